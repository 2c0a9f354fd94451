"""Static checks of kernel building blocks that need no GPU."""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_sort16_network_sorts_every_binary_input():
    """0-1 principle: a comparator network sorts all inputs iff it sorts all 2^16 0/1 inputs."""
    src = open(os.path.join(REPO, "popbam_amd", "csrc", "call_kernel.hip")).read()
    body = src[src.index("void sort16_desc"):src.index("#undef CS")]
    pairs = [tuple(map(int, m)) for m in re.findall(r"CS\((\d+), (\d+)\)", body)]
    assert pairs and all(i < j < 16 for i, j in pairs)
    for x in range(1 << 16):
        a = [(x >> i) & 1 for i in range(16)]
        for i, j in pairs:
            if a[i] < a[j]:
                a[i], a[j] = a[j], a[i]
        assert all(a[i] >= a[i + 1] for i in range(15)), f"input {x:#06x} not sorted"
