"""Static checks of kernel building blocks that need no GPU."""
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _network(name):
    src = open(os.path.join(REPO, "popbam_amd", "csrc", "call_kernel.hip")).read()
    start = src.index(name)
    body = src[start:src.index("#undef CS", start)]
    return [tuple(map(int, m)) for m in re.findall(r"CS\((\d+), (\d+)\)", body)]


@pytest.mark.parametrize("n_wires", [1, 2, 3, 5, 8, 11, 12, 13, 16])
def test_pruned_sort16_network_sorts_every_binary_input(n_wires):
    """0-1 principle: a comparator network sorts all inputs iff it sorts all 0/1 inputs.  The
    kernel prunes the 16-wire network to its first N wires (comparators with j >= N dropped,
    wires >= N hold the minimum); check every N the kernel can use."""
    pairs = _network("void sortn_desc")
    assert len(pairs) == 63 and all(i < j < 16 for i, j in pairs)
    # the kernel returns after the first 19 comparators (the 8-wire sorter) when N <= 8
    kept = [(i, j) for i, j in (pairs[:19] if n_wires <= 8 else pairs) if j < n_wires]
    x = np.arange(1 << n_wires, dtype=np.uint32)
    a = ((x[:, None] >> np.arange(n_wires, dtype=np.uint32)) & 1).astype(np.uint8)
    for i, j in kept:
        hi = np.maximum(a[:, i], a[:, j])
        lo = np.minimum(a[:, i], a[:, j])
        a[:, i], a[:, j] = hi, lo
    assert (a[:, :-1] >= a[:, 1:]).all()
    if n_wires == 8:
        assert len(kept) == 19
    if n_wires == 12:
        assert len(kept) == 42
