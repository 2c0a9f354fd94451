"""The PBG_BOUNDS debug build (popbam_amd/variants/bounds/libpopbam_gpu.so: every key load of the
call kernels checked against [block_off[0], block_off[last]), pbg_common.h) needs a positive
control: a green bounds run only shows that no check fired.  With PBG_BOUNDS_SELFTEST=1 the bounds
build takes the batch's last 16-byte key chunk out of the allowed range, so correct kernels, which
read it, must trip the check, and pbg_check must report PBG_E_BATCH with the bounds message -- on
the rows-only pipeline (scan / list pass / queues) and on the consensus-word kernel.  Without it
the same calls are clean, and the product build ignores the variable."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOUNDS_LIB = os.path.join(REPO, "popbam_amd", "variants", "bounds", "libpopbam_gpu.so")

SNIPPET = r"""
import sys, torch
sys.path.insert(0, {repo!r})
from popbam_amd import _lib, workload
ctx = _lib.Context(workload.default_params({n}), 0)
L = 64 * 300
syn = workload.SynthPileup(ctx, L, 10, 0xC0FFEE02 + {n})
hp = workload.HotPath(ctx, syn, [(0, L)], 0)
out = []
for words in (False, True):
    cb = torch.zeros(L * {n}, dtype=torch.int64, device="cuda") if words else None
    hp.call(cb=cb)
    rc = ctx.lib.pbg_check(ctx.h, None)
    out.append("%d:%s" % (rc, ctx.lib.pbg_last_error(ctx.h).decode() if rc else ""))
ctx.close()
print("|".join(out))
"""


def _run(lib, selftest, n):
    env = dict(os.environ, PBG_BOUNDS_SELFTEST=str(selftest))
    if lib:
        env["POPBAM_GPU_LIB"] = lib
    else:
        env.pop("POPBAM_GPU_LIB", None)
    r = subprocess.run([sys.executable, "-c", SNIPPET.format(repo=REPO, n=n)], env=env, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.strip().splitlines()[-1].split("|")


@pytest.mark.gpu
@pytest.mark.parametrize("n", [12, 96])
def test_bounds_build_positive_control(gpu_lib, n):
    assert os.path.exists(BOUNDS_LIB), "build it with __graft_entry__.build() (make bounds)"
    fired = _run(BOUNDS_LIB, 1, n)
    for res in fired:
        rc, msg = res.split(":", 1)
        assert int(rc) == -6 and "PBG_BOUNDS" in msg, fired
    assert _run(BOUNDS_LIB, 0, n) == ["0:", "0:"]


@pytest.mark.gpu
def test_product_build_ignores_bounds_selftest(gpu_lib):
    assert _run(None, 1, 12) == ["0:", "0:"]
