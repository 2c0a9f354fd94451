"""The PBG_BOUNDS debug build (popbam_amd/variants/bounds/libpopbam_gpu.so, pbg_common.h) checks
every key LOAD of the call kernels against [block_off[0], block_off[last]) and every device STORE
and bump against its array's allocation -- the scan's queue records (inside D.raw and inside the
block's own region: r05's one GPU fault was a queue-region base computed past D.raw), the deep-task
list, the info bytes, the rows, the per-block pending masks / queue counts, the consensus words and
the statistics workspace (pool slices, ZnS lists, omega / Wall lists).  A green bounds run only
shows that no check fired, so each class has a positive control: PBG_BOUNDS_SELFTEST=<class> cuts
that class's checked range (keys: the batch's last chunk; queue / info / block: half the array;
deep: all of it; rows / words: half the batch; pool: half of every slice) and correct kernels must
trip exactly that check, with pbg_check reporting PBG_E_BATCH and the class's own message -- on the
rows-only pipeline (scan / list pass / queues / folds), on the consensus-word kernels and on the
window statistics.  Without a self-test the same calls are clean, and the product build ignores
the variable."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BOUNDS_LIB = os.path.join(REPO, "popbam_amd", "variants", "bounds", "libpopbam_gpu.so")

# three calls per run: the rows-only call, the consensus-word call, the window statistics over
# one window of the whole batch (more segregating rows than LDS keeps: its rows go to the pool)
# with ZnS (its lists at fixed places)
SNIPPET = r"""
import sys, torch
sys.path.insert(0, {repo!r})
from popbam_amd import _lib, workload
ctx = _lib.Context(workload.default_params({n}), 0)
L = 64 * 1000
syn = workload.SynthPileup(ctx, L, 10, 0xC0FFEE02 + {n})
hp = workload.HotPath(ctx, syn, [(0, L // 2), (L // 2, L)], _lib.PBG_S_NUCDIV | _lib.PBG_S_SFS | _lib.PBG_S_ZNS)
out = []
def check():
    rc = ctx.lib.pbg_check(ctx.h, None)
    out.append("%d:%s" % (rc, ctx.lib.pbg_last_error(ctx.h).decode() if rc else ""))
hp.call()
check()
cb = torch.zeros(L * {n}, dtype=torch.int64, device="cuda")
hp.call(cb=cb)
check()
hp.call()
torch.cuda.synchronize()
ctx.lib.pbg_check(ctx.h, None)   # the rows-only call again (its flags, if any, cleared)
hp.window_stats()
check()
ctx.close()
print("|".join(out))
"""

# class -> (message fragment, fires on: rows-only call, consensus-word call, statistics)
MODES = {
    "keys": ("loaded keys outside", (True, True, False)),
    "queue": ("queue record", (True, False, False)),
    "info": ("info byte", (True, True, False)),
    "deep": ("deep-task", (True, True, False)),
    "block": ("pending mask", (True, False, False)),
    "rows": ("a row was stored", (True, True, False)),
    "words": ("consensus word", (False, True, False)),
    "pool": ("statistics workspace store", (False, False, True)),
}


def _run(lib, selftest, n):
    env = dict(os.environ)
    env.pop("PBG_BOUNDS_SELFTEST", None)
    if selftest:
        env["PBG_BOUNDS_SELFTEST"] = selftest
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
def test_bounds_build_clean_without_selftest(gpu_lib, n):
    assert os.path.exists(BOUNDS_LIB), "build it with __graft_entry__.build() (make bounds)"
    assert _run(BOUNDS_LIB, None, n) == ["0:", "0:", "0:"]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [12, 96])
@pytest.mark.parametrize("mode", list(MODES))
def test_bounds_build_positive_control(gpu_lib, n, mode):
    """Each class's check fires on exactly the calls that store (or load) into that class."""
    assert os.path.exists(BOUNDS_LIB), "build it with __graft_entry__.build() (make bounds)"
    frag, where = MODES[mode]
    res = _run(BOUNDS_LIB, mode, n)
    for fires, r in zip(where, res):
        rc, msg = r.split(":", 1)
        if fires:
            assert int(rc) == -6 and "PBG_BOUNDS" in msg and frag in msg, (mode, res)
        else:
            assert r == "0:", (mode, res)


@pytest.mark.gpu
def test_bounds_selftest_1_is_the_key_class(gpu_lib):
    """PBG_BOUNDS_SELFTEST=1 (r05's spelling) still means the key-load control."""
    res = _run(BOUNDS_LIB, "1", 12)
    assert [r.split(":", 1)[0] for r in res] == ["-6", "-6", "0"], res


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["keys", "queue", "pool"])
def test_product_build_ignores_bounds_selftest(gpu_lib, mode):
    assert _run(None, mode, 12) == ["0:", "0:", "0:"]
