#!/usr/bin/env python3
"""Real-data probe: the rows-only call on the configs[2]-shaped synthetic batch with a fraction
of the reference soft-masked (lower-case runs, as RepeatMasker leaves ~half of a mammalian
genome).  POPBAM compares the reference case-sensitively, so no read
matches a lower-case base and every called task of such a position leaves the scan's
reference-only test for its list (uniform / one-error settling) or the overflow kernel.
Prints the call time per fraction and checks the rows against the consensus-word call."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from popbam_amd import _lib, workload  # noqa: E402

n_sites = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
fracs = [float(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0.0, 0.1, 0.25, 0.5]
ctx = _lib.Context(workload.default_params(12), 0)
syn = workload.SynthPileup(ctx, n_sites, 10, 0xC0FFEE02)
hp = workload.HotPath(ctx, syn, [(0, n_sites)], 0)
ref0 = syn.ref.clone()
out = []
for frac in fracs:
    run = 5000
    pos = torch.arange(n_sites, device="cuda")
    masked = (pos % (run * 100)) < int(frac * run * 100)
    r = ref0.clone()
    letter = ((r & 0x7F) == ord("A")) | ((r & 0x7F) == ord("C")) | ((r & 0x7F) == ord("G")) | ((r & 0x7F) == ord("T"))
    r = torch.where(masked & letter, r | 0x20, r)
    syn.ref.copy_(r)
    hp.call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        hp.call()
    e1.record()
    torch.cuda.synchronize()
    ctx.sync_check()
    ms = e0.elapsed_time(e1) / 3
    fast = hp.rows.clone()
    cb = torch.empty(n_sites * 12, dtype=torch.int64, device="cuda")
    hp.call(cb=cb)
    torch.cuda.synchronize()
    same = bool(torch.equal(fast, hp.rows))
    del cb
    out.append({"masked_fraction": frac, "call_ms": round(ms, 3), "Msites_per_s_call": round(n_sites / ms / 1e3, 1),
                "rows_identical_to_word_path": same})
    print(json.dumps(out[-1]), flush=True)
ctx.close()
