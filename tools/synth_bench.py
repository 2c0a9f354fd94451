"""The synthetic pileup generator alone (pbg_synth_pileup into device buffers), for timing under a
kernel trace: `python tools/synth_bench.py [--samples 24] [--sites 33554432] [--reps 5]`.
Prints the mean wall time per generation (HIP events on the stream) and the key count."""
import argparse
import ctypes as C
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from popbam_amd import _lib, workload  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--samples", type=int, default=24)
ap.add_argument("--sites", type=int, default=1 << 25)
ap.add_argument("--depth", type=int, default=10)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--seed", type=lambda s: int(s, 0), default=0xC0FFEE04)
a = ap.parse_args()
ctx = _lib.Context(workload.default_params(a.samples), 0)
syn = workload.SynthPileup(ctx, a.sites, a.depth, a.seed)
st = torch.cuda.current_stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
syn.generate(st, sync=False)
torch.cuda.synchronize()
e0.record(st)
for _ in range(a.reps):
    syn.generate(st, sync=False)
e1.record(st)
torch.cuda.synchronize()
ctx.sync_check()
ms = e0.elapsed_time(e1) / a.reps
print(json.dumps({"ms_per_generation": round(ms, 4), "keys": syn.n_keys, "sites": a.sites, "samples": a.samples,
                  "key_GBps": round(2 * syn.n_keys / (ms * 1e-3) / 1e9, 1),
                  "lib": ctx.lib.pbg_build_info().decode()}))
