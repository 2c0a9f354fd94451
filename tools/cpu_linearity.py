#!/usr/bin/env python3
"""CPU-baseline linearity check: POPBAM itself (oracle/_ref/popbam) runs
nucdiv, sfs and ld -w 10 as three single-threaded processes on BAMs of the first 200 k, 1 M and
5 M positions of the synthetic genome (tests/ref_baseline.py), at 12 and 24 samples; the
summed wall time per position must be flat in the prefix length for bench.py's 200 k-position
sample to stand for the 5 Msite prefix BASELINE.md asks for.  Writes one JSON document."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import ref_baseline  # noqa: E402

out = {"binary": "oracle/_ref/popbam (POPBAM 0.3 built from /root/reference)", "window": 10000, "runs": []}
for n, seed in ((12, 0xC0FFEE02), (24, 0xC0FFEE04)):
    for L in (200_000, 1_000_000, 5_000_000):
        t0 = time.perf_counter()
        d = ref_baseline.make_inputs(f"/tmp/popbam_lin_v3_{seed:x}_{L}_{n}", seed, L, n)
        tb = time.perf_counter() - t0
        t = ref_baseline.time_reference(d, L, 10_000, 1)
        r = {"samples": n, "sites": L, "bam_write_s": round(tb, 1), "wall_s": {k: round(v, 3) for k, v in t["single"].items()},
             "total_s": round(t["single_total_s"], 3), "us_per_site": round(t["single_total_s"] / L * 1e6, 4),
             "Msites_per_s": round(L / t["single_total_s"] / 1e6, 6)}
        out["runs"].append(r)
        print(json.dumps(r), flush=True)
json.dump(out, open(sys.argv[1] if len(sys.argv) > 1 else "cpu_linearity.json", "w"), indent=1)
