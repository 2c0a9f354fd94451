#!/usr/bin/env python3
"""Copy a GPU session's rocprofv3 results from gpurun_out/ into profiles/<tag>_* and derive
the per-launch HBM traffic of the dominant kernel (profiles/pmc_call_scan_kernel.json, read by bench.py).

FETCH_SIZE on gfx950 reports half the bytes of wide coalesced streaming reads
(MI355X_MICROARCH.md, HBM/rocprofv3 section): it is doubled here.  FETCH_SIZE and WRITE_SIZE
come from separate --pmc passes (tools/gpu_round.sh).  Usage: tools/profile_summary.py TAG
"""
import csv
import collections
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "gpurun_out")
PROF = os.path.join(REPO, "profiles")


def per_kernel(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


def main():
    tag = sys.argv[1]
    rnd = tag.split("s")[0] if tag.startswith("r") else "misc"
    global PROF
    top = PROF
    PROF = os.path.join(top, rnd)
    os.makedirs(PROF, exist_ok=True)
    shutil.copy(os.path.join(OUT, "prof_trace", "run_kernel_stats.csv"), os.path.join(PROF, f"{tag}_kernel_stats.csv"))
    bench = open(os.path.join(OUT, "bench.log")).read().strip().splitlines()[-1]
    b = json.loads(bench)
    open(os.path.join(PROF, f"{tag}_bench.json"), "w").write(bench + "\n")
    fetch = per_kernel(os.path.join(OUT, "prof_fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(OUT, "prof_write", "run_counter_collection.csv"))
    lines = ["kernel,fetch_size_kib_avg,fetch_bytes_corrected,write_size_kib_avg"]
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, 0.0), write.get(k, 0.0)
        lines.append(f"{k},{f:.3f},{int(f * 1024 * 2)},{w:.3f}")
    open(os.path.join(PROF, f"{tag}_pmc_hbm.csv"), "w").write("\n".join(lines) + "\n")
    k = b["roofline"]["kernel"]
    cfg = b["config"]
    pmc = {"kernel": k, "sites": cfg["sites_per_gpu"], "samples": cfg["samples"], "depth": cfg["mean_depth"],
           "fetch_size_kib": fetch[k], "write_size_kib": write[k], "fetch_correction": 2.0,
           "hbm_bytes_per_launch": int(fetch[k] * 1024 * 2 + write[k] * 1024),
           "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) on bench.py --steps 2, {tag}",
           "algorithmic_bytes_per_launch": b["roofline"]["bytes_per_launch"], "layout": "keys16",
           "pieces": cfg.get("pieces", 1)}
    json.dump(pmc, open(os.path.join(top, f"pmc_{k}.json"), "w"), indent=1)
    print(json.dumps(pmc, indent=1))


if __name__ == "__main__":
    main()
