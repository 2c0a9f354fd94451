#!/usr/bin/env python3
"""Per-launch HBM bytes of every kernel from rocprofv3 --pmc passes (FETCH_SIZE doubled: gfx950
counts half of wide streaming reads, MI355X_MICROARCH.md; WRITE_SIZE as is), written as
profiles/pmc_traffic_c<config>.json with the source hash of this tree (bench.source_hash) and
the bench shape, plus a per-round copy under profiles/$PROFDIR (default r06/) and a copy under
the counter directory (gpurun_out/..., which a GPU box hands back).
usage: pmc_traffic.py <pmc dir with p*/ passes> <tag> <bench args...>"""
import collections
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
root, tag, bargs = sys.argv[1], sys.argv[2], sys.argv[3:]
sys.argv = ["bench.py"] + bargs
import bench  # noqa: E402

args = bench.parse()
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName") or "?"
        name = k.split("(")[0].split("<")[0].replace("void ", "").replace("pbg::", "").strip()
        cn = r.get("Counter_Name") or r.get("Counter-Name")
        acc[name][cn].append(float(r.get("Counter_Value") or r.get("Counter-Value") or 0))
kern = {}
for name, cs in acc.items():
    fe = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) if cs.get("FETCH_SIZE") else 0.0
    wr = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) if cs.get("WRITE_SIZE") else 0.0
    kern[name] = {"fetch_bytes_x2": int(fe * 2 * 1024), "write_bytes": int(wr * 1024),
                  "hbm_bytes": int(fe * 2 * 1024 + wr * 1024), "launches": len(cs.get("FETCH_SIZE", []))}
if "call_scan_kernel" not in kern:
    sys.exit("no call_scan_kernel in the counter files")
if args.config == 2:
    shape = {"sites": args.sites, "samples": args.samples, "depth": args.depth, "pieces": args.pieces}
else:
    shape = {"contigs": args.contigs, "contig_len": args.contig_len, "samples": args.samples, "depth": args.depth,
             "chunk": args.chunk, "world": 1}
call = sum(kern.get(k, {}).get("hbm_bytes", 0) for k in bench.CALL_KERNELS)
out = {"src_sha": bench.source_hash(), "config": args.config, "shape": shape, "tag": tag,
       "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), bench.py {' '.join(bargs)}, {tag}",
       "fetch_correction": 2.0, "call_stage_hbm_bytes": call, "kernels": kern}
os.makedirs(os.path.join(REPO, "profiles", os.environ.get("PROFDIR", "r06")), exist_ok=True)
for path in (os.path.join(REPO, "profiles", f"pmc_traffic_c{args.config}.json"),
             os.path.join(REPO, "profiles", os.environ.get("PROFDIR", "r06"), f"{tag}_pmc_traffic_c{args.config}.json"),
             os.path.join(root, f"pmc_traffic_c{args.config}.json")):
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
print(json.dumps({k: v["hbm_bytes"] for k, v in kern.items()}))
