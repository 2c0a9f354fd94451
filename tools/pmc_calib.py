#!/usr/bin/env python3
"""FETCH_SIZE / WRITE_SIZE calibration on gfx950 (tools/ubench/fetch_calib.hip): per access
pattern, the known bytes the kernel moves divided by the counter's bytes (counter KiB * 1024).
usage: pmc_calib.py <dir with p1 (FETCH_SIZE) and p2 (WRITE_SIZE) passes> <known-bytes json line>"""
import csv
import glob
import json
import os
import sys

root, known = sys.argv[1], json.loads(open(sys.argv[2]).read().strip().splitlines()[0])
cnt = {}
for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = (r.get("Kernel_Name") or "?").split("(")[0].split("<")[0].replace("void ", "").strip()
        cn = r.get("Counter_Name")
        cnt.setdefault(k, {}).setdefault(cn, []).append(float(r.get("Counter_Value") or 0))
out = {}
for k, b in known.items():
    c = cnt.get(k, {})
    name = "WRITE_SIZE" if k.startswith("store") else "FETCH_SIZE"
    if name in c:
        v = sum(c[name]) * 1024
        out[k] = {"known_bytes": b, "counter": name, "counter_bytes": int(v), "bytes_per_counter_byte": round(b / v, 4)}
print(json.dumps(out, indent=1))
