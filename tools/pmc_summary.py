#!/usr/bin/env python3
"""Per-kernel mean of every counter in rocprofv3 --pmc pass directories (pN/**/run_counter_collection.csv),
FETCH_SIZE doubled (gfx950 reports half of wide streaming reads, MI355X_MICROARCH.md), plus derived
ratios for the SQ counters (quad-cycle units: ACTIVE_INST_VALU * 4 / WAVE_CYCLES ...)."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r.get("Kernel_Name") or r.get("Kernel-Name") or r.get("KernelName")
        name = (k or "?").split("(")[0].split("<")[0].replace("void ", "").replace("pbg::", "")
        cn = r.get("Counter_Name") or r.get("Counter-Name")
        v = float(r.get("Counter_Value") or r.get("Counter-Value") or 0)
        acc[name][cn].append(v)
rows = []
for name, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    if "FETCH_SIZE" in m:
        m["FETCH_SIZE_x2_bytes"] = m["FETCH_SIZE"] * 2 * 1024
    if "WRITE_SIZE" in m:
        m["WRITE_SIZE_bytes"] = m["WRITE_SIZE"] * 1024
    if m.get("SQ_WAVES"):
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"):
            if c in m:
                m[c + "_per_wave"] = m[c] / m["SQ_WAVES"]
    if m.get("SQ_WAVE_CYCLES"):
        for c in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS"):
            if c in m:
                m[c + "_frac_of_wave_cycles"] = m[c] / m["SQ_WAVE_CYCLES"]
    rows.append((name, m))
for name, m in sorted(rows, key=lambda x: -x[1].get("SQ_WAVE_CYCLES", x[1].get("FETCH_SIZE", 0))):
    print(name)
    for c in sorted(m):
        print(f"    {c:44s} {m[c]:.6g}")
