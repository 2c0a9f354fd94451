#!/usr/bin/env python3
"""Print the kernels of the second-to-last step of a rocprofv3 kernel trace (start / end / duration
in microseconds relative to that step's call_scan_kernel), to see which call-stage kernel ends last."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("call_scan")]
i0 = idx[-2] if len(idx) > 1 else idx[-1]
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i0 + 12]:
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{r['Kernel_Name'][:32]:32s} {s:9.1f} {e:9.1f} {e - s:8.1f} stream={r.get('Stream_Id', '')}")
