#!/usr/bin/env python3
"""Print a rocprofv3 --stats kernel summary (run_kernel_stats.csv): name, calls, mean ms, share."""
import csv
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    print(path)
    for r in rows:
        print(f"  {r['Name'][:48]:48s} calls={int(r['Calls']):5d} avg_ms={float(r['AverageNs']) / 1e6:9.4f} "
              f"pct={float(r['Percentage']):6.2f}")
