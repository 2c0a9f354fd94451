#!/bin/bash
# rocprofv3 kernel trace (--stats) of a short bench run; prints per-kernel mean durations.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/prof_q
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/gpurun_out/prof_q" -o run \
  -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/prof_q.log 2>&1 || exit $?
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/prof_q/run_kernel_stats.csv")):
    print(f"{r['Name'][:44]:44s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:8.4f}")
PY
