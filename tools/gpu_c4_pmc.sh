#!/bin/bash
# HBM counters of one configs[4] pass (FETCH_SIZE / WRITE_SIZE, one counter set per process, each
# under its own kill timeout), summarised per kernel by tools/pmc_summary.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/c4/pmc; export TMPDIR=/tmp
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1)); rm -rf "gpurun_out/c4/pmc/p$i"
  timeout -s KILL 300 rocprofv3 --pmc $set -T --output-format csv -d "$R/gpurun_out/c4/pmc/p$i" -o run \
    -- python3 "$R/bench.py" --config 4 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/c4/pmc/p$i.log 2>&1 \
    || { echo "pmc pass $i failed"; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/c4/pmc > gpurun_out/c4/pmc/summary.txt && head -60 gpurun_out/c4/pmc/summary.txt
