#!/bin/bash
# SQ/TA counter passes over a short bench run (one --pmc pass each, separate processes).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---sites 10000000 --steps 2 --warmup 0 --cpu-sample 0}
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc/list_avail.txt 2>&1
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -T --output-format csv -d "$R/gpurun_out/pmc/p$i" -o run \
    -- python3 "$R/bench.py" $ARGS > gpurun_out/pmc/p$i.log 2>&1 || exit $?
done
exit 0
