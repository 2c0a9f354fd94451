#!/bin/bash
# HBM traffic of the call kernels on THIS source tree: rocprofv3 FETCH_SIZE and WRITE_SIZE in
# separate --pmc passes (one counter set per process, each under its own kill timeout) over one
# bench.py step, summarised by tools/pmc_traffic.py into profiles/pmc_traffic_c<config>.json
# (keyed by bench.source_hash(); bench.py reports roofline.traffic only for a matching tree).
# usage: tools/pmc_traffic.sh <config> <tag> [extra bench args]
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
CFG=${1:-2}; TAG=${2:-r04}; shift 2
D=gpurun_out/pmc_c$CFG; rm -rf "$D"; mkdir -p "$D"
ARGS="--config $CFG --steps 1 --warmup 0 --cpu-sample 0 --parity-windows 0 --e2e-chunk -1 --cli-sample 0 $*"
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $set -T --output-format csv -d "$R/$D/p$i" -o run \
    -- python3 "$R/bench.py" $ARGS > "$D/p$i.log" 2>&1 || { echo "pmc pass $i ($set) failed"; tail -5 "$D/p$i.log"; exit 1; }
done
python3 tools/pmc_summary.py "$D" > "$D/summary.txt" || exit 1
python3 tools/pmc_traffic.py "$D" "$TAG" $ARGS || exit 1
mkdir -p "profiles/${PROFDIR:-r06}"; cp "$D/summary.txt" "profiles/${PROFDIR:-r06}/${TAG}_pmc_hbm_summary_c$CFG.txt"
