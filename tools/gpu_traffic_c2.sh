#!/bin/bash
# HBM counters of the configs[2] call on this tree (profiles/pmc_traffic_c2.json), then the default bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/final; export TMPDIR=/tmp
bash tools/pmc_traffic.sh 2 r05f || exit 1
timeout -k 10 400 python bench.py > gpurun_out/final/bench_c2_final.json 2> gpurun_out/final/bench_c2_final.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/final/bench_c2_final.json')); r=d['roofline']; print('c2', d['value'], d['ms_per_step'], r['frac'], r.get('traffic'), r.get('traffic_ratio'))"
