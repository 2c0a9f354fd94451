#!/bin/bash
# configs[3] HBM counters of this tree (profiles/pmc_traffic_c3.json), then a configs[3] line
# that reports them (roofline.traffic for a matching source hash and shape).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/final; mkdir -p $O; export TMPDIR=/tmp
bash tools/pmc_traffic.sh 3 r05g || exit 1
timeout -k 10 400 python bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 > $O/bench_c3_traffic.json 2> $O/bench_c3_traffic.err || { tail -5 $O/bench_c3_traffic.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c3_traffic.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c3', d['value'], r['frac'], r['traffic'], r['traffic_ratio'], d['parity_sampled'], d['rows_crosscheck']['identical'])"
