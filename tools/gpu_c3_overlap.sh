#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/final; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 --overlap > $O/bench_c3_overlap.json 2> $O/bench_c3_overlap.err || { tail -5 $O/bench_c3_overlap.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c3_overlap.json').read().strip().splitlines()[-1]); print('c3ov', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity_sampled'], d['rows_crosscheck']['identical'])"
