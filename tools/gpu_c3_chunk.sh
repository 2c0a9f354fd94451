#!/bin/bash
# configs[3] (or CFG=4) pass time by chunk size (serial pass).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; C=${CFG:-3}; O=gpurun_out/c${C}_chunk; mkdir -p $O; export TMPDIR=/tmp
for ch in ${CHUNKS:-33554432 67108864 134217728}; do
  timeout -k 10 400 python bench.py --config $C --steps 2 --warmup 1 --cpu-sample 0 --chunk $ch > $O/c${C}_$ch.json 2> $O/c${C}_$ch.err || { tail -5 $O/c${C}_$ch.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c${C}_$ch.json').read().strip().splitlines()[-1]); print('chunk $ch', d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['roofline']['frac'], d['parity_sampled'], d['rows_crosscheck']['identical'])"
done
