#!/bin/bash
# configs[3] default (serial) and --overlap lines at the default chunk.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/c3_modes; mkdir -p $O; export TMPDIR=/tmp
for m in "" "--overlap"; do
  t=${m:-serial}; t=${t#--}
  timeout -k 10 400 python bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 $m > $O/c3_$t.json 2> $O/c3_$t.err || { tail -5 $O/c3_$t.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/c3_$t.json').read().strip().splitlines()[-1]); print('$t', d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['roofline']['frac'], d['parity_sampled'], d['rows_crosscheck']['identical'])"
done
