#!/bin/bash
# configs[3] window stage, product vs a variant library (POPBAM_GPU_LIB).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/c3_ab; mkdir -p $O; export TMPDIR=/tmp
for v in product ${AB:-}; do
  L=""; [ "$v" != product ] && L=$R/popbam_amd/variants/$v/libpopbam_gpu.so
  POPBAM_GPU_LIB=$L timeout -k 10 300 python bench.py --allow-variant --config 3 --steps 1 --warmup 1 --cpu-sample 0 > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python3 -c "
import json,sys
d=json.loads(open('$O/$v.json').read().strip().splitlines()[-1])
print('$v', d['value'], d['ms_per_step'], 'scan', d['roofline']['ms_per_launch'], 'call', d['call_stage']['ms_per_pass'], 'win', d['window_stage']['ms_per_pass'])"
done
