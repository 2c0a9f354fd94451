#!/bin/bash
# configs[2] bench, product vs a variant library, alternating (run-order balanced).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/bench_ab; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
for v in product ${AB:-}; do
  L=""; [ "$v" != product ] && L=$R/popbam_amd/variants/$v/libpopbam_gpu.so
  POPBAM_GPU_LIB=$L timeout -k 10 300 python bench.py --allow-variant --steps 20 --warmup 3 --cpu-sample 0 --cli-sample 0 --e2e-chunk -1 > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -5 $O/${v}_$rep.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/${v}_$rep.json').read().strip().splitlines()[-1])
print('$v', $rep, d['value'], d['ms_per_step'], 'scan', d['roofline']['ms_per_launch'], 'call', d['call_stage']['ms_serial'], 'stats', d['window_stats']['ms_serial'])"
done; done
