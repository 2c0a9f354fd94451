#!/bin/bash
# configs[4] line (2 timed passes), library variants VS (popbam_amd/variants/NAME, tools/variant.sh),
# alternating, 2 reps: value, step, scan per chunk and frac, call stage per pass.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/c4ab; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do for v in ${VS:-w64 w128 w192}; do
  POPBAM_GPU_LIB=$R/popbam_amd/variants/$v/libpopbam_gpu.so timeout -k 10 300 python bench.py --allow-variant --config 4 --steps 2 --warmup 1 --cpu-sample 0 --parity-windows 0 > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -5 $O/${v}_$rep.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/${v}_$rep.json').read().strip().splitlines()[-1])
print('$v', $rep, d['value'], d['ms_per_step'], 'scan', d['roofline']['ms_per_launch'], d['roofline']['frac'], 'call', d['call_stage']['ms_per_pass'], d.get('parity_sampled'))"
done; done
