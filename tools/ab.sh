#!/bin/bash
# A/B timing of library variants (popbam_amd/variants/NAME/libpopbam_gpu.so) with bench.py.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/ab
ARGS=${BENCH_ARGS:---sites 10000000 --steps 5 --warmup 1 --cpu-sample 0}
for v in "$@"; do
  POPBAM_GPU_LIB=$R/popbam_amd/variants/$v/libpopbam_gpu.so timeout -k 10 120 python3 bench.py --allow-variant $ARGS > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err || exit $?
  python3 -c "import json,sys; d=json.load(open('gpurun_out/ab/$v.json')); print('$v', d['roofline']['ms_per_launch'], d['window_stats']['ms_serial'], d['call_stage']['ms_library_events'], d['value'])"
done
