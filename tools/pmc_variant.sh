#!/bin/bash
# SQ counter pass over one library variant: tools/pmc_variant.sh NAME "COUNTERS"
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/pmcv; export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---sites 10000000 --steps 2 --warmup 0 --cpu-sample 0}
POPBAM_GPU_LIB=$R/popbam_amd/variants/$1/libpopbam_gpu.so timeout -s KILL 120 rocprofv3 --pmc $2 -T --output-format csv -d "$R/gpurun_out/pmcv/$1" -o run \
    -- python3 "$R/bench.py" --allow-variant $ARGS > gpurun_out/pmcv/$1.log 2>&1
