#!/bin/bash
# rocprofv3 kernel trace of a short bench run for one variant: tools/trace.sh NAME
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/trace; export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---sites 10000000 --steps 3 --warmup 1 --cpu-sample 0}
for v in "$@"; do
POPBAM_GPU_LIB=$R/popbam_amd/variants/$v/libpopbam_gpu.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/gpurun_out/trace/$v" -o run \
    -- python3 "$R/bench.py" --allow-variant $ARGS > gpurun_out/trace/$v.log 2>&1 || exit $?
echo "== $v"; cut -d, -f1-4 gpurun_out/trace/$v/run_kernel_stats.csv | head -8
done
