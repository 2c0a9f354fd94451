set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
BENCH_ARGS="--steps 10 --warmup 2 --cpu-sample 0" bash tools/ab.sh head two head two || exit 1
POPBAM_GPU_LIB=$R/popbam_amd/variants/two/libpopbam_gpu.so timeout -k 10 700 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests > gpurun_out/pytest_two.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_two.log; exit 1; }
tail -2 gpurun_out/pytest_two.log
