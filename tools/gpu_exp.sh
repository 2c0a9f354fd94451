set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
BENCH_ARGS="--steps 10 --warmup 2 --cpu-sample 0" bash tools/ab.sh head dg64 dg32 head dg64 dg32 || exit 1
timeout -k 10 400 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_golden.py -k "call or rows_only or fixture or deep or golden" > gpurun_out/pytest_call.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_call.log; exit 1; }
tail -2 gpurun_out/pytest_call.log
