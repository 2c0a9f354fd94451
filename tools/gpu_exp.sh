set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench/fadd_chain || exit 1
BENCH_ARGS="--steps 5 --warmup 1 --cpu-sample 0" bash tools/ab.sh f32row dq2row dq1 dq8 main || exit 1
timeout -k 10 400 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_scale.py -k "call or rows_only or fixture or pipelined" > gpurun_out/pytest_call.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_call.log; exit 1; }
tail -2 gpurun_out/pytest_call.log
