set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
BENCH_ARGS="--steps 10 --warmup 2 --cpu-sample 0" bash tools/ab.sh head zfix head zfix || exit 1
timeout -k 10 700 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_golden.py tests/test_wide_samples.py tests/test_genome.py tests/test_cli.py > gpurun_out/pytest_stats.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_stats.log; exit 1; }
tail -2 gpurun_out/pytest_stats.log
