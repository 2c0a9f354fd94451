set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_scale.py -k "pipelined" > gpurun_out/pytest_pipe.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_pipe.log; exit 1; }
tail -1 gpurun_out/pytest_pipe.log
for p in 1 2 3 4 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --cpu-sample 0 --pieces $p > gpurun_out/bench_p$p.json 2>gpurun_out/bench_p$p.err || { tail -3 gpurun_out/bench_p$p.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_p$p.json')); print('pieces $p', d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['call_stage']['ms_library_events'], d['window_stats']['ms_serial'])"
done
