set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
BENCH_ARGS="--steps 5 --warmup 1 --cpu-sample 0 --pieces 1" bash tools/ab.sh zlin zall zg0 zg0_u4 zg0_u8 || exit 1
timeout -k 10 700 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests > gpurun_out/pytest_all.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_all.log; exit 1; }
tail -2 gpurun_out/pytest_all.log
for p in 1 2 4; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --cpu-sample 0 --pieces $p > gpurun_out/bench_p$p.json 2>gpurun_out/bench_p$p.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/bench_p$p.json')); print('pieces $p', d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['call_stage']['ms_library_events'], d['window_stats']['ms_serial'])"
done
