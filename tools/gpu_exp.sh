set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
BENCH_ARGS="--steps 10 --warmup 2 --cpu-sample 0" bash tools/ab.sh head cf cf_pw1 cf_pw2 head cf || exit 1
export TMPDIR=/tmp
rm -rf gpurun_out/prof_q
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/gpurun_out/prof_q" -o run \
  -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof_q.log 2>&1 || exit 1
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_q/run_kernel_stats.csv')):
    print(f\"{r['Name'][:40]:40s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:8.4f}\")
" | head -9
timeout -k 10 700 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests > gpurun_out/pytest_all.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_all.log; exit 1; }
tail -2 gpurun_out/pytest_all.log
