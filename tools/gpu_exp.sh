set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread tests > gpurun_out/pytest_all.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_all.log; exit 1; }
tail -2 gpurun_out/pytest_all.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 200 python3 bench.py > gpurun_out/bench.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['call_stage']['ms_library_events'], d['window_stats']['ms_serial'])"
