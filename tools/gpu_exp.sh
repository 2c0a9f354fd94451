set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 200 python3 bench.py --cpu-sample 0 > gpurun_out/bench_final.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/bench_final.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['call_stage']['ms_library_events'], d['window_stats']['ms_serial'])"
