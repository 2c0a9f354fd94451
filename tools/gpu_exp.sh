set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/ab3
timeout -k 10 200 python3 bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/ab3/c3.json 2> gpurun_out/ab3/c3.err || { tail -3 gpurun_out/ab3/c3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab3/c3.json')); print('c3', d['value'], d['ms_per_step'], d['roofline'])"
timeout -k 10 300 python3 bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/ab3/c4.json 2> gpurun_out/ab3/c4.err || { tail -3 gpurun_out/ab3/c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab3/c4.json')); print('c4', d['value'], d['ms_per_step'], d['roofline'])"
