#!/bin/bash
# r04 session 11: run-order check of the base / cur scan difference (cur base cur base), then the
# configs[4] and configs[3] lines (parity_sampled + chunk rows cross-check).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/s11; mkdir -p $O; export TMPDIR=/tmp
O=$O VARIANTS="cur base cur base" bash tools/gpu_r04_s6.sh 2>&1 | grep -E "==|scan|slow|pend|zns"
timeout -k 10 600 python bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c4.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['alone'], d.get('parity_sampled'), d.get('rows_crosscheck'), d.get('window_stage'))"
timeout -k 10 600 python bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c3.json')); print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_sampled'), d.get('rows_crosscheck'), d.get('window_stage'))"
