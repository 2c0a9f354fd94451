#!/bin/bash
# Round-end check: the -m gpu suite + smoke, then the configs[2] bench line (with baselines) and the
# configs[4] / configs[3] lines (no CPU baseline).  Every GPU step has its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/final; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/final/pytest_gpu.log; tail -3 gpurun_out/final/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/final/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final/bench_c2.json 2> gpurun_out/final/bench_c2.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/final/bench_c2.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/final/bench_c4.json 2> gpurun_out/final/bench_c4.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/final/bench_c4.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/final/bench_c3.json 2> gpurun_out/final/bench_c3.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/final/bench_c3.json')); print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'])"
exit 0
