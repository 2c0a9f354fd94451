#!/bin/bash
# configs[4] (200 Msites x 96 samples, overlapping 1 kb / 500 bp windows, nucdiv + sfs + haplo
# EHHS) on one GPU: the bench line with the CPU port baseline and a rocprofv3 kernel trace of one
# pass; then the configs[3] bench line.  Every GPU step has its own time limit; stops at the first
# failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/c4; export TMPDIR=/tmp
timeout -k 10 600 python bench.py --config 4 --steps 2 --warmup 1 > gpurun_out/c4/bench.json 2> gpurun_out/c4/bench.err || exit $?
cat gpurun_out/c4/bench.json
rm -rf gpurun_out/c4/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/gpurun_out/c4/prof" -o run \
  -- python3 "$R/bench.py" --config 4 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/c4/prof.log 2>&1 || exit $?
python3 tools/kstats.py gpurun_out/c4/prof/run_kernel_stats.csv
if [ "${C3:-1}" = "1" ]; then
  timeout -k 10 600 python bench.py --config 3 --steps 2 --warmup 1 > gpurun_out/c4/bench_c3.json 2> gpurun_out/c4/bench_c3.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c4/bench_c3.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
fi
exit 0
