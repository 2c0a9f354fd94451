#!/bin/bash
# Round-end check: PBG_BOUNDS build under the parity tests, the default bench line, a kernel trace of
# the configs[2] step, and its HBM counters (profiles/pmc_traffic_c2.json for this tree).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/final; mkdir -p $O; export TMPDIR=/tmp
bash tools/gpu_bounds.sh || exit 1
timeout -k 10 400 python bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { tail -5 $O/bench_c2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c2.json')); print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic'))"
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/$O/prof" -o run \
  -- python3 "$R/bench.py" --steps 20 --warmup 3 --cpu-sample 0 --cli-sample 0 > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python3 tools/kstats.py $O/prof/run_kernel_stats.csv | head -12
bash tools/pmc_traffic.sh 2 r06 || exit 1
for c in 3 4; do
  timeout -k 10 400 python bench.py --config $c --steps 2 --warmup 1 --cpu-sample 0 > $O/bench_c$c.json 2> $O/bench_c$c.err || { tail -5 $O/bench_c$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_c$c.json').read().strip().splitlines()[-1]); print('c$c', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity_sampled'], d['rows_crosscheck']['identical'])"
done
