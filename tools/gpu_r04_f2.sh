#!/bin/bash
# r04 final check 2: HBM counters of this tree (configs[2] and configs[4]: FETCH_SIZE and
# WRITE_SIZE in separate passes -> profiles/pmc_traffic_c*.json), a kernel trace of the default
# bench, the default bench line (which then reports the counters as roofline.traffic), and the
# PBG_BOUNDS build under the call-path tests.  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/f2; mkdir -p $O; export TMPDIR=/tmp
bash tools/pmc_traffic.sh 2 r04f2 || exit 1
bash tools/pmc_traffic.sh 4 r04f2 --steps 1 || exit 1
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/$O/prof" -o run \
  -- python3 "$R/bench.py" --steps 10 --warmup 2 --cpu-sample 0 --parity-windows 0 --e2e-chunk -1 --cli-sample 0 \
  > $O/prof.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
python3 tools/kstats.py $O/prof/run_kernel_stats.csv | head -12
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], json.dumps(d['roofline'])[:900], d['call_stage'].get('traffic_ratio'), d.get('parity_sampled'), d.get('rows_crosscheck', {}).get('identical'))"
BOUNDS_TIMEOUT=700 bash tools/gpu_bounds.sh || exit 1
