#!/bin/bash
# r04 final check 4b: HBM counters of the round's last tree (configs[2], configs[4]), a kernel
# trace of the default bench, and the default bench line reporting them.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/f4; mkdir -p $O; export TMPDIR=/tmp
bash tools/pmc_traffic.sh 2 r04f4 || exit 1
bash tools/pmc_traffic.sh 4 r04f4 --steps 1 || exit 1
rm -rf $O/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/$O/prof" -o run \
  -- python3 "$R/bench.py" --steps 10 --warmup 2 --cpu-sample 0 --parity-windows 0 --e2e-chunk -1 --cli-sample 0 \
  > $O/prof.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
python3 tools/kstats.py $O/prof/run_kernel_stats.csv > $O/kstats.txt; head -12 $O/kstats.txt
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d.get('parity_sampled'), d.get('rows_crosscheck',{}).get('identical'), (d.get('cli') or {}).get('x_over_popbam_all_cores'))"
timeout -k 10 600 python bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c4.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['alone']['frac'], d['roofline']['traffic_ratio'], d.get('parity_sampled'), d.get('rows_crosscheck',{}).get('identical'), d.get('window_stage',{}).get('ms_per_pass'))"
