#!/bin/bash
# rocprofv3 kernel traces of the configs[3] / configs[4] lines (one timed pass each) on the final
# tree: the scan's per-launch mean beside the lines' HIP-event figure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r06f; mkdir -p $O; export TMPDIR=/tmp
for c in 3 4; do
  rm -rf $O/prof_c$c
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/$O/prof_c$c" -o run \
    -- python3 "$R/bench.py" --config $c --steps 1 --warmup 1 --cpu-sample 0 --parity-windows 0 > $O/prof_c$c.log 2>&1 || { tail -5 $O/prof_c$c.log; exit 1; }
  python3 tools/kstats.py $O/prof_c$c/run_kernel_stats.csv | head -8
  grep '^{"metric"' $O/prof_c$c.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('line', d['value'], d['roofline']['ms_per_launch'], d['roofline']['frac'])"
done
