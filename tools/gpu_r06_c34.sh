#!/bin/bash
# Round-6 configs[3] / configs[4] evidence on the final tree: the bench line (2 timed passes),
# then the HBM counters of one pass (profiles/pmc_traffic_c<N>.json, this tree's hash) and the
# bench line again, now carrying them.  CFGS selects the configs (default "3 4").
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r06; mkdir -p $O; export TMPDIR=/tmp
for c in ${CFGS:-3 4}; do
  PROFDIR=r06 bash tools/pmc_traffic.sh $c ${TAG:-r06} || exit 1
  timeout -k 10 600 python bench.py --config $c --steps 2 --warmup 1 > $O/bench_c$c.json 2> $O/bench_c$c.err || { tail -5 $O/bench_c$c.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_c$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c$c', d['value'], d['ms_per_step'], r['ms_per_launch'], r['frac'], r['traffic_ratio'], d['parity_sampled'], d['rows_crosscheck']['identical'], (d.get('window_stage') or {}).get('ms_per_pass'))"
done
