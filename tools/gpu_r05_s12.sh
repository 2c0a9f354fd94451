#!/bin/bash
# r05 step 12: configs[4] line (serial and overlapped), CLI probe (fresh native processes).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05s12; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 > $O/c4_serial.json 2> $O/c4_serial.err || { tail -5 $O/c4_serial.err; exit 1; }
timeout -k 10 400 python bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 --overlap > $O/c4_overlap.json 2> $O/c4_overlap.err || { tail -5 $O/c4_overlap.err; exit 1; }
for f in c4_serial c4_overlap; do python3 -c "
import json
d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], 'scan', d['roofline']['ms_per_launch'], d['roofline']['frac'], 'call', d['call_stage']['ms_per_pass'], 'win', d['window_stage']['ms_per_pass'], d['parity_sampled'], d['rows_crosscheck']['identical'])"; done
timeout -k 10 600 python -u tools/cli_probe.py > $O/cli_probe.json 2> $O/cli_probe.err || { tail -5 $O/cli_probe.err; exit 1; }
tail -c 800 $O/cli_probe.json
