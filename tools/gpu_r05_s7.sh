#!/bin/bash
# r05 step 7: configs[3] pass serial and overlapped (two streams) on the new generator.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05s7; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 > $O/c3_serial.json 2> $O/c3_serial.err || { tail -5 $O/c3_serial.err; exit 1; }
cat $O/c3_serial.json
timeout -k 10 500 python bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 --overlap > $O/c3_overlap.json 2> $O/c3_overlap.err || { tail -5 $O/c3_overlap.err; exit 1; }
cat $O/c3_overlap.json
