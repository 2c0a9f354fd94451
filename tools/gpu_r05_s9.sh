#!/bin/bash
# r05 step 9: generator timing, product (split) vs template-locality experiments, configs[3] shape.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05s9; mkdir -p $O; export TMPDIR=/tmp
SYNTH_ARGS="--samples 24 --sites 33554432 --reps 5" bash tools/gpu_synth_ab.sh ${AB:-synadj synadj32} > $O/synth_c3.log 2>&1 || { cat $O/synth_c3.log; exit 1; }
cat $O/synth_c3.log
