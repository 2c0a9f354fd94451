#!/bin/bash
# r05 step 5: generator rework -- its parity tests (device generator vs the oracle's, chunked
# genome pass), then the generator timing at the configs[3] / configs[4] chunk shapes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05s5; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_genome.py -x -q -m gpu -p no:cacheprovider \
  --timeout 200 --timeout-method thread -k "generator or chunked or serial or rows_only or call_kernel" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
SYNTH_ARGS="--samples 24 --sites 33554432 --reps 5" bash tools/gpu_synth_ab.sh ${AB:-} > $O/synth_c3.log 2>&1 || exit 1
cat $O/synth_c3.log
[ -n "${SKIP96:-}" ] || SYNTH_ARGS="--samples 96 --sites 8388608 --reps 5 --seed 0xC0FFEE05" bash tools/gpu_synth_ab.sh ${AB:-} > $O/synth_c4.log 2>&1 || exit 1
cat $O/synth_c4.log
