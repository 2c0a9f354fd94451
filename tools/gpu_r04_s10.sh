#!/bin/bash
# r04 session 10: call-path parity after the pend-fold rework, then base vs cur kernel traces.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/s10; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_genome.py tests/test_wide_samples.py tests/test_gpu_golden.py \
  -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "rows_only or consensus_word or call_kernel or fixture or stream or pipelined or inconsistent or wide or chunked or golden" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
O=$O VARIANTS="base cur" bash tools/gpu_r04_s6.sh 2>&1 | tail -20
