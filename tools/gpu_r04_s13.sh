#!/bin/bash
# r04 session 13: soft-masked reference runs (parity + call time), the call-path tests, and
# base vs cur kernel traces after the overflow kernel's shortcut settling.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/s13; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_scale.py tests/test_wide_samples.py tests/test_gpu_golden.py \
  -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "soft_masked or rows_only or consensus_word or call_kernel or fixture or inconsistent or wide or golden" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/softmask_probe.py 10000000 > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
grep masked $O/probe.log
O=$O VARIANTS="base cur base cur" bash tools/gpu_r04_s6.sh 2>&1 | grep -E "==|scan|slow|overflow|pend"
