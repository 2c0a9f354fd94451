#!/bin/bash
# r05 step 14: generator parity tests, then the configs[2] A/B (step 13).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05s14; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_genome.py -x -q -m gpu -p no:cacheprovider \
  --timeout 200 --timeout-method thread -k "generator or chunked or serial or rows_only or call_kernel" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r05_s13.sh
