#!/bin/bash
# r05 step 3: PBG_BOUNDS positive control, mixed-quality scale parity, CLI probe (phases).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05s3; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_bounds_build.py -x -v -m gpu -p no:cacheprovider --timeout 200 \
    --timeout-method thread > $O/pytest_bounds.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_bounds.log; tail -4 $O/pytest_bounds.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_mixed_quality.py -x -v -m gpu -p no:cacheprovider --timeout 120 \
    --timeout-method thread --durations=0 > $O/pytest_mixed.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_mixed.log; tail -8 $O/pytest_mixed.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/cli_probe.py > $O/cli_probe.json 2> $O/cli_probe.err
rc=$?; tail -c 600 $O/cli_probe.json; exit $rc
