#!/bin/bash
# r04 final check 4a: the whole -m gpu suite + smoke, then the PBG_BOUNDS build under the
# call-path tests, on the round's last tree.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/f4; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 \
    --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
BOUNDS_TIMEOUT=360 K_EXPR="host_stream or chunked or serial or overlapping or inconsistent or rows_only or soft_masked or fixture" bash tools/gpu_bounds.sh || exit 1
