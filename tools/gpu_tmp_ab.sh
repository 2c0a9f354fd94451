export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_mixed_quality.py tests/test_compact.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k "call_kernel or rows_only or soft_masked or inconsistent or mixed or compact" > gpurun_out/pytest_pre.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_pre.log; [ $rc -ne 0 ] && exit $rc
AB="base fold" bash tools/gpu_bench_ab.sh
