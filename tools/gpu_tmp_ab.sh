export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
POPBAM_GPU_LIB=$R/popbam_amd/variants/zg4/libpopbam_gpu.so timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k "window_stats_match and n12" > gpurun_out/pytest_zns.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_zns.log; [ $rc -ne 0 ] && exit $rc
AB="zg2 zg4" bash tools/gpu_bench_ab.sh
