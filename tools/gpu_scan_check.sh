#!/bin/bash
# Call-path parity (scale, chunked genome, golden fixtures) on the product library, then the
# configs[2] A/B against a variant library (AB=<name>, tools/gpu_bench_ab.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/scan_check; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py tests/test_genome.py tests/test_gpu_golden.py -x -q -m gpu \
  -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_bench_ab.sh
