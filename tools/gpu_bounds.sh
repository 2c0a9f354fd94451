#!/bin/bash
# The PBG_BOUNDS debug build (every key load of the call kernels checked against
# [block_off[0], block_off[last]), pbg_common.h) under the host-stream, chunked-genome, fixture
# and scale parity tests; log -> gpurun_out/bounds/pytest.log.  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/bounds
test -f popbam_amd/variants/bounds/libpopbam_gpu.so || { echo "bounds build missing"; exit 1; }
POPBAM_GPU_LIB=$R/popbam_amd/variants/bounds/libpopbam_gpu.so timeout -k 10 ${BOUNDS_TIMEOUT:-600} \
  python -u -m pytest tests/test_gpu_scale.py tests/test_genome.py tests/test_gpu_golden.py tests/test_wide_samples.py \
  -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "${K_EXPR:-host_stream or chunked or serial or overlapping or golden or inconsistent or rows_only or call_kernel or u16_wrap or wide}" \
  > gpurun_out/bounds/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc (POPBAM_GPU_LIB=variants/bounds, PBG_BOUNDS)" >> gpurun_out/bounds/pytest.log
tail -3 gpurun_out/bounds/pytest.log
exit $rc
