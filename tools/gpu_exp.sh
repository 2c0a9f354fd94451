set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
POPBAM_GPU_LIB=$R/popbam_amd/variants/sstats/libpopbam_gpu.so timeout -k 10 120 python3 bench.py --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/sstats.log 2>&1 || exit 1
grep "slow-kernel classes" gpurun_out/sstats.log | tail -2
