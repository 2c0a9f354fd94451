#!/bin/bash
# r04 session 18: mid-block list pass at <= 24 samples (ms) vs HEAD (base): configs[2] traces
# (run-order balanced) and the soft-masked probe under each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/s18; mkdir -p $O; export TMPDIR=/tmp
O=$O VARIANTS="base ms base ms" bash tools/gpu_r04_s6.sh 2>&1 | grep -E "==|call_scan|call_overflow"
for v in base ms; do
  POPBAM_GPU_LIB=$R/popbam_amd/variants/$v/libpopbam_gpu.so timeout -k 10 300 python3 tools/softmask_probe.py 10000000 > $O/probe_$v.log 2>&1 || { tail -3 $O/probe_$v.log; exit 1; }
  echo "probe $v"; grep masked $O/probe_$v.log
done
