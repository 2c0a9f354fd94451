#!/bin/bash
# SQ counter passes (instruction mix, wave states) over a short bench run: tools/pmc_sq.sh with
# BENCH_ARGS; summary -> gpurun_out/pmc/summary.txt.  Then a kernel trace of the same run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
PASSES="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
  bash tools/pmc_sq.sh || exit 1
mkdir -p gpurun_out/trace
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/trace" -o run --output-format csv \
  -- python3 "$R/bench.py" ${BENCH_ARGS:---steps 2 --warmup 1 --cpu-sample 0} > gpurun_out/trace/bench.log 2>&1 || exit 1
f=$(find gpurun_out/trace -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -d, -f1-4
