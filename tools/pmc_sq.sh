#!/bin/bash
# SQ (and TCC) counter passes over a short configs[2] bench run, one --pmc pass per process,
# each under its own kill timeout; then the per-kernel summary (tools/pmc_summary.py).
#   PASSES: ';'-separated counter sets (default: instruction mix + wave states)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---steps 2 --warmup 1 --cpu-sample 0}
DEF="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT;FETCH_SIZE;WRITE_SIZE"
IFS=';' read -ra SETS <<< "${PASSES:-$DEF}"
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  rm -rf "gpurun_out/pmc/p$i"
  timeout -s KILL 120 rocprofv3 --pmc $set -T --output-format csv -d "$R/gpurun_out/pmc/p$i" -o run \
    -- python3 "$R/bench.py" $ARGS > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i ($set) failed"; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt && cat gpurun_out/pmc/summary.txt
