#!/bin/bash
# r05 step 8: counter list of the box, then SQ / GRBM / TA counters of the generator (split kernel)
# at the configs[3] chunk shape, one counter set per process under its own kill timeout.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05s8; mkdir -p $O/pmc; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || echo "counter list failed"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC" \
           "GRBM_GUI_ACTIVE GRBM_COUNT" "TA_TA_BUSY TA_BUFFER_WAVEFRONTS" "TA_BUFFER_READ_WAVEFRONTS TA_BUFFER_WRITE_WAVEFRONTS" \
           "TD_TD_BUSY TD_TC_STALL"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -T --output-format csv -d "$R/$O/pmc/p$i" -o run \
    -- python3 "$R/tools/synth_bench.py" --samples 24 --sites 33554432 --reps 2 > $O/pmc/p$i.log 2>&1 || { echo "pmc pass $i ($set) failed"; tail -3 $O/pmc/p$i.log; }
done
python3 tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt; grep -A60 "^synth_keys_split_kernel" $O/pmc_summary.txt | head -70
