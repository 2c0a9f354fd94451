#!/bin/bash
# r05 step 6: generator variants (no stores / no template loads / neither / reach-only loads) at
# the configs[3] chunk shape, then SQ counters of the product generator there.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05s6; mkdir -p $O; export TMPDIR=/tmp
SYNTH_ARGS="--samples 24 --sites 33554432 --reps 5" bash tools/gpu_synth_ab.sh synx1 synx2 synx3 synx4 > $O/synth_c3.log 2>&1 || { cat $O/synth_c3.log; exit 1; }
cat $O/synth_c3.log
mkdir -p $O/pmc
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -T --output-format csv -d "$R/$O/pmc/p$i" -o run \
    -- python3 "$R/tools/synth_bench.py" --samples 24 --sites 33554432 --reps 2 > $O/pmc/p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $O/pmc > $O/pmc_summary.txt && grep -A40 "^synth_keys_kernel" $O/pmc_summary.txt
