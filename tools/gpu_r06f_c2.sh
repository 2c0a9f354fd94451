#!/bin/bash
# Round-6 final-tree configs[2] evidence: a rocprofv3 kernel trace of the bench step (20 steps), the
# HBM counters (FETCH_SIZE / WRITE_SIZE passes -> profiles/pmc_traffic_c2.json, this tree's hash),
# the SQ instruction-mix / wave-state passes, then the full bench line (cpu_baseline, streamed
# boundary, CLI) carrying the counters.  Every GPU step under its own time limit; stops at the
# first failure.  Outputs under gpurun_out/r06f (copied into profiles/r06/ by hand).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r06f; mkdir -p $O; export TMPDIR=/tmp
rm -rf $O/prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/$O/prof_c2" -o run \
  -- python3 "$R/bench.py" --steps 20 --warmup 3 --cpu-sample 0 --cli-sample 0 > $O/prof_c2.log 2>&1 || { tail -5 $O/prof_c2.log; exit 1; }
python3 tools/kstats.py $O/prof_c2/run_kernel_stats.csv | head -14
PROFDIR=r06 bash tools/pmc_traffic.sh 2 r06f || exit 1
BENCH_ARGS="--steps 2 --warmup 1 --cpu-sample 0 --cli-sample 0 --e2e-chunk -1 --parity-windows 0" \
PASSES="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
  bash tools/pmc_sq.sh > /dev/null || exit 1
cp gpurun_out/pmc/summary.txt $O/r06f_pmc_sq_summary_c2.txt
timeout -k 10 600 python bench.py > $O/bench_c2_full.json 2> $O/bench_c2_full.err || { tail -5 $O/bench_c2_full.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c2_full.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c2', d['value'], d['ms_per_step'], r['ms_per_launch'], r['frac'], r['traffic'], r['traffic_ratio'], d['parity_sampled'], d['window_stats'])"
# LDS counters of the step's kernels (ZnS: LDS-array cycles and bank-conflict cycles), last so a
# failure here loses nothing above
BENCH_ARGS="--steps 2 --warmup 1 --cpu-sample 0 --cli-sample 0 --e2e-chunk -1 --parity-windows 0" \
PASSES="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS" \
  bash tools/pmc_sq.sh > /dev/null || exit 1
cp gpurun_out/pmc/summary.txt $O/r06f_pmc_lds_summary_c2.txt
