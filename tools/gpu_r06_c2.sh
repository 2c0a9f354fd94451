#!/bin/bash
# Round-6 configs[2] evidence on the final tree: a rocprofv3 kernel trace of the bench step
# (20 steps), the HBM counters (FETCH_SIZE / WRITE_SIZE passes -> profiles/pmc_traffic_c2.json)
# and the SQ instruction-mix / wave-state passes.  Every GPU step under its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r06; mkdir -p $O; export TMPDIR=/tmp
rm -rf $O/prof_c2
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/$O/prof_c2" -o run \
  -- python3 "$R/bench.py" --steps 20 --warmup 3 --cpu-sample 0 --cli-sample 0 > $O/prof_c2.log 2>&1 || { tail -5 $O/prof_c2.log; exit 1; }
python3 tools/kstats.py $O/prof_c2/run_kernel_stats.csv | head -14
PROFDIR=r06 bash tools/pmc_traffic.sh 2 r06 || exit 1
BENCH_ARGS="--steps 2 --warmup 1 --cpu-sample 0 --cli-sample 0 --e2e-chunk -1 --parity-windows 0" \
PASSES="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU;SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" \
  bash tools/pmc_sq.sh > /dev/null || exit 1
cp gpurun_out/pmc/summary.txt $O/r06_pmc_sq_summary_c2.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-sample 0 --cli-sample 0 --e2e-chunk -1 > $O/bench_c2_traffic.json 2> $O/bench_c2_traffic.err || exit 1
python3 -c "import json; d=json.load(open('$O/bench_c2_traffic.json')); r=d['roofline']; print('c2', d['value'], r['ms_per_launch'], r['frac'], r['traffic'], r['traffic_ratio'], r['traffic_split'])"
