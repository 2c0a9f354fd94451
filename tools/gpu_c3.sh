#!/bin/bash
# configs[3] (3 Gbp x 24 samples, streamed) on one GPU: the bench line with POPBAM's own CPU
# baseline, a rocprofv3 kernel trace of one pass, and FETCH_SIZE / WRITE_SIZE passes (one
# counter set per process, each under its own kill timeout).  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/c3; export TMPDIR=/tmp
timeout -k 10 900 python bench.py --config 3 --steps 2 --warmup 1 ${BENCH3_ARGS:-} > gpurun_out/c3/bench.json \
    2> gpurun_out/c3/bench.err || exit $?
cat gpurun_out/c3/bench.json
rm -rf gpurun_out/c3/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/gpurun_out/c3/prof" -o run \
  -- python3 "$R/bench.py" --config 3 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/c3/prof.log 2>&1 || exit $?
python3 tools/kstats.py gpurun_out/c3/prof/run_kernel_stats.csv
bash tools/gpu_c3_pmc.sh
