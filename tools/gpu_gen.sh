#!/bin/bash
# Generator check: parity tests of the synthetic pileup + genome pass, then a kernel trace of a
# configs[2] bench (generator kernels once) and a configs[3] bench line.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_genome.py -x -q -p no:cacheprovider --timeout 300 \
    --timeout-method thread -k "${K_EXPR:-generator or genome or chunked}" > gpurun_out/pytest_gen.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gen.log; tail -3 gpurun_out/pytest_gen.log
[ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/prof_gen
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/gpurun_out/prof_gen" -o run \
  -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof_gen.log 2>&1 || exit $?
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/prof_gen/run_kernel_stats.csv")):
    print(f"{r['Name'][:44]:44s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:8.4f}")
PY
timeout -k 10 400 python bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 ${BENCH3_ARGS:-} > gpurun_out/b_c3.log 2>&1 || exit $?
tail -c 2500 gpurun_out/b_c3.log
timeout -k 10 400 python bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 --overlap > gpurun_out/b_c3o.log 2>&1 || exit $?
tail -c 2500 gpurun_out/b_c3o.log
