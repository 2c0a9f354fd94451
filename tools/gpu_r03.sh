#!/bin/bash
# Round-3 GPU session: the -m gpu suite (optional), smoke, the configs[2] bench line, the configs[3]
# bench line with POPBAM's own CPU baseline, and a rocprofv3 kernel trace of each.
# Every GPU step has its own time limit; the script stops at the first failure.
#   SKIP_TESTS=1   skip the pytest/smoke step      K_EXPR   pytest -k filter
#   C3=0           skip configs[3]                 PROF=0   skip the kernel traces
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 \
      --timeout-method thread -k "${K_EXPR:-}" > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
  tail -1 gpurun_out/smoke.log
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || exit $?
cat gpurun_out/bench_c2.json
if [ "${C3:-1}" = "1" ]; then
  timeout -k 10 900 python bench.py --config 3 --steps 2 --warmup 1 ${BENCH3_ARGS:-} > gpurun_out/bench_c3.json \
      2> gpurun_out/bench_c3.err || exit $?
  cat gpurun_out/bench_c3.json
fi
if [ "${PROF:-1}" = "1" ]; then
  rm -rf gpurun_out/prof_c2 gpurun_out/prof_c3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/gpurun_out/prof_c2" -o run \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof_c2.log 2>&1 || exit $?
  if [ "${C3:-1}" = "1" ]; then
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/gpurun_out/prof_c3" -o run \
      -- python3 "$R/bench.py" --config 3 --steps 1 --warmup 1 --cpu-sample 0 > gpurun_out/prof_c3.log 2>&1 || exit $?
  fi
  python3 tools/kstats.py gpurun_out/prof_c2/run_kernel_stats.csv
  [ -f gpurun_out/prof_c3/run_kernel_stats.csv ] && python3 tools/kstats.py gpurun_out/prof_c3/run_kernel_stats.csv
fi
exit 0
