#!/bin/bash
# A focused GPU session: selected parity tests (TESTS, K_EXPR), the configs[2] bench line, and a
# rocprofv3 kernel trace of it (PROF=1).  Every GPU step has its own time limit; the script stops
# at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest $TESTS -x -q -m gpu -p no:cacheprovider --timeout 200 \
      --timeout-method thread -k "${K_EXPR:-}" > gpurun_out/pytest_quick.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_quick.log; tail -3 gpurun_out/pytest_quick.log
  [ $rc -ne 0 ] && exit $rc
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python bench.py --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || exit $?
  cat gpurun_out/bench_q.json
fi
if [ "${PROF:-1}" = "1" ]; then
  rm -rf gpurun_out/prof_q
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/gpurun_out/prof_q" -o run \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-sample 0 ${BENCH_ARGS:-} > gpurun_out/prof_q.log 2>&1 || exit $?
  python3 tools/kstats.py gpurun_out/prof_q/run_kernel_stats.csv
fi
exit 0
