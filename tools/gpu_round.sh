#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace + HBM counters.
# Stops at the first fault / timeout (exit codes > 1 from pytest, any failure afterwards).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -q -m gpu -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit $?
if [ "${PROFILE:-0}" = "1" ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/gpurun_out/prof_trace" -o run \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof_trace.log 2>&1 || exit $?
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$R/gpurun_out/prof_fetch" -o run \
    -- python3 "$R/bench.py" --steps 2 --warmup 0 --cpu-sample 0 > gpurun_out/prof_fetch.log 2>&1 || exit $?
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$R/gpurun_out/prof_write" -o run \
    -- python3 "$R/bench.py" --steps 2 --warmup 0 --cpu-sample 0 > gpurun_out/prof_write.log 2>&1 || exit $?
fi
exit 0
