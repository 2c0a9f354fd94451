#!/bin/bash
# Full -m gpu suite + smoke, a rocprofv3 kernel trace of one configs[4] pass, then an optional
# A/B of library variants (AB="a b ..." via tools/ab.sh).  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
rm -rf gpurun_out/prof_c4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/gpurun_out/prof_c4" -o run \
  -- python3 "$R/bench.py" --config 4 --steps 1 --warmup 0 --cpu-sample 0 > gpurun_out/prof_c4.log 2>&1 || exit $?
python3 tools/kstats.py gpurun_out/prof_c4/run_kernel_stats.csv
if [ -n "${AB:-}" ]; then bash tools/ab.sh $AB || exit $?; fi
exit 0
