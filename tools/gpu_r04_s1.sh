#!/bin/bash
# r04 session 1: new / changed GPU tests + smoke, the PBG_BOUNDS run, the configs[2] bench line
# (sampled oracle parity), a kernel trace, and the HBM counters of this tree.  Stops at the
# first failure; every GPU step under its own time limit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/s1; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py tests/test_genome.py -x -q -m gpu -p no:cacheprovider \
  --timeout 200 --timeout-method thread -k "inconsistent or serial or host_stream" > gpurun_out/s1/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/s1/pytest.log; tail -3 gpurun_out/s1/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s1/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/s1/smoke.log
bash tools/gpu_bounds.sh || exit $?
timeout -k 10 400 python bench.py > gpurun_out/s1/bench.json 2> gpurun_out/s1/bench.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/s1/bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_sampled'), d['parity_sample']['seconds'])"
rm -rf gpurun_out/s1/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/gpurun_out/s1/prof" -o run \
  -- python3 "$R/bench.py" --steps 5 --warmup 1 --cpu-sample 0 --parity-windows 0 > gpurun_out/s1/prof.log 2>&1 || exit $?
python3 tools/kstats.py gpurun_out/s1/prof/run_kernel_stats.csv
bash tools/pmc_traffic.sh 2 r04s1 || exit $?
exit 0
