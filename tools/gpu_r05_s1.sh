#!/bin/bash
# r05 step 1: the native command line on the GPU: every golden case as a fresh bin/popbam
# process, the rank and small-piece variants, then the CLI probe on the 5 Mbp BAM.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05s1; mkdir -p $O; export TMPDIR=/tmp
nproc > $O/host.txt; python -c "import os; print(len(os.sched_getaffinity(0)))" >> $O/host.txt
cat /sys/fs/cgroup/cpu.max >> $O/host.txt 2>&1; env | grep -E "OMP|MAX_JOBS" >> $O/host.txt
timeout -k 10 900 python -u -m pytest tests/test_native_cli.py tests/test_feeder.py -x -q -m gpu -p no:cacheprovider \
    --timeout 120 --timeout-method thread > $O/pytest_native.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_native.log; tail -3 $O/pytest_native.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/cli_probe.py > $O/cli_probe.json 2> $O/cli_probe.err
rc=$?; tail -c 3000 $O/cli_probe.json; exit $rc
