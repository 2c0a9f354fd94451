#!/bin/bash
# r05 step 2: INTEGRATION.md's binding on the GPU, the native command line again (walk during
# GPU init, table file, fast exit), the Python CLI tests, then the CLI probe.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05s2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_integration.py tests/test_native_cli.py tests/test_cli.py -x -q -m gpu \
    -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u tools/cli_probe.py > $O/cli_probe.json 2> $O/cli_probe.err
rc=$?; tail -c 1500 $O/cli_probe.json; exit $rc
