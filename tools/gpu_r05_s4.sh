#!/bin/bash
# r05 step 4: process-exit cost by allocation size, CLI probe (push internals), then SQ counters
# and a kernel trace of a short configs[2] bench (generator + scan instruction mix).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/r05s4; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python3 tools/teardown_probe.py > $O/teardown.jsonl 2>&1 || { tail -5 $O/teardown.jsonl; exit 1; }
tail -24 $O/teardown.jsonl | cut -c1-200
timeout -k 10 600 python -u tools/cli_probe.py > $O/cli_probe.json 2> $O/cli_probe.err || exit 1
bash tools/gpu_pmc_sq.sh > $O/pmc.log 2>&1; rc=$?; tail -5 $O/pmc.log; cp -r gpurun_out/pmc/summary.txt $O/ 2>/dev/null
exit $rc
