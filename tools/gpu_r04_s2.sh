#!/bin/bash
# r04 session 2: the full -m gpu suite + smoke (streamed pbg_run, feeder key stream, CLI), then the
# configs[2] bench line (C-ABI end_to_end, the CLI on a 5 Mbp BAM beside POPBAM on all cores).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/s2; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 \
    --timeout-method thread > gpurun_out/s2/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/s2/pytest_gpu.log; tail -3 gpurun_out/s2/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/s2/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/s2/bench.json 2> gpurun_out/s2/bench.err || exit $?
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/s2/bench.json"))
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d.get("parity_sampled"))
print(json.dumps(d.get("end_to_end"))[:800])
print(json.dumps(d.get("cli"))[:3000])
PY
exit 0
