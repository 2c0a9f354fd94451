#!/bin/bash
# r04 session 9: kernel traces base (previous head) vs cur, then the default bench line
# (parity_sampled + the full-size rows cross-check).  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/s9; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -x -q -m gpu -p no:cacheprovider --timeout 200 \
  --timeout-method thread -k "consensus_word" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
O=$O VARIANTS="base cur" bash tools/gpu_r04_s6.sh 2>&1 | tail -20
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/s9/bench.json"))
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["call_stage"], d.get("window_stats"))
print(d.get("parity_sampled"), d.get("rows_crosscheck"))
print(json.dumps(d.get("cli"))[-400:])
PY
