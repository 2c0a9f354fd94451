#!/bin/bash
# r04 session 4: FETCH_SIZE / WRITE_SIZE calibration of the call kernels' access widths
# (tools/ubench/fetch_calib, one counter per pass), then the default bench line (CLI identity
# against POPBAM after the .fai fix).  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/s4; export TMPDIR=/tmp
rm -rf gpurun_out/s4/calib
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$R/gpurun_out/s4/calib/p1" -o run \
  -- "$R/tools/ubench/fetch_calib" > gpurun_out/s4/calib_known.json 2> gpurun_out/s4/calib_p1.err || { tail -5 gpurun_out/s4/calib_p1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$R/gpurun_out/s4/calib/p2" -o run \
  -- "$R/tools/ubench/fetch_calib" > /dev/null 2> gpurun_out/s4/calib_p2.err || { tail -5 gpurun_out/s4/calib_p2.err; exit 1; }
python3 tools/pmc_calib.py gpurun_out/s4/calib gpurun_out/s4/calib_known.json | tee gpurun_out/s4/calib.json
timeout -k 10 700 python bench.py > gpurun_out/s4/bench.json 2> gpurun_out/s4/bench.err || { tail -5 gpurun_out/s4/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/s4/bench.json"))
print(d["value"], d["ms_per_step"], d["roofline"], d.get("parity_sampled"))
print(json.dumps(d.get("end_to_end"))[:700])
print(json.dumps(d.get("cli"))[:3500])
PY
exit 0
