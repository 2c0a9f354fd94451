#!/bin/bash
# r04 session 5: FETCH_SIZE / WRITE_SIZE calibration (tools/ubench/fetch_calib, one counter per
# pass); window-statistics parity after the per-site nucdiv sums / restricted calc_nhaps bits /
# register merge; the default bench line; configs[4] with the window stage timed alone.
# Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/s5; mkdir -p $O; export TMPDIR=/tmp
rm -rf $O/calib
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$R/$O/calib/p1" -o run \
  -- "$R/tools/ubench/fetch_calib" > $O/calib_known.json 2> $O/calib_p1.err || { tail -5 $O/calib_p1.err; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$R/$O/calib/p2" -o run \
  -- "$R/tools/ubench/fetch_calib" > /dev/null 2> $O/calib_p2.err || { tail -5 $O/calib_p2.err; exit 1; }
python3 tools/pmc_calib.py $O/calib $O/calib_known.json > $O/calib.json; cat $O/calib.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -x -q -m gpu -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "window_stats or u16_wrap or sfs_bins" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/s5/bench.json"))
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d.get("parity_sampled"), d.get("window_stats"))
print(json.dumps(d.get("end_to_end"))[:500])
print(json.dumps(d.get("cli"))[:2500])
PY
timeout -k 10 600 python bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c4.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_sampled'), d.get('window_stage'))"
exit 0
