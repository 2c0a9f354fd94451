#!/bin/bash
# r04 final check 3: the GPU tests that drive the host feeder (CLI, golden fixtures through the
# command line) after the feeder changes, then the default bench line (CLI at 5 Mbp) and the
# configs[4] / configs[3] lines.  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/f3; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_cli.py tests/test_gpu_golden.py tests/test_wide_samples.py tests/test_feeder.py \
  -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/f3/bench.json"))
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d["roofline"]["traffic"], d.get("parity_sampled"), d.get("rows_crosscheck", {}).get("identical"))
c = d.get("cli") or {}
print({k: c.get(k) for k in ("Msites_per_s_in_process", "x_over_popbam_all_cores", "identical_to_reference", "feeder_threads")})
print(json.dumps(c.get("commands", {}).get("nucdiv", {}).get("phases")))
PY
timeout -k 10 600 python bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c4.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d.get('parity_sampled'), d.get('rows_crosscheck',{}).get('identical'), d.get('window_stage',{}).get('ms_per_pass'))"
timeout -k 10 600 python bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_c3.json')); print('c3', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_sampled'), d.get('rows_crosscheck',{}).get('identical'))"
