#!/bin/bash
# r04 session 3: window-statistics parity after the kernel rework (pair sums per population
# pair, bit matrix for calc_nhaps, host-chosen LDS slice, XCD-aware window order), the configs[2]
# bench line, an A/B of the scan's mid-block list pass (PBG_SCAN_LISTK) with scan FETCH_SIZE, and
# configs[4] (bench line + kernel trace).  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/s3; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_golden.py tests/test_wide_samples.py tests/test_genome.py \
  -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "window_stats or u16_wrap or sfs_bins or golden or wide or overlapping or chunked or serial or stream" > gpurun_out/s3/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/s3/pytest.log; tail -3 gpurun_out/s3/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/s3/bench.json 2> gpurun_out/s3/bench.err || { tail -5 gpurun_out/s3/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/s3/bench.json"))
print(d["value"], d["ms_per_step"], d["roofline"]["frac"], d.get("parity_sampled"), d["window_stats"])
print(json.dumps(d.get("end_to_end"))[:700])
print(json.dumps(d.get("cli"))[:3500])
PY
BENCH_ARGS="--sites 50000000 --steps 5 --warmup 1 --cpu-sample 0 --parity-windows 0" bash tools/ab.sh base listk1 listk2 listk3 || exit $?
for v in base listk1 listk2 listk3; do
  POPBAM_GPU_LIB=$R/popbam_amd/variants/$v/libpopbam_gpu.so timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -T --output-format csv \
    -d "$R/gpurun_out/s3/pmc_$v" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --cpu-sample 0 --parity-windows 0 \
    --e2e-chunk -1 --cli-sample 0 > gpurun_out/s3/pmc_$v.log 2>&1 || { echo "pmc $v failed"; exit 1; }
  python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
acc = {}
for f in glob.glob(f"gpurun_out/s3/pmc_{v}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = (r.get("Kernel_Name") or "?").split("(")[0].split("<")[0].replace("void ", "").replace("pbg::", "")
        acc.setdefault(k, []).append(float(r.get("Counter_Value") or 0))
for k in ("call_scan_kernel", "call_slow_kernel"):
    if k in acc:
        print(v, k, "FETCH x2 GB per launch:", round(sum(acc[k]) / len(acc[k]) * 2 * 1024 / 1e9, 3))
PY
done
timeout -k 10 600 python bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/s3/bench_c4.json 2> gpurun_out/s3/bench_c4.err || { tail -5 gpurun_out/s3/bench_c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/s3/bench_c4.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_sampled'))"
rm -rf gpurun_out/s3/prof_c4
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/gpurun_out/s3/prof_c4" -o run \
  -- python3 "$R/bench.py" --config 4 --steps 1 --warmup 0 --cpu-sample 0 --parity-windows 0 > gpurun_out/s3/prof_c4.log 2>&1 || exit $?
python3 tools/kstats.py gpurun_out/s3/prof_c4/run_kernel_stats.csv
exit 0
