#!/bin/bash
# r04 session 17: configs[4] scan without the list pass's s_waitcnt(0) (nowait) vs cur, then the
# wide-sample parity tests under nowait
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/s17; mkdir -p $O; export TMPDIR=/tmp
for v in cur nowait cur nowait; do
  export POPBAM_GPU_LIB=$R/popbam_amd/variants/$v/libpopbam_gpu.so
  rm -rf $O/prof_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/$O/prof_$v" -o run \
    -- python3 "$R/bench.py" --config 4 --steps 1 --warmup 0 --cpu-sample 0 --parity-windows 0 \
    > $O/prof_$v.json 2> $O/prof_$v.err || { echo "variant $v failed"; tail -5 $O/prof_$v.err; exit 1; }
  echo "== $v $(python3 -c "import json; d=json.load(open('$O/prof_$v.json')); print(d['value'], d['ms_per_step'], d['roofline']['alone'])")"
  python3 tools/kstats.py $O/prof_$v/run_kernel_stats.csv | grep -E "call_scan"
done
export POPBAM_GPU_LIB=$R/popbam_amd/variants/nowait/libpopbam_gpu.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_wide_samples.py tests/test_gpu_golden.py -x -q -m gpu \
  -p no:cacheprovider --timeout 300 --timeout-method thread -k "rows_only or call_kernel or consensus_word or wide or golden or soft_masked" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log
