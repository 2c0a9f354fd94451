#!/bin/bash
# r04 session 16: configs[3] (24 samples) scan with info bytes in LDS (cur) vs in HBM with the
# 64-entry list settle (linf12: the wide path from 13 samples up)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/s16; mkdir -p $O; export TMPDIR=/tmp
for v in ${VARIANTS:-cur linf12 cur linf12}; do
  export POPBAM_GPU_LIB=$R/popbam_amd/variants/$v/libpopbam_gpu.so
  rm -rf $O/prof_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/$O/prof_$v" -o run \
    -- python3 "$R/bench.py" --config 3 --steps 1 --warmup 0 --cpu-sample 0 --parity-windows 0 \
    > $O/prof_$v.json 2> $O/prof_$v.err || { echo "variant $v failed"; tail -5 $O/prof_$v.err; exit 1; }
  echo "== $v $(python3 -c "import json; d=json.load(open('$O/prof_$v.json')); print(d['value'], d['ms_per_step'], d['roofline']['alone'])")"
  python3 tools/kstats.py $O/prof_$v/run_kernel_stats.csv | grep -E "call_"
done
