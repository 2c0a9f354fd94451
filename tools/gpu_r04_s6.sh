#!/bin/bash
# r04 session 6: kernel traces of library variants (ZnS adder priority; slow kernel without its
# network / without its fold -- timing experiments) at configs[2].  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=${O:-gpurun_out/s6}; mkdir -p $O; export TMPDIR=/tmp
for v in ${VARIANTS:-base zprio3 nonet nofold}; do
  rm -rf $O/prof_$v
  export POPBAM_GPU_LIB=$R/popbam_amd/variants/$v/libpopbam_gpu.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/$O/prof_$v" -o run \
    -- python3 "$R/bench.py" --steps 5 --warmup 1 --cpu-sample 0 --parity-windows 0 --e2e-chunk -1 --cli-sample 0 \
    > $O/prof_$v.json 2> $O/prof_$v.err || { echo "variant $v failed"; tail -5 $O/prof_$v.err; exit 1; }
  echo "== $v $(python3 -c "import json; d=json.load(open('$O/prof_$v.json')); print(d['value'], d['ms_per_step'])")"
  python3 tools/kstats.py $O/prof_$v/run_kernel_stats.csv | grep -E "call_|window_" 
done
exit 0
