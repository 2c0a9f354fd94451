#!/bin/bash
# Generator A/B: tools/synth_bench.py --allow-variant (configs[3] chunk shape by default) under a kernel trace for
# the product library and each variant named (popbam_amd/variants/NAME).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/synth_ab; mkdir -p $O; export TMPDIR=/tmp
ARGS=${SYNTH_ARGS:---samples 24 --sites 33554432 --reps 5}
for v in product "$@"; do
  L=""; [ "$v" != product ] && L=$R/popbam_amd/variants/$v/libpopbam_gpu.so
  rm -rf $O/$v
  POPBAM_GPU_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/$O/$v" -o run \
    -- python3 "$R/tools/synth_bench.py" $ARGS > $O/$v.log 2>&1 || { tail -3 $O/$v.log; exit 1; }
  echo "== $v $(grep ms_per_generation $O/$v.log)"
  f=$(find $O/$v -name "*kernel_stats.csv" | head -1); grep -E "synth_" "$f" | cut -d, -f1-4
done
