set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base skipz skipzs skipzsn; do
  rm -rf gpurun_out/prof_v
  POPBAM_GPU_LIB=$R/popbam_amd/variants/$v/libpopbam_gpu.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$R/gpurun_out/prof_v" -o run \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-sample 0 > gpurun_out/prof_v.log 2>&1 || exit 1
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_v/run_kernel_stats.csv')):
    if r['Name'].startswith('window'): print('$v', r['Name'][:28], round(float(r['AverageNs'])/1e3, 1), 'us')
"
done
