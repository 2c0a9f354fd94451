set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/ab3
for v in head main head main; do
  if [ $v = main ]; then L=""; else L=$R/popbam_amd/variants/$v/libpopbam_gpu.so; fi
  POPBAM_GPU_LIB=$L timeout -k 10 200 python3 bench.py --config 3 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/ab3/$v.json 2> gpurun_out/ab3/$v.err || { echo "$v failed"; tail -2 gpurun_out/ab3/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab3/$v.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['roofline']['frac'], d['call_stage'])"
done
timeout -k 10 300 python3 bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/ab3/c4.json 2> gpurun_out/ab3/c4.err || { echo "c4 failed"; tail -2 gpurun_out/ab3/c4.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/ab3/c4.json')); print('c4', d['value'], d['ms_per_step'], d['roofline']['ms_per_launch'], d['call_stage'])"
