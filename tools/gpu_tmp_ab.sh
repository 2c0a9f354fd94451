export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
AB="pad7 pad6 exp6 exp6pad6" bash tools/gpu_bench_ab.sh
