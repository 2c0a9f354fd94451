#!/bin/bash
# r04 session 7: call-path parity after the fold changes (batched info loads, bit-rank select)
# and the ZnS adder priority, then kernel traces of base (previous head) vs cur.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/s7; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_golden.py tests/test_wide_samples.py tests/test_genome.py \
  -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "window_stats or rows_only or call_kernel or fixture or stream or pipelined or wide or golden or chunked or overlapping or inconsistent or u16_wrap" > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-sample 0 --parity-windows 0 --e2e-chunk -1 \
  --cli-sample 0 > $O/bench_w2.json 2> $O/bench_w2.err || { tail -5 $O/bench_w2.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_w2.json')); print('w2 rehearsal (2 ranks, one GPU)', d['n_gpus'], d['value'], d['ms_per_step'])"

exit 0
