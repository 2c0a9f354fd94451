#!/bin/bash
# Overflow-kernel check: wide-sample / scale parity tests, the configs[4] bench line, then an
# A/B of library variants (tools/ab.sh) at configs[2].  Stops at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wide_samples.py tests/test_gpu_scale.py -x -q -m gpu -p no:cacheprovider \
    --timeout 300 --timeout-method thread -k "${K_EXPR:-}" > gpurun_out/pytest_ovf.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_ovf.log; tail -3 gpurun_out/pytest_ovf.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --config 4 --steps 2 --warmup 1 --cpu-sample 0 > gpurun_out/c4_ovf.json 2> gpurun_out/c4_ovf.err || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/c4_ovf.json')); print('c4', d['value'], d['ms_per_step'], d['call_stage'])"
if [ -n "${AB:-}" ]; then bash tools/ab.sh $AB || exit $?; fi
exit 0
