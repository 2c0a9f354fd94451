#!/bin/bash
# r05 step 11: generator parity + timing (step 5), then configs[3] with the window stage.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; export TMPDIR=/tmp
bash tools/gpu_r05_s5.sh || exit 1
bash tools/gpu_r05_s10.sh || exit 1
