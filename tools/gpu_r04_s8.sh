#!/bin/bash
# r04 session 8: kernel traces of library variants at configs[2] (previous head, current tree,
# ZnS chain order, ZnS timing experiments, scan occupancy experiments).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/s8; mkdir -p $O
O=$O VARIANTS="${VARIANTS:-base cur zsort zexp1 zexp2 occ6 occ4}" bash tools/gpu_r04_s6.sh 2>&1 | tail -60
