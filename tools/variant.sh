#!/bin/bash
# Build an experimental variant of libpopbam_gpu.so with extra defines:
#   bash tools/variant.sh NAME -DFOO=1 ...   ->  popbam_amd/variants/NAME/libpopbam_gpu.so
# (git-ignored; load it with POPBAM_GPU_LIB=... for A/B timing on the GPU box).  Every variant is
# built with -DPBG_EXPERIMENT=1 (the experiment switches compile only then; pbg_build_info() of
# the variant says "experiment").
# SRC=<dir> builds from another source tree (e.g. a `git archive` of an earlier commit).
set -e
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=$R/popbam_amd/variants/$NAME
mkdir -p "$OUT/build"
F="-O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-function -DPBG_EXPERIMENT=1 $*"
C=${SRC:-$R/popbam_amd/csrc}
H=/opt/rocm/bin/hipcc
$H $F --offload-arch=gfx950 -c -o $OUT/build/call.o $C/call_kernel.hip &
$H $F --offload-arch=gfx950 -c -o $OUT/build/stats.o $C/stats_kernel.hip &
$H $F -x hip --offload-arch=gfx950 -c -o $OUT/build/api.o $C/api.cpp &
$H $F -x hip --offload-arch=gfx950 -c -o $OUT/build/stream.o $C/stream.cpp &
$H $F -c -o $OUT/build/tables.o $C/host_tables.cpp &
$H $F -c -o $OUT/build/format.o $C/format.cpp &
wait || exit 1
$H -shared -fPIC --offload-arch=gfx950 -o $OUT/libpopbam_gpu.so $OUT/build/*.o
rm -rf "$OUT/build"
echo "$OUT/libpopbam_gpu.so"
