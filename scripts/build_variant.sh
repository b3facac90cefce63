#!/bin/bash
# Measurement builds of libdlamd.so with extra -D flags (kernel variants for A/B runs on one box:
# DLAMD_LIB=scripts/_build/<name>/libdlamd.so python bench.py ...).  Rebuilds the sources that
# read the flags (capi.hip, mix_tile.hip, mix_trace.hip, mix_multi.hip) and links them with the
# default build's other objects.   Usage: scripts/build_variant.sh <name> -DFOO=1 ...
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
SRC=distributed-learning_amd/csrc
OBJ=distributed-learning_amd/_lib/obj
OUT=scripts/_build/$NAME
mkdir -p $OUT
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-result"
VAR="capi mix_tile mix_trace mix_multi mlp_fused"
for f in $VAR; do /opt/rocm/bin/hipcc $FLAGS "$@" -c $SRC/$f.hip -o $OUT/$f.o & done
wait
OTHERS=$(ls $OBJ/*.o | grep -v -E "/(capi|mix_tile|mix_trace|mix_multi|mlp_fused)\.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libdlamd.so $OUT/*.o $OTHERS
echo "built $OUT/libdlamd.so ($*)"
