#!/bin/bash
# Measurement build of libdlamd.so with extra -D flags on mix_tile.hip only (A/B builds,
# -D knobs), linked with the default build's other objects:
#   scripts/build_tile_variant.sh <name> -DFOO=1 ...  ->  scripts/_build/<name>/libdlamd.so
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
OBJ=distributed-learning_amd/_lib/obj
OUT=scripts/_build/$NAME
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall \
    -Wno-unused-result "$@" -c distributed-learning_amd/csrc/mix_tile.hip -o $OUT/mix_tile.o
OTHERS=$(ls $OBJ/*.o | grep -v "/mix_tile\.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libdlamd.so $OUT/mix_tile.o $OTHERS
echo "built $OUT/libdlamd.so ($*)"
