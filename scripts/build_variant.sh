#!/bin/bash
# Measurement build of libdlamd.so with extra -D flags on ONE source file (A/B builds), linked
# with the default build's other objects:
#   scripts/build_variant.sh <source.hip> <name> -DFOO=1 ...  ->  scripts/_build/<name>/libdlamd.so
set -e
cd "$(dirname "$0")/.."
SRC=$1; NAME=$2; shift 2
OBJ=distributed-learning_amd/_lib/obj
OUT=scripts/_build/$NAME
BASE=$(basename $SRC .hip)
mkdir -p $OUT
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall \
    -Wno-unused-result "$@" -c distributed-learning_amd/csrc/$SRC -o $OUT/$BASE.o
OTHERS=$(ls $OBJ/*.o | grep -v "/$BASE\.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUT/libdlamd.so $OUT/$BASE.o $OTHERS
echo "built $OUT/libdlamd.so ($*)"
