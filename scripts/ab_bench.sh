#!/bin/bash
# Same-box A/B of two builds of libdlamd.so on one bench line, alternating, each run under its
# own time limit: scripts/ab_bench.sh <out_dir> <base.so> <reps> <bench args...>
# (DLAMD_LIB selects the build; the in-tree one is "new").  Trouble (rc >= 2) ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; BASE=$2; REPS=$3; shift 3
mkdir -p $O
for i in $(seq 1 $REPS); do
    for v in base new; do
        if [ $v = base ]; then L=$BASE; else L=; fi
        DLAMD_LIB=$L timeout -k 10 300 python bench.py "$@" > $O/${v}_$i.log 2>&1
        rc=$?
        echo "$v $i rc=$rc $(grep -o '"value": [0-9.]*' $O/${v}_$i.log | head -1)"
        if [ $rc -ne 0 ]; then exit $rc; fi
    done
done
