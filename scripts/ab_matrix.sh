#!/bin/bash
# Same-box interleaved A/B of several libdlamd.so builds on one bench line:
#   scripts/ab_matrix.sh <out_dir> <reps> "<name>=<lib or 'new'> ..." <bench args...>
# ('new' = the in-tree build).  Each run under its own time limit; trouble ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; REPS=$2; LIBS=$3; shift 3
mkdir -p $O
for i in $(seq 1 $REPS); do
    for nv in $LIBS; do
        n=${nv%%=*}; L=${nv#*=}
        [ "$L" = new ] && L=
        DLAMD_LIB=$L timeout -k 10 300 python bench.py "$@" > $O/${n}_$i.log 2>&1
        rc=$?
        echo "$n $i rc=$rc $(grep -o '"value": [0-9.]*' $O/${n}_$i.log | head -1)"
        if [ $rc -ne 0 ]; then tail -5 $O/${n}_$i.log; exit $rc; fi
    done
done
