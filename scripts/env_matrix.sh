#!/bin/bash
# Same-box interleaved runs of one bench line under several environment settings:
#   scripts/env_matrix.sh <out_dir> <reps> "<name>:<VAR=val,VAR=val or ->" ... -- <bench args...>
# Each run under its own time limit; trouble ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$1; REPS=$2; shift 2
V=()
while [ "$1" != "--" ]; do V+=("$1"); shift; done
shift
mkdir -p $O
for i in $(seq 1 $REPS); do
    for nv in "${V[@]}"; do
        n=${nv%%:*}; e=${nv#*:}
        [ "$e" = "-" ] && e=
        env ${e//,/ } timeout -k 10 300 python bench.py "$@" > $O/${n}_$i.log 2>&1
        rc=$?
        echo "$n $i rc=$rc $(grep -o '"value": [0-9.]*' $O/${n}_$i.log | head -1) $(grep -o '"frac_of_measured_triad": [0-9.]*' $O/${n}_$i.log | head -1)"
        if [ $rc -ne 0 ]; then tail -5 $O/${n}_$i.log; exit $rc; fi
    done
done
