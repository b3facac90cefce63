#!/bin/bash
# c3 resident layouts interleaved on one box: rows (default) against the column-tiled layout at
# tile widths 64 (the planner's), 32, 16 and 8 (784 = 49 x 16: W1's rows start on a 16-column
# tile boundary at T <= 16).  Each run under its own time limit; trouble ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-r14/c3_layout}; REPS=${2:-2}
mkdir -p $O
for i in $(seq 1 $REPS); do
    for v in rows t64 t32 t16 t8; do
        case $v in
            rows) a="--c3-layout rows";;
            t*) a="--c3-layout tiled --c3-tile-cols ${v#t}";;
        esac
        timeout -k 10 300 python bench.py --workload c3 --no-cpu $a > $O/${v}_$i.log 2>&1
        rc=$?
        echo "$v $i rc=$rc $(grep -o '"value": [0-9.]*' $O/${v}_$i.log | head -1) $(grep -o '"launch_ms": [0-9.]*' $O/${v}_$i.log | head -2 | tr '\n' ' ')"
        if [ $rc -ne 0 ]; then tail -5 $O/${v}_$i.log; exit $rc; fi
    done
done
