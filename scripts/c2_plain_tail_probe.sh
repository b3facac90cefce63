#!/bin/bash
# Measurement of a since-removed build knob (DLAMD_PLAIN_TAIL: the last k output rows of a round stored plainly); results in profiles/r11/c2_plain_tail/ and DESIGN.md section 4 "Stores".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c2tail; mkdir -p $O
for rep in 1 2; do
  for k in 0 128 256 512 1024; do
    DLAMD_PLAIN_TAIL=$k timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu > $O/t${k}_$rep.log 2>&1 || exit $?
    echo "t$k rep $rep: $(grep -o '"value": [0-9.]*' $O/t${k}_$rep.log | head -1)"
  done
done
