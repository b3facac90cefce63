#!/bin/bash
# Round-4 session L: plain (MALL-allocating) stores for the last output rows of a halo round,
# so the next round's pack and the split scheme's boundary window read them on-die
# (DLAMD_PLAIN_TAIL = rows, a measurement knob of that build, since removed): one rank of 8 and 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11l; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -1 $O/$name.log | cut -c1-200;
         if [ $rc -ne 0 ]; then exit $rc; fi; }
for rep in 1 2; do
  for k in 0 96 176 256; do
    DLAMD_PLAIN_TAIL=$k step c4rank_t${k}_$rep 200 python bench.py --workload c4-rank --steps 50 --warmup 5
  done
done
for k in 0 128 256; do
  DLAMD_PLAIN_TAIL=$k step c4rank4_t$k 200 python bench.py --workload c4-rank --rank-of 4 --steps 30 --warmup 3
done
