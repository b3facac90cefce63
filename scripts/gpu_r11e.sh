#!/bin/bash
# Round-4 session E: the halo pack probe, and one rank of the 2- and 4-GPU c4 partitions.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11e; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -2 $O/$name.log | cut -c1-300;
         if [ $rc -ne 0 ]; then exit $rc; fi; }
step pack_probe 120 scripts/bin/pack_probe
step c4rank_of4 240 python bench.py --workload c4-rank --rank-of 4 --steps 30 --warmup 3
step c4rank_of2 240 python bench.py --workload c4-rank --rank-of 2 --steps 20 --warmup 3
