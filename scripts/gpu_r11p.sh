#!/bin/bash
# Round-4 session P: c3 row-major against column-tiled X / G (A/B pairs on one box).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11p; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; grep -o '"value": [0-9.]*' $O/$name.log | head -1;
         if [ $rc -ne 0 ]; then exit $rc; fi; }
for i in 1 2; do
  step rows$i 240 python bench.py --workload c3 --steps 100 --warmup 10 --no-cpu
  step tiled$i 240 python bench.py --workload c3 --steps 100 --warmup 10 --no-cpu --c3-layout tiled
done
