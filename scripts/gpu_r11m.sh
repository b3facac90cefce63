#!/bin/bash
# Round-4 session M: the c3 and c4 lines citing their round-4 profiles by kernel instance.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11m; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -1 $O/$name.log | cut -c1-200;
         if [ $rc -ne 0 ]; then exit $rc; fi; }
step c3 300 python bench.py --workload c3 --steps 50 --warmup 5 --no-cpu
step c4 300 python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu
