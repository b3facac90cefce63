#!/bin/bash
# Round-4 session F: three-pass halo rounds at C = 1 (one rank of 2), non-temporal pack stores:
# the full-size c4 halo tests at 8 / 4 / 2 ranks, then one rank of 8 / 4 / 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11f; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -2 $O/$name.log | cut -c1-300;
         if [ $rc -ne 0 ] && ! { [ "${SOFT:-0}" = 1 ] && [ $rc -eq 1 ]; }; then exit $rc; fi; }
SOFT=1 step tests 600 python -u -m pytest tests/test_sharding_gpu.py -v -m gpu --timeout 300 --timeout-method thread
if grep -q -i -E "hipError|illegal|memory access fault|HSA_STATUS_ERROR|Aborted" $O/tests.log; then
    echo "device error in the tests: stopping"; exit 4; fi
step c4rank 240 python bench.py --workload c4-rank --steps 50 --warmup 5
step c4rank_of4 240 python bench.py --workload c4-rank --rank-of 4 --steps 30 --warmup 3
step c4rank_of2 240 python bench.py --workload c4-rank --rank-of 2 --steps 20 --warmup 3
