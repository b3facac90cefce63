#!/bin/bash
# Round-4 session G: per-peer contiguous send runs (boundary rows grouped by peer, halo blocks
# in the sender's order): the sharding GPU tests, one rank of 8 / 4 / 2, and the layer-1 probe
# with MALL-flushed (cold) timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11g; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -2 $O/$name.log | cut -c1-300;
         if [ $rc -ne 0 ] && ! { [ "${SOFT:-0}" = 1 ] && [ $rc -eq 1 ]; }; then exit $rc; fi; }
SOFT=1 step tests 600 python -u -m pytest tests/test_sharding_gpu.py -v -m gpu --timeout 300 --timeout-method thread
if grep -q -i -E "hipError|illegal|memory access fault|HSA_STATUS_ERROR|Aborted" $O/tests.log; then
    echo "device error in the tests: stopping"; exit 4; fi
step c4rank 240 python bench.py --workload c4-rank --steps 50 --warmup 5
step c4rank_of4 240 python bench.py --workload c4-rank --rank-of 4 --steps 30 --warmup 3
step c4rank_of2 240 python bench.py --workload c4-rank --rank-of 2 --steps 20 --warmup 3
step l1_probe 180 scripts/bin/l1_x6_dma_probe
