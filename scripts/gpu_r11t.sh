#!/bin/bash
# Round-4 session T: split rounds whose boundary launch reads the boundary rows' stepped values
# from the send blocks (one [send | halo] buffer): sharding GPU tests, one rank of 8 / 4 / 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11t; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -1 $O/$name.log | cut -c1-200;
         if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 600 python -u -m pytest tests/test_sharding_gpu.py -q -m gpu --timeout 300 --timeout-method thread
step c4rank 240 python bench.py --workload c4-rank --steps 50 --warmup 5
step c4rank_of4 240 python bench.py --workload c4-rank --rank-of 4 --steps 30 --warmup 3
step c4rank_of2 240 python bench.py --workload c4-rank --rank-of 2 --steps 20 --warmup 3
