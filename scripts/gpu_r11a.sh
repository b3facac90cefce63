#!/bin/bash
# Round-4 session A: halo-on-tiled tests, the one-rank-of-8 c4 bench, the c2 headline and its
# rocprofv3 trace + PMC passes.  Each GPU step has its own limit; trouble ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11a; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -4 $O/$name.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 900 python -u -m pytest tests/test_sharding_gpu.py tests/test_mix_gpu.py tests/test_mix_ragged_gpu.py tests/test_abi.py -x -v -m gpu --timeout 300 --timeout-method thread
step c4rank 300 python bench.py --workload c4-rank --steps 50 --warmup 5
step c2 400 python bench.py --steps 20 --warmup 3
step c4ba 300 python bench.py --workload c4-ba --steps 30 --warmup 3 --no-cpu
DLAMD_HUB_ROWS=0 step c4ba_nohub 300 python bench.py --workload c4-ba --steps 30 --warmup 3 --no-cpu
bash scripts/gpu_profile.sh r11a/c2prof --steps 20 --warmup 3 --no-cpu --no-fdla-probe
