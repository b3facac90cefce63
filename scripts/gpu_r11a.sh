#!/bin/bash
# Round-4 session A: halo-on-tiled tests, the one-rank-of-8 c4 bench, the c2 headline and its
# rocprofv3 trace + PMC passes.  Each GPU step has its own limit; trouble ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11a; mkdir -p $O
# (SOFT=1: a test failure, pytest's exit 1, does not stop the script; a fault, abort or timeout does)
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -4 $O/$name.log;
         if [ $rc -ne 0 ] && ! { [ "${SOFT:-0}" = 1 ] && [ $rc -eq 1 ]; }; then exit $rc; fi; }
SOFT=1 step tests 900 python -u -m pytest tests/test_sharding_gpu.py tests/test_mix_gpu.py tests/test_mix_ragged_gpu.py tests/test_mix_trace_gpu.py tests/test_batched_ann_gpu.py tests/test_abi.py -v -m gpu --timeout 300 --timeout-method thread
# a device fault surfacing as a Python exception (a failed test, exit 1) still ends the session
if grep -q -i -E "hipError|illegal|memory access fault|HSA_STATUS_ERROR|Aborted" $O/tests.log; then
    echo "device error in the tests: stopping"; exit 4; fi
step c4rank 300 python bench.py --workload c4-rank --steps 50 --warmup 5
step c2 400 python bench.py --steps 20 --warmup 3
step c4ba 300 python bench.py --workload c4-ba --steps 30 --warmup 3 --no-cpu
DLAMD_HUB_ROWS=0 step c4ba_nohub 300 python bench.py --workload c4-ba --steps 30 --warmup 3 --no-cpu
bash scripts/gpu_profile.sh r11a/c2prof --steps 20 --warmup 3 --no-cpu --no-fdla-probe
