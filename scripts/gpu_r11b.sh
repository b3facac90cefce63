#!/bin/bash
# Round-4 session B: the halo tests after the one-launch pack, the one-rank-of-8 c4 round's
# workgroup / tile-width variants, the hub-lane check on c4-ba, rocprofv3 trace + FETCH / WRITE
# passes of both, and the N = 2 gloo rehearsals of the multi-GPU lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11b; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -3 $O/$name.log | cut -c1-400;
         if [ $rc -ne 0 ] && ! { [ "${SOFT:-0}" = 1 ] && [ $rc -eq 1 ]; }; then exit $rc; fi; }
SOFT=1 step tests 600 python -u -m pytest tests/test_sharding_gpu.py tests/test_mix_trace_gpu.py tests/test_mix_ragged_gpu.py -v -m gpu --timeout 300 --timeout-method thread
if grep -q -i -E "hipError|illegal|memory access fault|HSA_STATUS_ERROR|Aborted" $O/tests.log; then
    echo "device error in the tests: stopping"; exit 4; fi
B="python bench.py --workload c4-rank --steps 50 --warmup 5"
step c4rank 240 $B
DLAMD_WG_PER_CU=1 step c4rank_wg1 240 $B
step c4rank_t8 240 $B --halo-tile-cols 8
step c4rank_t4 240 $B --halo-tile-cols 4
DLAMD_HUB_ROWS=256 step c4ba_hub256 240 python bench.py --workload c4-ba --steps 30 --warmup 3 --no-cpu
DLAMD_HUB_ROWS=0 step c4ba_hub0 240 python bench.py --workload c4-ba --steps 30 --warmup 3 --no-cpu
bash scripts/gpu_profile.sh r11b/c4rank --workload c4-rank --steps 20 --warmup 3 || exit $?
bash scripts/gpu_profile.sh r11b/c4ba --workload c4-ba --steps 20 --warmup 3 --no-cpu || exit $?
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step c4_gloo2 300 $R --master-port 29511 bench.py --gpus 2 --workload c4 --dist-backend gloo --steps 5 --warmup 1
