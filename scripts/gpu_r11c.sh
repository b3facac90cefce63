#!/bin/bash
# Round-4 session C: the three-pass tiled halo kernel, boundary-last packs and 256 hub rows:
# tests, the c4-rank and c4-ba (three irregular graphs) A/B, and the c4-rank profile.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11c; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -2 $O/$name.log | cut -c1-300;
         if [ $rc -ne 0 ] && ! { [ "${SOFT:-0}" = 1 ] && [ $rc -eq 1 ]; }; then exit $rc; fi; }
SOFT=1 step tests 600 python -u -m pytest tests/test_sharding_gpu.py tests/test_mix_ragged_gpu.py tests/test_mixer_gpu.py -v -m gpu --timeout 300 --timeout-method thread
if grep -q -i -E "hipError|illegal|memory access fault|HSA_STATUS_ERROR|Aborted" $O/tests.log; then
    echo "device error in the tests: stopping"; exit 4; fi
step c4rank 240 python bench.py --workload c4-rank --steps 50 --warmup 5
DLAMD_WG_PER_CU=1 step c4rank_wg1 240 python bench.py --workload c4-rank --steps 50 --warmup 5
for g in ba2 ba1 deg; do
  step c4ba_$g 240 python bench.py --workload c4-ba --irregular $g --steps 30 --warmup 3 --no-cpu
  DLAMD_HUB_ROWS=0 step c4ba_${g}_hub0 240 python bench.py --workload c4-ba --irregular $g --steps 30 --warmup 3 --no-cpu
done
DLAMD_HUB_ROWS=128 step c4ba_ba2_hub128 240 python bench.py --workload c4-ba --steps 30 --warmup 3 --no-cpu
bash scripts/gpu_profile.sh r11c/c4rank --workload c4-rank --steps 20 --warmup 3 || exit $?
