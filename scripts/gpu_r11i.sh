#!/bin/bash
# Round-4 session I: hidden forward phases double-buffered through the output activation
# (mlp_fused_kernel): c3 tests and smoke, then a same-box A/B of the c3 step against the previous
# kernel (scripts/bin/libdlamd_base.so, DLAMD_LIB).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11i; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -2 $O/$name.log | cut -c1-300;
         if [ $rc -ne 0 ] && ! { [ "${SOFT:-0}" = 1 ] && [ $rc -eq 1 ]; }; then exit $rc; fi; }
SOFT=1 step tests 600 python -u -m pytest tests/test_configs_gpu.py tests/test_batched_ann_gpu.py -v -m gpu --timeout 300 --timeout-method thread
if grep -q -i -E "hipError|illegal|memory access fault|HSA_STATUS_ERROR|Aborted" $O/tests.log; then
    echo "device error in the tests: stopping"; exit 4; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
for i in 1 2; do
  DLAMD_LIB=scripts/bin/libdlamd_base.so step c3_base$i 240 python bench.py --workload c3 --steps 100 --warmup 10 --no-cpu
  step c3_new$i 240 python bench.py --workload c3 --steps 100 --warmup 10 --no-cpu
done
