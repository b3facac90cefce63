#!/bin/bash
# Same-box A/B: the loads' waits forced before the staging barrier (in-tree) against the previous
# build (DL_AB_NO_LOADS_DONE), on c2, c4, c4-rank and c3; then the tile-kernel GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r13/wait
L="new=new old=scripts/_build/oldwait/libdlamd.so"
bash scripts/ab_matrix.sh r13/wait/c2 3 "$L" --steps 50 --warmup 5 --no-cpu --no-fdla-probe || exit $?
bash scripts/ab_matrix.sh r13/wait/c4 2 "$L" --workload c4 --steps 20 --warmup 3 --no-cpu || exit $?
bash scripts/ab_matrix.sh r13/wait/c4rank 2 "$L" --workload c4-rank --steps 50 --warmup 5 --no-cpu || exit $?
bash scripts/ab_matrix.sh r13/wait/c3 2 "$L" --workload c3 --steps 50 --warmup 5 --no-cpu || exit $?
timeout -k 10 900 python -u -m pytest tests/test_mix_gpu.py tests/test_mix_ragged_gpu.py tests/test_sharding_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r13/wait/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r13/wait/tests.log; exit $rc
