#!/bin/bash
# c3 bench per bgemm tile shape (DLAMD_BGEMM_SHAPE=<rows<=64>,<rows>64>), one JSON line each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for sh in 0,0 1,0 2,0 5,0 1,1 2,2 0,2 1,2; do
    echo "=== shape $sh"
    DLAMD_BGEMM_SHAPE=$sh timeout -k 10 200 python bench.py --workload c3 --steps 50 --warmup 5 --no-cpu > gpurun_out/c3_$sh.log 2>&1 || exit $?
    grep '^{' gpurun_out/c3_$sh.log | python -c "
import json,sys
r=json.loads(sys.stdin.read()); g=r['phases']['gradients']
print('$sh', round(r['ms_per_step'],4), 'grad_ms', round(g['launch_ms'],4), round(g['achieved'],1), 'TF')"
done
