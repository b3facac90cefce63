#!/bin/bash
# traced rows kernel at half the threads (DLAMD_TRACE_HALF=1): parity, then c2 traced pass speed
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/thalf; mkdir -p $O
DLAMD_TRACE_HALF=1 timeout -k 10 300 python -u -m pytest tests/test_mix_trace_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; echo "tests rc=$?"; tail -2 $O/tests.log
r() { n=$1; shift; timeout -k 10 200 "$@" > $O/$n.log 2>&1 || exit $?; python -c "
import json
for l in open('$O/$n.log'):
    if l.startswith('{'): d=json.loads(l); print('$n', round(d['value'],1))"; }
B="python bench.py --workload c2-gossip --trace --steps 10 --warmup 2 --no-cpu"
r base24 $B --rounds 24
r half24 env DLAMD_TRACE_HALF=1 $B --rounds 24
r half32 env DLAMD_TRACE_HALF=1 $B --rounds 32
r base24b $B --rounds 24
