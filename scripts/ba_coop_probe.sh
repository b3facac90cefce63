#!/bin/bash
# path 5 with wave 0's long-row product area: parity tests, then c4-ba against the previous build
# (scripts/_build/base) and with the area off (DLAMD_COOP=0)
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/bacoop; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_mix_ragged_gpu.py tests/test_plan_cpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
r() { n=$1; shift; timeout -k 10 200 "$@" > $O/$n.log 2>&1 || exit $?; python -c "
import json
for l in open('$O/$n.log'):
    if l.startswith('{'): d=json.loads(l); print('$n', round(d['value'],1), round(d['roofline']['frac'],3), d['config'].get('plan',{}).get('lds_bytes'))"; }
B="python bench.py --workload c4-ba --steps 30 --warmup 3 --no-cpu"
for g in ba2 ba1 deg; do
  r base_$g env DLAMD_LIB=scripts/_build/base/libdlamd.so $B --irregular $g
  r coop_$g $B --irregular $g
  r off_$g env DLAMD_COOP=0 $B --irregular $g
done
