#!/bin/bash
# c4-ba A/B of measurement builds: rounds/s and HBM fraction per variant, e.g. the tail caps of
# profiles/r10/ba_tail_cap (built in r10 with a -DMIX_TAIL_CAP measurement knob, since removed from
# the product source: those figures are recorded there; VARIANTS names other builds now)
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/bavar; mkdir -p $O
r() { n=$1; shift; timeout -k 10 200 "$@" > $O/$n.log 2>&1 || exit $?; python -c "
import json
for l in open('$O/$n.log'):
    if l.startswith('{'): d=json.loads(l); print('$n', round(d['value'],1), round(d['roofline']['frac'],3))"; }
B="python bench.py --workload c4-ba --steps 30 --warmup 3 --no-cpu"
for v in ${VARIANTS:-base cap32 cap0}; do
  L=""; [ $v != base ] && L=scripts/_build/$v/libdlamd.so
  for g in ${GRAPHS:-ba2 ba1 deg}; do
    r ${v}_$g env DLAMD_LIB=$L $B --irregular $g
  done
done
