#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only) over a probe binary.
# Usage: scripts/gpu_pmc_probe.sh <tag> <binary> [args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for grp in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_THRASHING_STALL_sum" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_STALL_MULTI_MISS_sum" \
           "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_HIT_sum TCC_MISS_sum" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT" \
           "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum"; do
    i=$((i+1))
    echo "=== pass $i: $grp"
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1
    rc=$?
    echo "rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
echo done
