#!/bin/bash
# PMC counter passes for the mix kernel (one counter group per rocprofv3 run; no trace domains
# besides --kernel-trace).  Usage: scripts/gpu_pmc.sh <tag> [bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-pmc}; shift
ARGS=${@:-"--steps 10 --warmup 2 --no-cpu"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"; do
    i=$((i+1))
    echo "=== pass $i: $grp"
    timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "mix_tile|stream_copy" --output-format csv -d $OUT/p$i -o run -- python bench.py $ARGS > $OUT/p$i.log 2>&1
    rc=$?
    echo "rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 $OUT/p$i.log; exit $rc; fi
done
echo done
