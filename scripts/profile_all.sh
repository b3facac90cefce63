#!/bin/bash
# rocprofv3 kernel trace + FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_profile.sh) of every
# bench line whose roofline.traffic cites a committed summary, into gpurun_out/<tag>/<line>/.
# Afterwards, on the CPU: scripts/profile_summary.py gpurun_out/<tag>/<line> profiles/<tag>/<line>
# (LAST=50 for c3: the timed graph steps).   Usage: scripts/profile_all.sh <tag> [lines...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
LINES=${@:-"c2 c3 c4 c4rank c4ba c4gather"}
for l in $LINES; do
    case $l in
        c2) A="--steps 20 --warmup 3 --no-cpu --no-fdla-probe" ;;
        c3) A="--workload c3 --steps 50 --warmup 5 --no-cpu" ;;
        c4) A="--workload c4 --steps 20 --warmup 3 --no-cpu" ;;
        c4rank) A="--workload c4-rank --steps 30 --warmup 3 --no-cpu" ;;
        c4ba) A="--workload c4-ba --steps 20 --warmup 3 --no-cpu" ;;
        c4gather) A="--workload c4-gather --steps 20 --warmup 3 --no-cpu" ;;
        *) echo "unknown line $l"; exit 2 ;;
    esac
    echo "=== $l: $A"
    bash scripts/gpu_profile.sh $TAG/$l $A || exit $?
done
echo done
