#!/bin/bash
# Round-4 session K: rocprofv3 + PMC of the c3 and c4 lines at the head (the bench's roofline
# traffic for them cited r10 / r05 profiles of earlier builds).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash scripts/gpu_profile.sh r11k/c3 --workload c3 --steps 50 --warmup 5 --no-cpu || exit $?
bash scripts/gpu_profile.sh r11k/c4 --workload c4 --steps 20 --warmup 3 --no-cpu || exit $?
