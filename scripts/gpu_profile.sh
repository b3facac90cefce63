#!/bin/bash
# rocprofv3 evidence for profiles/: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE in
# separate passes (no trace domains besides --kernel-trace, per the pool's rules).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
ARGS=${@:-"--steps 20 --warmup 3 --no-cpu"}
run() {
    local name=$1; shift
    echo "=== $name"
    timeout -k 10 400 rocprofv3 "$@" --output-format csv -d $OUT/$name -o run -- python bench.py $ARGS > $OUT/$name.log 2>&1
    local rc=$?
    echo "rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 $OUT/$name.log; exit $rc; fi
}
run trace --kernel-trace --stats
run fetch --kernel-trace --pmc FETCH_SIZE
run write --kernel-trace --pmc WRITE_SIZE
echo done
