#!/bin/bash
# The headline's evidence from ONE box in ONE call:
#   1. the driver's c2 line (bench.py --steps 20 --warmup 5) -> gpurun_out/r13/c2/bench.json
#   2. rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE passes of the same line
#   3. optional same-box A/B of another libdlamd.so build on the same line (AB_LIB, AB_REPS)
# Every step under its own time limit; any failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r13/c2
mkdir -p $O
ARGS=${BENCH_ARGS:-"--steps 20 --warmup 5"}
echo "=== bench $ARGS"
timeout -k 10 400 python bench.py $ARGS > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 3; }
tail -c 600 $O/bench.json
prof() {
    local name=$1; shift
    echo "=== $name"
    # (--no-fdla-probe: the per-edge-weight probe launches the same kernel instance on another
    # graph, and its launches would mix into the instance's average)
    timeout -k 10 400 rocprofv3 "$@" --output-format csv -d $O/$name -o run -- python bench.py $ARGS --no-cpu --no-fdla-probe > $O/$name.log 2>&1
    local rc=$?
    echo "rc=$rc"
    if [ $rc -ne 0 ]; then tail -20 $O/$name.log; exit $rc; fi
}
prof trace --kernel-trace --stats
prof fetch --kernel-trace --pmc FETCH_SIZE
prof write --kernel-trace --pmc WRITE_SIZE
if [ -n "$AB_LIB" ]; then
    bash scripts/ab_bench.sh r13/c2_ab "$AB_LIB" "${AB_REPS:-3}" $ARGS --no-cpu --no-fdla-probe || exit $?
fi
echo done
