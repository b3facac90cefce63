#!/bin/bash
# GPU session script: smoke -> gpu tests -> bench -> rocprof kernel trace.
# Each GPU step has its own time limit; a fault/abort/timeout (exit >= 2 except pytest's 1 for
# test failures) ends the script so nothing else touches the GPU after trouble.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
step() {  # name, timeout, cmd...
    local name=$1 t=$2; shift 2
    echo "=== $name: $*" | tee -a $OUT/steps.log
    timeout -k 10 "$t" "$@" > $OUT/$name.log 2>&1
    local rc=$?
    echo "=== $name rc=$rc" | tee -a $OUT/steps.log
    tail -5 $OUT/$name.log
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
MODE=${1:-all}
if [ "$MODE" = all ] || [ "$MODE" = test ]; then
    step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
    step pytest_gpu 1200 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread
fi
if [ "$MODE" = all ] || [ "$MODE" = bench ]; then
    step bench 600 python bench.py --steps 50 --warmup 5
fi
if [ "$MODE" = all ] || [ "$MODE" = workloads ]; then
    step bench_c3 600 python bench.py --workload c3 --steps 50 --warmup 5
    step bench_c4 600 python bench.py --workload c4 --steps 20 --warmup 3
fi
if [ "$MODE" = all ] || [ "$MODE" = prof ]; then
    step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 20 --warmup 3 --no-cpu
fi
echo "=== done"
