#!/bin/bash
# c3 with the local-step emission (the gradient kernel writes X - lr G): GPU tests of the c3
# paths, bench lines for both emissions, phase probe, rocprof trace + FETCH/WRITE passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/c3s
mkdir -p $OUT
set -o pipefail
s() { local n=$1 t=$2; shift 2; echo "=== $n"; timeout -k 10 "$t" "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "rc=$rc"; tail -3 $OUT/$n.log; [ $rc -eq 0 ] || exit $rc; }
s tests 400 python -u -m pytest tests/test_batched_ann_gpu.py tests/test_configs_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread -k "not c5"
s bench_step 300 python bench.py --workload c3 --steps 50 --warmup 5
s bench_grad 300 python bench.py --workload c3 --steps 50 --warmup 5 --c3-emit grad --no-cpu
s bench_step2 300 python bench.py --workload c3 --steps 50 --warmup 5 --no-cpu
s probe_grad 60 ./scripts/bin/mlp_probe x6 rows
s probe_step 60 ./scripts/bin/mlp_probe x6 rows step
ARGS="--workload c3 --steps 50 --warmup 5 --no-cpu"
s trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof/trace -o run -- python bench.py $ARGS
s fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/prof/fetch -o run -- python bench.py $ARGS
s write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/prof/write -o run -- python bench.py $ARGS
echo done
