#!/bin/bash
# Round-4 session U (final head; re-run as session V after the last sharding changes): the whole GPU suite, the smoke, the default bench line, and
# the N = 2 gloo rehearsal of the c4 agent partition (split rounds reading the send blocks).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11v; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -2 $O/$name.log | cut -c1-300;
         if [ $rc -ne 0 ] && ! { [ "${SOFT:-0}" = 1 ] && [ $rc -eq 1 ]; }; then exit $rc; fi; }
SOFT=1 step tests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
if grep -q -i -E "hipError|illegal|memory access fault|HSA_STATUS_ERROR|Aborted" $O/tests.log; then
    echo "device error in the tests: stopping"; exit 4; fi
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python bench.py
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step c4rank 240 python bench.py --workload c4-rank --steps 50 --warmup 5
step c4_gloo2 300 $R --master-port 29561 bench.py --gpus 2 --workload c4 --dist-backend gloo --steps 5 --warmup 1
