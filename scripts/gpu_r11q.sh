#!/bin/bash
# Round-4 session Q: the column sums' all-reduce deferred to the next round's mix (posted async,
# waited after the next pack and exchange): sharding GPU tests and the N = 2 gloo rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11q; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -1 $O/$name.log | cut -c1-200;
         if [ $rc -ne 0 ]; then exit $rc; fi; }
step tests 600 python -u -m pytest tests/test_sharding_gpu.py -q -m gpu --timeout 300 --timeout-method thread
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step c4_gloo2 300 $R --master-port 29531 bench.py --gpus 2 --workload c4 --dist-backend gloo --steps 5 --warmup 1
