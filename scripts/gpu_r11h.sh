#!/bin/bash
# Round-4 session H: the N = 2 multi-rank paths rehearsed on one GPU with gloo (the c4 agent
# partition with the peer-grouped boundary order and all three halo schemes; the default c2 line
# with its embedded c4 child), then the c4-rank profile at the head.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11h; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -2 $O/$name.log | cut -c1-400;
         if [ $rc -ne 0 ]; then exit $rc; fi; }
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step c4_gloo2 300 $R --master-port 29511 bench.py --gpus 2 --workload c4 --dist-backend gloo --steps 5 --warmup 1
step c2_gloo2 400 $R --master-port 29512 bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 1
bash scripts/gpu_profile.sh r11h/c4rank --workload c4-rank --steps 20 --warmup 3 || exit $?
