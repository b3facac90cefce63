#!/bin/bash
# Round-4 session B: the one-image traced kernel and the engine-order / hub tests, then the
# rocprofv3 trace + FETCH / WRITE passes of the one-rank-of-8 c4 round and the c4-ba round.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r11b; mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "=== $name"; timeout -k 10 "$t" "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "=== $name rc=$rc"; tail -4 $O/$name.log; if [ $rc -ne 0 ]; then exit $rc; fi; }
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
bash scripts/gpu_profile.sh r11b/c4rank --workload c4-rank --steps 20 --warmup 3 || exit $?
bash scripts/gpu_profile.sh r11b/c4ba --workload c4-ba --steps 20 --warmup 3 --no-cpu || exit $?
# the N > 1 paths rehearsed with 2 gloo ranks sharing the GPU (RCCL needs distinct GPUs): the
# c4 agent partition on the column-tiled layout, then the default line with its child probes
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1"
step c4_gloo2 300 $R --master-port 29511 bench.py --gpus 2 --workload c4 --dist-backend gloo --steps 5 --warmup 1
step c2_gloo2 600 $R --master-port 29512 bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 1 --no-cpu
