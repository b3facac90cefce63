#!/bin/bash
# Round 6 head check: smoke, the whole GPU suite, and the N > 1 bench path rehearsed with two
# gloo ranks sharing this one GPU (the driver's torchrun command shape).  Trouble ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r13/check
mkdir -p $O
timeout -k 10 400 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -3 $O/smoke.log
timeout -k 10 1500 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --no-cpu > $O/bench_gloo2.log 2>&1 || { tail -30 $O/bench_gloo2.log; exit 3; }
tail -c 1500 $O/bench_gloo2.log
echo done
