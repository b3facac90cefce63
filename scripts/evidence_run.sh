#!/bin/bash
# Every throughput figure README.md quotes, from one box in one call: each bench line under its
# own time limit into gpurun_out/evidence/ (copied to profiles/rNN/evidence/ afterwards).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/evidence${EVID_SUFFIX:-}
mkdir -p $O
bash scripts/gpu_steps.sh \
  "evidence${EVID_SUFFIX:-}/c2|300|python bench.py --steps 50 --warmup 5" \
  "evidence${EVID_SUFFIX:-}/c2_gossip64|200|python bench.py --workload c2-gossip --rounds 64 --steps 10 --warmup 2 --no-cpu" \
  "evidence${EVID_SUFFIX:-}/c2_trace24|200|python bench.py --workload c2-gossip --trace --rounds 24 --steps 10 --warmup 2 --no-cpu" \
  "evidence${EVID_SUFFIX:-}/c3|300|python bench.py --workload c3 --steps 50 --warmup 5" \
  "evidence${EVID_SUFFIX:-}/c4|200|python bench.py --workload c4 --steps 20 --warmup 3" \
  "evidence${EVID_SUFFIX:-}/c4_gossip64|200|python bench.py --workload c2-gossip --graph torus --agents 4096 --params 262144 --rounds 64 --relabel 0 --steps 10 --warmup 2 --no-cpu" \
  "evidence${EVID_SUFFIX:-}/c4_trace8|200|python bench.py --workload c2-gossip --graph torus --agents 4096 --params 262144 --trace --rounds 8 --relabel 0 --steps 10 --warmup 2 --no-cpu" \
  "evidence${EVID_SUFFIX:-}/c4_gather|200|python bench.py --workload c4-gather --steps 20 --warmup 3 --no-cpu" \
  "evidence${EVID_SUFFIX:-}/c4_ba|200|python bench.py --workload c4-ba --steps 20 --warmup 3 --no-cpu" \
  "evidence${EVID_SUFFIX:-}/c4_ba1|200|python bench.py --workload c4-ba --irregular ba1 --steps 20 --warmup 3 --no-cpu" \
  "evidence${EVID_SUFFIX:-}/c4_rank|200|python bench.py --workload c4-rank --steps 50 --warmup 5" \
  "evidence${EVID_SUFFIX:-}/c1|200|python bench.py --workload c1 --steps 4000 --warmup 1" \
  "evidence${EVID_SUFFIX:-}/mixer_eps|200|python scripts/mixer_eps_probe.py" \
  "evidence${EVID_SUFFIX:-}/c5|600|python bench.py --workload c5 --steps 10 --warmup 3"
