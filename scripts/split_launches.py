"""Split-scheme halo rounds (interior launch, then boundary launch) of one rank of the c4
partition alone on one GPU, for a kernel trace that separates the launches by instantiation:

    rocprofv3 --kernel-trace --stats -d gpurun_out/x -- python3 scripts/split_launches.py 8

(DLAMD_TILE_GROUP=1 before the command turns tile groups off for an A/B.)"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from distributed_learning_amd import engine, sharding  # noqa: E402


def main():
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    dev = torch.device("cuda", 0)
    csr, rows, cols, _ = bench.c4_torus()
    P, lr = 1 << 18, 1e-3
    rp = sharding.split_halo_plans(csr, sharding.torus_block_partition(rows, cols, world))[0]
    shard = sharding.HaloShard(rp, P, dev, sharding.ResidentHaloTransport(),
                               n_agents_total=csr.n_rows, overlap="split")
    gen = torch.Generator(device=dev).manual_seed(1)
    shard.X.normal_(generator=gen)
    G = engine.staggered_zeros(shard._shape(rp.n_local), 2, dev).normal_(generator=gen)
    for _ in range(rounds):
        shard.round(G=G, lr=lr, deviation=True)
    torch.cuda.synchronize()
    print(f"rank of {world}: {rounds} split rounds, boundary plan "
          f"{engine.plan_shape(shard.W_bnd_packed, P, tile_cols=shard.T)}", flush=True)


if __name__ == "__main__":
    main()
