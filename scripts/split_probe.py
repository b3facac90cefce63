"""Probe: a split halo round's boundary launch reading the boundary rows' stepped values from
the send blocks (HaloShard.W_bnd_packed, the default in the column-tiled layout) against
re-stepping them from x and g (the plain row_sets launch); one rank of the 8-, 4- and 2-way c4
partition alone on one GPU (sharding.ResidentHaloTransport), alternating in one process.
(profiles/r11/split_probe_side_stream.log has a third mode, from a since-removed build: the pack
posted from a side stream, 435 against 420 us at one rank of 8.)

    python scripts/split_probe.py
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402
from distributed_learning_amd import engine, sharding  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    csr, rows, cols, _ = bench.c4_torus()
    n, P, lr = csr.n_rows, 1 << 18, 1e-3
    out = {}
    for world in (8, 4, 2):
        rp = sharding.split_halo_plans(csr, sharding.torus_block_partition(rows, cols, world))[0]
        shard = sharding.HaloShard(rp, P, dev, sharding.ResidentHaloTransport(),
                                   n_agents_total=n, overlap="split")
        gen = torch.Generator(device=dev).manual_seed(1)
        shard.X.normal_(generator=gen)
        G = engine.staggered_zeros(shard._shape(rp.n_local), 2, dev).normal_(generator=gen)
        _, halo, _ = shard._buffers(0, P)
        halo.normal_(generator=gen)
        packed = shard.W_bnd_packed
        res = {"packed": [], "restep": []}
        for rep in range(3):
            for mode in res:
                shard.W_bnd_packed = packed if mode != "restep" else None
                for _ in range(5):
                    shard.round(G=G, lr=lr, deviation=True)
                torch.cuda.synchronize()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(30)]
                for a, b in ev:
                    a.record()
                    shard.round(G=G, lr=lr, deviation=True)
                    b.record()
                torch.cuda.synchronize()
                res[mode].append(float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3)
        out[world] = {k: [round(v, 1) for v in vs] for k, vs in res.items()}
        print(f"one rank of {world}: split round us, " +
              "; ".join(f"{k} {v}" for k, v in out[world].items()), flush=True)
        del shard, G
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
