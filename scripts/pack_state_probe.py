"""The c4-rank halo pack (one rank of 8: 96 boundary rows of 512, three peers) on the bench's own
buffers (HaloShard's staggered X, the bench's G, the [send | halo] buffer), timed with HIP
events after different predecessors: itself (warm), a read-only sweep of 1 GiB, a memset of
1 GiB, and the round's own mix launch.  Median of 20.
python scripts/pack_state_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from distributed_learning_amd import engine, sharding  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    csr, rows, cols, _ = bench.c4_torus()
    P, lr = 1 << 18, 1e-3
    parts = sharding.torus_block_partition(rows, cols, 8)
    rp = sharding.split_halo_plans(csr, parts)[0]
    shard = sharding.HaloShard(rp, P, dev, sharding.ResidentHaloTransport(), overlap="chunks")
    gen = torch.Generator(device=dev).manual_seed(1)
    shard.X.normal_(generator=gen)
    G = engine.staggered_zeros(shard._shape(rp.n_local), 2, dev).normal_(generator=gen)
    _, halo, _ = shard._buffers(0, P)
    halo.normal_(generator=gen)
    colsum = torch.empty(P, device=dev)
    dsq = torch.empty(rp.n_local, device=dev)
    mean_prev = torch.zeros(P, device=dev)
    flush = torch.empty(1 << 28, device=dev)          # 1 GiB
    stream = torch.cuda.current_stream(dev)

    preds = {
        "warm (pack after pack)": lambda: None,
        "after a 1-GiB read (sum)": lambda: flush.sum(),
        "after a 1-GiB memset": lambda: flush.fill_(0.5),
        "after the round's mix": lambda: shard.mix_chunk(0, P, halo, G, lr,
                                                        (mean_prev, colsum, dsq)),
    }
    out = {}
    for name, pre in preds.items():
        ts = []
        for i in range(23):
            pre()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            shard.pack(0, 0, P, G, lr)
            e1.record(stream)
            torch.cuda.synchronize()
            if i >= 3:
                ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        out[name] = {"median_us": ts[len(ts) // 2], "min_us": ts[0],
                     "frac": 12 * 96 * P / (ts[len(ts) // 2] / 1e6) / 8e12}
        print(json.dumps({name: out[name]}), flush=True)


if __name__ == "__main__":
    main()
