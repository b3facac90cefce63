"""Does recording a HIP timing-event pair around every round cost GPU time?  The c2 round and
one c4 rank's round (whole scheme), K rounds each, alternately with an event pair per round and
with one pair around all K; wall time per round and the kernel-only GPU time per round.

    python scripts/event_probe.py [--reps 3] [--steps 50]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=50)
    args = ap.parse_args()
    import bench
    from distributed_learning_amd import engine, sharding
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    g = torch.Generator(device=dev).manual_seed(0)

    def measure(name, step):
        for _ in range(5):
            step()
        torch.cuda.synchronize()
        for rep in range(args.reps):
            for mode in ("per-round", "span"):
                evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                       for _ in range(args.steps if mode == "per-round" else 1)]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if mode == "span":
                    evs[0][0].record(stream)
                for i in range(args.steps):
                    if mode == "per-round":
                        evs[i][0].record(stream)
                    step()
                    if mode == "per-round":
                        evs[i][1].record(stream)
                if mode == "span":
                    evs[0][1].record(stream)
                torch.cuda.synchronize()
                wall = (time.perf_counter() - t0) / args.steps * 1e3
                gpu = (np.mean([a.elapsed_time(b) for a, b in evs]) if mode == "per-round"
                       else evs[0][0].elapsed_time(evs[0][1]) / args.steps)
                print(f"{name:8s} rep {rep} {mode:9s} wall {wall:.4f} ms/round  events "
                      f"{gpu:.4f} ms/round", flush=True)

    csr, _ = bench.build_graph(1024)
    P = 1 << 20
    eng = engine.GossipEngine(csr, P, device=dev, X=torch.randn(1024, P, device=dev, generator=g))
    G = eng.layout_like(torch.randn(1024, P, device=dev, generator=g))
    measure("c2", lambda: eng.round(G=G, lr=1e-3, deviation=True))
    del eng, G
    torch.cuda.empty_cache()

    tcsr, rows, cols, _ = bench.c4_torus()
    parts = sharding.torus_block_partition(rows, cols, 8)
    rp = sharding.split_halo_plans(tcsr, parts)[0]
    P = 1 << 18
    shard = sharding.HaloShard(rp, P, dev, sharding.ResidentHaloTransport(), n_agents_total=4096,
                               overlap="chunks")
    shard.X.normal_(generator=g)
    Gs = engine.staggered_zeros(shard._shape(rp.n_local), 2, dev).normal_(generator=g)
    _, halo, _ = shard._buffers(0, P)
    halo.normal_(generator=g)
    measure("c4rank", lambda: shard.round(G=Gs, lr=1e-3, deviation=True))


if __name__ == "__main__":
    main()
