"""Does the HBM stream rate ramp after process start?  The c2 round (fused local step + mix +
deviation, tiled) timed in batches of 10 rounds from the first launch on, for ~3 s, then the
triad ceilings, then another round batch.  One JSON line per batch (t = seconds since the
first round).  python scripts/warm_probe.py [--batches B] [--triad-first]"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd import engine  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=120)
    ap.add_argument("--triad-first", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, P = 1024, 1 << 20
    csr, _ = bench.build_graph(n)
    g = torch.Generator(device=dev).manual_seed(0)
    eng = engine.GossipEngine(csr, P, device=dev, X=torch.randn(n, P, device=dev, generator=g),
                              layout="tiled")
    G = eng.layout_like(torch.randn(n, P, device=dev, generator=g))
    eng.reserve_workspace()
    torch.cuda.synchronize()
    if args.triad_first:
        c = bench.copy_ceiling(dev)
        print(json.dumps({"triad_first": c[1], "variants": c[2]}), flush=True)
    t_start = time.perf_counter()

    def batch(tag):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(10):
            eng.round(G=G, lr=1e-3, deviation=True)
        e.record()
        e.synchronize()
        ms = s.elapsed_time(e) / 10
        print(json.dumps({"tag": tag, "t": round(time.perf_counter() - t_start, 3),
                          "ms": round(ms, 4), "GBs": round(12 * n * P / ms / 1e6)}), flush=True)

    for _ in range(args.batches):
        batch("round")
    c = bench.copy_ceiling(dev)
    print(json.dumps({"triad_after": c[1], "variants": c[2]}), flush=True)
    for _ in range(10):
        batch("round_after")


if __name__ == "__main__":
    main()
