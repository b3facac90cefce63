"""Is the c3 round (256 agents) slow because of its SIZE (fixed per-launch costs over a 110 us
launch) or its SHAPE (256-row tiles)?  The same round at 1x / 4x / 16x the columns, with and
without the fused deviation.  python scripts/c3_scale_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd import engine  # noqa: E402
import bench  # noqa: E402
from c3_round_probe import time_it  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n, lr = 256, 0.05
    csr, _ = bench.build_graph(n)
    for mult in (1, 4, 16):
        P = 164608 * mult
        gen = torch.Generator(device=dev).manual_seed(0)
        X = torch.randn(n, P, device=dev, generator=gen)
        G = torch.randn(n, P, device=dev, generator=gen)
        for layout, T in (("rows", None), ("tiled", 64)):
            eng = engine.GossipEngine(csr, P, device=dev, X=X, layout=layout, tile_cols=T)
            Gl = eng.layout_like(G)
            for dv in (True, False):
                med, lo, hi = time_it(lambda: eng.round(G=Gl, lr=lr, deviation=dv))
                print(json.dumps({"mult": mult, "layout": layout, "dev": dv,
                                  "plan": eng.plan(deviation=dv), "us": med * 1e3,
                                  "GBs": 12 * n * P / (med / 1e3) / 1e9}), flush=True)
            del eng, Gl
            torch.cuda.empty_cache()
        del X, G
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
