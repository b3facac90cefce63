"""Probe: how much of the c2 round's box-to-box spread (436-454 rounds/s for one binary) is the
placement of X, G and Y in HBM.  Builds the c2 engine (1024 agents x 2^20, random 4-regular,
fused local step + mix + deviation) under several stagger steps between the three resident
buffers (engine.STAGGER_BYTES; 0 = packed allocations), each twice in alternation, and times
rounds with HIP events.

    python scripts/placement_probe.py
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from distributed_learning_amd import engine as E  # noqa: E402
from distributed_learning_amd.graph import (best_constant_weight, from_edge_weights,  # noqa: E402
                                            random_regular_edges)


def main():
    dev = torch.device("cuda", 0)
    n, P = 1024, 1 << 20
    edges = random_regular_edges(4, n, seed=0)
    verts = list(range(n))
    csr = from_edge_weights(edges, [best_constant_weight(edges, verts)] * len(edges), verts)
    base = E.STAGGER_BYTES
    steps = {"default (2 MiB + 64 KiB)": base, "packed (none)": None, "64 KiB": 64 << 10,
             "1 MiB + 64 KiB": (1 << 20) + (64 << 10), "4 MiB + 192 KiB": (4 << 20) + (192 << 10),
             "2 MiB + 320 KiB": (2 << 20) + (320 << 10)}
    res = {k: [] for k in steps}
    g = torch.Generator(device=dev).manual_seed(0)
    for rep in range(2):
        for name, st in steps.items():
            if st is None:
                os.environ["DLAMD_STAGGER"] = "0"
            else:
                os.environ.pop("DLAMD_STAGGER", None)
                E.STAGGER_BYTES = st
            X = torch.randn(n, P, device=dev, generator=g)
            eng = E.GossipEngine(csr, P, device=dev, X=X)
            del X
            G = eng.layout_like(torch.randn(n, P, device=dev, generator=g))
            mean = torch.empty(P, device=dev)
            for _ in range(5):
                eng.round(G=G, lr=1e-3, deviation=True, mean=mean)
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(30)]
            for a, b in ev:
                a.record()
                eng.round(G=G, lr=1e-3, deviation=True, mean=mean)
                b.record()
            torch.cuda.synchronize()
            ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
            res[name].append(ms)
            print(f"rep {rep} {name:>26}: {ms:.4f} ms = {12 * n * P / ms / 1e9:.2f} TB/s "
                  f"({1e3 / ms:.1f} rounds/s)", flush=True)
            del eng, G, mean
            torch.cuda.empty_cache()
            time.sleep(0.2)
    E.STAGGER_BYTES = base
    print(json.dumps({k: [round(v, 4) for v in vs] for k, vs in res.items()}))


if __name__ == "__main__":
    main()
