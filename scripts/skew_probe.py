"""Does the round's rate depend on where X, G and Y sit relative to each other in HBM?
(a) arena: one allocation holds X | G | Y (column-tiled c2 operands, 4 GiB each), G and Y shifted
    by `skew` extra bytes each;
(b) separate: three allocations (as the engine makes them), the operands starting `stagger` x
    slot bytes into their own allocation (slot 0, 1, 2 for X, G, Y).
The round (fused local step + mix + deviation) is timed per layout, twice, in one process, with
the triad in the round's shape on the arena as the reference.  python scripts/skew_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd import _lib, engine  # noqa: E402
import bench  # noqa: E402
from kbench import time_it  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    n, P = 1024, 1 << 20
    csr, _ = bench.build_graph(n)
    W = engine.DeviceCsr(csr, dev)
    T = engine.plan_shape(W, P, tile_cols=-1)["tile_cols"]
    shape = engine.tiled_shape(n, P, T)
    NP = n * P
    dev_sq = torch.empty(n, device=dev)
    dev_max = torch.empty(1, device=dev)
    ws = engine.Workspace(dev)
    lib = _lib.load()

    def time_round(X, G, Y):
        ms = sorted(time_it(lambda: engine.mix_round(W, X, Y, G=G, lr=1e-3, dev_sq=dev_sq,
                                                     dev_max=dev_max, workspace=ws,
                                                     tiled=(P, T)), 10) for _ in range(3))
        return 12 * NP / ms[1] / 1e6

    mode = sys.argv[1] if len(sys.argv) > 1 else "both"
    if mode in ("both", "arena"):
        skews = [0, 65536, (1 << 21) + 65536, 12 << 20]
        big = torch.randn(3 * NP + 2 * max(skews) // 4, device=dev)
        X = big[0:NP].view(shape)
        tri = sorted(time_it(lambda: _lib.check(lib.dl_stream_copy(
            _lib.ptr(X), _lib.ptr(big[2 * NP:]), NP, 6, _lib.stream_handle(dev)), "triad"), 10)
            for _ in range(3))
        print(json.dumps({"triad6_arena_GBs": 12 * NP / tri[1] / 1e6}), flush=True)
        for rep in range(2):
            for skew in skews:
                s = skew // 4
                G = big[NP + s:2 * NP + s].view(shape)
                Y = big[2 * NP + 2 * s:3 * NP + 2 * s].view(shape)
                print(json.dumps({"layout": "arena", "skew": skew,
                                  "round_GBs": time_round(X, G, Y)}), flush=True)
        del big, X, G, Y
        torch.cuda.empty_cache()
    if mode in ("both", "separate"):
        staggers = [0, 65536, (1 << 20) + 65536, (1 << 21) + 65536, (4 << 20) + 196608]
        pad = 2 * max(staggers) // 4
        bufs = [torch.randn(NP + pad, device=dev) for _ in range(3)]
        for rep in range(2):
            for st in staggers:
                X, G, Y = (bufs[i][i * st // 4:i * st // 4 + NP].view(shape) for i in range(3))
                print(json.dumps({"layout": "separate", "stagger": st,
                                  "round_GBs": time_round(X, G, Y)}), flush=True)


if __name__ == "__main__":
    main()
