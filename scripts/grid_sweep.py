"""Persistent-grid placement sweep for the fused round (local step + mix + deviation, tiled
layout) at c2 (1024 x 2^20, random 4-regular) and c4 (4096 x 2^18, torus) sizes:
DLAMD_GRID_MULT = k (workgroups = k x the resident count) x DLAMD_LDS_MIN (LDS per workgroup,
98304 bytes = at most one 1024-thread workgroup per CU).  HIP-event medians of 3 x reps rounds.
python scripts/grid_sweep.py [--reps R] [--cases c2,c4]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd import engine  # noqa: E402
import bench  # noqa: E402
from kbench import time_it  # noqa: E402

SHAPES = {"c2": (1024, 1 << 20, "rr4"), "c4": (4096, 1 << 18, "torus")}
POINTS = (("1", "0"), ("1", "98304"), ("2", "0"), ("2", "98304"), ("3", "0"), ("4", "0"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cases", default="c2,c4")
    ap.add_argument("--points", default="")   # mult:lds_min[:early_prefetch], e.g. "1:0,2:0:1"
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    print(json.dumps({"host": os.uname().nodename,
                      "triad_GBs": bench.copy_ceiling(dev)}), flush=True)
    for case in args.cases.split(","):
        n, P, kind = SHAPES[case]
        csr, _ = bench.build_graph(n, kind)
        g = torch.Generator(device=dev).manual_seed(0)
        eng = engine.GossipEngine(csr, P, device=dev,
                                  X=torch.randn(n, P, device=dev, generator=g), layout="tiled")
        G = eng.layout_like(torch.randn(n, P, device=dev, generator=g))
        for rep in range(2):
            pts = [tuple(p.split(":")) for p in args.points.split(",")] if args.points else POINTS
            for pt in pts:
                mult, lds_min = pt[0], pt[1]
                ep = pt[2] if len(pt) > 2 else "0"
                os.environ["DLAMD_GRID_MULT"] = mult
                os.environ["DLAMD_LDS_MIN"] = lds_min
                os.environ["DLAMD_EARLY_PREFETCH"] = ep
                ms = sorted(time_it(lambda: eng.round(G=G, lr=1e-3, deviation=True), args.reps)
                            for _ in range(3))
                plan = engine.plan_shape(eng.W, P, tile_cols=eng.T)
                print(json.dumps({"case": case, "mult": mult, "lds_min": lds_min, "ep": ep,
                                  "grid": plan["grid"], "lds": plan["lds_bytes"], "ms": ms[1],
                                  "GBs": 12 * n * P / ms[1] / 1e6, "spread": [ms[0], ms[2]]}),
                      flush=True)
        os.environ.pop("DLAMD_GRID_MULT")
        os.environ.pop("DLAMD_LDS_MIN")
        del eng, G
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
