"""Kernel-level timing of dl_mix_round variants (HIP events), one JSON line per variant.
python scripts/kbench.py [--reps R]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd import engine  # noqa: E402
from distributed_learning_amd.graph import from_edge_weights, random_regular_edges  # noqa: E402
import bench  # noqa: E402


def time_it(fn, reps):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cases", default="all")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    print(json.dumps({"copy_ceiling_GBs": bench.copy_ceiling(dev)}), flush=True)
    if args.cases == "tile2":
        # repeated sweep: tile width x shared weights x workgroups per CU
        for n, P, Ts in [(1024, 1 << 20, (8, 16, 32)), (512, 1 << 21, (16, 32)),
                         (2048, 1 << 19, (4, 8)), (256, 1 << 22, (32, 64))]:
            edges = random_regular_edges(4, n, seed=0)
            csr = from_edge_weights(edges, [0.2] * len(edges), list(range(n)))
            X = torch.randn(n, P, device=dev)
            G = torch.randn(n, P, device=dev)
            for T in Ts:
                for shared in (1, 0):
                    eng = engine.GossipEngine(csr, P, device=dev, X=X, layout="tiled",
                                              tile_cols=T)
                    eng.W.shared_row_weights = shared
                    Gl = eng.layout_like(G)
                    for wg in ("2", "1"):
                        os.environ["DLAMD_WG_PER_CU"] = wg
                        ms = sorted(time_it(lambda: eng.round(G=Gl, lr=1e-3, deviation=True),
                                            args.reps) for _ in range(3))
                        print(json.dumps({"n": n, "T": T, "shared": shared, "wg": wg,
                                          "ms": ms[1], "GBs": 12 * n * P / ms[1] / 1e6,
                                          "spread": [ms[0], ms[2]]}), flush=True)
                    os.environ.pop("DLAMD_WG_PER_CU")
                    del eng, Gl
            del X, G
        return
    if args.cases == "tile":
        # tile width x shared-weight sweep (tiled layout, SGD + deviation, the bench round)
        for n, P, Ts in [(1024, 1 << 20, (4, 8, 16, 32)), (512, 1 << 21, (8, 16, 32, 64)),
                         (4096, 1 << 18, (4,))]:
            edges = random_regular_edges(4, n, seed=0)
            csr = from_edge_weights(edges, [0.2] * len(edges), list(range(n)))
            X = torch.randn(n, P, device=dev)
            G = torch.randn(n, P, device=dev)
            for T in Ts:
                for shared in (1, 0):
                    try:
                        eng = engine.GossipEngine(csr, P, device=dev, X=X, layout="tiled",
                                                  tile_cols=T)
                        eng.W.shared_row_weights = shared
                        Gl = eng.layout_like(G)
                        ms = time_it(lambda: eng.round(G=Gl, lr=1e-3, deviation=True), args.reps)
                    except ValueError as ex:
                        print(json.dumps({"n": n, "T": T, "shared": shared, "error": str(ex)}))
                        continue
                    lds = engine.plan_shape(eng.W, P)  # row-major plan, for reference
                    print(json.dumps({"n": n, "P": P, "T": T, "shared": shared, "ms": ms,
                                      "GBs": 12 * n * P / ms / 1e6,
                                      "auto_plan_T": lds["tile_cols"]}), flush=True)
                    del eng, Gl
            del X, G
        return
    if args.cases == "nt":
        edges = random_regular_edges(4, 1024, seed=0)
        csr = from_edge_weights(edges, [0.2] * len(edges), list(range(1024)))
        X = torch.randn(1024, 1 << 20, device=dev)
        G = torch.randn(1024, 1 << 20, device=dev)
        eng = engine.GossipEngine(csr, 1 << 20, device=dev, X=X)
        Gl = eng.layout_like(G)
        for rep in range(2):
            for ntl in ("1",):
                for nts in ("1",):
                    os.environ["DLAMD_NT_STORE"] = nts
                    os.environ["DLAMD_NT_LOAD"] = ntl
                    ms = time_it(lambda: eng.round(G=Gl, lr=1e-3, deviation=True), args.reps)
                    print(json.dumps({"nt_load": ntl, "nt_store": nts, "ms": ms,
                                      "GBs": 12 * 1024 * (1 << 20) / ms / 1e6}), flush=True)
        return
    for n, P in [(1024, 1 << 20), (512, 1 << 21), (256, 1 << 22), (2048, 1 << 19)]:
        edges = random_regular_edges(4, n, seed=0)
        csr = from_edge_weights(edges, [0.2] * len(edges), sorted(set(u for e in edges for u in e)))
        X = torch.randn(n, P, device=dev)
        G = torch.randn(n, P, device=dev)
        for layout in ("tiled", "rows"):
            eng = engine.GossipEngine(csr, P, device=dev, X=X, layout=layout)
            Gl = eng.layout_like(G)
            for sgd in (False, True):
                for dv in (False, True):
                    g = Gl if sgd else None
                    ms = time_it(lambda: eng.round(G=g, lr=1e-3, deviation=dv), args.reps)
                    nbytes = (12 if sgd else 8) * n * P
                    print(json.dumps({"n": n, "P": P, "layout": layout, "sgd": sgd, "dev": dv,
                                      "ms": ms, "GBs": nbytes / ms / 1e6,
                                      "plan": eng.plan(deviation=dv)}), flush=True)
            del eng, Gl
        del X, G
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
