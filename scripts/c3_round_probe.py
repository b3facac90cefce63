"""c3 round shapes (256 agents x 164,560 params, fused local step + mix + deviation) under every
layout / tile / grid configuration, against the triad ceiling of the same byte count.
HIP events, median of 5 x 20 back-to-back rounds.  python scripts/c3_round_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd import engine  # noqa: E402
import bench  # noqa: E402


def time_it(fn, reps=20, rounds=5):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        out.append(s.elapsed_time(e) / reps)
    out.sort()
    return out[len(out) // 2], out[0], out[-1]


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="", help="comma list of case-name prefixes (all if empty)")
    ap.add_argument("--no-ceiling", action="store_true")
    ap.add_argument("--pad-cols", default="", help="comma list of padded row widths: the "
                    "default row-major plan at each (tile-count quantisation)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, P, lr = 256, 164560, 0.05
    csr, _ = bench.build_graph(n)
    alg = 12 * n * P
    if not args.no_ceiling:
        copy, triad, var = bench.copy_ceiling(dev, nbytes=256 * 164608 * 4, reps=20)
        print(json.dumps({"case": "ceiling", "copy_GBs": copy, "triad_GBs": triad,
                          "variants": var}), flush=True)
    gen = torch.Generator(device=dev).manual_seed(0)
    X0 = torch.randn(n, P, device=dev, generator=gen)
    G0 = torch.randn(n, P, device=dev, generator=gen)
    cases = [
        ("rows T128 balanced", "rows", None, 164608, {}),
        ("rows T128 grid256", "rows", None, 164608, {"DLAMD_BALANCE_GRID": "0"}),
        ("rows T128 nt", "rows", None, 164608, {"DLAMD_NT_STORE": "1"}),
        ("rows T64", "rows", None, 164608, {"DLAMD_MAX_TILE_CHUNKS": "16"}),
        ("rows T64 wg1", "rows", None, 164608, {"DLAMD_MAX_TILE_CHUNKS": "16",
                                                "DLAMD_WG_PER_CU": "1"}),
        ("rows T32", "rows", None, 164608, {"DLAMD_MAX_TILE_CHUNKS": "8"}),
        ("tiled T64", "tiled", 64, P, {}),
        ("tiled T64 mult1", "tiled", 64, P, {"DLAMD_GRID_MULT": "1"}),
        ("tiled T64 wg1", "tiled", 64, P, {"DLAMD_WG_PER_CU": "1"}),
        ("tiled T32", "tiled", 32, P, {}),
        ("tiled T128", "tiled", 128, P, {}),
        ("tiled T16", "tiled", 16, P, {}),
        # plan path 4: the CSR in registers (DLAMD_FORCE_REG, a test knob): no LDS CSR reads
        ("reg rows T64", "rows", None, 164608, {"DLAMD_FORCE_REG": "1",
                                                "DLAMD_MAX_TILE_CHUNKS": "16"}),
        ("reg tiled T64", "tiled", 64, P, {"DLAMD_FORCE_REG": "1"}),
        ("reg tiled T64 mult1", "tiled", 64, P, {"DLAMD_FORCE_REG": "1", "DLAMD_GRID_MULT": "1"}),
        ("reg tiled T32", "tiled", 32, P, {"DLAMD_FORCE_REG": "1"}),
    ]
    for w in [int(v) for v in args.pad_cols.split(",") if v]:
        cases.append((f"rows pad{w}", "rows", None, w, {}))
    want = [c for c in args.cases.split(",") if c]
    for name, layout, T, Pp, env in cases:
        if want and not any(name.startswith(w) for w in want):
            continue
        for k, v in env.items():
            os.environ[k] = v
        try:
            X = torch.nn.functional.pad(X0, (0, Pp - P))[:, :Pp].contiguous() if layout == "rows" else X0
            G = torch.nn.functional.pad(G0, (0, Pp - P))[:, :Pp].contiguous() if layout == "rows" else G0
            eng = engine.GossipEngine(csr, Pp, device=dev, X=X, layout=layout, tile_cols=T)
            Gl = eng.layout_like(G)
            plan = eng.plan(deviation=True)
            med, lo, hi = time_it(lambda: eng.round(G=Gl, lr=lr, deviation=True))
            nodev = time_it(lambda: eng.round(G=Gl, lr=lr, deviation=False))[0]
            print(json.dumps({"case": name, "plan": plan, "us": med * 1e3,
                              "us_no_deviation": nodev * 1e3,
                              "spread_us": [lo * 1e3, hi * 1e3],
                              "GBs": 12 * n * Pp / (med / 1e3) / 1e9,
                              "frac": 12 * n * Pp / (med / 1e3) / 1e9 / 8000.0}), flush=True)
            del eng, Gl, X, G
            torch.cuda.empty_cache()
        finally:
            for k in env:
                os.environ.pop(k, None)


if __name__ == "__main__":
    main()
