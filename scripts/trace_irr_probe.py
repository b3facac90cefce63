"""Probe: Mixer.mix(times, eps)'s traced passes on 4096-agent irregular graphs (mix_trace_irr_kernel:
the Barabasi-Albert graph of c4-ba, and a row-stochastic graph whose per-round column mean is
reduced from each round's outputs) against the loop they replace, one fused round + deviation +
a 4-byte readback per round.  P = 2^18 columns, the engine's column-tiled layout.

    python scripts/trace_irr_probe.py
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from distributed_learning_amd import engine as E  # noqa: E402
from distributed_learning_amd.graph import Csr, barabasi_albert_metropolis  # noqa: E402


def row_stochastic(n, lo, hi, seed):
    """Ring + random extra neighbours (degree lo..hi), random positive row weights summing to 1,
    the self entry at a random position: row- but not column-stochastic."""
    rng = np.random.default_rng(seed)
    adj = [set() for _ in range(n)]
    for i in range(n):
        adj[i].add((i + 1) % n)
        adj[(i + 1) % n].add(i)
    for i in range(n):
        want = int(rng.integers(lo, hi + 1))
        while len(adj[i]) < want:
            j = int(rng.integers(n))
            if j != i:
                adj[i].add(j)
                adj[j].add(i)
    rowptr, col, w = [0], [], []
    for i in range(n):
        nb = sorted(adj[i])
        ws = rng.uniform(0.5, 1.5, len(nb) + 1)
        ws = list(ws / ws.sum())
        pos = int(rng.integers(len(nb) + 1))
        col.extend(nb[:pos] + [i] + nb[pos:])
        w.extend(ws)
        rowptr.append(len(col))
    return Csr(rowptr, col, w, keys=list(range(n)))


def main():
    dev = torch.device("cuda", 0)
    out = {}
    cases = []
    for n, P in ((4096, 1 << 18), (2048, 1 << 19), (4096, 1 << 14)):
        cases += [(f"ba2 n={n} P={P}", n, P, barabasi_albert_metropolis(n, 2, 1)),
                  (f"row-stochastic deg 4..9 n={n} P={P}", n, P, row_stochastic(n, 4, 9, 7))]
    for name, n, P, csr in cases:
        g = torch.Generator(device=dev).manual_seed(0)
        X = torch.randn(n, P, device=dev, generator=g)
        eng = E.GossipEngine(csr, P, device=dev, X=X)
        del X
        K = eng.trace_max_rounds()
        rec = {"layout": eng.layout, "plan": eng.plan(), "rounds_per_pass": K}
        if K > 0:
            trace = torch.empty(K, device=dev)
            for _ in range(2):
                eng.rounds_traced(K, trace)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            passes = 10
            for _ in range(passes):
                eng.rounds_traced(K, trace)
                trace.cpu()          # the host tests the pass's K deviations
            rec["traced_rounds_per_s"] = passes * K / (time.perf_counter() - t0)
        for _ in range(3):
            eng.round(deviation=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        k = 30
        for _ in range(k):
            eng.round(deviation=True)
            float(eng.dev_max.item())   # the loop's per-round readback
        rec["loop_rounds_per_s"] = k / (time.perf_counter() - t0)
        out[name] = rec
        print(name, json.dumps(rec), flush=True)
        del eng
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
