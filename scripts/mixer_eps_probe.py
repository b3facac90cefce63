"""Mixer.mix(times, eps) wall time: the one-launch device loop (dl_mix_until) against the path
the Mixer takes when that loop is switched off (dl_mix_until_fits forced False): traced passes
(dl_mix_rounds_trace + one readback per pass) with eps set, one dl_mix_rounds pass without --
the per-round host loop (dl_mix_round + 4-byte readback per round) before round 2; same models,
same result.
Usage: python scripts/mixer_eps_probe.py  (GPU)."""
import logging
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from distributed_learning_amd import engine  # noqa: E402
from distributed_learning_amd.networks import ANNModel  # noqa: E402
from distributed_learning_amd.utils.consensus_simple import Mixer  # noqa: E402


def models(n, dims, seed):
    torch.manual_seed(seed)
    return {i: ANNModel(*dims).cuda() for i in range(n)}


def ring(n):
    return {i: {(i - 1) % n: 0.25, i: 0.5, (i + 1) % n: 0.25} for i in range(n)}


def flat(ms):
    return torch.stack([torch.cat([p.data.view(-1) for p in m.parameters()]) for m in ms.values()])


def run(n, dims, times, eps, resident, reps=20):
    log = logging.getLogger("probe")
    fits = engine.until_fits
    if not resident:
        engine.until_fits = lambda W, P: False
    try:
        out, best, done = None, 1e9, None
        ms = models(n, dims, 0)
        init = [p.data.clone() for m in ms.values() for p in m.parameters()]
        mx = Mixer(ms, ring(n), log)      # built once, mix() called repeatedly (notebook use)
        for r in range(reps):
            for p, q in zip([p for m in ms.values() for p in m.parameters()], init):
                p.data.copy_(q)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            done = mx.mix(times=times, eps=eps)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t0)
            out = flat(ms)
        return best, done, out
    finally:
        engine.until_fits = fits


def main():
    print(f"{'agents':>6} {'params':>7} {'times':>5} {'eps':>7} {'rounds':>6} "
          f"{'device ms':>9} {'passes ms':>9} {'x':>6}", flush=True)
    for n, dims in [(5, (30, 17, 5)), (8, (40, 20, 5)), (16, (20, 16, 4))]:
        for times, eps in [(1, 1e-3), (1, 1e-5), (10, None)]:
            td, kd, od = run(n, dims, times, eps, True)
            th, kh, oh = run(n, dims, times, eps, False)
            assert kd == kh and torch.equal(od, oh), (n, dims, times, eps, kd, kh)
            P = od.shape[1]
            print(f"{n:>6} {P:>7} {times:>5} {str(eps):>7} {kd:>6} {td * 1e3:>9.3f} "
                  f"{th * 1e3:>9.3f} {th / td:>6.1f}", flush=True)


if __name__ == "__main__":
    main()
