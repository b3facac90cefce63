"""Where the c1 asyncio facade's host time goes: the Titanic ring-8 run through
utils.consensus_asyncio with each schedule, the host gradients alone, and a cProfile of each.
python scripts/c1_facade_probe.py [--steps N]"""
import argparse
import asyncio
import cProfile
import io
import os
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributed_learning_amd import workloads  # noqa: E402
from distributed_learning_amd.networks.logreg_model_titanic import LogRegTitanic  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    d = np.load(os.path.join(ROOT, "tests", "golden", "titanic.npz"))
    nt = int(d["n_test"])
    Xtr, ytr = d["X"][nt:], d["y"][nt:]
    topo = [(i, (i + 1) % 8) for i in range(8)]
    shards = workloads.split_data(Xtr, ytr, list(range(8)))
    m = LogRegTitanic(7)
    w = np.zeros(7)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for t in range(8):
            m.gradient(*shards[t], w)
    print(f"host gradients alone: {args.steps / (time.perf_counter() - t0):.0f} steps/s")
    res = {}
    for sched in ("synchronous", "reference"):
        asyncio.run(workloads.consensus_gd(topo, Xtr, ytr, 5, convergence_eps=10, device=dev,
                                           consensus=sched))
        t0 = time.perf_counter()
        res[sched] = asyncio.run(workloads.consensus_gd(topo, Xtr, ytr, args.steps,
                                                        convergence_eps=10, device=dev,
                                                        consensus=sched))
        print(f"{sched}: {args.steps / (time.perf_counter() - t0):.0f} steps/s", flush=True)
        pr = cProfile.Profile()
        pr.enable()
        asyncio.run(workloads.consensus_gd(topo, Xtr, ytr, 100, convergence_eps=10, device=dev,
                                           consensus=sched))
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
        print(s.getvalue(), flush=True)
    same = all(np.array_equal(res["synchronous"][t], res["reference"][t]) for t in range(8))
    print(f"schedules bit-identical at eps 10: {same}")


if __name__ == "__main__":
    main()
