"""FDLA weight fixtures for the BASELINE graphs (tests/golden/fdla_*.npz).

The reference computes mixing weights with cvxpy (utils/fast_averaging.py:4-32), which is absent
here and on the GPU box; SURVEY §7 (ii)/(iii) asks for a host solver and committed weight
fixtures.  This script runs ``find_optimal_weights`` (the host barrier SDP) on

  * c2: networkx.random_regular_graph(4, 1024, seed=0)        -> fdla_rr4_1024.npz
  * c4: the 64 x 64 periodic torus (edge-transitive: the best-constant weight is the FDLA
        optimum; the Lanczos subgradient method is run from it as a numerical certificate)
                                                               -> fdla_torus64.npz

and stores the edge list (so the box never regenerates the graph), the per-edge weights in
edge-list order, gamma = ||I - L(w) - 11^T/n||_2 and the best-constant gamma it beats.

    python scripts/make_fdla_fixture.py [c2] [c4]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from distributed_learning_amd.graph import random_regular_edges, torus_edges  # noqa: E402
from distributed_learning_amd.utils.fast_averaging import find_optimal_weights  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


def make(name, edges, method):
    info = {}
    t0 = time.time()
    w, gamma = find_optimal_weights(edges, method=method, info=info, verbose=True)
    dt = time.time() - t0
    print(f"{name}: method={info['method']} gamma={gamma:.12f} best-constant "
          f"{info['gamma_best_constant']:.12f} ({info['iterations']} iterations, {dt:.0f} s)")
    np.savez_compressed(os.path.join(OUT, f"fdla_{name}.npz"), edges=np.asarray(edges, np.int32),
                        w=w, gamma=np.float64(gamma), method=np.asarray(info["method"]),
                        gamma_best_constant=np.float64(info["gamma_best_constant"]),
                        best_constant_weight=np.float64(info["best_constant_weight"]),
                        iterations=np.int64(info["iterations"]), solve_seconds=np.float64(dt))


if __name__ == "__main__":
    which = sys.argv[1:] or ["c2", "c4"]
    if "c2" in which:
        make("rr4_1024", random_regular_edges(4, 1024, seed=0), "sdp")
    if "c4" in which:
        make("torus64", torus_edges(64, 64), "subgradient")
