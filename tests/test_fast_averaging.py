"""Host fast-averaging solver (reference utils/fast_averaging.py, cvxpy SDP) against the known
answers the reference notebook recorded and the analytic optimum for rings."""
import networkx as nx
import numpy as np
import pytest

from distributed_learning_amd.graph import from_edge_weights
from distributed_learning_amd.utils.fast_averaging import find_optimal_weights, spectral_gamma


def test_notebook_kat(golden):
    nb = golden("notebook_outputs.json")
    w, g = find_optimal_weights([tuple(e) for e in nb["fa_kat_edges"]])
    np.testing.assert_allclose(w, nb["fa_kat_w"], atol=1e-6)
    assert g == pytest.approx(nb["fa_kat_gamma"], abs=1e-8)


def test_hexagonal_lattice(golden):
    nb = golden("notebook_outputs.json")
    edges = list(nx.hexagonal_lattice_graph(2, 2, periodic=True).edges)
    _, g = find_optimal_weights(edges)
    assert g == pytest.approx(nb["fa_hex_lattice_2_2_periodic_gamma"], abs=1e-7)


def test_ring_analytic(golden):
    nb = golden("notebook_outputs.json")
    w, g = find_optimal_weights([(i, (i + 1) % 8) for i in range(8)])
    np.testing.assert_allclose(w, nb["fa_ring8_w"], atol=1e-7)
    assert g == pytest.approx(nb["fa_ring8_gamma"], abs=1e-8)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_optimality_certificate(seed):
    """The returned gamma is the spectral radius of W - J/n, and no uniform weight beats it."""
    g = nx.connected_watts_strogatz_graph(16, 4, 0.5, seed=seed)
    edges = list(g.edges)
    w, gamma = find_optimal_weights(edges)
    assert gamma == pytest.approx(spectral_gamma(edges, w), abs=1e-12)
    best_uniform = min(spectral_gamma(edges, [a] * len(edges)) for a in np.linspace(0.01, 0.6, 120))
    assert gamma <= best_uniform + 1e-9
    # the mixing matrix built from these weights is doubly stochastic
    W = from_edge_weights(edges, w).dense()
    np.testing.assert_allclose(W.sum(0), 1, atol=1e-12)
    np.testing.assert_allclose(W.sum(1), 1, atol=1e-12)


def test_vertex_order_self_loops_and_large_fallback():
    edges = [("b", "a"), ("a", "c"), ("c", "c"), ("c", "b")]
    w, g = find_optimal_weights(edges)
    assert w[2] == 0.0 and g < 1
    ring = [(i, (i + 1) % 500) for i in range(500)]
    w, g = find_optimal_weights(ring, max_dense=400)          # best-constant fallback
    assert np.allclose(w, w[0]) and g < 1
