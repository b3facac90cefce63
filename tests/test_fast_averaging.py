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


def test_vertex_order_self_loops_and_explicit_methods():
    edges = [("b", "a"), ("a", "c"), ("c", "c"), ("c", "b")]
    w, g = find_optimal_weights(edges)
    assert w[2] == 0.0 and g < 1
    ring = [(i, (i + 1) % 500) for i in range(500)]
    info = {}
    w, g = find_optimal_weights(ring, method="best_constant", info=info)
    assert info["method"] == "best_constant"             # asked for, and recorded
    assert np.allclose(w, w[0]) and g == pytest.approx(info["gamma_best_constant"], abs=1e-12)
    with pytest.raises(ValueError):
        find_optimal_weights(ring, method="cvxpy")


def test_auto_switches_to_subgradient_and_says_so():
    """Above max_sdp the Lanczos subgradient method runs (never a silent best-constant): it never
    returns worse than the best-constant weights and lands near the SDP optimum."""
    edges = list(nx.connected_watts_strogatz_graph(40, 4, 0.5, seed=3).edges)
    info_sg, info_sdp = {}, {}
    w, g = find_optimal_weights(edges, max_sdp=16, info=info_sg)
    assert info_sg["method"] == "subgradient"
    assert g == pytest.approx(spectral_gamma(edges, w), abs=1e-10)
    assert g <= info_sg["gamma_best_constant"] + 1e-12
    _, g_sdp = find_optimal_weights(edges, info=info_sdp)
    assert info_sdp["method"] == "sdp" and g_sdp <= g + 1e-9
    assert g - g_sdp < 0.5 * (info_sg["gamma_best_constant"] - g_sdp) + 1e-6


def test_edge_transitive_torus_best_constant_is_optimal():
    """On an edge-transitive graph (8 x 8 torus) the SDP optimum is the uniform best-constant
    weight: what makes ``best_constant`` exact for config c4's torus."""
    from distributed_learning_amd.graph import torus_edges
    edges = torus_edges(8, 8)
    info = {}
    w, g = find_optimal_weights(edges, info=info)
    assert info["method"] == "sdp"
    assert g == pytest.approx(info["gamma_best_constant"], abs=1e-7)
    np.testing.assert_allclose(w, info["best_constant_weight"], atol=1e-4)


@pytest.mark.parametrize("name", ["rr4_1024", "torus64"])
def test_committed_config_weights(golden, name):
    """The committed FDLA weights of the BASELINE graphs (scripts/make_fdla_fixture.py): c2's
    random 4-regular 1024-agent graph (barrier SDP) and c4's 64 x 64 torus.  gamma is recomputed
    here from the weights, the c2 weights beat the best constant, and W = I - L(w) is doubly
    stochastic and symmetric."""
    d = golden(f"fdla_{name}.npz")
    edges = [tuple(int(x) for x in e) for e in d["edges"]]
    w = d["w"]
    if name == "rr4_1024":
        assert str(d["method"]) == "sdp"
        assert spectral_gamma(edges, w) == pytest.approx(float(d["gamma"]), abs=1e-9)
        assert float(d["gamma"]) < float(d["gamma_best_constant"]) - 0.015
        assert not np.allclose(w, w[0])                    # genuinely per-edge weights
    else:
        assert float(d["gamma"]) == pytest.approx(float(d["gamma_best_constant"]), abs=1e-12)
    W = from_edge_weights(edges, w).dense()
    np.testing.assert_allclose(W.sum(0), 1, atol=1e-12)
    np.testing.assert_allclose(W, W.T, atol=0)
