"""BASELINE config c1 as one launch (dl_consensus_gd) against the synchronous restatement of the
reference's Titanic consensus GD (oracle/mixer_ref.consensus_gd, itself pinned bit for bit to the
reference's 4000-step asyncio run) and against that run's golden final weights.  The gradient's
dot products sum in a different order than numpy's BLAS, so the weights agree within 1e-9
relative; the Jacobi iteration counts exactly."""
import numpy as np
import pytest

from oracle import mixer_ref as M

pytestmark = pytest.mark.gpu


def titanic(golden):
    d = golden("titanic.npz")
    nt = int(d["n_test"])
    return d, d["X"][nt:], d["y"][nt:]


@pytest.mark.parametrize("topo_name,eps,iters", [("ring8", 10, 300), ("ring8", 1e-3, 60),
                                                 ("k4", 1e-6, 40), ("grid5", 1e-2, 50)])
def test_matches_synchronous_restatement(golden, cuda, topo_name, eps, iters):
    from distributed_learning_amd import workloads
    _, X, y = titanic(golden)
    topo = {"ring8": [(i, (i + 1) % 8) for i in range(8)],
            "k4": [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)],
            "grid5": [(0, 1), (1, 2), (2, 3), (3, 4), (0, 4), (1, 3)]}[topo_name]
    want, ks = M.consensus_gd(topo, X, y, iters, conv_eps=eps)
    got, kd = workloads.consensus_gd_device(topo, X, y, iters, convergence_eps=eps, device=cuda)
    assert list(kd) == ks
    for t in want:
        np.testing.assert_allclose(got[t], want[t], rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("eps,iters", [(10, 300), (1e-3, 60)])
def test_ring8_fast_averaging_weights(golden, cuda, eps, iters):
    """BASELINE c1's wording, "ring with fast-averaging weights": the ring's FDLA weights are one
    weight on every edge, w* = 1 / (3 - cos(2 pi / 8)) (find_optimal_weights, pinned by
    tests/test_fast_averaging.py), mixed as x' = x(1 - 2 w*) + w* sum_j x_j.  The one-launch run
    equals the restatement with that weight (same Jacobi counts, 1e-9 relative)."""
    from distributed_learning_amd import workloads
    from distributed_learning_amd.utils.fast_averaging import find_optimal_weights
    _, X, y = titanic(golden)
    topo = [(i, (i + 1) % 8) for i in range(8)]
    w, _ = find_optimal_weights(topo)
    assert np.allclose(w, w[0]) and abs(w[0] - 1 / (3 - np.cos(2 * np.pi / 8))) < 1e-8
    want, ks = M.consensus_gd(topo, X, y, iters, conv_eps=eps, edge_weight=float(w[0]))
    got, kd = workloads.consensus_gd_device(topo, X, y, iters, convergence_eps=eps, device=cuda,
                                            edge_weight=float(w[0]))
    assert list(kd) == ks
    for t in want:
        np.testing.assert_allclose(got[t], want[t], rtol=1e-9, atol=1e-12)


def test_reference_4000_step_run(golden, cuda):
    """The reference's ring-8, eps = 10, 4000-step asyncio run (golden final weights)."""
    from distributed_learning_amd import workloads
    d, X, y = titanic(golden)
    topo = [(i, (i + 1) % 8) for i in range(8)]
    got, kd = workloads.consensus_gd_device(topo, X, y, int(d["ring8_steps"]), convergence_eps=10,
                                            device=cuda)
    assert (kd == 1).all()
    w = np.stack([got[t] for t in d["ring8_tokens"].tolist()])
    np.testing.assert_allclose(w, d["ring8_eps10_final_w"], rtol=1e-9, atol=1e-12)
    acc = workloads.accuracy(w[0], d["X"][:int(d["n_test"])], d["y"][:int(d["n_test"])])
    assert abs(acc - 0.7978) < 6e-3   # the reference run's agent-0 accuracy


def test_validation(cuda):
    import ctypes

    from distributed_learning_amd import _lib
    lib = _lib.load()
    a = _lib.DlConsensusGdArgs()
    assert lib.dl_consensus_gd(ctypes.byref(a), 10, None) == _lib.DL_ERR_INVALID
