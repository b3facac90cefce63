"""GPU parity of the one-launch Mixer loop (dl_mix_until: rounds, deviation and the stop test of
utils/consensus_simple/mixer.py:18-41 in one workgroup) against the oracle's restatement of the
reference loop (oracle/mixer_ref.mixer_mix) and the reference-generated Mixer fixture.
The iterate must be bit-exact and the round count equal; the deviation trace within 1e-5
relative (np.linalg.norm sums in BLAS order)."""
import logging

import numpy as np
import pytest
import torch

from oracle import mixer_ref as M
from test_mix_gpu import bits, graph_csr

pytestmark = pytest.mark.gpu


def engine():
    from distributed_learning_amd import engine as E
    return E


def run_until(csr, X, times, eps, cuda, max_rounds=4096, inplace=True):
    E = engine()
    W = E.DeviceCsr(csr, cuda)
    Xd = torch.from_numpy(X).to(cuda)
    Y = Xd if inplace else torch.full_like(Xd, float("nan"))
    status = torch.zeros(2, dtype=torch.int32, device=cuda)
    trace = torch.full((max_rounds + 1,), -1.0, device=cuda)
    E.mix_until(W, Xd, Y, times, eps, max_rounds, status, trace)
    n, stopped = status.tolist()
    return Y.cpu().numpy(), n, stopped, trace[:n + 1].cpu().numpy()


CASES = [(5, 617, 3, 1), (8, 1000, 4, 2), (16, 63, 3, 3), (3, 1, 2, 4), (40, 200, 5, 5),
         (2, 4096, 2, 6)]


@pytest.mark.parametrize("n,P,deg,seed", CASES)
@pytest.mark.parametrize("times,eps", [(1, None), (7, None), (0, None), (1, 1e-2), (10, 1e-1),
                                       (0, 5e-2)])
def test_matches_reference_loop(cuda, n, P, deg, seed, times, eps):
    csr = graph_csr(n, deg, seed=seed, weights="uniform")
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, P), dtype=np.float32)
    want, want_n = M.mixer_mix(X, csr.rowptr, csr.col, csr.w, times=times, eps=eps)
    got, n_done, stopped, trace = run_until(csr, X, times, eps, cuda, inplace=seed % 2 == 0)
    assert stopped == 1 and n_done == want_n
    assert np.array_equal(bits(got), bits(want))
    if eps is not None:
        ref, Z = [], X
        ref.append(M.deviation(Z).max())
        for _ in range(n_done):
            Z = M.mix_once(Z, csr.rowptr, csr.col, csr.w)
            ref.append(M.deviation(Z).max())
        np.testing.assert_allclose(trace, ref, rtol=1e-5, atol=1e-12)


def test_round_cap_and_continuation(cuda):
    """A loop cut by max_rounds reports stopped == 0; re-entering with the remaining times
    reproduces the uncut run bit for bit."""
    csr = graph_csr(12, 3, seed=9, weights="uniform")
    X = np.random.default_rng(9).standard_normal((12, 300), dtype=np.float32)
    want, want_n = M.mixer_mix(X, csr.rowptr, csr.col, csr.w, times=5, eps=1e-4)
    assert want_n > 10
    done, Z = 0, X
    while True:
        Z, n, stopped, _ = run_until(csr, Z, max(5 - done, 0), 1e-4, cuda, max_rounds=3)
        done += n
        if stopped:
            break
        assert n == 3
    assert done == want_n and np.array_equal(bits(Z), bits(want))


def test_stop_compares_in_float32(cuda):
    """eps is compared as float32 (numpy >= 2: np.float32 < Python float casts the float):
    a threshold between the deviation and its float32 neighbour above does not stop."""
    csr = graph_csr(4, 2, seed=1, weights="uniform")
    X = np.random.default_rng(1).standard_normal((4, 8), dtype=np.float32)
    _, _, _, tr = run_until(csr, X, 0, 1e9, cuda)
    d0 = np.float32(tr[0])
    eps = float(d0) * (1 + 1e-9)          # float32(eps) == d0: d0 < eps is False in numpy 2
    assert np.float32(eps) == d0 and not (d0 < eps)
    _, n, _, _ = run_until(csr, X, 0, eps, cuda, max_rounds=1)
    assert n == 1


def test_mixer_debug_log_replays_every_evaluation(cuda, monkeypatch):
    """Mixer.mix(times, eps) on the one-launch path logs one 'max deviation' line per
    evaluation (times_done + 1), also across launches cut by the round cap."""
    from distributed_learning_amd.networks import ANNModel
    from distributed_learning_amd.utils.consensus_simple import Mixer
    from distributed_learning_amd.utils.consensus_simple import mixer as mixer_mod

    class Rec(logging.Handler):
        def __init__(self):
            super().__init__()
            self.lines = []

        def emit(self, record):
            self.lines.append(record.getMessage())

    log = logging.getLogger("until")
    log.setLevel(logging.DEBUG)
    h = Rec()
    log.addHandler(h)
    torch.manual_seed(0)
    keys = list("abcdef")
    topo = {k: {keys[(i - 1) % 6]: 0.25, k: 0.5, keys[(i + 1) % 6]: 0.25}
            for i, k in enumerate(keys)}
    init = {k: ANNModel(30, 17, 5).to(cuda) for k in keys}
    X0 = np.stack([torch.cat([p.data.reshape(-1) for p in init[k].parameters()]).cpu().numpy()
                   for k in keys])
    rp, cl, w = M.topology_to_csr(topo)
    want, want_n = M.mixer_mix(X0, rp, cl, w, times=2, eps=1e-3)
    monkeypatch.setattr(mixer_mod.Mixer, "_UNTIL_ROUNDS", 5)
    mixer = Mixer(init, topo, log)
    assert mixer.mix(times=2, eps=1e-3) == want_n
    devs = [ln for ln in h.lines if ln.startswith("Mixer calculate max deviation")]
    assert len(devs) == want_n + 1
    got = np.stack([torch.cat([p.data.reshape(-1) for p in init[k].parameters()]).cpu().numpy()
                    for k in keys])
    assert np.array_equal(bits(got), bits(want))
    log.removeHandler(h)
