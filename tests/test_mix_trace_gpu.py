"""GPU parity of the traced multi-round pass (dl_mix_rounds_trace: K rounds in one HBM pass plus
the K per-round max deviations) and of the Mixer.mix(times, eps) path built on it, against the
oracle's restatement of the reference loop (oracle/mixer_ref: mix_once, deviation, mixer_mix;
utils/consensus_simple/mixer.py:18-66).  Iterates bit-exact, round counts equal, deviations
within 1e-5 relative or the mean-rounding noise floor 8 sqrt(P) eps32 max|mean| (the kernel
takes the column mean of the pass input, exact for doubly stochastic W; numpy re-sums it)."""
import logging

import numpy as np
import pytest
import torch

from oracle import cref
from oracle import mixer_ref as M
from test_mix_gpu import bits

pytestmark = pytest.mark.gpu


def E():
    from distributed_learning_amd import engine
    return engine


def rr_csr(n, seed):
    from distributed_learning_amd.graph import (best_constant_weight, from_edge_weights,
                                                random_regular_edges)
    edges = random_regular_edges(4, n, seed=seed)
    w = best_constant_weight(edges, list(range(n)))
    return from_edge_weights(edges, [w] * len(edges), list(range(n)))


def metropolis_csr(n, p, seed):
    """Erdos-Renyi graph (plus a ring, connected) with Metropolis weights: irregular, symmetric,
    doubly stochastic -- the CSR-in-LDS path of the kernel."""
    from distributed_learning_amd.graph import from_edge_weights
    rng = np.random.default_rng(seed)
    es = {(i, (i + 1) % n) for i in range(n)}
    for i in range(n):
        for j in range(i + 1, n):
            if rng.random() < p:
                es.add((i, j))
    edges = sorted((min(a, b), max(a, b)) for a, b in es)
    deg = np.zeros(n, int)
    for a, b in edges:
        deg[a] += 1
        deg[b] += 1
    w = [1.0 / (1 + max(deg[a], deg[b])) for a, b in edges]
    return from_edge_weights(edges, w, list(range(n)))


def noise_floor(X):
    return 8 * np.sqrt(X.shape[1]) * np.finfo(np.float32).eps * np.abs(X.mean(axis=0)).max()


def torus_csr(side):
    from distributed_learning_amd.graph import (best_constant_weight, from_edge_weights,
                                                torus_edges)
    edges = torus_edges(side, side)
    n = side * side
    w = best_constant_weight(edges, list(range(n)))
    return from_edge_weights(edges, [w] * len(edges), list(range(n)))


# rr4 rows run mix_trace_rows_kernel (4 / 2 / 1 agents per thread at 1024 / 300 / 64 agents,
# ragged at 300; 256, 512 and 1024 agents fill every slot: the unguarded FULL instantiations);
# metropolis rows (irregular) the chunk-major planes kernel.  Above 1024 agents the wide kernel
# (one column chunk per step, 2 or 4 agents per thread): rr4 2048 (FULL, CSR in registers), rr4
# 3000 (ragged, 4 per thread), the c4 torus (4096, FULL), sparse Metropolis 1500 (CSR in LDS)
# The one-image kernel (mix_trace_irr_kernel: register head + LDS tail CSR, one 4-column chunk
# per step) takes the rest: Barabasi-Albert 4096 (irregular above 2048 agents, 3-entry head) and
# W that are row- but not column-stochastic at 300 / 1500 / 4096 agents (1 / 2 / 4 per thread;
# every round's column mean reduced from its outputs).
CASES = [("rr4", 64, 4096, 0), ("rr4", 1024, 256, 1), ("metro", 50, 1000, 2),
         ("metro", 7, 4, 3), ("rr4", 16, 65536, 4), ("rr4", 300, 512, 5), ("rr4", 1000, 128, 6),
         ("rr4", 256, 1024, 7), ("rr4", 512, 512, 8), ("rr4", 2048, 256, 9),
         ("rr4", 3000, 128, 10), ("torus", 4096, 256, 11), ("metro_sparse", 1500, 192, 12),
         ("ba", 4096, 256, 13), ("rowstoch", 4096, 128, 14), ("rowstoch", 300, 256, 15),
         ("rowstoch", 1500, 128, 16)]
T_TILED = 16
# the column-tiled layout needs whole tiles: widths that are not a multiple of T run row-major only
LAYOUT_CASES = [(c, lay) for c in CASES for lay in ("rows", "tiled")
                if lay == "rows" or c[2] % T_TILED == 0]


def make(kind, n, seed):
    if kind == "rr4":
        return rr_csr(n, seed)
    if kind == "torus":
        return torus_csr(int(round(n ** 0.5)))
    if kind == "ba":
        from distributed_learning_amd.graph import barabasi_albert_metropolis
        return barabasi_albert_metropolis(n, 2, seed)
    if kind == "rowstoch":
        from test_mix_ragged_gpu import dense_irregular
        return dense_irregular(n, 4, 9, seed, row_stochastic=True)
    return metropolis_csr(n, 3.0 / n if kind == "metro_sparse" else 0.1, seed)


@pytest.mark.parametrize("case,layout", LAYOUT_CASES)
def test_trace_pass_matches_round_by_round(cuda, case, layout):
    kind, n, P, seed = case
    e = E()
    csr = make(kind, n, seed)
    assert csr.doubly_stochastic == (kind != "rowstoch")
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, P), dtype=np.float32)
    W = e.DeviceCsr(csr, cuda)
    Xd = torch.from_numpy(X).to(cuda)
    tiled = None
    if layout == "tiled":
        T = T_TILED
        Xd = e.to_tiled(Xd, T)
        tiled = (P, T)
    Yd = torch.full_like(Xd, float("nan"))
    kmax = e.trace_max_rounds(W, Xd, Yd, tiled=tiled)
    assert kmax >= 4
    K = min(kmax, 23)
    trace = torch.full((K,), -1.0, device=cuda)
    X0 = Xd.clone()
    e.mix_rounds_trace(W, Xd, Yd, K, trace, tiled=tiled)
    assert torch.equal(Xd, X0)                     # the pass input is left intact
    got = (e.from_tiled(Yd, P) if tiled else Yd).cpu().numpy()
    Z, ref, floor = X, [], []
    for _ in range(K):
        Z = M.mix_once(Z, csr.rowptr, csr.col, csr.w)
        ref.append(M.deviation(Z).max())
        floor.append(noise_floor(Z))    # (row-stochastic W: the mean moves every round)
    assert np.array_equal(bits(got), bits(Z))
    np.testing.assert_allclose(trace.cpu().numpy(), ref, rtol=1e-5, atol=max(floor))


@pytest.mark.parametrize("n", [1024, 300])
def test_trace_rows_and_planes_kernels_agree(cuda, monkeypatch, n):
    """The agent-major kernel (default for register-cached regular graphs) and the chunk-major
    planes kernel (DLAMD_TRACE_PLANES=1) give the same bits and traces within rounding."""
    e = E()
    csr = rr_csr(n, 7)
    X = torch.from_numpy(np.random.default_rng(7).standard_normal((n, 1024), dtype=np.float32)).to(cuda)
    W = e.DeviceCsr(csr, cuda)
    out = {}
    for planes in (False, True):
        if planes:
            monkeypatch.setenv("DLAMD_TRACE_PLANES", "1")
        Y = torch.full_like(X, float("nan"))
        K = min(e.trace_max_rounds(W, X, Y), 20)
        tr = torch.empty(K, device=cuda)
        e.mix_rounds_trace(W, X, Y, K, tr)
        out[planes] = (Y.cpu(), tr.cpu())
    assert torch.equal(out[False][0], out[True][0])
    torch.testing.assert_close(out[False][1], out[True][1], rtol=1e-5, atol=1e-6)


def test_trace_plan_rejects_unsupported(cuda):
    from test_mix_gpu import graph_csr
    e = E()
    X = torch.randn(8, 64, device=cuda)
    Y = torch.empty_like(X)
    # random directed neighbours: not doubly stochastic -> the one-image kernel (per-round means)
    assert e.trace_max_rounds(e.DeviceCsr(graph_csr(8, 3, seed=0), cuda), X, Y) == 24
    big = torch.randn(4100, 64, device=cuda)       # above 4096 agents
    assert e.trace_max_rounds(e.DeviceCsr(rr_csr(4100, 0), cuda), big, torch.empty_like(big)) == 0
    # above 2048 agents: register-cached regular graphs keep the double-buffered wide kernel (8
    # rounds), irregular ones the one-image kernel (4 rounds at 4 agents per thread)
    mid = torch.randn(3000, 64, device=cuda)
    assert e.trace_max_rounds(e.DeviceCsr(metropolis_csr(3000, 1.0 / 3000, 1), cuda), mid,
                              torch.empty_like(mid)) == 4
    assert e.trace_max_rounds(e.DeviceCsr(rr_csr(3000, 0), cuda), mid, torch.empty_like(mid)) == 8
    # an irregular graph whose CSR does not fit LDS beside one image: no traced pass
    from test_mix_ragged_gpu import dense_irregular
    dense = dense_irregular(4096, 14, 20, 2)
    assert dense.nnz - 5 * 4096 > 65535 // 8
    assert e.trace_max_rounds(e.DeviceCsr(dense, cuda), torch.randn(4096, 64, device=cuda),
                              torch.empty(4096, 64, device=cuda)) == 0
    W = e.DeviceCsr(rr_csr(8, 0), cuda)
    k = e.trace_max_rounds(W, X, Y)
    with pytest.raises(ValueError, match="rounds must be"):
        e.mix_rounds_trace(W, X, Y, k + 1, torch.empty(k + 1, device=cuda))


class _Rec(logging.Handler):
    def __init__(self):
        super().__init__()
        self.lines = []

    def emit(self, record):
        self.lines.append(record.getMessage())


@pytest.mark.parametrize("times,eps,kmax", [(1, 1e-2, 256), (1, 1e-2, 5), (40, 1e-1, 7),
                                             (3, 5e-1, 4), (1, 1e-4, 64)])
def test_mixer_traced_path_matches_reference_loop(cuda, monkeypatch, times, eps, kmax):
    """Mixer.mix(times, eps) on models too large for the one-workgroup loop goes through the
    traced passes: same round count, same bits, one debug line per evaluation."""
    from distributed_learning_amd import engine
    from distributed_learning_amd.networks import ANNModel
    from distributed_learning_amd.utils.consensus_simple import Mixer
    from distributed_learning_amd.utils.consensus_simple import mixer as mixer_mod
    calls = []
    real = engine.mix_rounds_trace
    monkeypatch.setattr(engine, "mix_rounds_trace",
                        lambda *a, **k: (calls.append(a[3]), real(*a, **k))[1])
    monkeypatch.setattr(mixer_mod.Mixer, "_TRACE_MAX_ROUNDS", kmax)
    log = logging.getLogger("traced")
    log.setLevel(logging.DEBUG)
    h = _Rec()
    log.addHandler(h)
    torch.manual_seed(1)
    n = 24
    keys = [f"agent{i}" for i in range(n)]
    csr = rr_csr(n, 5)
    topo = {}
    for i, k in enumerate(keys):
        row = range(csr.rowptr[i], csr.rowptr[i + 1])
        topo[k] = {keys[csr.col[e]]: float(csr.w[e]) for e in row}
    models = {k: ANNModel(60, 40, 10).to(cuda) for k in keys}
    X0 = np.stack([torch.cat([p.data.reshape(-1) for p in models[k].parameters()]).cpu().numpy()
                   for k in keys])
    assert not engine.until_fits(engine.DeviceCsr(csr, cuda), X0.shape[1])
    rp, cl, w = M.topology_to_csr(topo)
    want, want_n = M.mixer_mix(X0, rp, cl, w, times=times, eps=eps)
    mixer = Mixer(models, topo, log)
    assert mixer.mix(times=times, eps=eps) == want_n
    assert calls, "the traced pass was not used"
    got = np.stack([torch.cat([p.data.reshape(-1) for p in models[k].parameters()]).cpu().numpy()
                    for k in keys])
    assert np.array_equal(bits(got), bits(want))
    devs = [ln for ln in h.lines if ln.startswith("Mixer calculate max deviation")]
    assert len(devs) == want_n + 1
    log.removeHandler(h)


def test_mixer_traced_stop_tie_uses_row_order_mean(cuda):
    """A traced max deviation within rounding of eps is re-evaluated on that round's iterate
    with the row-order (numpy) column mean, so the integer round count Mixer.mix returns is the
    reference loop's (mixer.py:40-41).  The test finds rounds where the traced value and numpy's
    differ by >= 1 ulp while the row-order recheck reproduces numpy's bits, puts eps between the
    two values, and checks the stop round for each such round."""
    from distributed_learning_amd import engine
    from distributed_learning_amd.networks import ANNModel
    from distributed_learning_amd.utils.consensus_simple import Mixer
    torch.manual_seed(3)
    n, K = 24, 24
    keys = [f"agent{i}" for i in range(n)]
    csr = rr_csr(n, 7)
    topo = {k: {keys[csr.col[e]]: float(csr.w[e]) for e in range(csr.rowptr[i], csr.rowptr[i + 1])}
            for i, k in enumerate(keys)}
    init = {k: ANNModel(60, 40, 10) for k in keys}
    X0 = np.stack([torch.cat([p.data.reshape(-1) for p in init[k].parameters()]).numpy()
                   for k in keys])
    P = X0.shape[1]
    rp, cl, w = M.topology_to_csr(topo)
    ref, Z = [], X0
    for _ in range(K):
        Z = M.mix_once(Z, rp, cl, w)
        ref.append(np.float32(M.deviation(Z).max()))
    W = engine.DeviceCsr(csr, cuda)
    Pp = -(-P // 64) * 64
    Xd = torch.nn.functional.pad(torch.from_numpy(X0).to(cuda), (0, Pp - P))
    Yd = torch.empty_like(Xd)
    trace = torch.empty(K, device=cuda)
    engine.mix_rounds_trace(W, Xd, Yd, K, trace)
    traced = [np.float32(v) for v in trace.tolist()]
    m = Mixer({k: init[k].to(cuda) for k in keys}, topo, logging.getLogger("tie"))
    m._dev()
    recheck = [m._recheck_deviation(W, Xd, r + 1, P) for r in range(K)]
    cands = [r for r in range(1, K) if traced[r] != ref[r] and recheck[r] == ref[r]
             and ref[r - 1] > max(traced[r], ref[r])]
    assert cands, "no round where the traced value and numpy's differ"
    for r in cands[:3]:
        lo = min(traced[r], ref[r])
        eps = float(np.nextafter(lo, np.float32(np.inf)))   # lo < eps <= the other one
        _, want_n = M.mixer_mix(X0, rp, cl, w, times=1, eps=eps)
        if ref[r] < eps:
            assert want_n == r + 1      # the reference stops exactly at this round
        models = {k: ANNModel(60, 40, 10).to(cuda) for k in keys}
        for k in keys:
            models[k].load_state_dict(init[k].state_dict())
        got_n = Mixer(models, topo, logging.getLogger("tie")).mix(times=1, eps=eps)
        assert got_n == want_n, (r, traced[r], ref[r], eps)


def test_full_size_c2_gossip_traced_pass(cuda):
    """BASELINE config c2 as pure gossip at full size (1024 agents x 2^20, random 4-regular
    graph, best-constant weights): one traced pass of 24 rounds (Mixer.mix(times, eps)'s device
    path) -- column slices of the final iterate bit-exact against 24 oracle rounds on the slice,
    the pass input left intact, and every round's max deviation against the fused deviation of
    24 single-round launches of the same iterates."""
    from distributed_learning_amd.graph import from_edge_weights, random_regular_edges
    e = E()
    n, P, K = 1024, 1 << 20, 24
    edges = random_regular_edges(4, n, seed=0)
    csr = from_edge_weights(edges, [0.25] * len(edges))
    assert csr.doubly_stochastic
    W = e.DeviceCsr(csr, cuda)
    g = torch.Generator(device=cuda).manual_seed(2)
    X = torch.randn(n, P, device=cuda, generator=g)
    T = 16
    Xt = e.to_tiled(X, T)
    Yt = torch.empty_like(Xt)
    assert e.trace_max_rounds(W, Xt, Yt, tiled=(P, T)) >= K
    trace = torch.full((K,), -1.0, device=cuda)
    X0 = Xt.clone()
    e.mix_rounds_trace(W, Xt, Yt, K, trace, tiled=(P, T))
    torch.cuda.synchronize()
    assert torch.equal(Xt, X0)
    del X0
    Y = e.from_tiled(Yt, P)
    for c0, c1 in [(0, 2048), (P - 2048, P), (500001, 500001 + 771)]:
        Z = X[:, c0:c1].cpu().numpy()
        for _ in range(K):
            Z = cref.mix_round(Z, csr.rowptr, csr.col, csr.w)
        assert np.array_equal(bits(Y[:, c0:c1].cpu().numpy()), bits(Z)), (c0, c1)
    # the same 24 rounds one launch each, with the single-round kernel's fused deviation
    eng = e.GossipEngine(csr, P, device=cuda, X=X)
    ref = []
    for _ in range(K):
        eng.round(deviation=True)
        ref.append(float(eng.dev_max.item()))
    assert torch.equal(eng.rows(), Y)
    floor = 8 * np.sqrt(P) * np.finfo(np.float32).eps * float(X.mean(0).abs().max())
    np.testing.assert_allclose(trace.cpu().numpy(), ref, rtol=1e-5, atol=floor)


def test_full_size_c4_gossip_traced_pass(cuda):
    """BASELINE config c4 (64 x 64 torus, 4096 agents x 2^18, best-constant weights) as
    Mixer.mix(times, eps)'s device path: one traced pass of 8 rounds through the wide kernel
    (column-tiled T = 4, 4 agents per thread, CSR in registers) -- column slices bit-exact
    against 8 oracle rounds, the input intact, and every round's max deviation against the fused
    deviation of 8 single-round launches."""
    e = E()
    n, P, K = 4096, 1 << 18, 8
    csr = torus_csr(64)
    W = e.DeviceCsr(csr, cuda)
    g = torch.Generator(device=cuda).manual_seed(4)
    X = torch.randn(n, P, device=cuda, generator=g)
    T = 4
    Xt = e.to_tiled(X, T)
    Yt = torch.empty_like(Xt)
    assert e.trace_max_rounds(W, Xt, Yt, tiled=(P, T)) == K
    trace = torch.full((K,), -1.0, device=cuda)
    X0 = Xt.clone()
    e.mix_rounds_trace(W, Xt, Yt, K, trace, tiled=(P, T))
    torch.cuda.synchronize()
    assert torch.equal(Xt, X0)
    del X0
    Y = e.from_tiled(Yt, P)
    for c0, c1 in [(0, 512), (P - 512, P), (100001, 100001 + 303)]:
        Z = X[:, c0:c1].cpu().numpy()
        for _ in range(K):
            Z = cref.mix_round(Z, csr.rowptr, csr.col, csr.w)
        assert np.array_equal(bits(Y[:, c0:c1].cpu().numpy()), bits(Z)), (c0, c1)
    eng = e.GossipEngine(csr, P, device=cuda, X=X)
    ref = []
    for _ in range(K):
        eng.round(deviation=True)
        ref.append(float(eng.dev_max.item()))
    assert torch.equal(eng.rows(), Y)
    floor = 8 * np.sqrt(P) * np.finfo(np.float32).eps * float(X.mean(0).abs().max())
    np.testing.assert_allclose(trace.cpu().numpy(), ref, rtol=1e-5, atol=floor)


@pytest.mark.parametrize("times,eps", [(1, 2e-1), (20, 1e-1), (3, 5e-1)])
def test_mixer_traced_path_4096_agents(cuda, monkeypatch, times, eps):
    """Mixer.mix(times, eps) over the c4 torus (4096 models) takes traced passes of 8 rounds
    through the wide kernel: the reference loop's round count and bits, one debug line per
    evaluation (stops inside the first pass, and in later passes)."""
    from distributed_learning_amd import engine
    from distributed_learning_amd.utils.consensus_simple import Mixer
    calls = []
    real = engine.mix_rounds_trace
    monkeypatch.setattr(engine, "mix_rounds_trace",
                        lambda *a, **k: (calls.append(a[3]), real(*a, **k))[1])
    log = logging.getLogger("traced4096")
    log.setLevel(logging.DEBUG)
    h = _Rec()
    log.addHandler(h)
    torch.manual_seed(2)
    csr = torus_csr(64)
    n = csr.n_rows
    topo = {i: {int(csr.col[e]): float(csr.w[e]) for e in range(csr.rowptr[i], csr.rowptr[i + 1])}
            for i in range(n)}
    models = {i: torch.nn.Linear(24, 8).to(cuda) for i in range(n)}
    X0 = np.stack([torch.cat([p.data.reshape(-1) for p in models[i].parameters()]).cpu().numpy()
                   for i in range(n)])
    rp, cl, w = M.topology_to_csr(topo)
    want, want_n = M.mixer_mix(X0, rp, cl, w, times=times, eps=eps)
    assert Mixer(models, topo, log).mix(times=times, eps=eps) == want_n
    assert calls and set(calls) == {8}, calls
    got = np.stack([torch.cat([p.data.reshape(-1) for p in models[i].parameters()]).cpu().numpy()
                    for i in range(n)])
    assert np.array_equal(bits(got), bits(want))
    devs = [ln for ln in h.lines if ln.startswith("Mixer calculate max deviation")]
    assert len(devs) == want_n + 1
    log.removeHandler(h)
