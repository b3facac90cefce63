"""GPU parity of the multi-round kernel (dl_mix_rounds: K rounds on LDS-resident tiles, one HBM
pass) against K one-round launches, the reference-generated fixtures and the Mixer drop-in.
Mixing must be bit-exact; the final deviation within 1e-5 relative."""
import numpy as np
import pytest
import torch

from oracle import mixer_ref as M
from test_mix_gpu import bits, check_dev, dev_floor, graph_csr

pytestmark = pytest.mark.gpu


def engine():
    from distributed_learning_amd import engine as E
    return E


@pytest.mark.parametrize("case,rounds", [("a", [10, 200]), ("b", [10])])
def test_reference_fixture_in_one_pass(golden, cuda, case, rounds):
    """X after 10 / 200 rounds of the reference's Mixer._mix_params_once, from one launch."""
    from distributed_learning_amd.graph import Csr
    E = engine()
    d = golden("mix_rr4_n64.npz")
    csr = Csr(d[f"{case}_rowptr"], d[f"{case}_cols"], d[f"{case}_w"])
    for r in rounds:
        eng = E.GossipEngine(csr, d[f"{case}_X0"].shape[1], device=cuda,
                             X=torch.from_numpy(d[f"{case}_X0"]).to(cuda))
        plan = E.rounds_plan(eng.W, eng.X, eng.Y, tiled=(eng.P, eng.T))
        assert plan is not None and plan["path"] == 3
        eng.rounds(r)
        torch.cuda.synchronize()
        assert np.array_equal(bits(eng.rows().cpu().numpy()), bits(d[f"{case}_X{r}"])), r


@pytest.mark.parametrize("n,P,deg,layout", [(64, 4096, 4, "tiled"), (1024, 4096, 4, "tiled"),
                                            (100, 1024, 5, "rows"), (256, 2048, 8, "tiled"),
                                            (3, 64, 2, "rows"), (1500, 512, 3, "tiled")])
@pytest.mark.parametrize("sgd", [False, True])
def test_k_rounds_equal_k_launches(cuda, n, P, deg, layout, sgd):
    E = engine()
    rng = np.random.default_rng(n + P)
    csr = graph_csr(n, deg, seed=n)
    X = rng.standard_normal((n, P), dtype=np.float32)
    G = rng.standard_normal((n, P), dtype=np.float32) if sgd else None
    K = 7
    a = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda), layout=layout)
    b = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda), layout=layout)
    Ga = a.layout_like(torch.from_numpy(G).to(cuda)) if sgd else None
    tiled = (a.P, a.T) if layout == "tiled" else None
    assert E.rounds_plan(a.W, a.X, a.Y, tiled=tiled) is not None
    a.rounds(K, G=Ga, lr=0.01)
    for i in range(K):
        b.round(G=Ga if i == 0 else None, lr=0.01 if i == 0 else 0.0)
    torch.cuda.synchronize()
    assert np.array_equal(bits(a.rows().cpu().numpy()), bits(b.rows().cpu().numpy()))


@pytest.mark.parametrize("n,P", [(1024, 2048), (4096, 512)])
@pytest.mark.parametrize("nt", ["0", "1"])
@pytest.mark.parametrize("dev", [False, True])
def test_full_slot_variants_both_store_kinds(cuda, monkeypatch, n, P, nt, dev):
    """N = KV * SLOTS on a degree-4 regular graph (c2's 1024 agents at 4 chunks, c4's 4096 at
    1): the unguarded mix_multi_kernel instantiations (MODE 1 plain / 2 non-temporal stores,
    chosen by DLAMD_NT_STORE here, by the output size in production) against K one-round
    launches with the local step before the first round, and the fused final deviation."""
    from distributed_learning_amd.graph import best_constant_weight, random_regular_edges, \
        uniform_weights
    monkeypatch.setenv("DLAMD_NT_STORE", nt)
    E = engine()
    edges = random_regular_edges(4, n, seed=n)
    csr = uniform_weights(edges, best_constant_weight(edges))
    assert csr.doubly_stochastic and csr.shared_row_weights
    rng = np.random.default_rng(n + int(nt))
    X = rng.standard_normal((n, P), dtype=np.float32)
    G = rng.standard_normal((n, P), dtype=np.float32)
    a = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda), layout="tiled")
    b = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda), layout="tiled")
    Ga = a.layout_like(torch.from_numpy(G).to(cuda))
    assert E.rounds_plan(a.W, a.X, a.Y, tiled=(a.P, a.T)) is not None
    K = 6
    mean = torch.empty(P, device=cuda)
    a.rounds(K, G=Ga, lr=0.01, deviation=dev, mean=mean if dev else None)
    for i in range(K):
        b.round(G=Ga if i == 0 else None, lr=0.01 if i == 0 else 0.0)
    torch.cuda.synchronize()
    Y = a.rows().cpu().numpy()
    assert np.array_equal(bits(Y), bits(b.rows().cpu().numpy()))
    if dev:
        check_dev(Y, a.dev_sq.cpu().numpy(), float(a.dev_max.item()), mean.cpu().numpy())


@pytest.mark.parametrize("layout", ["tiled", "rows"])
def test_final_deviation_doubly_stochastic(cuda, layout):
    from distributed_learning_amd.graph import best_constant_weight, random_regular_edges, \
        uniform_weights
    E = engine()
    n, P = 512, 8192
    edges = random_regular_edges(4, n, seed=1)
    csr = uniform_weights(edges, best_constant_weight(edges))
    assert csr.doubly_stochastic and csr.shared_row_weights
    rng = np.random.default_rng(7)
    X = rng.standard_normal((n, P), dtype=np.float32)
    eng = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda), layout=layout)
    mean = torch.empty(P, device=cuda)
    eng.rounds(5, deviation=True, mean=mean)
    torch.cuda.synchronize()
    Y = eng.rows().cpu().numpy()
    Yw = X
    for _ in range(5):
        Yw = M.mix_once(Yw, csr.rowptr, csr.col, csr.w)
    assert np.array_equal(bits(Y), bits(Yw))
    check_dev(Y, eng.dev_sq.cpu().numpy(), float(eng.dev_max.item()), mean.cpu().numpy())


def test_torus_4096_csr_in_registers(cuda):
    """c4's 64 x 64 torus: with the CSR in registers two 4096-agent tile images fit LDS."""
    from distributed_learning_amd.graph import best_constant_weight, torus_edges, uniform_weights
    E = engine()
    edges = torus_edges(64, 64)
    csr = uniform_weights(edges, best_constant_weight(edges))
    rng = np.random.default_rng(2)
    X = rng.standard_normal((4096, 256), dtype=np.float32)
    a = E.GossipEngine(csr, 256, device=cuda, X=torch.from_numpy(X).to(cuda))
    assert E.rounds_plan(a.W, a.X, a.Y, tiled=(a.P, a.T)) is not None
    b = E.GossipEngine(csr, 256, device=cuda, X=torch.from_numpy(X).to(cuda))
    a.rounds(3, deviation=True)
    for i in range(3):
        b.round(deviation=i == 2)
    torch.cuda.synchronize()
    assert torch.equal(a.X, b.X)
    torch.testing.assert_close(a.dev_sq, b.dev_sq, rtol=1e-5, atol=0)


def test_unsupported_falls_back_to_single_rounds(cuda):
    """6000 agents (general CSR): two tile images do not fit LDS -> k one-round launches."""
    E = engine()
    csr = graph_csr(6000, 3, seed=5)
    rng = np.random.default_rng(2)
    X = rng.standard_normal((6000, 64), dtype=np.float32)
    a = E.GossipEngine(csr, 64, device=cuda, X=torch.from_numpy(X).to(cuda), layout="rows")
    assert E.rounds_plan(a.W, a.X, a.Y) is None
    b = E.GossipEngine(csr, 64, device=cuda, X=torch.from_numpy(X).to(cuda), layout="rows")
    a.rounds(3)
    for _ in range(3):
        b.round()
    torch.cuda.synchronize()
    assert torch.equal(a.X, b.X)


def test_mixer_times_uses_one_pass(cuda):
    """Mixer.mix(times=K) with eps=None on models too large for the one-workgroup loop
    (dl_mix_until): one dl_mix_rounds pass over padded rows, equal to the reference fold applied
    K times to the flattened models."""
    import logging

    from distributed_learning_amd.networks import ANNModel
    from distributed_learning_amd.utils.consensus_simple import Mixer
    torch.manual_seed(0)
    keys = ["a", "b", "c", "d", "e"]
    models = {k: ANNModel(300, 40, 5).to(cuda) for k in keys}
    topo = {"a": {"a": 0.5, "b": 0.25, "e": 0.25}, "b": {"b": 0.5, "a": 0.25, "c": 0.25},
            "c": {"c": 0.5, "b": 0.25, "d": 0.25}, "d": {"d": 0.5, "c": 0.25, "e": 0.25},
            "e": {"e": 0.5, "d": 0.25, "a": 0.25}}
    X0 = np.stack([torch.cat([p.data.reshape(-1) for p in models[k].parameters()]).cpu().numpy()
                   for k in keys])
    rp, cl, w = M.topology_to_csr(topo)
    from distributed_learning_amd import engine as E
    from distributed_learning_amd.graph import from_topology
    assert not E.until_fits(E.DeviceCsr(from_topology(topo), cuda), X0.shape[1])
    want = X0
    for _ in range(9):
        want = M.mix_once(want, rp, cl, w)
    mixer = Mixer(models, topo, logging.getLogger("t"))
    assert mixer.mix(times=9) == 9
    got = np.stack([torch.cat([p.data.reshape(-1) for p in models[k].parameters()]).cpu().numpy()
                    for k in keys])
    assert np.array_equal(bits(got), bits(want))


def test_lds_slot_order_is_transparent(cuda):
    """An engine holding its rows in an LDS slot order (graph.lds_slot_order) gives every agent
    the same bits as the agent-order engine, one round or K rounds."""
    from distributed_learning_amd.graph import (best_constant_weight, lds_conflicts,
                                                lds_slot_order, random_regular_edges,
                                                uniform_weights)
    E = engine()
    n, P = 1024, 2048
    edges = random_regular_edges(4, n, seed=0)
    csr = uniform_weights(edges, best_constant_weight(edges), list(range(n)))
    order, c0, c1 = lds_slot_order(csr, 4, moves=20000)
    assert c1 < c0 and lds_conflicts(csr, 4, order) == c1
    rng = np.random.default_rng(3)
    X = torch.from_numpy(rng.standard_normal((n, P), dtype=np.float32)).to(cuda)
    G = torch.from_numpy(rng.standard_normal((n, P), dtype=np.float32)).to(cuda)
    a = E.GossipEngine(csr, P, device=cuda, X=X)
    b = E.GossipEngine(csr, P, device=cuda, X=X, order=order)
    a.round(G=a.layout_like(G), lr=0.1, deviation=True)
    b.round(G=b.layout_like(G), lr=0.1, deviation=True)
    a.rounds(9, deviation=True)
    b.rounds(9, deviation=True)
    torch.cuda.synchronize()
    assert torch.equal(a.rows(), b.rows())
    torch.testing.assert_close(a.agent_dev_sq(), b.agent_dev_sq(), rtol=1e-5, atol=0)


def test_lds_slot_order_traced_is_transparent(cuda):
    """The traced pass (chunk-major images, one agent per lane) under its own slot order
    (lds_slot_order with chunks = 1): same bits per agent as the agent-order engine, and the
    same per-round max deviations up to the mean's summation order."""
    from distributed_learning_amd.graph import (best_constant_weight, lds_conflicts,
                                                lds_slot_order, random_regular_edges,
                                                uniform_weights)
    E = engine()
    n, P = 1024, 4096
    edges = random_regular_edges(4, n, seed=0)
    csr = uniform_weights(edges, best_constant_weight(edges), list(range(n)))
    order, c0, c1 = lds_slot_order(csr, 1, moves=20000)
    assert c1 < c0 and lds_conflicts(csr, 1, order) == c1
    rng = np.random.default_rng(5)
    X = torch.from_numpy(rng.standard_normal((n, P), dtype=np.float32)).to(cuda)
    a = E.GossipEngine(csr, P, device=cuda, X=X)
    b = E.GossipEngine(csr, P, device=cuda, X=X, order=order)
    K = min(12, a.trace_max_rounds())
    assert K >= 1 and b.trace_max_rounds() >= K
    ta = torch.empty(K, dtype=torch.float32, device=cuda)
    tb = torch.empty(K, dtype=torch.float32, device=cuda)
    a.rounds_traced(K, ta)
    b.rounds_traced(K, tb)
    torch.cuda.synchronize()
    assert torch.equal(a.rows(), b.rows())
    torch.testing.assert_close(ta, tb, rtol=1e-5, atol=1e-6)


def test_mixer_times_slot_order_bits(cuda, monkeypatch):
    """Mixer.mix(times=K), eps=None, on 1024 agents of a random 4-regular graph (small models, so
    the multi-round pass runs 16-column tiles, 4 float4 chunks per row, where bank conflicts
    matter): the rows go to the device in dl_lds_slot_order's order (not the identity), the
    multi-round pass really runs on that ordered CSR, and every model ends with the reference
    fold's bits; a second call reuses the cached order.  A fractional ``times`` runs
    ceil(times) rounds, as the reference's ``times_done >= times`` loop does."""
    import logging

    from test_mix_trace_gpu import rr_csr

    from distributed_learning_amd import engine as E
    from distributed_learning_amd.networks import ANNModel
    from distributed_learning_amd.utils.consensus_simple import Mixer
    from distributed_learning_amd.utils.consensus_simple import mixer as mixer_mod
    torch.manual_seed(2)
    n = 1024
    keys = [f"agent{i}" for i in range(n)]
    csr = rr_csr(n, 9)
    topo = {}
    for i, k in enumerate(keys):
        topo[k] = {keys[csr.col[e]]: float(csr.w[e]) for e in range(csr.rowptr[i], csr.rowptr[i + 1])}
    models = {k: ANNModel(8, 4, 2).to(cuda) for k in keys}
    X0 = np.stack([torch.cat([p.data.reshape(-1) for p in models[k].parameters()]).cpu().numpy()
                   for k in keys])
    rp, cl, w = M.topology_to_csr(topo)
    want = X0
    for _ in range(7 + 3):
        want = M.mix_once(want, rp, cl, w)
    calls = []
    real = E.mix_rounds

    def spy(W, X, Y, rounds, *a, **kw):
        calls.append((W, rounds))
        return real(W, X, Y, rounds, *a, **kw)
    monkeypatch.setattr(mixer_mod._engine, "mix_rounds", spy)
    mixer = Mixer(models, topo, logging.getLogger("t"))
    assert mixer.mix(times=7) == 7
    ordered = mixer._ordered
    assert ordered is not None and ordered[3] is not None and ordered[3] != keys
    assert calls and calls[-1] == (ordered[2], 7)          # the pass ran on the ordered CSR
    assert mixer.mix(times=2.5) == 3                        # ceil, like the reference loop
    assert mixer._ordered is ordered and calls[-1] == (ordered[2], 3)
    got = np.stack([torch.cat([p.data.reshape(-1) for p in models[k].parameters()]).cpu().numpy()
                    for k in keys])
    assert np.array_equal(bits(got), bits(want))


def test_mixer_slot_order_skipped_when_it_cannot_pay(cuda):
    """No slot-order search when the multi-round pass will not run (an irregular graph) or the
    graph is small: the Mixer keeps topology order and caches that decision."""
    import logging

    from distributed_learning_amd.networks import ANNModel
    from distributed_learning_amd.utils.consensus_simple import Mixer
    torch.manual_seed(3)
    keys = [f"a{i}" for i in range(80)]
    topo = {k: {k: 0.5, keys[(i + 1) % 80]: 0.25, keys[(i - 1) % 80]: 0.25} for i, k in
            enumerate(keys)}
    topo[keys[0]] = {keys[0]: 0.4, keys[1]: 0.2, keys[79]: 0.2, keys[40]: 0.2}   # irregular
    topo[keys[40]] = {keys[40]: 0.3, keys[41]: 0.25, keys[39]: 0.25, keys[0]: 0.2}
    models = {k: ANNModel(60, 40, 10).to(cuda) for k in keys}
    mixer = Mixer(models, topo, logging.getLogger("t"))
    assert mixer.mix(times=4) == 4
    assert mixer._ordered is not None and mixer._ordered[3] is None
