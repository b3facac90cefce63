"""Plan path 5: irregular graphs of thousands of agents whose CSR does not fit LDS beside a column
tile of every agent (per-edge weights: 4 B weight + 2 B id per entry).  The tile kernel keeps
each row's first min(min_row_nnz, 5) CSR entries in registers and stages only the rest in LDS
(fp32 weight + u16 row per entry), so the round still streams X, G and X' once instead of taking the gather
kernel.  The reference's Mixer takes any dict-of-dicts topology (utils/consensus_simple/
mixer.py:43-49); the fold order is the row's CSR order, head then tail, so the result is the
reference's left fold bit for bit."""
import numpy as np
import pytest
import torch

from oracle import cref

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def eng_mod():
    from distributed_learning_amd import engine
    return engine


def check_dev(Y, dev_sq, dev_max, mean=None):
    want = cref.deviation_sq(Y)
    m = cref.column_mean(Y)
    floor = 8 * np.sqrt(Y.shape[1]) * np.finfo(np.float32).eps * np.abs(m).max()
    d_got, d_want = np.sqrt(dev_sq), np.sqrt(want)
    assert np.all(np.abs(d_got - d_want) <= 1e-5 * d_want + floor)
    assert abs(dev_max - d_want.max()) <= 1e-5 * d_want.max() + floor
    if mean is not None:
        np.testing.assert_allclose(mean, m, rtol=1e-5, atol=1e-6 * np.abs(m).max())


def ba(n, m, seed):
    from distributed_learning_amd.graph import barabasi_albert_metropolis
    return barabasi_albert_metropolis(n, m, seed)


def dense_irregular(n, lo, hi, seed, row_stochastic=False):
    """Every agent on a ring (degree 2) plus random extra neighbours up to degree lo..hi,
    Metropolis weights (or, row_stochastic, random positive weights normalised per row: W is
    then not doubly stochastic and the fused deviation takes its second LDS pass)."""
    from distributed_learning_amd.graph import Csr
    rng = np.random.default_rng(seed)
    adj = [set() for _ in range(n)]
    for i in range(n):
        adj[i].add((i + 1) % n)
        adj[(i + 1) % n].add(i)
    target = rng.integers(lo, hi + 1, n)
    for i in range(n):
        while len(adj[i]) < target[i]:
            j = int(rng.integers(n))
            if j != i:
                adj[i].add(j)
                adj[j].add(i)
    rowptr, col, w = [0], [], []
    for i in range(n):
        nb = sorted(adj[i], key=lambda j: (j * 7919 + i) % n)   # not sorted by id
        if row_stochastic:
            ws = list(rng.uniform(0.5, 1.5, len(nb) + 1))
            tot = sum(ws)
            ws = [x / tot for x in ws]
            pos = int(rng.integers(len(nb) + 1))   # the self entry anywhere in the row
            ids = nb[:pos] + [i] + nb[pos:]
        else:
            mw = [1.0 / (1.0 + max(len(adj[i]), len(adj[j]))) for j in nb]
            ids, ws = [i] + nb, [1.0 - sum(mw)] + mw
        col.extend(ids)
        w.extend(ws)
        rowptr.append(len(col))
    return Csr(rowptr, col, w, keys=list(range(n)))


CASES = {
    # name: (graph builder, register head the planner must pick, forced)
    "ba2_4096": (lambda: ba(4096, 2, 1), 3, False),   # the fixture-B construction at c4 scale
    # a tree (leaves have 2 entries): its CSR (72 KiB) fits LDS beside the tile, and path 5
    # still runs it (irregular, > 2048 agents: 430 vs 250 rounds/s for path 1's CSR loop)
    "ba1_4096": (lambda: ba(4096, 1, 2), 2, False),
    "deg5to9_4096": (lambda: dense_irregular(4096, 4, 8, 3), 5, False),
    "deg9to12_2048": (lambda: dense_irregular(2048, 8, 11, 4), 5, False),   # 2 rows per thread
    "ba2_3001": (lambda: ba(3001, 2, 5), 3, False),   # ragged last row pass (CSR fits LDS)
    # 2048 agents, CSR fits LDS beside a 2-chunk tile: path 5 only when forced
    "ba2_2048": (lambda: ba(2048, 2, 6), 3, True),
    # a 3-entry head whose tail fits LDS at 6 B per entry but not at 8 B (the split format)
    "deg2to7_4096": (lambda: rim(4096, 2, 7, 1), 3, False),
}


def rim(n, lo, hi, seed):
    from distributed_learning_amd.graph import random_irregular_metropolis
    return random_irregular_metropolis(n, lo, hi, seed)


@pytest.mark.parametrize("layout", ["tiled", "rows"])
@pytest.mark.parametrize("case", sorted(CASES))
def test_register_head_lds_tail(cuda, monkeypatch, case, layout):
    """Fused local step + mix + deviation through path 5: bit-exact with the oracle's CSR-order
    fold, deviation within 1e-5; the forced gather kernel gives the same bits."""
    E = eng_mod()
    build, head, forced = CASES[case]
    if forced:
        monkeypatch.setenv("DLAMD_FORCE_REG", "1")
    csr = build()
    n = csr.n_rows
    assert not csr.uniform_row_nnz and csr.min_row_nnz >= head
    P = 1024 + 32
    rng = np.random.default_rng(n + head)
    X = rng.standard_normal((n, P), dtype=np.float32)
    G = rng.standard_normal((n, P), dtype=np.float32)
    want = cref.mix_round(X, csr.rowptr, csr.col, csr.w, G=G, lr=0.02)
    eng = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda), layout=layout)
    plan = eng.plan()
    assert plan["path"] == 5 and plan["tile_cols"] == 4, plan
    ntail = csr.nnz - head * n
    assert plan["lds_bytes"] >= n * 16 + 6 * ntail
    # 8-byte {weight, row} pairs whenever they fit LDS (heads < 5), else 6 B per entry
    pairs = head < 5 and n * 16 + 256 + 8 * ntail <= 163840
    assert (plan["lds_bytes"] >= n * 16 + 8 * ntail) == pairs, (plan, ntail)
    mean = torch.empty(P, device=cuda)
    eng.round(G=eng.layout_like(torch.from_numpy(G).to(cuda)), lr=0.02, deviation=True, mean=mean)
    torch.cuda.synchronize()
    assert np.array_equal(bits(eng.rows().cpu().numpy()), bits(want))
    check_dev(want, eng.agent_dev_sq().cpu().numpy(), float(eng.dev_max.item()),
              mean.cpu().numpy())
    if head < 5:
        # the result above ran with the leading rows' tails folded four column lanes each
        # (dl_mix_args.n_hub_rows: every leading row with a tail, up to 256)
        assert 0 < eng.W.hub_rows <= 256, eng.W.hub_rows
    # plain mix (no local step, no deviation) through the same path, rows in agent order
    # instead of the engine's default row-length order: the same bits
    eng2 = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda), layout=layout,
                          order=None)
    assert eng2.plan()["path"] == 5 and eng2.order is None
    eng2.round()
    torch.cuda.synchronize()
    assert np.array_equal(bits(eng2.rows().cpu().numpy()),
                          bits(cref.mix_round(X, csr.rowptr, csr.col, csr.w)))
    if layout == "rows" and case == "ba2_4096":
        monkeypatch.setenv("DLAMD_FORCE_GATHER", "1")
        W = E.DeviceCsr(csr, cuda)
        assert E.plan_shape(W, P)["path"] == 2
        Y = torch.empty(n, P, device=cuda)
        E.mix_round(W, torch.from_numpy(X).to(cuda), Y, G=torch.from_numpy(G).to(cuda), lr=0.02)
        torch.cuda.synchronize()
        assert np.array_equal(bits(Y.cpu().numpy()), bits(want))


def test_row_stochastic_two_pass_deviation(cuda):
    """A W that is row- but not column-stochastic, the self entry at varying row positions: the
    fused deviation cannot take the mean from the inputs and re-mixes the tile in a second LDS
    pass (head + tail again); same bits, exact-mean deviation."""
    E = eng_mod()
    csr = dense_irregular(4096, 4, 9, 7, row_stochastic=True)
    assert not csr.doubly_stochastic and csr.min_row_nnz >= 5
    P = 512
    rng = np.random.default_rng(11)
    X = rng.standard_normal((4096, P), dtype=np.float32)
    eng = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda))
    assert eng.plan()["path"] == 5
    mean = torch.empty(P, device=cuda)
    eng.round(deviation=True, mean=mean)
    torch.cuda.synchronize()
    want = cref.mix_round(X, csr.rowptr, csr.col, csr.w)
    assert np.array_equal(bits(eng.rows().cpu().numpy()), bits(want))
    check_dev(want, eng.agent_dev_sq().cpu().numpy(), float(eng.dev_max.item()),
              mean.cpu().numpy())


@pytest.mark.parametrize("rounds", [1, 10])
def test_reference_fixture_b_through_path5(cuda, golden, monkeypatch, rounds):
    """The reference-run fixture B (Barabasi-Albert 64 agents, Metropolis weights, string keys,
    `Mixer._mix_params_once` snapshots) forced through the register-head + LDS-tail kernel
    (DLAMD_FORCE_REG=1; at 64 agents the CSR would fit LDS): bit-identical after 1 and 10
    rounds.  Fixture A (random 4-regular, uniform weights) likewise through path 4."""
    from distributed_learning_amd.graph import Csr
    E = eng_mod()
    d = golden("mix_rr4_n64.npz")
    monkeypatch.setenv("DLAMD_FORCE_REG", "1")
    for tag, path in (("b", 5), ("a", 4)):
        csr = Csr(d[f"{tag}_rowptr"], d[f"{tag}_cols"], d[f"{tag}_w"])
        X0 = d[f"{tag}_X0"]
        for layout in ("tiled", "rows"):
            eng = E.GossipEngine(csr, X0.shape[1], device=cuda,
                                 X=torch.from_numpy(X0).to(cuda), layout=layout)
            assert eng.plan()["path"] == path, (tag, layout, eng.plan())
            if path == 5:
                assert eng.W.hub_rows > 0   # the leading rows' tails on four lanes each
            for _ in range(rounds):
                eng.round()
            torch.cuda.synchronize()
            assert np.array_equal(bits(eng.rows().cpu().numpy()), bits(d[f"{tag}_X{rounds}"])), \
                (tag, layout)


@pytest.mark.parametrize("hubs", [0, 5, 64])
def test_fixture_b_hub_row_counts(cuda, golden, monkeypatch, hubs):
    """dl_mix_args.n_hub_rows (DLAMD_HUB_ROWS override) only moves which lanes fold the leading
    rows' LDS tails (one column each, CSR order): none, some, and every row of fixture B --
    including rows whose tail is empty -- give the reference's bits after 10 rounds."""
    from distributed_learning_amd.graph import Csr
    E = eng_mod()
    d = golden("mix_rr4_n64.npz")
    monkeypatch.setenv("DLAMD_FORCE_REG", "1")
    monkeypatch.setenv("DLAMD_HUB_ROWS", str(hubs))
    csr = Csr(d["b_rowptr"], d["b_cols"], d["b_w"])
    X0 = d["b_X0"]
    eng = E.GossipEngine(csr, X0.shape[1], device=cuda, X=torch.from_numpy(X0).to(cuda))
    assert eng.plan()["path"] == 5 and eng.W.hub_rows == hubs
    for _ in range(10):
        eng.round()
    torch.cuda.synchronize()
    assert np.array_equal(bits(eng.rows().cpu().numpy()), bits(d["b_X10"]))


def test_plan_csr_reports_path5_and_refuses_bad_promise(cuda):
    """dl_mix_plan_csr sees min_row_nnz (dl_mix_plan_shape assumes uniform rows and reports the
    gather path for the same sizes); a min_row_nnz above nnz / n_rows is refused."""
    import ctypes
    from distributed_learning_amd import _lib
    E = eng_mod()
    csr = ba(4096, 2, 1)
    W = E.DeviceCsr(csr, cuda)
    assert E.plan_shape(W, 1 << 18, tile_cols=-1)["path"] == 5
    lib = _lib.load()
    pl = _lib.DlMixPlan()
    _lib.check(lib.dl_mix_plan_shape(4096, 0, 1 << 18, csr.nnz, 0, 0, 1, 0, ctypes.byref(pl)),
               "plan")
    assert pl.path == 2
    W.min_row_nnz = csr.nnz // 4096 + 1
    with pytest.raises(Exception):
        Y = torch.empty(4096, 64, device=cuda)
        E.mix_round(W, torch.zeros(4096, 64, device=cuda), Y)


@pytest.mark.parametrize("times,eps", [(1, 0.5), (2, None)])
def test_mixer_4096_irregular_models(cuda, times, eps):
    """The drop-in Mixer over 4096 models on the Barabasi-Albert graph (the reference's
    dict-of-dicts topology, mixer.py:43-49): the round loop runs on a column-tiled copy of X
    through plan path 5 -- the reference loop's round count and bits (mixer.py:18-41)."""
    import logging
    from oracle import mixer_ref as M
    from distributed_learning_amd.utils.consensus_simple import Mixer
    from distributed_learning_amd.utils.consensus_simple import mixer as mixer_mod
    from distributed_learning_amd import engine as E
    csr = ba(4096, 2, 3)
    n = csr.n_rows
    topo = {i: {int(csr.col[e]): float(csr.w[e]) for e in range(csr.rowptr[i], csr.rowptr[i + 1])}
            for i in range(n)}
    torch.manual_seed(5)
    models = {i: torch.nn.Linear(24, 8).to(cuda) for i in range(n)}
    X0 = np.stack([torch.cat([p.data.reshape(-1) for p in models[i].parameters()]).cpu().numpy()
                   for i in range(n)])
    rp, cl, w = M.topology_to_csr(topo)
    want, want_n = M.mixer_mix(X0, rp, cl, w, times=times, eps=eps)
    m = Mixer(models, topo, logging.getLogger("ba4096"))
    W = m._device_csr()
    assert m._loop_tile_cols(W, X0.shape[1]) == 4
    assert E.plan_shape(W, X0.shape[1], tile_cols=4)["path"] == 5
    assert m.mix(times=times, eps=eps) == want_n
    got = np.stack([torch.cat([p.data.reshape(-1) for p in models[i].parameters()]).cpu().numpy()
                    for i in range(n)])
    assert np.array_equal(bits(got), bits(want))


def test_wrong_min_row_nnz_promise_stays_in_bounds(cuda):
    """dlamd.h: a wrong dl_csr.min_row_nnz promise gives wrong, never out-of-bounds, results.
    Here two rows (one in the middle, the last) have 2 entries while the CSR promises 5 -- the
    promise still passes the host's global check (5 n <= nnz) -- so path 5 runs with a register
    head longer than those rows: the kernel clamps every CSR index it derives into the CSR and
    the LDS tail.  The launch completes, and the rows before the first short row
    (their heads and tails are exact) still equal the oracle's fold bit for bit."""
    from distributed_learning_amd.graph import Csr
    E = eng_mod()
    base = dense_irregular(3000, 4, 8, 9)
    n, k = base.n_rows, 1500
    rowptr, col, w = [0], [], []
    for r in range(n):
        e0, e1 = base.rowptr[r], base.rowptr[r + 1]
        keep = 2 if r in (k, n - 1) else e1 - e0
        col.extend(base.col[e0:e0 + keep])
        w.extend(base.w[e0:e0 + keep])
        rowptr.append(len(col))
    csr = Csr(rowptr, col, w, keys=list(range(n)))
    assert csr.min_row_nnz == 2 and 5 * n <= csr.nnz
    W = E.DeviceCsr(csr, cuda)
    W.min_row_nnz = 5                      # the wrong promise
    assert E.plan_shape(W, 1024, deviation=False)["path"] == 5
    P = 1024
    rng = np.random.default_rng(5)
    X = rng.standard_normal((n, P), dtype=np.float32)
    Xd = torch.from_numpy(X).to(cuda)
    Y = torch.zeros_like(Xd)
    E.mix_round(W, Xd, Y)
    torch.cuda.synchronize()
    want = cref.mix_round(X, csr.rowptr, csr.col, csr.w)
    assert np.array_equal(bits(Y[:k - 100].cpu().numpy()), bits(want[:k - 100]))


@pytest.mark.parametrize("times,eps", [(1, 0.3), (5, 0.02)])
def test_mixer_traced_row_stochastic_4096(cuda, monkeypatch, times, eps):
    """Mixer.mix(times, eps) over 4096 models whose topology is row- but not column-stochastic
    (the graph of test_row_stochastic_two_pass_deviation: the reference Mixer takes any
    dict-of-dicts weights, mixer.py:47, and tests eps after every round, :27-32, 40-41).  The
    loop runs as traced passes (dl_mix_rounds_trace on the one-image kernel, every round's column
    mean reduced from its outputs) -- not one launch and readback per round -- and returns the
    reference loop's round count and bits."""
    import logging
    from oracle import mixer_ref as M
    from distributed_learning_amd.utils.consensus_simple import Mixer
    from distributed_learning_amd.utils.consensus_simple import mixer as mixer_mod
    csr = dense_irregular(4096, 4, 9, 7, row_stochastic=True)
    n = csr.n_rows
    topo = {i: {int(csr.col[e]): float(csr.w[e]) for e in range(csr.rowptr[i], csr.rowptr[i + 1])}
            for i in range(n)}
    torch.manual_seed(9)
    models = {i: torch.nn.Linear(24, 8).to(cuda) for i in range(n)}
    X0 = np.stack([torch.cat([p.data.reshape(-1) for p in models[i].parameters()]).cpu().numpy()
                   for i in range(n)])
    rp, cl, w = M.topology_to_csr(topo)
    want, want_n = M.mixer_mix(X0, rp, cl, w, times=times, eps=eps)
    assert want_n >= 3                 # several rounds, so the passes are what runs
    calls = []
    real = mixer_mod._engine.mix_rounds_trace

    def traced(*a, **k):
        calls.append(a[3])
        return real(*a, **k)
    monkeypatch.setattr(mixer_mod._engine, "mix_rounds_trace", traced)
    m = Mixer(models, topo, logging.getLogger("rowstoch4096"))
    assert m.mix(times=times, eps=eps) == want_n
    assert calls and all(k == 4 for k in calls), calls
    got = np.stack([torch.cat([p.data.reshape(-1) for p in models[i].parameters()]).cpu().numpy()
                    for i in range(n)])
    assert np.array_equal(bits(got), bits(want))


def test_mixer_row_stochastic_4096_wide_models_take_the_round_loop(cuda, monkeypatch):
    """The same 4096-model row-stochastic topology with 9696 parameters per model: above
    Mixer._TRACE_IRR4_MAX_COLS columns the one-image traced kernel at 4 agents per thread is
    slower than one fused round per launch (scripts/trace_irr_probe.py), so Mixer.mix(times, eps)
    runs the round loop -- the reference loop's round count and bits either way."""
    import logging
    from oracle import mixer_ref as M
    from distributed_learning_amd.utils.consensus_simple import Mixer
    from distributed_learning_amd.utils.consensus_simple import mixer as mixer_mod
    csr = dense_irregular(4096, 4, 9, 7, row_stochastic=True)
    n = csr.n_rows
    topo = {i: {int(csr.col[e]): float(csr.w[e]) for e in range(csr.rowptr[i], csr.rowptr[i + 1])}
            for i in range(n)}
    torch.manual_seed(10)
    models = {i: torch.nn.Linear(100, 96).to(cuda) for i in range(n)}
    X0 = np.stack([torch.cat([p.data.reshape(-1) for p in models[i].parameters()]).cpu().numpy()
                   for i in range(n)])
    assert X0.shape[1] > Mixer._TRACE_IRR4_MAX_COLS
    rp, cl, w = M.topology_to_csr(topo)
    want, want_n = M.mixer_mix(X0, rp, cl, w, times=3, eps=0.05)
    calls = []
    real = mixer_mod._engine.mix_rounds_trace

    def traced(*a, **k):
        calls.append(a[3])
        return real(*a, **k)
    monkeypatch.setattr(mixer_mod._engine, "mix_rounds_trace", traced)
    m = Mixer(models, topo, logging.getLogger("rowstoch4096wide"))
    assert m.mix(times=3, eps=0.05) == want_n
    assert not calls, calls
    got = np.stack([torch.cat([p.data.reshape(-1) for p in models[i].parameters()]).cpu().numpy()
                    for i in range(n)])
    assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize("case", ["ba2_4096", "ba1_4096"])
def test_hub_rows_keep_deviation_bits(cuda, monkeypatch, case):
    """dlamd.h n_hub_rows: with a doubly stochastic W the fused deviation's bits (dev_sq, the
    max and the column mean) do not depend on how many leading rows the hub lanes fold -- they
    add a tile's squared deviations in the owner's (dx^2 + dy^2) + (dz^2 + dw^2) order."""
    E = eng_mod()
    csr = CASES[case][0]()
    n, P = csr.n_rows, 2048
    rng = np.random.default_rng(17)
    X = rng.standard_normal((n, P), dtype=np.float32)
    G = rng.standard_normal((n, P), dtype=np.float32)
    out = {}
    for hubs in ("0", "64", None):
        if hubs is None:
            monkeypatch.delenv("DLAMD_HUB_ROWS", raising=False)
        else:
            monkeypatch.setenv("DLAMD_HUB_ROWS", hubs)
        eng = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda))
        assert eng.plan()["path"] == 5 and eng.W.doubly_stochastic
        mean = torch.empty(P, device=cuda)
        eng.round(G=eng.layout_like(torch.from_numpy(G).to(cuda)), lr=0.02, deviation=True,
                  mean=mean)
        torch.cuda.synchronize()
        out[hubs] = (eng.W.hub_rows, bits(eng.rows().cpu().numpy()),
                     bits(eng.agent_dev_sq().cpu().numpy()), bits(eng.dev_max.cpu().numpy()),
                     bits(mean.cpu().numpy()))
    assert out["0"][0] == 0 and out[None][0] > 0
    for hubs in ("64", None):
        for k in range(1, 5):
            assert np.array_equal(out[hubs][k], out["0"][k]), (hubs, k)
