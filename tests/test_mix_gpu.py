"""GPU parity of the fused mix kernels (through libdlamd.so) against the CPU oracle and the
reference-generated fixtures.  Mixing must be bit-exact; deviations within 1e-5 relative."""
import numpy as np
import pytest
import torch

from oracle import cref, mixer_ref as M

pytestmark = pytest.mark.gpu

DEV_RTOL = 1e-5  # north_star: disagreement within 1e-5 relative in fp32


def dev_floor(mean, P):
    """Noise floor of a deviation: the fused kernel sums the column mean as a tree, numpy (the
    reference, mixer.py:61) as a sequential fold; the two means differ by a few ulp, which moves
    ||x_a - mean|| by up to ~sqrt(P) * ulp(|mean|).  Near consensus the reference's own value is
    at this floor, so parity there is an absolute bound, not a relative one."""
    return 8.0 * np.sqrt(P) * np.finfo(np.float32).eps * float(np.max(np.abs(mean)))


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


def eng_mod():
    from distributed_learning_amd import engine
    return engine


def graph_csr(n, deg, seed, self_pos="random", weights="random"):
    from distributed_learning_amd.graph import Csr
    rng = np.random.default_rng(seed)
    rp, cl, w = [0], [], []
    for a in range(n):
        nb = list(rng.choice(n, size=min(deg, n), replace=False)) if n > 1 else []
        nb = [int(x) for x in nb if x != a]
        pos = int(rng.integers(0, len(nb) + 1))
        row = nb[:pos] + [a] + nb[pos:]
        cl += row
        w += list(rng.uniform(-0.3, 0.9, len(row)) if weights == "random"
                  else [1.0 / len(row)] * len(row))
        rp.append(len(cl))
    return Csr(rp, cl, w)


def run_round(csr, X, G=None, lr=0.0, dev=True, cuda=None):
    E = eng_mod()
    Xd = torch.from_numpy(X).to(cuda)
    W = E.DeviceCsr(csr, cuda)
    Y = torch.empty_like(Xd)
    Gd = torch.from_numpy(G).to(cuda) if G is not None else None
    dsq = torch.empty(X.shape[0], device=cuda) if dev else None
    dmax = torch.empty(1, device=cuda) if dev else None
    mean = torch.empty(X.shape[1], device=cuda) if dev else None
    E.mix_round(W, Xd, Y, G=Gd, lr=lr, dev_sq=dsq, dev_max=dmax, mean=mean)
    torch.cuda.synchronize()
    out = Y.cpu().numpy()
    if dev:
        return out, dsq.cpu().numpy(), float(dmax.item()), mean.cpu().numpy()
    return out


def check_dev(Y, dsq, dmax, mean):
    want_mean = M.column_mean(Y)
    np.testing.assert_allclose(mean, want_mean, rtol=1e-5, atol=1e-6)
    want = cref.deviation_sq(Y)
    floor = dev_floor(want_mean, Y.shape[1])
    np.testing.assert_allclose(np.sqrt(dsq), np.sqrt(want), rtol=DEV_RTOL, atol=floor)
    assert dmax == pytest.approx(np.sqrt(want).max(), rel=DEV_RTOL, abs=floor)


@pytest.mark.parametrize("case,rounds", [("a", [1, 10, 200]), ("b", [1, 10])])
def test_reference_fixture_rounds(golden, cuda, case, rounds):
    from distributed_learning_amd.graph import Csr
    E = eng_mod()
    d = golden("mix_rr4_n64.npz")
    csr = Csr(d[f"{case}_rowptr"], d[f"{case}_cols"], d[f"{case}_w"])
    eng = E.GossipEngine(csr, d[f"{case}_X0"].shape[1], device=cuda,
                         X=torch.from_numpy(d[f"{case}_X0"]).to(cuda))
    assert eng.plan()["path"] == 1 and eng.layout == "tiled"
    done = 0
    for r in rounds:
        while done < r:
            eng.round(deviation=True)
            done += 1
        torch.cuda.synchronize()
        got = eng.rows().cpu().numpy()
        assert np.array_equal(bits(got), bits(d[f"{case}_X{r}"])), f"round {r}"
        np.testing.assert_allclose(np.sqrt(eng.dev_sq.cpu().numpy()), d[f"{case}_dev{r}"],
                                   rtol=DEV_RTOL, atol=dev_floor(M.column_mean(got), got.shape[1]))


SHAPES = [(1, 5, 1), (2, 7, 2), (8, 7, 3), (33, 129, 4), (64, 4096, 4), (100, 1000, 5),
          (300, 777, 8), (1024, 4100, 4), (1500, 64, 6), (2048, 256, 4), (4096, 64, 4)]


@pytest.mark.parametrize("n,P,deg", SHAPES)
@pytest.mark.parametrize("sgd", [False, True])
def test_mix_shapes_bit_exact(cuda, n, P, deg, sgd):
    rng = np.random.default_rng(n * 7 + P)
    csr = graph_csr(n, deg, seed=n + P)
    X = rng.standard_normal((n, P), dtype=np.float32)
    G = rng.standard_normal((n, P), dtype=np.float32) if sgd else None
    lr = 0.05
    Y, dsq, dmax, mean = run_round(csr, X, G, lr, dev=True, cuda=cuda)
    want = cref.mix_round(X, csr.rowptr, csr.col, csr.w, G=G, lr=lr)
    assert np.array_equal(bits(Y), bits(want))
    if n > 1:
        check_dev(Y, dsq, dmax, mean)
    else:
        assert np.all(dsq == 0) and dmax == 0.0


@pytest.mark.parametrize("sgd", [False, True])
def test_row_major_ragged_last_pass(cuda, sgd):
    """Row-major tiles whose last pass is ragged (256 agents: 515 tiles of 128 columns on the
    balanced grid) and a guarded 5-column tail behind them: bits and deviations as the oracle's."""
    n, P = 256, 515 * 128 + 5
    rng = np.random.default_rng(11)
    csr = graph_csr(n, 4, seed=3)
    X = rng.standard_normal((n, P), dtype=np.float32)
    G = rng.standard_normal((n, P), dtype=np.float32) if sgd else None
    Y, dsq, dmax, mean = run_round(csr, X, G, 0.05, dev=True, cuda=cuda)
    want = cref.mix_round(X, csr.rowptr, csr.col, csr.w, G=G, lr=0.05)
    assert np.array_equal(bits(Y), bits(want))
    check_dev(Y, dsq, dmax, mean)


def test_regular_graph_skips_rowptr(cuda):
    from distributed_learning_amd.graph import Csr
    E = eng_mod()
    n, P = 512, 2048
    rp = np.arange(0, n * 5 + 1, 5)
    rng = np.random.default_rng(5)
    cl = np.concatenate([np.r_[a, rng.choice(n, 4, replace=False)] for a in range(n)])
    csr = Csr(rp, cl, np.full(cl.size, 0.2))
    assert csr.uniform_row_nnz == 5
    X = rng.standard_normal((n, P), dtype=np.float32)
    for layout in ("rows", "tiled"):
        eng = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda), layout=layout)
        assert eng.plan()["regular"] == 1
        eng.round()
        assert np.array_equal(bits(eng.rows().cpu().numpy()), bits(M.mix_once(X, rp, cl, csr.w)))


def test_unaligned_operands_use_guarded_path(cuda):
    """Column-offset views (16-byte misaligned, odd leading dimension)."""
    E = eng_mod()
    n, P = 77, 513
    csr = graph_csr(n, 4, seed=11)
    rng = np.random.default_rng(2)
    big = torch.from_numpy(rng.standard_normal((n, P + 3), dtype=np.float32)).to(cuda)
    gbig = torch.from_numpy(rng.standard_normal((n, P + 2), dtype=np.float32)).to(cuda)
    X, G = big[:, 1:P + 1], gbig[:, 2:P + 2]
    Yb = torch.zeros(n, P + 5, device=cuda)
    Y = Yb[:, 3:P + 3]
    E.mix_round(E.DeviceCsr(csr, cuda), X, Y, G=G, lr=0.1)
    torch.cuda.synchronize()
    want = cref.mix_round(X.cpu().numpy(), csr.rowptr, csr.col, csr.w, G=G.cpu().numpy(), lr=0.1)
    assert np.array_equal(bits(Y.cpu().numpy()), bits(want))
    assert torch.all(Yb[:, :3] == 0) and torch.all(Yb[:, P + 3:] == 0)


@pytest.mark.parametrize("n,P", [(64, 1000), (1024, 2048), (5000, 300)])
def test_gather_path_bit_exact(cuda, monkeypatch, n, P):
    monkeypatch.setenv("DLAMD_FORCE_GATHER", "1")
    rng = np.random.default_rng(n)
    csr = graph_csr(n, 5, seed=n)
    X = rng.standard_normal((n, P), dtype=np.float32)
    G = rng.standard_normal((n, P), dtype=np.float32)
    Y, dsq, dmax, mean = run_round(csr, X, G, 0.01, dev=True, cuda=cuda)
    want = cref.mix_round(X, csr.rowptr, csr.col, csr.w, G=G, lr=0.01)
    assert np.array_equal(bits(Y), bits(want))
    check_dev(Y, dsq, dmax, mean)
    # the column mean on this path is numpy's sequential sum, bit for bit
    assert np.array_equal(bits(mean), bits(np.mean(want, axis=0)))


@pytest.mark.parametrize("force_gather", [False, True])
def test_halo_rows_equal_full_mix(cuda, monkeypatch, force_gather):
    """Split the agents into local rows + halo rows (already stepped, as a remote rank sends
    them): the local rows of the result equal the single-device round."""
    from distributed_learning_amd.graph import Csr
    if force_gather:
        monkeypatch.setenv("DLAMD_FORCE_GATHER", "1")
    E = eng_mod()
    n, P, n_loc = 200, 1030, 120
    full = graph_csr(n, 4, seed=3)
    rng = np.random.default_rng(4)
    X = rng.standard_normal((n, P), dtype=np.float32)
    G = rng.standard_normal((n, P), dtype=np.float32)
    lr = 0.02
    want = cref.mix_round(X, full.rowptr, full.col, full.w, G=G, lr=lr)
    local = Csr(full.rowptr[:n_loc + 1], full.col[:full.rowptr[n_loc]],
                full.w[:full.rowptr[n_loc]], n_src=n)
    Xd = torch.from_numpy(X).to(cuda)
    Gd = torch.from_numpy(G).to(cuda)
    rows = torch.arange(n_loc, n, dtype=torch.int32, device=cuda)
    halo = torch.empty(n - n_loc, P, device=cuda)
    E.step_rows(Xd, rows, halo, G=Gd, lr=lr)
    Y = torch.empty(n_loc, P, device=cuda)
    E.mix_round(E.DeviceCsr(local, cuda), Xd[:n_loc], Y, G=Gd[:n_loc], lr=lr, halo=halo)
    torch.cuda.synchronize()
    assert np.array_equal(bits(Y.cpu().numpy()), bits(want[:n_loc]))


def test_deviation_only_and_helpers(cuda):
    E = eng_mod()
    rng = np.random.default_rng(9)
    for n, P in [(2, 3), (64, 5000), (1024, 4096), (3000, 100)]:
        X = rng.standard_normal((n, P), dtype=np.float32)
        Xd = torch.from_numpy(X).to(cuda)
        mean = torch.empty(P, device=cuda)
        dsq, dmax = E.deviation(Xd, mean_out=mean)
        torch.cuda.synchronize()
        check_dev(X, dsq.cpu().numpy(), float(dmax.item()), mean.cpu().numpy())
        cs = E.column_sum(Xd).cpu().numpy()
        want_cs = X[0].copy()
        for r in range(1, n):
            want_cs = want_cs + X[r]
        assert np.array_equal(bits(cs), bits(want_cs))
        assert E.max_column_std(Xd).item() == np.float32(X.std(axis=0).max())
    X = rng.standard_normal((1, 10), dtype=np.float32)
    dsq, dmax = E.deviation(torch.from_numpy(X).to(cuda))
    assert float(dsq.item()) == 0.0 and float(dmax.item()) == 0.0


def test_full_size_round_column_slices(cuda):
    """BASELINE config c2 at full size (1024 agents x 2^20 params, random 4-regular graph,
    fused local step + deviation): columns are independent, so any column slice must equal
    the oracle run on that slice; the deviation is checked against the full oracle."""
    from distributed_learning_amd.graph import from_edge_weights, random_regular_edges
    E = eng_mod()
    n, P = 1024, 1 << 20
    edges = random_regular_edges(4, n, seed=0)
    csr = from_edge_weights(edges, [0.2] * len(edges))
    g = torch.Generator(device=cuda).manual_seed(0)
    X = torch.randn(n, P, device=cuda, generator=g)
    G = torch.randn(n, P, device=cuda, generator=g)
    eng = E.GossipEngine(csr, P, device=cuda, X=X)
    plan = eng.plan(deviation=True)
    assert plan["path"] == 1 and plan["tile_cols"] == 16 and eng.layout == "tiled"
    eng.round(G=eng.layout_like(G), lr=1e-3, deviation=True)
    torch.cuda.synchronize()
    Y = eng.rows()
    for c0, c1 in [(0, 4096), (P - 4096, P), (123456, 123456 + 999)]:
        want = cref.mix_round(X[:, c0:c1].cpu().numpy(), csr.rowptr, csr.col, csr.w,
                              G=G[:, c0:c1].cpu().numpy(), lr=1e-3)
        assert np.array_equal(bits(Y[:, c0:c1].cpu().numpy()), bits(want)), (c0, c1)
    Yh = Y.cpu().numpy()
    want_dsq = cref.deviation_sq(Yh)
    np.testing.assert_allclose(np.sqrt(eng.dev_sq.cpu().numpy()), np.sqrt(want_dsq),
                               rtol=DEV_RTOL)


def test_full_size_round_fdla_weights(cuda):
    """BASELINE config c2 at full size with the mixing weights north_star names: the per-edge
    FDLA weights of the c2 graph from utils/fast_averaging.py's SDP (the committed
    tests/golden/fdla_rr4_1024.npz, the weights bench.py's fdla_probe times every run; W = I -
    L(w), every row its own weights: shared_row_weights 0, all n(d + 1) weights staged).  Fused
    local step + mix + deviation over 1024 agents x 2^20 params in the column-tiled layout:
    column slices bit-exact against oracle/cref, the fused deviation within 1e-5 of the oracle's.
    Reference: utils/fast_averaging.py:4-32 (weights), utils/consensus_simple/mixer.py:47."""
    import os
    from distributed_learning_amd.graph import first_appearance_vertices, from_edge_weights
    E = eng_mod()
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "fdla_rr4_1024.npz"))
    edges = [tuple(int(x) for x in e) for e in d["edges"]]
    csr = from_edge_weights(edges, d["w"], sorted(first_appearance_vertices(edges)))
    n, P, lr = csr.n_rows, 1 << 20, 1e-3
    assert n == 1024 and not csr.shared_row_weights and csr.doubly_stochastic
    g = torch.Generator(device=cuda).manual_seed(12)
    X = torch.randn(n, P, device=cuda, generator=g)
    G = torch.randn(n, P, device=cuda, generator=g)
    eng = E.GossipEngine(csr, P, device=cuda, X=X)
    plan = eng.plan(deviation=True)
    assert plan["path"] == 1 and eng.layout == "tiled"
    eng.round(G=eng.layout_like(G), lr=lr, deviation=True)
    torch.cuda.synchronize()
    Y = eng.rows()
    for c0, c1 in [(0, 4096), (P - 4096, P), (654321, 654321 + 777)]:
        want = cref.mix_round(X[:, c0:c1].cpu().numpy(), csr.rowptr, csr.col, csr.w,
                              G=G[:, c0:c1].cpu().numpy(), lr=lr)
        assert np.array_equal(bits(Y[:, c0:c1].cpu().numpy()), bits(want)), (c0, c1)
    want_dsq = cref.deviation_sq(Y.cpu().numpy())
    np.testing.assert_allclose(np.sqrt(eng.dev_sq.cpu().numpy()), np.sqrt(want_dsq),
                               rtol=DEV_RTOL)
    assert float(eng.dev_max.item()) == pytest.approx(float(np.sqrt(want_dsq.max())),
                                                      rel=DEV_RTOL)


def test_full_size_c4_torus_column_slices(cuda):
    """BASELINE config c4 at full size on one GPU (64 x 64 torus, 4096 agents x 2^18 params,
    best-constant weights, fused local step + deviation, the engine's column-tiled layout):
    column slices bit-exact against the oracle; size-independent properties of the whole round
    -- W doubly stochastic, so every column sum of the stepped inputs is preserved (fp64 sums
    on the device, within fp32 rounding), and the fused deviation equals an fp64 recomputation
    from the output."""
    import math
    from distributed_learning_amd.graph import from_edge_weights, torus_edges
    E = eng_mod()
    n, P, lr = 4096, 1 << 18, 1e-3
    e = torus_edges(64, 64)
    w = 2.0 / (2.0 - 2.0 * math.cos(2 * math.pi / 64) + 8.0)
    csr = from_edge_weights(e, [w] * len(e), list(range(n)))
    g = torch.Generator(device=cuda).manual_seed(4)
    X = torch.randn(n, P, device=cuda, generator=g)
    G = torch.randn(n, P, device=cuda, generator=g)
    eng = E.GossipEngine(csr, P, device=cuda, X=X)
    plan = eng.plan(deviation=True)
    assert plan["path"] == 1 and eng.layout == "tiled"
    eng.round(G=eng.layout_like(G), lr=lr, deviation=True)
    torch.cuda.synchronize()
    Y = eng.rows()
    for c0, c1 in [(0, 2048), (P - 2048, P), (77777, 77777 + 513)]:
        want = cref.mix_round(X[:, c0:c1].cpu().numpy(), csr.rowptr, csr.col, csr.w,
                              G=G[:, c0:c1].cpu().numpy(), lr=lr)
        assert np.array_equal(bits(Y[:, c0:c1].cpu().numpy()), bits(want)), (c0, c1)
    T = X - np.float32(lr) * G          # the stepped inputs, rounded as the kernel does
    cs_in, cs_out = T.double().sum(0), Y.double().sum(0)
    scale = T.double().abs().sum(0)
    assert float(((cs_out - cs_in).abs() / scale).max()) < 1e-5
    del T
    Yd = Y.double()
    dsq = ((Yd - Yd.mean(0)) ** 2).sum(1)
    del Yd
    np.testing.assert_allclose(np.sqrt(eng.dev_sq.cpu().numpy()), np.sqrt(dsq.cpu().numpy()),
                               rtol=DEV_RTOL)
    assert float(eng.dev_max.item()) == pytest.approx(float(dsq.max().sqrt()), rel=DEV_RTOL)


@pytest.mark.parametrize("layout,P", [("rows", 10 ** 6), ("rows", 10 ** 6 + 3),
                                      ("tiled", 10 ** 6 + 8)])
def test_full_size_tail_columns(cuda, layout, P):
    """the tail test at P = 10^6 (and ragged widths: 10^6 + 3 is not float4-aligned, so
    the row-major round takes the guarded tail launch; 10^6 + 8 pads the last 16-column tile),
    1024 agents, fused local step + deviation.  Column slices at both ends equal the oracle;
    the fused deviation equals the two-pass dl_deviation of the result."""
    from distributed_learning_amd.graph import from_edge_weights, random_regular_edges
    E = eng_mod()
    n = 1024
    edges = random_regular_edges(4, n, seed=0)
    csr = from_edge_weights(edges, [0.2] * len(edges))
    g = torch.Generator(device=cuda).manual_seed(1)
    X = torch.randn(n, P, device=cuda, generator=g)
    G = torch.randn(n, P, device=cuda, generator=g)
    eng = E.GossipEngine(csr, P, device=cuda, X=X, layout=layout)
    eng.round(G=eng.layout_like(G), lr=1e-3, deviation=True)
    torch.cuda.synchronize()
    Y = eng.rows()
    for c0, c1 in [(0, 1000), (P - 1037, P)]:
        want = cref.mix_round(X[:, c0:c1].cpu().numpy(), csr.rowptr, csr.col, csr.w,
                              G=G[:, c0:c1].cpu().numpy(), lr=1e-3)
        assert np.array_equal(bits(Y[:, c0:c1].cpu().numpy()), bits(want)), (c0, c1)
    dsq, _ = E.deviation(Y.contiguous())
    torch.testing.assert_close(eng.dev_sq, dsq, rtol=DEV_RTOL, atol=0)


@pytest.mark.parametrize("n,P,deg", [(64, 4096, 4), (100, 1000, 5), (1024, 4100, 4), (7, 33, 3),
                                     (300, 777, 8)])
def test_tiled_layout_round_trip_and_parity(cuda, n, P, deg):
    """Resident column-tiled layout: same bits as the row-major round and the oracle, padded
    tail columns stay zero, deviation matches, conversions round-trip."""
    E = eng_mod()
    rng = np.random.default_rng(n + 3 * P)
    csr = graph_csr(n, deg, seed=n * P)
    X = rng.standard_normal((n, P), dtype=np.float32)
    G = rng.standard_normal((n, P), dtype=np.float32)
    eng = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda), layout="tiled")
    assert np.array_equal(bits(eng.rows().cpu().numpy()), bits(X))
    mean = torch.empty(P, device=cuda)
    eng.round(G=eng.layout_like(torch.from_numpy(G).to(cuda)), lr=0.03, deviation=True,
              mean=mean)
    torch.cuda.synchronize()
    want = cref.mix_round(X, csr.rowptr, csr.col, csr.w, G=G, lr=0.03)
    assert np.array_equal(bits(eng.rows().cpu().numpy()), bits(want))
    check_dev(want, eng.dev_sq.cpu().numpy(), float(eng.dev_max.item()), mean.cpu().numpy())
    T = eng.T
    if P % T:
        assert torch.all(eng.X[-1, :, P % T:] == 0)
    dsq, dmax = eng.deviation()
    check_dev(want, dsq.cpu().numpy(), float(dmax.item()), M.column_mean(want))


@pytest.mark.parametrize("layout", ["tiled", "rows"])
def test_doubly_stochastic_mean_from_inputs(cuda, layout):
    """For doubly stochastic W the fused deviation takes the column mean from the round's inputs
    (one LDS pass); it must agree with the general two-pass path and with the oracle."""
    from distributed_learning_amd.graph import from_edge_weights, random_regular_edges
    E = eng_mod()
    n, P = 512, 8192 + 40
    edges = random_regular_edges(4, n, seed=3)
    csr = from_edge_weights(edges, [0.19] * len(edges), list(range(n)))
    assert csr.doubly_stochastic
    rng = np.random.default_rng(8)
    X = rng.standard_normal((n, P), dtype=np.float32)
    G = rng.standard_normal((n, P), dtype=np.float32)
    want = cref.mix_round(X, csr.rowptr, csr.col, csr.w, G=G, lr=0.02)
    out = {}
    for ds in (1, 0):
        eng = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda), layout=layout)
        eng.W.doubly_stochastic = ds
        mean = torch.empty(P, device=cuda)
        eng.round(G=eng.layout_like(torch.from_numpy(G).to(cuda)), lr=0.02, deviation=True,
                  mean=mean)
        torch.cuda.synchronize()
        assert np.array_equal(bits(eng.rows().cpu().numpy()), bits(want))
        check_dev(want, eng.dev_sq.cpu().numpy(), float(eng.dev_max.item()), mean.cpu().numpy())
        out[ds] = eng.dev_sq.cpu().numpy()
    np.testing.assert_allclose(out[1], out[0], rtol=1e-5)


@pytest.mark.parametrize("layout", ["tiled", "rows"])
def test_torus_4096_shared_weights_bit_exact(cuda, layout):
    """The c4 graph (64x64 torus, uniform best-constant weights, 4096 agents): the shared-weight
    LDS tile path is bit-identical to the oracle and to the per-entry-weight path (which at this
    size is the gather kernel)."""
    import math
    from distributed_learning_amd.graph import from_edge_weights, torus_edges
    E = eng_mod()
    n, P = 4096, 1024 + 20
    e = torus_edges(64, 64)
    w = 2.0 / (2.0 - 2.0 * math.cos(2 * math.pi / 64) + 8.0)
    csr = from_edge_weights(e, [w] * len(e), list(range(n)))
    rng = np.random.default_rng(64)
    X = rng.standard_normal((n, P), dtype=np.float32)
    G = rng.standard_normal((n, P), dtype=np.float32)
    want = cref.mix_round(X, csr.rowptr, csr.col, csr.w, G=G, lr=0.01)
    eng = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda), layout=layout)
    assert eng.plan()["path"] == 1
    mean = torch.empty(P, device=cuda)
    eng.round(G=eng.layout_like(torch.from_numpy(G).to(cuda)), lr=0.01, deviation=True, mean=mean)
    torch.cuda.synchronize()
    assert np.array_equal(bits(eng.rows().cpu().numpy()), bits(want))
    check_dev(want, eng.dev_sq.cpu().numpy(), float(eng.dev_max.item()), mean.cpu().numpy())
    # the same graph with per-entry weights (no shared flag): the CSR no longer fits LDS beside
    # the tile -> the register-CSR tile kernel (path 4), and the gather kernel when forced;
    # same bits
    W = E.DeviceCsr(csr, cuda)
    W.shared_row_weights = 0
    assert E.plan_shape(W, P)["path"] == 4
    Y = torch.empty(n, P, device=cuda)
    E.mix_round(W, torch.from_numpy(X).to(cuda), Y, G=torch.from_numpy(G).to(cuda), lr=0.01)
    torch.cuda.synchronize()
    assert np.array_equal(bits(Y.cpu().numpy()), bits(want))


def _per_edge_regular(kind, n, seed):
    """A degree-4 regular graph with genuinely per-edge symmetric weights (doubly stochastic)."""
    from distributed_learning_amd.graph import from_edge_weights, random_regular_edges, torus_edges
    edges = torus_edges(64, n // 64) if kind == "torus" else random_regular_edges(4, n, seed=seed)
    w = np.random.default_rng(seed).uniform(0.12, 0.24, len(edges))
    return from_edge_weights(edges, list(w), sorted({v for e in edges for v in e}))


@pytest.mark.parametrize("kind,n", [("torus", 4096), ("rr4", 4096), ("rr4", 3600)])
@pytest.mark.parametrize("layout", ["tiled", "rows"])
def test_register_csr_tile_path(cuda, monkeypatch, kind, n, layout):
    """Regular graphs of thousands of agents with per-edge weights: the CSR (n * 5 weights + ids)
    does not fit LDS beside a column tile of every agent, so the tile kernel keeps each thread's
    rows' CSR in registers (path 4) instead of falling back to the gather kernel.  Fused local
    step + mix + deviation: bit-exact with the oracle, deviation within 1e-5; the forced gather
    path gives the same bits."""
    E = eng_mod()
    csr = _per_edge_regular(kind, n, seed=n)
    assert not csr.shared_row_weights and csr.doubly_stochastic
    P = 2048 + 64
    rng = np.random.default_rng(n)
    X = rng.standard_normal((n, P), dtype=np.float32)
    G = rng.standard_normal((n, P), dtype=np.float32)
    want = cref.mix_round(X, csr.rowptr, csr.col, csr.w, G=G, lr=0.02)
    eng = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda), layout=layout)
    assert eng.plan()["path"] == 4, eng.plan()
    mean = torch.empty(P, device=cuda)
    eng.round(G=eng.layout_like(torch.from_numpy(G).to(cuda)), lr=0.02, deviation=True, mean=mean)
    torch.cuda.synchronize()
    assert np.array_equal(bits(eng.rows().cpu().numpy()), bits(want))
    check_dev(want, eng.dev_sq.cpu().numpy(), float(eng.dev_max.item()), mean.cpu().numpy())
    if layout == "rows":
        monkeypatch.setenv("DLAMD_FORCE_GATHER", "1")
        Y, dsq, dmax, mean_g = run_round(csr, X, G=G, lr=0.02, cuda=cuda)
        assert np.array_equal(bits(Y), bits(want))
        check_dev(want, dsq, dmax, mean_g)



@pytest.mark.parametrize("edges,w", [
    ([(0, 1), (0, 2), (0, 3), (1, 4), (4, 2)], [1 / 3, 1 / 3, 1 / 2, 1 / 3, 1 / 3]),
    ([(9, 1), (1, 17), (17, 33), (33, 9), (9, 17)], [0.2, 0.25, 0.3, 0.15, 0.1])])
def test_tcp_run_once_round(cuda, edges, w):
    """a7: ConsensusAgent.run_once of every agent (consensus_tcp/agent.py:204-207) as one
    dl_mix_round over graph.from_tcp_weights: bit-exact with the fp32 CSR fold, within fp32
    rounding of the reference's fp64-promoted update."""
    from distributed_learning_amd.graph import from_tcp_weights
    E = eng_mod()
    csr = from_tcp_weights(edges, w)
    rng = np.random.default_rng(3)
    X = rng.standard_normal((csr.n_rows, 1000), dtype=np.float32)
    Y = torch.empty(X.shape, device=cuda)
    E.mix_round(E.DeviceCsr(csr, cuda), torch.from_numpy(X).to(cuda), Y)
    got = Y.cpu().numpy()
    assert np.array_equal(bits(got), bits(M.mix_once(X, csr.rowptr, csr.col, csr.w)))
    want = M.tcp_run_once(edges, w, {k: X[i] for i, k in enumerate(csr.keys)})
    np.testing.assert_allclose(got, np.stack([want[k] for k in csr.keys]), rtol=1e-5, atol=1e-6)



def shared_weight_graph(n, seed, doubly=True):
    """A random 4-regular graph whose every row carries the same weight sequence (CSR
    shared_row_weights: the tile kernel's unrolled degree-5 rows with the weights in scalar
    registers).  doubly: the best-constant weights (W doubly stochastic, the tile mean taken
    from the staged inputs); else one asymmetric sequence whose columns do not sum to 1 (the
    two-pass tile mean)."""
    from distributed_learning_amd.graph import Csr, random_regular_edges
    edges = random_regular_edges(4, n, seed=seed)
    nbrs = [[] for _ in range(n)]
    for u, v in edges:
        nbrs[u].append(v)
        nbrs[v].append(u)
    seq = [0.2] * 5 if doubly else [0.4, 0.3, 0.1, 0.15, 0.05]
    rp, cl, w = [0], [], []
    for a in range(n):
        cl += [a] + nbrs[a]
        w += seq
        rp.append(len(cl))
    csr = Csr(rp, cl, w, keys=list(range(n)))
    assert csr.shared_row_weights and csr.uniform_row_nnz == 5
    assert bool(csr.doubly_stochastic) == doubly
    return csr


@pytest.mark.parametrize("T", [4, 8, 16, 32, 64, 128])
@pytest.mark.parametrize("doubly", [True, False])
def test_tiled_widths_shared_weights(cuda, T, doubly):
    """Every column-tiled width (C = 1 .. 32 float4 chunks per row: the cross-lane sums on DPP,
    v_permlane16/32_swap and ds_bpermute, the per-lane deviation partials at <= 4 passes per
    thread) with the fused step and deviation on a shared-weight degree-4 graph: bit-exact
    rounds, deviation and mean within tolerance, both tile-mean paths."""
    E = eng_mod()
    n, P = 256, 128 * 24 + 64
    csr = shared_weight_graph(n, seed=T, doubly=doubly)
    rng = np.random.default_rng(T + 7 * doubly)
    X = rng.standard_normal((n, P), dtype=np.float32)
    G = rng.standard_normal((n, P), dtype=np.float32)
    eng = E.GossipEngine(csr, P, device=cuda, X=torch.from_numpy(X).to(cuda), layout="tiled",
                         tile_cols=T)
    plan = eng.plan()
    assert plan["path"] == 1 and plan["tile_cols"] == T, plan
    mean = torch.empty(P, device=cuda)
    eng.round(G=eng.layout_like(torch.from_numpy(G).to(cuda)), lr=0.03, deviation=True,
              mean=mean)
    torch.cuda.synchronize()
    want = cref.mix_round(X, csr.rowptr, csr.col, csr.w, G=G, lr=0.03)
    assert np.array_equal(bits(eng.rows().cpu().numpy()), bits(want))
    check_dev(want, eng.dev_sq.cpu().numpy(), float(eng.dev_max.item()), mean.cpu().numpy())


def test_row_sums(cuda):
    """dl_row_sums (a chunked halo round's deviation and its max in one launch): column sums of
    the partial rows in a fixed order, max of their square roots."""
    E = eng_mod()
    rng = np.random.default_rng(5)
    parts = torch.from_numpy(rng.random((3, 1000), dtype=np.float32)).to(cuda)
    sums = torch.empty(1000, device=cuda)
    mx = torch.empty(1, device=cuda)
    E.row_sums(parts, sums, mx)
    torch.cuda.synchronize()
    want = parts.cpu().double().sum(0).float().numpy()
    np.testing.assert_allclose(sums.cpu().numpy(), want, rtol=1e-6)
    assert float(mx.item()) == pytest.approx(float(np.sqrt(want).max()), rel=1e-6)
    # max_zeroed: the caller (a partial-rows dl_mix_round's dev_max) already set the word to 0
    sums2, mx2 = torch.empty(1000, device=cuda), torch.zeros(1, device=cuda)
    E.row_sums(parts, sums2, mx2, max_zeroed=True)
    torch.cuda.synchronize()
    assert torch.equal(sums2, sums) and torch.equal(mx2, mx)
