"""Kernel-configuration planning on the host (no GPU): dl_mix_plan_csr picks the register-CSR tile
kernels for graphs whose CSR does not fit LDS beside a tile of every agent -- path 4 (regular, all
five entries in registers) and path 5 (irregular: a register head of min(min_row_nnz, 5) entries
and an LDS tail of 8-byte pairs, or 6 bytes per entry when 8 do not fit) -- and the traced
multi-round pass for up to 4096 agents (dl_mix_trace_plan's round caps)."""
import ctypes

import numpy as np
import pytest

from distributed_learning_amd import _lib, engine, graph

LDS = 163840


def plan(csr, n_params=1 << 18, tile_cols=-1):
    return engine.plan_shape(engine.DeviceCsr(csr, "cpu"), n_params, deviation=True,
                             tile_cols=tile_cols)


def test_barabasi_albert_takes_path5_with_pairs():
    csr = graph.barabasi_albert_metropolis(4096, 2, 1)
    assert csr.min_row_nnz == 3 and not csr.uniform_row_nnz and csr.doubly_stochastic
    p = plan(csr)
    ntail = csr.nnz - 3 * 4096
    assert p["path"] == 5 and p["tile_cols"] == 4 and p["regular"] == 0
    # tile + mean scratch + 8-byte {weight, row} pairs
    assert p["lds_bytes"] == 4096 * 16 + 256 + (8 * ntail + 15) // 16 * 16
    assert plan(csr, tile_cols=0)["path"] == 5      # row-major operands too


def test_tail_falls_back_to_six_bytes():
    csr = graph.random_irregular_metropolis(4096, 2, 7, 1)
    ntail = csr.nnz - 3 * csr.n_rows
    assert 4096 * 16 + 256 + 8 * ntail > LDS >= 4096 * 16 + 256 + 6 * ntail
    p = plan(csr)
    assert p["path"] == 5 and p["lds_bytes"] == 4096 * 16 + 256 + (6 * ntail + 15) // 16 * 16


def test_too_dense_for_path5_takes_gather():
    csr = graph.random_irregular_metropolis(4096, 2, 8, 1)    # tail > 6 B x 16k entries
    assert plan(csr, tile_cols=0)["path"] == 2


def test_irregular_above_2048_prefers_path5_even_when_csr_fits():
    tree = graph.barabasi_albert_metropolis(4096, 1, 2)        # CSR 72 KB: fits beside the tile
    assert plan(tree)["path"] == 5
    small = graph.barabasi_albert_metropolis(2048, 2, 6)       # 2 chunks per tile on path 1
    p = plan(small)
    assert p["path"] == 1 and p["tile_cols"] == 8


def test_regular_graphs_keep_their_paths():
    import math
    e = graph.torus_edges(64, 64)
    w = 2.0 / (2.0 - 2.0 * math.cos(2 * math.pi / 64) + 8.0)
    shared = graph.from_edge_weights(e, [w] * len(e), list(range(4096)))
    assert plan(shared)["path"] == 1                           # 5 shared weights: CSR in LDS
    W = engine.DeviceCsr(shared, "cpu")
    W.shared_row_weights = 0                                    # per-entry weights
    assert engine.plan_shape(W, 1 << 18, tile_cols=-1)["path"] == 4


def test_plan_shape_without_min_row_nnz_cannot_see_path5():
    csr = graph.barabasi_albert_metropolis(4096, 2, 1)
    lib = _lib.load()
    pl = _lib.DlMixPlan()
    _lib.check(lib.dl_mix_plan_shape(4096, 0, 1 << 18, csr.nnz, 0, 0, 1, 0, ctypes.byref(pl)),
               "plan")
    assert pl.path == 2
    # a promise no row set can keep (more entries per row than nnz / n_rows): never path 5
    W = _lib.DlCsr(None, None, None, 4096, csr.nnz, 0, 1, 0, csr.nnz // 4096 + 1)
    pl.path = 0
    lib.dl_mix_plan_csr(ctypes.byref(W), 0, 1 << 18, 1, -1, ctypes.byref(pl))
    assert pl.path != 5


def test_min_row_nnz_and_row_length_order():
    csr = graph.barabasi_albert_metropolis(512, 2, 3)
    d = np.diff(csr.rowptr)
    assert csr.min_row_nnz == d.min() == 3
    order = graph.row_length_order(csr)
    assert sorted(order.tolist()) == list(range(512))
    assert np.all(np.diff(d[order]) <= 0)                       # descending row lengths
    p = graph.permuted(csr, order)
    assert p.min_row_nnz == 3 and p.nnz == csr.nnz


@pytest.mark.parametrize("n,want", [(1024, 24), (1500, 16), (2048, 16), (3000, 8), (4096, 8)])
def test_trace_round_caps(n, want):
    """dl_mix_trace_plan for register-cached regular graphs: 24 rounds per traced pass at 1024
    agents (rows kernel), 16 at up to 2048 and 8 at up to 4096 (wide kernel: every agent's
    per-round deviation in registers)."""
    edges = graph.random_regular_edges(4, n, seed=0)
    w = graph.best_constant_weight(edges, list(range(n)))
    csr = graph.from_edge_weights(edges, [w] * len(edges), list(range(n)))
    lib = _lib.load()
    W = engine.DeviceCsr(csr, "cpu")
    args = _lib.DlMixArgs()
    args.x = ctypes.c_void_p(16)           # never dereferenced by the planner
    args.y = ctypes.c_void_p(1 << 40)
    args.ldx = args.ldy = 1024
    args.n_params = 1024
    args.W = _lib.DlCsr(ctypes.c_void_p(64), ctypes.c_void_p(64), ctypes.c_void_p(64), n, csr.nnz,
                        W.uniform_row_nnz, 1, W.shared_row_weights, W.min_row_nnz)
    k = ctypes.c_int32(0)
    _lib.check(lib.dl_mix_trace_plan(ctypes.byref(args), ctypes.byref(k)), "trace plan")
    assert k.value == want


def test_hub_rows_of_a_row_length_order(monkeypatch):
    """engine.hub_rows (dl_mix_args.n_hub_rows for plan path 5): the leading rows of a
    descending row-length order with LDS tails (more than ``tail`` entries, default 0), capped
    at 256; DLAMD_HUB_ROWS overrides it.  The plan reports the register head it is
    measured against (ABI 8 dl_mix_plan.head / tail_fmt)."""
    csr = graph.barabasi_albert_metropolis(4096, 2, 1)
    p = plan(csr)
    assert p["path"] == 5 and p["head"] == 3 and p["tail_fmt"] == 2
    order = graph.row_length_order(csr)
    pc = graph.permuted(csr, order)
    lens = np.diff(pc.rowptr)
    assert np.all(np.diff(lens) <= 0)               # descending
    h = engine.hub_rows(pc, p["head"])
    assert h == 256 and np.all(lens[:h] - 3 > 0)
    assert engine.hub_rows(csr, p["head"]) < h or lens[0] == np.diff(csr.rowptr)[0]
    monkeypatch.setenv("DLAMD_HUB_ROWS", "0")
    assert engine.hub_rows(pc, 3) == 0
    monkeypatch.setenv("DLAMD_HUB_ROWS", "999")
    assert engine.hub_rows(pc, 3) == 256
    # a graph whose longest rows fit the register head has none
    monkeypatch.delenv("DLAMD_HUB_ROWS")
    short = graph.Csr([0, 2, 4, 6], [0, 1, 1, 2, 0, 2], [0.5] * 6)
    assert engine.hub_rows(short, 2) == 0


def test_traced_plan_takes_any_topology_that_fits():
    """dl_mix_trace_plan (ABI 8): a row-stochastic W or an irregular graph above 2048 agents
    runs traced passes on the one-image kernel (24 / 12 / 4 rounds per pass at <= 1024 / 2048 /
    4096 agents); a CSR too large for LDS beside one image is refused."""
    lib = _lib.load()

    def trace_rounds(csr, P=256):
        a = _lib.DlMixArgs()
        a.x, a.y = 1 << 20, 1 << 36
        a.ldx = a.ldy = P
        a.n_params = P
        W = engine.DeviceCsr(csr, "cpu")   # sizes and flags; the pointers are never read here
        a.W = _lib.DlCsr(16, 16, 16, W.n_rows, W.nnz, W.uniform_row_nnz, W.doubly_stochastic,
                         W.shared_row_weights, W.min_row_nnz)
        k = ctypes.c_int32(0)
        rc = lib.dl_mix_trace_plan(ctypes.byref(a), ctypes.byref(k))
        return k.value if rc == 0 else -rc
    ba = graph.barabasi_albert_metropolis(4096, 2, 1)
    assert ba.doubly_stochastic and trace_rounds(ba) == 4
    rs = graph.Csr([0, 2, 4, 6], [0, 1, 1, 2, 0, 2], [0.7, 0.3, 0.4, 0.6, 0.5, 0.5])
    assert not rs.doubly_stochastic and trace_rounds(rs) == 24
    rr = graph.from_edge_weights(graph.random_regular_edges(4, 1500, seed=1),
                                 [0.2] * 3000, list(range(1500)))
    assert trace_rounds(rr) == 16        # doubly stochastic: the double-buffered wide kernel
    dense = graph.random_irregular_metropolis(4096, 14, 20, 2)
    assert trace_rounds(dense) == -_lib.DL_ERR_UNSUPPORTED
