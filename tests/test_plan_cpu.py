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
