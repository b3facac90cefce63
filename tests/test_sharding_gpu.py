"""Agent-partitioned halo rounds on one MI355X with virtual ranks (threads + LocalTransport):
the HIP halo path (dl_step_rows + dl_mix_round with n_halo) equals the single-device round."""
import threading

import numpy as np
import pytest
import torch

from distributed_learning_amd import sharding
from distributed_learning_amd.graph import best_constant_weight, from_edge_weights, torus_edges

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("layout", ["rows", "tiled"])
@pytest.mark.parametrize("world,chunk,overlap", [(2, None, "chunks"), (4, 300, "chunks"),
                                                 (8, 1000, "chunks"), (2, None, "split"),
                                                 (4, None, "split"), (8, None, "split")])
def test_virtual_ranks_equal_single_device(cuda, world, chunk, overlap, layout):
    from distributed_learning_amd import engine as E
    R, C, P = 16, 16, 2048
    edges = torus_edges(R, C)
    verts = list(range(R * C))
    csr = from_edge_weights(edges, [best_constant_weight(edges, verts)] * len(edges), verts)
    g = torch.Generator(device=cuda).manual_seed(5)
    X = torch.randn(R * C, P, device=cuda, generator=g)
    G = torch.randn(R * C, P, device=cuda, generator=g)
    ref = E.GossipEngine(csr, P, device=cuda, X=X, layout="rows")
    for _ in range(3):
        ref.round(G=G, lr=0.01)
    plans = (sharding.split_halo_plans if overlap == "split" else sharding.halo_plans)(
        csr, sharding.torus_block_partition(R, C, world))
    tr = sharding.LocalTransport(world)
    shards = []
    for pl in plans:
        sh = sharding.HaloShard(pl, P, cuda, tr.endpoint(pl.rank), chunk_cols=chunk,
                                n_agents_total=R * C, overlap=overlap, layout=layout)
        assert sh.layout == layout
        ids = torch.as_tensor(pl.local, device=cuda)
        sh.load_rows(X[ids])
        shards.append((sh, sh.layout_like(G[ids]), ids))
    errs = []

    def run(sh, Gl):
        try:
            for _ in range(3):
                sh.round(G=Gl, lr=0.01)
            sh.dev = sh.deviation()
        except Exception as e:  # pragma: no cover
            errs.append(e)
    ths = [threading.Thread(target=run, args=(sh, Gl)) for sh, Gl, _ in shards]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
    torch.cuda.synchronize()
    full = ref.rows()
    for sh, _, ids in shards:
        assert torch.equal(sh.rows().view(torch.int32), full[ids].view(torch.int32))
    dsq, dmax = ref.deviation()
    for sh, _, ids in shards:
        assert float(sh.dev[1].item()) == pytest.approx(float(dmax.item()), rel=1e-5)
        np.testing.assert_allclose(sh.dev[0].cpu().numpy(), dsq[ids].cpu().numpy(), rtol=1e-5)


@pytest.mark.parametrize("layout", ["rows", "tiled"])
@pytest.mark.parametrize("world,chunk,overlap", [(2, None, "chunks"), (4, 300, "chunks"),
                                                 (8, 1000, "chunks"), (4, None, "split"),
                                                 (8, None, "split")])
def test_lagged_deviation_in_the_halo_round(cuda, world, chunk, overlap, layout):
    """HaloShard.round(deviation=True): the kernel measures its input rows against the previous
    round's all-reduced mean and publishes the column sums of its stepped inputs (no HBM pass of
    its own).  Iterates stay bit-identical to the single-device round; round i returns the
    deviation of the iterate it started from within 1e-5 relative of ``GossipEngine.deviation``
    on that iterate (the mean differs only by summation order)."""
    from distributed_learning_amd import engine as E
    # rows: a ragged tail tile (guarded launch); tiled: whole tiles (the layout's requirement)
    R, C, P = 16, 16, 2048 + (36 if layout == "rows" else 0)
    edges = torus_edges(R, C)
    verts = list(range(R * C))
    csr = from_edge_weights(edges, [best_constant_weight(edges, verts)] * len(edges), verts)
    g = torch.Generator(device=cuda).manual_seed(7)
    X = torch.randn(R * C, P, device=cuda, generator=g)
    G = torch.randn(R * C, P, device=cuda, generator=g)
    ref = E.GossipEngine(csr, P, device=cuda, X=X, layout="rows")
    want = []
    for _ in range(4):
        want.append(tuple(t.clone() for t in ref.deviation()))   # engine buffers are reused
        ref.round(G=G, lr=0.01)
    plans = (sharding.split_halo_plans if overlap == "split" else sharding.halo_plans)(
        csr, sharding.torus_block_partition(R, C, world))
    tr = sharding.LocalTransport(world)
    shards = []
    for pl in plans:
        sh = sharding.HaloShard(pl, P, cuda, tr.endpoint(pl.rank), chunk_cols=chunk,
                                n_agents_total=R * C, overlap=overlap, layout=layout)
        assert sh.layout == layout
        ids = torch.as_tensor(pl.local, device=cuda)
        sh.load_rows(X[ids])
        shards.append((sh, sh.layout_like(G[ids]), ids))
    errs = []

    def run(sh, Gl):
        try:
            sh.got = [sh.round(G=Gl, lr=0.01, deviation=True) for _ in range(4)]
        except Exception as e:  # pragma: no cover
            errs.append(e)
    ths = [threading.Thread(target=run, args=(sh, Gl)) for sh, Gl, _ in shards]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
    torch.cuda.synchronize()
    full = ref.rows()
    for sh, _, ids in shards:
        assert torch.equal(sh.rows().view(torch.int32), full[ids].view(torch.int32))
        for (dsq, dmax), (wsq, wmax) in zip(sh.got, want):
            np.testing.assert_allclose(dsq.cpu().numpy(), wsq[ids].cpu().numpy(), rtol=1e-5)
            assert float(dmax.item()) == pytest.approx(float(wmax.item()), rel=1e-5)


def _gloo_worker(rank, world, port, chunk, out_dir, overlap="chunks", layout="auto"):
    """One rank of a real multi-process run on the shared GPU: torch.distributed gloo with the
    host-staged transport, the HIP halo path, checked against the single-device round."""
    import os
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from distributed_learning_amd import engine as E
    dev = torch.device("cuda", 0)
    R, C, P = 16, 16, 2048
    edges = torus_edges(R, C)
    verts = list(range(R * C))
    csr = from_edge_weights(edges, [best_constant_weight(edges, verts)] * len(edges), verts)
    g = torch.Generator(device=dev).manual_seed(9)
    X = torch.randn(R * C, P, device=dev, generator=g)
    G = torch.randn(R * C, P, device=dev, generator=g)
    plan = (sharding.split_halo_plans if overlap == "split" else sharding.halo_plans)(
        csr, sharding.torus_block_partition(R, C, world))[rank]
    tr = sharding.dist_transport()
    assert isinstance(tr, sharding.StagedTransport)
    sh = sharding.HaloShard(plan, P, dev, tr, chunk_cols=chunk, n_agents_total=R * C,
                            overlap=overlap, layout=layout)
    ids = torch.as_tensor(plan.local, device=dev)
    sh.load_rows(X[ids])
    Gl = sh.layout_like(G[ids])
    for _ in range(3):
        sh.round(G=Gl, lr=0.01)
    dsq, dmax = sh.deviation()
    ref = E.GossipEngine(csr, P, device=dev, X=X, layout="rows")
    for _ in range(3):
        ref.round(G=G, lr=0.01)
    rsq, rmax = ref.deviation()
    torch.cuda.synchronize()
    ok = torch.equal(sh.rows().view(torch.int32), ref.rows()[ids].view(torch.int32))
    ok = ok and abs(float(dmax.item()) - float(rmax.item())) <= 1e-5 * float(rmax.item())
    ok = ok and bool(torch.allclose(dsq, rsq[ids], rtol=1e-5, atol=0))
    with open(os.path.join(out_dir, f"ok{rank}"), "w") as f:
        f.write(f"{int(ok)} halo={plan.n_halo} peers={sorted(plan.halo_from)} layout={sh.layout}")
    dist.destroy_process_group()


@pytest.mark.parametrize("world,chunk,overlap,layout", [(2, None, "chunks", "rows"),
                                                        (4, 700, "chunks", "tiled"),
                                                        (4, None, "split", "tiled")])
def test_processes_over_gloo_equal_single_device(cuda, tmp_path, world, chunk, overlap, layout):
    """world processes share the GPU and exchange halos through torch.distributed (gloo, staged
    through the host): the multi-process protocol of bench --workload c4 with the HIP kernels."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_gloo_worker, args=(world, port, chunk, str(tmp_path), overlap, layout),
             nprocs=world, join=True)
    for r in range(world):
        txt = (tmp_path / f"ok{r}").read_text()
        assert txt.startswith("1 "), (r, txt)


@pytest.mark.parametrize("layout", ["rows", "tiled"])
@pytest.mark.parametrize("overlap", ["chunks", "split"])
def test_virtual_ranks_random_graph_bfs_partition(cuda, overlap, layout):
    """A random 4-regular graph with per-edge weights, agents split by greedy BFS over 3 virtual
    ranks (irregular halos, every rank a different row-set shape): 3 rounds bit-identical to the
    single-device round, with the lagged deviation within 1e-5 of the exact one."""
    from distributed_learning_amd import engine as E
    from distributed_learning_amd.graph import random_regular_edges
    n, P, world = 300, 1024 + (20 if layout == "rows" else 0), 3
    edges = random_regular_edges(4, n, seed=11)
    rng = np.random.default_rng(3)
    csr = from_edge_weights(edges, list(rng.uniform(0.05, 0.2, len(edges))), list(range(n)))
    g = torch.Generator(device=cuda).manual_seed(2)
    X = torch.randn(n, P, device=cuda, generator=g)
    G = torch.randn(n, P, device=cuda, generator=g)
    ref = E.GossipEngine(csr, P, device=cuda, X=X, layout="rows")
    want = []
    for _ in range(3):
        want.append(tuple(t.clone() for t in ref.deviation()))
        ref.round(G=G, lr=0.02)
    parts = sharding.greedy_bfs_partition(csr, world)
    plans = (sharding.split_halo_plans if overlap == "split" else sharding.halo_plans)(csr, parts)
    tr = sharding.LocalTransport(world)
    shards = []
    for pl in plans:
        sh = sharding.HaloShard(pl, P, cuda, tr.endpoint(pl.rank), n_agents_total=n,
                                overlap=overlap, chunk_cols=None if overlap == "split" else 512,
                                layout=layout)
        assert sh.layout == layout
        ids = torch.as_tensor(pl.local, device=cuda)
        sh.load_rows(X[ids])
        shards.append((sh, sh.layout_like(G[ids]), ids))
    errs = []

    def run(sh, Gl):
        try:
            sh.got = [sh.round(G=Gl, lr=0.02, deviation=True) for _ in range(3)]
        except Exception as e:  # pragma: no cover
            errs.append(e)
    ths = [threading.Thread(target=run, args=(sh, Gl)) for sh, Gl, _ in shards]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
    torch.cuda.synchronize()
    full = ref.rows()
    for sh, _, ids in shards:
        assert torch.equal(sh.rows().view(torch.int32), full[ids].view(torch.int32))
        for (dsq, dmax), (wsq, wmax) in zip(sh.got, want):
            np.testing.assert_allclose(dsq.cpu().numpy(), wsq[ids].cpu().numpy(), rtol=1e-5)
            assert float(dmax.item()) == pytest.approx(float(wmax.item()), rel=1e-5)


C4_RANK_SHAPES = {8: (512, 96, [32, 32, 32]), 4: (1024, 128, [64, 64]), 2: (2048, 128, [128])}


@pytest.mark.parametrize("overlap", ["chunks", "split"])
@pytest.mark.parametrize("world", [8, 4, 2])
def test_c4_ranks_full_size_tiled(cuda, overlap, world):
    """BASELINE config c4 at full size on one GPU: the 64 x 64 torus x 2^18 params split over 8
    virtual ranks (32 x 16 blocks: 512 local + 96 halo rows each; at 4 ranks 1024 + 128 rows from
    two peers, at 2 ranks 2048 + 128 from one -- T = 16 / 8 / 4, three row passes each),
    column-tiled X / Y / G with per-peer tiled halo blocks -- the per-rank kernel an N-GPU run
    launches.  Three rounds with
    the lagged deviation are bit-identical to the single-device round, which itself equals the
    oracle's C restatement (oracle/cref) on a column slice; every lagged deviation is within 1e-5
    of the exact one.  Reference: the neighbour exchange it replaces,
    utils/consensus_asyncio.py:96-118 and consensus_tcp/agent.py:204-207."""
    from distributed_learning_amd import engine as E
    from distributed_learning_amd.graph import from_edge_weights as few
    from oracle import cref
    import math
    rows = cols = 64
    n, P, lr = rows * cols, 1 << 18, 1e-3
    n_local, n_halo, blocks = C4_RANK_SHAPES[world]
    edges = torus_edges(rows, cols)
    wc = 2.0 / (2.0 - 2.0 * math.cos(2 * math.pi / cols) + 8.0)
    csr = few(edges, [wc] * len(edges), list(range(n)))
    g = torch.Generator(device=cuda).manual_seed(41)
    X = torch.randn(n, P, device=cuda, generator=g)
    G = torch.randn(n, P, device=cuda, generator=g)
    cs = slice(1000, 1000 + 96)        # oracle column slice
    Xs, Gs = X[:, cs].cpu().numpy(), G[:, cs].cpu().numpy()
    ref = E.GossipEngine(csr, P, device=cuda, X=X)
    assert ref.layout == "tiled"
    Gt = ref.layout_like(G)
    want = []
    for _ in range(3):
        want.append(tuple(t.clone() for t in ref.deviation()))
        ref.round(G=Gt, lr=lr)
        Xs = cref.mix_round(Xs, csr.rowptr, csr.col, csr.w, G=Gs, lr=lr)
    del Gt
    full = ref.rows()
    assert np.array_equal(full[:, cs].cpu().numpy().view(np.uint32), Xs.view(np.uint32))
    del ref
    plans = (sharding.split_halo_plans if overlap == "split" else sharding.halo_plans)(
        csr, sharding.torus_block_partition(rows, cols, world))
    tr = sharding.LocalTransport(world)
    shards = []
    for pl in plans:
        assert (pl.n_local, pl.n_halo, len(pl.halo_from)) == (n_local, n_halo, len(blocks))
        sh = sharding.HaloShard(pl, P, cuda, tr.endpoint(pl.rank), n_agents_total=n,
                                overlap=overlap, chunk_cols=P // 8 if overlap == "chunks" else None)
        assert sh.layout == "tiled" and sh.halo_blocks == blocks
        if overlap == "split" and sh.W_bnd_packed is not None:
            # the boundary launch (276 / 372 / 384 source rows) walks groups of 2 / 4 / 8 data
            # tiles as one kernel tile of 32 columns (dl_mix_plan.n_tiles)
            bp = E.plan_shape(sh.W_bnd_packed, P, tile_cols=sh.T)
            assert bp["tile_cols"] == sh.T and bp["n_tiles"] == P // 32, bp
        ids = torch.as_tensor(pl.local, device=cuda)
        sh.load_rows(X[ids])
        shards.append((sh, sh.layout_like(G[ids]), ids))
    del X, G
    errs = []

    def run(sh, Gl):
        try:
            sh.got = [sh.round(G=Gl, lr=lr, deviation=True) for _ in range(3)]
        except Exception as e:  # pragma: no cover
            errs.append(e)
    ths = [threading.Thread(target=run, args=(sh, Gl)) for sh, Gl, _ in shards]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert not errs, errs
    torch.cuda.synchronize()
    for sh, _, ids in shards:
        assert torch.equal(sh.rows().view(torch.int32), full[ids].view(torch.int32))
        for (dsq, dmax), (wsq, wmax) in zip(sh.got, want):
            np.testing.assert_allclose(dsq.cpu().numpy(), wsq[ids].cpu().numpy(), rtol=1e-5)
            assert float(dmax.item()) == pytest.approx(float(wmax.item()), rel=1e-5)


class _Row(torch.nn.Module):
    """One agent's flattened parameter vector as a model (Mixer flattens model.parameters())."""

    def __init__(self, x):
        super().__init__()
        self.p = torch.nn.Parameter(x.clone())


@pytest.mark.parametrize("overlap", ["split", "chunks"])
@pytest.mark.parametrize("world", [8, 4, 2])
def test_halo_mix_stop_rule_equals_single_device_mixer(cuda, world, overlap):
    """HaloShard.mix(times, eps) -- Mixer.mix's stop rule (utils/consensus_simple/mixer.py:18-41)
    on the agent partition, lagged rounds with a one-round rollback -- on 8 / 4 / 2 virtual ranks
    of the c4 torus (64 x 64 agents, reduced to 4096 params): for several (times, eps), eps
    strictly between two rounds' deviations and within a few ulps of one, times_done and every
    agent's bits equal the single-device drop-in Mixer's on the same models."""
    import logging
    import math
    from distributed_learning_amd.graph import from_edge_weights as few
    from distributed_learning_amd.utils.consensus_simple import Mixer
    from oracle import mixer_ref as M
    rows = cols = 64
    n, P = rows * cols, 4096
    edges = torus_edges(rows, cols)
    wc = 2.0 / (2.0 - 2.0 * math.cos(2 * math.pi / cols) + 8.0)
    csr = few(edges, [wc] * len(edges), list(range(n)))
    topo = {a: {int(csr.col[e]): float(csr.w[e]) for e in range(csr.rowptr[a], csr.rowptr[a + 1])}
            for a in range(n)}
    g = torch.Generator(device=cuda).manual_seed(17)
    X0 = torch.randn(n, P, device=cuda, generator=g)
    # the oracle's deviation sequence (mixer.py:51-66) picks the eps values
    Xh, d = X0.cpu().numpy(), []
    for _ in range(6):
        d.append(np.float32(M.deviation(Xh).max()))
        Xh = M.mix_once(Xh, csr.rowptr, csr.col, csr.w)
    cases = [(1, float(np.sqrt(float(d[2]) * float(d[3])))), (4, float(np.sqrt(float(d[1]) *
                                                                                float(d[2])))),
             (0, float(d[0]) * 2), (1, float(d[4]) * (1 + 4e-7)), (2, None)]
    plans = (sharding.split_halo_plans if overlap == "split" else sharding.halo_plans)(
        csr, sharding.torus_block_partition(rows, cols, world))
    for times, eps in cases:
        models = {a: _Row(X0[a]) for a in range(n)}
        want_n = Mixer(models, topo, logging.getLogger("test")).mix(times, eps)
        want = torch.stack([models[a].p.data for a in range(n)])
        tr = sharding.LocalTransport(world)
        shards, errs = [], []
        for pl in plans:
            sh = sharding.HaloShard(pl, P, cuda, tr.endpoint(pl.rank), n_agents_total=n,
                                    overlap=overlap,
                                    chunk_cols=P // 2 if overlap == "chunks" else None)
            ids = torch.as_tensor(pl.local, device=cuda)
            sh.load_rows(X0[ids])
            shards.append((sh, ids))

        def run(sh):
            try:
                sh.done = sh.mix(times, eps)
            except Exception as e:  # pragma: no cover
                errs.append(e)
        ths = [threading.Thread(target=run, args=(sh,)) for sh, _ in shards]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        assert not errs, errs
        torch.cuda.synchronize()
        for sh, ids in shards:
            assert sh.done == want_n, (times, eps, sh.done, want_n)
            assert torch.equal(sh.rows().view(torch.int32), want[ids].view(torch.int32))
