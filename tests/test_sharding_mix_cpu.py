"""The agent-partitioned path over real gloo processes on the CPU (oracle ops stand in for the
device kernels; the halo protocol, the lagged deviation and the stop rule are the product's):

* ``HaloShard.mix(times, eps)`` -- the reference's ``Mixer.mix`` stop rule
  (utils/consensus_simple/mixer.py:18-41) on a partition: the round count and the returned
  iterate equal the single-process oracle's for several (times, eps), near-ties included;
* the exact geometry of the driver's 8-GPU job: the 64 x 64 torus of c4 in 2 x 4 blocks of
  32 x 16 agents (3 peers per rank: the blocks above and below are one peer across the wrap),
  column-tiled operands and per-peer halo blocks, all three overlap schemes (whole, chunks,
  split) with the lagged deviation, bit-exact against single-process oracle rounds
  (consensus_asyncio.py:96-118's neighbour exchange, replaced by the halo exchange)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from distributed_learning_amd import sharding
from distributed_learning_amd.graph import best_constant_weight, from_edge_weights, torus_edges
from oracle import mixer_ref as M


_WEIGHT = {}


def torus_csr(r, c, w=None):
    """The r x c torus with its best-constant weight (computed once per process: a dense
    eigendecomposition at 4096 agents; the spawned ranks get it from the parent)."""
    edges = torus_edges(r, c)
    verts = list(range(r * c))
    if w is None:
        if (r, c) not in _WEIGHT:
            _WEIGHT[(r, c)] = best_constant_weight(edges, verts)
        w = _WEIGHT[(r, c)]
    return from_edge_weights(edges, [w] * len(edges), verts)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    torch.set_num_threads(1)          # world ranks on the container's cores
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def _counting(sh):
    """Count the exact near-tie re-evaluations HaloShard.mix makes."""
    calls = [0]
    orig = sh.exact_max_deviation

    def wrapped(A=None):
        calls[0] += 1
        return orig(A)
    sh.exact_max_deviation = wrapped
    return calls


def _mix_worker(rank, world, port, side, P, out_dir, cases, overlap, layout, w):
    _init(rank, world, port)
    from shard_oracle_ops import OracleOps
    csr = torus_csr(side, side, w)
    n = side * side
    parts = sharding.torus_block_partition(side, side, world)
    plan = (sharding.split_halo_plans if overlap == "split" else sharding.halo_plans)(
        csr, parts)[rank]
    X0 = np.random.default_rng(11).standard_normal((n, P), dtype=np.float32)
    sh = sharding.HaloShard(plan, P, "cpu", sharding.dist_transport(), n_agents_total=n,
                            ops=OracleOps(), overlap=overlap, layout=layout)
    calls = _counting(sh)
    for i, (times, eps) in enumerate(cases):
        sh.load_rows(torch.from_numpy(X0[plan.local].copy()))
        calls[0] = 0
        done = sh.mix(times, eps)
        np.save(os.path.join(out_dir, f"x{rank}_{i}.npy"), sh.rows().numpy())
        np.save(os.path.join(out_dir, f"n{rank}_{i}.npy"), np.asarray([done, calls[0]]))
    np.save(os.path.join(out_dir, f"ids{rank}.npy"), plan.local)
    dist.destroy_process_group()


def _deviations(X, csr, k):
    """The oracle's max deviation of X_0 .. X_k (mixer.py:51-66)."""
    out = []
    for _ in range(k + 1):
        out.append(np.float32(M.deviation(X).max()))
        X = M.mix_once(X, csr.rowptr, csr.col, csr.w)
    return out


def _check_mix(tmp_path, world, side, P, cases, overlap, layout, want_recheck=()):
    csr = torus_csr(side, side)
    mp.spawn(_mix_worker, args=(world, _free_port(), side, P, str(tmp_path), cases, overlap,
                                layout, _WEIGHT[(side, side)]), nprocs=world, join=True)
    X0 = np.random.default_rng(11).standard_normal((side * side, P), dtype=np.float32)
    for i, (times, eps) in enumerate(cases):
        want, want_n = M.mixer_mix(X0, csr.rowptr, csr.col, csr.w, times, eps)
        for r in range(world):
            ids = np.load(tmp_path / f"ids{r}.npy")
            done, rechecks = np.load(tmp_path / f"n{r}_{i}.npy")
            assert done == want_n, (i, times, eps, r, done, want_n)
            got = np.load(tmp_path / f"x{r}_{i}.npy")
            assert np.array_equal(got.view(np.uint32), want[ids].view(np.uint32)), (i, r)
            if i in want_recheck:
                assert rechecks >= 1, (i, r)


def _cases(side, P):
    """(times, eps) pairs around the oracle's own deviation sequence: stops strictly between two
    rounds' deviations, a times bound that dominates, eps above the start (times 0: no round at
    all), eps None, and two near-ties a few ulps either side of a round's exact deviation."""
    csr = torus_csr(side, side)
    X0 = np.random.default_rng(11).standard_normal((side * side, P), dtype=np.float32)
    d = _deviations(X0, csr, 7)
    mid = lambda k: float(np.sqrt(float(d[k]) * float(d[k + 1])))   # noqa: E731
    return [(1, mid(3)), (6, mid(2)), (0, float(d[0]) * 2), (3, None), (0, mid(0)),
            (1, float(d[5]) * (1 + 4e-7)), (1, float(d[5]) * (1 - 4e-7))]


@pytest.mark.parametrize("overlap,layout", [("chunks", "tiled"), ("split", "tiled"),
                                            ("chunks", "rows")])
def test_halo_mix_stop_rule_two_gloo_ranks(tmp_path, overlap, layout):
    """HaloShard.mix(times, eps) on 2 gloo ranks of an 8 x 8 torus: times_done and the returned
    bits equal the oracle's Mixer.mix for every case; the near-tie cases re-evaluate the
    lagged deviation exactly (the single-device Mixer's tie rule)."""
    P = 24
    _check_mix(tmp_path, 2, 8, P, _cases(8, P), overlap, layout, want_recheck=(5, 6))


def _geom_worker(rank, world, port, P, out_dir, w):
    _init(rank, world, port)
    from shard_oracle_ops import OracleOps
    side, n = 64, 64 * 64
    csr = torus_csr(side, side, w)
    parts = sharding.torus_block_partition(side, side, world)
    rng = np.random.default_rng(3)
    X = rng.standard_normal((n, P), dtype=np.float32)
    G = rng.standard_normal((n, P), dtype=np.float32)
    tr = sharding.dist_transport()
    for scheme, overlap, chunk in (("whole", "chunks", None), ("chunks", "chunks", P // 2),
                                   ("split", "split", None)):
        plan = (sharding.split_halo_plans if overlap == "split" else sharding.halo_plans)(
            csr, parts)[rank]
        sh = sharding.HaloShard(plan, P, "cpu", tr, chunk_cols=chunk, n_agents_total=n,
                                ops=OracleOps(), overlap=overlap, layout="tiled")
        assert sh.layout == "tiled" and len(sh.chunks()) == (2 if scheme == "chunks" else 1)
        sh.load_rows(torch.from_numpy(X[plan.local].copy()))
        Gl = sh.layout_like(torch.from_numpy(G[plan.local].copy()))
        devs = [float(sh.round(G=Gl, lr=0.05, deviation=True)[1]) for _ in range(2)]
        np.save(os.path.join(out_dir, f"{scheme}_x{rank}.npy"), sh.rows().numpy())
        np.save(os.path.join(out_dir, f"{scheme}_dev{rank}.npy"), np.asarray(devs))
        np.save(os.path.join(out_dir, f"{scheme}_ids{rank}.npy"), plan.local)
        np.save(os.path.join(out_dir, f"{scheme}_peers{rank}.npy"),
                np.asarray([len(plan.send_to), len(plan.halo_from), plan.n_local, plan.n_halo]))
    dist.destroy_process_group()


def test_c4_geometry_eight_gloo_ranks(tmp_path):
    """The driver's N = 8 agent partition on the CPU: 64 x 64 torus, 2 x 4 blocks of 512
    agents with 96 halo rows from 3 peers each, column-tiled, lagged deviation; whole, chunks
    and split rounds bit-identical to single-process oracle rounds, each round's lagged
    deviation within 1e-5 of the oracle's deviation of the iterate it started from."""
    world, P = 8, 64
    csr = torus_csr(64, 64)
    mp.spawn(_geom_worker, args=(world, _free_port(), P, str(tmp_path), _WEIGHT[(64, 64)]),
             nprocs=world, join=True)
    rng = np.random.default_rng(3)
    X = rng.standard_normal((4096, P), dtype=np.float32)
    G = rng.standard_normal((4096, P), dtype=np.float32)
    devs = []
    want = X
    for _ in range(2):
        devs.append(M.deviation(want).max())
        want = M.mix_once(M.sgd_step(want, G, 0.05), csr.rowptr, csr.col, csr.w)
    for scheme in ("whole", "chunks", "split"):
        for r in range(world):
            peers, halo_from, n_local, n_halo = np.load(tmp_path / f"{scheme}_peers{r}.npy")
            assert (peers, halo_from, n_local, n_halo) == (3, 3, 512, 96), (scheme, r)
            ids = np.load(tmp_path / f"{scheme}_ids{r}.npy")
            got = np.load(tmp_path / f"{scheme}_x{r}.npy")
            assert np.array_equal(got.view(np.uint32), want[ids].view(np.uint32)), (scheme, r)
            np.testing.assert_allclose(np.load(tmp_path / f"{scheme}_dev{r}.npy"), devs,
                                       rtol=1e-5)


def test_c4_geometry_stop_rule_eight_gloo_ranks(tmp_path):
    """HaloShard.mix(times, eps) on the same 8-rank geometry (split rounds, column-tiled; a
    reduced column count): the reference's round count and iterate."""
    side, P = 64, 8
    csr = torus_csr(side, side)
    X0 = np.random.default_rng(11).standard_normal((side * side, P), dtype=np.float32)
    d = _deviations(X0, csr, 4)
    cases = [(1, float(np.sqrt(float(d[2]) * float(d[3])))), (2, None)]
    _check_mix(tmp_path, 8, side, P, cases, "split", "tiled")
