"""Agent-partitioned halo rounds on one MI355X with virtual ranks (threads + LocalTransport):
the HIP halo path (dl_step_rows + dl_mix_round with n_halo) equals the single-device round."""
import threading

import numpy as np
import pytest
import torch

from distributed_learning_amd import sharding
from distributed_learning_amd.graph import best_constant_weight, from_edge_weights, torus_edges

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,chunk", [(2, None), (4, 300), (8, 1000)])
def test_virtual_ranks_equal_single_device(cuda, world, chunk):
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
    plans = sharding.halo_plans(csr, sharding.torus_block_partition(R, C, world))
    tr = sharding.LocalTransport(world)
    shards = []
    for pl in plans:
        sh = sharding.HaloShard(pl, P, cuda, tr.endpoint(pl.rank), chunk_cols=chunk,
                                n_agents_total=R * C)
        ids = torch.as_tensor(pl.local, device=cuda)
        sh.X = X[ids].contiguous()
        shards.append((sh, G[ids].contiguous(), ids))
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
        assert torch.equal(sh.X.view(torch.int32), full[ids].view(torch.int32))
    dsq, dmax = ref.deviation()
    for sh, _, ids in shards:
        assert float(sh.dev[1].item()) == pytest.approx(float(dmax.item()), rel=1e-5)
        np.testing.assert_allclose(sh.dev[0].cpu().numpy(), dsq[ids].cpu().numpy(), rtol=1e-5)
