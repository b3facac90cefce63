"""Batched per-agent MLP gradients (config c3) against plain PyTorch fp32 autograd, one
ANNModel per agent (reference networks/ann_model.py + torch.nn.CrossEntropyLoss)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _flat_grads(m):
    return torch.cat([p.grad.reshape(-1) for p in m.parameters()])


@pytest.mark.parametrize("n,b,dims", [(4, 64, (784, 150, 10)), (7, 33, (50, 40, 7)),
                                      (3, 5, (20, 15, 3))])
def test_gradients_match_autograd(cuda, n, b, dims):
    from distributed_learning_amd.networks import ANNModel
    from distributed_learning_amd.networks.batched_ann import BatchedANN
    din, dh, dout = dims
    torch.manual_seed(0)
    models = [ANNModel(din, dh, dout).to(cuda) for _ in range(n)]
    X = torch.stack([torch.cat([p.data.reshape(-1) for p in m.parameters()]) for m in models])
    data = torch.randn(n, b, din, device=cuda)
    labels = torch.randint(0, dout, (n, b), device=cuda, dtype=torch.int32)
    bann = BatchedANN(n, b, din, dh, dout, device=cuda)
    assert bann.P == X.shape[1]
    G = torch.full_like(X, float("nan"))
    loss = bann.gradients(X, data, labels, G).clone()
    torch.cuda.synchronize()
    for a, m in enumerate(models):
        m.zero_grad()
        ref_loss = torch.nn.functional.cross_entropy(m(data[a]), labels[a].long())
        ref_loss.backward()
        ref = _flat_grads(m)
        assert torch.isfinite(G[a]).all()
        scale = ref.abs().max().item()
        np.testing.assert_allclose(G[a].cpu().numpy(), ref.cpu().numpy(), rtol=1e-4,
                                   atol=1e-5 * scale)
        assert loss[a].item() == pytest.approx(ref_loss.item(), rel=1e-5)


def test_consensus_sgd_round_with_batched_grads(cuda):
    """One c3 round: G from the batched kernels, then the fused local step + mix; equals the
    per-agent autograd step followed by the oracle mix (to fp32 GEMM rounding)."""
    from distributed_learning_amd import engine
    from distributed_learning_amd.graph import from_edge_weights, random_regular_edges
    from distributed_learning_amd.networks import ANNModel
    from distributed_learning_amd.networks.batched_ann import BatchedANN
    from oracle import cref
    n, b = 16, 32
    torch.manual_seed(1)
    models = [ANNModel(64, 32, 10).to(cuda) for _ in range(n)]
    X = torch.stack([torch.cat([p.data.reshape(-1) for p in m.parameters()]) for m in models])
    data = torch.randn(n, b, 64, device=cuda)
    labels = torch.randint(0, 10, (n, b), device=cuda, dtype=torch.int32)
    edges = random_regular_edges(4, n, seed=0)
    csr = from_edge_weights(edges, [0.2] * len(edges), list(range(n)))
    bann = BatchedANN(n, b, 64, 32, 10, device=cuda)
    eng = engine.GossipEngine(csr, bann.P, device=cuda, X=X, layout="rows")
    G = torch.empty_like(X)
    bann.gradients(eng.X, data, labels, G)
    eng.round(G=G, lr=0.1)
    torch.cuda.synchronize()
    grads = []
    for a, m in enumerate(models):
        m.zero_grad()
        torch.nn.functional.cross_entropy(m(data[a]), labels[a].long()).backward()
        grads.append(_flat_grads(m))
    want = cref.mix_round(X.cpu().numpy(), csr.rowptr, csr.col, csr.w,
                          G=torch.stack(grads).cpu().numpy(), lr=0.1)
    np.testing.assert_allclose(eng.rows().cpu().numpy(), want, rtol=1e-5, atol=1e-6)
