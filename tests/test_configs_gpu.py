"""BASELINE configs c3 and c5 at their stated shapes on the GPU.

c3: 256 agents x ANNModel(784, 150, 10), B = 64, random 4-regular graph -- three consensus SGD
    steps of ``workloads.MLPConsensusSGD``.  Every step is checked in two parts:
      * gradients: the fused kernel's G against per-agent torch autograd.  fp32 GEMMs in two
        different summation orders cannot agree bitwise, so the bar is stated against the truth
        (the same autograd in fp64): the kernel's error is within 2x torch fp32's own error per
        agent, and its norm-wise relative error is below 1e-5;
      * round: X' == W (X - lr G) computed by the C oracle (oracle/cref.mix_round) from the same
        X and the kernel's own G -- bit for bit (the mix is exact, tests/test_mix_gpu.py).
c5: Wide-ResNet-16-4.  3 agents of the full model against the reference-style CPU loop
    (oracle/consensus_sgd_ref: per-agent torch modules + optim.SGD + the numpy Mixer round), and
    the full 64-agent, B = 64 step with property checks: two agents' local SGD steps against
    standalone torch models, the round bit-exact from the stepped rows, the deviation against
    the oracle, the agent mean preserved by the doubly stochastic W.
"""
import os

import numpy as np
import pytest
import torch

os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")

pytestmark = pytest.mark.gpu


def _flat_grads(m):
    return torch.cat([p.grad.reshape(-1) for p in m.parameters()])


def _load(model, vec):
    off = 0
    for p in model.parameters():
        n = p.numel()
        p.data.copy_(vec[off:off + n].view_as(p))
        off += n


def test_c3_full_shape_three_steps(cuda):
    from distributed_learning_amd import engine
    from distributed_learning_amd.graph import from_edge_weights, random_regular_edges
    from distributed_learning_amd.networks import ANNModel
    from distributed_learning_amd.networks.batched_ann import BatchedANN
    from distributed_learning_amd.workloads import MLPConsensusSGD
    from oracle import cref
    n, b, dims, lr = 256, 64, (784, 150, 10), 0.05
    gen = torch.Generator(device=cuda).manual_seed(0)
    edges = random_regular_edges(4, n, seed=0)
    csr = from_edge_weights(edges, [0.2] * len(edges), list(range(n)))
    bann = BatchedANN(n, b, *dims, device=cuda)
    assert bann.path == "fused" and bann.P == 164_560
    torch.manual_seed(0)
    X0 = torch.stack([torch.cat([p.data.reshape(-1) for p in ANNModel(*dims).parameters()])
                      for _ in range(n)]).to(cuda)
    data = torch.randn(n, b, dims[0], device=cuda, generator=gen)
    labels = torch.randint(0, dims[2], (n, b), device=cuda, generator=gen, dtype=torch.int32)
    P = bann.P
    cols = MLPConsensusSGD.padded_params(csr, P, cuda)
    eng = engine.GossipEngine(csr, cols, device=cuda,
                              X=torch.nn.functional.pad(X0, (0, cols - P)), layout="rows")
    sgd = MLPConsensusSGD(bann, eng, data, labels, lr=lr)
    m32, m64 = ANNModel(*dims).to(cuda), ANNModel(*dims).to(cuda).double()
    worst_ratio, worst_rel = 0.0, 0.0
    for step in range(3):
        X = eng.X[:, :P].clone()
        sgd.step()
        torch.cuda.synchronize()
        G = sgd.G[:, :P]
        for a in range(n):
            g = []
            for m, dt in ((m32, torch.float32), (m64, torch.float64)):
                _load(m, X[a].to(dt))
                m.zero_grad()
                torch.nn.functional.cross_entropy(m(data[a].to(dt)), labels[a].long()).backward()
                g.append(_flat_grads(m))
            truth = g[1]
            err_kernel = (G[a].double() - truth).abs().max().item()
            err_torch = (g[0].double() - truth).abs().max().item()
            rel = ((G[a].double() - truth).norm() / truth.norm()).item()
            worst_rel = max(worst_rel, rel)
            worst_ratio = max(worst_ratio, err_kernel / max(err_torch, 1e-12))
            assert rel < 1e-5, (step, a, rel)
            assert err_kernel <= 2.0 * err_torch + 1e-9, (step, a, err_kernel, err_torch)
        want = cref.mix_round(X.cpu().numpy(), csr.rowptr, csr.col, csr.w,
                              G=G.cpu().numpy(), lr=lr)
        got = eng.X[:, :P].cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), step
        assert torch.all(eng.X[:, P:] == 0)
    print(f"c3 gradients: worst kernel/torch-fp32 error ratio {worst_ratio:.2f}, "
          f"worst norm-wise relative error vs fp64 {worst_rel:.2e}")


def _wrn_reference(n, arch, X0):
    from distributed_learning_amd.networks.wide_resnet import Wide_ResNet
    from oracle import consensus_sgd_ref as R
    models = []
    for a in range(n):
        m = Wide_ResNet(*arch)
        R.load_flat(m, X0[a])
        models.append(m)
    return models


def test_c5_wrn16_4_three_agents_vs_reference_loop(cuda):
    """The full WRN-16-4 (2,751,146 params) on 3 agents, B = 4, 2 steps vs the CPU reference
    loop (momentum 0.9, weight decay 5e-4, lr 0.02 as Man_Colab cell 19).  fp32 on both sides
    with different conv summation orders (MIOpen vs the CPU): 2e-5 of the parameter scale."""
    from distributed_learning_amd.graph import Csr
    from distributed_learning_amd.workloads import WRNConsensusSGD
    from oracle import consensus_sgd_ref as R
    from oracle import mixer_ref
    n, B, arch = 3, 4, (16, 4, 0.0, 10)
    topo = {0: {0: 0.5, 1: 0.25, 2: 0.25}, 1: {1: 0.5, 0: 0.25, 2: 0.25},
            2: {2: 0.5, 1: 0.25, 0: 0.25}}
    rp, cols, w = mixer_ref.topology_to_csr(topo)
    csr = Csr(rp, cols, w)
    g = torch.Generator().manual_seed(4)
    data = torch.randn(n, B, 3, 32, 32, generator=g)
    labels = torch.randint(0, 10, (n, B), generator=g)
    wl = WRNConsensusSGD(csr, B, *arch, lr=0.02, momentum=0.9, weight_decay=5e-4, device=cuda,
                         seed=5, data=data.to(cuda), labels=labels.to(cuda))
    assert wl.P == 2_751_146
    X0 = wl.params().cpu().numpy().copy()
    models = _wrn_reference(n, arch, X0)
    opts = [torch.optim.SGD(m.parameters(), lr=0.02, momentum=0.9, weight_decay=5e-4,
                            foreach=False) for m in models]
    ref_losses = R.consensus_sgd_steps(models, opts, data, labels, rp, cols, w, 2)
    for _ in range(2):
        wl.step()
    torch.cuda.synchronize()
    got = wl.params().cpu().numpy()
    want = np.stack([R.flatten(m) for m in models])
    scale = np.maximum(np.abs(want), 1e-2)
    assert np.max(np.abs(got - want) / scale) < 2e-5
    np.testing.assert_allclose(wl.loss.cpu().numpy(), ref_losses[-1], rtol=1e-5)
    np.testing.assert_allclose(np.sqrt(wl.dev_sq.cpu().numpy()), mixer_ref.deviation(got),
                               rtol=1e-5)


def test_c5_wrn16_4_sixty_four_agents_step(cuda):
    """BASELINE c5 itself: 64 agents x WRN-16-4, B = 64, random 4-regular graph, one step."""
    from distributed_learning_amd.graph import (best_constant_weight, random_regular_edges,
                                                uniform_weights)
    from distributed_learning_amd.networks.wide_resnet import Wide_ResNet
    from distributed_learning_amd.workloads import WRNConsensusSGD
    from oracle import cref, mixer_ref
    n, B = 64, 64
    edges = random_regular_edges(4, n, seed=0)
    csr = uniform_weights(edges, best_constant_weight(edges))
    wl = WRNConsensusSGD(csr, B, 16, 4, lr=0.02, momentum=0.9, weight_decay=5e-4, device=cuda,
                         seed=0, streams=8)
    X0 = wl.params().clone()
    wl.step()
    torch.cuda.synchronize()
    P = wl.P
    S = wl.S[:, :P]
    X1 = wl.params()
    assert torch.isfinite(X1).all() and torch.isfinite(wl.loss).all()
    # the round, bit for bit, from the stepped rows
    want = cref.mix_round(S.cpu().numpy(), csr.rowptr, csr.col, csr.w)
    assert np.array_equal(X1.cpu().numpy().view(np.uint32), want.view(np.uint32))
    # doubly stochastic W: the agent mean of S is preserved (fp32 rounding)
    torch.testing.assert_close(X1.double().mean(0), S.double().mean(0), rtol=0, atol=1e-6)
    np.testing.assert_allclose(np.sqrt(wl.dev_sq.cpu().numpy()),
                               mixer_ref.deviation(X1.cpu().numpy()), rtol=1e-5)
    # two agents' local steps against standalone torch modules (first SGD step: buf = g + wd x)
    for a in (0, 37):
        m = Wide_ResNet(16, 4, 0.0, 10).to(cuda)
        _load(m, X0[a])
        m.zero_grad()
        loss = torch.nn.functional.cross_entropy(m(wl.data[a]), wl.labels[a])
        loss.backward()
        opt = torch.optim.SGD(m.parameters(), lr=0.02, momentum=0.9, weight_decay=5e-4)
        opt.step()
        ref = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
        scale = ref.abs().clamp_min(1e-2)
        assert ((S[a] - ref).abs() / scale).max().item() < 1e-5, a
        assert wl.loss[a].item() == pytest.approx(loss.item(), rel=1e-5)
