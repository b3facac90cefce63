"""Config c5 on the GPU: the local-step kernel (dl_sgd_step) against its C oracle and against
torch.optim.SGD, and the resident WRN consensus-SGD workload against the reference-style loop
(per-agent torch modules + optim.SGD on the CPU, then the numpy Mixer round)."""
import os

import numpy as np
import pytest
import torch

os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")   # small test shapes: skip MIOpen's search

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,p,ld,inplace,momentum,nesterov", [
    (5, 4096, 4096, False, 0.9, False),      # float4 path
    (3, 1001, 1003, True, 0.9, False),       # scalar path, in place
    (4, 2048, 2052, False, 0.0, False),      # no momentum buffer
    (2, 640, 640, True, 0.9, True),          # Nesterov
])
def test_sgd_step_matches_oracle(cuda, n, p, ld, inplace, momentum, nesterov):
    from distributed_learning_amd.workloads import sgd_step
    from oracle import cref
    rng = np.random.default_rng(5)
    X = rng.standard_normal((n, ld)).astype(np.float32)
    Xd = torch.from_numpy(X).to(cuda)[:, :p]
    Md = torch.zeros(n, ld, device=cuda)[:, :p] if momentum else None
    Sd = Xd if inplace else torch.full((n, ld), float("nan"), device=cuda)[:, :p]
    x = X[:, :p].copy()
    buf = np.zeros_like(x) if momentum else None
    for step in range(3):
        G = rng.standard_normal((n, p)).astype(np.float32)
        out = sgd_step(Xd, torch.from_numpy(G).to(cuda), Md, out=Sd, lr=0.05,
                       momentum=momentum, weight_decay=5e-4, nesterov=nesterov, first=step == 0)
        x = cref.sgd_step(x, G, buf, lr=0.05, momentum=momentum, weight_decay=5e-4,
                          nesterov=nesterov, first=step == 0)
        got = out.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), x.view(np.uint32)), step
        if not inplace:
            Xd.copy_(out)
        if momentum:
            assert np.array_equal(Md.cpu().numpy().view(np.uint32), buf.view(np.uint32))


def test_sgd_step_vs_torch_optimizer(cuda):
    """torch.optim.SGD on the GPU (foreach kernels): at most one ulp apart (its fused
    add-with-alpha is an fma when the compiler contracts it, as the kernel's explicit fma)."""
    from distributed_learning_amd.workloads import sgd_step
    torch.manual_seed(0)
    X = torch.randn(4, 8192, device=cuda)
    ps = [torch.nn.Parameter(X[i].clone()) for i in range(4)]
    opt = torch.optim.SGD(ps, lr=0.02, momentum=0.9, weight_decay=5e-4)
    M = torch.zeros_like(X)
    for step in range(3):
        G = torch.randn_like(X)
        for i, p in enumerate(ps):
            p.grad = G[i].clone()
        opt.step()
        sgd_step(X, G, M, lr=0.02, momentum=0.9, weight_decay=5e-4, first=step == 0)
        want = torch.stack([p.detach() for p in ps])
        ulp = (want.view(torch.int32) - X.view(torch.int32)).abs().max().item()
        assert ulp <= 1, ulp


def _reference_models(n, arch, seed, X0):
    from distributed_learning_amd.networks.wide_resnet import Wide_ResNet
    from oracle import consensus_sgd_ref as R
    models = []
    for a in range(n):
        m = Wide_ResNet(*arch)
        R.load_flat(m, X0[a])
        models.append(m)
    return models


@pytest.mark.parametrize("streams", [1, 2])
def test_wrn_consensus_matches_reference_loop(cuda, streams):
    """2 steps of 4 agents (WRN-10-1, B = 6) on a ring with per-agent weights: the resident
    workload vs one CPU torch module + optim.SGD per agent and the numpy Mixer round.  Tolerance
    1e-5 relative in fp32 (MIOpen's and the CPU's conv summation orders differ; the mix itself
    is bit-exact, tested elsewhere)."""
    from distributed_learning_amd.graph import Csr
    from distributed_learning_amd.workloads import WRNConsensusSGD
    from oracle import consensus_sgd_ref as R
    from oracle import mixer_ref
    n, B, arch = 4, 6, (10, 1, 0.0, 10)
    topo = {0: {0: 0.5, 1: 0.25, 3: 0.25}, 1: {1: 0.6, 0: 0.25, 2: 0.15},
            2: {2: 0.6, 1: 0.15, 3: 0.25}, 3: {3: 0.5, 2: 0.25, 0: 0.25}}
    rp, cols, w = mixer_ref.topology_to_csr(topo)
    csr = Csr(rp, cols, w)
    g = torch.Generator().manual_seed(3)
    data = torch.randn(n, B, 3, 32, 32, generator=g)
    labels = torch.randint(0, 10, (n, B), generator=g)
    wl = WRNConsensusSGD(csr, B, *arch, lr=0.05, momentum=0.9, weight_decay=5e-4, device=cuda,
                         seed=7, streams=streams, data=data.to(cuda), labels=labels.to(cuda))
    X0 = wl.params().cpu().numpy().copy()
    models = _reference_models(n, arch, 7, X0)
    opts = [torch.optim.SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4,
                            foreach=False) for m in models]
    ref_losses = R.consensus_sgd_steps(models, opts, data, labels, rp, cols, w, 2)
    for _ in range(2):
        wl.step()
    torch.cuda.synchronize()
    got = wl.params().cpu().numpy()
    want = np.stack([R.flatten(m) for m in models])
    scale = np.maximum(np.abs(want), 1e-2)
    assert np.max(np.abs(got - want) / scale) < 1e-5
    np.testing.assert_allclose(wl.loss.cpu().numpy(), ref_losses[-1], rtol=1e-5)
    # the padding columns stay exactly zero; the fused deviation is the Mixer's
    assert not wl.X[:, wl.P:].any()
    dev = mixer_ref.deviation(got)
    np.testing.assert_allclose(np.sqrt(wl.dev_sq.cpu().numpy()), dev, rtol=1e-5)
    # the module parameters are views of X's rows (nothing copied per step)
    p0 = next(wl.models[1].parameters())
    assert p0.data_ptr() == wl.X[1].data_ptr()


@pytest.fixture
def deterministic_convs():
    """MIOpen's default conv/BN solvers are not run-to-run deterministic (split-K atomics): two
    eager runs differ by ~1e-8 after one step.  Deterministic solvers make runs comparable bit
    for bit."""
    old = torch.backends.cudnn.deterministic
    torch.backends.cudnn.deterministic = True
    yield
    torch.backends.cudnn.deterministic = old


def test_wrn_graph_replay_matches_eager(cuda, deterministic_convs):
    """The hipGraph replay of a step is the eager step, bit for bit."""
    from distributed_learning_amd.graph import best_constant_weight, uniform_weights
    from distributed_learning_amd.workloads import WRNConsensusSGD
    edges = [(i, (i + 1) % 4) for i in range(4)]
    csr = uniform_weights(edges, best_constant_weight(edges))
    kw = dict(depth=10, widen=1, lr=0.05, device=cuda, seed=1)
    a = WRNConsensusSGD(csr, 4, **kw)
    b = WRNConsensusSGD(csr, 4, **kw)
    a.step()
    b.step()
    b.capture()
    for _ in range(2):
        a.step()
    b.replay(2)
    torch.cuda.synchronize()
    assert torch.equal(a.params(), b.params())
    assert torch.equal(a.M, b.M) and torch.equal(a.loss, b.loss)
    assert a.steps_done == b.steps_done == 3
