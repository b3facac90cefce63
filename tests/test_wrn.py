"""Config c5 host side on the CPU: the Wide-ResNet restatement (parameter count and Mixer
flatten order), the analytic FLOP count, and the local-step oracle (torch.optim.SGD restated in C)
against torch's own CPU optimizer."""
import numpy as np
import pytest
import torch

from distributed_learning_amd.networks.wide_resnet import Wide_ResNet
from distributed_learning_amd.workloads import wrn_flops_per_image
from oracle import cref


def test_wrn16_4_parameters():
    m = Wide_ResNet(16, 4, 0.0, 10)
    names = [n for n, _ in m.named_parameters()]
    assert sum(p.numel() for p in m.parameters()) == 2_751_146
    assert len(names) == 60
    # registration order = the Mixer flatten order (mixer.py:68-69)
    assert names[:6] == ["conv1.weight", "conv1.bias", "layer1.0.bn1.weight",
                         "layer1.0.bn1.bias", "layer1.0.conv1.weight", "layer1.0.conv1.bias"]
    assert names[10:12] == ["layer1.0.shortcut.0.weight", "layer1.0.shortcut.0.bias"]
    assert names[-4:] == ["bn1.weight", "bn1.bias", "linear.weight", "linear.bias"]
    with pytest.raises(ValueError):
        Wide_ResNet(15, 4, 0.0, 10)


@pytest.mark.parametrize("depth,widen", [(16, 4), (10, 1), (28, 2)])
def test_flops_formula_matches_hooks(depth, widen):
    m = Wide_ResNet(depth, widen, 0.0, 10)
    macs = []

    def hook(mod, inp, out):
        if isinstance(mod, torch.nn.Conv2d):
            k = mod.kernel_size[0] * mod.kernel_size[1]
            macs.append(out.numel() * mod.in_channels * k)
        elif isinstance(mod, torch.nn.Linear):
            macs.append(out.numel() * mod.in_features)
    for mod in m.modules():
        mod.register_forward_hook(hook)
    with torch.no_grad():
        m(torch.zeros(1, 3, 32, 32))
    fwd, total = wrn_flops_per_image(depth, widen, 10)
    assert fwd == 2 * sum(macs)
    assert total == 3 * fwd - 2 * 3 * 16 * 9 * 32 * 32


@pytest.mark.parametrize("momentum,damp,wd,nesterov", [(0.9, 0.0, 5e-4, False),
                                                       (0.0, 0.0, 1e-2, False),
                                                       (0.5, 0.1, 0.0, False),
                                                       (0.9, 0.0, 1e-3, True)])
def test_sgd_oracle_is_torch_sgd(momentum, damp, wd, nesterov):
    """oracle/mix_ref.c ref_sgd_step == torch.optim.SGD.step (CPU, single-tensor), bit for bit,
    over three steps (the first one clones the gradient into the buffer)."""
    rng = np.random.default_rng(1)
    X = rng.standard_normal((3, 1031)).astype(np.float32)
    ps = [torch.nn.Parameter(torch.from_numpy(X[i].copy())) for i in range(3)]
    opt = torch.optim.SGD(ps, lr=0.02, momentum=momentum, dampening=damp, weight_decay=wd,
                          nesterov=nesterov, foreach=False)
    buf = np.zeros_like(X) if momentum else None
    x = X.copy()
    for step in range(3):
        G = rng.standard_normal(X.shape).astype(np.float32)
        for i, p in enumerate(ps):
            p.grad = torch.from_numpy(G[i].copy())
        opt.step()
        x = cref.sgd_step(x, G, buf, lr=0.02, momentum=momentum, dampening=damp,
                          weight_decay=wd, nesterov=nesterov, first=step == 0)
        want = np.stack([p.detach().numpy() for p in ps])
        assert np.array_equal(want.view(np.uint32), x.view(np.uint32)), step
