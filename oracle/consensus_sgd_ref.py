"""Reference-style consensus SGD loop on the CPU (TEST INFRASTRUCTURE ONLY).

Restates the training loop the reference's consensus notebooks drive (Man_Colab.ipynb cells
19-23: per-agent ``optimizer.step()`` with optim.SGD(momentum, weight_decay), then
``Mixer.mix``) with one torch ``nn.Module`` + optimizer per agent, exactly as the reference
holds them:
  * local step: ``zero_grad``, ``CrossEntropyLoss``, ``backward``, ``step`` per agent;
  * mix: ``Mixer._get_flatten_model_params`` (mixer.py:68-69: fp32 flatten in
    ``model.parameters()`` order) -> ``_mix_params_once`` (mixer.py:43-49, numpy left fold:
    ``mixer_ref.mix_once``) -> ``_load_flatten_params_to_model`` (mixer.py:71-76).
Used only as the checker of ``workloads.WRNConsensusSGD`` in tests/test_wrn_gpu.py.
"""
import numpy as np
import torch

from . import mixer_ref


def flatten(model, dtype=torch.float32):
    """mixer.py:68-69 (dtype=float64 only for the tests' fp64 truth runs)"""
    return torch.cat([p.data.to(dtype).view(-1) for p in model.parameters()]).numpy()


def load_flat(model, vec):
    """mixer.py:71-76"""
    off = 0
    for p in model.parameters():
        n = p.numel()
        p.data.copy_(torch.from_numpy(vec[off:off + n]).view_as(p).to(p.dtype))
        off += n


def consensus_sgd_steps(models, optimizers, data, labels, rowptr, cols, w, steps,
                        dtype=torch.float32):
    """``steps`` rounds of (local SGD step per agent, one Mixer round).  Returns the per-agent
    losses of every step ([steps][N]).  dtype=float64 (models, data and the mix in fp64) is the
    tests' accuracy yardstick, not a reference behaviour."""
    losses = []
    for _ in range(steps):
        ls = []
        for a, (m, opt) in enumerate(zip(models, optimizers)):
            opt.zero_grad()
            loss = torch.nn.functional.cross_entropy(m(data[a].to(dtype)), labels[a])
            loss.backward()
            opt.step()
            ls.append(float(loss.detach()))
        X = np.stack([flatten(m, dtype) for m in models])
        Y = mixer_ref.mix_once(X, rowptr, cols, w)
        for m, y in zip(models, Y):
            load_flat(m, y)
        losses.append(ls)
    return losses
