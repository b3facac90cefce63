"""Generates tests/golden/mlp_grad_small.npz: per-agent ANNModel gradients from CPU autograd,
the fixture ``__graft_entry__.smoke()`` checks one ``dl_mlp_grad`` launch against.

Three agents of ``ANNModel(52, 40, 7)`` (the reference's networks/ann_model.py:4-45 layer stack,
restated in distributed_learning_amd/networks/ann_model.py), a batch of 64 rows each,
``torch.nn.CrossEntropyLoss`` (mean over the batch) as in the c3 workload.  The parameters are
stored as the flattened fp32 rows the engine keeps (registration order, mixer.py:68-69); the
reference gradients are computed by torch autograd in fp64 on exactly those fp32 values, so the
fixture holds the exact gradient the fp32 kernel approximates.

    python tests/golden/make_mlp_grad_fixture.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    sys.path.insert(0, ROOT)
    from distributed_learning_amd.networks import ANNModel
    n, b, din, dh, dout = 3, 64, 52, 40, 7
    torch.manual_seed(0)
    models = [ANNModel(din, dh, dout) for _ in range(n)]
    X = torch.stack([torch.cat([p.data.reshape(-1) for p in m.parameters()]) for m in models])
    gen = torch.Generator().manual_seed(1)
    data = torch.randn(n, b, din, generator=gen)
    labels = torch.randint(0, dout, (n, b), generator=gen, dtype=torch.int32)
    G, loss = [], []
    for a, m in enumerate(models):
        m = m.double()
        m.zero_grad()
        l = torch.nn.functional.cross_entropy(m(data[a].double()), labels[a].long())
        l.backward()
        G.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]))
        loss.append(l.detach())
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "mlp_grad_small.npz"),
                        X=X.numpy(), data=data.numpy(), labels=labels.numpy(),
                        G=torch.stack(G).numpy(), loss=torch.stack(loss).numpy(),
                        dims=np.array([din, dh, dout]))


if __name__ == "__main__":
    main()
