"""Diagnose eager vs eager vs hipGraph replay differences of WRNConsensusSGD (small config)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from distributed_learning_amd.graph import best_constant_weight, uniform_weights  # noqa: E402
from distributed_learning_amd.workloads import WRNConsensusSGD  # noqa: E402


def diff(a, b):
    d = (a - b).abs()
    return f"max abs {d.max().item():.3e}  n diff {(d > 0).sum().item()}"


dev = torch.device("cuda", 0)
torch.backends.cudnn.deterministic = len(sys.argv) > 1 and sys.argv[1] == "det"
print("deterministic", torch.backends.cudnn.deterministic)
edges = [(i, (i + 1) % 4) for i in range(4)]
csr = uniform_weights(edges, best_constant_weight(edges))
kw = dict(depth=10, widen=1, lr=0.05, device=dev, seed=1)
a, b, c = (WRNConsensusSGD(csr, 4, **kw) for _ in range(3))
for w in (a, b, c):
    w.step()
torch.cuda.synchronize()
print("after step 1: a-b", diff(a.params(), b.params()), " a-c", diff(a.params(), c.params()))
print("G a-b", diff(a.G, b.G), "G a-c", diff(a.G, c.G))
c.capture()
a.step()
b.step()
c.replay(1)
torch.cuda.synchronize()
print("after step 2: a-b", diff(a.params(), b.params()), " a-c", diff(a.params(), c.params()))
print("G a-b", diff(a.G, b.G), "G a-c", diff(a.G, c.G))
print("loss a", a.loss.tolist(), "c", c.loss.tolist())
for (n, p), (_, q) in zip(a.models[0].named_parameters(), c.models[0].named_parameters()):
    d = (p.grad - q.grad).abs().max().item()
    if d > 0:
        print("  grad diff", n, f"{d:.3e}", f"|g| {p.grad.abs().max().item():.3e}")
