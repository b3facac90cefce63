"""Dump dl_mlp_grad's gradients and losses at c3's shapes (256 agents x ANNModel(784, 150, 10),
fixed seeds) to an .npz, so two builds (DLAMD_LIB) can be compared bit for bit:
    python scripts/mlp_bits.py out.npz            # one build
    python scripts/mlp_bits.py --compare a.npz b.npz
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    if sys.argv[1] == "--compare":
        a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
        for k in a.files:
            same = np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32))
            print(f"{k}: {'identical' if same else 'DIFFERENT'}"
                  + ("" if same else f" (max abs diff {np.abs(a[k] - b[k]).max():.3e})"))
            if not same:
                sys.exit(1)
        return
    import torch
    from distributed_learning_amd.networks.batched_ann import BatchedANN
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    n = 256
    bann = BatchedANN(n, 64, 784, 150, 10, device=dev)
    P = bann.P
    ld = -(-P // 64) * 64
    X = torch.zeros(n, ld, device=dev)
    X[:, :P] = 0.05 * torch.randn(n, P, device=dev, generator=g)
    data = torch.randn(n, 64, 784, device=dev, generator=g)
    labels = torch.randint(0, 10, (n, 64), device=dev, generator=g, dtype=torch.int32)
    G = torch.zeros(n, ld, device=dev)
    loss = bann.gradients(X[:, :P], data, labels, G[:, :P])
    torch.cuda.synchronize()
    np.savez(sys.argv[1], G=G[:, :P].cpu().numpy(), loss=loss.cpu().numpy())


if __name__ == "__main__":
    main()
