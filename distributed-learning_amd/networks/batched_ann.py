"""Batched per-agent ANNModel gradients on the GPU (BASELINE config c3).

The reference trains each agent's ``ANNModel`` (networks/ann_model.py:4-45) separately with torch
autograd and a cross-entropy loss; consensus then mixes the flattened parameters (mixer.py:69).
Here all agents' parameters are rows of one matrix X[N, P] (the Mixer flatten order: fc1.w,
fc1.b, fc2.w, fc2.b, fc3.w, fc3.b, fc4.w, fc4.b), and one step runs 4 forward and 7 backward
batched fp32-MFMA GEMMs over every agent at once (``dl_bgemm``), with bias/activation fused into
the forward epilogues, activation derivatives fused into the backward ones, and weight/bias
gradients written directly into each agent's row of G -- the G that the fused local step of
``dl_mix_round`` consumes.  No per-agent Python loop, no autograd graph.
"""
import ctypes
import os

import numpy as np
import torch

from .. import _lib
from .ann_model import ANNModel


def fused_supported(batch, input_dim, hidden_dim, output_dim):
    """Shapes the one-launch kernel (dl_mlp_grad, csrc/mlp_fused.hip) covers."""
    return batch == 64 and input_dim % 4 == 0 and 0 < hidden_dim <= 152 and hidden_dim % 2 == 0 and 0 < output_dim <= 16


class BatchedANN:
    """path: "fused" (dl_mlp_grad: every agent's forward + loss + backward, activations in LDS),
    "layers" (11 dl_bgemm launches) or "auto" (fused when the shapes allow it).

    split (fused path, gradient output): run dl_mlp_grad's two-launch form -- everything up to
    dZ1, then dW1 over x's column tiles on two workgroups per agent -- with a workspace
    (dl_mlp_args.workspace); the same bits as the one-launch form.  Measured slower (dW1 52.8 us
    as a launch of its own against ~42 inside the fused one, profiles/r14/README.md), so "auto"
    is off unless DLAMD_MLP_SPLIT=1 (a measurement knob)."""

    def __init__(self, n_agents, batch, input_dim=784, hidden_dim=150, output_dim=10,
                 device="cuda", path="auto", split="auto"):
        self.N, self.B = int(n_agents), int(batch)
        self.din, self.dh, self.dout = int(input_dim), int(hidden_dim), int(output_dim)
        if self.dout > 64:
            raise ValueError("the cross-entropy head supports at most 64 classes")
        self.device = torch.device(device)
        self.offsets = {}
        off = 0
        for name, shape in ANNModel.param_shapes(self.din, self.dh, self.dout):
            self.offsets[name] = off
            off += int(np.prod(shape))
        self.P = off
        f = lambda *s: torch.empty(*s, dtype=torch.float32, device=self.device)  # noqa: E731
        self.H1, self.H2, self.H3 = (f(self.N, self.B, self.dh) for _ in range(3))
        self.Z4 = f(self.N, self.B, self.dout)
        self.dZ4 = f(self.N, self.B, self.dout)
        self.dZa, self.dZb = f(self.N, self.B, self.dh), f(self.N, self.B, self.dh)
        self.loss = f(self.N)
        ok = fused_supported(self.B, self.din, self.dh, self.dout)
        if path not in ("auto", "fused", "layers"):
            raise ValueError(f"unknown path {path!r}")
        if path == "fused" and not ok:
            raise ValueError("these shapes are not covered by the fused kernel")
        self.path = "fused" if (path == "auto" and ok) else ("layers" if path == "auto" else path)
        if split == "auto":
            split = os.environ.get("DLAMD_MLP_SPLIT", "0") == "1"
        self.ws = None
        if split and self.path == "fused":
            nb = _lib.load().dl_mlp_workspace_bytes(self.N)
            self.ws = torch.empty(-(-nb // 4), dtype=torch.float32, device=self.device)

    # -------------------------------------------------------------- helpers
    def _gemm(self, M, N, K, A, lda, sA, ta, B, ldb, sB, tb, C, ldc, sC, epi="none", bias=None,
              H=None, rowsum=None, labels=None, loss=None):
        lib = _lib.load()

        def p(t, off=0):
            if t is None:
                return None
            return ctypes.c_void_p(t.data_ptr() + 4 * off)
        args = _lib.DlBgemmArgs(
            self.N, M, N, K, p(*A), lda, sA, int(ta), p(*B), ldb, sB, int(tb), p(*C), ldc, sC,
            _lib.EPI[epi], p(*bias) if bias else None, bias[0].stride(0) if bias else 0,
            p(H) if H is not None else None, self.dh if H is not None else 0,
            self.B * self.dh if H is not None else 0,
            p(*rowsum) if rowsum else None, rowsum[0].stride(0) if rowsum else 0,
            p(labels), labels.stride(0) if labels is not None else 0, p(loss))
        _lib.check(lib.dl_bgemm(ctypes.byref(args), _lib.stream_handle(self.device)), "dl_bgemm")

    def gradients(self, X, data, labels, G, lr=None):
        """G[a] = d loss_a / d params_a for every agent.  X, G: [N, P] row-major fp32 (row stride
        may exceed P), or -- fused path only -- the engine's column-tiled [tiles, N, T] tensors
        (tiles * T >= P); data: [N, B, input_dim] fp32; labels: [N, B] int32.  Returns the
        per-agent mean cross-entropy (device tensor [N]).

        lr (fused path only): G instead receives the local SGD step X - lr * grad, rounded as
        the fused round's step rounds it (dl_mlp_args.out_mode 1), so a plain round of G equals
        the fused round of X and the gradient bit for bit (row-major: G's row stride must equal
        X's)."""
        lib = _lib.load()
        step = lr is not None
        if step and self.path != "fused":
            raise ValueError("the local-step output (lr=...) needs the fused kernel")
        mode = (1, float(lr)) if step else (0, 0.0)
        ws = _lib.ptr(self.ws) if self.ws is not None else None
        N, B, din, dh, dout, P = self.N, self.B, self.din, self.dh, self.dout, self.P
        if tuple(data.shape) != (N, B, din) or not data.is_contiguous():
            raise ValueError(f"data must be contiguous [{N}, {B}, {din}] fp32")
        if tuple(labels.shape) != (N, B) or labels.dtype != torch.int32:
            raise ValueError(f"labels must be int32 [{N}, {B}]")
        if X.dim() == 3:
            if self.path != "fused":
                raise ValueError("the column-tiled layout needs the fused kernel")
            tiles, n, T = X.shape
            if n != N or tiles * T < P or tuple(G.shape) != tuple(X.shape) or \
                    not X.is_contiguous() or not G.is_contiguous() or \
                    X.dtype != torch.float32 or G.dtype != torch.float32:
                raise ValueError(f"expected contiguous fp32 [tiles, {N}, T] tensors covering {P} "
                                 "columns")
            args = _lib.DlMlpArgs(N, B, din, dh, dout, _lib.ptr(X), 0, _lib.ptr(data), B * din,
                                  _lib.ptr(labels), labels.stride(0), _lib.ptr(G), 0,
                                  _lib.ptr(self.loss), T, *mode, ws)
            _lib.check(lib.dl_mlp_grad(ctypes.byref(args), _lib.stream_handle(self.device)),
                       "dl_mlp_grad")
            return self.loss
        for t, shape in ((X, (N, P)), (G, (N, P))):
            if tuple(t.shape) != shape or t.stride(1) != 1 or t.dtype != torch.float32:
                raise ValueError(f"expected a row-major fp32 [{N}, {P}] tensor")
        aligned = all(t.data_ptr() % 16 == 0 for t in (X, G, data)) and \
            X.stride(0) % 4 == 0 and G.stride(0) % 4 == 0
        if self.path == "fused" and not aligned:
            raise ValueError("the fused kernel needs 16-byte aligned X, G, data with row strides "
                             "% 4 == 0 (pad the parameter rows)")
        if self.path == "fused":
            args = _lib.DlMlpArgs(N, B, din, dh, dout, _lib.ptr(X), X.stride(0), _lib.ptr(data),
                                  B * din, _lib.ptr(labels), labels.stride(0), _lib.ptr(G),
                                  G.stride(0), _lib.ptr(self.loss), 0, *mode, ws)
            _lib.check(lib.dl_mlp_grad(ctypes.byref(args), _lib.stream_handle(self.device)),
                       "dl_mlp_grad")
            return self.loss
        sx, sg = X.stride(0), G.stride(0)
        o = self.offsets
        hs = B * dh
        # ---- forward: H1 = relu(x W1^T + b1), H2 = tanh(.), H3 = elu(.), Z4 = H3 W4^T + b4
        self._gemm(B, dh, din, (data,), din, B * din, 0, (X, o["fc1.weight"]), din, sx, 1,
                   (self.H1,), dh, hs, "bias_relu", bias=(X, o["fc1.bias"]))
        self._gemm(B, dh, dh, (self.H1,), dh, hs, 0, (X, o["fc2.weight"]), dh, sx, 1,
                   (self.H2,), dh, hs, "bias_tanh", bias=(X, o["fc2.bias"]))
        self._gemm(B, dh, dh, (self.H2,), dh, hs, 0, (X, o["fc3.weight"]), dh, sx, 1,
                   (self.H3,), dh, hs, "bias_elu", bias=(X, o["fc3.bias"]))
        if B <= 64:   # logits + cross-entropy head in one launch (one tile per agent)
            self._gemm(B, dout, dh, (self.H3,), dh, hs, 0, (X, o["fc4.weight"]), dh, sx, 1,
                       (self.dZ4,), dout, B * dout, "bias_xent", bias=(X, o["fc4.bias"]),
                       labels=labels, loss=self.loss)
        else:
            self._gemm(B, dout, dh, (self.H3,), dh, hs, 0, (X, o["fc4.weight"]), dh, sx, 1,
                       (self.Z4,), dout, B * dout, "bias", bias=(X, o["fc4.bias"]))
            _lib.check(lib.dl_xent_grad(_lib.ptr(self.Z4), B * dout, _lib.ptr(labels), B,
                                        _lib.ptr(self.dZ4), B * dout, _lib.ptr(self.loss), N, B,
                                        dout, _lib.stream_handle(self.device)), "dl_xent_grad")
        # ---- backward (weight grads straight into G rows, bias grads as row sums of dZ^T)
        self._gemm(dout, dh, B, (self.dZ4,), dout, B * dout, 1, (self.H3,), dh, hs, 0,
                   (G, o["fc4.weight"]), dh, sg, rowsum=(G, o["fc4.bias"]))
        self._gemm(B, dh, dout, (self.dZ4,), dout, B * dout, 0, (X, o["fc4.weight"]), dh, sx, 0,
                   (self.dZa,), dh, hs, "delu", H=self.H3)                  # dZ3
        self._gemm(dh, dh, B, (self.dZa,), dh, hs, 1, (self.H2,), dh, hs, 0,
                   (G, o["fc3.weight"]), dh, sg, rowsum=(G, o["fc3.bias"]))
        self._gemm(B, dh, dh, (self.dZa,), dh, hs, 0, (X, o["fc3.weight"]), dh, sx, 0,
                   (self.dZb,), dh, hs, "dtanh", H=self.H2)                 # dZ2
        self._gemm(dh, dh, B, (self.dZb,), dh, hs, 1, (self.H1,), dh, hs, 0,
                   (G, o["fc2.weight"]), dh, sg, rowsum=(G, o["fc2.bias"]))
        self._gemm(B, dh, dh, (self.dZb,), dh, hs, 0, (X, o["fc2.weight"]), dh, sx, 0,
                   (self.dZa,), dh, hs, "drelu", H=self.H1)                 # dZ1
        self._gemm(dh, din, B, (self.dZa,), dh, hs, 1, (data,), din, B * din, 0,
                   (G, o["fc1.weight"]), din, sg, rowsum=(G, o["fc1.bias"]))
        return self.loss

    def flops_per_step(self):
        B, din, dh, dout = self.B, self.din, self.dh, self.dout
        fwd = 2 * B * (din * dh + 2 * dh * dh + dh * dout)
        bwd_w = fwd
        bwd_x = 2 * B * (dout * dh + 2 * dh * dh)
        return self.N * (fwd + bwd_w + bwd_x)
