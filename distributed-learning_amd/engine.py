"""Device-resident gossip engine: the agent matrix X[N, P] lives in HBM and every round is one
call into libdlamd (``dl_mix_round``): fused local step + sparse mix + disagreement.

This replaces, per round, the reference's Python loop of ``Mixer._mix_params_once``
(utils/consensus_simple/mixer.py:43-49) and ``_get_deviation_dict`` (:57-66), which allocate a
fresh fp32 array per agent and term.  Flattening models to X happens once per ``mix()`` call
(mixer.py:26), not per round.
"""
import ctypes
import os

import numpy as np
import torch

from . import _lib
from .graph import Csr


class DeviceCsr:
    """A Csr uploaded to the device (int32 indices, fp32 weights)."""

    def __init__(self, csr: Csr, device):
        if csr.n_src > 65535 * 4 or csr.nnz >= 2 ** 31:
            raise ValueError("graph too large for the int32 CSR ABI")
        self.csr = csr
        self.device = torch.device(device)
        self.rowptr = torch.as_tensor(csr.rowptr.astype(np.int32), device=self.device)
        self.col = torch.as_tensor(csr.col.astype(np.int32), device=self.device)
        self.w = torch.as_tensor(csr.w.astype(np.float32), device=self.device)
        self.n_rows = csr.n_rows
        self.n_src = csr.n_src
        self.n_local = csr.n_local      # local source rows (n_rows unless a partition row set)
        self.nnz = csr.nnz
        self.uniform_row_nnz = csr.uniform_row_nnz
        self.doubly_stochastic = int(csr.doubly_stochastic)
        self.shared_row_weights = int(csr.shared_row_weights)
        self.min_row_nnz = csr.min_row_nnz
        self.hub_rows = 0       # dl_mix_args.n_hub_rows (plan path 5 hint; GossipEngine sets it)

    def c_struct(self):
        return _lib.DlCsr(_lib.ptr(self.rowptr), _lib.ptr(self.col), _lib.ptr(self.w),
                          self.n_rows, self.nnz, self.uniform_row_nnz, self.doubly_stochastic,
                          self.shared_row_weights, self.min_row_nnz)


def _ld(t):
    if t.dim() != 2 or t.stride(1) != 1:
        raise ValueError("expected a 2-D row-major tensor with unit column stride")
    return t.stride(0)


def _check(t, name, rows, cols, device):
    if t.dtype != torch.float32:
        raise ValueError(f"{name} must be float32 (got {t.dtype})")
    if t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")
    if t.shape[0] != rows or t.shape[1] != cols:
        raise ValueError(f"{name} has shape {tuple(t.shape)}, expected ({rows}, {cols})")


def plan_shape(W: DeviceCsr, n_params, deviation=True, tile_cols=0):
    """dl_mix_plan_csr: the kernel configuration for this graph's sizes and flags (no tensors
    needed).  tile_cols: 0 row-major, > 0 column-tiled of that width, -1 choose the tiled width."""
    lib = _lib.load()
    plan = _lib.DlMixPlan()
    w = _lib.DlCsr(None, None, None, W.n_rows, W.nnz, W.uniform_row_nnz, W.doubly_stochastic,
                   W.shared_row_weights, W.min_row_nnz)   # sizes and flags only
    _lib.check(lib.dl_mix_plan_csr(ctypes.byref(w), W.n_src - W.n_rows, int(n_params),
                                   int(bool(deviation)), int(tile_cols), ctypes.byref(plan)),
               "dl_mix_plan_csr")
    return {f: getattr(plan, f) for f, _ in plan._fields_}


def tiled_shape(n_rows, n_params, tile_cols):
    return ((n_params + tile_cols - 1) // tile_cols, n_rows, tile_cols)


def to_tiled(X, tile_cols, out=None):
    """Row-major [n, P] -> column-tiled [ceil(P/T), n, T] (zero-padded last tile)."""
    lib = _lib.load()
    n, P = X.shape
    out = torch.empty(tiled_shape(n, P, tile_cols), dtype=torch.float32,
                      device=X.device) if out is None else out
    _lib.check(lib.dl_to_tiled(_lib.ptr(X), _ld(X), n, P, tile_cols, _lib.ptr(out),
                               _lib.stream_handle(X.device)), "dl_to_tiled")
    return out


def from_tiled(Xt, n_params, out=None):
    """Column-tiled [tiles, n, T] -> row-major [n, P]."""
    lib = _lib.load()
    _, n, T = Xt.shape
    out = torch.empty(n, n_params, dtype=torch.float32, device=Xt.device) if out is None else out
    _lib.check(lib.dl_from_tiled(_lib.ptr(Xt), n, n_params, T, _lib.ptr(out), _ld(out),
                                 _lib.stream_handle(Xt.device)), "dl_from_tiled")
    return out


def _check_tiled(t, name, shape, device):
    if t.dtype != torch.float32 or t.device != device or tuple(t.shape) != tuple(shape) or \
            not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous float32 tensor of shape {tuple(shape)} "
                         f"on {device} (got {tuple(t.shape)}, {t.dtype}, {t.device})")


def _tiled_ld(t, name, rows, n_params, tile_cols, device):
    """Block rows (dl_mix_args ld* in the column-tiled layout) of a [tiles, rows, T] operand: a
    contiguous tiled matrix, or a view of whole rows / whole tiles of a wider one (a partition
    row set X[:, a:b], a column chunk X[t0:t1]); its tile stride is ld*T floats."""
    tiles = (n_params + tile_cols - 1) // tile_cols
    if t.dtype != torch.float32 or t.device != device or t.dim() != 3 or \
            tuple(t.shape) != (tiles, rows, tile_cols) or t.stride(2) != 1 or \
            t.stride(1) != tile_cols or (tiles > 1 and t.stride(0) % tile_cols) or \
            (tiles > 1 and t.stride(0) < rows * tile_cols):
        raise ValueError(f"{name} must be a float32 [tiles={tiles}, rows={rows}, T={tile_cols}] "
                         f"column-tiled tensor (or a row / tile view of one) on {device} "
                         f"(got {tuple(t.shape)}, strides {t.stride()}, {t.dtype}, {t.device})")
    return t.stride(0) // tile_cols if tiles > 1 else rows


def mix_args_tiled(W: DeviceCsr, n_params, tile_cols, X, Y, G=None, lr=0.0, dev_sq=None,
                   dev_max=None, mean=None, halo=None, halo_blocks=None):
    """dl_mix_args for column-tiled operands (3-D [tiles, rows, T] tensors or row / tile views of
    them).  X (and G) hold the W.n_local local source rows, Y the W.n_rows output rows; halo rows
    (W.n_src > W.n_local) come from ``halo``, a contiguous buffer of per-peer tiled blocks of
    ``halo_blocks`` rows each (dlamd.h n_halo_blocks; None = one block)."""
    dev = W.device
    ldx = _tiled_ld(X, "X", W.n_local, n_params, tile_cols, dev)
    ldy = _tiled_ld(Y, "Y", W.n_rows, n_params, tile_cols, dev)
    ldg = _tiled_ld(G, "G", W.n_local, n_params, tile_cols, dev) if G is not None else 0
    n_halo = W.n_src - W.n_local
    blocks = None
    if n_halo > 0:
        tiles = (n_params + tile_cols - 1) // tile_cols
        if halo is None:
            raise ValueError(f"graph has {n_halo} halo rows but no halo buffer was given")
        if halo.dtype != torch.float32 or halo.device != dev or not halo.is_contiguous() or \
                halo.numel() < tiles * n_halo * tile_cols:
            raise ValueError(f"halo must be a contiguous float32 buffer of >= {tiles} x {n_halo} "
                             f"x {tile_cols} floats on {dev}")
        hb = [int(b) for b in halo_blocks] if halo_blocks is not None else []
        if hb and sum(hb) != n_halo:
            raise ValueError(f"halo_blocks {hb} do not sum to the {n_halo} halo rows")
        blocks = (ctypes.c_int32 * max(len(hb), 1))(*hb) if hb else None
    args = _lib.DlMixArgs(
        _lib.ptr(X), ldx, _lib.ptr(Y), ldy, int(n_params), W.c_struct(), _lib.ptr(G), ldg,
        float(lr), _lib.ptr(halo) if n_halo > 0 else None, 0, n_halo, _lib.ptr(dev_sq),
        _lib.ptr(dev_max), _lib.ptr(mean), int(tile_cols), None, None,
        W.n_local if W.n_local != W.n_rows else 0, len(blocks) if blocks is not None else 0,
        ctypes.cast(blocks, ctypes.c_void_p) if blocks is not None else None)
    args._keep = blocks   # the host block table must outlive the call
    args.n_hub_rows = int(getattr(W, "hub_rows", 0))
    return args


def mix_args(W: DeviceCsr, X, Y, G=None, lr=0.0, halo=None, dev_sq=None, dev_max=None,
             mean=None):
    """Build the dl_mix_args struct for X -> Y (shapes checked here, the rest in the ABI).
    X (and G) hold the W.n_local local source rows, Y the W.n_rows output rows."""
    n, P = W.n_rows, X.shape[1]
    _check(X, "X", W.n_local, P, W.device)
    _check(Y, "Y", n, P, W.device)
    if G is not None:
        _check(G, "G", W.n_local, P, W.device)
    n_halo = W.n_src - W.n_local
    if n_halo > 0:
        if halo is None:
            raise ValueError(f"graph has {n_halo} halo rows but no halo buffer was given")
        _check(halo, "halo", n_halo, P, W.device)
    args = _lib.DlMixArgs(
        _lib.ptr(X), _ld(X), _lib.ptr(Y), _ld(Y), P, W.c_struct(),
        _lib.ptr(G), _ld(G) if G is not None else 0, float(lr),
        _lib.ptr(halo) if n_halo > 0 else None, _ld(halo) if n_halo > 0 else 0, n_halo,
        _lib.ptr(dev_sq), _lib.ptr(dev_max), _lib.ptr(mean), 0, None, None,
        W.n_local if W.n_local != n else 0)
    args.n_hub_rows = int(getattr(W, "hub_rows", 0))
    return args


class Workspace:
    """Grow-only device scratch buffer handed to the ABI calls."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.buf = None

    def get(self, nbytes):
        if self.buf is None or self.buf.numel() < nbytes:
            self.buf = torch.empty(max(int(nbytes), 256), dtype=torch.uint8, device=self.device)
        return self.buf

    def ptr_size(self, nbytes):
        b = self.get(nbytes)
        return _lib.ptr(b), b.numel()


def mix_round(W: DeviceCsr, X, Y, G=None, lr=0.0, halo=None, dev_sq=None, dev_max=None,
              mean=None, workspace: Workspace = None, tiled=None, mean_prev=None,
              colsum_out=None, halo_blocks=None):
    """One consensus round on the current stream: Y = W (X - lr G) [+ deviation of Y].
    ``tiled=(n_params, tile_cols)``: X, G, Y are in the column-tiled layout (``halo`` then a
    buffer of per-peer tiled blocks of ``halo_blocks`` rows, see ``mix_args_tiled``).
    Halo rounds (``halo`` rows): ``mean_prev`` (the global column mean of X), ``colsum_out`` and
    ``dev_sq`` together give the lagged deviation -- dev_sq = ||x_a - mean_prev||^2 of the
    INPUT rows, colsum_out = this rank's column sums of X - lr G (include/dlamd.h).  Without
    dev_sq / dev_max (column-tiled only) the round leaves its [R, n_local] partial rows in
    ``workspace`` -- then a float32 tensor slice the caller reduces (``row_sums``) -- and returns
    R, which the ABI reports from the launch itself (dl_mix_args.partial_rows_out, ABI 9).
    Otherwise returns None."""
    lib = _lib.load()
    if tiled is not None:
        P = tiled[0]
        args = mix_args_tiled(W, tiled[0], tiled[1], X, Y, G, lr, dev_sq, dev_max, mean, halo,
                              halo_blocks)
    else:
        P = X.shape[1]
        args = mix_args(W, X, Y, G, lr, halo, dev_sq, dev_max, mean)
    for name, t in (("mean_prev", mean_prev), ("colsum_out", colsum_out)):
        if t is not None:
            if t.dtype != torch.float32 or t.device != W.device or t.numel() < P or \
                    t.dim() != 1 or t.stride(0) != 1:
                raise ValueError(f"{name} must be a contiguous float32 [n_params] device tensor")
            setattr(args, name, _lib.ptr(t))
    n_parts = None
    if mean_prev is not None and dev_sq is None:
        # the partial-rows mode: only into a caller-placed slice the caller reduces itself (with
        # the internal workspace the partials would be dropped and the round have no deviation)
        if not isinstance(workspace, torch.Tensor):
            raise ValueError("a lagged halo round without dev_sq leaves its deviation partial "
                             "rows in the workspace: pass dev_sq, or a tensor workspace to "
                             "reduce with row_sums")
        n_parts = ctypes.c_int32(-1)
        args.partial_rows_out = ctypes.pointer(n_parts)
    if isinstance(workspace, torch.Tensor):   # a caller-placed slice (partial rows it reduces)
        if workspace.device != W.device or not workspace.is_contiguous():
            raise ValueError("a tensor workspace must be a contiguous tensor on W's device")
        wp, wn = _lib.ptr(workspace), workspace.numel() * workspace.element_size()
    else:
        workspace = workspace or Workspace(W.device)
        wp, wn = workspace.ptr_size(lib.dl_mix_workspace_bytes(max(W.n_rows, W.n_local),
                                                               W.n_src - W.n_local, P))
    _lib.check(lib.dl_mix_round(ctypes.byref(args), wp, wn, _lib.stream_handle(W.device)),
               "dl_mix_round")
    return None if n_parts is None else int(n_parts.value)


def mix_rounds(W: DeviceCsr, X, Y, rounds, G=None, lr=0.0, dev_sq=None, dev_max=None, mean=None,
               workspace: Workspace = None, tiled=None):
    """``rounds`` mixing rounds in one HBM pass: Y = W^rounds (X - lr G) (dl_mix_rounds; the local
    step once, before the first round).  Returns False, launching nothing, when the multi-round
    kernel does not fit this graph/layout (the caller then loops ``mix_round``)."""
    lib = _lib.load()
    if tiled is not None:
        P = tiled[0]
        args = mix_args_tiled(W, tiled[0], tiled[1], X, Y, G, lr, dev_sq, dev_max, mean)
    else:
        P = X.shape[1]
        args = mix_args(W, X, Y, G, lr, None, dev_sq, dev_max, mean)
    workspace = workspace or Workspace(W.device)
    wp, wn = workspace.ptr_size(lib.dl_mix_workspace_bytes(W.n_rows, 0, P))
    rc = lib.dl_mix_rounds(ctypes.byref(args), int(rounds), wp, wn, _lib.stream_handle(W.device))
    if rc == _lib.DL_ERR_UNSUPPORTED:
        return False
    _lib.check(rc, "dl_mix_rounds")
    return True


def trace_max_rounds(W: DeviceCsr, X, Y, tiled=None):
    """dl_mix_trace_plan: the most rounds one traced pass can run, or 0 when the traced kernel
    does not fit this graph/layout (then the caller loops ``mix_round``)."""
    lib = _lib.load()
    args = (mix_args_tiled(W, tiled[0], tiled[1], X, Y) if tiled is not None
            else mix_args(W, X, Y))
    k = ctypes.c_int32(0)
    rc = lib.dl_mix_trace_plan(ctypes.byref(args), ctypes.byref(k))
    if rc == _lib.DL_ERR_UNSUPPORTED:
        return 0
    _lib.check(rc, "dl_mix_trace_plan")
    return int(k.value)


def mix_rounds_trace(W: DeviceCsr, X, Y, rounds, trace, workspace: Workspace = None,
                     tiled=None):
    """dl_mix_rounds_trace: Y = W^rounds X in one HBM pass and trace[r] = the max deviation
    after round r + 1 (device float32[rounds]).  X is left unmodified."""
    lib = _lib.load()
    args = (mix_args_tiled(W, tiled[0], tiled[1], X, Y) if tiled is not None
            else mix_args(W, X, Y))
    if trace.dtype != torch.float32 or trace.device != W.device or trace.numel() < rounds:
        raise ValueError("trace must be a float32 device tensor of at least `rounds` entries")
    workspace = workspace or Workspace(W.device)
    wp, wn = workspace.ptr_size(lib.dl_mix_trace_workspace_bytes(W.n_rows, int(rounds)))
    _lib.check(lib.dl_mix_rounds_trace(ctypes.byref(args), int(rounds), _lib.ptr(trace), wp, wn,
                                       _lib.stream_handle(W.device)), "dl_mix_rounds_trace")


def rounds_plan(W: DeviceCsr, X, Y, deviation=False, tiled=None):
    """dl_mix_rounds_plan: the multi-round configuration, or None when it does not fit."""
    lib = _lib.load()
    dummy = torch.empty(1, dtype=torch.float32, device=W.device) if deviation else None
    if tiled is not None:
        args = mix_args_tiled(W, tiled[0], tiled[1], X, Y, None, 0.0, dummy, dummy, None)
    else:
        args = mix_args(W, X, Y, None, 0.0, None, dummy, dummy, None)
    plan = _lib.DlMixPlan()
    rc = lib.dl_mix_rounds_plan(ctypes.byref(args), ctypes.byref(plan))
    if rc == _lib.DL_ERR_UNSUPPORTED:
        return None
    _lib.check(rc, "dl_mix_rounds_plan")
    return {f: getattr(plan, f) for f, _ in plan._fields_}


def rounds_plan_shape(W: DeviceCsr, n_params, deviation=False, tile_cols=0):
    """dl_mix_rounds_plan_shape: the multi-round configuration for row-major (tile_cols 0) or
    column-tiled operands of these sizes, or None when the multi-round kernel does not fit."""
    lib = _lib.load()
    plan = _lib.DlMixPlan()
    rc = lib.dl_mix_rounds_plan_shape(W.n_rows, int(n_params), W.nnz, W.uniform_row_nnz,
                                      W.shared_row_weights, W.doubly_stochastic,
                                      int(bool(deviation)), int(tile_cols), ctypes.byref(plan))
    if rc == _lib.DL_ERR_UNSUPPORTED:
        return None
    _lib.check(rc, "dl_mix_rounds_plan_shape")
    return {f: getattr(plan, f) for f, _ in plan._fields_}


def until_fits(W: DeviceCsr, n_params):
    """True when dl_mix_until holds these agents' whole vectors in one workgroup's LDS."""
    return W.n_src == W.n_rows and bool(_lib.load().dl_mix_until_fits(W.n_rows, int(n_params),
                                                                       W.nnz))


def mix_until(W: DeviceCsr, X, Y, times, eps=None, max_rounds=4096, status=None,
              dev_trace=None):
    """``Mixer.mix``'s loop (mixer.py:18-41) in one launch on the current stream: rounds until
    ``(eps is None or max deviation < float32(eps)) and done >= times`` or ``max_rounds``.
    Y may be X.  ``status`` (device int32[2]) receives (rounds done, 1 if the stop rule held);
    ``dev_trace`` (device float32[max_rounds + 1], eps only) every evaluated max deviation.
    Does not synchronise."""
    P = X.shape[1]
    _check(X, "X", W.n_rows, P, W.device)
    _check(Y, "Y", W.n_rows, P, W.device)
    if W.n_src != W.n_rows:
        raise ValueError("mix_until needs a square W (no halo rows)")
    if status is None or status.dtype != torch.int32 or status.numel() < 2:
        raise ValueError("status must be a device int32 tensor of >= 2 elements")
    if dev_trace is not None and (dev_trace.dtype != torch.float32 or
                                  dev_trace.numel() < max_rounds + 1):
        raise ValueError("dev_trace must be float32 with >= max_rounds + 1 elements")
    args = _lib.DlMixUntilArgs(
        _lib.ptr(X), _ld(X), _lib.ptr(Y), _ld(Y), P, W.c_struct(), int(times),
        0 if eps is None else 1, float(np.float32(eps)) if eps is not None else 0.0,
        int(max_rounds), _lib.ptr(status), _lib.ptr(dev_trace) if eps is not None else None)
    _lib.check(_lib.load().dl_mix_until(ctypes.byref(args), _lib.stream_handle(W.device)),
               "dl_mix_until")


def mix_plan(W: DeviceCsr, X, Y, G=None, deviation=False):
    lib = _lib.load()
    dummy = torch.empty(1, dtype=torch.float32, device=W.device) if deviation else None
    args = mix_args(W, X, Y, G, 0.0, None, dummy, dummy, None)
    plan = _lib.DlMixPlan()
    _lib.check(lib.dl_mix_plan_query(ctypes.byref(args), ctypes.byref(plan)), "dl_mix_plan_query")
    return {f: getattr(plan, f) for f, _ in plan._fields_}


def deviation(X, dev_sq=None, dev_max=None, mean_in=None, mean_out=None,
              workspace: Workspace = None):
    """dev_sq[a] = ||x_a - mean||^2 and dev_max = max_a ||x_a - mean|| (mixer.py:51-66)."""
    lib = _lib.load()
    n, P = X.shape
    dev = X.device
    if dev_sq is None:
        dev_sq = torch.empty(n, dtype=torch.float32, device=dev)
    if dev_max is None:
        dev_max = torch.empty(1, dtype=torch.float32, device=dev)
    workspace = workspace or Workspace(dev)
    wp, wn = workspace.ptr_size(lib.dl_deviation_workspace_bytes(n, P))
    _lib.check(lib.dl_deviation(_lib.ptr(X), _ld(X), n, P, _lib.ptr(mean_in), _lib.ptr(dev_sq),
                                _lib.ptr(dev_max), _lib.ptr(mean_out), wp, wn,
                                _lib.stream_handle(dev)), "dl_deviation")
    return dev_sq, dev_max


def deviation_tiled(Xt, n_params, dev_sq=None, dev_max=None, mean_out=None,
                    workspace: Workspace = None):
    lib = _lib.load()
    _, n, T = Xt.shape
    dev = Xt.device
    if dev_sq is None:
        dev_sq = torch.empty(n, dtype=torch.float32, device=dev)
    if dev_max is None:
        dev_max = torch.empty(1, dtype=torch.float32, device=dev)
    workspace = workspace or Workspace(dev)
    wp, wn = workspace.ptr_size(lib.dl_deviation_workspace_bytes(n, n_params))
    _lib.check(lib.dl_deviation_tiled(_lib.ptr(Xt), n, int(n_params), T, _lib.ptr(dev_sq),
                                      _lib.ptr(dev_max), _lib.ptr(mean_out), wp, wn,
                                      _lib.stream_handle(dev)), "dl_deviation_tiled")
    return dev_sq, dev_max


def row_sums(parts, sums=None, max_sqrt=None, max_zeroed=False):
    """dl_row_sums: sums[a] = sum_b parts[b][a] (fixed order), max_sqrt[0] = max sqrt(sums) --
    a chunked round's per-agent deviation and its max in one launch (max_zeroed: max_sqrt
    already holds 0, as a partial-rows dl_mix_round given it as dev_max leaves it)."""
    lib = _lib.load()
    if parts.dim() != 2 or not parts.is_contiguous() or parts.dtype != torch.float32:
        raise ValueError("parts must be a contiguous float32 [n_parts, n_rows] tensor")
    nb, n = parts.shape
    _lib.check(lib.dl_row_sums(_lib.ptr(parts), nb, n, _lib.ptr(sums), _lib.ptr(max_sqrt),
                               int(bool(max_zeroed)), _lib.stream_handle(parts.device)),
               "dl_row_sums")
    return sums, max_sqrt


def column_sum(X, out=None):
    lib = _lib.load()
    n, P = X.shape
    out = torch.empty(P, dtype=torch.float32, device=X.device) if out is None else out
    _lib.check(lib.dl_column_sum(_lib.ptr(X), _ld(X), n, P, _lib.ptr(out),
                                 _lib.stream_handle(X.device)), "dl_column_sum")
    return out


def max_column_std(X):
    lib = _lib.load()
    n, P = X.shape
    out = torch.empty(1, dtype=torch.float32, device=X.device)
    _lib.check(lib.dl_max_column_std(_lib.ptr(X), _ld(X), n, P, _lib.ptr(out),
                                     _lib.stream_handle(X.device)), "dl_max_column_std")
    return out


def step_rows(X, rows, out, G=None, lr=0.0):
    """out[i] = X[rows[i]] - lr * G[rows[i]] (halo send buffers)."""
    lib = _lib.load()
    n_sel = rows.numel()
    P = X.shape[1]
    _lib.check(lib.dl_step_rows(_lib.ptr(X), _ld(X), _lib.ptr(G), _ld(G) if G is not None else 0,
                                float(lr), _lib.ptr(rows), n_sel, P, _lib.ptr(out), _ld(out),
                                _lib.stream_handle(X.device)), "dl_step_rows")
    return out


def step_rows_tiled_peers(X, rows, row0, outs, G=None, lr=0.0):
    """dl_step_rows_tiled_peers: every peer's halo block in one launch -- peer b's rows are
    rows[row0[b]:row0[b+1]] (one int32 device tensor, peers concatenated), its block
    outs[b] = [tiles, n_b, T] (contiguous)."""
    lib = _lib.load()
    tiles, _, T = X.shape
    if rows.dtype != torch.int32 or rows.device != X.device:
        raise ValueError("rows must be a device int32 tensor (every entry < X.shape[1]: checked "
                         "once by the caller, a bad row faults the GPU)")
    n = len(outs)
    if len(row0) != n + 1 or row0[0] != 0 or row0[-1] != rows.numel():
        raise ValueError("row0 must be [0, ..., rows.numel()] with one entry per peer + 1")
    xl = _tiled_ld(X, "X", X.shape[1], tiles * T, T, X.device)
    gl = _tiled_ld(G, "G", G.shape[1], tiles * T, T, X.device) if G is not None else 0
    if G is not None and G.shape[1] < X.shape[1]:   # the kernel reads G at X's row ids
        raise ValueError("G has fewer rows than X")
    for b, o in enumerate(outs):
        _check_tiled(o, f"outs[{b}]", (tiles, row0[b + 1] - row0[b], T), X.device)
    r0 = (ctypes.c_int32 * (n + 1))(*row0)
    op = (ctypes.c_void_p * n)(*[o.data_ptr() for o in outs])
    _lib.check(lib.dl_step_rows_tiled_peers(_lib.ptr(X), xl, _lib.ptr(G), gl, float(lr),
                                            _lib.ptr(rows), n, r0, op, tiles * T, T,
                                            _lib.stream_handle(X.device)),
               "dl_step_rows_tiled_peers")
    return outs


def step_rows_tiled(X, rows, out, G=None, lr=0.0):
    """Column-tiled dl_step_rows_tiled: out[t, i] = X[t, rows[i]] - lr * G[t, rows[i]] for every
    tile t -- one peer's halo block [tiles, n_sel, T] (X, G: [tiles, rows, T] or tile views)."""
    lib = _lib.load()
    tiles, _, T = X.shape
    n_sel = rows.numel()
    if rows.dtype != torch.int32 or rows.device != X.device:
        raise ValueError("rows must be a device int32 tensor (every entry < X.shape[1]: checked "
                         "once by the caller, a bad row faults the GPU)")
    xl = _tiled_ld(X, "X", X.shape[1], tiles * T, T, X.device)
    gl = _tiled_ld(G, "G", G.shape[1], tiles * T, T, X.device) if G is not None else 0
    if G is not None and G.shape[1] < X.shape[1]:
        raise ValueError("G has fewer rows than X")
    _check_tiled(out, "out", (tiles, n_sel, T), X.device)
    _lib.check(lib.dl_step_rows_tiled(_lib.ptr(X), xl, _lib.ptr(G), gl, float(lr),
                                      _lib.ptr(rows), n_sel, tiles * T, T, _lib.ptr(out),
                                      _lib.stream_handle(X.device)), "dl_step_rows_tiled")
    return out


def perron_round(Y, rowptr, col, eps, conv_eps, weight=None, mean_weight=1.0, max_iter=1 << 30,
                 workspace: Workspace = None, conv_eps_rows=None):
    """In-place asyncio-style consensus round on Y (fp32 or fp64).  Returns the iteration count."""
    lib = _lib.load()
    if Y.dtype not in (torch.float32, torch.float64):
        raise ValueError("perron_round supports float32 and float64")
    dtype = 1 if Y.dtype == torch.float64 else 0
    n, P = Y.shape
    iters = torch.zeros(1, dtype=torch.int32, device=Y.device)
    workspace = workspace or Workspace(Y.device)
    wp, wn = workspace.ptr_size(lib.dl_perron_workspace_bytes(dtype, n, P))
    args = _lib.DlPerronArgs(dtype, _lib.ptr(Y), _ld(Y), n, P, _lib.ptr(rowptr), _lib.ptr(col),
                             _lib.ptr(weight), float(mean_weight), float(eps), float(conv_eps),
                             int(min(max_iter, 2 ** 31 - 1)), _lib.ptr(iters),
                             _lib.ptr(conv_eps_rows))
    _lib.check(lib.dl_perron_round(ctypes.byref(args), wp, wn, _lib.stream_handle(Y.device)),
               "dl_perron_round")
    return int(iters.item())


class PerronRounds:
    """Repeated ``dl_perron_round`` calls on HOST values of one shape -- the asyncio facade's
    synchronous schedule, where every round starts from the agents' numpy values and returns
    numpy values (consensus_asyncio.py:209-312).  Pinned host staging, the device buffers, the
    argument struct and the workspace are made once; a round is then one H2D copy of the values
    and weights, one launch, one D2H copy of the result and the iteration count, and ONE stream
    synchronisation (``perron_round`` allocates and syncs per call: 2.2 ms per Titanic step
    through the facade)."""

    def __init__(self, rowptr, col, n, P, dtype, device):
        lib = _lib.load()
        self.lib, self.n, self.P = lib, int(n), int(P)
        self.device = torch.device(device)
        tdt = torch.float64 if dtype == torch.float64 else torch.float32
        self.dtype = tdt
        pin = dict(pin_memory=True)
        self.h_y = torch.empty((n, P), dtype=tdt, **pin)
        self.h_w = torch.empty(n, dtype=torch.float64, **pin)
        self.h_out = torch.empty((n, P), dtype=tdt, **pin)
        self.h_it = torch.empty(1, dtype=torch.int32, **pin)
        self.y = torch.empty((n, P), dtype=tdt, device=self.device)
        self.w = torch.empty(n, dtype=torch.float64, device=self.device)
        self.it = torch.zeros(1, dtype=torch.int32, device=self.device)
        # per-agent convergence eps (agents built with different convergence_eps): pinned
        # staging + device buffer made once, copied only when the values change
        self.h_conv = torch.empty(n, dtype=torch.float64, **pin)
        self.h_conv_np = self.h_conv.numpy()
        self.conv_rows = torch.empty(n, dtype=torch.float64, device=self.device)
        self._conv_key = None
        self.rowptr, self.col = rowptr, col
        self.ws = Workspace(self.device)
        wp, wn = self.ws.ptr_size(lib.dl_perron_workspace_bytes(1 if tdt == torch.float64 else 0,
                                                                 n, P))
        self.wp, self.wn = wp, wn
        self.args = _lib.DlPerronArgs(1 if tdt == torch.float64 else 0, _lib.ptr(self.y), P, n,
                                      P, _lib.ptr(rowptr), _lib.ptr(col), _lib.ptr(self.w), 1.0,
                                      0.0, 0.0, 1, _lib.ptr(self.it), None)
        self.h_y_np, self.h_w_np = self.h_y.numpy(), self.h_w.numpy()
        self.h_out_np, self.h_it_np = self.h_out.numpy(), self.h_it.numpy()

    def run(self, values, weights, mean_weight, eps, conv_eps, max_iter, conv_eps_rows=None):
        """values: n arrays of P elements (any shape), weights: n floats.  Returns (result
        [n, P] numpy copy, iterations)."""
        np.stack([np.asarray(v, dtype=self.h_y_np.dtype).reshape(-1) for v in values],
                 out=self.h_y_np)
        self.h_w_np[:] = weights
        with torch.cuda.device(self.device):
            self.y.copy_(self.h_y, non_blocking=True)
            self.w.copy_(self.h_w, non_blocking=True)
            a = self.args
            a.mean_weight, a.eps, a.conv_eps = float(mean_weight), float(eps), float(conv_eps)
            a.max_iter = int(min(max_iter, 2 ** 31 - 1))
            if conv_eps_rows is None:
                a.conv_eps_rows = None
            else:
                key = tuple(float(e) for e in conv_eps_rows)
                if len(key) != self.n:
                    raise ValueError(f"conv_eps_rows needs {self.n} entries (got {len(key)})")
                if key != self._conv_key:
                    self.h_conv_np[:] = key
                    self.conv_rows.copy_(self.h_conv, non_blocking=True)
                    self._conv_key = key
                a.conv_eps_rows = _lib.ptr(self.conv_rows)
            _lib.check(self.lib.dl_perron_round(ctypes.byref(a), self.wp, self.wn,
                                                _lib.stream_handle(self.device)),
                       "dl_perron_round")
            self.h_out.copy_(self.y, non_blocking=True)
            self.h_it.copy_(self.it, non_blocking=True)
            torch.cuda.current_stream(self.device).synchronize()
        return self.h_out_np.copy(), int(self.h_it_np[0])


HUB_TAIL = 0   # plan path 5: rows with more tail entries than this are folded by column lanes


def hub_rows(csr, head, tail=HUB_TAIL, cap=256):
    """dl_mix_args.n_hub_rows for plan path 5: the leading rows (a descending row-length order
    puts the longest first) whose LDS tails exceed ``tail`` entries, at most ``cap`` -- 256 rows
    = every thread of the workgroup folds one column of one of them.  Measured on c4-ba
    (Barabasi-Albert m = 2, 4096 x 2^18): 440 rounds/s with 256 such rows against 387 with none
    and 380 with only the 24 rows of more than 32 tail entries (profiles/r11/session_b): the
    4-way split pays when it spreads over the whole workgroup.  DLAMD_HUB_ROWS=k overrides it
    (0 = off; measurements)."""
    env = os.environ.get("DLAMD_HUB_ROWS")
    if env is not None:
        return max(0, min(int(env), cap, csr.n_rows))
    lens = np.diff(np.asarray(csr.rowptr)) - int(head)
    k = 0
    while k < min(cap, len(lens)) and lens[k] > tail:
        k += 1
    return k


# Resident operands of the one-round kernel are streamed together, tile t of X, G and Y at the
# same moment.  When their buffers start an exact multiple of a large power of two apart (4 GiB
# allocations placed back to back), the three streams alias in HBM and the round loses up to
# 15 % (scripts/skew_probe.py, profiles/r05/skew_probe.log: 5.08-5.18 TB/s with X | G | Y packed
# at 4 GiB spacing vs 5.68-5.98 TB/s staggered).  Each large resident buffer therefore gets a
# padded allocation of its own and starts `slot` x (2 MiB + 64 KiB) into it.
STAGGER_BYTES = (2 << 20) + (64 << 10)
_STAGGER_MIN_BYTES = 64 << 20


def staggered_zeros(shape, slot, device):
    """torch.zeros(shape) fp32 on ``device``, placed at a stagger of ``slot`` (0..3) inside a
    padded allocation when it is large; DLAMD_STAGGER=0 turns the stagger off (measurements)."""
    numel = int(np.prod(shape))
    if numel * 4 < _STAGGER_MIN_BYTES or os.environ.get("DLAMD_STAGGER", "1") == "0":
        return torch.zeros(shape, dtype=torch.float32, device=device)
    step = STAGGER_BYTES // 4
    off = (int(slot) % 4) * step
    buf = torch.zeros(numel + 4 * step, dtype=torch.float32, device=device)
    return buf[off:off + numel].view(shape)


class GossipEngine:
    """N agents x P params resident in HBM, mixed by a fixed sparse W.

    ``round(G, lr)`` runs one consensus round  X <- W (X - lr G)  (ping-pong buffers, no host
    synchronisation); with ``deviation=True`` it also leaves ||x_a - mean||^2 in ``dev_sq`` and
    max_a ||x_a - mean|| in ``dev_max`` (device tensors).

    layout="tiled" (default when the graph fits the LDS tile kernel) keeps X, Y and G in the
    column-tiled layout [ceil(P/T)][N][T]: every tile the kernel stages is one contiguous HBM
    block, so the stream runs at copy speed even when T*4 bytes is a short row segment.
    Row-major data goes in and out through ``load_rows`` / ``rows`` / ``layout_like``.
    """

    def __init__(self, csr: Csr, n_params, device="cuda", X=None, layout="auto", tile_cols=None,
                 order="auto"):
        """order (optional, ``graph.lds_slot_order``): order[slot] = agent, the row order of the
        resident matrices.  ``load_rows`` / ``layout_like`` / ``rows`` take and return agent
        order; ``dev_sq`` is per slot (``agent_dev_sq()`` in agent order).  "auto": the agents
        by descending row length (``graph.row_length_order``) when the round runs the
        register-head + LDS-tail kernel (plan path 5, irregular graphs of thousands of agents),
        else agent order (None)."""
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.order = None
        if isinstance(order, str):
            if order != "auto":
                raise ValueError("order must be a permutation, None or 'auto'")
            order = None
            tc = 0 if layout == "rows" else (int(tile_cols) if tile_cols else -1)
            if plan_shape(DeviceCsr(csr, self.device), int(n_params), deviation=True,
                          tile_cols=tc)["path"] == 5:
                from .graph import row_length_order
                order = row_length_order(csr)
        if order is not None:
            from .graph import permuted
            order = np.asarray(order, np.int64)
            if sorted(order.tolist()) != list(range(csr.n_rows)):
                raise ValueError("order must be a permutation of the agents")
            csr = permuted(csr, order)
            self.order = torch.as_tensor(order, device=self.device)
        self.W = DeviceCsr(csr, self.device)
        self.n, self.P = csr.n_rows, int(n_params)
        plan = plan_shape(self.W, self.P, deviation=True,
                          tile_cols=int(tile_cols) if tile_cols else -1)
        if plan["path"] == 5:
            self.W.hub_rows = hub_rows(csr, plan["head"])
        tiled_ok = plan["path"] in (1, 4, 5) and plan["tile_cols"] >= 4 and self.W.n_src == self.n
        if layout == "auto":
            layout = "tiled" if tiled_ok else "rows"
        if layout == "tiled" and not tiled_ok:
            raise ValueError("this graph does not fit the LDS tile kernel; use layout='rows'")
        self.layout = layout
        self.T = (int(tile_cols) if tile_cols else plan["tile_cols"]) if layout == "tiled" else 0
        self.dev_sq = torch.zeros(self.n, dtype=torch.float32, device=self.device)
        self.dev_max = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.ws = Workspace(self.device)
        self._slot = 0      # stagger slot of the next resident buffer (X, Y, G, ...)
        self.X = self.layout_like(X) if X is not None else self._empty()
        self.Y = self._empty()

    def _empty(self):
        shape = (tiled_shape(self.n, self.P, self.T) if self.layout == "tiled"
                 else (self.n, self.P))
        self._slot += 1
        return staggered_zeros(shape, self._slot - 1, self.device)

    def layout_like(self, A):
        """A row-major [N, P] tensor in this engine's resident layout (G, X, ...)."""
        if A.shape != (self.n, self.P):
            raise ValueError(f"expected shape ({self.n}, {self.P}), got {tuple(A.shape)}")
        A = A.to(self.device, torch.float32)
        if self.order is not None:
            A = A.index_select(0, self.order)          # agent order -> slot order (a copy)
        # always a buffer of its own: the engine ping-pongs X/Y and must never write into the
        # caller's tensor
        out = self._empty()
        if self.layout == "tiled":
            return to_tiled(A, self.T, out=out)
        return out.copy_(A)

    def load_rows(self, X):
        self.X = self.layout_like(X)

    def rows(self):
        """The agent matrix as a row-major [N, P] tensor in agent order (a conversion in the
        tiled layout or under a slot order)."""
        R = from_tiled(self.X, self.P) if self.layout == "tiled" else self.X
        if self.order is not None:
            out = torch.empty_like(R)
            out[self.order] = R
            return out
        return R

    def agent_dev_sq(self):
        """dev_sq in agent order."""
        if self.order is None:
            return self.dev_sq
        out = torch.empty_like(self.dev_sq)
        out[self.order] = self.dev_sq
        return out

    def reserve_workspace(self, deviation=True):
        """Allocate the round's scratch now (so a hipGraph capture allocates nothing)."""
        if deviation:
            lib = _lib.load()
            self.ws.get(lib.dl_mix_workspace_bytes(self.n, self.W.n_src - self.n, self.P))

    def round(self, G=None, lr=0.0, deviation=False, mean=None, halo=None, src=None):
        """G must already be in the resident layout (``layout_like``).  src (optional, resident
        layout): mix it instead of X -- e.g. the local step X - lr G a gradient kernel already
        formed -- into the new X; X itself is then only the buffer the next round writes."""
        mix_round(self.W, self.X if src is None else src, self.Y, G=G, lr=lr, halo=halo,
                  dev_sq=self.dev_sq if deviation else None,
                  dev_max=self.dev_max if deviation else None, mean=mean, workspace=self.ws,
                  tiled=(self.P, self.T) if self.layout == "tiled" else None)
        self.X, self.Y = self.Y, self.X

    def trace_max_rounds(self):
        """Most rounds one traced pass (``rounds_traced``) can run; 0 = not supported."""
        return trace_max_rounds(self.W, self.X, self.Y,
                                tiled=(self.P, self.T) if self.layout == "tiled" else None)

    def rounds_traced(self, k, trace):
        """k rounds X <- W^k X in one HBM pass; trace[r] = max deviation after round r + 1
        (device float32[k]; what Mixer.mix(times, eps) tests after every round)."""
        mix_rounds_trace(self.W, self.X, self.Y, int(k), trace, workspace=self.ws,
                         tiled=(self.P, self.T) if self.layout == "tiled" else None)
        self.X, self.Y = self.Y, self.X

    def rounds(self, k, G=None, lr=0.0, deviation=False, mean=None):
        """k rounds  X <- W^k (X - lr G)  (the local step once, before the first round): one
        dl_mix_rounds pass when the multi-round kernel fits, else k one-round launches.  With
        ``deviation`` the final iterate's ||x_a - mean||^2 lands in ``dev_sq``."""
        k = int(k)
        if k < 1:
            return
        tiled = (self.P, self.T) if self.layout == "tiled" else None
        if mix_rounds(self.W, self.X, self.Y, k, G=G, lr=lr,
                      dev_sq=self.dev_sq if deviation else None,
                      dev_max=self.dev_max if deviation else None, mean=mean, workspace=self.ws,
                      tiled=tiled):
            self.X, self.Y = self.Y, self.X
            return
        for i in range(k):
            last = i == k - 1
            self.round(G=G if i == 0 else None, lr=lr if i == 0 else 0.0,
                       deviation=deviation and last, mean=mean if last else None)

    def deviation(self, mean_out=None):
        if self.layout == "tiled":
            return deviation_tiled(self.X, self.P, self.dev_sq, self.dev_max, mean_out, self.ws)
        return deviation(self.X, self.dev_sq, self.dev_max, mean_out=mean_out, workspace=self.ws)

    def plan(self, deviation=True):
        p = plan_shape(self.W, self.P, deviation, tile_cols=self.T)
        p["layout"] = self.layout
        return p
