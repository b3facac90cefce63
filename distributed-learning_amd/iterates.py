"""Device iterates of the asyncio consensus round (utils/consensus_asyncio.py:209-312).

In the reference every agent step produces a new numpy array ``y`` and messages carry it by
reference: a neighbour keeps mixing the array it received even after the sender has moved on
(:281, :284).  Here an iterate is an fp64 slot of one device arena per network, and a message
carries an :class:`Iterate` handle.  The slot is freed when the last handle dies (CPython
reference counting frees it exactly when the reference's array would be), so a slot referenced by
a queued message or a neighbour's half-collected value set is never overwritten.  All launches go
to one stream in order, so a slot reused after its last reader is safe without synchronisation.

Arithmetic (libdlamd ``dl_async_load`` / ``dl_async_update`` / ``dl_async_read``) reproduces
numpy's fp64 results bit for bit, including the reduction order of ``np.sum(list, axis=0)`` and
the NEP 50 dtype of the pre-scale (``include/dlamd.h``).
"""
import ctypes

import numpy as np
import torch

from . import _lib


class Iterate:
    """Handle of one agent iterate (the reference's ``y`` array)."""
    __slots__ = ("_store", "slot", "f32", "shape", "scalar")

    def __init__(self, store, slot, f32, shape, scalar):
        self._store, self.slot, self.f32, self.shape, self.scalar = store, slot, f32, shape, scalar

    def __del__(self):
        st = self._store
        if st is not None:
            st._free.append(self.slot)

    def value(self):
        return self._store.result(self)

    def __repr__(self):
        return repr(self.value())

    def __str__(self):
        return str(self.value())

    def __format__(self, spec):
        return format(self.value(), spec)


class DeviceIterates:
    """fp64 iterate arena on one device.  Not thread-safe: the asyncio protocol runs on one
    event-loop thread, as the reference's does."""

    def __init__(self, device=None, capacity=64):
        lib = _lib.load()
        if device is None:
            if not torch.cuda.is_available():
                raise RuntimeError("the HIP consensus iterates need a GPU (no CPU fallback)")
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = torch.device(device)
        self._lib = lib
        self._ld = 0
        self._arena = None
        self._cap = 0
        self._free = []
        self._flags = torch.zeros(2, dtype=torch.int32, device=self.device)
        self._parity = 0
        self._verdict = ctypes.c_int32(0)
        self._upd = _lib.DlAsyncUpdateArgs()
        self._upd.flags = _lib.ptr(self._flags)
        self._grow(capacity, 1)
        self.updates = 0

    # ------------------------------------------------------------------ arena management
    def _grow(self, cap, ld):
        ld = max(ld, self._ld)
        cap = max(cap, self._cap)
        if ld == self._ld and cap == self._cap:
            return
        with torch.cuda.device(self.device):
            arena = torch.empty((cap, ld), dtype=torch.float64, device=self.device)
            if self._arena is not None:
                arena[:self._cap, :self._ld].copy_(self._arena)
        self._free.extend(range(self._cap, cap))
        self._arena, self._cap, self._ld = arena, cap, ld

    def _slot(self):
        if not self._free:
            self._grow(2 * self._cap, self._ld)
        return self._free.pop()

    def _stream(self):
        return _lib.stream_handle(self.device)

    # ------------------------------------------------------------------ arithmetic
    def load(self, value, weight, mean_weight):
        """``y = value * weight / mean_weight`` (consensus_asyncio.py:231)."""
        arr = np.asarray(value)
        scalar = arr.ndim == 0
        # numpy's own (NEP 50) promotion of this exact expression decides the arithmetic dtype:
        # Python scalars are weak, numpy scalars and arrays strong
        probe = value if scalar else np.zeros((0,), arr.dtype)
        dt = np.asarray(probe * weight / mean_weight).dtype
        if dt not in (np.float32, np.float64):
            raise TypeError(f"run_round value of dtype {arr.dtype} (arithmetic {dt}) is not "
                            "supported; pass float32/float64 values")
        f32 = dt == np.float32
        n = self._size(arr.shape)
        if n > self._ld:
            self._grow(self._cap, n)
        slot = self._slot()
        src = np.ascontiguousarray(arr, dtype=np.float64).reshape(-1)
        a = _lib.DlAsyncLoadArgs()
        a.arena, a.ld, a.n_params, a.slot = self._arena.data_ptr(), self._ld, n, slot
        a.mode = 1 if f32 else 0
        a.src = src.ctypes.data
        a.weight = float(np.float32(weight)) if f32 else float(weight)
        a.mean_weight = float(np.float32(mean_weight)) if f32 else float(mean_weight)
        _lib.check(self._lib.dl_async_load(ctypes.byref(a), self._stream()), "dl_async_load")
        return Iterate(self, slot, f32, arr.shape, scalar)

    def update(self, y, nbrs, keep, eps, conv_eps):
        """One agent step ``y*(1 - eps*deg) + eps*np.sum(nbrs, axis=0)`` (:295) and its
        convergence verdict ``all((y' - v) <= conv_eps)`` (:297).  Synchronous: returns
        (new iterate, verdict)."""
        d = len(nbrs)
        if d > _lib.DL_ASYNC_MAX_NBRS:
            raise ValueError(f"{d} neighbours: the device step supports at most "
                             f"{_lib.DL_ASYNC_MAX_NBRS}")
        for v in nbrs:
            if v.shape != y.shape:
                raise ValueError(f"neighbour value shape {v.shape} != {y.shape}")
        out = self._slot()
        a = self._upd
        a.arena, a.ld = self._arena.data_ptr(), self._ld
        a.n_params = self._size(y.shape)
        a.self_slot, a.out_slot, a.n_nbrs = y.slot, out, d
        for j, v in enumerate(nbrs):
            a.nbr_slots[j] = v.slot
        a.sum_f32 = 1 if d and all(v.f32 for v in nbrs) else 0
        a.keep, a.eps, a.conv_eps = float(keep), float(eps), float(conv_eps)
        a.parity = self._parity
        _lib.check(self._lib.dl_async_update(ctypes.byref(a), ctypes.byref(self._verdict),
                                             self._stream()), "dl_async_update")
        # flipped only once the step ran: a call refused by the argument checks launches no
        # kernel, so the other parity's flag word was not zeroed for the next step
        self._parity ^= 1
        self.updates += 1
        return Iterate(self, out, False, y.shape, y.scalar), bool(self._verdict.value)

    def result(self, y):
        """Host copy of an iterate: ndarray of the value's shape (fp32 only for an fp32
        pre-scaled value, every step's output is fp64 as numpy's is), np.float64 for a
        Python-scalar value."""
        n = self._size(y.shape)
        buf = np.empty(n, np.float64)
        _lib.check(self._lib.dl_async_read(self._arena.data_ptr(), self._ld, y.slot, n,
                                           buf.ctypes.data, self._stream()), "dl_async_read")
        if y.scalar:
            return np.float64(buf[0])
        return buf.astype(np.float32 if y.f32 else np.float64, copy=False).reshape(y.shape)

    @staticmethod
    def _size(shape):
        n = int(np.prod(shape)) if shape else 1
        if n < 1:
            raise ValueError("run_round values must hold at least one element")
        return n
