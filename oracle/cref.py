"""ctypes binding of oracle/mix_ref.c (TEST INFRASTRUCTURE ONLY; see oracle/__init__.py)."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "_build", "libmixref.so")
_lib = None


def build():
    import subprocess
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            build()
        L = ctypes.CDLL(_LIB)
        P = ctypes.c_void_p
        i32, i64, f32 = ctypes.c_int32, ctypes.c_int64, ctypes.c_float
        L.ref_mix_round.argtypes = [P, i64, P, i64, f32, P, i64, i32, i64, P, P, P, P, i64]
        L.ref_mix_round.restype = None
        L.ref_column_mean.argtypes = [P, i64, i32, i64, P]
        L.ref_column_mean.restype = None
        L.ref_deviation_sq.argtypes = [P, i64, i32, i64, P, P]
        L.ref_deviation_sq.restype = None
        L.ref_sgd_step.argtypes = [P, i64, P, i64, P, i64, P, i64, i32, i64, f32, f32, f32, f32,
                                   i32, i32]
        L.ref_sgd_step.restype = None
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def mix_round(X, rowptr, cols, w, G=None, lr=0.0, block=4096):
    """C restatement of Mixer._mix_params_once (+ optional fused ``x - lr*g``)."""
    X = np.ascontiguousarray(X, np.float32)
    n, p = X.shape
    out = np.empty_like(X)
    rp = np.ascontiguousarray(rowptr, np.int64)
    cl = np.ascontiguousarray(cols, np.int64)
    ww = np.ascontiguousarray(w, np.float64)
    scratch = None
    if G is not None:
        G = np.ascontiguousarray(G, np.float32)
        scratch = np.empty((n, block), np.float32)
    lib().ref_mix_round(_p(X), p, _p(G), p, float(lr), _p(out), p, n, p, _p(rp), _p(cl), _p(ww),
                        _p(scratch), block)
    return out


def column_mean(X):
    X = np.ascontiguousarray(X, np.float32)
    m = np.empty(X.shape[1], np.float32)
    lib().ref_column_mean(_p(X), X.shape[1], X.shape[0], X.shape[1], _p(m))
    return m


def deviation_sq(X, mean=None):
    X = np.ascontiguousarray(X, np.float32)
    if mean is None:
        mean = column_mean(X)
    d = np.empty(X.shape[0], np.float64)
    lib().ref_deviation_sq(_p(X), X.shape[1], X.shape[0], X.shape[1], _p(mean), _p(d))
    return d


def sgd_step(X, G, buf=None, lr=0.1, momentum=0.0, dampening=0.0, weight_decay=0.0,
             nesterov=False, first=False):
    """C restatement of torch.optim.SGD.step over agent rows.  Returns the stepped X; ``buf`` is
    updated in place (a new zero buffer when None and momentum != 0)."""
    X = np.ascontiguousarray(X, np.float32)
    G = np.ascontiguousarray(G, np.float32)
    n, p = X.shape
    if momentum != 0.0 and buf is None:
        buf = np.zeros_like(X)
    out = np.empty_like(X)
    lib().ref_sgd_step(_p(X), p, _p(G), p, _p(buf), p, _p(out), p, n, p, float(lr),
                       float(momentum), float(dampening), float(weight_decay), int(nesterov),
                       int(first))
    return out
