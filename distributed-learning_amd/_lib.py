"""ctypes binding of libdlamd.so (the C ABI declared in include/dlamd.h).

This is the only door from Python into the HIP kernels.  It fails loudly: if the shared library
is missing or was built without gfx950 code, importing a consumer raises instead of silently
running anything on the CPU.  Tensor arguments are torch CUDA(HIP) tensors; only raw device
pointers, sizes and the current HIP stream cross the boundary.
"""
import ctypes
import os

import torch  # loads torch's HIP runtime first, so libdlamd.so binds to the same one

_HERE = os.path.dirname(os.path.abspath(__file__))
# DLAMD_LIB: another build of the same ABI (A/B measurements of kernel variants on one box)
LIB_PATH = os.environ.get("DLAMD_LIB") or os.path.join(_HERE, "_lib", "libdlamd.so")

DL_OK, DL_ERR_INVALID, DL_ERR_WORKSPACE, DL_ERR_HIP, DL_ERR_UNSUPPORTED = 0, 1, 2, 3, 4

_vp = ctypes.c_void_p
_i32, _i64, _f32, _f64, _sz = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_double, \
    ctypes.c_size_t


class DlCsr(ctypes.Structure):
    _fields_ = [("row_ptr", _vp), ("col", _vp), ("w", _vp), ("n_rows", _i32), ("nnz", _i32),
                ("uniform_row_nnz", _i32), ("doubly_stochastic", _i32),
                ("shared_row_weights", _i32), ("min_row_nnz", _i32)]


class DlMixArgs(ctypes.Structure):
    _fields_ = [("x", _vp), ("ldx", _i64), ("y", _vp), ("ldy", _i64), ("n_params", _i64),
                ("W", DlCsr), ("g", _vp), ("ldg", _i64), ("lr", _f32), ("halo", _vp),
                ("ldh", _i64), ("n_halo", _i32), ("dev_sq", _vp), ("dev_max", _vp),
                ("mean", _vp), ("tile_cols", _i32), ("mean_prev", _vp), ("colsum_out", _vp),
                ("n_local_src", _i32), ("n_halo_blocks", _i32), ("halo_block_rows", _vp),
                ("n_hub_rows", _i32), ("partial_rows_out", ctypes.POINTER(_i32))]


class DlMixUntilArgs(ctypes.Structure):
    _fields_ = [("x", _vp), ("ldx", _i64), ("y", _vp), ("ldy", _i64), ("n_params", _i64),
                ("W", DlCsr), ("times", _i32), ("use_eps", _i32), ("eps", _f32),
                ("max_rounds", _i32), ("status", _vp), ("dev_trace", _vp)]


class DlConsensusGdArgs(ctypes.Structure):
    _fields_ = [("X", _vp), ("y", _vp), ("shard_ptr", _vp), ("n_agents", _i32),
                ("n_features", _i32), ("row_ptr", _vp), ("col", _vp), ("eps", _f64),
                ("conv_eps", _f64), ("mean_weight", _f64), ("tau", _f64), ("steps", _vp),
                ("iterations", _i32), ("max_iter", _i32), ("w", _vp), ("iters_out", _vp)]


class DlMixPlan(ctypes.Structure):
    _fields_ = [("path", _i32), ("tile_cols", _i32), ("grid", _i32), ("lds_bytes", _i32),
                ("n_tiles", _i32), ("regular", _i32), ("head", _i32), ("tail_fmt", _i32)]


class DlPerronArgs(ctypes.Structure):
    _fields_ = [("dtype", _i32), ("y", _vp), ("ldy", _i64), ("n_rows", _i32), ("n_params", _i64),
                ("row_ptr", _vp), ("col", _vp), ("weight", _vp), ("mean_weight", _f64),
                ("eps", _f64), ("conv_eps", _f64), ("max_iter", _i32), ("iters_out", _vp),
                ("conv_eps_rows", _vp)]


DL_ASYNC_MAX_NBRS = 64


class DlAsyncLoadArgs(ctypes.Structure):
    _fields_ = [("arena", _vp), ("ld", _i64), ("n_params", _i64), ("slot", _i32), ("mode", _i32),
                ("src", _vp), ("weight", _f64), ("mean_weight", _f64)]


class DlAsyncUpdateArgs(ctypes.Structure):
    _fields_ = [("arena", _vp), ("ld", _i64), ("n_params", _i64), ("self_slot", _i32),
                ("out_slot", _i32), ("n_nbrs", _i32), ("nbr_slots", _i32 * DL_ASYNC_MAX_NBRS),
                ("sum_f32", _i32), ("keep", _f64), ("eps", _f64), ("conv_eps", _f64),
                ("flags", _vp), ("parity", _i32)]


class DlBgemmArgs(ctypes.Structure):
    _fields_ = [("batch", _i32), ("M", _i32), ("N", _i32), ("K", _i32),
                ("A", _vp), ("lda", _i64), ("sA", _i64), ("ta", _i32),
                ("B", _vp), ("ldb", _i64), ("sB", _i64), ("tb", _i32),
                ("C", _vp), ("ldc", _i64), ("sC", _i64), ("epi", _i32),
                ("bias", _vp), ("s_bias", _i64), ("H", _vp), ("ldh", _i64), ("sH", _i64),
                ("rowsum", _vp), ("s_rowsum", _i64),
                ("labels", _vp), ("s_labels", _i64), ("loss", _vp)]


class DlSgdArgs(ctypes.Structure):
    _fields_ = [("x", _vp), ("ldx", _i64), ("g", _vp), ("ldg", _i64), ("buf", _vp), ("ldb", _i64),
                ("out", _vp), ("ldo", _i64), ("n_rows", _i32), ("n_params", _i64), ("lr", _f32),
                ("momentum", _f32), ("dampening", _f32), ("weight_decay", _f32),
                ("nesterov", _i32), ("first", _i32)]


class DlMlpArgs(ctypes.Structure):
    _fields_ = [("n_agents", _i32), ("batch", _i32), ("input_dim", _i32), ("hidden_dim", _i32),
                ("output_dim", _i32), ("X", _vp), ("ldx", _i64), ("data", _vp), ("s_data", _i64),
                ("labels", _vp), ("s_labels", _i64), ("G", _vp), ("ldg", _i64), ("loss", _vp),
                ("tile_cols", _i32), ("out_mode", _i32), ("lr", ctypes.c_float),
                ("workspace", _vp)]


EPI = {"none": 0, "bias": 1, "bias_relu": 2, "bias_tanh": 3, "bias_elu": 4, "drelu": 5,
       "dtanh": 6, "delu": 7, "bias_xent": 8}

# exported symbol -> (restype, argtypes); tests check every one is exported
SIGNATURES = {
    "dl_abi_version": (_i32, []),
    "dl_last_error": (ctypes.c_char_p, []),
    "dl_mix_workspace_bytes": (_sz, [_i32, _i32, _i64]),
    "dl_mix_plan_query": (_i32, [ctypes.POINTER(DlMixArgs), ctypes.POINTER(DlMixPlan)]),
    "dl_mix_plan_shape": (_i32, [_i32, _i32, _i64, _i32, _i32, _i32, _i32, _i32,
                                 ctypes.POINTER(DlMixPlan)]),
    "dl_mix_plan_csr": (_i32, [ctypes.POINTER(DlCsr), _i32, _i64, _i32, _i32,
                               ctypes.POINTER(DlMixPlan)]),
    "dl_mix_round": (_i32, [ctypes.POINTER(DlMixArgs), _vp, _sz, _vp]),
    "dl_mix_rounds_plan": (_i32, [ctypes.POINTER(DlMixArgs), ctypes.POINTER(DlMixPlan)]),
    "dl_mix_rounds_plan_shape": (_i32, [_i32, _i64, _i32, _i32, _i32, _i32, _i32, _i32,
                                        ctypes.POINTER(DlMixPlan)]),
    "dl_mix_rounds": (_i32, [ctypes.POINTER(DlMixArgs), _i32, _vp, _sz, _vp]),
    "dl_mix_trace_plan": (_i32, [ctypes.POINTER(DlMixArgs), ctypes.POINTER(_i32)]),
    "dl_mix_trace_workspace_bytes": (_sz, [_i32, _i32]),
    "dl_mix_rounds_trace": (_i32, [ctypes.POINTER(DlMixArgs), _i32, _vp, _vp, _sz, _vp]),
    "dl_mix_until_fits": (_i32, [_i32, _i64, _i32]),
    "dl_mix_until": (_i32, [ctypes.POINTER(DlMixUntilArgs), _vp]),
    "dl_consensus_gd": (_i32, [ctypes.POINTER(DlConsensusGdArgs), _i32, _vp]),
    "dl_deviation_workspace_bytes": (_sz, [_i32, _i64]),
    "dl_deviation": (_i32, [_vp, _i64, _i32, _i64, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "dl_deviation_tiled": (_i32, [_vp, _i32, _i64, _i32, _vp, _vp, _vp, _vp, _sz, _vp]),
    "dl_to_tiled": (_i32, [_vp, _i64, _i32, _i64, _i32, _vp, _vp]),
    "dl_from_tiled": (_i32, [_vp, _i32, _i64, _i32, _vp, _i64, _vp]),
    "dl_column_sum": (_i32, [_vp, _i64, _i32, _i64, _vp, _vp]),
    "dl_max_column_std": (_i32, [_vp, _i64, _i32, _i64, _vp, _vp]),
    "dl_row_sums": (_i32, [_vp, _i32, _i32, _vp, _vp, _i32, _vp]),
    "dl_step_rows": (_i32, [_vp, _i64, _vp, _i64, _f32, _vp, _i32, _i64, _vp, _i64, _vp]),
    "dl_step_rows_tiled": (_i32, [_vp, _i32, _vp, _i32, _f32, _vp, _i32, _i64, _i32, _vp, _vp]),
    "dl_step_rows_tiled_peers": (_i32, [_vp, _i32, _vp, _i32, _f32, _vp, _i32, _vp, _vp, _i64,
                                        _i32, _vp]),
    "dl_stream_copy": (_i32, [_vp, _vp, _i64, _i32, _vp]),
    "dl_sgd_step": (_i32, [ctypes.POINTER(DlSgdArgs), _vp]),
    "dl_mlp_workspace_bytes": (_sz, [_i32]),
    "dl_mlp_grad": (_i32, [ctypes.POINTER(DlMlpArgs), _vp]),
    "dl_bgemm": (_i32, [ctypes.POINTER(DlBgemmArgs), _vp]),
    "dl_xent_grad": (_i32, [_vp, _i64, _vp, _i64, _vp, _i64, _vp, _i32, _i32, _i32, _vp]),
    "dl_perron_workspace_bytes": (_sz, [_i32, _i32, _i64]),
    "dl_perron_round": (_i32, [ctypes.POINTER(DlPerronArgs), _vp, _sz, _vp]),
    "dl_async_load": (_i32, [ctypes.POINTER(DlAsyncLoadArgs), _vp]),
    "dl_async_update": (_i32, [ctypes.POINTER(DlAsyncUpdateArgs), ctypes.POINTER(_i32), _vp]),
    "dl_async_read": (_i32, [_vp, _i64, _i32, _i64, _vp, _vp]),
    "dl_lds_slot_order": (_i32, [_i32, _i32, _vp, _i32, _i64, ctypes.c_uint64, _vp, _vp]),
}

ABI_VERSION = 10
_lib = None


class DlError(RuntimeError):
    pass


def load():
    """Load libdlamd.so (once).  Raises ImportError when the HIP library has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build the HIP extension first "
            "(python -c 'import __graft_entry__ as g; g.build()'); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        if os.environ.get("DLAMD_LIB") and not hasattr(lib, name):
            continue   # an older build under A/B: entry points it predates stay unbound
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    v = lib.dl_abi_version()
    # (an older build under A/B, DLAMD_LIB: ABI 8 reads dl_mix_args up to n_hub_rows, ABI 9
    # dl_mlp_args up to lr, and never sees the fields added after them)
    if v != ABI_VERSION and not (os.environ.get("DLAMD_LIB") and v in (8, 9)):
        raise ImportError(f"libdlamd ABI {lib.dl_abi_version()} != expected {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc, what):
    if rc == DL_OK:
        return
    msg = load().dl_last_error().decode(errors="replace")
    if rc == DL_ERR_INVALID:
        raise ValueError(f"{what}: {msg}")
    raise DlError(f"{what} failed (status {rc}): {msg}")


def ptr(t):
    """Device pointer of a CUDA tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("libdlamd operates on device tensors; got a CPU tensor")
    return ctypes.c_void_p(t.data_ptr())


def stream_handle(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
