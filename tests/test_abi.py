"""CPU checks of the C-ABI boundary: libdlamd.so loads, exports every entry point that
include/dlamd.h declares, and the ctypes struct layouts match the C compiler's."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "dlamd.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dl_[a-z_]+)\s*\(", src)))


def test_library_loads_and_exports_every_declared_symbol():
    import distributed_learning_amd  # noqa: F401
    from distributed_learning_amd import _lib
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(lib, n), f"{n} declared in dlamd.h but not exported"
        assert n in _lib.SIGNATURES, f"{n} has no ctypes signature"
    assert lib.dl_abi_version() == _lib.ABI_VERSION == 10
    assert set(_lib.SIGNATURES) == set(names)
    # (ABI 9, 10) entries are tagged in the header
    src = open(HEADER).read()
    assert "#define DLAMD_ABI_VERSION 10" in src
    for tagged in ("(ABI 9) sums[a] = sum_b parts", "(ABI 9) nullable HOST pointer",
                   "(ABI 9) A column-tiled halo round", "(ABI 10) nullable: the two-launch",
                   "size_t dl_mlp_workspace_bytes(int32_t n_agents);   /* (ABI 10) */"):
        assert tagged in src, tagged


def test_struct_layout_matches_c(tmp_path):
    from distributed_learning_amd import _lib
    prog = tmp_path / "layout.c"
    prog.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "dlamd.h"\n'
                    'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu\\n",'
                    'sizeof(dl_csr), sizeof(dl_mix_args), offsetof(dl_mix_args, W),'
                    'offsetof(dl_mix_args, lr), offsetof(dl_mix_args, partial_rows_out),'
                    'sizeof(dl_mix_plan), sizeof(dl_perron_args));'
                    'printf("%zu %zu %zu %zu %zu %zu\\n", sizeof(dl_sgd_args), offsetof(dl_sgd_args, lr),'
                    'sizeof(dl_mlp_args), offsetof(dl_mlp_args, lr),'
                    'offsetof(dl_mlp_args, workspace), sizeof(dl_bgemm_args));'
                    'return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)],
                   check=True)
    c = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True,
                                        check=True).stdout.split()]
    py = [ctypes.sizeof(_lib.DlCsr), ctypes.sizeof(_lib.DlMixArgs), _lib.DlMixArgs.W.offset,
          _lib.DlMixArgs.lr.offset, _lib.DlMixArgs.partial_rows_out.offset,
          ctypes.sizeof(_lib.DlMixPlan),
          ctypes.sizeof(_lib.DlPerronArgs), ctypes.sizeof(_lib.DlSgdArgs),
          _lib.DlSgdArgs.lr.offset, ctypes.sizeof(_lib.DlMlpArgs), _lib.DlMlpArgs.lr.offset,
          _lib.DlMlpArgs.workspace.offset, ctypes.sizeof(_lib.DlBgemmArgs)]
    assert c == py


def test_invalid_arguments_are_reported_not_crashed():
    """Validation runs before any device call, so it is testable without a GPU."""
    from distributed_learning_amd import _lib
    lib = _lib.load()
    args = _lib.DlMixArgs()  # all NULL / zero
    rc = lib.dl_mix_round(ctypes.byref(args), None, 0, None)
    assert rc == _lib.DL_ERR_INVALID
    assert b"n_rows" in lib.dl_last_error()
    with pytest.raises(ValueError):
        _lib.check(rc, "dl_mix_round")
    rc = lib.dl_deviation(None, 0, 0, 0, None, None, None, None, None, 0, None)
    assert rc == _lib.DL_ERR_INVALID
    rc = lib.dl_step_rows(None, 0, None, 0, 0.0, None, -1, 0, None, 0, None)
    assert rc == _lib.DL_ERR_INVALID


def test_shared_row_weights_flag_and_plan():
    """A uniform-weight regular graph (the c4 torus) sets shared_row_weights; the planner then
    stages one row's weights and the 4096-agent torus fits the LDS tile kernel; the flag without
    a regular graph is rejected before any device call."""
    import math
    from distributed_learning_amd import _lib, graph
    e = graph.torus_edges(64, 64)
    w = 2.0 / (2.0 - 2.0 * math.cos(2 * math.pi / 64) + 8.0)
    csr = graph.from_edge_weights(e, [w] * len(e), list(range(4096)))
    assert csr.uniform_row_nnz == 5 and csr.shared_row_weights and csr.doubly_stochastic
    bumpy = graph.Csr(csr.rowptr, csr.col, csr.w.copy())
    bumpy.w[7] = np.nextafter(np.float32(bumpy.w[7]), np.float32(1))
    assert not bumpy.shared_row_weights
    lib = _lib.load()
    plans = []
    for shared in (0, 1):
        pl = _lib.DlMixPlan()
        _lib.check(lib.dl_mix_plan_shape(4096, 0, 1 << 18, csr.nnz, 5, shared, 1, -1,
                                         ctypes.byref(pl)), "plan")
        plans.append((pl.path, pl.tile_cols, pl.lds_bytes))
    # per-entry weights: the CSR does not fit LDS beside the tile, so the regular graph keeps
    # each thread's rows' CSR in registers (path 4; the gather path when that cannot run)
    assert plans[0][0] == 4
    assert plans[1][:2] == (1, 4) and plans[1][2] <= 160 * 1024
    args = _lib.DlMixArgs()
    args.x = args.y = 16
    args.n_params = 8
    args.ldx = args.ldy = 8
    args.W = _lib.DlCsr(16, 16, 16, 4, 10, 0, 0, 1)   # shared weights on an irregular CSR
    rc = lib.dl_mix_round(ctypes.byref(args), None, 0, None)
    assert rc == _lib.DL_ERR_INVALID and b"shared_row_weights" in lib.dl_last_error()


@pytest.mark.parametrize("n,T", [(1024, 16), (512, 32), (256, 64), (2048, 8), (4096, 4),
                                 (64, 128), (7, 128)])
def test_tiled_width_choice(n, T):
    """dl_mix_plan_shape(tile_cols=-1) picks the widest tile of <= 64 KiB (profiles/HISTORY.md §5) for
    degree-4 graphs with one shared weight sequence."""
    from distributed_learning_amd import _lib
    lib = _lib.load()
    pl = _lib.DlMixPlan()
    nnz = 5 * n
    _lib.check(lib.dl_mix_plan_shape(n, 0, 1 << 20, nnz, 5, 1, 1, -1, ctypes.byref(pl)), "plan")
    assert pl.path == 1 and pl.tile_cols == T
    assert pl.tile_cols * n * 4 <= 65536 or pl.tile_cols == 4
    # at C = 4 one resident workgroup per CU, else two when LDS allows; the persistent grid is
    # oversubscribed 2x by default (DLAMD_GRID_MULT)
    if T == 16:
        assert pl.grid <= 2 * 256
        os.environ["DLAMD_GRID_MULT"] = "1"
        try:
            _lib.check(lib.dl_mix_plan_shape(n, 0, 1 << 20, nnz, 5, 1, 1, -1, ctypes.byref(pl)),
                       "plan")
        finally:
            os.environ.pop("DLAMD_GRID_MULT")
        assert pl.grid <= 256


def test_new_entry_points_validate_before_any_device_call():
    """dl_sgd_step, dl_mlp_grad, dl_mix_rounds(_plan): bad arguments come back as status codes
    with a message, nothing is launched (runs without a GPU)."""
    from distributed_learning_amd import _lib
    lib = _lib.load()
    a = _lib.DlSgdArgs()
    a.n_rows, a.n_params = 4, 16
    assert lib.dl_sgd_step(ctypes.byref(a), None) == _lib.DL_ERR_INVALID   # null pointers
    a.x = a.g = a.out = 16
    a.ldx = a.ldg = a.ldo = 16
    a.momentum = 0.9                                                        # ... no buffer
    assert lib.dl_sgd_step(ctypes.byref(a), None) == _lib.DL_ERR_INVALID
    assert b"momentum" in lib.dl_last_error()
    a.momentum, a.nesterov = 0.0, 1
    assert lib.dl_sgd_step(ctypes.byref(a), None) == _lib.DL_ERR_INVALID
    assert b"Nesterov" in lib.dl_last_error()
    m = _lib.DlMlpArgs(4, 32, 784, 150, 10)                                 # batch 32
    assert lib.dl_mlp_grad(ctypes.byref(m), None) == _lib.DL_ERR_UNSUPPORTED
    m = _lib.DlMlpArgs(4, 64, 784, 150, 10)
    m.tile_cols = 6                                                         # not a power of 2
    assert lib.dl_mlp_grad(ctypes.byref(m), None) == _lib.DL_ERR_INVALID
    P = 150 * 784 + 150 + 2 * (150 * 150 + 150) + 10 * 150 + 10
    m = _lib.DlMlpArgs(4, 64, 784, 150, 10, 16, P + 48, 1 << 36, 64 * 784, 1 << 38, 64,
                       1 << 40, P + 48, None, 0, 2, 0.1)                  # out_mode 2
    assert lib.dl_mlp_grad(ctypes.byref(m), None) == _lib.DL_ERR_INVALID
    assert b"out_mode" in lib.dl_last_error()
    m.out_mode, m.ldg = 1, P + 112                                          # step, ldg != ldx
    assert lib.dl_mlp_grad(ctypes.byref(m), None) == _lib.DL_ERR_INVALID
    assert b"ldg == ldx" in lib.dl_last_error()
    # (ABI 10) the two-launch workspace: one [64][156] fp32 image per agent, 16-byte aligned,
    # disjoint from X and G
    assert lib.dl_mlp_workspace_bytes(256) == 256 * 64 * 156 * 4
    assert lib.dl_mlp_workspace_bytes(0) == 0
    m.out_mode, m.ldg = 0, P + 48
    m.workspace = (1 << 42) + 4                                             # misaligned
    assert lib.dl_mlp_grad(ctypes.byref(m), None) == _lib.DL_ERR_INVALID
    assert b"workspace" in lib.dl_last_error()
    m.workspace = (1 << 40) + 4096                                          # inside G
    assert lib.dl_mlp_grad(ctypes.byref(m), None) == _lib.DL_ERR_INVALID
    assert b"workspace" in lib.dl_last_error()
    x = _lib.DlMixArgs()
    x.x, x.y, x.n_params, x.ldx, x.ldy = 256, 1 << 20, 64, 64, 64
    x.W = _lib.DlCsr(16, 16, 16, 4, 12, 3, 1, 1)
    assert lib.dl_mix_rounds(ctypes.byref(x), 0, None, 0, None) == _lib.DL_ERR_INVALID
    assert b"rounds" in lib.dl_last_error()
    x.n_halo, x.halo, x.ldh = 2, 4096, 64
    pl = _lib.DlMixPlan()
    assert lib.dl_mix_rounds_plan(ctypes.byref(x), ctypes.byref(pl)) == _lib.DL_ERR_UNSUPPORTED
    assert b"halo" in lib.dl_last_error()


def test_mix_until_validates_and_sizes():
    """dl_mix_until / dl_mix_until_fits: argument errors and the LDS fit come back as status
    codes before any launch (runs without a GPU)."""
    from distributed_learning_amd import _lib
    lib = _lib.load()
    assert lib.dl_mix_until_fits(8, 617, 24) == 1
    assert lib.dl_mix_until_fits(8, 2048, 24) == 1     # 2 x 64 KiB images + mean + CSR
    assert lib.dl_mix_until_fits(8, 4096, 24) == 0
    assert lib.dl_mix_until_fits(8, 1 << 20, 24) == 0
    assert lib.dl_mix_until_fits(0, 10, 0) == 0
    u = _lib.DlMixUntilArgs()
    assert lib.dl_mix_until(None, None) == _lib.DL_ERR_INVALID
    assert lib.dl_mix_until(ctypes.byref(u), None) == _lib.DL_ERR_INVALID
    u.x = u.y = 256
    u.status = 64
    u.n_params = u.ldx = u.ldy = 64
    u.W = _lib.DlCsr(16, 16, 16, 4, 12, 3, 0, 0)
    assert lib.dl_mix_until(ctypes.byref(u), None) == _lib.DL_ERR_INVALID   # max_rounds 0
    assert b"max_rounds" in lib.dl_last_error()
    u.max_rounds = 1
    u.y = 512                                                                # partial overlap
    assert lib.dl_mix_until(ctypes.byref(u), None) == _lib.DL_ERR_INVALID
    assert b"overlaps" in lib.dl_last_error()
    u.y = 256                                                                # in place
    u.n_params = u.ldx = u.ldy = 1 << 20
    assert lib.dl_mix_until(ctypes.byref(u), None) == _lib.DL_ERR_UNSUPPORTED
    assert b"LDS" in lib.dl_last_error()


def test_tiled_halo_arguments_validate_without_a_gpu():
    """ABI 8 (column-tiled halo rounds): the per-peer block table, the tiled ld* (block rows)
    and the whole-tile requirement are checked on the host, before any launch; the planner picks
    a tile width for every source row (local + halo) that divides n_params and keeps the halo
    kernel at <= 4 row passes per thread (runs without a GPU)."""
    from distributed_learning_amd import _lib
    lib = _lib.load()
    pl = _lib.DlMixPlan()
    # the c4 rank of 8: 512 local rows + 96 halo rows, 2^18 params -> T = 16 (608 x 16 x 16 B)
    _lib.check(lib.dl_mix_plan_shape(512, 96, 1 << 18, 5 * 512, 5, 1, 1, -1, ctypes.byref(pl)),
               "plan")
    assert pl.path == 1 and pl.tile_cols == 16
    # a width that does not divide n_params is halved until it does
    _lib.check(lib.dl_mix_plan_shape(512, 96, 1000, 5 * 512, 5, 1, 1, -1, ctypes.byref(pl)),
               "plan")
    assert pl.tile_cols == 8
    # more than 4 passes of 1024 threads at C chunks: a narrower tile (here 3000 + 100 rows)
    _lib.check(lib.dl_mix_plan_shape(3000, 100, 1 << 16, 5 * 3000, 5, 1, 1, -1, ctypes.byref(pl)),
               "plan")
    assert (3100 * pl.tile_cols // 4) <= 4 * 1024
    assert pl.n_tiles * pl.tile_cols == 1 << 16            # no tile groups at 3100 rows

    def args(**kw):
        a = _lib.DlMixArgs()
        a.x, a.y, a.halo = 1 << 20, 1 << 30, 1 << 34
        a.n_params, a.tile_cols = 64, 16
        a.W = _lib.DlCsr(16, 16, 16, 4, 20, 5, 1, 1, 5)
        a.n_halo = 4
        for k, v in kw.items():
            setattr(a, k, v)
        return a

    def err(a):
        rc = lib.dl_mix_round(ctypes.byref(a), None, 0, None)
        return rc, lib.dl_last_error()

    rows = (ctypes.c_int32 * 2)(1, 2)          # sums to 3, not n_halo = 4
    rc, msg = err(args(n_halo_blocks=2, halo_block_rows=ctypes.cast(rows, ctypes.c_void_p)))
    assert rc == _lib.DL_ERR_INVALID and b"sum" in msg
    rc, msg = err(args(n_halo_blocks=2, halo_block_rows=None))
    assert rc == _lib.DL_ERR_INVALID and b"halo_block_rows" in msg
    rc, msg = err(args(n_halo_blocks=17))
    assert rc == _lib.DL_ERR_INVALID and b"n_halo_blocks" in msg
    zero = (ctypes.c_int32 * 2)(4, 0)
    rc, msg = err(args(n_halo_blocks=2, halo_block_rows=ctypes.cast(zero, ctypes.c_void_p)))
    assert rc == _lib.DL_ERR_INVALID and b"<= 0" in msg
    rc, msg = err(args(n_params=72))           # not whole tiles of 16
    assert rc == _lib.DL_ERR_INVALID and b"tile_cols" in msg
    rc, msg = err(args(ldx=2))                  # block rows below the local rows
    assert rc == _lib.DL_ERR_INVALID and b"ldx" in msg
    rc, msg = err(args(tile_cols=0, ldx=64, ldy=64, ldh=64, n_halo_blocks=1))
    assert rc == _lib.DL_ERR_INVALID and b"n_halo_blocks" in msg
    rc, msg = err(args(y=(1 << 34) + 64))       # y inside the halo blocks
    assert rc == _lib.DL_ERR_INVALID and b"halo" in msg
    rc, msg = err(args(n_hub_rows=-1))
    assert rc == _lib.DL_ERR_INVALID and b"n_hub_rows" in msg
    # the lagged deviation: mean_prev and colsum_out together; without dev_sq the round leaves
    # its partial rows in the workspace (column-tiled only), so dev_max alone is accepted there
    # and the row-major layout refuses it -- all before any device call
    rc, msg = err(args(mean_prev=1 << 36))
    assert rc == _lib.DL_ERR_INVALID and b"lagged" in msg
    rc, msg = err(args(tile_cols=0, ldx=64, ldy=64, ldh=64, mean_prev=1 << 36,
                       colsum_out=(1 << 36) + 4096, dev_max=(1 << 36) + 8192))
    assert rc == _lib.DL_ERR_INVALID and b"column-tiled" in msg
    # (ABI 9) the partial-rows mode needs partial_rows_out: a caller that forgets dev_sq gets an
    # error, not a round whose deviation nobody reduces
    rc, msg = err(args(mean_prev=1 << 36, colsum_out=(1 << 36) + 4096))
    assert rc == _lib.DL_ERR_INVALID and b"partial_rows_out" in msg
    n_parts = ctypes.c_int32(-7)
    rc, msg = err(args(mean_prev=1 << 36, colsum_out=(1 << 36) + 4096,
                       partial_rows_out=ctypes.pointer(n_parts)))
    assert rc == _lib.DL_ERR_WORKSPACE, msg   # accepted: only the missing workspace is refused
    assert n_parts.value == 0                  # cleared before anything can fail
    # dl_row_sums: outputs and sizes checked on the host
    assert lib.dl_row_sums(None, 2, 8, 1 << 20, None, 0, None) == _lib.DL_ERR_INVALID
    assert lib.dl_row_sums(1 << 20, 2, 8, None, None, 1, None) == _lib.DL_ERR_INVALID
    # dl_step_rows_tiled: arguments before any launch
    assert lib.dl_step_rows_tiled(None, 4, None, 0, 0.0, None, 2, 64, 16, None, None) == \
        _lib.DL_ERR_INVALID
    assert lib.dl_step_rows_tiled(1 << 20, 4, None, 0, 0.0, 1 << 22, 2, 64, 12, 1 << 24,
                                  None) == _lib.DL_ERR_INVALID          # T not a power of 2
    assert lib.dl_step_rows_tiled(1 << 20, 4, None, 0, 0.0, 1 << 22, 2, 64, 16,
                                  (1 << 20) + 16, None) == _lib.DL_ERR_INVALID   # out overlaps x
    assert b"overlaps" in lib.dl_last_error()


@pytest.mark.parametrize("n,nnz,uni,ds,shared,minr,want", [
    (100, 350, 0, 0, 0, 3, 24),        # row-stochastic W: one-image kernel, every round's mean
    (1500, 5250, 0, 0, 0, 3, 12),      # ... 2 agents per thread
    (4096, 5 * 4096, 5, 0, 0, 5, 4),   # ... 4 agents per thread, up to 4096 agents
    (3000, 9000, 0, 1, 0, 3, 4),       # irregular doubly stochastic above 2048 agents
    (512, 5 * 512, 5, 1, 1, 5, 32),    # two-image kernels
    (1024, 5 * 1024, 5, 1, 1, 5, 24),  # register-cached regular graph above 512 agents
    (2048, 5 * 2048, 5, 1, 1, 5, 16),  # wide kernel
    (4096, 5 * 4096, 5, 1, 1, 5, 8),
])
def test_trace_plan_matches_the_header(n, nnz, uni, ds, shared, minr, want):
    """dlamd.h's dl_mix_rounds_trace contract, checked on the host (no device call): any W --
    row-stochastic ones included -- up to 4096 agents, and the rounds per pass it documents."""
    from distributed_learning_amd import _lib
    lib = _lib.load()
    a = _lib.DlMixArgs()
    a.x, a.y, a.n_params = 1 << 20, 1 << 36, 4096
    a.ldx = a.ldy = 4096
    a.W = _lib.DlCsr(1 << 40, 1 << 41, 1 << 42, n, nnz, uni, ds, shared, minr)
    k = ctypes.c_int32(0)
    _lib.check(lib.dl_mix_trace_plan(ctypes.byref(a), ctypes.byref(k)), "trace plan")
    assert k.value == want


def test_trace_plan_refusals_match_the_header():
    """What the header says dl_mix_rounds_trace does not take comes back DL_ERR_UNSUPPORTED with
    a message: more than 4096 agents, a local step (g), n_params not a multiple of 4, halo rows."""
    from distributed_learning_amd import _lib
    lib = _lib.load()

    def plan(n=100, **kw):
        a = _lib.DlMixArgs()
        a.x, a.y, a.n_params = 1 << 20, 1 << 36, 4096
        a.ldx = a.ldy = a.ldg = 4096
        a.W = _lib.DlCsr(1 << 40, 1 << 41, 1 << 42, n, 3 * n, 0, 0, 0, 3)
        for key, v in kw.items():
            setattr(a, key, v)
        k = ctypes.c_int32(0)
        return lib.dl_mix_trace_plan(ctypes.byref(a), ctypes.byref(k)), lib.dl_last_error()

    assert plan()[0] == _lib.DL_OK
    rc, msg = plan(n=5000)
    assert rc == _lib.DL_ERR_UNSUPPORTED and b"5000" in msg
    rc, msg = plan(g=1 << 38)
    assert rc == _lib.DL_ERR_UNSUPPORTED and b"g must be NULL" in msg
    rc, msg = plan(n_params=4094, ldx=4096, ldy=4096)
    assert rc == _lib.DL_ERR_UNSUPPORTED and b"multiple of 4" in msg
    rc, msg = plan(n_halo=4, halo=1 << 39, ldh=4096)
    assert rc == _lib.DL_ERR_UNSUPPORTED and b"halo" in msg


def test_tile_groups_plan_without_a_gpu(monkeypatch):
    """A column-tiled halo round of few source rows walks g consecutive data tiles as one kernel
    tile (the split scheme's boundary launch: 92 output rows over 276 sources at T = 16 -> g = 2;
    372 at T = 8 -> 4; 384 at T = 4 -> 8): n_tiles counts kernel tiles, tile_cols stays the data
    width, the kernel keeps <= 4 row passes per thread; DLAMD_TILE_GROUP=1 turns groups off, and
    the whole round's 608 rows or a round without halo rows never group (runs without a GPU)."""
    from distributed_learning_amd import _lib
    lib = _lib.load()
    P = 1 << 18

    def plan(rows, halo, T):
        pl = _lib.DlMixPlan()
        _lib.check(lib.dl_mix_plan_shape(rows, halo, P, 5 * rows, 5, 1, 1, T, ctypes.byref(pl)),
                   "plan")
        assert pl.path == 1 and pl.tile_cols == T
        return pl
    for rows, halo, T, g in [(92, 184, 16, 2), (124, 248, 8, 4), (128, 256, 4, 8)]:
        pl = plan(rows, halo, T)
        assert pl.n_tiles == P // (T * g), (rows, halo, T, pl.n_tiles)
        assert (rows + halo) * (T * g // 4) <= 4 * 1024
    assert plan(512, 96, 16).n_tiles == P // 16
    assert plan(276, 0, 16).n_tiles == P // 16
    monkeypatch.setenv("DLAMD_TILE_GROUP", "1")
    assert plan(92, 184, 16).n_tiles == P // 16
    monkeypatch.setenv("DLAMD_TILE_GROUP", "2")
    assert plan(124, 248, 8).n_tiles == P // 16
