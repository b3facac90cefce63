"""CPU checks of the BUILT gfx950 code object (no GPU): the streaming kernels of the headline
paths still carry their non-temporal cache hints.

Round 5 lost them without any test noticing: the tile kernel chooses non-temporal or plain
loads and stores at run time (dl::TileArgs nt_load / nt_store), and the optimizer merged the two
arms of that choice -- identical instructions but for the hint -- and kept the plain one.  The
c2 round fell from 446 to 427 rounds/s on one box (profiles/r13/c2_matrix).  The kernels now
stream through buffer instructions whose cache policy is a constant operand (mix_tile.hip
buf_ld4 / buf_st4); this test disassembles libdlamd.so's device code and checks every
instantiation the bench lines launch for both arms."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "distributed-learning_amd", "_lib", "libdlamd.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"

pytestmark = pytest.mark.skipif(not (os.path.exists(LIB) and
                                     os.path.exists(os.path.join(LLVM, "llvm-objdump"))),
                                reason="needs the built library and the ROCm LLVM tools")


@pytest.fixture(scope="module")
def code_objects(tmp_path_factory):
    """The gfx950 code objects of every linked translation unit (one offload bundle each)."""
    d = tmp_path_factory.mktemp("isa")
    fat = d / "fat.bin"
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", LIB,
                    str(d / "host.o")], check=True, capture_output=True)
    data = fat.read_bytes()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    out = []
    for j, s in enumerate(starts):
        b = d / f"b{j}.bin"
        b.write_bytes(data[s:starts[j + 1] if j + 1 < len(starts) else len(data)])
        co = d / f"d{j}.co"
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                            f"--input={b}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                            f"--output={co}"], capture_output=True)
        if r.returncode == 0 and co.exists() and co.stat().st_size:
            out.append(co)
    assert out, "no gfx950 code object in libdlamd.so"
    return out


def _disasm(code_objects, pattern):
    """Disassembly of the one kernel whose mangled name matches ``pattern``."""
    for co in code_objects:
        syms = subprocess.run([f"{LLVM}/llvm-readelf", "-sW", str(co)], capture_output=True,
                              text=True, check=True).stdout
        hits = sorted({s for s in re.findall(r"(_ZN2dl\S+)", syms)
                       if re.fullmatch(pattern, s)})
        if hits:
            assert len(hits) == 1, hits
            return subprocess.run([f"{LLVM}/llvm-objdump", "-d",
                                   f"--disassemble-symbols={hits[0]}", str(co)],
                                  capture_output=True, text=True, check=True).stdout
    raise AssertionError(f"kernel {pattern} not in the code object")


def _tile(c, kv, sgd, dev, halo, rd, lag, rag):
    b = lambda v: "1" if v else "0"   # noqa: E731
    return (rf"_ZN2dl12_GLOBAL__N_115mix_tile_kernelILi{c}ELi{kv}ELb{b(sgd)}ELb{b(dev)}ELb1"
            rf"ELi{halo}ELb1ELi{rd}ELb{b(lag)}ELi{rag}EEEvNS_8TileArgsE")


@pytest.mark.parametrize("what,pattern,kv", [
    ("c2 round", _tile(4, 4, True, True, 0, 0, False, 0), 4),
    ("c4 round", _tile(1, 4, True, True, 0, 0, False, 0), 4),
    ("c3 round", _tile(16, 4, True, True, 0, 0, False, 0), 4),
    ("c4 per-edge weights (path 4)", _tile(1, 4, True, True, 0, 5, False, 0), 4),
    ("c4-ba (path 5)", _tile(1, 4, True, True, 0, 3, False, 2), 4),
    ("c4 rank of 8 (halo, lagged)", _tile(4, 3, True, False, 2, 0, True, 0), 3),
])
def test_round_kernels_stream_non_temporally(code_objects, what, pattern, kv):
    """Both arms of the run-time policy exist: non-temporal loads of x and g for every row pass,
    and a non-temporal store of X' beside the plain one (an X' that fits the MALL)."""
    asm = _disasm(code_objects, pattern)
    loads = re.findall(r"(?:global|buffer)_load_dwordx4[^\n]*", asm)
    stores = re.findall(r"(?:global|buffer)_store_dwordx4[^\n]*", asm)
    nt_loads = [x for x in loads if re.search(r"\bnt\b", x)]
    nt_stores = [x for x in stores if re.search(r"\bnt\b", x)]
    assert len(nt_loads) >= 2 * kv, (what, len(nt_loads), len(loads))
    assert nt_stores and len(stores) > len(nt_stores), (what, len(nt_stores), len(stores))


def test_halo_pack_stores_non_temporally(code_objects):
    """The halo pack's send blocks are read once, by the peers' receives (dlamd.h)."""
    asm = _disasm(code_objects, r"_ZN2dl12_GLOBAL__N_122step_rows_tiled_kernel\S*liii")
    stores = re.findall(r"(?:global|buffer)_store_dwordx4[^\n]*", asm)
    assert stores and all(re.search(r"\bnt\b", s) for s in stores)


def test_mlp_layer1_ring_waits_are_counted(code_objects):
    """The c3 gradient kernel's layer-1 producer keeps three slices' loads in flight (7 float4
    loads a slice per producer lane); the waits before a slice's LDS stores must count the two
    younger sets' loads: vmcnt(20) down to vmcnt(14), at the ring's loop head too.  When the
    scheduler interleaved the first sets' loads, the loop-head wait became vmcnt(0) and drained
    the ring every few slices (fixed: c3 +0.5-1 %, profiles/r14/l1order)."""
    asm = _disasm(code_objects,
                  r"_ZN2dl12_GLOBAL__N_116mlp_fused_kernelILb0ELb1ELb0ELb0EEEvNS0_7MlpArgsE")
    waits = [int(x) for x in re.findall(r"s_waitcnt\s+vmcnt\((\d+)\)", asm)]
    ring = list(range(20, 13, -1))
    runs = sum(waits[i:i + 7] == ring for i in range(len(waits)))
    assert runs >= 3, (runs, waits[:60])   # one per register set of the unrolled ring


def test_mlp_bf16_split_is_packed(code_objects):
    """The exact three-way bf16 split of the c3 gradient kernel converts pairs: one
    v_cvt_pk_bf16_f32 per plane and pair, the remainders by v_pk_add_f32.  Element-wise, the same
    kernel had 1722 conversions and 62 packed adds; packed, 738 and 408 (c3 +1.1 %, bit-identical,
    profiles/r14/splitpk).  A regression to per-element conversions shows as the count jumping."""
    asm = _disasm(code_objects,
                  r"_ZN2dl12_GLOBAL__N_116mlp_fused_kernelILb0ELb1ELb0ELb0EEEvNS0_7MlpArgsE")
    cvt = len(re.findall(r"v_cvt_pk_bf16_f32", asm))
    pk_add = len(re.findall(r"v_pk_add_f32", asm))
    assert 0 < cvt <= 1000 and pk_add >= 300, (cvt, pk_add)
