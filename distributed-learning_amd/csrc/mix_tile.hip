// Fused gossip-mixing kernels for gfx950 (MI355X).
//
// Hot path: one consensus round X' = W (X - lr G) over a sparse agent graph, plus the
// disagreement ||x'_a - mean(x')|| -- the work of Mixer._mix_params_once and
// Mixer._get_deviation_dict (utils/consensus_simple/mixer.py:43-66) after a local step.
//
// Design: the mix is column-independent, so a workgroup owns a column tile of
// T = 4*C floats for ALL agents.  The tile (n_src x T fp32) is staged once in LDS; every
// neighbour read is an LDS read, so each element of X and G crosses HBM exactly once and each
// element of X' is written once (12 B per element-round with the local step, 8 B without),
// independent of the graph.  Workgroups are persistent (grid = CUs) and prefetch the next
// tile's X/G rows into registers while mixing the current one from LDS, so HBM streaming
// overlaps the LDS phase.  The CSR is staged in LDS once per workgroup (16-bit column ids), so
// the mix phase issues no vector-memory loads that would queue behind the prefetch (vmcnt is
// in-order on CDNA).  Products and sums are separate fp32 ops in CSR order (-ffp-contract=off),
// which reproduces the reference's left fold bit for bit.
#include <mutex>
#include <set>
#include <type_traits>
#include <utility>

#include "dl_internal.h"

namespace dl {
namespace {

__device__ __forceinline__ float4 zero4() { return make_float4(0.f, 0.f, 0.f, 0.f); }

typedef float f32x4 __attribute__((ext_vector_type(4)));

// 16-byte non-temporal load (global_load_dwordx4 ... nt): streamed once, keep it out of L2/MALL
__device__ __forceinline__ float4 nt_load4(const float4 *p) {
    const f32x4 x = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(p));
    return make_float4(x.x, x.y, x.z, x.w);
}

// 16-byte non-temporal store (global_store_dwordx4 ... nt)
__device__ __forceinline__ void nt_store4(float4 v, float4 *p) {
    f32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f32x4 *>(p));
}

// FAST-path streams of a tile through buffer instructions whose cache policy is an immediate.
// The non-temporal hint is a runtime choice (dl::TileArgs nt_load / nt_store), and two global
// accesses that differ only in it are one instruction to the optimizer, which merged the two
// arms of that choice and dropped the hint (round 5: every load and store of the c2 round plain,
// 446 -> 427 rounds/s on one box).  Buffer loads and stores carry the policy as an operand that
// must stay a constant, so the arms stay two instructions; tests/test_kernel_isa.py checks the
// built code object for them.  Base = a uniform tile pointer, 32-bit offsets as for the global
// forms (the host admits this path only when every operand spans < 4 GiB); the resource's
// record count is the whole 32-bit range, so no access is clipped.
constexpr int kBufNT = 2;   // cache-policy operand: nt (gfx950)
typedef unsigned int u32x4v __attribute__((vector_size(16)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void *base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, -1, 0x00020000);
}

template <int AUX>
__device__ __forceinline__ float4 buf_ld4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    const f32x4 v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX));
    return make_float4(v.x, v.y, v.z, v.w);
}

template <int AUX>
__device__ __forceinline__ void buf_st4(float4 v, __amdgpu_buffer_rsrc_t r, uint32_t off) {
    const f32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, x), r, off, 0, AUX);
}

// Load 4 consecutive floats starting at column c0 of `row`; columns >= P read as 0.
__device__ __forceinline__ float4 ld4(const float *__restrict__ row, int64_t c0, int64_t P,
                                      bool vec) {
    if (vec && c0 + 3 < P) return *reinterpret_cast<const float4 *>(row + c0);
    float4 v = zero4();
    if (c0 < P) v.x = row[c0];
    if (c0 + 1 < P) v.y = row[c0 + 1];
    if (c0 + 2 < P) v.z = row[c0 + 2];
    if (c0 + 3 < P) v.w = row[c0 + 3];
    return v;
}

__device__ __forceinline__ void st4(float *__restrict__ row, int64_t c0, int64_t P, bool vec,
                                    float4 v) {
    if (vec && c0 + 3 < P) {
        *reinterpret_cast<float4 *>(row + c0) = v;
        return;
    }
    if (c0 < P) row[c0] = v.x;
    if (c0 + 1 < P) row[c0 + 1] = v.y;
    if (c0 + 2 < P) row[c0 + 2] = v.z;
    if (c0 + 3 < P) row[c0 + 3] = v.w;
}

// x - lr*g with two roundings (numpy: x - np.float32(lr) * g).
__device__ __forceinline__ float4 local_step(float4 x, float4 g, float lr) {
    float4 t;
    t.x = x.x - lr * g.x;
    t.y = x.y - lr * g.y;
    t.z = x.z - lr * g.z;
    t.w = x.w - lr * g.w;
    return t;
}

__device__ __forceinline__ void axpy4(float4 &acc, float w, float4 v) {
    acc.x = acc.x + w * v.x;
    acc.y = acc.y + w * v.y;
    acc.z = acc.z + w * v.z;
    acc.w = acc.w + w * v.w;
}

__device__ __forceinline__ void add4(float4 &a, float4 b) {
    a.x = a.x + b.x;
    a.y = a.y + b.y;
    a.z = a.z + b.z;
    a.w = a.w + b.w;
}

// v + v[lane ^ m] across the wave (m a power of two, a compile-time constant after unrolling),
// without the LDS unit where gfx950 has a register path: xor 1 / 2 are DPP quad permutes, xor
// 16 / 32 the v_permlane16/32_swap pair (their two results are {v, partner} per lane, in some
// order: the sum is the same IEEE add); xor 4 / 8 stay ds_bpermute.  Bit-identical to
// v + __shfl_xor(v, m) (a + b == b + a).
__device__ __forceinline__ float xor_add(float v, int m) {
    if (m == 1)
        return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));
    if (m == 2)
        return v + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));
    if (m == 16) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v),
                                                        false, false);
        return __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    if (m == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v),
                                                        false, false);
        return __uint_as_float(r[0]) + __uint_as_float(r[1]);
    }
    return v + __shfl_xor(v, m);
}

__device__ __forceinline__ float4 shfl_xor4(float4 v, int m) {
    v.x = xor_add(v.x, m);
    v.y = xor_add(v.y, m);
    v.z = xor_add(v.z, m);
    v.w = xor_add(v.w, m);
    return v;
}

// C    : float4 chunks per row in a tile (T = 4*C columns)
// KV   : row passes per thread (rows s + k*SLOTS, k < KV); R <= KV * SLOTS
// SGD  : fused local step x - lr*g on local rows before mixing
// DEV  : fused column mean + per-agent ||y_a - mean||^2 (needs all agents in the tile)
// MIX  : false = deviation of x only (no LDS staging, no output rows)
// HALO : 1, 2: source rows [n_loc, n_src) come from the halo buffer (1: row-major rows of ldh; 2:
//        column-tiled per-peer blocks, dl_mix_args.n_halo_blocks); output rows [0, n_rows) follow the
//        CSR and need not be source rows (n_loc != n_rows: an interior or boundary row set of
//        an agent partition, sharding.py)
// FAST : every tile is full and every operand 16-byte aligned (float4 path with 32-bit
//        offsets from a uniform tile base); false = guarded scalar path (tail, unaligned)
// RD   : 0 = CSR staged in LDS; RD > 0 = regular graph with RD entries per row whose CSR does
//        not fit LDS beside the tile (per-edge weights on thousands of agents): every thread
//        keeps its KV rows' weights and LDS row indices in registers (a thread mixes exactly
//        the rows it stages), loaded once per workgroup.
// Tiles cover columns [col_base + t*T, ...) for t < n_tiles.  Lanes whose row does not exist
// (the last, ragged pass) re-read row 0 -- an L1 hit -- and never write LDS or y, so every
// pass is straight-line code and the loads of the next tile stay in flight during the mix.
// LAG  : halo rounds only: ||x_a - mean_prev||^2 of every local source row while it is staged
//        (the deviation of the previous round's iterate against its all-reduced global mean) and
//        this rank's column sums of the stepped inputs t into colsum_out -- all-reduced over the
//        ranks, the numerator of the next mean_prev (sum(W t) = sum(t): W doubly stochastic).
// RAG  : (with RD > 0) an irregular graph whose every row has >= RD entries (dl_csr.min_row_nnz):
//        each row's first RD entries in registers as above, the rest ("tail", nnz - RD*n_rows
//        entries) staged once per workgroup in LDS behind the tile; row r's tail is
//        [rowptr[r] - RD*r, rowptr[r+1] - RD*(r+1)) there.  RAG = 2: {weight, row} pairs of 8 B
//        (one ds_read_b64 per entry, +4 % on c4-ba); RAG = 1: fp32 weights then u16 rows (6 B,
//        for tails that do not fit LDS at 8 B).  The fold runs the
//        register head, then the tail, in CSR order: still the reference's left fold.
// Waves per SIMD the compiler must leave room for: 8 (<= 64 VGPRs, two 1024-thread workgroups
// per CU) for the grouped halo launch of few rows (C >= 8 at <= 3 passes, the split scheme's
// boundary launch, latency-bound at one workgroup a CU), else no constraint
template <int C, int KV, int HALO, bool LAG>
constexpr int tile_waves_per_eu() {
    return (HALO == 2 && C >= 8 && KV <= 3 && !LAG) ? 8 : 1;
}

template <int C, int KV, bool SGD, bool DEV, bool MIX, int HALO, bool FAST, int RD = 0,
          bool LAG = false, int RAG = 0>
__global__ void __attribute__((amdgpu_flat_work_group_size(1, kTileThreads),
                               amdgpu_waves_per_eu(tile_waves_per_eu<C, KV, HALO, LAG>())))
mix_tile_kernel(TileArgs a) {
    constexpr bool PACK = RAG == 2;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    float4 *tile = reinterpret_cast<float4 *>(smem);
    constexpr int NT = kTileThreads;
    constexpr int SLOTS = NT / C;  // rows covered per pass
    constexpr int T = 4 * C;
    const int tid = threadIdx.x;
    const int c = tid & (C - 1);
    const int s = tid / C;
    const int R = a.n_src;
    const int Nr = a.n_rows;
    const int NL = a.n_loc;   // source rows [0, NL) from x (stepped), [NL, R) from the halo
    const int64_t P = a.n_params;
    const int nnz = a.nnz;

    // staged CSR: n_w weights (all nnz, or one row's when every row shares them), u16 columns,
    // u16 row_ptr unless the graph is regular
    float *lw = reinterpret_cast<float *>(smem + a.csr_off);
    uint16_t *lcol = reinterpret_cast<uint16_t *>(smem + a.csr_off + 4u * (uint32_t)a.n_w);
    uint16_t *lrp = lcol + nnz;
    // register CSR: weights, and the float4 LDS index (col * C + c < 2^16: the host admits
    // KV <= 4 at C <= 2, i.e. at most 4096 rows) packed two per register
    constexpr int NRC = RD > 0 ? KV * RD : 1;
    float rw[NRC];
    uint32_t ri[(NRC + 1) / 2];
    // RAG: per pass, this row's tail in LDS: start (low 16 bits) and length (high 16 bits)
    uint32_t rdesc[RAG ? KV : 1];
    const int ntail = RAG ? nnz - RD * Nr : 0;
    float *ltw = reinterpret_cast<float *>(smem + a.csr_off);
    uint16_t *ltc = reinterpret_cast<uint16_t *>(smem + a.csr_off + 4u * (uint32_t)ntail);
    uint2 *ltp = reinterpret_cast<uint2 *>(smem + a.csr_off);   // RAG == 2
    // RAG, hub rows: rows [0, NH) (the longest ones, in a row-length order) are each folded by
    // four lanes, one column each, instead of by their owner alone: a Barabasi-Albert hub's tail
    // (169 entries at c4-ba) is one lane's serial chain, and column lanes fold it with scalar
    // ops, twice the entries per LDS round trip.  Each column keeps its CSR-order left fold, so
    // the bits are the owner's.  The lanes are the LAST 4 NH threads (their own rows are the
    // shortest); the owners skip those rows.  NH is wave-uniform (host: <= 256).
    // (not at a five-entry head: beside its 30 head registers the hub loop spills)
    const int NH = (RAG && RD < 5) ? a.n_hub : 0;
    const int hl = tid - (NT - 4 * NH);           // >= 0: hub lane
    const bool hub_lane = RAG && RD < 5 && hl >= 0;
    const int hr = hub_lane ? hl >> 2 : 0, hc = hl & 3;
    uint2 *hubp = reinterpret_cast<uint2 *>(smem + a.hub_off);
    uint32_t hdesc = 0u;   // hub lane: its row's tail [start, start + len) in the LDS tail
    if (hub_lane) {
        const int e0 = a.rowptr[hr], e1 = a.rowptr[hr + 1];
        const int st = min(max(e0 - RD * hr, 0), ntail);
        hdesc = (uint32_t)st | ((uint32_t)min(max(e1 - e0 - RD, 0), ntail - st) << 16);
    }
    float hacc = 0.f;      // hub lane: its row's squared deviation over the tiles (hub_dev)
    if (RD > 0) {
#pragma unroll
        for (int i = 0; i < (NRC + 1) / 2; ++i) ri[i] = 0u;
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const int r = s + k * SLOTS;
            const int rr = r < Nr ? r : 0;
            const int e0 = RAG ? a.rowptr[rr] : rr * RD;
#pragma unroll
            for (int e = 0; e < RD; ++e) {
                const int j = k * RD + e;
                // (RAG: a wrong min_row_nnz promise -- a row shorter than the head -- gives
                // wrong results but never reads past the CSR: indices are clamped into it)
                const int idx = RAG ? min(max(e0 + e, 0), nnz - 1) : e0 + e;
                rw[j] = a.w[idx];
                ri[j >> 1] |= ((uint32_t)a.col[idx] * C + c) << (16 * (j & 1));
            }
            if (RAG) {
                // this row's tail [st, st + ln) in the LDS tail, clamped into [0, ntail) for the
                // same reason
                const int e1 = a.rowptr[rr + 1];
                const int st = min(max(e0 - RD * rr, 0), ntail);
                const int ln = min(max(e1 - e0 - RD, 0), ntail - st);
                rdesc[k] = r < Nr ? (uint32_t)st | ((uint32_t)ln << 16) : 0u;
            }
        }
        if (RAG) {
            // stage the tail: first a row id per tail slot (u16, in the tile area, which the
            // first tile's staging overwrites only after the barrier below), then every thread
            // copies tail slots t = tid, tid + NT, ... -- coalesced loads whatever the degrees
            uint16_t *trow = reinterpret_cast<uint16_t *>(smem);
#pragma unroll
            for (int k = 0; k < KV; ++k) {
                const uint32_t t0 = rdesc[k] & 0xffffu, tn = rdesc[k] >> 16;
                for (uint32_t t = 0; t < tn; ++t) trow[t0 + t] = (uint16_t)(s + k * SLOTS);
            }
            __syncthreads();
            for (int t = tid; t < ntail; t += NT) {
                const int r = trow[t];
                // (clamped: with a wrong min_row_nnz promise a slot may hold no row of its own)
                const int e = min(t + RD * (r + 1), nnz - 1);
                const float we = a.w[e];
                const int ce = a.col[e];
                if (PACK) {
                    ltp[t] = make_uint2(__float_as_uint(we), (uint32_t)(ce * C + c));
                } else {
                    ltw[t] = we;
                    ltc[t] = (uint16_t)(ce * C + c);
                }
            }
            // hub rows: their register heads as {weight, row} pairs behind the tail, for the
            // four column lanes that fold each one (below)
            for (int i = tid; i < NH * RD; i += NT) {
                const int h = i / RD, e = i - (i / RD) * RD;
                const int idx = min(max(a.rowptr[h] + e, 0), nnz - 1);
                hubp[i] = make_uint2(__float_as_uint(a.w[idx]), (uint32_t)a.col[idx]);
            }
            __syncthreads();
        }
    }
    const int reg = a.regular;

    // FAST-path byte offsets: lane row s / chunk c; pass k adds k * step
    // (row stride = ld*4 in the row-major layout, T*4 in the column-tiled one).  Tile groups
    // (a.grp > 1, column-tiled halo rounds): chunk c lies in data tile gt = c >> cd_sh of the group, at
    // chunk c & (2^cd_sh - 1) of it -- gt data-tile strides further (< 4 GiB: 32-bit, checked
    // by the host like every FAST offset)
    const int grp = (HALO == 2 && a.grp > 1) ? a.grp : 1;   // the host groups halo rounds only
    const int gt = grp > 1 ? c >> a.cd_sh : 0;
    const uint32_t lc = 16u * (uint32_t)(grp > 1 ? c & ((1 << a.cd_sh) - 1) : c);
    const uint32_t cx = lc + (uint32_t)gt * (uint32_t)a.xts;   // row 0's chunk c in x
    const uint32_t cgx = SGD ? lc + (uint32_t)gt * (uint32_t)a.gts : 0u;
    uint32_t ox = (uint32_t)s * a.xrs + cx;
    const uint32_t sx = (uint32_t)SLOTS * a.xrs;
    uint32_t og = SGD ? (uint32_t)s * a.grs + cgx : 0u;
    const uint32_t sg = SGD ? (uint32_t)SLOTS * a.grs : 0u;
    uint32_t oy = (uint32_t)s * a.yrs + lc + (uint32_t)gt * (uint32_t)a.yts;
    const uint32_t sy = (uint32_t)SLOTS * a.yrs;
    // byte address of tile t's first element (row 0) in x / g / y
    auto tile_base = [&](const void *p, int64_t ts, int tile_id) {
        return reinterpret_cast<const char *>(p) + (a.tiled ? 0 : a.col_base * 4) +
               (int64_t)tile_id * grp * ts;
    };
    float4 *scratch = reinterpret_cast<float4 *>(smem + a.scratch_off);

    // HALO == 2 (column-tiled halo, FAST): per pass, the byte offset of this lane's halo row in
    // tile 0 and its per-tile stride -- one [n_tiles][rows_b][T] block per peer, so a row's tile
    // stride is its block's rows_b*T*4, picked by an unrolled select over the block table (no
    // dynamic indexing of the kernel arguments).  Local passes keep 16c / 0 (not read).  Two
    // registers per pass: the host keeps this instantiation at KV <= 4 (no spills).
    constexpr bool HT = HALO == 2;
    const int Td = T / grp;   // data tile width
    uint32_t hoff[HT ? KV : 1], hstr[HT ? KV : 1];
    if (HT) {
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const int h = s + k * SLOTS - NL;
            uint32_t o = lc, st = 0u;
            if (h >= 0 && h < R - NL) {
                {
                    int r0 = 0, r1 = R - NL;
                    uint32_t bo = 0u;
#pragma unroll
                    for (int b = 1; b < kMaxHaloBlocks; ++b) {
                        if (b < a.n_hblk && h >= a.hblk_row0[b]) {
                            r0 = a.hblk_row0[b];
                            bo = a.hblk_off[b];
                        }
                    }
#pragma unroll
                    for (int b = 1; b <= kMaxHaloBlocks; ++b)
                        if (b <= a.n_hblk && a.hblk_row0[b] > h && a.hblk_row0[b - 1] <= h)
                            r1 = a.hblk_row0[b];
                    o += bo + (uint32_t)(h - r0) * (uint32_t)(Td * 4);
                    st = (uint32_t)(r1 - r0) * (uint32_t)(Td * 4);
                    o += (uint32_t)gt * st;   // this chunk's data tile of the group
                }
            }
            hoff[k] = o;
            hstr[k] = st;
        }
    }

    float4 px[KV], pg[KV];
    float4 pm = zero4();             // LAG: this lane's chunk of mean_prev, prefetched with px
    float lacc[LAG ? KV : 1];        // LAG: per-pass partial ||x - mean_prev||^2 of the chunk
#pragma unroll
    for (int k = 0; k < (LAG ? KV : 1); ++k) lacc[k] = 0.f;
    // per-agent ||y - mean||^2 accumulators, spread over the C lanes of a row group: lane c keeps
    // the passes k with k % C == c (slot k / C), so ceil(KV / C) registers instead of KV.
    constexpr int ND = KV <= C ? 1 : KV / C;
    float dacc[ND];
#pragma unroll
    for (int k = 0; k < ND; ++k) dacc[k] = 0.f;
    // LD (C > 1, KV <= 4): each lane instead keeps its own chunk's partial of every pass's row,
    // and the row group's C lanes are summed ONCE, after the last tile -- no cross-lane
    // reduction per pass and tile (log2 C ds_bpermutes per pass: at c3's 256 x 164,608 round
    // they were 20-30 us of a 117-us launch, scripts/c3_scale_probe.py)
    constexpr bool LD = DEV && C > 1 && KV <= 4;

    float ldev[LD ? KV : 1];
#pragma unroll
    for (int k = 0; k < (LD ? KV : 1); ++k) ldev[k] = 0.f;

    auto prefetch = [&](int tile_id) {
        const int64_t col0 = a.col_base + (int64_t)tile_id * T;
        // (FAST tiles are whole: row-major tails take the guarded launch, and a column-tiled
        // partition round needs n_params % T == 0, checked by the host)
        if (LAG)
            pm = FAST ? *reinterpret_cast<const float4 *>(a.mean_prev + col0 + 4 * c)
                      : ld4(a.mean_prev, col0 + 4 * c, P, false);
        if (FAST && HALO) {
            // local rows from x/g (32-bit offsets), halo rows from the halo buffer (row-major,
            // ldh; or per-peer tiled blocks, hoff/hstr); the per-lane base select keeps every
            // pass straight-line code
            const char *xt = tile_base(a.x, a.xts, tile_id);
            const char *gtb = SGD ? tile_base(a.g, a.gts, tile_id) : nullptr;
            const char *ht = reinterpret_cast<const char *>(a.halo) + (HT ? 0 : col0 * 4);
#pragma unroll
            for (int k = 0; k < KV; ++k) {
                const int r = s + k * SLOTS;
                const bool loc = r < NL;
                const bool ok = r < R;
                const uint32_t oh = HT ? hoff[k] + (uint32_t)(tile_id * grp) * hstr[k]
                                       : (uint32_t)(r - NL) * a.hrs + 16u * c;
                const char *bx = loc || !ok ? xt : ht;
                const uint32_t o1 = loc ? ox + k * sx : ok ? oh : cx;
                const float4 *p1 = reinterpret_cast<const float4 *>(bx + o1);
                px[k] = (a.nt_load & 1) ? nt_load4(p1) : *p1;
                if (SGD) {
                    const float4 *p2 =
                        reinterpret_cast<const float4 *>(gtb + (loc ? og + k * sg : cgx));
                    pg[k] = (a.nt_load & 2) ? nt_load4(p2) : *p2;
                }
            }
        } else if (FAST) {
            const __amdgpu_buffer_rsrc_t rx = buf_rsrc(tile_base(a.x, a.xts, tile_id));
            const __amdgpu_buffer_rsrc_t rg = buf_rsrc(SGD ? tile_base(a.g, a.gts, tile_id)
                                                           : tile_base(a.x, a.xts, tile_id));
            // one straight-line loop per load policy (bit 0: x non-temporal, bit 1: g)
            auto loads = [&](auto ax, auto ag) {
#pragma unroll
                for (int k = 0; k < KV; ++k) {
                    const bool ok = s + k * SLOTS < R;
                    px[k] = buf_ld4<decltype(ax)::value>(rx, ok ? ox + k * sx : cx);
                    if (SGD) pg[k] = buf_ld4<decltype(ag)::value>(rg, ok ? og + k * sg : cgx);
                }
            };
            using NT = std::integral_constant<int, kBufNT>;
            using PL = std::integral_constant<int, 0>;
            if (a.nt_load == 3) loads(NT{}, NT{});
            else if (a.nt_load == 1) loads(NT{}, PL{});
            else if (a.nt_load == 2) loads(PL{}, NT{});
            else loads(PL{}, PL{});
        } else {
            const int64_t cc = col0 + 4 * c;
#pragma unroll
            for (int k = 0; k < KV; ++k) {
                int r = s + k * SLOTS;
                if (r >= R) r = 0;
                const bool local = !HALO || r < NL;
                const float *row = local ? a.x + (int64_t)r * a.ldx
                                         : a.halo + (int64_t)(r - NL) * a.ldh;
                px[k] = ld4(row, cc, P, FAST);
                if (SGD) pg[k] = local ? ld4(a.g + (int64_t)r * a.ldg, cc, P, FAST) : zero4();
            }
        }
    };

    // y_a = sum_e w_e * t_{col_e} for agent ag, chunk c: left fold in CSR order from +0.0
    // (mixer.py:47); reads only LDS.
    const bool wshared = a.n_w != nnz;  // weight of entry e is lw[e - e0]
    // regular rows of 5 entries sharing one weight sequence (a degree-4 graph with uniform
    // weights: c2, c3, c4): the 5 weights in scalar registers from row 0's CSR, the row's 5
    // column ids and then its 5 tile values read back to back -- 6 LDS round trips a row
    // become 2 (the same products and sums in the same order: the same bits)
    const bool reg5 = MIX && RD == 0 && KV <= 4 && reg == 5 && wshared;
    float w5[5];
#pragma unroll
    for (int e = 0; e < 5; ++e) w5[e] = reg5 ? a.w[e] : 0.f;
    auto mix_row = [&](int ag) {
        if (reg5) {
            uint32_t ci[5];
#pragma unroll
            for (int e = 0; e < 5; ++e) ci[e] = lcol[ag * 5 + e];
            float4 v[5];
#pragma unroll
            for (int e = 0; e < 5; ++e) v[e] = tile[ci[e] * C + c];
            float4 acc = zero4();
#pragma unroll
            for (int e = 0; e < 5; ++e) axpy4(acc, w5[e], v[e]);
            return acc;
        }
        int e0, e1;
        if (reg) {
            e0 = ag * reg;
            e1 = e0 + reg;
        } else {
            e0 = lrp[ag];
            e1 = lrp[ag + 1];
        }
        const float *wr = wshared ? lw - e0 : lw;
        float4 acc = zero4();
        for (int e = e0; e < e1; ++e) axpy4(acc, wr[e], tile[lcol[e] * C + c]);
        return acc;
    };

    // the same fold from the register CSR of this thread's pass k: k is a runtime value in the
    // rolled pass loop, so entry e of pass k is picked by a select chain over the KV passes
    // (statically indexed registers, no scratch)
    auto mix_row_reg = [&](int k) {
        float4 acc = zero4();
#pragma unroll
        for (int e = 0; e < (RD > 0 ? RD : 1); ++e) {
            float w = rw[e];
            uint32_t idx = ri[e >> 1] >> (16 * (e & 1));
#pragma unroll
            for (int kk = 1; kk < KV; ++kk) {
                const int j = kk * RD + e;
                w = k == kk ? rw[j] : w;
                idx = k == kk ? ri[j >> 1] >> (16 * (j & 1)) : idx;
            }
            axpy4(acc, w, tile[idx & 0xffffu]);
        }
        if (RAG) {   // the row's entries past the register head, from LDS, in CSR order
            uint32_t d = rdesc[0];
#pragma unroll
            for (int kk = 1; kk < (RAG ? KV : 1); ++kk) d = k == kk ? rdesc[kk] : d;
            // TU entries per step with their reads issued first: a hub row's tail (169
            // entries on the c4-ba graph) is one lane's serial chain, and read-then-fold per
            // entry exposed two dependent LDS latencies each (4.5 ms per round, LDS-bound)
            uint32_t t = d & 0xffffu;
            const uint32_t t1 = t + (d >> 16);
            // (eight per step spill; one at a five-entry head: beside its 30 head registers even
            // two per step spill 84 VGPRs in the local-step + deviation instantiation)
            constexpr int TU = RD >= 5 ? 1 : 4;
            auto tail_w = [&](uint32_t i) {
                if (PACK) return __uint_as_float(ltp[i].x);
                return ltw[i];
            };
            auto tail_c = [&](uint32_t i) -> uint32_t {
                if (PACK) return ltp[i].y;
                return ltc[i];
            };
            // The fold runs on (x, y) / (z, w) pairs (v_pk_mul_f32 / v_pk_add_f32 round every
            // lane as the scalar ops do: same bits): a hub row's chain is one lane's, so its
            // length is the VALU issue of a wave -- four packed ops per entry instead of eight
            // (c4-ba 338 -> 363 rounds/s)
            typedef float f32x2 __attribute__((ext_vector_type(2)));
            f32x2 lo = {acc.x, acc.y}, hi = {acc.z, acc.w};
            auto fold = [&](float w, const float4 &v) {
                if (RD < 5) {   // (at a five-entry head the pairs spill)
                    const f32x2 w2 = {w, w};
                    lo = lo + w2 * f32x2{v.x, v.y};
                    hi = hi + w2 * f32x2{v.z, v.w};
                } else {
                    lo.x = lo.x + w * v.x;
                    lo.y = lo.y + w * v.y;
                    hi.x = hi.x + w * v.z;
                    hi.y = hi.y + w * v.w;
                }
            };
            if constexpr (RD >= 5) {   // the pairs and the unroll spill beside a 5-entry head
                for (; t < t1; ++t) axpy4(acc, tail_w(t), tile[tail_c(t)]);
                return acc;
            }
            auto pairs = [&](uint32_t t0, float (&w4)[TU], uint32_t (&c4)[TU]) {
#pragma unroll
                for (int u = 0; u < TU; ++u) {
                    if (PACK) {
                        const uint2 pr = ltp[t0 + u];
                        w4[u] = __uint_as_float(pr.x);
                        c4[u] = pr.y;
                    } else {
                        w4[u] = ltw[t0 + u];
                        c4[u] = ltc[t0 + u];
                    }
                }
            };
            // (software-pipelining the next step's pair reads over this step's tile reads and
            // folds measured 3 % slower: c4-ba 367 vs 379 rounds/s)
            if constexpr (TU > 1) for (; t + TU <= t1; t += TU) {
                float w4[TU];
                uint32_t c4[TU];
                pairs(t, w4, c4);
                float4 v4[TU];
#pragma unroll
                for (int u = 0; u < TU; ++u) v4[u] = tile[c4[u]];
#pragma unroll
                for (int u = 0; u < TU; ++u) fold(w4[u], v4[u]);
            }
            for (; t < t1; ++t) fold(tail_w(t), tile[tail_c(t)]);
            acc = make_float4(lo.x, lo.y, hi.x, hi.y);
        }
        return acc;
    };

    // hub lane: column hc of row hr, the row's left fold in CSR order (register head's entries
    // from the hub area, then the tail) on scalars -- the same IEEE operations per column as
    // mix_row_reg's float4 / pair fold, so the same bits; eight entries' reads issued per step
    auto hub_fold = [&]() {
        const float *tf = reinterpret_cast<const float *>(tile);
        float acc = 0.f;
#pragma unroll
        for (int e = 0; e < (RD > 0 ? RD : 1); ++e) {
            const uint2 pr = hubp[hr * RD + e];
            acc = acc + __uint_as_float(pr.x) * tf[pr.y * 4u + hc];
        }
        uint32_t t = hdesc & 0xffffu;
        const uint32_t t1 = t + (hdesc >> 16);
        auto entry = [&](uint32_t i, float &w, uint32_t &ci) {
            if (PACK) {
                const uint2 pr = ltp[i];
                w = __uint_as_float(pr.x);
                ci = pr.y;
            } else {
                w = ltw[i];
                ci = ltc[i];
            }
        };
        constexpr int HU = 8;
        for (; t + HU <= t1; t += HU) {
            float w8[HU], v8[HU];
            uint32_t c8[HU];
#pragma unroll
            for (int u = 0; u < HU; ++u) entry(t + u, w8[u], c8[u]);
#pragma unroll
            for (int u = 0; u < HU; ++u) v8[u] = tf[c8[u] * 4u + hc];
#pragma unroll
            for (int u = 0; u < HU; ++u) acc = acc + w8[u] * v8[u];
        }
        for (; t < t1; ++t) {
            float w;
            uint32_t ci;
            entry(t, w, ci);
            acc = acc + w * tf[ci * 4u + hc];
        }
        return acc;
    };
    auto pick = [](const float4 &v, int i) {
        return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
    };
    // hub lanes: a tile's (dx^2 + dy^2) + (dz^2 + dw^2) over the row's four column lanes, the
    // owner's dev_add order, so dev_sq does not depend on n_hub_rows (all four lanes get it)
    auto hub_dev = [&](float d) {
        float v = d * d;
        v = xor_add(v, 1);
        return xor_add(v, 2);
    };

    // column mean of the tile over all agents from per-thread partial sums: thread -> wave
    // (lanes with the same c) -> LDS scratch -> every thread sums the 16 wave partials in order
    // (reading them once per wave and adding across the wave's slot lanes with shuffles instead
    // measured no faster, profiles/r12)
    auto tile_mean = [&](float4 cs) {
#pragma unroll
        for (int m = C; m < 64; m <<= 1) cs = shfl_xor4(cs, m);
        const int wave = tid >> 6, lane = tid & 63;
        if (lane < C) scratch[wave * C + lane] = cs;
        __syncthreads();
        float4 mean = zero4();
#pragma unroll
        for (int wv = 0; wv < NT / 64; ++wv) add4(mean, scratch[wv * C + c]);
        const float n = (float)Nr;
        mean.x = mean.x / n;
        mean.y = mean.y / n;
        mean.z = mean.z / n;
        mean.w = mean.w / n;
        return mean;
    };

    auto dev_add = [&](int k, float4 y, float4 mean) {  // k may be a runtime pass index
        const float dx = y.x - mean.x, dy = y.y - mean.y;
        const float dz = y.z - mean.z, dw = y.w - mean.w;
        float v = (dx * dx + dy * dy) + (dz * dz + dw * dw);
        if constexpr (LD) {   // (k is a runtime pass index: a select per register)
#pragma unroll
            for (int j = 0; j < KV; ++j) ldev[j] += j == k ? v : 0.f;
            return;
        }
#pragma unroll
        for (int m = 1; m < C; m <<= 1) v = xor_add(v, m);  // sum over the row group
        const bool mine = (k % C) == c;
#pragma unroll
        for (int j = 0; j < ND; ++j) dacc[j] += (mine && j == k / C) ? v : 0.f;
    };

    const int trun = a.tile_run;
    int tile_id = trun ? (int)blockIdx.x * trun : (int)blockIdx.x;
    const int tile_end = trun ? min(tile_id + trun, a.n_tiles) : a.n_tiles;
    const int tstep = trun ? 1 : (int)gridDim.x;
    if (tile_id < tile_end) prefetch(tile_id);
    // the LDS CSR is staged after the first tile's loads are issued: its loads (an L2 hit for
    // every workgroup but the first) then wait behind the tile's instead of delaying them, and
    // the first staging barrier below publishes it
    if (RD == 0 && MIX) {
        for (int i = tid; i < a.n_w; i += NT) lw[i] = a.w[i];
        for (int i = tid; i < nnz; i += NT) lcol[i] = (uint16_t)a.col[i];
        if (!a.regular)
            for (int i = tid; i <= Nr; i += NT) lrp[i] = (uint16_t)a.rowptr[i];
    }
    for (; tile_id < tile_end; tile_id += tstep) {
        // opaque per tile: keeps LICM from hoisting one offset register per pass
        asm volatile("" : "+v"(ox), "+v"(og), "+v"(oy));
        const int64_t col0 = a.col_base + (int64_t)tile_id * T;
        const int nxt = tile_id + tstep;
        if (MIX) {
            // stage the (stepped) tile of every source row in LDS
            float4 cst = zero4();  // column partial sums of t (doubly stochastic W only)
#pragma unroll
            for (int k = 0; k < KV; ++k) {
                const int r = s + k * SLOTS;
                float4 t = px[k];
                // lagged deviation of the input, local rows only: this lane's chunk of
                // ||x_r - mean_prev||^2, summed over the row group's lanes once, at the end
                if (LAG && r < NL) {
                    const float dx = t.x - pm.x, dy = t.y - pm.y;
                    const float dz = t.z - pm.z, dw = t.w - pm.w;
                    lacc[k] += (dx * dx + dy * dy) + (dz * dz + dw * dw);
                }
                if (SGD && (!HALO || r < NL)) t = local_step(t, pg[k], a.lr);
                if (r < R) {
                    tile[r * C + c] = t;
                    if (DEV || (LAG && r < NL)) add4(cst, t);
                }
            }
            // mean(W t) = mean(t) when W is doubly stochastic: reduce the column sums of the
            // inputs under the staging barrier instead of re-mixing the tile afterwards.  A halo
            // round (LAG) publishes its local rows' sums of t: all-reduced over the ranks they are
            // the sum of the whole (doubly stochastic) round's output
            const bool mfi = DEV && a.mean_from_inputs;
            constexpr bool lsum = LAG;
            if (mfi || lsum) {
#pragma unroll
                for (int m = C; m < 64; m <<= 1) cst = shfl_xor4(cst, m);
                if ((tid & 63) < C) scratch[(tid >> 6) * C + (tid & 63)] = cst;
            }
            __syncthreads();
            // the next tile's loads go out first: they land while we mix from LDS.  Issued after
            // the staging barrier: issuing it before (right after the staging writes) measured
            // 10 % slower (scripts/grid_sweep.py, profiles/r05/grid_sweep_early_prefetch.log; the
            // register-head + LDS-tail kernel, one workgroup per CU, 10 % slower too: c4-ba 327
            // vs 361 rounds/s).  And ahead of the tile mean's scratch reads (-1 to -5 us on c3's
            // 100-us round, profiles/r12)
            if (nxt < tile_end) prefetch(nxt);
            float4 mean_t = zero4();
            if (mfi || lsum) {
#pragma unroll
                for (int wv = 0; wv < NT / 64; ++wv) add4(mean_t, scratch[wv * C + c]);
                if (lsum && s == 0) st4(a.colsum_out, col0 + 4 * c, P, FAST, mean_t);
                const float n = (float)Nr;
                mean_t.x = mean_t.x / n;
                mean_t.y = mean_t.y / n;
                mean_t.z = mean_t.z / n;
                mean_t.w = mean_t.w / n;
            }
            float *yt = const_cast<float *>(
                reinterpret_cast<const float *>(tile_base(a.y, a.yts, tile_id)));
            float4 cs = zero4();
            float hy = 0.f;   // hub lane: column hc of row hr (plain store: few rows)
            if (RAG && hub_lane) {
                hy = hub_fold();
                *reinterpret_cast<float *>(reinterpret_cast<char *>(yt) + (uint32_t)hr * a.yrs +
                                           4u * (uint32_t)hc) = hy;
                if (DEV) {
                    if (mfi) {
                        hacc += hub_dev(hy - pick(mean_t, hc));
                    } else {
                        cs.x += hc == 0 ? hy : 0.f;
                        cs.y += hc == 1 ? hy : 0.f;
                        cs.z += hc == 2 ? hy : 0.f;
                        cs.w += hc == 3 ? hy : 0.f;
                    }
                }
            }
            const __amdgpu_buffer_rsrc_t ry = buf_rsrc(yt);
            auto store_y = [&](int k, int ag, const float4 &acc) {
                if (FAST) {
                    if (a.nt_store)
                        buf_st4<kBufNT>(acc, ry, oy + (uint32_t)k * sy);
                    else
                        buf_st4<0>(acc, ry, oy + (uint32_t)k * sy);
                } else {
                    st4(a.y + (int64_t)ag * a.ldy, col0 + 4 * c, P, false, acc);
                }
            };
            // passes stay rolled: interleaving them would hold KV accumulators at once on top
            // of the 2*KV prefetch registers (and mixing every pass before reducing the tile
            // mean behind a second barrier measured 4-9 % slower on c2 / c4, profiles/r12)
#pragma unroll 1
            for (int k = 0; k < KV; ++k) {
                const int ag = s + k * SLOTS;
                if (ag < Nr && !(RAG && ag < NH)) {   // (hub rows: folded by their lanes above)
                    const float4 acc = RD > 0 ? mix_row_reg(k) : mix_row(ag);
                    store_y(k, ag, acc);
                    if (DEV) {
                        if (mfi)
                            dev_add(k, acc, mean_t);
                        else
                            add4(cs, acc);
                    }
                }
            }
            if (mfi && a.mean != nullptr && s == 0) st4(a.mean, col0 + 4 * c, P, FAST, mean_t);
            if (DEV && !mfi) {
                const float4 mean = tile_mean(cs);
                if (a.mean != nullptr && s == 0) st4(a.mean, col0 + 4 * c, P, FAST, mean);
                // second LDS pass: recompute y (same order, same bits) instead of holding it
#pragma unroll 1
                for (int k = 0; k < KV; ++k) {
                    const int ag = s + k * SLOTS;
                    if (ag < Nr && !(RAG && ag < NH))
                        dev_add(k, RD > 0 ? mix_row_reg(k) : mix_row(ag), mean);
                }
                if (RAG && hub_lane) hacc += hub_dev(hy - pick(mean, hc));
            }
        } else {
            float4 cur[KV];
            float4 cs = zero4();
#pragma unroll
            for (int k = 0; k < KV; ++k) {
                cur[k] = px[k];
                if (s + k * SLOTS < Nr) add4(cs, cur[k]);
            }
            if (nxt < tile_end) prefetch(nxt);
            const float4 mean = tile_mean(cs);
            if (a.mean != nullptr && s == 0) st4(a.mean, col0 + 4 * c, P, FAST, mean);
#pragma unroll
            for (int k = 0; k < KV; ++k)
                if (s + k * SLOTS < Nr) dev_add(k, cur[k], mean);
        }
        __syncthreads();  // tile and scratch are rewritten by the next iteration
    }
    if (LAG) {
#pragma unroll
        for (int k = 0; k < (LAG ? KV : 1); ++k) {
            float v = lacc[k];
#pragma unroll
            for (int m = 1; m < C; m <<= 1) v = xor_add(v, m);   // over the row group
            const int ag = s + k * SLOTS;   // a local source row
            if (c == 0 && ag < NL) a.dev_partial[(int64_t)blockIdx.x * NL + ag] = v;
        }
        if (a.dev_max_zero != nullptr && blockIdx.x == 0 && tid == 0) *a.dev_max_zero = 0u;
    }
    if (LD) {
#pragma unroll
        for (int k = 0; k < (LD ? KV : 1); ++k) {
            float v = ldev[k];
#pragma unroll
            for (int m = 1; m < C; m <<= 1) v = xor_add(v, m);   // over the row group
            const int ag = s + k * SLOTS;
            if (c == 0 && ag < Nr) a.dev_partial[(int64_t)blockIdx.x * Nr + ag] = v;
        }
        if (a.dev_max_zero != nullptr && blockIdx.x == 0 && tid == 0) *a.dev_max_zero = 0u;
    } else if (DEV) {
#pragma unroll
        for (int j = 0; j < ND; ++j) {
            const int k = j * C + c;  // the pass this lane's slot j holds
            const int ag = s + k * SLOTS;
            if (k < KV && ag < Nr && !(RAG && ag < NH))
                a.dev_partial[(int64_t)blockIdx.x * Nr + ag] = dacc[j];
        }
        if (RAG && NH > 0) {   // hub rows: every lane of the row holds the same sum (hub_dev)
            if (hub_lane && hc == 0) a.dev_partial[(int64_t)blockIdx.x * Nr + hr] = hacc;
        }
        if (a.dev_max_zero != nullptr && blockIdx.x == 0 && tid == 0) *a.dev_max_zero = 0u;
    }
}

// General path (graphs whose tile does not fit LDS): one wave per (agent, 256 columns); the
// agent index is wave-uniform so CSR reads are scalar loads; neighbour rows come from L2/MALL.
// AGENT_FAST: blockIdx.x walks the agent groups of one 256-column chunk before the next chunk
// (grid.x = agent groups), so the chunk of every row -- X and G, 2 KiB per agent -- is read by all
// its neighbours while it is still in L2 / MALL; otherwise blockIdx.x walks the columns of one
// agent group (neighbour rows are re-read from HBM by every agent that gathers them).
template <bool SGD, bool AGENT_FAST>
__global__ void __launch_bounds__(256) mix_gather_kernel(TileArgs a) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int grp = AGENT_FAST ? blockIdx.x : blockIdx.y;
    const int chunk = AGENT_FAST ? blockIdx.y : blockIdx.x;
    const int ag = grp * 4 + wave;
    if (ag >= a.n_rows) return;
    const int64_t P = a.n_params;
    const int64_t c0 = ((int64_t)chunk * 64 + lane) * 4;
    if (c0 >= P) return;
    const bool vec = a.vec != 0;
    const int Nr = a.n_rows;
    const int e0 = a.rowptr[ag], e1 = a.rowptr[ag + 1];
    float4 acc = zero4();
    for (int e = e0; e < e1; ++e) {
        const int n = a.col[e];
        const float wv = a.w[e];
        const float *row = n < Nr ? a.x + (int64_t)n * a.ldx : a.halo + (int64_t)(n - Nr) * a.ldh;
        float4 v = ld4(row, c0, P, vec);
        if (SGD && n < Nr) v = local_step(v, ld4(a.g + (int64_t)n * a.ldg, c0, P, vec), a.lr);
        axpy4(acc, wv, v);
    }
    st4(a.y + (int64_t)ag * a.ldy, c0, P, vec, acc);
}

// dev_sq[a] = sum_b partial[b][a] (fixed order per lane group, fp64), dev_max = max sqrt.
// Block = 64 agents x 16 part-lanes; each lane sums parts j, j+16, ... then LDS combine in a
// fixed order, so the result is deterministic.  dev_max (zeroed by the launcher) takes one
// atomicMax per block on the bits of a non-negative float.
__global__ void __launch_bounds__(1024) dev_reduce_kernel(const float *__restrict__ partial,
                                                          int nparts, int n_rows,
                                                          float *__restrict__ dev_sq,
                                                          unsigned int *__restrict__ dev_max) {
    __shared__ double red[16][64];
    const int ai = threadIdx.x & 63, j = threadIdx.x >> 6;
    const int ag = blockIdx.x * 64 + ai;
    double s = 0.0;
    if (ag < n_rows) {
        // eight partials in flight per lane, added in the same order as one at a time (the sum
        // is bit-identical): a dependent load per add left this launch latency-bound (11.8 us for
        // c2's 512 x 1024 partials, profiles/r08)
        int b = j;
        for (; b + 16 * 7 < nparts; b += 16 * 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = partial[(int64_t)(b + 16 * u) * n_rows + ag];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += (double)v[u];
        }
        for (; b < nparts; b += 16) s += (double)partial[(int64_t)b * n_rows + ag];
    }
    red[j][ai] = s;
    __syncthreads();
    float f = 0.f;
    if (j == 0 && ag < n_rows) {
        double t = red[0][ai];
        for (int k = 1; k < 16; ++k) t += red[k][ai];
        f = (float)t;
        if (dev_sq) dev_sq[ag] = f;
    }
    if (j == 0) {
        float mx = sqrtf(f);
        for (int m = 32; m >= 1; m >>= 1) mx = fmaxf(mx, __shfl_xor(mx, m));
        if (ai == 0 && dev_max) atomicMax(dev_max, __float_as_uint(mx));
    }
}

// Streaming copy (HBM ceiling measurement), float4.  Each workgroup moves 256 x U float4 per
// step with all U loads of a thread in flight before its stores; NT = non-temporal stores.
template <int U, bool NT, bool NTL = false>
__global__ void __launch_bounds__(256) stream_copy_kernel(const float4 *__restrict__ src,
                                                          float4 *__restrict__ dst, int64_t n4) {
    const int64_t step = (int64_t)gridDim.x * 256 * U;
    for (int64_t base = (int64_t)blockIdx.x * 256 * U; base < n4; base += step) {
        float4 v[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t i = base + j * 256 + threadIdx.x;
            if (i < n4) v[j] = NTL ? nt_load4(src + i) : src[i];
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t i = base + j * 256 + threadIdx.x;
            if (i < n4) {
                if (NT)
                    nt_store4(v[j], dst + i);
                else
                    dst[i] = v[j];
            }
        }
    }
}

// Streaming triad y = x - 1e-3 g (HBM ceiling of the 2-read : 1-write round traffic),
// grid-stride, U float4 per stream per thread in flight, non-temporal loads and stores.
template <int U>
__global__ void stream_triad_kernel(const float4 *__restrict__ x, const float4 *__restrict__ g,
                                    float4 *__restrict__ y, int64_t n4) {
    const int64_t step = (int64_t)gridDim.x * blockDim.x * U;
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x * U; base < n4; base += step) {
        float4 a[U], b[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t i = base + j * blockDim.x + threadIdx.x;
            if (i < n4) {
                a[j] = nt_load4(x + i);
                b[j] = nt_load4(g + i);
            }
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int64_t i = base + j * blockDim.x + threadIdx.x;
            if (i < n4) nt_store4(local_step(a[j], b[j], 1e-3f), y + i);
        }
    }
}

// The same triad in the round's own access shape: persistent 1024-thread workgroups on a 2x
// oversubscribed grid, each streaming whole 64-KiB blocks per operand (4 float4 per thread per
// stream), the next block's loads issued before the current block's stores.  Ragged tails are
// not handled: n4 must be a multiple of 4096 (checked by the launcher).
__global__ void __launch_bounds__(1024) stream_triad_tile_kernel(const float4 *__restrict__ x,
                                                                 const float4 *__restrict__ g,
                                                                 float4 *__restrict__ y,
                                                                 int64_t n_blocks) {
    constexpr int R = 4;
    int64_t t = blockIdx.x;
    if (t >= n_blocks) return;
    float4 a[R], b[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        a[r] = nt_load4(x + t * 4096 + r * 1024 + threadIdx.x);
        b[r] = nt_load4(g + t * 4096 + r * 1024 + threadIdx.x);
    }
    for (; t < n_blocks; t += gridDim.x) {
        float4 o[R];
#pragma unroll
        for (int r = 0; r < R; ++r) o[r] = local_step(a[r], b[r], 1e-3f);
        const int64_t tn = t + gridDim.x < n_blocks ? t + gridDim.x : t;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            a[r] = nt_load4(x + tn * 4096 + r * 1024 + threadIdx.x);
            b[r] = nt_load4(g + tn * 4096 + r * 1024 + threadIdx.x);
        }
#pragma unroll
        for (int r = 0; r < R; ++r) nt_store4(o[r], y + t * 4096 + r * 1024 + threadIdx.x);
    }
}

template <int C, int KV, bool SGD, bool DEV, bool MIX, int HALO, bool FAST, int RD = 0,
          bool LAG = false, int RAG = 0>
hipError_t launch_one(const TileArgs &a, int grid, int lds, hipStream_t s) {
    auto k = mix_tile_kernel<C, KV, SGD, DEV, MIX, HALO, FAST, RD, LAG, RAG>;
    hipError_t e = allow_full_lds(reinterpret_cast<const void *>(k));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(grid), dim3(kTileThreads), lds, s, a);
    return hipGetLastError();
}

template <int C, int KV, bool FAST, int H>
hipError_t launch_part(const TileArgs &a, bool sgd, int grid, int lds, hipStream_t s) {
    if (tile_lag(a))   // lagged: previous iterate vs mean_prev, colsum_out for the next
        return sgd ? launch_one<C, KV, true, false, true, H, FAST, 0, true>(a, grid, lds, s)
                   : launch_one<C, KV, false, false, true, H, FAST, 0, true>(a, grid, lds, s);
    return sgd ? launch_one<C, KV, true, false, true, H, FAST>(a, grid, lds, s)
               : launch_one<C, KV, false, false, true, H, FAST>(a, grid, lds, s);
}

template <int C, int KV, bool FAST>
hipError_t launch_mode(const TileArgs &a, bool sgd, bool dev, bool mix, int grid, int lds,
                       hipStream_t s) {
    if (!mix) return launch_one<C, KV, false, true, false, 0, FAST>(a, grid, lds, s);
    if (tile_partitioned(a)) {  // halo rows / a row set: the exact deviation needs the global mean
        if (a.tiled && a.n_src > a.n_loc) {   // column-tiled halo blocks: FAST, KV <= 4 only
            if constexpr (FAST && KV <= 4) return launch_part<C, KV, FAST, 2>(a, sgd, grid, lds, s);
            return hipErrorInvalidValue;
        }
        return launch_part<C, KV, FAST, 1>(a, sgd, grid, lds, s);
    }
    if (sgd) return dev ? launch_one<C, KV, true, true, true, 0, FAST>(a, grid, lds, s)
                        : launch_one<C, KV, true, false, true, 0, FAST>(a, grid, lds, s);
    return dev ? launch_one<C, KV, false, true, true, 0, FAST>(a, grid, lds, s)
               : launch_one<C, KV, false, false, true, 0, FAST>(a, grid, lds, s);
}

// FAST kernels: every C x KV in {2,4,8}; guarded kernels: every C, KV = 8.
template <int C>
hipError_t launch_fast_c(const TileArgs &a, int kv, bool sgd, bool dev, bool mix, int grid,
                         int lds, hipStream_t s) {
    if (kv <= 2) return launch_mode<C, 2, true>(a, sgd, dev, mix, grid, lds, s);
    // a column-tiled halo round of 2..3 row passes (c4 at 8 GPUs: 512 + 96 rows at C = 4; at 2
    // GPUs 2048 + 128 rows at C = 1) runs three passes instead of four: the fourth would only
    // re-read row 0 (45 % of the staging loads dead at 608 rows, 47 % at 2176)
    if (kv == 3 && a.tiled && a.n_src > a.n_loc && C <= 8)
        return launch_part<C, 3, true, 2>(a, sgd, grid, lds, s);
    if (kv <= 4) return launch_mode<C, 4, true>(a, sgd, dev, mix, grid, lds, s);
    return launch_mode<C, 8, true>(a, sgd, dev, mix, grid, lds, s);
}

}  // namespace

int tile_passes(int chunks, int n_src, bool fast) {
    const int slots = kTileThreads / chunks;
    const int need = (n_src + slots - 1) / slots;
    if (!fast) return kRowsPerThread;
    return need <= 2 ? 2 : need <= 4 ? 4 : 8;
}

// Register-CSR tile kernels, FAST path, no halo rows, C = 1 (T = 4 columns), KV in {2, 4} rows
// per thread, i.e. up to 4096 agents.  (C = 2 at KV = 4 spills; at KV = 2 -- 1024 agents -- a
// CSR that fits a 5-entry register head fits LDS too.)
//   head == 0: regular graphs of 5 entries per row, the whole CSR in registers (path 4);
//   head  > 0: rows of >= head entries, the first `head` in registers, the rest in LDS (path 5).
template <int KV, int RD, int RAG>
hipError_t launch_reg_kv(const TileArgs &a, bool sgd, bool dev, int grid, int lds, hipStream_t s) {
    if (sgd)
        return dev ? launch_one<1, KV, true, true, true, 0, true, RD, false, RAG>(a, grid, lds, s)
                   : launch_one<1, KV, true, false, true, 0, true, RD, false, RAG>(a, grid, lds, s);
    return dev ? launch_one<1, KV, false, true, true, 0, true, RD, false, RAG>(a, grid, lds, s)
               : launch_one<1, KV, false, false, true, 0, true, RD, false, RAG>(a, grid, lds, s);
}

template <int RD, int RAG>
hipError_t launch_reg(const TileArgs &a, bool sgd, bool dev, int grid, int lds, hipStream_t s) {
    return tile_passes(1, a.n_src, true) <= 2 ? launch_reg_kv<2, RD, RAG>(a, sgd, dev, grid, lds, s)
                                              : launch_reg_kv<4, RD, RAG>(a, sgd, dev, grid, lds, s);
}

bool reg_csr_supported(int chunks, int n_rows, int regular, int n_halo) {
    return regular == 5 && n_halo == 0 && chunks == 1 && tile_passes(chunks, n_rows, true) <= 4;
}

int reg_head_rows(int min_row_nnz) {
    return min_row_nnz >= 5 ? 5 : min_row_nnz >= 3 ? 3 : min_row_nnz >= 2 ? 2 : 0;
}

bool reg_tail_supported(int chunks, int n_rows, int head, int n_halo) {
    return head > 0 && n_halo == 0 && chunks == 1 && tile_passes(chunks, n_rows, true) <= 4;
}

hipError_t launch_mix_tile_reg(const TileArgs &a, int chunks, int head, int tail_fmt, bool sgd,
                               bool dev, int grid, int lds, hipStream_t s) {
    if (head == 0) {
        if (!reg_csr_supported(chunks, a.n_rows, a.regular, a.n_src - a.n_rows))
            return hipErrorInvalidValue;
        return launch_reg<5, 0>(a, sgd, dev, grid, lds, s);
    }
    if (!reg_tail_supported(chunks, a.n_rows, head, a.n_src - a.n_rows) ||
        a.nnz < head * a.n_rows || (tail_fmt != 1 && tail_fmt != 2) ||
        (head >= 5 && tail_fmt != 1))
        return hipErrorInvalidValue;
    const bool pk = tail_fmt == 2;
    switch (head) {
        case 5: return launch_reg<5, 1>(a, sgd, dev, grid, lds, s);
        case 3: return pk ? launch_reg<3, 2>(a, sgd, dev, grid, lds, s)
                          : launch_reg<3, 1>(a, sgd, dev, grid, lds, s);
        case 2: return pk ? launch_reg<2, 2>(a, sgd, dev, grid, lds, s)
                          : launch_reg<2, 1>(a, sgd, dev, grid, lds, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_mix_tile(const TileArgs &a, int chunks, bool sgd, bool dev, bool mix, int grid,
                           int lds, bool fast, hipStream_t s) {
    if (fast) {
        int kv = tile_passes(chunks, a.n_src, true);
        const int need = (a.n_src + kTileThreads / chunks - 1) / (kTileThreads / chunks);
        if (need == 3 && mix && a.tiled && a.n_src > a.n_loc) kv = 3;   // (launch_fast_c)
        switch (chunks) {
            case 1: return launch_fast_c<1>(a, kv, sgd, dev, mix, grid, lds, s);
            case 2: return launch_fast_c<2>(a, kv, sgd, dev, mix, grid, lds, s);
            case 4: return launch_fast_c<4>(a, kv, sgd, dev, mix, grid, lds, s);
            case 8: return launch_fast_c<8>(a, kv, sgd, dev, mix, grid, lds, s);
            case 16: return launch_fast_c<16>(a, kv, sgd, dev, mix, grid, lds, s);
            case 32: return launch_fast_c<32>(a, kv, sgd, dev, mix, grid, lds, s);
            default: return hipErrorInvalidValue;
        }
    }
    switch (chunks) {
        case 1: return launch_mode<1, 8, false>(a, sgd, dev, mix, grid, lds, s);
        case 2: return launch_mode<2, 8, false>(a, sgd, dev, mix, grid, lds, s);
        case 4: return launch_mode<4, 8, false>(a, sgd, dev, mix, grid, lds, s);
        case 8: return launch_mode<8, 8, false>(a, sgd, dev, mix, grid, lds, s);
        case 16: return launch_mode<16, 8, false>(a, sgd, dev, mix, grid, lds, s);
        case 32: return launch_mode<32, 8, false>(a, sgd, dev, mix, grid, lds, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t allow_full_lds(const void *k) {
    static std::mutex mu;
    static std::set<std::pair<const void *, int>> done;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(mu);
    if (done.count({k, dev})) return hipSuccess;
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes);
    if (e == hipSuccess) done.insert({k, dev});
    return e;
}

uint32_t csr_lds_bytes(int32_t n_rows, int32_t nnz, int32_t regular, int32_t n_w) {
    if (nnz > 65535 || n_rows > 65535) return 0;
    uint32_t b = 4u * (uint32_t)n_w + 2u * (uint32_t)nnz;
    if (!regular) b += 2u * (uint32_t)(n_rows + 1);
    return (b + 15u) & ~15u;
}

hipError_t launch_mix_gather(const TileArgs &a, bool sgd, hipStream_t s) {
    const unsigned chunks = (unsigned)((a.n_params + 255) / 256);
    const unsigned groups = (unsigned)((a.n_rows + 3) / 4);
    // DLAMD_GATHER_ORDER=columns keeps the column-fastest order (measurement knob)
    const char *o = getenv("DLAMD_GATHER_ORDER");
    const bool agent_fast = !(o && o[0] == 'c') && chunks <= 65535;
    if (agent_fast) {
        dim3 grid(groups, chunks);
        if (sgd)
            hipLaunchKernelGGL((mix_gather_kernel<true, true>), grid, dim3(256), 0, s, a);
        else
            hipLaunchKernelGGL((mix_gather_kernel<false, true>), grid, dim3(256), 0, s, a);
    } else {
        dim3 grid(chunks, groups);
        if (sgd)
            hipLaunchKernelGGL((mix_gather_kernel<true, false>), grid, dim3(256), 0, s, a);
        else
            hipLaunchKernelGGL((mix_gather_kernel<false, false>), grid, dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_dev_reduce(const float *partial, int nparts, int n_rows, float *dev_sq,
                             float *dev_max, hipStream_t s, bool max_zeroed) {
    if (dev_max && !max_zeroed) {
        hipError_t e = hipMemsetAsync(dev_max, 0, sizeof(float), s);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(dev_reduce_kernel, dim3((n_rows + 63) / 64), dim3(1024), 0, s, partial,
                       nparts, n_rows, dev_sq, reinterpret_cast<unsigned int *>(dev_max));
    return hipGetLastError();
}

hipError_t launch_stream_copy(const float *src, float *dst, int64_t n_floats, int variant,
                              hipStream_t s) {
    const int64_t n4 = n_floats / 4;
    if (variant >= 4) {
        auto x = reinterpret_cast<const float4 *>(src);
        auto y = reinterpret_cast<float4 *>(dst);
        if (variant == 6) {
            if (n4 % 4096) return hipErrorInvalidValue;
            const int64_t nb = n4 / 4096;
            int dev = 0, cus = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
                cus <= 0)
                cus = 256;
            int64_t grid = 2 * (int64_t)cus;
            if (grid > nb) grid = nb;
            if (grid < 1) return hipSuccess;
            hipLaunchKernelGGL(stream_triad_tile_kernel, dim3((unsigned)grid), dim3(1024), 0, s, x,
                               x + n4, y, nb);
        } else if (variant == 4)
            hipLaunchKernelGGL(stream_triad_kernel<1>, dim3(256), dim3(512), 0, s, x, x + n4, y, n4);
        else
            hipLaunchKernelGGL(stream_triad_kernel<4>, dim3(1024), dim3(256), 0, s, x, x + n4, y, n4);
        return hipGetLastError();
    }
    const int U = variant == 0 ? 1 : variant == 3 ? 4 : 8;
    int64_t grid = (n4 + 256 * U - 1) / (256 * U);
    const int64_t gmax = variant == 0 ? 256 * 8 : variant == 3 ? 256 * 32 : 256 * 4;
    if (grid > gmax) grid = gmax;
    if (grid < 1) grid = 1;
    auto f4s = reinterpret_cast<const float4 *>(src);
    auto f4d = reinterpret_cast<float4 *>(dst);
    switch (variant) {
        case 0: hipLaunchKernelGGL((stream_copy_kernel<1, false>), dim3((unsigned)grid), dim3(256), 0, s, f4s, f4d, n4); break;
        case 1: hipLaunchKernelGGL((stream_copy_kernel<8, false>), dim3((unsigned)grid), dim3(256), 0, s, f4s, f4d, n4); break;
        case 2: hipLaunchKernelGGL((stream_copy_kernel<8, true>), dim3((unsigned)grid), dim3(256), 0, s, f4s, f4d, n4); break;
        default: hipLaunchKernelGGL((stream_copy_kernel<4, true, true>), dim3((unsigned)grid), dim3(256), 0, s, f4s, f4d, n4); break;
    }
    return hipGetLastError();
}

}  // namespace dl
