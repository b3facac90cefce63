// Multi-round gossip mixing in one HBM pass (gfx950): Y = W^K (X - lr G) for K >= 1 rounds.
//
// `Mixer.mix(times=K)` (utils/consensus_simple/mixer.py:18-38, eps=None) runs K consecutive
// rounds of `_mix_params_once` (:43-49) with nothing in between, and pure gossip averaging (the
// BASELINE c2 config) is exactly that.  The mix is column-independent: column p of X' depends
// only on column p of X.  So a workgroup that holds a column tile of ALL agents in LDS can run
// every one of the K rounds on it before writing it back: HBM sees each element of X (and G) read
// once and Y written once per K rounds instead of per round, and the rounds run at LDS speed.
// Two tile images ping-pong in LDS (round r reads one, writes the other, one barrier per round);
// the last round writes HBM directly from registers (non-temporal) and, for doubly stochastic W,
// accumulates the final deviation against the column mean of the staged tile (mean(W t) =
// mean(t)).  Every round folds in CSR order with separate fp32 products and sums
// (-ffp-contract=off), so K rounds here are bit-identical to K launches of the one-round kernel
// and to K calls of the reference's fold.  The next tile's X (and G) rows are prefetched into
// registers while the current tile's rounds run.
#include "dl_internal.h"

#include <type_traits>

namespace dl {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 mm_zero4() { return make_float4(0.f, 0.f, 0.f, 0.f); }

__device__ __forceinline__ float4 mm_nt_load4(const float4 *p) {
    const f32x4 x = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(p));
    return make_float4(x.x, x.y, x.z, x.w);
}

__device__ __forceinline__ void mm_nt_store4(float4 v, float4 *p) {
    f32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f32x4 *>(p));
}

__device__ __forceinline__ const float4 *mm_at(const void *base, uint32_t off) {
    return reinterpret_cast<const float4 *>(reinterpret_cast<const char *>(base) + off);
}

// C: float4 chunks per tile row (T = 4C columns); KV: rows per thread (agents s + k*SLOTS);
// SGD: local step x - lr g applied once, before the first round; DEV: final deviation.
// RE > 0: regular graph with RE entries per row whose weights every row shares (best-constant /
// analytic FA weights): each thread keeps its rows' neighbour byte offsets and the RE weights in
// registers for the whole launch, so a round issues only the RE neighbour reads and one write
// per output chunk (no CSR reads from LDS).  RE = 0: CSR from LDS.
// FAST tiles only (every tile full and 16-byte aligned; the column-tiled layout always is).
// MODE 1 / 2: N == KV * SLOTS (every slot an agent): the image fill and the output stores carry
// no ragged guard and the store kind is fixed (1 plain, 2 non-temporal).  With guarded stores or
// a run-time store-kind branch, the compiler's wait-count tracking could not count the stores
// issued after the prefetch and waited for the previous tile's stores to drain (vmcnt(0))
// before the image fill of every tile.  MODE 0: guarded, store kind from a.nt_store.
template <int C, int KV, bool SGD, bool DEV, int RE, int MODE>
__global__ void __launch_bounds__(kTileThreads) mix_multi_kernel(TileArgs a, int rounds) {
    constexpr bool FULL = MODE > 0;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int NT = kTileThreads;
    constexpr int SLOTS = NT / C;
    const int tid = threadIdx.x;
    const int c = tid & (C - 1);
    const int s = tid / C;
    const int Nr = a.n_rows;
    const int nnz = a.nnz;
    float4 *img0 = reinterpret_cast<float4 *>(smem);
    float4 *img1 = img0 + (size_t)Nr * C;
    float *lw = reinterpret_cast<float *>(smem + a.csr_off);
    uint16_t *lcol = reinterpret_cast<uint16_t *>(smem + a.csr_off + 4u * (uint32_t)a.n_w);
    uint16_t *lrp = lcol + nnz;
    float4 *scratch = reinterpret_cast<float4 *>(smem + a.scratch_off);
    const int reg = a.regular;
    if constexpr (RE == 0) {   // RE > 0 keeps its CSR in registers: nothing staged in LDS
        for (int i = tid; i < a.n_w; i += NT) lw[i] = a.w[i];
        for (int i = tid; i < nnz; i += NT) lcol[i] = (uint16_t)a.col[i];
        if (!reg)
            for (int i = tid; i <= Nr; i += NT) lrp[i] = (uint16_t)a.rowptr[i];
    }
    const bool wshared = a.n_w != nnz;

    uint32_t ox = (uint32_t)s * a.xrs + 16u * c;
    const uint32_t sx = (uint32_t)SLOTS * a.xrs;
    uint32_t og = SGD ? (uint32_t)s * a.grs + 16u * c : 0u;
    const uint32_t sg = SGD ? (uint32_t)SLOTS * a.grs : 0u;
    uint32_t oy = (uint32_t)s * a.yrs + 16u * c;
    const uint32_t sy = (uint32_t)SLOTS * a.yrs;
    auto tile_base = [&](const void *p, int64_t ts, int tile_id) {
        return reinterpret_cast<const char *>(p) + (a.tiled ? 0 : a.col_base * 4) +
               (int64_t)tile_id * ts;
    };

    float4 px[KV], pg[KV];
    auto prefetch = [&](int tile_id) {
        const char *xt = tile_base(a.x, a.xts, tile_id);
        const char *gt = SGD ? tile_base(a.g, a.gts, tile_id) : nullptr;
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const bool ok = FULL || s + k * SLOTS < Nr;   // ragged: re-read row 0 (L1 hit)
            px[k] = mm_nt_load4(mm_at(xt, ok ? ox + k * sx : 16u * c));
            if (SGD) pg[k] = mm_nt_load4(mm_at(gt, ok ? og + k * sg : 16u * c));
        }
    };

    // one agent's output chunk from an LDS image: left fold in CSR order from +0.0 (mixer.py:47)
    auto mix_row = [&](const float4 *src, int ag) {
        int e0, e1;
        if (reg) {
            e0 = ag * reg;
            e1 = e0 + reg;
        } else {
            e0 = lrp[ag];
            e1 = lrp[ag + 1];
        }
        const float *wr = wshared ? lw - e0 : lw;
        float4 acc = mm_zero4();
        for (int e = e0; e < e1; ++e) {
            const float w = wr[e];
            const float4 v = src[lcol[e] * C + c];
            acc.x = acc.x + w * v.x;
            acc.y = acc.y + w * v.y;
            acc.z = acc.z + w * v.z;
            acc.w = acc.w + w * v.w;
        }
        return acc;
    };

    // register-cached CSR (RE > 0): byte offset of each neighbour's chunk c inside an image
    uint32_t coff[KV][RE > 0 ? RE : 1];
    float wreg[RE > 0 ? RE : 1];
    bool self_ok = true;   // every row of this thread lists itself first (the diagonal of W)
    if constexpr (RE > 0) {
#pragma unroll
        for (int e = 0; e < RE; ++e) wreg[e] = a.w[e];
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const int ag = FULL || s + k * SLOTS < Nr ? s + k * SLOTS : 0;
            self_ok = self_ok && a.col[ag * RE] == ag;
#pragma unroll
            for (int e = 0; e < RE; ++e)
                coff[k][e] = ((uint32_t)a.col[ag * RE + e] * C + c) * 16u;
        }
    }
    // Every row's first entry its own agent (W = I - L(w) with the diagonal first,
    // graph.from_edge_weights: c2, c4): that operand is the value this very thread produced for
    // the row in the previous round (or staged), so it is kept in a register (own[k]) and the
    // round reads 4 neighbours from LDS instead of 5 -- same operand, same fold, same bits.
    // Decided per wave (a wave vote, no LDS: a uniform branch, so the skipped read is not
    // issued; __syncthreads_and would add static LDS beside the full dynamic allocation).
    const bool self0 = RE > 0 && __all(self_ok ? 1 : 0) != 0;
    float4 own[RE > 0 ? KV : 1];
#pragma unroll
    for (int k = 0; k < (RE > 0 ? KV : 1); ++k) own[k] = mm_zero4();
    auto mix_row_reg = [&](const float4 *src, int k, auto selfc) {
        constexpr bool SELF = decltype(selfc)::value;
        const char *base = reinterpret_cast<const char *>(src);
        float4 acc = mm_zero4();
#pragma unroll
        for (int e = 0; e < (RE > 0 ? RE : 1); ++e) {
            float4 v;
            if (SELF && e == 0)
                v = own[k];
            else
                v = *reinterpret_cast<const float4 *>(base + coff[k][e]);
            const float w = wreg[e];
            acc.x = acc.x + w * v.x;
            acc.y = acc.y + w * v.y;
            acc.z = acc.z + w * v.z;
            acc.w = acc.w + w * v.w;
        }
        return acc;
    };
    auto out_row = [&](const float4 *src, int k, int ag, auto selfc) {
        if constexpr (RE > 0) return mix_row_reg(src, k, selfc);
        return mix_row(src, ag);
    };

    constexpr int ND = KV <= C ? 1 : KV / C;
    float dacc[ND];
#pragma unroll
    for (int k = 0; k < ND; ++k) dacc[k] = 0.f;

    // The tile loop is rotated: stage (image fill + column mean) of the next tile runs after
    // this tile's output stores, and its prefetch is issued right after, so every path into
    // the fill has the same loads-then-stores order and the fill waits only for the loads
    // (vmcnt(4..7) rather than vmcnt(0), which also drained the previous tile's stores).
    int tile_id = blockIdx.x;
    float4 mean = mm_zero4();
    auto stage = [&]() {
        float4 cst = mm_zero4();
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const int r = s + k * SLOTS;
            float4 t = px[k];
            if (SGD) {
                t.x = t.x - a.lr * pg[k].x;
                t.y = t.y - a.lr * pg[k].y;
                t.z = t.z - a.lr * pg[k].z;
                t.w = t.w - a.lr * pg[k].w;
            }
            if (RE > 0) own[k] = t;
            if (FULL || r < Nr) {
                img0[r * C + c] = t;
                if (DEV) {
                    cst.x += t.x;
                    cst.y += t.y;
                    cst.z += t.z;
                    cst.w += t.w;
                }
            }
        }
        if (DEV) {   // column sums of the staged tile (W doubly stochastic: the final mean)
#pragma unroll
            for (int m = C; m < 64; m <<= 1) {
                cst.x += __shfl_xor(cst.x, m);
                cst.y += __shfl_xor(cst.y, m);
                cst.z += __shfl_xor(cst.z, m);
                cst.w += __shfl_xor(cst.w, m);
            }
            if ((tid & 63) < C) scratch[(tid >> 6) * C + (tid & 63)] = cst;
        }
        __syncthreads();
        mean = mm_zero4();
        if (DEV) {
#pragma unroll 2   // (fully unrolled, the 16 reads are hoisted: 64 VGPRs at once, spills)
            for (int wv = 0; wv < NT / 64; ++wv) {
                const float4 q = scratch[wv * C + c];
                mean.x += q.x;
                mean.y += q.y;
                mean.z += q.z;
                mean.w += q.w;
            }
            const float n = (float)Nr;
            mean.x = mean.x / n;
            mean.y = mean.y / n;
            mean.z = mean.z / n;
            mean.w = mean.w / n;
        }
    };
    // prefetches past the last tile re-read the last tile instead (unconditional loads keep the
    // count exact; 64 KB per workgroup per pass)
    const int last = a.n_tiles - 1;
    if (tile_id < a.n_tiles) {
        prefetch(tile_id);
        stage();
        prefetch(min(tile_id + (int)gridDim.x, last));
    }
    // the tile loop twice, with and without the own-operand register (self0 is wave-uniform:
    // one branch here, none inside the rounds)
    auto tiles = [&](auto selfc) {
    for (; tile_id < a.n_tiles; tile_id += gridDim.x) {
        asm volatile("" : "+v"(ox), "+v"(og), "+v"(oy));
        const int nxt = min(tile_id + (int)gridDim.x, last);
        const float4 *src = img0;
        float4 *dst = img1;
        for (int r = 0; r + 1 < rounds; ++r) {
#pragma unroll
            for (int k = 0; k < KV; ++k) {
                const int ag = s + k * SLOTS;
                if (FULL || ag < Nr) {
                    const float4 o = out_row(src, k, ag, selfc);
                    dst[ag * C + c] = o;
                    if (RE > 0) own[k] = o;
                }
                // one output row at a time: keeps the RE neighbour reads of the next row from
                // being hoisted above this one's (register pressure at 1024 threads)
                __builtin_amdgcn_sched_barrier(0);
            }
            __syncthreads();
            const float4 *t = src;
            src = dst;
            dst = const_cast<float4 *>(t);
        }
        const char *yt = tile_base(a.y, a.yts, tile_id);
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const int ag = s + k * SLOTS;
            if (FULL || ag < Nr) {
                const float4 y = out_row(src, k, ag, selfc);
                float4 *py = const_cast<float4 *>(mm_at(yt, oy + (uint32_t)k * sy));
                if (MODE == 2 || (MODE == 0 && a.nt_store))
                    mm_nt_store4(y, py);
                else
                    *py = y;
                if (DEV) {
                    const float dx = y.x - mean.x, dy = y.y - mean.y;
                    const float dz = y.z - mean.z, dw = y.w - mean.w;
                    float v = (dx * dx + dy * dy) + (dz * dz + dw * dw);
#pragma unroll
                    for (int m = 1; m < C; m <<= 1) v += __shfl_xor(v, m);
                    const bool mine = (k % C) == c;
#pragma unroll
                    for (int j = 0; j < ND; ++j) dacc[j] += (mine && j == k / C) ? v : 0.f;
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (DEV && a.mean != nullptr && s == 0) {
            const int64_t col0 = a.col_base + (int64_t)tile_id * 4 * C + 4 * c;
            *reinterpret_cast<float4 *>(a.mean + col0) = mean;
        }
        __syncthreads();   // both images and the scratch are rewritten by the next tile
        stage();   // the next tile (past the end: a re-read of the last one, then unused)
        prefetch(min(nxt + (int)gridDim.x, last));   // lands while the next tile's rounds run
    }
    };
    // (pure gossip only, and not at C = 2 x KV = 4 with the deviation: beside those registers
    // the second copy spills)
    if constexpr (RE > 0 && !SGD && !(C == 2 && KV == 4 && DEV)) {
        if (self0)
            tiles(std::true_type{});
        else
            tiles(std::false_type{});
    } else {
        tiles(std::false_type{});
    }
    if (DEV) {
#pragma unroll
        for (int j = 0; j < ND; ++j) {
            const int k = j * C + c;
            const int ag = s + k * SLOTS;
            if (k < KV && ag < Nr) a.dev_partial[(int64_t)blockIdx.x * Nr + ag] = dacc[j];
        }
        if (a.dev_max_zero != nullptr && blockIdx.x == 0 && tid == 0) *a.dev_max_zero = 0u;
    }
}

template <int C, int KV, bool SGD, bool DEV, int RE, int MODE>
hipError_t launch_mode(const TileArgs &a, int rounds, int grid, int lds, hipStream_t s) {
    const void *k = reinterpret_cast<const void *>(mix_multi_kernel<C, KV, SGD, DEV, RE, MODE>);
    hipError_t e = allow_full_lds(k);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((mix_multi_kernel<C, KV, SGD, DEV, RE, MODE>), dim3(grid),
                       dim3(kTileThreads), lds, s, a, rounds);
    return hipGetLastError();
}

template <int C, int KV, bool SGD, bool DEV, int RE>
hipError_t launch_one(const TileArgs &a, int rounds, int grid, int lds, hipStream_t s) {
    // the unguarded variant for the register-CSR graphs whose N fills every slot (c2, c4)
    if (RE > 0 && a.n_rows == KV * (kTileThreads / C))
        return a.nt_store ? launch_mode<C, KV, SGD, DEV, RE, RE ? 2 : 0>(a, rounds, grid, lds, s)
                          : launch_mode<C, KV, SGD, DEV, RE, RE ? 1 : 0>(a, rounds, grid, lds, s);
    return launch_mode<C, KV, SGD, DEV, RE, 0>(a, rounds, grid, lds, s);
}

template <int C, int KV, int RE>
hipError_t launch_re(const TileArgs &a, int rounds, bool sgd, bool dev, int grid, int lds,
                     hipStream_t s) {
    if (sgd)
        return dev ? launch_one<C, KV, true, true, RE>(a, rounds, grid, lds, s)
                   : launch_one<C, KV, true, false, RE>(a, rounds, grid, lds, s);
    return dev ? launch_one<C, KV, false, true, RE>(a, rounds, grid, lds, s)
               : launch_one<C, KV, false, false, RE>(a, rounds, grid, lds, s);
}

template <int C, int KV>
hipError_t launch_kv(const TileArgs &a, int rounds, bool sgd, bool dev, int grid, int lds,
                     hipStream_t s) {
    // register-cached CSR for the degree-4 regular graphs with shared weights (c2, c4 shapes);
    // the same test as csr_in_registers() on the host, which then reserves no LDS for the CSR
    if constexpr (KV <= 4) {
        if (a.regular == 5 && a.n_w == 5)
            return launch_re<C, KV, 5>(a, rounds, sgd, dev, grid, lds, s);
    }
    return launch_re<C, KV, 0>(a, rounds, sgd, dev, grid, lds, s);
}

template <int C>
hipError_t launch_c(const TileArgs &a, int rounds, bool sgd, bool dev, int grid, int lds,
                    hipStream_t s) {
    const int kv = tile_passes(C, a.n_rows, true);
    if (kv <= 2) return launch_kv<C, 2>(a, rounds, sgd, dev, grid, lds, s);
    if (kv <= 4) return launch_kv<C, 4>(a, rounds, sgd, dev, grid, lds, s);
    return launch_kv<C, 8>(a, rounds, sgd, dev, grid, lds, s);
}

}  // namespace

hipError_t launch_mix_multi(const TileArgs &a, int chunks, int rounds, bool sgd, bool dev,
                            int grid, int lds, hipStream_t s) {
    switch (chunks) {
        case 1: return launch_c<1>(a, rounds, sgd, dev, grid, lds, s);
        case 2: return launch_c<2>(a, rounds, sgd, dev, grid, lds, s);
        case 4: return launch_c<4>(a, rounds, sgd, dev, grid, lds, s);
        case 8: return launch_c<8>(a, rounds, sgd, dev, grid, lds, s);
        case 16: return launch_c<16>(a, rounds, sgd, dev, grid, lds, s);
        case 32: return launch_c<32>(a, rounds, sgd, dev, grid, lds, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace dl
