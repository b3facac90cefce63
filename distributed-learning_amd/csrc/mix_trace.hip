// K gossip rounds in one HBM pass WITH the per-round disagreement trace (gfx950):
// `Mixer.mix(times, eps)` (utils/consensus_simple/mixer.py:18-41) with eps set evaluates
// max_a ||x_a - mean(X)|| (:51-66) after every round and stops at the first round r >= times
// whose value is below eps.  mix_multi_kernel already runs K rounds on LDS-resident column tiles
// (mixing is column-independent); the stop test is what kept eps-loops on one HBM-bound launch
// per round.  Here every workgroup also accumulates, for each of the K rounds, every agent's
// squared deviation over its own columns; one reduce launch turns the per-workgroup traces
// [grid][K][N] into the K per-round max deviations.  The host then finds the stop round
// and, if it lies inside the pass, re-runs that many rounds from the pass's input (still intact:
// X -> Y).  The rounds are the same CSR-order fp32 fold as the one-round kernel, so the iterates
// are bit-identical to round-by-round mixing.
//
// Geometry: one agent per thread (N <= 1024), C float4 column chunks per step (the widest of
// 4, 2, 1 whose two images fit LDS), the per-round squared deviations in registers, so nothing
// is shuffled or atomically added per round.  LDS: two images 2 x N x C x 16 B, the CSR (unless
// register-cached), a 16 x C float4 mean scratch.  W must be doubly stochastic: the column mean of every
// round equals the mean of the pass's input chunk (mean(W t) = mean(t)), as in the fused
// one-round deviation.
#include "dl_internal.h"

#include <cstdlib>
#include <type_traits>

namespace dl {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// (lo, hi) += w * v on v's (x, y) / (z, w) halves: each v_pk_mul_f32 / v_pk_add_f32 rounds every
// lane as the scalar ops do, so the fold's bits are those of acc.x = acc.x + w * v.x, ... .  The
// pairs are the halves of the ds_read_b128 registers.  (Written per component, the deviation's
// sums let the vectorizer pair (x, z) / (y, w): three moves per neighbour, and each LDS read
// waited for before the next was issued -- the rows kernel ran 1978 instead of 2520 rounds/s.)
__device__ __forceinline__ void fold2(f32x2 &lo, f32x2 &hi, float w, const f32x4 &v) {
    const f32x2 w2 = {w, w};
    lo = lo + w2 * __builtin_shufflevector(v, v, 0, 1);
    hi = hi + w2 * __builtin_shufflevector(v, v, 2, 3);
}

// ||(lo, hi) - (mlo, mhi)||^2 summed as (dx^2 + dy^2) + (dz^2 + dw^2)
__device__ __forceinline__ float dev2(const f32x2 &lo, const f32x2 &hi, const f32x2 &mlo,
                                      const f32x2 &mhi) {
    const f32x2 dl = lo - mlo, dh = hi - mhi;
    const f32x2 ql = dl * dl, qh = dh * dh;
    return (ql.x + ql.y) + (qh.x + qh.y);
}

__device__ __forceinline__ float4 tr_load4(const char *p) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}

// Plain (write-back) stores: a lane writes its agent's C chunks with C instructions, each one
// 16 B per lane at the agent stride, so every instruction covers only part of each line.
// Through L2 the C partial writes of a line merge before it is written back; non-temporal
// stores sent them to HBM as partial-line writes (WRITE_SIZE 2.8x the bytes, profiles/r05/trace).
__device__ __forceinline__ void tr_store4(float4 v, char *p) {
    *reinterpret_cast<float4 *>(p) = v;
}

// Lane exchange inside a quad as a DPP modifier on a VALU move (quad_perm [1,0,3,2] /
// [2,3,0,1]): __shfl_xor compiles to ds_bpermute_b32, an LDS instruction, and the traced rows
// kernel would issue 8 of them per thread per round next to its 24 image accesses.
__device__ __forceinline__ float quad_xor1(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}
__device__ __forceinline__ float quad_xor2(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
}

// RE > 0: regular graph of RE entries per row sharing row 0's weights, CSR in registers.
// C: float4 column chunks per agent per step (T = 4C columns): a round does C outputs per thread
// between barriers.  The per-round deviations live in registers (dacc[r], the round loop
// unrolled up to kTraceRounds; 118 VGPRs at C = 4, no spills).  Measured against an LDS trace
// [rounds][N] (rolled loop, which leaves room for two images only at C <= 2 for 1024 agents):
// 1218 rounds/s at C = 2 vs 1589 at C = 4 here (c2 sizes, profiles/r05/trace_bench.log).
template <int RE, int C>
__global__ void __launch_bounds__(kTileThreads) mix_trace_kernel(TileArgs a, int rounds) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int KR = kTraceRounds;
    const int tid = threadIdx.x;
    const int N = a.n_rows;
    const bool mine = tid < N;
    // images chunk-major [C][N]: lanes (consecutive agents) reading random neighbours of one
    // chunk plane hit 16-byte slots spread over all banks; agent-major [N][C] rows (64 B at C = 4)
    // put every neighbour of a chunk on the same quarter of the banks (890 vs 1589 rounds/s at c2)
    float4 *img0 = reinterpret_cast<float4 *>(smem);
    float4 *img1 = img0 + N * C;
    float4 *scratch = reinterpret_cast<float4 *>(smem + a.scratch_off);   // [16][C]
    float *lw = reinterpret_cast<float *>(smem + a.csr_off);
    uint16_t *lcol = reinterpret_cast<uint16_t *>(smem + a.csr_off + 4u * (uint32_t)a.n_w);
    uint16_t *lrp = lcol + a.nnz;
    const int reg = a.regular;
    const bool wshared = a.n_w != a.nnz;

    if constexpr (RE == 0) {
        for (int i = tid; i < a.n_w; i += kTileThreads) lw[i] = a.w[i];
        for (int i = tid; i < a.nnz; i += kTileThreads) lcol[i] = (uint16_t)a.col[i];
        if (!reg)
            for (int i = tid; i <= N; i += kTileThreads) lrp[i] = (uint16_t)a.rowptr[i];
    }
    uint32_t coff[RE > 0 ? RE : 1];
    float wreg[RE > 0 ? RE : 1];
    if constexpr (RE > 0) {
        const int ag = mine ? tid : 0;
#pragma unroll
        for (int e = 0; e < RE; ++e) {
            coff[e] = (uint32_t)a.col[ag * RE + e] * 16u;
            wreg[e] = a.w[e];
        }
    }
    // agent tid's output chunk c: left fold in CSR order from +0.0 (mixer.py:47), as pairs
    auto mix = [&](const float4 *src, int c, f32x2 &lo, f32x2 &hi) {
        lo = f32x2{0.f, 0.f};
        hi = f32x2{0.f, 0.f};
        if constexpr (RE > 0) {
            const char *base = reinterpret_cast<const char *>(src + c * N);
            f32x4 v[RE];
#pragma unroll
            for (int e = 0; e < RE; ++e) v[e] = *reinterpret_cast<const f32x4 *>(base + coff[e]);
#pragma unroll
            for (int e = 0; e < RE; ++e) fold2(lo, hi, wreg[e], v[e]);
        } else {
            int e0, e1;
            if (reg) {
                e0 = tid * reg;
                e1 = e0 + reg;
            } else {
                e0 = lrp[tid];
                e1 = lrp[tid + 1];
            }
            const float *wr = wshared ? lw - e0 : lw;
            const f32x4 *sv = reinterpret_cast<const f32x4 *>(src + c * N);
            for (int e = e0; e < e1; ++e) fold2(lo, hi, wr[e], sv[lcol[e]]);
        }
    };
    // byte offset of (agent tid, chunk q) in an operand laid out in lc-chunk tiles (lc a power
    // of two; the step index is wave-uniform, so the tile part is scalar arithmetic)
    const int lsh = __builtin_ctz((unsigned)a.lchunks);
    const int64_t lmask = (int64_t)a.lchunks - 1;
    const int64_t xrow = (int64_t)tid * a.xrs, yrow = (int64_t)tid * a.yrs;
    auto off = [&](int64_t ts, int64_t row, int64_t q) {
        return (q >> lsh) * ts + row + (q & lmask) * 16;
    };
    const char *xb = reinterpret_cast<const char *>(a.x);
    char *yb = reinterpret_cast<char *>(a.y);
    const int64_t nsteps = a.n_tiles;   // steps of C float4 column chunks
    float dacc[KR];   // this agent's squared deviation after each round (registers)
#pragma unroll
    for (int r = 0; r < KR; ++r) dacc[r] = 0.f;
    float4 px[C];
#pragma unroll
    for (int c = 0; c < C; ++c) px[c] = make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t q = blockIdx.x;
    if (q < nsteps && mine) {
#pragma unroll
        for (int c = 0; c < C; ++c) px[c] = tr_load4(xb + off(a.xts, xrow, q * C + c));
    }
    __syncthreads();   // CSR staged
    for (; q < nsteps; q += gridDim.x) {
#pragma unroll
        for (int c = 0; c < C; ++c) {
            if (mine) img0[c * N + tid] = px[c];
            float4 cs = mine ? px[c] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int m = 1; m < 64; m <<= 1) {
                cs.x += __shfl_xor(cs.x, m);
                cs.y += __shfl_xor(cs.y, m);
                cs.z += __shfl_xor(cs.z, m);
                cs.w += __shfl_xor(cs.w, m);
            }
            if ((tid & 63) == 0) scratch[(tid >> 6) * C + c] = cs;
        }
        __syncthreads();
        float4 mean[C];
        const float n = (float)N;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            float4 m4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 2   // (fully unrolled, the 16 reads are hoisted: 64 VGPRs at once, spills)
            for (int wv = 0; wv < kTileThreads / 64; ++wv) {
                const float4 p = scratch[wv * C + c];
                m4.x += p.x;
                m4.y += p.y;
                m4.z += p.z;
                m4.w += p.w;
            }
            mean[c] = make_float4(m4.x / n, m4.y / n, m4.z / n, m4.w / n);
        }
        const int64_t qn = q + gridDim.x;
        if (qn < nsteps && mine) {   // lands during the rounds
#pragma unroll
            for (int c = 0; c < C; ++c) px[c] = tr_load4(xb + off(a.xts, xrow, qn * C + c));
        }
        const float4 *src = img0;
        float4 *dst = img1;
#pragma unroll
        for (int r = 0; r < KR; ++r) {
            if (r < rounds) {
                if (mine) {
                    float d = 0.f;
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        f32x2 lo, hi;
                        mix(src, c, lo, hi);
                        const float4 y = make_float4(lo.x, lo.y, hi.x, hi.y);
                        if (r + 1 < rounds)
                            dst[c * N + tid] = y;
                        else
                            tr_store4(y, yb + off(a.yts, yrow, q * C + c));
                        d += dev2(lo, hi, f32x2{mean[c].x, mean[c].y}, f32x2{mean[c].z, mean[c].w});
                    }
                    dacc[r] += d;
                }
                __syncthreads();   // dst complete before it is read; img0/scratch reuse
                const float4 *t = src;
                src = dst;
                dst = const_cast<float4 *>(t);
            }
        }
    }
    if (mine) {
#pragma unroll
        for (int r = 0; r < KR; ++r)
            if (r < rounds) a.dev_partial[((int64_t)blockIdx.x * rounds + r) * N + tid] = dacc[r];
    }
}

// Agent-major variant for register-cached regular graphs (RE = 5) at C = 4: the images are rows
// [N][4] float4 (64 B per agent, all 16 columns of the step) and lane = (row, chunk) as in
// mix_multi_kernel: thread (s, c) produces chunk c of agents s + k * 256, k < KV.  A 16-lane
// ds_read_b128 group then reads 4 neighbour rows x 4 chunks, so it is conflict-free when those
// 4 rows sit on distinct slots mod 4 (graph.lds_slot_order with chunks = 4: a random 4-regular
// graph of 1024 agents reaches 51 extra cycles per round-tile, against 335 x 4 planes for the
// chunk-major images at their best order).  Per round the 4 chunk lanes of an agent add their
// squared deviations with two quad shuffles; lane c keeps agent s + c * 256's trace in dacc.
//
// The pass's last round (the one that stores Y) is peeled out of the round loop and FULL
// (N == KV * SLOTS, every slot an agent) drops the ragged guards: with the image fill and the
// output stores conditional, the compiler's wait-count tracking could not count the stores
// issued after the prefetch, so each tile waited for the previous tile's output stores to drain
// (vmcnt(0)) before filling the image and issuing the next prefetch (≈1.3 ms per pass at c2).
template <int KV, int KR, bool FULL>
__global__ void __launch_bounds__(kTileThreads) mix_trace_rows_kernel(TileArgs a, int rounds) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int C = 4, RE = 5;
    constexpr int SLOTS = kTileThreads / C;
    const int tid = threadIdx.x;
    const int c = tid & (C - 1);
    const int s = tid / C;
    const int N = a.n_rows;
    float4 *img0 = reinterpret_cast<float4 *>(smem);
    float4 *img1 = img0 + N * C;
    float4 *scratch = reinterpret_cast<float4 *>(smem + a.scratch_off);   // [16][C]
    float wreg[RE];
#pragma unroll
    for (int e = 0; e < RE; ++e) wreg[e] = a.w[e];
    // own operand: when every row's first CSR entry is the row itself (W = I - L(w)), the thread
    // that produced agent ag's chunk in round r folds it from a register in round r + 1 -- four
    // LDS reads a row instead of five (as in mix_multi_kernel); a wave vote picks the
    // instantiation.  The LDS offsets (< 64 KiB: N <= 1024 rows of 64 B) are packed two to a
    // register, which pays for the own values' registers
    bool self_ok = true;
#pragma unroll
    for (int k = 0; k < KV; ++k) {
        const int ag = FULL || s + k * SLOTS < N ? s + k * SLOTS : 0;
        self_ok = self_ok && a.col[ag * RE] == ag;
    }
    const bool self0 = __all(self_ok);
    const int lsh = __builtin_ctz((unsigned)a.lchunks);
    const int64_t lmask = (int64_t)a.lchunks - 1;
    auto off = [&](int64_t ts, int64_t row, int64_t q) {
        return (q >> lsh) * ts + row + (q & lmask) * 16;
    };
    const char *xb = reinterpret_cast<const char *>(a.x);
    char *yb = reinterpret_cast<char *>(a.y);
    const int64_t nsteps = a.n_tiles;
    float dacc[KR];
#pragma unroll
    for (int r = 0; r < KR; ++r) dacc[r] = 0.f;
    float dlast = 0.f;   // the last round's (dacc[rounds - 1] stays 0)
    float4 px[KV];
    auto prefetch = [&](int64_t q) {
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const int ag = FULL || s + k * SLOTS < N ? s + k * SLOTS : 0;   // ragged: row 0
            px[k] = tr_load4(xb + off(a.xts, (int64_t)ag * a.xrs, q * C + c));
        }
    };
    auto tiles = [&](auto selfc) {
    constexpr bool SELF = decltype(selfc)::value;
    constexpr int E0 = SELF ? 1 : 0;              // first entry read from LDS
    constexpr int NO = (RE - E0 + 1) / 2;         // offset registers per pass (two per register)
    uint32_t coff[KV][NO];
#pragma unroll
    for (int k = 0; k < KV; ++k) {
        const int ag = FULL || s + k * SLOTS < N ? s + k * SLOTS : 0;
#pragma unroll
        for (int j = 0; j < NO; ++j) {
            const int e = E0 + 2 * j;
            const uint32_t o1 = ((uint32_t)a.col[ag * RE + e] * C + c) * 16u;
            const uint32_t o2 = e + 1 < RE ? ((uint32_t)a.col[ag * RE + e + 1] * C + c) * 16u : 0u;
            coff[k][j] = o1 | (o2 << 16);
        }
    }
    float4 selfv[SELF ? KV : 1];   // this thread's agents' chunks of the current round
    // the fold as (x, y) / (z, w) pairs (fold2), the neighbour reads issued first
    auto mix = [&](const float4 *src, int k, f32x2 &lo, f32x2 &hi) {
        const char *base = reinterpret_cast<const char *>(src);
        f32x4 v[RE];
        if (SELF) v[0] = f32x4{selfv[k].x, selfv[k].y, selfv[k].z, selfv[k].w};
#pragma unroll
        for (int e = E0; e < RE; ++e) {
            const uint32_t w2 = coff[k][(e - E0) >> 1];
            const uint32_t o = (e - E0) & 1 ? w2 >> 16 : w2 & 0xffffu;
            v[e] = *reinterpret_cast<const f32x4 *>(base + o);
        }
        lo = f32x2{0.f, 0.f};
        hi = f32x2{0.f, 0.f};
#pragma unroll
        for (int e = 0; e < RE; ++e) fold2(lo, hi, wreg[e], v[e]);
    };
    int64_t q = blockIdx.x;
    if (q < nsteps) prefetch(q);
    for (; q < nsteps; q += gridDim.x) {
        float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const int ag = s + k * SLOTS;
            if (SELF) selfv[k] = px[k];
            if (FULL || ag < N) {
                img0[ag * C + c] = px[k];
                cs.x += px[k].x;
                cs.y += px[k].y;
                cs.z += px[k].z;
                cs.w += px[k].w;
            }
        }
#pragma unroll
        for (int m = C; m < 64; m <<= 1) {
            cs.x += __shfl_xor(cs.x, m);
            cs.y += __shfl_xor(cs.y, m);
            cs.z += __shfl_xor(cs.z, m);
            cs.w += __shfl_xor(cs.w, m);
        }
        if ((tid & 63) < C) scratch[(tid >> 6) * C + (tid & 63)] = cs;
        __syncthreads();
        float4 mean = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 2
        for (int wv = 0; wv < kTileThreads / 64; ++wv) {
            const float4 p = scratch[wv * C + c];
            mean.x += p.x;
            mean.y += p.y;
            mean.z += p.z;
            mean.w += p.w;
        }
        const float n = (float)N;
        mean = make_float4(mean.x / n, mean.y / n, mean.z / n, mean.w / n);
        const f32x2 mlo = {mean.x, mean.y}, mhi = {mean.z, mean.w};
        if (q + gridDim.x < nsteps) prefetch(q + gridDim.x);   // lands during the rounds
        const float4 *src = img0;
        float4 *dst = img1;
        // one round src -> dst (LDS) or, the pass's last, src -> Y; acc += this lane's agent's
        // squared deviation
        auto round = [&](bool last, float &acc) {
            float own = 0.f;
#pragma unroll
            for (int k = 0; k < KV; ++k) {
                const int ag = s + k * SLOTS;
                float v = 0.f;
                if (FULL || ag < N) {
                    f32x2 lo, hi;
                    mix(src, k, lo, hi);
                    const float4 y = make_float4(lo.x, lo.y, hi.x, hi.y);
                    if (!last) {
                        dst[ag * C + c] = y;
                        if (SELF) selfv[k] = y;
                    } else {
                        tr_store4(y, yb + off(a.yts, (int64_t)ag * a.yrs, q * C + c));
                    }
                    v = dev2(lo, hi, mlo, mhi);
                }
                v += quad_xor1(v);   // the agent's 4 chunk lanes (whole wave active)
                v += quad_xor2(v);
                own += k == c ? v : 0.f;
            }
            acc += own;
            __syncthreads();   // dst complete before it is read; img0/scratch reuse
            const float4 *t = src;
            src = dst;
            dst = const_cast<float4 *>(t);
        };
#pragma unroll
        for (int r = 0; r + 1 < KR; ++r)
            if (r + 1 < rounds) round(false, dacc[r]);
        round(true, dlast);
    }
    };
    if (self0)
        tiles(std::true_type{});
    else
        tiles(std::false_type{});
    const int mine_ag = s + c * SLOTS;
    if (c < KV && (FULL || mine_ag < N)) {
#pragma unroll
        for (int r = 0; r < KR; ++r)
            if (r < rounds)
                a.dev_partial[((int64_t)blockIdx.x * rounds + r) * N + mine_ag] =
                    r == rounds - 1 ? dlast : dacc[r];
    }
}

// Wide variant: 1024 < N <= 4096 agents (the c4 torus) at C = 1 (T = 4 columns per step), KV =
// ceil(N / 1024) agents per thread (s + k * 1024), every lane its agents' only chunk.  Two images
// of 4096 agents are 128 KiB, so the CSR stays in registers (RE = 5, shared weights, as in
// mix_multi_kernel) or, for up to 2048 agents, in LDS (RE = 0).  The per-round squared
// deviations of a thread's KV agents live in registers for the whole pass (dacc[KV][KR]), which
// caps a pass at KR rounds; the last round, which stores Y, is peeled as in the rows kernel.
template <int KV, int KR, int RE, bool FULL>
__global__ void __launch_bounds__(kTileThreads) mix_trace_wide_kernel(TileArgs a, int rounds) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int SLOTS = kTileThreads;
    const int tid = threadIdx.x;
    const int s = tid;
    const int N = a.n_rows;
    float4 *img0 = reinterpret_cast<float4 *>(smem);
    float4 *img1 = img0 + N;
    float4 *scratch = reinterpret_cast<float4 *>(smem + a.scratch_off);   // [16]
    float *lw = reinterpret_cast<float *>(smem + a.csr_off);
    uint16_t *lcol = reinterpret_cast<uint16_t *>(smem + a.csr_off + 4u * (uint32_t)a.n_w);
    uint16_t *lrp = lcol + a.nnz;
    const int reg = a.regular;
    const bool wshared = a.n_w != a.nnz;
    if constexpr (RE == 0) {
        for (int i = tid; i < a.n_w; i += kTileThreads) lw[i] = a.w[i];
        for (int i = tid; i < a.nnz; i += kTileThreads) lcol[i] = (uint16_t)a.col[i];
        if (!reg)
            for (int i = tid; i <= N; i += kTileThreads) lrp[i] = (uint16_t)a.rowptr[i];
    }
    uint32_t coff[KV][RE > 0 ? RE : 1];
    float wreg[RE > 0 ? RE : 1];
    if constexpr (RE > 0) {
#pragma unroll
        for (int e = 0; e < RE; ++e) wreg[e] = a.w[e];
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const int ag = FULL || s + k * SLOTS < N ? s + k * SLOTS : 0;
#pragma unroll
            for (int e = 0; e < RE; ++e) coff[k][e] = (uint32_t)a.col[ag * RE + e] * 16u;
        }
    }
    // agent s + k * SLOTS's output from an image: left fold in CSR order from +0.0, as pairs
    auto mix = [&](const float4 *src, int k, f32x2 &lo, f32x2 &hi) {
        lo = f32x2{0.f, 0.f};
        hi = f32x2{0.f, 0.f};
        if constexpr (RE > 0) {
            const char *base = reinterpret_cast<const char *>(src);
            f32x4 v[RE];
#pragma unroll
            for (int e = 0; e < RE; ++e) v[e] = *reinterpret_cast<const f32x4 *>(base + coff[k][e]);
#pragma unroll
            for (int e = 0; e < RE; ++e) fold2(lo, hi, wreg[e], v[e]);
        } else {
            const int ag = s + k * SLOTS;
            int e0, e1;
            if (reg) {
                e0 = ag * reg;
                e1 = e0 + reg;
            } else {
                e0 = lrp[ag];
                e1 = lrp[ag + 1];
            }
            const float *wr = wshared ? lw - e0 : lw;
            const f32x4 *sv = reinterpret_cast<const f32x4 *>(src);
            for (int e = e0; e < e1; ++e) fold2(lo, hi, wr[e], sv[lcol[e]]);
        }
    };
    const int lsh = __builtin_ctz((unsigned)a.lchunks);
    const int64_t lmask = (int64_t)a.lchunks - 1;
    auto off = [&](int64_t ts, int64_t row, int64_t q) {
        return (q >> lsh) * ts + row + (q & lmask) * 16;
    };
    const char *xb = reinterpret_cast<const char *>(a.x);
    char *yb = reinterpret_cast<char *>(a.y);
    const int64_t nsteps = a.n_tiles;
    float dacc[KV][KR];
#pragma unroll
    for (int k = 0; k < KV; ++k)
#pragma unroll
        for (int r = 0; r < KR; ++r) dacc[k][r] = 0.f;
    float dlast[KV];   // the last round's (dacc[.][rounds - 1] stays 0)
#pragma unroll
    for (int k = 0; k < KV; ++k) dlast[k] = 0.f;
    float4 px[KV];
    auto prefetch = [&](int64_t q) {
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const int ag = FULL || s + k * SLOTS < N ? s + k * SLOTS : 0;   // ragged: row 0
            px[k] = tr_load4(xb + off(a.xts, (int64_t)ag * a.xrs, q));
        }
    };
    int64_t q = blockIdx.x;
    if (q < nsteps) prefetch(q);
    if (RE == 0) __syncthreads();   // CSR staged
    for (; q < nsteps; q += gridDim.x) {
        float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const int ag = s + k * SLOTS;
            if (FULL || ag < N) {
                img0[ag] = px[k];
                cs.x += px[k].x;
                cs.y += px[k].y;
                cs.z += px[k].z;
                cs.w += px[k].w;
            }
        }
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) {
            cs.x += __shfl_xor(cs.x, m);
            cs.y += __shfl_xor(cs.y, m);
            cs.z += __shfl_xor(cs.z, m);
            cs.w += __shfl_xor(cs.w, m);
        }
        if ((tid & 63) == 0) scratch[tid >> 6] = cs;
        __syncthreads();
        float4 mean = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 2
        for (int wv = 0; wv < kTileThreads / 64; ++wv) {
            const float4 p = scratch[wv];
            mean.x += p.x;
            mean.y += p.y;
            mean.z += p.z;
            mean.w += p.w;
        }
        const float n = (float)N;
        mean = make_float4(mean.x / n, mean.y / n, mean.z / n, mean.w / n);
        const f32x2 mlo = {mean.x, mean.y}, mhi = {mean.z, mean.w};
        if (q + gridDim.x < nsteps) prefetch(q + gridDim.x);   // lands during the rounds
        const float4 *src = img0;
        float4 *dst = img1;
        // one round src -> dst (LDS) or, the pass's last, src -> Y; acc[k] += agent k's squared
        // deviation
        auto round = [&](bool last, auto &&acc_of) {
#pragma unroll
            for (int k = 0; k < KV; ++k) {
                const int ag = s + k * SLOTS;
                if (FULL || ag < N) {
                    f32x2 lo, hi;
                    mix(src, k, lo, hi);
                    const float4 y = make_float4(lo.x, lo.y, hi.x, hi.y);
                    if (!last)
                        dst[ag] = y;
                    else
                        tr_store4(y, yb + off(a.yts, (int64_t)ag * a.yrs, q));
                    acc_of(k) += dev2(lo, hi, mlo, mhi);
                }
                // one output at a time (register pressure at 1024 threads, as mix_multi_kernel)
                __builtin_amdgcn_sched_barrier(0);
            }
            __syncthreads();   // dst complete before it is read; img0/scratch reuse
            const float4 *t = src;
            src = dst;
            dst = const_cast<float4 *>(t);
        };
#pragma unroll
        for (int r = 0; r + 1 < KR; ++r)
            if (r + 1 < rounds) round(false, [&](int k) -> float & { return dacc[k][r]; });
        round(true, [&](int k) -> float & { return dlast[k]; });
    }
#pragma unroll
    for (int k = 0; k < KV; ++k) {
        const int ag = s + k * SLOTS;
        if (FULL || ag < N) {
#pragma unroll
            for (int r = 0; r < KR; ++r)
                if (r < rounds)
                    a.dev_partial[((int64_t)blockIdx.x * rounds + r) * N + ag] =
                        r == rounds - 1 ? dlast[k] : dacc[k][r];
        }
    }
}

// Traced passes for the graphs the double-buffered kernels above cannot hold: irregular graphs
// of more than 2048 agents (Barabasi-Albert hubs, per-entry weights), and any W that is not
// doubly stochastic (GM).  One LDS image [N] of one column chunk per step and the CSR as in plan
// path 5: each row's first RD entries in registers, the rest behind the image.  With one image
// a round folds every output into registers, waits for all reads of the image, then writes it
// back (two barriers a round instead of one ping-pong barrier).  GM: mean(W x) != mean(x), so
// every round's column mean is reduced from its outputs (wave shuffles + a 16-entry scratch)
// before the deviations of that round -- what Mixer._get_deviation_dict computes after every
// round (mixer.py:51-66).  The fold is the reference's left fold in CSR order (head, then tail)
// as in the other kernels: bit-identical.  KV agents per thread (rows tid + k * 1024), KR rounds
// per pass (their deviations in VGPRs).
// NW (narrow): 2-column chunks (8-byte image entries) and a 6-byte tail (fp32 weights, then u16
// rows) for CSRs that do not fit LDS beside a 16-byte image with 8-byte pairs (a row-stochastic
// graph of 4096 agents and 41k entries: 32 KiB image + 123 KiB tail).
template <int KV, int KR, int RD, bool GM, bool NW>
__global__ void __launch_bounds__(kTileThreads) mix_trace_irr_kernel(TileArgs a, int rounds) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int NT = kTileThreads;
    typedef typename std::conditional<NW, f32x2, f32x4>::type vec;
    const int tid = threadIdx.x;
    const int N = a.n_rows;
    const int nnz = a.nnz;
    vec *img = reinterpret_cast<vec *>(smem);
    float4 *scratch = reinterpret_cast<float4 *>(smem + a.scratch_off);   // [16]
    const int ntail = nnz - RD * N;
    uint2 *ltp = reinterpret_cast<uint2 *>(smem + a.csr_off);                        // !NW
    float *ltw = reinterpret_cast<float *>(smem + a.csr_off);                        // NW
    uint16_t *ltc = reinterpret_cast<uint16_t *>(smem + a.csr_off + 4u * (uint32_t)ntail);
    constexpr int NRC = RD > 0 ? KV * RD : 1;
    float rw[NRC];
    uint32_t ri[(NRC + 1) / 2];
    uint32_t rdesc[KV];   // row's LDS tail: start (low 16 bits), length (high 16 bits)
#pragma unroll
    for (int i = 0; i < (NRC + 1) / 2; ++i) ri[i] = 0u;
#pragma unroll
    for (int k = 0; k < KV; ++k) {
        const int r = tid + k * NT;
        const int rr = r < N ? r : 0;
        const int e0 = a.rowptr[rr], e1 = a.rowptr[rr + 1];
#pragma unroll
        for (int e = 0; e < (RD > 0 ? RD : 0); ++e) {
            const int j = k * RD + e;
            // (clamped into the CSR: a wrong min_row_nnz promise gives wrong results only)
            const int idx = min(max(e0 + e, 0), nnz - 1);
            rw[j] = a.w[idx];
            ri[j >> 1] |= (uint32_t)a.col[idx] << (16 * (j & 1));
        }
        const int st = min(max(e0 - RD * rr, 0), ntail);
        const int ln = min(max(e1 - e0 - RD, 0), ntail - st);
        rdesc[k] = r < N ? (uint32_t)st | ((uint32_t)ln << 16) : 0u;
    }
    {   // stage the tail: a row id per tail slot (u16), then the entries
        // (!NW: the map in the image area; NW: in the upper half of the weights array, so
        // batches of reads, a barrier, then writes: weight t lands on map slot 2t - ntail < t,
        // already read)
        uint16_t *trow = NW ? reinterpret_cast<uint16_t *>(smem + a.csr_off + 2u * (uint32_t)ntail)
                            : reinterpret_cast<uint16_t *>(smem);
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const uint32_t t0 = rdesc[k] & 0xffffu, tn = rdesc[k] >> 16;
            for (uint32_t t = 0; t < tn; ++t) trow[t0 + t] = (uint16_t)(tid + k * NT);
        }
        __syncthreads();
        if constexpr (NW) {
            for (int base = 0; base < ntail; base += 4 * NT) {
                int rid[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int t = base + u * NT + tid;
                    rid[u] = t < ntail ? trow[t] : 0;
                }
                __syncthreads();
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int t = base + u * NT + tid;
                    if (t < ntail) {
                        const int e = min(t + RD * (rid[u] + 1), nnz - 1);
                        ltw[t] = a.w[e];
                        ltc[t] = (uint16_t)a.col[e];
                    }
                }
                __syncthreads();
            }
        } else {
            for (int t = tid; t < ntail; t += NT) {
                const int e = min(t + RD * (trow[t] + 1), nnz - 1);
                ltp[t] = make_uint2(__float_as_uint(a.w[e]), (uint32_t)a.col[e]);
            }
            __syncthreads();
        }
    }
    // (lo, hi) += w * v: the pair fold of the 16-byte image; lo += w * v on the 8-byte one
    auto fold1 = [&](f32x2 &lo, f32x2 &hi, float w, const vec &v) {
        if constexpr (NW) {
            const f32x2 w2 = {w, w};
            lo = lo + w2 * v;
        } else {
            fold2(lo, hi, w, v);
        }
    };
    auto entry = [&](uint32_t i, float &w, uint32_t &ci) {
        if constexpr (NW) {
            w = ltw[i];
            ci = ltc[i];
        } else {
            const uint2 pr = ltp[i];
            w = __uint_as_float(pr.x);
            ci = pr.y;
        }
    };
    // agent tid + k * 1024's output from the image: register head, then the LDS tail, TU
    // entries' reads issued per step
    auto fold = [&](int k, f32x2 &lo, f32x2 &hi) {
        lo = f32x2{0.f, 0.f};
        hi = f32x2{0.f, 0.f};
#pragma unroll
        for (int e = 0; e < (RD > 0 ? RD : 0); ++e) {
            const int j = k * RD + e;
            const uint32_t idx = (ri[j >> 1] >> (16 * (j & 1))) & 0xffffu;
            fold1(lo, hi, rw[j], img[idx]);
        }
        uint32_t t = rdesc[k] & 0xffffu;
        const uint32_t t1 = t + (rdesc[k] >> 16);
        constexpr int TU = KV >= 4 ? 1 : 4;   // (4 agents' outputs: fewer in flight)
        for (; t + TU <= t1; t += TU) {
            float w4[TU];
            uint32_t c4[TU];
            vec v4[TU];
#pragma unroll
            for (int u = 0; u < TU; ++u) entry(t + u, w4[u], c4[u]);
#pragma unroll
            for (int u = 0; u < TU; ++u) v4[u] = img[c4[u]];
#pragma unroll
            for (int u = 0; u < TU; ++u) fold1(lo, hi, w4[u], v4[u]);
        }
        for (; t < t1; ++t) {
            float w;
            uint32_t ci;
            entry(t, w, ci);
            fold1(lo, hi, w, img[ci]);
        }
    };
    // column mean of this step's chunk over every agent: per-thread sums -> wave -> scratch
    auto reduce_mean = [&](float4 cs) {
#pragma unroll
        for (int m = 1; m < 64; m <<= 1) {
            cs.x += __shfl_xor(cs.x, m);
            cs.y += __shfl_xor(cs.y, m);
            if (!NW) {
                cs.z += __shfl_xor(cs.z, m);
                cs.w += __shfl_xor(cs.w, m);
            }
        }
        if ((tid & 63) == 0) scratch[tid >> 6] = cs;
    };
    auto read_mean = [&]() {
        float4 m4 = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 2
        for (int wv = 0; wv < NT / 64; ++wv) {
            const float4 p = scratch[wv];
            m4.x += p.x;
            m4.y += p.y;
            m4.z += p.z;
            m4.w += p.w;
        }
        const float n = (float)N;
        return make_float4(m4.x / n, m4.y / n, m4.z / n, m4.w / n);
    };
    const int lsh = __builtin_ctz((unsigned)a.lchunks);
    const int64_t lmask = (int64_t)a.lchunks - 1;
    // byte offset of (agent row, step q): 16-byte chunks, or (NW) 8-byte halves of them
    auto off = [&](int64_t ts, int64_t row, int64_t q) {
        const int64_t c4 = NW ? q >> 1 : q;
        return (c4 >> lsh) * ts + row + (c4 & lmask) * 16 + (NW ? (q & 1) * 8 : 0);
    };
    const char *xb = reinterpret_cast<const char *>(a.x);
    char *yb = reinterpret_cast<char *>(a.y);
    const int64_t nsteps = a.n_tiles;
    float dacc[KV][KR];
#pragma unroll
    for (int k = 0; k < KV; ++k)
#pragma unroll
        for (int r = 0; r < KR; ++r) dacc[k][r] = 0.f;
    vec px[KV];
    // (lane ids laundered per step: hoisted out of the step loop, the KV agents' 64-bit load and
    // store addresses took 16 VGPRs and spilled)
    int ltid = tid;
    auto prefetch = [&](int64_t q) {
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const int ag = ltid + k * NT < N ? ltid + k * NT : 0;   // ragged: row 0 (L1 hit)
            px[k] = __builtin_nontemporal_load(
                reinterpret_cast<const vec *>(xb + off(a.xts, (int64_t)ag * a.xrs, q)));
        }
    };
    auto comps = [](const vec &v) {   // as float4 (NW: z = w = 0)
        if constexpr (NW)
            return make_float4(v.x, v.y, 0.f, 0.f);
        else
            return make_float4(v.x, v.y, v.z, v.w);
    };
    int64_t q = blockIdx.x;
    if (q < nsteps) prefetch(q);
    for (; q < nsteps; q += gridDim.x) {
        asm volatile("" : "+v"(ltid));
        float4 cs = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int k = 0; k < KV; ++k) {
            const int ag = tid + k * NT;
            if (ag < N) {
                img[ag] = px[k];
                const float4 v = comps(px[k]);
                cs.x += v.x;
                cs.y += v.y;
                cs.z += v.z;
                cs.w += v.w;
            }
        }
        if (!GM) reduce_mean(cs);   // mean(W^r x) = mean(x): one mean per step
        __syncthreads();
        float4 mean = GM ? make_float4(0.f, 0.f, 0.f, 0.f) : read_mean();
        // the next step's chunk lands during the rounds (at 4 agents per thread after them: the
        // prefetch registers beside 4 agents' head CSR and outputs spill)
        constexpr bool PF = KV < 4;
        if (PF && q + gridDim.x < nsteps) prefetch(q + gridDim.x);
        // (the round loop stays rolled: unrolled, four agents' folds of every round were
        // interleaved and spilled; a round's deviations go to their slot by predicated adds)
#pragma unroll 1
        for (int r = 0; r < rounds; ++r) {
            {
                const bool last = r + 1 == rounds;
                f32x2 ylo[KV], yhi[KV];
#pragma unroll
                for (int k = 0; k < KV; ++k) {
                    if (tid + k * NT < N) fold(k, ylo[k], yhi[k]);
                    __builtin_amdgcn_sched_barrier(0);
                }
                __syncthreads();   // every read of the image is done
                float4 ys = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
                for (int k = 0; k < KV; ++k) {
                    const int ag = tid + k * NT;
                    if (ag < N) {
                        vec y;
                        if constexpr (NW)
                            y = ylo[k];
                        else
                            y = f32x4{ylo[k].x, ylo[k].y, yhi[k].x, yhi[k].y};
                        if (!last)
                            img[ag] = y;
                        else
                            *reinterpret_cast<vec *>(
                                yb + off(a.yts, (int64_t)(ltid + k * NT) * a.yrs, q)) = y;
                        ys.x += ylo[k].x;
                        ys.y += ylo[k].y;
                        ys.z += NW ? 0.f : yhi[k].x;
                        ys.w += NW ? 0.f : yhi[k].y;
                    }
                }
                if (GM) {   // this round's column mean, from its outputs
                    reduce_mean(ys);
                    __syncthreads();   // (also: the image complete before the next round reads)
                    mean = read_mean();
                } else if (!last) {
                    __syncthreads();   // the image complete before the next round reads it
                }
                const f32x2 mlo = {mean.x, mean.y}, mhi = {mean.z, mean.w};
#pragma unroll
                for (int k = 0; k < KV; ++k) {
                    float d = 0.f;
                    if (tid + k * NT < N) {
                        if constexpr (NW) {
                            const f32x2 dd = ylo[k] - mlo, q2 = dd * dd;
                            d = q2.x + q2.y;
                        } else {
                            d = dev2(ylo[k], yhi[k], mlo, mhi);
                        }
                    }
#pragma unroll
                    for (int j = 0; j < KR; ++j) dacc[k][j] += j == r ? d : 0.f;
                }
            }
        }
        // (GM) the last round's scratch reads finish before the next step writes scratch: that
        // write comes after round 0's first barrier
        if (!PF && q + gridDim.x < nsteps) prefetch(q + gridDim.x);
    }
#pragma unroll
    for (int k = 0; k < KV; ++k) {
        const int ag = tid + k * NT;
        if (ag < N) {
#pragma unroll
            for (int r = 0; r < KR; ++r)
                if (r < rounds) a.dev_partial[((int64_t)blockIdx.x * rounds + r) * N + ag] = dacc[k][r];
        }
    }
}

// out[r] = max_a sqrt(sum_b partial[b][r][a]) (fp64 sum in workgroup order, then float, as
// dev_reduce's dev_sq); one workgroup per round.
__global__ void __launch_bounds__(1024) trace_reduce_kernel(const float *__restrict__ partial,
                                                            int nparts, int rounds, int n,
                                                            float *__restrict__ out) {
    __shared__ float red[16];
    const int r = blockIdx.x, tid = threadIdx.x;
    float best = 0.f;
    for (int ag = tid; ag < n; ag += 1024) {
        // eight partials in flight, added in the same order (bit-identical to one at a time)
        double s = 0.0;
        int b = 0;
        for (; b + 7 < nparts; b += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = partial[((int64_t)(b + u) * rounds + r) * n + ag];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += (double)v[u];
        }
        for (; b < nparts; ++b) s += (double)partial[((int64_t)b * rounds + r) * n + ag];
        best = fmaxf(best, sqrtf((float)s));
    }
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) best = fmaxf(best, __shfl_xor(best, m));
    if ((tid & 63) == 0) red[tid >> 6] = best;
    __syncthreads();
    if (tid == 0) {
        float m = red[0];
        for (int i = 1; i < 16; ++i) m = fmaxf(m, red[i]);
        out[r] = m;
    }
}

template <int RE, int C>
hipError_t launch_rc(const TileArgs &a, int rounds, int grid, int lds, hipStream_t s) {
    const void *k = reinterpret_cast<const void *>(mix_trace_kernel<RE, C>);
    hipError_t e = allow_full_lds(k);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((mix_trace_kernel<RE, C>), dim3(grid), dim3(kTileThreads), lds, s, a,
                       rounds);
    return hipGetLastError();
}

template <int KV, int KR>
hipError_t launch_rows(const TileArgs &a, int rounds, int grid, int lds, hipStream_t s) {
    const bool full = a.n_rows == KV * (kTileThreads / 4);
    const void *k = full ? reinterpret_cast<const void *>(mix_trace_rows_kernel<KV, KR, true>)
                         : reinterpret_cast<const void *>(mix_trace_rows_kernel<KV, KR, false>);
    hipError_t e = allow_full_lds(k);
    if (e != hipSuccess) return e;
    if (full)
        hipLaunchKernelGGL((mix_trace_rows_kernel<KV, KR, true>), dim3(grid), dim3(kTileThreads),
                           lds, s, a, rounds);
    else
        hipLaunchKernelGGL((mix_trace_rows_kernel<KV, KR, false>), dim3(grid), dim3(kTileThreads),
                           lds, s, a, rounds);
    return hipGetLastError();
}

template <int RE>
hipError_t launch_re(const TileArgs &a, int chunks, int rounds, int grid, int lds,
                     hipStream_t s) {
    switch (chunks) {
        case 1: return launch_rc<RE, 1>(a, rounds, grid, lds, s);
        case 2: return launch_rc<RE, 2>(a, rounds, grid, lds, s);
        case 4: return launch_rc<RE, 4>(a, rounds, grid, lds, s);
        default: return hipErrorInvalidValue;
    }
}

template <int KV, int RE>
hipError_t launch_wide(const TileArgs &a, int rounds, int grid, int lds, hipStream_t s) {
    constexpr int KR = KV > 2 ? kWideTraceRounds4 : kWideTraceRounds2;
    const bool full = a.n_rows == KV * kTileThreads;
    const void *k = full ? reinterpret_cast<const void *>(mix_trace_wide_kernel<KV, KR, RE, true>)
                         : reinterpret_cast<const void *>(mix_trace_wide_kernel<KV, KR, RE, false>);
    hipError_t e = allow_full_lds(k);
    if (e != hipSuccess) return e;
    if (full)
        hipLaunchKernelGGL((mix_trace_wide_kernel<KV, KR, RE, true>), dim3(grid),
                           dim3(kTileThreads), lds, s, a, rounds);
    else
        hipLaunchKernelGGL((mix_trace_wide_kernel<KV, KR, RE, false>), dim3(grid),
                           dim3(kTileThreads), lds, s, a, rounds);
    return hipGetLastError();
}

template <int KV, int RD, bool GM>
hipError_t launch_irr3(const TileArgs &a, bool narrow, int rounds, int grid, int lds,
                       hipStream_t s) {
    constexpr int KR = irr_trace_rounds(KV);
    auto k = narrow ? mix_trace_irr_kernel<KV, KR, RD, GM, true>
                    : mix_trace_irr_kernel<KV, KR, RD, GM, false>;
    hipError_t e = allow_full_lds(reinterpret_cast<const void *>(k));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(grid), dim3(kTileThreads), lds, s, a, rounds);
    return hipGetLastError();
}

template <int KV, bool GM>
hipError_t launch_irr2(const TileArgs &a, int head, bool narrow, int rounds, int grid, int lds,
                       hipStream_t s) {
    switch (head) {
        case 0: return launch_irr3<KV, 0, GM>(a, narrow, rounds, grid, lds, s);
        case 2: return launch_irr3<KV, 2, GM>(a, narrow, rounds, grid, lds, s);
        case 3: return launch_irr3<KV, 3, GM>(a, narrow, rounds, grid, lds, s);
        case 5: return launch_irr3<KV, 5, GM>(a, narrow, rounds, grid, lds, s);
        default: return hipErrorInvalidValue;
    }
}

template <bool GM>
hipError_t launch_irr1(const TileArgs &a, int head, bool narrow, int rounds, int grid, int lds,
                       hipStream_t s) {
    if (a.n_rows <= kTileThreads)
        return launch_irr2<1, GM>(a, head, narrow, rounds, grid, lds, s);
    if (a.n_rows <= 2 * kTileThreads)
        return launch_irr2<2, GM>(a, head, narrow, rounds, grid, lds, s);
    return launch_irr2<4, GM>(a, head, narrow, rounds, grid, lds, s);
}

}  // namespace

hipError_t launch_mix_trace_irr(const TileArgs &a, int head, bool general_mean, bool narrow,
                                int rounds, int grid, int lds, float *trace_out, hipStream_t s) {
    if (rounds < 1 || rounds > irr_trace_rounds(irr_trace_kv(a.n_rows)) || a.n_rows < 2 ||
        a.n_rows > 4 * kTileThreads || a.lchunks < 1)
        return hipErrorInvalidValue;
    hipError_t e = general_mean ? launch_irr1<true>(a, head, narrow, rounds, grid, lds, s)
                                : launch_irr1<false>(a, head, narrow, rounds, grid, lds, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(trace_reduce_kernel, dim3(rounds), dim3(1024), 0, s, a.dev_partial, grid,
                       rounds, a.n_rows, trace_out);
    return hipGetLastError();
}

hipError_t launch_mix_trace(const TileArgs &a, int chunks, int rounds, int grid, int lds,
                            float *trace_out, hipStream_t s) {
    const bool in_regs = a.regular == 5 && a.n_w == 5;
    if (rounds < 1 || rounds > trace_max_rounds(a.n_rows, in_regs, chunks))
        return hipErrorInvalidValue;
    hipError_t e;
    if (a.n_rows > kTileThreads) {   // the wide kernel: C = 1, KV agents per thread
        if (chunks != 1 || a.lchunks < 1 || (!in_regs && a.n_rows > 2 * kTileThreads))
            return hipErrorInvalidValue;
        if (a.n_rows <= 2 * kTileThreads)
            e = in_regs ? launch_wide<2, 5>(a, rounds, grid, lds, s)
                        : launch_wide<2, 0>(a, rounds, grid, lds, s);
        else
            e = launch_wide<4, 5>(a, rounds, grid, lds, s);
    } else if (trace_uses_rows(a.n_rows, in_regs, chunks)) {
        // agent-major rows (mix_trace_rows_kernel); DLAMD_TRACE_PLANES=1 keeps the chunk-major
        // planes for comparison
        if (a.n_rows <= 256)
            e = launch_rows<1, kTraceRounds>(a, rounds, grid, lds, s);
        else if (a.n_rows <= 512)
            e = launch_rows<2, kTraceRounds>(a, rounds, grid, lds, s);
        else
            e = launch_rows<4, kRowsTraceRounds>(a, rounds, grid, lds, s);
    } else {
        e = in_regs ? launch_re<5>(a, chunks, rounds, grid, lds, s)
                    : launch_re<0>(a, chunks, rounds, grid, lds, s);
    }
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(trace_reduce_kernel, dim3(rounds), dim3(1024), 0, s, a.dev_partial, grid,
                       rounds, a.n_rows, trace_out);
    return hipGetLastError();
}

}  // namespace dl
