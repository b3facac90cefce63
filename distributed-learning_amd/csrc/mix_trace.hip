// K gossip rounds in one HBM pass WITH the per-round disagreement trace (gfx950):
// `Mixer.mix(times, eps)` (utils/consensus_simple/mixer.py:18-41) with eps set evaluates
// max_a ||x_a - mean(X)|| (:51-66) after every round and stops at the first round r >= times
// whose value is below eps.  mix_multi_kernel already runs K rounds on LDS-resident column tiles
// (mixing is column-independent); the stop test is what kept eps-loops on one HBM-bound launch
// per round.  Here every workgroup also accumulates, for each of the K rounds, every agent's
// squared deviation over its own columns in an LDS trace [K][N]; one reduce launch turns the
// per-workgroup traces into the K per-round max deviations.  The host then finds the stop round
// and, if it lies inside the pass, re-runs that many rounds from the pass's input (still intact:
// X -> Y).  The rounds are the same CSR-order fp32 fold as the one-round kernel, so the iterates
// are bit-identical to round-by-round mixing.
//
// Geometry: one agent per thread (N <= 1024), one float4 column chunk per tile step, so a
// thread's trace slot is a single LDS word it alone updates (no shuffles, no atomics).  LDS:
// two chunk images 2 x N x 16 B, the trace K x N x 4 B, the CSR (unless register-cached), a
// 16-float4 mean scratch.  W must be doubly stochastic: the column mean of every round equals
// the mean of the pass's input chunk (mean(W t) = mean(t)), as in the fused one-round deviation.
#include "dl_internal.h"

namespace dl {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 tr_load4(const char *p) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ void tr_store4(float4 v, char *p) {
    f32x4 x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<f32x4 *>(p));
}

// RE > 0: regular graph of RE entries per row sharing row 0's weights, CSR in registers.
template <int RE>
__global__ void __launch_bounds__(kTileThreads) mix_trace_kernel(TileArgs a, int rounds) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x;
    const int N = a.n_rows;
    const bool mine = tid < N;
    float4 *img0 = reinterpret_cast<float4 *>(smem);
    float4 *img1 = img0 + N;
    float *trace = reinterpret_cast<float *>(smem + a.trace_off);
    float4 *scratch = reinterpret_cast<float4 *>(smem + a.scratch_off);
    float *lw = reinterpret_cast<float *>(smem + a.csr_off);
    uint16_t *lcol = reinterpret_cast<uint16_t *>(smem + a.csr_off + 4u * (uint32_t)a.n_w);
    uint16_t *lrp = lcol + a.nnz;
    const int reg = a.regular;
    const bool wshared = a.n_w != a.nnz;

    if (mine)
        for (int r = 0; r < rounds; ++r) trace[r * N + tid] = 0.f;
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
    // agent tid's output chunk: left fold in CSR order from +0.0 (mixer.py:47)
    auto mix = [&](const float4 *src) {
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (RE > 0) {
            const char *base = reinterpret_cast<const char *>(src);
#pragma unroll
            for (int e = 0; e < RE; ++e) {
                const float4 v = *reinterpret_cast<const float4 *>(base + coff[e]);
                const float w = wreg[e];
                acc.x = acc.x + w * v.x;
                acc.y = acc.y + w * v.y;
                acc.z = acc.z + w * v.z;
                acc.w = acc.w + w * v.w;
            }
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
            for (int e = e0; e < e1; ++e) {
                const float w = wr[e];
                const float4 v = src[lcol[e]];
                acc.x = acc.x + w * v.x;
                acc.y = acc.y + w * v.y;
                acc.z = acc.z + w * v.z;
                acc.w = acc.w + w * v.w;
            }
        }
        return acc;
    };
    // byte offset of (agent tid, chunk q) in an operand laid out in lc-chunk tiles
    const int64_t lc = a.lchunks;
    auto off = [&](int64_t ts, uint32_t rs, int64_t q) {
        return (q / lc) * ts + (int64_t)tid * rs + (q % lc) * 16;
    };
    const char *xb = reinterpret_cast<const char *>(a.x);
    char *yb = reinterpret_cast<char *>(a.y);
    const int64_t nq = a.n_tiles;   // float4 column chunks
    float4 px = make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t q = blockIdx.x;
    if (q < nq && mine) px = tr_load4(xb + off(a.xts, a.xrs, q));
    __syncthreads();   // CSR and trace initialised
    for (; q < nq; q += gridDim.x) {
        if (mine) img0[tid] = px;
        float4 cs = mine ? px : make_float4(0.f, 0.f, 0.f, 0.f);
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
        for (int wv = 0; wv < kTileThreads / 64; ++wv) {
            const float4 p = scratch[wv];
            mean.x += p.x;
            mean.y += p.y;
            mean.z += p.z;
            mean.w += p.w;
        }
        const float n = (float)N;
        mean.x = mean.x / n;
        mean.y = mean.y / n;
        mean.z = mean.z / n;
        mean.w = mean.w / n;
        const int64_t qn = q + gridDim.x;
        if (qn < nq && mine) px = tr_load4(xb + off(a.xts, a.xrs, qn));   // lands during the rounds
        const float4 *src = img0;
        float4 *dst = img1;
        for (int r = 0; r < rounds; ++r) {
            if (mine) {
                const float4 y = mix(src);
                if (r + 1 < rounds)
                    dst[tid] = y;
                else
                    tr_store4(y, yb + off(a.yts, a.yrs, q));
                const float dx = y.x - mean.x, dy = y.y - mean.y;
                const float dz = y.z - mean.z, dw = y.w - mean.w;
                trace[r * N + tid] += (dx * dx + dy * dy) + (dz * dz + dw * dw);
            }
            __syncthreads();   // dst complete before it is read; img0/scratch reuse next chunk
            const float4 *t = src;
            src = dst;
            dst = const_cast<float4 *>(t);
        }
    }
    if (mine)
        for (int r = 0; r < rounds; ++r)
            a.dev_partial[((int64_t)blockIdx.x * rounds + r) * N + tid] = trace[r * N + tid];
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
        double s = 0.0;
        for (int b = 0; b < nparts; ++b) s += (double)partial[((int64_t)b * rounds + r) * n + ag];
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

template <int RE>
hipError_t launch_re(const TileArgs &a, int rounds, int grid, int lds, hipStream_t s) {
    const void *k = reinterpret_cast<const void *>(mix_trace_kernel<RE>);
    hipError_t e = allow_full_lds(k);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(mix_trace_kernel<RE>, dim3(grid), dim3(kTileThreads), lds, s, a, rounds);
    return hipGetLastError();
}

}  // namespace

hipError_t launch_mix_trace(const TileArgs &a, int rounds, int grid, int lds, float *trace_out,
                            hipStream_t s) {
    const bool in_regs = a.regular == 5 && a.n_w == 5;
    hipError_t e = in_regs ? launch_re<5>(a, rounds, grid, lds, s)
                           : launch_re<0>(a, rounds, grid, lds, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(trace_reduce_kernel, dim3(rounds), dim3(1024), 0, s, a.dev_partial, grid,
                       rounds, a.n_rows, trace_out);
    return hipGetLastError();
}

}  // namespace dl
