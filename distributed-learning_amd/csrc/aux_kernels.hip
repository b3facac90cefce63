// Auxiliary kernels around the mixing hot path (gfx950):
//   column sums / means           (np.mean numerator, mixer.py:61; multi-GPU global mean)
//   per-agent deviation rows      (mixer.py:65 against a given mean)
//   max column std                (mixer.py:82-84 intent)
//   boundary-row local step pack  (multi-GPU halo send buffers)
//   Perron / asyncio Jacobi round (consensus_asyncio.py:231-310), fp32 and fp64
#include "dl_internal.h"

#include <cstdlib>

namespace dl {
namespace {

// sum over rows in row order (bit-identical to numpy's add.reduce over axis 0), optional /div.
__global__ void __launch_bounds__(256) column_sum_kernel(const float *__restrict__ x, int64_t ldx,
                                                         int n_rows, int64_t n_params,
                                                         float *__restrict__ out, float div) {
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= n_params) return;
    float s = x[p];
    for (int r = 1; r < n_rows; ++r) s = s + x[(int64_t)r * ldx + p];
    out[p] = div > 0.f ? s / div : s;
}

// partial[b][a] = sum over columns of block b of (x[a,p] - mean[p])^2
__global__ void __launch_bounds__(256) dev_rows_kernel(const float *__restrict__ x, int64_t ldx,
                                                       int n_rows, int64_t n_params,
                                                       const float *__restrict__ mean,
                                                       float *__restrict__ partial, int nparts) {
    __shared__ float red[4];
    const int ag = blockIdx.y;
    const int64_t span = (n_params + nparts - 1) / nparts;
    const int64_t p0 = (int64_t)blockIdx.x * span;
    const int64_t p1 = p0 + span < n_params ? p0 + span : n_params;
    const float *row = x + (int64_t)ag * ldx;
    float acc = 0.f;
    for (int64_t p = p0 + threadIdx.x; p < p1; p += 256) {
        const float d = row[p] - mean[p];
        acc += d * d;
    }
    for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0)
        partial[(int64_t)blockIdx.x * n_rows + ag] = (red[0] + red[1]) + (red[2] + red[3]);
}

// numpy std(axis=0): mean = sum/N; var = sum((x-mean)^2)/N; std = sqrt(var); then max over p.
__global__ void __launch_bounds__(256) max_column_std_kernel(const float *__restrict__ x,
                                                             int64_t ldx, int n_rows,
                                                             int64_t n_params,
                                                             unsigned int *__restrict__ out_bits) {
    __shared__ float red[4];
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    float sd = 0.f;
    if (p < n_params) {
        float s = x[p];
        for (int r = 1; r < n_rows; ++r) s = s + x[(int64_t)r * ldx + p];
        const float n = (float)n_rows;
        const float m = s / n;
        float d0 = x[p] - m;
        float v = d0 * d0;
        for (int r = 1; r < n_rows; ++r) {
            const float d = x[(int64_t)r * ldx + p] - m;
            v = v + d * d;
        }
        sd = sqrtf(v / n);
    }
    for (int m = 32; m >= 1; m >>= 1) sd = fmaxf(sd, __shfl_xor(sd, m));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sd;
    __syncthreads();
    if (threadIdx.x == 0) {
        const float b = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
        atomicMax(out_bits, __float_as_uint(b));  // non-negative floats order like their bits
    }
}

__global__ void __launch_bounds__(256) step_rows_kernel(const float *__restrict__ x, int64_t ldx,
                                                        const float *__restrict__ g, int64_t ldg,
                                                        float lr, const int32_t *__restrict__ rows,
                                                        int n_sel, int64_t n_params,
                                                        float *__restrict__ out, int64_t ldo) {
    const int i = blockIdx.y;
    const int r = rows[i];
    for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < n_params;
         p += (int64_t)gridDim.x * 256) {
        float v = x[(int64_t)r * ldx + p];
        if (g) v = v - lr * g[(int64_t)r * ldg + p];
        out[(int64_t)i * ldo + p] = v;
    }
}

// Column-tiled form, every peer of a halo exchange in one launch.  The selected rows of all peers
// are concatenated (peer b's in [row0[b], row0[b+1])); one tile's work is L = n_sel * T/4 float4
// lanes (row i, chunk cc).  A workgroup holds `sub` lane groups of lp >= L threads (lp = L
// rounded up to a wave when L < 256, so a 96-row exchange keeps 3 of 4 lanes busy instead of
// 3 of 8), group s walking tiles t0 + s, t0 + s + sub, ... of the workgroup's ONE contiguous run
// of tiles, four tiles' loads in flight before their stores (peer, row and offsets computed
// once; no division in the loop).  x / g tiles are [x_rows][T] / [g_rows][T] blocks; peer b's
// output is its own contiguous block [n_tiles][n_b][T] (one RCCL send buffer).
__global__ void __launch_bounds__(256) step_rows_tiled_kernel(
    const float4 *__restrict__ x, int x_rows, const float4 *__restrict__ g, int g_rows, float lr,
    const int32_t *__restrict__ rows, PackPeers pp, int64_t n_tiles, int tcq, int lp, int sub) {
    const int s = threadIdx.x / lp;
    const int q = blockIdx.x * lp + (threadIdx.x - s * lp);
    const int n_sel = pp.row0[pp.n];
    if (s >= sub || q >= n_sel * tcq) return;
    const int i = q / tcq, cc = q - (q / tcq) * tcq;
    // this row's peer: an unrolled select over the <= kMaxPackPeers table (kernel arguments
    // are not indexed dynamically)
    float4 *ob = pp.out[0];
    int r0 = 0, nb = pp.row0[1];
#pragma unroll
    for (int b = 1; b < kMaxPackPeers; ++b) {
        if (b < pp.n && i >= pp.row0[b]) {
            ob = pp.out[b];
            r0 = pp.row0[b];
            nb = pp.row0[b + 1] - pp.row0[b];
        }
    }
    const int64_t r = rows[i];
    const int64_t xs = (int64_t)x_rows * tcq, gs = (int64_t)g_rows * tcq, os = (int64_t)nb * tcq;
    const float4 *xp = x + r * tcq + cc;
    const float4 *gp = g ? g + r * tcq + cc : nullptr;
    float4 *op = ob + (int64_t)(i - r0) * tcq + cc;
    // one contiguous run of tiles per workgroup: its reads and writes stay inside a few MB
    // instead of striding the whole matrix (pack 104 -> 96 us at c4's rank of 8)
    constexpr int U = 4;
    const int64_t per = (n_tiles + gridDim.y - 1) / gridDim.y;
    const int64_t t0 = (int64_t)blockIdx.y * per;
    const int64_t t_end = t0 + per < n_tiles ? t0 + per : n_tiles;
    typedef float f4 __attribute__((ext_vector_type(4)));
    int64_t t = t0 + s;
    for (; t + (U - 1) * sub < t_end; t += U * sub) {
        float4 v[U], w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v[u] = xp[(t + u * sub) * xs];
            if (gp) w[u] = gp[(t + u * sub) * gs];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (gp) {
                v[u].x = v[u].x - lr * w[u].x;
                v[u].y = v[u].y - lr * w[u].y;
                v[u].z = v[u].z - lr * w[u].z;
                v[u].w = v[u].w - lr * w[u].w;
            }
            // non-temporal: the send blocks are read once, by the peers' RCCL receives (the pack
            // alone 52.9 -> 47.9 us at the c4 rank-of-8 shape, scripts/pack_probe.hip)
            __builtin_nontemporal_store(f4{v[u].x, v[u].y, v[u].z, v[u].w},
                                        reinterpret_cast<f4 *>(op + (t + u * sub) * os));
        }
    }
    for (; t < t_end; t += sub) {
        float4 v = xp[t * xs];
        if (gp) {
            const float4 w = gp[t * gs];
            v.x = v.x - lr * w.x;
            v.y = v.y - lr * w.y;
            v.z = v.z - lr * w.z;
            v.w = v.w - lr * w.w;
        }
        __builtin_nontemporal_store(f4{v.x, v.y, v.z, v.w}, reinterpret_cast<f4 *>(op + t * os));
    }
}

// ---------------------------------------------------------------- local optimizer step
// torch.optim.SGD.step (single-tensor form, torch/optim/sgd.py) over a block of agent rows, in
// the rounding of torch's fused add-with-alpha (one fma per `add(.., alpha=..)`):
//   d = fma(wd, x, g)                                   grad.add(param, alpha=weight_decay)
//   buf = first ? d : fma(1 - dampening, d, mu * buf)   buf.mul_(momentum).add_(grad, alpha=1-damp)
//   d = nesterov ? fma(mu, buf, d) : buf                grad.add(buf, alpha=momentum)
//   out = fma(-lr, d, x)                                param.add_(grad, alpha=-lr)
// out may alias x (in-place step) or be the round's input buffer (step fused into the ping-pong).
typedef float v4f __attribute__((ext_vector_type(4)));

struct SgdParams {
    float lr, mu, damp, wd;
    int first, nesterov;
};

__device__ __forceinline__ float sgd_elem(float x, float g, float &b, const SgdParams &p) {
    float d = p.wd != 0.f ? __builtin_fmaf(p.wd, x, g) : g;
    if (p.mu != 0.f) {
        b = p.first ? d : __builtin_fmaf(1.f - p.damp, d, p.mu * b);
        d = p.nesterov ? __builtin_fmaf(p.mu, b, d) : b;
    }
    return __builtin_fmaf(-p.lr, d, x);
}

template <bool VEC>
__global__ void __launch_bounds__(256) sgd_step_kernel(const float *x, int64_t ldx,
                                                       const float *__restrict__ g, int64_t ldg,
                                                       float *__restrict__ buf, int64_t ldb,
                                                       float *out, int64_t ldo, int64_t n_params,
                                                       SgdParams p) {
    const int r = blockIdx.y;
    const float *xr = x + (int64_t)r * ldx;
    const float *gr = g + (int64_t)r * ldg;
    float *br = buf ? buf + (int64_t)r * ldb : nullptr;
    float *orow = out + (int64_t)r * ldo;
    const int64_t stride = (int64_t)gridDim.x * 256;
    if (VEC) {
        const int64_t n4 = n_params >> 2;
        for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += stride) {
            const v4f xv = __builtin_nontemporal_load(reinterpret_cast<const v4f *>(xr) + i);
            const v4f gv = __builtin_nontemporal_load(reinterpret_cast<const v4f *>(gr) + i);
            v4f bv = br && !p.first ? reinterpret_cast<const v4f *>(br)[i] : v4f{0.f, 0.f, 0.f, 0.f};
            v4f ov;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float b = bv[k];
                ov[k] = sgd_elem(xv[k], gv[k], b, p);
                bv[k] = b;
            }
            if (br) reinterpret_cast<v4f *>(br)[i] = bv;
            reinterpret_cast<v4f *>(orow)[i] = ov;
        }
    } else {
        for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_params; i += stride) {
            float b = br && !p.first ? br[i] : 0.f;
            const float o = sgd_elem(xr[i], gr[i], b, p);
            if (br) br[i] = b;
            orow[i] = o;
        }
    }
}

// ---------------------------------------------------------------- Perron / asyncio round
// One Jacobi iteration on element i of an [R, TP] tile held in LDS (cur), neighbour sums in
// socket order (np.sum(list, axis=0): first term, then left fold), then scale.
template <typename DT>
__device__ __forceinline__ DT perron_update(const DT *cur, int r, int p, int TP,
                                            const int32_t *__restrict__ rp,
                                            const int32_t *__restrict__ col, double eps,
                                            DT conv, const double *conv_rows, bool &fail) {
    const int e0 = rp[r], e1 = rp[r + 1];
    const int cnt = e1 - e0;
    DT s = (DT)0;
    if (cnt > 0) {
        s = cur[col[e0] * TP + p];
        for (int e = e0 + 1; e < e1; ++e) s = s + cur[col[e] * TP + p];
    }
    const DT dcoef = (DT)(1.0 - eps * (double)cnt);
    const DT t1 = cur[r * TP + p] * dcoef;
    const DT t2 = (DT)eps * s;
    const DT yn = t1 + t2;
    if (conv_rows) conv = (DT)conv_rows[r];
    for (int e = e0; e < e1; ++e) {
        const DT v = cur[col[e] * TP + p];
        if (!((yn - v) <= conv)) fail = true;
    }
    return yn;
}

template <typename DT>
__device__ __forceinline__ DT prescale(DT v, const double *weight, double mean_w, int r) {
    if (weight == nullptr) return v;
    const DT t = v * (DT)weight[r];
    return t / (DT)mean_w;
}

// All columns in one tile: the whole round (until every agent has converged) in one launch.
template <typename DT>
__global__ void __launch_bounds__(1024) perron_single_kernel(PerronArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int R = a.n_rows;
    const int TP = (int)a.n_params;
    const int E = R * TP;
    DT *buf0 = reinterpret_cast<DT *>(smem);
    DT *buf1 = buf0 + E;
    int *flags = reinterpret_cast<int *>(buf1 + E);
    DT *y = reinterpret_cast<DT *>(a.y);
    for (int i = threadIdx.x; i < E; i += 1024) {
        const int r = i / TP, p = i - r * TP;
        buf0[i] = prescale<DT>(y[(int64_t)r * a.ldy + p], a.weight, a.mean_weight, r);
    }
    if (threadIdx.x < 2) flags[threadIdx.x] = 0;
    __syncthreads();
    const DT conv = (DT)a.conv_eps;
    DT *cur = buf0, *nxt = buf1;
    int it = 0;
    while (it < a.max_iter) {
        ++it;
        bool fail = false;
        for (int i = threadIdx.x; i < E; i += 1024) {
            const int r = i / TP, p = i - r * TP;
            nxt[i] = perron_update<DT>(cur, r, p, TP, a.rowptr, a.col, a.eps, conv, a.conv_rows, fail);
        }
        if (__any(fail) && (threadIdx.x & 63) == 0) atomicOr(&flags[it & 1], 1);
        __syncthreads();
        DT *t = cur;
        cur = nxt;
        nxt = t;
        const bool done = flags[it & 1] == 0;
        if (threadIdx.x == 0) flags[(it + 1) & 1] = 0;  // next iteration's flag; read after barrier
        __syncthreads();
        if (done) break;
    }
    for (int i = threadIdx.x; i < E; i += 1024) {
        const int r = i / TP, p = i - r * TP;
        y[(int64_t)r * a.ldy + p] = cur[i];
    }
    if (threadIdx.x == 0) a.iters_out[0] = it;
}

// Column tile of TP columns: one iteration, global in -> global out, global not-converged flag.
template <typename DT>
__global__ void __launch_bounds__(1024) perron_step_kernel(PerronArgs a, int TP, const DT *yin,
                                                           int64_t ldin, DT *yout, int64_t ldout,
                                                           int do_prescale) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int R = a.n_rows;
    const int64_t p0 = (int64_t)blockIdx.x * TP;
    const int64_t P = a.n_params;
    DT *cur = reinterpret_cast<DT *>(smem);
    const int E = R * TP;
    for (int i = threadIdx.x; i < E; i += 1024) {
        const int r = i / TP, p = i - r * TP;
        DT v = (DT)0;
        if (p0 + p < P) {
            v = yin[(int64_t)r * ldin + p0 + p];
            if (do_prescale) v = prescale<DT>(v, a.weight, a.mean_weight, r);
        }
        cur[i] = v;
    }
    __syncthreads();
    const DT conv = (DT)a.conv_eps;
    bool fail = false;
    for (int i = threadIdx.x; i < E; i += 1024) {
        const int r = i / TP, p = i - r * TP;
        if (p0 + p >= P) continue;
        bool f = false;
        const DT yn = perron_update<DT>(cur, r, p, TP, a.rowptr, a.col, a.eps, conv, a.conv_rows, f);
        fail |= f;
        yout[(int64_t)r * ldout + p0 + p] = yn;
    }
    if (__any(fail) && (threadIdx.x & 63) == 0) atomicOr(a.notconv, 1);
}

// row-major [n_rows][ld] <-> column-tiled [n_tiles][n_rows][T] (tail columns of the last tile
// are zero-filled when packing and skipped when unpacking)
__global__ void __launch_bounds__(256) tile_convert_kernel(const float *__restrict__ src,
                                                           float *__restrict__ dst, int64_t ld,
                                                           int n_rows, int64_t n_params, int T,
                                                           int to_tiled) {
    const int64_t n_tiles = (n_params + T - 1) / T;
    const int64_t total = n_tiles * n_rows * T;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * 256) {
        const int64_t t = i / ((int64_t)n_rows * T);
        const int64_t rem = i - t * n_rows * T;
        const int64_t r = rem / T;
        const int64_t col = t * T + (rem - r * T);
        if (to_tiled)
            dst[i] = col < n_params ? src[r * ld + col] : 0.f;
        else if (col < n_params)
            dst[r * ld + col] = src[i];
    }
}

}  // namespace

hipError_t launch_tile_convert(const float *src, float *dst, int64_t ld, int n_rows, int64_t n_params,
                               int tile_cols, bool to_tiled, hipStream_t s) {
    const int64_t total = ((n_params + tile_cols - 1) / tile_cols) * n_rows * tile_cols;
    int64_t grid = (total + 255) / 256;
    if (grid > 8192) grid = 8192;
    hipLaunchKernelGGL(tile_convert_kernel, dim3((unsigned)grid), dim3(256), 0, s, src, dst, ld,
                       n_rows, n_params, tile_cols, (int)to_tiled);
    return hipGetLastError();
}

int dev_rows_parts(int64_t n_params) {
    int64_t parts = (n_params + 8191) / 8192;
    if (parts < 1) parts = 1;
    if (parts > 256) parts = 256;
    return (int)parts;
}

hipError_t launch_column_sum(const float *x, int64_t ldx, int n_rows, int64_t n_params,
                             float *colsum, float div, hipStream_t s) {
    hipLaunchKernelGGL(column_sum_kernel, dim3((unsigned)((n_params + 255) / 256)), dim3(256), 0,
                       s, x, ldx, n_rows, n_params, colsum, div);
    return hipGetLastError();
}

hipError_t launch_dev_rows(const float *x, int64_t ldx, int n_rows, int64_t n_params,
                           const float *mean, float *partial, int nparts, hipStream_t s) {
    hipLaunchKernelGGL(dev_rows_kernel, dim3(nparts, n_rows), dim3(256), 0, s, x, ldx, n_rows,
                       n_params, mean, partial, nparts);
    return hipGetLastError();
}

hipError_t launch_max_column_std(const float *x, int64_t ldx, int n_rows, int64_t n_params,
                                 float *out, hipStream_t s) {
    hipError_t e = hipMemsetAsync(out, 0, sizeof(float), s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(max_column_std_kernel, dim3((unsigned)((n_params + 255) / 256)), dim3(256),
                       0, s, x, ldx, n_rows, n_params, reinterpret_cast<unsigned int *>(out));
    return hipGetLastError();
}

hipError_t launch_step_rows(const float *x, int64_t ldx, const float *g, int64_t ldg, float lr,
                            const int32_t *rows, int n_sel, int64_t n_params, float *out,
                            int64_t ldo, hipStream_t s) {
    int64_t bx = (n_params + 255) / 256;
    if (bx > 1024) bx = 1024;
    hipLaunchKernelGGL(step_rows_kernel, dim3((unsigned)bx, n_sel), dim3(256), 0, s, x, ldx, g,
                       ldg, lr, rows, n_sel, n_params, out, ldo);
    return hipGetLastError();
}

hipError_t launch_step_rows_tiled(const float *x, int x_rows, const float *g, int g_rows,
                                  float lr, const int32_t *rows, const PackPeers &pp,
                                  int64_t n_tiles, int tile_cols, hipStream_t s) {
    const int tcq = tile_cols / 4;
    const int64_t lanes = (int64_t)pp.row0[pp.n] * tcq;
    const int64_t bx = (lanes + 255) / 256;
    if (bx > 65535 || pp.n < 1 || pp.n > kMaxPackPeers) return hipErrorInvalidValue;
    // lane groups: one tile's lanes rounded up to a wave, as many groups as fit 256 threads
    const int lp = lanes >= 256 ? 256 : (int)((lanes + 63) / 64 * 64);
    const int sub = 256 / lp;
    // about 2048 resident threads per CU over 256 CUs; each lane group walks >= 4 tiles
    int64_t gy = (256 * 2048) / (bx * 256);
    // DLAMD_PACK_RUN=n (a measurement knob): runs of n tiles per workgroup instead
    static const int64_t pack_run = [] {
        const char *pr = getenv("DLAMD_PACK_RUN");
        return pr ? (int64_t)atoi(pr) : (int64_t)0;
    }();
    if (pack_run > 0) gy = (n_tiles + pack_run - 1) / pack_run;
    const int64_t gmax = (n_tiles + 4 * sub - 1) / (4 * sub);
    if (gy > gmax) gy = gmax;
    if (gy > 65535) gy = 65535;
    if (gy < 1) gy = 1;
    hipLaunchKernelGGL(step_rows_tiled_kernel, dim3((unsigned)bx, (unsigned)gy), dim3(256), 0, s,
                       reinterpret_cast<const float4 *>(x), x_rows,
                       reinterpret_cast<const float4 *>(g), g_rows, lr, rows, pp, n_tiles, tcq, lp, sub);
    return hipGetLastError();
}

hipError_t launch_sgd_step(const float *x, int64_t ldx, const float *g, int64_t ldg, float *buf,
                           int64_t ldb, float *out, int64_t ldo, int n_rows, int64_t n_params,
                           float lr, float mu, float damp, float wd, int first, int nesterov,
                           bool vec, hipStream_t s) {
    const SgdParams p{lr, mu, damp, wd, first, nesterov};
    const int64_t work = vec ? n_params >> 2 : n_params;
    int64_t bx = (work + 255) / 256;
    // ~16 workgroups per CU over all rows, each thread a few float4s (grid-stride)
    int64_t cap = (8192 + n_rows - 1) / n_rows;
    if (cap < 1) cap = 1;
    if (bx > cap) bx = cap;
    if (vec)
        hipLaunchKernelGGL(sgd_step_kernel<true>, dim3((unsigned)bx, n_rows), dim3(256), 0, s, x,
                           ldx, g, ldg, buf, ldb, out, ldo, n_params, p);
    else
        hipLaunchKernelGGL(sgd_step_kernel<false>, dim3((unsigned)bx, n_rows), dim3(256), 0, s, x,
                           ldx, g, ldg, buf, ldb, out, ldo, n_params, p);
    return hipGetLastError();
}

int perron_tile_cols(int dtype, int n_rows, int64_t n_params) {
    const int64_t sz = dtype == 1 ? 8 : 4;
    if (2 * (int64_t)n_rows * n_params * sz + 16 <= kLdsBytes) return (int)n_params;  // single
    int64_t tp = (kLdsBytes - 16) / ((int64_t)n_rows * sz);
    if (tp > 1024) tp = 1024;
    return (int)(tp < 1 ? 0 : tp);
}

hipError_t launch_perron_single(const PerronArgs &a, int dtype, int tile_cols, hipStream_t s) {
    const int64_t sz = dtype == 1 ? 8 : 4;
    const int lds = (int)(2 * (int64_t)a.n_rows * tile_cols * sz + 16);
    const void *k = dtype == 1 ? reinterpret_cast<const void *>(perron_single_kernel<double>)
                               : reinterpret_cast<const void *>(perron_single_kernel<float>);
    hipError_t e = allow_full_lds(k);
    if (e != hipSuccess) return e;
    if (dtype == 1)
        hipLaunchKernelGGL(perron_single_kernel<double>, dim3(1), dim3(1024), lds, s, a);
    else
        hipLaunchKernelGGL(perron_single_kernel<float>, dim3(1), dim3(1024), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_perron_step(const PerronArgs &a, int dtype, int tile_cols, const void *yin,
                              void *yout, bool do_prescale, hipStream_t s) {
    const int64_t sz = dtype == 1 ? 8 : 4;
    const int lds = (int)((int64_t)a.n_rows * tile_cols * sz);
    const unsigned grid = (unsigned)((a.n_params + tile_cols - 1) / tile_cols);
    const int64_t ldin = yin == a.y ? a.ldy : a.n_params;
    const int64_t ldout = yout == a.y ? a.ldy : a.n_params;
    if (dtype == 1) {
        auto k = perron_step_kernel<double>;
        hipError_t e = allow_full_lds(reinterpret_cast<const void *>(k));
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k, dim3(grid), dim3(1024), lds, s, a, tile_cols,
                           static_cast<const double *>(yin), ldin, static_cast<double *>(yout),
                           ldout, (int)do_prescale);
    } else {
        auto k = perron_step_kernel<float>;
        hipError_t e = allow_full_lds(reinterpret_cast<const void *>(k));
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k, dim3(grid), dim3(1024), lds, s, a, tile_cols,
                           static_cast<const float *>(yin), ldin, static_cast<float *>(yout),
                           ldout, (int)do_prescale);
    }
    return hipGetLastError();
}

}  // namespace dl
