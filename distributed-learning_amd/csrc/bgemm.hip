// Batched per-agent GEMMs on fp32 MFMA (v_mfma_f32_16x16x4_f32) for BASELINE config c3:
// every agent trains its own ANNModel (reference networks/ann_model.py:4-45) on its own batch,
// so forward and backward are 256 independent small GEMMs per layer.  One launch covers all
// agents (blockIdx.z = agent); epilogues fuse bias + activation (forward), the activation
// derivative (backward) or the whole cross-entropy head (last layer), and weight gradients land
// directly in the agent's row of G, in the parameter order Mixer flattens (mixer.py:69), ready
// for the fused local step of dl_mix_round.
//
// C[b] (M x N) = op(A[b]) (M x K) . op(B[b]) (K x N)
//   TA: A stored [K][M] (A = stored^T), else [M][K];   TB: B stored [N][K], else [K][N].
// 64x64 block tile, 4 waves each owning a 32x32 quadrant = 2x2 MFMA 16x16 tiles.  The K loop
// walks slices of BK = 32 staged in LDS (k-major, so MFMA fragment reads are conflict-free); the
// next slice is loaded into registers while the current one feeds the MFMAs, so the global
// latency of a slice hides behind 32 MFMAs per wave instead of stalling every step (these
// GEMMs are small -- M = 64 batch rows -- and were latency-bound with one slice in flight).
// f32 MFMA is a k-ordered f32 fma chain (exact fp32, cdna_hip_programming.md §3).
#include <cstdlib>

#include "dl_internal.h"

namespace dl {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 32;

template <bool TA>
__device__ __forceinline__ float load_a(const float *A, int64_t lda, int m, int k, int M, int K) {
    if (m >= M || k >= K) return 0.f;
    return TA ? A[(int64_t)k * lda + m] : A[(int64_t)m * lda + k];
}
template <bool TB>
__device__ __forceinline__ float load_b(const float *B, int64_t ldb, int k, int n, int K, int N) {
    if (k >= K || n >= N) return 0.f;
    return TB ? B[(int64_t)n * ldb + k] : B[(int64_t)k * ldb + n];
}

// element e (< BM*BK) of a slice -> (row, k) of op(A) / (k, col) of op(B); consecutive threads
// walk the stored contiguous dimension, so global loads coalesce
template <bool TA, int BM>
__device__ __forceinline__ void a_coord(int e, int &m, int &k) {
    if (TA) { m = e % BM; k = e / BM; }
    else    { k = e % BK; m = e / BK; }
}
template <bool TB, int BN>
__device__ __forceinline__ void b_coord(int e, int &k, int &n) {
    if (TB) { k = e % BK; n = e / BK; }
    else    { n = e % BN; k = e / BN; }
}

__device__ __forceinline__ float act_fwd(int epi, float z) {
    switch (epi) {
        case EPI_BIAS_RELU: return z > 0.f ? z : 0.f;
        case EPI_BIAS_TANH: return tanhf(z);
        case EPI_BIAS_ELU: return z > 0.f ? z : expm1f(z);
        default: return z;
    }
}

// derivative of the activation expressed through its OUTPUT h (what the forward kept)
__device__ __forceinline__ float act_grad(int epi, float h) {
    switch (epi) {
        case EPI_DRELU: return h > 0.f ? 1.f : 0.f;
        case EPI_DTANH: return 1.f - h * h;
        case EPI_DELU: return h > 0.f ? 1.f : h + 1.f;
        default: return 1.f;
    }
}

// softmax cross-entropy of one logits row held one class per lane (classes <= 64):
// writes dZ = (softmax - onehot) / rows and returns the row's loss / rows (meaningful on all
// lanes).  torch.nn.CrossEntropyLoss, mean reduction.
__device__ __forceinline__ float xent_row(float v, int lane, int classes, int label, int rows,
                                          float *dz_row) {
    float mx = lane < classes ? v : -INFINITY;
    for (int m = 32; m >= 1; m >>= 1) mx = fmaxf(mx, __shfl_xor(mx, m));
    const float e = lane < classes ? expf(v - mx) : 0.f;
    float sum = e;
    for (int m = 32; m >= 1; m >>= 1) sum += __shfl_xor(sum, m);
    if (lane < classes) dz_row[lane] = (e / sum - (lane == label ? 1.f : 0.f)) / (float)rows;
    const float zl = __shfl(v, label);
    return (logf(sum) + mx - zl) / (float)rows;
}

// Block tile BM x BN = (16 TM WM) x (16 TN WN): the 4 waves form a WM x WN grid and each owns
// TM x TN MFMA 16x16 tiles.  Shapes used (launch_bgemm): 64 x 160 (WM 4, TN 10) for the
// batch-row GEMMs -- one workgroup per agent covers a 150-wide layer with 6 % padding instead of
// 28 % -- 160 x 64 (TM 10, WN 4) for the weight gradients (all 150 rows of dW in one tile, so
// each input slice is read once), and 64 x 64 (2 x 2 waves of 2 x 2) for the cross-entropy head.
template <bool TA, bool TB, int WM, int TM, int WN, int TN, bool XENT>
__global__ void __launch_bounds__(256) bgemm_kernel(BgemmArgs p) {
    static_assert(WM * WN == 4, "4 waves");
    constexpr int BM = 16 * TM * WM, BN = 16 * TN * WN;
    constexpr int SA = BM * BK / 256, SB = BN * BK / 256;  // staged elements per thread
    static_assert(SA * 256 == BM * BK && SB * 256 == BN * BK, "slice must split over 256 threads");
    static_assert(!XENT || (BM == 64 && BN == 64), "cross-entropy head uses the 64 x 64 tile");
    __shared__ float As[BK][BM + 4];
    __shared__ float Bs[BK][BN + 4];
    __shared__ float Zs[XENT ? BM : 1][XENT ? BN + 1 : 1];
    __shared__ float lpart[4];
    // XCD-aware work order (cdna_hip_programming.md T1, bijective form): the 1-D grid's
    // blocks round-robin over the 8 XCDs; give each XCD a contiguous run of (agent, tile) work
    // items so the tiles of one agent -- which re-read the same input slab -- share an L2.
    const int gx = (p.N + BN - 1) / BN, gy = (p.M + BM - 1) / BM;
    int tile_x, tile_y, b;
    {
        const int nwg = gridDim.x, id = blockIdx.x;
        const int q = nwg / 8, r = nwg % 8, xcd = id % 8;
        const int w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + id / 8;
        tile_x = w % gx;
        tile_y = (w / gx) % gy;
        b = w / (gx * gy);
    }
    const int m0 = tile_y * BM, n0 = tile_x * BN;
    const float *A = p.A + (int64_t)b * p.sA;
    const float *B = p.B + (int64_t)b * p.sB;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = (wave / WN) * 16 * TM, wn = (wave % WN) * 16 * TN;
    f32x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // bias gradient: row sums of op(A), one thread per tile row, k in order
    const bool want_rs = p.rowsum != nullptr && tile_x == 0;
    float rsum = 0.f;

    float ra[SA], rb[SB];
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < SA; ++i) {
            int m, k;
            a_coord<TA, BM>(tid + i * 256, m, k);
            ra[i] = load_a<TA>(A, p.lda, m0 + m, k0 + k, p.M, p.K);
        }
#pragma unroll
        for (int i = 0; i < SB; ++i) {
            int k, n;
            b_coord<TB, BN>(tid + i * 256, k, n);
            rb[i] = load_b<TB>(B, p.ldb, k0 + k, n0 + n, p.K, p.N);
        }
    };
    load(0);
    for (int k0 = 0; k0 < p.K; k0 += BK) {
#pragma unroll
        for (int i = 0; i < SA; ++i) {
            int m, k;
            a_coord<TA, BM>(tid + i * 256, m, k);
            As[k][m] = ra[i];
        }
#pragma unroll
        for (int i = 0; i < SB; ++i) {
            int k, n;
            b_coord<TB, BN>(tid + i * 256, k, n);
            Bs[k][n] = rb[i];
        }
        __syncthreads();
        if (k0 + BK < p.K) load(k0 + BK);  // in flight during this slice's MFMAs
        if (want_rs && tid < BM) {
#pragma unroll 8
            for (int kk = 0; kk < BK; ++kk) rsum += As[kk][tid];
        }
#pragma unroll
        for (int kk = 0; kk < BK; kk += 4) {
            const int kl = kk + (lane >> 4);
            float af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; ++i) af[i] = As[kl][wm + 16 * i + (lane & 15)];
#pragma unroll
            for (int j = 0; j < TN; ++j) bf[j] = Bs[kl][wn + 16 * j + (lane & 15)];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        __syncthreads();
    }
    if (want_rs && tid < BM && m0 + tid < p.M) p.rowsum[(int64_t)b * p.sR + m0 + tid] = rsum;
    // epilogue: C/D map col = lane & 15, row = 4 * (lane >> 4) + r
    float *C = p.C + (int64_t)b * p.sC;
    const float *bias = p.bias ? p.bias + (int64_t)b * p.sBias : nullptr;
    const float *H = p.H ? p.H + (int64_t)b * p.sH : nullptr;
    if (XENT) {
        // logits of the whole [M x classes] block (one tile per agent) -> LDS, then one wave
        // per row group: softmax cross-entropy, dZ -> C, loss summed in a fixed order
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = wm + 16 * i + 4 * (lane >> 4) + r;
                    const int n = wn + 16 * j + (lane & 15);
                    Zs[m][n] = acc[i][j][r] + ((bias && n < p.N) ? bias[n] : 0.f);
                }
        __syncthreads();
        float lsum = 0.f;
        for (int m = wave; m < p.M; m += 4) {
            const int label = p.labels[(int64_t)b * p.sLab + m];
            lsum += xent_row(Zs[m][lane], lane, p.N, label, p.M, C + (int64_t)m * p.ldc);
        }
        if (lane == 0) lpart[wave] = lsum;
        __syncthreads();
        if (p.loss != nullptr && tid == 0)
            p.loss[b] = (lpart[0] + lpart[1]) + (lpart[2] + lpart[3]);
        return;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + wm + 16 * i + 4 * (lane >> 4) + r;
                const int n = n0 + wn + 16 * j + (lane & 15);
                if (m >= p.M || n >= p.N) continue;
                float v = acc[i][j][r];
                if (p.epi >= EPI_BIAS && p.epi <= EPI_BIAS_ELU) {
                    if (bias) v = v + bias[n];
                    v = act_fwd(p.epi, v);
                } else if (p.epi >= EPI_DRELU && p.epi <= EPI_DELU) {
                    v = v * act_grad(p.epi, H[(int64_t)m * p.ldh + n]);
                }
                C[(int64_t)m * p.ldc + n] = v;
            }
}

// Stand-alone cross-entropy head (dl_xent_grad): dZ = (softmax(z) - onehot(y)) / B per agent
// and the per-agent mean loss.  One workgroup per agent, wave w takes rows w, w+4, ...; the
// loss is summed in a fixed order (deterministic).
__global__ void __launch_bounds__(256) xent_grad_kernel(const float *__restrict__ Z, int64_t sZ,
                                                        const int32_t *__restrict__ y, int64_t sY,
                                                        float *__restrict__ dZ, int64_t sD,
                                                        float *__restrict__ loss, int rows,
                                                        int classes) {
    __shared__ float part[4];
    const int b = blockIdx.x;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    float lsum = 0.f;
    for (int row = wave; row < rows; row += 4) {
        const float *z = Z + (int64_t)b * sZ + (int64_t)row * classes;
        const float v = lane < classes ? z[lane] : 0.f;
        lsum += xent_row(v, lane, classes, y[(int64_t)b * sY + row], rows,
                         dZ + (int64_t)b * sD + (int64_t)row * classes);
    }
    if (lane == 0) part[wave] = lsum;
    __syncthreads();
    if (loss != nullptr && threadIdx.x == 0) loss[b] = (part[0] + part[1]) + (part[2] + part[3]);
}

// Tile shape per GEMM.  Shapes (WM x TM rows, WN x TN cols of 16x16 MFMA tiles):
//   0: 64 x 64  (2x2 waves of 2x2)    1: 32 x 64 (2x1, 2x2)    2: 32 x 32 (2x1, 2x1)
//   3: 64 x 160 (4x1, 1x10)           4: 160 x 64 (1x10, 4x1)  5: 16 x 64 (1x1, 4x1)
// The cross-entropy head always uses shape 0.  DLAMD_BGEMM_SHAPE=<rows<=64>,<rows>64>
// overrides the defaults (a measurement knob).
int bgemm_shape(const BgemmArgs &p) {
    static int small = -1, large = -1;
    if (small < 0) {
        small = 0;
        large = 0;
        if (const char *v = getenv("DLAMD_BGEMM_SHAPE")) {
            if (v[0] >= '0' && v[0] <= '5') small = v[0] - '0';
            if (v[1] == ',' && v[2] >= '0' && v[2] <= '5') large = v[2] - '0';
        }
    }
    return p.M <= 64 ? small : large;
}

template <bool TA, bool TB>
void launch_t(const BgemmArgs &p, hipStream_t s) {
    const unsigned batch = (unsigned)p.batch;
    auto grid = [&](int bm, int bn) {  // 1-D: the kernel maps block ids to (agent, tile)
        return dim3((unsigned)((p.N + bn - 1) / bn) * (unsigned)((p.M + bm - 1) / bm) * batch);
    };
    if (p.epi == EPI_BIAS_XENT) {
        hipLaunchKernelGGL((bgemm_kernel<TA, TB, 2, 2, 2, 2, true>), grid(64, 64), dim3(256), 0, s, p);
        return;
    }
    switch (bgemm_shape(p)) {
        case 1: hipLaunchKernelGGL((bgemm_kernel<TA, TB, 2, 1, 2, 2, false>), grid(32, 64), dim3(256), 0, s, p); break;
        case 2: hipLaunchKernelGGL((bgemm_kernel<TA, TB, 2, 1, 2, 1, false>), grid(32, 32), dim3(256), 0, s, p); break;
        case 3: hipLaunchKernelGGL((bgemm_kernel<TA, TB, 4, 1, 1, 10, false>), grid(64, 160), dim3(256), 0, s, p); break;
        case 4: hipLaunchKernelGGL((bgemm_kernel<TA, TB, 1, 10, 4, 1, false>), grid(160, 64), dim3(256), 0, s, p); break;
        case 5: hipLaunchKernelGGL((bgemm_kernel<TA, TB, 1, 1, 4, 1, false>), grid(16, 64), dim3(256), 0, s, p); break;
        default: hipLaunchKernelGGL((bgemm_kernel<TA, TB, 2, 2, 2, 2, false>), grid(64, 64), dim3(256), 0, s, p); break;
    }
}

}  // namespace

hipError_t launch_bgemm(const BgemmArgs &p, hipStream_t s) {
    if (p.ta && p.tb)
        launch_t<true, true>(p, s);
    else if (p.ta)
        launch_t<true, false>(p, s);
    else if (p.tb)
        launch_t<false, true>(p, s);
    else
        launch_t<false, false>(p, s);
    return hipGetLastError();
}

hipError_t launch_xent_grad(const float *Z, int64_t sZ, const int32_t *y, int64_t sY, float *dZ,
                            int64_t sD, float *loss, int batch, int rows, int classes,
                            hipStream_t s) {
    hipLaunchKernelGGL(xent_grad_kernel, dim3((unsigned)batch), dim3(256), 0, s, Z, sZ, y, sY, dZ,
                       sD, loss, rows, classes);
    return hipGetLastError();
}

}  // namespace dl
