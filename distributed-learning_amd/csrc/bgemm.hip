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
#include "dl_internal.h"

namespace dl {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 64, BN = 64, BK = 32;
constexpr int kStage = BM * BK / 256;  // elements of A (and of B) each thread stages per slice

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
template <bool TA>
__device__ __forceinline__ void a_coord(int e, int &m, int &k) {
    if (TA) { m = e & (BM - 1); k = e / BM; }
    else    { k = e & (BK - 1); m = e / BK; }
}
template <bool TB>
__device__ __forceinline__ void b_coord(int e, int &k, int &n) {
    if (TB) { k = e & (BK - 1); n = e / BK; }
    else    { n = e & (BN - 1); k = e / BN; }
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

template <bool TA, bool TB, bool XENT>
__global__ void __launch_bounds__(256) bgemm_kernel(BgemmArgs p) {
    __shared__ float As[BK][BM + 4];
    __shared__ float Bs[BK][BN + 4];
    __shared__ float rs[4][BM];  // row sums of op(A) per k quarter (bias gradients)
    __shared__ float Zs[XENT ? BM : 1][BN + 1];
    const int b = blockIdx.z;
    const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
    const float *A = p.A + (int64_t)b * p.sA;
    const float *B = p.B + (int64_t)b * p.sB;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
    f32x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool want_rs = p.rowsum != nullptr && blockIdx.x == 0;
    float rsum = 0.f;  // partial row sum of op(A): row tid & 63, k quarter tid >> 6

    float ra[kStage], rb[kStage];
    auto load = [&](int k0) {
#pragma unroll
        for (int i = 0; i < kStage; ++i) {
            const int e = tid + i * 256;
            int m, k, kb, n;
            a_coord<TA>(e, m, k);
            b_coord<TB>(e, kb, n);
            ra[i] = load_a<TA>(A, p.lda, m0 + m, k0 + k, p.M, p.K);
            rb[i] = load_b<TB>(B, p.ldb, k0 + kb, n0 + n, p.K, p.N);
        }
    };
    load(0);
    for (int k0 = 0; k0 < p.K; k0 += BK) {
#pragma unroll
        for (int i = 0; i < kStage; ++i) {
            const int e = tid + i * 256;
            int m, k, kb, n;
            a_coord<TA>(e, m, k);
            b_coord<TB>(e, kb, n);
            As[k][m] = ra[i];
            Bs[kb][n] = rb[i];
        }
        __syncthreads();
        if (k0 + BK < p.K) load(k0 + BK);  // in flight during this slice's MFMAs
        if (want_rs) {
#pragma unroll
            for (int kk = 0; kk < BK / 4; ++kk) rsum += As[(tid >> 6) * (BK / 4) + kk][tid & 63];
        }
#pragma unroll
        for (int kk = 0; kk < BK; kk += 4) {
            const int kl = kk + (lane >> 4);
            const float a0 = As[kl][wm + (lane & 15)];
            const float a1 = As[kl][wm + 16 + (lane & 15)];
            const float b0 = Bs[kl][wn + (lane & 15)];
            const float b1 = Bs[kl][wn + 16 + (lane & 15)];
            acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
        }
        __syncthreads();
    }
    if (want_rs) {
        rs[tid >> 6][tid & 63] = rsum;
        __syncthreads();
        if (tid < 64 && m0 + tid < p.M)
            p.rowsum[(int64_t)b * p.sR + m0 + tid] =
                (rs[0][tid] + rs[1][tid]) + (rs[2][tid] + rs[3][tid]);
    }
    // epilogue: C/D map col = lane & 15, row = 4 * (lane >> 4) + r
    float *C = p.C + (int64_t)b * p.sC;
    const float *bias = p.bias ? p.bias + (int64_t)b * p.sBias : nullptr;
    const float *H = p.H ? p.H + (int64_t)b * p.sH : nullptr;
    if (XENT) {
        // logits of the whole [M x classes] block (one tile per agent) -> LDS, then one wave
        // per row group: softmax cross-entropy, dZ -> C, loss summed in a fixed order
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
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
            lsum += xent_row(Zs[m][lane < BN ? lane : 0], lane, p.N, label, p.M,
                             C + (int64_t)m * p.ldc);
        }
        if (lane == 0) rs[wave][0] = lsum;
        __syncthreads();
        if (p.loss != nullptr && tid == 0)
            p.loss[b] = (rs[0][0] + rs[1][0]) + (rs[2][0] + rs[3][0]);
        return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
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

template <bool TA, bool TB>
void launch_t(const BgemmArgs &p, dim3 grid, hipStream_t s) {
    if (p.epi == EPI_BIAS_XENT)
        hipLaunchKernelGGL((bgemm_kernel<TA, TB, true>), grid, dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL((bgemm_kernel<TA, TB, false>), grid, dim3(256), 0, s, p);
}

}  // namespace

hipError_t launch_bgemm(const BgemmArgs &p, hipStream_t s) {
    dim3 grid((unsigned)((p.N + BN - 1) / BN), (unsigned)((p.M + BM - 1) / BM), (unsigned)p.batch);
    if (p.ta && p.tb)
        launch_t<true, true>(p, grid, s);
    else if (p.ta)
        launch_t<true, false>(p, grid, s);
    else if (p.tb)
        launch_t<false, true>(p, grid, s);
    else
        launch_t<false, false>(p, grid, s);
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
