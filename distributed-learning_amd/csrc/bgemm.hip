// Batched per-agent GEMMs on fp32 MFMA (v_mfma_f32_16x16x4_f32) for BASELINE config c3:
// every agent trains its own ANNModel (reference networks/ann_model.py:4-45) on its own batch,
// so forward and backward are 256 independent small GEMMs per layer.  One launch covers all
// agents (blockIdx.z = agent); epilogues fuse bias + activation (forward) or the activation
// derivative (backward), and weight gradients land directly in the agent's row of G, in the
// parameter order Mixer flattens (mixer.py:69), ready for the fused local step of dl_mix_round.
//
// C[b] (M x N) = op(A[b]) (M x K) . op(B[b]) (K x N)
//   TA: A stored [K][M] (A = stored^T), else [M][K];   TB: B stored [N][K], else [K][N].
// 64x64 block tile, K-step 16 staged in LDS (k-major, so MFMA fragment reads are conflict-free),
// 4 waves each owning a 32x32 quadrant = 2x2 MFMA 16x16 tiles.  f32 MFMA is a k-ordered f32 fma
// chain (exact fp32, cdna_hip_programming.md §3).
#include "dl_internal.h"

namespace dl {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 64, BN = 64, BK = 16;

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

template <bool TA, bool TB>
__global__ void __launch_bounds__(256) bgemm_kernel(BgemmArgs p) {
    __shared__ float As[BK][BM + 4];
    __shared__ float Bs[BK][BN + 4];
    __shared__ float rs[4][BM];  // row sums of op(A) per wave quarter (bias gradients)
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
    float rsum = 0.f;  // thread's partial row sum of op(A) (rows tid & 63, k quarter tid >> 6)

    for (int k0 = 0; k0 < p.K; k0 += BK) {
        // stage A (64 x 16) and B (16 x 64): 1024 elements each, 4 per thread
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int e = tid + i * 256;
            int m, k;
            if (TA) {  // consecutive threads along m (contiguous in memory)
                m = e & 63;
                k = e >> 6;
            } else {  // consecutive threads along k
                k = e & 15;
                m = e >> 4;
            }
            As[k][m] = load_a<TA>(A, p.lda, m0 + m, k0 + k, p.M, p.K);
            int kb, n;
            if (TB) {
                kb = e & 15;
                n = e >> 4;
            } else {
                n = e & 63;
                kb = e >> 6;
            }
            Bs[kb][n] = load_b<TB>(B, p.ldb, k0 + kb, n0 + n, p.K, p.N);
        }
        __syncthreads();
        if (want_rs) {
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) rsum += As[(tid >> 6) * 4 + kk][tid & 63];
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
                } else if (p.epi >= EPI_DRELU) {
                    v = v * act_grad(p.epi, H[(int64_t)m * p.ldh + n]);
                }
                C[(int64_t)m * p.ldc + n] = v;
            }
}

// Cross-entropy head: dZ = (softmax(z) - onehot(y)) / B per agent, and the per-agent mean loss
// (torch.nn.CrossEntropyLoss, mean reduction).  One wave per (agent, row); classes <= 64.
__global__ void __launch_bounds__(256) xent_grad_kernel(const float *__restrict__ Z, int64_t sZ,
                                                        const int32_t *__restrict__ y, int64_t sY,
                                                        float *__restrict__ dZ, int64_t sD,
                                                        float *__restrict__ loss, int rows,
                                                        int classes) {
    const int b = blockIdx.y;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (row >= rows) return;
    const float *z = Z + (int64_t)b * sZ + (int64_t)row * classes;
    const float v = lane < classes ? z[lane] : -INFINITY;
    float mx = v;
    for (int m = 32; m >= 1; m >>= 1) mx = fmaxf(mx, __shfl_xor(mx, m));
    const float e = lane < classes ? expf(v - mx) : 0.f;
    float sum = e;
    for (int m = 32; m >= 1; m >>= 1) sum += __shfl_xor(sum, m);
    const int label = y[(int64_t)b * sY + row];
    if (lane < classes) {
        const float pr = e / sum;
        dZ[(int64_t)b * sD + (int64_t)row * classes + lane] =
            (pr - (lane == label ? 1.f : 0.f)) / (float)rows;
    }
    if (loss != nullptr && lane == label)
        atomicAdd(&loss[b], (logf(sum) + mx - v) / (float)rows);
}

}  // namespace

hipError_t launch_bgemm(const BgemmArgs &p, hipStream_t s) {
    dim3 grid((unsigned)((p.N + BN - 1) / BN), (unsigned)((p.M + BM - 1) / BM), (unsigned)p.batch);
    if (p.ta && p.tb)
        hipLaunchKernelGGL((bgemm_kernel<true, true>), grid, dim3(256), 0, s, p);
    else if (p.ta)
        hipLaunchKernelGGL((bgemm_kernel<true, false>), grid, dim3(256), 0, s, p);
    else if (p.tb)
        hipLaunchKernelGGL((bgemm_kernel<false, true>), grid, dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL((bgemm_kernel<false, false>), grid, dim3(256), 0, s, p);
    return hipGetLastError();
}

hipError_t launch_xent_grad(const float *Z, int64_t sZ, const int32_t *y, int64_t sY, float *dZ,
                            int64_t sD, float *loss, int batch, int rows, int classes,
                            hipStream_t s) {
    if (loss) {
        hipError_t e = hipMemsetAsync(loss, 0, sizeof(float) * batch, s);
        if (e != hipSuccess) return e;
    }
    dim3 grid((unsigned)((rows + 3) / 4), (unsigned)batch);
    hipLaunchKernelGGL(xent_grad_kernel, grid, dim3(256), 0, s, Z, sZ, y, sY, dZ, sD, loss, rows,
                       classes);
    return hipGetLastError();
}

}  // namespace dl
