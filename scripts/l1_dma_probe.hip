// Probe: c3's layer 1 (H1 = relu(x W1^T + b1), per agent 64 x 784 by 784 x 150, 256 agents, one
// 512-thread workgroup per agent) with LDS-DMA staging (global_load_lds_dwordx4 straight into a
// 3-slice LDS ring, no register staging, no split) and the fp32 MFMA (v_mfma_f32_16x16x4_f32) on
// all 8 waves.  The question: does staging by LDS-DMA take layer 1 from the
// 43-46 us of the warp-specialised bf16x6 kernel (csrc/mlp_fused.hip) towards its ~28 us memory
// floor (670 KB per CU at ~24 GB/s per CU, MI355X_MICROARCH.md "Indexed rows") and ~25 us fp32
// MFMA floor?  Times 50 launches with hip events; checks 4 agents against a CPU fp64 reference.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o scripts/bin/l1_dma_probe scripts/l1_dma_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#define CHECK(x)                                                                     \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                \
        }                                                                            \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int NT = 512, MB = 64, DIN = 784, DH = 150, BK = 32;
constexpr int NROWS = 192;                 // W1 rows staged per slice (150 real, clamped pad)
constexpr int SLICE_F4 = (MB + NROWS) * 8; // float4 per slice image: 2048 = 32 KB
#ifndef RING
#define RING 3
#endif
#ifndef FRAG_FIRST
#define FRAG_FIRST 1
#endif
#ifndef ORDER_ST
#define ORDER_ST 0
#endif
#ifndef NODMA
#define NODMA 0   // 1: no staging at all (the MFMA loop on whatever the ring holds)
#endif
#ifndef NOMMA
#define NOMMA 0   // 1: stream the slices only (no fragment reads, no MFMAs)
#endif

#define VMCNT(n) (((n) & 0xF) | (((n) >> 4) << 14) | (0x7 << 4) | (0xF << 8))

// LDS slot of (row, float4 chunk c) inside an image: 8 chunks per row, chunk swizzled by row & 7
__device__ __forceinline__ int slot(int row, int c) { return row * 8 + (c ^ (row & 7)); }

template <int S>
__global__ void __launch_bounds__(NT) l1_dma(const float *__restrict__ X, long ldx,
                                             const float *__restrict__ data, float *__restrict__ H,
                                             int reps) {
    extern __shared__ f32x4 lds[];   // [S][SLICE_F4]
    const int a = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const float *W1 = X + (long)a * ldx;
    const float *x = data + (long)a * MB * DIN;
    const int ns = (DIN + BK - 1) / BK;   // 25
    // DMA instruction i of a slice (32 per slice, 4 per wave): LDS float4 slots [64i, 64i + 64);
    // lane -> slot 64i + lane -> (row, position) -> the chunk that position holds
    auto issue = [&](int sl, int buf) {
        if (NODMA) return;
        const int k0 = sl * BK;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = wave * 4 + j;
            const int sl_lin = i * 64 + lane;
            const int row = sl_lin >> 3, pos = sl_lin & 7;
            const int c = pos ^ (row & 7);
            int k = k0 + 4 * c;
            k = k < DIN ? k : DIN - 4;            // K tail: clamped (zeroed in the A fragment)
            const float *src = row < MB ? x + (long)row * DIN + k
                                        : W1 + (long)(row - MB < DH ? row - MB : DH - 1) * DIN + k;
            __builtin_amdgcn_global_load_lds((const void *)src,
                                             (lds_void *)(lds + buf * SLICE_F4 + i * 64), 16, 0, 0);
        }
    };
    // wave w: M-tile (w & 3) x N-tiles 5 (w >> 2) .. + 4 (16 x 16 each)
    const int mt = wave & 3, nt0 = 5 * (wave >> 2);
    const int r16 = lane & 15, g = lane >> 4;   // lane group g supplies k = 8g + s at step s
    float bias[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) {
        const int n = 16 * (nt0 + t) + r16;
        bias[t] = n < DH ? W1[DH * DIN + n] : 0.f;   // b1 follows W1 (Mixer order)
    }
    for (int rep = 0; rep < reps; ++rep) {
        f32x4 acc[5];
#pragma unroll
        for (int t = 0; t < 5; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < S - 1; ++s) issue(s, s);
        for (int sl = 0; sl < ns; ++sl) {
            // this wave's DMAs of slice sl done (the later S - 2 slices' stay in flight), then
            // every wave's: the barrier also retires every wave's reads of slice sl - 1's buffer
            // outstanding after slice sl's 4 DMAs: the later issued slices' (4 each)
            const int later = (sl + S - 2 < ns ? S - 2 : ns - 1 - sl);
            if (later >= 2) __builtin_amdgcn_s_waitcnt(VMCNT(8));
            else if (later == 1) __builtin_amdgcn_s_waitcnt(VMCNT(4));
            else __builtin_amdgcn_s_waitcnt(VMCNT(0));
            __builtin_amdgcn_s_barrier();
            if (sl + S - 1 < ns) issue(sl + S - 1, (sl + S - 1) % S);
            if (NOMMA) continue;
            const f32x4 *img = lds + (sl % S) * SLICE_F4;
            const int arow = 16 * mt + r16;
            f32x4 a0 = img[slot(arow, 2 * g)], a1 = img[slot(arow, 2 * g + 1)];
            // every fragment of the slice read first, one wait, then the 40 MFMAs back to back
            // (read-wait-4 MFMAs per N-tile left the matrix core idle for an LDS latency each)
            f32x4 b[5][2];
#pragma unroll
            for (int t = 0; t < 5; ++t) {
                const int brow = MB + 16 * (nt0 + t) + r16;
                b[t][0] = img[slot(brow, 2 * g)];
                b[t][1] = img[slot(brow, 2 * g + 1)];
            }
            if (sl == ns - 1 && g >= 2) a0 = a1 = f32x4{0.f, 0.f, 0.f, 0.f};   // k >= 784
#if FRAG_FIRST
            __builtin_amdgcn_sched_barrier(0);
#endif
#if ORDER_ST   // k step outer, N-tile inner: five independent accumulators between dependent MFMAs
#pragma unroll
            for (int s = 0; s < 8; ++s)
#pragma unroll
                for (int t = 0; t < 5; ++t)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(s < 4 ? a0[s] : a1[s - 4],
                                                                  b[t][s >> 2][s & 3], acc[t], 0, 0, 0);
#else
#pragma unroll
            for (int t = 0; t < 5; ++t) {
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s], b[t][0][s], acc[t], 0, 0, 0);
#pragma unroll
                for (int s = 0; s < 4; ++s)
                    acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[s], b[t][1][s], acc[t], 0, 0, 0);
            }
#endif
        }
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();
        // C/D map of 16x16x4: lane (col = lane & 15, rows 4 * (lane >> 4) + r)
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            const int n = 16 * (nt0 + t) + r16;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = 16 * mt + 4 * g + r;
                const float v = acc[t][r] + bias[t];
                if (n < DH) H[((long)a * MB + m) * DH + n] = v > 0.f ? v : 0.f;
            }
        }
    }
}

// K-major storage (x^T [784][64], W1^T [784][150] per agent): a K slice of 32 is two contiguous
// blocks (8 KB + 18.75 KB) instead of 224 row segments of 128 B.  LDS images [k][64] and
// [k][150] filled linearly by LDS-DMA (27 wave-instructions per slice, 4 per wave, the extra
// ones re-load the last granule); fragments by ds_read_b32 (consecutive lanes, consecutive
// rows: conflict-free).
constexpr int XT_F4 = BK * MB / 4;                  // 512
constexpr int WT_F4 = BK * DH / 4;                  // 1200
constexpr int KSLICE_F4 = XT_F4 + 1216 + 64;        // image 1728 float4 (27 KB) + a spare pad
template <int S>
__global__ void __launch_bounds__(NT) l1_dma_kmaj(const float *__restrict__ XT, long ldx,
                                                  const float *__restrict__ dataT,
                                                  float *__restrict__ H) {
    extern __shared__ f32x4 lds[];
    const int a = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const float *W1T = XT + (long)a * ldx;             // [784][150]
    const float *xT = dataT + (long)a * MB * DIN;      // [784][64]
    const int ns = (DIN + BK - 1) / BK;
    auto issue = [&](int sl, int buf) {
        const long k0 = (long)sl * BK;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = wave * 4 + j;                // 0..31: 8 x^T, 19 W1^T, 5 spare
            int f = i * 64 + lane;                     // float4 index inside the slice image
            const f32x4 *src;
            if (i < 8) {
                src = reinterpret_cast<const f32x4 *>(xT + k0 * MB) + f;
                if (k0 * MB + 4 * f >= (long)DIN * MB) src = reinterpret_cast<const f32x4 *>(xT) ;
            } else {
                int fw = f - XT_F4;
                if (fw >= WT_F4 || k0 * DH + 4 * fw >= (long)DIN * DH) fw = 0;   // spare / tail
                src = reinterpret_cast<const f32x4 *>(W1T + k0 * DH) + fw;
                if (k0 * DH + 4 * fw >= (long)DIN * DH) src = reinterpret_cast<const f32x4 *>(W1T);
            }
            if (i >= 27) f = XT_F4 + 1216;             // spare granules: the pad area
            __builtin_amdgcn_global_load_lds((const void *)src,
                                             (lds_void *)(lds + buf * KSLICE_F4 + (f & ~63)), 16,
                                             0, 0);
        }
    };
    const int mt = wave & 3, nt0 = 5 * (wave >> 2);
    const int r16 = lane & 15, g = lane >> 4;
    float bias[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) {
        const int n = 16 * (nt0 + t) + r16;
        bias[t] = n < DH ? W1T[DH * DIN + n] : 0.f;
    }
    f32x4 acc[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < S - 1; ++s) issue(s, s);
    for (int sl = 0; sl < ns; ++sl) {
        const int later = (sl + S - 2 < ns ? S - 2 : ns - 1 - sl);
        if (later >= 2) __builtin_amdgcn_s_waitcnt(VMCNT(8));
        else if (later == 1) __builtin_amdgcn_s_waitcnt(VMCNT(4));
        else __builtin_amdgcn_s_waitcnt(VMCNT(0));
        __builtin_amdgcn_s_barrier();
        if (sl + S - 1 < ns) issue(sl + S - 1, (sl + S - 1) % S);
        if (NOMMA) continue;
        const float *img = reinterpret_cast<const float *>(lds + (sl % S) * KSLICE_F4);
        const float *wimg = img + 4 * XT_F4;
        const int steps = DIN - sl * BK >= BK ? BK / 4 : (DIN - sl * BK) / 4;
        for (int j = 0; j < steps; ++j) {
            const int k = 4 * j + g;
            const float av = img[k * MB + 16 * mt + r16];
#pragma unroll
            for (int t = 0; t < 5; ++t) {
                const int n = 16 * (nt0 + t) + r16;
                const float bv = wimg[k * DH + (n < DH ? n : DH - 1)];
                acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[t], 0, 0, 0);
            }
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 5; ++t) {
        const int n = 16 * (nt0 + t) + r16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = 16 * mt + 4 * g + r;
            const float v = acc[t][r] + bias[t];
            if (n < DH) H[((long)a * MB + m) * DH + n] = v > 0.f ? v : 0.f;
        }
    }
}

int main(int argc, char **argv) {
    const int N = 256;
    const long P = (long)DH * DIN + DH + 2 * (DH * DH + DH) + 10 * DH + 10;
    const long ld = (P + 63) / 64 * 64;
    std::vector<float> hx(N * ld), hd((long)N * MB * DIN);
    unsigned s = 1;
    auto rnd = [&] { s = s * 1664525u + 1013904223u; return ((s >> 8) & 0xffff) / 65536.f - 0.5f; };
    for (auto &v : hx) v = 0.1f * rnd();
    for (auto &v : hd) v = rnd();
    float *X, *D, *H;
    CHECK(hipMalloc(&X, hx.size() * 4));
    CHECK(hipMalloc(&D, hd.size() * 4));
    CHECK(hipMalloc(&H, (long)N * MB * DH * 4));
    CHECK(hipMemcpy(X, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(D, hd.data(), hd.size() * 4, hipMemcpyHostToDevice));
    auto k = l1_dma<RING>;
    const int lds = RING * SLICE_F4 * 16;
    CHECK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    hipLaunchKernelGGL(k, dim3(N), dim3(NT), lds, 0, X, ld, D, H, 1);
    CHECK(hipDeviceSynchronize());
    // check 4 agents in fp64
    std::vector<float> hh((long)N * MB * DH);
    CHECK(hipMemcpy(hh.data(), H, hh.size() * 4, hipMemcpyDeviceToHost));
    double maxrel = 0;
    for (int a : {0, 77, 128, 255})
        for (int m = 0; m < MB; ++m)
            for (int n = 0; n < DH; ++n) {
                double acc = hx[a * ld + DH * DIN + n], nrm = std::fabs(acc);
                for (int kk = 0; kk < DIN; ++kk) {
                    const double p = (double)hd[((long)a * MB + m) * DIN + kk] * hx[a * ld + (long)n * DIN + kk];
                    acc += p;
                    nrm += std::fabs(p);
                }
                const double want = acc > 0 ? acc : 0;
                const double got = hh[((long)a * MB + m) * DH + n];
                maxrel = std::fmax(maxrel, std::fabs(got - want) / nrm);
            }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int iters = 50;
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k, dim3(N), dim3(NT), lds, 0, X, ld, D, H, 1);
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k, dim3(N), dim3(NT), lds, 0, X, ld, D, H, 1);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    const double bytes = (double)N * (MB + DH) * DIN * 4;
    printf("l1_dma ring=%d: %.2f us per launch (256 agents), %.2f GB/s per CU, %.1f TB/s; "
           "max |err|/sum|terms| vs fp64 = %.2e\n",
           RING, us, bytes / 256 / (us * 1e-6) / 1e9, bytes / (us * 1e-6) / 1e12, maxrel);
    // ---- K-major storage of the same data
    std::vector<float> hxt(N * ld, 0.f), hdt((long)N * MB * DIN);
    for (int a = 0; a < N; ++a) {
        for (int n = 0; n < DH; ++n)
            for (int kk = 0; kk < DIN; ++kk) hxt[a * ld + (long)kk * DH + n] = hx[a * ld + (long)n * DIN + kk];
        for (int n = 0; n < DH; ++n) hxt[a * ld + DH * DIN + n] = hx[a * ld + DH * DIN + n];
        for (int m = 0; m < MB; ++m)
            for (int kk = 0; kk < DIN; ++kk)
                hdt[((long)a * DIN + kk) * MB + m] = hd[((long)a * MB + m) * DIN + kk];
    }
    CHECK(hipMemcpy(X, hxt.data(), hxt.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(D, hdt.data(), hdt.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemset(H, 0, (long)N * MB * DH * 4));
    auto k2 = l1_dma_kmaj<RING>;
    const int lds2 = RING * KSLICE_F4 * 16;
    CHECK(hipFuncSetAttribute((const void *)k2, hipFuncAttributeMaxDynamicSharedMemorySize, lds2));
    hipLaunchKernelGGL(k2, dim3(N), dim3(NT), lds2, 0, X, ld, D, H);
    CHECK(hipDeviceSynchronize());
    std::vector<float> hh2((long)N * MB * DH);
    CHECK(hipMemcpy(hh2.data(), H, hh2.size() * 4, hipMemcpyDeviceToHost));
    double maxd = 0;
    for (long i = 0; i < (long)hh.size(); ++i) maxd = std::fmax(maxd, std::fabs(hh2[i] - hh[i]) / (std::fabs(hh[i]) + 1e-3));
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k2, dim3(N), dim3(NT), lds2, 0, X, ld, D, H);
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k2, dim3(N), dim3(NT), lds2, 0, X, ld, D, H);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us2 = ms * 1e3 / iters;
    printf("l1_dma_kmajor ring=%d: %.2f us per launch, %.2f GB/s per CU, %.1f TB/s; max rel diff "
           "vs the row-major kernel %.2e\n",
           RING, us2, bytes / 256 / (us2 * 1e-6) / 1e9, bytes / (us2 * 1e-6) / 1e12, maxd);
    return 0;
}
