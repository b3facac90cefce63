// Probe: c3's layer 1 (H1 = relu(x W1^T + b1), 256 agents x [64 x 784] by
// [784 x 150], one 512-thread workgroup per agent) with LDS-DMA staging of the RAW fp32 slices
// (global_load_lds_dwordx4 into an S-slice ring, no producer waves, no register staging) and the
// bf16x6 products on the bf16 matrix cores, every wave splitting its own fragments in registers
// (8 consecutive k of one row = two ds_read_b128 -> three bf16x8 planes).  r10's
// scripts/l1_dma_probe.hip paired the same ring with the fp32 MFMA (47-48 us: the fp32 matrix
// work alone 39.5 us) and streamed the slices alone in 27.6 us; the kernel's layer 1 (4 producer
// waves load + split into bf16 planes, 4 MFMA waves) measured 46.2 us.  Here all 8 waves run
// 30 bf16 MFMAs per slice (6/16 of the fp32 time) and split 6 fragments each.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o scripts/bin/l1_x6_dma_probe scripts/l1_x6_dma_probe.hip
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
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int NT = 512, MB = 64, DIN = 784, DH = 150, BK = 32;
constexpr int NROWS = 192;                 // W1 rows staged per slice (150 real, clamped pad)
constexpr int SLICE_F4 = (MB + NROWS) * 8; // float4 per slice image: 2048 = 32 KB

#define VMCNT(n) (((n) & 0xF) | (((n) >> 4) << 14) | (0x7 << 4) | (0xF << 8))

__device__ __forceinline__ int slot(int row, int c) { return row * 8 + (c ^ (row & 7)); }

__device__ __forceinline__ void split2(float x0, float x1, bf16x2 &h, bf16x2 &m, bf16x2 &l) {
    h = bf16x2{(__bf16)x0, (__bf16)x1};
    const float r0 = x0 - (float)h[0], r1 = x1 - (float)h[1];
    m = bf16x2{(__bf16)r0, (__bf16)r1};
    l = bf16x2{(__bf16)(r0 - (float)m[0]), (__bf16)(r1 - (float)m[1])};
}
__device__ __forceinline__ void split8(const f32x4 &x0, const f32x4 &x1, bf16x8 &h, bf16x8 &m,
                                       bf16x8 &l) {
    bf16x2 h0, m0, l0, h1, m1, l1, h2, m2, l2, h3, m3, l3;
    split2(x0.x, x0.y, h0, m0, l0);
    split2(x0.z, x0.w, h1, m1, l1);
    split2(x1.x, x1.y, h2, m2, l2);
    split2(x1.z, x1.w, h3, m3, l3);
    h = bf16x8{h0[0], h0[1], h1[0], h1[1], h2[0], h2[1], h3[0], h3[1]};
    m = bf16x8{m0[0], m0[1], m1[0], m1[1], m2[0], m2[1], m3[0], m3[1]};
    l = bf16x8{l0[0], l0[1], l1[0], l1[1], l2[0], l2[1], l3[0], l3[1]};
}
__device__ __forceinline__ f32x4 mfma_bf(const bf16x8 &a, const bf16x8 &b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void mfma_x6(const bf16x8 &ah, const bf16x8 &am, const bf16x8 &al,
                                        const bf16x8 &bh, const bf16x8 &bm, const bf16x8 &bl,
                                        f32x4 &big, f32x4 &small) {
    small = mfma_bf(al, bh, small);
    small = mfma_bf(ah, bl, small);
    small = mfma_bf(am, bm, small);
    small = mfma_bf(am, bh, small);
    small = mfma_bf(ah, bm, small);
    big = mfma_bf(ah, bh, big);
}

// MODE 0: DMA ring + per-wave split + bf16x6 MFMAs; 1: the slices streamed only; 2: no DMA
// (the split + MFMA loop on whatever the ring holds)
template <int S, int MODE>
__global__ void __launch_bounds__(NT) l1_x6(const float *__restrict__ X, long ldx,
                                            const float *__restrict__ data, float *__restrict__ H) {
    extern __shared__ f32x4 lds[];   // [S][SLICE_F4]
    const int a = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const float *W1 = X + (long)a * ldx;
    const float *x = data + (long)a * MB * DIN;
    const int ns = (DIN + BK - 1) / BK;   // 25
    auto issue = [&](int sl, int buf) {
        if (MODE == 2) return;
        const int k0 = sl * BK;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = wave * 4 + j;
            const int sl_lin = i * 64 + lane;
            const int row = sl_lin >> 3, pos = sl_lin & 7;
            const int c = pos ^ (row & 7);
            int k = k0 + 4 * c;
            k = k < DIN ? k : DIN - 4;
            const float *src = row < MB ? x + (long)row * DIN + k
                                        : W1 + (long)(row - MB < DH ? row - MB : DH - 1) * DIN + k;
            __builtin_amdgcn_global_load_lds((const void *)src,
                                             (lds_void *)(lds + buf * SLICE_F4 + i * 64), 16, 0, 0);
        }
    };
    const int mt = wave & 3, nt0 = 5 * (wave >> 2);
    const int r16 = lane & 15, g = lane >> 4;
    float bias[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) {
        const int n = 16 * (nt0 + t) + r16;
        bias[t] = n < DH ? W1[DH * DIN + n] : 0.f;
    }
    f32x4 acc[5], sml[5];
#pragma unroll
    for (int t = 0; t < 5; ++t) acc[t] = sml[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < S - 1; ++s) issue(s, s);
    for (int sl = 0; sl < ns; ++sl) {
        const int later = (sl + S - 2 < ns ? S - 2 : ns - 1 - sl);
        if (later >= 3) __builtin_amdgcn_s_waitcnt(VMCNT(12));
        else if (later == 2) __builtin_amdgcn_s_waitcnt(VMCNT(8));
        else if (later == 1) __builtin_amdgcn_s_waitcnt(VMCNT(4));
        else __builtin_amdgcn_s_waitcnt(VMCNT(0));
        __builtin_amdgcn_s_barrier();
        if (sl + S - 1 < ns) issue(sl + S - 1, (sl + S - 1) % S);
        if (MODE == 1) continue;
        const f32x4 *img = lds + (sl % S) * SLICE_F4;
        const int arow = 16 * mt + r16;
        f32x4 a0 = img[slot(arow, 2 * g)], a1 = img[slot(arow, 2 * g + 1)];
        f32x4 b[5][2];
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            const int brow = MB + 16 * (nt0 + t) + r16;
            b[t][0] = img[slot(brow, 2 * g)];
            b[t][1] = img[slot(brow, 2 * g + 1)];
        }
        if (sl == ns - 1 && g >= 2) a0 = a1 = f32x4{0.f, 0.f, 0.f, 0.f};   // k >= 784
        bf16x8 ah, am, al;
        split8(a0, a1, ah, am, al);
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            bf16x8 bh, bm, bl;
            split8(b[t][0], b[t][1], bh, bm, bl);
            mfma_x6(ah, am, al, bh, bm, bl, acc[t], sml[t]);
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 5; ++t) {
        const int n = 16 * (nt0 + t) + r16;
        acc[t] += sml[t];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = 16 * mt + 4 * g + r;
            const float v = acc[t][r] + bias[t];
            if (n < DH) H[((long)a * MB + m) * DH + n] = v > 0.f ? v : 0.f;
        }
    }
}

// ---- warp-specialised forms (the kernel's layer-1 structure): waves 4-7 produce bf16 planes of
// slice s (x [64][32] and W1 [160][32], three planes each, l1_wofs layout) while waves 0-3 run
// slice s - 1's 60 bf16 MFMAs (M-tile = wave, all ten N-tiles); two plane images, one barrier per
// slice.  DMA = false: the kernel's producers (register-staged loads, L1_RING = 4 sets in
// flight).  DMA = true: the producers DMA raw fp32 slices into a 2-slot LDS ring and split them
// from LDS (one iteration of lead: slice s + 2 issued after the barrier that retires slice s's
// raw reads).
constexpr int XPL = MB * BK * 2;                 // 4096 B per x plane
constexpr int L1P = 160 * BK * 2;                // 10240 B per W1 plane
constexpr int IMGB = 3 * XPL + 3 * L1P;          // 43008
constexpr int RAW_F4 = (MB + 160) * 8;           // 1792 float4 = 28 KB per raw slice
__device__ __forceinline__ uint32_t l1_wofs(int n, int k) {
    return (uint32_t)(n * 64 + ((((k >> 3) ^ (n >> 2)) & 3) << 4) + (k & 7) * 2);
}
__device__ __forceinline__ void split4(const f32x4 &x, bf16x4 &h, bf16x4 &m, bf16x4 &l) {
    bf16x2 h0, m0, l0, h1, m1, l1;
    split2(x.x, x.y, h0, m0, l0);
    split2(x.z, x.w, h1, m1, l1);
    h = bf16x4{h0[0], h0[1], h1[0], h1[1]};
    m = bf16x4{m0[0], m0[1], m1[0], m1[1]};
    l = bf16x4{l0[0], l0[1], l1[0], l1[1]};
}

// BLK: x and W1 slice-blocked ([25][64][32] and [25][150][32] per agent, the last slice zero
// padded; b1 after W1's blocks): every slice of either operand is one contiguous block
template <bool DMA, bool BLK = false>
__global__ void __launch_bounds__(NT) l1_ws(const float *__restrict__ X, long ldx,
                                            const float *__restrict__ data, float *__restrict__ H) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char *img0 = smem;                                        // two plane images
    f32x4 *raw = reinterpret_cast<f32x4 *>(smem + 2 * IMGB);  // DMA: two raw slots
    const int a = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const float *W1 = X + (long)a * ldx;
    const float *x = data + (long)a * (BLK ? 25 * MB * BK : MB * DIN);
    const int ns = (DIN + BK - 1) / BK, din = DIN, dh = DH;
    if (wave >= 4) {
        const int pt = tid - NT / 2;
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        // write one float4 of (row, chunk c) of slice k0 as planes into img
        auto put = [&](char *img, int row, int c, int k0, f32x4 v) {
            bf16x4 h, m, l;
            if (row < MB) {
                split4(k0 + 4 * c < din ? v : z, h, m, l);
                const uint32_t o = l1_wofs(row, 4 * c);
                *reinterpret_cast<bf16x4 *>(img + o) = h;
                *reinterpret_cast<bf16x4 *>(img + XPL + o) = m;
                *reinterpret_cast<bf16x4 *>(img + 2 * XPL + o) = l;
            } else {
                const int n = row - MB;
                split4(n < dh && k0 + 4 * c < din ? v : z, h, m, l);
                const uint32_t o = l1_wofs(n, 4 * c);
                char *wpl = img + 3 * XPL;
                *reinterpret_cast<bf16x4 *>(wpl + o) = h;
                *reinterpret_cast<bf16x4 *>(wpl + L1P + o) = m;
                *reinterpret_cast<bf16x4 *>(wpl + 2 * L1P + o) = l;
            }
        };
        if constexpr (DMA) {
            auto issue = [&](int sl) {   // 28 wave-instructions per slice, 7 per producer wave
                const int k0 = sl * BK;
                f32x4 *dst = raw + (sl & 1) * RAW_F4;
#pragma unroll
                for (int j = 0; j < 7; ++j) {
                    const int i = (wave - 4) * 7 + j;
                    const int e = i * 64 + lane, row = e >> 3, c = (e & 7) ^ (row & 7);
                    int k = k0 + 4 * c;
                    k = k < din ? k : din - 4;
                    const float *src = row < MB ? x + (long)row * din + k
                                                : W1 + (long)(row - MB < dh ? row - MB : dh - 1) * din + k;
                    __builtin_amdgcn_global_load_lds((const void *)src, (lds_void *)(dst + i * 64),
                                                     16, 0, 0);
                }
            };
            issue(0);
            issue(1);
            __builtin_amdgcn_s_waitcnt(VMCNT(7));   // own slice-0 DMAs
            __builtin_amdgcn_s_barrier();           // everyone's
            for (int sl = 0; sl < ns; ++sl) {
                const f32x4 *src = raw + (sl & 1) * RAW_F4;
                f32x4 v[7];
#pragma unroll
                for (int i = 0; i < 7; ++i) v[i] = src[pt + i * 256];
#pragma unroll
                for (int i = 0; i < 7; ++i) {
                    const int e = pt + i * 256, row = e >> 3, c = (e & 7) ^ (row & 7);
                    put(img0 + (sl & 1) * IMGB, row, c, sl * BK, v[i]);
                }
                // own DMAs of slice sl + 1 landed, then the barrier: everyone's landed, every
                // raw read of slice sl retired, every consumer done with the other image
                __builtin_amdgcn_s_waitcnt(VMCNT(0));
                __builtin_amdgcn_s_barrier();
                if (sl + 2 < ns) issue(sl + 2);
            }
        } else {
            constexpr int R = 4;
            f32x4 rx[R][2], rw[R][5];
            auto load = [&](int set, int sl) {
                const int k0 = sl * BK;
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int e = pt + i * 256, r = e / 8, c = 4 * (e % 8);
                    rx[set][i] = BLK ? *reinterpret_cast<const f32x4 *>(x + ((long)sl * MB + r) * BK + c)
                                     : *reinterpret_cast<const f32x4 *>(
                                           x + (long)r * din + (k0 + c < din ? k0 + c : din - 4));
                }
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    const int e = pt + i * 256, r = e / 8, c = 4 * (e % 8);
                    const int rr = r < dh ? r : dh - 1;
                    rw[set][i] = BLK ? *reinterpret_cast<const f32x4 *>(W1 + ((long)sl * dh + rr) * BK + c)
                                     : *reinterpret_cast<const f32x4 *>(
                                           W1 + (long)rr * din + (k0 + c < din ? k0 + c : din - 4));
                }
            };
            auto store = [&](int set, int sl, char *img) {
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int e = pt + i * 256;
                    put(img, e / 8, e % 8, sl * BK, rx[set][i]);
                }
#pragma unroll
                for (int i = 0; i < 5; ++i) {
                    const int e = pt + i * 256;
                    put(img, MB + e / 8, e % 8, sl * BK, rw[set][i]);
                }
            };
#pragma unroll
            for (int j = 0; j < R; ++j) load(j, j < ns ? j : ns - 1);
            for (int s0 = 0; s0 < ns; s0 += R) {
#pragma unroll
                for (int j = 0; j < R; ++j) {
                    const int sl = s0 + j;
                    if (sl < ns) store(j, sl, img0 + (sl & 1) * IMGB);
                    load(j, sl + R < ns ? sl + R : ns - 1);
                    if (sl < ns) __syncthreads();
                }
            }
        }
    } else {
        f32x4 acc[10], sml[10];
#pragma unroll
        for (int t = 0; t < 10; ++t) acc[t] = sml[t] = f32x4{0.f, 0.f, 0.f, 0.f};
        float bv[10];
#pragma unroll
        for (int t = 0; t < 10; ++t) {
            const int n = 16 * t + (lane & 15);
            bv[t] = n < dh ? W1[BLK ? 25 * dh * BK + n : dh * din + n] : 0.f;
        }
        const int m = wave * 16 + (lane & 15), hq = lane >> 4;
        auto compute = [&](const char *img) {
            const uint32_t oa = l1_wofs(m, 8 * hq);
            const bf16x8 ah = *reinterpret_cast<const bf16x8 *>(img + oa);
            const bf16x8 am = *reinterpret_cast<const bf16x8 *>(img + XPL + oa);
            const bf16x8 al = *reinterpret_cast<const bf16x8 *>(img + 2 * XPL + oa);
            const char *wpl = img + 3 * XPL;
#pragma unroll
            for (int t = 0; t < 10; ++t) {
                const uint32_t ob = l1_wofs(16 * t + (lane & 15), 8 * hq);
                const bf16x8 bh = *reinterpret_cast<const bf16x8 *>(wpl + ob);
                const bf16x8 bm = *reinterpret_cast<const bf16x8 *>(wpl + L1P + ob);
                const bf16x8 bl = *reinterpret_cast<const bf16x8 *>(wpl + 2 * L1P + ob);
                mfma_x6(ah, am, al, bh, bm, bl, acc[t], sml[t]);
            }
        };
        if constexpr (DMA) __builtin_amdgcn_s_barrier();   // the producers' slice-0 DMA barrier
        for (int sl = 0; sl < ns; ++sl) {
            if (sl > 0) compute(img0 + ((sl - 1) & 1) * IMGB);
            if constexpr (DMA) __builtin_amdgcn_s_barrier();
            else __syncthreads();
        }
        compute(img0 + ((ns - 1) & 1) * IMGB);
#pragma unroll
        for (int t = 0; t < 10; ++t) {
            acc[t] += sml[t];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = wave * 16 + 4 * hq + r, n = 16 * t + (lane & 15);
                const float v = acc[t][r] + bv[t];
                if (n < dh) H[((long)a * MB + row) * DH + n] = v > 0.f ? v : 0.f;
            }
        }
    }
}

template <bool DMA, bool BLK = false>
int run_ws(const char *name, float *X, long ld, float *D, float *H, int N,
           const std::vector<float> &ref) {
    auto k = l1_ws<DMA, BLK>;
    const int lds = 2 * IMGB + (DMA ? 2 * RAW_F4 * 16 : 0);
    CHECK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    CHECK(hipMemset(H, 0, (long)N * MB * DH * 4));
    hipLaunchKernelGGL(k, dim3(N), dim3(NT), lds, 0, X, ld, D, H);
    CHECK(hipDeviceSynchronize());
    std::vector<float> hh((long)N * MB * DH);
    CHECK(hipMemcpy(hh.data(), H, hh.size() * 4, hipMemcpyDeviceToHost));
    long diff = 0;
    for (long i = 0; i < (long)hh.size(); ++i) diff += hh[i] != ref[i];
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int iters = 50;
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k, dim3(N), dim3(NT), lds, 0, X, ld, D, H);
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k, dim3(N), dim3(NT), lds, 0, X, ld, D, H);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    const double bytes = (double)N * (MB + DH) * DIN * 4;
    const double cu = cold_us([&] { hipLaunchKernelGGL(k, dim3(N), dim3(NT), lds, 0, X, ld, D, H); });
    printf("%-40s: %6.2f us per launch (cold %6.2f), %5.2f GB/s per CU; elements differing from "
           "the per-wave split kernel: %ld\n", name, us, cu, bytes / 256 / (us * 1e-6) / 1e9, diff);
    return 0;
}

// Cold timing: the inputs (x 51 MB + W1 120 MB) fit the 256-MB MALL, so back-to-back launches
// read them on-die; in the c3 step they come from HBM behind the round's 500 MB.  cold_us
// reads a 1-GiB buffer before each launch and times the launch alone.
static float *g_flush = nullptr;
// read-only flush: 1 GiB streamed through L2 and the MALL, nothing left dirty (a memset leaves
// 256 MB of dirty lines whose write-back lands in the timed launch)
__global__ void __launch_bounds__(256) flush_read(const float4 *__restrict__ p, long n, float *out) {
    float acc = 0.f;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const float4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.678f) out[0] = acc;   // keeps the loads alive; never true for zeros
}
template <typename L>
double cold_us(L launch) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    double tot = 0;
    const int iters = 30;
    for (int i = 0; i < iters; ++i) {
        hipLaunchKernelGGL(flush_read, dim3(4096), dim3(256), 0, 0,
                           reinterpret_cast<const float4 *>(g_flush), (1L << 30) / 16, g_flush);
        (void)hipEventRecord(e0);
        launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        tot += ms;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return tot * 1e3 / iters;
}

template <int S, int MODE>
int run(const char *name, float *X, long ld, float *D, float *H, int N, bool check,
        const std::vector<float> &hx, const std::vector<float> &hd) {
    auto k = l1_x6<S, MODE>;
    const int lds = S * SLICE_F4 * 16;
    CHECK(hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    hipLaunchKernelGGL(k, dim3(N), dim3(NT), lds, 0, X, ld, D, H);
    CHECK(hipDeviceSynchronize());
    double maxrel = -1;
    if (check) {
        std::vector<float> hh((long)N * MB * DH);
        CHECK(hipMemcpy(hh.data(), H, hh.size() * 4, hipMemcpyDeviceToHost));
        maxrel = 0;
        for (int a : {0, 77, 128, 255})
            for (int m = 0; m < MB; ++m)
                for (int n = 0; n < DH; ++n) {
                    double acc = hx[a * ld + DH * DIN + n], nrm = std::fabs(acc);
                    for (int kk = 0; kk < DIN; ++kk) {
                        const double p = (double)hd[((long)a * MB + m) * DIN + kk] *
                                         hx[a * ld + (long)n * DIN + kk];
                        acc += p;
                        nrm += std::fabs(p);
                    }
                    const double want = acc > 0 ? acc : 0;
                    const double got = hh[((long)a * MB + m) * DH + n];
                    maxrel = std::fmax(maxrel, std::fabs(got - want) / nrm);
                }
    }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int iters = 50;
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(k, dim3(N), dim3(NT), lds, 0, X, ld, D, H);
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(k, dim3(N), dim3(NT), lds, 0, X, ld, D, H);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / iters;
    const double bytes = (double)N * (MB + DH) * DIN * 4;
    const double cu = cold_us([&] { hipLaunchKernelGGL(k, dim3(N), dim3(NT), lds, 0, X, ld, D, H); });
    printf("%-28s ring=%d: %6.2f us per launch (cold %6.2f), %5.2f GB/s per CU; max |err|/sum|terms| "
           "vs fp64 = %.2e\n", name, S, us, cu, bytes / 256 / (us * 1e-6) / 1e9, maxrel);
    return 0;
}

int main() {
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
    CHECK(hipMalloc(&g_flush, 1L << 30));
    CHECK(hipMemset(g_flush, 0, 1L << 30));
    CHECK(hipMemcpy(X, hx.data(), hx.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(D, hd.data(), hd.size() * 4, hipMemcpyHostToDevice));
    int rc = 0;
    rc |= run<3, 0>("dma + split + bf16x6", X, ld, D, H, N, true, hx, hd);
    rc |= run<4, 0>("dma + split + bf16x6", X, ld, D, H, N, true, hx, hd);
    rc |= run<2, 0>("dma + split + bf16x6", X, ld, D, H, N, true, hx, hd);
    rc |= run<3, 1>("stream only", X, ld, D, H, N, false, hx, hd);
    rc |= run<4, 1>("stream only", X, ld, D, H, N, false, hx, hd);
    rc |= run<3, 2>("split + bf16x6 only (no dma)", X, ld, D, H, N, false, hx, hd);
    // the per-wave split kernel's H1 (ring 3) as the bit reference: same products, same order
    rc |= run<3, 0>("dma + split + bf16x6 (reference H1)", X, ld, D, H, N, false, hx, hd);
    std::vector<float> ref((long)N * MB * DH);
    CHECK(hipMemcpy(ref.data(), H, ref.size() * 4, hipMemcpyDeviceToHost));
    rc |= run_ws<false>("warp-specialised, register producers", X, ld, D, H, N, ref);
    rc |= run_ws<true>("warp-specialised, DMA producers", X, ld, D, H, N, ref);
    rc |= run_ws<false>("warp-specialised, register producers", X, ld, D, H, N, ref);
    rc |= run_ws<true>("warp-specialised, DMA producers", X, ld, D, H, N, ref);
    // slice-blocked copies of the same x and W1 (+ b1)
    {
        const long ldb = ((long)25 * DH * BK + DH + 63) / 64 * 64;
        std::vector<float> hxb(N * ldb, 0.f), hdb((long)N * 25 * MB * BK, 0.f);
        for (int a = 0; a < N; ++a) {
            for (int n = 0; n < DH; ++n)
                for (int kk = 0; kk < DIN; ++kk)
                    hxb[a * ldb + ((long)(kk / BK) * DH + n) * BK + kk % BK] = hx[a * ld + (long)n * DIN + kk];
            for (int n = 0; n < DH; ++n) hxb[a * ldb + 25L * DH * BK + n] = hx[a * ld + (long)DH * DIN + n];
            for (int m = 0; m < MB; ++m)
                for (int kk = 0; kk < DIN; ++kk)
                    hdb[(long)a * 25 * MB * BK + ((long)(kk / BK) * MB + m) * BK + kk % BK] =
                        hd[((long)a * MB + m) * DIN + kk];
        }
        float *Xb, *Db;
        CHECK(hipMalloc(&Xb, hxb.size() * 4));
        CHECK(hipMalloc(&Db, hdb.size() * 4));
        CHECK(hipMemcpy(Xb, hxb.data(), hxb.size() * 4, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(Db, hdb.data(), hdb.size() * 4, hipMemcpyHostToDevice));
        rc |= run_ws<false, true>("warp-specialised, register, BLOCKED", Xb, ldb, Db, H, N, ref);
        rc |= run_ws<false, false>("warp-specialised, register producers", X, ld, D, H, N, ref);
        rc |= run_ws<false, true>("warp-specialised, register, BLOCKED", Xb, ldb, Db, H, N, ref);
    }
    return rc;
}
