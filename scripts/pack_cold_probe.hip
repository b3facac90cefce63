// Probe: the c4-rank halo pack COLD (the 1.7-GB mix launch before it in the real round evicts
// the MALL), at its real shape -- 96 boundary rows (the last 96 of 512, 32 per peer for 3 peers)
// of a column-tiled [16384][512][16] x and g, t = x - lr g into three contiguous per-peer blocks
// [16384][32][16] -- against the same bytes read from a compact boundary-only source
// [16384][96][16] (what a layout keeping the boundary rows in their own block would read).  A
// 1-GiB flush before every timed launch (memset, read sweep or non-temporal store sweep); each launch timed alone with events.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/bin/pack_cold_probe scripts/pack_cold_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
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

constexpr int SEL = 96, TQ = 4;   // T = 16: 4 float4 per row segment
constexpr long NT = 16384;        // 2^18 / 16 tiles

// src rows: row0 + i of [NT][src_rows][16]; workgroup = one contiguous run of tiles, lane groups
// of 384 lanes (96 rows x 4 chunks) -> 256-thread blocks hold 1 group of 384?  use 384 threads.
template <int U>
__global__ void __launch_bounds__(384) pack_runs(const float4 *__restrict__ x,
                                                 const float4 *__restrict__ g, int src_rows,
                                                 int row0, float lr, float4 *__restrict__ o0,
                                                 float4 *__restrict__ o1, float4 *__restrict__ o2,
                                                 long per) {
    const int q = threadIdx.x, i = q / TQ, cc = q % TQ, b = i / 32;
    float4 *ob = b == 0 ? o0 : b == 1 ? o1 : o2;
    const long xs = (long)src_rows * TQ, os = 32L * TQ;
    const float4 *xp = x + (long)(row0 + i) * TQ + cc, *gp = g + (long)(row0 + i) * TQ + cc;
    float4 *op = ob + (long)(i - 32 * b) * TQ + cc;
    const long t0 = blockIdx.x * per, t1 = t0 + per < NT ? t0 + per : NT;
    typedef float f4 __attribute__((ext_vector_type(4)));
    long t = t0;
    for (; t + U <= t1; t += U) {
        float4 v[U], w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v[u] = xp[(t + u) * xs];
            w[u] = gp[(t + u) * xs];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            __builtin_nontemporal_store(f4{v[u].x - lr * w[u].x, v[u].y - lr * w[u].y,
                                           v[u].z - lr * w[u].z, v[u].w - lr * w[u].w},
                                        reinterpret_cast<f4 *>(op + (t + u) * os));
        }
    }
    for (; t < t1; ++t) {
        const float4 v = xp[t * xs], w = gp[t * xs];
        __builtin_nontemporal_store(f4{v.x - lr * w.x, v.y - lr * w.y, v.z - lr * w.z,
                                       v.w - lr * w.w},
                                    reinterpret_cast<f4 *>(op + t * os));
    }
}

// a plain read-only sweep of the same bytes (x and g segments only, no stores): the read floor
template <int U>
__global__ void __launch_bounds__(384) read_runs(const float4 *__restrict__ x,
                                                 const float4 *__restrict__ g, int src_rows,
                                                 int row0, long per, float *sink) {
    const int q = threadIdx.x, i = q / TQ, cc = q % TQ;
    const long xs = (long)src_rows * TQ;
    const float4 *xp = x + (long)(row0 + i) * TQ + cc, *gp = g + (long)(row0 + i) * TQ + cc;
    const long t0 = blockIdx.x * per, t1 = t0 + per < NT ? t0 + per : NT;
    float acc = 0.f;
    for (long t = t0; t + U <= t1; t += U) {
        float4 v[U], w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v[u] = xp[(t + u) * xs];
            w[u] = gp[(t + u) * xs];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u].x + w[u].y;
    }
    if (acc == 12345.678f) sink[0] = acc;
}

// read-only sweep of the flush buffer: evicts the MALL without leaving dirty lines behind
__global__ void __launch_bounds__(256) sweep(const float4 *__restrict__ p, long n, float *sink) {
    float acc = 0.f;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        const float4 v = p[i];
        acc += v.x;
    }
    if (acc == 12345.678f) sink[0] = acc;
}

// sweep of the pack's own source buffers (x then g), non-temporal or plain loads: what the mix
// launch before the pack does to the lines the pack then reads
template <bool NTL>
__global__ void __launch_bounds__(256) src_sweep(const float4 *__restrict__ x,
                                                 const float4 *__restrict__ g, long n, float *sink) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    float acc = 0.f;
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        if (NTL) {
            const f4 a = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(x + i));
            const f4 b = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(g + i));
            acc += a.x + b.y;
        } else {
            acc += x[i].x + g[i].y;
        }
    }
    if (acc == 12345.678f) sink[0] = acc;
}

// non-temporal store sweep of the flush buffer (what the c4 mix launch's output stores are)
__global__ void __launch_bounds__(256) nt_fill(float4 *__restrict__ p, long n, float v) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        __builtin_nontemporal_store(f4{v, v, v, v}, reinterpret_cast<f4 *>(p + i));
}

int main() {
    const long n_x = NT * 512 * 16, n_b = NT * SEL * 16, n_o = NT * 32 * 16;
    float *x, *g, *xb, *gb, *o[3], *flush, *sink;
    CHECK(hipMalloc(&x, n_x * 4));
    CHECK(hipMalloc(&g, n_x * 4));
    CHECK(hipMalloc(&xb, n_b * 4));
    CHECK(hipMalloc(&gb, n_b * 4));
    for (int b = 0; b < 3; ++b) CHECK(hipMalloc(&o[b], n_o * 4));
    const size_t fl = 1ul << 30;
    CHECK(hipMalloc(&flush, fl));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(x, 0, n_x * 4));
    CHECK(hipMemset(g, 0, n_x * 4));
    CHECK(hipMemset(xb, 0, n_b * 4));
    CHECK(hipMemset(gb, 0, n_b * 4));
    const float lr = 0.01f;
    const double bytes = 3.0 * SEL * NT * 16 * 4, rbytes = 2.0 * SEL * NT * 16 * 4;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    int mode = 0;   // 1: memset flush, 2: read-only sweep, 3: non-temporal store sweep
    auto time = [&](const char *name, double nbytes, bool cold, auto launch) -> int {
        std::vector<float> v;
        for (int i = 0; i < 23; ++i) {
            if (cold && mode == 1) CHECK(hipMemsetAsync(flush, i & 0xff, fl));
            if (cold && mode == 2)
                hipLaunchKernelGGL(sweep, dim3(4096), dim3(256), 0, 0, (const float4 *)flush,
                                   (long)(fl / 16), sink);
            if (cold && mode == 3)
                hipLaunchKernelGGL(nt_fill, dim3(4096), dim3(256), 0, 0, (float4 *)flush,
                                   (long)(fl / 16), (float)i);
            if (cold && (mode == 4 || mode == 5)) {
                if (mode == 4)
                    hipLaunchKernelGGL(src_sweep<true>, dim3(4096), dim3(256), 0, 0,
                                       (const float4 *)x, (const float4 *)g, n_x / 4, sink);
                else
                    hipLaunchKernelGGL(src_sweep<false>, dim3(4096), dim3(256), 0, 0,
                                       (const float4 *)x, (const float4 *)g, n_x / 4, sink);
            }
            CHECK(hipEventRecord(e0));
            launch();
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (i >= 3) v.push_back(ms * 1e3f);
        }
        std::sort(v.begin(), v.end());
        const double us = v[v.size() / 2];
        printf("%-44s %s %7.2f us (min %6.2f)  %5.2f TB/s  %5.1f %% of 8 TB/s\n", name,
               !cold ? "warm      " : mode == 1 ? "cold-memset" : mode == 2 ? "cold-read  " : mode == 3 ? "cold-ntfill" : mode == 4 ? "src-ntload " : "src-plain  ", us, v[0], nbytes / (us * 1e-6) / 1e12,
               nbytes / (us * 1e-6) / 8e12 * 100);
        return 0;
    };
    int rc = 0;
    for (int m : {4, 5, 2, 0}) {
        mode = m;
        const bool cold = m != 0;
        for (long per : {16L, 64L}) {
            const long nb = (NT + per - 1) / per;
            char nm[96];
            snprintf(nm, sizeof nm, "pack strided src (last 96 of 512), run %ld", per);
            rc |= time(nm, bytes, cold, [&] {
                hipLaunchKernelGGL((pack_runs<4>), dim3(nb), dim3(384), 0, 0, (const float4 *)x,
                                   (const float4 *)g, 512, 512 - SEL, lr, (float4 *)o[0],
                                   (float4 *)o[1], (float4 *)o[2], per);
            });
            snprintf(nm, sizeof nm, "pack compact src [NT][96][16], run %ld", per);
            rc |= time(nm, bytes, cold, [&] {
                hipLaunchKernelGGL((pack_runs<4>), dim3(nb), dim3(384), 0, 0, (const float4 *)xb,
                                   (const float4 *)gb, SEL, 0, lr, (float4 *)o[0],
                                   (float4 *)o[1], (float4 *)o[2], per);
            });
            snprintf(nm, sizeof nm, "read only strided, run %ld", per);
            rc |= time(nm, rbytes, cold, [&] {
                hipLaunchKernelGGL((read_runs<4>), dim3(nb), dim3(384), 0, 0, (const float4 *)x,
                                   (const float4 *)g, 512, 512 - SEL, per, sink);
            });
            snprintf(nm, sizeof nm, "read only compact, run %ld", per);
            rc |= time(nm, rbytes, cold, [&] {
                hipLaunchKernelGGL((read_runs<4>), dim3(nb), dim3(384), 0, 0, (const float4 *)xb,
                                   (const float4 *)gb, SEL, 0, per, sink);
            });
        }
    }
    return rc;
}
