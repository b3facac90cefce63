// Probe: the c4-rank halo pack (step_rows_tiled_kernel, csrc/aux_kernels.hip) at its real shape --
// 96 boundary rows (the last 96 of 512 in the boundary-last order, 32 per peer for 3 peers) of a
// column-tiled [16384][512][16] x and g, t = x - lr g written into three contiguous per-peer
// blocks [16384][32][16] -- against variants of its geometry: tiles in flight per thread (U),
// workgroups per launch, and non-temporal stores of the send blocks (read by the peers, never
// again here).  Session D measured the kernel at 69 us = 54 % of spec for 302 MB.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/bin/pack_probe scripts/pack_probe.hip
#include <hip/hip_runtime.h>

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

constexpr int ROWS = 512, SEL = 96, PEERS = 3, TQ = 4;   // T = 16: 4 float4 per row segment
constexpr long NT = 16384;                                 // 2^18 / 16 tiles

template <int U, bool NTS>
__global__ void __launch_bounds__(256) pack(const float4 *__restrict__ x, const float4 *__restrict__ g,
                                            float lr, float4 *__restrict__ o0, float4 *__restrict__ o1,
                                            float4 *__restrict__ o2) {
    const int q = blockIdx.x * 256 + threadIdx.x;
    if (q >= SEL * TQ) return;
    const int i = q / TQ, cc = q % TQ;
    const int b = i / 32;
    float4 *ob = b == 0 ? o0 : b == 1 ? o1 : o2;
    const long r = ROWS - SEL + i;
    const long xs = (long)ROWS * TQ, os = 32L * TQ;
    const float4 *xp = x + r * TQ + cc, *gp = g + r * TQ + cc;
    float4 *op = ob + (long)(i - 32 * b) * TQ + cc;
    long t = blockIdx.y;
    const long gy = gridDim.y;
    for (; t + (U - 1) * gy < NT; t += U * gy) {
        float4 v[U], w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v[u] = xp[(t + u * gy) * xs];
            w[u] = gp[(t + u * gy) * xs];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v[u].x = v[u].x - lr * w[u].x;
            v[u].y = v[u].y - lr * w[u].y;
            v[u].z = v[u].z - lr * w[u].z;
            v[u].w = v[u].w - lr * w[u].w;
            if (NTS) {
                typedef float f4 __attribute__((ext_vector_type(4)));
                const f4 vv = {v[u].x, v[u].y, v[u].z, v[u].w};
                __builtin_nontemporal_store(vv, reinterpret_cast<f4 *>(op + (t + u * gy) * os));
            } else {
                op[(t + u * gy) * os] = v[u];
            }
        }
    }
    for (; t < NT; t += gy) {
        float4 v = xp[t * xs];
        const float4 w = gp[t * xs];
        v.x = v.x - lr * w.x;
        v.y = v.y - lr * w.y;
        v.z = v.z - lr * w.z;
        v.w = v.w - lr * w.w;
        op[t * os] = v;
    }
}

// tile-major variant: a workgroup owns whole tiles (all 96 rows x 4 chunks = 384 lanes -> 2 tiles
// per 768 threads would not divide; use 384-thread groups), every thread one float4 per tile,
// consecutive tiles per workgroup (contiguous 6 KB reads per tile and operand)
template <int U>
__global__ void __launch_bounds__(384) pack_tiles(const float4 *__restrict__ x,
                                                  const float4 *__restrict__ g, float lr,
                                                  float4 *__restrict__ o0, float4 *__restrict__ o1,
                                                  float4 *__restrict__ o2, long per) {
    const int q = threadIdx.x, i = q / TQ, cc = q % TQ, b = i / 32;
    float4 *ob = b == 0 ? o0 : b == 1 ? o1 : o2;
    const long xs = (long)ROWS * TQ, os = 32L * TQ;
    const float4 *xp = x + (long)(ROWS - SEL + i) * TQ + cc, *gp = g + (long)(ROWS - SEL + i) * TQ + cc;
    float4 *op = ob + (long)(i - 32 * b) * TQ + cc;
    const long t0 = blockIdx.x * per, t1 = t0 + per < NT ? t0 + per : NT;
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
            v[u].x = v[u].x - lr * w[u].x;
            v[u].y = v[u].y - lr * w[u].y;
            v[u].z = v[u].z - lr * w[u].z;
            v[u].w = v[u].w - lr * w[u].w;
            op[(t + u) * os] = v[u];
        }
    }
    for (; t < t1; ++t) {
        float4 v = xp[t * xs];
        const float4 w = gp[t * xs];
        v.x = v.x - lr * w.x;
        v.y = v.y - lr * w.y;
        v.z = v.z - lr * w.z;
        v.w = v.w - lr * w.w;
        op[t * os] = v;
    }
}

int main() {
    const long n_x = NT * ROWS * 16, n_o = NT * 32 * 16;
    float *x, *g, *o[3];
    CHECK(hipMalloc(&x, n_x * 4));
    CHECK(hipMalloc(&g, n_x * 4));
    for (int b = 0; b < 3; ++b) CHECK(hipMalloc(&o[b], n_o * 4));
    {
        std::vector<float> h(n_x);
        for (long i = 0; i < n_x; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
        CHECK(hipMemcpy(x, h.data(), n_x * 4, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(g, h.data(), n_x * 4, hipMemcpyHostToDevice));
    }
    const float lr = 0.01f;
    const double bytes = 3.0 * SEL * NT * 16 * 4;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    std::vector<float> ref(n_o);
    auto time = [&](const char *name, auto launch) -> int {
        launch();
        CHECK(hipDeviceSynchronize());
        std::vector<float> h(n_o);
        CHECK(hipMemcpy(h.data(), o[1], n_o * 4, hipMemcpyDeviceToHost));
        long diff = 0;
        if (ref[0] == 0.f && ref[1] == 0.f) ref = h;
        for (long i = 0; i < n_o; ++i) diff += h[i] != ref[i];
        for (int i = 0; i < 5; ++i) launch();
        CHECK(hipEventRecord(e0));
        const int iters = 100;
        for (int i = 0; i < iters; ++i) launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / iters;
        printf("%-36s %7.2f us  %5.2f TB/s  %5.1f %% of 8 TB/s  (diff %ld)\n", name, us,
               bytes / (us * 1e-6) / 1e12, bytes / (us * 1e-6) / 8e12 * 100, diff);
        return 0;
    };
    int rc = 0;
    for (int gy : {512, 1024, 2048, 4096}) {
        char nm[64];
        snprintf(nm, sizeof nm, "strided U=4 gy=%d", gy);
        rc |= time(nm, [&] { hipLaunchKernelGGL((pack<4, false>), dim3(2, gy), dim3(256), 0, 0,
                                                (const float4 *)x, (const float4 *)g, lr,
                                                (float4 *)o[0], (float4 *)o[1], (float4 *)o[2]); });
        snprintf(nm, sizeof nm, "strided U=8 gy=%d", gy);
        rc |= time(nm, [&] { hipLaunchKernelGGL((pack<8, false>), dim3(2, gy), dim3(256), 0, 0,
                                                (const float4 *)x, (const float4 *)g, lr,
                                                (float4 *)o[0], (float4 *)o[1], (float4 *)o[2]); });
        snprintf(nm, sizeof nm, "strided U=4 gy=%d nt stores", gy);
        rc |= time(nm, [&] { hipLaunchKernelGGL((pack<4, true>), dim3(2, gy), dim3(256), 0, 0,
                                                (const float4 *)x, (const float4 *)g, lr,
                                                (float4 *)o[0], (float4 *)o[1], (float4 *)o[2]); });
    }
    for (long per : {8L, 16L, 32L, 64L}) {
        char nm[64];
        snprintf(nm, sizeof nm, "tile runs of %ld, U=4", per);
        const long nb = (NT + per - 1) / per;
        rc |= time(nm, [&] { hipLaunchKernelGGL((pack_tiles<4>), dim3(nb), dim3(384), 0, 0,
                                                (const float4 *)x, (const float4 *)g, lr,
                                                (float4 *)o[0], (float4 *)o[1], (float4 *)o[2], per); });
        snprintf(nm, sizeof nm, "tile runs of %ld, U=8", per);
        rc |= time(nm, [&] { hipLaunchKernelGGL((pack_tiles<8>), dim3(nb), dim3(384), 0, 0,
                                                (const float4 *)x, (const float4 *)g, lr,
                                                (float4 *)o[0], (float4 *)o[1], (float4 *)o[2], per); });
    }
    return rc;
}
