// HBM probe for gfx950: read-only, write-only and copy streaming kernels over a sweep of
// geometries, to find the access pattern that reaches the HBM ceiling (the mix kernel's target).
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/hbm_probe scripts/hbm_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// grid-stride, U float4 per thread per step (all loads before the stores)
template <int U, bool NT_LOAD, bool NT_STORE>
__global__ void copy_k(const f32x4 *__restrict__ s, f32x4 *__restrict__ d, long n4) {
    const long step = (long)gridDim.x * blockDim.x * U;
    for (long base = (long)blockIdx.x * blockDim.x * U; base < n4; base += step) {
        f32x4 v[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            long i = base + (long)j * blockDim.x + threadIdx.x;
            if (i < n4) v[j] = NT_LOAD ? __builtin_nontemporal_load(s + i) : s[i];
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            long i = base + (long)j * blockDim.x + threadIdx.x;
            if (i < n4) {
                if (NT_STORE)
                    __builtin_nontemporal_store(v[j], d + i);
                else
                    d[i] = v[j];
            }
        }
    }
}

// contiguous chunk per workgroup (each WG streams its own contiguous range)
template <int U>
__global__ void copy_chunk_k(const f32x4 *__restrict__ s, f32x4 *__restrict__ d, long n4) {
    const long per = (n4 + gridDim.x - 1) / gridDim.x;
    const long b0 = (long)blockIdx.x * per, b1 = b0 + per < n4 ? b0 + per : n4;
    for (long base = b0; base < b1; base += (long)blockDim.x * U) {
        f32x4 v[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            long i = base + (long)j * blockDim.x + threadIdx.x;
            if (i < b1) v[j] = s[i];
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            long i = base + (long)j * blockDim.x + threadIdx.x;
            if (i < b1) d[i] = v[j];
        }
    }
}

// triad y = x - lr*g: two read streams, one write stream (the traffic of the fused SGD + mix
// round, 12 B per element), grid-stride, U float4 per stream per thread
template <int U, bool NT>
__global__ void triad_k(const f32x4 *__restrict__ x, const f32x4 *__restrict__ g,
                        f32x4 *__restrict__ y, long n4, float lr) {
    const long step = (long)gridDim.x * blockDim.x * U;
    for (long base = (long)blockIdx.x * blockDim.x * U; base < n4; base += step) {
        f32x4 a[U], b[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            long i = base + (long)j * blockDim.x + threadIdx.x;
            if (i < n4) {
                a[j] = NT ? __builtin_nontemporal_load(x + i) : x[i];
                b[j] = NT ? __builtin_nontemporal_load(g + i) : g[i];
            }
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            long i = base + (long)j * blockDim.x + threadIdx.x;
            if (i < n4) {
                f32x4 v = a[j] - lr * b[j];
                if (NT) __builtin_nontemporal_store(v, y + i);
                else y[i] = v;
            }
        }
    }
}

// contiguous chunk per workgroup, triad (each WG streams its own range, like the tile kernel)
template <int U>
__global__ void triad_chunk_k(const f32x4 *__restrict__ x, const f32x4 *__restrict__ g,
                              f32x4 *__restrict__ y, long n4, float lr) {
    const long per = (n4 + gridDim.x - 1) / gridDim.x;
    const long b0 = (long)blockIdx.x * per, b1 = b0 + per < n4 ? b0 + per : n4;
    for (long base = b0; base < b1; base += (long)blockDim.x * U) {
        f32x4 a[U], b[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            long i = base + (long)j * blockDim.x + threadIdx.x;
            if (i < b1) {
                a[j] = __builtin_nontemporal_load(x + i);
                b[j] = __builtin_nontemporal_load(g + i);
            }
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            long i = base + (long)j * blockDim.x + threadIdx.x;
            if (i < b1) __builtin_nontemporal_store(a[j] - lr * b[j], y + i);
        }
    }
}

template <int U>
__global__ void read_k(const f32x4 *__restrict__ s, long n4, float *out) {
    const long step = (long)gridDim.x * blockDim.x * U;
    f32x4 acc = {0, 0, 0, 0};
    for (long base = (long)blockIdx.x * blockDim.x * U; base < n4; base += step) {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            long i = base + (long)j * blockDim.x + threadIdx.x;
            if (i < n4) acc += s[i];
        }
    }
    float t = acc.x + acc.y + acc.z + acc.w;
    if (t == 12345.678f) out[0] = t;  // keep the loads alive
}

template <int U, bool NT>
__global__ void write_k(f32x4 *__restrict__ d, long n4) {
    const long step = (long)gridDim.x * blockDim.x * U;
    f32x4 v = {1, 2, 3, 4};
    for (long base = (long)blockIdx.x * blockDim.x * U; base < n4; base += step) {
#pragma unroll
        for (int j = 0; j < U; ++j) {
            long i = base + (long)j * blockDim.x + threadIdx.x;
            if (i < n4) {
                if (NT)
                    __builtin_nontemporal_store(v, d + i);
                else
                    d[i] = v;
            }
        }
    }
}

template <typename F>
float time_ms(F f, int reps) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    f();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CHECK(hipEventRecord(b));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

int triad_main(long bytes) {
    // x, g, y of `bytes` each; traffic = 3 * bytes per launch
    const long n4 = bytes / 16;
    f32x4 *x, *g, *y;
    CHECK(hipMalloc(&x, bytes));
    CHECK(hipMalloc(&g, bytes));
    CHECK(hipMalloc(&y, bytes));
    CHECK(hipMemset(x, 0, bytes));
    CHECK(hipMemset(g, 0, bytes));
    const int reps = 10;
    const double traffic = 3.0 * bytes;
    for (int bs : {256, 512, 1024})
        for (int gr : {256, 512, 1024, 2048, 4096, 8192, 16384}) {
            auto pr = [&](const char *name, float ms) {
                printf("{\"kernel\":\"%s\",\"block\":%d,\"grid\":%d,\"ms\":%.4f,\"GBs\":%.1f}\n",
                       name, bs, gr, ms, traffic / ms / 1e6);
            };
            pr("triad_u1_nt", time_ms([&] { triad_k<1, true><<<gr, bs>>>(x, g, y, n4, 1e-3f); }, reps));
            pr("triad_u2_nt", time_ms([&] { triad_k<2, true><<<gr, bs>>>(x, g, y, n4, 1e-3f); }, reps));
            pr("triad_u4_nt", time_ms([&] { triad_k<4, true><<<gr, bs>>>(x, g, y, n4, 1e-3f); }, reps));
            pr("triad_u4", time_ms([&] { triad_k<4, false><<<gr, bs>>>(x, g, y, n4, 1e-3f); }, reps));
            pr("triad_chunk_u2", time_ms([&] { triad_chunk_k<2><<<gr, bs>>>(x, g, y, n4, 1e-3f); }, reps));
            fflush(stdout);
        }
    return 0;
}

int main(int argc, char **argv) {
    const long bytes = (argc > 1 ? atol(argv[1]) : 4096L) << 20;  // MiB
    if (argc > 2 && argv[2][0] == 't') return triad_main(bytes);
    const long n4 = bytes / 16;
    f32x4 *s, *d;
    float *o;
    CHECK(hipMalloc(&s, bytes));
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMalloc(&o, 4));
    CHECK(hipMemset(s, 0, bytes));
    CHECK(hipMemset(d, 0, bytes));
    const int reps = 10;
    const int grids[] = {256, 512, 1024, 2048, 4096, 8192};
    const int blocks[] = {256, 512, 1024};
    for (int bs : blocks)
        for (int g : grids) {
            auto pr = [&](const char *name, float ms, double traffic) {
                printf("{\"kernel\":\"%s\",\"block\":%d,\"grid\":%d,\"ms\":%.4f,\"GBs\":%.1f}\n", name,
                       bs, g, ms, traffic / ms / 1e6);
            };
            pr("read_u4", time_ms([&] { read_k<4><<<g, bs>>>(s, n4, o); }, reps), bytes);
            pr("read_u8", time_ms([&] { read_k<8><<<g, bs>>>(s, n4, o); }, reps), bytes);
            pr("write_u4", time_ms([&] { write_k<4, false><<<g, bs>>>(d, n4); }, reps), bytes);
            pr("write_u4_nt", time_ms([&] { write_k<4, true><<<g, bs>>>(d, n4); }, reps), bytes);
            pr("copy_u1", time_ms([&] { copy_k<1, false, false><<<g, bs>>>(s, d, n4); }, reps), 2.0 * bytes);
            pr("copy_u4", time_ms([&] { copy_k<4, false, false><<<g, bs>>>(s, d, n4); }, reps), 2.0 * bytes);
            pr("copy_u4_nt", time_ms([&] { copy_k<4, false, true><<<g, bs>>>(s, d, n4); }, reps), 2.0 * bytes);
            pr("copy_u4_ntld", time_ms([&] { copy_k<4, true, true><<<g, bs>>>(s, d, n4); }, reps), 2.0 * bytes);
            pr("copy_u8_nt", time_ms([&] { copy_k<8, false, true><<<g, bs>>>(s, d, n4); }, reps), 2.0 * bytes);
            pr("copy_chunk_u4", time_ms([&] { copy_chunk_k<4><<<g, bs>>>(s, d, n4); }, reps), 2.0 * bytes);
            fflush(stdout);
        }
    printf("{\"kernel\":\"hipMemcpyDtoD\",\"ms\":%.4f,\"GBs\":%.1f}\n",
           time_ms([&] { CHECK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0)); }, reps),
           2.0 * bytes / time_ms([&] { CHECK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0)); }, reps) / 1e6);
    return 0;
}
