// Does LDS-DMA staging (global_load_lds_dwordx4) stream the mix round's 2-read : 1-write traffic
// faster than register staging?  Triad y = x - lr*g over 1024-thread persistent workgroups:
//   reg_tile  : the mix kernel's scheme -- each thread loads its float4 of x and g for the next tile
//               into registers (nt), tile t is written to LDS, barrier, read back, stored (nt);
//   glds<S>   : x and g of tile t+S-1 DMA'd straight into LDS slot (t+S-1)%S, counted vmcnt wait
//               for tile t, raw s_barrier, read, nt store.  S = 2, 3 stages.
// One "tile" = TILE float4 per stream per workgroup (TILE = 1024 * R, R float4 per thread).
// Result (profiles/r04/glds_probe.log, 4 GiB per stream): register staging with 64-KiB tiles per
// stream (R = 4) 5.84-5.95 TB/s; glds 5.54-5.67 TB/s at best, and that figure is an upper bound:
// the counted vmcnt wait is not sufficient (the verify step reports stale LDS reads), so the
// glds variant waited less than a correct one would.  LDS-DMA staging is not a lever here.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/glds_probe scripts/glds_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));     \
            exit(1);                                                                      \
        }                                                                                 \
    } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

// s_waitcnt with only vmcnt constrained (gfx9 encoding: vmcnt[3:0] + [15:14], expcnt[6:4],
// lgkmcnt[11:8])
#define VMCNT(n) (((n) & 0xF) | (((n) >> 4) << 14) | (0x7 << 4) | (0xF << 8))

template <int R>
__global__ __launch_bounds__(1024) void reg_tile_k(const f32x4 *__restrict__ x,
                                                   const f32x4 *__restrict__ g,
                                                   f32x4 *__restrict__ y, int ntiles, float lr) {
    extern __shared__ f32x4 lds[];  // [2][R*1024]
    const int tid = threadIdx.x;
    int t = blockIdx.x;
    if (t >= ntiles) return;
    f32x4 a[R], b[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        a[r] = __builtin_nontemporal_load(x + (long)t * R * 1024 + r * 1024 + tid);
        b[r] = __builtin_nontemporal_load(g + (long)t * R * 1024 + r * 1024 + tid);
    }
    for (; t < ntiles; t += gridDim.x) {
#pragma unroll
        for (int r = 0; r < R; ++r) lds[r * 1024 + tid] = a[r] - lr * b[r];
        __syncthreads();
        const int tn = t + gridDim.x < ntiles ? t + gridDim.x : t;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            a[r] = __builtin_nontemporal_load(x + (long)tn * R * 1024 + r * 1024 + tid);
            b[r] = __builtin_nontemporal_load(g + (long)tn * R * 1024 + r * 1024 + tid);
        }
        // read a neighbour's element (another wave's) so the barrier is real
#pragma unroll
        for (int r = 0; r < R; ++r)
            __builtin_nontemporal_store(lds[r * 1024 + (tid ^ 64)], y + (long)t * R * 1024 + r * 1024 + tid);
        __syncthreads();
    }
}

template <int R, int S>
__global__ __launch_bounds__(1024) void glds_k(const f32x4 *__restrict__ x,
                                               const f32x4 *__restrict__ g,
                                               f32x4 *__restrict__ y, int ntiles, float lr) {
    extern __shared__ f32x4 lds[];  // [S][2][R*1024]
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int step = gridDim.x;
    int t0 = blockIdx.x;
    if (t0 >= ntiles) return;
    auto issue = [&](int t, int slot) {
        const f32x4 *xs = x + (long)t * R * 1024, *gs = g + (long)t * R * 1024;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int off = r * 1024 + wave * 64;  // wave-uniform LDS base, lane-linear
            __builtin_amdgcn_global_load_lds((const void *)(xs + off + lane),
                                             (lds_void *)(lds + (slot * 2 + 0) * R * 1024 + off), 16, 0, 3);
            __builtin_amdgcn_global_load_lds((const void *)(gs + off + lane),
                                             (lds_void *)(lds + (slot * 2 + 1) * R * 1024 + off), 16, 0, 3);
        }
    };
#pragma unroll
    for (int s = 0; s < S - 1; ++s) {
        const int t = t0 + s * step;
        issue(t < ntiles ? t : t0, s);
    }
    int slot = 0;
    for (int t = t0; t < ntiles; t += step) {
        const int tn = t + (S - 1) * step;
        issue(tn < ntiles ? tn : t, (slot + S - 1) % S);
        // outstanding after tile t's 2R DMAs: (S-1) later tiles' 2R DMAs + (S-1) tiles' R stores
        __builtin_amdgcn_s_waitcnt(VMCNT((S - 1) * 3 * R));
        __builtin_amdgcn_s_barrier();
        const f32x4 *lx = lds + (slot * 2 + 0) * R * 1024, *lg = lds + (slot * 2 + 1) * R * 1024;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int i = r * 1024 + (tid ^ 64);
            __builtin_nontemporal_store(lx[i] - lr * lg[i], y + (long)t * R * 1024 + r * 1024 + tid);
        }
        __builtin_amdgcn_s_waitcnt(VMCNT(63) & ~(0xF << 8));  // lgkmcnt(0): LDS reads done
        __builtin_amdgcn_s_barrier();                          // before the slot is refilled
        slot = slot + 1 == S ? 0 : slot + 1;
    }
    __builtin_amdgcn_s_waitcnt(VMCNT(0));
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

template <int R>
void run_r(f32x4 *x, f32x4 *g, f32x4 *y, long n4, int ncu, double traffic, f32x4 *h, f32x4 *hx, f32x4 *hg) {
    const int ntiles = (int)(n4 / (R * 1024));
    const int reps = 10;
    auto pr = [&](const char *name, int grid, size_t lds, float ms) {
        printf("{\"kernel\":\"%s\",\"R\":%d,\"grid\":%d,\"lds\":%zu,\"ms\":%.4f,\"GBs\":%.1f}\n", name, R, grid,
               lds, ms, traffic / ms / 1e6);
        fflush(stdout);
    };
    auto verify = [&](const char *name) {
        CHECK(hipMemcpy(h, y, 16 * 4096, hipMemcpyDeviceToHost));
        for (int i = 0; i < 4096; ++i) {
            const int j = (i & ~1023) | ((i & 1023) ^ 64);
            const float want = hx[j].x - 1e-3f * hg[j].x;
            if (h[i].x != want) {
                printf("MISMATCH %s R=%d i=%d %g vs %g\n", name, R, i, h[i].x, want);
                return;
            }
        }
    };
    for (int grid : {ncu, 2 * ncu}) {
        size_t lds = 2 * R * 1024 * 16;
        if (lds <= 160 * 1024) {
            (void)hipFuncSetAttribute((const void *)reg_tile_k<R>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            pr("reg_tile", grid, lds, time_ms([&] { reg_tile_k<R><<<grid, 1024, lds>>>(x, g, y, ntiles, 1e-3f); }, reps));
            verify("reg_tile");
        }
        lds = 2 * 2 * R * 1024 * 16;
        if (lds <= 160 * 1024) {
            (void)hipFuncSetAttribute((const void *)glds_k<R, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            CHECK(hipMemset(y, 0, 16 * 4096));
            pr("glds_s2", grid, lds, time_ms([&] { glds_k<R, 2><<<grid, 1024, lds>>>(x, g, y, ntiles, 1e-3f); }, reps));
            verify("glds_s2");
        }
        lds = 3 * 2 * R * 1024 * 16;
        if (lds <= 160 * 1024) {
            (void)hipFuncSetAttribute((const void *)glds_k<R, 3>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            CHECK(hipMemset(y, 0, 16 * 4096));
            pr("glds_s3", grid, lds, time_ms([&] { glds_k<R, 3><<<grid, 1024, lds>>>(x, g, y, ntiles, 1e-3f); }, reps));
            verify("glds_s3");
        }
    }
}

int main(int argc, char **argv) {
    const long bytes = (argc > 1 ? atol(argv[1]) : 4096L) << 20;  // MiB per stream
    const long n4 = bytes / 16;
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    f32x4 *x, *g, *y;
    CHECK(hipMalloc(&x, bytes));
    CHECK(hipMalloc(&g, bytes));
    CHECK(hipMalloc(&y, bytes));
    f32x4 *hx = (f32x4 *)malloc(16 * 4096), *hg = (f32x4 *)malloc(16 * 4096), *h = (f32x4 *)malloc(16 * 4096);
    for (int i = 0; i < 4096; ++i) {
        hx[i] = f32x4{(float)i, 1, 2, 3};
        hg[i] = f32x4{(float)(i % 7), 1, 2, 3};
    }
    CHECK(hipMemset(x, 0, bytes));
    CHECK(hipMemset(g, 0, bytes));
    CHECK(hipMemcpy(x, hx, 16 * 4096, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(g, hg, 16 * 4096, hipMemcpyHostToDevice));
    const double traffic = 3.0 * bytes;
    for (int rep = 0; rep < 2; ++rep) {
        run_r<1>(x, g, y, n4, ncu, traffic, h, hx, hg);
        run_r<2>(x, g, y, n4, ncu, traffic, h, hx, hg);
        run_r<4>(x, g, y, n4, ncu, traffic, h, hx, hg);
    }
    return 0;
}
