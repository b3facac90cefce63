// Config c1 as ONE launch (gfx950): the Titanic notebook's consensus gradient descent
// (notebooks/Titanic Consensus GD test.ipynb cells 12-14: every agent takes a local GD step on
// its shard of the L2-regularised logistic loss, networks/logreg_model_titanic.py:16-20, then
// runs one asyncio consensus round weighted by its shard size, utils/consensus_asyncio.py:209-312)
// for all agents and all iterations inside one workgroup, fp64.
//
// Through the asyncio facade an iteration costs ~0.8 ms of host work (numpy gradients, asyncio
// scheduling, a launch, two copies and a synchronisation per round) for 7 parameters per agent.
// Here the shards stay in LDS, each wave computes an agent's gradient (lanes over rows, a
// shuffle reduction per feature), and the round is the synchronous Jacobi of dl_perron_round
// (pre-scale y = w * n_a / mean_n, y <- y (1 - eps deg) + eps sum_nbr y, one-sided convergence
// test against the neighbours' previous values) -- the same arithmetic, in the same order, as
// perron_update in aux_kernels.hip.  The gradient's sums run in a different order than numpy's
// BLAS dot products, so parity with the reference is a tolerance (tests/test_consensus_gd_gpu.py).
#include "dl_internal.h"

namespace dl {
namespace {

constexpr int kGdThreads = 512;
constexpr int kGdMaxF = 16;

__device__ __forceinline__ double gd_wave_sum(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
    return v;
}

// LDS: w [R][F] | y0, y1 [R][F] (Jacobi ping-pong) | flag | X [rows][F] | labels [rows]
__global__ void __launch_bounds__(kGdThreads) consensus_gd_kernel(GdArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    constexpr int NW = kGdThreads / 64;
    const int R = a.n_agents, F = a.n_features, E = R * F;
    const int rows = a.shard_ptr[R];
    double *w = reinterpret_cast<double *>(smem);
    double *y0 = w + E;
    double *y1 = y0 + E;
    int *flag = reinterpret_cast<int *>(y1 + E);
    double *Xs = reinterpret_cast<double *>(smem + a.x_off);
    double *ys = Xs + (int64_t)rows * F;
    const double *X = a.x_in_lds ? Xs : a.X;
    const double *Y = a.x_in_lds ? ys : a.y;
    if (a.x_in_lds) {
        for (int i = tid; i < rows * F; i += kGdThreads) Xs[i] = a.X[i];
        for (int i = tid; i < rows; i += kGdThreads) ys[i] = a.y[i];
    }
    for (int i = tid; i < E; i += kGdThreads) w[i] = a.w[i];
    __syncthreads();

    for (int it = 0; it < a.iterations; ++it) {
        // ---- local GD step, one wave per agent:
        // grad_j = -(sum_i y_i sigmoid(-y_i x_i.w) x_ij) / n + tau w_j ;  w <- w - step grad
        for (int ag = wave; ag < R; ag += NW) {
            const int r0 = a.shard_ptr[ag], n = a.shard_ptr[ag + 1] - r0;
            double acc[kGdMaxF];
#pragma unroll
            for (int j = 0; j < kGdMaxF; ++j) acc[j] = 0.0;
            for (int i = lane; i < n; i += 64) {
                const double *xr = X + (int64_t)(r0 + i) * F;
                const double yi = Y[r0 + i];
                double z = 0.0;
#pragma unroll
                for (int j = 0; j < kGdMaxF; ++j)
                    if (j < F) z = z + xr[j] * w[ag * F + j];
                const double t = -yi * z;                  // -y * (X @ w)
                const double c = yi * (1.0 / (1.0 + exp(-t)));   // y * sigmoid(-y X w)
#pragma unroll
                for (int j = 0; j < kGdMaxF; ++j)
                    if (j < F) acc[j] = acc[j] + c * xr[j];
            }
#pragma unroll
            for (int j = 0; j < kGdMaxF; ++j)
                if (j < F) acc[j] = gd_wave_sum(acc[j]);
            double mine = 0.0;
#pragma unroll
            for (int j = 0; j < kGdMaxF; ++j)
                if (j == lane) mine = acc[j];
            if (lane < F) {
                const double wj = w[ag * F + lane];
                const double g = -mine / (double)n + a.tau * wj;
                const double wn = wj - a.steps[it] * g;
                // pre-scale for the round: y = v * weight / mean_weight (weight = shard size)
                y0[ag * F + lane] = wn * (double)n / a.mean_weight;
            }
        }
        if (tid == 0) flag[0] = 0;
        __syncthreads();
        // ---- consensus round: synchronous Jacobi until every agent's one-sided test holds
        const double *cur = y0;
        double *nxt = y1;
        int k = 0;
        while (k < a.max_iter) {
            ++k;
            bool fail = false;
            for (int i = tid; i < E; i += kGdThreads) {
                const int r = i / F, p = i - r * F;
                const int e0 = a.rowptr[r], e1 = a.rowptr[r + 1];
                double s = 0.0;
                if (e1 > e0) {
                    s = cur[a.col[e0] * F + p];
                    for (int e = e0 + 1; e < e1; ++e) s = s + cur[a.col[e] * F + p];
                }
                const double dcoef = 1.0 - a.eps * (double)(e1 - e0);
                const double yn = cur[i] * dcoef + a.eps * s;
                for (int e = e0; e < e1; ++e)
                    if (!((yn - cur[a.col[e] * F + p]) <= a.conv_eps)) fail = true;
                nxt[i] = yn;
            }
            if (__any(fail) && lane == 0) atomicOr(&flag[0], 1);
            __syncthreads();
            const bool done = flag[0] == 0;
            __syncthreads();                 // everyone has read the flag
            if (tid == 0) flag[0] = 0;
            const double *t = cur;
            cur = nxt;
            nxt = const_cast<double *>(t);
            __syncthreads();                 // flag reset visible; nxt free to overwrite
            if (done) break;
        }
        for (int i = tid; i < E; i += kGdThreads) w[i] = cur[i];
        if (tid == 0 && a.iters_out) a.iters_out[it] = k;
        __syncthreads();
    }
    for (int i = tid; i < E; i += kGdThreads) a.w[i] = w[i];
}

}  // namespace

int64_t gd_lds_bytes(int n_agents, int n_features, int rows, bool x_in_lds, int64_t *x_off) {
    const int64_t E = (int64_t)n_agents * n_features;
    int64_t off = (3 * E * 8 + 4 + 15) / 16 * 16;
    *x_off = off;
    if (x_in_lds) off += (int64_t)rows * n_features * 8 + (int64_t)rows * 8;
    return off;
}

hipError_t launch_consensus_gd(const GdArgs &a, int lds_bytes, hipStream_t s) {
    const void *k = reinterpret_cast<const void *>(consensus_gd_kernel);
    hipError_t e = allow_full_lds(k);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(consensus_gd_kernel, dim3(1), dim3(kGdThreads), lds_bytes, s, a);
    return hipGetLastError();
}

}  // namespace dl
