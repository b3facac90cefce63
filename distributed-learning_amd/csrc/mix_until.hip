// Mixer.mix(times, eps) in ONE launch when every agent's whole parameter vector fits LDS (gfx950).
//
// utils/consensus_simple/mixer.py:18-41 loops
//     stop = (eps is None or max_a ||x_a - mean(x)|| < eps) and times_done >= times
//     while not stop: x <- W x (the _mix_params_once fold, :43-49); times_done += 1
// and evaluates the deviation (:51-66) before the first round and after every round.  For the
// models the reference mixes this way (ANNModel / small CNNs on a handful of agents) X is a few
// tens of KB, so a host-driven loop is launch- and readback-bound: one launch and one 4-byte
// device->host copy per round.  Here one workgroup holds X in LDS (two images, ping-pong) and
// runs the whole loop: fold, column mean, per-agent norm, the stop test, all on the device; the
// host reads the round count once.  A round cap (max_rounds) bounds the launch; the caller
// re-enters with the remaining `times` to continue a loop the cap cut.
//
// Numerics: the fold is the same left fold in CSR order as dl_mix_round (bit-identical to the
// reference, -ffp-contract=off); the column mean is the rows summed in order then divided by N
// (np.mean axis 0, bit-identical); the norm is a per-lane then tree sum of squares (the
// reference's np.linalg.norm sums in BLAS order, so this is within rounding of it, not
// bit-identical); the comparison is float32 against float32(eps), as numpy >= 2 compares an
// np.float32 with a Python float (NEP 50).
#include "dl_internal.h"

namespace dl {
namespace {

__device__ __forceinline__ float4 mu_zero4() { return make_float4(0.f, 0.f, 0.f, 0.f); }

__device__ __forceinline__ float mu_wave_sum(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
    return v;
}

__device__ __forceinline__ float mu_wave_max(float v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m));
    return v;
}

// LDS: img0 | img1 ([N][C4] float4 each) | mean [C4] float4 | w [nnz] | col [nnz] | rowptr [N+1]
//      | devsq [N] | ctl (max deviation)
__global__ void __launch_bounds__(1024) mix_until_kernel(UntilArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int NT = 1024;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int N = a.n_rows;
    const int C4 = a.chunks;
    const int P = (int)a.n_params;
    const int E4 = N * C4;
    const int nnz = a.nnz;
    float4 *img0 = reinterpret_cast<float4 *>(smem);
    float4 *img1 = img0 + E4;
    float4 *mean = img1 + E4;
    float *lw = reinterpret_cast<float *>(mean + C4);
    int *lcol = reinterpret_cast<int *>(lw + nnz);
    int *lrp = lcol + nnz;
    float *devsq = reinterpret_cast<float *>(lrp + N + 1);
    float *ctl = devsq + N;

    for (int i = tid; i < nnz; i += NT) {
        lw[i] = a.w[i];
        lcol[i] = a.col[i];
    }
    for (int i = tid; i <= N; i += NT) lrp[i] = a.rowptr[i];
    {   // X -> img0, columns P..4*C4 zero (zeros mix to zeros and add nothing to a norm)
        float *f = reinterpret_cast<float *>(img0);
        const int L = 4 * C4;
        for (int i = tid; i < N * L; i += NT) {
            const int r = i / L, p = i - r * L;
            f[i] = p < P ? a.x[(int64_t)r * a.ldx + p] : 0.f;
        }
    }
    __syncthreads();

    // max_a ||x_a - mean|| of an image (all threads return the same value)
    auto max_deviation = [&](const float4 *src) {
        for (int c = tid; c < C4; c += NT) {
            float4 s = src[c];
            for (int r = 1; r < N; ++r) {
                const float4 v = src[r * C4 + c];
                s.x = s.x + v.x;
                s.y = s.y + v.y;
                s.z = s.z + v.z;
                s.w = s.w + v.w;
            }
            const float n = (float)N;
            mean[c] = make_float4(s.x / n, s.y / n, s.z / n, s.w / n);
        }
        __syncthreads();
        for (int r = wave; r < N; r += NT / 64) {
            float v = 0.f;
            for (int c = lane; c < C4; c += 64) {
                const float4 x = src[r * C4 + c], m = mean[c];
                const float dx = x.x - m.x, dy = x.y - m.y, dz = x.z - m.z, dw = x.w - m.w;
                v += (dx * dx + dy * dy) + (dz * dz + dw * dw);
            }
            v = mu_wave_sum(v);
            if (lane == 0) devsq[r] = v;
        }
        __syncthreads();
        if (wave == 0) {
            float m = 0.f;
            for (int r = lane; r < N; r += 64) m = fmaxf(m, sqrtf(devsq[r]));
            m = mu_wave_max(m);
            if (lane == 0) ctl[0] = m;
        }
        __syncthreads();
        const float d = ctl[0];
        __syncthreads();   // ctl is rewritten by the next evaluation
        return d;
    };

    const float4 *src = img0;
    float4 *dst = img1;
    int done = 0;
    bool stop;
    if (a.use_eps) {
        const float d = max_deviation(src);
        if (tid == 0 && a.dev_trace) a.dev_trace[0] = d;
        stop = d < a.eps && done >= a.times;
    } else {
        stop = done >= a.times;
    }
    while (!stop && done < a.max_rounds) {
        for (int i = tid; i < E4; i += NT) {
            const int r = i / C4, c = i - r * C4;
            float4 acc = mu_zero4();
            for (int e = lrp[r]; e < lrp[r + 1]; ++e) {
                const float w = lw[e];
                const float4 v = src[lcol[e] * C4 + c];
                acc.x = acc.x + v.x * w;
                acc.y = acc.y + v.y * w;
                acc.z = acc.z + v.z * w;
                acc.w = acc.w + v.w * w;
            }
            dst[i] = acc;
        }
        __syncthreads();
        const float4 *t = src;
        src = dst;
        dst = const_cast<float4 *>(t);
        ++done;
        if (a.use_eps) {
            const float d = max_deviation(src);
            if (tid == 0 && a.dev_trace) a.dev_trace[done] = d;
            stop = d < a.eps && done >= a.times;
        } else {
            stop = done >= a.times;
        }
    }

    {
        const float *f = reinterpret_cast<const float *>(src);
        const int L = 4 * C4;
        for (int i = tid; i < N * L; i += NT) {
            const int r = i / L, p = i - r * L;
            if (p < P) a.y[(int64_t)r * a.ldy + p] = f[i];
        }
    }
    if (tid == 0) {
        a.status[0] = done;
        a.status[1] = stop ? 1 : 0;
    }
}

}  // namespace

int64_t until_lds_bytes(int n_rows, int64_t n_params, int nnz) {
    const int64_t c4 = (n_params + 3) / 4;
    return 2 * (int64_t)n_rows * c4 * 16 + c4 * 16 + 8 * (int64_t)nnz + 4 * (int64_t)(n_rows + 1) +
           4 * (int64_t)n_rows + 16;
}

hipError_t launch_mix_until(const UntilArgs &a, hipStream_t s) {
    const int64_t lds = until_lds_bytes(a.n_rows, a.n_params, a.nnz);
    const void *k = reinterpret_cast<const void *>(mix_until_kernel);
    hipError_t e = allow_full_lds(k);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(mix_until_kernel, dim3(1), dim3(1024), (unsigned)lds, s, a);
    return hipGetLastError();
}

}  // namespace dl
