// Per-agent arithmetic of the reference's asyncio consensus round under its own message
// schedule (utils/consensus_asyncio.py:209-312).  The host façade replays the message protocol
// (who answers which request with which iterate, when DONE is seen) on asyncio; every
// arithmetic step lands here.  Iterates are fp64 slots of a caller-owned arena; a slot index
// plays the role of the numpy array a reference message carries.
//
// Bit-exactness with numpy (fp64, -ffp-contract=off, every product and sum rounded separately):
//   pre-scale (:231)  y0 = (v * w) / m                       in fp64, or in fp32 (NEP 50 weak
//                                                             Python scalars with fp32 values)
//   step (:295)       y' = y * keep + eps * S                keep = 1 - eps*deg, host-computed
//   S = np.sum(list_of_values, axis=0): numpy reduces a (d, P) stack along axis 0 as a left fold
//   from the +0.0 identity when P > 1; a (d,) stack (P == 1, scalar values) along its contiguous
//   axis with the pairwise kernel -- sequential for d < 8, eight interleaved accumulators
//   combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) plus a sequential tail for d >= 8 (checked
//   against numpy 2.2 for d < 40).  All-fp32 inputs (pre-scaled fp32 values) sum in fp32.
//   verdict (:297)    all_j all_p ((y' - v_j) <= conv_eps)   NaN compares false, as in numpy.
#include <cstring>

#include "../../include/dlamd.h"
#include "dl_internal.h"

namespace {

constexpr int kThreads = 256;

template <typename T>
__device__ __forceinline__ T pairwise_sum(const double *const *v, int d) {
    if (d < 8) {
        T r = T(0);
        for (int j = 0; j < d; ++j) r = r + T(*v[j]);
        return r;
    }
    T acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = T(*v[k]);
    int i = 8;
    for (; i < d - (d % 8); i += 8) {
#pragma unroll
        for (int k = 0; k < 8; ++k) acc[k] = acc[k] + T(*v[i + k]);
    }
    T r = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    for (; i < d; ++i) r = r + T(*v[i]);
    return T(0) + r;
}

struct UpdateParams {
    double *arena;
    int64_t ld;
    int64_t n;
    int32_t self_slot, out_slot, n_nbrs, sum_f32;
    int32_t nbr[DL_ASYNC_MAX_NBRS];
    double keep, eps, conv;
    int32_t *flags;
    int32_t parity;
};

__global__ void __launch_bounds__(kThreads) async_update_kernel(UpdateParams a) {
    const double *self = a.arena + (int64_t)a.self_slot * a.ld;
    double *out = a.arena + (int64_t)a.out_slot * a.ld;
    int bad = 0;
    if (a.n == 1) {
        // numpy's contiguous-axis pairwise reduction of a (d,) stack
        if (threadIdx.x == 0 && blockIdx.x == 0) {
            const double *v[DL_ASYNC_MAX_NBRS];
            for (int j = 0; j < a.n_nbrs; ++j) v[j] = a.arena + (int64_t)a.nbr[j] * a.ld;
            const double s = a.sum_f32 ? double(pairwise_sum<float>(v, a.n_nbrs))
                                       : pairwise_sum<double>(v, a.n_nbrs);
            const double t1 = self[0] * a.keep;
            const double t2 = a.eps * s;
            const double y = t1 + t2;
            out[0] = y;
            for (int j = 0; j < a.n_nbrs; ++j) bad |= !((y - *v[j]) <= a.conv);
        }
    } else {
        const int64_t stride = (int64_t)gridDim.x * kThreads;
        for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < a.n; p += stride) {
            double s;
            if (a.sum_f32) {
                float f = 0.0f;
                for (int j = 0; j < a.n_nbrs; ++j) f = f + float(a.arena[(int64_t)a.nbr[j] * a.ld + p]);
                s = double(f);
            } else {
                s = 0.0;
                for (int j = 0; j < a.n_nbrs; ++j) s = s + a.arena[(int64_t)a.nbr[j] * a.ld + p];
            }
            const double t1 = self[p] * a.keep;
            const double t2 = a.eps * s;
            const double y = t1 + t2;
            out[p] = y;
            for (int j = 0; j < a.n_nbrs; ++j)
                bad |= !((y - a.arena[(int64_t)a.nbr[j] * a.ld + p]) <= a.conv);
        }
    }
    bad = __syncthreads_or(bad);
    if (threadIdx.x == 0) {
        if (bad) atomicOr(a.flags + a.parity, 1);
        if (blockIdx.x == 0) a.flags[a.parity ^ 1] = 0;
    }
}

__global__ void __launch_bounds__(kThreads) async_load_kernel(double *y, int64_t n, int mode,
                                                              double w, double m) {
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    for (int64_t p = (int64_t)blockIdx.x * kThreads + threadIdx.x; p < n; p += stride) {
        if (mode == 1) {
            const float t = float(y[p]) * float(w);
            y[p] = double(t / float(m));
        } else {
            const double t = y[p] * w;
            y[p] = t / m;
        }
    }
}

int grid_for(int64_t n) {
    const int64_t g = (n + kThreads - 1) / kThreads;
    return (int)(g < 1 ? 1 : (g > 1024 ? 1024 : g));
}

}  // namespace

extern "C" int dl_async_load(const dl_async_load_args *a, dl_stream_t stream) {
    if (!a || !a->arena || !a->src || a->n_params < 1 || a->ld < a->n_params || a->slot < 0 ||
        (a->mode != 0 && a->mode != 1))
        return dl::fail_msg(DL_ERR_INVALID, "dl_async_load: bad arguments");
    hipStream_t s = static_cast<hipStream_t>(stream);
    double *y = a->arena + (int64_t)a->slot * a->ld;
    hipError_t e = hipMemcpyAsync(y, a->src, (size_t)a->n_params * sizeof(double),
                                  hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return dl::fail_msg(DL_ERR_HIP, "dl_async_load: value upload failed");
    hipLaunchKernelGGL(async_load_kernel, dim3(grid_for(a->n_params)), dim3(kThreads), 0, s, y,
                       a->n_params, a->mode, a->weight, a->mean_weight);
    e = hipGetLastError();
    return e == hipSuccess ? DL_OK : dl::fail_msg(DL_ERR_HIP, "dl_async_load: launch failed");
}

extern "C" int dl_async_update(const dl_async_update_args *a, int32_t *converged_host,
                               dl_stream_t stream) {
    if (!a || !a->arena || !a->flags || a->n_params < 1 || a->ld < a->n_params ||
        a->n_nbrs < 0 || (a->parity != 0 && a->parity != 1))
        return dl::fail_msg(DL_ERR_INVALID, "dl_async_update: bad arguments");
    if (a->n_nbrs > DL_ASYNC_MAX_NBRS)
        return dl::fail_msg(DL_ERR_UNSUPPORTED, "dl_async_update: more than 64 neighbours");
    if (a->self_slot < 0 || a->out_slot < 0 || a->out_slot == a->self_slot)
        return dl::fail_msg(DL_ERR_INVALID, "dl_async_update: bad slot");
    UpdateParams p;
    p.arena = a->arena;
    p.ld = a->ld;
    p.n = a->n_params;
    p.self_slot = a->self_slot;
    p.out_slot = a->out_slot;
    p.n_nbrs = a->n_nbrs;
    p.sum_f32 = a->sum_f32 ? 1 : 0;
    for (int j = 0; j < a->n_nbrs; ++j) {
        if (a->nbr_slots[j] < 0 || a->nbr_slots[j] == a->out_slot)
            return dl::fail_msg(DL_ERR_INVALID, "dl_async_update: bad neighbour slot");
        p.nbr[j] = a->nbr_slots[j];
    }
    for (int j = a->n_nbrs; j < DL_ASYNC_MAX_NBRS; ++j) p.nbr[j] = 0;
    p.keep = a->keep;
    p.eps = a->eps;
    p.conv = a->conv_eps;
    p.flags = a->flags;
    p.parity = a->parity;
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(async_update_kernel, dim3(a->n_params == 1 ? 1 : grid_for(a->n_params)),
                       dim3(kThreads), 0, s, p);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return dl::fail_msg(DL_ERR_HIP, "dl_async_update: launch failed");
    if (converged_host) {
        int32_t bad = 0;
        e = hipMemcpyAsync(&bad, a->flags + a->parity, sizeof(int32_t), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return dl::fail_msg(DL_ERR_HIP, "dl_async_update: verdict readback");
        *converged_host = bad ? 0 : 1;
    }
    return DL_OK;
}

extern "C" int dl_async_read(const double *arena, int64_t ld, int32_t slot, int64_t n_params,
                             double *host_out, dl_stream_t stream) {
    if (!arena || !host_out || n_params < 1 || ld < n_params || slot < 0)
        return dl::fail_msg(DL_ERR_INVALID, "dl_async_read: bad arguments");
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipError_t e = hipMemcpyAsync(host_out, arena + (int64_t)slot * ld,
                                  (size_t)n_params * sizeof(double), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return e == hipSuccess ? DL_OK : dl::fail_msg(DL_ERR_HIP, "dl_async_read: readback failed");
}
