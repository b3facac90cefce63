// Fused per-agent ANNModel gradients (BASELINE config c3) on fp32 MFMA, one workgroup per agent.
//
// The reference trains every agent's ANNModel (networks/ann_model.py:4-45: 784 -> 150 ReLU ->
// 150 Tanh -> 150 ELU -> 10, torch.nn.CrossEntropyLoss) with its own autograd pass.  The layered
// path (bgemm.hip) runs that as 11 batched GEMM launches; each is a small GEMM (64 batch rows)
// whose per-slice global->LDS latency, not the matrix cores, sets its time.  Here one 512-thread
// workgroup runs an agent's whole forward + cross-entropy + backward:
//   * the three 64 x 150 activations stay in LDS for the whole pass (3 x 39 KiB), and the
//     backward overwrites each in place with its dZ once its weight gradient is done;
//   * only the agent's parameter row of X, its input batch (read twice) and its gradient row of
//     G touch HBM: ~1.7 MB per agent, every byte once;
//   * weights stream through one LDS staging area; a hidden phase's whole weight matrix is in
//     registers (requested during the phase before, load_all_w) while the MFMAs consume it;
//   * weight gradients go from the MFMA accumulators straight into the agent's row of G (the
//     Mixer flatten order, mixer.py:69), and the per-agent loss is summed in a fixed order
//     (deterministic, hipGraph-replay stable);
//   * bias gradients db = sum_b dZ[b][:] ride along in the weight-gradient MFMAs: the layer's
//     input image carries a column of ones at index K (H1/H2/H3 column dh, the last x chunk's
//     column din), whose tile column is db -- no serial 64-row column sums at the phase ends.
// LDS strides per access (ds_read_b32 banks are dword mod 32 per 32-lane half,
// MI355X_MICROARCH.md §LDS):
//   [row][k] images read by 16 rows x 4 k   -> stride = 4 (mod 8)  floats  (36, 156): 2-way (a
//     ds_read_b64 pairing of k that is conflict-free measured no faster: not the bottleneck)
//   [k][col] images read by 16 cols x 4 k   -> stride = 16 (mod 32) floats (176): conflict-free
//   [k][col] images read by 32 cols x 2 k (32x32x2) -> stride = 32 (mod 64) floats (288)
// f32 MFMA (16x16x4) products are exact fp32 fma chains; summation order differs from
// autograd's BLAS, so parity is a tolerance (tests/test_batched_ann_gpu.py).
#include "dl_internal.h"

#include <type_traits>

namespace dl {
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));


constexpr int NTHR = 512;     // 8 waves, 2 per SIMD
constexpr int MB = 64;        // batch rows per agent
constexpr int LDH = 156;      // activation row stride: dh <= 152 columns + zero pad
constexpr int BK = 32;        // K slice of the staged GEMMs
constexpr int LDS1 = 36;      // [row][BK] slices
constexpr int LDT = 176;      // [k][col] slices (cols <= 160)
constexpr int LDZ = 17;       // logits / dZ4 [64][16 (+1)]
constexpr int LDW4 = 156;     // W4 image [16][dh] for the logits

constexpr int H_FLOATS = MB * LDH;                        // one activation buffer
constexpr int STAGE_FLOATS = MB * LDS1 + 160 * LDS1;      // largest staging use (layer 1)
constexpr int Z_FLOATS = MB * LDZ;
constexpr int LDS_FLOATS = 3 * H_FLOATS + STAGE_FLOATS + Z_FLOATS + 16;
static_assert(160 * LDS1 + MB * LDS1 >= 32 * LDT, "staging area holds a [32][176] slice");
static_assert(160 * LDS1 + MB * LDS1 >= 16 * LDW4, "staging area holds W4");
static_assert(LDS_FLOATS * 4 <= kLdsBytes, "fits one CU's LDS");

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

typedef float f32x16 __attribute__((ext_vector_type(16)));
__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}


// ---- fp32 GEMM on the bf16 matrix cores ("bf16x6").  Every fp32 operand x is split exactly into
// three bf16 pieces x = h + m + l (h = bf16(x), m = bf16(x - h), l = bf16(x - h - m); each
// difference is exact, so h + m + l carries x's 24 significand bits).  A product a*b is then
// the six terms whose magnitude reaches 2^-16 |ab|: hh + (hm + mh) + (hl + lh + mm); the three
// dropped terms are below 2^-23 |ab| together, i.e. at fp32 rounding level.  bf16 x bf16
// products are exact in the fp32 accumulators.  hh goes to one accumulator, the five smaller
// terms to a second one that is added at the end, so the big accumulator's rounding is the fp32
// MFMA's own.  v_mfma_f32_16x16x32_bf16 does 16x the FLOPs per cycle of v_mfma_f32_16x16x4_f32,
// so the six products cost 6/16 of the fp32 MFMA time (MI355X_MICROARCH.md, matrix cores).
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mfma_bf(const bf16x8 &a, const bf16x8 &b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// split two floats into their (h, m, l) bf16 pairs (v_cvt_pk_bf16_f32, round to nearest even)
#ifndef DL_SPLIT_PK
#define DL_SPLIT_PK 1
#endif
typedef float f32x2 __attribute__((ext_vector_type(2)));
#if DL_SPLIT_PK
// both lanes of a pair at once: one packed conversion per plane, the bf16 pair widened back to
// fp32 by two bit operations, the remainders by one packed subtraction (exact: x - bf16(x) is
// representable), 9 VALU instructions per pair instead of 17 element-wise ones
__device__ __forceinline__ f32x2 widen2(bf16x2 v) {
    const uint32_t u = __builtin_bit_cast(uint32_t, v);
    return f32x2{__builtin_bit_cast(float, u << 16), __builtin_bit_cast(float, u & 0xffff0000u)};
}
__device__ __forceinline__ void split2(float x0, float x1, bf16x2 &h, bf16x2 &m, bf16x2 &l) {
    const f32x2 x = {x0, x1};
    h = __builtin_convertvector(x, bf16x2);
    const f32x2 r = x - widen2(h);
    m = __builtin_convertvector(r, bf16x2);
    l = __builtin_convertvector(r - widen2(m), bf16x2);
}
#else
__device__ __forceinline__ void split2(float x0, float x1, bf16x2 &h, bf16x2 &m, bf16x2 &l) {
    h = bf16x2{(__bf16)x0, (__bf16)x1};
    const float r0 = x0 - (float)h[0], r1 = x1 - (float)h[1];
    m = bf16x2{(__bf16)r0, (__bf16)r1};
    l = bf16x2{(__bf16)(r0 - (float)m[0]), (__bf16)(r1 - (float)m[1])};
}
#endif

__device__ __forceinline__ void split4(const f32x4 &x, bf16x4 &h, bf16x4 &m, bf16x4 &l) {
    bf16x2 h0, m0, l0, h1, m1, l1;
    split2(x.x, x.y, h0, m0, l0);
    split2(x.z, x.w, h1, m1, l1);
    h = bf16x4{h0[0], h0[1], h1[0], h1[1]};
    m = bf16x4{m0[0], m0[1], m1[0], m1[1]};
    l = bf16x4{l0[0], l0[1], l1[0], l1[1]};
}

__device__ __forceinline__ f32x16 mfma_bf32(const bf16x8 &a, const bf16x8 &b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// the same six products on v_mfma_f32_32x32x16_bf16 (32 x 32 tiles)
__device__ __forceinline__ void mfma32_x6(const bf16x8 &ah, const bf16x8 &am, const bf16x8 &al,
                                          const bf16x8 &bh, const bf16x8 &bm, const bf16x8 &bl,
                                          f32x16 &big, f32x16 &small) {
    small = mfma_bf32(al, bh, small);
    small = mfma_bf32(ah, bl, small);
    small = mfma_bf32(am, bm, small);
    small = mfma_bf32(am, bh, small);
    small = mfma_bf32(ah, bm, small);
    big = mfma_bf32(ah, bh, big);
}

// acc_big += Ah Bh;  acc_small += Al Bh + Ah Bl + Am Bm + Am Bh + Ah Bm  (smallest terms first)
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


// Two LDS images (layer 1 on the fp32 MFMA): slice s + 1 is written into the other image while the
// MFMAs read slice s, so each slice costs one barrier and the LDS writes overlap the matrix work.
// The register set of slice s + 1 was issued two compute phases before it is stored.
template <typename Set, typename Load, typename Store, typename Compute>
__device__ __forceinline__ void pipeline_db(int ns, Load load, Store store, Compute compute) {
    Set A, B;
    load(A, 0);
    if (ns > 1) load(B, 1);
    store(A, 0);
    __syncthreads();
    for (int s = 0; s < ns; s += 2) {
        if (s + 2 < ns) load(A, s + 2);
        compute(s, 0);
        if (s + 1 < ns) store(B, 1);
        __syncthreads();
        if (s + 1 < ns) {
            if (s + 3 < ns) load(B, s + 3);
            compute(s + 1, 1);
            if (s + 2 < ns) store(A, 0);
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------- parameter addressing
// One agent's row of X or G: parameter p -> element address, row-major (base + p) or in the
// engine's column-tiled layout [ceil(P/T)][n_agents][T] (tile p >> sh, lane p & (T - 1)), so the
// same kernel reads the tiled X the c3 round streams at copy speed.
// Offsets are 32-bit (the ABI checks that every offset from an agent's base fits).
template <bool TILED>
struct PRow {
    float *base;        // row-major: X + a * ld;  tiled: X + a * T
    int tstride;        // tiled: n_agents * T
    int sh;             // tiled: log2 T
    __device__ __forceinline__ float *at(int p) const {
        if constexpr (TILED) return base + ((p >> sh) * tstride + (p & ((1 << sh) - 1)));
        return base + p;
    }
};

// [rows][ld] matrix inside a parameter row (a weight or bias, Mixer order offsets)
template <bool TILED>
struct ParMat {
    static constexpr bool kLinear = !TILED;   // element (r, c) at a fixed row stride ld
    PRow<TILED> row;
    int off;
    int ld;
    __device__ __forceinline__ float *at(int r, int c) const { return row.at(off + r * ld + c); }
};

// one gradient value into G (plain store: non-temporal G stores, so that X' and the batch could
// stay in the MALL, measured 3722 vs 3722 steps/s, profiles/HISTORY.md section 5)
__device__ __forceinline__ void gstore(float *p, float v) {
    *p = v;
}

// The G addresses of this lane's part of a finished 32 x 32 MFMA tile: register r holds row
// i0 + (r & 3) + 8 (r >> 2) of column j (C/D map); every store instruction writes two 128-B runs.
// Column j == cols is the ones column of the input image: its values are the bias gradient.
// f(r, address) for every register that lands in the matrix.
template <typename M, typename F>
__device__ __forceinline__ void tile_addrs(int i0, int j, const M &m, int rows, int cols,
                                           const M &bias, F f) {
    if (j > cols) return;
    if (j == cols) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int i = i0 + (r & 3) + 8 * (r >> 2);
            if (i < rows) f(r, bias.at(0, i));
        }
        return;
    }
    if (i0 + 27 < rows) {   // every row of this lane's 16 (i0 + 0..3, + 8.., + 16.., + 24..)
        // one base address per lane, the 16 rows as ld-strided 32-bit offsets from it: no
        // per-store bounds branch (exec juggling) and no 64-bit address math per store
        if constexpr (M::kLinear) {
            float *p = m.at(i0, j);
            const int ld = m.ld;
#pragma unroll
            for (int r = 0; r < 16; ++r) f(r, p + ((r & 3) + 8 * (r >> 2)) * ld);
        } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) f(r, m.at(i0 + (r & 3) + 8 * (r >> 2), j));
        }
        return;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int i = i0 + (r & 3) + 8 * (r >> 2);
        if (i < rows) f(r, m.at(i, j));
    }
}

// What the kernel writes at a G address (dl_mlp_args.out_mode): the gradient g, or (STEP) the
// local SGD step t = x - lr g of the same parameter, rounded fl(x - fl(lr g)) exactly as
// dl_mix_round's fused step (mix_tile.hip sgd_step), so a plain round of T is bit-identical to
// the fused round of X and G -- and reads one matrix instead of two.  x is read from X at the
// element's own address shifted by dx = G - X (the two share the agent-row geometry), into
// registers before the tile's MFMA chain (xo), so its latency hides behind the chain and every
// store of the tile issues back to back.
template <bool STEP>
struct GOut {
    float lr;
    int64_t dx;   // G address - X address of the same element, in floats
    template <typename M>
    __device__ __forceinline__ void prefetch(f32x16 &xo, int i0, int j, const M &m, int rows,
                                             int cols, const M &bias) const {
        if constexpr (STEP)
            tile_addrs(i0, j, m, rows, cols, bias,
                       [&](int r, float *p) { xo[r] = *(const float *)(p - dx); });
    }
    __device__ __forceinline__ void put(float *p, float v, float x) const {
        if constexpr (STEP) gstore(p, x - lr * v);
        else gstore(p, v);
    }
    __device__ __forceinline__ void put(float *p, float v) const {   // x read here (small tiles)
        if constexpr (STEP) gstore(p, *(const float *)(p - dx) - lr * v);
        else gstore(p, v);
    }
};

// Store a finished tile (xo: the prefetched x values of a STEP output).  (Issuing these stores
// interleaved with the next tile's MFMA chain measured slower: dW1 53 -> 64 us.)
template <bool STEP, typename M>
__device__ __forceinline__ void store_tile(const f32x16 &v, const f32x16 &xo, int i0, int j,
                                           const M &m, int rows, int cols, const M &bias,
                                           const GOut<STEP> &o) {
    tile_addrs(i0, j, m, rows, cols, bias, [&](int r, float *p) { o.put(p, v[r], xo[r]); });
}

// plain row-major matrix (the agent's input batch)
struct PlainMat {
    const float *p;
    int64_t ld;
    __device__ __forceinline__ const float *at(int r, int c) const {
        return p + (int64_t)r * ld + c;
    }
};

// ---------------------------------------------------------------- staging (global -> LDS)
// rows x BK slice of a row-major [rows][ld] matrix, columns [k0, k0 + BK), zero outside
// [0, n_rows) x [0, K), into S[r * LDS1 + c].  Register-prefetched: load() then store().
// Every load issues unconditionally from a clamped in-range address and the out-of-range
// elements are zeroed in store(), at the registers' only use: a load the compiler may branch
// around, or a select right after it, makes the wait before the store a vmcnt(0) that drains
// every slice in flight (as the layer-1 producer measured).
template <int ROWS>
struct RowSlice {
    static constexpr int PER = (ROWS * BK + NTHR - 1) / NTHR;
    float v[PER];
    int k0_, nr_, K_;
    template <typename M>
    __device__ __forceinline__ void load(const M &W, int n_rows, int K, int k0) {
        k0_ = k0;
        nr_ = n_rows;
        K_ = K;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x + i * NTHR;
            const int r = e / BK, c = e % BK;
            v[i] = *W.at(r < n_rows ? r : n_rows - 1, k0 + c < K ? k0 + c : K - 1);
        }
    }
    __device__ __forceinline__ void store(float *S) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x + i * NTHR;
            const int r = e / BK, c = e % BK;
            if (e < ROWS * BK) S[r * LDS1 + c] = (r < nr_ && k0_ + c < K_) ? v[i] : 0.f;
        }
    }
};

// float4 form for 16-byte aligned rows (layer 1: x and W1 with din % 4 == 0)
template <int ROWS>
struct RowSlice4 {
    static constexpr int Q = BK / 4;
    static constexpr int PER = (ROWS * Q + NTHR - 1) / NTHR;
    f32x4 v[PER];
    template <typename M>   // 4 consecutive parameters never straddle a tile (T % 4 == 0)
    __device__ __forceinline__ void load(const M &W, int n_rows, int K, int k0) {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x + i * NTHR;
            const int r = e / Q, c = 4 * (e % Q);
            v[i] = (e < ROWS * Q && r < n_rows && k0 + c < K)
                       ? *reinterpret_cast<const f32x4 *>(W.at(r, k0 + c))
                       : f32x4{0.f, 0.f, 0.f, 0.f};
        }
    }
    __device__ __forceinline__ void store(float *S) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x + i * NTHR;
            if (e < ROWS * Q) *reinterpret_cast<f32x4 *>(S + (e / Q) * LDS1 + 4 * (e % Q)) = v[i];
        }
    }
};

// bf16x6 layer-1 planes: x [64][32] and W1 [160][32] bf16 per plane (64-byte rows, no pad),
// split once when the producer waves stage them.  A lane's fragment is 8 consecutive k of one
// row = one ds_read_b128 per plane; the 16-byte chunk c of row n sits at chunk c ^ ((n >> 2) & 3),
// so the 16 rows a read spans cover all 64 banks.
#ifndef DL_L1_RING
#define DL_L1_RING 3
#endif
// layer-1 slices in flight (producer register sets): with the loop-head waits counted, three
// measured best (c3 3881-3891 steps/s against 3830-3868 for four, 3808-3818 for six; two noisy,
// profiles/r14/l1ring*)
constexpr int L1_RING = DL_L1_RING;
#ifndef DL_DW_QUAD
#define DL_DW_QUAD 1   // hidden dW phases: the 25th 32 x 32 tile as four 16 x 16 quadrants
#endif
#ifndef DL_L1_TILING
#define DL_L1_TILING 1   // layer-1 MFMA waves: 2 M-tiles x 5 N-tiles each (0: 1 x 10)
#endif
constexpr int L1P_BYTES = 160 * BK * 2;           // 10240 per plane
__device__ __forceinline__ uint32_t l1_wofs(int n, int k) {   // byte offset in a plane
    return (uint32_t)(n * 64 + ((((k >> 3) ^ (n >> 2)) & 3) << 4) + (k & 7) * 2);
}

// BK rows [k0, k0 + BK) of a row-major [K][ld] matrix, columns [0, n_cols), zero outside, into
// S[kl * LDT + n] (cols < 160)
struct ColSlice {   // loads unconditional, zeroing in store() (see RowSlice)
    static constexpr int PER = BK * 160 / NTHR;  // 10
    float v[PER];
    int k0_, nc_, K_;
    template <typename M>
    __device__ __forceinline__ void load(const M &W, int n_cols, int K, int k0) {
        k0_ = k0;
        nc_ = n_cols;
        K_ = K;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x + i * NTHR;
            const int kl = e / 160, n = e % 160;
            v[i] = *W.at(k0 + kl < K ? k0 + kl : K - 1, n < n_cols ? n : n_cols - 1);
        }
    }
    __device__ __forceinline__ void store(float *S) const {
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x + i * NTHR;
            const int kl = e / 160, n = e % 160;
            S[kl * LDT + n] = (n < nc_ && k0_ + kl < K_) ? v[i] : 0.f;
        }
    }
};

__device__ __forceinline__ float act_fwd(int layer, float z) {
    if (layer == 0) return z > 0.f ? z : 0.f;   // ReLU
    if (layer == 1) return tanhf(z);            // Tanh
    return z > 0.f ? z : expm1f(z);             // ELU(alpha = 1)
}
// derivative through the layer's OUTPUT h (what the forward kept)
__device__ __forceinline__ float act_grad(int layer, float h) {
    if (layer == 0) return h > 0.f ? 1.f : 0.f;
    if (layer == 1) return 1.f - h * h;
    return h > 0.f ? 1.f : h + 1.f;
}

// ------------------------------------------------------------- [64 x 160] output GEMM tiles
// wave w owns M-tile (w & 3) and the five N-tiles 5 * (w >> 2) + t.  acc = sum_k A(m,k) B(n,k)
// with A(m, k) = Alds[m * lda + k] and B(n, k) = Blds[n * LDS1 + k] (staged [n][k] slice) or
// Blds[k * LDT + n] (staged [k][n] slice).
// KS k-steps of 4 (BK / 4: a whole slice; dZ3's K = dout <= 16 needs 4: the slice's rows from
// dout on are zero, exact-zero products, left out)
template <bool B_KMAJOR, int KS = BK / 4>
__device__ __forceinline__ void mma_rows64(f32x4 (&acc)[5], const float *A, int lda,
                                           const float *Bs) {
    // a whole BK slice, software-pipelined: the fragments of k-step s + 1 are read while the
    // five MFMAs of step s issue, so LDS latency hides behind the matrix core instead of
    // alternating with it (the barriers around a slice put all waves in the same phase).  K tails
    // need no guard: staged slices are zero beyond K and LDS holds only finite values.
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m = (wave & 3) * 16 + (lane & 15);
    const int n0 = (wave >> 2) * 80 + (lane & 15);
    float a[2], b[2][5];
    auto read = [&](int s, int buf) {
        const int k = 4 * s + (lane >> 4);
        a[buf] = A[m * lda + k];
#pragma unroll
        for (int t = 0; t < 5; ++t) {
            const int n = n0 + 16 * t;
            b[buf][t] = B_KMAJOR ? Bs[k * LDT + n] : Bs[n * LDS1 + k];
        }
    };
    read(0, 0);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
        if (s + 1 < KS) read(s + 1, (s + 1) & 1);
#pragma unroll
        for (int t = 0; t < 5; ++t) acc[t] = mfma4(a[s & 1], b[s & 1][t], acc[t]);
    }
}

__device__ __forceinline__ void zero(f32x4 (&acc)[5]) {
#pragma unroll
    for (int t = 0; t < 5; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// C/D fragment -> (row, col) of the [64 x 160] output: row = 16 (w & 3) + 4 (lane >> 4) + r,
// col = 80 (w >> 2) + 16 t + (lane & 15)
template <typename F>
__device__ __forceinline__ void epi_rows64(const f32x4 (&acc)[5], F f) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            f((wave & 3) * 16 + 4 * (lane >> 4) + r, (wave >> 2) * 80 + 16 * t + (lane & 15),
              acc[t][r]);
}

// The five bias values of this lane's output columns (epi_rows64's n for t = 0..4), loaded
// before the layer's MFMAs so their latency hides behind them instead of stalling the epilogue.
template <typename M>
__device__ __forceinline__ void load_bias5(const M &bias, int dh, float (&bv)[5]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int t = 0; t < 5; ++t) {
        const int n = (wave >> 2) * 80 + 16 * t + (lane & 15);
        bv[t] = n < dh ? *bias.at(0, n) : 0.f;
    }
}

// epi_rows64 with the N-tile index t passed along (for per-column values held in registers)
template <typename F>
__device__ __forceinline__ void epi_rows64_t(const f32x4 (&acc)[5], F f) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            f((wave & 3) * 16 + 4 * (lane >> 4) + r, (wave >> 2) * 80 + 16 * t + (lane & 15), t,
              acc[t][r]);
}

// ---- bf16x6 hidden phases (X6).  A staged weight slice is split once, by the threads that stage
// it, into three bf16 planes [160 n][32 k] (l1_wofs layout, as layer 1's W1 planes: a lane's B
// fragment is one ds_read_b128 per plane).  The LDS-resident fp32 activation operand is split per
// fragment in registers (8 consecutive k of one row: two ds_read_b128).  Per K slice a wave then
// issues 30 bf16 MFMAs (16 cycles each) instead of 40 fp32 ones (32 cycles each) and 17 wide LDS
// reads instead of 48 ds_read_b32.
constexpr int HPL = 160 * BK * 2;   // bytes per plane
static_assert(3 * HPL <= STAGE_FLOATS * 4, "three W planes fit the staging area");
typedef float f32x2 __attribute__((ext_vector_type(2)));

// forward: B(n, k) = W[n][k0 + k], rows [0, n_rows), as 8-byte pairs (even dh, even offsets)
struct RowPairs {
    static constexpr int PER = 160 * BK / 2 / NTHR;   // 5 pairs per thread
    f32x2 v[PER];
    int k0_, nr_, K_;
    template <typename M>
    __device__ __forceinline__ void load(const M &W, int n_rows, int K, int k0) {
        k0_ = k0;
        nr_ = n_rows;
        K_ = K;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x + i * NTHR;
            const int r = e / (BK / 2), c = 2 * (e % (BK / 2));
            v[i] = *reinterpret_cast<const f32x2 *>(
                W.at(r < n_rows ? r : n_rows - 1, k0 + c < K ? k0 + c : K - 2));
        }
    }
    __device__ __forceinline__ void store(float *S) const {
        char *pl = reinterpret_cast<char *>(S);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x + i * NTHR;
            const int r = e / (BK / 2), c = 2 * (e % (BK / 2));
            const f32x2 x = (r < nr_ && k0_ + c < K_) ? v[i] : f32x2{0.f, 0.f};
            bf16x2 h, m, l;
            split2(x.x, x.y, h, m, l);
            const uint32_t o = l1_wofs(r, c);
            *reinterpret_cast<bf16x2 *>(pl + o) = h;
            *reinterpret_cast<bf16x2 *>(pl + HPL + o) = m;
            *reinterpret_cast<bf16x2 *>(pl + 2 * HPL + o) = l;
        }
    }
};

// backward: B(n, k) = W[k0 + k][n] (rows k of W, K = dk), staged transposed into the same planes;
// a thread holds rows k, k + 1 of one column n (two coalesced scalar loads)
struct ColPairs {
    static constexpr int PER = 160 * BK / 2 / NTHR;   // 5
    float v0[PER], v1[PER];
    int k0_, nc_, K_;
    template <typename M>
    __device__ __forceinline__ void load(const M &W, int n_cols, int K, int k0) {
        k0_ = k0;
        nc_ = n_cols;
        K_ = K;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x + i * NTHR;
            const int n = e % 160, k = k0 + 2 * (e / 160);
            const int nn = n < n_cols ? n : n_cols - 1;
            v0[i] = *W.at(k < K ? k : K - 1, nn);
            v1[i] = *W.at(k + 1 < K ? k + 1 : K - 1, nn);
        }
    }
    __device__ __forceinline__ void store(float *S) const {
        char *pl = reinterpret_cast<char *>(S);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int e = threadIdx.x + i * NTHR;
            const int n = e % 160, kl = 2 * (e / 160), k = k0_ + kl;
            const bool ok = n < nc_;
            bf16x2 h, m, l;
            split2(ok && k < K_ ? v0[i] : 0.f, ok && k + 1 < K_ ? v1[i] : 0.f, h, m, l);
            const uint32_t o = l1_wofs(n, kl);
            *reinterpret_cast<bf16x2 *>(pl + o) = h;
            *reinterpret_cast<bf16x2 *>(pl + HPL + o) = m;
            *reinterpret_cast<bf16x2 *>(pl + 2 * HPL + o) = l;
        }
    }
};

__device__ __forceinline__ bf16x8 cat8(const bf16x4 &a, const bf16x4 &b) {
    return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// split 8 consecutive fp32 values (two float4) into their three bf16x8 planes
__device__ __forceinline__ void split8(const f32x4 &x0, const f32x4 &x1, bf16x8 &h, bf16x8 &m,
                                       bf16x8 &l) {
    bf16x4 h0, m0, l0, h1, m1, l1;
    split4(x0, h0, m0, l0);
    split4(x1, h1, m1, l1);
    h = cat8(h0, h1);
    m = cat8(m0, m1);
    l = cat8(l0, l1);
}

// One K slice of the [64 x 160] output on the bf16 cores: acc/sml[t] += A[m][0..31] B[n][0..31]
// for this wave's M-tile (w & 3) and N-tiles 5 (w >> 2) + t (epi_rows64's C/D map).  A is fp32
// [m][lda] in LDS (16-byte aligned rows), B the three staged planes.
__device__ __forceinline__ void mma_x6_rows64(f32x4 (&acc)[5], f32x4 (&sml)[5], const float *A,
                                              int lda, const float *Bp) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m = (wave & 3) * 16 + (lane & 15), q = lane >> 4;
    const char *pl = reinterpret_cast<const char *>(Bp);
    const f32x4 *ar = reinterpret_cast<const f32x4 *>(A + m * lda + 8 * q);
    bf16x8 ah, am, al;
    split8(ar[0], ar[1], ah, am, al);
#pragma unroll
    for (int t = 0; t < 5; ++t) {
        const uint32_t ob = l1_wofs((wave >> 2) * 80 + 16 * t + (lane & 15), 8 * q);
        const bf16x8 bh = *reinterpret_cast<const bf16x8 *>(pl + ob);
        const bf16x8 bm = *reinterpret_cast<const bf16x8 *>(pl + HPL + ob);
        const bf16x8 bl = *reinterpret_cast<const bf16x8 *>(pl + 2 * HPL + ob);
        mfma_x6(ah, am, al, bh, bm, bl, acc[t], sml[t]);
    }
}

// Whole-matrix register sets for the hidden phases : every K slice of a hidden weight
// (dh <= 160 -> five slices, 10 floats per thread each) is requested at once, and each set is
// re-issued with the NEXT phase's slice of the same index as soon as its own slice is in LDS
// ("rolling"): the next phase's weights are in flight during this phase's remaining MFMAs and
// epilogue, so a phase waits one HBM latency at most instead of one per pair of slices (the
// two-slice pipeline was latency-bound: the same phases without MFMAs took 6-9 us of 10-12).
// Five slices run whatever dh is (slices past dh stage zeros: exact zero products), so every
// load and store is unconditional and the waits before the stores stay counted.
constexpr int NSL = 5;
static_assert(NSL * BK >= 152, "five K slices cover dh <= 152");
template <typename Set, typename M>
__device__ __forceinline__ void load_all_w(Set (&w)[NSL], const M &W, int dh) {
#pragma unroll
    for (int s = 0; s < NSL; ++s) w[s].load(W, dh, dh, s * BK);
}
template <typename Set, typename M>
__device__ __forceinline__ void load_all_wt(Set (&w)[NSL], const M &W, int dk, int dh) {
#pragma unroll
    for (int s = 0; s < NSL; ++s) w[s].load(W, dh, dk, s * BK);
}

// Forward hidden layer from a whole-matrix set: roll(s) runs right after slice s is stored (it
// re-issues w[s] with the next phase's slice s, or does nothing).
// X6: W slices staged as bf16 planes (RowPairs) and the MFMAs on the bf16 cores; else fp32
// [n][k] slices (RowSlice) on the fp32 MFMA.
template <bool X6, typename M, typename Set, typename Roll>
__device__ __forceinline__ void forward_hidden_all(const M &bias, int dh, const float *Hin,
                                                   float *Hout, float *stage, int layer,
                                                   Set (&w)[NSL], Roll roll) {
    f32x4 acc[5], sml[5];
    zero(acc);
    zero(sml);
    float bv[5];
    load_bias5(bias, dh, bv);
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
        w[s].store(stage);
        __syncthreads();
        roll(s);
        if constexpr (X6) mma_x6_rows64(acc, sml, Hin + s * BK, LDH, stage);
        else mma_rows64<false>(acc, Hin + s * BK, LDH, stage);
        __syncthreads();
    }
    if constexpr (X6) {
#pragma unroll
        for (int t = 0; t < 5; ++t) acc[t] += sml[t];
    }
    epi_rows64_t(acc, [&](int m, int n, int t, float v) {
        if (n < dh) Hout[m * LDH + n] = act_fwd(layer, v + bv[t]);
    });
}

// Backward through a hidden layer from a whole-matrix set of W^T slices (K = dk <= 160 rows)
// X6: W^T slices staged as transposed bf16 planes (ColPairs); else fp32 [k][n] (ColSlice)
template <bool X6, typename Set, typename Roll>
__device__ __forceinline__ void backward_dz_all(int dh, const float *dZ, int ldz, float *Hio,
                                                float *stage, int layer, Set (&w)[NSL],
                                                Roll roll) {
    f32x4 acc[5], sml[5];
    zero(acc);
    zero(sml);
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
        w[s].store(stage);
        __syncthreads();
        roll(s);
        if constexpr (X6) mma_x6_rows64(acc, sml, dZ + s * BK, ldz, stage);
        else mma_rows64<true>(acc, dZ + s * BK, ldz, stage);
        __syncthreads();
    }
    if constexpr (X6) {
#pragma unroll
        for (int t = 0; t < 5; ++t) acc[t] += sml[t];
    }
    epi_rows64(acc, [&](int m, int n, float v) {
        if (n < dh) Hio[m * LDH + n] = v * act_grad(layer, Hio[m * LDH + n]);
    });
}

// dZ3 = (dZ4 W4) * elu'(H3) in place: K = dout <= BK, so one W4^T slice (A, issued during the
// layer-3 forward); next() runs after the MFMAs, before the epilogue.
template <typename Next>
__device__ __forceinline__ void backward_dz_one(int dh, const float *dZ, int ldz, float *Hio,
                                                float *stage, int layer, const ColSlice &A,
                                                Next next) {
    f32x4 acc[5];
    zero(acc);
    A.store(stage);
    __syncthreads();
    mma_rows64<true, 4>(acc, dZ, ldz, stage);   // K = dout <= 16
    __syncthreads();
    next();
    epi_rows64(acc, [&](int m, int n, float v) {
        if (n < dh) Hio[m * LDH + n] = v * act_grad(layer, Hio[m * LDH + n]);
    });
}

// Weight gradient of a hidden layer: dW[i][j] = sum_b dZ[b][i] Hin[b][j] (both LDS-resident,
// [64][LDH]), i, j < dh, straight into G; bias gradient db[i] = sum_b dZ[b][i] from Hin's ones
// column j = dh (N-tile 4).
// 25 tiles of 32 x 32 (v_mfma_f32_32x32x2_f32: half the operand reads of 16x16x4 per flop),
// wave w computes tiles w, w + 8, w + 16 (, 24) one after the other, so each tile's stores
// overlap the next tile's MFMAs (one accumulator: the 32x32x2 issue interval equals its
// dependent latency).  C/D: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5): every
// store instruction writes two 128-B runs.
template <bool STEP, typename M>
__device__ __forceinline__ void weight_grad_hidden(const float *dZ, const float *Hin, int dh,
                                                   const M &gW, const M &gb,
                                                   const GOut<STEP> &o) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // tiles 0..23 three per wave; the 25th (rows and columns 128..159) as four 16 x 16 quadrants
    // on waves 4..7 -- one per SIMD -- instead of a fourth whole tile on wave 0, whose SIMD then
    // ran seven tiles against six (DL_DW_QUAD=0: the whole tile)
    constexpr int NT = DL_DW_QUAD ? 24 : 25;
    for (int t = wave; t < NT; t += 8) {    // one tile at a time (one accumulator)
        f32x16 acc, xo;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
        const int ia = (t / 5) * 32 + (lane & 31), jb = (t % 5) * 32 + (lane & 31);
        o.prefetch(xo, (t / 5) * 32 + 4 * (lane >> 5), jb, gW, dh, dh, gb);
#pragma unroll 8
        for (int ks = 0; ks < MB / 2; ++ks) {
            const int b = 2 * ks + (lane >> 5);
            acc = mfma32(dZ[b * LDH + ia], Hin[b * LDH + jb], acc);
        }
        store_tile(acc, xo, (t / 5) * 32 + 4 * (lane >> 5), jb, gW, dh, dh, gb, o);
    }
    if (DL_DW_QUAD && wave >= 4 && dh > 128) {
        const int q = wave - 4, i0 = 128 + 16 * (q >> 1), j0 = 128 + 16 * (q & 1);
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < MB / 4; ++ks) {
            const int b = 4 * ks + (lane >> 4);
            acc = mfma4(dZ[b * LDH + i0 + (lane & 15)], Hin[b * LDH + j0 + (lane & 15)], acc);
        }
        const int j = j0 + (lane & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = i0 + 4 * (lane >> 4) + r;
            if (i < dh && j < dh) o.put(gW.at(i, j), acc[r]);
            if (i < dh && j == dh) o.put(gb.at(0, i), acc[r]);   // Hin's ones column: the bias
        }
    }
}

struct MlpArgs {
    const float *X;
    int64_t ldx;
    const float *data;
    int64_t s_data;
    const int32_t *labels;
    int64_t s_lab;
    float *G;
    int64_t ldg;
    float *loss;
    int32_t din, dh, dout;
    int32_t tsh;        // column-tiled X and G: log2 of the tile width (0 = row-major)
    int64_t tstride;    // column-tiled: n_agents * T floats per tile
    uint64_t *stamps;   // nullable: per-phase wall clocks of every workgroup (scripts/mlp_probe)
    float lr;           // STEP: G receives x - lr g
    float *ws;          // split path: one [MB][LDH] image per agent (H1, then dZ1 in place)
    int32_t dw_ct;      // split path: dW1 column tiles (32 columns) per workgroup
};

#define STAMP(i) \
    if (p.stamps && threadIdx.x == 0) p.stamps[(int64_t)blockIdx.x * 16 + (i)] = wall_clock64()

// L1X6: layer 1, dW1 and the hidden forward / dZ GEMMs on the bf16 matrix cores with the exact
// 3-way split (bf16x6, above; the hidden dW tiles stay on the fp32 MFMA: a per-fragment split of
// both batch-strided operands measured no faster); false = everything on the fp32 MFMA
// (DLAMD_MLP_L1=fp32, a measurement knob)
// STEP: G receives the local step T = X - lr G instead of the gradient (GOut)
// DZ1_OUT: the two-launch path's first launch (below): dZ1 into p.ws instead of dW1
template <bool TILED, bool L1X6, bool STEP, bool DZ1_OUT = false>
__global__ void __launch_bounds__(NTHR) mlp_fused_kernel(MlpArgs p) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float *H1 = lds, *H2 = lds + H_FLOATS, *H3 = lds + 2 * H_FLOATS;
    float *stage = lds + 3 * H_FLOATS;
    float *Zs = stage + STAGE_FLOATS;
    float *lpart = Zs + Z_FLOATS;
    const int a = blockIdx.x;
    const int din = p.din, dh = p.dh, dout = p.dout;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    PRow<TILED> Xr, Gr;
    if constexpr (TILED) {
        Xr = {const_cast<float *>(p.X) + ((int64_t)a << p.tsh), (int)p.tstride, p.tsh};
        Gr = {p.G + ((int64_t)a << p.tsh), (int)p.tstride, p.tsh};
    } else {
        Xr = {const_cast<float *>(p.X) + (int64_t)a * p.ldx, 0, 0};
        Gr = {p.G + (int64_t)a * p.ldg, 0, 0};
    }
    const float *x = p.data + (int64_t)a * p.s_data;
    const GOut<STEP> go{p.lr, (int64_t)(Gr.base - Xr.base)};
    // parameter offsets in the Mixer flatten order (fc1.w, fc1.b, fc2.w, fc2.b, ...)
    STAMP(0);
    if (p.stamps && threadIdx.x == 0) p.stamps[(int64_t)blockIdx.x * 16 + 14] = __builtin_amdgcn_s_memtime();
    const int o_w1 = 0, o_b1 = dh * din, o_w2 = o_b1 + dh, o_b2 = o_w2 + dh * dh,
              o_w3 = o_b2 + dh, o_b3 = o_w3 + dh * dh, o_w4 = o_b3 + dh, o_b4 = o_w4 + dout * dh;
    using PM = ParMat<TILED>;
    auto mat = [&](const PRow<TILED> &r, int off, int ld) { return PM{r, off, ld}; };

    // a forward phase's whole W, requested during the phase before, and the same for the
    // backward phases' W^T: bf16-plane pair sets (X6) or fp32 slices
    using WSet = std::conditional_t<L1X6, RowPairs, RowSlice<160>>;
    using TSet = std::conditional_t<L1X6, ColPairs, ColSlice>;
    WSet w5[NSL];
    TSet t5[NSL];
    ColSlice ta;            // dZ3's W4^T slice (K = dout)
    // zero all of LDS: K tails and padded tiles then read only finite values (zeros where
    // they meet a zero-filled staged operand), and the activation pads start at zero
    for (int e = tid; e < LDS_FLOATS / 4; e += NTHR)
        reinterpret_cast<f32x4 *>(lds)[e] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    if (tid < MB) H1[tid * LDH + dh] = 1.f;   // ones column: db2 in dW2's MFMAs

    // ---- layer 1: H1 = relu(x W1^T + b1), K = din from HBM: x and W1 slices double-buffered in
    // LDS (the H2/H3 space, free until layer 2), the next two register-prefetched
    if constexpr (L1X6) {
        // Warp-specialised: waves 4-7 (one per SIMD) load slice s + 2 from HBM and split slice
        // s into bf16 planes while waves 0-3 (the other wave of each SIMD) run slice s - 1's
        // MFMAs, one barrier per slice.  (Both roles in every wave, split between barriers,
        // measured: the split VALU and the LDS stores did not overlap the MFMAs -- 47.8 us.)
        // Images: x planes [64][32] and W1 planes [160][32] (bf16, l1_wofs layout), 43 KB each,
        // two of them across H2, H3 and the staging area (contiguous, all free until layer 2).
        constexpr int XPL = MB * BK * 2;                    // 4096 bytes per x plane
        constexpr int IMGB = 3 * XPL + 3 * L1P_BYTES;       // 43008
        static_assert(2 * IMGB <= (2 * H_FLOATS + STAGE_FLOATS) * 4, "two L1 images fit");
        char *img0 = reinterpret_cast<char *>(H2);
        const int ns = (din + BK - 1) / BK;
        if (wave >= 4) {
            const int pt = tid - NTHR / 2;                  // 0..255
            constexpr int XQ = MB * BK / 4 / (NTHR / 2);    // 2 float4 of x per thread
            constexpr int WQ = 160 * BK / 4 / (NTHR / 2);   // 5 float4 of W1 per thread
            f32x4 rx[L1_RING][XQ], rw[L1_RING][WQ];   // L1_RING slices in flight
            const PM W1 = mat(Xr, o_w1, din);
            // Every load instruction issues unconditionally (out-of-range lanes read a clamped
            // in-range address and are zeroed by a select afterwards): a load the compiler may
            // skip -- a branch around it, or a slice not fetched -- makes the number of younger
            // loads unknown, and the wait before a set's LDS store degrades to vmcnt(0), which
            // drains every slice in flight (measured on this kernel: all 61 waits were vmcnt(0)).
            auto load = [&](int set, int sl) {
                const int k0 = sl * BK;
#pragma unroll
                for (int i = 0; i < XQ; ++i) {
                    const int e = pt + i * (NTHR / 2), r = e / 8, c = 4 * (e % 8);
                    rx[set][i] = *reinterpret_cast<const f32x4 *>(
                        x + (int64_t)r * din + (k0 + c < din ? k0 + c : din - 4));
                }
#pragma unroll
                for (int i = 0; i < WQ; ++i) {
                    const int e = pt + i * (NTHR / 2), r = e / 8, c = 4 * (e % 8);
                    rw[set][i] = *reinterpret_cast<const f32x4 *>(
                        W1.at(r < dh ? r : dh - 1, k0 + c < din ? k0 + c : din - 4));
                }
            };
            // the out-of-range lanes are zeroed here, at the registers' only use (a select next
            // to the load would be the load's first use, and the wait would move there)
            auto store = [&](int set, int sl, char *img) {
                const int k0 = sl * BK;
                const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int i = 0; i < XQ; ++i) {
                    const int e = pt + i * (NTHR / 2), r = e / 8, c = 4 * (e % 8);
                    bf16x4 h, m, l;
                    split4(k0 + c < din ? rx[set][i] : z, h, m, l);
                    const uint32_t o = l1_wofs(r, c);
                    *reinterpret_cast<bf16x4 *>(img + o) = h;
                    *reinterpret_cast<bf16x4 *>(img + XPL + o) = m;
                    *reinterpret_cast<bf16x4 *>(img + 2 * XPL + o) = l;
                }
                char *wpl = img + 3 * XPL;
#pragma unroll
                for (int i = 0; i < WQ; ++i) {
                    const int e = pt + i * (NTHR / 2), r = e / 8, c = 4 * (e % 8);
                    bf16x4 h, m, l;
                    split4(r < dh && k0 + c < din ? rw[set][i] : z, h, m, l);
                    const uint32_t o = l1_wofs(r, c);
                    *reinterpret_cast<bf16x4 *>(wpl + o) = h;
                    *reinterpret_cast<bf16x4 *>(wpl + L1P_BYTES + o) = m;
                    *reinterpret_cast<bf16x4 *>(wpl + 2 * L1P_BYTES + o) = l;
                }
            };
            // loads past the last slice re-read it (unconditional issue, see load).  The
            // scheduling barriers keep the first sets' loads in set order: interleaved by the
            // scheduler, the wait before set 0's LDS store at the loop head was vmcnt(0), which
            // drained the whole ring every L1_RING slices.
#pragma unroll
            for (int j = 0; j < L1_RING; ++j) {
                load(j, j < ns ? j : ns - 1);
                __builtin_amdgcn_sched_barrier(0);
            }
            for (int s0 = 0; s0 < ns; s0 += L1_RING) {
#pragma unroll
                for (int j = 0; j < L1_RING; ++j) {   // register set j holds slice s0 + j
                    const int sl = s0 + j;
                    if (sl < ns) store(j, sl, img0 + (sl & 1) * IMGB);
                    load(j, sl + L1_RING < ns ? sl + L1_RING : ns - 1);
                    if (sl < ns) __syncthreads();
                }
            }
        } else {
            // wave c: M-tiles 2 (c & 1), 2 (c & 1) + 1 x N-tiles 5 (c >> 1) .. + 4, so a wave reads
            // 2 A and 5 B fragments (x 3 planes) a slice instead of 1 and 10: the four MFMA waves'
            // LDS reads drop from 132 to 84 KB a slice for the same 60 MFMAs each.  Every tile's
            // products and their order are unchanged.
            constexpr int MT = DL_L1_TILING ? 2 : 1, NT = 10 / MT;
            const int m0 = DL_L1_TILING ? 2 * (wave & 1) : wave, n0 = DL_L1_TILING ? NT * (wave >> 1) : 0;
            f32x4 acc[MT][NT], sml[MT][NT];
#pragma unroll
            for (int mi = 0; mi < MT; ++mi)
#pragma unroll
                for (int t = 0; t < NT; ++t) acc[mi][t] = sml[mi][t] = f32x4{0.f, 0.f, 0.f, 0.f};
            float bv[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int n = 16 * (n0 + t) + (lane & 15);
                bv[t] = n < dh ? *Xr.at(o_b1 + n) : 0.f;
            }
            const int hq = lane >> 4;
            auto compute = [&](const char *img) {
                bf16x8 ah[MT], am[MT], al[MT];
#pragma unroll
                for (int mi = 0; mi < MT; ++mi) {
                    const uint32_t oa = l1_wofs(16 * (m0 + mi) + (lane & 15), 8 * hq);
                    ah[mi] = *reinterpret_cast<const bf16x8 *>(img + oa);
                    am[mi] = *reinterpret_cast<const bf16x8 *>(img + XPL + oa);
                    al[mi] = *reinterpret_cast<const bf16x8 *>(img + 2 * XPL + oa);
                }
                const char *wpl = img + 3 * XPL;
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    const uint32_t ob = l1_wofs(16 * (n0 + t) + (lane & 15), 8 * hq);
                    const bf16x8 bh = *reinterpret_cast<const bf16x8 *>(wpl + ob);
                    const bf16x8 bm = *reinterpret_cast<const bf16x8 *>(wpl + L1P_BYTES + ob);
                    const bf16x8 bl = *reinterpret_cast<const bf16x8 *>(wpl + 2 * L1P_BYTES + ob);
#pragma unroll
                    for (int mi = 0; mi < MT; ++mi)
                        mfma_x6(ah[mi], am[mi], al[mi], bh, bm, bl, acc[mi][t], sml[mi][t]);
                }
            };
            for (int sl = 0; sl < ns; ++sl) {
                if (sl > 0) compute(img0 + ((sl - 1) & 1) * IMGB);
                __syncthreads();
            }
            compute(img0 + ((ns - 1) & 1) * IMGB);
#pragma unroll
            for (int mi = 0; mi < MT; ++mi)
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    acc[mi][t] += sml[mi][t];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = 16 * (m0 + mi) + 4 * hq + r, n = 16 * (n0 + t) + (lane & 15);
                        if (n < dh) H1[row * LDH + n] = act_fwd(0, acc[mi][t][r] + bv[t]);
                    }
                }
        }
        load_all_w(w5, mat(Xr, o_w2, dh), dh);   // layer 2's weights
        __syncthreads();   // every consumer is done with the images before H2/H3 are written
    } else {
        f32x4 acc[5];
        zero(acc);
        float bv[5];
        load_bias5(mat(Xr, o_b1, 0), dh, bv);
        constexpr int IMG = MB * LDS1 + 160 * LDS1;   // one [x | W1] slice image
        static_assert(2 * IMG <= 2 * H_FLOATS, "two slice images fit the H2/H3 space");
        struct L1 {
            RowSlice4<MB> x;
            RowSlice4<160> w;
        };
        pipeline_db<L1>(
            (din + BK - 1) / BK,
            [&](L1 &v, int s) {
                v.x.load(PlainMat{x, din}, MB, din, s * BK);
                v.w.load(mat(Xr, o_w1, din), dh, din, s * BK);
            },
            [&](const L1 &v, int buf) {
                v.x.store(H2 + buf * IMG);
                v.w.store(H2 + buf * IMG + MB * LDS1);
            },
            [&](int s, int buf) {
                mma_rows64<false>(acc, H2 + buf * IMG, LDS1, H2 + buf * IMG + MB * LDS1);
            });
        load_all_w(w5, mat(Xr, o_w2, dh), dh);   // layer 2's weights
        epi_rows64_t(acc, [&](int m, int n, int t, float v) {
            if (n < dh) H1[m * LDH + n] = act_fwd(0, v + bv[t]);
        });
    }
    if (tid < MB) {   // ones columns: db3 in dW3's MFMAs (H2), db4 in dW4's (H3)
        H2[tid * LDH + dh] = 1.f;
        H3[tid * LDH + dh] = 1.f;
    }
    __syncthreads();
    STAMP(1);
    forward_hidden_all<L1X6>(mat(Xr, o_b2, 0), dh, H1, H2, stage, 1, w5,
                       [&](int sl) { w5[sl].load(mat(Xr, o_w3, dh), dh, dh, sl * BK); });
    __syncthreads();
    STAMP(2);
    // the logits' operands from HBM (W4 image values, b4, this wave's labels), issued now so they
    // land while layer 3 runs instead of stalling the head
    constexpr int W4PER = (16 * LDW4 + NTHR - 1) / NTHR;
    float w4v[W4PER];
#pragma unroll
    for (int i = 0; i < W4PER; ++i) {
        const int e = tid + i * NTHR;
        const int n = e / LDW4, k = e % LDW4;
        w4v[i] = (e < 16 * LDW4 && n < dout && k < dh) ? *Xr.at(o_w4 + n * dh + k) : 0.f;
    }
    const float b4v = (lane & 15) < dout ? *Xr.at(o_b4 + (lane & 15)) : 0.f;
    // this lane's two rows of the cross-entropy head (row wave + 8 i, i = 4 pass + lane / 16)
    int lab2[2];
#pragma unroll
    for (int ps = 0; ps < 2; ++ps)
        lab2[ps] = p.labels[(int64_t)a * p.s_lab + wave + 8 * (4 * ps + (lane >> 4))];
    forward_hidden_all<L1X6>(mat(Xr, o_b3, 0), dh, H2, H3, stage, 2, w5, [&](int sl) {
        if (sl == NSL - 1) ta.load(mat(Xr, o_w4, dh), dh, dout, 0);   // dZ3's W4^T (dout <= 16)
    });
    STAMP(3);
    // ---- logits Z = H3 W4^T + b4 (waves 0-3, one 16 x 16 tile each), W4 image [16][LDW4]
#pragma unroll
    for (int i = 0; i < W4PER; ++i) {
        const int e = tid + i * NTHR;
        if (e < 16 * LDW4) stage[e] = w4v[i];
    }
    __syncthreads();
    if (wave < 4) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        const int m = wave * 16 + (lane & 15);
        // fixed trip count (dh <= 152): columns dh.. of the W4 image are zero, so the extra
        // k-steps add exact zeros (H3's ones column meets a zero)
#pragma unroll
        for (int kk = 0; kk < 152; kk += 4) {
            const int k = kk + (lane >> 4);
            acc = mfma4(H3[m * LDH + k], stage[(lane & 15) * LDW4 + k], acc);
        }
        const int n = lane & 15;
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (n < dout) Zs[(wave * 16 + 4 * (lane >> 4) + r) * LDZ + n] = acc[r] + b4v;
    }
    __syncthreads();
    // ---- cross-entropy head (torch.nn.CrossEntropyLoss, mean): dZ4 = (softmax - onehot) / 64
    // Four rows per pass, one per 16-lane group (lane & 15 = the class, dout <= 16): the max and
    // sum butterflies need 4 exchange steps instead of 6, over 2 passes instead of 8 rows one
    // at a time.  The same bits: the 64-lane butterfly's first two steps only combined each
    // value with -inf / +0 from lanes >= dout.  The per-row loss terms go back to lane 0 and are
    // summed in row order, as before.
    {
        const int g = lane >> 4, c = lane & 15;
        float tq[2];
#pragma unroll
        for (int ps = 0; ps < 2; ++ps) {
            const int m = wave + 8 * (4 * ps + g);
            const float v = c < dout ? Zs[m * LDZ + c] : 0.f;
            float mx = c < dout ? v : -INFINITY;
            for (int s = 8; s >= 1; s >>= 1) mx = fmaxf(mx, __shfl_xor(mx, s));
            const float e = c < dout ? expf(v - mx) : 0.f;
            float sum = e;
            for (int s = 8; s >= 1; s >>= 1) sum += __shfl_xor(sum, s);
            const int label = lab2[ps];
            const float zl = __shfl(v, 16 * g + label);
            if (c < dout) Zs[m * LDZ + c] = (e / sum - (c == label ? 1.f : 0.f)) / (float)MB;
            tq[ps] = (logf(sum) + mx - zl) / (float)MB;
        }
        float lsum = 0.f;
#pragma unroll
        for (int i = 0; i < MB / 8; ++i) lsum += __shfl(tq[i / 4], 16 * (i % 4));
        if (lane == 0) lpart[wave] = lsum;
    }
    __syncthreads();
    if (tid == 0 && p.loss)
        p.loss[a] = ((lpart[0] + lpart[1]) + (lpart[2] + lpart[3])) +
                    ((lpart[4] + lpart[5]) + (lpart[6] + lpart[7]));
    STAMP(4);
    // ---- dW4 = dZ4^T H3 [dout x dh] (one M-tile, N-tiles w and w + 8), db4
    {
        for (int nt = wave; nt < 10; nt += 8) {
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
            for (int kk = 0; kk < MB; kk += 4) {
                const int b = kk + (lane >> 4);
                acc = mfma4(Zs[b * LDZ + (lane & 15)], H3[b * LDH + nt * 16 + (lane & 15)], acc);
            }
            const int j = nt * 16 + (lane & 15);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = 4 * (lane >> 4) + r;
                if (i < dout && j < dh) go.put(Gr.at(o_w4 + i * dh + j), acc[r]);
                if (i < dout && j == dh) go.put(Gr.at(o_b4 + i), acc[r]);   // H3's ones column
            }
        }
    }
    __syncthreads();
    // ---- dZ3 = (dZ4 W4) * elu'(H3) in place, K = dout
    backward_dz_one(dh, Zs, LDZ, H3, stage, 2, ta,   // dZ2's W3^T lands during dW3
                    [&] { load_all_wt(t5, mat(Xr, o_w3, dh), dh, dh); });
    __syncthreads();
    STAMP(5);
    weight_grad_hidden(H3, H2, dh, mat(Gr, o_w3, dh), mat(Gr, o_b3, 0), go);
    __syncthreads();
    STAMP(6);
    backward_dz_all<L1X6>(dh, H3, LDH, H2, stage, 1, t5,    // dZ2 into H2; dZ1's W2^T rolls in
                    [&](int sl) { t5[sl].load(mat(Xr, o_w2, dh), dh, dh, sl * BK); });
    __syncthreads();
    STAMP(7);
    weight_grad_hidden(H2, H1, dh, mat(Gr, o_w2, dh), mat(Gr, o_b2, 0), go);
    __syncthreads();
    STAMP(8);
    backward_dz_all<L1X6>(dh, H2, LDH, H1, stage, 0, t5, [](int) {});   // dZ1 into H1
    __syncthreads();
    STAMP(9);
    // ---- dW1 = dZ1^T x [dh x din], K = the 64 batch rows.
    if constexpr (DZ1_OUT) {   // dZ1 (with H1's ones column and zero pads) for mlp_dw1_kernel
        f32x4 *out = reinterpret_cast<f32x4 *>(p.ws + (int64_t)a * H_FLOATS);
        for (int e = tid; e < H_FLOATS / 4; e += NTHR) out[e] = reinterpret_cast<const f32x4 *>(H1)[e];
    } else if constexpr (L1X6) {
        // bf16x6 on v_mfma_f32_32x32x16_bf16.  Both operands are batch-major in LDS, the MFMA
        // wants 8 consecutive k (= batch rows) per lane, so both are split once into bf16 planes
        // stored TRANSPOSED, [row][64 batch] (128-byte rows, 16-byte chunk q of row r at
        // q ^ ((r >> 1) & 7): a 16-lane group of a fragment read covers every bank):
        //   dZ1^T planes [160][64] in the H2/H3 space (free: dZ2, dZ3 consumed), split once;
        //   x chunk planes [96][64] in H1 (free once dZ1 is split), per 96-column chunk, the
        //   next two chunks' x register-prefetched during the MFMAs.
        // Wave items = (N-tile, M-tile) 32 x 32 tiles of the chunk, K = 64 = 4 k-steps x 6
        // products; tiles stored straight into G as before (store_tile).  db1 from x's ones
        // column (din).
        constexpr int CW = 96;                          // chunk columns (3 N-tiles)
        constexpr int ROWB = MB * 2;                    // 128 bytes per transposed plane row
        constexpr int AP = 160 * ROWB;                  // dZ1^T plane bytes
        constexpr int XP = CW * ROWB;                   // x chunk plane bytes
        static_assert(3 * AP <= 2 * H_FLOATS * 4, "dZ1^T planes fit the H2/H3 space");
        static_assert(3 * XP <= H_FLOATS * 4, "x chunk planes fit H1");
        char *aplanes = reinterpret_cast<char *>(H2);
        // x chunk planes, double-buffered so a chunk's planes go in while the previous chunk's
        // tiles run (one barrier a chunk): even chunks in H1, odd ones in the staging area (two
        // planes) and the H2/H3 space past the dZ1^T planes (the third)
        static_assert(2 * XP <= STAGE_FLOATS * 4 && 3 * AP + XP <= 2 * H_FLOATS * 4,
                      "the second x plane buffer fits the staging area and the H2/H3 tail");
        char *xbuf[2][3] = {{reinterpret_cast<char *>(H1), reinterpret_cast<char *>(H1) + XP,
                             reinterpret_cast<char *>(H1) + 2 * XP},
                            {reinterpret_cast<char *>(stage), reinterpret_cast<char *>(stage) + XP,
                             aplanes + 3 * AP}};
        auto tofs = [](int r, int b) {   // byte offset of (row r, batch b) in a transposed plane
            return (uint32_t)(r * ROWB + ((((b >> 3) ^ (r >> 1)) & 7) << 4) + (b & 7) * 2);
        };
        // one item = 4 batch rows x 4 columns: 4 float4 in, 4 columns x 3 planes of bf16x4 out
        auto split_store = [&](const f32x4 (&v)[4], int b0, int c, char *planes, int pbytes) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                bf16x4 h, m, l;
                split4(f32x4{v[0][j], v[1][j], v[2][j], v[3][j]}, h, m, l);
                const uint32_t o = tofs(c + j, b0);
                *reinterpret_cast<bf16x4 *>(planes + o) = h;
                *reinterpret_cast<bf16x4 *>(planes + pbytes + o) = m;
                *reinterpret_cast<bf16x4 *>(planes + 2 * pbytes + o) = l;
            }
        };
        constexpr int XITEMS = (MB / 4) * (CW / 4);    // 384 items per chunk
        f32x4 xva[4], xvb[4];                          // two chunks in flight
        const bool xt = tid < XITEMS;
        // lanes past the items load an item's address too (their registers are never used)
        const int xi = xt ? tid : tid - XITEMS;
        const int xb0 = 4 * (xi / (CW / 4)), xc = 4 * (xi % (CW / 4));
        // Every lane issues its four loads unconditionally from a clamped address, and the
        // columns from din on (the ones column din, db1, then zeros) are substituted at the
        // registers' single use (chunk, below): a load the compiler may branch around made the
        // wait before that use a vmcnt(0), which also drained every G store of the tiles just
        // issued (all nine chunk waits of this phase, in the ISA).
        auto load = [&](f32x4 (&xv)[4], int c0) {
            const int c = c0 + xc < din ? c0 + xc : din - 4;
#pragma unroll
            for (int i = 0; i < 4; ++i)
                xv[i] = *reinterpret_cast<const f32x4 *>(x + (int64_t)(xb0 + i) * din + c);
        };
        load(xva, 0);
        load(xvb, CW);
        // dZ1^T planes from H1 (fp32 [b][LDH]; columns dh.. hold the ones column / zeros and
        // only feed rows >= dh, which store_tile skips)
        for (int e = tid; e < (MB / 4) * 40; e += NTHR) {
            const int b0 = 4 * (e / 40), i0 = 4 * (e % 40);
            f32x4 v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
                v[i] = i0 + 3 < LDH ? *reinterpret_cast<const f32x4 *>(H1 + (b0 + i) * LDH + i0)
                                    : f32x4{0.f, 0.f, 0.f, 0.f};
            split_store(v, b0, i0, aplanes, AP);
        }
        __syncthreads();   // H1 (dZ1 fp32) is read: the x planes may overwrite it
        const int nc = (din + CW) / CW;          // through column din (the ones column)
        const PM gw1 = mat(Gr, o_w1, din), gb1 = mat(Gr, o_b1, 0);
        const int r = lane & 31, hh = lane >> 5;
        // (the barrier after a chunk's planes also orders the previous chunk's tiles, all waves,
        // before the planes of the chunk after it overwrite that buffer)
        auto chunk = [&](int ci, f32x4 (&xv)[4], int odd) {
            char *const *xp = xbuf[odd];
            if (xt) {
                // column din is the ones column (db1); din % 4 == 0 puts it at a float4 start
                const int c = ci * CW + xc;
                f32x4 v[4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    v[i] = c < din ? xv[i]
                           : c == din ? f32x4{1.f, 0.f, 0.f, 0.f} : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    bf16x4 h, m, l;
                    split4(f32x4{v[0][j], v[1][j], v[2][j], v[3][j]}, h, m, l);
                    const uint32_t o = tofs(xc + j, xb0);
                    *reinterpret_cast<bf16x4 *>(xp[0] + o) = h;
                    *reinterpret_cast<bf16x4 *>(xp[1] + o) = m;
                    *reinterpret_cast<bf16x4 *>(xp[2] + o) = l;
                }
            }
            __syncthreads();
            const int c0 = ci * CW;
            // (unconditional: past the last chunk it re-reads the last one, never used)
            load(xv, ci + 2 < nc ? c0 + 2 * CW : (nc - 1) * CW);
            const int ntc = min(CW / 32, (din + 1 - c0 + 31) / 32);
            for (int it = wave; it < 5 * ntc; it += 8) {
                const int nt = it % ntc, t = it / ntc;
                f32x16 big, sml, xo;
#pragma unroll
                for (int q = 0; q < 16; ++q) big[q] = sml[q] = 0.f;
                go.prefetch(xo, 32 * t + 4 * hh, c0 + 32 * nt + r, gw1, dh, din, gb1);
#pragma unroll
                for (int ks = 0; ks < MB / 16; ++ks) {
                    const int b = 16 * ks + 8 * hh;
                    const uint32_t oa = tofs(32 * t + r, b), ob = tofs(32 * nt + r, b);
                    const bf16x8 ah = *reinterpret_cast<const bf16x8 *>(aplanes + oa);
                    const bf16x8 am = *reinterpret_cast<const bf16x8 *>(aplanes + AP + oa);
                    const bf16x8 al = *reinterpret_cast<const bf16x8 *>(aplanes + 2 * AP + oa);
                    const bf16x8 bh = *reinterpret_cast<const bf16x8 *>(xp[0] + ob);
                    const bf16x8 bm = *reinterpret_cast<const bf16x8 *>(xp[1] + ob);
                    const bf16x8 bl = *reinterpret_cast<const bf16x8 *>(xp[2] + ob);
                    mfma32_x6(ah, am, al, bh, bm, bl, big, sml);
                }
                big += sml;
                store_tile(big, xo, 32 * t + 4 * hh, c0 + 32 * nt + r, gw1, dh, din, gb1, go);
            }
        };
        // chunks in pairs, the second of the last pair run even past nc (no tiles then: ntc <= 0),
        // so the loads and waits are the same straight-line code every pair
        for (int ci = 0; ci < nc; ci += 2) {
            chunk(ci, xva, 0);
            chunk(ci + 1, xvb, 1);
        }
    } else {
    // fp32: dW1 by 256-column chunks of x, staged in the H2/H3 space (free now: dZ2 and dZ3
    // are consumed); wave w owns the chunk's 32-column N-tile w and all five 32-row M-tiles
    // (v_mfma_f32_32x32x2_f32); the next chunk is loaded during the MFMAs.  db1.
        constexpr int CW = 256, LDC = 288;   // chunk width, row stride (= 32 mod 64)
        static_assert(MB * LDC <= 2 * H_FLOATS, "x chunk fits the H2/H3 space");
        float *xs = H2;
        constexpr int PER = MB * CW / 4 / NTHR;   // 8 float4 per thread
        f32x4 xv[PER];
        auto load = [&](int c0) {
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int e = tid + i * NTHR;
                const int b = e / (CW / 4), c = 4 * (e % (CW / 4));
                // column din is the ones column (db1); din % 4 == 0 puts it at a float4 start
                xv[i] = c0 + c < din ? *reinterpret_cast<const f32x4 *>(x + (int64_t)b * din + c0 + c)
                        : c0 + c == din ? f32x4{1.f, 0.f, 0.f, 0.f} : f32x4{0.f, 0.f, 0.f, 0.f};
            }
        };
        const int nc = (din + CW) / CW;          // through column din (the ones column)
        const PM gw1 = mat(Gr, o_w1, din), gb1 = mat(Gr, o_b1, 0);
        load(0);
        for (int ci = 0; ci < nc; ++ci) {
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int e = tid + i * NTHR;
                *reinterpret_cast<f32x4 *>(xs + (e / (CW / 4)) * LDC + 4 * (e % (CW / 4))) = xv[i];
            }
            __syncthreads();
            const int c0 = ci * CW;
            if (ci + 1 < nc) load(c0 + CW);
            // (N-tile, M-tile) items of this chunk round-robin over the waves, one 32 x 32 tile at a
            // time: its 16 stores go out while the wave's next tile runs on the matrix core (the
            // G writes of dW1 are a quarter of the kernel's HBM traffic)
            const int ntc = min(CW / 32, (din + 1 - c0 + 31) / 32);
            for (int it = wave; it < 5 * ntc; it += 8) {
                const int nt = it % ntc, t = it / ntc;
                const int nl = 32 * nt + (lane & 31);
                f32x16 acc, xo;
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[r] = 0.f;
                go.prefetch(xo, 32 * t + 4 * (lane >> 5), c0 + nl, gw1, dh, din, gb1);
#pragma unroll 8
                for (int ks = 0; ks < MB / 2; ++ks) {
                    const int b = 2 * ks + (lane >> 5);
                    acc = mfma32(H1[b * LDH + 32 * t + (lane & 31)], xs[b * LDC + nl], acc);
                }
                store_tile(acc, xo, 32 * t + 4 * (lane >> 5), c0 + nl, gw1, dh, din, gb1, go);
            }
            __syncthreads();
        }
    }
    STAMP(10);
    if (p.stamps && threadIdx.x == 0) p.stamps[(int64_t)blockIdx.x * 16 + 15] = __builtin_amdgcn_s_memtime();
}

// ---------------------------------------------------------------- two-launch path
// With a workspace (dl_mlp_args.workspace) dW1 -- the gradient's last phase, 470 KB of G writes
// and the 200 KB batch re-read per agent -- runs as a launch of its own: mlp_fused_kernel<DZ1_OUT>
// writes each agent's dZ1 image ([MB][LDH], H1's ones column at dh, zero pads) into the
// workspace, and mlp_dw1_kernel spreads x's 32-column tiles over two workgroups per agent, each
// with one producer wave staging tiles and five MFMA waves, small LDS, two per CU.  Every split,
// product and summation order is the fused dW1's, so both paths give the same bits
// (tests/test_batched_ann_gpu.py).
constexpr int DW_THR = 384;            // wave 5 stages x tiles, waves 0-4 own dW1 rows 32w..
constexpr int DW_RING = 3;             // x tiles in flight in the producer's registers
constexpr int DW_ROWB = MB * 2;        // 128 bytes per transposed plane row
constexpr int DW_XP = 32 * DW_ROWB;    // one x tile's plane (4096)
__device__ __forceinline__ uint32_t dw_tofs(int r, int b) {   // the fused dW1's plane layout
    return (uint32_t)(r * DW_ROWB + ((((b >> 3) ^ (r >> 1)) & 7) << 4) + (b & 7) * 2);
}

template <bool TILED>
__global__ void __launch_bounds__(DW_THR, 3) mlp_dw1_kernel(MlpArgs p) {
    __shared__ __attribute__((aligned(16))) char xpl[2 * 3 * DW_XP];
    const int din = p.din, dh = p.dh, ct = p.dw_ct;
    const int ntiles = (din + 1 + 31) / 32;          // through the ones column din
    const int wpa = (ntiles + ct - 1) / ct;
    const int a = blockIdx.x / wpa, part = blockIdx.x - a * wpa;
    const int j0 = part * ct, nt = min(ntiles, j0 + ct) - j0;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const float *x = p.data + (int64_t)a * p.s_data;
    if (wave == 5) {
        // items of 2 batch rows x 4 columns, four per lane (256 per tile); every load issues
        // unconditionally from a clamped address, the columns from din on (the ones column din,
        // then zeros) substituted at the single use (fused dW1)
        constexpr int Q = 4;
        f32x4 xv[DW_RING][Q][2];
        auto load = [&](int set, int t) {
            const int j = j0 + t;
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int idx = lane + 64 * q, b0 = 2 * (idx >> 3), xc = 4 * (idx & 7);
                const int c = 32 * j + xc < din ? 32 * j + xc : din - 4;
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    xv[set][q][i] = *reinterpret_cast<const f32x4 *>(x + (int64_t)(b0 + i) * din + c);
            }
        };
        auto store = [&](int set, int t) {
            const int j = j0 + t;
            char *pl = xpl + (t & 1) * (3 * DW_XP);
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const int idx = lane + 64 * q, b0 = 2 * (idx >> 3), xc = 4 * (idx & 7);
                const int c = 32 * j + xc;
                f32x4 v[2];
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    v[i] = c < din ? xv[set][q][i]
                           : c == din ? f32x4{1.f, 0.f, 0.f, 0.f} : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    bf16x2 h, m, l;
                    split2(v[0][jj], v[1][jj], h, m, l);
                    const uint32_t o = dw_tofs(xc + jj, b0);
                    *reinterpret_cast<bf16x2 *>(pl + o) = h;
                    *reinterpret_cast<bf16x2 *>(pl + DW_XP + o) = m;
                    *reinterpret_cast<bf16x2 *>(pl + 2 * DW_XP + o) = l;
                }
            }
        };
        // (loads past the last tile re-read it: unconditional issue.)  The scheduling barriers
        // keep the first sets' loads in set order: interleaved, the wait before set 0's LDS
        // store at the loop head became vmcnt(0), draining the whole ring every DW_RING tiles.
#pragma unroll
        for (int k = 0; k < DW_RING; ++k) {
            load(k, k < nt ? k : nt - 1);
            __builtin_amdgcn_sched_barrier(0);
        }
        for (int s0 = 0; s0 < nt; s0 += DW_RING) {
#pragma unroll
            for (int k = 0; k < DW_RING; ++k) {   // register set k holds tile s0 + k
                const int t = s0 + k;
                if (t < nt) store(k, t);
                load(k, t + DW_RING < nt ? t + DW_RING : nt - 1);
                if (t < nt) __syncthreads();
            }
        }
        return;
    }
    PRow<TILED> Xr, Gr;
    if constexpr (TILED) {
        Xr = {const_cast<float *>(p.X) + ((int64_t)a << p.tsh), (int)p.tstride, p.tsh};
        Gr = {p.G + ((int64_t)a << p.tsh), (int)p.tstride, p.tsh};
    } else {
        Xr = {const_cast<float *>(p.X) + (int64_t)a * p.ldx, 0, 0};
        Gr = {p.G + (int64_t)a * p.ldg, 0, 0};
    }
    const GOut<false> go{0.f, 0};
    const ParMat<TILED> gw1{Gr, 0, din}, gb1{Gr, dh * din, 0};
    const int r = lane & 31, hh = lane >> 5;
    // A: dZ1^T rows 32 wave + r (zero from LDH on, as the fused planes), batch rows
    // 16 ks + 8 hh .. + 7, split once into registers
    bf16x8 ah[MB / 16], am[MB / 16], al[MB / 16];
    {
        const float *dz = p.ws + (int64_t)a * H_FLOATS;
        const int i = 32 * wave + r;
        const int ic = i < LDH ? i : LDH - 1;
#pragma unroll
        for (int ks = 0; ks < MB / 16; ++ks) {
            float v[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const float d = dz[(16 * ks + 8 * hh + q) * LDH + ic];
                v[q] = i < LDH ? d : 0.f;
            }
            split8(f32x4{v[0], v[1], v[2], v[3]}, f32x4{v[4], v[5], v[6], v[7]}, ah[ks], am[ks],
                   al[ks]);
        }
    }
    auto compute = [&](int t) {
        const int j = j0 + t;
        const char *pl = xpl + (t & 1) * (3 * DW_XP);
        f32x16 big, sml, xo = {};   // (xo: the step output's x values, unused here)
#pragma unroll
        for (int q = 0; q < 16; ++q) big[q] = sml[q] = 0.f;
#pragma unroll
        for (int ks = 0; ks < MB / 16; ++ks) {
            const uint32_t ob = dw_tofs(r, 16 * ks + 8 * hh);
            const bf16x8 bh = *reinterpret_cast<const bf16x8 *>(pl + ob);
            const bf16x8 bm = *reinterpret_cast<const bf16x8 *>(pl + DW_XP + ob);
            const bf16x8 bl = *reinterpret_cast<const bf16x8 *>(pl + 2 * DW_XP + ob);
            mfma32_x6(ah[ks], am[ks], al[ks], bh, bm, bl, big, sml);
        }
        big += sml;
        store_tile(big, xo, 32 * wave + 4 * hh, 32 * j + r, gw1, dh, din, gb1, go);
    };
    for (int t = 0; t < nt; ++t) {
        if (t > 0) compute(t - 1);
        __syncthreads();
    }
    compute(nt - 1);
}

}  // namespace

int mlp_fused_supported(int batch, int din, int dh, int dout) {
    return batch == MB && din > 0 && din % 4 == 0 && dh > 0 && dh <= 152 && dh % 2 == 0 && dout > 0 &&
           dout <= 16;
}

size_t mlp_workspace_floats(int n_agents) { return (size_t)n_agents * H_FLOATS; }

hipError_t launch_mlp_fused(const float *X, int64_t ldx, const float *data, int64_t s_data,
                            const int32_t *labels, int64_t s_lab, float *G, int64_t ldg,
                            float *loss, int n_agents, int din, int dh, int dout, int tile_cols,
                            bool step, float lr, float *ws, hipStream_t s) {
    int tsh = 0;
    while (tile_cols > 0 && (1 << tsh) < tile_cols) ++tsh;
    static const bool l1_fp32 = [] {
        const char *v = getenv("DLAMD_MLP_L1");
        return v && v[0] == 'f';
    }();
    // dW1 column tiles per workgroup (split path): 13 = two workgroups per agent
    static const int dw_ct = [] {
        const char *v = getenv("DLAMD_MLP_DW1_CT");
        const int c = v ? atoi(v) : 13;
        return c > 0 ? c : 13;
    }();
    MlpArgs p{X, ldx, data, s_data, labels, s_lab, G, ldg, loss, din, dh, dout, tsh,
              (int64_t)n_agents * tile_cols, nullptr, lr, ws, dw_ct};
    auto go = [&](auto kern) {
        hipError_t e = allow_full_lds(reinterpret_cast<const void *>(kern));
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(kern, dim3((unsigned)n_agents), dim3(NTHR),
                           LDS_FLOATS * sizeof(float), s, p);
        return hipGetLastError();
    };
    auto split = [&](auto head, auto dw1) {
        hipError_t e = go(head);
        if (e != hipSuccess) return e;
        const int wpa = ((din + 1 + 31) / 32 + dw_ct - 1) / dw_ct;
        hipLaunchKernelGGL(dw1, dim3((unsigned)(n_agents * wpa)), dim3(DW_THR), 0, s, p);
        return hipGetLastError();
    };
    auto pick = [&](auto tiled) {
        constexpr bool T = decltype(tiled)::value;
        // (the local-step output keeps one launch)
        if (ws && !l1_fp32 && !step)
            return split(mlp_fused_kernel<T, true, false, true>, mlp_dw1_kernel<T>);
        if (step)
            return l1_fp32 ? go(mlp_fused_kernel<T, false, true>) : go(mlp_fused_kernel<T, true, true>);
        return l1_fp32 ? go(mlp_fused_kernel<T, false, false>) : go(mlp_fused_kernel<T, true, false>);
    };
    return tile_cols > 0 ? pick(std::true_type{}) : pick(std::false_type{});
}

}  // namespace dl
