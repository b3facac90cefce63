// Internal launcher interface between the C ABI (capi.hip) and the kernel files.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdlib>

namespace dl {

constexpr int kTileThreads = 1024;      // 16 waves: one workgroup per CU owns a column tile
constexpr int kRowsPerThread = 8;       // prefetch depth: rows x chunks <= 8 * 1024 float4
constexpr int kLdsBytes = 163840;       // 160 KiB LDS per CU on gfx950
constexpr int kMaxChunks = 32;          // T <= 128 columns per tile

struct TileArgs {
    const float *x;
    int64_t ldx;
    const float *halo;
    int64_t ldh;
    const float *g;
    int64_t ldg;
    float *y;
    int64_t ldy;
    const int32_t *rowptr;
    const int32_t *col;
    const float *w;
    int32_t n_rows;   // output rows (local agents)
    int32_t n_src;    // rows staged in LDS = n_loc + n_halo
    int32_t n_loc;    // source rows read from x (and stepped with g); n_rows unless the round
                      // mixes one row set of an agent partition from a wider local window
    int32_t nnz;
    int32_t regular;  // >0: every row has exactly `regular` entries (row_ptr not staged)
    int32_t n_w;      // weights staged in LDS: nnz, or `regular` when every row shares row 0's
    int32_t mean_from_inputs;  // 1: W doubly stochastic -> tile mean taken from the staged t
    int32_t nt_store;          // 1: non-temporal stores of y (FAST path)
    int32_t nt_load;           // non-temporal loads (FAST path): bit 0 x / halo, bit 1 g
    int64_t n_params;
    int32_t n_tiles;
    int64_t col_base; // first column of tile 0
    float lr;
    int32_t vec;      // 1: x/g/y/halo 16-byte aligned and ld % 4 == 0
    uint32_t csr_off; // byte offset of the staged CSR in LDS
    uint32_t scratch_off; // byte offset of the 16 x C float4 mean scratch in LDS
    // FAST-path strides in bytes: tile stride (next tile's row 0) and row stride.
    //   row-major:      xts = T*4,          xrs = ldx*4   (tile base also offset by col_base)
    //   column-tiled:   xts = n_rows*T*4,   xrs = T*4     (block [n_rows][T] per tile)
    int32_t tiled;
    int64_t xts, gts, yts;
    uint32_t xrs, grs, yrs;
    uint32_t hrs;     // halo row stride in bytes (ldh*4)
    int32_t lchunks;     // mix_trace_kernel: float4 chunks per operand tile (1 = row-major)
    float *dev_partial;  // [gridDim.x][n_rows] per-workgroup partial ||y_a - mean||^2
                         // (lagged halo deviation: [gridDim.x][n_loc], one per source row)
    float *mean;         // [n_params] nullable
    unsigned int *dev_max_zero;  // nullable: workgroup 0 zeroes it (dev_reduce's atomicMax target,
                                 // so that launch needs no memset of its own)
    const float *mean_prev;      // halo rounds: global column mean of x (lagged deviation)
    float *colsum_out;           // halo rounds: this rank's column sums of y
    // column-tiled halo (tiled != 0, n_src > n_loc): n_hblk per-peer blocks back to back; block
    // b holds halo rows [hblk_row0[b], hblk_row0[b + 1]) as [n_tiles][rows_b][T], starting
    // hblk_off[b] bytes into `halo`
    int32_t n_hblk;
    int32_t hblk_row0[17];
    uint32_t hblk_off[16];
    // path 5: rows [0, n_hub) folded by four column lanes each; their register heads as
    // {weight, row} pairs at LDS byte offset hub_off
    int32_t n_hub;
    uint32_t hub_off;
    // column-tiled partition rounds (FAST): one kernel tile = `grp` consecutive data tiles of T
    // columns (chunk c of a kernel row is chunk c & (2^cd_sh - 1) of data tile c >> cd_sh), so a
    // short launch moves grp times the bytes per pass; grp = 1 (the default) is the plain tile
    int32_t grp;
    int32_t cd_sh;
    int32_t tile_run;          // 0: workgroup b walks tiles b, b + grid, ...; > 0: the run
                               // [b * tile_run, (b + 1) * tile_run) (DLAMD_TILE_RUN, a knob)
};
constexpr int kMaxHaloBlocks = 16;

// LDS bytes the staged CSR needs (0 if it cannot be staged: > 65535 rows/entries).
// Raise kernel k's dynamic-LDS limit to the whole CU (kLdsBytes), once per (kernel, device):
// launches then make no attribute call, so they are capturable in a hipGraph and carry no
// per-launch driver work.
hipError_t allow_full_lds(const void *k);

// n_w = weights staged (nnz, or the row degree when all rows share one weight sequence).
uint32_t csr_lds_bytes(int32_t n_rows, int32_t nnz, int32_t regular, int32_t n_w);

hipError_t launch_mix_tile(const TileArgs &a, int chunks, bool sgd, bool dev, bool mix, int grid,
                           int lds_bytes, bool fast, hipStream_t s);
// true when a launch of this plan runs the halo instantiation with the lagged deviation
// a round of an agent partition: halo source rows, or output rows that are not the source rows
inline bool tile_partitioned(const TileArgs &a) {
    return a.n_src != a.n_rows || a.n_loc != a.n_rows;
}
inline bool tile_lag(const TileArgs &a) {
    return tile_partitioned(a) && (a.mean_prev != nullptr || a.colsum_out != nullptr);
}
hipError_t launch_mix_gather(const TileArgs &a, bool sgd, hipStream_t s);
// Tile kernel with the CSR in registers (regular graphs of 5 entries per row whose CSR does not
// fit LDS beside the tile): FAST path only, no halo, chunks 1, <= 4 rows per thread.
bool reg_csr_supported(int chunks, int n_rows, int regular, int n_halo);
// ... and its irregular form: every row has >= min_row_nnz entries; the first reg_head_rows()
// of each row in registers, the remaining nnz - head * n_rows entries in LDS (8 B each)
int reg_head_rows(int min_row_nnz);   // 5, 3, 2 or 0 (no register head)
bool reg_tail_supported(int chunks, int n_rows, int head, int n_halo);
// head 0: the regular register-CSR kernel (path 4); head > 0: head + LDS tail (path 5), the
// tail as {weight, row} pairs of 8 B (tail_fmt 2, heads < 5) or weights + u16 rows (1: 6 B)
hipError_t launch_mix_tile_reg(const TileArgs &a, int chunks, int head, int tail_fmt, bool sgd,
                               bool dev, int grid, int lds, hipStream_t s);
// rows per thread (KV) the FAST tile kernels use for n_src rows at `chunks` float4 per row
int tile_passes(int chunks, int n_src, bool fast);
// K rounds of mixing on LDS-resident tiles (mix_multi.hip); FAST tiles only, no halo rows
hipError_t launch_mix_multi(const TileArgs &a, int chunks, int rounds, bool sgd, bool dev,
                            int grid, int lds, hipStream_t s);
// K rounds on LDS-resident column chunks with the per-round max deviation trace
// (mix_trace.hip): mix_trace_kernel + trace_reduce into trace_out[rounds]
constexpr int kTraceRounds = 32;   // rounds per traced pass (per-round deviations in VGPRs)
// mix_trace_rows_kernel at 4 agents per thread keeps 4 agents' CSR offsets and prefetch
// registers: its trace depth is capped so the per-round deviations fit VGPRs (122, no spills)
constexpr int kRowsTraceRounds = 24;
// mix_trace_wide_kernel (1024 < N <= 4096 agents, one chunk per step, KV = 2 or 4 agents per
// thread) keeps every agent's per-round deviation of the pass in registers (KV x rounds VGPRs):
// 16 rounds per pass at KV = 2, 8 at KV = 4 (12 spilled 20-30 VGPRs there)
constexpr int kWideTraceRounds2 = 16;
constexpr int kWideTraceRounds4 = 8;
inline int wide_trace_rounds(int n_rows) {
    return n_rows > 2 * kTileThreads ? kWideTraceRounds4 : kWideTraceRounds2;
}
// the agent-major traced kernel serves register-cached regular graphs at C = 4;
// DLAMD_TRACE_PLANES=1 keeps the chunk-major planes kernel (comparison runs)
inline bool trace_uses_rows(int n_rows, bool in_regs, int chunks) {
    return in_regs && chunks == 4 && n_rows <= kTileThreads &&
           std::getenv("DLAMD_TRACE_PLANES") == nullptr;
}
inline int trace_max_rounds(int n_rows, bool in_regs, int chunks) {
    if (n_rows > kTileThreads) return wide_trace_rounds(n_rows);
    return trace_uses_rows(n_rows, in_regs, chunks) && n_rows > kTileThreads / 2 ? kRowsTraceRounds
                                                                                  : kTraceRounds;
}
hipError_t launch_mix_trace(const TileArgs &a, int chunks, int rounds, int grid, int lds,
                            float *trace_out, hipStream_t s);
// mix_trace_irr_kernel (one image, register head + LDS tail of 8-byte pairs, one 4-column
// chunk per step): irregular graphs of more than 2048 agents and W that are not doubly
// stochastic (general_mean: every round's column mean from its outputs).  KV agents per thread,
// irr_trace_rounds(KV) rounds per pass.
constexpr int irr_trace_kv(int n_rows) {
    return n_rows <= kTileThreads ? 1 : n_rows <= 2 * kTileThreads ? 2 : 4;
}
constexpr int irr_trace_rounds(int kv) { return kv == 1 ? 24 : kv == 2 ? 12 : 4; }
// narrow: 2-column steps (8-byte image entries) and a 6-byte LDS tail, for larger CSRs
hipError_t launch_mix_trace_irr(const TileArgs &a, int head, bool general_mean, bool narrow,
                                int rounds, int grid, int lds, float *trace_out, hipStream_t s);
// max_zeroed: an earlier launch on the stream already zeroed dev_max (TileArgs::dev_max_zero)
hipError_t launch_dev_reduce(const float *partial, int nparts, int n_rows, float *dev_sq,
                             float *dev_max, hipStream_t s, bool max_zeroed = false);
hipError_t launch_column_sum(const float *x, int64_t ldx, int n_rows, int64_t n_params,
                             float *colsum, float scale, hipStream_t s);
hipError_t launch_dev_rows(const float *x, int64_t ldx, int n_rows, int64_t n_params,
                           const float *mean, float *partial, int nparts, hipStream_t s);
int dev_rows_parts(int64_t n_params);
hipError_t launch_stream_copy(const float *src, float *dst, int64_t n_floats, int variant,
                              hipStream_t s);
hipError_t launch_tile_convert(const float *src, float *dst, int64_t ld, int n_rows, int64_t n_params,
                               int tile_cols, bool to_tiled, hipStream_t s);
hipError_t launch_max_column_std(const float *x, int64_t ldx, int n_rows, int64_t n_params,
                                 float *out, hipStream_t s);
hipError_t launch_step_rows(const float *x, int64_t ldx, const float *g, int64_t ldg, float lr,
                            const int32_t *rows, int n_sel, int64_t n_params, float *out,
                            int64_t ldo, hipStream_t s);
// a halo pack's peers: peer b's rows are rows[row0[b], row0[b+1]), its tiled block goes to out[b]
constexpr int kMaxPackPeers = 16;
struct PackPeers {
    int32_t n;
    int32_t row0[kMaxPackPeers + 1];
    float4 *out[kMaxPackPeers];
};
hipError_t launch_step_rows_tiled(const float *x, int x_rows, const float *g, int g_rows,
                                  float lr, const int32_t *rows, const PackPeers &pp,
                                  int64_t n_tiles, int tile_cols, hipStream_t s);
hipError_t launch_sgd_step(const float *x, int64_t ldx, const float *g, int64_t ldg, float *buf,
                           int64_t ldb, float *out, int64_t ldo, int n_rows, int64_t n_params,
                           float lr, float mu, float damp, float wd, int first, int nesterov,
                           bool vec, hipStream_t s);

struct PerronArgs {
    void *y;
    int64_t ldy;
    void *ybuf;       // workspace ping-pong buffer [n_rows, n_params] (multi-tile only)
    int32_t n_rows;
    int64_t n_params;
    const int32_t *rowptr;
    const int32_t *col;
    const double *weight;
    double mean_weight;
    double eps;
    double conv_eps;
    int32_t max_iter;
    int32_t *iters_out;
    int32_t *notconv;  // workspace flag (multi-tile)
    const double *conv_rows;  // nullable per-row conv eps
};
int perron_tile_cols(int dtype, int n_rows, int64_t n_params);
hipError_t launch_perron_single(const PerronArgs &a, int dtype, int tile_cols, hipStream_t s);
hipError_t launch_perron_step(const PerronArgs &a, int dtype, int tile_cols, const void *yin,
                              void *yout, bool prescale, hipStream_t s);

// Mixer.mix(times, eps) loop in one workgroup (mix_until.hip)
struct UntilArgs {
    const float *x;
    int64_t ldx;
    float *y;
    int64_t ldy;
    int64_t n_params;
    int32_t chunks;   // float4 chunks per LDS row: ceil(n_params / 4)
    int32_t n_rows;
    int32_t nnz;
    const int32_t *rowptr;
    const int32_t *col;
    const float *w;
    int32_t times;
    int32_t use_eps;
    float eps;
    int32_t max_rounds;
    int32_t *status;
    float *dev_trace;
};
int64_t until_lds_bytes(int n_rows, int64_t n_params, int nnz);
hipError_t launch_mix_until(const UntilArgs &a, hipStream_t s);

// c1 consensus GD, all agents and iterations in one workgroup (consensus_gd.hip)
struct GdArgs {
    const double *X;
    const double *y;
    const int32_t *shard_ptr;
    int32_t n_agents;
    int32_t n_features;
    const int32_t *rowptr;
    const int32_t *col;
    double eps;
    double conv_eps;
    double mean_weight;
    double tau;
    const double *steps;
    int32_t iterations;
    int32_t max_iter;
    double *w;
    int32_t *iters_out;
    int32_t x_in_lds;
    int64_t x_off;
};
int64_t gd_lds_bytes(int n_agents, int n_features, int rows, bool x_in_lds, int64_t *x_off);
hipError_t launch_consensus_gd(const GdArgs &a, int lds_bytes, hipStream_t s);

enum Epi {
    EPI_NONE = 0,
    EPI_BIAS = 1,
    EPI_BIAS_RELU = 2,
    EPI_BIAS_TANH = 3,
    EPI_BIAS_ELU = 4,
    EPI_DRELU = 5,
    EPI_DTANH = 6,
    EPI_DELU = 7,
    EPI_BIAS_XENT = 8
};

struct BgemmArgs {
    int32_t batch, M, N, K;
    const float *A;
    int64_t lda, sA;
    int32_t ta;
    const float *B;
    int64_t ldb, sB;
    int32_t tb;
    float *C;
    int64_t ldc, sC;
    int32_t epi;
    const float *bias;
    int64_t sBias;
    const float *H;
    int64_t ldh, sH;
    float *rowsum;
    int64_t sR;
    const int32_t *labels;
    int64_t sLab;
    float *loss;
};
hipError_t launch_bgemm(const BgemmArgs &p, hipStream_t s);
hipError_t launch_xent_grad(const float *Z, int64_t sZ, const int32_t *y, int64_t sY, float *dZ,
                            int64_t sD, float *loss, int batch, int rows, int classes,
                            hipStream_t s);

int mlp_fused_supported(int batch, int din, int dh, int dout);
hipError_t launch_mlp_fused(const float *X, int64_t ldx, const float *data, int64_t s_data,
                            const int32_t *labels, int64_t s_lab, float *G, int64_t ldg,
                            float *loss, int n_agents, int din, int dh, int dout, int tile_cols,
                            bool step, float lr, float *ws, hipStream_t s);
// the split gradient path's workspace (dl_mlp_args.workspace), in floats
size_t mlp_workspace_floats(int n_agents);

// sets dl_last_error()'s message (capi.hip) and returns code: for host-only entry points
// defined outside capi.hip
int fail_msg(int code, const char *msg);

}  // namespace dl
