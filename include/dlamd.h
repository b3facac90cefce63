/* dlamd.h -- C ABI of the MI355X consensus-mixing engine (libdlamd.so).
 *
 * The reference (Malkovsky/distributed-learning) is pure Python; it has no native/FFI boundary.
 * Each entry point below replaces one reference Python routine on the gossip hot path and is
 * what a binding (ctypes here) calls in its place:
 *
 *   dl_mix_round        <- Mixer._mix_params_once        utils/consensus_simple/mixer.py:43-49
 *                          (+ the local step x -= lr*g that a training loop runs before mixing,
 *                           Titanic Consensus GD test.ipynb:903-907, and the deviation pass of
 *                           Mixer._get_deviation_dict mixer.py:57-66, fused)
 *   dl_deviation        <- Mixer._get_deviation_dict / _get_max_deviation   mixer.py:51-66
 *   dl_max_column_std   <- Mixer.get_max_parameters_std                     mixer.py:82-84
 *   dl_perron_round     <- ConsensusAgent.run_round mixing loop             consensus_asyncio.py:231-310
 *                          (synchronous Jacobi form: every agent at the same iteration)
 *   dl_async_load / dl_async_update / dl_async_read
 *                       <- ConsensusAgent.run_round's per-agent arithmetic under the reference's
 *                          own message schedule: pre-scale :231, step :295, verdict :297
 *   dl_step_rows        <- (multi-GPU) boundary rows x - lr*g packed for the halo exchange that
 *                          replaces the per-neighbour value messages of consensus_asyncio.py:236-284
 *   dl_column_sum       <- the np.mean numerator of mixer.py:61 (multi-GPU global mean)
 *   dl_mix_rounds       <- Mixer.mix(times=K) with eps=None: K rounds in one HBM pass  mixer.py:18-38
 *   dl_mix_rounds_trace <- Mixer.mix(times, eps) when X does not fit one workgroup: K rounds in
 *                          one HBM pass plus the K per-round max deviations  mixer.py:18-41, 51-66
 *   dl_mix_until        <- Mixer.mix(times, eps): loop, deviation and stop rule in one launch
 *                          mixer.py:18-41
 *   dl_consensus_gd     <- the Titanic notebook's consensus GD run (local logreg steps,
 *                          networks/logreg_model_titanic.py:16-20, + run_round per iteration)
 *   dl_sgd_step, dl_mlp_grad, dl_bgemm, dl_xent_grad <- the per-agent training steps of configs
 *                          c3/c5 (torch.optim.SGD, ANNModel autograd)
 *
 * Conventions
 *   - Every pointer argument is a DEVICE pointer owned by the caller; nothing is allocated inside.
 *     Scratch comes from the caller's workspace (size from the *_workspace_bytes query).
 *   - Calls are stream-ordered and asynchronous (no host synchronisation) unless stated.
 *   - Matrices are row-major: row a = agent a, `ld*` = row stride in elements.
 *   - No exceptions cross the ABI. Return value: 0 on success, otherwise a dl_status code;
 *     dl_last_error() returns a thread-local message for the last failure on this thread.
 *   - Reentrant across streams; the only process-wide state is a per-device property cache.
 */
#ifndef DLAMD_H
#define DLAMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DLAMD_ABI_VERSION 10

typedef void *dl_stream_t; /* hipStream_t; NULL = the legacy default stream */

enum dl_status {
    DL_OK = 0,
    DL_ERR_INVALID = 1,   /* bad argument (shape, null pointer, alias, range) */
    DL_ERR_WORKSPACE = 2, /* workspace too small or misaligned */
    DL_ERR_HIP = 3,       /* a HIP runtime call failed; message has the hipError string */
    DL_ERR_UNSUPPORTED = 4
};

/* Mixing matrix W in CSR form (device pointers).  Row a lists its (source row, weight) pairs in
 * the reference's dict insertion order (mixer.py:47) -- that order is the fp32 summation order,
 * and the result is bit-identical to the reference's left fold when it is kept.  Source rows
 * index [0, n_rows) = local agents, [n_rows, n_rows + n_halo) = halo rows (with
 * dl_mix_args.n_local_src = L: [0, L) local, [L, L + n_halo) halo). */
typedef struct dl_csr {
    const int32_t *row_ptr; /* [n_rows + 1] */
    const int32_t *col;     /* [nnz] */
    const float *w;         /* [nnz] fp32 (the reference casts the Python float to fp32) */
    int32_t n_rows;
    int32_t nnz;
    int32_t uniform_row_nnz; /* > 0 promises row_ptr[a] == a * uniform_row_nnz for every row
                                (regular graphs); lets the LDS kernel skip staging row_ptr.
                                0 = general CSR.  Checked: nnz == n_rows * uniform_row_nnz. */
    int32_t doubly_stochastic; /* 1 promises every column of W sums to 1 (as rows do for the
                                  reference's mixing matrices), so mean(W t) = mean(t): the fused
                                  deviation then takes the column mean from the staged inputs and
                                  needs one LDS pass instead of two.  0 = general W. */
    int32_t shared_row_weights; /* 1 promises (with uniform_row_nnz > 0) that every row's weight
                                   sequence equals row 0's, w[a*d + k] == w[k] bit for bit (a
                                   uniform edge weight: best-constant or analytic FA weights on a
                                   regular graph).  The LDS kernel then stages d weights instead
                                   of nnz, which fits ~2x more agents per tile.  w is still the
                                   full [nnz] array.  0 = per-entry weights. */
    int32_t min_row_nnz; /* (ABI 6) > 0 promises every row has at least this many entries (any
                            graph with a self weight per row: >= 1; Barabasi-Albert m = 2 with
                            self weights: 3).  When the CSR does not fit LDS beside a tile of all
                            agents (thousands of agents, per-edge weights), the tile kernel then
                            keeps each row's first min(min_row_nnz, 5) entries in registers and
                            only the remaining nnz - head * n_rows entries in LDS (plan path 5)
                            instead of taking the gather path.  Checked: min_row_nnz * n_rows <=
                            nnz; a wrong promise gives wrong (never out-of-bounds) results.
                            0 = unknown. */
} dl_csr;

typedef struct dl_mix_args {
    const float *x;     /* [n_rows, ldx] parameters before the round */
    int64_t ldx;
    float *y;           /* [n_rows, ldy] parameters after the round; must not overlap x */
    int64_t ldy;
    int64_t n_params;   /* columns per agent */
    dl_csr W;
    const float *g;     /* nullable [n_rows, ldg]: fused local step x <- x - lr*g first */
    int64_t ldg;
    float lr;
    const float *halo;  /* nullable [n_halo, ldh]: remote rows, already stepped */
    int64_t ldh;
    int32_t n_halo;
    float *dev_sq;      /* nullable [n_rows]: ||y_a - mean_b(y_b)||^2  (n_halo > 0: see mean_prev) */
    float *dev_max;     /* nullable [1]: max_a sqrt(dev_sq[a])          (n_halo > 0: see mean_prev) */
    float *mean;        /* nullable [n_params]: mean_b(y_b)              (needs n_halo == 0) */
    int32_t tile_cols;  /* 0: x, g, y row-major with ld*.  T > 0: x, g, y in the column-tiled
                           layout [ceil(n_params/T)][rows][T] (each tile one contiguous block,
                           last tile zero-padded); T must be the plan's tile_cols
                           (dl_mix_plan_query on the row-major args).  (ABI 8) In this layout
                           ldx / ldg / ldy are the ROWS of each operand's tiled blocks (tile
                           stride ld*T floats), 0 = the default (n_local_src for x and g, n_rows
                           for y): a partition row set passes x / g / y offset by whole rows into
                           wider blocks.  ldh is ignored; the halo is n_halo_blocks tiled blocks
                           (below). */
    /* Agent-partitioned rounds (n_halo > 0) with the deviation pipelined one round behind: the
     * global column mean of y needs every rank's rows, so this round's kernel publishes its
     * share of it and measures the PREVIOUS round's iterate -- its input x, staged anyway --
     * against the previous mean.  No HBM pass beyond the round's own. */
    const float *mean_prev; /* nullable [n_params] (n_halo > 0 or n_local_src > n_rows only; with
                               colsum_out and dev_sq):
                               the global column mean of x (the previous round's all-reduced
                               colsum_out / N): dev_sq[a] = ||x_a - mean_prev||^2, dev_max =
                               max sqrt (nullable).  With dev_sq NULL the round leaves its
                               partial sums in the workspace instead -- rows [0, R) of
                               n_local_src floats, column-tiled layout only, R written to
                               *partial_rows_out (ABI 9: required in this mode) -- for the caller
                               to reduce (one dl_row_sums over several column chunks' partial
                               rows placed back to back); a dev_max is then only set to 0, for
                               that dl_row_sums (max_zeroed = 1). */
    float *colsum_out;      /* nullable [n_params] (as mean_prev): sum over the local source rows of
                               the stepped inputs t = x - lr*g, in a fixed order.  Summed over all
                               ranks it is the column sum of the round's output when the global W
                               is doubly stochastic (the numerator of the next mean_prev). */
    /* Row sets of an agent partition (sharding.py, interior/boundary split): 0 = n_rows.
     * Otherwise source rows [0, n_local_src) come from x (and g, stepped), [n_local_src,
     * n_local_src + n_halo) from halo, and the n_rows OUTPUT rows follow the CSR -- they need
     * not be the first source rows: an interior launch mixes rows [0, n_I) of a rank's window
     * from all its local rows while the halo is in flight; a boundary launch passes x (and g)
     * offset to the first local row the boundary rows read, and y offset to the first boundary
     * row.  Needs n_rows <= n_local_src + n_halo, the LDS tile kernel, no fused exact deviation
     * (dev_sq / dev_max / mean only as the lagged deviation, which is then per SOURCE row:
     * dev_sq[n_local_src]; workspace dl_mix_workspace_bytes(max(n_rows, n_local_src), ...)). */
    int32_t n_local_src;
    /* (ABI 8) Halo rows in the column-tiled layout (tile_cols > 0, n_halo > 0): `halo` holds
     * n_halo_blocks blocks back to back (0 = one block of n_halo rows), block b of
     * halo_block_rows[b] rows laid out [ceil(n_params/T)][halo_block_rows[b]][T] -- one block per
     * peer, so that each peer's halo is ONE contiguous receive buffer of the exchange.  Halo row
     * h of the CSR (source row n_local_src + h) is row h - (rows of blocks before b) of block b.
     * halo_block_rows is a HOST array of n_halo_blocks <= 16 positive counts summing to n_halo.
     * The whole halo must span < 4 GiB.  Row-major layout: n_halo_blocks must be 0. */
    int32_t n_halo_blocks;
    const int32_t *halo_block_rows;
    /* (ABI 8) Plan path 5 only (ignored elsewhere), a performance hint: the first n_hub_rows rows
     * (<= 256; the longest ones first, as in a descending row-length order) are each folded by
     * four lanes, one column each, instead of by one lane.  A Barabasi-Albert hub's CSR row is
     * a serial fp32 fold (the reference's order); split by column it is four shorter scalar
     * chains.  Any value gives the same y bits (each column keeps its left fold), and with a
     * doubly stochastic W the same dev_sq / dev_max / mean bits (the hub lanes add a tile's
     * squared deviations in the owner's order).  With a general W (two-pass deviation) the
     * column mean gathers the hub rows in another lane order, so dev_sq and mean may differ in
     * the last bits across n_hub_rows values.  The kernel uses fewer rows when their register
     * heads do not fit LDS. */
    int32_t n_hub_rows;
    /* (ABI 9) nullable HOST pointer; REQUIRED in the partial-rows mode (a halo round with mean_prev
     * and colsum_out but no dev_sq, see mean_prev), which is refused without it, so a caller that
     * forgets dev_sq gets an error instead of a round with no deviation.  dl_mix_round writes the
     * number of deviation partial rows the launch left in the workspace (0 when it wrote none)
     * before it returns -- on the host, no synchronisation: a caller placing several column
     * chunks' rows back to back starts the next chunk's slice there. */
    int32_t *partial_rows_out;
} dl_mix_args;

/* Which kernel configuration dl_mix_round picks (introspection for tests and the bench). */
typedef struct dl_mix_plan {
    int32_t path;       /* 1 = LDS tile kernel (all agents x T columns per tile), 2 = gather kernel,
                           3 = multi-round LDS kernel (dl_mix_rounds), 4 = tile kernel with the
                           CSR in registers (regular graphs of 5 entries per row whose CSR does
                           not fit LDS beside the tile), 5 = tile kernel with each row's first
                           entries in registers and the rest in LDS (irregular graphs with
                           W.min_row_nnz >= 2 whose CSR does not fit LDS beside the tile) */
    int32_t tile_cols;  /* T: columns per tile (path 1) */
    int32_t grid;       /* workgroups launched */
    int32_t lds_bytes;  /* dynamic LDS per workgroup */
    int32_t n_tiles;    /* tiles one launch walks.  (ABI 9) A column-tiled halo round of few
                           source rows walks groups of 2, 4 or 8 consecutive data tiles as one
                           kernel tile, so n_tiles = n_params / (tile_cols x group) and
                           n_tiles x tile_cols < n_params there; tile_cols stays the data
                           layout's width */
    int32_t regular;    /* 1 if every row has the same entry count (CSR row_ptr not staged) */
    int32_t head;       /* (ABI 8) path 5: CSR entries per row kept in registers (2, 3 or 5);
                           path 4: 5; else 0 */
    int32_t tail_fmt;   /* (ABI 8) path 5: LDS tail entries of 8 B {weight, row} (2) or 6 B (1) */
} dl_mix_plan;

int dl_abi_version(void);
const char *dl_last_error(void);

size_t dl_mix_workspace_bytes(int32_t n_rows, int32_t n_halo, int64_t n_params);
/* Plan from shapes only (no pointers): what dl_mix_round would pick for these sizes, with
 * (deviation) / without the fused deviation.  tile_cols: 0 = row-major operands; > 0 = operands
 * in the column-tiled layout of that width; -1 = choose the width for a column-tiled layout
 * (plan->tile_cols; 0 with the row-major plan if no tile of all rows fits LDS). */
int dl_mix_plan_shape(int32_t n_rows, int32_t n_halo, int64_t n_params, int32_t nnz,
                      int32_t uniform_row_nnz, int32_t shared_row_weights, int32_t deviation,
                      int32_t tile_cols, dl_mix_plan *plan);
/* (ABI 6) The same from a CSR descriptor (only its sizes and flags are read, pointers may be
 * NULL): min_row_nnz included, which dl_mix_plan_shape cannot express (it assumes
 * uniform_row_nnz). */
int dl_mix_plan_csr(const dl_csr *W, int32_t n_halo, int64_t n_params, int32_t deviation,
                    int32_t tile_cols, dl_mix_plan *plan);
int dl_mix_plan_query(const dl_mix_args *args, dl_mix_plan *plan);
int dl_mix_round(const dl_mix_args *args, void *workspace, size_t ws_bytes, dl_stream_t stream);

/* `rounds` consecutive mixing rounds in ONE pass over HBM:  y = W^rounds (x - lr g).
 * Replaces `Mixer.mix(times=rounds)` with eps=None (mixer.py:18-38: `times` calls of
 * _mix_params_once, :43-49, nothing in between) and pure gossip averaging (BASELINE c2).  The
 * mix is column-independent, so each workgroup runs every round on an LDS-resident tile of all
 * agents before writing it back: HBM traffic is that of one round, whatever `rounds` is.  Bit-
 * identical to `rounds` calls of dl_mix_round (same fold order each round).  g (nullable): the
 * local step is applied once, before the first round.  dev_sq / dev_max / mean describe the
 * final iterate and need a doubly stochastic W.  Needs two tile images of all agents in LDS, no
 * halo rows, 16-byte aligned operands and (row-major) n_params a multiple of the tile width;
 * otherwise returns DL_ERR_UNSUPPORTED and the caller loops dl_mix_round.  Workspace:
 * dl_mix_workspace_bytes (deviation only).  dl_mix_rounds_plan reports the configuration
 * (path 3) or DL_ERR_UNSUPPORTED. */
int dl_mix_rounds_plan(const dl_mix_args *args, dl_mix_plan *plan);
/* The same from sizes alone (no operands): the configuration dl_mix_rounds would use for
 * row-major (tile_cols 0) or column-tiled operands of n_rows x n_params, or
 * DL_ERR_UNSUPPORTED.  Lets a caller decide on an LDS slot order before X exists. */
int dl_mix_rounds_plan_shape(int32_t n_rows, int64_t n_params, int32_t nnz,
                             int32_t uniform_row_nnz, int32_t shared_row_weights,
                             int32_t doubly_stochastic, int32_t deviation, int32_t tile_cols,
                             dl_mix_plan *plan);
int dl_mix_rounds(const dl_mix_args *args, int32_t rounds, void *workspace, size_t ws_bytes,
                  dl_stream_t stream);

/* `rounds` mixing rounds in one HBM pass, y = W^rounds x, with the per-round disagreement
 * trace[r] = max_a ||x_a^(r+1) - mean(x^(r+1))||_2 (device float[rounds]) for r < rounds -- what
 * Mixer.mix(times, eps) (mixer.py:18-41) evaluates after every round (_get_max_deviation,
 * :51-55, 57-66).  The caller finds the first round whose value is below eps (and >= times); if
 * it lies inside the pass it re-runs that many rounds from x with dl_mix_rounds / dl_mix_round
 * (x is not modified).  Rounds are the dl_mix_round fold (bit-identical).
 *   W: any CSR.  A doubly stochastic W (W.doubly_stochastic = 1) takes the column mean of x
 *     once (mean(W x) = mean(x)); any other W -- row-stochastic or general -- gets every round's
 *     column mean reduced from that round's own outputs before its deviations (the one-image
 *     kernel, "GM").  Irregular graphs above 2048 agents also take the one-image kernel.
 *   Sizes: 2 <= n_rows <= 4096; no halo rows (n_halo == 0, n_local_src 0 or n_rows); g must be
 *     NULL; n_params % 4 == 0; 16-byte aligned operands, row-major or column-tiled (tile_cols, a
 *     multiple of 4 on the one-image kernel).  Rounds per pass (dl_mix_trace_plan): two-image
 *     kernels 32, or 24 above 512 agents of a register-cached regular graph (degree 4, shared
 *     weights), 16 / 8 above 1024 / 2048 agents; the one-image kernel 24 / 12 / 4 at <= 1024 /
 *     <= 2048 / <= 4096 agents.
 *   LDS: two column images of all agents beside the CSR, or else one image [n_rows] float4 plus
 *     the CSR past each row's register head (min(min_row_nnz, 5) entries) as 8-byte pairs; when
 *     that does not fit, a narrow image [n_rows] float2 with 6-byte tail entries.  Limits: at
 *     most 65535 CSR entries past the register heads, and image + tail + 256 B <= 160 KiB.
 *     Otherwise DL_ERR_UNSUPPORTED (the caller loops dl_mix_round).
 * Workspace: dl_mix_trace_workspace_bytes(n_rows, rounds). */
int dl_mix_trace_plan(const dl_mix_args *args, int32_t *max_rounds);
size_t dl_mix_trace_workspace_bytes(int32_t n_rows, int32_t rounds);
int dl_mix_rounds_trace(const dl_mix_args *args, int32_t rounds, float *trace, void *workspace,
                        size_t ws_bytes, dl_stream_t stream);

/* Mixer.mix(times, eps) (utils/consensus_simple/mixer.py:18-41) as ONE launch: the loop
 *     stop = (!use_eps || max_a ||x_a - mean|| < eps) && done >= times
 *     while (!stop && done < max_rounds) { x <- W x; ++done; }
 * runs on one workgroup with x resident in LDS (two images of n_rows x ceil(n_params/4)*4 fp32
 * plus the CSR: dl_mix_until_fits).  Rounds are the dl_mix_round fold (bit-identical); the
 * deviation is evaluated before the first round and after each one, as the reference does; the
 * test is float32 against float32(eps) (numpy >= 2 semantics of np.float32 < float).
 * status (device int32[2]) receives {rounds done, 1 if the stop rule held / 0 if max_rounds cut
 * the loop}; a caller continues a cut loop with times' = times - done on y.  dev_trace (nullable,
 * device float[max_rounds + 1], use_eps only) receives the max deviation of every evaluation in
 * order (index 0 = before the first round) for the reference's per-round debug log.  y may be x
 * itself (same ld); otherwise it must not overlap x.  W must be square (col < n_rows). */
typedef struct dl_mix_until_args {
    const float *x;     /* [n_rows, ldx] */
    int64_t ldx;
    float *y;           /* [n_rows, ldy]: x after the last round */
    int64_t ldy;
    int64_t n_params;
    dl_csr W;
    int32_t times;      /* minimum rounds (mixer.py:18 `times`, >= 0) */
    int32_t use_eps;    /* 0 = eps None: exactly `times` rounds */
    float eps;          /* float32(eps) */
    int32_t max_rounds; /* >= 1: rounds this launch may run */
    int32_t *status;    /* device int32[2] */
    float *dev_trace;   /* nullable device float[max_rounds + 1] */
} dl_mix_until_args;

/* BASELINE config c1 as one launch: `iterations` rounds of the Titanic notebook's consensus GD
 * (cells 12-14) for every agent, fp64 -- per agent a local step on its shard of the L2-regularised
 * logistic loss (networks/logreg_model_titanic.py:16-20)
 *     w <- w - steps[it] * ( -(sum_i y_i sigmoid(-y_i x_i.w) x_i) / n_a + tau w )
 * then one asyncio consensus round (consensus_asyncio.py:209-312) weighted by the shard sizes n_a:
 * the dl_perron_round Jacobi (pre-scale w n_a / mean_weight, y <- y (1 - eps deg) + eps sum_nbr y,
 * until every agent's one-sided test against its neighbours' previous values holds, at most
 * max_iter iterations).  Agent a owns rows [shard_ptr[a], shard_ptr[a+1]) of X [rows][n_features]
 * and y; row_ptr/col list each agent's neighbours in its socket order (no self loops).  w (device,
 * [n_agents][n_features]) holds the start weights and receives the final ones; iters_out
 * (nullable, device int32[iterations]) the Jacobi iterations of each round.  One workgroup:
 * n_features <= 16, and the agents' values, shards (if they fit LDS, else read from L2) and the
 * step sizes (host-computed, e.g. alpha (it+1)^-0.5) are device memory. */
typedef struct dl_consensus_gd_args {
    const double *X;
    const double *y;
    const int32_t *shard_ptr;   /* [n_agents + 1], shard_ptr[0] == 0 */
    int32_t n_agents;
    int32_t n_features;
    const int32_t *row_ptr;     /* [n_agents + 1] neighbour lists */
    const int32_t *col;
    double eps;                 /* 0.95 / max degree (consensus_asyncio.py:78-86) */
    double conv_eps;
    double mean_weight;         /* mean shard size */
    double tau;
    const double *steps;        /* [iterations] */
    int32_t iterations;
    int32_t max_iter;
    double *w;
    int32_t *iters_out;
} dl_consensus_gd_args;
int dl_consensus_gd(const dl_consensus_gd_args *args, int32_t total_rows, dl_stream_t stream);

/* 1 when dl_mix_until takes these sizes in one workgroup's LDS, else 0. */
int dl_mix_until_fits(int32_t n_rows, int64_t n_params, int32_t nnz);
int dl_mix_until(const dl_mix_until_args *args, dl_stream_t stream);

/* Deviation of x from its column mean: dev_sq[a] = ||x_a - mean||^2, dev_max = max sqrt(dev_sq).
 * mean_in nullable: when given (e.g. a global mean all-reduced across GPUs) it is used instead
 * of the local column mean.  mean_out nullable.  Returns zeros when n_rows <= 1 (mixer.py:58-59). */
size_t dl_deviation_workspace_bytes(int32_t n_rows, int64_t n_params);
int dl_deviation(const float *x, int64_t ldx, int32_t n_rows, int64_t n_params,
                 const float *mean_in, float *dev_sq, float *dev_max, float *mean_out,
                 void *workspace, size_t ws_bytes, dl_stream_t stream);

/* Deviation of x held in the column-tiled layout (see dl_mix_args.tile_cols). */
int dl_deviation_tiled(const float *x, int32_t n_rows, int64_t n_params, int32_t tile_cols,
                       float *dev_sq, float *dev_max, float *mean_out, void *workspace,
                       size_t ws_bytes, dl_stream_t stream);

/* Layout conversion between row-major [n_rows][ld] and column-tiled [ceil(P/T)][n_rows][T]
 * (the resident layout of the engine: one HBM-contiguous block per LDS tile). */
int dl_to_tiled(const float *src, int64_t ld, int32_t n_rows, int64_t n_params, int32_t tile_cols,
                float *dst, dl_stream_t stream);
int dl_from_tiled(const float *src, int32_t n_rows, int64_t n_params, int32_t tile_cols, float *dst,
                  int64_t ld, dl_stream_t stream);

/* colsum[p] = sum_a x[a, p], rows added in order (numerator of np.mean, mixer.py:61). */
int dl_column_sum(const float *x, int64_t ldx, int32_t n_rows, int64_t n_params, float *colsum,
                  dl_stream_t stream);

/* (ABI 9) sums[a] = sum_b parts[b][a] over n_parts rows of n_rows floats (fixed order, fp64), max_sqrt[0]
 * = max_a sqrt(sums[a]); either output nullable.  The per-agent ||x_a - mean||^2 of a round run
 * as several column chunks (their partial rows back to back in parts, see mean_prev), and their
 * max -- the _get_max_deviation of mixer.py:51-55 over the whole round -- in one launch.
 * max_zeroed = 1: max_sqrt already holds 0 (a dl_mix_round given it as dev_max without dev_sq
 * zeroes it), so no memset is queued before the reduce. */
int dl_row_sums(const float *parts, int32_t n_parts, int32_t n_rows, float *sums, float *max_sqrt,
                int32_t max_zeroed, dl_stream_t stream);

/* out[0] = max_p std_a(x[a, p]) (population std, the intent of mixer.py:82-84). */
int dl_max_column_std(const float *x, int64_t ldx, int32_t n_rows, int64_t n_params, float *out,
                      dl_stream_t stream);

/* Host-only (no device work): agent -> LDS image row-slot order for the multi-round kernels'
 * neighbour gathers.  col: [n_rows][degree] neighbour agent ids in CSR entry order (the
 * reference's topology dict order, mixer.py:43-49); chunks: float4 chunks per image row and lane
 * (4 = dl_mix_rounds' agent-major rows at 16 columns, 1 = dl_mix_rounds_trace's chunk-major
 * planes).  A greedy random-swap search over `moves` moves (seeded) that lowers the number of
 * ds_read_b128 16-lane groups' repeated 16-byte bank slots; order[slot] = agent (out, n_rows);
 * conflicts[0] / [1] = extra LDS cycles per round before / after.  Relabelling keeps every row's
 * entry order, so the iterates are bit-identical per agent.  Same objective and move rule as
 * graph.lds_slot_order (Python), with incremental counts.  Not in the reference: it has no
 * device layout to order. */
int dl_lds_slot_order(int32_t n_rows, int32_t degree, const int32_t *col, int32_t chunks,
                      int64_t moves, uint64_t seed, int32_t *order, int64_t *conflicts);

/* out[i, :] = x[rows[i], :] - lr * g[rows[i], :]  (g nullable: plain copy).  Packs the boundary
 * rows a GPU sends to its neighbours in the multi-GPU halo exchange. */
int dl_step_rows(const float *x, int64_t ldx, const float *g, int64_t ldg, float lr,
                 const int32_t *rows, int32_t n_sel, int64_t n_params, float *out, int64_t ldo,
                 dl_stream_t stream);

/* (ABI 8) The same in the column-tiled layout: x [ceil(n_params/T)][x_rows][T] and g (nullable)
 * [..][g_rows][T] -> out [ceil(n_params/T)][n_sel][T] (one peer's halo block of dl_mix_args,
 * padded columns included).  Packs a rank's boundary rows for one peer of the exchange; a column
 * chunk of whole tiles is x / g / out offset to its first tile.  16-byte aligned pointers. */
int dl_step_rows_tiled(const float *x, int32_t x_rows, const float *g, int32_t g_rows, float lr,
                       const int32_t *rows, int32_t n_sel, int64_t n_params, int32_t tile_cols,
                       float *out, dl_stream_t stream);
/* (ABI 8) The same for every peer of an exchange in ONE launch: peer b's rows are
 * rows[row0[b] .. row0[b+1]) and its block [ceil(n_params/T)][row0[b+1] - row0[b]][T] goes to
 * outs[b].  row0 (n_peers + 1 entries, row0[0] = 0) and outs (n_peers device pointers) are HOST
 * arrays; n_peers <= 16.  Both tiled packs store non-temporally (the blocks are read once, by the
 * peers' receives). */
int dl_step_rows_tiled_peers(const float *x, int32_t x_rows, const float *g, int32_t g_rows,
                             float lr, const int32_t *rows, int32_t n_peers, const int32_t *row0,
                             float *const *outs, int64_t n_params, int32_t tile_cols,
                             dl_stream_t stream);

/* Local optimizer step of config c5 (Man_Colab.ipynb cell 19: optimizer = optim.SGD,
 * {'momentum': 0.9, 'weight_decay': 5e-4}, lr 0.02), i.e. torch.optim.SGD.step (torch/optim/sgd.py,
 * single-tensor form) applied to every agent row at once, with torch's rounding (one fma per
 * add-with-alpha):
 *   d = g + wd*x;  buf = first ? d : mu*buf + (1-dampening)*d;  d = nesterov ? d + mu*buf : buf;
 *   out = x - lr*d
 * out may be x itself (in place, as optimizer.step) or a separate buffer, e.g. the input of the
 * following dl_mix_round (the parameters stay put and the round writes them back).  buf
 * (momentum buffer) is read unless `first` and always written when momentum != 0. */
typedef struct dl_sgd_args {
    const float *x; int64_t ldx;    /* [n_rows, ldx] parameters */
    const float *g; int64_t ldg;    /* [n_rows, ldg] gradients */
    float *buf; int64_t ldb;        /* [n_rows, ldb] momentum buffers (nullable if momentum == 0) */
    float *out; int64_t ldo;        /* [n_rows, ldo] stepped parameters (== x or disjoint) */
    int32_t n_rows;
    int64_t n_params;
    float lr, momentum, dampening, weight_decay;
    int32_t nesterov;
    int32_t first;                  /* 1: buf = d (torch's first step: clone of the gradient) */
} dl_sgd_args;
int dl_sgd_step(const dl_sgd_args *args, dl_stream_t stream);

/* dst[i] = src[i] for n_floats floats (float4 streaming copy; variant 0: one load in flight
 * per thread, 1: eight, 2: eight + non-temporal stores, 3: four + non-temporal loads and
 * stores on a 8192-workgroup grid).  Variants 4 and 5 are the triad
 * dst[i] = src[i] - 1e-3 * src[n_floats + i] (src holds 2 * n_floats floats): two read streams
 * and one write stream, the traffic of the fused local step + mix round (12 B per element);
 * 4: one float4 per stream in flight, 512-thread workgroups x 256; 5: four, 256 x 1024; 6: the
 * round's own shape (persistent 1024-thread workgroups on 2 x CUs, 64-KiB blocks per stream,
 * next block loaded before the current one is stored; n_floats % 16384 == 0); all
 * non-temporal.  Not on the reference path: the bench uses them to measure the HBM streaming
 * ceilings next to the mix kernel's achieved bandwidth. */
int dl_stream_copy(const float *src, float *dst, int64_t n_floats, int32_t variant,
                   dl_stream_t stream);

/* One asyncio consensus round (consensus_asyncio.py:209-312) restated as synchronous Jacobi:
 *   y0_a = v_a * weight_a / mean_weight                              (:231)
 *   y_a <- y_a * (1 - eps*deg_a) + eps * sum_{j in N(a)} y_j           (:295, sum then scale)
 *   flag_a = all_j all_p (y_a - y_j_previous <= conv_eps)              (:297, one-sided)
 * iterated until every flag is set (master DONE, :170-174) or max_iter.  `y` holds the values on
 * entry and the result on exit; iters_out (device int32[1]) receives the iteration count.
 * The adjacency (no self loops) lists neighbours in the agent's socket order (:104-114).
 * When all columns fit one tile the loop runs inside one launch; otherwise this call iterates on
 * the host and SYNCHRONISES the stream once per iteration. */
typedef struct dl_perron_args {
    int32_t dtype;            /* 0 = fp32, 1 = fp64 */
    void *y;                  /* [n_rows, ldy] */
    int64_t ldy;
    int32_t n_rows;
    int64_t n_params;
    const int32_t *row_ptr;   /* [n_rows + 1] adjacency */
    const int32_t *col;       /* [nnz] */
    const double *weight;     /* nullable [n_rows]: pre-scale weights (NULL: no pre-scale) */
    double mean_weight;
    double eps;
    double conv_eps;
    int32_t max_iter;
    int32_t *iters_out;       /* device [1] */
    const double *conv_eps_rows; /* nullable [n_rows]: per-agent convergence eps (an agent's own
                                    ConsensusAgent(convergence_eps=...)); overrides conv_eps */
} dl_perron_args;

size_t dl_perron_workspace_bytes(int32_t dtype, int32_t n_rows, int64_t n_params);
int dl_perron_round(const dl_perron_args *args, void *workspace, size_t ws_bytes,
                    dl_stream_t stream);

/* ---------------------------------------------------------------- asyncio message schedule
 * The reference's asyncio round is NOT synchronous Jacobi after the first round: each agent
 * answers REQUEST_VALUE with whatever iterate it holds when the request is served, drops
 * other-round messages (consensus_asyncio.py:276-278) and sees DONE only between exchanges
 * (:241-252, :260-265), so an agent may mix a neighbour's iterate t+1 or t-2 into its own step
 * t, and agents stop at different iteration counts.  The host façade
 * (utils/consensus_asyncio.py) replays that message protocol on asyncio exactly and sends every
 * arithmetic step here.  Iterates live in a caller-owned device arena of fp64 slots
 * ([n_slots][ld]); a message carries a slot index, as the reference's carries its numpy array.
 *
 * dl_async_load: y0 = v * weight / mean_weight (:231) into `slot`.  `src` is HOST memory holding
 *   n_params doubles (the caller converts fp32/int values exactly).  mode 0: numpy computes in
 *   fp64 (fp64 values, or a strong fp64/int64 weight); mode 1: in fp32 (fp32 values with Python
 *   scalar weights, NEP 50) -- weight and mean_weight already rounded to fp32 by the caller.
 *   Stream-ordered; the pageable host copy is consumed before return.
 * dl_async_update: one agent step (:295, :297)
 *     y' = y * keep + eps * S,  S = np.sum([v_0 .. v_{d-1}], axis=0) in arrival order,
 *     converged = all_j all_p ((y' - v_j) <= conv_eps)
 *   keep = 1 - eps*deg (np.float64, computed by the caller), each product and sum rounded
 *   separately.  S follows numpy's reduction exactly: a left fold from +0.0 when n_params > 1;
 *   for n_params == 1 numpy's pairwise sum (8 accumulators once d >= 8); in fp32 when every v_j
 *   is an fp32 pre-scaled value (sum_f32 = 1), else in fp64.  `flags` is a device int32[2]
 *   (zeroed once by the caller): the launch ORs violations into flags[parity] and zeroes
 *   flags[parity ^ 1] for the next launch.  converged_host (nullable): when set, the call copies
 *   the verdict there and SYNCHRONISES the stream (the protocol needs it before the agent's next
 *   message, :301-310).
 * dl_async_read: copies n_params doubles of `slot` to host memory and synchronises the stream. */
#define DL_ASYNC_MAX_NBRS 64
typedef struct dl_async_load_args {
    double *arena;            /* [n_slots][ld] */
    int64_t ld;
    int64_t n_params;
    int32_t slot;
    int32_t mode;             /* 0 = fp64, 1 = fp32 */
    const double *src;        /* host [n_params] */
    double weight;
    double mean_weight;
} dl_async_load_args;
int dl_async_load(const dl_async_load_args *args, dl_stream_t stream);

typedef struct dl_async_update_args {
    double *arena;            /* [n_slots][ld] */
    int64_t ld;
    int64_t n_params;
    int32_t self_slot;        /* the agent's current iterate y */
    int32_t out_slot;         /* receives y' (must differ from every input slot) */
    int32_t n_nbrs;           /* <= DL_ASYNC_MAX_NBRS, in arrival order */
    int32_t nbr_slots[DL_ASYNC_MAX_NBRS];
    int32_t sum_f32;
    double keep;
    double eps;
    double conv_eps;
    int32_t *flags;           /* device int32[2] */
    int32_t parity;
} dl_async_update_args;
int dl_async_update(const dl_async_update_args *args, int32_t *converged_host,
                    dl_stream_t stream);
int dl_async_read(const double *arena, int64_t ld, int32_t slot, int64_t n_params,
                  double *host_out, dl_stream_t stream);

/* ---------------------------------------------------------------- batched per-agent GEMMs
 * BASELINE config c3: every agent trains its own ANNModel (networks/ann_model.py:4-45) on its own
 * batch; the reference runs torch autograd per agent.  Here one launch covers all agents:
 *   C[b] = epi( op(A[b]) . op(B[b]) )      b < batch,  op(A) is M x K,  op(B) is K x N
 * ta: A stored [K][M] (row stride lda) instead of [M][K];  tb: B stored [N][K] instead of [K][N].
 * epi: DL_EPI_BIAS[_RELU|_TANH|_ELU] add bias[b][n] then activate (forward);
 *      DL_EPI_D{RELU,TANH,ELU} multiply by the activation derivative read from the layer's
 *      OUTPUT H[b] (ldh) (backward);  rowsum (nullable) receives sum_k op(A)[b][m][k] (the
 *      bias gradient when op(A) = dZ^T).
 *      DL_EPI_BIAS_XENT (M <= 64 rows = the batch, N <= 64 classes): add bias -> logits z, then
 *      the torch.nn.CrossEntropyLoss head in the same launch: C[b] receives
 *      dZ = (softmax(z) - onehot(labels[b])) / M and loss[b] (nullable) the mean loss; labels
 *      must lie in [0, N).  Deterministic (fixed-order sums).
 * fp32 MFMA (16x16x4), exact fp32 products. */
enum dl_epilogue {
    DL_EPI_NONE = 0, DL_EPI_BIAS = 1, DL_EPI_BIAS_RELU = 2, DL_EPI_BIAS_TANH = 3,
    DL_EPI_BIAS_ELU = 4, DL_EPI_DRELU = 5, DL_EPI_DTANH = 6, DL_EPI_DELU = 7,
    DL_EPI_BIAS_XENT = 8
};
typedef struct dl_bgemm_args {
    int32_t batch, M, N, K;
    const float *A; int64_t lda, sA; int32_t ta;  /* sA: batch stride (elements) */
    const float *B; int64_t ldb, sB; int32_t tb;
    float *C; int64_t ldc, sC;
    int32_t epi;
    const float *bias; int64_t s_bias;
    const float *H; int64_t ldh, sH;
    float *rowsum; int64_t s_rowsum;
    const int32_t *labels; int64_t s_labels;   /* DL_EPI_BIAS_XENT: [batch][M] class ids */
    float *loss;                               /* DL_EPI_BIAS_XENT: nullable [batch] */
} dl_bgemm_args;
int dl_bgemm(const dl_bgemm_args *args, dl_stream_t stream);

/* Cross-entropy head (torch.nn.CrossEntropyLoss, mean): dZ[b] = (softmax(Z[b]) - onehot(y[b]))
 * / rows and loss[b] (nullable) = mean_r (logsumexp(Z[b][r]) - Z[b][r][y]).  Z, dZ: [batch]
 * [rows][classes] with batch strides; classes <= 64. */
int dl_xent_grad(const float *Z, int64_t sZ, const int32_t *y, int64_t sY, float *dZ, int64_t sD,
                 float *loss, int32_t batch, int32_t rows, int32_t classes, dl_stream_t stream);

/* Whole-model per-agent gradients of ANNModel (networks/ann_model.py:4-45) in ONE launch: every
 * agent's forward (Linear-ReLU-Linear-Tanh-Linear-ELU-Linear), torch.nn.CrossEntropyLoss (mean)
 * and backward, one workgroup per agent with its activations resident in LDS.  Replaces the
 * 11-launch dl_bgemm sequence for the shapes it supports (batch == 64, input_dim % 4 == 0,
 * even hidden_dim <= 152, output_dim <= 16); other shapes return DL_ERR_UNSUPPORTED and the caller
 * uses dl_bgemm.
 *   X [n_agents, ldx]: parameter rows in the Mixer flatten order (mixer.py:68-69: fc1.weight,
 *     fc1.bias, fc2.weight, fc2.bias, fc3.weight, fc3.bias, fc4.weight, fc4.bias);
 *   data [n_agents][batch][input_dim] (agent stride s_data), labels [n_agents][batch] int32 in
 *     [0, output_dim);  G [n_agents, ldg]: receives d loss_a / d params_a (same order; columns
 *     beyond the parameter count untouched);  loss nullable [n_agents]: mean cross-entropy.
 *   tile_cols T > 0: X and G are instead in the column-tiled layout of dl_mix_args
 *     ([ceil(P/T)][n_agents][T], T a power of two >= 4; ldx, ldg ignored), the resident layout
 *     the fused round streams fastest.
 *   out_mode 1 (ABI 7): G receives the local SGD step T = X - lr G instead of the gradient, each
 *     element rounded fl(x - fl(lr g)) as dl_mix_round's fused step computes it, so a round of T
 *     (dl_mix_round with G = NULL) gives bit-for-bit the X' of the fused round of X and G while
 *     streaming one matrix instead of two; row-major needs ldg == ldx.  0: the gradient.
 *   workspace (ABI 10) nullable, else dl_mlp_workspace_bytes(n_agents) 16-byte aligned bytes:
 *     the gradients run as two launches instead of one -- everything up to dZ1, then dW1 with
 *     x's column tiles spread over two workgroups per agent; the same bits as the one-launch
 *     path (measured slower at c3's shapes: an experiment's reproducible form).  The workspace
 *     holds each agent's dZ1 between the launches.  out_mode 1 ignores it (one launch).
 * X, data and G 16-byte aligned, ldx, ldg and s_data multiples of 4, G disjoint from X. */
typedef struct dl_mlp_args {
    int32_t n_agents, batch, input_dim, hidden_dim, output_dim;
    const float *X; int64_t ldx;
    const float *data; int64_t s_data;
    const int32_t *labels; int64_t s_labels;
    float *G; int64_t ldg;
    float *loss;
    int32_t tile_cols;   /* 0 = row-major X, G;  T > 0 = column-tiled (see above) */
    int32_t out_mode;    /* 0 = gradient, 1 = local step X - lr G (ABI 7) */
    float lr;            /* out_mode 1: the step size */
    float *workspace;    /* (ABI 10) nullable: the two-launch path (above) */
} dl_mlp_args;
size_t dl_mlp_workspace_bytes(int32_t n_agents);   /* (ABI 10) */
int dl_mlp_grad(const dl_mlp_args *args, dl_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* DLAMD_H */
