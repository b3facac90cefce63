// C ABI of libdlamd.so (include/dlamd.h): argument validation, kernel-configuration planning,
// workspace carving and error reporting.  No exceptions cross this boundary; every entry point
// returns a dl_status and leaves a thread-local message for dl_last_error().
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/dlamd.h"
#include "dl_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_fail(hipError_t e, const char *where) {
    return fail(DL_ERR_HIP, "%s: %s (%d)", where, hipGetErrorString(e), (int)e);
}

// Compute units of the current device (cached per device ordinal).
int device_cus() {
    static std::mutex mu;
    static int cache[64] = {0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    std::lock_guard<std::mutex> lock(mu);
    if (cache[dev] == 0) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            n <= 0)
            n = 256;
        cache[dev] = n;
    }
    return cache[dev];
}

constexpr size_t kAlign = 256;
size_t align_up(size_t v) { return (v + kAlign - 1) & ~(kAlign - 1); }
bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Workgroups of the one-round tile kernel per resident slot on the column-tiled layout: its
// persistent grid is oversubscribed 2x, the second half of the workgroups starting as the first ones retire.
// Measured on MI355X (scripts/grid_sweep.py, profiles/r05/grid_sweep.log): the c2 and c4 rounds
// stream at 5.90-5.93 TB/s with 2x against 5.28-5.41 TB/s with exactly one workgroup per CU, on
// the same box (3x: 5.74-5.80, 4x: 5.75-5.84).  Forcing one resident workgroup per CU through
// LDS changes nothing, so the gain is not co-residency.  Row-major operands (c3's N = 256 rows)
// keep one slot's grid (3247 vs 3206 steps/s).  DLAMD_GRID_MULT=k (1..8) overrides it.
int grid_mult() {
    const char *m = getenv("DLAMD_GRID_MULT");
    const int k = m ? atoi(m) : 2;
    return k < 1 ? 1 : (k > 8 ? 8 : k);
}

// ... for a launch of n_tiles tiles over `slots` resident workgroups: the 2x grid pays on long
// persistent launches (c2 / c4: 128 tile passes per slot); on short ones (c3 column-tiled: 2572
// tiles of 64 columns on 512 slots, 5 passes) the second wave of workgroups only adds its ramp:
// 105.3 vs 110.1 us with one slot's grid (scripts/c3_round_probe.py, profiles/r12/c3_round).
// An explicit DLAMD_GRID_MULT still applies everywhere.
int grid_mult_for(int64_t n_tiles, int64_t slots) {
    if (!getenv("DLAMD_GRID_MULT") && n_tiles < 16 * slots) return 1;
    return grid_mult();
}

// Upper bound of per-workgroup partial rows any path writes.
// MI355X Infinity Cache (MALL), shared by all XCDs
constexpr size_t kMallBytes = (size_t)256 << 20;

int max_parts() {
    int p = 2 * device_cus() * grid_mult();
    return p < 256 ? 256 : p;
}

bool overlaps(const void *a, size_t an, const void *b, size_t bn) {
    const char *x = static_cast<const char *>(a), *y = static_cast<const char *>(b);
    return x < y + bn && y < x + an;
}

struct Plan {
    dl_mix_plan pub;
    int chunks;
    bool dev;
    uint32_t csr_off, scratch_off;
    int head;       // path 5: CSR entries per row in registers (the rest in LDS)
    int tail_fmt;   // path 5: LDS tail entries of 8 B (2) or 6 B (1)
    int grp;        // path 1, column-tiled: data tiles per kernel tile (0 / 1: one)
};

// Workgroups per CU the tile kernel may use (LDS permitting): 2 unless DLAMD_WG_PER_CU=1
// (a measurement knob).
int wg_per_cu_cap() {
    const char *v = getenv("DLAMD_WG_PER_CU");
    return (v && v[0] == '1') ? 1 : 2;
}

// Persistent grid for n_tiles tiles and at most gmax workgroups: the fewest workgroups that
// still finish in the same number of passes, so every workgroup walks ceil(n_tiles/gmax) or one
// fewer tiles.  The time of a persistent HBM-bound launch is its longest workgroup's tile
// count; with gmax workgroups and a ragged last pass (c3: 1286 tiles on 256 CUs = 6 passes for
// an average of 5.02) the idle CUs of that pass are pure tail.  Fewer, evenly loaded workgroups
// keep the same number of passes while each one gets a larger share of HBM.
// DLAMD_BALANCE_GRID=0 (a measurement knob) keeps gmax.
int64_t balanced_grid(int64_t n_tiles, int64_t gmax) {
    if (gmax <= 0) return 1;
    if (n_tiles <= gmax) return n_tiles;
    const char *v = getenv("DLAMD_BALANCE_GRID");
    if (v && v[0] == '0') return gmax;
    const int64_t passes = (n_tiles + gmax - 1) / gmax;
    return (n_tiles + passes - 1) / passes;
}

int next_pow2_chunks(int64_t n_params) {
    int64_t need = (n_params + 3) / 4;
    int c = 1;
    while (c < dl::kMaxChunks && c < need) c <<= 1;
    return c;
}

// LDS bytes of the register-head + LDS-tail tile kernel (path 5) for R rows at c chunks, or 0
// when it does not apply: the nnz - head * R tail entries behind the tile and the mean scratch,
// 8 B per entry ({weight, row} pairs, *fmt = 2) when that fits, else 6 B (weights + u16 rows,
// *fmt = 1; the only form at a 5-entry head, whose registers leave no room for the pairs'
// unrolled loop); the tail's u16 row map (setup only) must fit the tile area.
int64_t reg_tail_lds(const dl_csr &W, int32_t R, int c, bool want_dev, int *head_out,
                     int *fmt_out = nullptr) {
    const int head = dl::reg_head_rows(W.min_row_nnz);
    if (W.uniform_row_nnz == 5 || !dl::reg_tail_supported(c, R, head, 0)) return 0;
    const int64_t ntail = (int64_t)W.nnz - (int64_t)head * R;
    if (ntail < 0 || ntail > 65535) return 0;
    const int64_t tile = (int64_t)R * c * 16;
    const int64_t scratch = want_dev ? (int64_t)(dl::kTileThreads / 64) * c * 16 : 0;
    if (tile > 65536 || 2 * ntail > tile) return 0;
    for (int fmt = head < 5 ? 2 : 1; fmt >= 1; --fmt) {
        const int64_t lds = tile + scratch + (((fmt == 2 ? 8 : 6) * ntail + 15) & ~(int64_t)15);
        if (lds > dl::kLdsBytes) continue;
        if (head_out) *head_out = head;
        if (fmt_out) *fmt_out = fmt;
        return lds;
    }
    return 0;
}

// DLAMD_FORCE_REG=1 (tests only): the register-CSR kernels (paths 4 / 5) wherever they apply,
// so the reference's small fixtures pin them too
bool force_reg_env() {
    const char *f = getenv("DLAMD_FORCE_REG");
    const char *g = getenv("DLAMD_FORCE_GATHER");
    return f && f[0] == '1' && !(g && g[0] == '1');
}

// R = every source row (local + halo); halo rounds have no register-CSR kernels
int choose_tiled_chunks(const dl_csr &W, int32_t R, uint32_t csr, bool want_dev, bool halo) {
    if (R > 65535) return 0;
    const bool reg_any = !halo && (dl::reg_csr_supported(1, R, W.uniform_row_nnz, 0) ||
                                   reg_tail_lds(W, R, 1, want_dev, nullptr) > 0);
    if (force_reg_env() && reg_any) return 1;
    if (csr > 0) {
        for (int c = dl::kMaxChunks; c >= 1; c >>= 1) {
            // (the column-tiled halo kernel runs at most 4 row passes per thread)
            if ((int64_t)R * c > (int64_t)(halo ? 4 : dl::kRowsPerThread) * dl::kTileThreads)
                continue;
            const int64_t tile = (int64_t)R * c * 16;
            if (tile > 65536 && c > 1) continue;
            const int64_t scratch = want_dev ? (int64_t)(dl::kTileThreads / 64) * c * 16 : 0;
            if (tile + csr + scratch <= dl::kLdsBytes) return c;
        }
    }
    if (halo) return 0;
    // the CSR does not fit beside any tile: the register-CSR kernels need LDS for the tile (and
    // path 5 for the CSR entries past each row's register head)
    const int64_t tile = (int64_t)R * 16;
    const int64_t scratch = want_dev ? (int64_t)(dl::kTileThreads / 64) * 16 : 0;
    if (dl::reg_csr_supported(1, R, W.uniform_row_nnz, 0) && tile <= 65536 &&
        tile + scratch <= dl::kLdsBytes)
        return 1;
    if (reg_tail_lds(W, R, 1, want_dev, nullptr) > 0) return 1;
    return 0;
}

// Local source rows of a round: n_local_src, or n_rows when 0 (dlamd.h).
inline int32_t local_src(const dl_mix_args *a) {
    return a->n_local_src > 0 ? a->n_local_src : a->W.n_rows;
}

// An irregular graph of more than 2048 agents takes the register-head + LDS-tail kernel (path 5)
// even when its whole CSR fits LDS beside the tile: above 2048 agents the tile is one 4-column
// chunk either way, and path 1's per-lane CSR loop from LDS (row pointers, weights and rows read
// per entry, a wave as long as its longest row) runs Barabasi-Albert m = 1 at 250 rounds/s
// against 430 for path 5 (4096 x 2^18, `bench.py --workload c4-ba --irregular ba1`).
bool prefer_reg_tail(const dl_csr &W, int32_t R, int c) {
    return c == 1 && R > 2048 && W.uniform_row_nnz == 0 && dl::reg_head_rows(W.min_row_nnz) > 0;
}

// Register-CSR plan for c chunks -- path 4 (regular, 5 entries per row, all in registers) or
// path 5 (rows of >= min_row_nnz entries: register head + LDS tail) -- or false when neither
// applies.
bool plan_reg(const dl_mix_args *a, int c, bool want_dev, Plan *pl) {
    const int32_t R = a->W.n_rows;
    if (a->n_halo > 0 || local_src(a) != R) return false;
    const int64_t tile = (int64_t)R * c * 16;
    const int64_t scratch = want_dev ? (int64_t)(dl::kTileThreads / 64) * c * 16 : 0;
    int head = 0;
    int64_t lds = 0;
    if (dl::reg_csr_supported(c, R, a->W.uniform_row_nnz, 0)) {
        lds = tile + scratch;
        if (lds > dl::kLdsBytes) return false;
    } else {
        lds = reg_tail_lds(a->W, R, c, want_dev, &head, &pl->tail_fmt);
        if (lds == 0) return false;
    }
    const int64_t T = 4 * c;
    const int64_t n_tiles = (a->n_params + T - 1) / T;
    if (n_tiles > 0x7fffffff) return false;
    int bpc = (int)(dl::kLdsBytes / lds);
    if (bpc > wg_per_cu_cap()) bpc = wg_per_cu_cap();
    pl->pub.path = head > 0 ? 5 : 4;
    pl->pub.tile_cols = (int32_t)T;
    pl->pub.grid = (int32_t)balanced_grid(
        n_tiles, (int64_t)device_cus() * bpc *
                     (a->tile_cols > 0 ? grid_mult_for(n_tiles, (int64_t)device_cus() * bpc) : 1));
    pl->pub.lds_bytes = (int32_t)lds;
    pl->pub.n_tiles = (int32_t)n_tiles;
    pl->pub.regular = head > 0 ? 0 : 1;
    pl->pub.head = head > 0 ? head : 5;
    pl->pub.tail_fmt = head > 0 ? pl->tail_fmt : 0;
    pl->chunks = c;
    pl->head = head;
    pl->csr_off = (uint32_t)(tile + scratch);   // path 5: the LDS tail
    pl->scratch_off = (uint32_t)tile;
    return true;
}

// Pick the kernel configuration for a mix round.
int plan_mix(const dl_mix_args *a, Plan *pl) {
    std::memset(pl, 0, sizeof *pl);
    const int32_t R = local_src(a) + a->n_halo;
    const int32_t nnz = a->W.nnz;
    // the halo round's column sums use the same LDS scratch as the fused deviation
    const bool want_dev = a->dev_sq || a->dev_max || a->mean || a->colsum_out;
    pl->dev = want_dev;
    const int reg = a->W.uniform_row_nnz > 0 ? 1 : 0;
    const int32_t n_w = (reg && a->W.shared_row_weights) ? a->W.uniform_row_nnz : nnz;
    const uint32_t csr = dl::csr_lds_bytes(a->W.n_rows, nnz, reg, n_w);
    int cmax = next_pow2_chunks(a->n_params);
    // DLAMD_MAX_TILE_CHUNKS=c (a measurement knob) caps the row-major tile at 4c columns
    if (const char *mc = getenv("DLAMD_MAX_TILE_CHUNKS")) {
        const int m = atoi(mc);
        while (m >= 1 && cmax > m) cmax >>= 1;
    }
    // DLAMD_FORCE_GATHER=1 (tests only) forces the general gather kernel; DLAMD_FORCE_REG=1
    // (tests only) the register-CSR kernels (paths 4 / 5) wherever they apply, so the reference's
    // small fixtures pin them too
    const char *force = getenv("DLAMD_FORCE_GATHER");
    const bool force_gather = force && force[0] == '1';
    const bool force_reg = force_reg_env();
    if (a->tile_cols > 0) {  // column-tiled layout: the tile width is fixed by the data
        const int c = a->tile_cols / 4;
        const int64_t tile = (int64_t)R * c * 16;
        const int64_t scratch = want_dev ? (int64_t)(dl::kTileThreads / 64) * c * 16 : 0;
        const int64_t lds = tile + csr + scratch;
        if ((csr == 0 || lds > dl::kLdsBytes || force_reg || prefer_reg_tail(a->W, R, c)) &&
            R <= 65535 && plan_reg(a, c, want_dev, pl))
            return DL_OK;
        if (csr == 0 || R > 65535 || (int64_t)R * c > (int64_t)dl::kRowsPerThread * dl::kTileThreads ||
            (a->n_halo > 0 && (int64_t)R * c > 4 * (int64_t)dl::kTileThreads) ||
            lds > dl::kLdsBytes)
            return fail(DL_ERR_INVALID, "dl_mix_round: tile_cols %d does not fit this graph "
                                        "(%d rows); query dl_mix_plan_query on row-major args",
                        a->tile_cols, R);
        int64_t n_tiles = (a->n_params + a->tile_cols - 1) / a->tile_cols;
        // tile groups: a halo round of few source rows (the split scheme's boundary launch,
        // 276 rows at 16 columns: 18 KB a tile, latency-bound) walks g <= 8 consecutive data tiles
        // as one kernel tile of 4cg columns, at <= 4 row passes per thread (the halo kernel's
        // limit); DLAMD_TILE_GROUP=g caps g (1: off, a measurement knob)
        int g = 1, cg = c;
        int64_t lds_g = lds;
        if (a->n_halo > 0) {
            int gcap = 8;
            if (const char *v = getenv("DLAMD_TILE_GROUP")) gcap = atoi(v);
            for (int gg = 8; gg >= 2; gg >>= 1) {
                if (gg > gcap) continue;
                const int cc = c * gg;
                const int64_t l = (int64_t)R * cc * 16 + csr +
                                  (want_dev ? (int64_t)(dl::kTileThreads / 64) * cc * 16 : 0);
                if (cc > dl::kMaxChunks || n_tiles % gg ||
                    (int64_t)R * cc > 4 * (int64_t)dl::kTileThreads || l > dl::kLdsBytes)
                    continue;
                g = gg;
                cg = cc;
                lds_g = l;
                break;
            }
        }
        n_tiles /= g;
        // two 1024-thread workgroups per CU when LDS allows, except at C = 4, where the second
        // workgroup's LDS traffic (4 rows of 64 B per 16 lanes: the most bank conflicts of any
        // C) costs more than its extra loads in flight (measured 5.5 vs 5.8 TB/s at N = 1024;
        // the c4 rank of 8's 608-row halo round: 69.1 vs 70.1 % of spec, profiles/r11/session_c)
        int bpc = (int)(dl::kLdsBytes / lds_g);
        if (bpc > wg_per_cu_cap()) bpc = wg_per_cu_cap();
        if (cg == 4) bpc = 1;
        // two 1024-thread workgroups share a CU only at <= 64 VGPRs.  Of the column-tiled halo
        // instantiations only those mix_tile.hip's tile_waves_per_eu caps are that small (C >= 8
        // at <= 3 row passes without the lagged deviation: 53-64 VGPRs, no spills); every other
        // one takes 66-123 (profiles/r13/vgprs.txt), so a grid sized for two would only queue
        // them (rank-of 4 / 2 halo mix 1.5 / 2 % slower, profiles/r12/halo_grid/)
        if (a->n_halo > 0) {
            const int64_t slots = dl::kTileThreads / cg;
            const bool capped = cg >= 8 && (R + slots - 1) / slots <= 3 && !a->mean_prev &&
                                !a->colsum_out;
            if (!capped) bpc = 1;
        }
        const int64_t grid =
            balanced_grid(n_tiles, (int64_t)device_cus() * (bpc < 1 ? 1 : bpc) *
                                   grid_mult_for(n_tiles, (int64_t)device_cus() *
                                                              (bpc < 1 ? 1 : bpc)));
        pl->pub.path = 1;
        pl->pub.tile_cols = a->tile_cols;
        pl->pub.grid = (int32_t)grid;
        pl->pub.lds_bytes = (int32_t)lds_g;
        pl->pub.n_tiles = (int32_t)n_tiles;
        pl->pub.regular = reg;
        pl->chunks = cg;
        pl->grp = g;
        pl->csr_off = (uint32_t)((int64_t)R * cg * 16);
        pl->scratch_off = (uint32_t)((int64_t)R * cg * 16 + csr);
        return DL_OK;
    }
    if ((force_reg || (prefer_reg_tail(a->W, R, 1) && !force_gather)) && R <= 65535 &&
        a->n_params % 4 == 0 && plan_reg(a, 1, want_dev, pl))
        return DL_OK;
    // with the fused deviation, prefer the widest tile at <= 4 row passes per thread: the
    // kernel then keeps each lane's deviation partials in registers and reduces them once per
    // launch (mix_tile.hip LD); c3's 256 agents: 64-column tiles, 116 -> 105 us a round
    // (scripts/c3_round_probe.py, profiles/r12/c3_round)
    int cdev = 0;
    if (want_dev)
        for (int c = cmax; c >= 2; c >>= 1)
            if ((int64_t)R * c <= 4 * (int64_t)dl::kTileThreads) {
                cdev = c;
                break;
            }
    // ... and one workgroup per CU there: c3 3704-3729 against 3589-3610 steps/s with two
    // (same box, profiles/r12/c3_round/c3_rows_wg*.log)
    bool one_per_cu = false;
    if (cdev > 0 && cdev < cmax && a->n_params % (4 * cdev) == 0) {
        cmax = cdev;
        one_per_cu = true;
    }
    if (csr > 0 && R <= 65535 && !force_gather) {
        for (int c = cmax; c >= 1; c >>= 1) {
            if ((int64_t)R * c > (int64_t)dl::kRowsPerThread * dl::kTileThreads) continue;
            const int64_t tile = (int64_t)R * c * 16;
            const int64_t scratch = want_dev ? (int64_t)(dl::kTileThreads / 64) * c * 16 : 0;
            const int64_t lds = tile + csr + scratch;
            if (lds > dl::kLdsBytes) continue;
            const int64_t T = 4 * c;
            const int64_t n_tiles = (a->n_params + T - 1) / T;
            if (n_tiles > 0x7fffffff) continue;
            int bpc = (int)(dl::kLdsBytes / lds);
            if (bpc > wg_per_cu_cap()) bpc = wg_per_cu_cap();  // 1024 threads: <= 2 per CU
            if (one_per_cu && c == cmax) bpc = 1;
            const int64_t grid =
                balanced_grid(n_tiles, (int64_t)device_cus() * bpc);
            pl->pub.path = 1;
            pl->pub.tile_cols = (int32_t)T;
            pl->pub.grid = (int32_t)grid;
            pl->pub.lds_bytes = (int32_t)lds;
            pl->pub.n_tiles = (int32_t)n_tiles;
            pl->pub.regular = reg;
            pl->chunks = c;
            pl->csr_off = (uint32_t)tile;
            pl->scratch_off = (uint32_t)(tile + csr);
            return DL_OK;
        }
    }
    if (R <= 65535 && !force_gather) {
        if (a->n_params % 4 == 0 && plan_reg(a, 1, want_dev, pl)) return DL_OK;
    }
    if (a->W.n_rows > 4 * 65535)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_round: %d rows exceed the gather path limit",
                    a->W.n_rows);
    if (a->mean_prev || a->colsum_out)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_round: the lagged halo deviation needs the LDS "
                                        "tile kernel; this graph takes the gather path");
    if (local_src(a) != a->W.n_rows)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_round: n_local_src != n_rows needs the LDS tile "
                                        "kernel; this graph takes the gather path");
    pl->pub.path = 2;
    pl->pub.grid = (int32_t)(((a->n_params + 255) / 256) * ((a->W.n_rows + 3) / 4));
    pl->pub.regular = reg;
    return DL_OK;
}

int check_mix_args(const dl_mix_args *a) {
    if (!a) return fail(DL_ERR_INVALID, "dl_mix_round: args is NULL");
    const dl_csr &W = a->W;
    if (W.n_rows <= 0) return fail(DL_ERR_INVALID, "dl_mix_round: n_rows must be > 0 (got %d)", W.n_rows);
    if (a->n_params <= 0) return fail(DL_ERR_INVALID, "dl_mix_round: n_params must be > 0");
    if (a->n_halo < 0) return fail(DL_ERR_INVALID, "dl_mix_round: n_halo < 0");
    if (a->n_local_src < 0) return fail(DL_ERR_INVALID, "dl_mix_round: n_local_src < 0");
    const int32_t NL = local_src(a);
    // an interior / boundary row set of an agent partition (outputs need not be source rows)
    const bool part = NL != W.n_rows;
    if ((int64_t)W.n_rows > (int64_t)NL + a->n_halo)
        return fail(DL_ERR_INVALID, "dl_mix_round: n_rows %d > n_local_src + n_halo %lld",
                    W.n_rows, (long long)NL + a->n_halo);
    if (W.nnz < 0) return fail(DL_ERR_INVALID, "dl_mix_round: nnz < 0");
    if (a->n_hub_rows < 0) return fail(DL_ERR_INVALID, "dl_mix_round: n_hub_rows < 0");
    if (!a->x || !a->y || !W.row_ptr || (W.nnz > 0 && (!W.col || !W.w)))
        return fail(DL_ERR_INVALID, "dl_mix_round: null x/y/row_ptr/col/w");
    if (a->tile_cols < 0 || (a->tile_cols > 0 && (a->tile_cols % 4 || a->tile_cols < 4 ||
                                                   a->tile_cols > 4 * dl::kMaxChunks ||
                                                   (a->tile_cols & (a->tile_cols - 1)))))
        return fail(DL_ERR_INVALID, "dl_mix_round: tile_cols must be 0 or a power of two in [4, %d]",
                    4 * dl::kMaxChunks);
    const bool tiled = a->tile_cols > 0;
    if (!tiled && (a->ldx < a->n_params || a->ldy < a->n_params))
        return fail(DL_ERR_INVALID, "dl_mix_round: ldx/ldy smaller than n_params");
    if (!tiled && a->g && a->ldg < a->n_params)
        return fail(DL_ERR_INVALID, "dl_mix_round: ldg < n_params");
    // column-tiled: ld* = rows of each operand's tiled blocks (0 = the operand's own rows)
    if (tiled && (a->ldx < 0 || a->ldy < 0 || a->ldg < 0 || (a->ldx > 0 && a->ldx < NL) ||
                  (a->ldy > 0 && a->ldy < W.n_rows) || (a->g && a->ldg > 0 && a->ldg < NL) ||
                  a->ldx > 65535 * 4 || a->ldy > 65535 * 4 || a->ldg > 65535 * 4))
        return fail(DL_ERR_INVALID, "dl_mix_round: tiled ldx/ldg (>= n_local_src) or ldy (>= "
                                    "n_rows) out of range");
    if (a->n_halo > 0 && !a->halo)
        return fail(DL_ERR_INVALID, "dl_mix_round: n_halo > 0 needs a halo buffer");
    if (!tiled && a->n_halo > 0 && a->ldh < a->n_params)
        return fail(DL_ERR_INVALID, "dl_mix_round: n_halo > 0 needs halo with ldh >= n_params");
    if (!tiled && a->n_halo_blocks != 0)
        return fail(DL_ERR_INVALID, "dl_mix_round: n_halo_blocks is for the column-tiled layout");
    if (tiled && a->n_halo > 0) {
        if (a->n_halo_blocks < 0 || a->n_halo_blocks > dl::kMaxHaloBlocks ||
            (a->n_halo_blocks > 0 && !a->halo_block_rows))
            return fail(DL_ERR_INVALID, "dl_mix_round: n_halo_blocks must be 0..%d with "
                                        "halo_block_rows", dl::kMaxHaloBlocks);
        int64_t sum = 0;
        for (int b = 0; b < a->n_halo_blocks; ++b) {
            if (a->halo_block_rows[b] <= 0)
                return fail(DL_ERR_INVALID, "dl_mix_round: halo_block_rows[%d] <= 0", b);
            sum += a->halo_block_rows[b];
        }
        if (a->n_halo_blocks > 0 && sum != a->n_halo)
            return fail(DL_ERR_INVALID, "dl_mix_round: halo_block_rows sum to %lld, n_halo %d",
                        (long long)sum, a->n_halo);
        const int64_t ntl = (a->n_params + a->tile_cols - 1) / a->tile_cols;
        if (ntl * a->n_halo * a->tile_cols * 4 >= ((int64_t)1 << 32))
            return fail(DL_ERR_INVALID, "dl_mix_round: the tiled halo must span < 4 GiB");
    }
    // a column-tiled partition round reads mean_prev / colsum_out a float4 per chunk, tiles whole
    if (tiled && (a->n_halo > 0 || part) && a->n_params % a->tile_cols)
        return fail(DL_ERR_INVALID, "dl_mix_round: a column-tiled partition round needs "
                                    "n_params %% tile_cols == 0");
    if (W.uniform_row_nnz < 0 ||
        (W.uniform_row_nnz > 0 && (int64_t)W.uniform_row_nnz * W.n_rows != W.nnz))
        return fail(DL_ERR_INVALID, "dl_mix_round: uniform_row_nnz * n_rows != nnz");
    if (W.shared_row_weights && W.uniform_row_nnz <= 0)
        return fail(DL_ERR_INVALID, "dl_mix_round: shared_row_weights needs uniform_row_nnz > 0");
    if (W.min_row_nnz < 0 || (int64_t)W.min_row_nnz * W.n_rows > W.nnz)
        return fail(DL_ERR_INVALID, "dl_mix_round: min_row_nnz * n_rows > nnz");
    const bool halo_round = a->n_halo > 0 || part;
    if ((a->mean_prev || a->colsum_out) && !halo_round)
        return fail(DL_ERR_INVALID, "dl_mix_round: mean_prev / colsum_out are for halo rounds "
                                    "(n_halo > 0 or n_local_src != n_rows); local rounds fuse "
                                    "the exact deviation");
    if (a->mean && halo_round)
        return fail(DL_ERR_INVALID, "dl_mix_round: the column mean of a halo round is global: "
                                    "use colsum_out and an all-reduce");
    if ((a->dev_sq || a->dev_max || a->mean_prev || a->colsum_out) && halo_round &&
        !(a->mean_prev && a->colsum_out))
        return fail(DL_ERR_INVALID,
                    "dl_mix_round: a halo round's deviation is the lagged one: mean_prev, "
                    "colsum_out and dev_sq together, or both without dev_sq (partial rows left "
                    "in the workspace), or dl_column_sum + dl_deviation after it");
    if (halo_round && a->mean_prev && !a->dev_sq && a->tile_cols <= 0)
        return fail(DL_ERR_INVALID, "dl_mix_round: partial rows without dev_sq need the "
                                    "column-tiled layout (one launch, plan grid rows)");
    if (halo_round && a->mean_prev && !a->dev_sq && !a->partial_rows_out)
        return fail(DL_ERR_INVALID, "dl_mix_round: a lagged halo round without dev_sq leaves its "
                                    "deviation as partial rows: pass partial_rows_out (ABI 9) to "
                                    "receive their count, or dev_sq for the reduced deviation");
    // extents: a tiled operand of `rows` used rows inside blocks of `ld` rows spans (tiles - 1)
    // block strides plus its used rows of the last tile
    const int64_t Tc = a->tile_cols;
    const int64_t ntl = tiled ? (a->n_params + Tc - 1) / Tc : 0;
    auto tiled_b = [&](int64_t ld, int64_t rows) {
        return (size_t)(((ntl - 1) * ld + rows) * Tc * 4);
    };
    const size_t xb = tiled ? tiled_b(a->ldx ? a->ldx : NL, NL)
                            : ((size_t)(NL - 1) * a->ldx + a->n_params) * 4;
    const size_t yb = tiled ? tiled_b(a->ldy ? a->ldy : W.n_rows, W.n_rows)
                            : ((size_t)(W.n_rows - 1) * a->ldy + a->n_params) * 4;
    if (overlaps(a->x, xb, a->y, yb)) return fail(DL_ERR_INVALID, "dl_mix_round: y overlaps x");
    if (a->g) {
        const size_t gb = tiled ? tiled_b(a->ldg ? a->ldg : NL, NL)
                                : ((size_t)(NL - 1) * a->ldg + a->n_params) * 4;
        if (overlaps(a->g, gb, a->y, yb)) return fail(DL_ERR_INVALID, "dl_mix_round: y overlaps g");
    }
    if (a->n_halo > 0) {
        const size_t hb = tiled ? (size_t)(ntl * a->n_halo * Tc * 4)
                                : ((size_t)(a->n_halo - 1) * a->ldh + a->n_params) * 4;
        if (overlaps(a->halo, hb, a->y, yb))
            return fail(DL_ERR_INVALID, "dl_mix_round: y overlaps halo");
    }
    return DL_OK;
}

dl::TileArgs tile_args(const dl_mix_args *a) {
    dl::TileArgs t{};
    t.x = a->x;
    t.ldx = a->ldx;
    t.halo = a->halo;
    t.ldh = a->ldh;
    t.g = a->g;
    t.ldg = a->ldg;
    t.y = a->y;
    t.ldy = a->ldy;
    t.rowptr = a->W.row_ptr;
    t.col = a->W.col;
    t.w = a->W.w;
    t.n_rows = a->W.n_rows;
    t.n_loc = local_src(a);
    t.n_src = t.n_loc + a->n_halo;
    t.nnz = a->W.nnz;
    t.regular = a->W.uniform_row_nnz;
    t.n_w = (a->W.uniform_row_nnz > 0 && a->W.shared_row_weights) ? a->W.uniform_row_nnz
                                                                   : a->W.nnz;
    t.mean_from_inputs = (a->W.doubly_stochastic && t.n_src == t.n_rows) ? 1 : 0;
    {
        // X, G and X' are streamed exactly once per round: non-temporal loads and stores keep
        // them out of L2/MALL (measured +1.5 % on c2).  An X' that fits the 256-MB MALL is
        // stored plainly instead, so the next kernel's reads of it (the c3 gradient launch
        // reading X' as its parameters) can hit there: c3 +2 % steps/s (3743 vs 3668) -- but
        // not in a partitioned round, whose next launch is the next column chunk's pack and mix
        // (other columns): plain stores there left the following launch 16 % slower (one rank
        // of 8, two chunks of 256 MB: 421.7 against 383.5-387.5 us a round with them
        // non-temporal, profiles/r13/c4rank_env/).  DLAMD_NT_STORE=0/1 and DLAMD_NT_LOAD=0
        // force them.
        const char *nt = getenv("DLAMD_NT_STORE");
        const size_t y_bytes = (size_t)a->W.n_rows * (size_t)a->n_params * 4;
        const bool partitioned = a->n_halo > 0 || (a->n_local_src && a->n_local_src != a->W.n_rows);
        t.nt_store = nt ? (nt[0] == '0' ? 0 : 1) : (y_bytes > kMallBytes || partitioned ? 1 : 0);
        const char *ntl = getenv("DLAMD_NT_LOAD");
        t.nt_load = !ntl ? 3 : ntl[0] == '0' ? 0 : ntl[0] == 'x' ? 1 : ntl[0] == 'g' ? 2 : 3;
    }
    t.n_params = a->n_params;
    t.lr = a->lr;
    bool vec = aligned16(a->x) && aligned16(a->y) && a->ldx % 4 == 0 && a->ldy % 4 == 0;
    if (a->g) vec = vec && aligned16(a->g) && a->ldg % 4 == 0;
    if (a->halo) vec = vec && aligned16(a->halo) && a->ldh % 4 == 0;
    if (a->mean) vec = vec && aligned16(a->mean);
    if (a->mean_prev) vec = vec && aligned16(a->mean_prev);
    if (a->colsum_out) vec = vec && aligned16(a->colsum_out);
    t.mean_prev = a->mean_prev;
    t.colsum_out = a->colsum_out;
    // the float4 kernel addresses rows with 32-bit byte offsets from the tile base
    const int64_t lim = (int64_t)1 << 32;
    const int64_t R = t.n_loc > t.n_rows ? t.n_loc : t.n_rows;
    if (a->tile_cols > 0) {
        vec = aligned16(a->x) && aligned16(a->y) && (!a->g || aligned16(a->g)) &&
              (!a->mean || aligned16(a->mean)) && (!a->halo || aligned16(a->halo)) &&
              (!a->mean_prev || aligned16(a->mean_prev)) &&
              (!a->colsum_out || aligned16(a->colsum_out));
        t.tiled = 1;
        // per-peer halo blocks (check_mix_args: <= kMaxHaloBlocks, rows summing to n_halo,
        // the whole halo < 4 GiB)
        const int64_t Tc = a->tile_cols;
        const int64_t ntl = (a->n_params + Tc - 1) / Tc;
        const int nb = a->n_halo > 0 ? (a->n_halo_blocks > 0 ? a->n_halo_blocks : 1) : 0;
        t.n_hblk = nb;
        int32_t r0 = 0;
        for (int b = 0; b < nb; ++b) {
            t.hblk_row0[b] = r0;
            t.hblk_off[b] = (uint32_t)(ntl * r0 * Tc * 4);
            r0 += a->n_halo_blocks > 0 ? a->halo_block_rows[b] : a->n_halo;
        }
        t.hblk_row0[nb] = r0;
    } else if (((R - 1) * a->ldx + 128) * 4 >= lim || ((R - 1) * a->ldy + 128) * 4 >= lim ||
               (a->g && ((R - 1) * a->ldg + 128) * 4 >= lim) ||
               // a halo row's offset (row and column) is one 32-bit value
               (a->n_halo > 0 && (int64_t)a->n_halo * a->ldh * 4 >= lim)) {
        vec = false;
    }
    t.vec = vec ? 1 : 0;
    t.mean = a->mean;
    return t;
}

// Deviation of x (n_rows x n_params) via the two-pass path: mean (given or column mean), then
// per-row partial sums, then the fixed-order reduce.
int deviation_two_pass(const float *x, int64_t ldx, int32_t n_rows, int64_t n_params,
                       const float *mean_in, float *dev_sq, float *dev_max, float *mean_out,
                       char *ws, size_t ws_bytes, hipStream_t s) {
    const int parts = dl::dev_rows_parts(n_params);
    const size_t part_b = align_up((size_t)parts * n_rows * 4);
    const size_t mean_b = align_up((size_t)n_params * 4);
    if (ws_bytes < part_b + mean_b) return fail(DL_ERR_WORKSPACE, "deviation: workspace too small");
    float *partial = reinterpret_cast<float *>(ws);
    const float *mean = mean_in;
    if (!mean) {
        float *m = mean_out ? mean_out : reinterpret_cast<float *>(ws + part_b);
        hipError_t e = dl::launch_column_sum(x, ldx, n_rows, n_params, m, (float)n_rows, s);
        if (e != hipSuccess) return hip_fail(e, "column_sum");
        mean = m;
    } else if (mean_out && mean_out != mean_in) {
        hipError_t e = hipMemcpyAsync(mean_out, mean_in, (size_t)n_params * 4,
                                      hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return hip_fail(e, "mean copy");
    }
    hipError_t e = dl::launch_dev_rows(x, ldx, n_rows, n_params, mean, partial, parts, s);
    if (e != hipSuccess) return hip_fail(e, "dev_rows");
    e = dl::launch_dev_reduce(partial, parts, n_rows, dev_sq, dev_max, s);
    if (e != hipSuccess) return hip_fail(e, "dev_reduce");
    return DL_OK;
}

int zero_deviation(int32_t n_rows, float *dev_sq, float *dev_max, hipStream_t s) {
    if (dev_sq) {
        hipError_t e = hipMemsetAsync(dev_sq, 0, (size_t)n_rows * 4, s);
        if (e != hipSuccess) return hip_fail(e, "memset dev_sq");
    }
    if (dev_max) {
        hipError_t e = hipMemsetAsync(dev_max, 0, 4, s);
        if (e != hipSuccess) return hip_fail(e, "memset dev_max");
    }
    return DL_OK;
}

// Configuration of the multi-round kernel: two tile images of all agents in LDS beside the CSR.
// Returns DL_ERR_UNSUPPORTED (no message needed by callers that fall back) when it cannot run.
int plan_rounds(const dl_mix_args *a, Plan *pl) {
    std::memset(pl, 0, sizeof *pl);
    const int32_t R = a->W.n_rows;
    const bool want_dev = a->dev_sq || a->dev_max || a->mean;
    pl->dev = want_dev;
    if (a->n_halo > 0 || local_src(a) != a->W.n_rows)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds: halo rows need one exchange per round");
    if (want_dev && !a->W.doubly_stochastic)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds: the fused final deviation needs a doubly "
                                        "stochastic W");
    const int reg = a->W.uniform_row_nnz > 0 ? 1 : 0;
    const int32_t n_w = (reg && a->W.shared_row_weights) ? a->W.uniform_row_nnz : a->W.nnz;
    if (dl::csr_lds_bytes(R, a->W.nnz, reg, n_w) == 0 || R > 65535)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds: CSR too large");
    auto fits = [&](int c) {
        // degree-4 regular graphs with shared weights keep the CSR in registers (mix_multi.hip
        // launch_kv: uniform_row_nnz 5, 5 weights, <= 4 rows per thread): no LDS for it
        const bool in_regs = a->W.uniform_row_nnz == 5 && n_w == 5 &&
                             dl::tile_passes(c, R, true) <= 4;
        const uint32_t csr = in_regs ? 0u : dl::csr_lds_bytes(R, a->W.nnz, reg, n_w);
        const int64_t tile = (int64_t)R * c * 16;
        const int64_t scratch = want_dev ? (int64_t)(dl::kTileThreads / 64) * c * 16 : 0;
        return (int64_t)R * c <= (int64_t)dl::kRowsPerThread * dl::kTileThreads &&
               2 * tile + csr + scratch <= dl::kLdsBytes;
    };
    int c = 0;
    if (a->tile_cols > 0) {
        c = a->tile_cols / 4;
        if (!fits(c))
            return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds: two %d-column tiles of %d rows do "
                                            "not fit LDS", a->tile_cols, R);
    } else {
        for (int cc = next_pow2_chunks(a->n_params); cc >= 1; cc >>= 1)
            if (fits(cc) && a->n_params % (4 * cc) == 0) {
                c = cc;
                break;
            }
        if (c == 0)
            return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds: no full-tile row-major configuration");
    }
    const int64_t T = 4 * c;
    const int64_t n_tiles = (a->n_params + T - 1) / T;
    const int64_t tile = (int64_t)R * c * 16;
    const bool in_regs = a->W.uniform_row_nnz == 5 && n_w == 5 && dl::tile_passes(c, R, true) <= 4;
    const uint32_t csr = in_regs ? 0u : dl::csr_lds_bytes(R, a->W.nnz, reg, n_w);
    pl->chunks = c;
    pl->csr_off = (uint32_t)(2 * tile);
    pl->scratch_off = (uint32_t)(2 * tile + csr);
    pl->pub.path = 3;
    pl->pub.tile_cols = (int32_t)T;
    pl->pub.grid = (int32_t)balanced_grid(n_tiles, device_cus());
    pl->pub.lds_bytes = (int32_t)(2 * tile + csr +
                                  (want_dev ? (dl::kTileThreads / 64) * c * 16 : 0));
    pl->pub.n_tiles = (int32_t)n_tiles;
    pl->pub.regular = reg;
    return DL_OK;
}

// dl_mix_rounds_trace configuration: one agent per thread, C float4 column chunks per step.
struct TracePlan {
    int32_t max_rounds;  // rounds per traced pass (the per-round deviations live in VGPRs)
    int32_t grid, chunks;
    int64_t n_steps;
    uint32_t csr_off, scratch_off, lds;
    int32_t irr;   // 1: mix_trace_irr_kernel (one image, register head + LDS tail)
    int32_t head;  // irr: CSR entries per row in registers
    int32_t gm;    // irr: W not doubly stochastic, every round's mean from its outputs
    int32_t narrow;  // irr: 2-column steps, 6-byte tail entries
};

// mix_trace_irr_kernel's configuration: one [N] float4 image, each row's first `head` entries in
// registers and the rest as 8-byte {weight, row} pairs behind it, a 16 x float4 mean scratch.
// The tail's u16 row map (setup only) lives in the image area.
int plan_trace_irr(const dl_mix_args *a, TracePlan *tp) {
    const dl_csr &W = a->W;
    const int32_t N = W.n_rows;
    if (N < 2 || N > 4 * dl::kTileThreads || W.nnz > 65535 + 5 * (int64_t)N)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds_trace: no traced kernel for %d agents "
                                        "with %d CSR entries", N, W.nnz);
    int head = dl::reg_head_rows(W.min_row_nnz);
    int64_t ntail = (int64_t)W.nnz - (int64_t)head * N;
    if (ntail > 65535 || ntail < 0) {
        head = 0;
        ntail = W.nnz;
    }
    if (ntail > 65535)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds_trace: %lld CSR entries past the register "
                                        "heads (> 65535)", (long long)ntail);
    // 4-column steps with 8-byte {weight, row} tail pairs (the tail's row map in the image), or
    // 2-column steps with 6-byte tail entries when that does not fit
    bool narrow = false;
    uint32_t img = (uint32_t)N * 16u;
    uint32_t tail = (uint32_t)align_up((size_t)ntail * 8);
    if (2 * ntail > (int64_t)img || img + tail + 256u > (uint32_t)dl::kLdsBytes) {
        narrow = true;
        img = (uint32_t)align_up((size_t)N * 8u);
        tail = (uint32_t)align_up((size_t)ntail * 6);
        if (img + tail + 256u > (uint32_t)dl::kLdsBytes)
            return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds_trace: the CSR of %d agents (%d "
                                            "entries) does not fit LDS beside one image", N, W.nnz);
    }
    tp->irr = 1;
    tp->head = head;
    tp->gm = W.doubly_stochastic ? 0 : 1;
    tp->narrow = narrow ? 1 : 0;
    tp->chunks = 1;
    tp->csr_off = img;
    tp->scratch_off = img + tail;
    tp->lds = img + tail + 256u;
    tp->max_rounds = dl::irr_trace_rounds(dl::irr_trace_kv(N));
    tp->n_steps = a->n_params / (narrow ? 2 : 4);
    tp->grid = (int32_t)balanced_grid(tp->n_steps, device_cus());
    return DL_OK;
}

int plan_trace(const dl_mix_args *a, TracePlan *tp) {
    const int32_t N = a->W.n_rows;
    std::memset(tp, 0, sizeof *tp);
    if (a->n_halo > 0 || local_src(a) != a->W.n_rows)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds_trace: halo rows need one exchange per "
                                        "round");
    if (a->g)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds_trace: no local step (g must be NULL)");
    if (a->n_params % 4)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds_trace: n_params must be a multiple of 4");
    // a W that is not doubly stochastic (every round's mean from its outputs), or an irregular
    // graph above 2048 agents: the one-image kernel with the register head + LDS tail CSR
    if (!a->W.doubly_stochastic)
        return plan_trace_irr(a, tp);
    if (N > 2 * dl::kTileThreads && !(a->W.uniform_row_nnz == 5 && a->W.shared_row_weights))
        return plan_trace_irr(a, tp);
    // one agent per thread up to 1024 agents; above, mix_trace_wide_kernel (one column chunk per
    // step, up to 4 agents per thread; the CSR in registers above 2048 agents)
    if (N < 2 || N > 4 * dl::kTileThreads)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds_trace: needs 2..%d agents, got %d",
                    4 * dl::kTileThreads, N);
    if (a->n_params % 4)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds_trace: n_params must be a multiple of 4");
    const int reg = a->W.uniform_row_nnz > 0 ? 1 : 0;
    const int32_t n_w = (reg && a->W.shared_row_weights) ? a->W.uniform_row_nnz : a->W.nnz;
    const bool in_regs = a->W.uniform_row_nnz == 5 && n_w == 5;
    const uint32_t csr = in_regs ? 0u : dl::csr_lds_bytes(N, a->W.nnz, reg, n_w);
    if (!in_regs && csr == 0) return plan_trace_irr(a, tp);
    const bool wide = N > dl::kTileThreads;
    if (wide && !in_regs && N > 2 * dl::kTileThreads)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds_trace: above %d agents the traced pass "
                                        "keeps the CSR in registers (regular degree-4 graphs with "
                                        "shared weights)", 2 * dl::kTileThreads);
    const int64_t nq = a->n_params / 4;
    const int64_t lc = a->tile_cols > 0 ? a->tile_cols / 4 : 0;   // 0: row-major
    // widest chunk count whose two images fit LDS (a round then does C outputs per thread)
    tp->chunks = 0;
    for (int c = wide ? 1 : 4; c >= 1; c >>= 1) {
        const uint32_t img = 2u * (uint32_t)N * 16u * (uint32_t)c;
        const uint32_t scr = (uint32_t)align_up(img + csr);
        const uint32_t lds = scr + (dl::kTileThreads / 64) * 16u * (uint32_t)c;
        // a step's chunks must be whole (nq % c) and lie in one operand tile (lc % c)
        if (lds <= (uint32_t)dl::kLdsBytes && nq % c == 0 && (lc == 0 || lc % c == 0)) {
            tp->chunks = c;
            tp->csr_off = img;
            tp->scratch_off = scr;
            tp->lds = lds;
            break;
        }
    }
    if (tp->chunks == 0) return plan_trace_irr(a, tp);   // two images do not fit: one image
    tp->max_rounds = dl::trace_max_rounds(N, in_regs, tp->chunks);
    tp->n_steps = nq / tp->chunks;
    tp->grid = (int32_t)balanced_grid(tp->n_steps, device_cus());
    return DL_OK;
}

}  // namespace

namespace dl {
int fail_msg(int code, const char *msg) { return fail(code, "%s", msg); }
}  // namespace dl

extern "C" {

int dl_abi_version(void) { return DLAMD_ABI_VERSION; }

int dl_mix_trace_plan(const dl_mix_args *args, int32_t *max_rounds) {
    g_err.clear();
    if (!max_rounds) return fail(DL_ERR_INVALID, "dl_mix_trace_plan: max_rounds is NULL");
    int rc = check_mix_args(args);
    if (rc) return rc;
    TracePlan tp;
    rc = plan_trace(args, &tp);
    if (rc) return rc;
    *max_rounds = tp.max_rounds;
    return DL_OK;
}

size_t dl_mix_trace_workspace_bytes(int32_t n_rows, int32_t rounds) {
    if (n_rows <= 0 || rounds <= 0) return 0;
    return align_up((size_t)device_cus() * (size_t)rounds * (size_t)n_rows * 4) + kAlign;
}

int dl_mix_rounds_trace(const dl_mix_args *args, int32_t rounds, float *trace, void *workspace,
                        size_t ws_bytes, dl_stream_t stream) {
    g_err.clear();
    int rc = check_mix_args(args);
    if (rc) return rc;
    if (!trace) return fail(DL_ERR_INVALID, "dl_mix_rounds_trace: trace is NULL");
    TracePlan tp;
    rc = plan_trace(args, &tp);
    if (rc) return rc;
    if (rounds < 1 || rounds > tp.max_rounds)
        return fail(DL_ERR_INVALID, "dl_mix_rounds_trace: rounds must be in [1, %d] (one "
                                    "traced pass), got %d", tp.max_rounds, rounds);
    dl::TileArgs t = tile_args(args);
    if (!t.vec)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds_trace: operands must be 16-byte aligned "
                                        "float4 rows");
    const int32_t N = args->W.n_rows;
    if (tp.irr && t.tiled && args->tile_cols % 4)
        return fail(DL_ERR_INVALID, "dl_mix_rounds_trace: tile_cols must be a multiple of 4");
    if (t.tiled) {
        const int64_t T = args->tile_cols;
        t.lchunks = (int32_t)(T / 4);
        t.xts = (args->ldx ? args->ldx : (int64_t)N) * T * 4;
        t.yts = (args->ldy ? args->ldy : (int64_t)N) * T * 4;
        t.xrs = t.yrs = (uint32_t)(T * 4);
    } else {
        t.lchunks = 1;
        t.xts = t.yts = 16;
        t.xrs = (uint32_t)(args->ldx * 4);
        t.yrs = (uint32_t)(args->ldy * 4);
    }
    t.n_tiles = (int32_t)tp.n_steps;
    t.csr_off = tp.csr_off;
    t.scratch_off = tp.scratch_off;
    const size_t need = align_up((size_t)tp.grid * rounds * N * 4);
    char *ws = static_cast<char *>(workspace);
    if (!ws || (reinterpret_cast<uintptr_t>(ws) & 15u) || ws_bytes < need)
        return fail(DL_ERR_WORKSPACE, "dl_mix_rounds_trace: needs a 16-byte aligned workspace "
                                      "of %zu bytes (dl_mix_trace_workspace_bytes)", need);
    t.dev_partial = reinterpret_cast<float *>(ws);
    hipError_t e = tp.irr ? dl::launch_mix_trace_irr(t, tp.head, tp.gm != 0, tp.narrow != 0,
                                                      rounds, tp.grid,
                                                      (int)tp.lds, trace,
                                                      static_cast<hipStream_t>(stream))
                          : dl::launch_mix_trace(t, tp.chunks, rounds, tp.grid, (int)tp.lds, trace,
                                                 static_cast<hipStream_t>(stream));
    return e == hipSuccess ? DL_OK : hip_fail(e, "mix_trace_kernel launch");
}

int dl_mix_rounds_plan(const dl_mix_args *args, dl_mix_plan *plan) {
    g_err.clear();
    if (!plan) return fail(DL_ERR_INVALID, "dl_mix_rounds_plan: plan is NULL");
    int rc = check_mix_args(args);
    if (rc) return rc;
    Plan pl;
    rc = plan_rounds(args, &pl);
    if (rc) return rc;
    *plan = pl.pub;
    return DL_OK;
}

int dl_mix_rounds(const dl_mix_args *args, int32_t rounds, void *workspace, size_t ws_bytes,
                  dl_stream_t stream) {
    g_err.clear();
    int rc = check_mix_args(args);
    if (rc) return rc;
    if (rounds < 1) return fail(DL_ERR_INVALID, "dl_mix_rounds: rounds must be >= 1");
    Plan pl;
    rc = plan_rounds(args, &pl);
    if (rc) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int32_t Nr = args->W.n_rows;
    dl::TileArgs t = tile_args(args);
    if (!t.vec)
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_rounds: operands must be 16-byte aligned float4 "
                                        "rows");
    const int64_t T = pl.pub.tile_cols;
    if (t.tiled) {
        t.xts = (args->ldx ? args->ldx : (int64_t)Nr) * T * 4;
        t.gts = (args->ldg ? args->ldg : (int64_t)Nr) * T * 4;
        t.yts = (args->ldy ? args->ldy : (int64_t)Nr) * T * 4;
        t.xrs = t.grs = t.yrs = (uint32_t)(T * 4);
    } else {
        t.xts = t.gts = t.yts = T * 4;
        t.xrs = (uint32_t)(args->ldx * 4);
        t.grs = (uint32_t)(args->ldg * 4);
        t.yrs = (uint32_t)(args->ldy * 4);
    }
    t.n_tiles = pl.pub.n_tiles;
    t.col_base = 0;
    t.csr_off = pl.csr_off;
    t.scratch_off = pl.scratch_off;
    char *ws = static_cast<char *>(workspace);
    if (pl.dev) {
        const size_t need = align_up((size_t)pl.pub.grid * Nr * 4);
        if (!ws || (reinterpret_cast<uintptr_t>(ws) & 15u) || ws_bytes < need)
            return fail(DL_ERR_WORKSPACE, "dl_mix_rounds: deviation outputs need a 16-byte "
                                          "aligned workspace of %zu bytes", need);
        t.dev_partial = reinterpret_cast<float *>(ws);
        t.dev_max_zero = reinterpret_cast<unsigned int *>(args->dev_max);
    }
    hipError_t e = dl::launch_mix_multi(t, pl.chunks, rounds, args->g != nullptr, pl.dev,
                                        pl.pub.grid, pl.pub.lds_bytes, s);
    if (e != hipSuccess) return hip_fail(e, "mix_multi_kernel launch");
    if (pl.dev) {
        if (Nr <= 1) return zero_deviation(Nr, args->dev_sq, args->dev_max, s);
        e = dl::launch_dev_reduce(t.dev_partial, pl.pub.grid, Nr, args->dev_sq, args->dev_max, s,
                                  true);
        if (e != hipSuccess) return hip_fail(e, "dev_reduce launch");
    }
    return DL_OK;
}

int dl_mix_until_fits(int32_t n_rows, int64_t n_params, int32_t nnz) {
    if (n_rows <= 0 || n_params <= 0 || nnz < 0) return 0;
    return dl::until_lds_bytes(n_rows, n_params, nnz) <= dl::kLdsBytes ? 1 : 0;
}

int dl_mix_until(const dl_mix_until_args *a, dl_stream_t stream) {
    g_err.clear();
    if (!a) return fail(DL_ERR_INVALID, "dl_mix_until: args is NULL");
    const dl_csr &W = a->W;
    if (W.n_rows <= 0 || a->n_params <= 0 || W.nnz < 0)
        return fail(DL_ERR_INVALID, "dl_mix_until: n_rows, n_params must be > 0, nnz >= 0");
    if (!a->x || !a->y || !a->status || !W.row_ptr || (W.nnz > 0 && (!W.col || !W.w)))
        return fail(DL_ERR_INVALID, "dl_mix_until: null x/y/status/row_ptr/col/w");
    if (a->ldx < a->n_params || a->ldy < a->n_params)
        return fail(DL_ERR_INVALID, "dl_mix_until: ldx/ldy smaller than n_params");
    if (a->times < 0 || a->max_rounds < 1)
        return fail(DL_ERR_INVALID, "dl_mix_until: times must be >= 0 and max_rounds >= 1");
    if (W.uniform_row_nnz < 0 ||
        (W.uniform_row_nnz > 0 && (int64_t)W.uniform_row_nnz * W.n_rows != W.nnz))
        return fail(DL_ERR_INVALID, "dl_mix_until: uniform_row_nnz * n_rows != nnz");
    const size_t xb = ((size_t)(W.n_rows - 1) * a->ldx + a->n_params) * 4;
    const size_t yb = ((size_t)(W.n_rows - 1) * a->ldy + a->n_params) * 4;
    if (!(a->x == a->y && a->ldx == a->ldy) && overlaps(a->x, xb, a->y, yb))
        return fail(DL_ERR_INVALID, "dl_mix_until: y overlaps x (in place needs y == x, ldy == ldx)");
    if (!dl_mix_until_fits(W.n_rows, a->n_params, W.nnz))
        return fail(DL_ERR_UNSUPPORTED, "dl_mix_until: %d agents x %lld parameters (%lld bytes of "
                                        "LDS) do not fit one workgroup", W.n_rows,
                    (long long)a->n_params,
                    (long long)dl::until_lds_bytes(W.n_rows, a->n_params, W.nnz));
    dl::UntilArgs u{};
    u.x = a->x;
    u.ldx = a->ldx;
    u.y = a->y;
    u.ldy = a->ldy;
    u.n_params = a->n_params;
    u.chunks = (int32_t)((a->n_params + 3) / 4);
    u.n_rows = W.n_rows;
    u.nnz = W.nnz;
    u.rowptr = W.row_ptr;
    u.col = W.col;
    u.w = W.w;
    u.times = a->times;
    u.use_eps = a->use_eps ? 1 : 0;
    u.eps = a->eps;
    u.max_rounds = a->max_rounds;
    u.status = a->status;
    u.dev_trace = a->use_eps ? a->dev_trace : nullptr;
    hipError_t e = dl::launch_mix_until(u, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? DL_OK : hip_fail(e, "mix_until_kernel launch");
}

int dl_consensus_gd(const dl_consensus_gd_args *a, int32_t total_rows, dl_stream_t stream) {
    g_err.clear();
    if (!a) return fail(DL_ERR_INVALID, "dl_consensus_gd: args is NULL");
    if (!a->X || !a->y || !a->shard_ptr || !a->row_ptr || !a->steps || !a->w)
        return fail(DL_ERR_INVALID, "dl_consensus_gd: null X/y/shard_ptr/row_ptr/steps/w");
    if (a->n_agents <= 0 || a->n_features <= 0 || a->n_features > 16 || total_rows <= 0 ||
        a->iterations < 0 || a->max_iter < 1)
        return fail(DL_ERR_INVALID, "dl_consensus_gd: need n_agents > 0, 0 < n_features <= 16, "
                                    "rows > 0, iterations >= 0, max_iter >= 1");
    if (!(a->mean_weight > 0.0))
        return fail(DL_ERR_INVALID, "dl_consensus_gd: mean_weight must be > 0");
    int64_t x_off = 0;
    bool in_lds = dl::gd_lds_bytes(a->n_agents, a->n_features, total_rows, true, &x_off) <=
                  dl::kLdsBytes;
    const int64_t lds = dl::gd_lds_bytes(a->n_agents, a->n_features, total_rows, in_lds, &x_off);
    if (lds > dl::kLdsBytes)
        return fail(DL_ERR_UNSUPPORTED, "dl_consensus_gd: %d agents x %d features do not fit LDS",
                    a->n_agents, a->n_features);
    if (a->iterations == 0) return DL_OK;
    dl::GdArgs g{};
    g.X = a->X;
    g.y = a->y;
    g.shard_ptr = a->shard_ptr;
    g.n_agents = a->n_agents;
    g.n_features = a->n_features;
    g.rowptr = a->row_ptr;
    g.col = a->col;
    g.eps = a->eps;
    g.conv_eps = a->conv_eps;
    g.mean_weight = a->mean_weight;
    g.tau = a->tau;
    g.steps = a->steps;
    g.iterations = a->iterations;
    g.max_iter = a->max_iter;
    g.w = a->w;
    g.iters_out = a->iters_out;
    g.x_in_lds = in_lds ? 1 : 0;
    g.x_off = x_off;
    hipError_t e = dl::launch_consensus_gd(g, (int)lds, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? DL_OK : hip_fail(e, "consensus_gd_kernel launch");
}

const char *dl_last_error(void) { return g_err.c_str(); }

size_t dl_mix_workspace_bytes(int32_t n_rows, int32_t n_halo, int64_t n_params) {
    (void)n_halo;
    if (n_rows < 0 || n_params < 0) return 0;
    return align_up((size_t)max_parts() * (size_t)n_rows * 4) + align_up((size_t)n_params * 4) +
           kAlign;
}

int dl_mix_plan_query(const dl_mix_args *args, dl_mix_plan *plan) {
    g_err.clear();
    int rc = check_mix_args(args);
    if (rc) return rc;
    if (!plan) return fail(DL_ERR_INVALID, "dl_mix_plan_query: plan is NULL");
    Plan pl;
    rc = plan_mix(args, &pl);
    if (rc) return rc;
    *plan = pl.pub;
    return DL_OK;
}

int dl_mix_rounds_plan_shape(int32_t n_rows, int64_t n_params, int32_t nnz,
                             int32_t uniform_row_nnz, int32_t shared_row_weights,
                             int32_t doubly_stochastic, int32_t deviation, int32_t tile_cols,
                             dl_mix_plan *plan) {
    g_err.clear();
    if (!plan || n_rows <= 0 || n_params <= 0 || nnz < 0 || tile_cols < 0)
        return fail(DL_ERR_INVALID, "dl_mix_rounds_plan_shape: bad arguments");
    dl_mix_args a{};
    a.W.n_rows = n_rows;
    a.W.nnz = nnz;
    a.W.uniform_row_nnz = uniform_row_nnz;
    a.W.shared_row_weights = uniform_row_nnz > 0 ? shared_row_weights : 0;
    a.W.doubly_stochastic = doubly_stochastic;
    a.n_params = n_params;
    a.tile_cols = tile_cols;
    float dummy;
    if (deviation) a.dev_max = &dummy;
    Plan pl;
    const int rc = plan_rounds(&a, &pl);
    if (rc) return rc;
    *plan = pl.pub;
    return DL_OK;
}

namespace {
int plan_from_csr(const dl_csr &W, int32_t n_halo, int64_t n_params, int32_t deviation,
                  int32_t tile_cols, dl_mix_plan *plan, const char *who) {
    if (!plan || W.n_rows <= 0 || n_halo < 0 || n_params <= 0 || W.nnz < 0 || tile_cols < -1 ||
        W.min_row_nnz < 0)
        return fail(DL_ERR_INVALID, "%s: bad arguments", who);
    dl_mix_args a{};
    a.W = W;
    a.W.shared_row_weights = W.uniform_row_nnz > 0 ? W.shared_row_weights : 0;
    a.n_halo = n_halo;
    a.n_params = n_params;
    float dummy;
    if (deviation) a.dev_max = &dummy;
    if (tile_cols == -1) {  // pick the column-tiled width (a tile of every source row in LDS)
        const int reg = W.uniform_row_nnz > 0 ? 1 : 0;
        const int32_t n_w = (reg && a.W.shared_row_weights) ? W.uniform_row_nnz : W.nnz;
        const int64_t R = (int64_t)W.n_rows + n_halo;
        const int c = R > 65535 ? 0
                                : choose_tiled_chunks(a.W, (int32_t)R,
                                                      dl::csr_lds_bytes(W.n_rows, W.nnz, reg, n_w),
                                                      deviation != 0, n_halo > 0);
        tile_cols = 4 * c;   // 0: not tileable, report the row-major plan
        // a tiled halo round needs whole tiles (check_mix_args)
        if (n_halo > 0 && tile_cols > 0)
            while (tile_cols > 4 && n_params % tile_cols) tile_cols >>= 1;
        if (n_halo > 0 && tile_cols > 0 && n_params % tile_cols) tile_cols = 0;
    }
    a.tile_cols = tile_cols;
    Plan pl;
    int rc = plan_mix(&a, &pl);
    if (rc) return rc;
    *plan = pl.pub;
    return DL_OK;
}
}  // namespace

int dl_mix_plan_shape(int32_t n_rows, int32_t n_halo, int64_t n_params, int32_t nnz,
                      int32_t uniform_row_nnz, int32_t shared_row_weights, int32_t deviation,
                      int32_t tile_cols, dl_mix_plan *plan) {
    g_err.clear();
    dl_csr W{};
    W.n_rows = n_rows;
    W.nnz = nnz;
    W.uniform_row_nnz = uniform_row_nnz;
    W.shared_row_weights = shared_row_weights;
    W.min_row_nnz = uniform_row_nnz > 0 ? uniform_row_nnz : 0;
    return plan_from_csr(W, n_halo, n_params, deviation, tile_cols, plan, "dl_mix_plan_shape");
}

int dl_mix_plan_csr(const dl_csr *W, int32_t n_halo, int64_t n_params, int32_t deviation,
                    int32_t tile_cols, dl_mix_plan *plan) {
    g_err.clear();
    if (!W) return fail(DL_ERR_INVALID, "dl_mix_plan_csr: W is NULL");
    return plan_from_csr(*W, n_halo, n_params, deviation, tile_cols, plan, "dl_mix_plan_csr");
}

int dl_mix_round(const dl_mix_args *args, void *workspace, size_t ws_bytes, dl_stream_t stream) {
    g_err.clear();
    int rc = check_mix_args(args);
    if (rc) return rc;
    if (args->partial_rows_out) *args->partial_rows_out = 0;
    Plan pl;
    rc = plan_mix(args, &pl);
    if (rc) return rc;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int32_t Nr = args->W.n_rows;
    char *ws = static_cast<char *>(workspace);
    dl::TileArgs t = tile_args(args);
    // halo rounds with the lagged deviation: partials only when the deviation of x is asked for
    const bool lag = dl::tile_lag(t);
    const bool parts = pl.dev;   // a lagged halo round always writes its deviation partials
    const int32_t Np = lag ? t.n_loc : Nr;   // partial rows: lagged = one per local source row
    if (parts && (!ws || (reinterpret_cast<uintptr_t>(ws) & 15u)))
        return fail(DL_ERR_WORKSPACE, "dl_mix_round: deviation outputs need a 16-byte aligned "
                                      "workspace of dl_mix_workspace_bytes()");
    const bool sgd = args->g != nullptr;
    if ((pl.pub.path == 4 || pl.pub.path == 5) && !t.vec) {   // register-CSR: FAST-only
        // the gather kernel reads row-major operands only: column-tiled ones are refused as on
        // path 1, row-major ones take the gather path
        if (t.tiled)
            return fail(DL_ERR_INVALID, "dl_mix_round: tiled operands must be 16-byte aligned");
        pl.pub.path = 2;
    }
    if (pl.pub.path == 1 || pl.pub.path == 4 || pl.pub.path == 5) {
        // full tiles on the branch-free float4 kernel, the ragged tail tile (and unaligned
        // operands) on the guarded one; each launch writes its own deviation partial rows
        const bool reg_csr = pl.pub.path == 4 || pl.pub.path == 5;
        const int64_t T = pl.pub.tile_cols;
        if (t.tiled) {
            if (!t.vec)
                return fail(DL_ERR_INVALID, "dl_mix_round: tiled operands must be 16-byte aligned");
            // tile stride = the operand's block rows (ld*, 0 = its own rows) x T floats
            t.xts = (args->ldx ? args->ldx : t.n_loc) * T * 4;
            t.gts = (args->ldg ? args->ldg : t.n_loc) * T * 4;
            t.yts = (args->ldy ? args->ldy : (int64_t)Nr) * T * 4;
            t.xrs = t.grs = t.yrs = (uint32_t)(T * 4);
        } else {
            t.xts = t.gts = t.yts = T * 4;
            t.xrs = (uint32_t)(args->ldx * 4);
            t.grs = (uint32_t)(args->ldg * 4);
            t.yrs = (uint32_t)(args->ldy * 4);
            t.hrs = (uint32_t)(args->ldh * 4);
        }
        const int64_t n_full = t.tiled ? pl.pub.n_tiles : (t.vec ? args->n_params / T : 0);
        const int64_t n_tail = pl.pub.n_tiles - n_full;  // 0 or 1 when vec, else all tiles
        int grid_full = (int)(n_full < pl.pub.grid ? n_full : pl.pub.grid);
        int grid_tail = (int)(n_tail < pl.pub.grid ? n_tail : pl.pub.grid);
        const size_t need = align_up((size_t)(grid_full + grid_tail) * Np * 4);
        if (parts && ws_bytes < need)
            return fail(DL_ERR_WORKSPACE, "dl_mix_round: workspace %zu < %zu bytes", ws_bytes, need);
        t.csr_off = pl.csr_off;
        t.scratch_off = pl.scratch_off;
        if (pl.grp > 1) {   // tile groups: chunk c of a kernel row -> data tile c / (T / 4)
            t.grp = pl.grp;
            t.cd_sh = __builtin_ctz((unsigned)(T / 4));
        }
        float *partial = parts ? reinterpret_cast<float *>(ws) : nullptr;
        if (parts) t.dev_max_zero = reinterpret_cast<unsigned int *>(args->dev_max);
        int lds = pl.pub.lds_bytes;
        if (const char *v = getenv("DLAMD_LDS_MIN")) {  // measurement knob: LDS per workgroup
            const int m = atoi(v);                        // bounds workgroups per CU
            if (m > lds) lds = m < (int)dl::kLdsBytes ? m : (int)dl::kLdsBytes;
        }
        if (pl.pub.path == 5 && pl.head < 5 && args->n_hub_rows > 0) {
            // hub rows' register heads behind the LDS tail: as many as fit, <= 256
            const int hb = pl.head * 8;
            const int room = ((int)dl::kLdsBytes - lds) / hb;
            int nh = args->n_hub_rows < 256 ? args->n_hub_rows : 256;
            if (nh > Nr) nh = Nr;
            if (nh > room) nh = room;
            if (nh > 0) {
                t.n_hub = nh;
                t.hub_off = (uint32_t)((lds + 15) & ~15);
                lds = (int)t.hub_off + nh * hb;
                if (lds > (int)dl::kLdsBytes) {   // (alignment) fall back to no hub lanes
                    t.n_hub = 0;
                    lds = pl.pub.lds_bytes;
                }
            }
        }
        if (grid_full > 0) {
            t.n_tiles = (int32_t)n_full;
            t.col_base = 0;
            // row-major operands: each workgroup walks one contiguous run of tiles instead of
            // every grid-th tile, so its row segments follow each other in every row (c3's
            // 256 x 164,608 round: 103.8 against 105.3-107.3 us between events,
            // profiles/r13/c3_env/); the column-tiled layout keeps the grid stride (+0.4 % with
            // runs on c2, within noise).  DLAMD_TILE_RUN=0 / 1 forces it off / on.
            const char *v = getenv("DLAMD_TILE_RUN");
            const bool runs = v ? v[0] == '1' : !t.tiled;
            if (runs) t.tile_run = (int32_t)((n_full + grid_full - 1) / grid_full);
            t.dev_partial = partial;
            hipError_t e = reg_csr ? dl::launch_mix_tile_reg(t, pl.chunks, pl.head, pl.tail_fmt,
                                                             sgd, pl.dev, grid_full, lds, s)
                                   : dl::launch_mix_tile(t, pl.chunks, sgd, pl.dev, true,
                                                         grid_full, lds, true, s);
            if (e != hipSuccess) return hip_fail(e, "mix_tile_kernel launch");
        }
        if (grid_tail > 0) {
            if (reg_csr) return fail(DL_ERR_INVALID, "dl_mix_round: register-CSR plan with a tail");
            t.n_tiles = (int32_t)n_tail;
            t.col_base = n_full * T;
            t.tile_run = 0;
            t.dev_partial = parts ? partial + (size_t)grid_full * Np : nullptr;
            hipError_t e = dl::launch_mix_tile(t, pl.chunks, sgd, pl.dev, true, grid_tail,
                                               lds, false, s);
            if (e != hipSuccess) return hip_fail(e, "mix_tile_kernel (tail) launch");
        }
        if (parts) {
            if (Nr <= 1 && !lag) return zero_deviation(Nr, args->dev_sq, args->dev_max, s);
            // a lagged round without dev_sq leaves its partial rows to the caller (column
            // chunks reduced once, dl_row_sums) and says how many; its dev_max, if any, the
            // kernel zeroed
            if (lag && !args->dev_sq) {
                *args->partial_rows_out = grid_full + grid_tail;
                return DL_OK;
            }
            hipError_t e = dl::launch_dev_reduce(partial, grid_full + grid_tail, Np, args->dev_sq,
                                                 args->dev_max, s, true);
            if (e != hipSuccess) return hip_fail(e, "dev_reduce launch");
        }
        return DL_OK;
    }
    hipError_t e = dl::launch_mix_gather(t, sgd, s);
    if (e != hipSuccess) return hip_fail(e, "mix_gather_kernel launch");
    if (pl.dev) {
        if (Nr <= 1) return zero_deviation(Nr, args->dev_sq, args->dev_max, s);
        return deviation_two_pass(args->y, args->ldy, Nr, args->n_params, nullptr, args->dev_sq,
                                  args->dev_max, args->mean, ws, ws_bytes, s);
    }
    return DL_OK;
}

size_t dl_deviation_workspace_bytes(int32_t n_rows, int64_t n_params) {
    return dl_mix_workspace_bytes(n_rows, 0, n_params);
}

}  // extern "C"

namespace {

// One-pass deviation on the tile kernel (MIX = false): every agent of a column tile in one
// workgroup, column mean in LDS scratch.  tile_cols > 0: x in the column-tiled layout.
// Returns DL_ERR_UNSUPPORTED (without launching) when the agents do not fit one tile.
int deviation_one_pass(const float *x, int64_t ldx, int32_t tile_cols, int32_t n_rows,
                       int64_t n_params, float *dev_sq, float *dev_max, float *mean_out, char *ws,
                       size_t ws_bytes, hipStream_t s) {
    int c = tile_cols > 0 ? tile_cols / 4 : next_pow2_chunks(n_params);
    for (; c >= 1; c >>= 1) {
        if ((int64_t)n_rows * c <= (int64_t)dl::kRowsPerThread * dl::kTileThreads) break;
        if (tile_cols > 0) return DL_ERR_UNSUPPORTED;
    }
    if (c < 1) return DL_ERR_UNSUPPORTED;
    const int lds = (dl::kTileThreads / 64) * c * 16;
    const int64_t T = 4 * c;
    bool vec = aligned16(x) && (!mean_out || aligned16(mean_out));
    if (tile_cols == 0)
        vec = vec && ldx % 4 == 0 && ((int64_t)(n_rows - 1) * ldx + 128) * 4 < ((int64_t)1 << 32);
    else if (!vec)
        return fail(DL_ERR_INVALID, "dl_deviation_tiled: x must be 16-byte aligned");
    const int64_t n_tiles = (n_params + T - 1) / T;
    const int64_t n_full = tile_cols > 0 ? n_tiles : (vec ? n_params / T : 0);
    const int64_t n_tail = n_tiles - n_full;
    const int64_t gmax = (int64_t)device_cus() * 2;
    const int grid_full = (int)(n_full < gmax ? n_full : gmax);
    const int grid_tail = (int)(n_tail < gmax ? n_tail : gmax);
    if (ws_bytes < align_up((size_t)(grid_full + grid_tail) * n_rows * 4))
        return fail(DL_ERR_WORKSPACE, "dl_deviation: workspace too small");
    dl::TileArgs t{};
    t.x = x;
    t.ldx = ldx;
    t.n_rows = n_rows;
    t.n_src = n_rows;
    t.n_loc = n_rows;
    t.n_params = n_params;
    t.vec = vec ? 1 : 0;
    t.mean = mean_out;
    t.tiled = tile_cols > 0 ? 1 : 0;
    t.xts = tile_cols > 0 ? (int64_t)n_rows * T * 4 : T * 4;
    t.xrs = (uint32_t)(tile_cols > 0 ? T * 4 : ldx * 4);
    t.scratch_off = 0;
    float *partial = reinterpret_cast<float *>(ws);
    if (grid_full > 0) {
        t.n_tiles = (int32_t)n_full;
        t.col_base = 0;
        t.dev_partial = partial;
        hipError_t e = dl::launch_mix_tile(t, c, false, true, false, grid_full, lds, true, s);
        if (e != hipSuccess) return hip_fail(e, "dev tile launch");
    }
    if (grid_tail > 0) {
        t.n_tiles = (int32_t)n_tail;
        t.col_base = n_full * T;
        t.dev_partial = partial + (size_t)grid_full * n_rows;
        hipError_t e = dl::launch_mix_tile(t, c, false, true, false, grid_tail, lds, false, s);
        if (e != hipSuccess) return hip_fail(e, "dev tile (tail) launch");
    }
    hipError_t e = dl::launch_dev_reduce(partial, grid_full + grid_tail, n_rows, dev_sq, dev_max, s);
    if (e != hipSuccess) return hip_fail(e, "dev_reduce launch");
    return DL_OK;
}

}  // namespace

extern "C" {

int dl_deviation(const float *x, int64_t ldx, int32_t n_rows, int64_t n_params,
                 const float *mean_in, float *dev_sq, float *dev_max, float *mean_out,
                 void *workspace, size_t ws_bytes, dl_stream_t stream) {
    g_err.clear();
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (!x || n_rows <= 0 || n_params <= 0 || ldx < n_params)
        return fail(DL_ERR_INVALID, "dl_deviation: bad x/n_rows/n_params/ldx");
    char *ws = static_cast<char *>(workspace);
    if (!ws || (reinterpret_cast<uintptr_t>(ws) & 15u))
        return fail(DL_ERR_WORKSPACE, "dl_deviation: needs a 16-byte aligned workspace");
    if (n_rows <= 1) {
        if (mean_out) {
            hipError_t e = mean_in ? hipMemcpyAsync(mean_out, mean_in, (size_t)n_params * 4,
                                                    hipMemcpyDeviceToDevice, s)
                                   : hipMemcpy2DAsync(mean_out, (size_t)n_params * 4, x,
                                                      (size_t)ldx * 4, (size_t)n_params * 4, 1,
                                                      hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) return hip_fail(e, "dl_deviation mean copy");
        }
        return zero_deviation(n_rows, dev_sq, dev_max, s);
    }
    if (!mean_in) {
        int rc = deviation_one_pass(x, ldx, 0, n_rows, n_params, dev_sq, dev_max, mean_out, ws,
                                    ws_bytes, s);
        if (rc != DL_ERR_UNSUPPORTED) return rc;
    }
    return deviation_two_pass(x, ldx, n_rows, n_params, mean_in, dev_sq, dev_max, mean_out, ws,
                              ws_bytes, s);
}

int dl_deviation_tiled(const float *x, int32_t n_rows, int64_t n_params, int32_t tile_cols,
                       float *dev_sq, float *dev_max, float *mean_out, void *workspace,
                       size_t ws_bytes, dl_stream_t stream) {
    g_err.clear();
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (!x || n_rows <= 0 || n_params <= 0 || tile_cols < 4 || tile_cols > 4 * dl::kMaxChunks ||
        (tile_cols & (tile_cols - 1)))
        return fail(DL_ERR_INVALID, "dl_deviation_tiled: bad x/n_rows/n_params/tile_cols");
    char *ws = static_cast<char *>(workspace);
    if (!ws || (reinterpret_cast<uintptr_t>(ws) & 15u))
        return fail(DL_ERR_WORKSPACE, "dl_deviation_tiled: needs a 16-byte aligned workspace");
    if (n_rows <= 1) {
        if (mean_out) {
            hipError_t e = dl::launch_tile_convert(x, mean_out, n_params, 1, n_params, tile_cols,
                                                   false, s);
            if (e != hipSuccess) return hip_fail(e, "dl_deviation_tiled mean copy");
        }
        return zero_deviation(n_rows, dev_sq, dev_max, s);
    }
    int rc = deviation_one_pass(x, 0, tile_cols, n_rows, n_params, dev_sq, dev_max, mean_out, ws,
                                ws_bytes, s);
    if (rc == DL_ERR_UNSUPPORTED)
        return fail(DL_ERR_UNSUPPORTED, "dl_deviation_tiled: %d rows exceed one tile", n_rows);
    return rc;
}

int dl_to_tiled(const float *src, int64_t ld, int32_t n_rows, int64_t n_params, int32_t tile_cols,
                float *dst, dl_stream_t stream) {
    g_err.clear();
    if (!src || !dst || n_rows <= 0 || n_params <= 0 || ld < n_params || tile_cols <= 0)
        return fail(DL_ERR_INVALID, "dl_to_tiled: bad arguments");
    hipError_t e = dl::launch_tile_convert(src, dst, ld, n_rows, n_params, tile_cols, true,
                                           static_cast<hipStream_t>(stream));
    return e == hipSuccess ? DL_OK : hip_fail(e, "tile_convert launch");
}

int dl_from_tiled(const float *src, int32_t n_rows, int64_t n_params, int32_t tile_cols, float *dst,
                  int64_t ld, dl_stream_t stream) {
    g_err.clear();
    if (!src || !dst || n_rows <= 0 || n_params <= 0 || ld < n_params || tile_cols <= 0)
        return fail(DL_ERR_INVALID, "dl_from_tiled: bad arguments");
    hipError_t e = dl::launch_tile_convert(src, dst, ld, n_rows, n_params, tile_cols, false,
                                           static_cast<hipStream_t>(stream));
    return e == hipSuccess ? DL_OK : hip_fail(e, "tile_convert launch");
}

int dl_column_sum(const float *x, int64_t ldx, int32_t n_rows, int64_t n_params, float *colsum,
                  dl_stream_t stream) {
    g_err.clear();
    if (!x || !colsum || n_rows <= 0 || n_params <= 0 || ldx < n_params)
        return fail(DL_ERR_INVALID, "dl_column_sum: bad arguments");
    hipError_t e = dl::launch_column_sum(x, ldx, n_rows, n_params, colsum, 0.f,
                                         static_cast<hipStream_t>(stream));
    return e == hipSuccess ? DL_OK : hip_fail(e, "column_sum launch");
}

int dl_row_sums(const float *parts, int32_t n_parts, int32_t n_rows, float *sums, float *max_sqrt,
                int32_t max_zeroed, dl_stream_t stream) {
    g_err.clear();
    if (!parts || n_parts <= 0 || n_rows <= 0 || (!sums && !max_sqrt))
        return fail(DL_ERR_INVALID, "dl_row_sums: bad arguments");
    hipError_t e = dl::launch_dev_reduce(parts, n_parts, n_rows, sums, max_sqrt,
                                         static_cast<hipStream_t>(stream), max_zeroed != 0);
    return e == hipSuccess ? DL_OK : hip_fail(e, "dev_reduce launch");
}

int dl_max_column_std(const float *x, int64_t ldx, int32_t n_rows, int64_t n_params, float *out,
                      dl_stream_t stream) {
    g_err.clear();
    if (!x || !out || n_rows <= 0 || n_params <= 0 || ldx < n_params)
        return fail(DL_ERR_INVALID, "dl_max_column_std: bad arguments");
    hipError_t e = dl::launch_max_column_std(x, ldx, n_rows, n_params, out,
                                             static_cast<hipStream_t>(stream));
    return e == hipSuccess ? DL_OK : hip_fail(e, "max_column_std launch");
}

int dl_step_rows(const float *x, int64_t ldx, const float *g, int64_t ldg, float lr,
                 const int32_t *rows, int32_t n_sel, int64_t n_params, float *out, int64_t ldo,
                 dl_stream_t stream) {
    g_err.clear();
    if (n_sel == 0) return DL_OK;
    if (!x || !rows || !out || n_sel < 0 || n_sel > 65535 || n_params <= 0 || ldx < n_params ||
        ldo < n_params || (g && ldg < n_params))
        return fail(DL_ERR_INVALID, "dl_step_rows: bad arguments");
    hipError_t e = dl::launch_step_rows(x, ldx, g, ldg, lr, rows, n_sel, n_params, out, ldo,
                                        static_cast<hipStream_t>(stream));
    return e == hipSuccess ? DL_OK : hip_fail(e, "step_rows launch");
}

namespace {
int step_rows_tiled_peers(const float *x, int32_t x_rows, const float *g, int32_t g_rows, float lr,
                          const int32_t *rows, int32_t n_peers, const int32_t *row0,
                          float *const *outs, int64_t n_params, int32_t tile_cols,
                          dl_stream_t stream, const char *who) {
    if (!x || !rows || !row0 || !outs || n_peers < 1 || n_peers > dl::kMaxPackPeers ||
        n_params <= 0 || x_rows <= 0 || (g && g_rows <= 0) || tile_cols < 4 ||
        tile_cols > 4 * dl::kMaxChunks || (tile_cols & (tile_cols - 1)))
        return fail(DL_ERR_INVALID, "%s: bad arguments", who);
    if (!aligned16(x) || (g && !aligned16(g)))
        return fail(DL_ERR_INVALID, "%s: operands must be 16-byte aligned", who);
    const int64_t n_tiles = (n_params + tile_cols - 1) / tile_cols;
    dl::PackPeers pp{};
    pp.n = n_peers;
    if (row0[0] != 0) return fail(DL_ERR_INVALID, "%s: row0[0] must be 0", who);
    for (int b = 0; b < n_peers; ++b) {
        const int32_t nb = row0[b + 1] - row0[b];
        if (nb < 0 || row0[b + 1] > 65535)
            return fail(DL_ERR_INVALID, "%s: row0 must be non-decreasing, <= 65535", who);
        if (nb > 0 && (!outs[b] || !aligned16(outs[b])))
            return fail(DL_ERR_INVALID, "%s: out[%d] must be a 16-byte aligned pointer", who, b);
        const size_t ob = (size_t)n_tiles * nb * tile_cols * 4;
        if (nb > 0 && (overlaps(outs[b], ob, x, (size_t)n_tiles * x_rows * tile_cols * 4) ||
                       (g && overlaps(outs[b], ob, g, (size_t)n_tiles * g_rows * tile_cols * 4))))
            return fail(DL_ERR_INVALID, "%s: out[%d] overlaps x or g", who, b);
        pp.row0[b] = row0[b];
        pp.out[b] = reinterpret_cast<float4 *>(outs[b]);
    }
    pp.row0[n_peers] = row0[n_peers];
    if (row0[n_peers] == 0) return DL_OK;
    hipError_t e = dl::launch_step_rows_tiled(x, x_rows, g, g_rows, lr, rows, pp, n_tiles,
                                              tile_cols, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? DL_OK : hip_fail(e, "step_rows_tiled launch");
}
}  // namespace

int dl_step_rows_tiled(const float *x, int32_t x_rows, const float *g, int32_t g_rows, float lr,
                       const int32_t *rows, int32_t n_sel, int64_t n_params, int32_t tile_cols,
                       float *out, dl_stream_t stream) {
    g_err.clear();
    if (n_sel == 0) return DL_OK;
    if (n_sel < 0 || n_sel > 65535 || !out)
        return fail(DL_ERR_INVALID, "dl_step_rows_tiled: bad arguments");
    const int32_t row0[2] = {0, n_sel};
    float *outs[1] = {out};
    return step_rows_tiled_peers(x, x_rows, g, g_rows, lr, rows, 1, row0, outs, n_params,
                                 tile_cols, stream, "dl_step_rows_tiled");
}

int dl_step_rows_tiled_peers(const float *x, int32_t x_rows, const float *g, int32_t g_rows,
                             float lr, const int32_t *rows, int32_t n_peers, const int32_t *row0,
                             float *const *outs, int64_t n_params, int32_t tile_cols,
                             dl_stream_t stream) {
    g_err.clear();
    return step_rows_tiled_peers(x, x_rows, g, g_rows, lr, rows, n_peers, row0, outs, n_params,
                                 tile_cols, stream, "dl_step_rows_tiled_peers");
}

int dl_sgd_step(const dl_sgd_args *a, dl_stream_t stream) {
    g_err.clear();
    if (!a) return fail(DL_ERR_INVALID, "dl_sgd_step: null args");
    if (a->n_rows == 0 || a->n_params == 0) return DL_OK;
    if (!a->x || !a->g || !a->out || a->n_rows < 0 || a->n_rows > 65535 || a->n_params < 0 ||
        a->ldx < a->n_params || a->ldg < a->n_params || a->ldo < a->n_params)
        return fail(DL_ERR_INVALID, "dl_sgd_step: bad arguments (n_rows %d, n_params %lld)",
                    a->n_rows, (long long)a->n_params);
    if (a->momentum != 0.f && (!a->buf || a->ldb < a->n_params))
        return fail(DL_ERR_INVALID, "dl_sgd_step: momentum needs a buffer [n_rows, ldb >= n_params]");
    if (a->nesterov && (a->momentum <= 0.f || a->dampening != 0.f))
        return fail(DL_ERR_INVALID, "dl_sgd_step: Nesterov momentum requires a momentum and zero "
                                    "dampening");
    const size_t rb = (size_t)a->n_params * sizeof(float);
    if (a->out != a->x && overlaps(a->out, ((size_t)a->n_rows - 1) * a->ldo * 4 + rb, a->x,
                                   ((size_t)a->n_rows - 1) * a->ldx * 4 + rb))
        return fail(DL_ERR_INVALID, "dl_sgd_step: out must be x itself or not overlap it");
    float *buf = a->momentum != 0.f ? a->buf : nullptr;
    const bool vec = aligned16(a->x) && aligned16(a->g) && aligned16(a->out) &&
                     (!buf || aligned16(buf)) && (a->n_params & 3) == 0 && (a->ldx & 3) == 0 &&
                     (a->ldg & 3) == 0 && (a->ldo & 3) == 0 && (!buf || (a->ldb & 3) == 0);
    hipError_t e = dl::launch_sgd_step(a->x, a->ldx, a->g, a->ldg, buf, a->ldb, a->out, a->ldo,
                                       a->n_rows, a->n_params, a->lr, a->momentum, a->dampening,
                                       a->weight_decay, a->first ? 1 : 0, a->nesterov ? 1 : 0,
                                       vec, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? DL_OK : hip_fail(e, "sgd_step launch");
}

size_t dl_mlp_workspace_bytes(int32_t n_agents) {
    return n_agents > 0 ? dl::mlp_workspace_floats(n_agents) * sizeof(float) : 0;
}

int dl_mlp_grad(const dl_mlp_args *a, dl_stream_t stream) {
    g_err.clear();
    if (!a) return fail(DL_ERR_INVALID, "dl_mlp_grad: null args");
    if (a->n_agents == 0) return DL_OK;
    if (!dl::mlp_fused_supported(a->batch, a->input_dim, a->hidden_dim, a->output_dim))
        return fail(DL_ERR_UNSUPPORTED, "dl_mlp_grad: fused path needs batch 64, input_dim %% 4 "
                                        "== 0, even hidden_dim <= 152, output_dim <= 16 (got %d, "
                                        "%d, %d, %d)", a->batch, a->input_dim, a->hidden_dim,
                    a->output_dim);
    const int64_t din = a->input_dim, dh = a->hidden_dim, dout = a->output_dim;
    const int64_t P = dh * din + dh + 2 * (dh * dh + dh) + dout * dh + dout;
    const int32_t T = a->tile_cols;
    if (T < 0 || (T > 0 && (T < 4 || (T & (T - 1)) || (int64_t)T * a->n_agents > 0x7fffffff)))
        return fail(DL_ERR_INVALID, "dl_mlp_grad: tile_cols must be 0 or a power of two >= 4");
    if (a->n_agents < 0 || a->n_agents > 65535 || !a->X || !a->data || !a->labels || !a->G ||
        (T == 0 && (a->ldx < P || a->ldg < P)) || a->s_data < (int64_t)a->batch * din ||
        a->s_labels < a->batch)
        return fail(DL_ERR_INVALID, "dl_mlp_grad: bad arguments (agents %d, params %lld, ldx %lld, "
                                    "ldg %lld)", a->n_agents, (long long)P, (long long)a->ldx,
                    (long long)a->ldg);
    if (!aligned16(a->X) || !aligned16(a->data) || !aligned16(a->G) ||
        (T == 0 && ((a->ldx & 3) || (a->ldg & 3))) || (a->s_data & 3))
        return fail(DL_ERR_INVALID, "dl_mlp_grad: X, data, G must be 16-byte aligned with row "
                                    "strides % 4 == 0");
    const size_t tb = T ? (size_t)((P + T - 1) / T) * T * a->n_agents * 4 : 0;
    if (T && tb / 4 > 0x7fffffff)   // the kernel addresses an agent's tiled row with 32-bit offsets
        return fail(DL_ERR_UNSUPPORTED, "dl_mlp_grad: tiled X too large for 32-bit offsets");
    const size_t xb = T ? tb : ((size_t)a->n_agents - 1) * a->ldx * 4 + P * 4;
    const size_t gb = T ? tb : ((size_t)a->n_agents - 1) * a->ldg * 4 + P * 4;
    if (overlaps(a->X, xb, a->G, gb)) return fail(DL_ERR_INVALID, "dl_mlp_grad: G overlaps X");
    if (a->out_mode != 0 && a->out_mode != 1)
        return fail(DL_ERR_INVALID, "dl_mlp_grad: out_mode must be 0 (gradient) or 1 (step)");
    if (a->out_mode == 1 && T == 0 && a->ldg != a->ldx)
        return fail(DL_ERR_INVALID, "dl_mlp_grad: out_mode 1 needs ldg == ldx");
    if (a->workspace && (!aligned16(a->workspace) ||
                         overlaps(a->workspace, dl_mlp_workspace_bytes(a->n_agents), a->X, xb) ||
                         overlaps(a->workspace, dl_mlp_workspace_bytes(a->n_agents), a->G, gb)))
        return fail(DL_ERR_INVALID, "dl_mlp_grad: workspace must be 16-byte aligned and disjoint "
                                    "from X and G");
    hipError_t e = dl::launch_mlp_fused(a->X, a->ldx, a->data, a->s_data, a->labels, a->s_labels,
                                        a->G, a->ldg, a->loss, a->n_agents, a->input_dim,
                                        a->hidden_dim, a->output_dim, T, a->out_mode == 1,
                                        a->lr, a->workspace, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? DL_OK : hip_fail(e, "mlp_fused launch");
}

int dl_stream_copy(const float *src, float *dst, int64_t n_floats, int32_t variant,
                   dl_stream_t stream) {
    g_err.clear();
    if (!src || !dst || n_floats < 0 || (n_floats & 3) || !aligned16(src) || !aligned16(dst) ||
        variant < 0 || variant > 6 || (variant == 6 && n_floats % 16384))
        return fail(DL_ERR_INVALID, "dl_stream_copy: needs 16-byte aligned buffers, n %% 4 == 0, "
                                    "variant 0..6 (6: n %% 16384 == 0)");
    hipError_t e = dl::launch_stream_copy(src, dst, n_floats, variant,
                                          static_cast<hipStream_t>(stream));
    return e == hipSuccess ? DL_OK : hip_fail(e, "stream_copy launch");
}

int dl_bgemm(const dl_bgemm_args *a, dl_stream_t stream) {
    g_err.clear();
    if (!a || a->batch <= 0 || a->M <= 0 || a->N <= 0 || a->K <= 0 || !a->A || !a->B || !a->C ||
        a->batch > 65535 || a->epi < DL_EPI_NONE || a->epi > DL_EPI_BIAS_XENT)
        return fail(DL_ERR_INVALID, "dl_bgemm: bad sizes/pointers/epilogue");
    if ((a->ta ? a->lda < a->M : a->lda < a->K) || (a->tb ? a->ldb < a->K : a->ldb < a->N) ||
        a->ldc < a->N)
        return fail(DL_ERR_INVALID, "dl_bgemm: leading dimension too small");
    if (a->epi >= DL_EPI_DRELU && a->epi <= DL_EPI_DELU && (!a->H || a->ldh < a->N))
        return fail(DL_ERR_INVALID, "dl_bgemm: derivative epilogue needs H with ldh >= N");
    if (a->epi == DL_EPI_BIAS_XENT && (a->M > 64 || a->N > 64 || !a->labels))
        return fail(DL_ERR_INVALID, "dl_bgemm: cross-entropy epilogue needs M <= 64 rows, "
                                    "N <= 64 classes and labels");
    dl::BgemmArgs p{};
    p.batch = a->batch; p.M = a->M; p.N = a->N; p.K = a->K;
    p.A = a->A; p.lda = a->lda; p.sA = a->sA; p.ta = a->ta;
    p.B = a->B; p.ldb = a->ldb; p.sB = a->sB; p.tb = a->tb;
    p.C = a->C; p.ldc = a->ldc; p.sC = a->sC;
    p.epi = a->epi; p.bias = a->bias; p.sBias = a->s_bias;
    p.H = a->H; p.ldh = a->ldh; p.sH = a->sH;
    p.rowsum = a->rowsum; p.sR = a->s_rowsum;
    p.labels = a->labels; p.sLab = a->s_labels; p.loss = a->loss;
    hipError_t e = dl::launch_bgemm(p, static_cast<hipStream_t>(stream));
    return e == hipSuccess ? DL_OK : hip_fail(e, "bgemm launch");
}

int dl_xent_grad(const float *Z, int64_t sZ, const int32_t *y, int64_t sY, float *dZ, int64_t sD,
                 float *loss, int32_t batch, int32_t rows, int32_t classes, dl_stream_t stream) {
    g_err.clear();
    if (!Z || !y || !dZ || batch <= 0 || batch > 65535 || rows <= 0 || classes <= 0 ||
        classes > 64)
        return fail(DL_ERR_INVALID, "dl_xent_grad: bad arguments");
    hipError_t e = dl::launch_xent_grad(Z, sZ, y, sY, dZ, sD, loss, batch, rows, classes,
                                        static_cast<hipStream_t>(stream));
    return e == hipSuccess ? DL_OK : hip_fail(e, "xent_grad launch");
}

size_t dl_perron_workspace_bytes(int32_t dtype, int32_t n_rows, int64_t n_params) {
    const size_t sz = dtype == 1 ? 8 : 4;
    return align_up((size_t)n_rows * (size_t)n_params * sz) + kAlign;
}

int dl_perron_round(const dl_perron_args *a, void *workspace, size_t ws_bytes,
                    dl_stream_t stream) {
    g_err.clear();
    if (!a) return fail(DL_ERR_INVALID, "dl_perron_round: args is NULL");
    if (a->dtype != 0 && a->dtype != 1) return fail(DL_ERR_INVALID, "dl_perron_round: dtype");
    if (!a->y || !a->row_ptr || !a->iters_out || a->n_rows <= 0 || a->n_params <= 0 ||
        a->ldy < a->n_params || a->max_iter < 1)
        return fail(DL_ERR_INVALID, "dl_perron_round: bad arguments");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int tp = dl::perron_tile_cols(a->dtype, a->n_rows, a->n_params);
    if (tp <= 0)
        return fail(DL_ERR_UNSUPPORTED, "dl_perron_round: %d rows do not fit one LDS column",
                    a->n_rows);
    dl::PerronArgs p{};
    p.y = a->y;
    p.ldy = a->ldy;
    p.n_rows = a->n_rows;
    p.n_params = a->n_params;
    p.rowptr = a->row_ptr;
    p.col = a->col;
    p.weight = a->weight;
    p.mean_weight = a->mean_weight;
    p.eps = a->eps;
    p.conv_eps = a->conv_eps;
    p.max_iter = a->max_iter;
    p.iters_out = a->iters_out;
    p.conv_rows = a->conv_eps_rows;
    if (tp == a->n_params) {
        hipError_t e = dl::launch_perron_single(p, a->dtype, tp, s);
        return e == hipSuccess ? DL_OK : hip_fail(e, "perron_single launch");
    }
    // multi-tile: one launch per iteration, host checks the not-converged flag (synchronises)
    const size_t sz = a->dtype == 1 ? 8 : 4;
    const size_t buf_b = align_up((size_t)a->n_rows * a->n_params * sz);
    if (!workspace || ws_bytes < buf_b + kAlign)
        return fail(DL_ERR_WORKSPACE, "dl_perron_round: workspace too small");
    char *ws = static_cast<char *>(workspace);
    p.ybuf = ws;
    p.notconv = reinterpret_cast<int32_t *>(ws + buf_b);
    void *bufs[2] = {a->y, p.ybuf};
    int it = 0, cur = 0;
    int32_t host_flag = 1;
    while (it < a->max_iter) {
        ++it;
        hipError_t e = hipMemsetAsync(p.notconv, 0, 4, s);
        if (e != hipSuccess) return hip_fail(e, "perron flag memset");
        e = dl::launch_perron_step(p, a->dtype, tp, bufs[cur], bufs[cur ^ 1], it == 1, s);
        if (e != hipSuccess) return hip_fail(e, "perron_step launch");
        cur ^= 1;
        e = hipMemcpyAsync(&host_flag, p.notconv, 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) return hip_fail(e, "perron flag readback");
        if (host_flag == 0) break;
    }
    if (cur == 1) {
        hipError_t e = hipMemcpy2DAsync(a->y, (size_t)a->ldy * sz, p.ybuf, (size_t)a->n_params * sz,
                                        (size_t)a->n_params * sz, a->n_rows,
                                        hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return hip_fail(e, "perron copy-back");
    }
    hipError_t e = hipMemcpyAsync(a->iters_out, &it, 4, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    return e == hipSuccess ? DL_OK : hip_fail(e, "perron iters write");
}

}  // extern "C"
