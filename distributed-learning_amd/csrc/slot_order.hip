// Host-side LDS slot-order search (no kernels): the native form of graph.lds_slot_order.
//
// The multi-round kernels gather neighbour rows from LDS images with ds_read_b128, which a wave
// issues as four fixed 16-lane groups, one LDS cycle per group when its 16 lanes hit distinct
// 16-byte bank slots (MI355X_MICROARCH.md, LDS).  Relabelling agents -> image row slots changes
// which bank slot every neighbour read lands on while every row keeps its CSR entry order
// (= the reference's topology dict order, mixer.py:47), so mixing stays bit-identical per agent.
// This greedy swap search has the objective and the move rule of the Python restatement, with
// incremental per-(group, entry, bank) counts so one move costs O(d^2) instead of re-counting
// the touched groups: millions of moves per second, which is what the traced pass's layout
// (chunk-major planes, 16 bank slots per group) needs to get its conflicts down.
#include "../../include/dlamd.h"
#include "dl_internal.h"

#include <cstdint>
#include <cstdio>
#include <vector>

namespace {

// lane groups of ds_read_b128 (graph._B128_GROUPS)
const int kGroups[4][16] = {
    {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
    {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
    {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
    {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};

struct Search {
    int n, d, M;
    const int32_t *nbr;               // [n][d] agent ids
    std::vector<int32_t> order, slot_of, grp, cnt;   // cnt[(grp * d + e) * M + bank]
    std::vector<std::vector<int32_t>> rev;           // (x * d + e) with nbr[x][e] == agent

    int key(int s, int e) const {
        return (grp[s] * d + e) * M + slot_of[nbr[(int64_t)order[s] * d + e]] % M;
    }
};

uint64_t splitmix(uint64_t &s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

}  // namespace

extern "C" int dl_lds_slot_order(int32_t n_rows, int32_t degree, const int32_t *col,
                                 int32_t chunks, int64_t moves, uint64_t seed, int32_t *order,
                                 int64_t *conflicts) {
    if (!col || !order || !conflicts)
        return dl::fail_msg(DL_ERR_INVALID, "dl_lds_slot_order: null col/order/conflicts");
    if (n_rows < 1 || degree < 1 || moves < 0)
        return dl::fail_msg(DL_ERR_INVALID, "dl_lds_slot_order: n_rows, degree must be > 0, moves >= 0");
    if (chunks != 1 && chunks != 2 && chunks != 4 && chunks != 8)
        return dl::fail_msg(DL_ERR_INVALID, "dl_lds_slot_order: chunks must be 1, 2, 4 or 8");
    for (int64_t i = 0; i < (int64_t)n_rows * degree; ++i)
        if (col[i] < 0 || col[i] >= n_rows)
            return dl::fail_msg(DL_ERR_INVALID, "dl_lds_slot_order: col entry out of range");
    Search S;
    S.n = n_rows;
    S.d = degree;
    S.M = 16 / chunks;
    S.nbr = col;
    const int rpw = 64 / chunks;   // image rows per wave
    std::vector<int> local(rpw);
    for (int g = 0; g < 4; ++g)
        for (int L : kGroups[g]) local[L / chunks] = g;
    S.order.resize(n_rows);
    S.slot_of.resize(n_rows);
    S.grp.resize(n_rows);
    int ngrp = 0;
    for (int s = 0; s < n_rows; ++s) {
        S.order[s] = S.slot_of[s] = s;
        S.grp[s] = (s / rpw) * 4 + local[s % rpw];
        if (S.grp[s] + 1 > ngrp) ngrp = S.grp[s] + 1;
    }
    S.cnt.assign((size_t)ngrp * degree * S.M, 0);
    S.rev.resize(n_rows);
    for (int x = 0; x < n_rows; ++x)
        for (int e = 0; e < degree; ++e) S.rev[col[(int64_t)x * degree + e]].push_back(x * degree + e);
    int64_t cost = 0;
    for (int s = 0; s < n_rows; ++s)
        for (int e = 0; e < degree; ++e) cost += S.cnt[S.key(s, e)]++ > 0 ? 1 : 0;
    conflicts[0] = cost;

    // (slot, entry) pairs whose key a swap of agents a, b can change: the two swapped rows'
    // entries and every entry that names a or b.  Deduplicated so each is counted once.
    std::vector<int64_t> touched;
    auto collect = [&](int a, int b) {
        touched.clear();
        auto add = [&](int s, int e) {
            const int64_t p = (int64_t)s * degree + e;
            for (int64_t q : touched)
                if (q == p) return;
            touched.push_back(p);
        };
        for (int e = 0; e < degree; ++e) {
            add(S.slot_of[a], e);
            add(S.slot_of[b], e);
        }
        for (int32_t xe : S.rev[a]) add(S.slot_of[xe / degree], xe % degree);
        for (int32_t xe : S.rev[b]) add(S.slot_of[xe / degree], xe % degree);
    };
    // remove the touched pairs' keys, swap, add them back: returns the cost change
    auto swap_delta = [&](int a, int b) {
        int64_t delta = 0;
        for (int64_t p : touched) delta -= --S.cnt[S.key((int)(p / degree), (int)(p % degree))] > 0 ? 1 : 0;
        const int sa = S.slot_of[a], sb = S.slot_of[b];
        S.order[sa] = b;
        S.order[sb] = a;
        S.slot_of[a] = sb;
        S.slot_of[b] = sa;
        // the touched (slot, entry) positions are the same set after the swap: slots sa, sb
        // stay touched, and every entry naming a or b sits at an unchanged slot unless it is
        // a row of a or b (whose slots are exactly sa, sb)
        for (int64_t p : touched) delta += S.cnt[S.key((int)(p / degree), (int)(p % degree))]++ > 0 ? 1 : 0;
        return delta;
    };
    uint64_t rs = seed;
    for (int64_t m = 0; m < moves && cost > 0; ++m) {
        const int a = (int)(splitmix(rs) % (uint64_t)n_rows);
        const int b = (int)(splitmix(rs) % (uint64_t)n_rows);
        if (a == b) continue;
        collect(a, b);
        const int64_t delta = swap_delta(a, b);
        if (delta <= 0) {
            cost += delta;
        } else {
            swap_delta(a, b);   // b now sits at a's old slot: swapping again restores both
        }
    }
    for (int s = 0; s < n_rows; ++s) order[s] = S.order[s];
    conflicts[1] = cost;
    return DL_OK;
}
