"""Graph compiler: reference topology formats -> CSR mixing matrices (host side).

The reference feeds the mix from three places, each with its own vertex numbering and entry
order; the fp32 summation order of the kernel is the CSR entry order, so keeping the reference
order here is what makes the HIP mix bit-identical to it:

* ``Mixer`` dict-of-dicts (utils/consensus_simple/mixer.py:43-49): rows in ``topology`` key order,
  entries in ``topology[a].items()`` order, weights as given (cast to fp32 like numpy does).
* asyncio edge list (utils/consensus_asyncio.py:40, 104): tokens = ``list(set(flatten))``,
  neighbours in edge-list order, Perron weight ``eps = 0.95 / max_deg``.
* fast-averaging edge list + per-edge weights (utils/fast_averaging.py:9-14, consensus_tcp
  agent.py:204-207): vertices by first appearance, row a = ``(1 - sum w) x_a + sum w_j x_j``.
"""
from dataclasses import dataclass, field

import numpy as np


@dataclass
class Csr:
    """Host CSR of a mixing matrix.  Source rows [0, n_rows) are local agents; rows
    [n_rows, n_src) (multi-GPU only) are halo rows owned by other ranks.  A row set of an agent
    partition (sharding.py: interior / boundary rows) sets ``n_local``: source rows
    [0, n_local) are local, [n_local, n_src) halo, and the n_rows output rows need not be
    source rows (dl_mix_args.n_local_src)."""
    rowptr: np.ndarray          # int64 [n_rows + 1]
    col: np.ndarray             # int64 [nnz]
    w: np.ndarray               # float64 [nnz] (cast to fp32 on upload)
    keys: list = field(default_factory=list)   # agent key of each local row
    n_src: int = -1
    n_local: int = -1

    def __post_init__(self):
        self.rowptr = np.asarray(self.rowptr, np.int64)
        self.col = np.asarray(self.col, np.int64)
        self.w = np.asarray(self.w, np.float64)
        if self.n_local < 0:
            self.n_local = self.n_rows
        if self.n_src < 0:
            self.n_src = self.n_local
        if self.n_src < self.n_local:
            raise ValueError("n_src < n_local")
        if len(self.rowptr) < 1 or self.rowptr[0] != 0 or np.any(np.diff(self.rowptr) < 0):
            raise ValueError("row_ptr must start at 0 and be non-decreasing")
        if self.rowptr[-1] != len(self.col) or len(self.col) != len(self.w):
            raise ValueError("row_ptr[-1], len(col) and len(w) must agree")
        if len(self.col) and (self.col.min() < 0 or self.col.max() >= self.n_src):
            raise ValueError(f"column index out of range [0, {self.n_src})")

    @property
    def n_rows(self):
        return len(self.rowptr) - 1

    @property
    def nnz(self):
        return len(self.col)

    @property
    def uniform_row_nnz(self):
        d = np.diff(self.rowptr)
        return int(d[0]) if len(d) and d[0] > 0 and np.all(d == d[0]) else 0

    @property
    def min_row_nnz(self):
        """Fewest entries of any row (dl_csr.min_row_nnz): a register head of that many entries
        per row is exact for every row (plan path 5)."""
        d = np.diff(self.rowptr)
        return int(d.min()) if len(d) else 0

    @property
    def shared_row_weights(self):
        """Regular graph whose rows all carry row 0's fp32 weight sequence (bit for bit)."""
        d = self.uniform_row_nnz
        if d == 0:
            return False
        w32 = self.w.astype(np.float32).view(np.uint32).reshape(-1, d)
        return bool(np.all(w32 == w32[0]))

    @property
    def doubly_stochastic(self):
        """Every row and column of W sums to 1 (fp32 weights, 1e-6): mean(W x) = mean(x)."""
        if self.n_src != self.n_rows or self.n_rows == 0:
            return False
        w32 = self.w.astype(np.float32).astype(np.float64)
        row_id = np.repeat(np.arange(self.n_rows), np.diff(self.rowptr))
        rows = np.bincount(row_id, weights=w32, minlength=self.n_rows)
        cols = np.bincount(self.col, weights=w32, minlength=self.n_src)
        return bool(np.all(np.abs(rows - 1) < 1e-6) and np.all(np.abs(cols - 1) < 1e-6))

    def dense(self):
        W = np.zeros((self.n_rows, self.n_src))
        for a in range(self.n_rows):
            for e in range(self.rowptr[a], self.rowptr[a + 1]):
                W[a, self.col[e]] += self.w[e]
        return W


def from_topology(topology, keys=None):
    """dict-of-dicts (``Mixer`` format) -> Csr in dict insertion order (mixer.py:46-47).

    A neighbour that is not itself a key raises KeyError, as ``params[neighbor]`` does in the
    reference."""
    keys = list(topology) if keys is None else list(keys)
    index = {k: i for i, k in enumerate(keys)}
    rowptr, col, w = [0], [], []
    for a in keys:
        for n, wt in topology[a].items():
            if n not in index:
                raise KeyError(n)
            col.append(index[n])
            w.append(float(wt))
        rowptr.append(len(col))
    return Csr(rowptr, col, w, keys=keys)


def first_appearance_vertices(edges):
    """Vertex numbering of ``find_optimal_weights`` (fast_averaging.py:9-14)."""
    v = {}
    for (a, b) in edges:
        if a not in v:
            v[a] = len(v)
        if b not in v:
            v[b] = len(v)
    return list(v)


def from_edge_weights(edges, weights, vertices=None):
    """Fast-averaging weights -> W = I - L(w) (consensus_tcp/agent.py:204-207).

    Row a: diagonal ``1 - sum_j w_aj`` first, then its neighbours in edge-list order.  Self-loop
    edges carry no weight in L (fast_averaging.py:20) and are skipped."""
    vertices = first_appearance_vertices(edges) if vertices is None else list(vertices)
    index = {k: i for i, k in enumerate(vertices)}
    nbrs = {k: {} for k in vertices}
    for (u, v), wt in zip(edges, weights):
        if u == v:
            continue
        nbrs[u].setdefault(v, float(wt))
        nbrs[v].setdefault(u, float(wt))
    rowptr, col, w = [0], [], []
    for a in vertices:
        col.append(index[a])
        w.append(1.0 - sum(nbrs[a].values()))
        for n, wt in nbrs[a].items():
            col.append(index[n])
            w.append(wt)
        rowptr.append(len(col))
    return Csr(rowptr, col, w, keys=vertices)


def tcp_neighbors(edges, weights, token):
    """What a consensus_tcp agent folds: its neighbours in the order the master's set
    comprehension yields them (master.py:230-234, kept by the agent's dict, agent.py:92-96), each
    with the weight of the first topology edge joining the two (master.py:235-241)."""
    nbrs = {u if token == v else v for (u, v) in edges if token == u or token == v}
    own = [((u, v), c) for (u, v), c in zip(edges, weights) if u == token or v == token]
    return [(n, [c for ((u, v), c) in own if u == n or v == n][0]) for n in nbrs]


def from_tcp_weights(edges, weights, vertices=None):
    """W for ``ConsensusAgent.run_once`` (consensus_tcp/agent.py:204-207)::

        value = (1.0 - sum_j w_j) * value + np.sum([x_j * w_j for j in neighbours], axis=0)

    Row a lists the neighbours in ``tcp_neighbors`` order, then the diagonal ``1 - sum w`` (summed
    as np.sum does) LAST: the CSR left fold ``((x_1 w_1 + x_2 w_2) + ...) + d x_a`` is the
    neighbour sum followed by the diagonal term, bit for bit in the arithmetic's own dtype."""
    vertices = first_appearance_vertices(edges) if vertices is None else list(vertices)
    index = {k: i for i, k in enumerate(vertices)}
    rowptr, col, w = [0], [], []
    for a in vertices:
        nb = tcp_neighbors(edges, weights, a)
        for n, c in nb:
            col.append(index[n])
            w.append(float(c))
        col.append(index[a])
        w.append(float(1.0 - np.sum([c for _, c in nb])))
        rowptr.append(len(col))
    return Csr(rowptr, col, w, keys=vertices)


def asyncio_tokens(edges):
    """``ConsensusNetwork.tokens`` = ``list(set(np.array(topology).flatten()))`` (:40)."""
    return list(set(np.array(edges).flatten()))


def asyncio_adjacency(edges, tokens=None):
    """Neighbour lists in the order an asyncio agent builds its sockets (:104-114): edge-list
    order, duplicates collapsed, self loops dropped.  Returns (tokens, rowptr, col)."""
    tokens = asyncio_tokens(edges) if tokens is None else list(tokens)
    index = {t: i for i, t in enumerate(tokens)}
    rowptr, col = [0], []
    for t in tokens:
        nb = [u if t == v else v for (u, v) in edges if (t == u or t == v) and u != v]
        for n in dict.fromkeys(nb):
            col.append(index[n])
        rowptr.append(len(col))
    return tokens, np.asarray(rowptr, np.int64), np.asarray(col, np.int64)


def perron_eps(edges, tokens=None):
    """``ConsensusNetwork.__calc_eps`` (:78-86): 0.95 / max degree of the 0/1 adjacency."""
    tokens = asyncio_tokens(edges) if tokens is None else tokens
    E = np.array([[int((u, v) in edges or (v, u) in edges) for v in tokens] for u in tokens])
    return 0.95 / np.max(np.sum(E, axis=1))


def uniform_weights(edges, w, vertices=None):
    """Every edge weight ``w`` (e.g. the best-constant 2/(l2 + l_max)) -> W = I - w L."""
    vertices = first_appearance_vertices(edges) if vertices is None else vertices
    return from_edge_weights(edges, [w] * len(edges), vertices)


# ------------------------------------------------------------------ synthetic graphs
def random_regular_edges(d, n, seed):
    """Edge list of ``networkx.random_regular_graph(d, n, seed)`` (bench config c2)."""
    import networkx as nx
    return [(int(u), int(v)) for u, v in nx.random_regular_graph(d, n, seed=seed).edges()]


def barabasi_albert_metropolis(n, m, seed):
    """networkx.barabasi_albert_graph(n, m, seed) with Metropolis weights 1/(1 + max(d_i, d_j)),
    each row's self weight first, then the neighbours in adjacency order -- the construction of
    the reference-run fixture B (tests/golden/make_golden.py).  Irregular (hub rows of ~m*sqrt(n)
    entries), symmetric, doubly stochastic."""
    import networkx as nx
    g = nx.barabasi_albert_graph(n, m, seed=seed)
    deg = dict(g.degree())
    rowptr, col, w = [0], [], []
    for i in range(n):
        nb = list(g.adj[i])
        ws = [1.0 / (1.0 + max(deg[i], deg[j])) for j in nb]
        col.append(i)
        w.append(1.0 - sum(ws))
        col.extend(nb)
        w.extend(ws)
        rowptr.append(len(col))
    return Csr(rowptr, col, w, keys=list(range(n)))


def torus_edges(rows, cols):
    """2-D periodic torus (bench config c4): vertex r*cols + c, right and down neighbours."""
    edges = []
    for r in range(rows):
        for c in range(cols):
            a = r * cols + c
            edges.append((a, r * cols + (c + 1) % cols))
            edges.append((a, ((r + 1) % rows) * cols + c))
    return edges


def laplacian(edges, vertices=None):
    vertices = first_appearance_vertices(edges) if vertices is None else vertices
    index = {k: i for i, k in enumerate(vertices)}
    n = len(vertices)
    L = np.zeros((n, n))
    for (u, v) in edges:
        if u == v:
            continue
        i, j = index[u], index[v]
        if L[i, j] == 0:
            L[i, j] = L[j, i] = -1.0
    L[np.diag_indices(n)] = -L.sum(1)
    return L


def best_constant_weight(edges, vertices=None):
    """Best constant edge weight ``2 / (lambda_2 + lambda_max)`` of the unweighted Laplacian
    (Xiao & Boyd 2004); optimal for edge-transitive graphs (ring, torus)."""
    ev = np.linalg.eigvalsh(laplacian(edges, vertices))
    return 2.0 / (ev[1] + ev[-1])


# ------------------------------------------------------------------ LDS slot order
# ds_read_b128 services a wave in four fixed 16-lane groups, one LDS cycle each when the 16
# lanes hit distinct 4-bank slots (MI355X_MICROARCH.md §LDS): lanes {0-3,12-15,20-27},
# {4-11,16-19,28-31}, {32-35,44-47,52-59}, {36-43,48-51,60-63}.
_B128_GROUPS = ([0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)),
                list(range(4, 12)) + [16, 17, 18, 19] + list(range(28, 32)),
                [32, 33, 34, 35, 44, 45, 46, 47] + list(range(52, 60)),
                list(range(36, 44)) + [48, 49, 50, 51] + list(range(60, 64)))


def _slot_groups(n, chunks):
    """Group id of every LDS row slot for a tile of `chunks` float4 per row: rows whose
    neighbour reads share one ds_read_b128 lane group (lane = row * chunks + chunk)."""
    rows_per_wave = 64 // chunks
    local = np.empty(rows_per_wave, np.int64)
    for g, lanes in enumerate(_B128_GROUPS):
        for L in lanes:
            local[L // chunks] = g
    slots = np.arange(n)
    return (slots // rows_per_wave) * 4 + local[slots % rows_per_wave]


def lds_conflicts(csr, chunks, order=None):
    """Extra LDS cycles per round of the multi-round kernel's neighbour reads: for every lane
    group and CSR entry position e, rows beyond one on the same 16-byte bank slot (slot mod
    16 / chunks).  order[slot] = agent (None = identity)."""
    d = csr.uniform_row_nnz
    if d == 0 or chunks >= 16:
        return 0
    n = csr.n_rows
    order = np.arange(n) if order is None else np.asarray(order)
    slot_of = np.empty(n, np.int64)
    slot_of[order] = np.arange(n)
    M = 16 // chunks
    nbr = csr.col.reshape(n, d)
    grp = _slot_groups(n, chunks)
    cost = 0
    for e in range(d):
        key = grp * M + slot_of[nbr[order, e]] % M       # per slot: (group, bank slot)
        _, counts = np.unique(key, return_counts=True)
        cost += int(np.sum(counts - 1))
    return cost


def lds_slot_order(csr, chunks, moves=200000, seed=0):
    """Agent order for the LDS image (order[slot] = agent) that spreads every lane group's
    neighbour reads over distinct bank slots, by greedy slot swaps.  Regular graphs only
    (identity otherwise).  Relabelling keeps each row's CSR entry order, so mixing stays
    bit-identical per agent.  Returns (order, conflicts before, conflicts after)."""
    n, d = csr.n_rows, csr.uniform_row_nnz
    ident = np.arange(n)
    base = lds_conflicts(csr, chunks)
    if d == 0 or chunks >= 16 or n < 8:
        return ident, base, base
    M = 16 // chunks
    nbr = csr.col.reshape(n, d).tolist()
    grp = _slot_groups(n, chunks).tolist()
    rev = [[] for _ in range(n)]          # (x, e) with nbr[x][e] == a
    for x in range(n):
        for e in range(d):
            rev[nbr[x][e]].append((x, e))
    order = list(range(n))
    slot_of = list(range(n))
    members = {}
    for s in range(n):
        members.setdefault(grp[s], []).append(s)

    def pair_cost(g, e):
        seen = set()
        c = 0
        for s in members[g]:
            b = slot_of[nbr[order[s]][e]] % M
            if b in seen:
                c += 1
            else:
                seen.add(b)
        return c

    rng = np.random.default_rng(seed)
    picks = rng.integers(0, n, size=(moves, 2))
    cur = base
    for a, b in picks.tolist():
        if a == b:
            continue
        pairs = {(grp[slot_of[a]], e) for e in range(d)} | {(grp[slot_of[b]], e) for e in range(d)}
        for (x, e) in rev[a] + rev[b]:
            pairs.add((grp[slot_of[x]], e))
        sa, sb = slot_of[a], slot_of[b]
        order[sa], order[sb] = b, a
        slot_of[a], slot_of[b] = sb, sa
        pairs2 = {(grp[slot_of[a]], e) for e in range(d)} | {(grp[slot_of[b]], e) for e in range(d)}
        for (x, e) in rev[a] + rev[b]:
            pairs2.add((grp[slot_of[x]], e))
        pairs |= pairs2          # every (group, entry) the swap can change, before or after it
        after = sum(pair_cost(g, e) for g, e in pairs)
        order[sa], order[sb] = a, b
        slot_of[a], slot_of[b] = sa, sb
        before_u = sum(pair_cost(g, e) for g, e in pairs)
        if after <= before_u:
            order[sa], order[sb] = b, a
            slot_of[a], slot_of[b] = sb, sa
            cur += after - before_u
            if cur == 0:
                break
    order = np.asarray(order)
    return order, base, lds_conflicts(csr, chunks, order)


def lds_slot_order_native(csr, chunks, moves=4_000_000, seed=0):
    """lds_slot_order's search in libdlamd (dl_lds_slot_order, host C++ with incremental
    counts: ~100x the moves per second of the Python loop).  Same objective, move rule and
    return value (order, conflicts before, conflicts after); its own RNG, so a different order."""
    import ctypes
    from . import _lib
    n, d = csr.n_rows, csr.uniform_row_nnz
    if d == 0 or chunks >= 16 or n < 8:
        base = lds_conflicts(csr, chunks)
        return np.arange(n), base, base
    lib = _lib.load()
    col = np.ascontiguousarray(csr.col, dtype=np.int32)
    order = np.empty(n, np.int32)
    conf = np.zeros(2, np.int64)
    _lib.check(lib.dl_lds_slot_order(n, d, col.ctypes.data, int(chunks), int(moves), int(seed),
                                     order.ctypes.data, conf.ctypes.data), "dl_lds_slot_order")
    return order.astype(np.int64), int(conf[0]), int(conf[1])


def random_irregular_metropolis(n, lo, hi, seed):
    """Every agent on a ring (degree 2) plus random extra neighbours up to a degree drawn from
    lo..hi (no hubs: rows of lo+1 .. ~hi+3 entries), Metropolis weights, self weight first,
    neighbours in a scrambled (not sorted) order: an irregular graph without the Barabasi-Albert
    hubs (bench --workload c4-ba --irregular deg)."""
    rng = np.random.default_rng(seed)
    adj = [set() for _ in range(n)]
    for i in range(n):
        adj[i].add((i + 1) % n)
        adj[(i + 1) % n].add(i)
    target = rng.integers(lo, hi + 1, n)
    for i in range(n):
        while len(adj[i]) < target[i]:
            j = int(rng.integers(n))
            if j != i:
                adj[i].add(j)
                adj[j].add(i)
    rowptr, col, w = [0], [], []
    for i in range(n):
        nb = sorted(adj[i], key=lambda j: (j * 7919 + i) % n)
        mw = [1.0 / (1.0 + max(len(adj[i]), len(adj[j]))) for j in nb]
        col.extend([i] + nb)
        w.extend([1.0 - sum(mw)] + mw)
        rowptr.append(len(col))
    return Csr(rowptr, col, w, keys=list(range(n)))


def row_length_order(csr):
    """Agents by descending CSR row length (stable): order[slot] = agent.  The register-head +
    LDS-tail tile kernel (plan path 5) mixes rows s + k * 1024 in lane s of pass k, and a wave
    runs each pass for as long as its longest tail; with the rows in this order the 64 rows of a
    wave-pass have similar lengths (Barabasi-Albert 4096 agents: 628 -> 271 tail steps per tile,
    summed over wave-passes).  Every row keeps its entry order, so the bits do not change."""
    return np.argsort(-np.diff(csr.rowptr), kind="stable")


def permuted(csr, order):
    """The CSR of the same W with rows stored in slot order (row s = agent order[s]); every row
    keeps its entry order, so the fp32 fold of each agent is unchanged."""
    order = np.asarray(order)
    n = csr.n_rows
    slot_of = np.empty(n, np.int64)
    slot_of[order] = np.arange(n)
    rp, cl, w = [0], [], []
    for s in range(n):
        a = order[s]
        lo, hi = csr.rowptr[a], csr.rowptr[a + 1]
        cl.extend(slot_of[csr.col[lo:hi]].tolist())
        w.extend(csr.w[lo:hi].tolist())
        rp.append(len(cl))
    keys = [csr.keys[a] for a in order] if csr.keys else []
    return Csr(rp, cl, w, keys=keys)
