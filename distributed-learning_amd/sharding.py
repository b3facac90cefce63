"""Multi-GPU execution of the consensus round (one process per GPU, torch.distributed / RCCL).

Two decompositions of the agent matrix X[N, P]:

* ``StripeShard`` -- column stripes.  The mix is column-independent, so every rank owns
  X[:, p0:p1] for ALL agents and mixes it with no data exchange; the only collective per round is
  the all-reduce of the N per-agent squared-deviation partials (the stop test of
  Mixer.mix, mixer.py:40-66).  This is the weak-scaling decomposition bench.py uses.

* ``HaloShard`` -- agent partition (BASELINE config c4, 2-D torus).  Every rank owns a block of
  agents; cut edges become a halo exchange: each round a rank packs the stepped rows
  (x - lr*g) its neighbours need (``dl_step_rows``), exchanges them point-to-point
  (batched isend/irecv -> RCCL send/recv over xGMI), and mixes its rows with the received halo
  (``dl_mix_round`` with n_halo > 0).  The column range is processed in chunks so the exchange of
  chunk j+1 overlaps the mix of chunk j.  This replaces the per-neighbour value messages of the
  reference (consensus_asyncio.py:236-284, consensus_tcp/agent.py:174-201).

The transport is pluggable: ``DistTransport`` (torch.distributed, RCCL on GPU / gloo on CPU) and
``LocalTransport`` (in-process virtual ranks, used to test the halo logic on one device).
"""
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from .graph import Csr

# the column-tiled pack (dl_step_rows_tiled_peers) and halo mix (dl_mix_args.n_halo_blocks) take
# at most this many peers' blocks per launch (kMaxPackPeers / kMaxHaloBlocks, dlamd.h)
MAX_TILED_PEERS = 16


# ------------------------------------------------------------------ partitioning (host)
def contiguous_partition(n, world):
    """Agents [r*n/world, (r+1)*n/world) to rank r."""
    bounds = [(r * n) // world for r in range(world + 1)]
    return [np.arange(bounds[r], bounds[r + 1]) for r in range(world)]


def torus_block_partition(rows, cols, world):
    """2-D block partition of a rows x cols torus (vertex r*cols + c) into a pr x pc grid of
    blocks with pr * pc == world, choosing the grid with the smallest block perimeter."""
    best = None
    for pr in range(1, world + 1):
        if world % pr:
            continue
        pc = world // pr
        if rows % pr or cols % pc:
            continue
        per = 2 * (rows // pr + cols // pc)
        if best is None or per < best[0]:
            best = (per, pr, pc)
    if best is None:
        return contiguous_partition(rows * cols, world)
    _, pr, pc = best
    br, bc = rows // pr, cols // pc
    parts = []
    for q in range(world):
        qr, qc = divmod(q, pc)
        rr, cc = np.meshgrid(np.arange(qr * br, (qr + 1) * br), np.arange(qc * bc, (qc + 1) * bc),
                             indexing="ij")
        parts.append((rr * cols + cc).ravel())
    return parts


def greedy_bfs_partition(csr: Csr, world):
    """Balanced BFS-grown partition for general graphs (keeps neighbourhoods together)."""
    n = csr.n_rows
    target = [(r + 1) * n // world - r * n // world for r in range(world)]
    owner = -np.ones(n, np.int64)
    parts = []
    for r in range(world):
        seed = int(np.flatnonzero(owner < 0)[0])
        frontier, members = [seed], []
        owner[seed] = r
        while frontier and len(members) < target[r]:
            a = frontier.pop(0)
            members.append(a)
            for e in range(csr.rowptr[a], csr.rowptr[a + 1]):
                b = int(csr.col[e])
                if owner[b] < 0 and len(members) + len(frontier) < target[r]:
                    owner[b] = r
                    frontier.append(b)
            if not frontier and len(members) < target[r]:
                rest = np.flatnonzero(owner < 0)
                if len(rest):
                    owner[rest[0]] = r
                    frontier.append(int(rest[0]))
        for a in frontier:
            owner[a] = -1
        parts.append(np.asarray(sorted(members), np.int64))
    left = np.flatnonzero(owner < 0)
    if len(left):
        parts[-1] = np.asarray(sorted(list(parts[-1]) + list(left)), np.int64)
    return parts


def refine_partition(csr: Csr, parts, max_swaps=100_000):
    """Balanced Kernighan-Lin-style refinement of a partition: repeatedly swap the vertex pair
    (a in part A, b in part B) whose exchange removes the most cut edges (gain(a -> B) +
    gain(b -> A) - 2 [a ~ b] > 0), until no swap improves the cut.  Part sizes are unchanged;
    every swap strictly lowers the edge cut, so it terminates.  Edge weights are ignored (the
    halo is a function of adjacency only); the diagonal is not an edge.  Each part keeps its
    vertices in increasing id order."""
    n, world = csr.n_rows, len(parts)
    owner = np.empty(n, np.int64)
    for r, p in enumerate(parts):
        owner[p] = r
    rows = np.repeat(np.arange(n), np.diff(csr.rowptr))
    keep = csr.col != rows
    src, dst = rows[keep], csr.col[keep]
    adj = [[] for _ in range(n)]
    for u, v in zip(src.tolist(), dst.tolist()):
        adj[u].append(v)
    adj = [np.unique(np.asarray(a, np.int64)) for a in adj]
    C = np.zeros((n, world), np.int64)              # neighbours of v in each part
    for v in range(n):
        np.add.at(C[v], owner[adj[v]], 1)
    swaps = 0
    while swaps < max_swaps:
        gain = C - C[np.arange(n), owner][:, None]   # gain[v, B] of moving v to part B
        best = None
        for A in range(world):
            inA = np.flatnonzero(owner == A)
            for B in range(A + 1, world):
                inB = np.flatnonzero(owner == B)
                ga, gb = gain[inA, B], gain[inB, A]
                ia, ib = int(np.argmax(ga)), int(np.argmax(gb))
                a, b = int(inA[ia]), int(inB[ib])
                g = int(ga[ia] + gb[ib]) - 2 * int(b in adj[a])
                if g <= 0 and ga[ia] + gb[ib] > 0:
                    # the best pair is adjacent: try the runner-ups of each side
                    oa, ob = np.argsort(-ga)[:8], np.argsort(-gb)[:8]
                    for xa in oa:
                        for xb in ob:
                            gg = int(ga[xa] + gb[xb]) - 2 * int(int(inB[xb]) in adj[int(inA[xa])])
                            if gg > g:
                                g, a, b = gg, int(inA[xa]), int(inB[xb])
                if g > 0 and (best is None or g > best[0]):
                    best = (g, a, b, A, B)
        if best is None:
            break
        _, a, b, A, B = best
        for v, old, new in ((a, A, B), (b, B, A)):
            owner[v] = new
            for u in adj[v]:
                C[u, old] -= 1
                C[u, new] += 1
        swaps += 1
    return [np.flatnonzero(owner == r) for r in range(world)]


def graph_partition(csr: Csr, world):
    """General balanced partition (SURVEY 8e's METIS-like greedy): BFS-grown parts, then
    Kernighan-Lin swap refinement of the edge cut."""
    return refine_partition(csr, greedy_bfs_partition(csr, world))


@dataclass
class RankPlan:
    """Everything one rank needs for halo rounds."""
    rank: int
    local: np.ndarray                 # global ids of my agents (my row order)
    csr: Csr                          # rows = my agents; cols: [0, n_local) local, then halo
    halo_from: dict = field(default_factory=dict)   # peer -> global ids I receive (halo order)
    send_to: dict = field(default_factory=dict)     # peer -> my local row indices I send
    halo_offset: dict = field(default_factory=dict)  # peer -> first halo row of its block
    # boundary-last row order (split_halo_plans): rows [0, n_deep) are interior rows no
    # boundary row reads, [n_deep, n_interior) interior rows a boundary row reads,
    # [n_interior, n_local) boundary rows (they read halo rows).  -1: not in that order.
    n_deep: int = -1
    n_interior: int = -1
    # every column of the GLOBAL W sums to 1 (taken from the global Csr in halo_plans): the
    # lagged deviation's sum(W t) = sum(t) needs it, and one rank cannot see it from its rows
    doubly_stochastic: bool = False

    @property
    def n_local(self):
        return len(self.local)

    @property
    def n_halo(self):
        return self.csr.n_src - self.csr.n_rows

    def row_sets(self):
        """(interior CSR, boundary CSR) of a boundary-last plan, for the two launches of a split
        round (``HaloShard(overlap="split")``):

        * interior: output rows [0, n_interior), sources = every local row (no halo);
        * boundary: output rows [n_interior, n_local), sources = the local window
          [n_deep, n_local) then the halo, columns renumbered into that window.

        Each row keeps its entries in the same order, so both launches fold exactly as the
        single-device round does."""
        if self.n_interior < 0:
            raise ValueError("plan is not in boundary-last order (use split_halo_plans)")
        c, n, nd, ni = self.csr, self.n_local, self.n_deep, self.n_interior
        e_i = c.rowptr[ni]
        interior = Csr(c.rowptr[:ni + 1], c.col[:e_i], c.w[:e_i], n_src=n, n_local=n)
        col = c.col[e_i:] - nd            # local c -> c - n_deep; halo h -> (n - nd) + (h - n)
        if len(col) and col.min() < 0:
            raise ValueError("a boundary row reads a row before the window (n_deep)")
        boundary = Csr(c.rowptr[ni:] - e_i, col, c.w[e_i:], n_src=c.n_src - nd, n_local=n - nd)
        return interior, boundary


def _boundary_from_send(plan, peers):
    """The boundary launch of a split round with the boundary rows' stepped values read from
    this rank's send blocks (which the pack just wrote: x - lr g rounded as the mix kernel's own
    local step) instead of re-stepping x and g: sources [the interior window rows [n_deep,
    n_interior), stepped from x and g | the send blocks of ``peers`` in order | the halo],
    the entry order of every row kept.  None when some boundary row is in no send block."""
    c, n, nd, ni = plan.csr, plan.n_local, plan.n_deep, plan.n_interior
    where, off = {}, 0
    for q in peers:
        for i, r in enumerate(plan.send_to[q]):
            where.setdefault(int(r), off + i)
        off += len(plan.send_to[q])
    n_adj, n_send = ni - nd, off
    e_i = int(c.rowptr[ni])
    src = np.asarray(c.col[e_i:], np.int64)
    out = np.empty_like(src)
    for k, v in enumerate(src.tolist()):
        if v >= n:                       # halo row
            out[k] = n_adj + n_send + (v - n)
        elif v >= ni:                    # a boundary row: its stepped value in a send block
            if v not in where:
                return None
            out[k] = n_adj + where[v]
        elif v >= nd:                    # an interior row of the window
            out[k] = v - nd
        else:
            raise ValueError("a boundary row reads a row before the window (n_deep)")
    return Csr(np.asarray(c.rowptr[ni:]) - e_i, out, c.w[e_i:],
               n_src=n_adj + n_send + (c.n_src - n), n_local=n_adj)


def halo_plans(csr: Csr, parts):
    """Per-rank local CSR + halo lists for a partition of the agents of ``csr``.

    Entry order within a row is preserved (so the fp32 fold is identical to the single-device
    round); remote columns are renumbered into the halo block of their owner, blocks ordered by
    peer rank and, inside a block, in the owner's row order -- so a peer's send rows are its
    local rows in increasing order, and a plan whose send sets are contiguous row ranges
    (split_halo_plans) packs every peer's block from one contiguous run of rows."""
    world = len(parts)
    owner = np.empty(csr.n_rows, np.int64)
    pos = np.empty(csr.n_rows, np.int64)
    for r, p in enumerate(parts):
        owner[p] = r
        pos[p] = np.arange(len(p))
    plans = []
    need = [[set() for _ in range(world)] for _ in range(world)]   # need[r][q]: ids r wants
    for r, p in enumerate(parts):
        for a in p:
            for e in range(csr.rowptr[a], csr.rowptr[a + 1]):
                b = int(csr.col[e])
                if owner[b] != r:
                    need[r][owner[b]].add(b)
    for r, p in enumerate(parts):
        halo_from, halo_offset, hidx = {}, {}, {}
        off = 0
        for q in range(world):
            if need[r][q]:
                ids = np.asarray(sorted(need[r][q], key=lambda b: pos[b]), np.int64)
                halo_from[q] = ids
                halo_offset[q] = off
                for i, b in enumerate(ids):
                    hidx[int(b)] = len(p) + off + i
                off += len(ids)
        rowptr, col, w = [0], [], []
        for a in p:
            for e in range(csr.rowptr[a], csr.rowptr[a + 1]):
                b = int(csr.col[e])
                col.append(int(pos[b]) if owner[b] == r else hidx[b])
                w.append(float(csr.w[e]))
            rowptr.append(len(col))
        local_csr = Csr(rowptr, col, w, keys=[csr.keys[a] for a in p] if csr.keys else [],
                        n_src=len(p) + off)
        send_to = {q: np.sort(pos[np.asarray(sorted(need[q][r]), np.int64)])
                   for q in range(world) if need[q][r]}
        plans.append(RankPlan(r, np.asarray(p), local_csr, halo_from, send_to, halo_offset,
                              doubly_stochastic=bool(csr.doubly_stochastic)))
    return plans


def _peer_grouped(rows, sig):
    """Order boundary rows so that every peer's send set is one contiguous run: rows grouped by
    their signature (the set of peers that read them), the groups in an order where the groups
    holding any one peer are consecutive -- e.g. a 32 x 16 torus block's [left column | top-left
    corner | top and bottom rows | top-right corner | right column] -- found by search over
    the group orders when there are at most 8 groups (the torus blocks have 3 or 5), else by
    the groups' smallest peer.  Rows keep the partition's order inside a group."""
    groups = {}
    for r in rows:
        groups.setdefault(sig[r], []).append(r)
    keys = sorted(groups, key=lambda k: (min(k) if k else -1, len(k), sorted(k)))
    peers = sorted(set().union(*keys)) if keys else []

    def runs(order):
        tot = 0
        for p in peers:
            inside = [p in k for k in order]
            tot += sum(1 for i, v in enumerate(inside) if v and (i == 0 or not inside[i - 1]))
        return tot

    if 2 < len(keys) <= 8 and runs(keys) > len(peers):
        import itertools
        best, best_runs = keys, runs(keys)
        for perm in itertools.permutations(keys):
            r = runs(perm)
            if r < best_runs:
                best, best_runs = list(perm), r
                if r == len(peers):     # every peer one run: cannot do better
                    break
        keys = best
    return np.asarray([r for k in keys for r in groups[k]], np.int64)


def split_halo_plans(csr: Csr, parts):
    """halo_plans with every rank's agents in boundary-last order: [interior rows no boundary row
    reads | interior rows a boundary row reads | boundary rows (they read halo rows)], the first
    two groups in the partition's order, the boundary rows grouped by the peers that read them
    so that each peer's send rows are one contiguous run (the halo pack then reads whole
    segments: ``_peer_grouped``).  The interior rows mix while the halo is in flight, and the
    boundary rows read only the window [n_deep, n_local) of local rows plus the halo
    (RankPlan.row_sets).  Entry order within every row is kept (bit-identical rounds)."""
    first = halo_plans(csr, parts)
    new_parts, counts = [], []
    for pl in first:
        sig = [frozenset() for _ in range(pl.n_local)]
        for q, rows in pl.send_to.items():
            for r in rows:
                sig[int(r)] = sig[int(r)] | {q}
        c, n = pl.csr, pl.n_local
        row_of = np.repeat(np.arange(n), np.diff(c.rowptr))
        bnd = np.zeros(n, bool)
        bnd[row_of[c.col >= n]] = True
        adj = np.zeros(n, bool)          # interior rows a boundary row reads
        adj[c.col[bnd[row_of] & (c.col < n)]] = True
        adj &= ~bnd
        deep = ~bnd & ~adj
        order = np.concatenate([np.flatnonzero(deep), np.flatnonzero(adj),
                                _peer_grouped(np.flatnonzero(bnd), sig)])
        new_parts.append(pl.local[order])
        counts.append((int(deep.sum()), int(deep.sum() + adj.sum())))
    plans = halo_plans(csr, new_parts)
    for pl, (nd, ni) in zip(plans, counts):
        pl.n_deep, pl.n_interior = nd, ni
    return plans


# ------------------------------------------------------------------ transports
class DistTransport:
    """Point-to-point halo exchange over torch.distributed (RCCL on GPU, gloo on CPU)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group

    @property
    def rank(self):
        return self.dist.get_rank(self.group)

    def exchange(self, sends, recvs):
        """sends: {peer: tensor}, recvs: {peer: tensor}; returns a waitable handle list."""
        ops = []
        for q, t in sorted(recvs.items()):
            ops.append(self.dist.P2POp(self.dist.irecv, t, q, self.group))
        for q, t in sorted(sends.items()):
            ops.append(self.dist.P2POp(self.dist.isend, t, q, self.group))
        return self.dist.batch_isend_irecv(ops) if ops else []

    def all_reduce_(self, t, op="sum"):
        o = self.dist.ReduceOp.SUM if op == "sum" else self.dist.ReduceOp.MAX
        self.dist.all_reduce(t, op=o, group=self.group)
        return t

    def all_reduce_async(self, t, op="sum"):
        """all_reduce_ posted without ordering the current stream after it; ``.wait()`` on the
        returned handle does (RCCL: a stream wait, the host does not block)."""
        o = self.dist.ReduceOp.SUM if op == "sum" else self.dist.ReduceOp.MAX
        return self.dist.all_reduce(t, op=o, group=self.group, async_op=True)


class _Done:
    def wait(self):
        pass


class _StagedWork:
    def __init__(self, works, host, dev):
        self.works, self.host, self.dev = works, host, dev

    def wait(self):
        for w in self.works:
            w.wait()
        for q, t in self.dev.items():
            t.copy_(self.host[q], non_blocking=False)


class StagedTransport(DistTransport):
    """DistTransport for a backend that moves only host tensors (gloo): device buffers are
    copied to the host before the send and back after the receive.  This is how several ranks
    that share ONE GPU (the single-GPU box's rehearsal of the multi-GPU path) run the real
    protocol with the real kernels; RCCL ranks use DistTransport directly."""

    def exchange(self, sends, recvs):
        hs = {q: t.cpu() for q, t in sends.items()}          # synchronises the packing kernels
        hr = {q: torch.empty(t.shape, dtype=t.dtype) for q, t in recvs.items()}
        works = super().exchange(hs, hr)
        return [_StagedWork(works, hr, recvs)] if recvs else works

    def all_reduce_(self, t, op="sum"):
        h = t.cpu()
        super().all_reduce_(h, op)
        t.copy_(h)
        return t

    def all_reduce_async(self, t, op="sum"):
        self.all_reduce_(t, op)
        return _Done()


def dist_transport(backend=None, group=None):
    """The transport for the current process group: RCCL moves device buffers itself, gloo
    needs them staged through the host."""
    import torch.distributed as dist
    backend = backend or dist.get_backend(group)
    return StagedTransport(group) if backend == "gloo" else DistTransport(group)


class LocalTransport:
    """In-process virtual ranks (threads) sharing one device: tests and single-GPU rehearsal of
    the halo protocol.  ``endpoint(r)`` gives rank r a transport with the DistTransport API."""

    def __init__(self, world):
        import threading
        self.world = world
        self.cv = threading.Condition()
        self.box = {}        # (src, dst, seq) -> tensor
        self.seq = {}        # (src, dst) -> next sequence number (send side)
        self.rseq = {}       # (src, dst) -> next sequence number (recv side)
        self.red = {}        # all-reduce rendezvous: seq -> list of tensors

    def endpoint(self, rank):
        return _LocalEndpoint(self, rank)


class _LocalWork:
    def __init__(self, tr, key, dst):
        self.tr, self.key, self.dst = tr, key, dst

    def wait(self):
        with self.tr.cv:
            self.tr.cv.wait_for(lambda: self.key in self.tr.box, timeout=120)
            src = self.tr.box.pop(self.key)
        self.dst.copy_(src)


class _LocalEndpoint:
    def __init__(self, tr, rank):
        self.tr, self.rank_ = tr, rank
        self.ar = 0

    @property
    def rank(self):
        return self.rank_

    def exchange(self, sends, recvs):
        tr, me = self.tr, self.rank_
        clones = {q: t.clone() for q, t in sends.items()}
        for t in clones.values():
            if t.is_cuda:   # the receiver copies on its own stream: the clones must be done
                torch.cuda.current_stream(t.device).synchronize()
                break
        with tr.cv:
            for q, t in clones.items():
                k = tr.seq.get((me, q), 0)
                tr.seq[(me, q)] = k + 1
                tr.box[(me, q, k)] = t
            tr.cv.notify_all()
        works = []
        for q, t in recvs.items():
            k = tr.rseq.get((q, me), 0)
            tr.rseq[(q, me)] = k + 1
            works.append(_LocalWork(tr, (q, me, k), t))
        return works

    def all_reduce_(self, t, op="sum"):
        tr = self.tr
        k = self.ar
        self.ar += 1
        with tr.cv:
            lst = tr.red.setdefault(k, [None] * tr.world)
            lst[self.rank_] = t.clone()
            tr.cv.notify_all()
            tr.cv.wait_for(lambda: all(x is not None for x in tr.red[k]), timeout=120)
            parts = list(tr.red[k])
        acc = parts[0].clone()
        for x in parts[1:]:
            acc = acc + x if op == "sum" else torch.maximum(acc, x)
        t.copy_(acc)
        return t

    def all_reduce_async(self, t, op="sum"):
        self.all_reduce_(t, op)
        return _Done()


class ResidentHaloTransport:
    """One rank of an N-rank partition measured alone (``bench.py --workload c4-rank``): the
    received halo stays resident in its buffers from whatever filled them, sends go nowhere and
    the all-reduces see one rank.  Every kernel of the rank's round runs at its real shape
    (pack, interior / boundary or chunked mixes, the lagged deviation) with no interconnect in
    the timed region."""

    rank = 0

    def exchange(self, sends, recvs):
        return []

    def all_reduce_(self, t, op="sum"):
        return t


class HipOps:
    """Device compute of a shard: libdlamd kernels (the product path)."""

    def __init__(self, device):
        from . import engine as E
        self.E = E
        self.device = torch.device(device)
        self.ws = E.Workspace(self.device)

    def csr(self, csr):
        return self.E.DeviceCsr(csr, self.device)

    def step_rows(self, X, rows, out, G=None, lr=0.0):
        if X.dim() == 3:   # column-tiled [tiles, rows, T]
            return self.E.step_rows_tiled(X, rows, out, G=G, lr=lr)
        return self.E.step_rows(X, rows, out, G=G, lr=lr)

    def step_rows_peers(self, X, rows, row0, outs, G=None, lr=0.0):
        """Every peer's column-tiled halo block in one launch (dl_step_rows_tiled_peers)."""
        return self.E.step_rows_tiled_peers(X, rows, row0, outs, G=G, lr=lr)

    def mix(self, W, X, Y, G=None, lr=0.0, halo=None, lag=None, halo_blocks=None):
        """lag = (mean_prev, colsum_out, dev_sq[, dev_max]): the lagged deviation of a halo
        round (dev_max, nullable: max sqrt(dev_sq) from the same launch's reduce).
        Column-tiled operands are 3-D [tiles, rows, T] (views), the halo then a flat buffer of
        per-peer tiled blocks of ``halo_blocks`` rows."""
        tiled = (X.shape[0] * X.shape[2], X.shape[2]) if X.dim() == 3 else None
        mean_prev, colsum, dsq, dmax = (tuple(lag) + (None,))[:4] if lag is not None else \
            (None, None, None, None)
        self.E.mix_round(W, X, Y, G=G, lr=lr, halo=halo, dev_sq=dsq, dev_max=dmax,
                         mean_prev=mean_prev, colsum_out=colsum, workspace=self.ws, tiled=tiled,
                         halo_blocks=halo_blocks)

    def mix_partials(self, W, X, Y, G, lr, halo, mean_prev, colsum, parts, halo_blocks,
                     zero_max=None):
        """A column-tiled lagged halo round that leaves its [R, n_local] deviation partial rows
        at the start of ``parts`` (a float32 slice) instead of reducing them, and returns R as
        the launch reports it (dl_mix_args.partial_rows_out): the column chunks of a round then
        place their rows back to back and share one ``row_sums`` (one reduce launch a round, not
        one per chunk).  ``zero_max``: a [1] buffer the kernel sets to 0 for that reduce."""
        tiled = (X.shape[0] * X.shape[2], X.shape[2])
        return self.E.mix_round(W, X, Y, G=G, lr=lr, halo=halo, mean_prev=mean_prev,
                                colsum_out=colsum, dev_max=zero_max, workspace=parts, tiled=tiled,
                                halo_blocks=halo_blocks)

    def partial_rows_bound(self, W, width):
        """At most this many partial rows a lagged round of ``width`` columns writes: the ABI's
        own workspace bound (dl_mix_workspace_bytes) in rows of n_local floats."""
        lib = self.E._lib.load()
        nl = W.n_local
        return int(lib.dl_mix_workspace_bytes(max(W.n_rows, nl), W.n_src - nl, int(width))) // \
            (4 * nl) + 1

    def row_sums(self, parts, zeroed_max=None):
        """(sum over the rows of parts, max sqrt of it): a chunked round's deviation.
        ``zeroed_max``: a [1] buffer already set to 0 on the stream (mix_partials' zero_max)."""
        sums = torch.empty(parts.shape[1], dtype=torch.float32, device=parts.device)
        if zeroed_max is not None:
            return self.E.row_sums(parts, sums, zeroed_max, max_zeroed=True)
        mx = torch.empty(1, dtype=torch.float32, device=parts.device)
        return self.E.row_sums(parts, sums, mx)

    def column_sum(self, X):
        return self.E.column_sum(X)

    def deviation(self, X, mean):
        return self.E.deviation(X, mean_in=mean, workspace=self.ws)


# ------------------------------------------------------------------ execution
class StripeShard:
    """Column stripe of a GossipEngine-style state on this rank (all agents, P_local columns)."""

    def __init__(self, engine, transport=None):
        self.engine = engine
        self.transport = transport

    def round(self, G=None, lr=0.0, deviation=False):
        self.engine.round(G=G, lr=lr, deviation=deviation)
        if deviation and self.transport is not None:
            self.transport.all_reduce_(self.engine.dev_sq, "sum")
        return self.engine.dev_sq if deviation else None

    def max_deviation(self):
        return torch.sqrt(self.engine.dev_sq.max())


class HaloShard:
    """One rank's agent block with halo exchange.  X, Y (and the caller's G) are resident in the
    column-tiled layout [P/T][n_local][T] (``layout="tiled"``, the default when the plan allows
    it: every tile the kernel stages is one contiguous HBM block, 5.7-5.9 TB/s against 3.1-3.8
    for row-major tiles) or row-major [n_local, P] (``layout="rows"``).
    Row-major data goes in and out through ``load_rows`` / ``rows`` / ``layout_like``."""

    def __init__(self, plan: RankPlan, n_params, device, transport, chunk_cols=None,
                 n_agents_total=None, ops=None, doubly_stochastic=None, overlap="chunks",
                 layout="auto", tile_cols=None):
        """overlap="chunks": the columns are processed in chunks, the exchange of chunk j+1 in
        flight while chunk j is mixed.  overlap="split" (a boundary-last plan from
        split_halo_plans): ONE exchange of every column per round, in flight while the interior
        rows mix; the boundary rows mix after it lands (RankPlan.row_sets).
        layout: "auto" (tiled when the LDS tile kernel takes every local + halo row at a tile
        width dividing n_params), "tiled" or "rows"; tile_cols overrides the planner's width."""
        if overlap not in ("chunks", "split"):
            raise ValueError(f"overlap must be 'chunks' or 'split' (got {overlap!r})")
        if overlap == "split" and plan.n_interior < 0:
            raise ValueError("overlap='split' needs a boundary-last plan (split_halo_plans)")
        if layout not in ("auto", "tiled", "rows"):
            raise ValueError(f"layout must be 'auto', 'tiled' or 'rows' (got {layout!r})")
        self.overlap = overlap
        self.plan = plan
        self.P = int(n_params)
        self.device = torch.device(device)
        self.transport = transport
        self.ops = ops if ops is not None else HipOps(self.device)
        self.T = 0
        if layout != "rows":
            from .engine import plan_shape
            T = int(tile_cols) if tile_cols else \
                plan_shape(plan.csr, self.P, deviation=True, tile_cols=-1)["tile_cols"]
            # the tiled pack and the tiled halo mix take at most MAX_TILED_PEERS peers each
            # (kMaxPackPeers / kMaxHaloBlocks in csrc); the row-major path has no such limit
            many = max(len(plan.send_to), len(plan.halo_from)) > MAX_TILED_PEERS
            if layout == "tiled" and many:
                raise ValueError(f"layout='tiled' takes at most {MAX_TILED_PEERS} peers per rank "
                                 f"(this rank sends to {len(plan.send_to)} and receives from "
                                 f"{len(plan.halo_from)}); use layout='rows'")
            if T >= 4 and self.P % T == 0 and not many:
                self.T = T
            elif layout == "tiled":
                raise ValueError(f"no column-tiled plan for {plan.n_local} + {plan.n_halo} rows "
                                 f"x {self.P} params (tile width {T})")
        self.layout = "tiled" if self.T else "rows"
        self.W = self.ops.csr(plan.csr)
        self.W_bnd_packed, self.bnd_blocks = None, None
        if overlap == "split":
            ci, cb = plan.row_sets()
            self.W_int = self.ops.csr(ci) if plan.n_interior > 0 else None
            self.W_bnd = self.ops.csr(cb) if plan.n_interior < plan.n_local else None
        self.n_total = n_agents_total
        chunk = int(chunk_cols or self.P)
        if self.T:      # chunks of whole tiles
            chunk = max(self.T, chunk - chunk % self.T)
        self.chunk = chunk
        for q, rows in plan.send_to.items():   # (a row past X would fault the pack kernel)
            if len(rows) and (int(np.max(rows)) >= plan.n_local or int(np.min(rows)) < 0):
                raise ValueError(f"send rows for peer {q} index past the {plan.n_local} local rows")
        self.send_rows = {q: torch.as_tensor(rows.astype(np.int32), device=self.device)
                          for q, rows in plan.send_to.items()}
        # the tiled pack of every peer in one launch: rows concatenated in peer order
        self.send_peers = sorted(plan.send_to)
        self.send_row0 = np.concatenate(
            [[0], np.cumsum([len(plan.send_to[q]) for q in self.send_peers])]).astype(int).tolist()
        self.send_rows_cat = torch.as_tensor(
            np.concatenate([plan.send_to[q] for q in self.send_peers]).astype(np.int32)
            if self.send_peers else np.zeros(0, np.int32), device=self.device)
        # per-peer halo blocks in halo_offset order (dl_mix_args.n_halo_blocks)
        self.halo_blocks = [len(plan.halo_from[q]) for q in
                            sorted(plan.halo_from, key=lambda q: plan.halo_offset[q])]
        # column-tiled split rounds: the boundary launch reads the boundary rows' stepped values
        # from the send blocks, which sit right before the halo blocks in one buffer
        # (_buffers), as further halo blocks -- x and g of those rows are not read again
        if (overlap == "split" and self.T and plan.n_deep < plan.n_interior < plan.n_local and
                len(self.send_peers) + len(self.halo_blocks) <= MAX_TILED_PEERS):
            cbp = _boundary_from_send(plan, self.send_peers)
            if cbp is not None:
                self.W_bnd_packed = self.ops.csr(cbp)
                self.bnd_blocks = [len(plan.send_to[q]) for q in self.send_peers] + \
                    self.halo_blocks
        # X, Y (and the caller's G) stream together: staggered so they do not alias in HBM
        from .engine import staggered_zeros
        self.X = staggered_zeros(self._shape(plan.n_local), 0, self.device)
        self.Y = staggered_zeros(self._shape(plan.n_local), 1, self.device)
        self._bufs = {}
        self._both = {}   # (slot, width) -> the tiled [send blocks | halo] buffer
        self._mean = None          # global column mean of X (lagged deviation), once known
        # (all-reduce handle, column sums): the previous round's sums still being all-reduced;
        # the next round's pack and exchange are posted before the mix waits for them
        self._pending_sums = None
        # the lagged deviation needs sum(W t) = sum(t): W doubly stochastic over ALL agents.
        # One rank cannot see the global column sums, so halo_plans records them on the plan;
        # an explicit argument may only narrow that (False), never assert it.
        ds = bool(plan.doubly_stochastic)
        self.doubly_stochastic = ds if doubly_stochastic is None else (ds and bool(doubly_stochastic))

    # ---------------------------------------------------------------- layout
    def _shape(self, rows, width=None):
        width = self.P if width is None else width
        return (width // self.T, rows, self.T) if self.T else (rows, width)

    def _cols(self, A, c0, c1):
        """Columns [c0, c1) of a resident matrix: whole tiles (a contiguous view) when tiled."""
        return A[c0 // self.T:c1 // self.T] if self.T else A[:, c0:c1]

    def _rows(self, A, r0, r1=None):
        """Rows [r0, r1) of a resident matrix (a view)."""
        return A[:, r0:r1] if self.T else A[r0:r1]

    def layout_like(self, A):
        """A row-major [n_local, P] tensor in the resident layout (a copy; G, X, ...)."""
        n = self.plan.n_local
        if tuple(A.shape) != (n, self.P):
            raise ValueError(f"expected shape ({n}, {self.P}), got {tuple(A.shape)}")
        A = A.to(self.device, torch.float32)
        if not self.T:
            return A.contiguous()
        return A.reshape(n, self.P // self.T, self.T).permute(1, 0, 2).contiguous()

    def load_rows(self, X):
        """Set this rank's iterate from row-major [n_local, P] rows (forgets the lagged mean)."""
        self.X.copy_(self.layout_like(X))
        self._forget_mean()

    def _forget_mean(self):
        if self._pending_sums is not None:   # an all-reduce in flight: finish it, drop it
            self._pending_sums[0].wait()
            self._pending_sums = None
        self._mean = None

    @property
    def mean_prev(self):
        """The global column mean of X that the next lagged round measures against, or None.
        Reading it finishes the previous round's column-sum all-reduce first, so it is never a
        buffer still waiting to be filled."""
        self._mean_ready()
        return self._mean

    def _mean_ready(self):
        """Turn the previous round's all-reduced column sums into mean_prev (the current stream
        waits for that all-reduce here, after this round's pack and exchange were posted)."""
        if self._pending_sums is not None:
            work, sums, mp = self._pending_sums
            work.wait()
            torch.div(sums, float(self.n_total), out=mp)
            self._pending_sums = None

    def rows(self, A=None):
        """A resident matrix (default X) as row-major [n_local, P] (a copy when tiled)."""
        A = self.X if A is None else A
        if not self.T:
            return A
        return A.permute(1, 0, 2).reshape(A.shape[1], self.P)

    # ---------------------------------------------------------------- exchange + mix
    def _buffers(self, slot, width):
        """Send/halo buffers of one pipeline slot; chunks alternate between two slots so the
        exchange of chunk j+1 never lands in the halo chunk j is being mixed from.  Tiled: each
        peer's halo block [width/T][rows][T] is one contiguous receive buffer, the blocks back to
        back in one halo buffer (the kernel's n_halo_blocks table)."""
        key = (slot, width)
        if key not in self._bufs:
            pl = self.plan
            if self.T:
                nt = width // self.T
                # [send blocks in send_peers order | halo blocks]: one buffer, so a split
                # round's boundary launch reads both as one table of tiled blocks
                n_send = self.send_row0[-1]
                both = torch.empty((n_send + pl.n_halo) * width, device=self.device)
                send = {q: both[self.send_row0[b] * width:self.send_row0[b + 1] * width].view(
                    nt, self.send_row0[b + 1] - self.send_row0[b], self.T)
                    for b, q in enumerate(self.send_peers)}
                halo = both[n_send * width:]
                recv = {q: halo[pl.halo_offset[q] * width:
                                (pl.halo_offset[q] + len(ids)) * width].view(nt, len(ids), self.T)
                        for q, ids in pl.halo_from.items()}
                self._both[key] = both
            else:
                send = {q: torch.empty(self._shape(len(r), width), device=self.device)
                        for q, r in pl.send_to.items()}
                halo = torch.empty(pl.n_halo, width, device=self.device)
                recv = {q: halo[pl.halo_offset[q]:pl.halo_offset[q] + len(ids)]
                        for q, ids in pl.halo_from.items()}
            self._bufs[key] = (send, halo, recv)
        return self._bufs[key]

    def pack(self, slot, c0, c1, G=None, lr=0.0):
        """Stepped boundary rows x - lr*g of columns [c0, c1) for every peer."""
        send, halo, recv = self._buffers(slot, c1 - c0)
        Gc = self._cols(G, c0, c1) if G is not None else None
        Xc = self._cols(self.X, c0, c1)
        if self.T and self.send_peers and hasattr(self.ops, "step_rows_peers"):
            self.ops.step_rows_peers(Xc, self.send_rows_cat, self.send_row0,
                                     [send[q] for q in self.send_peers], G=Gc, lr=lr)
            return send, halo, recv
        for q, rows in self.send_rows.items():
            self.ops.step_rows(Xc, rows, send[q], G=Gc, lr=lr)
        return send, halo, recv

    def _mix(self, W, X, Y, G, lr, halo, lag, blocks=None):
        self.ops.mix(W, X, Y, G=G, lr=lr, halo=halo, lag=lag,
                     halo_blocks=(blocks or self.halo_blocks) if (self.T and halo is not None)
                     else None)

    def mix_chunk(self, c0, c1, halo, G=None, lr=0.0, lag=None):
        Gc = self._cols(G, c0, c1) if G is not None else None
        self._mix(self.W, self._cols(self.X, c0, c1), self._cols(self.Y, c0, c1), Gc, lr,
                  halo if self.plan.n_halo else None, lag)

    def chunks(self):
        return [(c, min(c + self.chunk, self.P)) for c in range(0, self.P, self.chunk)]

    def round(self, G=None, lr=0.0, deviation=False):
        """One round: the halo exchange of chunk j+1 is in flight while chunk j is mixed.
        (Stream order makes the reuse safe: a slot's next exchange is posted after the mix that
        read it, and the collective waits for the current stream.)

        deviation=True: the lagged deviation, with no HBM pass of its own.  Each chunk's kernel
        also measures its INPUT rows -- the previous round's iterate, which it stages anyway --
        against that iterate's global column mean (``mean_prev``), and publishes this rank's
        column sums of the stepped inputs; one all-reduce of those sums (n_params floats) gives
        the next round's ``mean_prev`` (the global W is doubly stochastic, so the sum of the
        round's output is the sum of its stepped inputs).  Returns (dev_sq of my agents,
        global max deviation) of the iterate this round started from -- the value
        ``deviation()`` would have returned before the round.  (Halo rounds cannot fuse the
        deviation of their own output: its global mean is only known after every rank's round.)
        The first lagged round computes the starting mean with one column-sum pass."""
        split = self.overlap == "split" and self.plan.n_halo > 0
        chunks = [(0, self.P)] if split else self.chunks()
        lag = None
        if deviation:
            if self.plan.n_halo == 0 or not self.doubly_stochastic:
                self._forget_mean()
                dev = self.deviation()
                self._mix_all(chunks, G, lr, None)
                return dev
            if self._mean is None:
                self._mean = self._global_mean(self.X)
            colsum = torch.empty(self.P, dtype=torch.float32, device=self.device)
            # one launch measures every local row (one chunk, or the split's interior launch):
            # its reduce also gives the max, no torch kernels of its own
            one = split or len(chunks) == 1
            dmax = torch.empty(1, dtype=torch.float32, device=self.device) if one else None
            prow = None if one else self._partial_rows(chunks)
            if prow is not None:
                # column-tiled chunks: every chunk's kernel leaves its partial rows right after
                # the previous chunk's in one buffer (the count each launch reports), and one
                # row_sums reduces them all (no reduce per chunk).  Sized by the ABI's bound for
                # every chunk, so a chunk's slice (to the end of the buffer) always holds its rows
                nl = self.plan.n_local
                flat = torch.empty(prow * nl + 64, dtype=torch.float32, device=self.device)
                parts = None     # the rows actually written, after the chunks (_mix_all)
                # the max's word, zeroed by the first chunk's kernel: no memset before the reduce
                prow = [0, flat, torch.empty(1, dtype=torch.float32, device=self.device)]
            else:
                parts = torch.empty(len(chunks), self.plan.n_local, dtype=torch.float32,
                                    device=self.device)
            lag = (self._mean, colsum, parts, dmax, prow)
        if split:
            self._split_round(G, lr, None if lag is None else (lag[0], lag[1], lag[2][0], lag[3]))
        else:
            self._mix_all(chunks, G, lr, lag)
        if lag is None:
            # a round that does not publish its column sums leaves mean_prev stale (the local
            # step moved the mean): the next lagged round recomputes it
            self._forget_mean()
            return None
        if dmax is not None:
            dev_sq, dev_max = parts[0], dmax
        elif lag[4] is not None:   # chunk partial rows: one launch, the max already zeroed
            rows, flat, zmax = lag[4]
            parts = flat[:rows * self.plan.n_local].view(rows, self.plan.n_local)
            dev_sq, dev_max = self.ops.row_sums(parts, zeroed_max=zmax)
        elif hasattr(self.ops, "row_sums"):   # chunks: one launch for the sum and the max
            dev_sq, dev_max = self.ops.row_sums(parts)
        else:
            dev_sq = parts.sum(0)
            dev_max = torch.sqrt(dev_sq.max()).reshape(1)
        # the max first (the caller may read it now), then the column sums in the background:
        # the next round posts its pack and exchange before its mix waits for them (_mean_ready)
        self.transport.all_reduce_(dev_max, "max")
        mp = torch.empty(self.P, dtype=torch.float32, device=self.device)
        post = getattr(self.transport, "all_reduce_async", None)   # (a transport may have none)
        if post is None:
            self.transport.all_reduce_(colsum, "sum")
            work = _Done()
        else:
            work = post(colsum, "sum")
        self._pending_sums = (work, colsum, mp)
        self._mean = mp       # filled by _mean_ready (next round, or the mean_prev property)
        return dev_sq, dev_max

    def reset_deviation_lag(self):
        """Forget the lagged mean.  Callers that write ``X`` directly (loading new parameters)
        must call this before the next ``round(deviation=True)``."""
        self._forget_mean()

    # ---------------------------------------------------------------- Mixer.mix on the partition
    # a lagged deviation this close to eps (relative, plus the mean-rounding floor) is
    # re-evaluated exactly before the stop test uses it: the same rule as the single-device
    # Mixer's traced passes (utils/consensus_simple/mixer.py, _TIE_RTOL)
    TIE_RTOL = 2e-5

    def mix(self, times=1, eps=None, max_rounds=1 << 20):
        """``Mixer.mix(times, eps)`` (utils/consensus_simple/mixer.py:18-41) on the agent
        partition: mix until ``(eps is None or max_a ||x_a - mean|| < eps) and done >= times``,
        the deviation over ALL agents, and return ``times_done``; X is left at that iterate (the
        reference writes it back into the models, :34-35).  Every rank calls it together.

        With eps set, each round is a lagged one (``round(deviation=True)``): round k + 1 mixes
        X_k and reports the deviation of X_k, so there is no deviation pass of its own.  When
        that report meets the stop rule the loop has already computed X_{k+1}; X_k is still in
        the ping-pong buffer and becomes X again -- the reference's iterate and round count,
        at the price of one round beyond the reference's.  A report within rounding of eps is
        re-evaluated on X_k with numpy's row-order column mean over every agent
        (``exact_max_deviation``), so the integer round count does not depend on the lagged
        mean's summation order.  The comparison is float32 against float32(eps), as numpy >= 2
        compares the reference's np.float32 deviation with a Python float."""
        n = int(self.n_total or 0)
        if n <= 1:                       # len(topology) <= 1 (mixer.py:19-20)
            return 0
        target = int(np.ceil(times))     # `times_done >= times` with integer rounds
        if eps is None:
            for _ in range(target):
                self.round()
            return target
        eps32 = np.float32(eps)
        floor = None
        k = 0
        while True:
            _, dmax = self.round(deviation=True)    # X_k -> X_{k+1}; reports X_k's deviation
            d = np.float32(float(dmax.reshape(-1)[0]))
            gap = abs(float(d) - float(eps32))
            if gap <= 0.1 * abs(float(eps32)):
                if floor is None:        # 8 sqrt(P) eps32 max|mean|, the Mixer's floor
                    ref = self.mean_prev if self.mean_prev is not None else \
                        self._global_mean(self.Y)
                    floor = 8.0 * np.sqrt(self.P) * float(np.finfo(np.float32).eps) * \
                        float(ref.abs().max())
                if gap <= self.TIE_RTOL * abs(float(eps32)) + floor:
                    d = self.exact_max_deviation(self.Y)
            if d < eps32 and k >= target:
                self.X, self.Y = self.Y, self.X      # back to X_k
                self._forget_mean()
                return k
            k += 1
            if k >= max_rounds:
                raise RuntimeError(f"HaloShard.mix: no stop after {max_rounds} rounds "
                                   f"(last max deviation {d}, eps {eps})")

    def exact_max_deviation(self, A=None):
        """max_a ||x_a - mean|| of the resident iterate A (default X) over every agent, with the
        column mean summed in global agent order as numpy does (mixer.py:61) -- what
        ``Mixer._recheck_deviation`` computes on one device.  Every rank places its rows at their
        global ids in a zero matrix and the ranks all-reduce it (x + 0 is exact, so each rank then
        holds the whole iterate), then the row-order column sum and the deviation.  A
        collective, costing an N x P all-reduce: the stop rule calls it only on near-ties."""
        A = self.X if A is None else A
        n = int(self.n_total)
        full = torch.zeros(n, self.P, dtype=torch.float32, device=self.device)
        full[torch.as_tensor(np.asarray(self.plan.local, np.int64), device=self.device)] = \
            self.rows(A)
        self.transport.all_reduce_(full, "sum")
        mean = self.ops.column_sum(full) / n
        _, dmax = self.ops.deviation(full, mean)
        return np.float32(float(dmax.reshape(-1)[0]))

    def _partial_rows(self, chunks):
        """Rows of one buffer that holds every column chunk's partial rows back to back (the
        ABI's bound per chunk, summed), or None where chunks reduce one by one (row-major
        layout, ops without mix_partials, rounds without halo rows)."""
        # (n_local % 4: every chunk's slice starts 16-byte aligned; DLAMD_CHUNK_PARTIALS=0, a
        # measurement knob, keeps one reduce per chunk)
        if not (self.T and self.plan.n_halo and self.plan.n_local % 4 == 0 and
                hasattr(self.ops, "mix_partials") and
                os.environ.get("DLAMD_CHUNK_PARTIALS", "1") != "0"):
            return None
        return sum(self.ops.partial_rows_bound(self.W, c1 - c0) for c0, c1 in chunks)

    def _mix_all(self, chunks, G, lr, lag):
        def post(j):
            c0, c1 = chunks[j]
            send, halo, recv = self.pack(j % 2, c0, c1, G, lr)
            return self.transport.exchange(send, recv), halo

        pend = post(0)
        self._mean_ready()
        for j, (c0, c1) in enumerate(chunks):
            nxt = post(j + 1) if j + 1 < len(chunks) else None
            works, halo = pend
            for w in works:
                w.wait()
            if lag is not None and lag[4] is not None:   # partial rows, reduced after the loop
                rows, flat, zmax = lag[4]
                Gc = self._cols(G, c0, c1) if G is not None else None
                got = self.ops.mix_partials(self.W, self._cols(self.X, c0, c1),
                                            self._cols(self.Y, c0, c1), Gc, lr,
                                            halo if self.plan.n_halo else None, lag[0][c0:c1],
                                            lag[1][c0:c1], flat[rows * self.plan.n_local:],
                                            self.halo_blocks, zero_max=zmax if j == 0 else None)
                if not got or got < 0:
                    raise RuntimeError(f"column chunk {j}: the lagged round reported {got} "
                                       f"deviation partial rows")
                lag[4][0] = rows + int(got)   # the next chunk's rows start after these
            else:
                cl = None if lag is None else (lag[0][c0:c1], lag[1][c0:c1], lag[2][j], lag[3])
                self.mix_chunk(c0, c1, halo, G, lr, cl)
            pend = nxt
        self.X, self.Y = self.Y, self.X

    def _split_round(self, G, lr, lag):
        """One exchange of the whole boundary; the interior rows mix from the local rows while
        it is in flight (and, with ``lag``, measure every local row -- the interior launch stages
        them all); the boundary rows mix from the window [n_deep, n_local) and the halo once it
        has landed."""
        pl = self.plan
        ni, nd, n = pl.n_interior, pl.n_deep, pl.n_local
        # (posting the pack and the exchange from a side stream, so that the interior launch need
        # not wait for the pack, measured slower: 435 against 420 us a round at one rank of 8,
        # scripts/split_probe.py -- the two launches contend for HBM)
        send, halo, recv = self.pack(0, 0, self.P, G, lr)
        works = self.transport.exchange(send, recv)
        self._mean_ready()
        if ni > 0:
            self._mix(self.W_int, self.X, self._rows(self.Y, 0, ni), G, lr, None, lag)
        for w in works:
            w.wait()
        if ni < n and self.W_bnd_packed is not None and ni > 0:
            # the window's interior rows stepped from x and g, the boundary rows' stepped values
            # from the send blocks, then the halo (one buffer, bnd_blocks)
            self._mix(self.W_bnd_packed, self._rows(self.X, nd, ni), self._rows(self.Y, ni),
                      None if G is None else self._rows(G, nd, ni), lr,
                      self._both[(0, self.P)], None, blocks=self.bnd_blocks)
        elif ni < n:
            self._mix(self.W_bnd, self._rows(self.X, nd), self._rows(self.Y, ni),
                      None if G is None else self._rows(G, nd), lr, halo,
                      None if ni > 0 else lag)
        self.X, self.Y = self.Y, self.X

    def _global_mean(self, X):
        colsum = self.ops.column_sum(self.rows(X))
        self.transport.all_reduce_(colsum, "sum")
        return colsum / float(self.n_total)

    def deviation(self):
        """Global ||x_a - mean||: column sums all-reduced into the global mean, then the local
        rows against it; returns (local dev_sq, global max deviation)."""
        X = self.rows()
        colsum = self.ops.column_sum(X)
        self.transport.all_reduce_(colsum, "sum")
        mean = colsum / float(self.n_total)
        dev_sq, dev_max = self.ops.deviation(X, mean)
        self.transport.all_reduce_(dev_max, "max")
        return dev_sq, dev_max
