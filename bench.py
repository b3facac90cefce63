"""Benchmark of the consensus hot path on MI355X (BASELINE.json metric).

One step = one consensus round over synthetic inputs resident in HBM: the fused local step
x <- x - lr*g, the sparse mix X <- W X over a random 4-regular graph of 1024 agents with
best-constant weights, and the per-agent disagreement ||x_a - mean|| with its max (the Mixer's
stop test).  At N GPUs every rank owns a column stripe of 2^20 parameters for all 1024 agents
(weak scaling; the mix is column-independent so the stripes need no data exchange) and the
per-agent deviation partials are all-reduced over RCCL every round, which is the round's real
exchange step.  ``value`` = rounds/s in units of the 1024 x 2^20 workload, summed over ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c2-mix|c3|c4]

Other BASELINE configs (not the headline line; run on request):
  c3  ANNModel MLP consensus SGD, 256 agents x 164,560 params, B=64 synthetic MNIST-shaped
      batches: batched per-agent gradients on fp32 MFMA (dl_bgemm) + the fused round.
      N>1: independent replicas (one 256-agent system per GPU).
  c4  64x64 periodic torus, 4096 agents x 2^18 params, best-constant weights.  N=1: the whole
      torus on one GPU (tiled layout).  N>1: agents partitioned into 2-D torus blocks, one per
      rank, boundary rows exchanged over RCCL send/recv every round (HaloShard), so the total
      work is fixed (strong scaling).
  c1  Titanic logistic-regression consensus GD, 8 agents on a ring (the reference's asyncio
      notebook run, convergence_eps 10): --steps GD iterations of every agent, each followed by
      its consensus round, in ONE dl_consensus_gd launch; the same run through the
      ConsensusNetwork / ConsensusAgent facade is reported beside it ("facade"); the CPU baseline
      is the synchronous numpy restatement.  Latency-bound by design (7 params per agent).
  c2-gossip  pure gossip averaging as Mixer.mix(times=K) (eps=None): K rounds per HBM pass on
      LDS-resident column tiles (dl_mix_rounds); rounds/s counts every round.  N>1: column
      stripes, no exchange.  --trace: Mixer.mix(times, eps) as passes of K <= 32 rounds that
      also return the K per-round max deviations (dl_mix_rounds_trace), read back every pass.
  c5  Wide-ResNet-16-4 consensus SGD, 64 agents x 2,751,146 params, B=64 synthetic CIFAR-shaped
      batches: per-agent PyTorch-ROCm (MIOpen) forward/backward into G's rows, dl_sgd_step
      (SGD momentum 0.9, wd 5e-4) and the fused round, one hipGraph per step.
      N>1: independent replicas.
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

XGMI_LINK_GBS = 153.0  # one xGMI link, one direction (MI355X: 7 links per GPU)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
FP32_MFMA_PEAK_TFLOPS = 157.3  # dense f32-input MFMA (MI355X_MICROARCH.md, peak FP32 matrix)
LDS_PEAK_GBS = 150000.0  # aggregate ds_read_b64/b128 with every CU streaming (MI355X_MICROARCH.md)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--workload", default="c2",
                   choices=["c1", "c2", "c2-mix", "c2-gossip", "c2-halo", "c3", "c4", "c4-rank",
                            "c4-gather", "c4-ba", "c5"])
    p.add_argument("--rank-of", type=int, default=8,
                   help="c4-rank: the GPU count of the partition whose rank 0 is measured alone")
    # 2: the cheapest chunk count on one GPU at rank-of 8 / 4 / 2 (433 / 746 / 1340 us a round
    # against 459 / 789 / 1346 at 4 and 494 / 833 / 1418 at 8, profiles/r12/c4rank_rankof)
    p.add_argument("--halo-chunks", default="2",
                   help="c4 / c4-rank: column chunks of the 'chunks' overlap scheme; a comma list "
                        "(c4-rank) times each count as its own scheme")
    p.add_argument("--halo-tile-cols", type=int, default=0,
                   help="c4-rank: column-tiled width of the rank's operands (0 = the planner's)")
    p.add_argument("--irregular", default="ba2", choices=["ba2", "ba1", "deg"],
                   help="c4-ba: Barabasi-Albert m=2 (the headline), m=1, or a hub-free random "
                        "graph of degree 2..6 (graph.random_irregular_metropolis)")
    p.add_argument("--order", default="auto", choices=["auto", "agents"],
                   help="c4-ba: engine row order (auto = by row length for plan path 5)")
    p.add_argument("--layout", default="auto", choices=["auto", "rows", "tiled"],
                   help="c2-gossip: resident layout of X (rows = the Mixer drop-in's row-major "
                        "flattened models)")
    p.add_argument("--graph", default="rr4", choices=["rr4", "circ4", "torus"],
                   help="c2-gossip: agent graph (circ4 = conflict-free control)")
    p.add_argument("--relabel", type=int, default=2_000_000,
                   help="c2-gossip: greedy slot-swap moves of graph.lds_slot_order_native (0 = agent "
                        "order; the default takes ~0.5 s on the host); spreads each ds_read_b128 "
                        "lane group over distinct banks")
    p.add_argument("--rounds", type=int, default=64,
                   help="c2-gossip: rounds per Mixer.mix(times=K) call (one HBM pass)")
    p.add_argument("--agents", type=int, default=1024)
    p.add_argument("--params", type=int, default=1 << 20)
    p.add_argument("--cpu-cols", type=int, default=1 << 18,
                   help="columns of the bounded CPU-baseline sample (all agents)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--trace", action="store_true",
                   help="c2-gossip: traced passes (Mixer.mix(times, eps) stop test every round)")
    p.add_argument("--no-graph", action="store_true", help="c3/c5: eager launches, no hipGraph")
    p.add_argument("--streams", type=int, default=8, help="c5: HIP streams the agents share")
    p.add_argument("--c3-emit", default="grad", choices=["step", "grad"],
                   help="c3: what the fused gradient kernel writes -- step: the local step "
                        "X - lr G, which the round then mixes (one matrix read); grad: G, and "
                        "the round forms X - lr G (reads X and G; default: 3503 vs 3159 "
                        "steps/s, profiles/r10/c3_step)")
    p.add_argument("--c3-layout", default="rows", choices=["rows", "tiled"],
                   help="c3: resident layout of X and G (tiled: the fused gradient kernel "
                        "addresses the round's column tiles; measured equal overall)")
    p.add_argument("--c3-tile-cols", type=int, default=0,
                   help="c3 tiled layout: the tile width (0: the planner's widest, 64)")
    p.add_argument("--batch", type=int, default=64, help="c5: images per agent per step")
    p.add_argument("--cudnn-benchmark", action=argparse.BooleanOptionalAction, default=True,
                   help="c5: torch.backends.cudnn.benchmark (MIOpen picks the fastest measured "
                        "solver per shape: 6.90 vs 6.66 steps/s; --no-cudnn-benchmark keeps the "
                        "default heuristic)")
    p.add_argument("--no-halo-probe", action="store_true",
                   help="N>1: skip the c4 agent-partition (RCCL halo exchange) probe that the "
                        "c2 line carries as its 'c4_halo' object")
    p.add_argument("--weights", default="best-constant", choices=["best-constant", "fdla"],
                   help="c2/c2-mix: mixing weights of the headline loop (fdla: the committed "
                        "per-edge FDLA SDP weights of the c2 graph, tests/golden/fdla_rr4_1024.npz)")
    p.add_argument("--no-fdla-probe", action="store_true",
                   help="c2 at N=1: skip the second measurement with per-edge FDLA weights")
    p.add_argument("--halo-overlap", default="both", choices=["both", "whole", "chunks", "split"],
                   help="c4 at N>1: halo overlap scheme(s) to time (sharding.HaloShard; both = "
                        "all three)")
    p.add_argument("--dist-backend", default="nccl",
                   help="nccl (= RCCL, default) or gloo (multi-rank rehearsal on one GPU)")
    return p.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_graph(n, kind="rr4"):
    """rr4: networkx random 4-regular graph (seed 0), the BASELINE graph; circ4: the circulant
    graph a ~ a+-1, a+-2 (a measurement control: every neighbour is a fixed slot offset, so the
    LDS reads of a lane group never conflict)."""
    from distributed_learning_amd.graph import (best_constant_weight, from_edge_weights,
                                                first_appearance_vertices, random_regular_edges)
    if kind == "circ4":
        edges = [(a, (a + d) % n) for a in range(n) for d in (1, 2)]
    elif kind == "torus":     # c4's periodic torus, side sqrt(n)
        from distributed_learning_amd.graph import torus_edges
        side = int(round(n ** 0.5))
        edges = torus_edges(side, side)
    else:
        edges = random_regular_edges(4, n, seed=0)
    verts = sorted(first_appearance_vertices(edges))
    w = best_constant_weight(edges, verts)
    return from_edge_weights(edges, [w] * len(edges), verts), w


FDLA_FIXTURE = os.path.join(ROOT, "tests", "golden", "fdla_rr4_1024.npz")


def build_fdla_graph(n):
    """The c2 graph with its per-edge FDLA weights (utils/fast_averaging.py's SDP, solved on the
    host by scripts/make_fdla_fixture.py and committed): W = I - L(w), every row its own weights
    (shared_row_weights = 0, so the kernel stages all n*(d+1) weights)."""
    from distributed_learning_amd.graph import first_appearance_vertices, from_edge_weights
    d = np.load(FDLA_FIXTURE)
    edges = [tuple(int(x) for x in e) for e in d["edges"]]
    if len(first_appearance_vertices(edges)) != n:
        raise ValueError(f"the FDLA fixture is for {len(first_appearance_vertices(edges))} agents")
    verts = sorted(first_appearance_vertices(edges))
    info = {"gamma": float(d["gamma"]), "gamma_best_constant": float(d["gamma_best_constant"]),
            "method": str(d["method"]), "source": os.path.relpath(FDLA_FIXTURE, ROOT)}
    return from_edge_weights(edges, d["w"], verts), info


def fdla_probe(dev, n, P, lr, steps=20, warmup=3):
    """The headline round (fused local step + mix + deviation, tiled layout) with the per-edge
    FDLA weights instead of the uniform best-constant ones: HIP-event time per launch."""
    from distributed_learning_amd import engine
    csr, info = build_fdla_graph(n)
    g = torch.Generator(device=dev).manual_seed(77)
    eng = engine.GossipEngine(csr, P, device=dev, X=torch.randn(n, P, device=dev, generator=g))
    G = eng.layout_like(torch.randn(n, P, device=dev, generator=g))
    plan = eng.plan(deviation=True)
    for _ in range(warmup):
        eng.round(G=G, lr=lr, deviation=True)
    stream = torch.cuda.current_stream(dev)
    sp = SpanEvents(steps, stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        sp.before(i)
        eng.round(G=G, lr=lr, deviation=True)
        sp.after(i)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    launch_ms = sp.ms()
    achieved = 12 * n * P / (launch_ms / 1e3) / 1e9
    del eng, G
    torch.cuda.empty_cache()
    return {"weights": "per-edge FDLA (SDP)", **info, "shared_row_weights": int(csr.shared_row_weights),
            "rounds_per_s": 1.0 / wall, "ms_per_step": wall * 1e3, "launch_ms": launch_ms,
            "achieved_GBs": achieved, "frac": achieved / HBM_PEAK_GBS, "plan": plan,
            "kernel_instance": kernel_name(plan, True, True, n)}


def copy_ceiling(dev, nbytes=4 << 30, reps=10):
    """Measured HBM ceilings (libdlamd dl_stream_copy) over 4 GiB streams: float4 copies
    (variants 0-3, read + write bytes) and the triad y = x - lr g (variants 4-6: two reads, one
    write -- the fused round's own traffic, 12 B per element; 6 in the round's access shape).
    Returns (best copy GB/s, best triad GB/s, per-variant GB/s)."""
    from distributed_learning_amd import _lib
    lib = _lib.load()
    a = torch.zeros(2 * nbytes // 4, dtype=torch.float32, device=dev)
    b = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    n = b.numel()

    best = {}
    for variant in (0, 1, 2, 3, 4, 5, 6):
        def cp():
            _lib.check(lib.dl_stream_copy(_lib.ptr(a), _lib.ptr(b), n, variant,
                                          _lib.stream_handle(dev)), "dl_stream_copy")
        cp()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(reps):
            cp()
        e.record()
        torch.cuda.synchronize()
        moved = (3 if variant >= 4 else 2) * nbytes
        best[variant] = moved / (s.elapsed_time(e) / 1e3 / reps) / 1e9
    del a, b
    return (max(best[v] for v in (0, 1, 2, 3)), max(best[v] for v in (4, 5, 6)), best)


def kernel_name(plan, sgd, dev, n_src, halo=0, lag=False):
    """The full mix_tile_kernel instantiation dl_mix_round launches for this plan (FAST path):
    mix_tile_kernel<C, KV, SGD, DEV, MIX, HALO, FAST, RD, LAG, RAG>(dl::TileArgs), as rocprofv3
    prints it.  Paths 4 / 5 keep RD = plan head entries in registers, path 5 its LDS tail in
    format RAG = plan tail_fmt; halo: 0 none, 1 row-major halo rows, 2 column-tiled halo blocks
    (the lagged-deviation instantiation of a partition round has DEV false, LAG true)."""
    c = plan["tile_cols"] // 4
    need = -(-n_src // (1024 // c))
    kv = 2 if need <= 2 else 4 if need <= 4 else 8
    if halo == 2 and need == 3 and c <= 8:   # the three-pass tiled halo instantiation
        kv = 3
    b = lambda v: "true" if v else "false"  # noqa: E731
    rd = plan.get("head", 0) if plan["path"] in (4, 5) else 0
    rag = plan.get("tail_fmt", 0) if plan["path"] == 5 else 0
    return (f"mix_tile_kernel<{c}, {kv}, {b(sgd)}, {b(dev)}, true, {halo}, true, {rd}, {b(lag)}, "
            f"{rag}>(dl::TileArgs)")


# the c2 line's committed evidence: rocprofv3 kernel trace + PMC passes of the same bench line,
# taken in the same gpurun call as the bench run saved beside it (bench.json)
PROFILE_C2 = os.path.join(ROOT, "profiles", "r13", "c2", "summary.json")


def profile_entry(kname, path=PROFILE_C2):
    """The committed rocprofv3 summary entry of this kernel instance (calls, avg_us, median_us,
    PMC bytes), or None if it was not profiled.  When the summary also holds the average over
    the profiled command's timed steps only (``graph_step_launches``: its last K launches of the
    instance, the warmup excluded), that is the entry's ``timed_avg_us``."""
    try:
        with open(path) as f:
            summ = json.load(f)
        kernels = summ["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    steps = summ.get("graph_step_launches", {})
    for name, e in kernels.items():
        if kname in name:
            e = dict(e)
            short = "mix_tile_kernel" if "mix_tile_kernel" in name else None
            if short and steps.get(f"{short}_kernels", [None])[0] == name:   # its own average
                e["timed_avg_us"] = steps[f"{short}_avg_us"]
            return e
    return None


def rocprof_fields(kname, bytes_per_launch, path=PROFILE_C2):
    """roofline fields from the committed profile itself: its kernel average as a launch time
    and the fraction of the HBM peak it implies (the same algorithmic bytes), beside the live
    HIP-event figures, so the line's frac can be checked against the profile it cites."""
    e = profile_entry(kname, path)
    if e is None or not e.get("avg_us"):
        return {}
    us = e.get("timed_avg_us") or e["avg_us"]    # the profiled command's timed rounds
    out = {"rocprof_launch_ms": us / 1e3,
           "rocprof_frac": bytes_per_launch / (us / 1e6) / 1e9 / HBM_PEAK_GBS}
    if e.get("median_us"):
        out["rocprof_median_ms"] = e["median_us"] / 1e3
    return out


def traffic_from_profile(kname, path=PROFILE_C2, bytes_hint=None):
    """HBM bytes per launch of this kernel from the committed rocprofv3 PMC summary
    (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction), or None if it was not profiled.  A kernel
    profiled at several launch sizes (``size_classes``: a whole round and its column chunks)
    gives the class nearest ``bytes_hint`` (the algorithmic bytes of the launch timed here)."""
    try:
        with open(path) as f:
            summ = json.load(f)
        kernels = summ["kernels"]
    except (OSError, ValueError, KeyError):
        return None, None
    for name, classes in summ.get("size_classes", {}).items():
        if kname in name and bytes_hint:
            c = min(classes, key=lambda c: abs(c["hbm_bytes_per_launch"] - bytes_hint))
            return c["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
    for name, e in kernels.items():
        if kname in name and "hbm_bytes_per_launch" in e:
            return e["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


def host_cpu():
    """The GPU box's host CPU: its model name (/proc/cpuinfo) and core counts, for every
    cpu_baseline record (the numpy restatement itself runs on one of them)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None
    return {"host_cpu": model or platform.processor() or platform.machine(),
            "host_cores": os.cpu_count(), "host_cores_usable": usable}


def cpu_baseline(csr, n, P, cols, sgd, lr, n_halo=0, lagged=False):
    """Bounded sample of the same round on the host: the reference algorithm restated in numpy
    (Mixer._mix_params_once + _get_deviation_dict, mixer.py:43-66, single thread) on all rows x
    `cols` columns, scaled to the full P (columns are independent).  Also the C restatement.

    n_halo > 0 (one rank of an agent partition): the CSR's n output rows read n local rows and
    n_halo halo rows (already stepped, as the exchange delivers them); lagged: the deviation is
    the halo round's -- ||x_a - mean_prev|| of the local input rows plus their column sums --
    instead of the exact one of the output."""
    from oracle import cref
    from oracle import mixer_ref as M
    rng = np.random.default_rng(0)
    X = rng.standard_normal((n, cols), dtype=np.float32)
    G = rng.standard_normal((n, cols), dtype=np.float32) if sgd else None
    H = rng.standard_normal((n_halo, cols), dtype=np.float32) if n_halo else None
    mp = rng.standard_normal(cols, dtype=np.float32) if lagged else None

    def dev(T, Y):
        if lagged:
            np.linalg.norm(X - mp, axis=1)
            M.column_mean(T[:n])
        else:
            M.deviation(Y)

    def np_round():
        T = M.sgd_step(X, G, lr) if sgd else X
        if n_halo:
            T = np.vstack([T, H])
        Y = M.mix_once(T, csr.rowptr, csr.col, csr.w)[:n]
        dev(T, Y)

    # the C restatement folds every source row's CSR row: halo rows get empty rows (output 0)
    rp = csr.rowptr if not n_halo else np.concatenate(
        [np.asarray(csr.rowptr), np.full(n_halo, csr.rowptr[-1])])
    Xc = X if not n_halo else np.vstack([X, H])
    Gc = G if not (n_halo and sgd) else np.vstack([G, np.zeros_like(H)])

    def c_round():
        Y = cref.mix_round(Xc, rp, csr.col, csr.w, G=Gc, lr=lr)[:n]
        if lagged:
            cref.deviation_sq(X, mp)
            cref.column_mean(Xc[:n])
        else:
            cref.deviation_sq(Y)

    out = {}
    for name, fn, reps in (("numpy", np_round, 3), ("c", c_round, 3)):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        dt = (time.perf_counter() - t0) / reps
        out[name] = (cols / P) / dt   # full-size rounds per second
    return out


def sample_cols(args, rows):
    """Columns of a CPU-baseline sample with half as many elements as the c2 line's (1024 agents
    x --cpu-cols): 10-20 s of host work whatever the row count (the restatement's per-row cost
    grows with the rows)."""
    return max(4, args.cpu_cols * 512 // rows // 4 * 4)


def cpu_record(csr, n, P, cols, lr, what, n_halo=0, lagged=False):
    """The cpu_baseline object of a mix-round line (N = 1): the numpy restatement's full-size
    rounds/s on one host core, the C restatement beside it, the sample and the host CPU."""
    cols = min(cols, P)
    cb = cpu_baseline(csr, n, P, cols, True, lr, n_halo=n_halo, lagged=lagged)
    rows = f"{n} agents" + (f" + {n_halo} halo rows" if n_halo else "")
    return {"value": cb["numpy"], "unit": "rounds/s", "cores": 1, "kind": "port",
            "sample": f"{rows} x {cols} of {P} columns, same graph; numpy restatement of "
                      f"Mixer._mix_params_once + {what} after x-lr*g (mixer.py:43-66), 3 rounds "
                      f"after one warm-up, scaled to the full column count",
            "c_port_value": cb["c"], **host_cpu()}


def max_over_ranks(v, world, dev):
    if world == 1:
        return v
    import torch.distributed as dist
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed_loop(step, args, world, dev):
    """W untimed warmup steps, then exactly K steps bracketed by barrier + synchronize on both
    sides; step(i) gets the timed index (None during warmup).  Returns max-over-ranks seconds."""
    for _ in range(args.warmup):
        step(None)
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    return max_over_ranks(time.perf_counter() - t0, world, dev)


def event_pairs(k, n):
    return [[torch.cuda.Event(enable_timing=True) for _ in range(n)] for _ in range(k)]


class SpanEvents:
    """One HIP timing-event pair around the K timed steps (``ms()`` = GPU time per step).  A pair
    around EVERY step would put two barrier packets between consecutive launches: 8-10 us of
    GPU idle a step, which the wall clock of the timed loop -- the line's ``value`` -- includes
    (c4-rank 0.368-0.378 against 0.359-0.360 ms a round, c2 +0.3 %; scripts/event_probe.py,
    profiles/r13/event_probe.log)."""

    def __init__(self, steps, stream):
        self.k, self.stream = steps, stream
        self.a = torch.cuda.Event(enable_timing=True)
        self.b = torch.cuda.Event(enable_timing=True)

    def before(self, i):
        if i == 0:
            self.a.record(self.stream)

    def after(self, i):
        if i == self.k - 1:
            self.b.record(self.stream)

    def ms(self):
        return self.a.elapsed_time(self.b) / self.k


def c3_init_rows(ann, gen):
    """Random-init ANNModel weights for every agent in the flattened row layout: the torch
    nn.Linear default, U(-1/sqrt(fan_in), 1/sqrt(fan_in)) for weight and bias."""
    from distributed_learning_amd.networks.ann_model import ANNModel
    X = torch.empty(ann.N, ann.P, device=ann.device)
    for name, shape in ANNModel.param_shapes(ann.din, ann.dh, ann.dout):
        layer = name.split(".")[0]
        fan_in = {"fc1": ann.din}.get(layer, ann.dh)
        o, sz = ann.offsets[name], int(np.prod(shape))
        bound = 1.0 / np.sqrt(fan_in)
        X[:, o:o + sz].uniform_(-bound, bound, generator=gen)
    return X


def c3_cpu_baseline(ann, csr, lr, n_agents_sample=16):
    """The reference's CPU path for one c3 step: a per-agent torch autograd step of ANNModel
    (networks/ann_model.py, CrossEntropyLoss) for every agent -- timed on a sample of agents and
    scaled -- plus the numpy restatement of Mixer._mix_params_once + _get_deviation_dict on all
    agents."""
    from oracle import mixer_ref as M
    from distributed_learning_amd.networks.ann_model import ANNModel
    torch.manual_seed(0)
    model = ANNModel(ann.din, ann.dh, ann.dout)
    loss_fn = torch.nn.CrossEntropyLoss()
    x = torch.randn(ann.B, ann.din)
    y = torch.randint(0, ann.dout, (ann.B,))
    opt = torch.optim.SGD(model.parameters(), lr=lr)

    def agent_step():
        opt.zero_grad()
        loss_fn(model(x), y).backward()
        opt.step()
    agent_step()
    t0 = time.perf_counter()
    for _ in range(n_agents_sample):
        agent_step()
    t_grad = (time.perf_counter() - t0) / n_agents_sample * ann.N
    rng = np.random.default_rng(0)
    X = rng.standard_normal((ann.N, ann.P), dtype=np.float32)
    t0 = time.perf_counter()
    Y = M.mix_once(X, csr.rowptr, csr.col, csr.w)
    M.deviation(Y)
    t_mix = time.perf_counter() - t0
    return 1.0 / (t_grad + t_mix), torch.get_num_threads(), t_grad, t_mix


def run_c3(args, dev, rank, world):
    """Config c3: MLP consensus SGD.  One step = batched per-agent gradients of ANNModel on a
    synthetic MNIST-shaped batch (4 forward + xent + 7 backward fp32-MFMA batched GEMMs, weight
    gradients written straight into G's rows, or with --c3-emit step the local step X - lr G) followed
    by the round X <- W (X - lr G) with the disagreement, over a random 4-regular graph of 256
    agents.  N>1: one independent
    256-agent system per GPU (replicas)."""
    from distributed_learning_amd import engine
    from distributed_learning_amd.networks.batched_ann import BatchedANN
    from distributed_learning_amd.workloads import MLPConsensusSGD
    n, B, lr = 256, 64, 0.05
    ann = BatchedANN(n, B, device=dev)
    P = ann.P
    csr, wconst = build_graph(n)
    gen = torch.Generator(device=dev).manual_seed(rank)
    X0 = c3_init_rows(ann, gen)
    data = torch.randn(n, B, ann.din, device=dev, generator=gen)
    labels = torch.randint(0, ann.dout, (n, B), device=dev, generator=gen, dtype=torch.int32)
    if ann.path == "fused" and args.c3_layout == "tiled":   # X, G column-tiled
        P_pad = P
        eng = engine.GossipEngine(csr, P, device=dev, X=X0, layout="tiled",
                                  tile_cols=args.c3_tile_cols or None)
    else:
        P_pad = MLPConsensusSGD.padded_params(csr, P, dev)   # zero columns: no ragged tail
        X0 = torch.nn.functional.pad(X0, (0, P_pad - P))
        eng = engine.GossipEngine(csr, P_pad, device=dev, X=X0, layout="rows")
    del X0
    sgd = MLPConsensusSGD(ann, eng, data, labels, lr, deviation=True,
                          emit=args.c3_emit if ann.path == "fused" else "grad")
    stream = torch.cuda.current_stream(dev)
    # phase times inside the real step order (round, then the gradient launch reading the X' it
    # left in the MALL): n_ev eager steps with a HIP event before, between and after the two
    # phases, all enqueued behind a device spin (torch.cuda._sleep) so the host is far ahead and
    # the events bracket GPU work only, not submission gaps.  (Back-to-back gradient launches run
    # without X' in the MALL: 177 us against rocprofv3's 159 us inside the step.)  The events'
    # own packets between the phases still cost: 169-173 us for the gradient launch against
    # 160.5 under rocprofv3 in the graph and 159-161 for the graph step minus the round
    # (profiles/r10/c3_phase_events), so the frac reported is the conservative one, with the
    # other two beside it.
    for _ in range(max(args.warmup, 2)):
        sgd.step()
    n_ev = max(min(args.steps, 20), 1)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(n_ev)]
    torch.cuda.synchronize()
    spin = hasattr(torch.cuda, "_sleep")
    if spin:
        torch.cuda._sleep(int(5e7))
    for a_, b_, c_ in evs:
        a_.record(stream)
        sgd.gradients()
        b_.record(stream)
        sgd.round()
        c_.record(stream)
    torch.cuda.synchronize()
    grad_ms = sum(a_.elapsed_time(b_) for a_, b_, _ in evs) / n_ev
    mix_ms = sum(b_.elapsed_time(c_) for _, b_, c_ in evs) / n_ev
    phase_how = ("HIP events around each phase of %d eager steps enqueued behind a device spin"
                 % n_ev if spin else "HIP events around each phase of %d eager steps" % n_ev)
    losses = [sgd.loss.mean()]
    use_graph = not args.no_graph
    if use_graph:
        sgd.capture()

    def step(i):
        if use_graph:
            sgd.replay(1)
        else:
            sgd.step()

    elapsed = timed_loop(step, args, world, dev)
    losses.append(sgd.loss.mean())
    # cross-check: the timed step minus the round phase (graph replay: no host gaps)
    grad_step_ms = max(elapsed / args.steps * 1e3 - mix_ms, 1e-6)
    grad_ms = max_over_ranks(grad_ms, world, dev)
    mix_ms = max_over_ranks(mix_ms, world, dev)
    flops = ann.flops_per_step()
    # algorithmic: the real columns only (padding is overhead); read T (step emission) or X and
    # G, write X'
    mix_bytes = (8 if sgd.emit == "step" else 12) * n * P
    tflops = flops / (grad_ms / 1e3) / 1e12
    gbs = mix_bytes / (mix_ms / 1e3) / 1e9
    if rank != 0:
        return
    # HBM bytes per launch from the committed PMC passes of this workload (profiles/r14/c3: the
    # final round-6 build; the local-step emission's from r10), and the kernel's rocprofv3 average over
    # the same command's timed graph steps
    c3_path = (os.path.join(ROOT, "profiles", "r14", "c3", "summary.json") if sgd.emit == "grad"
               else os.path.join(ROOT, "profiles", "r10", "c3_step", "summary.json"))
    if not os.path.exists(c3_path) and sgd.emit == "grad":
        c3_path = os.path.join(ROOT, "profiles", "r10", "c3", "summary.json")
    prof_us = None
    try:
        with open(c3_path) as f:
            summ = json.load(f)
        if ann.path == "fused":   # the timed graph steps' launches (not the warmup / phase ones)
            prof_us = summ.get("graph_step_launches", {}).get("mlp_fused_kernel_avg_us")
    except (OSError, ValueError, KeyError):
        pass
    c3_grad_traffic, c3_src = (traffic_from_profile("mlp_fused_kernel", c3_path)
                               if ann.path == "fused" and args.c3_layout == "rows"
                               else (None, None))
    c3_mix_traffic, _ = (traffic_from_profile(
        kernel_name(eng.plan(deviation=True), True, True, eng.n), c3_path)
        if args.c3_layout == "rows" else (None, None))
    grad_roof = {"bound": "mfma", "achieved": tflops, "peak": FP32_MFMA_PEAK_TFLOPS,
                 "unit": "TFLOP/s", "frac": tflops / FP32_MFMA_PEAK_TFLOPS,
                 "traffic": c3_grad_traffic, "traffic_source": c3_src if c3_grad_traffic else None,
                 "kernel": ("mlp_fused_kernel" + (" (writes X - lr G)" if sgd.emit == "step"
                                                  else "") if ann.path == "fused" else
                            "dl_bgemm x11 + dl_xent_grad") + f" ({phase_how})",
                 "flops_per_launch": flops, "launch_ms": grad_ms,
                 "step_minus_round_ms": grad_step_ms,
                 # the same kernel under rocprofv3 (committed profile of this command): its
                 # average duration and the fraction it gives
                 "rocprof_launch_ms": prof_us / 1e3 if prof_us else None,
                 "rocprof_frac": (flops / (prof_us / 1e6) / 1e12 / FP32_MFMA_PEAK_TFLOPS
                                  if prof_us else None),
                 "rocprof_source": os.path.relpath(c3_path, ROOT) if prof_us else None,
                 "arithmetic": "fp32 GEMMs: layer 1, dW1 and the hidden forward / dZ GEMMs on the "
                               "bf16 matrix cores as exact 3-way bf16 splits (six products, "
                               "csrc/mlp_fused.hip), the hidden dW tiles and the head on the fp32 "
                               "MFMA; achieved counts the fp32 FLOPs, peak is the fp32 MFMA peak"}
    mix_roof = {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": gbs / HBM_PEAK_GBS, "traffic": c3_mix_traffic,
                "traffic_source": c3_src if c3_mix_traffic else None,
                "kernel": "mix_tile_kernel (+dev_reduce) round" + (
                    " of T = X - lr G" if sgd.emit == "step" else " fusing X - lr G") +
                    f" ({phase_how})", "bytes_per_launch": mix_bytes,
                "launch_ms": mix_ms}
    dominant = grad_roof if grad_ms >= mix_ms else mix_roof
    cpu = None
    if not args.no_cpu and world == 1:   # the CPU baseline is an N=1 figure
        v, cores, tg, tm = c3_cpu_baseline(ann, csr, lr)
        cpu = {"value": v, "unit": "steps/s", "cores": cores, "kind": "port",
               "sample": f"torch CPU autograd step of ANNModel on 16 of {n} agents (B={B}), "
                         f"scaled to {n}: {tg:.3f} s; numpy restatement of the mix + deviation "
                         f"on all {n} x {P}: {tm:.3f} s",
               **host_cpu()}
    rec = {
        "metric": "c3 MLP consensus SGD steps/sec (256 agents x ANNModel 164,560 params)",
        "value": world * args.steps / elapsed,
        "unit": "steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic MNIST-shaped batches x ~ N(0,1) [{B}x784], labels uniform in 10 "
                f"classes, one fixed batch per agent resident in HBM; random-init weights",
        "config": {"workload": "c3: ANNModel consensus SGD (batched per-agent MFMA gradients + "
                               "fused round + deviation)",
                   "agents": n, "params": P, "params_padded": P_pad, "batch": B, "lr": lr,
                   "layout": eng.layout, "tile_cols": eng.T, "gradient_path": ann.path, "emit": sgd.emit,
                   "graph": "random 4-regular",
                   "weights": f"best-constant {wconst:.6f}",
                   "launch": "hipGraph replay per step" if use_graph else "eager",
                   "parallelism": f"{world} independent replicas" if world > 1 else "single GPU"},
        "roofline": dominant,
        "phases": {"gradients": grad_roof, "round": mix_roof},
        "cpu_baseline": cpu,
        "mean_loss_first_last": [float(v.item()) for v in losses],
    }
    print(json.dumps(rec), flush=True)


def per_edge_torus(rows, cols, seed=0):
    """The c4 torus with genuinely per-edge symmetric weights (best constant x (1 +- 10 %)):
    W = I - L(w) stays doubly stochastic, but with 4096 agents the per-entry CSR (120 KiB) no
    longer fits LDS beside a column tile of every agent, so dl_mix_round takes the general
    gather path."""
    import math
    from distributed_learning_amd import graph
    n = rows * cols
    edges = graph.torus_edges(rows, cols)
    wc = 2.0 / (2.0 - 2.0 * math.cos(2 * math.pi / cols) + 8.0)
    u = np.random.default_rng(seed).random(len(edges))
    return graph.from_edge_weights(edges, list(wc * (0.9 + 0.2 * u)), list(range(n))), n


def run_gather(args, dev, rank, world):
    """c4 with per-edge weights (``per_edge_torus``): 4096 agents x 2^18 params, one fused round
    (local step + mix + deviation) per step.  The per-entry CSR does not fit LDS beside a column
    tile of every agent, so the product path is the register-CSR tile kernel (plan path 4,
    column-tiled layout, fused deviation) -- ``value`` and ``roofline``.  The general gather
    kernel (path 2: neighbour rows from L2/MALL, two-pass deviation) is timed on the same graph
    as ``gather`` (forced).  N>1: replicas.

    ``--workload c4-ba``: the same on an IRREGULAR graph of the same size -- Barabasi-Albert
    (m = 2, seed 1) with Metropolis weights, the reference-run fixture B's construction at 4096
    agents (rows of 3 to 172 entries, 20,472 entries): plan path 5, each row's first 3 entries in
    registers and the other 8,184 in LDS behind the tile as 8-byte {weight, row} pairs, rows
    in the engine's row-length order (``--order agents`` keeps agent order)."""
    from distributed_learning_amd import engine, graph
    if args.workload == "c4-ba":
        if args.irregular == "deg":
            csr = graph.random_irregular_metropolis(4096, 2, 6, 1)
        else:
            csr = graph.barabasi_albert_metropolis(4096, 2 if args.irregular == "ba2" else 1, 1)
        n = csr.n_rows
        gname = ({"ba2": "c4-ba: Barabasi-Albert m=2 (seed 1)", "ba1": "c4-ba: Barabasi-Albert "
                  "m=1 (seed 1)", "deg": "c4-ba --irregular deg: ring + random degree 2..6"}
                 [args.irregular] + ", Metropolis weights, 4096 agents, fused local step + mix "
                 "+ deviation")
        kdesc = "mix_tile_kernel register head + LDS tail (+dev_reduce), HIP-event time"
        metric = "consensus rounds/sec, 4096 agents x 2^18 fp32 params, irregular graph"
        # the committed profile is of the Barabasi-Albert m = 2 graph only
        prof_dir = os.path.join(ROOT, "profiles", "r12", "c4ba") if args.irregular == "ba2" else None
    else:
        csr, n = per_edge_torus(64, 64)
        gname = ("c4-gather: 64x64 torus, per-edge weights (best constant x U[0.9, 1.1]), fused "
                 "local step + mix + deviation")
        kdesc = "mix_tile_kernel register-CSR (+dev_reduce), HIP-event time"
        metric = "consensus rounds/sec, 4096 agents x 2^18 fp32 params, per-edge weights"
        # the path-4 instance of this graph, profiled at the round-5 head (traffic null until
        # that summary exists: the r07 per-edge profile was of an older kernel)
        prof_dir = os.path.join(ROOT, "profiles", "r12", "c4gather")
    P, lr = 1 << 18, 1e-3
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    stream = torch.cuda.current_stream(dev)

    def timed(round_fn):
        sp = SpanEvents(args.steps, stream)

        def step(i):
            if i is not None:
                sp.before(i)
            round_fn()
            if i is not None:
                sp.after(i)
        elapsed = timed_loop(step, args, world, dev)
        return elapsed, sp.ms()

    # product path: register-CSR tile kernel, tiled layout, fused deviation
    eng = engine.GossipEngine(csr, P, device=dev, X=torch.randn(n, P, device=dev, generator=gen),
                              order="auto" if args.order == "auto" else None)
    G = eng.layout_like(torch.randn(n, P, device=dev, generator=gen))
    plan = eng.plan(deviation=True)
    plan["hub_rows"] = int(eng.W.hub_rows)       # rows folded by four column lanes (path 5)
    kname = kernel_name(plan, True, True, n)     # the instance this plan launches
    elapsed, launch_ms = timed(lambda: eng.round(G=G, lr=lr, deviation=True))
    del eng, G
    torch.cuda.empty_cache()
    # the general gather kernel on the same graph (row-major operands, forced)
    os.environ["DLAMD_FORCE_GATHER"] = "1"
    W = engine.DeviceCsr(csr, dev)
    X = engine.staggered_zeros((n, P), 0, dev).normal_(generator=gen)
    Gr = engine.staggered_zeros((n, P), 1, dev).normal_(generator=gen)
    Y = engine.staggered_zeros((n, P), 2, dev)
    dsq, dmax = torch.empty(n, device=dev), torch.empty(1, device=dev)
    ws = engine.Workspace(dev)
    gplan = engine.plan_shape(W, P, deviation=True)
    g_round = timed(lambda: engine.mix_round(W, X, Y, G=Gr, lr=lr, dev_sq=dsq, dev_max=dmax,
                                             workspace=ws))
    g_mix = timed(lambda: engine.mix_round(W, X, Y, G=Gr, lr=lr, workspace=ws))
    del os.environ["DLAMD_FORCE_GATHER"]
    bytes_per_round = 12 * n * P
    prof = os.path.join(prof_dir, "summary.json") if prof_dir else None
    traffic, src = traffic_from_profile(kname, prof) if prof else (None, None)
    g_traffic, g_src = traffic_from_profile("mix_gather_kernel", prof) if prof else (None, None)
    achieved = bytes_per_round / (launch_ms / 1e3) / 1e9
    g_achieved = bytes_per_round / (g_mix[1] / 1e3) / 1e9
    cpu = None
    if rank == 0 and not args.no_cpu and world == 1:   # the CPU baseline is an N=1 figure
        cpu = cpu_record(csr, n, P, sample_cols(args, n), lr, "_get_deviation_dict")
    if rank == 0:
        print(json.dumps({
            "metric": metric,
            "value": world * args.steps / elapsed, "unit": "rounds/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic X, G ~ N(0,1) resident in HBM",
            "config": {"workload": gname, "agents": n, "params": P, "nnz": csr.nnz,
                       "max_row_nnz": int(np.diff(csr.rowptr).max()), "plan": plan,
                       "parallelism": f"{world} independent replicas" if world > 1
                       else "single GPU"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": src,
                         "kernel": kdesc, "kernel_instance": kname,
                         "bytes_per_launch": bytes_per_round, "launch_ms": launch_ms},
            "gather": {"plan": gplan, "rounds_per_s_with_deviation": 1e3 / g_round[1],
                       "round_ms_with_deviation": g_round[1], "mix_launch_ms": g_mix[1],
                       "achieved": g_achieved, "frac": g_achieved / HBM_PEAK_GBS,
                       "traffic": g_traffic, "traffic_source": g_src,
                       "read_amplification": (g_traffic / bytes_per_round) if g_traffic else None,
                       "grid_order": os.environ.get("DLAMD_GATHER_ORDER", "agents")},
            "cpu_baseline": cpu,
        }), flush=True)


def _halo_schemes(args, dev, rank, world, csr, parts, P, lr, gen):
    """The agent-partitioned round on this rank (HaloShard over RCCL, strong scaling), the
    deviation lagged one round inside the round's own kernel (no extra HBM pass; one all-reduce
    of n_params column sums + one of the max).  Times each overlap scheme of --halo-overlap
    ("both" by default): "chunks" -- the boundary rows of each column chunk exchanged with RCCL
    send/recv while the previous chunk is mixed; "split" -- one exchange per round in flight
    while the interior rows mix, the boundary rows after it lands.  Returns the faster scheme's
    (elapsed, launch_ms, plan) and every scheme's figures."""
    from distributed_learning_amd import engine, sharding
    stream = torch.cuda.current_stream(dev)
    n = csr.n_rows
    G = None
    schemes = {}
    # "whole": one exchange, then one launch (no overlap, no per-chunk launches); "chunks":
    # --halo-chunks column chunks, the exchange of one overlapping the mix of the previous;
    # "split": the interior rows mix while the one exchange is in flight
    names = ["whole", "chunks", "split"] if args.halo_overlap == "both" else [args.halo_overlap]
    for name in names:
        # boundary-last row order for every scheme (the pack reads one contiguous run of rows)
        rp = sharding.split_halo_plans(csr, parts)[rank]
        shard = sharding.HaloShard(rp, P, dev, sharding.dist_transport(),
                                   chunk_cols=P // int(str(args.halo_chunks).split(",")[0])
                                   if name == "chunks" else None,
                                   n_agents_total=n, overlap="split" if name == "split" else
                                   "chunks")
        shard.X.normal_(generator=gen)
        if G is None:   # synthetic gradient rows, shared by both schemes (same shape and layout)
            G = engine.staggered_zeros(shard._shape(rp.n_local), 2, dev).normal_(generator=gen)
        sp = SpanEvents(args.steps, stream)

        def step(i, shard=shard, sp=sp):
            if i is not None:
                sp.before(i)
            shard.round(G=G, lr=lr, deviation=True)   # lagged deviation, in the round
            if i is not None:
                sp.after(i)
        el = timed_loop(step, args, world, dev)
        lm = max_over_ranks(sp.ms(), world, dev)
        extra = 8 * (rp.n_local - rp.n_deep) * P if name == "split" else 0
        schemes[name] = {"rounds_per_s": args.steps / el, "elapsed_s": el, "launch_ms": lm,
                         "layout": shard.layout, "tile_cols": shard.T,
                         "n_local": rp.n_local, "n_halo": rp.n_halo,
                         "n_interior": rp.n_interior if name == "split" else None,
                         "n_deep": rp.n_deep if name == "split" else None,
                         "reread_bytes_per_round": extra,
                         "halo_rows_per_peer": {int(q): len(ids) for q, ids in
                                                sorted(rp.halo_from.items())}}
        del shard
        torch.cuda.empty_cache()
    best = max(schemes, key=lambda k: schemes[k]["rounds_per_s"])
    plan = {"path": "halo", "overlap": best, "layout": schemes[best]["layout"],
            "tile_cols": schemes[best]["tile_cols"], "n_local": schemes[best]["n_local"],
            "n_halo": schemes[best]["n_halo"],
            "peers": sorted(schemes[best]["halo_rows_per_peer"])}
    return schemes[best]["elapsed_s"], schemes[best]["launch_ms"], plan, schemes


def _halo_xgmi(schemes, best, P, launch_ms):
    """xGMI figures of rank 0: halo bytes received per round and the busiest link's rate (one
    xGMI link per peer on the fully connected 8-GPU node) over the round time."""
    per_peer = schemes[best]["halo_rows_per_peer"]
    hb = sum(per_peer.values()) * P * 4
    link = max(per_peer.values()) * P * 4 if per_peer else 0
    out = {"halo_bytes_per_round": hb, "peers": len(per_peer),
           "busiest_link_bytes_per_round": link,
           "achieved_GBs": hb / (launch_ms / 1e3) / 1e9,
           "busiest_link_GBs": link / (launch_ms / 1e3) / 1e9,
           "peak_GBs_per_link": XGMI_LINK_GBS,
           "frac": link / (launch_ms / 1e3) / 1e9 / XGMI_LINK_GBS,
           "note": "received halo bytes over the rank's round time (HIP events); frac = the "
                   "busiest link's rate / one link's peak"}
    for v in schemes.values():
        lm = v["launch_ms"]
        v["hbm_frac"] = 12 * v["n_local"] * P / (lm / 1e3) / 1e9 / HBM_PEAK_GBS
        v["xgmi_frac"] = max(v["halo_rows_per_peer"].values()) * P * 4 / (lm / 1e3) / 1e9 / \
            XGMI_LINK_GBS if v["halo_rows_per_peer"] else 0.0
    return out


def _single_gpu_round(args, dev, csr, P, lr, gen):
    from distributed_learning_amd import engine
    stream = torch.cuda.current_stream(dev)
    n = csr.n_rows
    sp = SpanEvents(args.steps, stream)
    X = torch.randn(n, P, device=dev, generator=gen)
    eng = engine.GossipEngine(csr, P, device=dev, X=X)
    G = eng.layout_like(torch.randn(n, P, device=dev, generator=gen))
    del X
    plan = eng.plan(deviation=True)

    def step(i):
        if i is not None:
            sp.before(i)
        eng.round(G=G, lr=lr, deviation=True)
        if i is not None:
            sp.after(i)
    elapsed = timed_loop(step, args, 1, dev)
    return elapsed, sp.ms(), plan


def run_c4(args, dev, rank, world):
    """Config c4: 64x64 periodic torus, 4096 agents x 2^18 params, uniform best-constant weight
    2/(lambda_2 + 8).  N=1: the whole torus resident in the tiled layout, one fused round
    (local step + mix + deviation) per step.  N>1: 2-D torus blocks per rank (_halo_schemes:
    both overlap schemes timed, ``value`` the faster one's rate, both in the line)."""
    import math
    from distributed_learning_amd import graph, sharding
    rows = cols = 64
    n, P, lr = rows * cols, 1 << 18, 1e-3
    edges = graph.torus_edges(rows, cols)
    wconst = 2.0 / (2.0 - 2.0 * math.cos(2 * math.pi / cols) + 8.0)
    csr = graph.from_edge_weights(edges, [wconst] * len(edges), list(range(n)))
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    schemes = {}
    if world == 1:
        elapsed, launch_ms, plan = _single_gpu_round(args, dev, csr, P, lr, gen)
        bytes_per_round, halo_rows = 12 * n * P, 0
    else:
        parts = sharding.torus_block_partition(rows, cols, world)
        elapsed, launch_ms, plan, schemes = _halo_schemes(args, dev, rank, world, csr, parts, P,
                                                          lr, gen)
        bytes_per_round, halo_rows = 12 * plan["n_local"] * P, plan["n_halo"]
    if rank != 0:
        return
    achieved = bytes_per_round / (launch_ms / 1e3) / 1e9
    # single GPU: HBM bytes per launch from the committed PMC passes of this kernel instance
    # (profiles/r13/c4)
    c4_traffic, c4_src = (traffic_from_profile(
        kernel_name(plan, True, True, n), os.path.join(ROOT, "profiles", "r13", "c4",
                                                       "summary.json"))
        if world == 1 else (None, None))
    xgmi = _halo_xgmi(schemes, plan["overlap"], P, launch_ms) if world > 1 else None
    cpu = None
    if not args.no_cpu and world == 1:   # the CPU baseline is an N=1 figure
        cpu = cpu_record(csr, n, P, sample_cols(args, n), lr, "_get_deviation_dict")
    rec = {
        "metric": "c4 torus consensus rounds/sec (4096 agents x 2^18 fp32 params)",
        "value": args.steps / elapsed,
        "unit": "rounds/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (X, G ~ N(0,1) resident in HBM)",
        "config": {"workload": "c4: 64x64 torus, fused local step + mix + deviation",
                   "agents": n, "params": P, "weights": f"best-constant {wconst:.6f}",
                   "parallelism": f"2-D torus blocks x{world}, "
                                  f"{'RCCL' if args.dist_backend == 'nccl' else args.dist_backend}"
                                  f" halo exchange" if world > 1 else "single GPU", "plan": plan,
                   "deviation": "fused exact" if world == 1 else
                                "lagged one round, inside the round kernel (dlamd.h mean_prev)",
                   "halo_rows_rank0": halo_rows,
                   "halo_bytes_per_round_rank0": halo_rows * P * 4},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": c4_traffic,
                     "traffic_source": c4_src,
                     "kernel": "per-round HIP-event time (rank 0 local work)",
                     "bytes_per_launch": bytes_per_round, "launch_ms": launch_ms},
        "xgmi": xgmi,
        "dist": getattr(args, "dist_info", None),
        "overlap_schemes": schemes or None,
        "cpu_baseline": cpu,
    }
    print(json.dumps(rec), flush=True)


def c4_torus():
    import math
    from distributed_learning_amd import graph
    rows = cols = 64
    n = rows * cols
    wconst = 2.0 / (2.0 - 2.0 * math.cos(2 * math.pi / cols) + 8.0)
    csr = graph.from_edge_weights(graph.torus_edges(rows, cols), [wconst] * (2 * n),
                                  list(range(n)))
    return csr, rows, cols, wconst


def run_c4rank(args, dev, rank, world):
    """One rank of config c4's N-GPU agent partition, alone on one GPU (``--rank-of N``, default
    8): rank 0's 2-D torus block of the 64 x 64 torus x 2^18 params (N = 8: 32 x 16 = 512 local
    rows + 96 halo rows from 3 peers), column-tiled X / Y / G and per-peer tiled halo blocks
    resident in HBM, the halo buffers filled once and no interconnect in the timed region
    (``sharding.ResidentHaloTransport``).  This is the per-rank HBM work the 8-GPU round runs;
    xGMI is then the only thing the real run adds.  Each overlap scheme's whole round (pack the
    boundary rows for every peer + the mix launch(es) + the lagged deviation's bookkeeping) is
    timed, and the dominant kernel -- the halo-round mix_tile_kernel of the whole-round scheme
    (HALO = 2, LAG) -- on its own with HIP events: its algorithmic bytes per launch are
    4 B x P x (2 n_local read x and g + n_halo halo rows read + n_local written) + 8 P
    (mean_prev read, this rank's column sums written).  N>1 GPUs: independent replicas."""
    from distributed_learning_amd import engine, sharding
    csr, rows, cols, wconst = c4_torus()
    n, P, lr = csr.n_rows, 1 << 18, 1e-3
    parts = sharding.torus_block_partition(rows, cols, args.rank_of)
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    stream = torch.cuda.current_stream(dev)
    schemes = {}
    counts = [int(k) for k in str(args.halo_chunks).split(",")]
    names = {"whole": ("chunks", None)}
    for k in counts:
        names["chunks" if len(counts) == 1 else f"chunks{k}"] = ("chunks", P // k)
    names["split"] = ("split", None)
    G = kern = None
    for name, (overlap, chunk) in names.items():
        # boundary-last row order for every scheme: the rows the peers read are then one
        # contiguous run of each tile block, so the pack reads whole cache lines (the torus
        # block's left / right columns are every 16th row in partition order)
        rp = sharding.split_halo_plans(csr, parts)[0]
        shard = sharding.HaloShard(rp, P, dev, sharding.ResidentHaloTransport(),
                                   chunk_cols=chunk, n_agents_total=n, overlap=overlap,
                                   tile_cols=args.halo_tile_cols or None)
        shard.X.normal_(generator=gen)
        if G is None:   # synthetic gradient rows, shared by every scheme (same shape and layout)
            G = engine.staggered_zeros(shard._shape(rp.n_local), 2, dev).normal_(generator=gen)
        for c0, c1 in (shard.chunks() if overlap == "chunks" else [(0, P)]):
            for slot in (0, 1):
                _, halo, _ = shard._buffers(slot, c1 - c0)
                halo.normal_(generator=gen)     # the resident halo (an exchange's payload)
        sp = SpanEvents(args.steps, stream)

        def step(i, shard=shard, sp=sp):
            if i is not None:
                sp.before(i)
            shard.round(G=G, lr=lr, deviation=True)
            if i is not None:
                sp.after(i)
        el = timed_loop(step, args, 1, dev)
        lm = sp.ms()
        schemes[name] = {"overlap": overlap, "chunk_cols": shard.chunk, "rounds_per_s":
                         args.steps / el, "elapsed_s": el, "round_ms": lm,
                         "layout": shard.layout, "tile_cols": shard.T,
                         "n_local": rp.n_local, "n_halo": rp.n_halo,
                         "halo_blocks": shard.halo_blocks,
                         "n_interior": rp.n_interior if overlap == "split" else None,
                         "n_deep": rp.n_deep if overlap == "split" else None}
        if name == "whole":   # the dominant kernel alone: the halo-round mix launch + its pack
            _, halo, _ = shard._buffers(0, P)
            colsum = torch.empty(P, device=dev)
            dsq = torch.empty(rp.n_local, device=dev)
            mean_prev = torch.zeros(P, device=dev)
            kev, pev = event_pairs(args.steps, 2), event_pairs(args.steps, 2)
            for i in range(-args.warmup, args.steps):
                if i >= 0:
                    pev[i][0].record(stream)
                shard.pack(0, 0, P, G, lr)
                if i >= 0:
                    pev[i][1].record(stream)
                    kev[i][0].record(stream)
                shard.mix_chunk(0, P, halo, G, lr, (mean_prev, colsum, dsq))
                if i >= 0:
                    kev[i][1].record(stream)
            torch.cuda.synchronize()
            plan = engine.plan_shape(shard.W, P, deviation=True, tile_cols=shard.T)
            kb = 4 * P * (3 * rp.n_local + rp.n_halo) + 8 * P
            pb = 12 * P * sum(len(r) for r in rp.send_to.values())
            kern = {"mix_ms": float(np.mean([a.elapsed_time(b) for a, b in kev])),
                    "pack_ms": float(np.mean([a.elapsed_time(b) for a, b in pev])),
                    "mix_bytes": kb, "pack_bytes": pb, "plan": plan,
                    "kernel_instance": kernel_name(plan, True, False, rp.n_local + rp.n_halo,
                                                   halo=2, lag=True)}
        del shard
        torch.cuda.empty_cache()
    if rank != 0:
        return
    best = max(schemes, key=lambda k: schemes[k]["rounds_per_s"])
    for v in schemes.values():
        v["round_hbm_bytes"] = kern["mix_bytes"] + kern["pack_bytes"]
        v["round_hbm_frac"] = v["round_hbm_bytes"] / (v["round_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS
    achieved = kern["mix_bytes"] / (kern["mix_ms"] / 1e3) / 1e9
    traffic, src = traffic_from_profile(kern["kernel_instance"], os.path.join(
        ROOT, "profiles", "r13", "c4rank", "summary.json"), bytes_hint=kern["mix_bytes"])
    cpu = None
    if not args.no_cpu and world == 1:   # this rank's round on one host core
        rp = sharding.split_halo_plans(csr, parts)[0]
        cpu = cpu_record(rp.csr, rp.n_local, P, sample_cols(args, rp.n_local + rp.n_halo), lr,
                         "the lagged deviation (||x_a - mean_prev||, column sums)",
                         n_halo=rp.n_halo, lagged=True)
    rec = {
        "metric": f"c4 per-rank halo round, one rank of {args.rank_of} alone (64x64 torus, "
                  f"4096 agents x 2^18 fp32 params)",
        "value": schemes[best]["rounds_per_s"], "unit": "rounds/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": schemes[best]["elapsed_s"] / args.steps * 1e3,
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (X, G, halo ~ N(0,1) resident in HBM)",
        "config": {"workload": f"c4-rank: rank 0 of a {args.rank_of}-way 2-D torus block "
                               "partition, halo resident (no transport), fused local step + mix "
                               "+ lagged deviation", "agents_total": n, "params": P,
                   "weights": f"best-constant {wconst:.6f}", "rank_of": args.rank_of,
                   "parallelism": f"{world} independent replicas" if world > 1 else "single GPU",
                   "best_scheme": best},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": src,
                     "kernel": "halo-round mix_tile_kernel (column-tiled halo blocks, lagged "
                               "deviation), HIP events per launch",
                     "kernel_instance": kern["kernel_instance"],
                     "bytes_per_launch": kern["mix_bytes"], "launch_ms": kern["mix_ms"]},
        "pack": {"kernel": "step_rows_tiled_kernel x peers", "bytes": kern["pack_bytes"],
                 "ms": kern["pack_ms"],
                 "frac": kern["pack_bytes"] / (kern["pack_ms"] / 1e3) / 1e9 / HBM_PEAK_GBS},
        "plan": kern["plan"],
        "schemes": schemes,
        "cpu_baseline": cpu,
    }
    print(json.dumps(rec), flush=True)


def partition_report(csr, P, worlds=(2, 4, 8)):
    """Host-side partition of a graph for each GPU count: sharding.graph_partition (BFS growth +
    Kernighan-Lin refinement) against contiguous blocks -- cut edges, halo rows and halo bytes
    per round of every rank, peers, busiest-link bytes."""
    from distributed_learning_amd import sharding
    rows = np.repeat(np.arange(csr.n_rows), np.diff(csr.rowptr))
    out = {}
    for world in worlds:
        rec = {}
        for name, parts in (("graph_partition", sharding.graph_partition(csr, world)),
                            ("contiguous", sharding.contiguous_partition(csr.n_rows, world))):
            owner = np.empty(csr.n_rows, np.int64)
            for r, p in enumerate(parts):
                owner[p] = r
            keep = csr.col != rows
            cut = int(np.sum(owner[rows[keep]] != owner[csr.col[keep]]) // 2)
            plans = sharding.halo_plans(csr, parts)
            halo = [pl.n_halo for pl in plans]
            link = [max((len(ids) for ids in pl.halo_from.values()), default=0) for pl in plans]
            rec[name] = {"cut_edges": cut, "halo_rows_per_rank": halo,
                         "halo_bytes_per_round_max": max(halo) * P * 4,
                         "busiest_link_bytes_per_round": max(link) * P * 4,
                         "peers_max": max(len(pl.halo_from) for pl in plans)}
        out[str(world)] = rec
    return out


def run_c2halo(args, dev, rank, world):
    """The c2 graph agent-partitioned (a general partitioner for random graphs, halo
    bytes per GPU): networkx random_regular_graph(4, 1024, seed=0), best-constant weights, 2^20
    params per agent, the fused local step + mix + lagged deviation per round.  N=1: the single
    -device round and the host-side partition report for 2/4/8 GPUs.  N>1: graph_partition (BFS
    + Kernighan-Lin) over the ranks, both halo overlap schemes timed (_halo_schemes); strong
    scaling.  Random 4-regular graphs cut badly (most boundary agents read several remote rows),
    so this path is expected to be xGMI-bound -- the column stripes of the headline are the
    c2 decomposition; this line measures the general agent partition on the same graph."""
    from distributed_learning_amd import sharding
    n, P, lr = args.agents, args.params, 1e-3
    csr, wconst = build_graph(n)
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    schemes = {}
    report = partition_report(csr, P) if rank == 0 else None
    if world == 1:
        elapsed, launch_ms, plan = _single_gpu_round(args, dev, csr, P, lr, gen)
        bytes_per_round, halo_rows = 12 * n * P, 0
    else:
        parts = sharding.graph_partition(csr, world)
        elapsed, launch_ms, plan, schemes = _halo_schemes(args, dev, rank, world, csr, parts, P,
                                                          lr, gen)
        bytes_per_round, halo_rows = 12 * plan["n_local"] * P, plan["n_halo"]
    if rank != 0:
        return
    achieved = bytes_per_round / (launch_ms / 1e3) / 1e9
    cpu = None
    if not args.no_cpu and world == 1:   # the CPU baseline is an N=1 figure
        cpu = cpu_record(csr, n, P, sample_cols(args, n), lr, "_get_deviation_dict")
    rec = {
        "metric": "c2 graph agent-partitioned consensus rounds/sec (1024 agents x 2^20 fp32 "
                  "params, random 4-regular, halo exchange)",
        "value": args.steps / elapsed,
        "unit": "rounds/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (X, G ~ N(0,1) resident in HBM)",
        "config": {"workload": "c2-halo: c2 graph agent-partitioned, fused local step + mix + "
                               "deviation",
                   "agents": n, "params": P, "weights": f"best-constant {wconst:.6f}",
                   "partitioner": "sharding.graph_partition (BFS growth + Kernighan-Lin swaps)",
                   "parallelism": f"agent partition x{world}, "
                                  f"{'RCCL' if args.dist_backend == 'nccl' else args.dist_backend}"
                                  f" halo exchange" if world > 1 else "single GPU", "plan": plan,
                   "halo_rows_rank0": halo_rows},
        "partition_report": report,
        "roofline": {"bound": "hbm" if world == 1 else "xgmi", "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": None, "kernel": "per-round HIP-event time (rank 0 local work)",
                     "bytes_per_launch": bytes_per_round, "launch_ms": launch_ms},
        "xgmi": _halo_xgmi(schemes, plan["overlap"], P, launch_ms) if world > 1 else None,
        "dist": getattr(args, "dist_info", None),
        "overlap_schemes": schemes or None,
        "cpu_baseline": cpu,
    }
    print(json.dumps(rec), flush=True)


def c5_cpu_baseline(wl, csr, n_agents_sample=2):
    """The reference's CPU path for one c5 step: per agent a torch CPU forward/backward of
    Wide_ResNet on its batch and optim.SGD.step -- timed on a sample of agents and scaled --
    plus the numpy restatement of Mixer._mix_params_once + _get_deviation_dict on all agents."""
    from oracle import mixer_ref as M
    from distributed_learning_amd.networks.wide_resnet import Wide_ResNet
    torch.manual_seed(0)
    model = Wide_ResNet(*wl.arch)
    x = torch.randn(wl.B, 3, 32, 32)
    y = torch.randint(0, wl.arch[3], (wl.B,))
    opt = torch.optim.SGD(model.parameters(), lr=wl.lr, momentum=wl.momentum,
                          weight_decay=wl.wd)

    def agent_step():
        opt.zero_grad()
        torch.nn.functional.cross_entropy(model(x), y).backward()
        opt.step()
    agent_step()
    t0 = time.perf_counter()
    for _ in range(n_agents_sample):
        agent_step()
    t_grad = (time.perf_counter() - t0) / n_agents_sample * wl.N
    X = np.random.default_rng(0).standard_normal((wl.N, wl.P), dtype=np.float32)
    t0 = time.perf_counter()
    Y = M.mix_once(X, csr.rowptr, csr.col, csr.w)
    M.deviation(Y)
    t_mix = time.perf_counter() - t0
    return 1.0 / (t_grad + t_mix), torch.get_num_threads(), t_grad, t_mix


def run_c5(args, dev, rank, world):
    """Config c5: WRN-16-4 consensus SGD.  One step = every agent's forward + cross-entropy +
    backward on its own B-image batch (MIOpen fp32 convs, gradients accumulate straight into G's
    rows), the SGD-momentum local step (dl_sgd_step) and the fused mix + deviation round over a
    random 4-regular graph of 64 agents.  N>1: one independent 64-agent system per GPU."""
    from distributed_learning_amd.workloads import WRNConsensusSGD
    n, B = 64, args.batch
    csr, wconst = build_graph(n)
    torch.backends.cudnn.benchmark = args.cudnn_benchmark
    t0 = time.perf_counter()
    wl = WRNConsensusSGD(csr, B, device=dev, seed=1000 * rank, streams=args.streams)
    stream = torch.cuda.current_stream(dev)
    wl.step()                          # MIOpen finds every conv solution here
    torch.cuda.synchronize()
    log(f"c5: setup + first step {time.perf_counter() - t0:.1f} s")
    for _ in range(max(args.warmup, 1)):
        wl.step()
    n_ev = min(args.steps, 5)
    evs = event_pairs(n_ev, 3)
    for i in range(n_ev):
        evs[i][0].record(stream)
        wl._local_grads()
        evs[i][1].record(stream)
        wl._round(first=False)
        evs[i][2].record(stream)
        wl.steps_done += 1
    torch.cuda.synchronize()
    grad_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in evs]))
    mix_ms = float(np.mean([b.elapsed_time(c) for _, b, c in evs]))
    loss0 = float(wl.loss.mean().item())
    use_graph = not args.no_graph
    if use_graph:
        wl.capture()

    def step(i):
        if use_graph:
            wl.replay(1)
        else:
            wl.step()

    elapsed = timed_loop(step, args, world, dev)
    loss1 = float(wl.loss.mean().item())
    grad_ms = max_over_ranks(grad_ms, world, dev)
    mix_ms = max_over_ranks(mix_ms, world, dev)
    if rank != 0:
        return
    flops = wl.flops_per_step()
    ms_step = elapsed / args.steps * 1e3
    tflops = flops / (ms_step / 1e3) / 1e12
    mix_bytes = 28 * n * wl.P    # sgd step: read x, g, buf, write buf, s; round: read s, write x
    gbs = mix_bytes / (mix_ms / 1e3) / 1e9
    grad_roof = {"bound": "mfma", "achieved": tflops, "peak": FP32_MFMA_PEAK_TFLOPS,
                 "unit": "TFLOP/s", "frac": tflops / FP32_MFMA_PEAK_TFLOPS, "traffic": None,
                 "kernel": "MIOpen fp32 convs (per-agent forward + backward), whole step time",
                 "flops_per_launch": flops, "launch_ms": ms_step,
                 "eager_gradient_phase_ms": grad_ms}
    mix_roof = {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": gbs / HBM_PEAK_GBS, "traffic": None,
                "kernel": "sgd_step_kernel + mix_tile_kernel (+dev_reduce)",
                "bytes_per_launch": mix_bytes, "launch_ms": mix_ms}
    cpu = None
    if not args.no_cpu and world == 1:   # the CPU baseline is an N=1 figure
        v, cores, tg, tm = c5_cpu_baseline(wl, csr)
        cpu = {"value": v, "unit": "steps/s", "cores": cores, "kind": "port",
               "sample": f"torch CPU forward/backward + optim.SGD step of Wide_ResNet(16, 4) on 2 "
                         f"of {n} agents (B={B}), scaled to {n}: {tg:.2f} s; numpy restatement "
                         f"of the mix + deviation on all {n} x {wl.P}: {tm:.3f} s",
               **host_cpu()}
    rec = {
        "metric": "c5 WRN-16-4 consensus SGD steps/sec (64 agents x 2,751,146 params)",
        "value": world * args.steps / elapsed,
        "unit": "steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic CIFAR-10-shaped batches x ~ N(0,1) [{B}x3x32x32], labels uniform in "
                f"10 classes, one fixed batch per agent resident in HBM; default torch init",
        "config": {"workload": "c5: Wide-ResNet-16-4 consensus SGD (per-agent MIOpen convs, "
                               "SGD momentum step + fused round + deviation)",
                   "agents": n, "params": wl.P, "batch": B, "lr": wl.lr,
                   "momentum": wl.momentum, "weight_decay": wl.wd,
                   "graph": "random 4-regular", "weights": f"best-constant {wconst:.6f}",
                   "streams": args.streams, "cudnn_benchmark": args.cudnn_benchmark,
                   "miopen_find_mode": os.environ.get("MIOPEN_FIND_MODE", "default"),
                   "launch": "hipGraph replay per step" if use_graph else "eager",
                   "images_per_s": world * args.steps * n * B / elapsed,
                   "parallelism": f"{world} independent replicas" if world > 1 else "single GPU"},
        "roofline": grad_roof,
        "phases": {"gradients": grad_roof, "round": mix_roof},
        "cpu_baseline": cpu,
        "mean_loss_first_last": [loss0, loss1],
    }
    print(json.dumps(rec), flush=True)


def c1_cpu_baseline(Xtr, ytr, topo, steps):
    """The reference's c1 run restated synchronously in numpy (oracle/mixer_ref.jacobi_round,
    pinned bit for bit to the reference's 4000-step asyncio run by tests/test_oracle_golden.py)."""
    from oracle import mixer_ref as M
    toks = M.asyncio_tokens(topo)
    sh, tX, ty = {}, Xtr.copy(), ytr.copy()
    for i in range(len(toks)):
        ln = len(tX) // (len(toks) - i)
        sh[toks[i]] = (tX[:ln], ty[:ln])
        tX, ty = tX[ln:], ty[ln:]

    def grad(X, y, w, tau=1e-4):
        s = 1 / (1 + np.exp(y * (X @ w)))
        return -np.array([np.dot(y * s, X[:, j]) for j in range(X.shape[1])]) / X.shape[0] \
            + tau * w
    w = {t: np.zeros(Xtr.shape[1]) for t in toks}
    t0 = time.perf_counter()
    for it in range(steps):
        for t in toks:
            w[t] = w[t] - 0.1 * np.power(it + 1, -0.5) * grad(*sh[t], w[t])
        w, _ = M.jacobi_round(topo, w, {t: sh[t][0].shape[0] for t in toks}, 10)
    return steps / (time.perf_counter() - t0)


def run_c1(args, dev, rank, world):
    """Config c1: the Titanic consensus-GD notebook run (ring of 8 agents, fp64 logistic
    regression on the preprocessed data committed in tests/golden/titanic.npz).  Timed: all
    --steps GD iterations of every agent, each with its consensus round, in ONE dl_consensus_gd
    launch (workloads.ConsensusGDRun; shards, adjacency and step sizes resident beforehand).
    Also reported: the same run through the asyncio facade (host gradients, one dl_perron_round
    launch and readback per round), the drop-in API's own rate."""
    import asyncio

    from distributed_learning_amd import workloads
    d = np.load(os.path.join(ROOT, "tests", "golden", "titanic.npz"))
    nt = int(d["n_test"])
    Xtr, ytr = d["X"][nt:], d["y"][nt:]
    topo = [(i, (i + 1) % 8) for i in range(8)]
    run = workloads.ConsensusGDRun(topo, Xtr, ytr, args.steps, convergence_eps=10, device=dev)
    for _ in range(max(args.warmup, 1)):
        run.launch()
    torch.cuda.synchronize()
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run.launch()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, world, dev)
    w, ks = run.result()
    # BASELINE's wording for c1 is "ring with fast-averaging weights": the ring's FDLA optimum is
    # one weight on every edge, w* = 1/(3 - cos(2 pi/8)) (utils/fast_averaging.py), mixed as the
    # TCP agent's update.  The headline keeps the notebook's asyncio ConsensusNetwork (Perron eps
    # 0.95/max_deg, consensus_asyncio.py:78-86: the run whose output the reference recorded); the
    # FA-weight run is reported beside it.
    from distributed_learning_amd.utils.fast_averaging import find_optimal_weights
    fw, _ = find_optimal_weights(topo)
    fa = None
    if rank == 0 and np.allclose(fw, fw[0]):
        run_fa = workloads.ConsensusGDRun(topo, Xtr, ytr, args.steps, convergence_eps=10,
                                          device=dev, edge_weight=float(fw[0]))
        run_fa.launch()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        run_fa.launch()
        torch.cuda.synchronize()
        el_fa = time.perf_counter() - t2
        wfa, kfa = run_fa.result()
        fa = {"edge_weight": float(fw[0]), "value": args.steps / el_fa, "unit": "steps/s",
              "jacobi_iterations_per_round": sorted(set(int(k) for k in kfa)),
              "test_accuracy_agent0": workloads.accuracy(wfa[run_fa.tokens[0]], d["X"][:nt],
                                                         d["y"][:nt])}
    facade = None
    if rank == 0:
        # the drop-in API (the notebook's learning_instance: host LogRegTitanic gradients, await
        # run_round per iteration) under both facade schedules.  At convergence_eps 10 every
        # round is one Jacobi step in lockstep, so the two return the same bits
        # (tests/test_asyncio_gpu.py); "synchronous" is one dl_perron_round per round.
        fs = min(args.steps, 500)
        facade, outs = {}, {}
        for sched in ("synchronous", "reference"):
            asyncio.run(workloads.consensus_gd(topo, Xtr, ytr, 5, convergence_eps=10,
                                               device=dev, consensus=sched))
            t1 = time.perf_counter()
            outs[sched] = asyncio.run(workloads.consensus_gd(topo, Xtr, ytr, fs,
                                                             convergence_eps=10, device=dev,
                                                             consensus=sched))
            facade[sched] = fs / (time.perf_counter() - t1)
        facade = {"value": facade["synchronous"], "unit": "steps/s", "steps": fs,
                  "schedule": "synchronous",
                  "path": "utils.consensus_asyncio facade, schedule='synchronous': host "
                          "gradients + one dl_perron_round per round (pinned staging, one "
                          "synchronisation)",
                  "reference_schedule_value": facade["reference"],
                  "reference_schedule_path": "schedule='reference': the reference's asyncio "
                                             "message protocol replayed, every agent step on the "
                                             "device",
                  "schedules_bit_identical": all(
                      np.array_equal(outs["synchronous"][t], outs["reference"][t])
                      for t in outs["reference"])}
    if rank != 0:
        return
    acc = workloads.accuracy(w[0], d["X"][:nt], d["y"][:nt])
    cpu = None
    if not args.no_cpu and world == 1:
        cpu = {"value": c1_cpu_baseline(Xtr, ytr, topo, args.steps), "unit": "steps/s",
               "cores": 1, "kind": "port",
               "sample": f"the same {args.steps} GD iterations, synchronous numpy restatement of "
                         "the asyncio rounds (oracle/mixer_ref.jacobi_round)", **host_cpu()}
    rec = {
        "metric": "c1 Titanic consensus GD iterations/sec (8 agents, ring)",
        "value": world * args.steps / elapsed,
        "unit": "steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "Titanic train.csv preprocessed as the notebook does (tests/golden/titanic.npz)",
        "config": {"workload": "c1: ring-8 asyncio consensus GD, convergence_eps 10, step "
                               "0.1 (it+1)^-0.5, tau 1e-4",
                   "agents": 8, "params": int(Xtr.shape[1]),
                   "test_accuracy_agent0": acc,
                   "jacobi_iterations_per_round": sorted(set(int(k) for k in ks)),
                   "launch": "one dl_consensus_gd launch for all --steps iterations",
                   "parallelism": f"{world} independent replicas" if world > 1 else "single GPU"},
        "facade": facade,
        "weights": "asyncio Perron eps 0.95/max_deg = 0.475 (the notebook's ConsensusNetwork, "
                   "the reference-recorded run)",
        "fast_averaging_weights": fa,
        "roofline": {"bound": "latency", "achieved": None, "peak": None, "unit": None,
                     "frac": None, "traffic": None,
                     "kernel": "consensus_gd_kernel: one workgroup, 8 waves; per iteration a "
                               "64-lane gradient reduction per agent and barrier-separated "
                               "Jacobi sweeps over 56 fp64 values: latency-bound by design"},
        "cpu_baseline": cpu,
    }
    print(json.dumps(rec), flush=True)


def run_gossip(args, dev, rank, world):
    """c2 as pure gossip averaging: one step = Mixer.mix(times=K) with eps=None, i.e. K rounds
    X <- W X with nothing in between, run by dl_mix_rounds as ONE pass over HBM (every round on
    LDS-resident column tiles of all 1024 agents) plus the final disagreement.  Every round is
    bit-identical to the one-round kernel (tests/test_mix_rounds_gpu.py)."""
    from distributed_learning_amd import engine
    n, P, K = args.agents, args.params, args.rounds
    csr, wconst = build_graph(n, args.graph)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    order, conflicts = None, None
    if args.relabel > 0:
        from distributed_learning_amd.graph import lds_slot_order_native
        # the bank slot of a neighbour read depends on the image layout: mix_multi_kernel keeps
        # agent-major rows of T/4 chunks (lane = row * chunks + chunk), as does
        # mix_trace_rows_kernel; mix_trace_kernel (DLAMD_TRACE_PLANES=1) chunk-major planes with
        # one agent per lane (the slot order of chunks = 1)
        chunks = 1 if args.trace and os.environ.get("DLAMD_TRACE_PLANES") else engine.plan_shape(
            engine.DeviceCsr(csr, dev), P, deviation=True, tile_cols=-1)["tile_cols"] // 4
        t0 = time.perf_counter()
        order, c0, c1 = lds_slot_order_native(csr, chunks, moves=args.relabel)
        conflicts = {"before": c0, "after": c1, "search_s": time.perf_counter() - t0}
        log(f"c2-gossip: LDS slot order, bank conflicts {c0} -> {c1}")
    eng = engine.GossipEngine(csr, P, device=dev, X=torch.randn(n, P, device=dev, generator=g),
                              order=order, layout=args.layout)
    stream = torch.cuda.current_stream(dev)
    sp = SpanEvents(args.steps, stream)
    if args.trace:
        # Mixer.mix(times, eps) as the drop-in runs it for X too large for one workgroup: one
        # traced pass of K rounds + one readback of the K per-round max deviations per step
        kmax = eng.trace_max_rounds()
        if kmax < 1:
            raise SystemExit("c2-gossip --trace: the traced kernel does not fit this graph")
        K = min(K, kmax)
        plan = {"kernel": "mix_trace_wide_kernel" if n > 1024 else "mix_trace_rows_kernel",
                "max_rounds_per_pass": kmax, "layout": eng.layout}
        trace = torch.empty(K, dtype=torch.float32, device=dev)
        last = []

        def step(i):
            if i is not None:
                sp.before(i)
            eng.rounds_traced(K, trace)
            if i is not None:
                sp.after(i)
            last[:] = trace.tolist()     # the host stop test reads the K values every pass
    else:
        plan = engine.rounds_plan(eng.W, eng.X, eng.Y, deviation=True, tiled=(eng.P, eng.T))
        if plan is None:
            raise SystemExit("c2-gossip: the multi-round kernel does not fit this graph")

        def step(i):
            if i is not None:
                sp.before(i)
            eng.rounds(K, deviation=True)
            if i is not None:
                sp.after(i)

    elapsed = timed_loop(step, args, world, dev)
    launch_ms = max_over_ranks(sp.ms(), world, dev)
    if rank != 0:
        return
    cpu = None
    if not args.no_cpu and world == 1:
        # the reference's Mixer.mix(times=K), eps=None: K _mix_params_once folds (numpy
        # restatement, one host core) on all agents x a column sample, scaled to the full P
        from oracle import mixer_ref as M
        cols = min(args.cpu_cols, P)
        Xs = np.random.default_rng(0).standard_normal((n, cols), dtype=np.float32)
        M.mix_once(Xs, csr.rowptr, csr.col, csr.w)
        t0 = time.perf_counter()
        for _ in range(3):
            Xs = M.mix_once(Xs, csr.rowptr, csr.col, csr.w)
        dt = (time.perf_counter() - t0) / 3
        cpu = {"value": (cols / P) / dt, "unit": "rounds/s", "cores": 1, "kind": "port",
               "sample": f"{n} agents x {cols} of {P} columns, 3 rounds of the numpy "
                         "restatement of Mixer._mix_params_once, scaled to the full column count",
               **host_cpu()}
    nel = n * P
    hbm_bytes = 8 * nel                      # read X, write X' once per K rounds
    lds_bytes = K * nel * 4 * (5 + 1)        # per round: d + 1 = 5 neighbour reads + 1 write
    rounds_per_s = world * args.steps * K / elapsed
    rec = {
        "metric": "consensus rounds/sec, pure gossip averaging (Mixer.mix(times=K)), "
                  + (f"1024 agents x 1M fp32 params" if (n, P) == (1024, 1 << 20)
                     else f"{n} agents x {P} fp32 params"),
        "value": rounds_per_s,
        "unit": "rounds/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (X ~ N(0,1) resident in HBM; networkx random_regular_graph(4, 1024, "
                "seed=0))",
        "config": {"workload": (f"c2-gossip --trace: Mixer.mix(times, eps) passes of {K} rounds "
                                "(dl_mix_rounds_trace: one HBM pass + the per-round max "
                                "deviations, read back every pass)" if args.trace else
                                f"c2-gossip: Mixer.mix(times={K}) eps=None as one dl_mix_rounds "
                                "pass + final deviation"),
                   "agents": n, "params_per_gpu": P, "rounds_per_step": K,
                   "graph": {"rr4": "random 4-regular", "circ4": "circulant a+-1, a+-2",
                             "torus": "2-D periodic torus"}[args.graph], "weights": f"best-constant {wconst:.6f}",
                   "plan": plan, "lds_slot_order": conflicts,
                   "parallelism": f"column stripes x{world}" if world > 1 else "single GPU"},
        "roofline": {"bound": "lds", "achieved": lds_bytes / (launch_ms / 1e3) / 1e9,
                     "peak": LDS_PEAK_GBS, "unit": "GB/s",
                     "frac": lds_bytes / (launch_ms / 1e3) / 1e9 / LDS_PEAK_GBS,
                     "traffic": None,
                     "kernel": (f"{plan['kernel']} (+trace_reduce)" if args.trace else
                                "mix_multi_kernel (+dev_reduce)") + " per-step HIP-event time",
                     "bytes_per_launch": lds_bytes, "launch_ms": launch_ms,
                     "hbm_bytes_per_launch": hbm_bytes,
                     "hbm_GBs": hbm_bytes / (launch_ms / 1e3) / 1e9,
                     "round_equivalent_hbm_GBs": K * hbm_bytes / (launch_ms / 1e3) / 1e9},
        "cpu_baseline": cpu,
        "final_max_deviation": (float(last[-1]) if args.trace else float(eng.dev_max.item())),
    }
    print(json.dumps(rec), flush=True)


def halo_probe(world, backend, steps=20, warmup=3, timeout_s=240, workload="c4",
               stderr_lines=40):
    """The agent-partitioned path at this GPU count: bench --workload c4 (64 x 64 torus, 2-D
    blocks, boundary rows exchanged with RCCL send/recv over xGMI each round, overlapped with
    the mix of the previous column chunk) as a CHILD job on the same GPUs, after this job's own
    process group is gone.  It runs as a child under a time limit, so whatever it does, the c2
    line is still printed.  Returns the child's figures, or its failure with the tail of its
    stderr (``stderr_tail``)."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = {k: v for k, v in os.environ.items()
           if not k.startswith("TORCHELASTIC_") and k not in (
               "RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK",
               "GROUP_WORLD_SIZE", "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR",
               "MASTER_PORT")}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.join(ROOT, "bench.py"), "--workload", workload, "--gpus", str(world),
           "--steps", str(steps), "--warmup", str(warmup), "--dist-backend", backend]
    t0 = time.perf_counter()
    # the child's stderr goes to a file, so a failing or hung run leaves its traceback tail in
    # this line (the driver's one multi-GPU chance is otherwise undiagnosable from the record)
    import tempfile
    with tempfile.TemporaryFile("w+") as errf:
        p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=errf, env=env,
                             start_new_session=True, text=True)
        try:
            out, _ = p.communicate(timeout=timeout_s)
            status = None
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, signal.SIGKILL)
            out, _ = p.communicate()
            status = f"timeout after {timeout_s} s"
        errf.seek(0)
        err = errf.read()
    lines = [ln for ln in (out or "").splitlines() if ln.startswith("{")]
    if status is None and (p.returncode != 0 or not lines):
        status = f"exit {p.returncode}"
    if status is not None:
        errl = err.splitlines()
        tail = errl[-stderr_lines:]
        # torchrun ends with its own failure summary: keep the first rank traceback as well
        tb = next((i for i, ln in enumerate(errl) if ln.startswith("Traceback")), None)
        first_tb = "\n".join(errl[tb:tb + stderr_lines]) if tb is not None else ""
        return {"status": status, "cmd": " ".join(cmd[2:]), "wall_s": time.perf_counter() - t0,
                "stderr_first_traceback": first_tb[-6000:],
                "stderr_tail": "\n".join(tail)[-6000:],
                "stdout_tail": "\n".join((out or "").splitlines()[-5:])[-2000:]}
    r = json.loads(lines[-1])
    return {"status": "ok", "metric": r["metric"], "value": r["value"], "unit": r["unit"],
            "scaling": r["scaling"], "ms_per_step": r["ms_per_step"], "steps": r["steps"],
            "parallelism": r["config"]["parallelism"], "plan": r["config"]["plan"],
            "hbm": {k: r["roofline"][k] for k in ("achieved", "peak", "frac", "launch_ms")},
            "xgmi": r["xgmi"], "overlap_schemes": r.get("overlap_schemes"),
            "partition_report": r.get("partition_report"), "dist": r.get("dist"),
            "wall_s": time.perf_counter() - t0}


def label_decompositions(rec, world, h):
    """At N > 1 the c2 line carries two decompositions; say which is which.
    ``value`` is the column-stripe (P-split) rate: every rank mixes 2^20 columns of all 1024
    agents with no data exchange (one N-float all-reduce per round), SURVEY 8e's "upper bound"
    decomposition.  The agent partition of north_star (c) -- config c4's torus blocks with the
    RCCL halo exchange over xGMI, strong scaling -- is the child probe ``h``; its per-N figures
    are first-class fields: rounds/s, HBM and xGMI fractions, the winning overlap scheme."""
    rec["decomposition"] = "P-split upper bound"
    rec["config"]["parallelism"] = (f"column stripes x{world} (P-split upper bound, SURVEY 8e: no "
                                    f"data exchange, deviation all-reduce only)")
    ok = h.get("status") == "ok"
    rec["agent_partition"] = {
        "decomposition": "agent partition (north_star (c)): c4 64x64 torus 2-D blocks, RCCL "
                         "send/recv halo over xGMI, strong scaling",
        "status": h.get("status"),
        "rounds_per_s": h["value"] if ok else None,
        "hbm_frac": h["hbm"]["frac"] if ok else None,
        "xgmi_frac": h["xgmi"]["frac"] if ok and h.get("xgmi") else None,
        "overlap": h["plan"].get("overlap") if ok else None,
        "layout": (h["plan"].get("layout") if ok else None),
    }
    # (the flat keys of earlier rounds, kept for the driver's records)
    rec["c4_halo_rounds_per_s"] = rec["agent_partition"]["rounds_per_s"]
    rec["c4_halo_hbm_frac"] = rec["agent_partition"]["hbm_frac"]
    rec["c4_halo_xgmi_frac"] = rec["agent_partition"]["xgmi_frac"]
    rec["c4_halo_overlap"] = rec["agent_partition"]["overlap"]
    return rec


def dist_info(args, world):
    """What the process group saw (for the driver's one multi-GPU record): backend, world size,
    RCCL version, visible devices."""
    info = {"world_size_env": world, "backend": args.dist_backend if world > 1 else None,
            "visible_devices": torch.cuda.device_count()}
    if world > 1:
        import torch.distributed as dist
        info["world_size_pg"] = dist.get_world_size()
    try:
        v = torch.cuda.nccl.version()
        info["rccl_version"] = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
    except Exception as e:   # noqa: BLE001 -- diagnostics only
        info["rccl_version"] = f"unavailable ({type(e).__name__})"
    return info


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        log(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE")
    n_gpus = world
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)
    args.dist_info = dist_info(args, world)

    runners = {"c1": run_c1, "c2-gossip": run_gossip, "c2-halo": run_c2halo, "c3": run_c3,
               "c4": run_c4, "c4-rank": run_c4rank, "c4-gather": run_gather,
               "c4-ba": run_gather, "c5": run_c5}
    if args.workload in runners:
        runners[args.workload](args, dev, rank, world)
        if world > 1:
            dist.destroy_process_group()
        return

    from distributed_learning_amd import engine

    n, P = args.agents, args.params
    sgd = args.workload == "c2"
    lr = 1e-3
    if args.weights == "fdla":
        csr, finfo = build_fdla_graph(n)
        weights_desc = f"per-edge FDLA (SDP gamma {finfo['gamma']:.6f})"
    else:
        csr, wconst = build_graph(n)
        weights_desc = f"best-constant {wconst:.6f}"
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    X = torch.randn(n, P, device=dev, generator=g)
    G = torch.randn(n, P, device=dev, generator=g) if sgd else None
    eng = engine.GossipEngine(csr, P, device=dev, X=X)
    if G is not None:
        G = eng.layout_like(G)        # synthetic gradient resident in the engine's layout
    del X
    plan = eng.plan(deviation=True)

    # N > 1: every round's ||x_a - mean||^2 partials all-reduced over the column stripes (the
    # global deviation: the column mean is stripe-local).  The all-reduce of a round's copy is
    # posted asynchronously: the next round's launch does not wait for the collective (as at
    # N = 1, where the deviation stays on the device); all of them are waited for before the
    # timed region closes
    pending = []

    def reduce_dev():
        if world > 1:
            buf = eng.dev_sq.clone()     # the next round rewrites dev_sq
            pending.append((dist.all_reduce(buf, async_op=True), buf))

    def step():
        eng.round(G=G, lr=lr, deviation=True)
        reduce_dev()

    for _ in range(args.warmup):
        step()
    for w, _ in pending:
        w.wait()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    sp = SpanEvents(args.steps, stream)
    t0 = time.perf_counter()
    pending.clear()
    for i in range(args.steps):
        sp.before(i)
        eng.round(G=G, lr=lr, deviation=True)
        sp.after(i)
        reduce_dev()
    for w, _ in pending:
        w.wait()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    launch_ms = sp.ms()
    dev_sq_global = pending[-1][1] if pending else eng.dev_sq
    dev_max = float(torch.sqrt(dev_sq_global.max()).item())
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        lt = torch.tensor([launch_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(lt, op=dist.ReduceOp.MAX)
        launch_ms = float(lt.item())

    bytes_per_round = (12 if sgd else 8) * n * P          # algorithmic: read X (+G), write X'
    ms_per_step = elapsed / args.steps * 1e3
    value = n_gpus * args.steps / elapsed                 # 1024 x 2^20-equivalent rounds / s
    achieved = bytes_per_round / (launch_ms / 1e3) / 1e9  # GB/s of the fused round launch

    fdla = None
    if rank == 0 and world == 1 and sgd and args.weights == "best-constant" and \
            not args.no_fdla_probe:
        del eng, G
        torch.cuda.empty_cache()
        fdla = fdla_probe(dev, n, P, lr)
    if rank == 0:
        kname = kernel_name(plan, sgd, True, n)
        traffic, traffic_src = traffic_from_profile(kname)
        ceiling, triad, ceiling_variants = copy_ceiling(dev)
        cpu = None
        if not args.no_cpu and world == 1:   # the CPU baseline is an N=1 figure
            cb = cpu_baseline(csr, n, P, min(args.cpu_cols, P), sgd, lr)
            cpu = {"value": cb["numpy"], "unit": "rounds/s", "cores": 1, "kind": "port",
                   "sample": f"{n} agents x {min(args.cpu_cols, P)} of {P} columns, same graph; "
                             f"numpy restatement of Mixer._mix_params_once + "
                             f"_get_deviation_dict{' after x-lr*g' if sgd else ''}, 3 rounds, "
                             f"scaled to the full column count",
                   "c_port_value": cb["c"], **host_cpu()}
        rec = {
            "metric": "consensus rounds/sec + achieved HBM GB/s, 1024 agents x 1M fp32 params",
            "value": value,
            "unit": "rounds/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (X, G ~ N(0,1) resident in HBM; networkx random_regular_graph(4, "
                    "1024, seed=0))",
            "config": {"workload": "c2: pure gossip consensus round, fused local step + mix + "
                                   "deviation" if sgd else "c2-mix: mix + deviation",
                       "agents": n, "params_per_gpu": P, "graph": "random 4-regular",
                       "weights": weights_desc, "parallelism":
                           f"column stripes x{n_gpus}, deviation all-reduce" if n_gpus > 1
                           else "single GPU",
                       "plan": plan},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src, "kernel_instance": kname,
                         "kernel": "mix_tile_kernel (+dev_reduce): HIP events around the K "
                                   "timed rounds / K",
                         "bytes_per_launch": bytes_per_round, "launch_ms": launch_ms,
                         "measured_copy_ceiling_GBs": ceiling,
                         "measured_triad_ceiling_GBs": triad,
                         "frac_of_measured_triad": achieved / triad,
                         "stream_variants_GBs": ceiling_variants,
                         **rocprof_fields(kname, bytes_per_round)},
            "cpu_baseline": cpu,
            "final_max_deviation": dev_max,
            "fdla_weights": fdla,
            "dist": args.dist_info,
        }
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        if world > 1 and not args.no_halo_probe and sgd:
            del eng, G
            torch.cuda.empty_cache()
            # the general partitioner on the c2 graph itself (halo bytes per GPU)
            rec["c2_halo"] = halo_probe(world, args.dist_backend, timeout_s=180,
                                        workload="c2-halo")
            rec["c4_halo"] = h = halo_probe(world, args.dist_backend)
            label_decompositions(rec, world, h)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
