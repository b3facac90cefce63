"""Benchmark of the consensus hot path on MI355X (BASELINE.json metric).

One step = one consensus round over synthetic inputs resident in HBM: the fused local step
x <- x - lr*g, the sparse mix X <- W X over a random 4-regular graph of 1024 agents with
best-constant weights, and the per-agent disagreement ||x_a - mean|| with its max (the Mixer's
stop test).  At N GPUs every rank owns a column stripe of 2^20 parameters for all 1024 agents
(weak scaling; the mix is column-independent so the stripes need no data exchange) and the
per-agent deviation partials are all-reduced over RCCL every round, which is the round's real
exchange step.  ``value`` = rounds/s in units of the 1024 x 2^20 workload, summed over ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c2|c2-mix]
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

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--workload", default="c2", choices=["c2", "c2-mix"])
    p.add_argument("--agents", type=int, default=1024)
    p.add_argument("--params", type=int, default=1 << 20)
    p.add_argument("--cpu-cols", type=int, default=1 << 18,
                   help="columns of the bounded CPU-baseline sample (all agents)")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--dist-backend", default="nccl",
                   help="nccl (= RCCL, default) or gloo (multi-rank rehearsal on one GPU)")
    return p.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def build_graph(n):
    from distributed_learning_amd.graph import (best_constant_weight, from_edge_weights,
                                                first_appearance_vertices, random_regular_edges)
    edges = random_regular_edges(4, n, seed=0)
    verts = sorted(first_appearance_vertices(edges))
    w = best_constant_weight(edges, verts)
    return from_edge_weights(edges, [w] * len(edges), verts), w


def copy_ceiling(dev, nbytes=4 << 30, reps=10):
    """Measured HBM ceiling: float4 streaming copy (libdlamd dl_stream_copy) of a 4 GiB buffer,
    counting read + write bytes."""
    from distributed_learning_amd import _lib
    lib = _lib.load()
    a = torch.zeros(nbytes // 4, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)

    best = {}
    for variant in (0, 1, 2, 3):
        def cp():
            _lib.check(lib.dl_stream_copy(_lib.ptr(a), _lib.ptr(b), a.numel(), variant,
                                          _lib.stream_handle(dev)), "dl_stream_copy")
        cp()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(reps):
            cp()
        e.record()
        torch.cuda.synchronize()
        best[variant] = 2 * nbytes / (s.elapsed_time(e) / 1e3 / reps) / 1e9
    del a, b
    return max(best.values()), best


def kernel_name(plan, sgd, dev, n_src):
    """The mix_tile_kernel instantiation dl_mix_round launches for this plan (FAST path)."""
    c = plan["tile_cols"] // 4
    need = -(-n_src // (1024 // c))
    kv = 2 if need <= 2 else 4 if need <= 4 else 8
    b = lambda v: "true" if v else "false"  # noqa: E731
    return f"mix_tile_kernel<{c}, {kv}, {b(sgd)}, {b(dev)}, true, false, true>"


def traffic_from_profile(kname, path=os.path.join(ROOT, "profiles", "r01", "summary.json")):
    """HBM bytes per launch of this kernel from the committed rocprofv3 PMC summary
    (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction), or None if it was not profiled."""
    try:
        with open(path) as f:
            kernels = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None, None
    for name, e in kernels.items():
        if kname in name and "hbm_bytes_per_launch" in e:
            return e["hbm_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(csr, n, P, cols, sgd, lr):
    """Bounded sample of the same round on the host: the reference algorithm restated in numpy
    (Mixer._mix_params_once + _get_deviation_dict, single thread) on all agents x `cols`
    columns, scaled to the full P (columns are independent).  Also the C restatement."""
    from oracle import cref
    from oracle import mixer_ref as M
    rng = np.random.default_rng(0)
    X = rng.standard_normal((n, cols), dtype=np.float32)
    G = rng.standard_normal((n, cols), dtype=np.float32) if sgd else None

    def np_round():
        T = M.sgd_step(X, G, lr) if sgd else X
        Y = M.mix_once(T, csr.rowptr, csr.col, csr.w)
        M.deviation(Y)

    def c_round():
        Y = cref.mix_round(X, csr.rowptr, csr.col, csr.w, G=G, lr=lr)
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

    from distributed_learning_amd import engine

    n, P = args.agents, args.params
    sgd = args.workload == "c2"
    lr = 1e-3
    csr, wconst = build_graph(n)
    g = torch.Generator(device=dev).manual_seed(1000 + rank)
    X = torch.randn(n, P, device=dev, generator=g)
    G = torch.randn(n, P, device=dev, generator=g) if sgd else None
    eng = engine.GossipEngine(csr, P, device=dev, X=X)
    if G is not None:
        G = eng.layout_like(G)        # synthetic gradient resident in the engine's layout
    del X
    plan = eng.plan(deviation=True)

    def step():
        eng.round(G=G, lr=lr, deviation=True)
        if world > 1:
            dist.all_reduce(eng.dev_sq)   # global ||x_a - mean||^2 over all column stripes

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        eng.round(G=G, lr=lr, deviation=True)
        evs[i][1].record(stream)
        if world > 1:
            dist.all_reduce(eng.dev_sq)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    launch_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    dev_max = float(torch.sqrt(eng.dev_sq.max()).item())
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

    if rank == 0:
        kname = kernel_name(plan, sgd, True, n)
        traffic, traffic_src = traffic_from_profile(kname)
        ceiling, ceiling_variants = copy_ceiling(dev)
        cpu = None
        if not args.no_cpu:
            cb = cpu_baseline(csr, n, P, min(args.cpu_cols, P), sgd, lr)
            cpu = {"value": cb["numpy"], "unit": "rounds/s", "cores": 1, "kind": "port",
                   "sample": f"{n} agents x {min(args.cpu_cols, P)} of {P} columns, same graph; "
                             f"numpy restatement of Mixer._mix_params_once + "
                             f"_get_deviation_dict{' after x-lr*g' if sgd else ''}, 3 rounds, "
                             f"scaled to the full column count",
                   "c_port_value": cb["c"],
                   "host_cpu": platform.processor() or platform.machine(),
                   "host_cores": os.cpu_count()}
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
                       "weights": f"best-constant {wconst:.6f}", "parallelism":
                           f"column stripes x{n_gpus}, deviation all-reduce" if n_gpus > 1
                           else "single GPU",
                       "plan": plan},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src, "kernel_instance": kname,
                         "kernel": "mix_tile_kernel (+dev_reduce) per-round HIP-event time",
                         "bytes_per_launch": bytes_per_round, "launch_ms": launch_ms,
                         "measured_copy_ceiling_GBs": ceiling,
                         "copy_variants_GBs": ceiling_variants},
            "cpu_baseline": cpu,
            "final_max_deviation": dev_max,
        }
        print(json.dumps(rec), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
