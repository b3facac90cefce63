"""CPU checks of bench.py's contract pieces that no GPU run exercises on its own: the committed
rocprofv3 PMC summaries the bench lines cite for ``roofline.traffic`` must contain the kernel
instantiation the bench names (a template parameter added to the kernel once left the c2 line's
traffic at null), and the argument parser must accept the driver's command line."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_c2_headline_kernel_has_committed_traffic(bench):
    # c2: 1024 agents, column-tiled T = 16 (4 float4 chunks), fused local step and deviation
    name = bench.kernel_name({"tile_cols": 16, "path": 1}, sgd=True, dev=True, n_src=1024)
    traffic, src = bench.traffic_from_profile(name)
    assert traffic is not None, f"{name} not in the default PMC summary"
    # within 1 % of the algorithmic 12 * N * P bytes per round
    assert abs(traffic / (12 * 1024 * 2 ** 20) - 1) < 0.01
    assert src.startswith("profiles/")


def test_c3_kernels_have_committed_traffic(bench):
    path = os.path.join(ROOT, "profiles", "r14", "c3", "summary.json")
    for k in ("mlp_fused_kernel", "mix_tile_kernel<"):
        traffic, _ = bench.traffic_from_profile(k, path)
        assert traffic is not None and traffic > 0, k


def test_driver_command_line_parses(bench, monkeypatch):
    # the driver's N = 1 and N > 1 invocations, and the defaults
    for argv in (["bench.py"], ["bench.py", "--gpus", "8", "--steps", "20", "--warmup", "3"],
                 ["bench.py", "--workload", "c3"], ["bench.py", "--workload", "c5",
                                                    "--no-cudnn-benchmark"]):
        monkeypatch.setattr("sys.argv", argv)
        p = bench.parse()
        assert p.gpus >= 1 and p.steps >= 1 and p.warmup >= 0
    # c3's layout knobs (profiles/r14/c3_layout): rows by default, the planner's tile width unless
    # one is named
    monkeypatch.setattr("sys.argv", ["bench.py", "--workload", "c3"])
    p = bench.parse()
    assert p.c3_layout == "rows" and p.c3_tile_cols == 0 and p.c3_emit == "grad"
    monkeypatch.setattr("sys.argv", ["bench.py", "--workload", "c3", "--c3-layout", "tiled",
                                     "--c3-tile-cols", "32"])
    p = bench.parse()
    assert p.c3_layout == "tiled" and p.c3_tile_cols == 32


def test_halo_probe_failure_carries_child_stderr(bench):
    """A failing child run (here: 2 gloo ranks of bench --workload c4 on a host with no GPU, which
    die in torch.cuda.set_device) comes back with its traceback tail in the record, so a failed
    multi-GPU probe in the driver's one scaling run is diagnosable from the JSON line alone."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("needs a host without a GPU for the child to fail")
    rec = bench.halo_probe(2, "gloo", steps=1, warmup=0, timeout_s=240)
    assert rec["status"].startswith("exit"), rec
    assert "Error" in rec["stderr_tail"], rec
    # the rank's own traceback, not only torchrun's summary
    assert rec["stderr_first_traceback"].startswith("Traceback"), rec
    assert "set_device" in rec["stderr_first_traceback"] or "cuda" in \
        rec["stderr_first_traceback"].lower(), rec
    assert "bench.py" in rec["cmd"]


def test_multi_gpu_line_names_both_decompositions(bench):
    """At N > 1 the c2 line's ``value`` is the column-stripe (P-split) upper bound and the agent
    partition (the c4 RCCL halo child probe) is a first-class object: both are named."""
    rec = {"config": {"parallelism": "column stripes x8"}}
    h = {"status": "ok", "value": 321.0, "hbm": {"frac": 0.6}, "xgmi": {"frac": 0.4},
         "plan": {"overlap": "split", "layout": "tiled"}}
    bench.label_decompositions(rec, 8, h)
    assert rec["decomposition"] == "P-split upper bound"
    assert "P-split upper bound" in rec["config"]["parallelism"]
    ap = rec["agent_partition"]
    assert ap["rounds_per_s"] == 321.0 and ap["hbm_frac"] == 0.6 and ap["xgmi_frac"] == 0.4
    assert ap["overlap"] == "split" and ap["layout"] == "tiled"
    assert "agent partition" in ap["decomposition"]
    assert rec["c4_halo_rounds_per_s"] == 321.0
    # a failed child probe: the keys stay, with no figures
    rec2 = {"config": {"parallelism": ""}}
    bench.label_decompositions(rec2, 2, {"status": "exit 1"})
    assert rec2["agent_partition"]["rounds_per_s"] is None
    assert rec2["agent_partition"]["status"] == "exit 1"


def test_kernel_names_follow_the_plan(bench):
    """kernel_name builds the full instantiation rocprofv3 prints, from the plan (the
    c4-ba instance was hardcoded): path 1, path 4 (register CSR, RD 5) and path 5 (head, tail)."""
    p1 = bench.kernel_name({"path": 1, "tile_cols": 16}, True, True, 1024)
    assert p1 == "mix_tile_kernel<4, 4, true, true, true, 0, true, 0, false, 0>(dl::TileArgs)"
    p4 = bench.kernel_name({"path": 4, "tile_cols": 4, "head": 5, "tail_fmt": 0}, True, True, 4096)
    assert p4 == "mix_tile_kernel<1, 4, true, true, true, 0, true, 5, false, 0>(dl::TileArgs)"
    p5 = bench.kernel_name({"path": 5, "tile_cols": 4, "head": 2, "tail_fmt": 2}, True, True, 4096)
    assert p5 == "mix_tile_kernel<1, 4, true, true, true, 0, true, 2, false, 2>(dl::TileArgs)"
    h = bench.kernel_name({"path": 1, "tile_cols": 16}, True, False, 608, halo=2, lag=True)
    assert h == "mix_tile_kernel<4, 3, true, false, true, 2, true, 0, true, 0>(dl::TileArgs)"


def test_c4_rank_kernel_has_committed_traffic(bench):
    """The one-rank-of-8 c4 line's roofline cites the committed rocprofv3 PMC summary of its own
    kernel instance: the whole-round launches' class (the profile also holds the 8-chunk
    scheme's launches of the same instance), within 1 % of the algorithmic bytes."""
    alg = 4 * 2 ** 18 * (3 * 512 + 96) + 8 * 2 ** 18
    name = bench.kernel_name({"path": 1, "tile_cols": 16}, True, False, 608, halo=2, lag=True)
    traffic, src = bench.traffic_from_profile(
        name, os.path.join(ROOT, "profiles", "r13", "c4rank", "summary.json"), bytes_hint=alg)
    assert traffic is not None and src.startswith("profiles/")
    assert abs(traffic / alg - 1) < 0.01


def test_c4_ba_kernel_has_committed_traffic(bench):
    """The c4-ba line (plan path 5: register head of 3, packed LDS tail, 256 hub rows) finds its
    kernel instance in the committed profile, within 1 % of the algorithmic 12 B per element."""
    alg = 12 * 4096 * 2 ** 18
    name = bench.kernel_name({"path": 5, "tile_cols": 4, "head": 3, "tail_fmt": 2}, True, True,
                             4096)
    traffic, src = bench.traffic_from_profile(
        name, os.path.join(ROOT, "profiles", "r12", "c4ba", "summary.json"))
    assert traffic is not None and src.startswith("profiles/")
    # (round 5: 1.0106 x algorithmic on the profiling box, 1.0018 in round 4 -- every workgroup
    # stages the graph's LDS tail and hub heads, ~100 KB x 512 workgroups)
    assert abs(traffic / alg - 1) < 0.02


@pytest.mark.parametrize("rnd,workload,plan,n,alg", [
    ("r14", "c3", {"path": 1, "tile_cols": 64}, 256, 12 * 256 * 164608),
    ("r13", "c4", {"path": 1, "tile_cols": 4}, 4096, 12 * 4096 * 2 ** 18),
    ("r12", "c4gather", {"path": 4, "tile_cols": 4, "head": 5, "tail_fmt": 0}, 4096,
     12 * 4096 * 2 ** 18)])
def test_c3_c4_round_kernels_have_committed_traffic(bench, rnd, workload, plan, n, alg):
    """The c3, c4 and c4-gather lines' round kernels (full instance names from the plan) are in
    the round-5 profiles, within 1 % of the algorithmic 12 B per element."""
    traffic, src = bench.traffic_from_profile(
        bench.kernel_name(plan, True, True, n),
        os.path.join(ROOT, "profiles", rnd, workload, "summary.json"))
    assert traffic is not None and src.startswith(f"profiles/{rnd}/")
    assert abs(traffic / alg - 1) < 0.01


def test_every_line_carries_a_cpu_baseline(bench):
    """every BASELINE-config line reports the reference's CPU path beside it (N = 1),
    with the host CPU named -- no runner hard-codes a null cpu_baseline."""
    src = open(os.path.join(ROOT, "bench.py")).read()
    assert '"cpu_baseline": None' not in src
    info = bench.host_cpu()
    assert info["host_cpu"] and info["host_cores"] >= 1


def test_cpu_record_of_a_halo_rank(bench):
    """The c4-rank CPU baseline: one rank's local rows + halo rows through the numpy and C
    restatements (mixer.py:43-66), the lagged deviation, scaled to the full column count."""
    from distributed_learning_amd import sharding
    from distributed_learning_amd.graph import best_constant_weight, from_edge_weights, torus_edges
    edges = torus_edges(8, 8)
    csr = from_edge_weights(edges, [best_constant_weight(edges, list(range(64)))] * len(edges),
                            list(range(64)))
    rp = sharding.split_halo_plans(csr, sharding.torus_block_partition(8, 8, 4))[0]
    rec = bench.cpu_record(rp.csr, rp.n_local, 256, 64, 1e-3, "the lagged deviation",
                           n_halo=rp.n_halo, lagged=True)
    assert rec["value"] > 0 and rec["c_port_value"] > 0 and rec["cores"] == 1
    assert f"{rp.n_halo} halo rows" in rec["sample"] and rec["host_cpu"]
    whole = bench.cpu_record(csr, 64, 256, 64, 1e-3, "_get_deviation_dict")
    assert whole["value"] > 0 and "halo" not in whole["sample"]
    assert bench.sample_cols(type("A", (), {"cpu_cols": 1 << 18})(), 4096) == 1 << 15


def _c2_evidence(bench):
    """(the bench line saved beside the c2 profile, its kernel's summary entry): both from ONE
    gpurun call (scripts/r13_c2.sh), the directory bench.PROFILE_C2 names."""
    import json
    d = os.path.dirname(bench.PROFILE_C2)
    with open(os.path.join(d, "bench.json")) as f:
        line = json.loads([ln for ln in f.read().splitlines() if ln.startswith("{")][-1])
    name = bench.kernel_name({"tile_cols": 16, "path": 1}, sgd=True, dev=True, n_src=1024)
    return line, bench.profile_entry(name)


def test_c2_profile_backs_its_bench_line(bench):
    """the headline's cited profile must be evidence for the line's time.  The
    committed c2 profile was taken in the same call as the bench run saved beside it; its
    mix_tile_kernel average may not imply a round slower than that run's HIP-event launch time
    by more than 5 %, and the frac the line reports and the one the profile implies agree
    within 3 %."""
    line, e = _c2_evidence(bench)
    assert e is not None and e["calls"] >= 20
    us = e.get("timed_avg_us") or e["avg_us"]   # the profiled command's timed rounds
    rf = line["roofline"]
    assert us / 1e3 <= 1.05 * rf["launch_ms"], (us, rf["launch_ms"])
    prof_frac = rf["bytes_per_launch"] / (us / 1e6) / 1e9 / bench.HBM_PEAK_GBS
    assert abs(prof_frac / rf["frac"] - 1) < 0.03, (prof_frac, rf["frac"])
    # and the kernel average is no slower than the whole round the same call's bench timed
    assert us / 1e3 <= line["ms_per_step"] * 1.0 + 1e-9


def test_c2_line_reports_its_profile_fields(bench):
    """rocprof_frac / rocprof_launch_ms on the c2 line come from the cited summary itself."""
    _, e = _c2_evidence(bench)
    name = bench.kernel_name({"tile_cols": 16, "path": 1}, sgd=True, dev=True, n_src=1024)
    f = bench.rocprof_fields(name, 12 * 1024 * 2 ** 20)
    us = e.get("timed_avg_us") or e["avg_us"]
    assert f["rocprof_launch_ms"] == us / 1e3
    assert abs(f["rocprof_frac"] - 12 * 1024 * 2 ** 20 / (us * 1e3) / bench.HBM_PEAK_GBS) < 1e-12

