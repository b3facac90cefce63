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
    name = bench.kernel_name({"tile_cols": 16}, sgd=True, dev=True, n_src=1024)
    traffic, src = bench.traffic_from_profile(name)
    assert traffic is not None, f"{name} not in the default PMC summary"
    # within 1 % of the algorithmic 12 * N * P bytes per round
    assert abs(traffic / (12 * 1024 * 2 ** 20) - 1) < 0.01
    assert src.startswith("profiles/")


def test_c3_kernels_have_committed_traffic(bench):
    path = os.path.join(ROOT, "profiles", "r09", "c3", "summary.json")
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
