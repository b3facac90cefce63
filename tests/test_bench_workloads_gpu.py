"""bench.py's secondary workload lines run end to end on the GPU and print a well-formed line
(one short run each, in-process): one rank of the c4 agent partition (8- and 2-way, every halo
scheme) and the irregular c4-ba graph.  The default c2 line is the driver's own bench run."""
import importlib.util
import json
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod_gpu", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def run_line(bench, monkeypatch, capsys, argv):
    monkeypatch.setattr(sys, "argv", ["bench.py"] + argv)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    bench.main()
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")]
    assert lines, "no JSON line"
    return json.loads(lines[-1])


@pytest.mark.parametrize("rank_of", [8, 2])
def test_c4_rank_line(cuda, bench, monkeypatch, capsys, rank_of):
    d = run_line(bench, monkeypatch, capsys, ["--workload", "c4-rank", "--rank-of", str(rank_of),
                                              "--steps", "3", "--warmup", "1"])
    assert d["unit"] == "rounds/s" and d["value"] > 0
    assert set(d["schemes"]) == {"whole", "chunks", "split"}
    r = d["roofline"]
    assert r["bound"] == "hbm" and 0.2 < r["frac"] < 1.0, r
    assert 0.2 < d["pack"]["frac"] < 1.0, d["pack"]
    cpu = d["cpu_baseline"]        # this rank's round on one host core, the CPU named
    assert cpu["value"] > 0 and cpu["cores"] == 1 and cpu["host_cpu"], cpu


def test_c4_ba_line(cuda, bench, monkeypatch, capsys):
    d = run_line(bench, monkeypatch, capsys, ["--workload", "c4-ba", "--steps", "2", "--warmup",
                                              "1", "--no-cpu"])
    assert d["unit"] == "rounds/s" and d["value"] > 0
    assert d["config"]["plan"]["path"] == 5 and d["config"]["plan"]["hub_rows"] == 256
    assert 0.2 < d["roofline"]["frac"] < 1.0
