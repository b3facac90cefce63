"""The asyncio façade's message protocol (utils/consensus_asyncio.py, schedule="reference") against
the reference's own multi-round runs, on the CPU: the arithmetic is the oracle's numpy
restatement (oracle/async_ref.py, test double of the device iterates), so what these tests pin is
the SCHEDULE -- which neighbour iterate each step mixes, which messages are dropped as stale, when
each agent sees DONE.  The same fixtures run through the HIP arithmetic in
tests/test_asyncio_gpu.py."""
import asyncio

import numpy as np
import pytest

import asyncio_drivers as drv
from oracle.async_ref import NumpyIterates


def _ca():
    from distributed_learning_amd.utils import consensus_asyncio as ca
    return ca


def _cases(golden):
    return [str(k) for k in golden("asyncio_rounds.npz")["cases"]]


def test_every_multi_round_case_bit_exact(golden):
    d = golden("asyncio_rounds.npz")
    bad = []
    for key in _cases(golden):
        err, types_ok = drv.check_case(_ca(), d, key, NumpyIterates())
        if err != 0.0 or not types_ok:
            bad.append((key, err, types_ok))
    assert not bad, bad


def test_later_rounds_are_not_synchronous(golden):
    """The fixture really exercises the asynchronous interleaving: ring8 at eps 0.1, round 2,
    is far from every synchronous Jacobi iterate (the gap the synchronous façade had)."""
    d = golden("asyncio_graphs.npz")
    assert d["ring8_e1_r1_jacobi_err"] > 0.1
    key = "ring8_e1"
    toks = d[key + "_tokens"].tolist()
    edges = [tuple(int(x) for x in e) for e in d["ring8_edges"].tolist()]
    vals = [{t: d[key + f"_r{r}_values"][i] for i, t in enumerate(toks)} for r in range(2)]
    wts = {t: int(d[key + "_weights"][i]) for i, t in enumerate(toks)}
    _, res = asyncio.run(drv.multi_round(_ca(), edges, vals, wts, float(d[key + "_conv_eps"]),
                                         "gather", NumpyIterates()))
    for r in range(2):
        got = np.stack([res[r][t] for t in toks])
        assert np.array_equal(got, d[key + f"_r{r}_out"]), r


@pytest.mark.parametrize("name", ["k4", "ring8", "cycle3", "grid5", "rr4_16"])
def test_asyncio_graphs_every_round(golden, name):
    """Every round committed in asyncio_graphs.npz (``_r0_`` and ``_r1_``), bit for bit."""
    d = golden("asyncio_graphs.npz")
    edges = [tuple(int(x) for x in e) for e in d[f"{name}_edges"].tolist()]
    ei = 0
    while f"{name}_e{ei}_conv_eps" in d:
        key = f"{name}_e{ei}"
        toks = d[key + "_tokens"].tolist()
        rounds = 2 if key + "_r1_values" in d else 1
        vals = [{t: d[key + f"_r{r}_values"][i] for i, t in enumerate(toks)}
                for r in range(rounds)]
        wts = {t: int(d[key + "_weights"][i]) for i, t in enumerate(toks)}
        _, res = asyncio.run(drv.multi_round(_ca(), edges, vals, wts,
                                             float(d[key + "_conv_eps"]), "gather",
                                             NumpyIterates()))
        for r in range(rounds):
            got = np.stack([res[r][t] for t in toks])
            assert np.array_equal(got, d[key + f"_r{r}_out"]), (key, r)
        ei += 1


def test_titanic_notebook_runs_at_inexact_eps(golden):
    """Notebook-style consensus GD (cells 12-14 and the 'old' algorithm of cell 22) through the
    reference agents at convergence eps 1e-2 / 1e-4 / 1e-1: 300 steps, every agent's W."""
    d = golden("asyncio_rounds.npz")
    t = golden("titanic.npz")
    nt = int(t["n_test"])
    for key in [str(k) for k in d["titanic_runs"]]:
        w = drv.titanic_async(_ca(), d, key, t["X"][nt:], t["y"][nt:], NumpyIterates())
        assert np.array_equal(w, d[key + "_w"]), key


def test_self_loop_and_unknown_token_raise():
    ca = _ca()

    async def main():
        net = ca.ConsensusNetwork([(0, 1), (1, 1)], asyncio.Queue(), iterates=NumpyIterates())
        net.register_agent(ca.ConsensusAgent(0))
        with pytest.raises(ValueError):
            net.register_agent(ca.ConsensusAgent(1))
    asyncio.run(main())
    with pytest.raises(ValueError):
        ca.ConsensusNetwork([(0, 1)], None).register_agent(ca.ConsensusAgent(7))
    with pytest.raises(ValueError):
        ca.ConsensusNetwork([(0, 1)], None, schedule="bogus")


def test_shutdown_releases_a_waiting_round():
    """SHUTDOWN while an agent waits for its round (serve :129-133) returns SHUTDOWN (:248-249
    or the NEW_ROUND wait :222-224)."""
    ca = _ca()

    async def main():
        q = asyncio.Queue()
        net = ca.ConsensusNetwork([(0, 1), (1, 2)], q, iterates=NumpyIterates())
        agents = [ca.ConsensusAgent(t) for t in net.tokens]
        for a in agents:
            net.register_agent(a)
        serve = asyncio.create_task(net.serve())
        lone = asyncio.create_task(agents[0].run_round(np.ones(3), 1))
        await asyncio.sleep(0)
        await asyncio.sleep(0)
        await q.put(ca.SHUTDOWN)
        await serve
        return await lone
    assert asyncio.run(main()) == ca.SHUTDOWN
