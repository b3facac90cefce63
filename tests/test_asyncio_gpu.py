"""asyncio-API façade (ConsensusNetwork / ConsensusAgent.run_round) on the HIP Perron kernel,
checked against the reference's own runs (tests/golden/asyncio_graphs.npz, titanic.npz) and
the values the reference notebook printed."""
import asyncio

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ca():
    from distributed_learning_amd.utils import consensus_asyncio as ca
    return ca


async def _one_round(topology, values, weights, conv_eps):
    ca = _ca()
    q = asyncio.Queue()
    net = ca.ConsensusNetwork(topology, q)
    agents = [ca.ConsensusAgent(t, convergence_eps=conv_eps) for t in net.tokens]
    for a in agents:
        net.register_agent(a)
    serve = asyncio.create_task(net.serve())
    res = await asyncio.gather(*[a.run_round(values[a.token], weights[a.token]) for a in agents])
    await q.put(ca.SHUTDOWN)
    await serve
    return {a.token: r for a, r in zip(agents, res)}, net.last_round_iterations


@pytest.mark.parametrize("name", ["k4", "ring8", "cycle3", "grid5", "rr4_16"])
def test_run_round_matches_reference(golden, cuda, name):
    d = golden("asyncio_graphs.npz")
    edges = [tuple(e) for e in d[f"{name}_edges"].tolist()]
    ei = 0
    while f"{name}_e{ei}_conv_eps" in d:
        key = f"{name}_e{ei}"
        toks = d[key + "_tokens"].tolist()
        vals = {t: d[key + "_r0_values"][i] for i, t in enumerate(toks)}
        wts = {t: int(d[key + "_weights"][i]) for i, t in enumerate(toks)}
        out, k = asyncio.run(_one_round(edges, vals, wts, float(d[key + "_conv_eps"])))
        assert k == d[key + "_r0_k"], key
        got = np.stack([out[t] for t in toks])
        np.testing.assert_allclose(got, d[key + "_r0_out"], rtol=0, atol=1e-13)
        ei += 1


def test_scalar_values_and_shutdown(cuda):
    """Notebook cell 10 shape: scalar values, weights 1..5 -> weighted average on every agent."""
    ca = _ca()
    grid5 = [('center', 'west'), ('center', 'east'), ('center', 'north'), ('center', 'south'),
             ('west', 'north'), ('north', 'east'), ('east', 'south'), ('west', 'south')]

    async def main():
        q = asyncio.Queue()
        net = ca.ConsensusNetwork(grid5, q)
        agents = [ca.ConsensusAgent(t, convergence_eps=1e-6) for t in net.tokens]
        for a in agents:
            net.register_agent(a)
        serve = asyncio.create_task(net.serve())
        vals = {a.token: float(i + 1) for i, a in enumerate(agents)}
        res = await asyncio.gather(*[a.run_round(vals[a.token], i + 1)
                                     for i, a in enumerate(agents)])
        want = sum(vals[a.token] * (i + 1) for i, a in enumerate(agents)) / 15.0
        for r in res:
            assert isinstance(r, np.floating) and abs(r - want) < 1e-5
        # a round that never completes is released by SHUTDOWN
        lone = asyncio.create_task(agents[0].run_round(1.0, 1))
        await asyncio.sleep(0)
        await q.put(ca.SHUTDOWN)
        await serve
        assert await lone == ca.SHUTDOWN
    asyncio.run(main())
    with pytest.raises(ValueError):
        ca.ConsensusNetwork([(0, 1)], None).register_agent(ca.ConsensusAgent(7))


def test_titanic_ring8_consensus_gd_matches_reference(golden, cuda):
    """BASELINE config c1: the reference's 4000-step asyncio consensus GD (ring-8, eps=10)."""
    from distributed_learning_amd import workloads
    d = golden("titanic.npz")
    nt = int(d["n_test"])
    topo = [(i, (i + 1) % 8) for i in range(8)]
    w = asyncio.run(workloads.consensus_gd(topo, d["X"][nt:], d["y"][nt:],
                                           int(d["ring8_steps"]), convergence_eps=10))
    got = np.stack([w[t] for t in d["ring8_tokens"].tolist()])
    np.testing.assert_allclose(got, d["ring8_eps10_final_w"], rtol=0, atol=1e-12)


@pytest.mark.parametrize("topo", [
    [(0, 1), (0, 2), (0, 3), (1, 2), (1, 3), (2, 3)],                 # K4, nb cell 15
    [(0, 1), (1, 2), (2, 0)],                                           # cycle3, cell 17
])
def test_titanic_exact_consensus_equals_notebook(golden, cuda, topo):
    """4000 steps at convergence_eps 1e-10: every agent prints the centralised W to 8 digits
    and scores 0.797752808988764 (notebook cells 15-17)."""
    from distributed_learning_amd import workloads
    d = golden("titanic.npz")
    nb = golden("notebook_outputs.json")
    nt = int(d["n_test"])
    w = asyncio.run(workloads.consensus_gd(topo, d["X"][nt:], d["y"][nt:], 4000,
                                           convergence_eps=1e-10))
    for wt in w.values():
        np.testing.assert_allclose(wt, nb["titanic_consensus_w_4000"], atol=6e-8)
        assert workloads.accuracy(wt, d["X"][:nt], d["y"][:nt]) == nb["titanic_score"]
