"""Drivers that run the asyncio façade the way tests/golden/make_golden.py ran the reference
(same task creation order, so the event loop interleaves the agents the same way)."""
import asyncio

import numpy as np


def _network(ca, topology, conv_eps, iterates, shutdown):
    kw = {} if iterates is None else {"iterates": iterates}
    net = ca.ConsensusNetwork(topology, shutdown, **kw)
    agents = [ca.ConsensusAgent(t, convergence_eps=conv_eps) for t in net.tokens]
    for a in agents:
        net.register_agent(a)
    return net, agents


async def multi_round(ca, topology, values_per_round, weights, conv_eps, driver, iterates=None):
    """make_golden._async_multi on the façade: 'gather' or 'loop'."""
    shutdown = asyncio.Queue()
    net, agents = _network(ca, topology, conv_eps, iterates, shutdown)
    if driver == "gather":
        serve = asyncio.create_task(net.serve())
        results = []
        for values in values_per_round:
            tasks = [asyncio.create_task(a.run_round(values[a.token], weights[a.token]))
                     for a in agents]
            res = await asyncio.gather(*tasks)
            results.append({a.token: r for a, r in zip(agents, res)})
    else:
        async def instance(a):
            outs, w = [], values_per_round[0][a.token]
            for r in range(len(values_per_round)):
                w = await a.run_round(w * 0.5 + values_per_round[r][a.token], weights[a.token])
                outs.append(w)
            return outs
        tasks = [asyncio.create_task(instance(a)) for a in agents]
        serve = asyncio.create_task(net.serve())
        outs = await asyncio.gather(*tasks)
        results = [{a.token: outs[i][r] for i, a in enumerate(agents)}
                   for r in range(len(values_per_round))]
    await shutdown.put(ca.SHUTDOWN)
    await serve
    return [int(t) for t in net.tokens], results


def case_inputs(d, key):
    toks = d[key + "_tokens"].tolist()
    vals = d[key + "_values"]
    is_scalar = key.split("_")[-2] == "scalar"
    per_round = []
    for r in range(vals.shape[0]):
        if is_scalar:
            per_round.append({t: float(vals[r, i]) for i, t in enumerate(toks)})
        else:
            per_round.append({t: vals[r, i].copy() for i, t in enumerate(toks)})
    wts = {t: int(d[key + "_weights"][i]) for i, t in enumerate(toks)}
    edges = [tuple(int(x) for x in e) for e in d[key + "_edges"].tolist()]
    return edges, per_round, wts, float(d[key + "_conv_eps"]), key.split("_")[-1]


def check_case(ca, d, key, iterates=None):
    """Run one asyncio_rounds.npz case; returns the max abs difference (0.0 = bit-exact) and
    whether every returned object has the reference's type."""
    edges, vals, wts, ce, driver = case_inputs(d, key)
    toks, res = asyncio.run(multi_round(ca, edges, vals, wts, ce, driver, iterates))
    want = d[key + "_out"]
    got = np.stack([np.stack([np.asarray(res[r][t]) for t in toks]) for r in range(len(res))])
    types_ok = all((np.ndim(res[r][t]) == 0) == bool(d[key + "_out_is_scalar"])
                   for r in range(len(res)) for t in toks)
    return float(np.max(np.abs(got - want))), got.dtype == want.dtype and types_ok


def titanic_async(ca, d, key, X, y, iterates=None):
    """make_golden._titanic_async_runs on the façade (the notebook's learning_instance, with its
    in-place ``w -= ...`` on the returned array)."""
    from oracle.mixer_ref import logreg_gradient
    topo = [tuple(int(x) for x in e) for e in d[key + "_edges"].tolist()]
    ce, steps = float(d[key + "_conv_eps"]), int(d[key + "_steps"])
    algo = key.split("_")[-1]

    async def main():
        shutdown = asyncio.Queue()
        net, agents = _network(ca, topo, ce, iterates, shutdown)
        tokens = net.tokens
        shards, tmpX, tmpy = {}, X.copy(), y.copy()
        for i in range(len(tokens)):
            ln = len(tmpX) // (len(tokens) - i)
            shards[tokens[i]] = (tmpX[:ln], tmpy[:ln])
            tmpX, tmpy = tmpX[ln:], tmpy[ln:]

        async def learning_instance(Xs, ys, agent):
            alpha, tau = (1e-1, 1e-4) if algo == "sqrt" else (5e-4, 1e-4)
            w = np.zeros(Xs.shape[1])
            for it in range(steps):
                g = logreg_gradient(Xs, ys, w, tau)
                if algo == "sqrt":
                    w -= alpha * np.power(it + 1, -0.5) * g
                else:
                    w -= alpha * g
                w = await agent.run_round(w, Xs.shape[0])
                if algo == "old" and it % 2000 == 0:
                    alpha *= 0.99
            return w

        tasks = [asyncio.create_task(learning_instance(*shards[a.token], a)) for a in agents]
        asyncio.create_task(net.serve())
        res = await asyncio.gather(*tasks)
        await shutdown.put(ca.SHUTDOWN)
        return res

    return np.stack(asyncio.run(main()))
