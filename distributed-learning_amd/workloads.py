"""Reference workloads driven through the drop-in API (config c1 of BASELINE.json).

Titanic consensus GD (notebooks/Titanic Consensus GD test.ipynb, cells 12-14): every agent holds
a contiguous shard of the training set, takes a local GD step on the L2-regularised logistic
loss with step ``alpha * (it + 1) ** -0.5`` and then runs one asyncio consensus round weighted
by its shard size.  Data preparation (cells 2-4) lives with the caller; the tests feed the
preprocessed arrays committed under tests/golden/.
"""
import asyncio

import numpy as np

from .networks.logreg_model_titanic import LogRegTitanic
from .utils import consensus_asyncio as ca


def split_data(X, y, tokens):
    """``split_data`` (notebook cell 12): contiguous shards in ``tokens`` order."""
    tmpX, tmpy = X.copy(), y.copy()
    result = {}
    num = len(tokens)
    for i in range(num):
        ln = len(tmpX) // (num - i)
        result[tokens[i]] = (tmpX[:ln], tmpy[:ln])
        tmpX, tmpy = tmpX[ln:], tmpy[ln:]
    return result


async def _learning_instance(X, y, agent, iterations, alpha, tau, schedule):
    model = LogRegTitanic(X.shape[1], lr=alpha, tau=tau)
    w = np.zeros(X.shape[1])
    for it in range(iterations):
        grad = model.gradient(X, y, w)
        step = alpha * np.power(it + 1, -0.5) if schedule == "sqrt" else alpha
        w = w - step * grad
        w = await agent.run_round(w, X.shape[0])
    return w


async def consensus_gd(topology, X, y, iterations, alpha=1e-1, tau=1e-4, convergence_eps=1e-10,
                       schedule="sqrt", device=None):
    """``run`` of the notebook (cell 14) without plots.  Returns {token: final w}."""
    shutdown = asyncio.Queue()
    net = ca.ConsensusNetwork(topology, shutdown, device=device)
    agents = [ca.ConsensusAgent(t, convergence_eps=convergence_eps) for t in net.tokens]
    for a in agents:
        net.register_agent(a)
    shards = split_data(X, y, net.tokens)
    serve = asyncio.create_task(net.serve())
    res = await asyncio.gather(*[_learning_instance(*shards[a.token], a, iterations, alpha, tau,
                                                    schedule) for a in agents])
    await shutdown.put(ca.SHUTDOWN)
    await serve
    return {a.token: w for a, w in zip(agents, res)}


def accuracy(w, X, y):
    m = LogRegTitanic(X.shape[1])
    m.W = w
    return m.calc_accuracy(X, y)
