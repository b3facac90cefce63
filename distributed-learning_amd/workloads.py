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


class MLPConsensusSGD:
    """Config c3 (BASELINE.json): every agent trains its own ``ANNModel`` (networks/ann_model.py)
    on its own batch and the agents mix after every local step -- the training loop of the
    reference's consensus notebooks (Man_Colab.ipynb cells 12-23: local SGD step, then
    ``Mixer.mix``), with all agents resident in HBM.

    One ``step()`` = batched per-agent gradients (``BatchedANN.gradients`` -> G rows) followed by
    the fused round X <- W (X - lr G) and the disagreement (``GossipEngine.round``).  Every call
    is stream-ordered with no host synchronisation, so ``capture()`` can record a step as a
    hipGraph (two graphs: the engine ping-pongs X/Y) and ``replay()`` then runs steps with one
    graph launch each instead of ~15 kernel launches from Python."""

    def __init__(self, ann, eng, data, labels, lr, deviation=True):
        if eng.layout != "rows":
            raise ValueError("the batched gradients read X row-major: use GossipEngine(layout='rows')")
        if eng.n != ann.N or eng.P < ann.P:
            raise ValueError("engine and model disagree on agents/params")
        import torch
        self.ann, self.eng = ann, eng
        self.data, self.labels = data, labels
        self.lr, self.deviation = float(lr), bool(deviation)
        # The engine may carry zero padding columns [ann.P, eng.P) (a whole number of mix tiles:
        # no ragged tail launch).  They stay exactly zero -- G is zero there and W 0 = 0 -- and
        # add exact zeros to the deviation, so results are those of the unpadded round.
        self.G = torch.zeros(ann.N, eng.P, dtype=torch.float32, device=eng.device)
        self.graphs = None
        self._torch = torch

    @property
    def loss(self):
        """Per-agent mean cross-entropy of the last step (device tensor [N])."""
        return self.ann.loss

    @staticmethod
    def padded_params(csr, n_params, device):
        """n_params rounded up to the row-major mix tile width for this graph."""
        from .engine import DeviceCsr, plan_shape
        T = plan_shape(DeviceCsr(csr, device), n_params, deviation=True)["tile_cols"]
        return -(-n_params // T) * T if T else n_params

    def step(self):
        P = self.ann.P
        self.ann.gradients(self.eng.X[:, :P], self.data, self.labels, self.G[:, :P])
        self.eng.round(G=self.G, lr=self.lr, deviation=self.deviation)

    def capture(self):
        """Record one step per ping-pong parity.  Runs nothing: the engine state afterwards is
        what it was before."""
        torch = self._torch
        self.eng.reserve_workspace(self.deviation)
        graphs = []
        for _ in range(2):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self.step()               # records; swaps eng.X / eng.Y on the host
            graphs.append(g)
        self.graphs = graphs              # two swaps: eng.X is the original buffer again
        self._parity = 0

    def replay(self, steps=1):
        for _ in range(int(steps)):
            self.graphs[self._parity].replay()
            self._parity ^= 1
            self.eng.X, self.eng.Y = self.eng.Y, self.eng.X
