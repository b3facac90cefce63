"""asyncio consensus API (reference: utils/consensus_asyncio.py:1-312) on the HIP Perron kernel.

Same module surface: the message constants, ``ConsensusNetwork(topology, shutdown_q, debug)``
with ``register_agent`` / ``initialize_agents`` / ``serve`` / ``describe``, and
``ConsensusAgent(token, debug, convergence_eps)`` with ``await run_round(value, weight)``.

What changes is the transport.  The reference simulates sockets with asyncio.Queue pairs and
runs one Jacobi update per agent per message exchange (:234-310).  Its single rounds are
exactly the synchronous iterate y_k = (I - eps L)^k y_0 stopped at the first k where every
agent's one-sided test holds (checked against the reference in tests/test_oracle_golden.py).
Here the round is that synchronous iteration, executed for all agents at once in one kernel
launch (``dl_perron_round``): the network collects every agent's (value, weight) for the round,
runs the GPU loop, and resolves each agent's ``run_round`` with its row.

Deliberate differences: consecutive rounds are synchronous here, while the
reference's later rounds can interleave iterations of neighbouring agents; an unknown token
raises ValueError (the reference raises NameError on its undefined IllegalArgumentException,
:90); self-loop edges are ignored.
"""
import asyncio
import functools
import sys

import numpy as np
import torch

from .. import engine as _engine
from ..graph import asyncio_adjacency

NEW_ROUND = 'NEW_ROUND'
REQUEST_VALUE = 'REQUEST_VALUE'
CONVERGED = 'CONVERGED'
NOT_CONVERGED = 'NOT CONVERGED'
DONE = 'DONE'
NETWORK_READY = 'NETWORK_READY'
SHUTDOWN = 'SHUTDOWN'

MAX_MIX_ITERATIONS = 10_000_000  # the reference loops until DONE; this bounds a round


class ConsensusNetwork:
    def __init__(self, topology, shutdown_q, debug=False, device=None):
        self.topology = topology
        self.tokens = list(set(np.array(topology).flatten()))   # consensus_asyncio.py:40
        self.agents = dict()
        self.shutdown_q = shutdown_q
        self.running_round = False
        self.debug = debug
        self._device = torch.device(device) if device is not None else None
        self._ready = None
        self._pending = {}
        self._shutdown = False
        self._adj = None
        self.last_round_iterations = 0

    def _debug(self, *args, **kwargs):
        if self.debug:
            if 'file' not in kwargs.keys():
                print('Master:', *args, **kwargs, file=sys.stderr)
            else:
                print('Master:', *args, **kwargs)

    def _adjacency_matrix(self):
        return np.array([[int((u, v) in self.topology or (v, u) in self.topology)
                          for v in self.tokens] for u in self.tokens])

    def describe(self):
        """Spectral report (consensus_asyncio.py:59-76), computed on the host."""
        E = self._adjacency_matrix()
        outdeg = np.sum(E, axis=1)
        L = np.diag(outdeg) - E
        print('Laplacian:\n{}'.format(L))
        L_eig = np.linalg.eigvals(L)
        L_eig.sort()
        print('Eigenvalues: {}'.format(L_eig))
        print('Algebraic connectivity: {}'.format(L_eig[1]))
        P = np.eye(outdeg.shape[0]) - self._calc_eps() * L
        print('Perron matrix:\n{}'.format(P))
        P_eig = np.linalg.eigvals(P)
        P_eig.sort()
        print('Eigenvalues: {}'.format(P_eig))
        print('Convergence speed: {}'.format(np.abs(P_eig[1])))

    @functools.lru_cache
    def _calc_eps(self):
        """0.95 / max degree (consensus_asyncio.py:78-86)."""
        E = self._adjacency_matrix()
        outdeg = np.sum(E, axis=1)
        return 0.95 / np.max(outdeg)

    def register_agent(self, agent):
        if agent.token not in self.tokens:
            raise ValueError('Agent with token {} is not presented in given topology'
                             .format(agent.token))
        self.agents[agent.token] = agent
        self._debug(f'Got {len(self.agents.keys())}/{len(self.tokens)} agents')
        if len(self.agents.keys()) == len(self.tokens):
            self.initialize_agents()

    def initialize_agents(self):
        tokens, rp, cl = asyncio_adjacency(self.topology, self.tokens)
        dev = self._dev()
        self._adj = (torch.as_tensor(rp.astype(np.int32), device=dev),
                     torch.as_tensor(cl.astype(np.int32), device=dev))
        eps = self._calc_eps()
        for token, agent in self.agents.items():
            agent.set_master(self)
            agent.set_neighbors([tokens[c] for c in cl[rp[tokens.index(token)]:
                                                        rp[tokens.index(token) + 1]]])
            agent.set_epsilon(eps)
        self._ready_event().set()

    def _dev(self):
        if self._device is None:
            if not torch.cuda.is_available():
                raise RuntimeError("the HIP consensus network needs a GPU (no CPU fallback)")
            self._device = torch.device("cuda", torch.cuda.current_device())
        return self._device

    def _ready_event(self):
        if self._ready is None:
            self._ready = asyncio.Event()
        return self._ready

    async def serve(self):
        """Waits for SHUTDOWN on shutdown_q (consensus_asyncio.py:120-133); rounds themselves
        complete as soon as every agent has submitted its value."""
        self._debug('serving...')
        if self.shutdown_q is None:
            return
        while True:
            msg = await self.shutdown_q.get()
            if msg == SHUTDOWN:
                self._debug('===== SHUTDOWN =====')
                self._shutdown = True
                for fut in [f for (_, _, f) in self._pending.values()]:
                    if not fut.done():
                        fut.set_result(SHUTDOWN)
                self._pending.clear()
                return

    async def _submit(self, agent, value, weight):
        if self._shutdown:
            return SHUTDOWN
        if agent.token in self._pending:
            raise RuntimeError(f'agent {agent.token!r} is already in a round')
        fut = asyncio.get_running_loop().create_future()
        self._pending[agent.token] = (value, weight, fut)
        self._debug(f'got NEW_ROUND from "{agent.token}" with weight {weight}')
        if len(self._pending) == len(self.tokens):
            self._run_round()
        return await fut

    def _run_round(self):
        pending, self._pending = self._pending, {}
        self.running_round = True
        self._debug('===== STARTING A NEW ROUND =====')
        vals = [np.asarray(pending[t][0]) for t in self.tokens]
        shape = vals[0].shape
        dtype = np.result_type(*[v.dtype for v in vals], np.float32)
        tdt = torch.float32 if dtype == np.float32 else torch.float64
        Y = torch.as_tensor(np.stack([v.reshape(-1) for v in vals]).astype(
            np.float32 if tdt == torch.float32 else np.float64), device=self._dev())
        weights = np.asarray([float(pending[t][1]) for t in self.tokens], np.float64)
        mean_w = sum(pending[t][1] for t in self.tokens) / len(self.tokens)
        conv = np.asarray([self.agents[t].convergence_eps for t in self.tokens], np.float64)
        k = _engine.perron_round(
            Y, self._adj[0], self._adj[1], self._calc_eps(), float(conv[0]),
            weight=torch.as_tensor(weights, device=self._dev()), mean_weight=float(mean_w),
            max_iter=MAX_MIX_ITERATIONS,
            conv_eps_rows=None if np.all(conv == conv[0]) else torch.as_tensor(conv,
                                                                            device=self._dev()))
        self.last_round_iterations = k
        out = Y.cpu().numpy()
        self._debug('===== ALL NODES CONVERGED! DONE =====')
        self.running_round = False
        for i, t in enumerate(self.tokens):
            fut = pending[t][2]
            if not fut.done():
                y = out[i].reshape(shape)
                fut.set_result(y if shape else y[()])


class ConsensusAgent:
    def __init__(self, token, debug=False, convergence_eps=1e-4):
        self.token = token
        self.neighbors = []
        self.network = None
        self.network_ready = False
        self.consensus_eps = None
        self.convergence_eps = convergence_eps
        self.debug = debug
        self.round_counter = 0

    def _debug(self, *args, **kwargs):
        if self.debug:
            if 'file' not in kwargs.keys():
                print(f'Agent "{self.token}":', *args, **kwargs, file=sys.stderr)
            else:
                print(f'Agent "{self.token}":', *args, **kwargs)

    def set_master(self, network):
        self.network = network
        self._debug('heard from master')

    def set_neighbors(self, neighbors):
        self.neighbors = list(neighbors)
        self._debug('got neighbors from master')

    def set_epsilon(self, eps):
        self.consensus_eps = eps
        self._debug(f'got consensus epsilon from master: {self.consensus_eps}')

    async def run_round(self, value, weight):
        """One consensus round: returns this agent's weighted-average estimate
        sum_i x_i w_i / sum_i w_i (consensus_asyncio.py:209-312)."""
        self.round_counter += 1
        self._debug(f'running new round with v={value}, w={weight}')
        if not self.network_ready:
            if self.network is None:
                raise RuntimeError(f'agent {self.token!r} is not registered with a network')
            await self.network._ready_event().wait()
            self.network_ready = True
        res = await self.network._submit(self, value, weight)
        self._debug(f'final result: {res}')
        return res
