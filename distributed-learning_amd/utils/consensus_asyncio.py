"""asyncio consensus API (reference: utils/consensus_asyncio.py:1-312).

Same module surface: the message constants, ``ConsensusNetwork(topology, shutdown_q, debug)``
with ``register_agent`` / ``initialize_agents`` / ``serve`` / ``describe``, and
``ConsensusAgent(token, debug, convergence_eps)`` with ``await run_round(value, weight)``.

Two schedules.

``schedule="reference"`` (default) replays the reference's message protocol on asyncio, with
the same queues, tasks and waits in the same order, so the event loop interleaves the agents
exactly as it interleaves the reference's.  That matters after the first round: an agent serves
a neighbour's REQUEST_VALUE with whatever iterate it holds at that moment (:279-281), drops
messages of other rounds -- the previous round's unanswered requests and late values are still
queued when the next round starts (:276-278) -- and sees DONE only between exchanges
(:241-252, :260-265).  Agents then mix neighbour iterates of other iteration counts and stop at
different counts, which no synchronous iteration reproduces (asyncio_graphs.npz ring8_e1 round
2: 0.35 away from every Jacobi iterate).  The message payloads are device iterate handles
(``iterates.Iterate``); each step -- pre-scale :231, update :295, verdict :297 -- is one
``dl_async_update`` launch whose verdict is read back before the agent's next message, because
the protocol branches on it (:301-310).

``schedule="synchronous"`` runs the whole round for all agents as one ``dl_perron_round``
launch (synchronous Jacobi with the common stop rule).  It equals the reference's first round
of a network and any round in which the reference's agents stay in lockstep (every round at
convergence_eps 10, i.e. one step per round, as in the Titanic notebook's c1 run), and is the
fast path for large graphs.

Deliberate differences: an unknown token raises ValueError (the reference raises NameError on its
undefined IllegalArgumentException, :90); self-loop edges raise ValueError (the reference's agent
would wait forever on its own unanswered request).
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

MAX_MIX_ITERATIONS = 10_000_000  # synchronous schedule: the reference loops until DONE

_SCHEDULES = ("reference", "synchronous")


class _DoneSignal(Exception):
    """DONE seen while collecting neighbour values (:244-247, :262-265)."""


class _Shutdown(Exception):
    """SHUTDOWN seen while collecting neighbour values (:248-249, :266-267)."""


class ConsensusNetwork:
    """The master of consensus_asyncio.py:37-174."""

    def __init__(self, topology, shutdown_q, debug=False, device=None, schedule="reference",
                 iterates=None):
        if schedule not in _SCHEDULES:
            raise ValueError(f"schedule must be one of {_SCHEDULES}")
        self.topology = topology
        self.tokens = list(set(np.array(topology).flatten()))   # consensus_asyncio.py:40
        self.agents = dict()
        self.agents_sockets = dict()     # token -> (agent -> master, master -> agent)
        self.shutdown_q = shutdown_q
        self.running_round = False
        self.agent_new_round = dict()
        self.agent_weight = dict()
        self.agent_converged = dict()
        self.debug = debug
        self.schedule = schedule
        self._device = torch.device(device) if device is not None else None
        self._iterates = iterates
        # synchronous schedule state
        self._ready = None
        self._pending = {}
        self._shutdown = False
        self._adj = None
        self._rounds = {}       # (agents, values per agent, dtype) -> engine.PerronRounds
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

    def _dev(self):
        if self._device is None:
            if not torch.cuda.is_available():
                raise RuntimeError("the HIP consensus network needs a GPU (no CPU fallback)")
            self._device = torch.device("cuda", torch.cuda.current_device())
        return self._device

    def register_agent(self, agent):
        if agent.token not in self.tokens:
            raise ValueError('Agent with token {} is not presented in given topology'
                             .format(agent.token))
        self.agents[agent.token] = agent
        self._debug(f'Got {len(self.agents.keys())}/{len(self.tokens)} agents')
        if len(self.agents.keys()) == len(self.tokens):
            self.initialize_agents()

    def initialize_agents(self):
        if any(u == v for (u, v) in self.topology):
            raise ValueError("self-loop edges are not supported (the reference agent would wait "
                             "forever for its own reply)")
        if self.schedule == "synchronous":
            self._initialize_synchronous()
            return
        if self._iterates is None:
            from ..iterates import DeviceIterates
            self._iterates = DeviceIterates(self._dev())
        # master <-> agent links (:97-100), in registration order
        for token, agent in self.agents.items():
            up, down = asyncio.Queue(), asyncio.Queue()
            self.agents_sockets[token] = (up, down)
            agent.set_master((down, up))
        # agent <-> agent links (:102-114): one queue per direction, created by the first endpoint
        links = dict()
        for token, agent in self.agents.items():
            mine = dict()
            for u, v in self.topology:
                if token != u and token != v:
                    continue
                other = u if token == v else v
                pair = links.get((token, other))
                if pair is None:
                    inbound, outbound = asyncio.Queue(), asyncio.Queue()
                    links[(token, other)] = (inbound, outbound)
                    links[(other, token)] = (outbound, inbound)
                    pair = (inbound, outbound)
                mine[other] = pair
            agent.set_neighbors(mine)
            agent.set_epsilon(self._calc_eps())
            agent._iterates = self._iterates
        for token, (up, down) in self.agents_sockets.items():   # :117-118
            asyncio.create_task(down.put(NETWORK_READY), name='master put NETWORK_READY')

    # ------------------------------------------------------------------ master loop (:120-174)
    async def serve(self):
        if self.schedule == "synchronous":
            return await self._serve_synchronous()
        self._debug('serving...')
        self.agent_new_round = dict.fromkeys(self.tokens, False)
        self.agent_converged = dict.fromkeys(self.tokens, False)
        while True:
            stop = asyncio.create_task(self.shutdown_q.get(), name='master check shutdown')
            inbox = {token: asyncio.create_task(up.get(), name=f'master check agent "{token}"')
                     for token, (up, down) in self.agents_sockets.items()}
            done, pending = await asyncio.wait({stop}.union(set(inbox.values())),
                                               return_when=asyncio.FIRST_COMPLETED)
            if stop in done:
                self._debug('===== SHUTDOWN =====')
                for token, (up, down) in self.agents_sockets.items():
                    await down.put(SHUTDOWN)
                break
            for token, task in inbox.items():
                if task in done:
                    self._on_agent_message(token, task.result())
            for task in pending:
                task.cancel()
            if not self.running_round and all(self.agent_new_round.values()):
                await self._open_round()
            if self.debug:
                self._debug(f"checking DONE: {sum(map(int, self.agent_converged.values()))}"
                            f"/{len(self.tokens)} converged")
            if self.running_round and all(self.agent_converged.values()):
                await self._close_round()

    def _on_agent_message(self, token, msg):
        if isinstance(msg, tuple) and msg[0] == NEW_ROUND:
            if self.debug:
                self._debug(f'got NEW_ROUND from "{token}" with weight {msg[1]}')
            if self.running_round:
                self._debug(f'got NEW_ROUND from "{token}" but round is already running')
            self.agent_new_round[token] = True
            self.agent_weight[token] = msg[1]
        elif msg == CONVERGED or msg == NOT_CONVERGED:
            self._debug(f'got {"CONVERGED" if msg == CONVERGED else "NOT_CONVERGED"} '
                        f'from "{token}"')
            if not self.running_round:
                self._debug(f'got {msg} from "{token}" but round is not yet running')
            self.agent_converged[token] = msg == CONVERGED
        else:
            self._debug(f'got unexpected request from "{token}": {msg}')

    async def _open_round(self):
        self._debug('===== STARTING A NEW ROUND =====')
        self.running_round = True
        self.agent_new_round = dict.fromkeys(self.tokens, False)
        self.agent_converged = dict.fromkeys(self.tokens, False)
        mean_weight = sum(self.agent_weight.values()) / len(self.tokens)
        for token, (up, down) in self.agents_sockets.items():
            await down.put((NEW_ROUND, mean_weight))

    async def _close_round(self):
        self._debug('===== ALL NODES CONVERGED! DONE =====')
        self.running_round = False
        for token, (up, down) in self.agents_sockets.items():
            await down.put(DONE)

    # ------------------------------------------------------------------ synchronous schedule
    def _initialize_synchronous(self):
        tokens, rp, cl = asyncio_adjacency(self.topology, self.tokens)
        dev = self._dev()
        self._adj = (torch.as_tensor(rp.astype(np.int32), device=dev),
                     torch.as_tensor(cl.astype(np.int32), device=dev))
        eps = self._calc_eps()
        for token, agent in self.agents.items():
            agent.set_master(self)
            i = tokens.index(token)
            agent.set_neighbors({tokens[c]: None for c in cl[rp[i]:rp[i + 1]]})
            agent.set_epsilon(eps)
        if self._ready is None:
            self._ready = asyncio.Event()
        self._ready.set()

    async def _serve_synchronous(self):
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
        if self.debug:
            self._debug(f'got NEW_ROUND from "{agent.token}" with weight {weight}')
        if len(self._pending) == len(self.tokens):
            self._run_synchronous_round()
        return await fut

    def _run_synchronous_round(self):
        pending, self._pending = self._pending, {}
        self.running_round = True
        self._debug('===== STARTING A NEW ROUND =====')
        vals = [np.asarray(pending[t][0]) for t in self.tokens]
        shape = vals[0].shape
        dtype = np.result_type(*[v.dtype for v in vals], np.float32)
        tdt = torch.float32 if dtype == np.float32 else torch.float64
        weights = [float(pending[t][1]) for t in self.tokens]
        mean_w = sum(pending[t][1] for t in self.tokens) / len(self.tokens)
        conv = [self.agents[t].convergence_eps for t in self.tokens]
        # one context per value shape and dtype: pinned staging + device buffers made once, a
        # round is one H2D copy, one launch, one D2H copy and one synchronisation
        key = (len(vals), int(vals[0].size), tdt)
        ctx = self._rounds.get(key)
        if ctx is None:
            ctx = self._rounds[key] = _engine.PerronRounds(self._adj[0], self._adj[1], key[0],
                                                           key[1], tdt, self._dev())
        out, k = ctx.run(vals, weights, float(mean_w), self._calc_eps(), float(conv[0]),
                         MAX_MIX_ITERATIONS,
                         conv_eps_rows=None if all(c == conv[0] for c in conv) else conv)
        self.last_round_iterations = k
        self._debug('===== ALL NODES CONVERGED! DONE =====')
        self.running_round = False
        for i, t in enumerate(self.tokens):
            fut = pending[t][2]
            if not fut.done():
                y = out[i].reshape(shape)
                fut.set_result(y if shape else y[()])


class ConsensusAgent:
    """An agent of consensus_asyncio.py:177-312."""

    def __init__(self, token, debug=False, convergence_eps=1e-4):
        self.token = token
        self.neighbor_sockets = dict()   # token -> (inbound, outbound)
        self.master_sockets = None       # (master -> agent, agent -> master)
        self.network_ready = False
        self.consensus_eps = None
        self.convergence_eps = convergence_eps
        self.debug = debug
        self.round_counter = 0
        self.iterations = 0              # steps of the last round (diagnostic)
        self._iterates = None

    def _debug(self, *args, **kwargs):
        if self.debug:
            if 'file' not in kwargs.keys():
                print(f'Agent "{self.token}":', *args, **kwargs, file=sys.stderr)
            else:
                print(f'Agent "{self.token}":', *args, **kwargs)

    def set_master(self, master_sockets):
        self.master_sockets = master_sockets
        self._debug('heard from master')

    def set_neighbors(self, neighbor_sockets):
        self.neighbor_sockets = dict(neighbor_sockets)
        self._debug('got neighbors from master')

    def set_epsilon(self, eps):
        self.consensus_eps = eps
        self._debug(f'got consensus epsilon from master: {self.consensus_eps}')

    async def run_round(self, value, weight):
        """One consensus round: returns this agent's estimate of sum_i x_i w_i / sum_i w_i
        (consensus_asyncio.py:209-312)."""
        if isinstance(self.master_sockets, ConsensusNetwork):
            return await self._run_round_synchronous(value, weight)
        self.round_counter += 1
        if self.debug:   # (formatting numpy values costs ~10 us a call)
            self._debug(f'running new round with v={value}, w={weight}')
        inbox, outbox = self.master_sockets
        if not self.network_ready:                                   # :212-218
            self._debug('initialized. Waiting for NETWORK_READY')
            rdy = await inbox.get()
            self._debug(f'got {rdy}')
            self.network_ready = rdy == NETWORK_READY
            if not self.network_ready:
                return rdy
        self._debug('sending NEW_ROUND to master')                   # :220-227
        await outbox.put((NEW_ROUND, weight))
        resp = await inbox.get()
        if not isinstance(resp, tuple) or resp[0] != NEW_ROUND:
            return resp
        self._debug('NEW_ROUND ack!')
        store = self._iterates
        y = store.load(value, weight, resp[1])                      # :231
        keep = 1 - self.consensus_eps * len(self.neighbor_sockets)   # :295
        flagged = False
        self.iterations = 0
        while True:                                                  # :234
            self._debug('requesting values from neighbors')
            for token, (inbound, outbound) in self.neighbor_sockets.items():
                await outbound.put((REQUEST_VALUE, self.round_counter))
            try:
                received = await self._collect(y)
            except _DoneSignal:
                break
            except _Shutdown:
                return SHUTDOWN
            y, c = store.update(y, list(received.values()), keep, self.consensus_eps,
                                self.convergence_eps)                # :295-297
            self.iterations += 1
            if self.debug:
                self._debug(f'updated value = {y}, c={c}')
            if c != flagged:                                         # :301-310
                self._debug('sending CONVERGED to master' if c else 'sending NOT_CONVERGED to master')
                await outbox.put(CONVERGED if c else NOT_CONVERGED)
                flagged = c
        out = store.result(y)
        if self.debug:
            self._debug(f'final result: {out}')
        return out

    def _master_says(self, msg):
        if msg == DONE:
            self._debug('got DONE from master!!!')
            raise _DoneSignal
        if msg == SHUTDOWN:
            raise _Shutdown
        self._debug(f'Unexpected request from master: {msg}')

    async def _collect(self, y):
        """Gather one value per neighbour for this step while serving the neighbours' requests
        with the current iterate (:239-284).  DONE / SHUTDOWN from the master end it."""
        inbox = self.master_sockets[0]
        received = {}
        while len(received) != len(self.neighbor_sockets):
            if inbox.qsize() > 0:                                    # :242-252
                self._master_says(inbox.get_nowait())
                continue
            master = asyncio.create_task(inbox.get())
            watch = {token: asyncio.create_task(inbound.get())
                     for token, (inbound, outbound) in self.neighbor_sockets.items()}
            done, pending = await asyncio.wait({master}.union(set(watch.values())),
                                               return_when=asyncio.FIRST_COMPLETED)
            for task in pending:
                task.cancel()
            if master in done:                                       # :260-269
                self._master_says(master.result())
            for token, task in watch.items():                         # :270-284
                if task not in done:
                    continue
                msg = task.result()
                if not isinstance(msg, tuple) or len(msg) < 2:
                    self._debug(f'got unexpected request from "{token}": {msg}')
                if msg[1] != self.round_counter:
                    self._debug(f'! got request/response from "{token}" from previous round')
                    continue
                if isinstance(msg[0], str) and msg[0] == REQUEST_VALUE:
                    self._debug(f'sending values to "{token}"')
                    await self.neighbor_sockets[token][1].put((y, self.round_counter))
                else:
                    self._debug(f'got value from "{token}"')
                    received[token] = msg[0]
        return received

    async def _run_round_synchronous(self, value, weight):
        net = self.master_sockets
        self.round_counter += 1
        if self.debug:   # (formatting numpy values costs ~10 us a call)
            self._debug(f'running new round with v={value}, w={weight}')
        if not self.network_ready:
            await net._ready.wait()
            self.network_ready = True
        res = await net._submit(self, value, weight)
        if self.debug:
            self._debug(f'final result: {res}')
        return res
