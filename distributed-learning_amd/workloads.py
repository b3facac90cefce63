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
                       schedule="sqrt", device=None, consensus="reference"):
    """``run`` of the notebook (cell 14) without plots: the learning tasks are created first and
    the master's ``serve`` after them, as the notebook does.  ``consensus`` picks the façade's
    schedule ("reference": the reference's own message interleaving, each agent step on the
    device; "synchronous": one Jacobi launch per round).  Returns {token: final w}."""
    shutdown = asyncio.Queue()
    net = ca.ConsensusNetwork(topology, shutdown, device=device, schedule=consensus)
    agents = [ca.ConsensusAgent(t, convergence_eps=convergence_eps) for t in net.tokens]
    for a in agents:
        net.register_agent(a)
    shards = split_data(X, y, net.tokens)
    tasks = [asyncio.create_task(_learning_instance(*shards[a.token], a, iterations, alpha, tau,
                                                    schedule)) for a in agents]
    serve = asyncio.create_task(net.serve())
    res = await asyncio.gather(*tasks)
    await shutdown.put(ca.SHUTDOWN)
    await serve
    return {a.token: w for a, w in zip(agents, res)}


class ConsensusGDRun:
    """``consensus_gd`` with every agent and every iteration in ONE launch (dl_consensus_gd):
    the same shards (``split_data`` in ``ConsensusNetwork.tokens`` order), local steps and
    consensus rounds (weighted by shard size, ``convergence_eps`` one-sided test), fp64 on the
    device with no host round trip per iteration.  The constructor makes everything resident
    (shards, adjacency, step sizes, zero weights); ``launch()`` is stream-ordered; ``result()``
    copies back ({token: final w}, Jacobi iterations per round).
    ``edge_weight``: mix with a uniform per-edge weight w (x' = x(1 - w deg) + w sum_j x_j, the
    TCP agent's update with a fast-averaging weight, consensus_tcp/agent.py:204-207) instead of
    the asyncio network's Perron eps 0.95 / max degree (consensus_asyncio.py:78-86).  The FDLA
    optimum is such a uniform weight on edge-transitive graphs (ring, torus)."""

    def __init__(self, topology, X, y, iterations, alpha=1e-1, tau=1e-4, convergence_eps=1e-10,
                 schedule="sqrt", device=None, max_iter=10_000_000, edge_weight=None):
        import torch

        from . import _lib
        from .graph import asyncio_adjacency, perron_eps
        self._torch, self._lib = torch, _lib
        self.dev = torch.device(device) if device is not None else torch.device(
            "cuda", torch.cuda.current_device())
        self.tokens, rp, cl = asyncio_adjacency(topology)
        shards = split_data(X, y, self.tokens)
        Xs = np.concatenate([shards[t][0] for t in self.tokens]).astype(np.float64)
        ys = np.concatenate([shards[t][1] for t in self.tokens]).astype(np.float64)
        sizes = [shards[t][0].shape[0] for t in self.tokens]
        sp = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
        steps = np.asarray([alpha * np.power(it + 1, -0.5) if schedule == "sqrt" else alpha
                            for it in range(iterations)], np.float64)
        self.rows, self.iterations = int(Xs.shape[0]), int(iterations)
        F = X.shape[1]
        self.t = {k: torch.as_tensor(v, device=self.dev) for k, v in
                  dict(X=Xs, y=ys, sp=sp, rp=rp.astype(np.int32), cl=cl.astype(np.int32),
                       steps=steps if iterations else np.zeros(1),
                       w=np.zeros((len(self.tokens), F))).items()}
        self.iters = torch.zeros(max(iterations, 1), dtype=torch.int32, device=self.dev)
        t = self.t
        self.args = _lib.DlConsensusGdArgs(
            _lib.ptr(t["X"]), _lib.ptr(t["y"]), _lib.ptr(t["sp"]), len(self.tokens), F,
            _lib.ptr(t["rp"]), _lib.ptr(t["cl"]),
            float(perron_eps(topology, self.tokens) if edge_weight is None else edge_weight),
            float(convergence_eps), sum(sizes) / len(sizes), float(tau), _lib.ptr(t["steps"]),
            self.iterations, int(max_iter), _lib.ptr(t["w"]), _lib.ptr(self.iters))

    def launch(self, reset=True):
        """All iterations from zero weights (reset) on the current stream."""
        import ctypes
        if reset:
            self.t["w"].zero_()
        with self._torch.cuda.device(self.dev):
            self._lib.check(self._lib.load().dl_consensus_gd(
                ctypes.byref(self.args), self.rows, self._lib.stream_handle(self.dev)),
                "dl_consensus_gd")

    def result(self):
        wf = self.t["w"].cpu().numpy()
        return ({tok: wf[i] for i, tok in enumerate(self.tokens)},
                self.iters[:self.iterations].cpu().numpy())


def consensus_gd_device(topology, X, y, iterations, alpha=1e-1, tau=1e-4, convergence_eps=1e-10,
                        schedule="sqrt", device=None, max_iter=10_000_000, edge_weight=None):
    """One-launch ``consensus_gd`` (ConsensusGDRun).  Returns ({token: final w}, Jacobi
    iterations per round)."""
    run = ConsensusGDRun(topology, X, y, iterations, alpha, tau, convergence_eps, schedule,
                         device, max_iter, edge_weight)
    run.launch()
    return run.result()


def accuracy(w, X, y):
    m = LogRegTitanic(X.shape[1])
    m.W = w
    return m.calc_accuracy(X, y)


class MLPConsensusSGD:
    """Config c3 (BASELINE.json): every agent trains its own ``ANNModel`` (networks/ann_model.py)
    on its own batch and the agents mix after every local step -- the training loop of the
    reference's consensus notebooks (Man_Colab.ipynb cells 12-23: local SGD step, then
    ``Mixer.mix``), with all agents resident in HBM.

    One ``step()`` = batched per-agent gradients followed by the round X <- W (X - lr G) and the
    disagreement (``GossipEngine.round``).  emit="grad" (default): the kernel writes G and the
    fused round forms X - lr G on the fly (reads X and G).  emit="step" (fused kernel only): the
    gradient kernel writes the local step T = X - lr G itself and the round mixes T -- one matrix
    read instead of two, bit-identical X' -- but the kernel must then read every parameter again
    where its gradient is stored, and fc1.weight (72 % of them) is long out of the caches by
    then: at c3 the round saves 22 us and the gradient kernel loses 58 (3159 vs 3503 steps/s,
    PMC bytes per step 975 vs 985 MB; profiles/r10/c3_step).  ``G`` holds whichever was
    written.  Every call
    is stream-ordered with no host synchronisation, so ``capture()`` can record a step as a
    hipGraph (two graphs: the engine ping-pongs X/Y) and ``replay()`` then runs steps with one
    graph launch each instead of ~15 kernel launches from Python."""

    def __init__(self, ann, eng, data, labels, lr, deviation=True, emit="auto"):
        if eng.layout == "tiled" and ann.path != "fused":
            raise ValueError("the layered gradients read X row-major: use GossipEngine("
                             "layout='rows') or the fused kernel")
        if eng.n != ann.N or eng.P < ann.P:
            raise ValueError("engine and model disagree on agents/params")
        import torch
        self.ann, self.eng = ann, eng
        # an engine row order (GossipEngine(order=...), "auto" on plan-path-5 graphs) stores
        # agent eng.order[s] in row s: every per-agent input follows it, so each row still
        # trains on its own agent's batch (results per agent are those of agent order)
        if eng.order is not None:
            data = data.index_select(0, eng.order.to(data.device))
            labels = labels.index_select(0, eng.order.to(labels.device))
        self.data, self.labels = data, labels
        self.lr, self.deviation = float(lr), bool(deviation)
        if emit == "auto":
            emit = "grad"
        if emit not in ("step", "grad") or (emit == "step" and ann.path != "fused"):
            raise ValueError("emit must be 'grad', or 'step' with the fused gradient kernel")
        self.emit = emit
        # Row-major engines may carry zero padding columns [ann.P, eng.P) (a whole number of mix
        # tiles: no ragged tail launch); the tiled layout zero-pads its last tile itself.  Padding
        # stays exactly zero -- G is zero there and W 0 = 0 -- and adds exact zeros to the
        # deviation, so results are those of the unpadded round.
        self.G = torch.zeros_like(eng.X)
        self.graphs = None
        self._torch = torch

    @property
    def loss(self):
        """Per-row mean cross-entropy of the last step (device tensor [N]; row s is agent
        ``eng.order[s]`` under an engine row order, see ``agent_loss``)."""
        return self.ann.loss

    def agent_loss(self):
        """Per-agent mean cross-entropy of the last step, in agent order."""
        if self.eng.order is None:
            return self.ann.loss
        out = self._torch.empty_like(self.ann.loss)
        out[self.eng.order] = self.ann.loss
        return out

    @staticmethod
    def padded_params(csr, n_params, device):
        """n_params rounded up to the row-major mix tile width for this graph."""
        from .engine import DeviceCsr, plan_shape
        T = plan_shape(DeviceCsr(csr, device), n_params, deviation=True)["tile_cols"]
        return -(-n_params // T) * T if T else n_params

    def gradients(self):
        """The gradient phase alone: G (emit="grad") or T = X - lr G (emit="step")."""
        P = self.ann.P
        lr = self.lr if self.emit == "step" else None
        if self.eng.layout == "tiled":     # the fused kernel addresses the tiles directly
            self.ann.gradients(self.eng.X, self.data, self.labels, self.G, lr=lr)
        else:
            self.ann.gradients(self.eng.X[:, :P], self.data, self.labels, self.G[:, :P], lr=lr)

    def round(self):
        """The round phase alone (after ``gradients``)."""
        if self.emit == "step":
            self.eng.round(src=self.G, deviation=self.deviation)
        else:
            self.eng.round(G=self.G, lr=self.lr, deviation=self.deviation)

    def step(self):
        self.gradients()
        self.round()

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


def _sgd_args(X, G, M, out, lr, momentum, dampening, weight_decay, nesterov, first):
    from . import _lib
    return _lib.DlSgdArgs(_lib.ptr(X), X.stride(0), _lib.ptr(G), G.stride(0), _lib.ptr(M),
                          M.stride(0) if M is not None else 0, _lib.ptr(out), out.stride(0),
                          X.shape[0], X.shape[1], float(lr), float(momentum), float(dampening),
                          float(weight_decay), int(bool(nesterov)), int(bool(first)))


def sgd_step(X, G, M=None, out=None, lr=0.1, momentum=0.0, dampening=0.0, weight_decay=0.0,
             nesterov=False, first=False):
    """``dl_sgd_step``: torch.optim.SGD.step over agent rows (X, G, M, out: [N, P] row-major
    device tensors; out defaults to X, i.e. in place).  Stream-ordered, no host sync."""
    import ctypes

    from . import _lib
    out = X if out is None else out
    for name, t in (("X", X), ("G", G), ("M", M), ("out", out)):
        if t is None:
            continue
        if t.dtype.itemsize != 4 or not t.is_floating_point() or t.dim() != 2 or \
                t.stride(1) != 1 or tuple(t.shape) != tuple(X.shape) or t.device != X.device:
            raise ValueError(f"{name} must be a row-major float32 [N, P] tensor like X")
    if momentum != 0.0 and M is None:
        raise ValueError("momentum needs a buffer M")
    args = _sgd_args(X, G, M, out, lr, momentum, dampening, weight_decay, nesterov, first)
    _lib.check(_lib.load().dl_sgd_step(ctypes.byref(args), _lib.stream_handle(X.device)),
               "dl_sgd_step")
    return out


def wrn_flops_per_image(depth=16, widen=4, num_classes=10, hw=32):
    """Forward FLOPs of one image through Wide_ResNet (convs + linear, 2 per MAC), and the FLOPs of
    forward + backward (input and weight gradients; the first conv needs no input gradient)."""
    n = (depth - 4) // 6
    st = [16, 16 * widen, 32 * widen, 64 * widen]
    convs = [(3, st[0], 3, hw)]               # (cin, cout, k, output hw)
    cin, h = st[0], hw
    for i, s in enumerate([1, 2, 2]):
        for j in range(n):
            stride = s if j == 0 else 1
            cout = st[i + 1]
            ho = h // stride
            convs.append((cin, cout, 3, h))           # conv1 (stride 1)
            convs.append((cout, cout, 3, ho))         # conv2 (strided)
            if stride != 1 or cin != cout:
                convs.append((cin, cout, 1, ho))      # 1x1 shortcut
            cin, h = cout, ho
    fwd = [2 * ci * co * k * k * o * o for ci, co, k, o in convs] + [2 * st[3] * num_classes]
    total = sum(fwd)
    return total, total + 2 * total - fwd[0]


class WRNConsensusSGD:
    """Config c5 (BASELINE.json): every agent trains its own Wide-ResNet (WRN-16-4,
    networks/wide_resnet.py) with the optimizer of Man_Colab.ipynb cell 19 (SGD, momentum 0.9,
    weight decay 5e-4, lr 0.02) on its own CIFAR-shaped batch, and the agents mix after every
    local step (the ``MasterNode`` loop the notebook drives, cells 21-23: local step, then
    ``Mixer.mix``, mixer.py:18-49).

    Layout: all agents' parameters are the rows of one row-major X[N, P] in HBM -- the Mixer's
    flatten order (mixer.py:68-69) -- and every agent's ``nn.Module`` parameters are views of its
    row; their ``.grad`` are views of G's rows, so backward accumulates straight into G.  One
    ``step()``:
      1. G = 0; per agent: forward, cross-entropy, backward (PyTorch-ROCm convs, MIOpen), agents
         spread round-robin over ``streams`` HIP streams;
      2. ``dl_sgd_step``: torch.optim.SGD's update (momentum buffers M), written to the scratch
         S instead of in place;
      3. ``dl_mix_round``: X <- W S with the fused disagreement -- the parameters land back in
         X, so the module views never move and no copy or re-binding is needed.
    Every call is stream-ordered: ``capture()`` records a step as one hipGraph."""

    def __init__(self, csr, batch, depth=16, widen=4, dropout=0.0, num_classes=10, lr=0.02,
                 momentum=0.9, weight_decay=5e-4, device="cuda", X0=None, seed=0, streams=1,
                 deviation=True, data=None, labels=None):
        import torch

        from .engine import DeviceCsr, Workspace, plan_shape
        from .networks.wide_resnet import Wide_ResNet
        self._torch = torch
        self.device = torch.device(device)
        if self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.N, self.B = csr.n_rows, int(batch)
        self.lr, self.momentum, self.wd = float(lr), float(momentum), float(weight_decay)
        self.deviation = bool(deviation)
        self.arch = (int(depth), int(widen), float(dropout), int(num_classes))
        self.models = []
        with torch.random.fork_rng(devices=[]):     # default torch init, agent a seeded seed + a
            for a in range(self.N):
                torch.manual_seed(seed + a)
                self.models.append(Wide_ResNet(*self.arch).to(self.device))
        shapes = [p.shape for p in self.models[0].parameters()]
        self.P = sum(int(np.prod(s)) for s in shapes)
        self.W = DeviceCsr(csr, self.device)
        T = plan_shape(self.W, self.P, deviation=True)["tile_cols"] or 1
        self.ld = -(-self.P // max(T, 16)) * max(T, 16)   # zero padding: no ragged tail launch
        f = lambda: torch.zeros(self.N, self.ld, dtype=torch.float32, device=self.device)  # noqa
        self.X, self.S, self.G = f(), f(), f()
        self.M = f() if self.momentum != 0.0 else None
        with torch.no_grad():
            for a, m in enumerate(self.models):
                if X0 is None:
                    self.X[a, :self.P] = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
                else:
                    self.X[a, :self.P] = torch.as_tensor(X0[a], dtype=torch.float32)
                off = 0
                for p in m.parameters():
                    n = p.numel()
                    p.set_(self.X[a, off:off + n].view_as(p))
                    p.grad = self.G[a, off:off + n].view_as(p)
                    off += n
        self.dev_sq = torch.zeros(self.N, dtype=torch.float32, device=self.device)
        self.dev_max = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.loss = torch.zeros(self.N, dtype=torch.float32, device=self.device)
        self.ws = Workspace(self.device)
        if data is None:
            g = torch.Generator(device=self.device).manual_seed(seed)
            data = torch.randn(self.N, self.B, 3, 32, 32, device=self.device, generator=g)
            labels = torch.randint(0, num_classes, (self.N, self.B), device=self.device,
                                   generator=g)
        self.data, self.labels = data, labels
        self.n_streams = max(1, int(streams))
        self.streams = [torch.cuda.Stream(self.device) for _ in range(self.n_streams)] \
            if self.n_streams > 1 else []
        self.steps_done = 0
        self.graph = None

    def params(self):
        """Row-major [N, P] view of every agent's flattened parameters (Mixer order)."""
        return self.X[:, :self.P]

    def flops_per_step(self):
        return wrn_flops_per_image(self.arch[0], self.arch[1], self.arch[3])[1] * self.N * self.B

    def _local_grads(self):
        torch = self._torch
        F = torch.nn.functional
        self.G.zero_()
        main = torch.cuda.current_stream(self.device)
        for s in self.streams:
            s.wait_stream(main)
        for a, m in enumerate(self.models):
            ctx = torch.cuda.stream(self.streams[a % self.n_streams]) if self.streams else \
                _nullctx()
            with ctx:
                loss = F.cross_entropy(m(self.data[a]), self.labels[a])
                loss.backward()
                self.loss[a:a + 1].copy_(loss.detach().reshape(1))
        for s in self.streams:
            main.wait_stream(s)

    def _round(self, first):
        from .engine import mix_round
        sgd_step(self.X, self.G, self.M, out=self.S, lr=self.lr, momentum=self.momentum,
                 weight_decay=self.wd, first=first)
        mix_round(self.W, self.S, self.X, dev_sq=self.dev_sq if self.deviation else None,
                  dev_max=self.dev_max if self.deviation else None, workspace=self.ws)

    def step(self):
        self._local_grads()
        self._round(first=self.steps_done == 0)
        self.steps_done += 1

    def capture(self):
        """Record one step (after at least one eager step: the momentum buffers exist and every
        MIOpen solution is found) as a hipGraph.  Runs nothing."""
        torch = self._torch
        if self.steps_done == 0:
            raise RuntimeError("run one eager step before capture()")
        from . import _lib
        self.ws.get(_lib.load().dl_mix_workspace_bytes(self.N, 0, self.ld))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._local_grads()
            self._round(first=False)
        self.graph = g

    def replay(self, steps=1):
        for _ in range(int(steps)):
            self.graph.replay()
            self.steps_done += 1


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
