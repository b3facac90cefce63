"""numpy restatement of the reference gossip-mixing path (TEST INFRASTRUCTURE ONLY).

Each function cites the reference file:line it restates.  Parity pinned by
tests/test_oracle_golden.py against fixtures produced by running the reference.
"""
import numpy as np


def topology_to_csr(topology, keys=None):
    """dict-of-dicts topology -> CSR in *dict insertion order*.

    Row order = ``topology`` key order (``for agent in self.topology``, mixer.py:46);
    entry order within a row = ``topology[a].items()`` order (mixer.py:47).  The weight is the
    Python float as given; the fp32 cast happens where numpy does it (in the multiply).
    """
    keys = list(topology) if keys is None else list(keys)
    index = {k: i for i, k in enumerate(keys)}
    rowptr, cols, ws = [0], [], []
    for a in keys:
        for n, w in topology[a].items():
            cols.append(index[n])
            ws.append(float(w))
        rowptr.append(len(cols))
    return np.asarray(rowptr, np.int64), np.asarray(cols, np.int64), np.asarray(ws, np.float64)


def mix_once(X, rowptr, cols, w):
    """``Mixer._mix_params_once`` (utils/consensus_simple/mixer.py:43-49).

    ``sum(params[n] * weight for n, weight in topology[a].items())``: Python ``sum`` starts at
    int 0 and folds left; each product is ``fp32 array * python float`` (NEP 50: the float is
    cast to the array dtype first), each add rounds separately.
    """
    X = np.asarray(X)
    out = np.empty_like(X)
    dt = X.dtype.type
    for a in range(len(rowptr) - 1):
        acc = 0
        for e in range(rowptr[a], rowptr[a + 1]):
            acc = acc + X[cols[e]] * dt(w[e])
        out[a] = acc
    return out


def sgd_step(X, G, lr):
    """Local step ``x <- x - lr * g`` in the array dtype (fp32: separate mul and sub)."""
    return X - X.dtype.type(lr) * G


def column_mean(X):
    """``np.mean(stack, axis=0)`` (mixer.py:61): rows summed in order, then divided by N."""
    X = np.asarray(X)
    acc = X[0].copy()
    for r in range(1, X.shape[0]):
        acc = acc + X[r]
    return acc / X.dtype.type(X.shape[0])


def deviation(X):
    """``Mixer._get_deviation_dict`` (mixer.py:57-66) with ``basic_deviation_metric`` (:5-6).

    Returns per-row ``||x_a - mean||_2`` (in row order); zeros when there is <= 1 agent.
    """
    X = np.asarray(X)
    if X.shape[0] <= 1:
        return np.zeros(X.shape[0], X.dtype)
    m = column_mean(X)
    return np.asarray([np.linalg.norm(X[a] - m) for a in range(X.shape[0])], X.dtype)


def max_parameters_std(X):
    """Intended semantics of ``Mixer.get_max_parameters_std`` (mixer.py:82-84):
    ``np.stack(params).std(axis=0).max()`` (population std).  The reference line itself
    raises TypeError on numpy>=2 (np.stack of dict_values)."""
    return np.asarray(X).std(axis=0).max()


def mixer_mix(X, rowptr, cols, w, times=1, eps=None):
    """``Mixer.mix`` loop (mixer.py:18-38, stop rule :40-41).  Returns (X, times_done)."""
    if len(rowptr) - 1 <= 1:
        return X, 0
    done = 0

    def stop(P):
        return (eps is None or deviation(P).max() < eps) and done >= times

    while not stop(X):
        X = mix_once(X, rowptr, cols, w)
        done += 1
    return X, done


# ------------------------------------------------------------------ consensus_tcp update
def tcp_run_once(edges, weights, values):
    """One synchronous ``ConsensusAgent.run_once`` round of every agent
    (utils/consensus_tcp/agent.py:204-207; neighbours and weights as the master hands them out,
    master.py:227-243).  values: dict token -> ndarray; returns the new dict.  Restated directly
    (no CSR), in numpy's own promotion: np.float64(1 - S) * fp32 value is fp64."""
    out = {}
    for t, x in values.items():
        nbrs = {u if t == v else v for (u, v) in edges if t == u or t == v}
        own = list(filter(lambda uv_c: (uv_c[0][0] == t or uv_c[0][1] == t),
                          list(zip(edges, weights))))
        ew = {n: [c for ((u, v), c) in own if (u == n or v == n)][0] for n in nbrs}
        s = np.sum([ew[n] for n in ew])
        out[t] = (1.0 - s) * x + np.sum([values[n] * ew[n] for n in ew], axis=0)
    return out


# ------------------------------------------------------------------ asyncio consensus round
def asyncio_tokens(topology):
    """``ConsensusNetwork.tokens`` (utils/consensus_asyncio.py:40)."""
    return list(set(np.array(topology).flatten()))


def asyncio_neighbors(topology, token):
    """Neighbour order an agent sees (``initialize_agents``, consensus_asyncio.py:104-114)."""
    nb = [u if token == v else v for (u, v) in topology if token == u or token == v]
    return list(dict.fromkeys(nb))


def perron_eps(topology, tokens):
    """``ConsensusNetwork.__calc_eps`` (consensus_asyncio.py:78-86): 0.95 / max degree."""
    E = np.array([[int((u, v) in topology or (v, u) in topology) for v in tokens] for u in tokens])
    return 0.95 / np.max(np.sum(E, axis=1))


def jacobi_round(topology, values, weights, conv_eps, max_iter=1_000_000, edge_weight=None):
    """Synchronous restatement of one ``ConsensusAgent.run_round`` over all agents.

    values/weights: dicts token -> ndarray / number.  Pre-scale ``y = v * w / mean_w``
    (consensus_asyncio.py:231, mean_w from serve() :165); update
    ``y <- y*(1 - eps*deg) + eps*sum(nbr y)`` (:295); agent flag
    ``all((y - v) <= conv_eps for v in nbr values)`` with the neighbours' PRE-update values
    (:297); stop at the first iteration where every flag is set (master DONE, :170-174).
    Returns (dict token -> y, k).  ``edge_weight``: a uniform mixing weight per edge in place of
    the Perron eps (x' = x + w sum_j (x_j - x) in the (1 - w deg) form above: the TCP agent's
    update, consensus_tcp/agent.py:204-207, with a fast-averaging weight that is the same on
    every edge, as the FDLA optimum is on the ring).
    """
    tokens = asyncio_tokens(topology)
    eps = perron_eps(topology, tokens) if edge_weight is None else edge_weight
    nbrs = {t: asyncio_neighbors(topology, t) for t in tokens}
    mean_w = sum(weights[t] for t in tokens) / len(tokens)
    y = {t: values[t] * weights[t] / mean_w for t in tokens}
    for k in range(1, max_iter + 1):
        new, flags = {}, []
        for t in tokens:
            nv = [y[j] for j in nbrs[t]]
            s = np.sum(nv, axis=0) if nv else 0.0
            new[t] = y[t] * (1 - eps * len(nbrs[t])) + eps * s
            flags.append(bool(np.all([(new[t] - v) <= conv_eps for v in nv])))
        y = new
        if all(flags):
            return y, k
    return y, max_iter


def logreg_gradient(X, y, w, tau=1e-4):
    """``LogRegTitanic.gradient`` (networks/logreg_model_titanic.py:16-20)."""
    def sig(x):
        return 1.0 / (1.0 + np.exp(-x))
    return -np.array([np.dot(y * sig(-y * (X @ w)), X[:, j])
                      for j in range(X.shape[1])]) / X.shape[0] + tau * w


def consensus_gd(topology, X, y, iterations, alpha=1e-1, tau=1e-4, conv_eps=1e-10,
                 schedule="sqrt", edge_weight=None):
    """The Titanic notebook's consensus GD run (cells 12-14) restated synchronously: shards split
    in ``ConsensusNetwork.tokens`` order, a local step per agent, then ``jacobi_round`` weighted
    by shard size.  Pinned bit for bit to the reference's 4000-step asyncio run by
    tests/test_oracle_golden.py.  Returns ({token: w}, [Jacobi iterations per round])."""
    toks = asyncio_tokens(topology)
    sh, tX, ty = {}, X.copy(), y.copy()
    for i in range(len(toks)):
        ln = len(tX) // (len(toks) - i)
        sh[toks[i]] = (tX[:ln], ty[:ln])
        tX, ty = tX[ln:], ty[ln:]
    w = {t: np.zeros(X.shape[1]) for t in toks}
    ks = []
    for it in range(iterations):
        step = alpha * np.power(it + 1, -0.5) if schedule == "sqrt" else alpha
        for t in toks:
            w[t] = w[t] - step * logreg_gradient(*sh[t], w[t], tau)
        w, k = jacobi_round(topology, w, {t: sh[t][0].shape[0] for t in toks}, conv_eps,
                            edge_weight=edge_weight)
        ks.append(k)
    return w, ks
