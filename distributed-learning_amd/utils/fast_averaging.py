"""Fastest-distributed-linear-averaging weights (reference: utils/fast_averaging.py:4-32).

The reference states the FDLA SDP (Xiao & Boyd, 2004) for cvxpy:

    minimise  gamma   s.t.  -gamma I <= I - L(w) - 11^T/n <= gamma I,   L(w) >= 0,
    L(w) = A diag(w) A^T   (A: vertex-edge incidence, vertices numbered by first appearance)

and returns ``(w in edge-list order, gamma)``.  cvxpy is not available here (nor on the GPU box),
so this module solves the same problem on the host, as the north star prescribes ("the
fast-averaging weight optimisation stays on the host").  ``find_optimal_weights`` picks one of
three methods, and always says which one it used (``info``); nothing falls back silently.

``sdp`` (n <= ``max_sdp``, default): a primal log-barrier Newton method for the SDP itself, to a
duality gap of ``tol``.  Every constraint lives on the complement of the all-ones vector; each is
written in the full n-space with the ones direction pinned to eigenvalue 1 (e.g.
F1 = (gamma - 1) I + L + (2 - gamma) 11^T/n), so log det and inverses need no basis change.  The
edge generators a_e = e_i - e_j are sparse, so the Hessian block K = A^T F^-1 A is a GATHER of
four entries of F^-1 per edge pair (O(m^2)) instead of a product (O(m^2 n)): one Newton step costs
three n x n inverses plus an m x m Cholesky solve (~0.2 s at the c2 graph, n = 1024, m = 2048).

``subgradient`` (larger graphs): minimises gamma(w) = max(1 - lambda_2(L), lambda_n(L) - 1)
to first order (Xiao & Boyd 2004, sec. 5) -- Lanczos (scipy eigsh) for the k extreme eigenpairs
on both ends of the sparse Laplacian's spectrum, descent on their entropy-smoothed maximum with
backtracking -- from the best-constant start, keeping the best iterate.  It certifies its
result against the best-constant gamma (never worse).

``best_constant``: w_e = 2 / (lambda_2 + lambda_n) of the unweighted Laplacian.  This IS the FDLA
optimum on edge-transitive graphs (rings, tori: by symmetry the optimal weights can be taken
uniform and the uniform optimum balances lambda_2 against lambda_n), and only there; it is used
only when asked for, and ``info['method']`` records it.

Self-loop edges have a zero incidence column; their weight is free in the reference and returned
as 0 here.
"""
import numpy as np

from ..graph import first_appearance_vertices


def _edge_index(graph, vertices):
    index = {v: i for i, v in enumerate(vertices)}
    i = np.asarray([index[u] for (u, v) in graph], np.int64)
    j = np.asarray([index[v] for (u, v) in graph], np.int64)
    return i, j, i != j


def _incidence(graph, vertices):
    i, j, active = _edge_index(graph, vertices)
    n, m = len(vertices), len(graph)
    A = np.zeros((n, m))
    e = np.nonzero(active)[0]
    A[i[e], e] = 1.0
    A[j[e], e] = -1.0
    return A


def _laplacian(n, i, j, w):
    L = np.zeros((n, n))
    np.add.at(L, (i, i), w)
    np.add.at(L, (j, j), w)
    np.add.at(L, (i, j), -w)
    np.add.at(L, (j, i), -w)
    return L


def _sparse_laplacian(n, i, j, w):
    import scipy.sparse as sp
    rows = np.concatenate([i, j, i, j])
    cols = np.concatenate([i, j, j, i])
    vals = np.concatenate([w, w, -w, -w])
    return sp.csr_matrix((vals, (rows, cols)), shape=(n, n))


def spectral_gamma(graph, weights, vertices=None):
    """gamma(w) = ||I - L(w) - 11^T/n||_2 (the convergence factor the reference returns)."""
    vertices = first_appearance_vertices(graph) if vertices is None else vertices
    i, j, active = _edge_index(graph, vertices)
    n = len(vertices)
    w = np.where(active, np.asarray(weights, float), 0.0)
    Mt = np.eye(n) - _laplacian(n, i, j, w) - np.ones((n, n)) / n
    return float(np.max(np.abs(np.linalg.eigvalsh(Mt))))


def _extreme_laplacian_eigs(n, i, j, w, dense_limit=2048):
    """(lambda_2, u_2, lambda_n, u_n) of L(w) (smallest nonzero and largest)."""
    if n <= dense_limit:
        ev, U = np.linalg.eigh(_laplacian(n, i, j, w))
        return ev[1], U[:, 1], ev[-1], U[:, -1]
    from scipy.sparse.linalg import LinearOperator, eigsh
    L = _sparse_laplacian(n, i, j, w)
    lmax, umax = eigsh(L, k=1, which="LA", tol=1e-10)
    # lambda_2: largest eigenvalue of  c I - L  restricted to the complement of 1
    c = float(lmax[0]) * 1.01
    ones = np.ones(n) / np.sqrt(n)

    def mv(x):
        x = x - ones * (ones @ x)
        y = c * x - L @ x
        return y - ones * (ones @ y)
    op = LinearOperator((n, n), matvec=mv, dtype=np.float64)
    lt, ut = eigsh(op, k=1, which="LA", tol=1e-10)
    return c - float(lt[0]), ut[:, 0], float(lmax[0]), umax[:, 0]


def best_constant_weight(graph, vertices=None):
    """2 / (lambda_2 + lambda_n) of the unweighted Laplacian (simple graph: parallel edges count
    once), the best uniform edge weight."""
    vertices = first_appearance_vertices(graph) if vertices is None else vertices
    i, j, active = _edge_index(graph, vertices)
    pairs = {(min(a, b), max(a, b)) for a, b, on in zip(i.tolist(), j.tolist(), active) if on}
    pi = np.asarray([p[0] for p in pairs], np.int64)
    pj = np.asarray([p[1] for p in pairs], np.int64)
    l2, _, ln, _ = _extreme_laplacian_eigs(len(vertices), pi, pj, np.ones(len(pi)))
    return 2.0 / (l2 + ln)


# ------------------------------------------------------------------------------------ SDP
def _solve_sdp(n, i, j, w0, tol=1e-8, max_newton=100, verbose=False):
    """Barrier method for  min gamma  over (w, gamma)  (i, j: endpoints of the m active edges)."""
    m = len(i)
    J = np.full((n, n), 1.0 / n)
    I = np.eye(n)

    def mats(w, g):
        L = _laplacian(n, i, j, w)
        return [((g - 1.0) * I + L + (2.0 - g) * J, 1.0, True),
                ((g + 1.0) * I - L - g * J, -1.0, True),
                (L + J, 1.0, False)]

    def phi(w, g, t):
        val = t * g
        for F, _, _ in mats(w, g):
            try:
                C = np.linalg.cholesky(F)
            except np.linalg.LinAlgError:
                return np.inf
            val -= 2.0 * np.sum(np.log(np.diag(C)))
        return val

    l2, _, ln, _ = _extreme_laplacian_eigs(n, i, j, w0)
    w = np.asarray(w0, float).copy()
    g = max(1.0 - l2, ln - 1.0) + 1e-2
    nb = 3.0 * (n - 1)
    t = 10.0 * nb
    newton = 0
    while True:
        for _ in range(max_newton):
            grad = np.zeros(m + 1)
            H = np.zeros((m + 1, m + 1))
            grad[m] = t
            for F, s, has_g in mats(w, g):
                Fi = np.linalg.inv(F) - J          # complement-only inverse (ones-eigenvalue 1)
                Fi = 0.5 * (Fi + Fi.T)
                K = Fi[np.ix_(i, i)] - Fi[np.ix_(i, j)] - Fi[np.ix_(j, i)] + Fi[np.ix_(j, j)]
                grad[:m] -= s * np.diag(K)
                H[:m, :m] += K * K
                if has_g:
                    D = Fi[:, i] - Fi[:, j]         # F^-1 a_e
                    grad[m] -= np.trace(Fi)
                    H[m, m] += np.sum(Fi * Fi)
                    cross = s * np.einsum("ke,ke->e", D, D)
                    H[:m, m] += cross
                    H[m, :m] += cross
            try:
                C = np.linalg.cholesky(H)
                dx = -np.linalg.solve(C.T, np.linalg.solve(C, grad))
            except np.linalg.LinAlgError:
                dx = -np.linalg.lstsq(H, grad, rcond=None)[0]
            lam2 = float(-grad @ dx)
            newton += 1
            if lam2 / 2.0 <= 1e-10:
                break
            s, f0 = 1.0, phi(w, g, t)
            while s > 1e-14:
                f1 = phi(w + s * dx[:m], g + s * dx[m], t)
                if f1 <= f0 - 0.25 * s * lam2:
                    break
                s *= 0.5
            w, g = w + s * dx[:m], g + s * dx[m]
        if verbose:
            print(f"  barrier t={t:.3g} gamma={g:.12f} newton={newton}")
        if nb / t < tol:
            break
        t *= 20.0
    return w, g, newton


# ----------------------------------------------------------------------------- first order
def _spectrum_ends(n, i, j, w, k, dense_limit=2048):
    """k smallest nonzero and k largest Laplacian eigenpairs of L(w): (lo, U_lo, hi, U_hi)."""
    if n <= dense_limit:
        ev, U = np.linalg.eigh(_laplacian(n, i, j, w))
        return ev[1:1 + k], U[:, 1:1 + k], ev[-k:], U[:, -k:]
    from scipy.sparse.linalg import LinearOperator, eigsh
    L = _sparse_laplacian(n, i, j, w)
    hi, U_hi = eigsh(L, k=k, which="LA", tol=1e-9)
    c = float(hi.max()) * 1.01
    ones = np.ones(n) / np.sqrt(n)

    def mv(x):
        x = x - ones * (ones @ x)
        y = c * x - L @ x
        return y - ones * (ones @ y)
    lt, U_lo = eigsh(LinearOperator((n, n), matvec=mv, dtype=np.float64), k=k, which="LA",
                     tol=1e-9)
    return c - lt, U_lo, hi, U_hi


def _solve_subgradient(n, i, j, w0, iters=300, k=8, verbose=False):
    """First-order FDLA for graphs too large for the dense SDP: descent on the entropy-smoothed
    spectral norm  f_mu(w) = mu log sum exp(g/mu)  over the 2k extreme eigenvalue terms
    g = {1 - lambda_2..k+1} u {lambda_n-k+1..n - 1} of L(w) (Lanczos for the eigenpairs); the
    gradient of each term is -/+ (u[i] - u[j])^2 (Xiao & Boyd 2004, sec. 5).  Armijo
    backtracking on f_mu, mu shrinking with the gap; the best iterate (true gamma) is kept."""
    k = max(1, min(k, (n - 1) // 2))
    w = np.asarray(w0, float).copy()

    def terms(w):
        lo, U_lo, hi, U_hi = _spectrum_ends(n, i, j, w, k)
        g = np.concatenate([1.0 - lo, hi - 1.0])
        D = np.concatenate([-(U_lo[i] - U_lo[j]) ** 2, (U_hi[i] - U_hi[j]) ** 2], axis=1)
        return g, D

    def smooth(g, mu):
        gm = g.max()
        e = np.exp((g - gm) / mu)
        return gm + mu * np.log(e.sum()), e / e.sum()

    g, D = terms(w)
    best_w, best = w.copy(), float(g.max())
    mu = 0.05
    step, it = 1.0, 0
    for it in range(iters):
        f, p = smooth(g, mu)
        grad = D @ p
        gn = float(grad @ grad)
        if gn == 0.0:
            break
        while step > 1e-12:
            wn = w - step * grad
            gt, Dt = terms(wn)
            ft, _ = smooth(gt, mu)
            if ft <= f - 0.3 * step * gn:
                break
            step *= 0.5
        else:                      # no descent at this smoothing: sharpen and retry
            mu *= 0.5
            step = 1.0
            if mu < 1e-9:
                break
            continue
        w, g, D = wn, gt, Dt
        step *= 1.5
        if float(g.max()) < best:
            best, best_w = float(g.max()), w.copy()
        mu = max(mu * 0.98, 1e-9)
        if verbose and it % 25 == 0:
            print(f"  first-order it={it} gamma={g.max():.10f} best={best:.10f} mu={mu:.2e}")
    return best_w, best, iters


def find_optimal_weights(graph, method="auto", max_sdp=2048, tol=1e-8, info=None,
                         verbose=False):
    '''
    graph: list of pairs describing edges, e.g. [(0, 1), (0, 2), (1, 3)]
    Returns a list of corresponding weights and a convergence factor (lambda_2 of (I - L))
    (same contract as the reference, utils/fast_averaging.py:4-32)

    method: "auto" (the SDP up to ``max_sdp`` vertices, the Lanczos subgradient method above),
    "sdp", "subgradient" or "best_constant".  ``info`` (optional dict) receives the method
    used, the gamma of the best-constant weights it was certified against, and the iteration
    count.
    '''
    graph = [tuple(e) for e in graph]
    vertices = first_appearance_vertices(graph)
    n = len(vertices)
    rec = {} if info is None else info
    if n <= 1:
        rec.update(method="trivial", gamma_best_constant=0.0, iterations=0)
        return np.zeros(len(graph)), 0.0
    i, j, active = _edge_index(graph, vertices)
    ia, ja = i[active], j[active]
    wc = best_constant_weight(graph, vertices)
    # multi-edges share the pair's weight: start them at wc / multiplicity
    pair = np.minimum(ia, ja) * n + np.maximum(ia, ja)
    _, inv, cnt = np.unique(pair, return_inverse=True, return_counts=True)
    w0 = wc / cnt[inv]
    gamma_bc = _gamma(n, ia, ja, w0)
    if method == "auto":
        method = "sdp" if n <= max_sdp else "subgradient"
    if method == "sdp":
        wa, _, its = _solve_sdp(n, ia, ja, w0, tol=tol, verbose=verbose)
    elif method == "subgradient":
        wa, _, its = _solve_subgradient(n, ia, ja, w0, verbose=verbose)
    elif method == "best_constant":
        wa, its = w0, 0
    else:
        raise ValueError(f"unknown method {method!r}")
    w = np.zeros(len(graph))
    w[active] = wa
    gamma = _gamma(n, ia, ja, wa)
    rec.update(method=method, gamma_best_constant=gamma_bc, iterations=its,
               best_constant_weight=wc)
    return w, gamma


def _gamma(n, i, j, w):
    l2, _, ln, _ = _extreme_laplacian_eigs(n, i, j, w)
    return float(max(1.0 - l2, ln - 1.0))
