"""Fastest-distributed-linear-averaging weights (reference: utils/fast_averaging.py:4-32).

The reference states the FDLA SDP (Xiao & Boyd, 2004) for cvxpy:

    minimise  gamma   s.t.  -gamma I <= I - L(w) - 11^T/n <= gamma I,   L(w) >= 0,
    L(w) = A diag(w) A^T   (A: vertex-edge incidence, vertices numbered by first appearance)

and returns ``(w in edge-list order, gamma)``.  cvxpy is not available here (nor on the GPU box),
so this module solves the same SDP with a small primal barrier method, host-side, as the
north star prescribes ("the fast-averaging weight optimisation stays on the host").

Working in the (n-1)-dimensional complement of the all-ones vector (Q^T L Q, Q orthonormal)
removes the trivial eigenvalue: with b_e = Q^T a_e, L~(w) = sum_e w_e b_e b_e^T and the
constraints become  (gamma - 1) I + L~ >= 0,  (gamma + 1) I - L~ >= 0,  L~ >= 0.  Each constraint
derivative is rank one, so the barrier gradient and Hessian are K = B^T F^-1 B and K o K, and a
Newton step costs O(n^3 + m^2 n).  Self-loop edges have a zero incidence column; their weight is
free in the reference and returned as 0 here.

Large graphs (n > ``max_dense``): the dense solve gets slow, so ``find_optimal_weights`` falls
back to the best-constant weight 2 / (lambda_2 + lambda_n) of the unweighted Laplacian (optimal
for edge-transitive graphs such as rings and tori) unless ``force_sdp`` is set.
"""
import numpy as np

from ..graph import first_appearance_vertices


def _incidence(graph, vertices):
    index = {v: i for i, v in enumerate(vertices)}
    n, m = len(vertices), len(graph)
    A = np.zeros((n, m))
    for i, (u, v) in enumerate(graph):
        if u != v:
            A[index[u], i] = 1.0
            A[index[v], i] = -1.0
    return A


def _complement_basis(n):
    """Orthonormal basis of the complement of the all-ones vector (n x (n-1))."""
    Q, _ = np.linalg.qr(np.column_stack([np.ones(n) / np.sqrt(n), np.eye(n)[:, :n - 1]]))
    return Q[:, 1:]


def spectral_gamma(graph, weights, vertices=None):
    """gamma(w) = ||I - L(w) - 11^T/n||_2 (the convergence factor the reference returns)."""
    vertices = first_appearance_vertices(graph) if vertices is None else vertices
    A = _incidence(graph, vertices)
    n = len(vertices)
    Mt = np.eye(n) - A @ np.diag(np.asarray(weights, float)) @ A.T - np.ones((n, n)) / n
    return float(np.max(np.abs(np.linalg.eigvalsh(Mt))))


def _solve_fdla(B, tol=1e-10, max_newton=200):
    """Barrier method for  min gamma  over (w, gamma)  (B: (n-1) x m, rank-one generators)."""
    k, m = B.shape
    active = np.linalg.norm(B, axis=0) > 0
    I = np.eye(k)
    # strictly feasible start: small uniform weights keep L~ > 0 (connected graph) and
    # I - L~ inside the unit ball; gamma above the spectral radius
    w = np.where(active, 1.0 / (2.0 * max(1.0, float(np.max(np.sum(np.abs(B @ B.T), 1))))), 0.0)

    def Lt(w):
        return (B * w) @ B.T

    ev = np.linalg.eigvalsh(I - Lt(w))
    gamma = float(np.max(np.abs(ev))) + 0.5
    x = np.concatenate([w, [gamma]])
    nb = 3 * k  # barrier parameter (sum of the LMI sizes)

    def pieces(x):
        w, g = x[:m], x[m]
        L = Lt(w)
        return [((g - 1.0) * I + L, 1.0, 1.0), ((g + 1.0) * I - L, -1.0, 1.0), (L, 1.0, 0.0)]

    def feasible(x):
        for F, _, _ in pieces(x):
            try:
                np.linalg.cholesky(F)
            except np.linalg.LinAlgError:
                return False
        return True

    def phi(x, t):
        val = t * x[m]
        for F, _, _ in pieces(x):
            val -= 2.0 * np.sum(np.log(np.diag(np.linalg.cholesky(F))))
        return val

    t = 1.0
    while True:
        for _ in range(max_newton):
            g = np.zeros(m + 1)
            g[m] = t
            H = np.zeros((m + 1, m + 1))
            for F, sw, sg in pieces(x):
                Fi = np.linalg.inv(F)
                FiB = Fi @ B
                K = B.T @ FiB
                g[:m] -= sw * np.diag(K)
                H[:m, :m] += K * K
                if sg:
                    g[m] -= np.trace(Fi)
                    H[m, m] += np.sum(Fi * Fi)
                    cross = sw * np.einsum("ij,ij->j", FiB, FiB)
                    H[:m, m] += cross
                    H[m, :m] += cross
            H[:m, :m][np.ix_(~active, ~active)] += np.eye(int((~active).sum()))
            g[:m][~active] = 0.0
            try:
                dx = -np.linalg.solve(H, g)
            except np.linalg.LinAlgError:
                dx = -np.linalg.lstsq(H, g, rcond=None)[0]
            lam2 = float(-g @ dx)
            if lam2 / 2.0 <= 1e-12:
                break
            s, f0 = 1.0, phi(x, t)
            while s > 1e-12:
                xn = x + s * dx
                if feasible(xn) and phi(xn, t) <= f0 - 0.25 * s * lam2:
                    break
                s *= 0.5
            x = x + s * dx
        if nb / t < tol:
            break
        t *= 20.0
    return x[:m], x[m]


def find_optimal_weights(graph, max_dense=400, force_sdp=False, tol=1e-10):
    '''
    graph: list of pairs describing edges, e.g. [(0, 1), (0, 2), (1, 3)]
    Returns a list of corresponding weights and a convergence factor (lambda_2 of (I - L))
    (same contract as the reference, utils/fast_averaging.py:4-32)
    '''
    graph = [tuple(e) for e in graph]
    vertices = first_appearance_vertices(graph)
    n = len(vertices)
    if n <= 1:
        return np.zeros(len(graph)), 0.0
    A = _incidence(graph, vertices)
    if n > max_dense and not force_sdp:
        L0 = A @ A.T
        L0 = np.where(np.abs(L0) > 0, np.sign(L0) * np.minimum(np.abs(L0), 1), 0)
        np.fill_diagonal(L0, 0)
        L0 = np.diag(-L0.sum(1)) + L0
        ev = np.linalg.eigvalsh(L0)
        wc = 2.0 / (ev[1] + ev[-1])
        w = np.where(np.any(A != 0, axis=0), wc, 0.0)
        return w, spectral_gamma(graph, w, vertices)
    Q = _complement_basis(n)
    B = Q.T @ A
    w, gamma = _solve_fdla(B, tol=tol)
    w = np.where(np.any(A != 0, axis=0), w, 0.0)
    return w, float(spectral_gamma(graph, w, vertices))
