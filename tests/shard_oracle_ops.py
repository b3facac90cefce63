"""CPU stand-in for the device ops of a shard, built on the oracle (TEST INFRASTRUCTURE ONLY):
lets the multi-process (gloo) tests exercise the real halo protocol of sharding.HaloShard."""
import numpy as np
import torch

from oracle import cref
from oracle import mixer_ref as M


class OracleCsr:
    def __init__(self, csr):
        self.csr = csr
        self.n_rows, self.n_src = csr.n_rows, csr.n_src


class OracleOps:
    def __init__(self):
        pass

    def csr(self, csr):
        return OracleCsr(csr)

    def step_rows(self, X, rows, out, G=None, lr=0.0):
        Xn = X.numpy()[rows.numpy()]
        if G is not None:
            Xn = M.sgd_step(Xn, G.numpy()[rows.numpy()], lr)
        out.copy_(torch.from_numpy(np.ascontiguousarray(Xn)))
        return out

    def mix(self, W, X, Y, G=None, lr=0.0, halo=None, lag=None):
        T = X.numpy()
        if lag is not None:     # lagged deviation of the input rows + sums of the stepped rows
            mean_prev, colsum, dsq = lag
            D = (T - mean_prev.numpy()).astype(np.float64)
            dsq.copy_(torch.from_numpy((D * D).sum(1).astype(np.float32)))
        if G is not None:
            T = M.sgd_step(T, G.numpy(), lr)
        if lag is not None:
            colsum.copy_(torch.from_numpy(T.astype(np.float64).sum(0).astype(np.float32)))
        if halo is not None:
            T = np.concatenate([T, halo.numpy()])
        c = W.csr
        out = M.mix_once(np.ascontiguousarray(T), c.rowptr, c.col, c.w)
        Y.copy_(torch.from_numpy(out[:W.n_rows]))

    def column_sum(self, X):
        Xn = X.numpy()
        s = Xn[0].copy()
        for r in range(1, Xn.shape[0]):
            s = s + Xn[r]
        return torch.from_numpy(s)

    def deviation(self, X, mean):
        d = cref.deviation_sq(X.numpy(), mean.numpy().astype(np.float32))
        dsq = torch.from_numpy(d.astype(np.float32))
        return dsq, torch.sqrt(dsq.max()).reshape(1)
