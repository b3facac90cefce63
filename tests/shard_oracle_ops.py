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
        sel = (slice(None), rows.numpy()) if X.dim() == 3 else (rows.numpy(),)  # tiled: every tile
        Xn = X.numpy()[sel]
        if G is not None:
            Xn = M.sgd_step(Xn, G.numpy()[sel], lr)
        out.copy_(torch.from_numpy(np.ascontiguousarray(Xn)))
        return out

    @staticmethod
    def _rows(A):
        """A column-tiled [tiles, rows, T] view as row-major [rows, tiles*T] numpy."""
        return np.ascontiguousarray(A.numpy().transpose(1, 0, 2).reshape(A.shape[1], -1))

    def mix(self, W, X, Y, G=None, lr=0.0, halo=None, lag=None, halo_blocks=None):
        if X.dim() == 3:    # column-tiled operands: the same round on their row-major images
            nt, T_ = X.shape[0], X.shape[2]
            Hr = None
            if halo is not None:
                blocks, off = [], 0
                for nb in (halo_blocks or [W.n_src - X.shape[1]]):
                    blocks.append(halo[off:off + nt * nb * T_].view(nt, nb, T_))
                    off += nt * nb * T_
                Hr = torch.from_numpy(np.concatenate([self._rows(b) for b in blocks]))
            Yr = torch.empty(Y.shape[1], nt * T_)
            self.mix(W, torch.from_numpy(self._rows(X)), Yr,
                     None if G is None else torch.from_numpy(self._rows(G)), lr, Hr, lag)
            Y.copy_(Yr.reshape(Y.shape[1], nt, T_).permute(1, 0, 2))
            return
        T = X.numpy()
        if lag is not None:     # lagged deviation of the input rows + sums of the stepped rows
            mean_prev, colsum, dsq = lag[:3]
            D = (T - mean_prev.numpy()).astype(np.float64)
            dsq.copy_(torch.from_numpy((D * D).sum(1).astype(np.float32)))
            if len(lag) > 3 and lag[3] is not None:   # the launch's max as well
                lag[3].copy_(torch.sqrt(dsq.max()).reshape(1))
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
