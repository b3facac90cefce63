"""Drop-in ``Mixer`` (reference: utils/consensus_simple/mixer.py:1-84) on the HIP engine.

Same constructor, methods, return values, logging and stopping rule as the reference; the
difference is where the work runs.  Per ``mix()`` call the models are flattened once into a
device matrix X[N, P] (rows in ``topology`` key order, mixer.py:26/69); each round is one
``dl_mix_round`` launch (the reference's ``_mix_params_once`` fold, :43-49, bit-identical in
fp32), and when ``eps`` is given the same launch also produces the per-agent deviation
(:51-66) so the stop test costs one 4-byte readback per round.  With ``eps=None`` the ``times``
rounds have nothing in between, so they run as ONE ``dl_mix_rounds`` pass (every round on
LDS-resident column tiles, bit-identical to ``times`` single rounds).  The results are written
back into the models once at the end (:34-35, 71-76).
"""
import numpy as np
import torch

from ... import engine as _engine
from ...graph import from_topology

__all__ = ["Mixer", "basic_deviation_metric"]


def basic_deviation_metric(p1, p2):
    """mixer.py:5-6 (used only when a caller passes it, or a custom metric, explicitly)."""
    return np.linalg.norm(p1 - p2)


def _default_device():
    if not torch.cuda.is_available():
        raise RuntimeError("the HIP Mixer needs a GPU (no CPU fallback by design)")
    return torch.device("cuda", torch.cuda.current_device())


class Mixer(object):
    def __init__(self, models, topology, logger, dev_metric=None, device=None):
        self.models = models
        self.topology = topology
        self.logger = logger
        self.dev_metric = basic_deviation_metric
        self._custom_metric = dev_metric is not None
        if dev_metric is not None:
            self.dev_metric = dev_metric
        self._device = torch.device(device) if device is not None else None
        self._ws = None

    # ------------------------------------------------------------------ public API (:18-38)
    def mix(self, times=1, eps=None):
        if len(self.topology) <= 1:
            return 0

        self.logger.debug('Mixer start with times= {}, eps= {}'.format(times, eps))

        with torch.no_grad():
            times_done = 0
            W = self._device_csr()
            X = self._flatten_all()
            Y = torch.empty_like(X)
            fused_dev = eps is not None and not self._custom_metric
            dev_sq = torch.empty(X.shape[0], dtype=torch.float32, device=X.device)
            dev_max = torch.empty(1, dtype=torch.float32, device=X.device)

            stopping_criterion = self._update_stopping_criterion(X, times_done, times, eps)
            if not stopping_criterion and eps is None:
                # times rounds, no stop test in between: one pass over HBM (rows padded with
                # zero columns to whole tiles; zeros mix to zeros)
                P = X.shape[1]
                Pp = -(-P // 64) * 64
                Xp = torch.nn.functional.pad(X, (0, Pp - P)) if Pp != P else X
                Yp = torch.empty_like(Xp)
                if _engine.mix_rounds(W, Xp, Yp, times, workspace=self._wspace()):
                    X, times_done = Yp[:, :P], int(times)
                    stopping_criterion = True
            while not stopping_criterion:
                _engine.mix_round(W, X, Y, dev_sq=dev_sq if fused_dev else None,
                                  dev_max=dev_max if fused_dev else None, workspace=self._wspace())
                X, Y = Y, X
                times_done += 1
                stopping_criterion = self._update_stopping_criterion(
                    X, times_done, times, eps, fused=(dev_max if fused_dev else None))

            self._write_back(X)

        self.logger.debug('Mixer finished with {} times'.format(times_done))
        return times_done

    def get_parameters_deviation(self):
        """mixer.py:78-80: dict agent -> ||x_a - mean|| (np.float32, like np.linalg.norm)."""
        with torch.no_grad():
            X = self._flatten_all()
            return self._get_deviation_dict(X)

    def get_max_parameters_std(self):
        """mixer.py:82-84 (intended semantics: max over params of the population std over
        agents; the reference line itself fails on numpy>=2)."""
        with torch.no_grad():
            X = self._flatten_all()
            return np.float32(_engine.max_column_std(X).item())

    # ------------------------------------------------------------------ internals
    def _update_stopping_criterion(self, X, times_done, max_times, eps, fused=None):
        """mixer.py:40-41; the deviation is only evaluated when eps is set (short circuit)."""
        if eps is None:
            return times_done >= max_times
        if fused is not None:
            max_dev = np.float32(fused.item())
            self.logger.debug('Mixer calculate max deviation= {}'.format(max_dev))
        else:
            max_dev = self._get_max_deviation(X)
        return max_dev < eps and times_done >= max_times

    def _get_max_deviation(self, X):
        devs_list = self._get_deviation_dict(X).values()
        max_dev = max(devs_list)
        self.logger.debug('Mixer calculate max deviation= {}'.format(max_dev))
        return max_dev

    def _get_deviation_dict(self, X):
        keys = list(self.topology)
        if len(keys) <= 1:
            return {agent: 0.0 for agent in keys}
        if self._custom_metric:
            # arbitrary user metric on numpy vectors: mean on the GPU, metric on the host
            mean = torch.empty(X.shape[1], dtype=torch.float32, device=X.device)
            _engine.deviation(X, mean_out=mean, workspace=self._wspace())
            Xh, mh = X.cpu().numpy(), mean.cpu().numpy()
            return {agent: self.dev_metric(Xh[i], mh) for i, agent in enumerate(keys)}
        dev_sq, _ = _engine.deviation(X, workspace=self._wspace())
        d = np.sqrt(dev_sq.cpu().numpy().astype(np.float32))
        return {agent: d[i] for i, agent in enumerate(keys)}

    def _device_csr(self):
        csr = from_topology(self.topology)
        return _engine.DeviceCsr(csr, self._dev())

    def _dev(self):
        if self._device is None:
            self._device = _default_device()
        return self._device

    def _wspace(self):
        if self._ws is None:
            self._ws = _engine.Workspace(self._dev())
        return self._ws

    def _flatten_all(self):
        rows = [self._get_flatten_model_params(self.models[agent]) for agent in self.topology]
        return torch.stack(rows).contiguous()

    def _get_flatten_model_params(self, model):
        """mixer.py:68-69, kept on the device."""
        dev = self._dev()
        return torch.cat([p.data.to(device=dev, dtype=torch.float32).view(-1)
                          for p in model.parameters()])

    def _load_flatten_params_to_model(self, model, params):
        """mixer.py:71-76."""
        used_params = 0
        for p in model.parameters():
            cnt_params = p.numel()
            p.data.copy_(params[used_params:used_params + cnt_params].view(p.shape).to(p.dtype))
            used_params += cnt_params

    def _write_back(self, X):
        for i, agent in enumerate(self.topology):
            self._load_flatten_params_to_model(self.models[agent], X[i])
