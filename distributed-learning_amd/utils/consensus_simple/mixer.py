"""Drop-in ``Mixer`` (reference: utils/consensus_simple/mixer.py:1-84) on the HIP engine.

Same constructor, methods, return values, logging and stopping rule as the reference; the
difference is where the work runs.  Per ``mix()`` call the models are flattened once into a
device matrix X[N, P] (rows in ``topology`` key order, mixer.py:26/69).  When two copies of X
fit one workgroup's LDS (the reference's own use: small models on a handful of agents) the
whole loop -- rounds, deviation, stop test -- is ONE ``dl_mix_until`` launch and one readback
of the round count; the reference's per-evaluation debug log is replayed from the device's
trace of max deviations.  Otherwise each round is one
``dl_mix_round`` launch (the reference's ``_mix_params_once`` fold, :43-49, bit-identical in
fp32), and when ``eps`` is given the same launch also produces the per-agent deviation
(:51-66) so the stop test costs one 4-byte readback per round -- or, when the graph fits the
traced multi-round kernel (<= 1024 agents, or up to 4096 of a register-cached regular graph;
doubly stochastic W), K rounds run in one HBM pass
that also returns their K per-round max deviations (``dl_mix_rounds_trace``), and the stop
round is found on the host.  With ``eps=None`` the ``times``
rounds have nothing in between, so they run as ONE ``dl_mix_rounds`` pass (every round on
LDS-resident column tiles, bit-identical to ``times`` single rounds).  The results are written
back into the models once at the end (:34-35, 71-76).
"""
import logging
import math

import numpy as np
import torch

from ... import engine as _engine
from ...graph import from_topology, lds_slot_order_native, permuted

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
        self._csr = None   # (host Csr, DeviceCsr) of the last topology seen
        self._ordered = None   # (host Csr, n_params, DeviceCsr in slot order or None, agents)

    # ------------------------------------------------------------------ public API (:18-38)
    def mix(self, times=1, eps=None):
        if len(self.topology) <= 1:
            return 0

        self.logger.debug('Mixer start with times= {}, eps= {}'.format(times, eps))

        with torch.no_grad():
            times_done = 0
            W = self._device_csr()
            agents = None
            if eps is None and times >= 1 and not (
                    not self._custom_metric and _engine.until_fits(W, self._n_params())):
                # mix(times) with no stop test on a large X: when the multi-round pass will run,
                # the rows go into the device matrix in an LDS slot order (every agent keeps its
                # CSR entry order, so its bits are the same; the pass gathers neighbours with
                # fewer bank conflicts)
                W_ord, agents = self._ordered_csr(self._n_params())
                if agents is not None:
                    W = W_ord
            X = self._flatten_all(agents)
            if not self._custom_metric and _engine.until_fits(W, X.shape[1]):
                times_done = self._mix_resident(W, X, times, eps)
                self._write_back(X)
                self.logger.debug('Mixer finished with {} times'.format(times_done))
                return times_done
            Y = torch.empty_like(X)
            fused_dev = eps is not None and not self._custom_metric
            dev_sq = torch.empty(X.shape[0], dtype=torch.float32, device=X.device)
            dev_max = torch.empty(1, dtype=torch.float32, device=X.device)

            stopping_criterion = self._update_stopping_criterion(X, times_done, times, eps)
            if not stopping_criterion and fused_dev:
                X, times_done, stopping_criterion = self._mix_traced(W, X, times, eps)
            P = X.shape[1]
            # above _TRACE_TILED_ABOVE agents the remaining rounds run on a column-tiled copy of X
            # (a row-major tile of all agents is a short segment of every row)
            T = None
            if not stopping_criterion and (fused_dev or eps is None):
                T = self._loop_tile_cols(W, P)
            tl = None
            if T:
                tl = (P, T)
                X = _engine.to_tiled(X, T)
                Y = torch.empty_like(X)
            if not stopping_criterion and eps is None:
                # times rounds, no stop test in between: one pass over HBM (rows padded with
                # zero columns to whole tiles; zeros mix to zeros)
                if tl:
                    Yt = torch.empty_like(X)
                    if _engine.mix_rounds(W, X, Yt, math.ceil(times), workspace=self._wspace(),
                                          tiled=tl):
                        X, times_done = Yt, math.ceil(times)
                        stopping_criterion = True
                else:
                    Pp = -(-P // 64) * 64
                    Xp = torch.nn.functional.pad(X, (0, Pp - P)) if Pp != P else X
                    Yp = torch.empty_like(Xp)
                    if _engine.mix_rounds(W, Xp, Yp, math.ceil(times), workspace=self._wspace()):
                        X, times_done = Yp[:, :P], math.ceil(times)
                        stopping_criterion = True
            while not stopping_criterion:
                _engine.mix_round(W, X, Y, dev_sq=dev_sq if fused_dev else None,
                                  dev_max=dev_max if fused_dev else None, workspace=self._wspace(),
                                  tiled=tl)
                X, Y = Y, X
                times_done += 1
                stopping_criterion = self._update_stopping_criterion(
                    X, times_done, times, eps, fused=(dev_max if fused_dev else None))
            if tl:
                X = _engine.from_tiled(X, P)

            self._write_back(X, agents)

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
    _UNTIL_ROUNDS = 4096   # rounds per dl_mix_until launch (bounds one launch; the loop re-enters)

    def _mix_resident(self, W, X, times, eps):
        """mixer.py:27-32 on the device (dl_mix_until), X updated in place.  A launch cut by the
        round cap is continued with the remaining ``times``; its first evaluation repeats the
        previous launch's last one, so that log line is not repeated."""
        status = torch.empty(2, dtype=torch.int32, device=X.device)
        trace = None
        if eps is not None:
            trace = torch.empty(self._UNTIL_ROUNDS + 1, dtype=torch.float32, device=X.device)
        log = eps is not None and self.logger.isEnabledFor(logging.DEBUG)
        done, first = 0, True
        while True:
            _engine.mix_until(W, X, X, max(math.ceil(times) - done, 0), eps, self._UNTIL_ROUNDS,
                              status, trace)
            n, stopped = status.tolist()
            if log:
                for d in trace[:n + 1].tolist()[0 if first else 1:]:
                    self.logger.debug('Mixer calculate max deviation= {}'.format(np.float32(d)))
            done += n
            first = False
            if stopped:
                return done

    _TRACE_MIN_ROUNDS = 4     # below this many rounds per traced pass the round loop is as good
    _TRACE_MAX_ROUNDS = 256   # rounds per traced pass (LDS permitting)

    # The traced deviations take the column mean as a tree sum (and reuse the pass input's mean:
    # mean(W x) = mean(x)) while the reference takes numpy's row-order mean every round
    # (mixer.py:61-65): they agree to ~1e-5 relative or the mean-rounding floor.
    # A traced value that close to eps could flip the integer round count, so that round is
    # re-evaluated with the row-order two-pass deviation (dl_column_sum, as dl_mix_until does).
    _TIE_RTOL = 2e-5

    # The one-image traced kernel at 4 agents per thread (mix_trace_irr_kernel: irregular graphs,
    # or a W that is not doubly stochastic, above 2048 agents; 4 rounds per pass) keeps four
    # agents' register heads and spills, so per round it costs more than one fused round launch
    # once the columns outweigh the launch: 4096 agents, scripts/trace_irr_probe.py
    # (profiles/r11/trace_irr_probe.log), traced / loop rounds per second: Barabasi-Albert 3532 /
    # 5552 at 2^14 columns and 247 / 514 at 2^18, a row-stochastic graph 3536 / 3851 and 245 / 314
    # (the loop's fixed cost ~65 us a round against ~31, its per-column cost 11.9 ns against 15.4:
    # even near 9.7k columns).  Above this many columns such graphs take the round loop.
    _TRACE_IRR4_MAX_COLS = 8192
    _TRACE_IRR4_ROUNDS = 4

    # above this many agents the traced pass (mix_trace_wide_kernel: one 4-column chunk per step)
    # runs on a column-tiled copy of X: a row-major step reads a 16-byte segment of every row
    # (c4 torus, 4096 x 2^18: 486 rounds/s row-major against 2179 tiled, profiles/r10/trace4096)
    _TRACE_TILED_ABOVE = 1024

    def _loop_tile_cols(self, W, P):
        """Tile width of the column-tiled layout for the round loop above _TRACE_TILED_ABOVE
        agents (the LDS tile kernels: paths 1, 4, 5), else None (row-major)."""
        if W.n_rows <= self._TRACE_TILED_ABOVE or W.n_src != W.n_rows:
            return None
        plan = _engine.plan_shape(W, P, deviation=True, tile_cols=-1)
        return plan["tile_cols"] if plan["path"] in (1, 4, 5) and plan["tile_cols"] > 0 else None

    def _mix_traced(self, W, X, times, eps):
        """mixer.py:27-32 with eps set, in passes of K rounds (dl_mix_rounds_trace): each pass
        runs K rounds in one HBM pass and returns the K per-round max deviations, which are
        logged and tested in order exactly as the reference evaluates them after every round;
        a deviation within rounding of eps is re-evaluated on that round's iterate with the
        row-order mean (``_TIE_RTOL``).  When the stop round falls inside a pass, that many
        rounds are re-run from the pass's input (left intact).  Returns (X, times_done,
        stopped); stopped is False, with nothing done, when the traced kernel does not fit (the
        caller's round loop takes over).  Above ``_TRACE_TILED_ABOVE`` agents the passes run on
        a column-tiled copy of X (one conversion each way per call)."""
        P = X.shape[1]
        Pp = -(-P // 64) * 64
        cur = torch.nn.functional.pad(X, (0, Pp - P)) if Pp != P else X
        nxt = torch.empty_like(cur)
        # whether the traced kernel fits is decided before any layout copy: the
        # row-major plan has the tiled one's depth (one 4-column chunk per step above 1024 agents)
        K = min(_engine.trace_max_rounds(W, cur, nxt), self._TRACE_MAX_ROUNDS)
        if K < min(self._TRACE_MIN_ROUNDS, self._TRACE_MAX_ROUNDS):
            return X, 0, False
        if (W.n_rows > 2048 and K == self._TRACE_IRR4_ROUNDS and
                Pp > self._TRACE_IRR4_MAX_COLS):
            return X, 0, False
        tiled = None
        if W.n_rows > self._TRACE_TILED_ABOVE:
            tiled = (Pp, 4)
            cur = _engine.to_tiled(cur, 4)
            nxt = nxt.view(_engine.tiled_shape(W.n_rows, Pp, 4))   # same bytes, tiled shape
        trace = torch.empty(K, dtype=torch.float32, device=X.device)
        ws = self._wspace()
        done = 0
        floor = None
        while True:
            _engine.mix_rounds_trace(W, cur, nxt, K, trace, workspace=ws, tiled=tiled)
            stop_at = None
            for i, d in enumerate(trace.tolist()):
                max_dev = np.float32(d)
                gap = abs(float(max_dev) - float(eps))
                if gap <= 0.1 * abs(float(eps)):
                    if floor is None:
                        if W.doubly_stochastic:   # mean(W^k x) = mean(x): one column sum
                            ref = (_engine.column_sum(X) / X.shape[0]).abs().max()
                        else:   # a row-stochastic W keeps every mean inside X's entry range
                            ref = X.abs().max()
                        floor = 8.0 * np.sqrt(P) * float(np.finfo(np.float32).eps) * \
                            float(ref.item())
                    if gap <= self._TIE_RTOL * abs(float(eps)) + floor:
                        max_dev = self._recheck_deviation(W, cur, i + 1, P, tiled)
                self.logger.debug('Mixer calculate max deviation= {}'.format(max_dev))
                if max_dev < eps and done + i + 1 >= times:
                    stop_at = i + 1
                    break
            if stop_at is None:
                cur, nxt = nxt, cur
                done += K
                continue
            if stop_at < K:   # the same rounds again from the pass's input (bit-identical)
                nxt = self._rounds_from(W, cur, stop_at, ws, tiled)
            out = _engine.from_tiled(nxt, Pp) if tiled else nxt
            return out[:, :P], done + stop_at, True

    def _rounds_from(self, W, src, k, ws, tiled=None):
        """The iterate k rounds after ``src`` (bit-identical to k single rounds), src intact."""
        out = torch.empty_like(src)
        if _engine.mix_rounds(W, src, out, k, workspace=ws, tiled=tiled):
            return out
        bufs, a = (out, torch.empty_like(src)), src
        for j in range(k):
            _engine.mix_round(W, a, bufs[j % 2], workspace=ws, tiled=tiled)
            a = bufs[j % 2]
        return a

    def _recheck_deviation(self, W, src, k, P, tiled=None):
        """max_a ||x_a - mean|| of the iterate k rounds after src, with numpy's row-order column
        mean (mixer.py:61: dl_column_sum, then the division in fp32)."""
        Z = self._rounds_from(W, src, k, self._wspace(), tiled)
        if tiled:
            Z = _engine.from_tiled(Z, tiled[0])
        Z = Z[:, :P]
        mean = _engine.column_sum(Z) / Z.shape[0]
        _, dmax = _engine.deviation(Z, mean_in=mean, workspace=self._wspace())
        return np.float32(dmax.item())

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
        """The topology as a device CSR; re-uploaded only when the topology changed (the
        reference re-reads self.topology on every call, so it is re-derived every call)."""
        csr = from_topology(self.topology)
        if self._csr is not None:
            old = self._csr[0]
            if (np.array_equal(old.rowptr, csr.rowptr) and np.array_equal(old.col, csr.col) and
                    np.array_equal(old.w, csr.w) and old.n_src == csr.n_src):
                return self._csr[1]
        self._csr = (csr, _engine.DeviceCsr(csr, self._dev()))
        return self._csr[1]

    _SLOT_MOVES_PER_AGENT = 2000   # slot-order search moves (1024 agents: ~0.5 s, once)
    _SLOT_MOVES_MAX = 4_000_000    # cap: the search is host work spent before the first round
    _SLOT_MIN_AGENTS = 64          # below a few lane groups there is nothing to spread

    def _ordered_csr(self, n_params):
        """(DeviceCsr, agents) with the rows in dl_lds_slot_order's order for the multi-round
        kernel's agent-major images, or (None, None) when ordering cannot pay: the multi-round
        pass does not fit these sizes (dl_mix_rounds_plan_shape), the graph is irregular, or it
        is small.  The search uses the chunks per row of the plan the pass will run with, its
        moves are capped, and the result is cached per (topology, n_params);
        agents[slot] is the topology key of row slot."""
        self._device_csr()
        csr, W = self._csr
        key = (csr, int(n_params))
        if self._ordered is not None and self._ordered[0] is key[0] and \
                self._ordered[1] == key[1]:
            return self._ordered[2], self._ordered[3]
        W_ord, agents = None, None
        plan = _engine.rounds_plan_shape(W, -(-int(n_params) // 64) * 64)
        if plan is not None and csr.uniform_row_nnz and csr.n_rows >= self._SLOT_MIN_AGENTS:
            keys = list(self.topology)
            moves = min(self._SLOT_MOVES_PER_AGENT * csr.n_rows, self._SLOT_MOVES_MAX)
            order, _, _ = lds_slot_order_native(csr, plan["tile_cols"] // 4, moves=moves)
            W_ord = _engine.DeviceCsr(permuted(csr, order), self._dev())
            agents = [keys[a] for a in order]
        self._ordered = (key[0], key[1], W_ord, agents)
        return W_ord, agents

    def _n_params(self):
        return sum(p.numel() for p in self.models[next(iter(self.topology))].parameters())

    def _dev(self):
        if self._device is None:
            self._device = _default_device()
        return self._device

    def _wspace(self):
        if self._ws is None:
            self._ws = _engine.Workspace(self._dev())
        return self._ws

    def _flatten_all(self, agents=None):
        """X[N, P], rows in topology order (or in ``agents`` order): one concatenation of every
        parameter of every model (mixer.py:26/68-69)."""
        dev = self._dev()
        parts, sizes = [], []
        for agent in (self.topology if agents is None else agents):
            n = 0
            for p in self.models[agent].parameters():
                parts.append(p.data.to(device=dev, dtype=torch.float32).view(-1))
                n += p.numel()
            sizes.append(n)
        if len(set(sizes)) != 1:
            raise ValueError(f"models differ in parameter count: {sizes}")
        return torch.cat(parts).view(len(sizes), sizes[0])

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

    def _write_back(self, X, agents=None):
        """mixer.py:34-35 / 71-76 for every model, as one fused multi-tensor copy (row i belongs
        to agents[i], topology order by default)."""
        dst, src = [], []
        for i, agent in enumerate(self.topology if agents is None else agents):
            used = 0
            for p in self.models[agent].parameters():
                n = p.numel()
                dst.append(p.data)
                src.append(X[i, used:used + n].view(p.shape))
                used += n
        if dst and all(d.device == s.device for d, s in zip(dst, src)):
            torch._foreach_copy_(dst, src)
        else:
            for d, s in zip(dst, src):
                d.copy_(s)
