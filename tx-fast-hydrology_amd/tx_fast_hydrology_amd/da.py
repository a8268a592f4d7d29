"""Kalman filtering of the routing state with the covariance resident on the device.

Drop-in for ``tx_fast_hydrology/da.py`` (``KalmanFilter`` :14-136, ``KalmanSmoother``
:139-264): same constructor, hooks, attributes and update formulas.  The n x n covariances
live in HBM as float64 CUDA tensors and every covariance product runs in ``libmcroute.so``
(``engine.CovGraph``):

* prior   ``P- = A P A^T + Q``        ``_aqat_par`` as two bit-exact level-set sweeps
                                      (``mc_cov_aqat``), ``+ Q`` on the device;
* gain    ``K = P-[:, s] (P-[s, s] + R)^-1``, ``gain = K dz``  (rocSOLVER LU + f64 MFMA GEMM);
* posterior ``P+ = P- - K P-[s, :]``  (f64 MFMA GEMM, ``mc_kf_update``);
* ``_apply_gain`` on the device (``mc_cov_apply_gain``), added to the host model state.

``P_t_next`` / ``P_t_prev`` read as numpy arrays (a device-to-host copy per access) and accept
numpy arrays or CUDA tensors; ``P_t_next_device`` is the resident tensor.  The measurement
interpolation and the innovation ``dz`` (m values) are host work, as in the reference.
Tolerance against the reference: the sweeps are bit-exact; the LU solve and GEMM summation
orders differ from numpy's, so K, gain and P agree to ~1e-12 relative (tests/test_gpu_kalman.py).
"""
from __future__ import annotations

import copy
import datetime as _dt
import logging
import weakref

import numpy as np
import pandas as pd

from . import engine
from .callbacks import BaseCallback
from .nutils import interpolate_sample, topology_key

logger = logging.getLogger(__name__)

# filter -> (topology digest, its CovGraph); entries vanish with their filter
_FILTER_GRAPHS = weakref.WeakKeyDictionary()


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("the device Kalman filter needs a GPU (torch.cuda is not available)")
    return torch


def _to_device(P):
    torch = _torch()
    if isinstance(P, torch.Tensor):
        return P.to(device="cuda", dtype=torch.float64).contiguous()
    return torch.as_tensor(np.ascontiguousarray(P, dtype=np.float64), device="cuda")


def _to_host(P):
    return P.cpu().numpy()


class KalmanFilter(BaseCallback):
    """Linear Kalman filter on the routing state (reference ``da.py:14-136``).

    ``measurements``: DataFrame of gauge observations (UTC index, columns = reach ids of the
    model); ``Q_cov`` (n x n), ``R_cov`` (m x m), ``P_t_init`` (n x n).  The analysis runs at
    the simulation start and after every step while the model time is at or before the last
    measurement time.
    """

    def __init__(self, model, measurements, Q_cov, R_cov, P_t_init):
        self.model = model
        self.measurements = measurements
        self.Q_cov = Q_cov
        self.R_cov = R_cov
        self.P_t_next = P_t_init
        self.P_t_prev = P_t_init
        self.reach_ids = model.reach_ids
        self.gage_reach_ids = measurements.columns
        self.datetime = copy.deepcopy(model.datetime)
        self.num_measurements = measurements.shape[1]
        assert isinstance(measurements.index, pd.DatetimeIndex)
        assert measurements.index.tz == _dt.timezone.utc
        assert np.isin(measurements.columns, self.reach_ids).all()
        position = pd.Series(np.arange(len(self.reach_ids)), index=self.reach_ids)
        reach_indices = position.loc[self.gage_reach_ids].values.astype(int)
        s = np.zeros(model.n, dtype=bool)
        s[reach_indices] = True
        self.s = s
        # gauges in reach order, as the boolean mask selects them (da.py:37-44)
        order = np.argsort(reach_indices)
        if not (order == np.arange(self.num_measurements)).all():
            logger.warning("Measurement indices not sorted. Permuting columns...")
        self.reach_indices = reach_indices[order]
        self.measurements = self.measurements.iloc[:, order]
        self.R_cov = self.R_cov[order, :][:, order]
        self.saved_states = {}
        self.save_state()

    # -- covariances on the device ---------------------------------------------------------------
    @property
    def P_t_next(self):
        return _to_host(self._P_next)

    @P_t_next.setter
    def P_t_next(self, P):
        self._P_next = _to_device(P)

    @property
    def P_t_next_device(self):
        return self._P_next

    @property
    def P_t_prev(self):
        return _to_host(self._P_prev)

    @P_t_prev.setter
    def P_t_prev(self, P):
        self._P_prev = _to_device(P)

    @property
    def Q_cov(self):
        return _to_host(self._Q)

    @Q_cov.setter
    def Q_cov(self, Q):
        self._Q = _to_device(Q)

    # -- hooks -----------------------------------------------------------------------------------
    def __on_simulation_start__(self):
        if self.model.datetime > self.latest_timestamp:
            return None
        return self.filter()

    def __on_step_end__(self):
        if self.model.datetime > self.latest_timestamp:
            return None
        return self.filter()

    def __idle_steps__(self):
        # __on_step_end__ filters only while the model time is at or before the last
        # observation; model time only grows during a simulation
        return self.model.datetime > self.latest_timestamp

    @property
    def latest_measurement(self):
        return self.measurements.iloc[-1, :].values

    @property
    def latest_timestamp(self):
        return self.measurements.index[-1]

    def interpolate_input(self, datetime, method="linear"):
        codes = {"linear": 1, "nearest": 0}
        if method not in codes:
            raise ValueError
        times = self.measurements.index.astype(int).astype(float).values
        return interpolate_sample(float(datetime.value), times, self.measurements.values,
                                  method=codes[method])

    def _observed(self, datetime):
        return self.interpolate_input(datetime)

    def save_state(self):
        self.saved_states["datetime"] = self.datetime
        self.saved_states["P_t_next"] = self._P_next.clone()

    def load_state(self):
        self.datetime = self.saved_states["datetime"]
        self._P_next = self.saved_states["P_t_next"]

    # -- analysis --------------------------------------------------------------------------------
    def _graph(self):
        """This filter's CovGraph, rebuilt only when the model topology changes.  Kept in a
        weak map keyed by the filter (not in __dict__), so copies build their own handle and many
        bound filters (one per sub-basin, app.py:129-145) never evict each other."""
        m = self.model
        key, arrays = topology_key(m.startnodes[m.indegree == 0], m.endnodes, m.indegree)
        held = _FILTER_GRAPHS.get(self)
        if held is None or held[0] != key:
            if held is not None:
                held[1].close()
            held = (key, engine.CovGraph(arrays[1], arrays[2], arrays[0]))
            _FILTER_GRAPHS[self] = held
        graph = held[1]
        graph.set_coeffs(m.alpha, m.beta, m.chi)
        return graph

    def _analysis(self):
        """(prior P-, posterior P+, K, gain, dz, i_prior, o_prior) for the current model time."""
        model = self.model
        graph = self._graph()
        Z = self._observed(model.datetime)
        dz = Z - model.o_t_next[self.s]
        P_prior = graph.aqat(self._P_next, self._Q)
        P_post = graph.empty()
        P_post, K, gain = graph.kf_update(self.reach_indices, self.R_cov, dz, P_prior, P_post)
        return graph, P_prior, P_post, K, gain, dz

    def filter(self):
        """da.py:91-136 after a step: prior, gain, posterior, state update."""
        model = self.model
        P_prev = self._P_next
        i_t_next, o_t_next = model.i_t_next, model.o_t_next
        graph, _, P_post, K, gain, dz = self._analysis()
        i_gain, o_gain = graph.apply_gain(gain)
        i_t_next += i_gain
        o_t_next += o_gain
        model.i_t_next = i_t_next
        model.o_t_next = o_t_next
        self._P_next = P_post
        self._P_prev = P_prev
        self.K = K
        self.dz = dz
        self.gain = gain
        self.datetime = model.datetime


class KalmanSmoother(KalmanFilter):
    """Kalman filter that keeps every prior / posterior and runs the Rauch-Tung-Striebel
    smoother at the simulation end (reference ``da.py:139-264``).  ``P_f`` / ``P_p`` / ``P_s``
    map timestamps to device tensors; ``o_hat_s`` / ``i_hat_s`` are DataFrames as in the
    reference."""

    def __init__(self, model, measurements, Q_cov, R_cov, P_t_init):
        super().__init__(model, measurements, Q_cov, R_cov, P_t_init)
        self.N = len(measurements) - 1
        t0 = model.datetime
        self.datetimes = [t0]
        self.i_hat_f = {t0: model.i_t_next.copy()}
        self.o_hat_f = {t0: model.o_t_next.copy()}
        self.i_hat_p = {t0: model.i_t_next.copy()}
        self.o_hat_p = {t0: model.o_t_next.copy()}
        self.P_f = {t0: self._P_next.clone()}
        self.P_p = {t0: self._P_next.clone()}
        self.i_hat_s = None
        self.o_hat_s = None

    def __on_simulation_end__(self):
        return self.smooth()

    def _observed(self, datetime):
        # the smoother reads the measurement row at the model time (da.py:190)
        return self.measurements.loc[datetime].values

    def filter(self):
        """da.py:170-218: the filter step, keeping the prior and posterior estimates."""
        model = self.model
        P_prev = self._P_next
        i_prior, o_prior = model.i_t_next, model.o_t_next
        graph, P_prior, P_post, K, gain, dz = self._analysis()
        i_gain, o_gain = graph.apply_gain(gain)
        i_t_next = i_prior + i_gain
        o_t_next = o_prior + o_gain
        model.i_t_next = i_t_next
        model.o_t_next = o_t_next
        self._P_prev = P_prev
        self._P_next = P_post
        t = model.datetime
        self.i_hat_f[t] = i_t_next
        self.i_hat_p[t] = i_prior
        self.o_hat_f[t] = o_t_next
        self.o_hat_p[t] = o_prior
        self.P_p[t] = P_prior
        self.P_f[t] = P_post
        self.datetimes.append(t)
        self.K = K
        self.dz = dz
        self.gain = gain
        self.datetime = t

    def smooth(self):
        """Backward pass (da.py:220-264): J = (P_p[t+1]^-1 A P_f[t])^T,
        x_s[t] = x_f[t] + J (x_s[t+1] - x_p[t+1]), P_s[t] = P_f[t] + J (P_s[t+1] - P_p[t+1])."""
        from . import engine
        graph = self._graph()
        times = self.datetimes
        last = self.datetime
        P_s = {last: self.P_f[last]}
        i_s = {last: self.i_hat_f[last]}
        o_s = {last: self.o_hat_f[last]}
        for k in reversed(range(len(times) - 1)):
            t, t1 = times[k], times[k + 1]
            P_s[t], i_s[t], o_s[t] = engine.ks_step(
                graph, self.P_f[t], self.P_p[t1], P_s[t1], self.i_hat_f[t], self.i_hat_p[t1],
                i_s[t1], self.o_hat_f[t], self.o_hat_p[t1], o_s[t1])
        i_frame = pd.DataFrame.from_dict(i_s, orient="index")
        i_frame.columns = self.model.reach_ids
        o_frame = pd.DataFrame.from_dict(o_s, orient="index")
        o_frame.columns = self.model.reach_ids
        self.i_hat_s = i_frame
        self.o_hat_s = o_frame
        self.P_s = P_s
