"""Drop-ins for the module-level kernels of ``tx_fast_hydrology/nutils.py``.

Same names and positional arguments as the reference; the routing and covariance kernels run on
the device (``libmcroute.so``), bit-identical to the reference walks:

* ``_ax_bu`` (nutils.py:64-89), ``_ax`` (:91-114): ``mc_ax_bu_f64`` (``_ax`` is ``_ax_bu`` with
  ``gamma = 0`` and ``q = 0``, which adds ``+ 0.0`` to a value that is never ``-0.0``).
* ``_apply_gain`` (:116-134): ``mc_cov_apply_gain``.
* ``_ap``/``_ap_par`` (:143-170), ``_aqat``/``_aqat_par`` (:172-214): ``mc_cov_ap`` /
  ``mc_cov_aqat`` on the covariance resident in HBM; results are written into ``out`` with the
  reference's memory layout (``_aqat_par`` returns the transposed view of ``out``).

``interpolate_sample(s)`` and ``has_same_index`` are the host-side input helpers (the routing
path interpolates in-kernel); ``numba_init_inflows`` is the host scatter of ``init_states``.
"""
from __future__ import annotations

import collections
import hashlib

import numpy as np

from . import engine


def interpolate_sample(x, xp, fp, method=1):
    """Row of ``fp`` at ``x``: linear (method 1) or nearest (0) between the bracketing rows
    ``searchsorted(xp, x) - 1`` and ``searchsorted(xp, x)``, clamped to the first / last row
    (nutils.py:5-39)."""
    n = xp.shape[0]
    ix = np.searchsorted(xp, x)
    if ix == 0:
        return fp[0]
    if ix >= n:
        return fp[n - 1]
    dx_0 = x - xp[ix - 1]
    dx_1 = xp[ix] - x
    if method == 1:
        frac = dx_0 / (dx_0 + dx_1)
        return (1 - frac) * fp[ix - 1] + frac * fp[ix]
    if method == 0:
        return fp[ix - 1] if abs(dx_0) <= abs(dx_1) else fp[ix]
    raise ValueError("method must be 0 (nearest) or 1 (linear)")


def interpolate_samples(xs, xp, fp, method=1):
    out = np.zeros((len(xs), fp.shape[1]), dtype=np.float64)
    for k, x in enumerate(xs):
        out[k, :] = interpolate_sample(x, xp, fp, method=method)
    return out


def has_same_index(known_index, dataframe_index):
    return len(known_index) == len(dataframe_index) and all(
        a == b for a, b in zip(known_index, dataframe_index))


def numba_init_inflows(a, indices, b):
    np.add.at(a, indices, b)


def _ax_bu(startnodes, endnodes, alpha, beta, chi, gamma, i_t_prev, o_t_prev, q_t_next,
           indegree):
    return engine.ax_bu(startnodes, endnodes, alpha, beta, chi, gamma, i_t_prev, o_t_prev,
                        q_t_next, indegree)


def _ax(startnodes, endnodes, alpha, beta, chi, i_t_prev, o_t_prev, indegree):
    zeros = np.zeros(np.asarray(endnodes).size)
    return engine.ax_bu(startnodes, endnodes, alpha, beta, chi, zeros, i_t_prev, o_t_prev,
                        zeros, indegree)


_GRAPHS = collections.OrderedDict()
_GRAPHS_MAX = 64


def topology_key(startnodes, endnodes, indegree):
    """(digest, int64 arrays) of a topology: headwaters, endnodes, indegree."""
    arrays = [np.ascontiguousarray(a, dtype=np.int64) for a in (startnodes, endnodes, indegree)]
    return hashlib.sha1(b"|".join(a.tobytes() for a in arrays)).hexdigest(), arrays


def cov_graph(startnodes, endnodes, indegree):
    """Cached ``engine.CovGraph`` of a topology (headwaters ``startnodes``).  The least recently
    used graph is closed beyond ``_GRAPHS_MAX`` topologies; ``KalmanFilter`` keeps its own graph
    on the instance (da.py), so many bound filters do not cycle this cache."""
    key, arrays = topology_key(startnodes, endnodes, indegree)
    graph = _GRAPHS.get(key)
    if graph is None:
        while len(_GRAPHS) >= _GRAPHS_MAX:
            _GRAPHS.popitem(last=False)[1].close()
        graph = _GRAPHS[key] = engine.CovGraph(arrays[1], arrays[2], arrays[0])
    else:
        _GRAPHS.move_to_end(key)
    return graph


def _apply_gain(startnodes, endnodes, gain, indegree):
    return cov_graph(startnodes, endnodes, indegree).apply_gain(gain)


def _propagate(P, out, startnodes, endnodes, alpha, beta, chi, indegree, both):
    P = np.asarray(P)
    if P.ndim != 2 or P.shape[0] != P.shape[1]:
        raise AssertionError("P must be square")
    graph = cov_graph(startnodes, endnodes, indegree)
    graph.set_coeffs(alpha, beta, chi)
    res = graph.aqat(P) if both else graph.ap(P)
    host = res.cpu().numpy()
    if both:
        out[...] = host.T        # the reference fills out^T and returns the view out.T
        return out.T
    out[...] = host
    return out


def _ap(P, out, startnodes, endnodes, alpha, beta, chi, indegree):
    return _propagate(P, out, startnodes, endnodes, alpha, beta, chi, indegree, False)


def _ap_par(P, out, startnodes, endnodes, alpha, beta, chi, indegree):
    return _propagate(P, out, startnodes, endnodes, alpha, beta, chi, indegree, False)


def _aqat(P, out, startnodes, endnodes, alpha, beta, chi, indegree):
    return _propagate(P, out, startnodes, endnodes, alpha, beta, chi, indegree, True)


def _aqat_par(P, out, startnodes, endnodes, alpha, beta, chi, indegree):
    return _propagate(P, out, startnodes, endnodes, alpha, beta, chi, indegree, True)
