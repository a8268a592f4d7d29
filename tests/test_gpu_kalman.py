"""GPU parity of the full-covariance Kalman path (mc_cov_*, mc_kf_update, mc_ks_step) and of the
nutils drop-ins.

* ``_ap_par`` / ``_aqat_par`` / ``_apply_gain`` / ``_ax`` / ``_ax_bu``: BIT-EXACT against the
  golden vectors (the sweeps replay the reference walk with the same association and order) and
  against the oracle on larger random forests (LDS-resident and global-memory variants).
* ``KalmanFilter`` (g5) and ``KalmanSmoother`` (g11): the LU solve and the GEMMs sum in another
  order than numpy / OpenBLAS, so states, gains and covariances are compared with
  rtol 1e-9 (north-star tolerance 1e-6), covariance entries with atol 1e-9 on top.
"""
import numpy as np
import pandas as pd
import pytest

from api_helpers import golden_frame, golden_model
from oracle import oracle as orc
from tx_fast_hydrology_amd import nutils, synthetic
from tx_fast_hydrology_amd.da import KalmanFilter, KalmanSmoother

pytestmark = pytest.mark.gpu

RTOL = 1e-9
ATOL = 1e-9


def test_nutils_dropins_golden(golden):
    g = golden("g7_covariance.npz")
    end, deg = g["endnodes"], g["indegree"]
    heads = np.arange(end.size)[deg == 0]
    out = np.empty_like(g["P"])
    res = nutils._aqat_par(g["P"], out, heads, end, g["alpha"], g["beta"], g["chi"], deg)
    assert np.array_equal(res, g["aqat"])
    assert np.array_equal(out.T, g["aqat"])            # reference layout: out^T is returned
    res = nutils._ap_par(g["P"], np.empty_like(g["P"]), heads, end, g["alpha"], g["beta"],
                         g["chi"], deg)
    assert np.array_equal(res, g["ap"])
    ig, og = nutils._apply_gain(heads, end, g["gain"], deg)
    assert np.array_equal(ig, g["gain_i"]) and np.array_equal(og, g["gain_o"])
    ai, ao = nutils._ax(heads, end, g["alpha"], g["beta"], g["chi"], g["ip"], g["op"], deg)
    assert np.array_equal(ai, g["ax_i"]) and np.array_equal(ao, g["ax_o"])


@pytest.mark.parametrize("n", [700, 1500])      # staged (LDS) and global sweeps
def test_covariance_sweeps_random_forest(n):
    rng = np.random.default_rng(n)
    end = synthetic.river_network(n, 3, max(8, n // 20), rng)
    n = end.size
    start = np.arange(n)
    deg = orc.compute_indegree(start, end)
    heads = start[deg == 0]
    K, X, _ = synthetic.model_arrays(n, seed=1)
    a, b, c, _ = orc.muskingum_coeffs(K, X, 900.0)
    A = rng.normal(size=(n, n))
    P = A @ A.T / n
    want = orc.ap(P, heads, end, a, b, c, deg)
    got = nutils._ap_par(P, np.empty_like(P), heads, end, a, b, c, deg)
    assert np.array_equal(got, want)
    if n <= 1024:
        want = orc.aqat(P, heads, end, a, b, c, deg)
        got = nutils._aqat_par(P, np.empty_like(P), heads, end, a, b, c, deg)
        assert np.array_equal(got, want)


def _close(a, b, rtol=RTOL, atol=0.0):
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol)


def test_kalman_filter_golden(golden):
    g = golden("g5_kalman.npz")
    model = golden_model(g)
    df = golden_frame(g, model.reach_ids)
    gage_ids = [model.reach_ids[k] for k in g["gages"]]
    meas = pd.DataFrame(g["meas"], index=pd.DatetimeIndex(pd.to_datetime(g["meas_ns"], utc=True)),
                        columns=gage_ids)
    n = model.n
    Q = 2.0 * np.eye(n)
    kf = KalmanFilter(model, meas, Q, 1e-2 * np.eye(6), Q.copy())
    assert np.array_equal(kf.reach_indices, g["reach_indices"])
    model.bind_callback(kf, key="kf")
    rec = {"K": [], "gain": [], "dz": [], "pdiag": []}
    orig = kf.filter

    def wrapped():
        orig()
        rec["K"].append(kf.K.copy())
        rec["gain"].append(kf.gain.copy())
        rec["dz"].append(kf.dz.copy())
        rec["pdiag"].append(np.diag(kf.P_t_next).copy())
    kf.filter = wrapped
    os_, is_ = [], []
    for state in model.simulate(df):
        os_.append(state.o_t_next.copy())
        is_.append(state.i_t_next.copy())
    assert len(rec["K"]) == len(g["Kgain"])
    _close(np.array(rec["dz"]), g["dz"], atol=ATOL)
    _close(np.array(rec["K"]), g["Kgain"], atol=ATOL)
    _close(np.array(rec["gain"]), g["gain"], atol=ATOL)
    _close(np.array(rec["pdiag"]), g["pdiag"])
    _close(np.array(os_), g["o"])
    _close(np.array(is_), g["i"])
    _close(kf.P_t_next, g["P_final"], atol=ATOL)


def test_kalman_smoother_golden(golden):
    g = golden("g11_smoother.npz")
    model = golden_model(g)
    df = golden_frame(g, model.reach_ids)
    meas = pd.DataFrame(g["meas"], index=pd.DatetimeIndex(pd.to_datetime(g["meas_ns"], utc=True)),
                        columns=[model.reach_ids[k] for k in g["gages"]])
    n = model.n
    Q = 2.0 * np.eye(n)
    ks = KalmanSmoother(model, meas, Q, 1e-2 * np.eye(len(g["gages"])), Q.copy())
    model.bind_callback(ks, key="ks")
    os_ = [state.o_t_next.copy() for state in model.simulate(df)]
    _close(np.array(os_), g["o"])
    assert len(ks.datetimes) == int(g["n_times"])
    assert np.array_equal(ks.o_hat_s.index.asi8, g["os_ns"])
    _close(ks.o_hat_s.values, g["o_s"], atol=ATOL)
    _close(ks.i_hat_s.values, g["i_s"], atol=ATOL)
    times = sorted(ks.P_s)
    assert [t.value for t in times] == g["s_ns"].tolist()
    _close(np.array([ks.P_s[t].cpu().numpy() for t in times]), g["P_s"], rtol=1e-8, atol=1e-8)
