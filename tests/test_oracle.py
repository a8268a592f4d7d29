"""Pin the CPU oracle (oracle/) against the reference's golden vectors (tests/golden/).

CPU only.  Every comparison of discharges is bit-exact (np.array_equal on float64): the oracle
restates the reference's arithmetic in the same order with FMA contraction off.
"""
import hashlib

import numpy as np
import pytest

from oracle import oracle as orc


def _model_arrays(g):
    endnodes = g["endnodes"].astype(np.int64)
    n = endnodes.size
    start = np.arange(n, dtype=np.int64)
    indeg = orc.compute_indegree(start, endnodes)
    a, b, c, gm = orc.muskingum_coeffs(g["K"], g["X"], float(g["dt"]))
    i0 = orc.init_inflows(start, endnodes, g["o0"])
    return start, endnodes, indeg, (a, b, c, gm), i0


def _simulate_golden(g, n_steps=None):
    start, endnodes, indeg, coef, i0 = _model_arrays(g)
    xs = orc.step_times(int(g["start_ns"]), int(float(g["dt"]) * 1e9), int(g["idx_ns"].max()))
    if n_steps is not None:
        xs = xs[:n_steps]
    xp = g["idx_ns"].astype(float)
    out_o, out_i, _, _ = orc.simulate(start, endnodes, indeg, *coef, g["o0"], i0,
                                      xs.astype(float), xp, g["forcing"])
    return xs, out_o, out_i, i0, indeg, coef


def test_g1_ynetwork_bitexact(golden):
    g = golden("g1_ynet.npz")
    xs, o, i, i0, indeg, coef = _simulate_golden(g)
    assert np.array_equal(i0, g["init_i"])           # self-loop quirk (muskingum.py:417)
    assert np.array_equal(i0, [0, 0, 2, 2])
    assert np.array_equal(indeg, g["indegree"])
    for got, want in zip(coef, ("alpha", "beta", "chi", "gamma")):
        assert np.array_equal(got, g[want])
    assert np.array_equal(xs, g["t_ns"])
    assert np.array_equal(o, g["o"]) and np.array_equal(i, g["i"])


def test_g2_huc8_every_step_hash(golden):
    g = golden("g2_huc8.npz")
    xs, o, i, i0, _, _ = _simulate_golden(g)
    assert o.shape == (288, 1000)
    assert np.array_equal(i0, g["init_i"])
    assert np.array_equal(xs, g["t_ns"])
    keep = g["keep"]
    assert np.array_equal(o[keep], g["o_keep"]) and np.array_equal(i[keep], g["i_keep"])
    for t in range(288):
        assert hashlib.sha256(o[t].tobytes()).digest() == g["o_sha"][t].tobytes(), t
        assert hashlib.sha256(i[t].tobytes()).digest() == g["i_sha"][t].tobytes(), t


def test_g3_confluence_order(golden):
    g = golden("g3_confluence.npz")
    xs, o, i, _, _, _ = _simulate_golden(g, n_steps=int(g["n_steps"]))
    assert np.array_equal(o, g["o"]) and np.array_equal(i, g["i"])


def test_g6_dt_change_quirk(golden):
    g = golden("g6_dt_change.npz")
    endnodes = g["endnodes"]
    n = endnodes.size
    start = np.arange(n, dtype=np.int64)
    indeg = orc.compute_indegree(start, endnodes)
    heads = start[indeg == 0]
    coef = orc.muskingum_coeffs(g["K"], g["X"], 3600.0)
    o = g["o0"].copy()
    i = orc.init_inflows(start, endnodes, o)
    for k, td in enumerate(g["td"]):
        if td > 0 and float(td) != 3600.0:
            coef = orc.muskingum_coeffs(g["K"], g["X"], float(td))
        i, o = orc.ax_bu(heads, endnodes, *coef, i, o, g["q"][k], indeg)
        assert np.array_equal(np.stack(coef), g["coef"][k])
        assert np.array_equal(o, g["o"][k]) and np.array_equal(i, g["i"][k])


def test_g7_covariance_and_gain(golden):
    g = golden("g7_covariance.npz")
    endnodes = g["endnodes"]
    n = endnodes.size
    start = np.arange(n, dtype=np.int64)
    indeg = g["indegree"]
    heads = start[indeg == 0]
    args = (heads, endnodes, g["alpha"], g["beta"], g["chi"])
    assert np.array_equal(orc.aqat(g["P"], *args, indeg), g["aqat"])
    assert np.array_equal(orc.ap(g["P"], *args, indeg), g["ap"])
    ig, og = orc.apply_gain(heads, endnodes, g["gain"], indeg)
    assert np.array_equal(ig, g["gain_i"]) and np.array_equal(og, g["gain_o"])
    ai, ao = orc.ax(*args, g["ip"], g["op"], indeg)
    assert np.array_equal(ai, g["ax_i"]) and np.array_equal(ao, g["ax_o"])


@pytest.mark.parametrize("impl", ["c", "py"])
def test_g8_ax_bu_edge_cases(golden, impl):
    g = golden("g8_ax_bu_edge.npz")
    fn = orc.ax_bu if impl == "c" else orc.ax_bu_py
    for name in g["names"]:
        a = g[f"{name}_args"]
        i_n, o_n = fn(g[f"{name}_heads"], g[f"{name}_endnodes"], a[0], a[1], a[2], a[3], a[4],
                      a[5], a[6], g[f"{name}_indegree"])
        assert np.array_equal(i_n, g[f"{name}_i"]), name
        assert np.array_equal(o_n, g[f"{name}_o"]), name


def test_g9_interpolation(golden):
    g = golden("g9_interp.npz")
    for k, x in enumerate(g["xs"]):
        assert np.array_equal(orc.interpolate_sample(x, g["xp"], g["fp"], 1), g["lin"][k])
        assert np.array_equal(orc.interpolate_sample(x, g["xp"], g["fp"], 0), g["near"][k])


def test_g10_coefficients_and_init(golden):
    g = golden("g10_model_io.npz")
    for dt in (60, 300, 900, 3600, 86400):
        assert np.array_equal(np.stack(orc.muskingum_coeffs(g["K"], g["X"], float(dt))),
                              g[f"dt{dt}"])
    n = g["endnodes"].size
    start = np.arange(n, dtype=np.int64)
    assert np.array_equal(orc.compute_indegree(start, g["endnodes"]), g["indegree"])
    assert np.array_equal(orc.init_inflows(start, g["endnodes"], g["o0"]), g["init_i"])


def test_g5_kalman_analysis(golden):
    """da.py:91-136 restated in numpy; BLAS reductions allow last-bit differences."""
    g = golden("g5_kalman.npz")
    endnodes = g["endnodes"]
    n = endnodes.size
    start = np.arange(n, dtype=np.int64)
    indeg = orc.compute_indegree(start, endnodes)
    coef = orc.muskingum_coeffs(g["K"], g["X"], 3600.0)
    heads = start[indeg == 0]
    s = np.zeros(n, dtype=bool)
    s[g["gages"]] = True
    order = np.argsort(g["gages"])
    meas = g["meas"][:, order]
    R = 1e-2 * np.eye(6)
    Q = 2.0 * np.eye(n)
    P = Q.copy()
    o = g["o0"].copy()
    i = orc.init_inflows(start, endnodes, o)
    xp = g["idx_ns"].astype(float)
    mxp = g["meas_ns"].astype(float)
    t_ns = int(g["start_ns"])
    dt_ns = 3600 * 10**9

    def analyse(o, i, P, t_ns):
        Z = orc.interpolate_sample(float(t_ns), mxp, meas, 1)
        return orc.kalman_analysis(P, o, i, s, Z, Q, R, start, endnodes, indeg, *coef[:3])

    done = []

    def check(r):
        k = len(done)
        np.testing.assert_allclose(r["K"], g["Kgain"][k], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(r["gain"], g["gain"][k], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(r["dz"], g["dz"][k], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(np.diag(r["P"]), g["pdiag"][k], rtol=1e-9, atol=1e-12)
        done.append(k)
        return r["o"], r["i"], r["P"]

    o, i, P = check(analyse(o, i, P, t_ns))      # __on_simulation_start__ (da.py:49-54)
    for step in range(g["t_ns"].size):
        t_ns += dt_ns
        q = orc.interpolate_sample(float(t_ns), xp, g["forcing"], 1)
        i, o = orc.ax_bu(heads, endnodes, *coef, i, o, q, indeg)
        if t_ns <= g["meas_ns"].max():          # da.py:56-61
            o, i, P = check(analyse(o, i, P, t_ns))
        np.testing.assert_allclose(o, g["o"][step], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(i, g["i"][step], rtol=1e-9, atol=1e-12)
    assert len(done) == g["Kgain"].shape[0]
