"""GPU edge cases of the session API (empty and minimal inputs, maximum analysis
sizes): an empty network, a one-reach network, a zero-length horizon, the smallest ensemble
analysis and one deep enough in gauges that the E x E products take the split-K GEMM."""
import numpy as np
import pytest

from oracle import oracle as orc
from tx_fast_hydrology_amd import _native as nat
from tx_fast_hydrology_amd import engine, synthetic

pytestmark = pytest.mark.gpu


def _empty():
    z = np.zeros(0, dtype=np.int64)
    return engine.RoutingNet(z, z, z)


def test_empty_network_session():
    net = _empty()
    net.set_coeffs(*(np.zeros(0),) * 4)
    net.set_state(np.zeros(0), np.zeros(0))
    net.load_forcing(np.array([0.0, 3.6e12]), np.zeros((2, 0)))
    net.run(np.array([3e11, 6e11, 9e11]))
    o, i = net.fetch_outputs()
    assert o.shape == (3, 0) and i.shape == (3, 0)
    so, si = net.get_state()
    assert so.shape == (0,) and si.shape == (0,)
    other = _empty()
    other.set_coeffs(*(np.zeros(0),) * 4)
    other.copy_state_from(net)
    i_n, o_n = engine.ax_bu(np.zeros(0, np.int64), np.zeros(0, np.int64),
                            *(np.zeros(0),) * 7, np.zeros(0, np.int64))
    assert i_n.shape == (0,) and o_n.shape == (0,)


def test_zero_length_horizon_is_rejected():
    end = np.array([1, 1])
    indeg = orc.compute_indegree(np.arange(2), end)
    net = engine.RoutingNet(end, indeg, np.array([0]))
    net.set_coeffs(*(np.full(2, v) for v in (0.1, 0.2, 0.3, 0.4)))
    net.load_forcing(np.array([0.0]), np.ones((1, 2)))
    with pytest.raises(nat.RoutingError):
        net.run(np.zeros(0))


@pytest.mark.parametrize("slots,tile", [(64, 16), (192, 16)])
def test_single_reach_network(slots, tile):
    end = np.array([0])                     # one outlet (self-loop)
    start = np.arange(1)
    indeg = orc.compute_indegree(start, end)
    coef = orc.muskingum_coeffs(np.array([3600.0]), np.array([0.29]), 300.0)
    o0, i0 = np.array([2.5]), np.array([0.0])
    xp = np.array([0.0, 3.6e12, 7.2e12])
    fp = np.array([[1.0], [2.0], [0.5]])
    x = 3e11 * np.arange(1, 25)
    net = engine.RoutingNet(end, indeg, start[indeg == 0], slots=slots, tile=tile)
    net.set_coeffs(*coef)
    net.set_state(o0, i0)
    got_o, got_i = net.simulate(x, xp, fp)
    want_o, want_i, _, _ = orc.simulate(start, end, indeg, *coef, o0, i0, x, xp, fp)
    assert np.array_equal(got_o, want_o) and np.array_equal(got_i, want_i)


def _numpy_enkf(X, s, Y, R):
    E = X.shape[1]
    A = X - X.mean(1, keepdims=True)
    HA = A[s]
    W = np.linalg.solve(HA @ HA.T / (E - 1) + R, Y - X[s])
    return A @ (HA.T @ W) / (E - 1)


@pytest.mark.parametrize("E,m", [(2, 1), (16, 600), (48, 400)])
def test_enkf_extreme_shapes_vs_numpy(E, m):
    """E = 2 / one gauge (smallest analysis); m >> E (the E x E products are 600 / 400 gauges
    deep: split-K over workgroups with the in-order slice reduction)."""
    end = synthetic.river_network(5000, 6, 150, np.random.default_rng(E + m))
    n = end.size
    start = np.arange(n)
    indeg = orc.compute_indegree(start, end)
    K, Xk, _ = synthetic.model_arrays(n, seed=3)
    net = engine.RoutingNet(end, indeg, start[indeg == 0], members=E)
    net.set_coeffs(*orc.muskingum_coeffs(K, Xk, 300.0))
    rng = np.random.default_rng(9)
    X = rng.uniform(0.5, 5, n)[:, None] * rng.lognormal(0, 0.3, (n, E))
    I0 = rng.uniform(0, 5, (n, E))
    net.set_state(X, I0)
    s = np.sort(rng.choice(n, m, replace=False))
    R = 1e-2 * np.eye(m)
    Y = X[s].mean(1, keepdims=True) + 0.3 + rng.normal(0, 0.1, (m, E))
    net.enkf_analysis(s, Y, R)
    o, i = net.get_state()
    G = _numpy_enkf(X, s, Y, R)
    heads = start[indeg == 0]
    scale = max(np.abs(G).max(), 1e-300)
    for e in range(E):
        ig, og = orc.apply_gain(heads, end, G[:, e], indeg)
        np.testing.assert_allclose(o[:, e] - X[:, e], og, rtol=0, atol=1e-9 * scale)
        np.testing.assert_allclose(i[:, e] - I0[:, e], ig, rtol=0, atol=1e-8 * scale)


def _same(a, b):
    """bit-equal arrays, NaN where the other has NaN (float64 cells)"""
    return np.array_equal(a, b, equal_nan=True)


@pytest.mark.parametrize("mode", ["launches", "auto"])
def test_non_finite_inputs_match_reference(mode):
    """Non-finite inputs route exactly as the reference routes them: a step outside the forcing
    index copies the clamped row (nutils.py:24-27, so +-Inf stays +-Inf instead of (1 - 0) f +
    0 f = NaN), and a never-processed reach keeps o = 0 (nutils.py:68) whatever its state and
    forcing hold.  Every cell equals the oracle's, +-Inf and NaN included."""
    # 0 -> 1 <-> 2 (cycle: 1 and 2 are never processed), 6 -> 1, 3, 4 -> 5 (outlet), 7 -> 3,
    # 8..13 -> 5: eight upstreams, so 5's inflow fold runs through partial-sum nodes
    end = np.array([1, 2, 1, 5, 5, 5, 1, 3] + [5] * 6, dtype=np.int64)
    n = end.size
    start = np.arange(n, dtype=np.int64)
    indeg = orc.compute_indegree(start, end)
    heads = start[indeg == 0]
    K = np.full(n, 3600.0)
    X = np.full(n, 0.2)
    coef = orc.muskingum_coeffs(K, X, 300.0)
    o0 = np.linspace(1.0, 2.0, n)
    o0[2] = np.nan                                   # unrouted reach: state never read
    i0 = orc.init_inflows(start, end, np.nan_to_num(o0))
    xp = (1.7e18 + 3600e9 * np.arange(4)).astype(float)
    fp = np.full((4, n), 0.5)
    fp[1, 1] = np.nan                                # unrouted reach forcing
    fp[3, 7] = np.inf                                # last row: clamped steps copy it
    fp[0, 4] = -np.inf                               # first row, interpolated from step 1
    fp[1, 9] = np.inf                                # into the partial sums of reach 5
    fp[2, 12] = -np.inf                              # ... and later Inf - Inf = NaN
    x = xp[0] + 300e9 * np.arange(1, 61)             # 60 steps: the last 24 beyond xp[-1]
    want_o, want_i, want_so, want_si = orc.simulate(start, end, indeg, *coef, o0, i0, x, xp, fp)
    assert np.isinf(want_o[-1, 7]) and (want_o[:, 1] == 0).all()
    net = engine.RoutingNet(end, indeg, heads, slots=64, tile=16)
    net.set_mode(mode)
    net.set_coeffs(*coef)
    net.set_state(o0, i0)
    net.load_forcing(xp, fp)
    net.run(x)
    got_o, got_i = net.fetch_outputs()
    assert _same(got_o, want_o) and _same(got_i, want_i)
    so, si = net.get_state()
    assert _same(so, want_so) and _same(si, want_si)
    # the reach-major fetch, and one step at a time (mc_step: the forcing row is q itself)
    O, I = net.fetch_series()
    assert _same(O, want_o.T) and _same(I, want_i.T)
    net.set_state(o0, i0)
    q = np.array([0.5, np.nan, 0.5, np.inf, 0.5, -np.inf, 0.5, np.inf] + [0.25] * 6)
    q[11] = np.inf
    i1, o1 = net.step(q)
    wi, wo = orc.ax_bu(heads, end, *coef, i0, o0, q, indeg)
    assert _same(o1, wo) and _same(i1, wi)
    net.close()


@pytest.mark.parametrize("mode", ["launches", "auto"])
def test_overflow_through_partial_sums_matches_reference(mode):
    """Finite inputs whose fold overflows inside the partial sums of a high fan-in reach.  The
    resident kernel's fast form (finite state and forcing: partial sums carry a state, exact for
    finite values) reports the non-finite partial sum at the end of the horizon and the horizon
    is re-routed from its input state in the exact form: every cell equals the oracle's (+Inf
    from the overflow, NaN from Inf - Inf), and a set_state with finite values re-arms the fast
    form."""
    end = np.array([1, 2, 1, 5, 5, 5, 1, 3] + [5] * 6, dtype=np.int64)
    n = end.size
    start = np.arange(n, dtype=np.int64)
    indeg = orc.compute_indegree(start, end)
    heads = start[indeg == 0]
    coef = orc.muskingum_coeffs(np.full(n, 3600.0), np.full(n, 0.2), 300.0)
    o0 = np.linspace(1.0, 2.0, n)
    i0 = orc.init_inflows(start, end, o0)
    xp = (1.7e18 + 3600e9 * np.arange(4)).astype(float)
    fp = np.full((4, n), 0.5)
    fp[1:, 8:11] = 1.2e308                  # three huge tributaries: their sum overflows
    fp[2:, 12] = -1.5e308                   # ... and one huge negative one: Inf - Inf later
    x = xp[0] + 300e9 * np.arange(1, 41)
    want_o, want_i, want_so, want_si = orc.simulate(start, end, indeg, *coef, o0, i0, x, xp, fp)
    assert not np.isfinite(want_o[:, 5]).all() and np.isfinite(fp).all()
    net = engine.RoutingNet(end, indeg, heads, slots=64, tile=16)
    net.set_mode(mode)
    net.set_coeffs(*coef)
    net.set_state(o0, i0)
    net.load_forcing(xp, fp)
    net.run(x)
    got_o, got_i = net.fetch_outputs()
    assert _same(got_o, want_o) and _same(got_i, want_i)
    so, si = net.get_state()
    assert _same(so, want_so) and _same(si, want_si)
    # finite state again: the next horizon runs in the fast form (and is exact: no overflow)
    fp2 = np.full((4, n), 0.5)
    net.set_state(o0, i0)
    net.load_forcing(xp, fp2)
    net.run(x)
    w2 = orc.simulate(start, end, indeg, *coef, o0, i0, x, xp, fp2)
    g2 = net.fetch_outputs()
    assert _same(g2[0], w2[0]) and _same(g2[1], w2[1])
    net.close()


def _edge_net():
    # the network of the two tests above: a cycle (reaches 1, 2 never processed) and reach 5's
    # eight upstreams folded through partial-sum nodes
    end = np.array([1, 2, 1, 5, 5, 5, 1, 3] + [5] * 6, dtype=np.int64)
    n = end.size
    start = np.arange(n, dtype=np.int64)
    indeg = orc.compute_indegree(start, end)
    coef = orc.muskingum_coeffs(np.full(n, 3600.0), np.full(n, 0.2), 300.0)
    return start, end, indeg, start[indeg == 0], coef


@pytest.mark.parametrize("mode,sync,E", [("launches", 0, 3), ("auto", 0, 3), ("dataflow", 0, 3),
                                         ("dataflow", 1, 3), ("launches", 1, 3),
                                         ("launches", 0, 4), ("auto", 0, 4)])
def test_non_finite_ensemble_matches_reference(mode, sync, E):
    """The same contract for an ensemble session: member e is an independent reference run
    (SURVEY a5).  Member 0 carries the non-finite forcing and state of the single-member test,
    member 1 is finite, member 2 overflows inside reach 5's partial sums from finite inputs.
    A horizon (multi-launch) and one-step runs (member dataflow; classic and chunk-synchronous
    plans) give every cell of every member exactly as the oracle does."""
    start, end, indeg, heads, coef = _edge_net()
    n = end.size                 # E = 4: member 3 finite; even E runs two members per instance
    o0 = np.stack([np.linspace(1.0, 2.0, n)] * E, axis=1)
    o0[2, 0] = np.nan                                # unrouted reach: state never read
    i0 = np.stack([orc.init_inflows(start, end, np.nan_to_num(o0[:, e])) for e in range(E)], 1)
    xp = (1.7e18 + 3600e9 * np.arange(4)).astype(float)
    fp = np.full((4, n, E), 0.5)
    fp[1, 1, 0] = np.nan
    fp[3, 7, 0] = np.inf
    fp[0, 4, 0] = -np.inf
    fp[1, 9, 0] = np.inf
    fp[2, 12, 0] = -np.inf
    fp[1:, 8:11, 2] = 1.2e308
    fp[2:, 12, 2] = -1.5e308
    x = xp[0] + 300e9 * np.arange(1, 61)
    c = np.ascontiguousarray
    want = [orc.simulate(start, end, indeg, *coef, c(o0[:, e]), c(i0[:, e]), x, xp, c(fp[:, :, e]))
            for e in range(E)]
    net = engine.RoutingNet(end, indeg, heads, slots=64, tile=16, members=E, sync=sync)
    net.set_coeffs(*coef)
    if mode != "dataflow":                           # dataflow mode routes one step only
        net.set_mode(mode)
        net.set_state(o0, i0)
        net.load_forcing(xp, fp)
        net.run(x)
        got_o, got_i = net.fetch_outputs()
        so, si = net.get_state()
        for e in range(E):
            assert _same(got_o[:, :, e], want[e][0]) and _same(got_i[:, :, e], want[e][1])
            assert _same(so[:, e], want[e][2]) and _same(si[:, e], want[e][3])
    net.set_mode(mode)
    # one step at a time over the first hours, from the reference's own states
    o, i = o0.copy(), i0.copy()
    net.set_state(o, i)
    net.load_forcing(xp, fp)
    for t in range(14):
        net.run(x[t:t + 1])
        got_o, got_i = net.fetch_outputs()
        for e in range(E):
            assert _same(got_o[0, :, e], want[e][0][t]), (t, e)
            assert _same(got_i[0, :, e], want[e][1][t]), (t, e)
    path = {"launches": "launches", "auto": "dataflow", "dataflow": "dataflow"}
    assert net.mode()[1] == path[mode]
    # mc_step: the forcing row is q itself
    net.set_state(o0, i0)
    q = np.full((n, E), 0.25)
    q[[1, 3, 5, 7, 11], 0] = [np.nan, np.inf, -np.inf, np.inf, np.inf]
    q[8:11, 2] = 1.5e308
    i1, o1 = net.step(q)
    for e in range(E):
        wi, wo = orc.ax_bu(heads, end, *coef, c(i0[:, e]), c(o0[:, e]), c(q[:, e]), indeg)
        assert _same(o1[:, e], wo) and _same(i1[:, e], wi), e
    net.close()
