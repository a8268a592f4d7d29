"""GPU parity of the analysis step.

* `mc_apply_gain` is `_apply_gain` (nutils.py:116-134) applied as da.py:124-126 -> bit-exact vs
  the oracle, including networks with cycles / unprocessed reaches (golden g8 topologies).
* The ensemble Kalman analysis has no reference implementation, so parity is by construction
  ("EnKF known-answer test"): an ensemble whose anomalies have exact sample
  covariance P must give the reference gain K = P[:, s] (P[s, s] + R)^-1 (da.py:119) and, with
  identical observations in every member, the reference mean update (da.py:121-126).  Tolerance
  1e-11 relative (f64 MFMA products + Cholesky vs numpy's inverse).
* A randomized perturbed-observation analysis is checked against a float64 numpy restatement of
  the same ensemble formulas.
"""
import numpy as np
import pytest

from oracle import oracle as orc
from tx_fast_hydrology_amd import engine, synthetic

pytestmark = pytest.mark.gpu


def _net(end, members=1, slots=0, **kw):
    n = end.size
    start = np.arange(n)
    indeg = orc.compute_indegree(start, end)
    K, X, _ = synthetic.model_arrays(n, seed=n)
    coef = orc.muskingum_coeffs(K, X, 300.0)
    net = engine.RoutingNet(end, indeg, start[indeg == 0], slots=slots, members=members, **kw)
    net.set_coeffs(*coef)
    return net, start, indeg


def test_apply_gain_bitexact_golden_topologies(golden):
    g = golden("g8_ax_bu_edge.npz")
    rng = np.random.default_rng(0)
    for name in g["names"]:
        end, indeg, heads = g[f"{name}_endnodes"], g[f"{name}_indegree"], g[f"{name}_heads"]
        n = end.size
        net = engine.RoutingNet(end, indeg, heads, slots=64, tile=16)
        net.set_coeffs(*(np.full(n, v) for v in (0.1, 0.2, 0.3, 0.4)))
        o0, i0 = rng.uniform(0, 3, n), rng.uniform(0, 3, n)
        net.set_state(o0, i0)
        gain = rng.normal(0, 1, n)
        net.apply_gain(gain)
        ig, og = orc.apply_gain(heads, end, gain, indeg)
        o, i = net.get_state()
        assert np.array_equal(o, o0 + og), name
        assert np.array_equal(i, i0 + ig), name


def test_apply_gain_ensemble_per_member():
    end = synthetic.river_network(4000, 5, 150, np.random.default_rng(3))
    E = 5
    net, start, indeg = _net(end, members=E)
    n = end.size
    rng = np.random.default_rng(1)
    o0, i0 = rng.uniform(0, 3, (n, E)), rng.uniform(0, 3, (n, E))
    net.set_state(o0, i0)
    gain = rng.normal(0, 1, (n, E))
    net.apply_gain(gain)
    o, i = net.get_state()
    for e in range(E):
        ig, og = orc.apply_gain(start[indeg == 0], end, gain[:, e], indeg)
        assert np.array_equal(o[:, e], o0[:, e] + og), e
        assert np.array_equal(i[:, e], i0[:, e] + ig), e


def _kat_case(n, m, seed):
    rng = np.random.default_rng(seed)
    end = synthetic.river_network(n, 2, 25, rng)
    n = end.size
    B = rng.normal(0, 1, (n, n))
    P = B @ B.T / n + 0.5 * np.eye(n)                       # SPD forecast covariance
    L = np.linalg.cholesky(P)
    E = 2 * n
    Xp = np.sqrt((E - 1) / 2.0) * np.concatenate([L, -L], axis=1)   # exact sample cov = P
    xbar = rng.uniform(1, 5, n)
    s = np.sort(rng.choice(n, m, replace=False))
    R = 1e-2 * np.eye(m) + 1e-3 * np.ones((m, m))
    return end, P, E, Xp, xbar, s, R


def test_enkf_known_answer_gain_and_mean_update():
    end, P, E, Xp, xbar, s, R = _kat_case(48, 6, 11)
    n = end.size
    net, start, indeg = _net(end, members=E)
    X = xbar[:, None] + Xp
    i0 = np.random.default_rng(2).uniform(0, 1, (n, E))
    net.set_state(X, i0)
    K_ref = P[:, s] @ np.linalg.inv(P[np.ix_(s, s)] + R)             # da.py:119
    K = net.enkf_gain(s, R)
    np.testing.assert_allclose(K, K_ref, rtol=0, atol=1e-11 * np.abs(K_ref).max())
    # identical observations in every member: the mean follows da.py:121-126 exactly
    y = xbar[s] + np.random.default_rng(4).normal(0, 0.2, s.size)
    net.enkf_analysis(s, np.repeat(y[:, None], E, axis=1), R)
    o, i = net.get_state()
    gain_ref = K_ref @ (y - xbar[s])
    ig_ref, og_ref = orc.apply_gain(start[indeg == 0], end, gain_ref, indeg)
    tol = 1e-11 * max(np.abs(gain_ref).max(), 1.0)
    np.testing.assert_allclose(o.mean(1) - X.mean(1), og_ref, rtol=0, atol=tol)
    np.testing.assert_allclose(i.mean(1) - i0.mean(1), ig_ref, rtol=0, atol=tol)
    # anomalies are shrunk but stay centred: the mean of the increments is the mean gain


def _numpy_enkf(X, s, Y, R):
    E = X.shape[1]
    A = X - X.mean(1, keepdims=True)
    HA = A[s]
    C = HA @ HA.T / (E - 1) + R
    W = np.linalg.solve(C, Y - X[s])
    return A @ (HA.T @ W) / (E - 1)


def test_enkf_perturbed_observations_vs_numpy():
    end = synthetic.river_network(6000, 6, 200, np.random.default_rng(21))
    n = end.size
    E, m = 32, 40
    net, start, indeg = _net(end, members=E)
    rng = np.random.default_rng(5)
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
    scale = np.abs(G).max()
    for e in range(E):
        ig, og = orc.apply_gain(heads, end, G[:, e], indeg)
        np.testing.assert_allclose(o[:, e] - X[:, e], og, rtol=0, atol=1e-10 * scale)
        np.testing.assert_allclose(i[:, e] - I0[:, e], ig, rtol=0, atol=1e-10 * scale * 10)


def test_enkf_rejects_single_member_and_bad_R():
    from tx_fast_hydrology_amd import _native as nat
    end = synthetic.river_network(500, 1, 30, np.random.default_rng(1))
    net, start, indeg = _net(end)
    with pytest.raises(nat.RoutingError):
        net.enkf_gain(np.array([3, 7]), np.eye(2))
    net2, _, _ = _net(end, members=4)
    net2.set_state(np.ones((end.size, 4)), np.ones((end.size, 4)))   # zero spread
    with pytest.raises(nat.RoutingError):
        net2.enkf_gain(np.array([3, 7]), -np.eye(2))                 # not SPD


def test_enkf_failure_reported_after_a_later_success():
    """The factorisation status of every analysis is kept until the next synchronising call: a
    failed analysis followed by a successful one is still reported (once), and the failed
    analysis left the members unchanged (zeroed increment)."""
    from tx_fast_hydrology_amd import _native as nat
    end = synthetic.river_network(500, 1, 30, np.random.default_rng(1))
    n = end.size
    net, start, indeg = _net(end, members=4)
    X = np.ones((n, 4))
    net.set_state(X, X)                                   # zero spread: HA = 0
    s = np.array([3, 7])
    y = np.ones((2, 4))
    net.enkf_analysis(s, y, -np.eye(2))                   # C = R = -I: not SPD
    net.enkf_analysis(s, y, np.eye(2))                    # fine
    with pytest.raises(nat.RoutingError):
        net.get_state()
    o, i = net.get_state()                                # reported once
    assert np.array_equal(o, X) and np.array_equal(i, X)


def test_staged_driver_single_rank_equals_enkf_analysis():
    """ensemble.distributed_analysis with one rank runs the mc_ens_* stages on torch device
    buffers; it must reproduce RoutingNet.enkf_analysis exactly."""
    import torch
    from tx_fast_hydrology_amd import ensemble
    end = synthetic.river_network(5000, 4, 150, np.random.default_rng(8))
    n = end.size
    E, m = 16, 30
    rng = np.random.default_rng(9)
    X = rng.uniform(0.5, 5, n)[:, None] * rng.lognormal(0, 0.3, (n, E))
    I0 = rng.uniform(0, 5, (n, E))
    s = np.sort(rng.choice(n, m, replace=False))
    R = 2e-2 * np.eye(m)
    Y = ensemble.perturbed_observations(X[s].mean(1) + 0.2, R, E, rng)
    a, _, _ = _net(end, members=E)
    a.set_state(X, I0)
    a.enkf_analysis(s, Y, R)
    b, _, _ = _net(end, members=E)
    b.set_state(X, I0)
    ensemble.distributed_analysis(b, s, Y, R, device=torch.device("cuda", 0), staged=True)
    oa, ia = a.get_state()
    ob, ib = b.get_state()
    assert np.array_equal(oa, ob) and np.array_equal(ia, ib)


def test_comm_analysis_single_rank_equals_enkf_analysis():
    """The C ABI's own communicator (mc_comm_* over RCCL, no torch.distributed): one rank runs
    the whole program -- all-gathers, both all-to-alls (copies with one rank), the weights under
    the member -> slice all-to-all on the side stream -- and reproduces RoutingNet.enkf_analysis
    exactly (two ranks cannot share the one GPU of a test box under RCCL)."""
    end = synthetic.river_network(5000, 4, 150, np.random.default_rng(18))
    n = end.size
    E, m = 16, 30
    rng = np.random.default_rng(19)
    X = rng.uniform(0.5, 5, n)[:, None] * rng.lognormal(0, 0.3, (n, E))
    I0 = rng.uniform(0, 5, (n, E))
    s = np.sort(rng.choice(n, m, replace=False))
    R = 2e-2 * np.eye(m)
    Y = X[s] + rng.normal(0, 0.1, (m, E))
    a, _, _ = _net(end, members=E)
    a.set_state(X, I0)
    a.enkf_analysis(s, Y, R)
    b, _, _ = _net(end, members=E)
    b.set_state(X, I0)
    comm = engine.Communicator(1, 0, engine.Communicator.unique_id())
    for _ in range(2):                         # scratch reuse across analyses
        b.ens_analysis_dist(comm, s, Y, R)
        if _ == 0:
            a.enkf_analysis(s, Y, R)
    oa, ia = a.get_state()
    ob, ib = b.get_state()
    assert np.array_equal(oa, ob) and np.array_equal(ia, ib)
    comm.close()


# (16, 40), (48, 12): the one-workgroup SPD solve; (96, 150), (200, 260): E > 64, the
# factorisation and the two triangular solves of the large-ensemble path
@pytest.mark.parametrize("E,m", [(16, 40), (48, 12), (96, 150), (200, 260)])
def test_ensemble_space_solve_equals_observation_space(E, m):
    """Diagonal R with E <= m takes the E x E ensemble-space solve (push-through identity); a
    numerically identical R with a 1e-300 off-diagonal entry forces the m x m observation-space
    Cholesky.  Both must give the same analysis (and the numpy restatement)."""
    end = synthetic.river_network(3000, 4, 120, np.random.default_rng(31))
    n = end.size
    rng = np.random.default_rng(E + m)
    X = rng.uniform(0.5, 5, n)[:, None] * rng.lognormal(0, 0.3, (n, E))
    I0 = rng.uniform(0, 5, (n, E))
    s = np.sort(rng.choice(n, m, replace=False))
    R = np.diag(rng.uniform(5e-3, 5e-2, m))
    Y = X[s].mean(1, keepdims=True) + 0.2 + rng.normal(0, 0.1, (m, E))
    Rd = R.copy()
    Rd[0, 1] = Rd[1, 0] = 1e-300
    out = []
    for RR in (R, Rd):
        net, _, _ = _net(end, members=E)
        net.set_state(X, I0)
        net.enkf_analysis(s, Y, RR)
        out.append(net.get_state())
    G = _numpy_enkf(X, s, Y, R)
    scale = np.abs(G).max()
    for k in range(2):
        np.testing.assert_allclose(out[0][k], out[1][k], rtol=0, atol=1e-10 * scale * 10)
    start = np.arange(n)
    indeg = orc.compute_indegree(start, end)
    for e in range(0, E, 7):
        _, og = orc.apply_gain(start[indeg == 0], end, G[:, e], indeg)
        np.testing.assert_allclose(out[0][0][:, e] - X[:, e], og, rtol=0, atol=1e-10 * scale)


def test_enkf256_large_mean_and_zero_spread_reaches():
    """ADVICE r3 (slice_increments, E > 64): reaches whose members are identical get increments
    of exactly 0 (their outflow is unchanged bit for bit, as the reference's X - mean gives), and
    reaches with a large mean and a small spread keep their increments to spread-relative
    accuracy -- the member mean is taken out before the products, not after."""
    end = synthetic.river_network(3000, 4, 120, np.random.default_rng(33))
    n = end.size
    E, m = 256, 30
    net, start, indeg = _net(end, members=E)
    rng = np.random.default_rng(8)
    X = rng.uniform(0.5, 5, n)[:, None] * rng.lognormal(0, 0.3, (n, E))
    flat = rng.choice(n, 200, replace=False)               # zero spread
    X[flat] = rng.uniform(1, 10, 200)[:, None]
    big = np.setdiff1d(rng.choice(n, 300, replace=False), flat)   # mean 1e6, spread 1e-3
    X[big] = 1e6 + 1e-3 * rng.standard_normal((big.size, E))
    I0 = rng.uniform(0, 5, (n, E))
    net.set_state(X, I0)
    s = np.sort(rng.choice(np.setdiff1d(np.arange(n), np.concatenate([flat, big])), m,
                           replace=False))
    R = 1e-2 * np.eye(m)
    Y = X[s].mean(1, keepdims=True) + 0.3 + rng.normal(0, 0.1, (m, E))
    net.enkf_analysis(s, Y, R)
    o, _ = net.get_state()
    G = _numpy_enkf(X, s, Y, R)
    assert np.array_equal(o[flat], X[flat])                # 0 + 0 increments: bit-identical
    spread = np.abs(X[big] - X[big].mean(1, keepdims=True)).max()
    assert spread < 1e-2
    np.testing.assert_allclose(o[big] - X[big], G[big], rtol=0,
                               atol=1e-9 * np.abs(G[big]).max() + 1e-7 * spread)
    rest = np.setdiff1d(np.arange(n), np.concatenate([flat, big]))
    np.testing.assert_allclose(o[rest] - X[rest], G[rest], rtol=0, atol=1e-10 * np.abs(G).max())


@pytest.mark.parametrize("E,mode,sync", [(32, "auto", 0), (256, "auto", 0), (32, "auto", 1),
                                         (256, "auto", 1), (100, "launches", 1)])
def test_lazy_gain_folded_into_member_step(E, mode, sync):
    """The analysis increments are applied lazily: the next one-step member run applies them
    while it stages its inputs (launch_member_inputs with the pending gain) instead of a separate
    apply_gain pass.  An EnKF cycle run that way is bit-identical to the same cycle with the gain
    settled right after every analysis (get_state forces it), outputs included -- on the
    member-dataflow launch of classic and chunk-synchronous plans and on launches."""
    end = synthetic.river_network(5000, 5, 150, np.random.default_rng(4))
    n = end.size
    m = 25
    rng = np.random.default_rng(E)
    X = rng.uniform(0.5, 5, n)[:, None] * rng.lognormal(0, 0.3, (n, E))
    I0 = rng.uniform(0, 5, (n, E))
    xp = (1.7e18 + 3600e9 * np.arange(3)).astype(float)
    fp = rng.gamma(2.0, 0.5, (3, n, E))
    s = np.sort(rng.choice(n, m, replace=False))
    R = 1e-2 * np.eye(m)
    Ys = [X[s].mean(1, keepdims=True) + 0.2 + rng.normal(0, 0.1, (m, E)) for _ in range(3)]
    res = []
    for settle in (False, True):
        net, start, indeg = _net(end, members=E, slots=192, tile=16, sync=sync)
        net.set_mode(mode)
        net.set_state(X, I0)
        net.load_forcing(xp, fp)
        outs = []
        for k in range(3):
            net.run(xp[:1] + 300e9 * (k + 1))
            outs.append(net.fetch_outputs())
            net.enkf_analysis(s, Ys[k], R)
            if settle:
                net.get_state()
        want = mode if mode != "auto" else "dataflow"
        assert net.mode()[1] == want
        res.append((net.get_state(), outs))
        net.close()
    (sa, oa), (sb, ob) = res
    assert np.array_equal(sa[0], sb[0]) and np.array_equal(sa[1], sb[1])
    for (o1, i1), (o2, i2) in zip(oa, ob):
        assert np.array_equal(o1, o2) and np.array_equal(i1, i2)
