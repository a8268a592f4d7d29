"""GPU parity of the ensemble axis: every member of an E-member session is an
independent deterministic run with its own forcing and initial state, so each member column must
be bit-identical to the serial oracle run on that member's inputs."""
import numpy as np
import pytest

from oracle import oracle as orc
from tx_fast_hydrology_amd import engine, synthetic

pytestmark = pytest.mark.gpu


def _members(n, E, rows, seed):
    """Member forcing / state = base x lognormal(0, 0.3) multiplier per (reach, member), constant
    in time (SURVEY §8d ensemble generator)."""
    rng = np.random.default_rng(seed)
    xp, fp = synthetic.forcing(n, rows=rows, seed=seed)
    mult = rng.lognormal(0.0, 0.3, (n, E))
    fpe = fp[:, :, None] * mult[None, :, :]
    o0 = rng.uniform(0.5, 5.0, n)[:, None] * rng.lognormal(0.0, 0.3, (n, E))
    return xp.astype(float), np.ascontiguousarray(fpe), np.ascontiguousarray(o0)


def _case(n, basins, depth, seed, E, rows=7):
    end = synthetic.river_network(n, basins, depth, np.random.default_rng(seed))
    n = end.size
    start = np.arange(n)
    indeg = orc.compute_indegree(start, end)
    K, X, _ = synthetic.model_arrays(n, seed=seed)
    coef = orc.muskingum_coeffs(K, X, 300.0)
    xp, fpe, o0 = _members(n, E, rows, seed + 1)
    i0 = np.stack([orc.init_inflows(start, end, o0[:, e]) for e in range(E)], axis=1)
    return end, start, indeg, coef, xp, fpe, o0, i0


@pytest.mark.parametrize("n,E,slots,T,chain", [(3000, 5, 256, 60, 0), (1200, 64, 128, 25, 0),
                                               (5000, 3, 448, 100, 0), (1500, 4, 64, 40, 1),
                                               (1500, 4, 64, 40, 3)])
def test_ensemble_members_bitexact(n, E, slots, T, chain):
    """Every member bit-identical to its serial oracle run on the multi-launch path (workgroup
    output rows, kernels.hpp), including one-segment workgroups (64 lanes x 1 position) and odd
    segment counts (64 lanes x 3 positions)."""
    end, start, indeg, coef, xp, fpe, o0, i0 = _case(n, 4, 120, n + E, E)
    n = end.size
    x = xp[0] + 300e9 * np.arange(1, T + 1)
    net = engine.RoutingNet(end, indeg, start[indeg == 0], slots=slots, members=E, chain=chain)
    net.set_mode("launches")
    net.set_coeffs(*coef)
    net.set_state(o0, i0)
    got_o, got_i = net.simulate(x, xp, fpe)
    assert got_o.shape == (T, n, E)
    assert net.mode()[1] == "launches"
    so, si = net.get_state()
    ser_o, ser_i = net.fetch_series()
    for e in range(E):
        want_o, want_i, fo, fi = orc.simulate(start, end, indeg, *coef, o0[:, e], i0[:, e], x,
                                              xp, np.ascontiguousarray(fpe[:, :, e]))
        assert np.array_equal(got_o[:, :, e], want_o), e
        assert np.array_equal(got_i[:, :, e], want_i), e
        assert np.array_equal(so[:, e], fo) and np.array_equal(si[:, e], fi), e
        assert np.array_equal(ser_o[:, :, e], want_o.T), e
        assert np.array_equal(ser_i[:, :, e], want_i.T), e


def test_ensemble_continuation_and_member_zero_equals_deterministic():
    E = 4
    end, start, indeg, coef, xp, fpe, o0, i0 = _case(2500, 3, 90, 17, E)
    heads = start[indeg == 0]
    ens = engine.RoutingNet(end, indeg, heads, members=E)
    ens.set_coeffs(*coef)
    ens.set_state(o0, i0)
    ens.load_forcing(xp, fpe)
    det = engine.RoutingNet(end, indeg, heads)
    det.set_mode("launches")
    det.set_coeffs(*coef)
    det.set_state(o0[:, 0], i0[:, 0])
    det.load_forcing(xp, np.ascontiguousarray(fpe[:, :, 0]))
    x = xp[0] + 300e9 * np.arange(1, 91)
    for part in (x[:37], x[37:]):             # two horizons continue the state
        ens.run(part)
        det.run(part)
        eo, ei = ens.fetch_outputs()
        do, di = det.fetch_outputs()
        assert np.array_equal(eo[:, :, 0], do) and np.array_equal(ei[:, :, 0], di)
    want_o, want_i, _, _ = orc.simulate(start, end, indeg, *coef, o0[:, 2], i0[:, 2], x, xp,
                                        np.ascontiguousarray(fpe[:, :, 2]))
    assert np.array_equal(eo[:, :, 2], want_o[37:]) and np.array_equal(ei[:, :, 2], want_i[37:])


def test_ensemble_step_api():
    E = 6
    end, start, indeg, coef, xp, fpe, o0, i0 = _case(1500, 2, 60, 5, E)
    heads = start[indeg == 0]
    net = engine.RoutingNet(end, indeg, heads, members=E)
    net.set_coeffs(*coef)
    q = np.ascontiguousarray(fpe[0])
    i_n, o_n = net.step(q, o0, i0)
    assert i_n.shape == (end.size, E)
    for e in range(E):
        i_w, o_w = orc.ax_bu(heads, end, *coef, i0[:, e], o0[:, e], q[:, e], indeg)
        assert np.array_equal(o_n[:, e], o_w) and np.array_equal(i_n[:, e], i_w), e


def test_ensemble_rejects_dataflow_and_bad_shapes():
    from tx_fast_hydrology_amd import _native as nat
    E = 2
    end, start, indeg, coef, xp, fpe, o0, i0 = _case(800, 2, 40, 3, E)
    net = engine.RoutingNet(end, indeg, start[indeg == 0], members=E)
    net.set_coeffs(*coef)
    with pytest.raises(ValueError):
        net.set_state(o0[:, 0], i0[:, 0])
    net.set_state(o0, i0)
    net.load_forcing(xp, fpe)
    net.set_mode("dataflow")
    with pytest.raises(nat.RoutingError):
        net.run(xp[0] + 300e9 * np.arange(1, 5))


@pytest.mark.parametrize("n,E,slots,tile,mode", [
    (3000, 33, 256, 0, "dataflow"), (1200, 2, 128, 0, "dataflow"), (4000, 256, 384, 0, "dataflow"),
    (2500, 137, 192, 0, "dataflow"), (190_000, 32, 384, 0, "dataflow"),
    (190_000, 32, 192, 16, "dataflow"),
    (3000, 33, 256, 16, "sync"), (1200, 2, 128, 16, "sync"), (4000, 256, 192, 16, "sync"),
    (2500, 137, 192, 16, "sync"), (2500, 64, 192, 16, "sync"), (190_000, 32, 192, 16, "sync"),
    (190_000, 256, 192, 16, "sync")])
def test_member_dataflow_single_steps(n, E, slots, tile, mode):
    """One-step runs of an ensemble (the analysis cycle of the EnKF) as member-dataflow launches
    (member e of slot d at tick G[d] + e), on classic plans and on chunk-synchronous ones
    ("sync": one workgroup barrier per 4 ticks, 4-tick local edges between waves).  Several
    consecutive one-step runs (interpolated between forcing rows) then a multi-step run must
    equal every member's serial run."""
    depth = 1500 if n > 100_000 else 120
    end, start, indeg, coef, xp, fpe, o0, i0 = _case(n, 4 if n < 100_000 else 300, depth,
                                                      n + E, E)
    n = end.size
    sync = mode == "sync"
    mode = "dataflow" if sync else mode
    net = engine.RoutingNet(end, indeg, start[indeg == 0], slots=slots, tile=tile, members=E,
                            sync=int(sync))
    if sync:
        assert net.info["n_local"] > 0 or n < 3000
    net.set_mode(mode)
    net.set_coeffs(*coef)
    net.set_state(o0, i0)
    net.load_forcing(xp, fpe)
    x = xp[0] + 300e9 * np.arange(1, 16)          # 12 steps per forcing row: fractional rows
    outs_o, outs_i = [], []
    for k in range(5):
        net.run(x[k:k + 1])
        assert net.mode()[1] == mode, k
        oo, ii = net.fetch_outputs()
        outs_o.append(oo[0])
        outs_i.append(ii[0])
    net.set_mode("auto")                        # (dataflow mode refuses ensemble horizons)
    net.run(x[5:])
    assert net.mode()[1] == "launches"
    oo, ii = net.fetch_outputs()
    got_o = np.concatenate([np.array(outs_o), oo])
    got_i = np.concatenate([np.array(outs_i), ii])
    so, si = net.get_state()
    for e in range(E) if E <= 40 else list(range(0, E, 17)) + [E - 1]:
        want_o, want_i, fo, fi = orc.simulate(start, end, indeg, *coef, o0[:, e], i0[:, e], x,
                                              xp, np.ascontiguousarray(fpe[:, :, e]))
        assert np.array_equal(got_o[:, :, e], want_o), e
        assert np.array_equal(got_i[:, :, e], want_i), e
        assert np.array_equal(so[:, e], fo) and np.array_equal(si[:, e], fi), e


def test_member_dataflow_matches_launches_path():
    E = 20
    end, start, indeg, coef, xp, fpe, o0, i0 = _case(2000, 3, 80, 99, E)
    x = xp[0] + 300e9 * np.arange(1, 4)
    res = []
    for mode, sync in (("dataflow", 0), ("launches", 0), ("dataflow", 1), ("launches", 1)):
        net = engine.RoutingNet(end, indeg, start[indeg == 0], slots=256, tile=16, members=E,
                                sync=sync)
        net.set_mode(mode)
        net.set_coeffs(*coef)
        net.set_state(o0, i0)
        net.load_forcing(xp, fpe)
        seq = []
        for k in range(3):
            net.run(x[k:k + 1])
            seq.append(net.fetch_outputs())
        assert net.mode()[1] == mode
        res.append((seq, net.get_state()))
    for other in res[1:]:
        for (a_o, a_i), (b_o, b_i) in zip(res[0][0], other[0]):
            assert np.array_equal(a_o, b_o) and np.array_equal(a_i, b_i)
        assert all(np.array_equal(a, b) for a, b in zip(res[0][1], other[1]))


def test_copy_state_between_plans_continues_bitexact():
    """mc_net_copy_state: one-step runs on a 384-lane plan (member dataflow), the hand-over to a
    256-lane 64-tick plan for the rest of the horizon, and back: identical to the serial runs."""
    E = 12
    end, start, indeg, coef, xp, fpe, o0, i0 = _case(6000, 5, 150, 71, E)
    heads = start[indeg == 0]
    a = engine.RoutingNet(end, indeg, heads, slots=384, members=E)
    b = engine.RoutingNet(end, indeg, heads, slots=256, tile=64, members=E)
    for net in (a, b):
        net.set_coeffs(*coef)
        net.load_forcing(xp, fpe)
    a.set_state(o0, i0)
    x = xp[0] + 300e9 * np.arange(1, 41)
    for k in range(3):
        a.run(x[k:k + 1])
    b.copy_state_from(a)
    b.run(x[3:30])
    a.copy_state_from(b)
    a.run(x[30:31])
    b.copy_state_from(a)
    b.run(x[31:])
    so, si = b.get_state()
    with pytest.raises(Exception):
        a.copy_state_from(a)
    other = engine.RoutingNet(end, indeg, heads, members=E + 1)
    with pytest.raises(Exception):
        other.copy_state_from(a)
    for e in (0, 5, E - 1):
        _, _, fo, fi = orc.simulate(start, end, indeg, *coef, o0[:, e], i0[:, e], x, xp,
                                    np.ascontiguousarray(fpe[:, :, e]), keep_outputs=False)
        assert np.array_equal(so[:, e], fo) and np.array_equal(si[:, e], fi), e


def test_conus_scale_ensemble_members_bitexact():
    """Maximum size (BASELINE configs[4] network: 2.7M reaches, 4000 outlets, deepest path ~7000
    reaches, a schedule over thousands of workgroups): a 4-member, 24-step horizon on the
    multi-launch path; every member's final state and last-step outputs bit-identical to its
    serial oracle run."""
    E, T = 4, 24
    end = synthetic.river_network(2_700_000, 4000, 7000, np.random.default_rng(44))
    n = end.size
    start = np.arange(n)
    indeg = orc.compute_indegree(start, end)
    K, X, _ = synthetic.model_arrays(n, seed=44)
    coef = orc.muskingum_coeffs(K, X, 300.0)
    xp, fpe, o0 = _members(n, E, 3, 45)
    i0 = np.stack([orc.init_inflows(start, end, o0[:, e]) for e in range(E)], axis=1)
    x = xp[0] + 300e9 * np.arange(1, T + 1)
    net = engine.RoutingNet(end, indeg, start[indeg == 0], slots=256, members=E)
    assert net.info["nwg"] > 1000
    net.set_coeffs(*coef)
    net.set_state(o0, i0)
    net.load_forcing(xp, fpe)
    net.run(x)
    assert net.mode()[1] == "launches"
    so, si = net.get_state()
    last_o, last_i = net.fetch_outputs(T - 1, T)
    for e in range(E):
        _, _, fo, fi = orc.simulate(start, end, indeg, *coef, o0[:, e], i0[:, e], x, xp,
                                    np.ascontiguousarray(fpe[:, :, e]), keep_outputs=False)
        assert np.array_equal(so[:, e], fo) and np.array_equal(si[:, e], fi), e
        assert np.array_equal(last_o[0, :, e], fo) and np.array_equal(last_i[0, :, e], fi), e
