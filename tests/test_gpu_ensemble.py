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


@pytest.mark.parametrize("n,E,slots,T", [(3000, 5, 256, 60), (1200, 64, 128, 25),
                                         (5000, 3, 448, 100)])
def test_ensemble_members_bitexact(n, E, slots, T):
    end, start, indeg, coef, xp, fpe, o0, i0 = _case(n, 4, 120, n + E, E)
    n = end.size
    x = xp[0] + 300e9 * np.arange(1, T + 1)
    net = engine.RoutingNet(end, indeg, start[indeg == 0], slots=slots, members=E)
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
