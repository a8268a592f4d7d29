"""GPU parity of the member-vector ensemble sweep (csrc/vector.hip): lanes are members, one
wave routes 64 / H members of H node slots.  Every member column must be bit-identical to the
serial oracle run on that member's forcing and initial state, at every member width (E = 64:
one node per wave instruction; 32 and 16: two and four), both lane chains, several launch
lengths, continued horizons and the full Texas network."""
import numpy as np
import pytest

from oracle import oracle as orc
from tx_fast_hydrology_amd import engine, synthetic

from test_gpu_ensemble import _case

pytestmark = pytest.mark.gpu


def _check_members(net, start, end, indeg, coef, xp, fpe, o0, i0, x, got_o, got_i, members):
    so, si = net.get_state()
    for e in members:
        want_o, want_i, fo, fi = orc.simulate(start, end, indeg, *coef, o0[:, e], i0[:, e], x,
                                              xp, np.ascontiguousarray(fpe[:, :, e]))
        assert np.array_equal(got_o[:, :, e], want_o), e
        assert np.array_equal(got_i[:, :, e], want_i), e
        assert np.array_equal(so[:, e], fo) and np.array_equal(si[:, e], fi), e


# (nodes per wave instruction, waves per workgroup): every instantiated shape (kernels.hpp
# MCR_VEC_SHAPES); 0 = the automatic choice
@pytest.mark.parametrize("n,E,chain,tile,T,shape", [
    (3000, 64, 1, 16, 60, (0, 0)), (3000, 64, 1, 16, 33, (1, 8)), (2600, 64, 1, 32, 41, (1, 16)),
    (2500, 32, 1, 32, 40, (2, 8)), (2500, 64, 1, 32, 40, (2, 16)), (2500, 16, 1, 16, 37, (4, 4)),
    (2200, 16, 1, 16, 29, (4, 8)), (2300, 48, 1, 16, 31, (4, 16)), (4000, 32, 2, 16, 50, (2, 16)),
    (2000, 16, 2, 48, 30, (4, 8)), (2100, 32, 2, 16, 30, (4, 16)), (1500, 128, 1, 64, 25, (0, 0)),
    (1800, 48, 1, 16, 20, (0, 0))])
def test_vector_members_bitexact(n, E, chain, tile, T, shape):
    end, start, indeg, coef, xp, fpe, o0, i0 = _case(n, 4, 120, n + E + chain, E)
    n = end.size
    x = xp[0] + 300e9 * np.arange(1, T + 1)
    net = engine.RoutingNet(end, indeg, start[indeg == 0], slots=64, chain=chain, tile=tile,
                            members=E)
    net.set_mode("vector")
    net.set_vector_shape(*shape)
    net.set_coeffs(*coef)
    net.set_state(o0, i0)
    got_o, got_i = net.simulate(x, xp, fpe)
    assert net.mode()[1] == "vector"
    assert got_o.shape == (T, n, E)
    ser_o, ser_i = net.fetch_series()
    assert np.array_equal(ser_o, got_o.transpose(1, 0, 2))
    assert np.array_equal(ser_i, got_i.transpose(1, 0, 2))
    _check_members(net, start, end, indeg, coef, xp, fpe, o0, i0, x, got_o, got_i,
                   sorted({0, 1, E // 2, E - 1}))


def test_vector_matches_launches_and_continues():
    """Two continued horizons through the member-vector path equal the multi-launch path on
    the same plan bit for bit (outputs, inflows and state), and a one-step run in between (the
    member dataflow) hands its state over."""
    E = 32
    end, start, indeg, coef, xp, fpe, o0, i0 = _case(3500, 5, 150, 91, E)
    heads = start[indeg == 0]
    nets = []
    for mode in ("vector", "launches"):
        nt = engine.RoutingNet(end, indeg, heads, slots=64, chain=2, tile=16, members=E)
        nt.set_mode(mode)
        nt.set_coeffs(*coef)
        nt.set_state(o0, i0)
        nt.load_forcing(xp, fpe)
        nets.append(nt)
    x = xp[0] + 300e9 * np.arange(1, 71)
    for part in (x[:29], x[29:30], x[30:]):
        outs = []
        for nt in nets:
            if part.size == 1:
                nt.set_mode("auto")           # one step: the member dataflow
            nt.run(part)
            outs.append(nt.fetch_outputs() + nt.get_state())
            if part.size == 1:
                nt.set_mode("vector" if nt is nets[0] else "launches")
        assert nets[0].mode()[1] in ("vector", "dataflow")
        for a, b in zip(*outs):
            assert np.array_equal(a, b)


def test_vector_texas_members_bitexact():
    """Full Texas (190k reaches, deepest path ~1500) with 64 members for a 36-step horizon: the
    first, a middle and the last member against the serial oracle."""
    E, T = 64, 36
    end = synthetic.river_network(190_000, 300, 1500, np.random.default_rng(0))
    n = end.size
    start = np.arange(n)
    indeg = orc.compute_indegree(start, end)
    K, X, o_base = synthetic.model_arrays(n, seed=0)
    coef = orc.muskingum_coeffs(K, X, 300.0)
    xp, fp = synthetic.forcing(n, rows=4, seed=1)
    xp = xp.astype(float)
    o0, fpe = synthetic.ensemble(o_base, fp, E, seed=5)
    i0 = np.zeros(o0.shape)
    np.add.at(i0, end, o0)
    x = xp[0] + 300e9 * np.arange(1, T + 1)
    net = engine.RoutingNet(end, indeg, start[indeg == 0], slots=64, chain=1, tile=32, members=E)
    net.set_mode("vector")
    net.set_coeffs(*coef)
    net.set_state(o0, i0)
    got_o, got_i = net.simulate(x, xp, fpe)
    assert net.mode()[1] == "vector"
    _check_members(net, start, end, indeg, coef, xp, fpe, o0, i0, x, got_o, got_i, [0, 37, 63])


def test_vector_mode_rejects_ineligible():
    end, start, indeg, coef, xp, fpe, o0, i0 = _case(800, 2, 60, 5, 5)
    net = engine.RoutingNet(end, indeg, start[indeg == 0], slots=64, members=5)
    net.set_mode("vector")
    net.set_coeffs(*coef)
    net.set_state(o0, i0)
    net.load_forcing(xp, fpe)
    with pytest.raises(RuntimeError, match="member-vector"):
        net.run(xp[0] + 300e9 * np.arange(1, 5))
