"""CPU check of the schedule + kernel protocol: the host model of the HIP wavefront kernel
(tests/kernel_emulator.py), driven by the C++ plan, must reproduce the oracle bit-for-bit."""
import numpy as np
import pytest

from oracle import oracle as orc
from tx_fast_hydrology_amd import engine, synthetic

import kernel_emulator as emu


def _case(end, K, X, dt, o0):
    n = end.size
    start = np.arange(n)
    indeg = orc.compute_indegree(start, end)
    coef = orc.muskingum_coeffs(K, X, dt)
    i0 = orc.init_inflows(start, end, o0)
    return start, indeg, coef, i0


@pytest.mark.parametrize("chain", [2, 1, 3, 4])
@pytest.mark.parametrize("n,p_chain,slots,tile,T,rows", [
    (1, 0.0, 64, 32, 7, 3), (2, 1.0, 64, 1, 3, 2), (300, 0.9, 64, 4, 50, 5),
    (1500, 0.95, 128, 16, 40, 4), (900, 0.5, 64, 8, 13, 1), (700, 0.99, 64, 64, 1, 2),
    (2000, 0.97, 256, 32, 70, 7)])
def test_emulator_matches_oracle(n, p_chain, slots, tile, T, rows, chain):
    rng = np.random.default_rng(n * 7 + T)
    end = synthetic.random_forest(n, max(1, n // 400), rng, p_chain=p_chain)
    K = rng.uniform(1800, 7200, n)
    X = rng.uniform(0.1, 0.4, n)
    o0 = rng.uniform(0.5, 5, n)
    start, indeg, coef, i0 = _case(end, K, X, 300.0, o0)
    xp, fp = synthetic.forcing(n, rows=rows, seed=n)
    xp = xp.astype(float)
    x = xp[0] - 600e9 + 300e9 * np.arange(1, T + 1)
    want_o, want_i, _, _ = orc.simulate(start, end, indeg, *coef, o0, i0, x, xp, fp)
    plan = engine.Plan(end, indeg, start[indeg == 0], slots=slots, tile=tile, chain=chain)
    O, I = emu.run(plan, *coef, o0, i0, x, xp, fp)
    assert np.array_equal(O.T, want_o)
    assert np.array_equal(I.T, want_i)


@pytest.mark.parametrize("slots,tile,chain", [(64, 1, 2), (64, 8, 2), (128, 16, 2), (64, 8, 3),
                                              (128, 16, 4)])
def test_emulator_partial_sums_high_fan_in(slots, tile, chain):
    """Reaches with up to 30 routed upstreams read chains of partial-sum slots; the fold must
    stay bit-identical to the reference's rank-ordered accumulation."""
    rng = np.random.default_rng(slots + tile)
    end = synthetic.fan_in_forest(1500, rng)
    n = end.size
    K, X, o0 = synthetic.model_arrays(n, seed=5)
    start, indeg, coef, i0 = _case(end, K, X, 300.0, o0)
    assert indeg.max() > 8
    xp, fp = synthetic.forcing(n, rows=4, seed=6)
    xp = xp.astype(float)
    x = xp[0] + 300e9 * np.arange(1, 41)
    want_o, want_i, _, _ = orc.simulate(start, end, indeg, *coef, o0, i0, x, xp, fp)
    plan = engine.Plan(end, indeg, start[indeg == 0], slots=slots, tile=tile, chain=chain)
    assert plan.info["n_partial"] > 0
    O, I = emu.run(plan, *coef, o0, i0, x, xp, fp)
    assert np.array_equal(O.T, want_o) and np.array_equal(I.T, want_i)


@pytest.mark.parametrize("chain", [2, 4])
def test_emulator_river_network_and_golden_edges(golden, chain):
    end = synthetic.river_network(4000, 6, 150, np.random.default_rng(9))
    n = end.size
    K, X, o0 = synthetic.model_arrays(n, seed=3)
    start, indeg, coef, i0 = _case(end, K, X, 300.0, o0)
    xp, fp = synthetic.forcing(n, rows=3, seed=4)
    xp = xp.astype(float)
    x = xp[0] + 300e9 * np.arange(1, 31)
    want_o, want_i, _, _ = orc.simulate(start, end, indeg, *coef, o0, i0, x, xp, fp)
    plan = engine.Plan(end, indeg, start[indeg == 0], slots=128, tile=8, chain=chain)
    O, I = emu.run(plan, *coef, o0, i0, x, xp, fp)
    assert np.array_equal(O.T, want_o) and np.array_equal(I.T, want_i)
    g = golden("g8_ax_bu_edge.npz")
    for name in g["names"]:
        a = g[f"{name}_args"]
        plan = engine.Plan(g[f"{name}_endnodes"], g[f"{name}_indegree"], g[f"{name}_heads"],
                           slots=64, tile=4, chain=chain)
        O, I = emu.run(plan, a[0], a[1], a[2], a[3], a[5], a[4], np.array([0.0]),
                       np.array([0.0]), a[6][None, :])
        assert np.array_equal(O[:, 0], g[f"{name}_o"]), name
        assert np.array_equal(I[:, 0], g[f"{name}_i"]), name


@pytest.mark.parametrize("slots,chain,tile", [(8, 4, 16), (8, 4, 32), (4, 4, 16), (32, 1, 32)])
def test_emulator_member_plans(slots, chain, tile):
    """Narrow plans (8 or 4 lanes of 4 positions, or 32 lanes of one): the same launch / tick
    protocol on them reproduces the oracle (chained positions within a tick, cross-workgroup
    inputs from earlier launches, partial sums)."""
    rng = np.random.default_rng(slots * 100 + tile)
    end = synthetic.random_forest(2500, 6, rng, p_chain=0.9)
    n = end.size
    K, X, o0 = synthetic.model_arrays(n, seed=3)
    start, indeg, coef, i0 = _case(end, K, X, 300.0, o0)
    xp, fp = synthetic.forcing(n, rows=5, seed=4)
    xp = xp.astype(float)
    x = xp[0] + 300e9 * np.arange(1, 45)
    want_o, want_i, _, _ = orc.simulate(start, end, indeg, *coef, o0, i0, x, xp, fp)
    plan = engine.Plan(end, indeg, start[indeg == 0], slots=slots, tile=tile, chain=chain,
                       ext_cap=4)
    assert plan.info["slots"] == slots and plan.info["chain"] == chain
    O, I = emu.run(plan, *coef, o0, i0, x, xp, fp)
    assert np.array_equal(O.T, want_o)
    assert np.array_equal(I.T, want_i)


@pytest.mark.parametrize("slots,chain,tile", [(192, 2, 16), (128, 2, 16), (64, 1, 16),
                                              (192, 3, 16), (256, 2, 32)])
@pytest.mark.parametrize("kind", ["river", "fan_in"])
def test_emulator_sync_plans(slots, chain, tile, kind):
    """Chunk-synchronous plans (plan.hpp sync): unit-slack edges inside one wave, 4-tick local
    edges between the waves of a workgroup (read from the producer's output of tick k - 4).
    The emulator reads a local input only from ticks the producer already ran, so a schedule
    that violated the slack would read NaN."""
    rng = np.random.default_rng(slots * 3 + chain)
    if kind == "river":
        end = synthetic.river_network(6000, 6, 400, rng)
    else:
        end = synthetic.fan_in_forest(3000, rng)
    n = end.size
    K, X, o0 = synthetic.model_arrays(n, seed=3)
    start, indeg, coef, i0 = _case(end, K, X, 300.0, o0)
    xp, fp = synthetic.forcing(n, rows=4, seed=4)
    xp = xp.astype(float)
    x = xp[0] + 300e9 * np.arange(1, 31)
    want_o, want_i, _, _ = orc.simulate(start, end, indeg, *coef, o0, i0, x, xp, fp)
    plan = engine.Plan(end, indeg, start[indeg == 0], slots=slots, tile=tile, chain=chain,
                       sync=1)
    if slots > 64 and kind == "river":
        assert plan.info["n_local"] > 0
    O, I = emu.run(plan, *coef, o0, i0, x, xp, fp)
    assert np.array_equal(O.T, want_o) and np.array_equal(I.T, want_i)


def test_sync_plan_invariants():
    """Every unit-slack edge of a sync plan stays inside one wave of 64 lanes; every local edge
    has slack exactly 4 and stays inside its workgroup."""
    rng = np.random.default_rng(11)
    end = synthetic.river_network(20000, 20, 800, rng)
    n = end.size
    start = np.arange(n)
    indeg = orc.compute_indegree(start, end)
    plan = engine.Plan(end, indeg, start[indeg == 0], slots=192, tile=16, chain=2, sync=1)
    info, ex, ln, loc = plan.info, plan.export(), plan.export_links(), plan.export_local()
    RS = 2 * 192
    G = ex["G"]
    n_unit = n_loc = 0
    for d in np.flatnonzero(ln["flags"]):
        w = d // RS
        ne = ln["ext_off"][w + 1] - ln["ext_off"][w]
        for c in range(int(ln["up_cnt"][d])):
            code = int(ln["up4"][d] >> np.uint64(16 * c)) & 0xFFFF
            if code == 0x7FFF:
                continue
            if code & 0x8000:
                e = code & 0x7FFF
                if e >= ne:
                    src = loc["lx_src"][loc["lx_off"][w] + e - ne]
                    assert src // RS == w and G[d] == G[src] + 4
                    n_loc += 1
                continue
            u = w * RS + code
            assert G[d] == G[u] + 1
            assert (u % RS % 192) // 64 == (d % RS % 192) // 64     # same wave
            n_unit += 1
    assert n_loc == info["n_local"] > 0 and n_unit > 0
