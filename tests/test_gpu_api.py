"""GPU parity of the reference-API mirror: Muskingum / ModelCollection / AsyncSimulation /
CheckPoint routed by libmcroute.so, bit-exact against the golden vectors generated from the
reference (tests/golden/make_golden.py).  Both simulation paths run: the fused horizon (no
callbacks: one mc_run per horizon) and the step-by-step path (a bound callback: one mc_step per
step, hooks fired in between)."""
import asyncio
import hashlib

import numpy as np
import pandas as pd
import pytest

from api_helpers import golden_frame, golden_model, run
from tx_fast_hydrology_amd import engine
from tx_fast_hydrology_amd.callbacks import BaseCallback
from tx_fast_hydrology_amd.simulation import AsyncSimulation, CheckPoint

pytestmark = pytest.mark.gpu


class Recorder(BaseCallback):
    def __init__(self, model):
        self.model = model
        self.events = []

    def __on_simulation_start__(self):
        self.events.append(("start", self.model.datetime.value))

    def __on_step_start__(self):
        self.events.append(("step_start", self.model.datetime.value))

    def __on_step_end__(self):
        self.events.append(("step_end", self.model.datetime.value))

    def __on_simulation_end__(self):
        self.events.append(("end", self.model.datetime.value))


@pytest.mark.parametrize("callback", [False, True])
@pytest.mark.parametrize("name", ["g1_ynet.npz", "g3_confluence.npz", "g2_huc8.npz"])
def test_simulate_golden(golden, name, callback):
    g = golden(name)
    m = golden_model(g)
    rec = None
    if callback:
        rec = Recorder(m)
        m.bind_callback(rec, key="rec")
    o, i, t = run(m, golden_frame(g, m.reach_ids))
    assert isinstance(m._device.net, engine.RoutingNet)       # the HIP session routed it
    if "o_keep" in g:
        keep = g["keep"]
        assert np.array_equal(o[keep], g["o_keep"]) and np.array_equal(i[keep], g["i_keep"])
        sha = np.array([np.frombuffer(hashlib.sha256(np.ascontiguousarray(r)).digest(),
                                      np.uint8) for r in o])
        assert np.array_equal(sha, g["o_sha"])
        assert np.array_equal(t, g["t_ns"])
    else:
        k = len(g["o"])
        assert np.array_equal(o[:k], g["o"]) and np.array_equal(i[:k], g["i"])
        assert np.array_equal(t[:k], g["t_ns"])
    if rec is not None:
        T = len(t)
        assert rec.events[0][0] == "start" and rec.events[-1][0] == "end"
        assert [e for e, _ in rec.events[1:-1]] == ["step_start", "step_end"] * T
        assert [v for e, v in rec.events if e == "step_end"] == t.tolist()


def test_dt_change_quirk(golden):
    g = golden("g6_dt_change.npz")
    m = golden_model(g)
    for k, (q, td) in enumerate(zip(g["q"], g["td"])):
        m.step(q, timedelta=None if td < 0 else pd.Timedelta(int(td), unit="s"))
        assert np.array_equal(m.o_t_next, g["o"][k]) and np.array_equal(m.i_t_next, g["i"][k])
        assert m.datetime.value == g["t_ns"][k]


def test_fused_fallback_and_continuation(golden):
    g = golden("g3_confluence.npz")
    outs = []
    for fused in (True, False):
        m = golden_model(g)
        df = golden_frame(g, m.reach_ids)
        if not fused:
            m.bind_callback(BaseCallback(), key="noop")
        seq = []
        for k, state in enumerate(m.simulate(df, end_time=df.index[4])):
            seq.append(np.array(state.o_t_next))
            if k == 5:
                state.o_t_next = state.o_t_next * 0.75
        # a second horizon continues from the state left by the first
        for state in m.simulate(df):
            seq.append(np.array(state.o_t_next))
        outs.append(np.array(seq))
    assert np.array_equal(outs[0], outs[1])


def test_async_simulation_golden(golden):
    g = golden("g4_split_async.npz")
    whole = golden_model(g)
    df = golden_frame(g, whole.reach_ids)
    coll = whole.split(g["cuts"], create_state_space=False)
    sim = AsyncSimulation(coll, df)
    outputs = asyncio.run(sim.simulate())
    for name in g["names"]:
        p = f"sub{name}_"
        assert np.array_equal(outputs[str(name)].values, g[p + "o"]), name
        assert np.array_equal(sim.inputs[str(name)].values, g[p + "inputs"]), name
        assert np.array_equal(coll.models[str(name)].i_t_next, g[p + "init_i"]), name
    o, i, _ = run(golden_model(g), df)
    assert np.array_equal(o, g["o_whole"]) and np.array_equal(i, g["i_whole"])


def test_checkpoint_and_reload(golden):
    g = golden("g2_huc8.npz")
    m = golden_model(g)
    df = golden_frame(g, m.reach_ids)
    cp = CheckPoint(m, timedelta=3600.0)
    m.bind_callback(cp, key="cp")
    o, i, t = run(m, df)
    k = int(np.flatnonzero(t >= t[0] - 300 * 10**9 + 3600 * 10**9)[0])
    assert m.saved_states["datetime"].value == t[k]
    assert np.array_equal(m.saved_states["o_t_next"], o[k])
    # reload the checkpoint and re-route the rest without callbacks (fused): same series
    m.unbind_callback("cp")
    m.load_state()
    o2, i2, t2 = run(m, df)
    assert np.array_equal(o2, o[k + 1:]) and np.array_equal(i2, i[k + 1:])


class _Idle(BaseCallback):
    """A callback that never needs the steps: the per-sub-basin fused path still runs, but the
    device DAG does not (it requires no callbacks), so the host driver routes the collection."""

    def __idle_steps__(self):
        return True


def _split_case(n, n_cuts, seed, sibling_cuts=True):
    from api_helpers import model_dict
    from tx_fast_hydrology_amd import synthetic
    from tx_fast_hydrology_amd.muskingum import Muskingum
    rng = np.random.default_rng(seed)
    end = synthetic.river_network(n, 3, max(40, n // 60), rng)
    n = end.size
    K, X, o0 = synthetic.model_arrays(n, seed=seed)
    start = pd.Timestamp("2024-05-01T00:00:00Z")
    T = 24
    whole = Muskingum(model_dict(end, K, X, o0, start, 3600.0, name="whole"))
    idx = pd.date_range(start + pd.Timedelta(3600, unit="s"), periods=T, freq="1h", tz="UTC")
    df = pd.DataFrame(rng.gamma(2.0, 0.5, (T, n)), index=idx, columns=whole.reach_ids)
    indeg = whole.indegree
    cand = np.flatnonzero((indeg > 0) & (end != np.arange(n)))
    cuts = set(rng.choice(cand, size=n_cuts, replace=False).tolist())
    if sibling_cuts:
        # two cut reaches draining into the same entry reach: two corrections of one column
        for d in np.flatnonzero(indeg >= 2):
            ups = [u for u in np.flatnonzero(end == d) if indeg[u] > 0 and u != d]
            if len(ups) >= 2:
                cuts.update(ups[:2])
                break
    return whole, df, np.sort(np.array(sorted(cuts)))


@pytest.mark.parametrize("n,n_cuts", [(3000, 12), (20000, 60)])
def test_async_simulation_device_dag_equals_host_driver(n, n_cuts):
    """The device DAG (every sub-basin launched on its stream, corrections added on the device)
    is bit-identical to the host driver (outflow frames, corrected inputs, final states)."""
    res = []
    for device in (True, False):
        whole, df, cuts = _split_case(n, n_cuts, 7 + n)
        coll = whole.split(cuts, create_state_space=False)
        assert len(coll.models) > n_cuts
        if not device:
            for m in coll.models.values():
                m.bind_callback(_Idle(), key="idle")
        sim = AsyncSimulation(coll, df)
        outputs = asyncio.run(sim.simulate())
        res.append((outputs, sim.inputs,
                    {k: (m.o_t_next, m.i_t_next, m.o_t_prev, m.datetime)
                     for k, m in coll.models.items()}))
    (o_d, in_d, st_d), (o_h, in_h, st_h) = res
    assert o_d.keys() == o_h.keys()
    for k in o_h:
        assert np.array_equal(o_d[k].values, o_h[k].values), k
        assert o_d[k].index.equals(o_h[k].index), k
        assert np.array_equal(in_d[k].values, in_h[k].values), k
        for a, b in zip(st_d[k][:3], st_h[k][:3]):
            assert np.array_equal(a, b), k
        assert st_d[k][3] == st_h[k][3], k


@pytest.mark.parametrize("edit_step", [0, 40, 286])
def test_fused_coefficient_edit_mid_horizon_bitexact(golden, edit_step):
    """set_transmissive_boundary inside a simulate loop (reference muskingum.py:567-571): the
    reference reads the coefficients at every step (:450-453), so the edit applies from the next
    step.  The mirror's fused horizon notices it and routes the rest step by step: every step
    bit-exact against the oracle's run with the coefficients changed after step `edit_step`."""
    from oracle import oracle as orc
    g = golden("g2_huc8.npz")
    m = golden_model(g)
    df = golden_frame(g, m.reach_ids)
    cut = [3, 17, 250]
    coef0 = [np.array(a) for a in (m.alpha, m.beta, m.chi, m.gamma)]
    o0, i0 = np.array(m.o_t_next), np.array(m.i_t_next)
    o, i, t = [], [], []
    for k, state in enumerate(m.simulate(df)):
        o.append(np.array(state.o_t_next))
        i.append(np.array(state.i_t_next))
        t.append(state.datetime.value)
        if k == edit_step:
            state.set_transmissive_boundary(cut)
    o, i = np.array(o), np.array(i)
    x = np.array(t, dtype=np.int64).astype(float)
    xp = df.index.astype(np.int64).astype(float).values
    fp = np.ascontiguousarray(df.values)
    start = np.asarray(m.startnodes)
    coef1 = [a.copy() for a in coef0]
    for a, v in zip(coef1, (1.0, 0.0, 0.0, 0.0)):
        a[cut] = v
    e = edit_step + 1
    wo1, wi1, fo, fi = orc.simulate(start, m.endnodes, m.indegree, *coef0, o0, i0, x[:e], xp, fp)
    wo2, wi2, _, _ = orc.simulate(start, m.endnodes, m.indegree, *coef1, fo, fi, x[e:], xp, fp)
    assert np.array_equal(o, np.concatenate([wo1, wo2]))
    assert np.array_equal(i, np.concatenate([wi1, wi2]))
    assert isinstance(m._device.net, engine.RoutingNet)


def test_device_dag_give_up_falls_back_to_host_driver():
    """an upstream sub-basin's dataflow horizon that gives up (patience < 0) is
    re-routed by its session at the fetch, but the corrections already taken from it used
    incomplete outflows -- the device DAG detects the re-route and routes the collection with
    the host driver instead: still bit-identical to the host driver's run."""
    res = []
    rerouted = 0
    for device in (True, False):
        whole, df, cuts = _split_case(20000, 60, 7 + 20000)
        coll = whole.split(cuts, create_state_space=False)
        if device:
            for m in coll.models.values():
                m._device.session(m).set_flow_patience(-1)
        else:
            for m in coll.models.values():
                m.bind_callback(_Idle(), key="idle")
        sim = AsyncSimulation(coll, df)
        outputs = asyncio.run(sim.simulate())
        if device:
            rerouted = sum(m._device.net.reroutes() for m in coll.models.values())
        res.append((outputs, sim.inputs,
                    {k: (m.o_t_next, m.i_t_next, m.o_t_prev) for k, m in coll.models.items()}))
    assert rerouted > 0                      # some horizon gave up and was re-routed
    (o_d, in_d, st_d), (o_h, in_h, st_h) = res
    for k in o_h:
        assert np.array_equal(o_d[k].values, o_h[k].values), k
        assert np.array_equal(in_d[k].values, in_h[k].values), k
        for a, b in zip(st_d[k], st_h[k]):
            assert np.array_equal(a, b), k
