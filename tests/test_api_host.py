"""CPU tests of the reference-API mirror (tx_fast_hydrology_amd.muskingum / simulation / io /
callbacks): model descriptions, validation, JSON files, split, and the host logic of the fused
and step-by-step simulation paths.

Routing in this file goes through ``OracleNet`` (tests/api_helpers.py), a CPU test double of the
device session, so the host bookkeeping can be checked without a GPU; the same scenarios run on
the real HIP path in tests/test_gpu_api.py.  Expected values are the golden vectors generated
from the reference (tests/golden/make_golden.py).
"""
import asyncio
import hashlib
import json

import numpy as np
import pandas as pd
import pytest

from api_helpers import golden_frame, golden_model, model_dict, run, use_oracle_device
from tx_fast_hydrology_amd import io as tio
from tx_fast_hydrology_amd.callbacks import BaseCallback
from tx_fast_hydrology_amd.muskingum import (ModelCollection, Muskingum, load_model_file,
                                             load_nhd_geojson)
from tx_fast_hydrology_amd.simulation import AsyncSimulation, CheckPoint

T0 = pd.Timestamp("2024-05-01T00:00:00Z")


def _g10_model(golden):
    g = golden("g10_model_io.npz")
    return g, Muskingum(model_dict(g["endnodes"], g["K"], g["X"], g["o0"], T0, 300))


# ------------------------------------------------------------------ model description / setup
def test_setup_quirks_match_reference(golden):
    g, m = _g10_model(golden)
    assert np.array_equal(m.indegree, g["indegree"])
    assert np.array_equal(m.i_t_next, g["init_i"])          # add.at incl. self-loops
    assert np.array_equal(m.o_t_prev, m.o_t_next) and np.array_equal(m.i_t_prev, m.i_t_next)
    for dt in (60, 300, 900, 3600, 86400):
        want = g[f"dt{dt}"]
        got = np.stack([m.compute_alpha(m.K, m.X, float(dt)), m.compute_beta(m.K, m.X, float(dt)),
                        m.compute_chi(m.K, m.X, float(dt)), m.compute_gamma(m.K, m.X, float(dt))])
        assert np.array_equal(got, want), dt
    assert np.array_equal(m.alpha, g["dt300"][0]) and np.array_equal(m.gamma, g["dt300"][3])
    assert m.dt == 300.0 and m.saved_states["datetime"] == T0


def test_json_matches_reference_encoder(golden, tmp_path):
    g, m = _g10_model(golden)
    assert json.dumps(m.info, cls=tio.ModelEncoder) == str(g["json"])
    path = str(tmp_path / "m.json")
    m.dump_model_file(path)
    m2 = Muskingum.from_model_file(path)
    for key in ("startnodes", "endnodes", "K", "X", "o_t_next", "indegree", "alpha", "i_t_next"):
        assert np.array_equal(getattr(m2, key), getattr(m, key)), key
    assert m2.datetime == m.datetime and m2.timedelta == m.timedelta and m2.name == m.name
    obj = load_model_file(path)
    assert obj["n"] == m.n and obj["startnodes"].dtype == np.int64
    assert set(load_model_file(path, load_optional=False)) == {"dx", "paths", "n"}


def test_load_model_validation():
    n = 3
    good = model_dict(np.array([1, 2, 2]), np.full(n, 3600.0), np.full(n, 0.2), np.ones(n), T0, 60)
    bad = dict(good)
    del bad["K"]
    with pytest.raises(ValueError):
        Muskingum(bad)
    bad = dict(good, endnodes=good["endnodes"].astype(np.int32))
    with pytest.raises(TypeError):
        Muskingum(bad)
    bad = dict(good, K=np.full(n + 1, 3600.0))
    with pytest.raises(ValueError):
        Muskingum(bad)
    with pytest.raises(TypeError):
        Muskingum(42)
    m = Muskingum(dict(good))
    with pytest.raises(TypeError):
        m.datetime = "2024-05-01"
    with pytest.raises(ValueError):
        m.datetime = pd.Timestamp("2024-05-01")
    with pytest.raises(TypeError):
        m.timedelta = 60
    m.name = 7
    assert m.name == "7"


def test_defaults_and_lazy_state_space():
    n = 4
    d = model_dict(np.array([2, 2, 3, 3]), np.full(n, 3600.0), np.full(n, 0.29), np.ones(n), T0,
                   3600)
    for key in ("dx", "paths"):
        del d[key]
    m = Muskingum(d)
    assert m.dx is None and m.paths == []
    assert m._A is None                       # not materialised by the constructor
    assert m.A.shape == (n, n) and not m.A.any()
    m2 = Muskingum(dict(d), create_state_space=True)
    # o_next = A o_prev + B q for a network at rest: check against one explicit step
    heads = m2.startnodes[m2.indegree == 0]
    assert m2.A[3, 2] != 0 and m2.B[0, 0] == m2.gamma[0] and len(heads) == 2


def test_nhd_geojson(tmp_path):
    feats = [{"attributes": {"COMID": c, "toCOMID": t, "Shape_Length": 1.5 * k},
              "geometry": {"paths": [[[k, 0.0], [k + 1.0, 1.0]]]}}
             for k, (c, t) in enumerate([(11, 13), (12, 13), (13, 99)])]
    path = tmp_path / "nhd.json"
    path.write_text(json.dumps({"features": feats}))
    obj = load_nhd_geojson(str(path))
    assert obj["reach_ids"] == ["11", "12", "13"]
    assert obj["endnodes"].tolist() == [2, 2, 2]            # 99 is outside: outlet self-loop
    assert np.array_equal(obj["K"], np.full(3, 3600.0)) and obj["o_t"][0] == 1e-3
    m = Muskingum.from_nhd_geojson(str(path))
    assert m.indegree.tolist() == [0, 0, 2]


class _IdleCb(BaseCallback):
    def __idle_steps__(self):
        return True


# ------------------------------------------------------------------ routing host logic
@pytest.mark.parametrize("callback", [False, True])
def test_simulate_paths_golden(golden, monkeypatch, callback):
    nets = use_oracle_device(monkeypatch)
    for name, n_steps in (("g1_ynet.npz", None), ("g3_confluence.npz", None)):
        g = golden(name)
        m = golden_model(g)
        if callback:
            m.bind_callback(BaseCallback(), key="noop")
        o, i, t = run(m, golden_frame(g, m.reach_ids))
        k = len(g["o"])       # g3 keeps the first 50 of 54 steps
        assert np.array_equal(o[:k], g["o"]) and np.array_equal(i[:k], g["i"]), name
        assert np.array_equal(t[:k], g["t_ns"]), name
        assert m.o_t_next.flags.writeable
    assert all((net.runs == 0) == callback for net in nets)


def test_huc8_day_golden(golden, monkeypatch):
    use_oracle_device(monkeypatch)
    g = golden("g2_huc8.npz")
    m = golden_model(g)
    o, i, t = run(m, golden_frame(g, m.reach_ids))
    assert np.array_equal(t, g["t_ns"])
    assert np.array_equal(o[g["keep"]], g["o_keep"]) and np.array_equal(i[g["keep"]], g["i_keep"])
    sha = np.array([np.frombuffer(hashlib.sha256(np.ascontiguousarray(r)).digest(), np.uint8)
                    for r in o])
    assert np.array_equal(sha, g["o_sha"])


def test_column_order_check_sees_reach_id_edits(golden, monkeypatch):
    """The frame-in-reach-order check is cached per column Index; an in-place edit of the
    model's reach_ids list (two ids swapped) must select the frame's columns again."""
    use_oracle_device(monkeypatch)
    g = golden("g1_ynet.npz")
    m = golden_model(g)
    df = golden_frame(g, list(m.reach_ids))
    assert not np.array_equal(df.iloc[:, 0], df.iloc[:, 1])
    o_ref, _, _ = run(m, df)                     # caches the check for df.columns
    m.datetime = pd.Timestamp(int(g["start_ns"]), tz="UTC")
    m.init_states(o_t_next=g["o0"])
    m.reach_ids[0], m.reach_ids[1] = m.reach_ids[1], m.reach_ids[0]
    o_sw, _, _ = run(m, df)
    swapped = pd.DataFrame(df[m.reach_ids].values, index=df.index, columns=df.columns)
    o_exp, _, _ = run(golden_model(g), swapped)
    assert np.array_equal(o_sw, o_exp) and not np.array_equal(o_sw, o_ref)


def test_dt_change_quirk(golden, monkeypatch):
    use_oracle_device(monkeypatch)
    g = golden("g6_dt_change.npz")
    m = golden_model(g)
    for k, (q, td) in enumerate(zip(g["q"], g["td"])):
        m.step(q, timedelta=None if td < 0 else pd.Timedelta(int(td), unit="s"))
        assert np.array_equal(m.o_t_next, g["o"][k]) and np.array_equal(m.i_t_next, g["i"][k])
        assert m.datetime.value == g["t_ns"][k]
        assert np.array_equal(np.stack([m.alpha, m.beta, m.chi, m.gamma]), g["coef"][k])


def test_fused_horizon_falls_back_when_state_replaced(golden, monkeypatch):
    use_oracle_device(monkeypatch)
    g = golden("g3_confluence.npz")
    df = None
    results = []
    for fused in (True, False):
        m = golden_model(g)
        df = golden_frame(g, m.reach_ids)
        if not fused:
            m.bind_callback(BaseCallback(), key="noop")
        out = []
        for k, state in enumerate(m.simulate(df)):
            assert state.o_t_next.flags.writeable and state.i_t_next.flags.writeable
            out.append(np.array(state.o_t_next))
            if k == 7:    # a consumer nudges the state: the rest routes from it
                state.o_t_next = state.o_t_next * 1.5
                state.i_t_next = np.array(state.i_t_next)
        results.append(np.array(out))
    assert np.array_equal(results[0], results[1])
    assert not np.array_equal(results[0][8:50], g["o"][8:])
    assert np.array_equal(results[0][:8], g["o"][:8])


def test_fused_horizon_routes_in_place_edits(golden, monkeypatch):
    """``state.o_t_next[j] = obs`` inside the loop (valid in the reference, which allocates fresh
    arrays every step) is routed like the step-by-step path routes it."""
    use_oracle_device(monkeypatch)
    g = golden("g3_confluence.npz")
    results = []
    for fused in (True, False):
        m = golden_model(g)
        df = golden_frame(g, m.reach_ids)
        if not fused:
            m.bind_callback(BaseCallback(), key="noop")
        out = []
        for k, state in enumerate(m.simulate(df)):
            out.append(np.array(state.o_t_next))
            if k == 5:
                state.o_t_next[3] = 7.25
                state.i_t_next *= 0.5
        results.append(np.array(out))
    assert np.array_equal(results[0], results[1])
    assert not np.array_equal(results[0][6:50], g["o"][6:])


COEF_EDITS = {
    "transmissive": lambda m: m.set_transmissive_boundary([2, 5]),
    "element": lambda m: m.alpha.__setitem__(4, 0.25),
    "inplace_ufunc": lambda m: m.beta.__imul__(1.01),
    "copyto": lambda m: np.copyto(m.chi, m.chi * 0.99),
    "ufunc_at": lambda m: np.add.at(m.gamma, [1, 1, 3], 1e-3),
    "rebind": lambda m: setattr(m, "alpha", np.array(m.alpha) * 1.02),
    "dt_recompute": lambda m: m.compute_muskingum_coeffs(dt=450.0),
}


@pytest.mark.parametrize("edit", sorted(COEF_EDITS))
def test_fused_horizon_follows_coefficient_edits(golden, monkeypatch, edit):
    """The reference reads alpha..gamma at every step (muskingum.py:450-453): a coefficient
    change between two yields of a fused horizon applies from the next step, exactly as the
    step-by-step path (and the reference) routes it."""
    use_oracle_device(monkeypatch)
    g = golden("g3_confluence.npz")
    results = []
    for fused in (True, False):
        m = golden_model(g)
        df = golden_frame(g, m.reach_ids)
        if not fused:
            m.bind_callback(BaseCallback(), key="noop")
        out = []
        for k, state in enumerate(m.simulate(df)):
            out.append((np.array(state.o_t_next), np.array(state.i_t_next)))
            if k == 9:
                COEF_EDITS[edit](state)
        results.append(out)
    fo, so = (np.array([r[0] for r in res]) for res in results)
    fi, si = (np.array([r[1] for r in res]) for res in results)
    assert np.array_equal(fo, so) and np.array_equal(fi, si)
    assert not np.array_equal(fo[10:50], g["o"][10:])      # the edit changed the routing
    assert np.array_equal(fo[:10], g["o"][:10])


def test_coefficient_tracking_is_per_model():
    m = Muskingum(model_dict(np.array([2, 2, 3, 3]), np.full(4, 3600.0), np.full(4, 0.2),
                             np.ones(4), T0, 300))
    r0 = m._coef_rev[0]
    c = m.copy()
    c.alpha[0] = 9.0
    assert m._coef_rev[0] == r0 and m.alpha[0] != 9.0      # copies track (and own) their own
    m.alpha[1] = 0.5
    assert m._coef_rev[0] == r0 + 1
    view = m.beta[1:3]
    view[0] = 0.0                                           # writes through views count
    assert m._coef_rev[0] == r0 + 2
    before = m._coef_rev[0]
    _ = m.alpha * 2 + m.chi.sum()                           # reads never do
    assert m._coef_rev[0] == before and type(m.alpha * 2) is np.ndarray
    import pickle
    p = pickle.loads(pickle.dumps(m))
    p.gamma[0] = 1.0
    assert m._coef_rev[0] == before and p.gamma[0] == 1.0


def test_fused_horizon_final_state_owns_its_arrays(golden, monkeypatch):
    """The last two yielded steps are copies: after the horizon the model's state arrays hold
    no fetched block alive."""
    use_oracle_device(monkeypatch)
    g = golden("g3_confluence.npz")
    m = golden_model(g)
    for _ in m.simulate(golden_frame(g, m.reach_ids)):
        pass
    for key in ("o_t_next", "i_t_next", "o_t_prev", "i_t_prev"):
        assert getattr(m, key).base is None, key


def test_fused_horizon_early_break_leaves_writable_state(golden, monkeypatch):
    use_oracle_device(monkeypatch)
    g = golden("g3_confluence.npz")
    m = golden_model(g)
    for k, _ in enumerate(m.simulate(golden_frame(g, m.reach_ids))):
        if k == 3:
            break
    for key in ("o_t_next", "i_t_next", "o_t_prev", "i_t_prev"):
        assert getattr(m, key).flags.writeable, key
    m.init_states(o_t_next=np.ones(m.n))          # in-place writes of the reference API
    assert np.array_equal(m.o_t_next, np.ones(m.n))


def test_idle_callbacks_switch_to_fused(golden, monkeypatch):
    """A checkpoint that has been taken is idle: the rest of the horizon is one fused call."""
    nets = use_oracle_device(monkeypatch)
    g = golden("g3_confluence.npz")
    m = golden_model(g)
    cp = CheckPoint(m, timedelta=3 * float(g["dt"]))
    m.bind_callback(cp, key="cp")
    o, i, t = run(m, golden_frame(g, m.reach_ids))
    assert np.array_equal(o[:50], g["o"]) and np.array_equal(i[:50], g["i"])
    assert nets[-1].steps == 3 and nets[-1].runs == 1


def test_split_topology_golden(golden):
    g = golden("g4_split_async.npz")
    whole = golden_model(g)
    coll = whole.split(g["cuts"], create_state_space=False)
    assert sorted(coll.models, key=int) == [str(x) for x in g["names"]]
    for name in g["names"]:
        sub = coll.models[str(name)]
        p = f"sub{name}_"
        assert [int(r[1:]) for r in sub.reach_ids] == g[p + "reach_ids"].tolist()
        for key in ("startnodes", "endnodes", "indegree"):
            assert np.array_equal(getattr(sub, key), g[p + key]), (name, key)
        sinks = np.array([[int(c.downstream_model.name), c.upstream_index, c.downstream_index]
                          for c in sub.sinks]).reshape(-1, 3)
        assert np.array_equal(sinks, g[p + "sinks"])
    # the whole model is untouched
    assert np.array_equal(whole.endnodes, g["endnodes"])


@pytest.mark.parametrize("driver", ["device_dag", "host"])
def test_async_simulation_golden(golden, monkeypatch, driver):
    """Both AsyncSimulation drivers against the reference's own split + AsyncSimulation run:
    the device DAG (no callbacks; OracleNet stands in for the sessions and their on-device
    lateral corrections) and the host driver (an idle callback on every sub-basin)."""
    use_oracle_device(monkeypatch)
    g = golden("g4_split_async.npz")
    whole = golden_model(g)
    df = golden_frame(g, whole.reach_ids)
    coll = whole.split(g["cuts"], create_state_space=False)
    if driver == "host":
        for m in coll.models.values():
            m.bind_callback(_IdleCb(), key="idle")
    sim = AsyncSimulation(coll, df)
    outputs = asyncio.run(sim.simulate())
    assert hasattr(sim, "dag_phases") == (driver == "device_dag")
    for name in g["names"]:
        p = f"sub{name}_"
        assert np.array_equal(outputs[str(name)].values, g[p + "o"]), name
        assert np.array_equal(outputs[str(name)].index.asi8, g[p + "t_ns"])
        assert np.array_equal(sim.inputs[str(name)].values, g[p + "inputs"]), name
        # (the fixture's "init_i" is the sub-model inflow state after the run)
        assert np.array_equal(coll.models[str(name)].i_t_next, g[p + "init_i"]), name
    o, i, _ = run(golden_model(g), df)
    assert np.array_equal(o, g["o_whole"]) and np.array_equal(i, g["i_whole"])


def test_collection_file_round_trip(golden, tmp_path):
    g = golden("g4_split_async.npz")
    coll = golden_model(g).split(g["cuts"], create_state_space=False)
    path = str(tmp_path / "coll.json")
    coll.dump_model_collection(path)
    back = ModelCollection.from_file(path)
    assert set(back.models) == set(coll.models)
    for name, model in coll.models.items():
        other = back.models[name]
        assert np.array_equal(other.endnodes, model.endnodes)
        assert [(c.downstream_model.name, c.upstream_index, c.downstream_index)
                for c in other.sinks] == [(c.downstream_model.name, int(c.upstream_index),
                                           int(c.downstream_index)) for c in model.sinks]
    assert back.datetime == coll.datetime and back.timedelta == coll.timedelta


def test_checkpoint_saves_once(golden, monkeypatch):
    use_oracle_device(monkeypatch)
    g = golden("g3_confluence.npz")
    m = golden_model(g)
    df = golden_frame(g, m.reach_ids)
    cp = CheckPoint(m, timedelta=3 * float(g["dt"]))
    m.bind_callback(cp, key="cp")
    o, i, t = run(m, df)
    k = int(np.flatnonzero(t >= t[0] + 2 * int(g["dt"] * 1e9))[0])
    assert m.saved_states["datetime"].value == t[k]
    assert np.array_equal(m.saved_states["o_t_next"], g["o"][k]) and k < 50
    m.load_state()
    assert np.array_equal(m.o_t_next, g["o"][k]) and m.datetime.value == t[k]


def test_copy_does_not_share_device_session(golden, monkeypatch):
    use_oracle_device(monkeypatch)
    g = golden("g1_ynet.npz")
    m = golden_model(g)
    m.step(np.ones(m.n))
    c = m.copy()
    assert c._device.net is None and m._device.net is not None
    assert np.array_equal(c.o_t_next, m.o_t_next) and c.o_t_next is not m.o_t_next


def test_close_with_held_generator_keeps_state_readable(golden, monkeypatch):
    """close() inside a fused horizon settles the lazy inflow rows first, so the
    state stays readable, the generator can finish and the model routes again."""
    use_oracle_device(monkeypatch)
    g = golden("g3_confluence.npz")
    m = golden_model(g)
    df = golden_frame(g, m.reach_ids)
    gen = m.simulate(df)
    for k, _ in enumerate(gen):
        if k == 5:
            break
    m.close()
    assert np.array_equal(m.i_t_next, g["i"][5]) and np.array_equal(m.i_t_prev, g["i"][4])
    gen.close()                                     # its finally settles on the closed session
    m.step(np.zeros(m.n))                           # a new session
    assert np.isfinite(m.o_t_next).all()


def test_lazy_inflow_block_refuses_stale_or_closed_session(monkeypatch):
    from api_helpers import OracleNet
    from tx_fast_hydrology_amd.muskingum import _InflowBlock
    net = OracleNet(np.array([1, 1]), np.array([1, 0]), np.array([0]))
    net.out_i = np.zeros((4, 2))
    net.out_o = np.zeros((4, 2))
    blk = _InflowBlock(net, 0, 2, 2)
    net.runs += 1                                    # the session routed again
    with pytest.raises(RuntimeError, match="routed again"):
        blk.fetch()
    blk = _InflowBlock(net, 0, 2, 2)
    net.close()
    with pytest.raises(RuntimeError, match="closed"):
        blk.fetch()


def test_unpickle_model_with_eager_inflow_keys(golden):
    """A model pickled before the inflows became lazy properties keeps its inflow state."""
    import pickle
    g, m = _g10_model(golden)
    state = m.__getstate__()
    state["i_t_next"] = state.pop("_i_t_next")
    state["i_t_prev"] = state.pop("_i_t_prev")
    m2 = Muskingum.__new__(Muskingum)
    m2.__setstate__(state)
    assert np.array_equal(m2.i_t_next, m.i_t_next) and np.array_equal(m2.i_t_prev, m.i_t_prev)
    m3 = pickle.loads(pickle.dumps(m2))
    assert np.array_equal(m3.i_t_next, m.i_t_next)
