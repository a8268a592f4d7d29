"""Generate the golden vectors under tests/golden/ from the reference implementation.

TEST INFRASTRUCTURE ONLY.  Runs in the build container (where /root/reference exists), never on
the GPU box and never from the product.  The committed ``*.npz`` outputs are plain data (inputs +
expected outputs); no reference source or bytecode leaves this script.

How the reference is executed
-----------------------------
``tx_fast_hydrology/nutils.py:3`` imports ``numba`` which is not installed in this image.  All the
``@njit`` kernels in ``nutils.py`` are float64 code without ``fastmath``: numba lowers them to IEEE
double operations in source order with no FMA contraction, i.e. the same arithmetic CPython
performs.  The script therefore puts a throw-away module on ``sys.path`` whose ``njit`` is the
identity decorator and whose ``prange`` is ``range``, and a small
``asyncio.TaskGroup`` backport (``simulation.py:114`` needs Python >= 3.11; this image has 3.10).
Both live in a temporary directory that is deleted afterwards.  ``sys.dont_write_bytecode`` keeps
the read-only reference tree untouched.

Usage:  python tests/golden/make_golden.py [g11 ...]  (writes tests/golden/*.npz; names: only those)
"""
from __future__ import annotations

import asyncio
import hashlib
import json
import os
import shutil
import sys
import tempfile
import warnings

import numpy as np
import pandas as pd

REFERENCE = os.environ.get("TXFH_REFERENCE", "/root/reference")
OUT_DIR = os.path.dirname(os.path.abspath(__file__))

_SHIM = '''
def njit(*args, **kwargs):
    if len(args) == 1 and callable(args[0]) and not kwargs:
        return args[0]
    def deco(f):
        return f
    return deco
prange = range
'''


class _TaskGroup:
    """Minimal asyncio.TaskGroup for Python 3.10 (used only to drive the reference here)."""

    async def __aenter__(self):
        self._tasks = []
        return self

    def create_task(self, coro):
        task = asyncio.get_running_loop().create_task(coro)
        self._tasks.append(task)
        return task

    async def __aexit__(self, et, ev, tb):
        while True:
            pending = [t for t in self._tasks if not t.done()]
            if not pending:
                break
            await asyncio.wait(pending)
        for t in self._tasks:
            if t.exception() is not None:
                raise t.exception()
        return False


def _import_reference():
    sys.dont_write_bytecode = True
    tmp = tempfile.mkdtemp(prefix="numba_shim_")
    os.makedirs(os.path.join(tmp, "numba"))
    with open(os.path.join(tmp, "numba", "__init__.py"), "w") as f:
        f.write(_SHIM)
    sys.path.insert(0, tmp)
    sys.path.insert(0, REFERENCE)
    if not hasattr(asyncio, "TaskGroup"):
        asyncio.TaskGroup = _TaskGroup
    import tx_fast_hydrology.muskingum as mk
    import tx_fast_hydrology.nutils as nu
    import tx_fast_hydrology.simulation as sim
    import tx_fast_hydrology.da as da
    import tx_fast_hydrology.io as tio
    return tmp, mk, nu, sim, da, tio


def sha(a: np.ndarray) -> bytes:
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).digest()


def random_forest(n, n_outlets, rng, window=None, p_window=0.0):
    """Random forest in topological order, then randomly permuted (NHD order != topo order).

    Node k >= n_outlets drains to an earlier node: with prob ``p_window`` one of the ``window``
    most recent nodes (long chains), otherwise a uniformly random earlier node.
    Returns endnodes (int64) with outlets as self-loops.
    """
    parent = np.empty(n, dtype=np.int64)
    parent[:n_outlets] = np.arange(n_outlets)
    for k in range(n_outlets, n):
        if window and rng.random() < p_window:
            parent[k] = k - 1 - rng.integers(0, min(window, k))
        else:
            parent[k] = rng.integers(0, k)
    perm = rng.permutation(n)
    endnodes = np.empty(n, dtype=np.int64)
    endnodes[perm] = perm[parent]
    return endnodes


def make_model_dict(mk, endnodes, K, X, o_t, start, dt_s, name="m"):
    n = endnodes.size
    return {
        "name": name,
        "datetime": start,
        "timedelta": pd.to_timedelta(dt_s, unit="s"),
        "reach_ids": [f"r{i}" for i in range(n)],
        "startnodes": np.arange(n, dtype=np.int64),
        "endnodes": endnodes.astype(np.int64),
        "K": K.astype(np.float64),
        "X": X.astype(np.float64),
        "o_t": o_t.astype(np.float64),
        "dx": np.ones(n, dtype=np.float64),
        "paths": [[[[0.0, 0.0], [1.0, 1.0]]] for _ in range(n)],
    }


def run_simulate(model, df, every=1):
    """Drive Muskingum.simulate and record o/i of each step (reference CS-1)."""
    os_, is_, ts = [], [], []
    for state in model.simulate(df):
        os_.append(state.o_t_next.copy())
        is_.append(state.i_t_next.copy())
        ts.append(state.datetime.value)
    return np.array(os_), np.array(is_), np.array(ts, dtype=np.int64)


def forcing_frame(reach_ids, start, periods, freq, rng):
    idx = pd.date_range(start, periods=periods, freq=freq, tz="UTC")
    vals = rng.gamma(2.0, 0.5, size=(periods, len(reach_ids)))
    return pd.DataFrame(vals, index=idx, columns=reach_ids)


def save(name, **arrays):
    path = os.path.join(OUT_DIR, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path)} bytes)")


# --------------------------------------------------------------------------------------------
def g1_y_network(mk):
    """G1: Y network 0,1 -> 2 -> 3 (outlet), 5 steps, incl. the init_states self-loop quirk."""
    endnodes = np.array([2, 2, 3, 3], dtype=np.int64)
    n = 4
    start = pd.Timestamp("2024-05-01T00:00:00Z")
    d = make_model_dict(mk, endnodes, np.full(n, 3600.0), np.full(n, 0.29), np.ones(n), start, 3600)
    m = mk.Muskingum(d)
    init_i = m.i_t_next.copy()
    rng = np.random.default_rng(11)
    df = forcing_frame(m.reach_ids, "2024-05-01T01:00:00", 5, "1h", rng)
    o, i, ts = run_simulate(m, df)
    save("g1_ynet.npz", endnodes=endnodes, K=d["K"], X=d["X"], o0=d["o_t"], dt=3600.0,
         start_ns=start.value, idx_ns=df.index.asi8, forcing=df.values, init_i=init_i,
         indegree=m.indegree, alpha=m.alpha, beta=m.beta, chi=m.chi, gamma=m.gamma,
         o=o, i=i, t_ns=ts)


def g2_huc8(mk):
    """G2: ~1k-reach tree, 24 h @ 300 s, hourly forcing (config 1). Sparse o/i + per-step hashes."""
    rng = np.random.default_rng(2024)
    n = 1000
    endnodes = random_forest(n, 3, rng, window=4, p_window=0.85)
    K = rng.uniform(1800.0, 7200.0, n)
    X = rng.uniform(0.1, 0.4, n)
    o0 = rng.uniform(0.5, 5.0, n)
    start = pd.Timestamp("2024-05-01T00:00:00Z")
    d = make_model_dict(mk, endnodes, K, X, o0, start, 300)
    m = mk.Muskingum(d)
    init_i = m.i_t_next.copy()
    df = forcing_frame(m.reach_ids, "2024-05-01T00:00:00", 25, "1h", rng)
    o, i, ts = run_simulate(m, df)
    assert o.shape[0] == 288, o.shape
    keep = np.r_[np.arange(0, 288, 12), 287]
    save("g2_huc8.npz", endnodes=endnodes, K=K, X=X, o0=o0, dt=300.0, start_ns=start.value,
         idx_ns=df.index.asi8, forcing=df.values, init_i=init_i, keep=keep,
         o_keep=o[keep], i_keep=i[keep], t_ns=ts,
         o_sha=np.frombuffer(b"".join(sha(r) for r in o), dtype=np.uint8).reshape(-1, 32),
         i_sha=np.frombuffer(b"".join(sha(r) for r in i), dtype=np.uint8).reshape(-1, 32),
         o_sum=o.sum(axis=1), i_sum=i.sum(axis=1))


def g3_confluence(mk):
    """G3: a tree with 3- and 4-way confluences (pins the summation order), 50 steps."""
    rng = np.random.default_rng(33)
    # hand-built core: nodes 0..9 feed a 4-way confluence at 10, 11..13 a 3-way at 14, both drain
    # to 15 -> 16 (outlet); then append a random tree below 16 for breadth.
    parent = {0: 10, 1: 10, 2: 10, 3: 10, 4: 0, 5: 0, 6: 0, 7: 1, 8: 2, 9: 2,
              11: 14, 12: 14, 13: 14, 10: 15, 14: 15, 15: 16, 16: 16}
    n_core = 17
    n = 160
    par = np.empty(n, dtype=np.int64)
    for k, v in parent.items():
        par[k] = v
    for k in range(n_core, n):
        par[k] = rng.integers(0, k) if rng.random() < 0.5 else rng.choice([10, 14, 15, 16, 0, 2])
    # relabel so that the graph is still a forest: nodes >= n_core drain into earlier nodes, fine.
    perm = rng.permutation(n)
    endnodes = np.empty(n, dtype=np.int64)
    endnodes[perm] = perm[par]
    K = rng.uniform(1800.0, 7200.0, n)
    X = rng.uniform(0.1, 0.4, n)
    o0 = rng.uniform(0.5, 5.0, n)
    start = pd.Timestamp("2024-05-01T00:00:00Z")
    d = make_model_dict(mk, endnodes, K, X, o0, start, 600)
    m = mk.Muskingum(d)
    fan = np.bincount(endnodes, minlength=n) - (endnodes == np.arange(n))
    assert fan.max() >= 4
    init_i = m.i_t_next.copy()
    df = forcing_frame(m.reach_ids, "2024-05-01T00:00:00", 10, "1h", rng)
    o, i, ts = run_simulate(m, df, every=1)
    o, i, ts = o[:50], i[:50], ts[:50]
    save("g3_confluence.npz", endnodes=endnodes, K=K, X=X, o0=o0, dt=600.0, start_ns=start.value,
         idx_ns=df.index.asi8, forcing=df.values, init_i=init_i, o=o, i=i, t_ns=ts,
         n_steps=len(ts))


def g4_split_async(mk, sim):
    """G4: split into sub-basins + AsyncSimulation vs whole network (300 reaches, 3 cuts)."""
    rng = np.random.default_rng(44)
    n = 300
    endnodes = random_forest(n, 1, rng, window=3, p_window=0.8)
    K = rng.uniform(1800.0, 7200.0, n)
    X = rng.uniform(0.1, 0.4, n)
    o0 = rng.uniform(0.5, 5.0, n)
    t0 = pd.Timestamp("2024-05-01T01:00:00Z")
    start = t0 - pd.Timedelta(3600, unit="s")
    d = make_model_dict(mk, endnodes, K, X, o0, start, 3600)
    whole = mk.Muskingum(d)
    df = forcing_frame(whole.reach_ids, t0, 18, "1h", rng)
    # cut at three non-outlet reaches that have upstream area
    indeg = whole.indegree
    cand = np.flatnonzero((indeg > 0) & (endnodes != np.arange(n)))
    cuts = np.sort(rng.choice(cand, size=3, replace=False))
    coll = whole.split(cuts, create_state_space=False)
    o_whole, i_whole, _ = run_simulate(whole.copy(), df)
    simulation = sim.AsyncSimulation(coll, df)
    outputs = asyncio.run(simulation.simulate())
    names = sorted(outputs.keys(), key=int)
    sub = {}
    for name in names:
        mdl = coll.models[name]
        sub[f"sub{name}_reach_ids"] = np.array([int(r[1:]) for r in mdl.reach_ids])
        sub[f"sub{name}_startnodes"] = mdl.startnodes
        sub[f"sub{name}_endnodes"] = mdl.endnodes
        sub[f"sub{name}_indegree"] = mdl.indegree
        sub[f"sub{name}_o"] = outputs[name].values
        sub[f"sub{name}_t_ns"] = outputs[name].index.asi8
        sub[f"sub{name}_sinks"] = np.array([[int(c.downstream_model.name), c.upstream_index,
                                             c.downstream_index] for c in mdl.sinks]).reshape(-1, 3)
        sub[f"sub{name}_init_i"] = mdl.i_t_next
        sub[f"sub{name}_inputs"] = simulation.inputs[name].values
    save("g4_split_async.npz", endnodes=endnodes, K=K, X=X, o0=o0, dt=3600.0,
         start_ns=start.value, idx_ns=df.index.asi8, forcing=df.values, cuts=cuts,
         names=np.array([int(x) for x in names]), o_whole=o_whole, i_whole=i_whole, **sub)


def g5_kalman(mk, da):
    """G5: KalmanFilter (da.py:91-136) on 200 reaches with 6 gages (unsorted), 24 steps."""
    rng = np.random.default_rng(55)
    n = 200
    endnodes = random_forest(n, 2, rng, window=3, p_window=0.7)
    K = rng.uniform(1800.0, 7200.0, n)
    X = rng.uniform(0.1, 0.4, n)
    o0 = rng.uniform(0.5, 5.0, n)
    start = pd.Timestamp("2024-05-01T00:00:00Z")
    d = make_model_dict(mk, endnodes, K, X, o0, start, 3600)
    model = mk.Muskingum(d)
    df = forcing_frame(model.reach_ids, "2024-05-01T00:00:00", 25, "1h", rng)
    indeg = model.indegree
    gages = rng.choice(np.flatnonzero(indeg > 0), size=6, replace=False)  # deliberately unsorted
    gage_ids = [model.reach_ids[g] for g in gages]
    meas_idx = pd.date_range("2024-05-01T00:00:00", periods=13, freq="1h", tz="UTC")
    meas = pd.DataFrame(rng.uniform(0.5, 8.0, size=(13, 6)), index=meas_idx, columns=gage_ids)
    Q = 2.0 * np.eye(n)
    R = 1e-2 * np.eye(6)
    kf = da.KalmanFilter(model, meas, Q, R, Q.copy())
    model.bind_callback(kf, key="kf")
    Ks, gains, dzs, pdiag, os_, is_, ts = [], [], [], [], [], [], []
    # record the analysis done in __on_simulation_start__ as well
    orig_filter = kf.filter

    def rec():
        orig_filter()
        Ks.append(kf.K.copy())
        gains.append(kf.gain.copy())
        dzs.append(kf.dz.copy())
        pdiag.append(np.diag(kf.P_t_next).copy())
    kf.filter = rec
    for state in model.simulate(df):
        os_.append(state.o_t_next.copy())
        is_.append(state.i_t_next.copy())
        ts.append(state.datetime.value)
    save("g5_kalman.npz", endnodes=endnodes, K=K, X=X, o0=o0, dt=3600.0, start_ns=start.value,
         idx_ns=df.index.asi8, forcing=df.values, gages=gages, meas_ns=meas.index.asi8,
         meas=meas.values, Kgain=np.array(Ks), gain=np.array(gains), dz=np.array(dzs),
         pdiag=np.array(pdiag), o=np.array(os_), i=np.array(is_), t_ns=np.array(ts),
         P_final=kf.P_t_next, reach_indices=kf.reach_indices)


def g6_dt_change(mk):
    """G6: step(q, timedelta=1800 s) recomputes coefficients; later default steps keep them."""
    rng = np.random.default_rng(66)
    n = 50
    endnodes = random_forest(n, 1, rng, window=3, p_window=0.5)
    K = rng.uniform(1800.0, 7200.0, n)
    X = rng.uniform(0.1, 0.4, n)
    o0 = rng.uniform(0.5, 5.0, n)
    start = pd.Timestamp("2024-05-01T00:00:00Z")
    m = mk.Muskingum(make_model_dict(mk, endnodes, K, X, o0, start, 3600))
    qs = rng.gamma(2.0, 0.5, size=(4, n))
    tds = [None, 1800, None, 3600]
    os_, is_, ts, coef = [], [], [], []
    for q, td in zip(qs, tds):
        if td is None:
            m.step(q)
        else:
            m.step(q, timedelta=pd.Timedelta(td, unit="s"))
        os_.append(m.o_t_next.copy())
        is_.append(m.i_t_next.copy())
        ts.append(m.datetime.value)
        coef.append(np.stack([m.alpha, m.beta, m.chi, m.gamma]))
    save("g6_dt_change.npz", endnodes=endnodes, K=K, X=X, o0=o0, dt=3600.0, start_ns=start.value,
         q=qs, td=np.array([-1 if t is None else t for t in tds]), o=np.array(os_),
         i=np.array(is_), t_ns=np.array(ts), coef=np.array(coef))


def g7_covariance(mk, nu):
    """G7: _ap_par / _aqat_par / _apply_gain / _ax on 50 reaches."""
    rng = np.random.default_rng(77)
    n = 50
    endnodes = random_forest(n, 2, rng, window=3, p_window=0.6)
    K = rng.uniform(1800.0, 7200.0, n)
    X = rng.uniform(0.1, 0.4, n)
    m = mk.Muskingum(make_model_dict(mk, endnodes, K, X, np.ones(n),
                                     pd.Timestamp("2024-05-01T00:00:00Z"), 900))
    heads = m.startnodes[m.indegree == 0]
    A = rng.normal(size=(n, n))
    P = A @ A.T / n
    aqat = nu._aqat_par(P.copy(), np.empty((n, n)), heads, m.endnodes, m.alpha, m.beta, m.chi,
                        m.indegree)
    ap = nu._ap_par(P.copy(), np.empty((n, n)), heads, m.endnodes, m.alpha, m.beta, m.chi,
                    m.indegree)
    gain = rng.normal(size=n)
    ig, og = nu._apply_gain(heads, m.endnodes, gain, m.indegree)
    ip = rng.normal(size=n)
    op = rng.normal(size=n)
    ax_i, ax_o = nu._ax(heads, m.endnodes, m.alpha, m.beta, m.chi, ip, op, m.indegree)
    save("g7_covariance.npz", endnodes=endnodes, K=K, X=X, dt=900.0, alpha=m.alpha, beta=m.beta,
         chi=m.chi, gamma=m.gamma, indegree=m.indegree, P=P, aqat=aqat, ap=ap, gain=gain,
         gain_i=ig, gain_o=og, ip=ip, op=op, ax_i=ax_i, ax_o=ax_o)


def g8_ax_bu_edge(nu):
    """G8: raw _ax_bu on edge-case topologies (cycles, self loops, 3+-way, unprocessed reaches,
    negative coefficients, caller-supplied headwater lists)."""
    rng = np.random.default_rng(88)
    cases = {}
    # (a) random forests of several shapes, coefficients incl. negative alpha
    for c, (n, outs, win, pw) in enumerate([(1, 1, None, 0), (2, 1, None, 0), (7, 2, 2, 0.5),
                                             (64, 4, 3, 0.7), (500, 5, 5, 0.9), (333, 40, None, 0)]):
        endnodes = random_forest(n, outs, rng, window=win, p_window=pw)
        indeg = np.bincount(endnodes, minlength=n) - (endnodes == np.arange(n))
        heads = np.flatnonzero(indeg == 0).astype(np.int64)
        args = [rng.normal(size=n) for _ in range(7)]
        i_n, o_n = nu._ax_bu(heads, endnodes, *args[:4], args[4], args[5], args[6], indeg)
        cases[f"c{c}"] = (endnodes, heads, indeg, args, i_n, o_n)
    # (b) a 3-cycle fed by a tree plus a node downstream of the cycle (never processed)
    endnodes = np.array([1, 2, 3, 1, 3, 4, 7, 7, 6], dtype=np.int64)  # 1->2->3->1 cycle; 4->3; 5->4
    # node 5 drains to 4, 4 drains to 3 (in cycle); 6,8 -> 7 -> 7 outlet... fix 6/8:
    endnodes = np.array([1, 2, 3, 1, 3, 4, 7, 7, 7], dtype=np.int64)
    n = endnodes.size
    indeg = np.bincount(endnodes, minlength=n) - (endnodes == np.arange(n))
    heads = np.flatnonzero(indeg == 0).astype(np.int64)
    args = [rng.normal(size=n) for _ in range(7)]
    i_n, o_n = nu._ax_bu(heads, endnodes, *args[:4], args[4], args[5], args[6], indeg)
    cases["cycle"] = (endnodes, heads, indeg, args, i_n, o_n)
    # (c) indegree larger than the true count (reach never processed, its subtree's output piles up)
    endnodes = random_forest(40, 2, rng, window=2, p_window=0.5)
    indeg = np.bincount(endnodes, minlength=40) - (endnodes == np.arange(40))
    bump = int(np.flatnonzero(indeg > 0)[0])
    indeg2 = indeg.copy()
    indeg2[bump] += 1
    heads = np.flatnonzero(indeg2 == 0).astype(np.int64)
    args = [rng.normal(size=40) for _ in range(7)]
    i_n, o_n = nu._ax_bu(heads, endnodes, *args[:4], args[4], args[5], args[6], indeg2)
    cases["bigindeg"] = (endnodes, heads, indeg2, args, i_n, o_n)
    # (d) headwater list given in descending order (changes finalisation order of confluences)
    endnodes = random_forest(120, 1, rng)
    indeg = np.bincount(endnodes, minlength=120) - (endnodes == np.arange(120))
    heads = np.flatnonzero(indeg == 0)[::-1].astype(np.int64).copy()
    args = [rng.normal(size=120) for _ in range(7)]
    i_n, o_n = nu._ax_bu(heads, endnodes, *args[:4], args[4], args[5], args[6], indeg)
    cases["revheads"] = (endnodes, heads, indeg, args, i_n, o_n)
    flat = {}
    for k, (e, h, d, a, i_n, o_n) in cases.items():
        flat[f"{k}_endnodes"] = e
        flat[f"{k}_heads"] = h
        flat[f"{k}_indegree"] = d
        flat[f"{k}_args"] = np.stack(a)
        flat[f"{k}_i"] = i_n
        flat[f"{k}_o"] = o_n
    save("g8_ax_bu_edge.npz", names=np.array(list(cases.keys())), **flat)


def g9_interp(nu):
    """G9: interpolate_sample (nutils.py:5-39) at knots, between knots, and clamped ends."""
    rng = np.random.default_rng(99)
    idx = pd.date_range("2024-05-01T00:00:00", periods=25, freq="1h", tz="UTC")
    xp = idx.astype(int).astype(float).values
    fp = rng.gamma(2.0, 0.5, size=(25, 17))
    xs_ts = [idx[0] - pd.Timedelta(300, unit="s"), idx[0], idx[0] + pd.Timedelta(300, unit="s"),
             idx[3] + pd.Timedelta(1, unit="ns"), idx[7] + pd.Timedelta(1799, unit="s"),
             idx[12], idx[24], idx[24] + pd.Timedelta(5, unit="s"),
             idx[5] + pd.Timedelta(2100, unit="s")]
    xs = np.array([float(t.value) for t in xs_ts])
    lin = np.array([nu.interpolate_sample(x, xp, fp, method=1) for x in xs])
    near = np.array([nu.interpolate_sample(x, xp, fp, method=0) for x in xs])
    save("g9_interp.npz", xp=xp, fp=fp, xs=xs, lin=lin, near=near)


def g10_model_io(mk, tio):
    """G10: model JSON (ModelEncoder, muskingum.py:867-876) + indegree/coeff/init quirks."""
    rng = np.random.default_rng(1010)
    n = 30
    endnodes = random_forest(n, 2, rng, window=3, p_window=0.5)
    K = rng.uniform(1800.0, 7200.0, n)
    X = rng.uniform(0.1, 0.4, n)
    o0 = rng.uniform(0.5, 5.0, n)
    d = make_model_dict(mk, endnodes, K, X, o0, pd.Timestamp("2024-05-01T00:00:00Z"), 300)
    m = mk.Muskingum(d)
    text = json.dumps(m.info, cls=tio.ModelEncoder)
    coeffs = {}
    for dt in (60.0, 300.0, 900.0, 3600.0, 86400.0):
        coeffs[f"dt{int(dt)}"] = np.stack([m.compute_alpha(K, X, dt), m.compute_beta(K, X, dt),
                                           m.compute_chi(K, X, dt), m.compute_gamma(K, X, dt)])
    save("g10_model_io.npz", endnodes=endnodes, K=K, X=X, o0=o0, json=np.array(text),
         indegree=m.indegree, init_i=m.i_t_next, **coeffs)


def g11_smoother(mk, da):
    """G11: KalmanSmoother (da.py:139-264) on 60 reaches, 4 gages, 8 hourly steps: filter
    estimates, priors and the RTS-smoothed series."""
    rng = np.random.default_rng(1111)
    n = 60
    endnodes = random_forest(n, 2, rng, window=3, p_window=0.7)
    K = rng.uniform(1800.0, 7200.0, n)
    X = rng.uniform(0.1, 0.4, n)
    o0 = rng.uniform(0.5, 5.0, n)
    start = pd.Timestamp("2024-05-01T00:00:00Z")
    model = mk.Muskingum(make_model_dict(mk, endnodes, K, X, o0, start, 3600))
    df = forcing_frame(model.reach_ids, "2024-05-01T00:00:00", 9, "1h", rng)
    gages = np.sort(rng.choice(np.flatnonzero(model.indegree > 0), size=4, replace=False))
    meas_idx = pd.date_range("2024-05-01T00:00:00", periods=9, freq="1h", tz="UTC")
    meas = pd.DataFrame(rng.uniform(0.5, 8.0, size=(9, 4)), index=meas_idx,
                        columns=[model.reach_ids[g] for g in gages])
    Q = 2.0 * np.eye(n)
    R = 1e-2 * np.eye(4)
    ks = da.KalmanSmoother(model, meas, Q, R, Q.copy())
    model.bind_callback(ks, key="ks")
    os_, is_ = [], []
    for state in model.simulate(df):
        os_.append(state.o_t_next.copy())
        is_.append(state.i_t_next.copy())
    times = sorted(ks.P_s.keys())
    save("g11_smoother.npz", endnodes=endnodes, K=K, X=X, o0=o0, dt=3600.0,
         start_ns=start.value, idx_ns=df.index.asi8, forcing=df.values, gages=gages,
         meas_ns=meas.index.asi8, meas=meas.values, o=np.array(os_), i=np.array(is_),
         s_ns=np.array([t.value for t in times], dtype=np.int64),
         o_s=ks.o_hat_s.values, i_s=ks.i_hat_s.values,
         os_ns=ks.o_hat_s.index.asi8 if hasattr(ks.o_hat_s.index, "asi8") else
         np.array([pd.Timestamp(t).value for t in ks.o_hat_s.index]),
         P_s=np.array([ks.P_s[t] for t in times]),
         P_f_final=ks.P_f[times[-1]], n_times=np.array(len(ks.datetimes)))


def main():
    warnings.simplefilter("ignore")
    tmp, mk, nu, sim, da, tio = _import_reference()
    only = set(sys.argv[1:])
    if only:
        try:
            for name in sorted(only):
                {"g11": lambda: g11_smoother(mk, da)}[name]()
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
        return
    try:
        g1_y_network(mk)
        g2_huc8(mk)
        g3_confluence(mk)
        g4_split_async(mk, sim)
        g5_kalman(mk, da)
        g6_dt_change(mk)
        g7_covariance(mk, nu)
        g8_ax_bu_edge(nu)
        g9_interp(nu)
        g10_model_io(mk, tio)
        g11_smoother(mk, da)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
