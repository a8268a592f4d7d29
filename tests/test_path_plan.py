"""The member-path plan (paths.hpp, the one-step ensemble sweep of paths.hip) replayed on the CPU:
tasks in ticket order, each node folding its inputs exactly as the kernel does -- the chain
register, the previous node, the LDS ring of the task's earlier outputs, another task's bottom --
must reproduce the oracle's _ax_bu step (nutils.py:64-89) bit for bit, every ticket may only wait
for earlier tickets, and every ring read must find its value still in the ring."""
import numpy as np
import pytest

from oracle import oracle as orc
from tx_fast_hydrology_amd import engine, synthetic

KIND = {0: "chain", 1: "prev", 2: "local", 3: "ext"}
RING = 32
INLINE = 8


def replay(end, indeg, coef, o0, i0, q, **kw):
    """One step of every member column through the path plan; returns (i, o) like ax_bu."""
    n = end.size
    start = np.arange(n)
    plan = engine.Plan(end, indeg, start[indeg == 0], **kw)
    pp = plan.paths()
    alpha, beta, chi, gamma = coef
    task_off, seq, rec, ovf = pp["task_off"], pp["seq_reach"], pp["rec"], pp["ovf"].view(np.uint32)
    assert sorted(seq.tolist()) == list(range(n))            # every reach once
    E = o0.shape[1]
    o_new = np.full((n, E), np.nan)
    i_new = np.full((n, E), np.nan)
    bottom = {}                                              # task -> published output
    n_tasks = task_off.size - 1
    for t in range(n_tasks):
        ring = {}
        chainv = prevv = None
        for s in range(task_off[t], task_off[t + 1]):
            j = seq[s]
            r = rec[s].view(np.uint32)
            meta = int(r[0])
            n_in = meta & 0xffff
            codes = [int(r[4 + k]) if k < INLINE else int(ovf[int(r[12]) + k - INLINE])
                     for k in range(n_in)]
            I = np.zeros(E)
            for k, c in enumerate(codes):
                kind, pay = KIND[c >> 30], c & ((1 << 30) - 1)
                if kind == "chain":
                    v = chainv
                elif kind == "prev":
                    v = prevv
                elif kind == "local":
                    assert s - pay < RING and ring.get(pay % RING, (None,))[0] == pay, (t, s, pay)
                    v = ring[pay % RING][1]
                else:
                    assert pay < t, "a ticket waits for a later ticket"
                    v = bottom[pay]
                assert v is not None
                I = v.copy() if k == 0 else I + v
            o = 0.0 + (((alpha[j] * I + beta[j] * i0[j]) + chi[j] * o0[j]) + gamma[j] * q[j])
            if not meta & (1 << 16):                             # never processed: o stays 0
                o = np.zeros(E)
            o_new[j], i_new[j] = o, I
            prevv = o
            if meta & (1 << 17):
                chainv = o
            if meta & (1 << 19):
                ring[s % RING] = (s, o)
            if meta & (1 << 18):
                assert s == task_off[t + 1] - 1
                bottom[t] = o
    return i_new, o_new, pp


def _members(n, E, seed):
    rng = np.random.default_rng(seed)
    o0 = rng.uniform(0.5, 5.0, (n, E))
    i0 = rng.uniform(0.0, 5.0, (n, E))
    q = rng.uniform(0.0, 2.0, (n, E))
    return o0, i0, q


def _check(end, coef=None, E=3, seed=0, **kw):
    n = end.size
    start = np.arange(n)
    indeg = orc.compute_indegree(start, end)
    if coef is None:
        K, X, _ = synthetic.model_arrays(n, seed=seed)
        coef = orc.muskingum_coeffs(K, X, 300.0)
    o0, i0, q = _members(n, E, seed)
    got_i, got_o, pp = replay(end, indeg, coef, o0, i0, q, **kw)
    heads = start[indeg == 0]
    for e in range(E):
        wi, wo = orc.ax_bu(heads, end, *coef, np.ascontiguousarray(i0[:, e]),
                           np.ascontiguousarray(o0[:, e]), np.ascontiguousarray(q[:, e]), indeg)
        assert np.array_equal(got_o[:, e], wo), e
        assert np.array_equal(got_i[:, e], wi), e
    return pp


def test_golden_networks(golden):
    for name in ("g1_ynet.npz", "g3_confluence.npz"):
        g = golden(name)
        end = g["endnodes"]
        coef = orc.muskingum_coeffs(g["K"], g["X"], float(g["dt"]))
        _check(np.asarray(end, np.int64), coef=coef)


@pytest.mark.parametrize("n,p_chain,seed", [(1, 0.0, 1), (2, 1.0, 2), (300, 0.9, 3),
                                            (3000, 0.5, 4), (5000, 0.98, 5)])
def test_random_forests(n, p_chain, seed):
    rng = np.random.default_rng(seed)
    end = synthetic.random_forest(n, max(1, n // 500), rng, p_chain=p_chain)
    _check(end, seed=seed)


def test_high_fan_in_uses_overflow_inputs():
    # reaches with up to 30 upstreams: inputs beyond the record's inline codes
    n, fan = 2000, 25
    end = np.arange(n, dtype=np.int64)
    for j in range(n):
        hub = (j // fan) * fan
        end[j] = hub if j != hub else min(hub + fan, (n - 1) // fan * fan)
    pp = _check(end, seed=11)
    assert pp["ovf"].size > 0


def test_unrouted_reaches_and_cycles():
    # 0 -> 1 <-> 2 (never processed), 6 -> 1, 3, 4 -> 5, 7 -> 3, 8..13 -> 5
    end = np.array([1, 2, 1, 5, 5, 5, 1, 3] + [5] * 6, dtype=np.int64)
    _check(end, E=2)


def test_texas_scale_plan():
    """The bench's Texas network: the plan covers every reach, ring reads stay in the ring, and
    its critical path is a few percent of the reaches."""
    end = synthetic.river_network(190_000, 300, 1500, np.random.default_rng(0))
    pp = _check(end, E=1, seed=0)
    assert pp["task_off"].size - 1 < end.size // 4
