#!/usr/bin/env python3
"""Diagnostic: where the multi-launch path departs from the oracle on a random forest (which
reaches, which steps, what kind of slot feeds them).  python scripts/diag_launches.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tx-fast-hydrology_amd"), os.path.join(ROOT, "tests")]
from oracle import oracle as orc  # noqa: E402
from tx_fast_hydrology_amd import engine, synthetic  # noqa: E402


def case(n, T, p_chain, slots, tile, mode):
    rng = np.random.default_rng(n + T)
    end = synthetic.random_forest(n, max(1, n // 500), rng, p_chain=p_chain)
    K = rng.uniform(1800.0, 7200.0, n)
    X = rng.uniform(0.1, 0.4, n)
    start = np.arange(n)
    indeg = orc.compute_indegree(start, end)
    coef = orc.muskingum_coeffs(K, X, 300.0)
    o0 = np.random.default_rng(n).uniform(0.5, 5, n)
    i0 = orc.init_inflows(start, end, o0)
    xp, fp = synthetic.forcing(n, rows=5, seed=n)
    xp = xp.astype(float)
    x = xp[0] - 600e9 + 300e9 * np.arange(1, T + 1)
    want_o, want_i, _, _ = orc.simulate(start, end, indeg, *coef, o0, i0, x, xp, fp)
    heads = start[indeg == 0]
    net = engine.RoutingNet(end, indeg, heads, slots=slots, tile=tile)
    net.set_mode(mode)
    net.set_coeffs(*coef)
    net.set_state(o0, i0)
    got_o, got_i = net.simulate(x, xp, fp)
    bad_o = got_o != want_o
    bad_i = got_i != want_i
    info = net.info
    print(f"n={n} T={T} p={p_chain} slots={slots} tile={tile} mode={mode} path={net.mode()[1]} "
          f"bad_o={bad_o.sum()} bad_i={bad_i.sum()} n_partial={info['n_partial']} "
          f"gmax={info['gmax']}", flush=True)
    if bad_o.any() or bad_i.any():
        plan = engine.Plan(end, indeg, heads, slots=slots, tile=tile)
        ex = plan.export()
        ln = plan.export_links()
        pos, G = ex["pos"], ex["G"]
        indeg_all = np.bincount(end, minlength=n) - (end == start)
        for name, bad in (("o", bad_o), ("i", bad_i)):
            ts, js = np.nonzero(bad)
            if not ts.size:
                continue
            t0 = ts.min()
            first = sorted(set(js[ts == t0].tolist()))[:10]
            print(f"  {name}: first bad step {t0}, reaches {first}")
            for j in first[:5]:
                d = pos[j]
                w = d // (2 * slots)
                print(f"    reach {j}: slot {d} wg {w} G {G[d]} flag {ln['flags'][d]} "
                      f"up_cnt {ln['up_cnt'][d]} indeg {indeg_all[j]} got {got_o[t0, j] if name == 'o' else got_i[t0, j]!r} "
                      f"want {want_o[t0, j] if name == 'o' else want_i[t0, j]!r} "
                      f"k0 of step: {(G[d] + t0) % tile}")
    net.close()


if __name__ == "__main__":
    for args in [(5000, 40, 0.5, 512, 16, "launches"), (5000, 40, 0.5, 512, 48, "launches"),
                 (5000, 40, 0.5, 256, 16, "launches"), (5000, 40, 0.5, 192, 16, "auto"),
                 (5000, 40, 0.5, 192, 16, "launches"), (3000, 96, 0.95, 256, 32, "launches")]:
        case(*args)
