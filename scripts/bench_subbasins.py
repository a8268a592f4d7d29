#!/usr/bin/env python3
"""Sub-basin DAG timing: the full-Texas synthetic network split into >= 50
sub-basins (Muskingum.split at reaches with 1k-20k upstream reaches), routed for 24 h at 300 s
by AsyncSimulation (reference simulation.py:94-166)
  * on the device DAG (no callbacks: every sub-basin launched on its own session stream, the
    cut-edge corrections added on the device, outflows fetched after the last launch), and
  * by the host driver (an idle callback bound to every sub-basin: one fused horizon per
    sub-basin, its series fetched to pandas, corrections on the host between sub-basins),
checking that both give bit-identical outflow frames, corrected inputs and final states.
Prints one JSON line.   python scripts/bench_subbasins.py [--cuts 60] [--runs 2]
"""
import argparse
import asyncio
import json
import os
import sys
import time

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tx-fast-hydrology_amd"))
sys.path.insert(0, ROOT)

from tx_fast_hydrology_amd import synthetic  # noqa: E402
from tx_fast_hydrology_amd.callbacks import BaseCallback  # noqa: E402
from tx_fast_hydrology_amd.muskingum import Muskingum  # noqa: E402
from tx_fast_hydrology_amd.simulation import AsyncSimulation  # noqa: E402


class Idle(BaseCallback):
    def __idle_steps__(self):
        return True


def upstream_area(end):
    n = end.size
    start = np.arange(n)
    deg = np.bincount(end, minlength=n) - (end == start)
    area = np.ones(n, dtype=np.int64)
    left = deg.copy()
    stack = list(np.flatnonzero(deg == 0))
    while stack:
        j = stack.pop()
        d = end[j]
        if d != j:
            area[d] += area[j]
            left[d] -= 1
            if left[d] == 0:
                stack.append(d)
    return area


def build(cuts_wanted, T, seed=0):
    end = synthetic.river_network(190_000, 300, 1500, np.random.default_rng(0))
    n = end.size
    K, X, o0 = synthetic.model_arrays(n, seed=0)
    start = pd.Timestamp("2024-05-01T00:00:00Z")
    data = {"name": "texas", "datetime": start, "timedelta": pd.to_timedelta(300, unit="s"),
            "reach_ids": [f"r{j}" for j in range(n)], "startnodes": np.arange(n, dtype=np.int64),
            "endnodes": end.astype(np.int64), "K": K, "X": X, "o_t": o0,
            "dx": np.ones(n), "paths": [[] for _ in range(n)]}
    rng = np.random.default_rng(seed)
    idx = pd.date_range(start + pd.Timedelta(300, unit="s"), periods=T, freq="300s", tz="UTC")
    df = pd.DataFrame(rng.gamma(2.0, 0.5, (T, n)), index=idx, columns=data["reach_ids"])
    area = upstream_area(end)
    cand = np.flatnonzero((area >= 1000) & (area <= 20000) & (end != np.arange(n)))
    cuts = np.sort(rng.choice(cand, size=min(cuts_wanted, cand.size), replace=False))
    return data, df, cuts


def collection(data, cuts, device):
    coll = Muskingum(dict(data)).split(cuts, create_state_space=False)
    if not device:
        for m in coll.models.values():
            m.bind_callback(Idle(), key="idle")
    return coll


def run(coll, df):
    """One 24-h AsyncSimulation of the collection from its split-time state (the sessions of
    earlier runs are reused: routing time, not session construction)."""
    for m in coll.models.values():
        m.load_state()
    sim = AsyncSimulation(coll, df)
    t0 = time.perf_counter()
    outputs = asyncio.run(sim.simulate())
    return time.perf_counter() - t0, outputs, sim


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cuts", type=int, default=60)
    ap.add_argument("--T", type=int, default=288)
    ap.add_argument("--runs", type=int, default=2)
    a = ap.parse_args()
    data, df, cuts = build(a.cuts, a.T)
    times = {}
    res = {}
    phases = None
    for device in (True, False):
        coll = collection(data, cuts, device)
        ts = []
        for r in range(a.runs + 1):       # the first run builds the device sessions
            dt, outputs, sim = run(coll, df)
            if r:
                ts.append(dt)
                if device and (phases is None or dt <= min(ts)):
                    phases = {k: round(v, 2) for k, v in getattr(sim, "dag_phases", {}).items()}
        times[device] = min(ts)
        res[device] = (outputs, sim, coll)
    (o_d, s_d, c_d), (o_h, s_h, c_h) = res[True], res[False]
    same = o_d.keys() == o_h.keys()
    for k in o_h:
        same = same and np.array_equal(o_d[k].values, o_h[k].values)
        same = same and np.array_equal(s_d.inputs[k].values, s_h.inputs[k].values)
        same = same and np.array_equal(c_d.models[k].o_t_next, c_h.models[k].o_t_next)
        same = same and np.array_equal(c_d.models[k].i_t_next, c_h.models[k].i_t_next)
    sizes = sorted(m.n for m in c_d.models.values())
    print(json.dumps({
        "workload": f"full-Texas synthetic network split into {len(sizes)} sub-basins "
                    f"({len(cuts)} cuts), 24 h @ 300 s ({a.T} steps), AsyncSimulation",
        "sub_basins": len(sizes), "largest": sizes[-1], "median": sizes[len(sizes) // 2],
        "device_dag_s": round(times[True], 4), "host_driver_s": round(times[False], 4),
        "speedup": round(times[False] / times[True], 2), "bit_identical": bool(same),
        "device_dag_phases_ms": phases}),
        flush=True)
    if not same:
        sys.exit(1)


if __name__ == "__main__":
    main()
