#!/usr/bin/env python3
"""Full-covariance Kalman filter on a HUC-8-size sub-basin: the da.py workload
through the reference API (Muskingum + KalmanFilter bound as a callback), on the device.

Workload: synthetic 1,000-reach sub-basin (BASELINE configs[0] size), 24 h at dt = 300 s, hourly
forcing; 20 gauges observed hourly for the first 2 h, so the filter runs at the simulation start
and after each of the first 24 steps (da.py:49-61); Q = 2 I, R = 1e-2 I, P0 = Q (app.py:137-139).

Prints one JSON line: ms per 24-h horizon (routing + 25 analyses, host state round trips
included), ms per analysis (prior A P A^T + Q, gain, posterior, gain application), the
covariance-sweep kernel time per analysis from HIP events, and the CPU baseline: the oracle's
restatement of KalmanFilter.filter (C _ax sweeps + NumPy inv / GEMM, oracle.kalman_analysis) on
a bounded sample of the same analyses.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tx-fast-hydrology_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--gauges", type=int, default=20)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    import pandas as pd
    import torch

    from api_helpers import model_dict
    from oracle import oracle as orc
    from tx_fast_hydrology_amd import synthetic
    from tx_fast_hydrology_amd.da import KalmanFilter
    from tx_fast_hydrology_amd.muskingum import Muskingum

    rng = np.random.default_rng(0)
    end = synthetic.river_network(args.n, 5, 120, rng)
    n = end.size
    K, X, o0 = synthetic.model_arrays(n, seed=0)
    t0 = pd.Timestamp("2024-05-01T00:00:00Z")
    base = Muskingum(model_dict(end, K, X, o0, t0, 300))
    idx = pd.date_range(t0, periods=25, freq="1h", tz="UTC")
    df = pd.DataFrame(np.random.default_rng(1).gamma(2.0, 0.5, (25, n)), index=idx,
                      columns=base.reach_ids)
    gauges = np.sort(np.random.default_rng(7).choice(np.flatnonzero(base.indegree > 0),
                                                     args.gauges, replace=False))
    meas = pd.DataFrame(np.random.default_rng(8).uniform(0.5, 8.0, (3, gauges.size)),
                        index=idx[:3], columns=[base.reach_ids[g] for g in gauges])
    Q = 2.0 * np.eye(n)
    R = 1e-2 * np.eye(gauges.size)

    def horizon():
        m = base.copy()
        kf = KalmanFilter(m, meas, Q, R, Q.copy())
        m.bind_callback(kf, key="kf")
        calls = [0]
        orig = kf.filter

        def counted():
            calls[0] += 1
            orig()
        kf.filter = counted
        for _ in m.simulate(df):
            pass
        torch.cuda.synchronize()
        return calls[0], kf

    horizon()                                            # warmup (graph compile, allocations)
    t = time.perf_counter()
    for _ in range(args.steps):
        n_an, kf = horizon()
    ms_horizon = (time.perf_counter() - t) / args.steps * 1e3

    # one analysis in isolation: device time of its parts
    m = base.copy()
    kf = KalmanFilter(m, meas, Q, R, Q.copy())
    graph = kf._graph()
    P = kf.P_t_next_device
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    reps = 20
    sweep_ms = upd_ms = 0.0
    for _ in range(reps):
        ev[0].record()
        prior = graph.aqat(P, kf._Q)
        ev[1].record()
        graph.kf_update(kf.reach_indices, kf.R_cov, np.ones(gauges.size), prior, graph.empty(),
                        want_K=False)
        ev[2].record()
        torch.cuda.synchronize()
        sweep_ms += ev[0].elapsed_time(ev[1]) / reps
        upd_ms += ev[1].elapsed_time(ev[2]) / reps
    t = time.perf_counter()
    for _ in range(reps):
        kf.filter()
    torch.cuda.synchronize()
    ms_filter = (time.perf_counter() - t) / reps * 1e3
    # algorithmic bytes of the prior: 2 sweeps (read x, read the inflow list of x, write o:
    # (2 + in-list) x 8 B per element) + transpose (16 B) + Q add (24 B) per element
    inl = np.bincount(end, minlength=n).mean()
    prior_bytes = n * n * (2 * (2 + inl) * 8 + 16 + 24)

    cpu = None
    if not args.no_cpu:
        heads = np.arange(n)[base.indegree == 0]
        Pc = Q.copy()
        o, i = base.o_t_next.copy(), base.i_t_next.copy()
        s = gauges
        reps_c, t_c = 0, 0.0
        while t_c < args.cpu_seconds or reps_c == 0:
            c0 = time.perf_counter()
            r = orc.kalman_analysis(Pc, o, i, s, np.ones(s.size) + o[s], Q, R, np.arange(n), end,
                                    base.indegree, base.alpha, base.beta, base.chi)
            t_c += time.perf_counter() - c0
            reps_c += 1
            Pc = r["P"]
        per = t_c / reps_c
        cpu = {"value": per * 1e3, "unit": "ms per analysis", "cores": 1, "kind": "port",
               "sample": f"{reps_c} x KalmanFilter.filter on the same {n}-reach network "
                         f"(oracle: C _ax sweeps + NumPy inv/GEMM), {t_c:.1f} s"}

    line = {
        "workload": f"huc8-kf: {n}-reach sub-basin, full-covariance KalmanFilter "
                    f"({gauges.size} gauges, {n_an} analyses per 24 h horizon @ 300 s), "
                    "reference API (Muskingum + KalmanFilter callback)",
        "ms_per_horizon": round(ms_horizon, 3),
        "analyses_per_horizon": n_an,
        "ms_per_analysis": round(ms_filter, 4),
        "prior_device_ms": round(sweep_ms, 4),
        "update_device_ms": round(upd_ms, 4),
        "prior_algorithmic_GBs": round(prior_bytes / (sweep_ms * 1e-3) / 1e9, 2),
        "levels": int(graph_levels(end, base.indegree)),
        "cpu_baseline": cpu,
        "speedup_per_analysis": (cpu["value"] / ms_filter) if cpu else None,
    }
    print(json.dumps(line), flush=True)


def graph_levels(end, indeg):
    n = end.size
    left = indeg.copy()
    lvl = np.zeros(n, dtype=np.int64)
    stack = list(np.flatnonzero(indeg == 0))
    while stack:
        j = stack.pop()
        d = end[j]
        if d == j:
            continue
        lvl[d] = max(lvl[d], lvl[j] + 1)
        left[d] -= 1
        if left[d] == 0:
            stack.append(d)
    return lvl.max() + 1


if __name__ == "__main__":
    main()
