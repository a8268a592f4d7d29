#!/usr/bin/env python3
"""Diagnostic: one-step member runs on the member paths vs the member-dataflow launch (device
time of the step's kernels, HIP events), on a straight chain (one task: the per-node latency) and
on the bench's Texas network.  python scripts/diag_paths.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tx-fast-hydrology_amd")]
from oracle import oracle as orc  # noqa: E402
from tx_fast_hydrology_amd import engine, synthetic  # noqa: E402


def run(end, E, mode, reps=20, slots=192, tile=16):
    n = end.size
    start = np.arange(n)
    indeg = orc.compute_indegree(start, end)
    K, X, o0 = synthetic.model_arrays(n, seed=1)
    coef = orc.muskingum_coeffs(K, X, 300.0)
    net = engine.RoutingNet(end, indeg, start[indeg == 0], slots=slots, tile=tile, members=E)
    net.set_mode(mode)
    net.set_coeffs(*coef)
    o = np.repeat(o0[:, None], E, axis=1)
    net.set_state(o, np.zeros((n, E)))
    xp = (1.7e18 + 3600e9 * np.arange(3)).astype(float)
    net.load_forcing(xp, np.full((3, n, E), 0.5))
    net.run(xp[:1] + 300e9)
    net.synchronize()
    net.reset_timing()
    net.set_timing(True)
    t0 = time.perf_counter()
    for k in range(reps):
        net.run(xp[:1] + 300e9 * (k + 2))
    net.synchronize()
    wall = (time.perf_counter() - t0) / reps * 1e3
    tm = net.timing()
    path = net.mode()[1]
    net.close()
    return path, tm["kernel_ms"] / max(tm["launches"], 1), wall


if __name__ == "__main__":
    chain = np.minimum(np.arange(4000) + 1, 3999).astype(np.int64)
    texas = synthetic.river_network(190_000, 300, 1500, np.random.default_rng(0))
    for name, end in (("chain4000", chain), ("texas", texas)):
        for E in (32, 64, 256):
            for mode in ("paths", "dataflow"):
                path, kms, wall = run(end, E, mode)
                print(f"{name} E={E} {path}: step kernel {kms:.3f} ms, wall {wall:.3f} ms",
                      flush=True)
