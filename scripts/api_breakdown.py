#!/usr/bin/env python3
"""Where the drop-in API horizon goes (Muskingum.simulate over Texas, T = 288), phase by phase
as Muskingum._simulate_fused runs them: forcing frame -> contiguous array, forcing upload,
state upload, device run, block fetches into pinned host rows (with the device's row digests),
the host digest check of every yielded step, and the whole generator.  Prints one JSON line.
    python scripts/api_breakdown.py
"""
import json
import os
import sys
import time

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tx-fast-hydrology_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from tx_fast_hydrology_amd import engine, muskingum  # noqa: E402


def best(fn, runs=3):
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return 1e3 * min(ts)


def main():
    args = bench.parse([], world=1)
    net, wl = bench.build_workload(args)
    n, x = wl.n, wl.x
    T = x.size
    reach_ids = [f"r{j}" for j in range(n)]
    idx = pd.DatetimeIndex(pd.to_datetime(wl.xp_ns, utc=True))
    df = pd.DataFrame(wl.fp, index=idx, columns=reach_ids)
    block = max(1, muskingum._FETCH_BLOCK_VALUES // n)
    res = {"steps": T, "n": n, "block_steps": block, "bytes_fetched": 2 * 8 * n * T}
    res["frame_to_array_ms"] = best(lambda: np.ascontiguousarray(df.values, dtype=np.float64))
    fp = np.ascontiguousarray(df.values, dtype=np.float64)
    res["load_forcing_ms"] = best(lambda: net.load_forcing(wl.xp, fp))
    res["set_state_ms"] = best(lambda: net.set_state(wl.o0, wl.i0))

    def run_only():
        net.run(x)
        net.synchronize()
    res["run_ms"] = best(run_only)
    blocks = []

    def run_fetch():
        blocks.clear()
        net.run(x)
        dig = muskingum._host_array((2, T), np.uint64)
        tks = []
        for b0 in range(0, T, block):
            b1 = min(T, b0 + block)
            oo = muskingum._host_array((b1 - b0, n), np.float64)
            ii = muskingum._host_array((b1 - b0, n), np.float64)
            tks.append(net.fetch_outputs_async(b0, b1, oo, ii, dig[0, b0:b1], dig[1, b0:b1]))
            blocks.append((oo, ii))
        for tk in tks:
            net.fetch_wait(tk)
    res["run_fetch_pinned_ms"] = best(run_fetch)
    res["fetch_gbs"] = round(res["bytes_fetched"] / (res["run_fetch_pinned_ms"] -
                                                      res["run_ms"]) / 1e6, 2)

    def overlap():
        """The yield loop's device/host overlap: enqueue every block, then wait block by block
        and digest its rows (what _simulate_fused does between yields, minus the model)."""
        net.run(x)
        dig = muskingum._host_array((2, T), np.uint64)
        t0 = time.perf_counter()
        tks = []
        bl = []
        for b0 in range(0, T, block):
            b1 = min(T, b0 + block)
            oo = muskingum._host_array((b1 - b0, n), np.float64)
            ii = muskingum._host_array((b1 - b0, n), np.float64)
            tks.append(net.fetch_outputs_async(b0, b1, oo, ii, dig[0, b0:b1], dig[1, b0:b1]))
            bl.append((oo, ii))
        t1 = time.perf_counter()
        first = None
        for (oo, ii), tk in zip(bl, tks):
            net.fetch_wait(tk)
            if first is None:
                first = time.perf_counter()
            for k in range(oo.shape[0]):
                engine.host_digest(oo[k])
                engine.host_digest(ii[k])
        t2 = time.perf_counter()
        res["enqueue_ms"] = 1e3 * (t1 - t0)
        res["first_block_ms"] = 1e3 * (first - t0)
        res["wait_and_digest_loop_ms"] = 1e3 * (t2 - t0)
    overlap()
    overlap()

    def digests():
        for oo, ii in blocks:
            for k in range(oo.shape[0]):
                engine.host_digest(oo[k])
                engine.host_digest(ii[k])
    res["host_digests_ms"] = best(digests)
    net.close()
    res["api_ms"] = bench.api_timing(wl)
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}),
          flush=True)


if __name__ == "__main__":
    main()
