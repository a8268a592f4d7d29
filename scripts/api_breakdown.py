#!/usr/bin/env python3
"""Where the drop-in API horizon goes (Muskingum.simulate over Texas, T = 288): device run,
output fetch to host, per-step edit digests, and the whole generator.  Prints one JSON line.
    python scripts/api_breakdown.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tx-fast-hydrology_amd"))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from tx_fast_hydrology_amd import muskingum  # noqa: E402


def main():
    args = bench.parse([], world=1)
    net, wl = bench.build_workload(args)
    x = wl.x
    T = x.size
    chunk = max(1, muskingum._HORIZON_CHUNK_VALUES // wl.n)
    res = {}
    for r in range(3):
        t0 = time.perf_counter()
        for c0 in range(0, T, chunk):
            net.run(x[c0:c0 + chunk])
            net.synchronize()
        res["run_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        outs = []
        for c0 in range(0, T, chunk):
            net.run(x[c0:c0 + chunk])
            outs.append(net.fetch_outputs())
        res["run_fetch_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        for oo, ii in outs:
            for k in range(oo.shape[0]):
                muskingum._digest(oo[k])
                muskingum._digest(ii[k])
        res["digest_once_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        for oo, ii in outs:
            oo.copy()
            ii.copy()
        res["host_copy_s"] = time.perf_counter() - t0
        del outs
    net.close()
    res["api_s"] = bench.api_timing(wl) / 1e3
    res["steps"] = T
    res["bytes_fetched"] = 2 * 8 * wl.n * T
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
