#!/usr/bin/env python3
"""Diagnostic: launch trace of one bench horizon (mc_set_trace).  Prints, per launch, the number
of workgroups, their dispatch spread, mean prologue / tick-loop time and the launch span, and
saves the raw records to gpurun_out/trace_<tag>.npz.
    python scripts/trace_launches.py [tag] [--slots S --tile T ...]  (bench.py workload flags)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "t"
    sys.argv = [sys.argv[0]] + [a for a in sys.argv[1:] if a != tag]
    args = bench.parse()
    import torch
    torch.cuda.set_device(0)
    net, wl = bench.build_workload(args)
    for _ in range(2):
        net.run(wl.x)
    net.set_trace(True)
    net.run(wl.x)
    net.synchronize()
    rec, khz = net.trace()
    us = 1e3 / khz                                   # microseconds per clock tick
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", f"trace_{tag}.npz"), rec=rec, khz=khz)
    t00 = rec[:, 2].min()
    print(f"clock {khz} kHz, {rec.shape[0]} records, {rec[:, 0].max() + 1} launches")
    print("launch  nwg  start_us  spread_us  prolog_us  loop_us(mean/max)  span_us  xcds")
    for k in np.unique(rec[:, 0]):
        r = rec[rec[:, 0] == k]
        st, lp, en = r[:, 2], r[:, 3], r[:, 4]
        xcc = (r[:, 5] >> 16) & 0xf if False else None
        print(f"{k:5d} {len(r):5d} {(st.min() - t00) * us:9.1f} {(st.max() - st.min()) * us:9.2f}"
              f" {((lp - st).mean()) * us:9.2f} {((en - lp).mean()) * us:8.2f}/"
              f"{((en - lp).max()) * us:7.2f} {(en.max() - st.min()) * us:8.2f}")
    hw = rec[:, 5]
    print("hw_id sample:", [hex(v) for v in hw[:8]])


if __name__ == "__main__":
    main()
