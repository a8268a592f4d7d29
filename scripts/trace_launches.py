#!/usr/bin/env python3
"""Diagnostic: launch trace of one bench horizon (mc_set_trace).  Prints, per launch, the number
of workgroups, dispatch spread, mean prologue / tick-loop time, shader cycles per tick and the
launch span, then a one-line summary; saves the raw records to gpurun_out/trace_<tag>.npz.
    python scripts/trace_launches.py [tag] [--quiet] [bench.py workload flags]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def summarize(rec, khz, tile, quiet=False):
    us = 1e3 / khz                                   # microseconds per wall-clock tick
    t00 = rec[:, 2].min()
    lines = []
    spans, loops_tail, cyc_tail, pro = [], [], [], []
    for k in np.unique(rec[:, 0]):
        r = rec[rec[:, 0] == k]
        st, lp, en = r[:, 2], r[:, 3], r[:, 4]
        cyc = (r[:, 7] - r[:, 6]) / tile
        ghz = (r[:, 7] - r[:, 6]).sum() / ((en - lp).sum() * us * 1e3)
        span = (en.max() - st.min()) * us
        spans.append(span)
        pro.append(((lp - st).mean()) * us)
        if len(r) <= 32:
            loops_tail.append(((en - lp).mean()) * us)
            cyc_tail.append(cyc.mean())
        lines.append(f"{k:5d} {len(r):5d} {(st.min() - t00) * us:9.1f} "
                     f"{(st.max() - st.min()) * us:7.2f} {pro[-1]:7.2f} "
                     f"{((en - lp).mean()) * us:7.2f}/{((en - lp).max()) * us:6.2f} "
                     f"{cyc.mean():7.0f}/{cyc.max():6.0f} {ghz:5.2f} {span:8.2f}")
    total = (rec[:, 4].max() - t00) * us
    if not quiet:
        print("launch  nwg  start_us spread prolog loop_us(mean/max) cyc/tick(mean/max) GHz span")
        print("\n".join(lines))
    heavy = sum(s for s, k in zip(spans, np.unique(rec[:, 0]))
                if (rec[:, 0] == k).sum() > 32)
    print(f"SUMMARY total_us={total:.1f} sum_span_us={sum(spans):.1f} heavy_span_us={heavy:.1f} "
          f"tail_launches={len(loops_tail)} tail_loop_us={np.mean(loops_tail):.2f} "
          f"tail_cyc_per_tick={np.mean(cyc_tail):.0f} mean_prolog_us={np.mean(pro):.2f}")


def summarize_flow(rec, khz, gmin, gmax, T):
    """One dataflow launch: per-workgroup tick rate and when each workgroup's loop started."""
    us = 1e3 / khz
    st, lp, en = rec[:, 2], rec[:, 3], rec[:, 4]
    t0 = st.min()
    w = rec[:, 1]
    kb = gmin[w] & ~7
    ticks = ((gmax[w] + T + 7) & ~7) - kb
    ns_tick = (en - lp) * us * 1e3 / ticks
    cyc_tick = (rec[:, 7] - rec[:, 6]) / ticks
    last = np.argsort(-(en - t0))[:5]
    print(f"workgroups {len(rec)}  span_us {(en.max() - t0) * us:.1f}  "
          f"start spread {(st.max() - t0) * us:.2f}  prologue(incl. first wait) mean "
          f"{((lp - st) * us).mean():.2f} max {((lp - st) * us).max():.2f}")
    print("ns/tick percentiles 10/50/90/max:",
          np.round(np.percentile(ns_tick, [10, 50, 90, 100]), 1),
          " cycles/tick median", np.round(np.median(cyc_tick)))
    for i in last:
        print(f"  last: wg {w[i]} gmin {gmin[w[i]]} gmax {gmax[w[i]]} loop start "
              f"{(lp[i] - t0) * us:.1f} us end {(en[i] - t0) * us:.1f} us, {ticks[i]} ticks, "
              f"{ns_tick[i]:.0f} ns/tick")
    # wall time at which each workgroup's loop started vs its first tick label
    order = np.argsort(kb)
    print("loop start vs first tick (every 76th workgroup by gmin): ",
          [(int(kb[i]), round(float((lp[i] - t0) * us), 1)) for i in order[::76]])
    print(f"SUMMARY total_us={(en.max() - t0) * us:.1f} median_ns_per_tick={np.median(ns_tick):.0f}")


def wg_windows(plan):
    """G range of every workgroup's node slots (chain * slots per workgroup, padding
    excluded)."""
    ex, ln = plan.export(), plan.export_links()
    rs = plan.info["chain"] * plan.info["slots"]
    G = ex["G"].reshape(-1, rs)
    used = ln["flags"].reshape(G.shape) != 0
    return np.where(used, G, 1 << 30).min(1), np.where(used, G, -1).max(1)


def main():
    argv = sys.argv[1:]
    quiet = "--quiet" in argv
    argv = [a for a in argv if a != "--quiet"]
    tag = argv[0] if argv and not argv[0].startswith("-") else "t"
    sys.argv = [sys.argv[0]] + [a for a in argv if a != tag]
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
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", f"trace_{tag}.npz"), rec=rec, khz=khz)
    print(f"[{tag}] clock {khz} kHz, {rec.shape[0]} records, {rec[:, 0].max() + 1} launches, "
          f"path {net.mode()[1]}")
    if net.mode()[1] == "dataflow":
        from tx_fast_hydrology_amd import engine
        heads = np.flatnonzero(wl.indeg == 0)
        plan = engine.Plan(wl.end, wl.indeg, heads, slots=net.info["slots"],
                           tile=net.info["tile"], chain=net.info["chain"])
        gmin, gmax = wg_windows(plan)
        summarize_flow(rec, khz, gmin, gmax, len(wl.x))
    else:
        summarize(rec, khz, net.info["tile"], quiet)


if __name__ == "__main__":
    main()
