#!/usr/bin/env python3
"""Benchmark: reach·timesteps/s of the Muskingum routing hot path on MI355X.

Workload (BASELINE.json configs[1]): the full-Texas-scale synthetic network (190k reaches,
~300 outlets, deepest flow path ~1500 reaches), deterministic run, 24 h at dt = 300 s
(T = 288 steps), hourly lateral-inflow forcing (25 rows).  One bench "step" = one whole 24-h
horizon routed by `mc_run` (forcing interpolation + network routing for all 288 timesteps),
inputs and outputs resident in HBM.

Multi-GPU (`torch.distributed.run --nproc-per-node N`): the deterministic run does not shard
 -- every rank routes its own independent replica (different forcing seed), no
data-path collective; value = reach·timesteps of all ranks / max-over-ranks time ("weak").

Prints ONE JSON line on rank 0 with `roofline` (HIP-event timed wavefront launches against the
HBM roofline, algorithmic 72 B per reach·timestep) and `cpu_baseline` (the serial
C transliteration of the reference loop, oracle/, timed on this host; rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tx-fast-hydrology_amd"))
sys.path.insert(0, ROOT)

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E peak (MI355X_MICROARCH.md, spec)
BYTES_PER_UNIT = 72.0        # 7 f64 reads + 2 f64 writes per reach·timestep


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--n", type=int, default=190_000)
    ap.add_argument("--basins", type=int, default=300)
    ap.add_argument("--depth", type=int, default=1500)
    ap.add_argument("--T", type=int, default=288)
    ap.add_argument("--dt", type=float, default=300.0)
    # 0 = per workload: 448 lanes + the helper wave make the deterministic Texas network one
    # resident dataflow launch; ensembles run the multi-launch path at 256
    ap.add_argument("--slots", type=int, default=0)
    ap.add_argument("--members", type=int, default=1,
                    help="ensemble members (BASELINE configs[2]: 64); 1 = deterministic")
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--timing-runs", type=int, default=3)
    return ap.parse_args()


def measured_traffic(info, n, T):
    """HBM bytes per launch of the routing kernel measured with rocprofv3 PMC counters for this
    exact workload (scripts/hbm_traffic.py -> profiles/*_hbm_traffic.json), newest first."""
    import glob
    want = {"slots": info["slots"], "tile": info["tile"], "n": n, "T": T}
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_hbm_traffic.json")), reverse=True):
        try:
            rec = json.load(open(f))
        except (OSError, ValueError):
            continue
        if rec.get("workload") == want:
            rec["file"] = os.path.relpath(f, ROOT)
            return rec
    return None


def build_workload(args, rank=0):
    """Texas-scale synthetic network, coefficients, state and forcing, loaded into a RoutingNet.
    Returns (net, w): w holds the host arrays (w.x = step times of one horizon)."""
    from types import SimpleNamespace

    from tx_fast_hydrology_amd import engine, synthetic

    end = synthetic.river_network(args.n, args.basins, args.depth, np.random.default_rng(0))
    n = end.size
    K, X, o0 = synthetic.model_arrays(n, seed=0)
    start = np.arange(n, dtype=np.int64)
    indeg = np.bincount(end, minlength=n) - (end == start)
    heads = start[indeg == 0]
    dt = args.dt
    alpha = (dt - 2 * K * X) / (2 * K * (1 - X) + dt)          # muskingum.py:332-347
    beta = (dt + 2 * K * X) / (2 * K * (1 - X) + dt)
    chi = (2 * K * (1 - X) - dt) / (2 * K * (1 - X) + dt)
    gamma = dt / (K * (1 - X) + dt / 2)
    rows = int(np.ceil(args.T * dt / 3600.0)) + 1
    xp_ns, fp = synthetic.forcing(n, rows=rows, seed=1 + rank)
    xp = xp_ns.astype(float)
    x = xp[0] + dt * 1e9 * np.arange(1, args.T + 1)
    E = args.members
    if E > 1:
        o0, fp = synthetic.ensemble(o0, fp, E, seed=5 + 7 * rank)
    i0 = np.zeros(o0.shape)
    np.add.at(i0, end, o0)                                      # muskingum.py:416-417

    slots = args.slots or (448 if E == 1 else 256)
    net = engine.RoutingNet(end, indeg, heads, slots=slots, tile=args.tile, members=E)
    net.set_coeffs(alpha, beta, chi, gamma)
    net.set_state(o0, i0)
    net.load_forcing(xp, fp)
    w = SimpleNamespace(n=n, start=start, end=end, indeg=indeg, alpha=alpha, beta=beta, chi=chi,
                        gamma=gamma, o0=o0, i0=i0, x=x, xp=xp, fp=fp, rows=rows, dt=dt, E=E)
    return net, w


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)

    from oracle import oracle as orc  # noqa: F401  (cpu_baseline leg only)

    # ---- workload -------------------------------------------------------------------------
    t_setup = time.time()
    net, wl = build_workload(args, rank)
    n, x = wl.n, wl.x
    info = net.info
    setup_s = time.time() - t_setup

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    # ---- warmup + timed region -------------------------------------------------------------
    for _ in range(args.warmup):
        net.run(x)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        net.run(x)
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    E = wl.E
    units = float(n) * E * args.T * args.steps * world
    value = units / elapsed

    # ---- roofline of the dominant kernel (HIP events around every wavefront launch) --------
    net.reset_timing()
    net.set_timing(True)
    for _ in range(args.timing_runs):
        net.run(x)
    net.synchronize()
    tm = net.timing()
    net.set_timing(False)
    launch_ms = tm["kernel_ms"] / max(tm["launches"], 1)
    # 72 B per reach·timestep deterministic, 40 + 32/E per reach·member·timestep
    per_unit = BYTES_PER_UNIT if E == 1 else 40.0 + 32.0 / E
    bytes_per_launch = per_unit * n * E * args.T * args.timing_runs / max(tm["launches"], 1)
    achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
    traffic = measured_traffic(info, n, args.T) if E == 1 else None
    roofline = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                "traffic": traffic["traffic_bytes_per_launch"] if traffic else None,
                "traffic_source": traffic["file"] if traffic else None,
                "kernel": "wavefront_flow" if net.mode()[1] == "dataflow" else "wavefront_det",
                "launches_per_step": tm["launches"] / args.timing_runs,
                "avg_launch_us": round(launch_ms * 1e3, 3),
                "kernel_ms_per_step": round(tm["kernel_ms"] / args.timing_runs, 4)}

    # ---- CPU baseline (serial transliteration of the reference loop, rank 0 at N=1) --------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and E > 1:
        # E independent member runs over the host cores the box gives this job (OpenMP)
        cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
        ms = min(E, cores)
        o_s = np.ascontiguousarray(wl.o0[:, :ms])
        i_s = np.ascontiguousarray(wl.i0[:, :ms])
        fps = np.ascontiguousarray(wl.fp[:, :, :ms])
        reps, t_cpu = 0, 0.0
        while t_cpu < args.cpu_seconds or reps == 0:
            c0 = time.perf_counter()
            o_s, i_s = orc.simulate_members(wl.start, wl.end, wl.indeg, wl.alpha, wl.beta,
                                            wl.chi, wl.gamma, o_s, i_s, x, wl.xp, fps,
                                            threads=cores)
            t_cpu += time.perf_counter() - c0
            reps += 1
        cpu = {"value": float(n) * ms * args.T * reps / t_cpu,
               "unit": "reach·member·timesteps/s", "cores": cores, "kind": "port",
               "sample": f"{reps} x full 24 h horizon (T={args.T}) of {ms} members on the same "
                         f"{n}-reach network, C member loop (-O3 -ffp-contract=off, OpenMP "
                         f"over members), {t_cpu:.1f} s"}
    elif rank == 0 and world == 1 and not args.no_cpu:
        o_s, i_s = wl.o0.copy(), wl.i0.copy()
        reps, t_cpu = 0, 0.0
        while t_cpu < args.cpu_seconds or reps == 0:
            c0 = time.perf_counter()
            orc.simulate(wl.start, wl.end, wl.indeg, wl.alpha, wl.beta, wl.chi, wl.gamma, o_s,
                         i_s, x, wl.xp, wl.fp, keep_outputs=False)
            t_cpu += time.perf_counter() - c0
            reps += 1
        cpu = {"value": float(n) * args.T * reps / t_cpu, "unit": "reach·timesteps/s",
               "cores": 1, "kind": "port",
               "sample": f"{reps} x full 24 h horizon (T={args.T}) on the same {n}-reach "
                         f"network, serial C (-O3 -ffp-contract=off), {t_cpu:.1f} s"}

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "reach·timesteps/s" if E == 1 else "reach·member·timesteps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": ("texas-det (BASELINE configs[1]): full-Texas synthetic "
                                    "network, deterministic, 24 h @ 300 s") if E == 1 else
                                   (f"texas-ens{E} (BASELINE configs[2]): full-Texas synthetic "
                                    f"network, {E}-member ensemble forecast, 24 h @ 300 s"),
                       "members": E,
                       "n_reaches": n, "outlets": int((wl.end == wl.start).sum()),
                       "max_height": info["max_height"], "T": args.T, "dt_s": wl.dt,
                       "forcing_rows": wl.rows, "parallelism": f"replicas x{world}",
                       "slots": info["slots"], "tile": info["tile"], "nwg": info["nwg"],
                       "schedule_ticks": info["gmax"] + args.T, "setup_s": round(setup_s, 2)},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        if cpu:
            line["speedup_vs_cpu"] = value / cpu["value"]
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
