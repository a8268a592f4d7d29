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
    # 0 = per workload: 192 lanes (2 node slots each) + the helper wave make the deterministic
    # Texas network one resident dataflow launch (two workgroups per CU); ensemble forecasts run
    # the multi-launch path at 256
    ap.add_argument("--slots", type=int, default=0)
    ap.add_argument("--members", type=int, default=1,
                    help="ensemble members (BASELINE configs[2]: 64); 1 = deterministic")
    ap.add_argument("--enkf", action="store_true",
                    help="BASELINE configs[3]: --members is the TOTAL ensemble, sharded over the "
                         "ranks, with the ensemble Kalman analysis at every step of the first "
                         "2 h (hourly gauge observations)")
    ap.add_argument("--gauges", type=int, default=500)
    ap.add_argument("--obs-hours", type=float, default=2.0)
    ap.add_argument("--one-plan", action="store_true",
                    help="EnKF: route the forecast on the analysis plan too (no hand-over)")
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--chain", type=int, default=0,
                    help="node slots per lane (plan.hpp lane chains); 0 = per workload")
    ap.add_argument("--vec-shape", default="",
                    help="route with the member-vector sweep at shape H:W (node slots per wave "
                         "instruction, waves per workgroup; 0 = automatic)")
    ap.add_argument("--conus", action="store_true",
                    help="BASELINE configs[4]: CONUS NWM-scale synthetic network (2.7M reaches, "
                         "4000 outlets, deepest path ~7000 reaches); --members per GPU (default "
                         "16: the 128-member ensemble over 8 GPUs, one 16-member shard per rank)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--timing-runs", type=int, default=3)
    return apply_presets(ap.parse_args())


def measured_traffic(info, n, T, E=1):
    """HBM bytes per launch of the routing kernel measured with rocprofv3 PMC counters for this
    exact workload (scripts/hbm_traffic.py -> profiles/*_hbm_traffic.json), newest first."""
    import glob
    want = {"slots": info["slots"], "tile": info["tile"], "n": n, "T": T}
    if E > 1:
        want["E"] = E
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_hbm_traffic*.json")),
                    reverse=True):
        try:
            rec = json.load(open(f))
        except (OSError, ValueError):
            continue
        if rec.get("workload") == want:
            rec["file"] = os.path.relpath(f, ROOT)
            return rec
    return None


def apply_presets(args):
    if args.conus:
        args.n, args.basins, args.depth = 2_700_000, 4000, 7000
        if args.members == 1:
            args.members = 16
    return args


def build_workload(args, rank=0, world=1):
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
    # replicas route different forcing per rank; the sharded EnKF ensemble is ONE ensemble
    xp_ns, fp = synthetic.forcing(n, rows=rows, seed=1 if args.enkf else 1 + rank)
    xp = xp_ns.astype(float)
    x = xp[0] + dt * 1e9 * np.arange(1, args.T + 1)
    E = args.members
    enkf = None
    if args.enkf:
        if E % world or E < 2:
            raise SystemExit("--enkf needs >= 2 members, divisible by the number of ranks")
        El = E // world
        o_base = o0
        o0, fp = synthetic.ensemble(o_base, fp, E, seed=5, cols=slice(rank * El, (rank + 1) * El))
        # gauges: non-headwater reaches (seed 7); hourly obs for the first 2 h, interpolated at
        # every model step (da.py:71-81) -> one analysis per step; a "truth" 10 % above the
        # initial ensemble mean plus N(0, 0.1^2) noise; R = 1e-2 I (app.py:137-139)
        rng = np.random.default_rng(7)
        cand = np.flatnonzero(indeg > 0)
        gauges = np.sort(rng.choice(cand, min(args.gauges, cand.size), replace=False))
        m = gauges.size
        m_o = np.random.default_rng(6).lognormal(0.0, 0.3, (n, E))[gauges]
        truth = 1.1 * (o_base[gauges, None] * m_o).mean(1)
        R = 1e-2 * np.eye(m)
        n_an = int(round(args.obs_hours * 3600.0 / dt))
        obs_rng = np.random.default_rng(1000 + rank)
        Y = [np.ascontiguousarray(truth[:, None] + rng_k)
             for rng_k in (np.random.default_rng(100 + k).normal(0, 0.1, (m, 1)) +
                           obs_rng.normal(0, 0.1, (m, El)) for k in range(n_an))]
        enkf = SimpleNamespace(gauges=gauges, R=R, Y=Y, n_an=n_an, m=m, E_total=E)
        E = El
    elif E > 1:
        o0, fp = synthetic.ensemble(o0, fp, E, seed=5 + 7 * rank)
    i0 = np.zeros(o0.shape)
    np.add.at(i0, end, o0)                                      # muskingum.py:416-417

    # 192 lanes (3 compute waves + the helper: one wave per SIMD, two workgroups per CU) for
    # the resident dataflow kernels (det horizon, EnKF member steps); ensemble forecasts 256
    slots = args.slots or (192 if E == 1 or enkf is not None else 256)
    # ensemble forecasts (multi-launch path): 64-tick launches amortise the per-launch slot
    # loads (Texas ens64 14.1 -> 13.1 ms per horizon); the EnKF keeps 32, whose shorter
    # schedule its one-step member-dataflow launches pay for at every analysis
    # the dataflow workloads at a 16-tick cross-cluster slack (two chunks, the minimum): Texas
    # det 0.605 -> 0.594 ms
    tile = args.tile or (64 if E > 1 and enkf is None else 16)
    net = engine.RoutingNet(end, indeg, heads, slots=slots, tile=tile, members=E,
                            chain=args.chain)
    if args.vec_shape:         # the member-vector sweep (mcroute.h mode 3) at this shape
        net.set_mode("vector")
        net.set_vector_shape(*(int(v) for v in args.vec_shape.split(":")))
    net.set_coeffs(alpha, beta, chi, gamma)
    net.set_state(o0, i0)
    net.load_forcing(xp, fp)
    if enkf is not None and not args.one_plan:
        # the forecast after the last analysis runs on its own plan (256 lanes, 64-tick
        # launches: the multi-launch ensemble shape), the state handed over on the device
        fnet = engine.RoutingNet(end, indeg, heads, slots=256, tile=64, members=E)
        fnet.set_coeffs(alpha, beta, chi, gamma)
        fnet.load_forcing(xp, fp)
        enkf.fnet = fnet
    w = SimpleNamespace(n=n, start=start, end=end, indeg=indeg, alpha=alpha, beta=beta, chi=chi,
                        gamma=gamma, o0=o0, i0=i0, x=x, xp=xp, fp=fp, rows=rows, dt=dt, E=E,
                        enkf=enkf)
    return net, w


def workload_name(wl, E):
    if wl.enkf is not None:
        ek = wl.enkf
        return (f"texas-enkf{ek.E_total} (BASELINE configs[3]): full-Texas synthetic network, "
                f"{ek.E_total}-member ensemble, EnKF analysis at the first {ek.n_an} steps "
                f"({ek.m} gauges), 24 h @ 300 s")
    if wl.n > 1_000_000:
        return (f"conus-ens (BASELINE configs[4]): CONUS-scale synthetic network ({wl.n} "
                f"reaches), {E} members per GPU (128 over 8 GPUs), 24 h @ 300 s")
    if E == 1:
        return ("texas-det (BASELINE configs[1]): full-Texas synthetic network, deterministic, "
                "24 h @ 300 s")
    return (f"texas-ens{E} (BASELINE configs[2]): full-Texas synthetic network, {E}-member "
            f"ensemble forecast, 24 h @ 300 s")


def cpu_enkf_baseline(args, wl, orc):
    """Host baseline of the EnKF horizon on a bounded sample: min(E, cores) members through the C
    member loop (OpenMP) with a NumPy ensemble analysis at the analysis steps."""
    cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    ek = wl.enkf
    ms = min(wl.E, cores)
    o = np.ascontiguousarray(wl.o0[:, :ms])
    i = np.ascontiguousarray(wl.i0[:, :ms])
    fp = np.ascontiguousarray(wl.fp[:, :, :ms])
    x = wl.x
    g = ek.gauges
    coef = (wl.alpha, wl.beta, wl.chi, wl.gamma)
    heads = wl.start[wl.indeg == 0]
    reps, t = 0, 0.0
    while t < args.cpu_seconds or reps == 0:
        c0 = time.perf_counter()
        for k in range(ek.n_an):
            o, i = orc.simulate_members(wl.start, wl.end, wl.indeg, *coef, o, i, x[k:k + 1],
                                        wl.xp, fp, threads=cores)
            A = o - o.mean(1, keepdims=True)
            HA = A[g]
            W = np.linalg.solve(HA @ HA.T / (ms - 1) + ek.R, ek.Y[k][:, :ms] - o[g])
            G = A @ (HA.T @ W) / (ms - 1)
            for e in range(ms):
                ig, og = orc.apply_gain(heads, wl.end, np.ascontiguousarray(G[:, e]), wl.indeg)
                o[:, e] += og
                i[:, e] += ig
            o, i = np.ascontiguousarray(o), np.ascontiguousarray(i)
        o, i = orc.simulate_members(wl.start, wl.end, wl.indeg, *coef, o, i, x[ek.n_an:], wl.xp,
                                    fp, threads=cores)
        t += time.perf_counter() - c0
        reps += 1
    return {"value": float(wl.n) * ms * args.T * reps / t, "unit": "reach·member·timesteps/s",
            "cores": cores, "kind": "port",
            "sample": f"{reps} x full 24 h EnKF horizon (T={args.T}, {ek.n_an} analysis steps) "
                      f"of {ms} members on the same {wl.n}-reach network: C member loop "
                      f"(OpenMP) + NumPy ensemble analysis + C _apply_gain, {t:.1f} s"}


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
    net, wl = build_workload(args, rank, world)
    n, x = wl.n, wl.x
    from tx_fast_hydrology_amd import ensemble

    def horizon():
        """One bench step: a 24-h horizon (with the analysis steps of the EnKF workload)."""
        if wl.enkf is None:
            net.run(x)
            return
        ek = wl.enkf
        for k in range(ek.n_an):       # analysis at every model step while obs exist
            net.run(x[k:k + 1])
            ensemble.distributed_analysis(net, ek.gauges, ek.Y[k], ek.R)
        if getattr(ek, "fnet", None) is None:
            net.run(x[ek.n_an:])
            return
        ek.fnet.copy_state_from(net)
        ek.fnet.run(x[ek.n_an:])
        net.copy_state_from(ek.fnet)
    info = net.info
    setup_s = time.time() - t_setup

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    # ---- warmup + timed region -------------------------------------------------------------
    for _ in range(args.warmup):
        horizon()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        horizon()
    barrier()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    E = wl.E
    if wl.enkf is not None:            # one ensemble sharded over the ranks (strong scaling)
        units = float(n) * wl.enkf.E_total * args.T * args.steps
    else:                              # replicas: every rank routes its own run (weak)
        units = float(n) * E * args.T * args.steps * world
    value = units / elapsed

    # ---- roofline of the dominant kernel (HIP events around every wavefront launch) --------
    nets = [net] + ([wl.enkf.fnet] if getattr(wl.enkf, "fnet", None) is not None else [])
    for nt in nets:
        nt.reset_timing()
        nt.set_timing(True)
    for _ in range(args.timing_runs):
        horizon()
    tm = {"kernel_ms": 0.0, "launches": 0}
    for nt in nets:
        nt.synchronize()
        t_ = nt.timing()
        tm["kernel_ms"] += t_["kernel_ms"]
        tm["launches"] += t_["launches"]
        nt.set_timing(False)
    launch_ms = tm["kernel_ms"] / max(tm["launches"], 1)
    # 72 B per reach·timestep deterministic, 40 + 32/E per reach·member·timestep
    per_unit = BYTES_PER_UNIT if E == 1 else 40.0 + 32.0 / E
    bytes_per_launch = per_unit * n * E * args.T * args.timing_runs / max(tm["launches"], 1)
    achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
    traffic = measured_traffic(info, n, args.T, E) if wl.enkf is None else None
    roofline = {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6),
                "traffic": traffic["traffic_bytes_per_launch"] if traffic else None,
                "traffic_source": traffic["file"] if traffic else None,
                # measured HBM bytes per launch / launch time: the DRAM rate the kernel drives
                "traffic_gbs": (round(traffic["traffic_bytes_per_launch"] / (launch_ms * 1e-3)
                                      / 1e9, 3) if traffic else None),
                # the same DRAM rate as a fraction of the HBM peak: the routing recurrence keeps
                # coefficients and state in registers / LDS and is bound by its dependency chain
                # (schedule ticks x per-tick latency), not by DRAM bandwidth
                "dram_frac": (round(traffic["traffic_bytes_per_launch"] / (launch_ms * 1e-3)
                                    / 1e9 / HBM_PEAK_GBS, 4) if traffic else None),
                "algorithmic_bytes_per_unit": per_unit,
                "kernel": {"dataflow": "wavefront_flow", "vector": "wavefront_vec"}.get(
                    net.mode()[1], "wavefront_det"),
                "launches_per_step": tm["launches"] / args.timing_runs,
                "avg_launch_us": round(launch_ms * 1e3, 3),
                "kernel_ms_per_step": round(tm["kernel_ms"] / args.timing_runs, 4)}

    # ---- CPU baseline (serial transliteration of the reference loop, rank 0 at N=1) --------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and wl.enkf is not None:
        cpu = cpu_enkf_baseline(args, wl, orc)
    elif rank == 0 and world == 1 and not args.no_cpu and E > 1:
        # E independent member runs over the host cores the box gives this job (OpenMP)
        cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
        ms = min(E, cores)
        o_s = np.ascontiguousarray(wl.o0[:, :ms])
        i_s = np.ascontiguousarray(wl.i0[:, :ms])
        fps = np.ascontiguousarray(wl.fp[:, :, :ms])
        # bounded sample: consecutive 12-step chunks of the horizon (wrapping) until the budget
        steps_done, t_cpu, k = 0, 0.0, 0
        while t_cpu < args.cpu_seconds or steps_done == 0:
            xs = x[k:k + 12]
            c0 = time.perf_counter()
            o_s, i_s = orc.simulate_members(wl.start, wl.end, wl.indeg, wl.alpha, wl.beta,
                                            wl.chi, wl.gamma, o_s, i_s, xs, wl.xp, fps,
                                            threads=cores)
            t_cpu += time.perf_counter() - c0
            steps_done += xs.size
            k = (k + xs.size) % x.size
        cpu = {"value": float(n) * ms * steps_done / t_cpu,
               "unit": "reach·member·timesteps/s", "cores": cores, "kind": "port",
               "sample": f"{steps_done} timesteps (12-step chunks of the 24 h horizon, T={args.T}) "
                         f"of {ms} members on the same {n}-reach network, C member loop (-O3 "
                         f"-ffp-contract=off, OpenMP over members), {t_cpu:.1f} s"}
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
            "unit": ("reach·timesteps/s" if E == 1 and wl.enkf is None
                     else "reach·member·timesteps/s"),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            # one bench step = one whole T-step horizon (module docstring)
            "ms_per_step": elapsed / args.steps * 1e3,
            "ms_per_horizon": elapsed / args.steps * 1e3,
            "us_per_timestep": elapsed / args.steps / args.T * 1e6,
            "higher_is_better": True,
            "scaling": "strong" if wl.enkf is not None else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": workload_name(wl, E),
                       "members": wl.enkf.E_total if wl.enkf is not None else E,
                       "members_per_gpu": E,
                       "n_reaches": n, "outlets": int((wl.end == wl.start).sum()),
                       "max_height": info["max_height"], "T": args.T, "dt_s": wl.dt,
                       "forcing_rows": wl.rows,
                       "parallelism": (f"members sharded x{world}" if wl.enkf is not None
                                       else f"replicas x{world}"),
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
