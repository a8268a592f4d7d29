#!/usr/bin/env python3
"""Benchmark: reach·timesteps/s of the Muskingum routing hot path on MI355X.

Workloads (BASELINE.json configs, SURVEY §8d synthetic generators):
  * N = 1 default -- configs[1]: the full-Texas-scale synthetic network (190k reaches, ~300
    outlets, deepest flow path ~1500 reaches), deterministic, 24 h at dt = 300 s (T = 288),
    hourly lateral-inflow forcing (25 rows).  One bench "step" = one whole 24-h horizon routed
    by `mc_run` (forcing interpolation + routing of all 288 timesteps), inputs and outputs
    resident in HBM.
  * N > 1 default -- configs[3]: the 256-member Texas EnKF (ensemble Kalman analysis at every
    step of the first 2 h, 500 gauges, R = 1e-2 I) with the members SHARDED over the ranks
    (256 / N each; RCCL all-gather + all-to-all in the analysis, ensemble.py): strong scaling,
    value = reach·member·timesteps of the whole ensemble / max-over-ranks time.  The replicated
    deterministic run (every rank its own Texas replica, no collective, "weak") is measured
    after it and reported in the same line under "det_replicas".
  * --huc8 (configs[0]: one ~1k-reach HUC-8 sub-basin, deterministic, the reference's CPU
    path; its cpu_baseline is that path's serial loop), --members 64 (configs[2]), --conus (configs[4], one GPU's 16-member share), --enkf,
    --det (N > 1: the replicated deterministic line as the headline).

`--gpus N` without a launcher starts `torch.distributed.run --nproc-per-node N` on this script
as a CHILD process (never exec) and exits with its status; under a launcher, --gpus must equal
WORLD_SIZE.

Prints ONE JSON line on rank 0 with
  * `roofline`: the contract's algorithmic figure (SURVEY §8d bytes per unit / HIP-event launch
    time vs the HBM peak) and what bounds the kernel: `latency` (schedule ticks x the measured
    floor of the bare tick chain, mc_probe_tick_floor), `compulsory` (bytes the horizon must
    move: outflows written, forcing / coefficients / state read, state written) and `dram`
    (rocprofv3 PMC bytes of THIS build, profiles/*_hbm_traffic*.json, source-hash checked);
  * `cpu_baseline`: the oracle's C transliteration of the reference loop (oracle/, test
    infrastructure used only here) timed on this host's cores, on rank 0 at any N (after the
    timed region);
  * `emulated_shards` (--enkf --emulate-shards N at N = 1): the configs[3] horizon as N member
    shards on the one GPU, each shard's device time, and the projected N-GPU speed-up;
  * `api_ms_per_horizon` (det, N = 1): the drop-in `Muskingum.simulate` over the same horizon,
    host fetch of every step's outflows and inflows included.
"""
from __future__ import annotations

import argparse
import copy
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "tx-fast-hydrology_amd"))
sys.path.insert(0, ROOT)

METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E peak (MI355X_MICROARCH.md, spec)
BYTES_PER_UNIT = 72.0        # 7 f64 reads + 2 f64 writes per reach·timestep


def parse(argv=None, world=None):
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
    ap.add_argument("--members", type=int, default=None,
                    help="ensemble members (BASELINE configs[2]: 64); default 1 at N = 1, the "
                         "256-member EnKF at N > 1")
    ap.add_argument("--enkf", action="store_true",
                    help="BASELINE configs[3]: --members is the TOTAL ensemble, sharded over the "
                         "ranks, with the ensemble Kalman analysis at every step of the first "
                         "2 h (hourly gauge observations)")
    ap.add_argument("--det", action="store_true",
                    help="N > 1: the replicated deterministic run as the headline line")
    ap.add_argument("--gauges", type=int, default=500)
    ap.add_argument("--obs-hours", type=float, default=2.0)
    ap.add_argument("--one-plan", action="store_true",
                    help="EnKF: route the forecast on the analysis plan too (no hand-over)")
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--sync", type=int, default=None,
                    help="1 / 0: chunk-synchronous / classic plan for the dataflow sessions "
                         "(default: the session's own choice, engine.RoutingNet)")
    ap.add_argument("--fslots", type=int, default=256,
                    help="EnKF: lanes of the forecast plan (after the last analysis)")
    ap.add_argument("--ftile", type=int, default=64,
                    help="EnKF: launch length (ticks) of the forecast plan")
    ap.add_argument("--chain", type=int, default=0,
                    help="node slots per lane (plan.hpp lane chains); 0 = per workload")
    ap.add_argument("--conus", action="store_true",
                    help="BASELINE configs[4]: CONUS NWM-scale synthetic network (2.7M reaches, "
                         "4000 outlets, deepest path ~7000 reaches); --members per GPU (default "
                         "16: the 128-member ensemble over 8 GPUs, one 16-member shard per rank)")
    ap.add_argument("--huc8", action="store_true",
                    help="BASELINE configs[0]: one HUC-8 sub-basin (1000 reaches, one outlet, "
                         "deepest path ~100 reaches), deterministic")
    ap.add_argument("--mode", default="auto", choices=["auto", "launches", "dataflow"],
                    help="execution path (mcroute.h mc_set_mode)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-api", action="store_true", help="skip the Muskingum.simulate timing")
    ap.add_argument("--timing-runs", type=int, default=3)
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1: torch.distributed backend (nccl = RCCL over xGMI, one GPU per "
                         "rank; gloo: host-staged collectives, lets several ranks share one GPU "
                         "in the tests)")
    ap.add_argument("--emulate-shards", type=int, default=0,
                    help="--enkf at N = 1: also run the configs[3] horizon as this many member "
                         "shards on the one GPU (ensemble.emulated_analysis, the stage program "
                         "of the N-rank run) and report each shard's device time per horizon "
                         "and the projected N-GPU speed-up")
    ap.add_argument("--xgmi-gbs", type=float, default=50.0,
                    help="--emulate-shards: modelled per-peer, per-direction xGMI rate (GB/s) "
                         "for the collectives the emulation does as device copies")
    args = ap.parse_args(argv)
    if world is None:
        world = int(os.environ.get("WORLD_SIZE", "1"))
    return apply_presets(args, world)


def apply_presets(args, world=1):
    if args.huc8:
        args.n, args.basins, args.depth = 1000, 1, 100
        if args.members is None:
            args.members = 1                       # configs[0] is deterministic
    if args.conus:
        args.n, args.basins, args.depth = 2_700_000, 4000, 7000
        if args.members is None:
            args.members = 16
    if args.members is None:
        if world > 1 and not args.det:
            args.members, args.enkf = 256, True      # BASELINE configs[3], members sharded
        else:
            args.members = 1
    return args


def launch_plan(gpus, env):
    """("spawn", N): start N ranks of this script under torch.distributed.run as a child;
    ("run", world): this process is one of `world` ranks (or the only one).  A launcher whose
    world size differs from --gpus is an error (it would silently measure another GPU count)."""
    world = int(env.get("WORLD_SIZE", "1"))
    launched = "RANK" in env or "LOCAL_RANK" in env
    if gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if not launched and world == 1:
        return ("spawn", gpus) if gpus > 1 else ("run", 1)
    if gpus != world:
        raise SystemExit(f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
    return ("run", world)


def spawn_ranks(n):
    """One rank per GPU: torch.distributed.run on this script as a child process (never exec:
    on this pool a process that touched the GPU must not be replaced); its stdout is ours."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def measured_traffic(info, n, T, E=1):
    """HBM bytes per launch of the routing kernel measured with rocprofv3 PMC counters for this
    exact workload AND this build (scripts/hbm_traffic.py -> profiles/*_hbm_traffic*.json,
    stamped with _build.source_hash()), newest first.  A profile of another build is refused."""
    import glob

    from tx_fast_hydrology_amd._build import source_hash
    want = {"slots": info["slots"], "tile": info["tile"], "n": n, "T": T}
    if E > 1:
        want["E"] = E
    h = source_hash()
    stale = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_hbm_traffic*.json")),
                    reverse=True):
        try:
            rec = json.load(open(f))
        except (OSError, ValueError):
            continue
        if rec.get("workload") != want:
            continue
        if "launches_per_horizon" not in rec:
            # written before hbm_traffic.py selected the bench horizons only (round 4's det
            # profile averaged the drop-in API's launches in): never quoted
            continue
        if rec.get("source_hash") != h:
            stale = stale or os.path.relpath(f, ROOT)
            continue
        rec["file"] = os.path.relpath(f, ROOT)
        return rec, None
    return None, (f"no PMC profile of this build (source hash {h})" +
                  (f"; {stale} is of another build" if stale else ""))


def build_workload(args, rank=0, world=1):
    """Texas-scale synthetic network, coefficients, state and forcing, loaded into a RoutingNet.
    Returns (net, w): w holds the host arrays (w.x = step times of one horizon)."""
    from types import SimpleNamespace

    from tx_fast_hydrology_amd import engine, synthetic

    if getattr(args, "huc8", False):
        end = synthetic.huc8(seed=0, n=args.n, max_depth=args.depth)
    else:
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
    K_arr, X_arr = K, X
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
    # (0: the session's default, engine._det_shape -- one compute wave of single-slot lanes for
    # a small network such as HUC-8)
    slots = args.slots or (0 if E == 1 else 192 if enkf is not None else 256)
    # ensemble forecasts (multi-launch path): 64-tick launches amortise the per-launch slot
    # loads (Texas ens64 14.1 -> 13.1 ms per horizon); the dataflow workloads at a 16-tick
    # cross-cluster slack (two chunks, the minimum): Texas det 0.605 -> 0.594 ms
    tile = args.tile or (64 if E > 1 and enkf is None else 16)
    # the deterministic horizon runs a chunk-synchronous plan (the session's default); the EnKF
    # member steps keep the classic plan (same box: 397 vs 388 us per EnKF32 member step -- the
    # member tick waits on its staged cells, not on the barrier)
    sync = getattr(args, "sync", None)
    net = engine.RoutingNet(end, indeg, heads, slots=slots, tile=tile, members=E,
                            chain=args.chain, sync=sync)
    net.set_mode(getattr(args, "mode", "auto"))
    net.set_coeffs(alpha, beta, chi, gamma)
    net.set_state(o0, i0)
    net.load_forcing(xp, fp)
    if enkf is not None and not args.one_plan:
        # the forecast after the last analysis runs on its own plan (256 lanes, 64-tick
        # launches: the multi-launch ensemble shape), the state handed over on the device
        fnet = engine.RoutingNet(end, indeg, heads, slots=getattr(args, "fslots", 256),
                                 tile=getattr(args, "ftile", 64), members=E)
        # (the one-step mode "dataflow" selects the analysis plan's member-step path;
        # the forecast is a multi-step ensemble horizon: launches)
        fnet.set_mode("launches" if getattr(args, "mode", "auto") == "launches" else "auto")
        fnet.set_coeffs(alpha, beta, chi, gamma)
        fnet.load_forcing(xp, fp)
        enkf.fnet = fnet
    w = SimpleNamespace(n=n, start=start, end=end, indeg=indeg, alpha=alpha, beta=beta, chi=chi,
                        gamma=gamma, o0=o0, i0=i0, x=x, xp=xp, fp=fp, rows=rows, dt=dt, E=E,
                        enkf=enkf, K=K_arr, X=X_arr, xp_ns=xp_ns)
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
    if E == 1 and wl.n <= 10_000:
        return (f"huc8-det (BASELINE configs[0]): one synthetic HUC-8 sub-basin ({wl.n} "
                f"reaches, one outlet), deterministic, 24 h @ 300 s")
    if E == 1:
        return ("texas-det (BASELINE configs[1]): full-Texas synthetic network, deterministic, "
                "24 h @ 300 s")
    return (f"texas-ens{E} (BASELINE configs[2]): full-Texas synthetic network, {E}-member "
            f"ensemble forecast, 24 h @ 300 s")


def compulsory_bytes(n, E, T, rows):
    """Bytes one horizon must move at least (SURVEY §8d data, counted once): every step's
    outflow written (the inflows are recomputed from them, kernels.hpp), the forcing rows and
    the four coefficient arrays read, the state {o, i} read at the start and written at the
    end.  (The reference additionally writes every step's inflows: +T n E 8.)"""
    return 8.0 * n * (E * T + E * rows + 4 + 4 * E)


def run_horizon(net, wl):
    """One bench step: a 24-h horizon of the workload, with the EnKF cycle where configured --
    one-step member runs each followed by the (member-sharded) analysis while observations
    exist (da.py:56-61), then the forecast on its own plan with the state handed over on the
    device (tests/test_gpu_enkf_horizon.py checks exactly this sequence)."""
    x = wl.x
    if wl.enkf is None:
        net.run(x)
        return
    from tx_fast_hydrology_amd import ensemble
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


def run_emulated_horizon(nets, wls, stream, stage_ms=None, rec=None):
    """The configs[3] horizon as N = len(nets) member shards on one GPU (all sessions on the
    torch stream `stream`): each shard's one-step member run, the analysis through
    ensemble.emulated_analysis (the N-rank stage program, collectives as device copies), then
    each shard's forecast with the device hand-over.  rec(r, part, fn) wraps each shard's parts
    (timing); stage_ms collects the analysis stages' device times."""
    import torch

    from tx_fast_hydrology_amd import ensemble
    rec = rec or (lambda r, part, fn: fn())
    N = len(nets)
    ek0 = wls[0].enkf
    x = wls[0].x
    for k in range(ek0.n_an):
        for r in range(N):
            rec(r, "member_steps", lambda r=r: nets[r].run(x[k:k + 1]))
        with torch.cuda.stream(stream):
            ensemble.emulated_analysis(nets, ek0.gauges, [wls[r].enkf.Y[k] for r in range(N)],
                                       ek0.R, stage_ms=stage_ms)
    for r in range(N):
        f = wls[r].enkf.fnet

        def fc(r=r, f=f):
            f.copy_state_from(nets[r])
            f.run(x[ek0.n_an:])
            nets[r].copy_state_from(f)
        rec(r, "forecast", fc)


def enkf_restatement(wl, orc, o, i, fp, Y, cores, x_out=None):
    """Host restatement of the EnKF horizon (test infrastructure and the CPU baseline): the
    members through the C member loop (OpenMP), at each analysis step the observation-space
    analysis of da.py:112-126 with the ensemble sample covariance, A HA^T (HA HA^T / (E - 1) +
    R)^-1 (Y - HX) / (E - 1), applied by the C _apply_gain (nutils.py:116-134), then the forecast.
    Y: per analysis step [m][E].  Returns the final (o, i) [n][E] and, for steps listed in x_out,
    the forecast outputs {t: (o_t, i_t)}."""
    ek = wl.enkf
    E = o.shape[1]
    g = ek.gauges
    coef = (wl.alpha, wl.beta, wl.chi, wl.gamma)
    heads = wl.start[wl.indeg == 0]
    x = wl.x
    o, i = np.ascontiguousarray(o), np.ascontiguousarray(i)
    for k in range(ek.n_an):
        o, i = orc.simulate_members(wl.start, wl.end, wl.indeg, *coef, o, i, x[k:k + 1],
                                    wl.xp, fp, threads=cores)
        A = o - o.mean(1, keepdims=True)
        HA = A[g]
        W = np.linalg.solve(HA @ HA.T / (E - 1) + ek.R, Y[k] - o[g])
        G = A @ (HA.T @ W) / (E - 1)
        for e in range(E):
            ig, og = orc.apply_gain(heads, wl.end, np.ascontiguousarray(G[:, e]), wl.indeg)
            o[:, e] += og
            i[:, e] += ig
        o, i = np.ascontiguousarray(o), np.ascontiguousarray(i)
    outs = {}
    t0 = ek.n_an
    targets = sorted(set(x_out or []))
    for t1 in targets + [x.size]:
        if t1 > t0:
            o, i = orc.simulate_members(wl.start, wl.end, wl.indeg, *coef, o, i, x[t0:t1],
                                        wl.xp, fp, threads=cores)
            t0 = t1
        if t1 in targets:
            outs[t1 - 1] = (o.copy(), i.copy())
    return o, i, outs


def cpu_enkf_baseline(args, wl, orc):
    """Host baseline of the EnKF horizon on a bounded sample: min(E, cores) members through the C
    member loop (OpenMP) with a NumPy ensemble analysis at the analysis steps."""
    cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    ek = wl.enkf
    ms = min(wl.E, cores)
    fp = np.ascontiguousarray(wl.fp[:, :, :ms])
    Y = [y[:, :ms] for y in ek.Y]
    reps, t = 0, 0.0
    while t < args.cpu_seconds or reps == 0:
        c0 = time.perf_counter()
        enkf_restatement(wl, orc, wl.o0[:, :ms], wl.i0[:, :ms], fp, Y, cores)
        t += time.perf_counter() - c0
        reps += 1
    return {"value": float(wl.n) * ms * args.T * reps / t, "unit": "reach·member·timesteps/s",
            "cores": cores, "kind": "port",
            "sample": f"{reps} x full 24 h EnKF horizon (T={args.T}, {ek.n_an} analysis steps) "
                      f"of {ms} members on the same {wl.n}-reach network: C member loop "
                      f"(OpenMP) + NumPy ensemble analysis + C _apply_gain, {t:.1f} s"}


def cpu_baseline(args, wl, orc, E, x):
    n = wl.n
    if wl.enkf is not None:
        return cpu_enkf_baseline(args, wl, orc)
    if E > 1:
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
        return {"value": float(n) * ms * steps_done / t_cpu,
                "unit": "reach·member·timesteps/s", "cores": cores, "kind": "port",
                "sample": f"{steps_done} timesteps (12-step chunks of the 24 h horizon, "
                          f"T={args.T}) of {ms} members on the same {n}-reach network, C member "
                          f"loop (-O3 -ffp-contract=off, OpenMP over members), {t_cpu:.1f} s"}
    o_s, i_s = wl.o0.copy(), wl.i0.copy()
    reps, t_cpu = 0, 0.0
    while t_cpu < args.cpu_seconds or reps == 0:
        c0 = time.perf_counter()
        orc.simulate(wl.start, wl.end, wl.indeg, wl.alpha, wl.beta, wl.chi, wl.gamma, o_s,
                     i_s, x, wl.xp, wl.fp, keep_outputs=False)
        t_cpu += time.perf_counter() - c0
        reps += 1
    return {"value": float(n) * args.T * reps / t_cpu, "unit": "reach·timesteps/s",
            "cores": 1, "kind": "port",
            "sample": f"{reps} x full 24 h horizon (T={args.T}) on the same {n}-reach "
                      f"network, serial C (-O3 -ffp-contract=off), {t_cpu:.1f} s"}


def reach_order_timing(net, n, T, reps=5):
    """Device time to produce both series of the last horizon in the reference's layout
    (outflows and inflows, reach order, step-major [T][n]: mc_gather_outputs into device
    buffers), HIP events on the session stream, and the bytes that must move: the outflow rows
    read once, both series written."""
    import torch
    stream = torch.cuda.Stream()
    net.set_stream(stream.cuda_stream)
    o = torch.empty((T, n), dtype=torch.float64, device="cuda")
    i = torch.empty((T, n), dtype=torch.float64, device="cuda")
    with torch.cuda.stream(stream):
        net.gather_outputs(0, T, o, i)                 # warm-up
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(stream)
        for _ in range(reps):
            net.gather_outputs(0, T, o, i)
        b.record(stream)
    b.synchronize()
    net.set_stream(None)
    ms = a.elapsed_time(b) / reps
    moved = 3.0 * 8 * n * T
    return {"ms": round(ms, 4), "bytes": moved,
            "gbs": round(moved / (ms * 1e-3) / 1e9, 1),
            "frac": round(moved / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 3),
            "counts": "outflow rows read once + outflow and inflow series written (f64)"}


def api_timing(wl, runs=2):
    """ms per horizon of the drop-in API: Muskingum.simulate (tx_fast_hydrology interface,
    muskingum.py:499-536) over the same network, forcing frame and 24-h horizon, iterating
    every step (each yields fresh writable host arrays of that step's outflows and inflows)."""
    import pandas as pd

    from tx_fast_hydrology_amd.muskingum import Muskingum
    n = wl.n
    reach_ids = [f"r{j}" for j in range(n)]
    start = pd.Timestamp(int(wl.xp_ns[0]), tz="UTC")
    model = Muskingum({"name": "texas", "datetime": start,
                       "timedelta": pd.to_timedelta(wl.dt, unit="s"), "reach_ids": reach_ids,
                       "startnodes": wl.start.astype(np.int64),
                       "endnodes": wl.end.astype(np.int64), "K": wl.K.astype(np.float64),
                       "X": wl.X.astype(np.float64), "o_t": wl.o0.astype(np.float64)})
    idx = pd.DatetimeIndex(pd.to_datetime(wl.xp_ns, utc=True))
    df = pd.DataFrame(wl.fp, index=idx, columns=reach_ids)
    end_time = start + pd.to_timedelta(wl.dt * wl.x.size, unit="s")
    times = []
    for r in range(runs + 1):                  # the first run builds the device session
        model.datetime = start
        t0 = time.perf_counter()
        steps = 0
        for _ in model.simulate(df, end_time=end_time, o_t_init=wl.o0):
            steps += 1
        if r:
            times.append(time.perf_counter() - t0)
    assert steps == wl.x.size, steps
    model.close()
    return 1e3 * min(times)


def emulated_shards(args, t1_ms):
    """configs[3] as N member shards on ONE GPU: shard r is exactly rank r of the N-rank run (its
    workload from build_workload(args, r, N): members r*E/N .., its own observation draws), the
    member steps and forecast of each shard on one stream, the analyses through
    ensemble.emulated_analysis (every mc_ens_* stage with nranks = N, the collectives as device
    copies).  Reports each shard's device time per horizon (HIP events on that stream, the
    collectives' copies excluded), the bytes each rank would move in the collectives, their time
    at a modelled xGMI rate, and the projected N-GPU speed-up T(1 GPU) / T(rank)."""
    import torch

    from tx_fast_hydrology_amd import ensemble
    N = args.emulate_shards
    if args.members % N:
        raise SystemExit("--emulate-shards must divide --members")
    built = [build_workload(args, r, N) for r in range(N)]
    nets = [b[0] for b in built]
    wls = [b[1] for b in built]
    ek0 = wls[0].enkf
    x = wls[0].x
    stream = torch.cuda.Stream()
    sessions = nets + [w.enkf.fnet for w in wls if getattr(w.enkf, "fnet", None) is not None]
    for s_ in sessions:
        s_.set_stream(stream.cuda_stream)
    ev = lambda: torch.cuda.Event(enable_timing=True)   # noqa: E731
    spans = []                                          # (shard, part, start, end)

    def rec(r, part, fn):
        a, b = ev(), ev()
        a.record(stream)
        fn()
        b.record(stream)
        spans.append((r, part, a, b))

    def horizon(stage_ms):
        run_emulated_horizon(nets, wls, stream, stage_ms, rec)

    with torch.cuda.stream(stream):
        horizon({})                                     # warm-up (plans, buffers)
        stream.synchronize()
        spans.clear()
        reps = max(1, min(args.steps, 3))
        stage_ms = {}
        t0 = time.perf_counter()
        for _ in range(reps):
            horizon(stage_ms)
        stream.synchronize()
        wall_ms = (time.perf_counter() - t0) * 1e3 / reps
    per = [dict() for _ in range(N)]
    for r, part, a, b in spans:
        per[r][part] = per[r].get(part, 0.0) + a.elapsed_time(b) / reps
    for name, vals in stage_ms.items():
        if name.startswith("exchange"):
            continue
        for r in range(N):
            per[r]["analysis: " + name] = per[r].get("analysis: " + name, 0.0) + vals[r] / reps
    exch_copy_ms = sum(stage_ms.get("exchange (device copies)", [0.0])) / reps
    shard_ms = [sum(p.values()) for p in per]
    # bytes one rank sends per analysis (mc_ens_* layout): all-gather of HX and D (E x m each),
    # the member -> slice all-to-all and the increments back (E x S each per peer)
    E, m = wls[0].E, ek0.m
    S = nets[0].slice_size(N)
    ag = 2 * E * m * 8 * (N - 1)                        # each rank's blocks to N - 1 peers
    a2a = 2 * E * S * 8 * (N - 1)                       # E x S doubles to each peer, twice
    peers = min(N - 1, 7)                               # xGMI: one link per peer (7 per GPU)
    lat_us = 25.0                                       # per collective (RCCL small-message)
    model_ms = ek0.n_an * ((ag + a2a) / (peers * args.xgmi_gbs * 1e9) * 1e3 +
                           3 * lat_us * 1e-3)
    t_rank = max(shard_ms) + model_ms
    # the member -> slice all-to-all (half of a2a) runs on a side stream under the weights in
    # both drivers (ensemble.distributed_analysis, mc_ens_analysis_dist): with that overlap the
    # rank saves min(weights, that all-to-all) per analysis
    r_w = max(range(N), key=lambda r: shard_ms[r])
    w_ms = per[r_w].get("analysis: weights", 0.0)
    a2a_half_ms = ek0.n_an * (a2a / 2) / (peers * args.xgmi_gbs * 1e9) * 1e3
    t_rank_ov = t_rank - min(w_ms, a2a_half_ms)
    for s_ in sessions:
        s_.close()
    return {"shards": N, "members_per_shard": E, "t1_ms_per_horizon": round(t1_ms, 3),
            "shard_device_ms_per_horizon": [round(v, 3) for v in shard_ms],
            "shard_breakdown_ms": {k: [round(p.get(k, 0.0), 3) for p in per]
                                   for k in sorted(per[0])},
            "emulation_wall_ms_per_horizon": round(wall_ms, 3),
            "exchange_device_copies_ms_per_horizon": round(exch_copy_ms, 3),
            "collective_bytes_per_rank_per_analysis": {"all_gather": ag, "all_to_all": a2a},
            "collective_model": {"xgmi_gbs_per_peer": args.xgmi_gbs, "peers": peers,
                                 "latency_us_per_collective": lat_us,
                                 "ms_per_horizon": round(model_ms, 3),
                                 "note": "not measured (one GPU): bytes / (peers x rate) + 3 "
                                         "collective latencies per analysis, no overlap"},
            "projected_rank_ms_per_horizon": round(t_rank, 3),
            "projected_speedup": round(t1_ms / t_rank, 3),
            "projected_with_overlap": {
                "rank_ms_per_horizon": round(t_rank_ov, 3),
                "speedup": round(t1_ms / t_rank_ov, 3),
                "note": "the member -> slice all-to-all under the weights, as both drivers "
                        "issue it (side stream); still a model, not a measurement"}}


def main():
    args = parse()
    what, world = launch_plan(args.gpus, os.environ)
    if what == "spawn":
        sys.exit(spawn_ranks(world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    dist = None
    if world > 1:
        import datetime as _dt

        import torch.distributed as dist
        # gloo (tests): several ranks may share one GPU
        ndev = max(torch.cuda.device_count(), 1)
        torch.cuda.set_device(local if args.backend == "nccl" else local % ndev)
        dist.init_process_group(args.backend, timeout=_dt.timedelta(seconds=600))
    else:
        torch.cuda.set_device(0)

    from oracle import oracle as orc  # noqa: F401  (cpu_baseline leg only)
    from tx_fast_hydrology_amd import engine, ensemble

    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(v):
        if dist is None:
            return v
        tt = torch.tensor([v], dtype=torch.float64,
                          device="cuda" if args.backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    # ---- workload -------------------------------------------------------------------------
    t_setup = time.time()
    net, wl = build_workload(args, rank, world)
    n, x = wl.n, wl.x

    def horizon():
        """One bench step: a 24-h horizon (with the analysis steps of the EnKF workload)."""
        run_horizon(net, wl)
    info = net.info
    setup_s = time.time() - t_setup

    # ---- warmup + timed region -------------------------------------------------------------
    for _ in range(args.warmup):
        horizon()
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        horizon()
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
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
    per_net = []
    for nt in nets:
        nt.synchronize()
        per_net.append(nt.timing())
        nt.set_timing(False)
    T_k = args.T                       # timesteps the roofline kernel routes per horizon
    tm = per_net[-1] if len(nets) > 1 else per_net[0]
    members_steps = None
    if len(nets) > 1:
        # EnKF: the dominant kernel is the forecast (fnet, T - n_an of the T steps, most of the
        # device time); the member steps between analyses are reported beside it
        T_k = args.T - wl.enkf.n_an
        ms_ = per_net[0]
        members_steps = {"kernel": "wavefront_flow (member dataflow, one step per launch)",
                         "launches_per_step": ms_["launches"] / args.timing_runs,
                         "kernel_ms_per_step": round(ms_["kernel_ms"] / args.timing_runs, 4)}
    launches = max(tm["launches"], 1)
    launch_ms = tm["kernel_ms"] / launches
    path = (nets[-1] if len(nets) > 1 else net).mode()[1]
    kernel = "wavefront_flow" if path == "dataflow" else "wavefront_det"
    if path == "launches" and E >= 2 and E % 2 == 0 and \
            (len(nets) > 1 or not getattr(args, "sync", None)) and \
            os.environ.get("MCR_MEMBERS_MB", "2") != "1":
        kernel = "wavefront_members"      # two members per instance (capi.cpp run: memb2)
    # 72 B per reach·timestep deterministic, 40 + 32/E per reach·member·timestep
    per_unit = BYTES_PER_UNIT if E == 1 else 40.0 + 32.0 / E
    bytes_per_launch = per_unit * n * E * T_k * args.timing_runs / launches
    achieved = bytes_per_launch / (launch_ms * 1e-3) / 1e9
    launches_per_step = tm["launches"] / args.timing_runs
    comp = compulsory_bytes(n, E, T_k, wl.rows) / launches_per_step
    roofline = {"bound": "latency", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 6), "traffic": None,
                "algorithmic_bytes_per_unit": per_unit, "kernel": kernel,
                "launches_per_step": launches_per_step, "avg_launch_us": round(launch_ms * 1e3, 3),
                "kernel_ms_per_step": round(tm["kernel_ms"] / args.timing_runs, 4)}
    if members_steps is not None:
        roofline["timesteps_per_step"] = T_k
        roofline["member_steps"] = members_steps
    # the routing recurrence keeps coefficients and state in registers / LDS: it is bound by its
    # dependency chain (schedule ticks x per-tick latency), not by DRAM bandwidth
    if wl.enkf is None and E == 1 and path == "dataflow" and \
            (info["slots"], info["chain"]) in ((192, 2), (384, 2), (64, 1)):
        ticks = info["gmax"] + args.T
        ns_tick = engine.probe_tick_floor(info["slots"], info["chain"], 8192)
        floor_ms = ticks * ns_tick * 1e-6
        roofline["latency"] = {
            "schedule_ticks": ticks, "ns_per_tick": round(launch_ms * 1e6 / ticks, 2),
            "floor_ns_per_tick": round(ns_tick, 2), "floor_ms": round(floor_ms, 4),
            "frac": round(floor_ms / launch_ms, 4),
            "floor": "mc_probe_tick_floor: the bare tick chain of this kernel shape (LDS inputs, "
                     "chained updates, LDS outputs, barrier; %s per CU, no memory traffic), "
                     "measured now on this device"
                     % ("2 workgroups" if info["slots"] == 192 else "1 workgroup")}
    elif E > 1:
        # an ensemble horizon is throughput-bound: its critical path (the schedule's ticks at the
        # bare tick latency) is a small fraction of it, and the bound it is measured against is
        # the HBM roofline of the bytes it must move (compulsory, below)
        ticks = nets[-1].info["gmax"] + T_k
        ns_tick = engine.probe_tick_floor(192, 2, 8192)
        floor_ms = ticks * ns_tick * 1e-6
        roofline["bound"] = "hbm"
        roofline["latency"] = {
            "schedule_ticks": ticks, "floor_ns_per_tick": round(ns_tick, 2),
            "floor_ms": round(floor_ms, 4), "frac": round(floor_ms / (launch_ms *
                                                                       launches_per_step), 4),
            "floor": "critical path: schedule ticks x the bare tick latency of the 192-lane "
                     "dataflow tick (mc_probe_tick_floor), a lower bound for any ensemble path"}
    else:
        roofline["latency"] = None
    roofline["compulsory"] = {
        "bytes_per_launch": comp, "gbs": round(comp / (launch_ms * 1e-3) / 1e9, 3),
        "frac": round(comp / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        "counts": "outflows written + forcing, coefficients, state read + state written"}
    if wl.enkf is None:
        traffic, note = measured_traffic(info, n, args.T, E)
    else:
        traffic, note = None, "EnKF horizon: several kernels, no single-kernel PMC profile"
    if traffic:
        tb = traffic["traffic_bytes_per_launch"]
        roofline["traffic"] = tb
        roofline["dram"] = {"source": traffic["file"], "source_hash": traffic["source_hash"],
                            "bytes_per_launch": tb, "read_bytes": traffic["read_bytes"],
                            "write_bytes": traffic["write_bytes"],
                            "gbs": round(tb / (launch_ms * 1e-3) / 1e9, 3),
                            "frac": round(tb / (launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                            "over_compulsory": round(tb / comp, 3)}
    else:
        roofline["dram"] = {"source": None, "note": note}

    # ---- CPU baseline (transliteration of the reference loop, rank 0 at any N) --------------
    # north_star: "timed on the node's own host cores in the same run"; at N > 1 the other ranks
    # wait for rank 0 at the next barrier
    cpu = None
    if rank == 0 and not args.no_cpu:
        cpu = cpu_baseline(args, wl, orc, E, x)
    if world > 1:
        barrier()

    # ---- configs[3] as emulated member shards on this one GPU ---------------------------------
    shards = None
    if world == 1 and wl.enkf is not None and args.emulate_shards > 1:
        for nt in nets:
            nt.close()
        shards = emulated_shards(args, elapsed / args.steps * 1e3)

    # ---- the reference layout on the device (det, N = 1): both [T][n] series in reach order,
    # what _ax_bu returns every step (nutils.py:64-89), from the last horizon's outputs --------
    reach_order = None
    if world == 1 and E == 1 and wl.enkf is None:
        reach_order = reach_order_timing(net, n, args.T)

    # ---- the drop-in API over the same horizon (det, N = 1) ---------------------------------
    api_ms = None
    if world == 1 and E == 1 and wl.enkf is None and not args.no_api and wl.n < 1_000_000:
        api_ms = api_timing(wl)

    # ---- N > 1 EnKF headline: the replicated deterministic run as well ----------------------
    det_rep = None
    if world > 1 and wl.enkf is not None:
        for nt in nets:
            nt.close()
        dargs = copy.copy(args)
        dargs.members, dargs.enkf, dargs.slots, dargs.tile = 1, False, 0, 0
        dnet, dwl = build_workload(dargs, rank, world)
        for _ in range(max(args.warmup, 1)):
            dnet.run(dwl.x)
        barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            dnet.run(dwl.x)
        barrier()
        de = max_over_ranks(time.perf_counter() - t0)
        det_rep = {"value": float(dwl.n) * args.T * args.steps * world / de,
                   "unit": "reach·timesteps/s", "ms_per_horizon": de / args.steps * 1e3,
                   "scaling": "weak", "parallelism": f"replicas x{world}",
                   "workload": workload_name(dwl, 1)}
        dnet.close()

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
        if reach_order is not None:
            line["reach_order_ms"] = reach_order["ms"]
            line["reach_order"] = reach_order
        if api_ms is not None:
            line["api_ms_per_horizon"] = round(api_ms, 3)
            line["api_path"] = ("Muskingum.simulate over the same 24 h horizon, every step "
                                "iterated (host outflows and inflows of each step)")
        if det_rep is not None:
            line["det_replicas"] = det_rep
        if shards is not None:
            line["emulated_shards"] = shards
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
