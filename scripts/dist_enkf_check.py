#!/usr/bin/env python3
"""Multi-rank check of the member-sharded analysis on real devices (ensemble.py + mc_ens_*).
Launch with torch.distributed.run (the launcher never touches the GPU):
    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 scripts/dist_enkf_check.py [--backend gloo|nccl]
With one GPU and several ranks use gloo (device buffers are staged through host memory); with one
GPU per rank use nccl (RCCL).  Rank 0 also runs the whole ensemble in one session and compares."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tx-fast-hydrology_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--reaches", type=int, default=20000)
    ap.add_argument("--members", type=int, default=8, help="members per rank")
    ap.add_argument("--gauges", type=int, default=50)
    ap.add_argument("--capi", action="store_true",
                    help="run the analysis through the C ABI's own RCCL communicator "
                         "(mc_comm_* / mc_ens_analysis_dist; one GPU per rank); torch.distributed "
                         "(gloo) only hands the communicator id around and gathers the results")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from oracle import oracle as orc
    from tx_fast_hydrology_amd import engine, ensemble, synthetic

    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev)
    dist.init_process_group(args.backend)

    end = synthetic.river_network(args.reaches, 8, 300, np.random.default_rng(1))
    n = end.size
    start = np.arange(n)
    indeg = orc.compute_indegree(start, end)
    K, X_, _ = synthetic.model_arrays(n, seed=2)
    coef = orc.muskingum_coeffs(K, X_, 300.0)
    El, Et, m = args.members, args.members * world, args.gauges
    rng = np.random.default_rng(3)                               # same on every rank
    X = rng.uniform(0.5, 5, n)[:, None] * rng.lognormal(0, 0.3, (n, Et))
    I0 = rng.uniform(0, 5, (n, Et))
    s = np.sort(rng.choice(n, m, replace=False))
    R = 2e-2 * np.eye(m)
    Y = ensemble.perturbed_observations(X[s].mean(1) + 0.2, R, Et, rng)
    cols = slice(rank * El, (rank + 1) * El)

    net = engine.RoutingNet(end, indeg, start[indeg == 0], members=El)
    net.set_coeffs(*coef)
    net.set_state(np.ascontiguousarray(X[:, cols]), np.ascontiguousarray(I0[:, cols]))
    if args.capi:
        uid = [engine.Communicator.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = engine.Communicator(world, rank, uid[0])
        net.ens_analysis_dist(comm, s, np.ascontiguousarray(Y[:, cols]), R)
        net.synchronize()
    else:
        ensemble.distributed_analysis(net, s, np.ascontiguousarray(Y[:, cols]), R,
                                      device=torch.device("cuda", dev))
    o, i = net.get_state()
    ot = torch.from_numpy(np.ascontiguousarray(o))
    it = torch.from_numpy(np.ascontiguousarray(i))
    if args.backend == "nccl":
        ot, it = ot.cuda(), it.cuda()
    po = [torch.empty_like(ot) for _ in range(world)]
    pi = [torch.empty_like(it) for _ in range(world)]
    dist.all_gather(po, ot)
    dist.all_gather(pi, it)
    ok = True
    if rank == 0:
        got_o = np.concatenate([p.cpu().numpy() for p in po], axis=1)
        got_i = np.concatenate([p.cpu().numpy() for p in pi], axis=1)
        ref = engine.RoutingNet(end, indeg, start[indeg == 0], members=Et)
        ref.set_coeffs(*coef)
        ref.set_state(X, I0)
        ref.enkf_analysis(s, Y, R)
        ro, ri = ref.get_state()
        ok = np.array_equal(got_o, ro) and np.array_equal(got_i, ri)
        err = max(np.abs(got_o - ro).max(), np.abs(got_i - ri).max())
        print(f"DIST_ENKF world={world} members/rank={El} backend={args.backend} capi={args.capi} "
              f"bitexact={ok} maxabs={err:.3e} gain_scale={np.abs(ro - X).max():.3e}",
              flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
