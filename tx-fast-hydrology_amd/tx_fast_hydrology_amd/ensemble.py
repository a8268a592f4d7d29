"""Member-sharded ensemble analysis across GPUs: one process per GPU, E local members
each, torch.distributed (backend "nccl" = RCCL over xGMI) for the exchange.

The forecast needs no communication.  The analysis (mcroute.h, mc_ens_* stages) exchanges:
  * all-gather of the gauge outflows HX and innovations D (m x E per rank: ~0.1 MB),
  * all-to-all of the member states into reach slices (each rank gets ALL members of 1/N of the
    reaches) and all-to-all of the increments back: ns x E x (N-1)/N doubles each way per rank
    -- 1/N of what an all-gather of the anomalies would move.
Every rank forms the same m x m system C = HA HA^T/(Et-1) + R, W = C^-1 D and Z = HA^T W/(Et-1)
from the gathered gauge data; the slice increments G = A Z are dense f64 MFMA products.

`net` is a RoutingNet with the ens_* stage methods (or any object with the same methods, e.g. the
NumPy model in tests/).  With one rank the stages equal RoutingNet.enkf_analysis.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


_SIDE = {}      # device index -> the side stream analyses run on when the caller's is the null stream


def _world(group):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def _host_staged(t: torch.Tensor) -> bool:
    # gloo has no device collectives: stage device buffers through host memory (tests on one
    # GPU with several ranks; production uses the nccl backend on device buffers)
    return t.is_cuda and dist.get_backend() == "gloo"


def _all_gather(out: torch.Tensor, inp: torch.Tensor, group) -> None:
    if _host_staged(inp):
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


def _all_to_all(out: torch.Tensor, inp: torch.Tensor, group) -> None:
    if _host_staged(inp):
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, group=group)


def distributed_analysis(net, gauges, y_local, R, device=None, group=None,
                         staged=False) -> None:
    """Ensemble Kalman update of all ranks' members.  gauges [m] (same on every rank), y_local
    [m, E] observations of this rank's members, R [m, m].  staged=True runs the mc_ens_* stages
    even with one rank (tests)."""
    N, _ = _world(group)
    if N == 1 and not staged and hasattr(net, "enkf_analysis"):
        # one rank: the staged form's pack / unpack are identities and there is nothing to
        # exchange; the whole update is one library call (same kernels, same results)
        net.enkf_analysis(gauges, y_local, R)
        return
    E = net.E
    m = int(np.asarray(gauges).size)
    Et = E * N
    S = net.slice_size(N)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    if device.type == "cuda" and hasattr(net, "set_stream"):
        # the session's kernels and torch's collectives must be ordered on one stream, and it
        # must not be the null stream (the session maps a NULL stream to its own, unordered one)
        caller = torch.cuda.current_stream(device)
        if caller.cuda_stream == 0:
            # one side stream per device, kept: the session then stays on it from one analysis
            # to the next (set_stream synchronises only when the stream changes)
            side = _SIDE.get(device.index)
            if side is None:
                side = _SIDE[device.index] = torch.cuda.Stream(device)
            side.wait_stream(caller)
            with torch.cuda.stream(side):
                distributed_analysis(net, gauges, y_local, R, group=group, device=device,
                                     staged=staged)
            caller.wait_stream(side)
            return
        net.set_stream(caller.cuda_stream)
    f64 = dict(dtype=torch.float64, device=device)
    HX = torch.empty((E, m), **f64)
    D = torch.empty((E, m), **f64)
    net.ens_gauges(gauges, y_local, HX, D)
    if N > 1:
        HXall = torch.empty((Et, m), **f64)
        Dall = torch.empty((Et, m), **f64)
        _all_gather(HXall, HX, group)
        _all_gather(Dall, D, group)
    else:
        HXall, Dall = HX, D
    send = torch.empty(N * E * S, **f64)
    net.ens_pack(N, send)
    if N > 1:
        Xs = torch.empty_like(send)
        _all_to_all(Xs, send, group)
    else:
        Xs = send
    Gs = torch.empty(Et * S, **f64)
    net.ens_slice_update(N, m, Xs, HXall, Dall, R, Gs)
    if N > 1:
        Grecv = torch.empty_like(Gs)
        _all_to_all(Grecv, Gs, group)
    else:
        Grecv = Gs
    net.ens_unpack_apply(N, Grecv)


def perturbed_observations(y, R, members, rng) -> np.ndarray:
    """y [m] -> y + eps_e, eps_e ~ N(0, R) per member: [m, members]."""
    L = np.linalg.cholesky(np.asarray(R, dtype=float))
    return np.asarray(y, float)[:, None] + L @ rng.standard_normal((len(y), members))
