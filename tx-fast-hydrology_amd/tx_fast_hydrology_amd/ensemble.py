"""Member-sharded ensemble analysis across GPUs: one process per GPU, E local members
each, torch.distributed (backend "nccl" = RCCL over xGMI) for the exchange.

The forecast needs no communication.  The analysis (mcroute.h, mc_ens_* stages) exchanges:
  * all-gather of the gauge outflows HX and innovations D (m x E per rank: ~0.1 MB),
  * all-to-all of the member states into reach slices (each rank gets ALL members of 1/N of the
    reaches) and all-to-all of the increments back: ns x E x (N-1)/N doubles each way per rank
    -- 1/N of what an all-gather of the anomalies would move.
Every rank forms the same analysis weights Z (Et x Et, from the gathered gauge data only) while
its member -> slice all-to-all is in flight, then the slice increments G = A Z (dense f64 MFMA).

One analysis is ONE per-rank program (`_program`, a generator that yields its collectives), run
by two drivers:
  * `distributed_analysis`: this rank's program, collectives on torch.distributed;
  * `emulated_analysis`: the programs of N member shards in ONE process, stepped in lockstep, the
    collectives as device copies -- the same stage calls with nranks = N, exactly as N GPUs would
    make them, on one GPU (the configs[3] 8-shard layout is testable and measurable on a 1-GPU box).

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


def _all_gather(out: torch.Tensor, inp: torch.Tensor, group, async_op=False):
    if _host_staged(inp):
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
        return None
    return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)


def _all_to_all(out: torch.Tensor, inp: torch.Tensor, group, async_op=False):
    if _host_staged(inp):
        o = out.cpu()
        dist.all_to_all_single(o, inp.cpu(), group=group)
        out.copy_(o)
        return None
    return dist.all_to_all_single(out, inp, group=group, async_op=async_op)


# ---- the per-rank program ---------------------------------------------------------------------
# It yields ("exchange", ops, wait) with ops a list of ("all_gather" | "all_to_all", out, inp):
# the driver starts the collectives in order and, with wait, makes the stream wait for them before
# it resumes the program; without wait it sends back a token the program later yields as
# ("wait", token).  ("stage", name) marks the start of a compute stage (timing in the emulator).

def _program(net, gauges, y_local, R, N, device):
    E = net.E
    m = int(np.asarray(gauges).size)
    Et = E * N
    S = net.slice_size(N)
    f64 = dict(dtype=torch.float64, device=device)
    split = hasattr(net, "ens_weights") and hasattr(net, "ens_increments")
    yield ("stage", "gauges+pack")
    HX = torch.empty((E, m), **f64)
    D = torch.empty((E, m), **f64)
    net.ens_gauges(gauges, y_local, HX, D)
    send = torch.empty(N * E * S, **f64)
    net.ens_pack(N, send)
    if N > 1:
        HXall = torch.empty((Et, m), **f64)
        Dall = torch.empty((Et, m), **f64)
        Xs = torch.empty_like(send)
        yield ("exchange", [("all_gather", HXall, HX), ("all_gather", Dall, D)], True)
    else:
        HXall, Dall, Xs = HX, D, send
    Gs = torch.empty(Et * S, **f64)
    if split:
        # the weights need only the gauge data: formed while the slices travel
        pending = None
        if N > 1:
            pending = yield ("exchange", [("all_to_all", Xs, send)], False)
        yield ("stage", "weights")
        net.ens_weights(N, m, HXall, Dall, R)
        if pending is not None:
            yield ("wait", pending)
        yield ("stage", "increments")
        net.ens_increments(N, Xs, Gs)
    else:
        if N > 1:
            yield ("exchange", [("all_to_all", Xs, send)], True)
        yield ("stage", "slice_update")
        net.ens_slice_update(N, m, Xs, HXall, Dall, R, Gs)
    if N > 1:
        Grecv = torch.empty_like(Gs)
        yield ("exchange", [("all_to_all", Grecv, Gs)], True)
    else:
        Grecv = Gs
    yield ("stage", "unpack_apply")
    net.ens_unpack_apply(N, Grecv)


def _on_side_stream(device, fn):
    """Run fn() on a kept side stream of `device`, ordered after and before the caller's stream
    (the session must not run on the null stream: it maps a NULL stream to its own, unordered
    one).  Returns fn's result."""
    caller = torch.cuda.current_stream(device)
    side = _SIDE.get(device.index)
    if side is None:
        # one side stream per device, kept: sessions then stay on it from one analysis to the
        # next (set_stream synchronises only when the stream changes)
        side = _SIDE[device.index] = torch.cuda.Stream(device)
    side.wait_stream(caller)
    with torch.cuda.stream(side):
        r = fn()
    caller.wait_stream(side)
    return r


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
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    if device.type == "cuda" and hasattr(net, "set_stream"):
        # the session's kernels and torch's collectives must be ordered on one stream
        caller = torch.cuda.current_stream(device)
        if caller.cuda_stream == 0:
            _on_side_stream(device, lambda: distributed_analysis(
                net, gauges, y_local, R, group=group, device=device, staged=staged))
            return
        net.set_stream(caller.cuda_stream)
    prog = _program(net, gauges, y_local, R, N, device)
    reply = None
    try:
        while True:
            req = prog.send(reply)
            reply = None
            if req[0] == "exchange":
                _, ops, wait = req
                works = []
                for kind, out, inp in ops:
                    f = _all_gather if kind == "all_gather" else _all_to_all
                    works.append(f(out, inp, group, async_op=not wait))
                if not wait:
                    reply = works
            elif req[0] == "wait":
                for w in req[1]:
                    if w is not None:
                        w.wait()   # the current stream waits for the collective (no host wait)
    except StopIteration:
        pass


def emulated_analysis(nets, gauges, y_parts, R, device=None, stage_ms=None) -> None:
    """The member-sharded analysis of N = len(nets) shards in one process: shard r (session
    nets[r], E local members each, rank-major member blocks) runs exactly the stage calls rank r
    of `distributed_analysis` makes -- nranks = N in every mc_ens_* call -- with the all-gathers
    and all-to-alls done as device copies between the sessions' buffers.  All sessions must be
    on `device` (one GPU).  stage_ms: optional dict that receives, per stage name, the list of
    the N shards' device times in ms (HIP events; exchanges under "exchange")."""
    N = len(nets)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    stream = None
    if device.type == "cuda":
        if torch.cuda.current_stream(device).cuda_stream == 0:
            _on_side_stream(device, lambda: emulated_analysis(nets, gauges, y_parts, R, device,
                                                              stage_ms))
            return
        stream = torch.cuda.current_stream(device)
        for net in nets:
            if hasattr(net, "set_stream"):
                net.set_stream(stream.cuda_stream)
    progs = [_program(nets[r], gauges, y_parts[r], R, N, device) for r in range(N)]
    timing = stage_ms is not None and stream is not None
    spans = []                               # (stage name, shard, start event, end event)

    def event():
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream)
        return ev

    replies = [None] * N
    while True:
        reqs = []
        for r in range(N):
            # run shard r up to its next exchange (or its end); every shard's stage calls are
            # enqueued on the one stream in shard order, so a stage's span is its kernels alone
            cur = None
            while True:
                try:
                    req = progs[r].send(replies[r])
                except StopIteration:
                    req = None
                replies[r] = None
                if timing and (req is None or req[0] in ("stage", "exchange", "wait")):
                    ev = event()
                    if cur is not None:
                        spans.append((cur[0], r, cur[1], ev))
                    cur = (req[1], ev) if req is not None and req[0] == "stage" else None
                if req is None or req[0] != "stage":
                    break
            reqs.append(req)
        if all(q is None for q in reqs):
            break
        kinds = {q[0] if q is not None else None for q in reqs}
        if len(kinds) != 1:
            raise RuntimeError(f"shard programs out of step: {kinds}")
        if reqs[0][0] == "wait":
            continue                          # the exchange was done when it was issued
        e0 = event() if timing else None
        n_ops = len(reqs[0][1])
        for k in range(n_ops):
            kind = reqs[0][1][k][0]
            outs = [q[1][k][1] for q in reqs]
            inps = [q[1][k][2] for q in reqs]
            if kind == "all_gather":
                cat = torch.cat([t.reshape(-1) for t in inps])
                for o in outs:
                    o.view(-1).copy_(cat)
            else:                             # all_to_all_single, equal splits
                chunks = [t.view(N, -1) for t in inps]
                for r, o in enumerate(outs):
                    ov = o.view(N, -1)
                    for q in range(N):        # block q of shard r's result: shard q's block r
                        ov[q].copy_(chunks[q][r])
        if timing:
            spans.append(("exchange (device copies)", 0, e0, event()))
        for r in range(N):
            replies[r] = [] if not reqs[r][2] else None
    if timing:
        stream.synchronize()
        for name, r, a, b in spans:
            stage_ms.setdefault(name, [0.0] * N)[r] += a.elapsed_time(b)


def perturbed_observations(y, R, members, rng) -> np.ndarray:
    """y [m] -> y + eps_e, eps_e ~ N(0, R) per member: [m, members]."""
    L = np.linalg.cholesky(np.asarray(R, dtype=float))
    return np.asarray(y, float)[:, None] + L @ rng.standard_normal((len(y), members))
