"""Python handles over the C ABI (include/mcroute.h).

* ``ax_bu``      -- drop-in for ``tx_fast_hydrology.nutils._ax_bu`` (nutils.py:64-89): same
                    positional arguments, returns fresh ``(i_t_next, o_t_next)`` arrays.
* ``Plan``       -- host-only topology compiler (usable without a GPU).
* ``RoutingNet`` -- device-resident session: coefficients, state, forcing and outputs live in
                    HBM; ``run`` routes a whole horizon in one call.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as nat
from ._native import f64, i64, ptr


def _params(slots=0, tile=0, ext_cap=0, chain=0, sync=0):
    return nat.PlanParams(int(slots), int(tile), int(ext_cap), int(chain), int(sync))


# Resident shapes of a single-member session (lanes, slots per lane, ns per tick): one compute
# wave of single-slot lanes ticks at ~0.29 us, 192 lanes x 2 at ~0.44 us but over a shorter
# schedule (chained slots cost no tick).  Same-box sweeps (profiles/r05v_shapes.txt): HUC-8
# 0.114 vs 0.162 ms per horizon, 4,000 reaches 0.163 vs 0.179; from ~12,000 reaches the 192 x 2
# schedule wins (0.269 vs 0.338).
_DET_SHAPES = ((64, 1, 0.29), (192, 2, 0.44))
_DET_SHAPE_MAX_N = 50_000
_DET_SHAPE_T = 288            # nominal horizon for the estimate: (schedule + T) ticks


# (lanes, chain) shapes of the dataflow kernel that run chunk-synchronous plans
# (kernels.hpp MCR_SYNC_SHAPES)
SYNC_SHAPES = {(64, 1), (64, 2), (128, 2), (192, 2), (256, 2), (192, 3)}

_det_shape_cache: dict = {}


def _det_shape(end, deg, heads, chain):
    """(lanes, chain) of a single-member session's default plan: the shape whose schedule of a
    nominal horizon ticks least long (host plans of both, small networks only).  The decision
    is cached by topology, so the sub-basin DAG's many sessions plan each network once here.
    The shape is fixed for the session's lifetime (set_members keeps the plan)."""
    if chain or end.size == 0 or end.size > _DET_SHAPE_MAX_N:
        return 192, chain
    import hashlib
    key = hashlib.sha1(b"".join(np.ascontiguousarray(a).tobytes()
                                for a in (end, deg, heads))).hexdigest()
    hit = _det_shape_cache.get(key)
    if hit is not None:
        return hit
    if len(_det_shape_cache) > 4096:
        _det_shape_cache.clear()
    _det_shape_cache[key] = shape = _det_shape_plan(end, deg, heads, chain)
    return shape


def _det_shape_plan(end, deg, heads, chain):
    best = None
    for lanes, k, ns_tick in _DET_SHAPES:
        try:
            p = Plan(end, deg, heads, slots=lanes, tile=16, chain=k,
                     sync=1 if (lanes, k) in SYNC_SHAPES else 0)
        except Exception:       # (a shape the plan cannot build: keep the other)
            continue
        est = (p.info["gmax"] + _DET_SHAPE_T) * ns_tick
        p.close()
        if best is None or est < best[0]:
            best = (est, lanes, k)
    return (best[1], best[2]) if best else (192, chain)


class Plan:
    """Compiled schedule of a network (no device memory)."""

    def __init__(self, endnodes, indegree, headwaters, slots=0, tile=0, ext_cap=0, chain=0,
                 sync=0):
        L = nat.lib()
        self._end = i64(endnodes)
        self._deg = i64(indegree)
        self._heads = i64(headwaters)
        self.n = self._end.size
        if self._deg.size != self.n:
            raise ValueError("indegree and endnodes must have the same length")
        h = ctypes.c_void_p()
        p = _params(slots, tile, ext_cap, chain, sync)
        nat.check(L.mc_plan_create(self.n, ptr(self._end), ptr(self._deg), ptr(self._heads),
                                   self._heads.size, ctypes.byref(p), ctypes.byref(h)))
        self._h = h

    @property
    def info(self) -> dict:
        info = nat.PlanInfo()
        nat.check(nat.lib().mc_plan_get_info(self._h, ctypes.byref(info)))
        return info.as_dict()

    def export(self) -> dict:
        info = self.info
        rank = np.empty(self.n, dtype=np.int64)
        pos = np.empty(self.n, dtype=np.int64)
        G = np.empty(info["nslots"], dtype=np.int32)
        slot_reach = np.empty(info["nslots"], dtype=np.int64)
        nat.check(nat.lib().mc_plan_export(self._h, ptr(rank), ptr(pos), ptr(G),
                                           ptr(slot_reach)))
        return dict(rank=rank, pos=pos, G=G, slot_reach=slot_reach)

    def export_links(self) -> dict:
        info = self.info
        ns, nwg = info["nslots"], info["nwg"]
        out = dict(flags=np.empty(ns, np.uint8), up_cnt=np.empty(ns, np.uint8),
                   up4=np.empty(ns, np.uint64), ext_off=np.empty(nwg + 1, np.int32),
                   ext_src=np.empty(info["n_ext"], np.int64),
                   ext_g=np.empty(info["n_ext"], np.int32))
        nat.check(nat.lib().mc_plan_export_links(
            self._h, *(ptr(out[k]) for k in ("flags", "up_cnt", "up4", "ext_off", "ext_src",
                                             "ext_g"))))
        return out

    def export_local(self) -> dict:
        """Local edges of a chunk-synchronous plan: lx_off [nwg + 1], lx_src [n_local]."""
        info = self.info
        out = dict(lx_off=np.zeros(info["nwg"] + 1, np.int32),
                   lx_src=np.empty(max(info["n_local"], 1), np.int32))
        nat.check(nat.lib().mc_plan_export_local(self._h, ptr(out["lx_off"]),
                                                 ptr(out["lx_src"])))
        out["lx_src"] = out["lx_src"][: info["n_local"]]
        return out

    def schedule(self, T: int):
        """(off [n_launch + 1], list): workgroups run by each launch of a T-step horizon."""
        nl = ctypes.c_int64()
        nls = ctypes.c_int64()
        L = nat.lib()
        nat.check(L.mc_plan_schedule(self._h, int(T), ctypes.byref(nl), ctypes.byref(nls), None,
                                     None))
        off = np.empty(nl.value + 1, dtype=np.int64)
        lst = np.empty(max(nls.value, 1), dtype=np.int32)
        nat.check(L.mc_plan_schedule(self._h, int(T), ctypes.byref(nl), ctypes.byref(nls),
                                     ptr(off), ptr(lst)))
        return off, lst[: nls.value]

    def close(self):
        if getattr(self, "_h", None):
            nat.lib().mc_plan_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


class Communicator:
    """Member-sharding communicator of the C ABI (mcroute.h mc_comm_*): nranks processes, one GPU
    each, over RCCL, without torch.distributed.  Rank 0 makes the id (``unique_id()``) and hands
    it to the others by any channel; every rank then constructs ``Communicator(nranks, rank,
    id)`` (collective).  ``RoutingNet.ens_analysis_dist(comm, ...)`` runs one analysis."""

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        nat.check(nat.lib().mc_comm_unique_id(ctypes.cast(buf, ctypes.c_void_p)))
        return bytes(buf)

    def __init__(self, nranks: int, rank: int, uid: bytes):
        if len(uid) != 128:
            raise ValueError("the communicator id is 128 bytes (Communicator.unique_id())")
        self.nranks, self.rank = int(nranks), int(rank)
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(uid)
        h = ctypes.c_void_p()
        nat.check(nat.lib().mc_comm_init(self.nranks, self.rank,
                                         ctypes.cast(buf, ctypes.c_void_p), ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            nat.lib().mc_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


class RoutingNet:
    """Device-resident routing session for one network (one HIP device, one stream).

    With ``members`` = E > 1 the session routes an ensemble: per-reach arrays are [n, E]
    (member innermost), forcing [n_rows, n, E], step-major outputs [T, n, E] (mcroute.h).
    """

    def __init__(self, endnodes, indegree, headwaters, slots=0, tile=0, ext_cap=0, members=1,
                 chain=0, sync=None):
        L = nat.lib()
        end = i64(endnodes)
        deg = i64(indegree)
        heads = i64(headwaters)
        self.n = end.size
        if deg.size != self.n:
            raise ValueError("indegree and endnodes must have the same length")
        h = ctypes.c_void_p()
        if slots == 0 and members == 1:
            # the resident dataflow launch: 192 lanes x 2 slots (3 compute waves + the helper,
            # one wave per SIMD; Texas det 0.61 ms vs 0.66 at 384 lanes and 0.82 through the
            # multi-launch path at 256), or for a small network whichever of that and one
            # compute wave of single-slot lanes ticks its horizon faster; cross-cluster slack of
            # two chunks (0.605 -> 0.594 ms)
            slots, chain = _det_shape(end, deg, heads, chain)
            tile = tile or 16
            if sync is None:
                # chunk-synchronous plan (plan.hpp): one workgroup barrier per 4 ticks
                sync = 1 if (slots, chain or 2) in SYNC_SHAPES else 0
        p = _params(slots, tile, ext_cap, chain, sync or 0)
        nat.check(L.mc_net_create(self.n, ptr(end), ptr(deg), ptr(heads), heads.size,
                                  ctypes.byref(p), ctypes.byref(h)))
        self._h = h
        self.T = 0
        self.E = 1
        self.runs = 0          # routing calls so far (mc_run / mc_step replace the outputs)
        if members != 1:
            self.set_members(members)

    def set_members(self, members: int):
        """Number of ensemble members (zeroes the state, drops forcing and outputs)."""
        nat.check(nat.lib().mc_net_set_members(self._h, int(members)))
        self.E = int(members)
        self.T = 0

    def _shape(self, *lead):
        return (*lead, self.n) if self.E == 1 else (*lead, self.n, self.E)

    # -- configuration -------------------------------------------------------------------
    @property
    def info(self) -> dict:
        info = nat.PlanInfo()
        nat.check(nat.lib().mc_net_get_info(self._h, ctypes.byref(info)))
        return info.as_dict()

    def set_stream(self, hip_stream: int | None):
        """Route on an external hipStream_t (None / 0: the session's own).  Switching streams
        synchronises the old one; setting the current stream again is free."""
        h = int(hip_stream or 0)
        if getattr(self, "_stream", None) == h:
            return
        nat.check(nat.lib().mc_net_set_stream(self._h, ctypes.c_void_p(h)))
        self._stream = h

    def set_coeffs(self, alpha, beta, chi, gamma):
        a, b, c, g = f64(alpha), f64(beta), f64(chi), f64(gamma)
        for v in (a, b, c, g):
            if v.size != self.n:
                raise ValueError("coefficient arrays must have n entries")
        nat.check(nat.lib().mc_set_coeffs(self._h, ptr(a), ptr(b), ptr(c), ptr(g)))

    def set_state(self, o_t_next, i_t_next):
        o, i = f64(o_t_next), f64(i_t_next)
        if o.size != self.n * self.E or i.size != self.n * self.E:
            raise ValueError(f"state arrays must be {self._shape()}")
        nat.check(nat.lib().mc_set_state(self._h, ptr(o), ptr(i)))

    def get_state(self):
        o = np.empty(self._shape())
        i = np.empty(self._shape())
        nat.check(nat.lib().mc_get_state(self._h, ptr(o), ptr(i)))
        return o, i

    def copy_state_from(self, other: "RoutingNet"):
        """This session's (o, i) := other's, device to device (mc_net_copy_state).  Both
        sessions route the same network with the same member count; their plans may differ
        (e.g. a 384-lane plan for one-step assimilation runs and a 256-lane, 64-tick plan for
        the forecast)."""
        nat.check(nat.lib().mc_net_copy_state(self._h, other._h))

    def add_lateral_correction(self, reach: int, src: "RoutingNet", src_reach: int,
                               o_start: float, alpha: float, beta: float, gamma: float):
        """Forcing row r of `reach` += alpha I(r+1) / gamma + beta I(r) / gamma, I = the outflow
        series of `src_reach` in src's last horizon (I(0) = o_start): the sub-basin coupling of
        the reference's AsyncSimulation, on the device and ordered on the streams
        (mcroute.h mc_net_lateral_correction)."""
        nat.check(nat.lib().mc_net_lateral_correction(
            self._h, int(reach), src._h, int(src_reach), float(o_start), float(alpha),
            float(beta), float(gamma)))

    def reroutes(self) -> int:
        """Horizons re-routed with launches after a dataflow wait gave up."""
        c = ctypes.c_int64()
        nat.check(nat.lib().mc_net_reroutes(self._h, ctypes.byref(c)))
        return c.value

    # -- routing -------------------------------------------------------------------------
    def step(self, q_t_next, o_t_prev=None, i_t_prev=None):
        """One timestep; returns fresh (i_t_next, o_t_next) like nutils._ax_bu."""
        q = f64(q_t_next)
        if q.size != self.n * self.E:
            raise ValueError(f"q must be {self._shape()}")
        o = None if o_t_prev is None else f64(o_t_prev)
        i = None if i_t_prev is None else f64(i_t_prev)
        if (o is None) != (i is None):
            raise ValueError("pass both o_t_prev and i_t_prev, or neither")
        i_out = np.empty(self._shape())
        o_out = np.empty(self._shape())
        nat.check(nat.lib().mc_step(self._h, ptr(o), ptr(i), ptr(q), ptr(i_out), ptr(o_out)))
        self.runs += 1
        return i_out, o_out

    # -- ensemble analysis -------------------------------------------------
    def apply_gain(self, gain):
        """_apply_gain (nutils.py:116-134) applied to the session state: o += gain, i += one-hop
        gain (da.py:124-126).  gain: [n] or [n, E]."""
        g = f64(gain)
        if g.size != self.n * self.E:
            raise ValueError(f"gain must be {self._shape()}")
        nat.check(nat.lib().mc_apply_gain(self._h, ptr(g)))

    def enkf_analysis(self, gauges, y, R):
        """Ensemble Kalman update of the member states: gauges [m] reach indices, y [m, E]
        observations per member, R [m, m] observation-error covariance."""
        gs, yy, RR = i64(gauges), f64(y), f64(R)
        m = gs.size
        if yy.shape != (m, self.E) or RR.shape != (m, m):
            raise ValueError("y must be [m, E] and R [m, m]")
        nat.check(nat.lib().mc_enkf_analysis(self._h, m, ptr(gs), ptr(yy), ptr(RR)))

    def ens_analysis_dist(self, comm: "Communicator", gauges, y_local, R) -> None:
        """One member-sharded analysis of this rank's E members over `comm` (RCCL;
        mcroute.h mc_ens_analysis_dist): gauges [m] and R [m, m] identical on every rank,
        y_local [m, E] this rank's perturbed observations."""
        g = i64(gauges)
        y = f64(y_local)
        Rm = f64(R)
        m = g.size
        if y.shape != (m, self.E) or Rm.shape != (m, m):
            raise ValueError("y_local must be [m, E] and R [m, m]")
        nat.check(nat.lib().mc_ens_analysis_dist(self._h, comm._h, m, ptr(g), ptr(y), ptr(Rm)))
    def enkf_gain(self, gauges, R):
        """Kalman gain of the current ensemble, K = P H^T (H P H^T + R)^-1, as [n, m]."""
        gs, RR = i64(gauges), f64(R)
        m = gs.size
        K = np.empty((self.n, m))
        nat.check(nat.lib().mc_enkf_gain(self._h, m, ptr(gs), ptr(RR), ptr(K)))
        return K

    # stages of the member-sharded analysis (mcroute.h; driven by ensemble.py).  Buffers are
    # device tensors (anything with .data_ptr()) allocated by the caller on the session's stream.
    def slice_size(self, nranks: int) -> int:
        S = ctypes.c_int64()
        nat.check(nat.lib().mc_ens_slice_size(self._h, int(nranks), ctypes.byref(S)))
        return S.value

    def ens_gauges(self, gauges, y, HX, D):
        gs, yy = i64(gauges), f64(y)
        if yy.shape != (gs.size, self.E):
            raise ValueError("y must be [m, E]")
        nat.check(nat.lib().mc_ens_gauges(self._h, gs.size, ptr(gs), ptr(yy),
                                          ctypes.c_void_p(HX.data_ptr()),
                                          ctypes.c_void_p(D.data_ptr())))

    def ens_pack(self, nranks, send):
        nat.check(nat.lib().mc_ens_pack(self._h, int(nranks), ctypes.c_void_p(send.data_ptr())))

    def ens_slice_update(self, nranks, m, Xs, HXall, Dall, R, Gs):
        RR = f64(R)
        nat.check(nat.lib().mc_ens_slice_update(
            self._h, int(nranks), int(m), ctypes.c_void_p(Xs.data_ptr()),
            ctypes.c_void_p(HXall.data_ptr()), ctypes.c_void_p(Dall.data_ptr()), ptr(RR),
            ctypes.c_void_p(Gs.data_ptr())))

    def ens_weights(self, nranks, m, HXall, Dall, R):
        RR = f64(R)
        nat.check(nat.lib().mc_ens_weights(
            self._h, int(nranks), int(m), ctypes.c_void_p(HXall.data_ptr()),
            ctypes.c_void_p(Dall.data_ptr()), ptr(RR)))

    def ens_increments(self, nranks, Xs, Gs):
        nat.check(nat.lib().mc_ens_increments(self._h, int(nranks), ctypes.c_void_p(Xs.data_ptr()),
                                              ctypes.c_void_p(Gs.data_ptr())))

    def ens_unpack_apply(self, nranks, Grecv):
        nat.check(nat.lib().mc_ens_unpack_apply(self._h, int(nranks),
                                                ctypes.c_void_p(Grecv.data_ptr())))

    def load_forcing(self, xp, fp):
        xp = f64(xp)
        fp = f64(fp)
        if fp.shape != self._shape(xp.size):
            raise ValueError(f"forcing must be {self._shape(xp.size)}, got {fp.shape}")
        nat.check(nat.lib().mc_load_forcing(self._h, xp.size, ptr(xp), ptr(fp)))

    def load_forcing_series(self, xp, fp_series):
        """load_forcing with the forcing reach-major: fp_series [n, n_rows] (or [n, n_rows, E]),
        e.g. the transpose view of a frame's values that is C-contiguous without a copy."""
        xp = f64(xp)
        fp = f64(fp_series)
        want = (self.n, xp.size) if self.E == 1 else (self.n, xp.size, self.E)
        if fp.shape != want:
            raise ValueError(f"forcing series must be {want}, got {fp.shape}")
        nat.check(nat.lib().mc_load_forcing_series(self._h, xp.size, ptr(xp), ptr(fp)))

    def run(self, x):
        """Route len(x) steps on the device (asynchronous; outputs stay resident)."""
        x = f64(x)
        nat.check(nat.lib().mc_run(self._h, x.size, ptr(x)))
        self.T = x.size
        self.runs += 1

    def fetch_outputs(self, t0=0, t1=None):
        """Step-major host copies (out_o[t][j](e), out_i[t][j](e)) of steps [t0, t1)."""
        t1 = self.T if t1 is None else t1
        out_o = np.empty(self._shape(t1 - t0))
        out_i = np.empty(self._shape(t1 - t0))
        nat.check(nat.lib().mc_fetch_outputs(self._h, t0, t1, ptr(out_o), ptr(out_i)))
        return out_o, out_i

    def fetch_outputs_async(self, t0, t1, out_o, out_i, digest_o=None, digest_i=None) -> int:
        """Queue the copy of steps [t0, t1) into the host arrays out_o / out_i ([t1 - t0, n(, E)]
        float64, C-contiguous; pinned memory for an asynchronous full-speed copy) and their row
        digests (uint64 [t1 - t0], see host_digest).  Returns a ticket; the arrays are complete
        after fetch_wait(ticket)."""
        shape = self._shape(t1 - t0)
        for a in (out_o, out_i):
            if a is not None and (a.dtype != np.float64 or a.shape != shape or
                                  not a.flags.c_contiguous):
                raise ValueError(f"output arrays must be C-contiguous float64 {shape}")
        for d in (digest_o, digest_i):
            if d is not None and (d.dtype != np.uint64 or d.shape != (t1 - t0,) or
                                  not d.flags.c_contiguous):
                raise ValueError(f"digest arrays must be C-contiguous uint64 [{t1 - t0}]")
        ticket = ctypes.c_int64()
        nat.check(nat.lib().mc_fetch_outputs_async(self._h, int(t0), int(t1), ptr(out_o),
                                                   ptr(out_i), ptr(digest_o), ptr(digest_i),
                                                   ctypes.byref(ticket)))
        # the buffers must outlive the queued copies
        self._fetching = getattr(self, "_fetching", {})
        self._fetching[ticket.value] = (out_o, out_i, digest_o, digest_i)
        return ticket.value

    def gather_outputs(self, t0, t1, dev_o=None, dev_i=None):
        """Steps [t0, t1) of the last run's outflows / inflows in reach order, step-major, into
        device tensors (anything with .data_ptr(), float64 [t1 - t0, n(, E)]) on the session
        stream (mcroute.h mc_gather_outputs); nothing is copied to the host."""
        for t in (dev_o, dev_i):
            if t is not None and t.numel() != (t1 - t0) * self.n * self.E:
                raise ValueError("device buffers must hold [t1 - t0, n(, E)] values")
        nat.check(nat.lib().mc_gather_outputs(
            self._h, int(t0), int(t1),
            ctypes.c_void_p(dev_o.data_ptr() if dev_o is not None else 0),
            ctypes.c_void_p(dev_i.data_ptr() if dev_i is not None else 0)))

    def fetch_wait(self, ticket: int):
        nat.check(nat.lib().mc_fetch_wait(self._h, int(ticket)))
        self._fetching.pop(int(ticket), None)

    def fetch_series(self):
        """Reach-major host copies (O[j][t](e), I[j][t](e)) of the last run."""
        shape = (self.n, self.T) if self.E == 1 else (self.n, self.T, self.E)
        O = np.empty(shape)
        I = np.empty(shape)
        nat.check(nat.lib().mc_fetch_series(self._h, ptr(O), ptr(I)))
        return O, I

    def simulate(self, x, xp, fp):
        self.load_forcing(xp, fp)
        self.run(x)
        return self.fetch_outputs()

    def synchronize(self):
        nat.check(nat.lib().mc_synchronize(self._h))

    # -- timing --------------------------------------------------------------------------
    def set_timing(self, enable: bool):
        nat.check(nat.lib().mc_set_timing(self._h, 1 if enable else 0))

    def reset_timing(self):
        nat.check(nat.lib().mc_reset_timing(self._h))

    def timing(self) -> dict:
        k = ctypes.c_double()
        n = ctypes.c_int64()
        r = ctypes.c_double()
        nat.check(nat.lib().mc_get_timing(self._h, ctypes.byref(k), ctypes.byref(n),
                                          ctypes.byref(r)))
        return dict(kernel_ms=k.value, launches=n.value, run_ms=r.value)

    MODES = {"auto": 0, "launches": 1, "dataflow": 2}

    def set_mode(self, mode: str):
        """Execution path: "auto" (default), "launches" or "dataflow" (mcroute.h
        mc_set_mode)."""
        nat.check(nat.lib().mc_set_mode(self._h, self.MODES[mode]))

    def set_flow_patience(self, wall_ticks: int):
        """Dataflow wait limit in 100 MHz wall-clock ticks (0 = default 2 s, < 0 = give up at
        once; a horizon whose wait gave up is re-routed with launches, mcroute.h)."""
        nat.check(nat.lib().mc_set_flow_patience(self._h, int(wall_ticks)))

    def mode(self) -> tuple:
        """(requested mode, path of the last run: "launches" / "dataflow" / None)."""
        m = ctypes.c_int()
        p = ctypes.c_int()
        nat.check(nat.lib().mc_get_mode(self._h, ctypes.byref(m), ctypes.byref(p)))
        names = {v: k for k, v in self.MODES.items()}
        return names[m.value], {1: "launches", 2: "dataflow"}.get(p.value)

    def set_trace(self, enable: bool):
        nat.check(nat.lib().mc_set_trace(self._h, 1 if enable else 0))

    def trace(self) -> tuple:
        """Launch trace of the last run: (records [m, 8] int64, clock_khz); see mcroute.h."""
        m = ctypes.c_int64()
        khz = ctypes.c_int64()
        nat.check(nat.lib().mc_get_trace(self._h, None, 0, ctypes.byref(m), ctypes.byref(khz)))
        out = np.zeros((m.value, 8), dtype=np.int64)
        nat.check(nat.lib().mc_get_trace(self._h, out.ctypes.data_as(ctypes.c_void_p), m.value,
                                         ctypes.byref(m), ctypes.byref(khz)))
        return out, khz.value

    def close(self):
        if getattr(self, "_h", None):
            nat.lib().mc_net_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def host_digest(a) -> np.ndarray:
    """Row digests (uint64) of a C-contiguous float64 array [rows, n] (a 1-D array is one row):
    the value mc_fetch_outputs_async forms on the device for the same row (mcroute.h
    mc_host_digest).  Host code, no GPU needed."""
    if a.dtype != np.float64 or not a.flags.c_contiguous:
        raise ValueError("host_digest needs a C-contiguous float64 array")
    rows = 1 if a.ndim == 1 else a.shape[0]
    n = a.size // max(rows, 1) if rows else 0
    out = np.empty(rows, dtype=np.uint64)
    nat.check(nat.lib().mc_host_digest(ptr(a), rows, n, ptr(out)))
    return out


class RowDigest:
    """Digests of a step's two rows (outflows, inflows) in one library call (mc_host_digest2):
    the per-yield edit check of Muskingum's fused horizons.  Rows: C-contiguous float64 [n]."""

    def __init__(self):
        self._fn = nat.lib().mc_host_digest2
        self._out = np.empty(2, dtype=np.uint64)
        self._p = self._out.ctypes.data

    def __call__(self, a, b):
        if not (a.flags.c_contiguous and b.flags.c_contiguous and a.dtype == np.float64 and
                b.dtype == np.float64 and a.size == b.size):
            raise ValueError("RowDigest needs two C-contiguous float64 rows of equal size")
        nat.check(self._fn(a.ctypes.data, b.ctypes.data, a.size, self._p))
        return int(self._out[0]), int(self._out[1])


def probe_tick_floor(slots=192, chain=2, ticks=8192) -> float:
    """Device ns per tick of the bare dataflow tick chain (mcroute.h mc_probe_tick_floor):
    the latency floor bench.py multiplies by the schedule length."""
    v = ctypes.c_double()
    nat.check(nat.lib().mc_probe_tick_floor(int(slots), int(chain), int(ticks),
                                            ctypes.byref(v)))
    return v.value


def ax_bu(startnodes, endnodes, alpha, beta, chi, gamma, i_t_prev, o_t_prev, q_t_next,
          indegree):
    """Drop-in for nutils._ax_bu (nutils.py:64-89) on the GPU: returns (i_t_next, o_t_next)."""
    heads = i64(startnodes)
    end = i64(endnodes)
    deg = i64(indegree)
    n = end.size
    a, b, c, g = f64(alpha), f64(beta), f64(chi), f64(gamma)
    ip, op, q = f64(i_t_prev), f64(o_t_prev), f64(q_t_next)
    i_out = np.empty(n)
    o_out = np.empty(n)
    nat.check(nat.lib().mc_ax_bu_f64(n, ptr(heads), heads.size, ptr(end), ptr(a), ptr(b), ptr(c),
                                     ptr(g), ptr(ip), ptr(op), ptr(q), ptr(deg), ptr(i_out),
                                     ptr(o_out)))
    return i_out, o_out


class CovGraph:
    """Covariance propagation and Kalman update on the device (mcroute.h ``mc_cov_*``,
    ``mc_kf_update``; reference ``nutils.py:91-214`` and ``da.py:91-136``).

    Matrices are row-major n x n float64 CUDA tensors (torch, on the current stream); the
    handle's stream follows ``torch.cuda.current_stream()`` at every call.
    """

    def __init__(self, endnodes, indegree, headwaters):
        import torch

        if not torch.cuda.is_available():
            raise nat.NativeUnavailable("CovGraph needs a GPU (torch.cuda is not available)")
        self._torch = torch
        end, deg, heads = i64(endnodes), i64(indegree), i64(headwaters)
        self.n = end.size
        if deg.size != self.n:
            raise ValueError("indegree and endnodes must have the same length")
        h = ctypes.c_void_p()
        nat.check(nat.lib().mc_cov_create(self.n, ptr(end), ptr(deg), ptr(heads), heads.size,
                                          ctypes.byref(h)))
        self._h = h

    def _sync_stream(self):
        """Order the next library call after the work queued on torch's current stream.

        The handle runs on a private torch stream (never the null stream, so the ordering is
        explicit): it waits for torch's current stream before every call, and ``_done`` makes
        torch's current stream wait for it afterwards."""
        t = self._torch
        if getattr(self, "_stream", None) is None:
            self._stream = t.cuda.Stream()
            nat.check(nat.lib().mc_cov_set_stream(self._h,
                                                  ctypes.c_void_p(self._stream.cuda_stream)))
        self._stream.wait_stream(t.cuda.current_stream())

    def _done(self, *tensors):
        t = self._torch
        for x in tensors:
            if x is not None:
                x.record_stream(self._stream)
        t.cuda.current_stream().wait_stream(self._stream)

    def _mat(self, P):
        t = self._torch
        if not isinstance(P, t.Tensor):
            P = t.as_tensor(np.ascontiguousarray(P, dtype=np.float64), device="cuda")
        if P.dtype != t.float64 or not P.is_cuda or P.shape != (self.n, self.n):
            raise ValueError(f"expected a float64 CUDA tensor of shape ({self.n}, {self.n})")
        return P.contiguous()

    def empty(self):
        return self._torch.empty((self.n, self.n), dtype=self._torch.float64, device="cuda")

    def set_coeffs(self, alpha, beta, chi):
        a, b, c = f64(alpha), f64(beta), f64(chi)
        if not (a.size == b.size == c.size == self.n):
            raise ValueError("coefficient arrays must have n entries")
        self._sync_stream()
        nat.check(nat.lib().mc_cov_set_coeffs(self._h, ptr(a), ptr(b), ptr(c)))
        self._done()

    def ap(self, P, out=None):
        """A P (_ap_par)."""
        P = self._mat(P)
        out = self.empty() if out is None else out
        self._sync_stream()
        nat.check(nat.lib().mc_cov_ap(self._h, ctypes.c_void_p(P.data_ptr()),
                                      ctypes.c_void_p(out.data_ptr())))
        self._done(P, out)
        return out

    def aqat(self, P, Q=None, out=None):
        """A P A^T (+ Q): _aqat_par then da.py:117."""
        P = self._mat(P)
        Q = None if Q is None else self._mat(Q)
        out = self.empty() if out is None else out
        self._sync_stream()
        nat.check(nat.lib().mc_cov_aqat(self._h, ctypes.c_void_p(P.data_ptr()),
                                        None if Q is None else ctypes.c_void_p(Q.data_ptr()),
                                        ctypes.c_void_p(out.data_ptr())))
        self._done(P, Q, out)
        return out

    def apply_gain(self, gain):
        """_apply_gain: (i_gain, o_gain) host arrays."""
        g = f64(gain)
        if g.size != self.n:
            raise ValueError("gain must have n entries")
        io, oo = np.empty(self.n), np.empty(self.n)
        self._sync_stream()
        nat.check(nat.lib().mc_cov_apply_gain(self._h, ptr(g), ptr(io), ptr(oo)))
        self._done()
        return io, oo

    def kf_update(self, s, R, dz, P_prior, P_post=None, want_K=True):
        """da.py:118-122: returns (P_post, K [n, m] or None, gain [n])."""
        s, R, dz = i64(s), f64(R), f64(dz)
        m = s.size
        if R.shape != (m, m) or dz.size != m:
            raise ValueError("R must be [m, m] and dz [m]")
        P_prior = self._mat(P_prior)
        P_post = P_prior if P_post is None else P_post
        K = np.empty((self.n, m)) if want_K else None
        gain = np.empty(self.n)
        self._sync_stream()
        nat.check(nat.lib().mc_kf_update(self._h, m, ptr(s), ptr(R), ptr(dz),
                                         ctypes.c_void_p(P_prior.data_ptr()),
                                         ctypes.c_void_p(P_post.data_ptr()), ptr(K), ptr(gain)))
        self._done(P_prior, P_post)
        return P_post, K, gain

    def close(self):
        if getattr(self, "_h", None):
            nat.lib().mc_cov_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def ks_step(graph, P_f, P_p1, P_s1, i_f, i_p1, i_s1, o_f, o_p1, o_s1):
    """One RTS backward step on the device (mc_ks_step, da.py:241-251): returns
    (P_s [device], i_s, o_s) for time t from the filter / prior / smoothed values at t, t+1."""
    n = graph.n
    P_f, P_p1, P_s1 = graph._mat(P_f), graph._mat(P_p1), graph._mat(P_s1)
    d = np.stack([f64(i_s1) - f64(i_p1), f64(o_s1) - f64(o_p1)])
    xf = np.ascontiguousarray(np.stack([f64(i_f), f64(o_f)]))
    xs = np.empty((2, n))
    P_s = graph.empty()
    graph._sync_stream()
    nat.check(nat.lib().mc_ks_step(graph._h, ctypes.c_void_p(P_f.data_ptr()),
                                   ctypes.c_void_p(P_p1.data_ptr()),
                                   ctypes.c_void_p(P_s1.data_ptr()),
                                   ctypes.c_void_p(P_s.data_ptr()), 2, ptr(xf), ptr(d), ptr(xs)))
    graph._done(P_f, P_p1, P_s1, P_s)
    return P_s, xs[0], xs[1]
