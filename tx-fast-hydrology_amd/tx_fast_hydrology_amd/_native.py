"""ctypes binding of libmcroute.so (include/mcroute.h).

There is no CPU fallback: if the HIP library is missing or cannot be loaded, every routing call
raises ``NativeUnavailable``.  Host-only entry points (the topology compiler) work without a GPU.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _build

MC_OK = 0
MC_E_INVALID = -1
MC_E_TOPOLOGY = -2
MC_E_HIP = -3
MC_E_NOMEM = -4
MC_E_STATE = -5


class NativeUnavailable(RuntimeError):
    """libmcroute.so is not built or cannot be loaded."""


class RoutingError(RuntimeError):
    """A libmcroute call returned an error status."""

    def __init__(self, code, message):
        super().__init__(f"[{code}] {message}")
        self.code = code


class TopologyError(RoutingError, ValueError):
    """The network cannot be scheduled (bad indices, inconsistent indegree, ...)."""


class PlanParams(ctypes.Structure):
    _fields_ = [("slots", ctypes.c_int32), ("tile", ctypes.c_int32),
                ("ext_cap", ctypes.c_int32), ("chain", ctypes.c_int32),
                ("sync", ctypes.c_int32)]


class PlanInfo(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int64), ("n_routed", ctypes.c_int64),
                ("n_clusters", ctypes.c_int64), ("n_cross", ctypes.c_int64),
                ("nslots", ctypes.c_int64), ("nwg", ctypes.c_int32), ("slots", ctypes.c_int32),
                ("tile", ctypes.c_int32), ("gmax", ctypes.c_int32),
                ("max_height", ctypes.c_int32), ("max_ext_wg", ctypes.c_int32),
                ("n_partial", ctypes.c_int64), ("n_ext", ctypes.c_int64),
                ("n_pairs", ctypes.c_int64), ("chain", ctypes.c_int32),
                ("n_local", ctypes.c_int32)]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


# every symbol declared in include/mcroute.h: name -> (restype, argtypes)
_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int
_pp = ctypes.POINTER(ctypes.c_void_p)
SIGNATURES = {
    "mc_last_error": (ctypes.c_char_p, []),
    "mc_version": (ctypes.c_int, []),
    "mc_plan_create": (_i32, [_i64, _vp, _vp, _vp, _i64, _vp, _pp]),
    "mc_plan_get_info": (_i32, [_vp, ctypes.POINTER(PlanInfo)]),
    "mc_plan_export": (_i32, [_vp, _vp, _vp, _vp, _vp]),
    "mc_plan_export_links": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mc_plan_export_local": (_i32, [_vp, _vp, _vp]),
    "mc_plan_schedule": (_i32, [_vp, _i64, ctypes.POINTER(ctypes.c_int64),
                                ctypes.POINTER(ctypes.c_int64), _vp, _vp]),
    "mc_plan_destroy": (_i32, [_vp]),
    "mc_ax_bu_f64": (_i32, [_i64, _vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                            _vp]),
    "mc_net_create": (_i32, [_i64, _vp, _vp, _vp, _i64, _vp, _pp]),
    "mc_net_destroy": (_i32, [_vp]),
    "mc_net_get_info": (_i32, [_vp, ctypes.POINTER(PlanInfo)]),
    "mc_net_set_stream": (_i32, [_vp, _vp]),
    "mc_net_copy_state": (_i32, [_vp, _vp]),
    "mc_set_coeffs": (_i32, [_vp, _vp, _vp, _vp, _vp]),
    "mc_set_state": (_i32, [_vp, _vp, _vp]),
    "mc_get_state": (_i32, [_vp, _vp, _vp]),
    "mc_step": (_i32, [_vp, _vp, _vp, _vp, _vp, _vp]),
    "mc_load_forcing": (_i32, [_vp, _i64, _vp, _vp]),
    "mc_run": (_i32, [_vp, _i64, _vp]),
    "mc_fetch_outputs": (_i32, [_vp, _i64, _i64, _vp, _vp]),
    "mc_fetch_series": (_i32, [_vp, _vp, _vp]),
    "mc_simulate": (_i32, [_vp, _i64, _vp, _i64, _vp, _vp, _vp, _vp]),
    "mc_synchronize": (_i32, [_vp]),
    "mc_set_timing": (_i32, [_vp, ctypes.c_int]),
    "mc_get_timing": (_i32, [_vp, ctypes.POINTER(ctypes.c_double),
                             ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)]),
    "mc_reset_timing": (_i32, [_vp]),
    "mc_net_set_members": (_i32, [_vp, _i64]),
    "mc_net_get_members": (_i32, [_vp, ctypes.POINTER(ctypes.c_int64)]),
    "mc_apply_gain": (_i32, [_vp, _vp]),
    "mc_enkf_analysis": (_i32, [_vp, _i64, _vp, _vp, _vp]),
    "mc_enkf_gain": (_i32, [_vp, _i64, _vp, _vp, _vp]),
    "mc_ens_slice_size": (_i32, [_vp, _i64, ctypes.POINTER(ctypes.c_int64)]),
    "mc_ens_gauges": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp]),
    "mc_ens_pack": (_i32, [_vp, _i64, _vp]),
    "mc_ens_slice_update": (_i32, [_vp, _i64, _i64, _vp, _vp, _vp, _vp, _vp]),
    "mc_load_forcing_series": (_i32, [_vp, _i64, _vp, _vp]),
    "mc_gather_outputs": (_i32, [_vp, _i64, _i64, _vp, _vp]),
    "mc_fetch_outputs_async": (_i32, [_vp, _i64, _i64, _vp, _vp, _vp, _vp,
                                      ctypes.POINTER(ctypes.c_int64)]),
    "mc_fetch_wait": (_i32, [_vp, _i64]),
    "mc_host_digest": (_i32, [_vp, _i64, _i64, _vp]),
    "mc_host_digest2": (_i32, [_vp, _vp, _i64, _vp]),
    "mc_ens_weights": (_i32, [_vp, _i64, _i64, _vp, _vp, _vp]),
    "mc_ens_increments": (_i32, [_vp, _i64, _vp, _vp]),
    "mc_ens_unpack_apply": (_i32, [_vp, _i64, _vp]),
    "mc_comm_unique_id": (_i32, [_vp]),
    "mc_comm_init": (_i32, [ctypes.c_int32, ctypes.c_int32, _vp, _pp]),
    "mc_comm_destroy": (_i32, [_vp]),
    "mc_ens_analysis_dist": (_i32, [_vp, _vp, _i64, _vp, _vp, _vp]),
    "mc_set_mode": (_i32, [_vp, ctypes.c_int]),
    "mc_set_flow_patience": (_i32, [_vp, _i64]),
    "mc_net_lateral_correction": (_i32, [_vp, _i64, _vp, _i64, ctypes.c_double, ctypes.c_double,
                                         ctypes.c_double, ctypes.c_double]),
    "mc_net_reroutes": (_i32, [_vp, ctypes.POINTER(ctypes.c_int64)]),
    "mc_probe_tick_floor": (_i32, [ctypes.c_int32, ctypes.c_int32, _i64, ctypes.POINTER(ctypes.c_double)]),
    "mc_get_mode": (_i32, [_vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "mc_set_trace": (_i32, [_vp, ctypes.c_int]),
    "mc_get_trace": (_i32, [_vp, _vp, _i64, ctypes.POINTER(ctypes.c_int64),
                            ctypes.POINTER(ctypes.c_int64)]),
    "mc_cov_create": (_i32, [_i64, _vp, _vp, _vp, _i64, _pp]),
    "mc_cov_destroy": (_i32, [_vp]),
    "mc_cov_set_stream": (_i32, [_vp, _vp]),
    "mc_cov_set_coeffs": (_i32, [_vp, _vp, _vp, _vp]),
    "mc_cov_ap": (_i32, [_vp, _vp, _vp]),
    "mc_cov_aqat": (_i32, [_vp, _vp, _vp, _vp]),
    "mc_cov_apply_gain": (_i32, [_vp, _vp, _vp, _vp]),
    "mc_kf_update": (_i32, [_vp, _i64, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    "mc_ks_step": (_i32, [_vp, _vp, _vp, _vp, _vp, _i64, _vp, _vp, _vp]),
    "mc_cov_synchronize": (_i32, [_vp]),
}

_lib = None


def lib_path() -> str:
    return os.environ.get("MCROUTE_LIB", _build.LIB_PATH)


def lib():
    """Load libmcroute.so (build it first when the toolchain is present and it is missing)."""
    global _lib
    if _lib is not None:
        return _lib
    path = lib_path()
    # PyTorch-ROCm ships its own HIP runtime (libamdhip64.so.7, rocBLAS, rocSOLVER).  One process
    # can hold only one: when torch is present it is loaded first, so that libmcroute.so binds
    # to the same runtime (loaded the other way round, torch finds no device) and device
    # tensors and streams can be shared with the engine.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(path):
        try:
            _build.build()
        except Exception as exc:  # noqa: BLE001 - report the real cause
            raise NativeUnavailable(f"{path} is missing and could not be built: {exc}") from exc
    try:
        L = ctypes.CDLL(path)
    except OSError as exc:
        raise NativeUnavailable(f"cannot load {path}: {exc}") from exc
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name, None)
        if fn is None and "MCROUTE_LIB" in os.environ:
            continue            # an explicitly chosen (older) build for an A/B run
        if fn is None:
            raise NativeUnavailable(f"{path} does not export {name}")
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc: int):
    if rc == MC_OK:
        return
    msg = lib().mc_last_error().decode(errors="replace")
    if rc == MC_E_TOPOLOGY:
        raise TopologyError(rc, msg)
    if rc == MC_E_INVALID:
        raise RoutingError(rc, msg)
    raise RoutingError(rc, msg)


def ptr(a):
    """Data pointer of a C-contiguous numpy array (None passes NULL)."""
    if a is None:
        return None
    return ctypes.c_void_p(a.ctypes.data)


def f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def i64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int64)
