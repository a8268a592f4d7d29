"""Muskingum routing model with the reference API, routed by the MI355X engine.

Drop-in for ``tx_fast_hydrology/muskingum.py``: same class and function names, constructor
arguments, attributes, validation errors, hook firing points and quirks.  What changes is
where the reach recurrence runs: ``step_iter`` calls the HIP wavefront kernels through the C ABI
(``include/mcroute.h``, ``mc_step``) instead of ``nutils._ax_bu`` (reference call site
``muskingum.py:456-457``), and ``simulate_iter`` routes whole horizons in one device call
(``mc_run``, forcing interpolation fused in-kernel) whenever no callback needs to observe the
individual steps.  There is no CPU fallback: without ``libmcroute.so`` or a GPU, routing raises.

Device sessions are created lazily on the first step and rebuilt when the topology arrays
change, so models can be constructed, split, serialised and inspected on a host without a GPU.

Reference anchors (file:line in ``tx_fast_hydrology/muskingum.py``):
  constructor :139-178, properties :180-250, ``load_model`` :252-300, file IO :302-320 and
  :839-944, ``compute_indegree`` :322-330, coefficients :332-360, state space :362-408,
  ``init_states`` :410-419, ``step_iter``/``step`` :435-483, ``simulate_iter``/``simulate``
  :499-565, ``save_state``/``load_state`` :573-588, callbacks :597-605, ``split`` :607-714,
  ``Connection`` :716-726, ``ModelCollection`` :728-836.
"""
from __future__ import annotations

import copy
import datetime as _dt
import json
import logging
import uuid

import numpy as np
import pandas as pd

from .callbacks import BaseCallback
from .io import DEFAULT_START_TIME, DEFAULT_TIMEDELTA, ModelDecoder, ModelEncoder

MIN_SLOPE = 1e-8

REQUIRED_FIELDS = frozenset({"name", "datetime", "timedelta", "reach_ids", "startnodes",
                             "endnodes", "K", "X", "o_t"})
OPTIONAL_FIELDS = frozenset({"paths", "dx"})

_log = logging.getLogger(__name__)

# Largest number of state values (steps x reaches) one fused device call routes before its
# outputs are fetched: 2 arrays x 8 B x 2^25 = 512 MiB of outputs per chunk.
_HORIZON_CHUNK_VALUES = 1 << 25
# Steps of a chunk are fetched in blocks of about this many values per array (32 MiB): the
# first block's steps are yielded while the later blocks are still being copied.
_FETCH_BLOCK_VALUES = 1 << 22


def _fire(callbacks, hook):
    for callback in list(callbacks.values()):
        getattr(callback, hook)()


class _CoefArray(np.ndarray):
    """A model's alpha / beta / chi / gamma (reference ``muskingum.py:332-360``): a plain float64
    array that counts writes.  The reference reads the coefficients at every step
    (``muskingum.py:450-453``), so a fused horizon must notice a change made between two yields
    (``set_transmissive_boundary``, ``compute_muskingum_coeffs``, ``model.alpha[j] = ...``,
    ``model.beta *= ...``, ``np.copyto(model.chi, ...)``) and route the rest step by step.
    Element writes, in-place ufuncs, ``ufunc.at`` and the in-place array methods and functions
    bump the shared revision counter ``_rev`` (views share it).  Results of other operations are
    plain arrays."""

    _rev = None

    def __array_finalize__(self, obj):
        self._rev = getattr(obj, "_rev", None)

    def _touch(self):
        if self._rev is not None:
            self._rev[0] += 1

    def __setitem__(self, key, value):
        super().__setitem__(key, value)
        self._touch()

    def __array_ufunc__(self, ufunc, method, *inputs, out=None, **kwargs):
        args = [x.view(np.ndarray) if isinstance(x, _CoefArray) else x for x in inputs]
        if out is not None:
            kwargs["out"] = tuple(o.view(np.ndarray) if isinstance(o, _CoefArray) else o
                                  for o in out)
        result = getattr(ufunc, method)(*args, **kwargs)
        if method == "at" and isinstance(inputs[0], _CoefArray):
            inputs[0]._touch()
        if out is not None:
            for o in out:
                if isinstance(o, _CoefArray):
                    o._touch()
            return out[0] if len(out) == 1 else out
        return result

    def __array_function__(self, func, types, args, kwargs):
        if func in _COEF_INPLACE_FUNCS and args and isinstance(args[0], _CoefArray):
            args[0]._touch()
        return super().__array_function__(func, types, args, kwargs)

    def fill(self, value):
        super().fill(value)
        self._touch()

    def put(self, *a, **k):
        super().put(*a, **k)
        self._touch()

    def sort(self, *a, **k):
        super().sort(*a, **k)
        self._touch()

    def partition(self, *a, **k):
        super().partition(*a, **k)
        self._touch()

    def __reduce__(self):
        # pickles / copies as a plain array; the owning model re-wraps it (_own_coefs)
        return self.view(np.ndarray).__reduce__()

    def __deepcopy__(self, memo):
        return np.array(self.view(np.ndarray), copy=True)


_COEF_INPLACE_FUNCS = frozenset({np.copyto, np.put, np.place, np.putmask, np.fill_diagonal,
                                 np.put_along_axis})


def _coef_property(name):
    attr = "_" + name

    def fget(self):
        return self.__dict__.get(attr)

    def fset(self, value):
        self.__dict__[attr] = self._coef_view(value)

    return property(fget, fset, doc=f"Muskingum coefficient {name} (per reach; tracked writes)")


def _host_array(shape, dtype):
    """Host array for fetched outputs: pinned (torch's caching host allocator, so a block freed
    by the caller is reused by the next horizon without a new page-locking) when a GPU is
    present, so the device copies run asynchronously at full PCIe speed."""
    try:
        import torch
        if torch.cuda.is_available():
            tdt = {np.dtype(np.float64): torch.float64, np.dtype(np.uint64): torch.uint64}
            return torch.empty(shape, dtype=tdt[np.dtype(dtype)], pin_memory=True).numpy()
    except (ImportError, KeyError, RuntimeError, TypeError):
        pass
    return np.empty(shape, dtype=dtype)


class _InflowBlock:
    """The inflow rows of one fetch block of a fused horizon (steps [b0, b1) of the session's
    last run), copied from the device only when a caller first reads one of them.  The
    reference's own caller reads only the outflows (simulation.py:126-130), so a horizon whose
    inflows nobody reads moves half the bytes over PCIe."""

    __slots__ = ("net", "run_id", "b0", "b1", "n", "rows", "digests")

    def __init__(self, net, b0, b1, n):
        self.net, self.run_id, self.b0, self.b1, self.n = net, net.runs, b0, b1, n
        self.rows = self.digests = None

    def fetch(self):
        if self.rows is None:
            if getattr(self.net, "_h", 1) is None:
                # Muskingum.close() settles its rows first; a block kept past that is an error
                raise RuntimeError("inflow rows were requested after their device session "
                                   "was closed")
            if self.net.runs != self.run_id:
                # the model settles its lazy rows before anything reruns its session
                raise RuntimeError("inflow rows of an earlier run were requested after the "
                                   "session routed again")
            rows = _host_array((self.b1 - self.b0, self.n), np.float64)
            dig = np.empty(self.b1 - self.b0, dtype=np.uint64)
            self.net.fetch_wait(self.net.fetch_outputs_async(self.b0, self.b1, None, rows,
                                                             None, dig))
            self.rows, self.digests = rows, dig
        return self.rows


class _LazyInflow:
    """``i_t_next`` of one yielded step until a caller reads it (``Muskingum.i_t_next``): then
    the step's row of its fetch block (a copy of its own for the last two steps, so the model's
    final state keeps no block alive)."""

    __slots__ = ("block", "k", "own", "value")

    def __init__(self, block, k, own):
        self.block, self.k, self.own, self.value = block, k, own, None

    def get(self):
        if self.value is None:
            row = self.block.fetch()[self.k]
            self.value = row.copy() if self.own else row
        return self.value

    def digest(self):
        return int(self.block.digests[self.k])


def _inflow_property(name):
    key = "_" + name

    def fget(self):
        v = self.__dict__.get(key)
        if isinstance(v, _LazyInflow):
            v = self.__dict__[key] = v.get()
        return v

    def fset(self, value):
        self.__dict__[key] = value

    return property(fget, fset, doc=f"{name} (host float64 [n]; a fused horizon fetches it from "
                                    "the device when it is first read)")


def _upload_forcing(net, xp, dataframe):
    """Forcing frame -> the session (mc_load_forcing): a frame whose float64 block is stored
    reach-major (any frame pandas copied or built column by column) goes up in its own layout
    (mc_load_forcing_series, no host transpose copy), else step-major."""
    vals = dataframe.values
    series = vals.T
    if vals.dtype == np.float64 and series.flags.c_contiguous and \
            hasattr(net, "load_forcing_series"):
        net.load_forcing_series(xp, series)
    else:
        net.load_forcing(xp, np.ascontiguousarray(vals, dtype=np.float64))


class _DeviceRouting:
    """Device session of one model: a ``RoutingNet`` plus the host snapshot of the topology and
    coefficients it was built from (rebuilt / re-uploaded when they change)."""

    def __init__(self):
        self.net = None
        self.topo = None
        self.coef = None
        self.columns = None     # (frame columns, reach_ids snapshot) last found in reach order

    def in_reach_order(self, cols, reach_ids):
        """True when the frame's columns are ``reach_ids`` in order.  Building an Index of the
        ids and comparing it costs ~20 ms at Texas size per horizon; a frame whose (immutable)
        column Index was already checked against the same ids is accepted after comparing the
        id list with the snapshot kept then (element identity first: well under 1 ms)."""
        ids = reach_ids if isinstance(reach_ids, list) else list(reach_ids)
        seen = self.columns
        if seen is not None and seen[0] is cols and seen[1] == ids:
            return True
        same = len(cols) == len(ids) and cols.equals(pd.Index(ids))
        self.columns = (cols, list(ids)) if same else None
        return same

    def session(self, model):
        from . import engine

        end = np.ascontiguousarray(model.endnodes, dtype=np.int64)
        deg = np.ascontiguousarray(model.indegree, dtype=np.int64)
        heads = np.ascontiguousarray(np.asarray(model.startnodes)[deg == 0], dtype=np.int64)
        topo = (end, deg, heads)
        if self.net is None or not all(np.array_equal(a, b) for a, b in zip(topo, self.topo)):
            if self.net is not None:
                self.net.close()
            self.net = engine.RoutingNet(end, deg, heads)
            self.topo = tuple(a.copy() for a in topo)
            self.coef = None
        coef = (model.alpha, model.beta, model.chi, model.gamma)
        if self.coef is None or not all(np.array_equal(a, b) for a, b in zip(coef, self.coef)):
            self.net.set_coeffs(*coef)
            self.coef = tuple(np.array(a, dtype=np.float64) for a in coef)
        return self.net

    def close(self):
        if self.net is not None:
            self.net.close()
        self.net = None
        self.topo = None
        self.coef = None


class Muskingum:
    """Muskingum routing over a river network (reference ``muskingum.py:20-138``).

    ``data`` is a model description dict (fields ``name``, ``datetime`` (UTC ``pd.Timestamp``),
    ``timedelta``, ``reach_ids``, ``startnodes``/``endnodes`` (int64), ``K``/``X``/``o_t``
    (float64), optional ``dx`` and ``paths``) or the path of a JSON model file.

    State: ``o_t_next``/``i_t_next`` (outflows/inflows at the current time) and
    ``o_t_prev``/``i_t_prev`` (previous step), host numpy arrays as in the reference; the device
    holds them only for the duration of a routing call.  ``A``/``B`` (state-space matrices) are
    materialised on first access instead of at construction: a dense n x n pair is 577 GB at
    Texas scale.
    """

    alpha = _coef_property("alpha")
    beta = _coef_property("beta")
    chi = _coef_property("chi")
    gamma = _coef_property("gamma")
    i_t_next = _inflow_property("i_t_next")
    i_t_prev = _inflow_property("i_t_prev")

    def __init__(self, data, load_optional=True, create_state_space=False, sparse=False):
        self.sparse = sparse
        self.callbacks = {}
        self.saved_states = {}
        self.sinks = []
        self.sources = []
        self._device = _DeviceRouting()
        self._A = None
        self._B = None
        if isinstance(data, dict):
            self.load_model(data, load_optional=load_optional)
        elif isinstance(data, str):
            self.load_model_file(data, load_optional=load_optional)
        else:
            raise TypeError("`data` must be a file path or dictionary.")
        self.logger = logging.getLogger(self.name)
        n = self.n
        self.o_t_prev = np.zeros(n, dtype=np.float64)
        self.i_t_next = np.zeros(n, dtype=np.float64)
        self.i_t_prev = np.zeros(n, dtype=np.float64)
        self.init_states(o_t_next=self.o_t_next)
        self.o_t_prev[:] = self.o_t_next
        self.i_t_prev[:] = self.i_t_next
        self.alpha = np.zeros(n, dtype=np.float64)
        self.beta = np.zeros(n, dtype=np.float64)
        self.chi = np.zeros(n, dtype=np.float64)
        self.gamma = np.zeros(n, dtype=np.float64)
        self.compute_muskingum_coeffs()
        if create_state_space:
            self.create_state_space()
        self.save_state()

    def _settle_inflows(self):
        """Materialise inflow rows still left on the device by a fused horizon (before anything
        routes on the session again, and before the model is copied)."""
        for name in ("i_t_next", "i_t_prev"):
            getattr(self, name)

    # -- copying: the device session is never shared or copied ---------------------------------
    def __getstate__(self):
        self._settle_inflows()
        state = self.__dict__.copy()
        state["_device"] = None
        return state

    def __setstate__(self, state):
        # a model pickled before the inflows became lazy properties stores them under their
        # public names, which the properties would shadow
        for key in ("i_t_next", "i_t_prev"):
            if key in state:
                state["_" + key] = state.pop(key)
        self.__dict__.update(state)
        self._device = _DeviceRouting()
        self._own_coefs()

    def __deepcopy__(self, memo):
        self._settle_inflows()
        clone = self.__class__.__new__(self.__class__)
        memo[id(self)] = clone
        for key, value in self.__dict__.items():
            if key == "_device":
                continue
            clone.__dict__[key] = copy.deepcopy(value, memo)
        clone._device = _DeviceRouting()
        clone._own_coefs()
        return clone

    # -- coefficient write tracking (see _CoefArray) ------------------------------------------
    def _coef_view(self, value):
        rev = self.__dict__.setdefault("_coef_rev", [0])
        rev[0] += 1
        v = np.asarray(value).view(_CoefArray)
        v._rev = rev
        return v

    def _own_coefs(self):
        """A revision counter of this model's own (after a copy or unpickling)."""
        self.__dict__["_coef_rev"] = [0]
        for name in ("alpha", "beta", "chi", "gamma"):
            a = self.__dict__.get("_" + name)
            if a is not None:
                setattr(self, name, a)

    def close(self):
        """Release the device session (it is recreated by the next routing call).  Inflow rows a
        fused horizon left on the session are copied to the host first, so the state stays
        readable (and a held simulate() generator can still settle)."""
        self._settle_inflows()
        self._device.close()

    # -- properties ----------------------------------------------------------------------------
    @property
    def info(self):
        return {
            "name": self.name,
            "datetime": self.datetime,
            "timedelta": self.timedelta,
            "reach_ids": self.reach_ids,
            "startnodes": self.startnodes,
            "endnodes": self.endnodes,
            "K": self.K,
            "X": self.X,
            "o_t": self.o_t_next,
            "dx": self.dx,
            "paths": self.paths,
        }

    @property
    def name(self):
        return self._name

    @name.setter
    def name(self, new_name):
        if not isinstance(new_name, str):
            new_name = str(new_name)
            getattr(self, "logger", _log).warning(f"`name` is not a string, converting to {new_name}")
        self._name = new_name

    @property
    def datetime(self):
        return self._datetime

    @datetime.setter
    def datetime(self, new_datetime):
        if not isinstance(new_datetime, pd.Timestamp):
            raise TypeError("New datetime must be of type `pd.Timestamp`")
        if new_datetime.tz != _dt.timezone.utc:
            raise ValueError("New datetime must be UTC.")
        self._datetime = new_datetime

    @property
    def timedelta(self):
        return self._timedelta

    @timedelta.setter
    def timedelta(self, new_timedelta):
        if not isinstance(new_timedelta, pd.Timedelta):
            raise TypeError("New timedelta must be of type `pd.Timedelta`")
        self._timedelta = new_timedelta

    @property
    def o_t(self):
        return self.o_t_next

    @o_t.setter
    def o_t(self, new_o_t):
        try:
            new_o_t = np.asarray(new_o_t, dtype=np.float64)
        except Exception as exc:
            raise TypeError("New `o_t` must be convertible to float64 np.ndarray") from exc
        self.o_t_next = new_o_t

    @property
    def dt(self):
        # timedelta.seconds ignores whole days (muskingum.py:247-250): kept
        return float(self.timedelta.seconds)

    @property
    def A(self):
        if self._A is None:
            self._A = self._zeros_square()
        return self._A

    @A.setter
    def A(self, value):
        self._A = value

    @property
    def B(self):
        if self._B is None:
            self._B = self._zeros_square()
        return self._B

    @B.setter
    def B(self, value):
        self._B = value

    def _zeros_square(self):
        if self.sparse:
            from scipy.sparse import lil_matrix
            return lil_matrix((self.n, self.n))
        return np.zeros((self.n, self.n), dtype=np.float64)

    # -- model description -----------------------------------------------------------------------
    def load_model(self, obj, load_optional=True):
        if not REQUIRED_FIELDS.issubset(obj.keys()):
            raise ValueError(f"Model field must contain fields {set(REQUIRED_FIELDS)}")
        typed = (("startnodes", np.int64), ("endnodes", np.int64), ("K", np.float64),
                 ("X", np.float64), ("o_t", np.float64))
        for key, dtype in typed:
            if not isinstance(obj[key], np.ndarray) or obj[key].dtype != dtype:
                raise TypeError("Typing of input arrays is incorrect.")
        if len({obj[key].size for key, _ in typed}) != 1:
            raise ValueError("Arrays are not the same length")
        defaults = {"name": str(uuid.uuid4()), "datetime": DEFAULT_START_TIME,
                    "timedelta": DEFAULT_TIMEDELTA, "dx": None, "paths": []}
        fields = REQUIRED_FIELDS | OPTIONAL_FIELDS if load_optional else REQUIRED_FIELDS
        for field in fields:
            if field in defaults:
                value = obj.setdefault(field, defaults[field])
            else:
                value = obj[field]
            setattr(self, field, value)
        self.n = self.startnodes.size
        self.indegree = self.compute_indegree(self.startnodes, self.endnodes)

    def load_model_file(self, file_path, load_optional=True):
        self.load_model(load_model_file(file_path, load_optional=load_optional))

    def dump_model_file(self, file_path, dump_optional=True):
        return dump_model_file(self.info, file_path, dump_optional=dump_optional)

    @classmethod
    def from_model_file(cls, file_path, load_optional=True, **kwargs):
        return cls(load_model_file(file_path, load_optional=load_optional), **kwargs)

    @classmethod
    def from_nhd_geojson(cls, file_path, **kwargs):
        return cls(load_nhd_geojson(file_path), **kwargs)

    # -- setup kernels (host, oracle-pinned) ------------------------------------------
    def compute_indegree(self, startnodes, endnodes):
        """Upstream count per reach: bincount of endnodes minus self-loops (:322-330)."""
        endnodes = np.asarray(endnodes)
        indegree = np.bincount(endnodes.ravel(), minlength=np.asarray(startnodes).size)
        loops = np.flatnonzero(endnodes == np.asarray(startnodes))
        np.subtract.at(indegree, loops, 1)
        return indegree

    def compute_alpha(self, K, X, dt):
        return (dt - 2 * K * X) / (2 * K * (1 - X) + dt)

    def compute_beta(self, K, X, dt):
        return (dt + 2 * K * X) / (2 * K * (1 - X) + dt)

    def compute_chi(self, K, X, dt):
        return (2 * K * (1 - X) - dt) / (2 * K * (1 - X) + dt)

    def compute_gamma(self, K, X, dt):
        return dt / (K * (1 - X) + dt / 2)

    def compute_muskingum_coeffs(self, K=None, X=None, dt=None):
        self.logger.info("Computing Muskingum coefficients...")
        K = self.K if K is None else K
        X = self.X if X is None else X
        dt = self.dt if dt is None else dt
        self.alpha[:] = self.compute_alpha(K, X, dt)
        self.beta[:] = self.compute_beta(K, X, dt)
        self.chi[:] = self.compute_chi(K, X, dt)
        self.gamma[:] = self.compute_gamma(K, X, dt)

    def create_state_space(self, overwrite_old=True):
        self.logger.info("Creating state-space system...")
        if overwrite_old:
            self._A = None
            self._B = None
        heads = self.startnodes[self.indegree == 0]
        self.A, self.B = self.muskingum_matrix(self.A, self.B, heads, self.endnodes, self.alpha,
                                               self.beta, self.chi, self.gamma, self.indegree)

    def muskingum_matrix(self, A, B, startnodes, endnodes, alpha, beta, chi, gamma, indegree):
        """Dense/sparse state-space matrices by the reference walk (:383-408): a reach's row is
        finalised when all its upstream rows are, then folded into its downstream row."""
        remaining = np.array(indegree, copy=True)
        for head in startnodes:
            j = head
            while remaining[j] == 0:
                down = endnodes[j]
                A[j, j] = chi[j]
                B[j, j] = gamma[j]
                if down != j:
                    A[down, j] += beta[down]
                    A[down] += alpha[down] * A[j]
                    B[down] += alpha[down] * B[j]
                remaining[down] -= 1
                j = down
        return A, B

    def init_states(self, o_t_next=None, i_t_next=None):
        if o_t_next is None:
            self.o_t_next[:] = 0.0
        else:
            self.o_t_next[:] = o_t_next[:]
        if i_t_next is None:
            # unbuffered scatter in index order, self-loops included (muskingum.py:415-417);
            # bincount adds the weights into a zeroed array in the same index order as np.add.at
            # (same bits), several times faster
            self.i_t_next[:] = np.bincount(self.endnodes, weights=self.o_t_next[self.startnodes],
                                           minlength=self.n)
        else:
            self.i_t_next[:] = i_t_next[:]

    # -- routing ---------------------------------------------------------------------------------
    def step_matrix(self, p_t_next, num_iter=1, inc_t=False):
        raise NotImplementedError

    def simulate_matrix(self, dataframe, **kwargs):
        raise NotImplementedError

    def step_iter(self, p_t_next, timedelta=None):
        """One timestep on the device (reference :435-465, kernel call :456-457)."""
        if timedelta is None:
            timedelta = self.timedelta
            dt = self.dt
        else:
            dt = float(timedelta.seconds)
        o_t_prev = self.o_t_next
        i_t_prev = self.i_t_next
        if dt != self.dt:
            # permanent until the next explicit change (reference quirk, golden g6)
            self.logger.warning("Timestep has changed. Recomputing Muskingum coefficients.")
            self.compute_muskingum_coeffs(dt=dt)
        _fire(self.callbacks, "__on_step_start__")
        self._settle_inflows()
        net = self._device.session(self)
        i_t_next, o_t_next = net.step(p_t_next, o_t_prev, i_t_prev)
        self.o_t_next = o_t_next
        self.o_t_prev = o_t_prev
        self.i_t_next = i_t_next
        self.i_t_prev = i_t_prev
        self.datetime += timedelta
        _fire(self.callbacks, "__on_step_end__")
        self.logger.debug(f"Stepped to time {self.datetime}")

    def step(self, p_t_next, timedelta=None):
        """Advance one timestep: new ``o_t_next`` / ``i_t_next`` from lateral inputs
        ``p_t_next`` (float64 [n]).  ``timedelta`` defaults to ``self.timedelta``."""
        return self.step_iter(p_t_next, timedelta=timedelta)

    def simulate_iter(self, dataframe, start_time=None, end_time=None, o_t_init=None, **kwargs):
        """Generator over timesteps (reference :499-536); yields ``self`` after each step.

        Without a ``timedelta`` override and while every bound callback is idle
        (``BaseCallback.__idle_steps__``; no callbacks at all is the common case), the remaining
        horizon is routed by the device in fused calls (``mc_run``: interpolation of the forcing rows and
        routing of every step in one launch) and the steps are then replayed on the host, each
        yielding fresh writable copies of the fetched outputs.  Editing a state array in place,
        replacing it, rebinding ``datetime`` or binding a non-idle callback between two yields
        switches the rest of the horizon to step-by-step routing from the state found, as the
        reference would route it; so does changing a coefficient array (``_CoefArray`` counts
        writes).  Topology is read when a fused call starts.

        Limit of the coefficient tracking: only writes through the model's own arrays (or their
        ndarray views created from them) are counted.  Writes through a base-class alias --
        ``np.asarray(model.alpha)`` (a plain ndarray sharing the memory), ``.view(np.ndarray)``,
        ``torch.from_numpy``, numba or ctypes buffers -- are NOT seen; a fused horizon then keeps
        routing with the coefficients uploaded when it started.  To change coefficients in the
        middle of a horizon, assign through the model (``model.alpha[j] = v``,
        ``model.alpha = new``) or bind a non-idle callback.
        """
        assert isinstance(dataframe.index, pd.DatetimeIndex)
        assert dataframe.index.tz == _dt.timezone.utc
        cols = dataframe.columns
        same_columns = self._device.in_reach_order(cols, self.reach_ids)
        assert same_columns or np.isin(self.reach_ids, cols).all()
        if end_time is None:
            end_time = dataframe.index.max()
        elif not isinstance(end_time, pd.Timestamp):
            raise TypeError("`end_time` must be of type `pd.Timestamp`")
        if start_time is not None:
            # (the reference builds, but never raises, an error when o_t_init is missing)
            self.datetime = start_time
        if o_t_init is not None:
            self.init_states(o_t_next=o_t_init)
        _fire(self.callbacks, "__on_simulation_start__")
        if not same_columns:        # (a frame already in reach order is used as it is)
            dataframe = dataframe[self.reach_ids]
        xp = dataframe.index.astype(int).astype(float).values
        fused = kwargs.get("timedelta") is None and self._callbacks_idle()
        if fused:
            yield from self._simulate_fused(dataframe, xp, end_time, kwargs)
        else:
            yield from self._simulate_steps(dataframe, xp, end_time, kwargs)
        _fire(self.callbacks, "__on_simulation_end__")

    def _simulate_steps(self, dataframe, xp, end_time, kwargs):
        from .nutils import interpolate_sample
        fp = dataframe.values
        while self.datetime < end_time:
            if kwargs.get("timedelta") is None and self._callbacks_idle():
                yield from self._simulate_fused(dataframe, xp, end_time, kwargs)
                return
            next_timestep = self.datetime + self.timedelta
            p_t_next = interpolate_sample(float(next_timestep.value), xp, fp)
            self.step_iter(p_t_next, **kwargs)
            yield self

    def _callbacks_idle(self):
        """True when no bound callback needs to see the remaining steps (``__idle_steps__``)."""
        return all(getattr(cb, "__idle_steps__", lambda: False)()
                   for cb in self.callbacks.values())

    def _simulate_fused(self, dataframe, xp, end_time, kwargs):
        xs = []
        t = self.datetime
        while t < end_time:
            t = t + self.timedelta
            xs.append(float(t.value))
        if not xs:
            return
        from . import engine
        self._settle_inflows()
        net = self._device.session(self)
        _upload_forcing(net, xp, dataframe)
        net.set_state(self.o_t_next, self.i_t_next)
        n, T = self.n, len(xs)
        chunk = max(1, _HORIZON_CHUNK_VALUES // max(n, 1))
        block = max(1, _FETCH_BLOCK_VALUES // max(n, 1))
        timedelta = self.timedelta
        rev = self._coef_rev[0]
        # the reference formats its per-step debug message unconditionally; formatting a
        # Timestamp costs more than the rest of a yielded step, so it is built only when emitted
        debug = self.logger.isEnabledFor(logging.DEBUG)
        d = self.__dict__
        pending = []          # fetch tickets not yet waited for
        try:
            for c0 in range(0, T, chunk):
                x = np.asarray(xs[c0:c0 + chunk])
                self._settle_inflows()          # rows of the previous chunk still on the device
                net.run(x)
                # the chunk's outflows in blocks: every block's copy (pinned host rows + the
                # device's row digests) is queued now; the steps of block b are yielded while
                # blocks b + 1, ... are still being copied.  The inflows stay on the device
                # until a caller reads one (_LazyInflow: the block's inflow rows are fetched then)
                blocks = []
                digests = _host_array((x.size,), np.uint64)
                for b0 in range(0, x.size, block):
                    b1 = min(x.size, b0 + block)
                    oo = _host_array((b1 - b0, n), np.float64)
                    tk = net.fetch_outputs_async(b0, b1, oo, None, digests[b0:b1], None)
                    pending.append(tk)
                    blocks.append((b0, oo, _InflowBlock(net, b0, b1, n), tk))
                for b0, oo, iblk, tk in blocks:
                    net.fetch_wait(tk)
                    pending.remove(tk)
                    for k in range(oo.shape[0]):
                        # a writable array of its own each step, as the reference allocates
                        # them (nutils.py:68-70): row k of a freshly fetched block (no other
                        # step shares its memory).  The last two steps of the horizon are
                        # copies, so the model's final state keeps no block alive.  A caller
                        # may edit a yielded array in place (state.o_t_next[j] = obs) or replace
                        # it, or change a coefficient; either is detected below (identity, the
                        # row digest the device formed before the copy, the coefficient
                        # revision) and the rest of the horizon is routed step by step from
                        # the state found
                        step = c0 + b0 + k
                        last = step >= T - 2
                        o_next = oo[k].copy() if last else oo[k]
                        i_ref = _LazyInflow(iblk, k, last)
                        self.o_t_prev = self.o_t_next
                        d["_i_t_prev"] = d.get("_i_t_next")    # (not materialised)
                        self.o_t_next = o_next
                        d["_i_t_next"] = i_ref
                        # (a UTC Timestamp plus a Timedelta: the setter's checks hold)
                        self._datetime = expected_time = self._datetime + timedelta
                        if debug:
                            self.logger.debug(f"Stepped to time {self.datetime}")
                        yield self
                        i_now = d.get("_i_t_next")
                        edited = (self.o_t_next is not o_next or
                                  int(engine.host_digest(o_next)[0]) != int(digests[b0 + k]))
                        if not edited and i_now is not i_ref:
                            # read (materialised) or replaced: an edit unless it is the row
                            # itself with the device's digest
                            edited = (i_now is not i_ref.value or
                                      int(engine.host_digest(i_now)[0]) != i_ref.digest())
                        if (edited or self._coef_rev[0] != rev or not self._callbacks_idle()
                                or self.datetime != expected_time
                                or self.timedelta != timedelta):
                            self._settle_inflows()
                            yield from self._simulate_steps(dataframe, xp, end_time, kwargs)
                            return
        finally:
            for tk in pending:
                net.fetch_wait(tk)
            self._settle_inflows()

    def simulate(self, dataframe, start_time=None, end_time=None, o_t_init=None, **kwargs):
        """Route over a time range; returns the ``simulate_iter`` generator (yields ``self``).

        ``dataframe``: lateral inputs (UTC ``DatetimeIndex``, one column per reach id);
        ``end_time`` defaults to the last forcing time; ``o_t_init`` resets the outflows.
        """
        return self.simulate_iter(dataframe, start_time=start_time, end_time=end_time,
                                  o_t_init=o_t_init, **kwargs)

    # -- state, hooks, copies ------------------------------------------------------------------
    def set_transmissive_boundary(self, index):
        self.alpha[index] = 1.0
        self.beta[index] = 0.0
        self.chi[index] = 0.0
        self.gamma[index] = 0.0

    def save_state(self):
        self.logger.info(f"Saving state for model {self.name} at time {self.datetime}...")
        self.saved_states["datetime"] = self.datetime
        self.saved_states["i_t_next"] = np.array(self.i_t_next, copy=True)
        self.saved_states["o_t_next"] = np.array(self.o_t_next, copy=True)
        _fire(self.callbacks, "__on_save_state__")

    def load_state(self):
        self.datetime = self.saved_states["datetime"]
        self.i_t_next = self.saved_states["i_t_next"]
        self.o_t_next = self.saved_states["o_t_next"]
        self.logger.info(f"Loading state for model {self.name} at time {self.datetime}...")
        _fire(self.callbacks, "__on_load_state__")

    def plot(self, ax, *args, **kwargs):
        for path in self.paths:
            for subpath in path:
                xy = np.asarray(subpath)
                ax.plot(xy[:, 0], xy[:, 1], *args, **kwargs)

    def bind_callback(self, callback, key="callback"):
        assert isinstance(callback, BaseCallback)
        self.callbacks[key] = callback

    def unbind_callback(self, key):
        return self.callbacks.pop(key)

    def copy(self):
        return copy.deepcopy(self)

    # -- sub-basins ----------------------------------------------------------------
    def split(self, indices, name=None, create_state_space=True):
        """Cut the network below each reach in ``indices`` and return a ``ModelCollection`` of
        the connected components, linked by ``Connection`` objects (reference :607-714).

        The cut reaches become outlets (self-loops); each downstream entry reach loses one
        indegree and has the upstream outflow removed from its inflow, so the collection routed
        with ``AsyncSimulation`` reproduces the whole network.
        """
        from scipy.sparse import coo_matrix
        from scipy.sparse.csgraph import connected_components

        whole = copy.deepcopy(self)
        cut_pos = np.asarray([np.flatnonzero(whole.startnodes == i).item() for i in indices])
        entry_pos = whole.endnodes[cut_pos]
        whole.endnodes[cut_pos] = indices
        n = whole.n
        adj = coo_matrix((np.ones(n, dtype=int), (whole.endnodes, whole.startnodes)),
                         shape=(n, n)).tolil()
        n_components, labels = connected_components(adj)
        index_map = pd.Series(np.arange(n), index=whole.startnodes)
        cut_comp = labels[cut_pos].astype(int).tolist()
        entry_comp = labels[entry_pos].astype(int).tolist()
        # per component: (downstream component, cut position, entry position); -1 = none
        links = []
        for k in range(n_components):
            if k in cut_comp:
                p = cut_comp.index(k)
                links.append((entry_comp[p], int(cut_pos[p]), int(entry_pos[p])))
            else:
                links.append((k, -1, -1))
        components = {}
        for k in range(n_components):
            sel = labels == k
            sub_start = whole.startnodes[sel]
            sub_end = whole.endnodes[sel]
            node_map = pd.Series(np.arange(len(sub_start)), index=sub_start)
            rows = index_map[sub_start].values
            sub = copy.deepcopy(whole, {id(a): a for a in _large_arrays(whole)})
            sub.name = str(k)
            sub.startnodes = np.arange(len(sub_start))
            sub.endnodes = node_map.loc[sub_end].values
            sub.n = len(sub.startnodes)
            sub.indegree = whole.indegree[rows]
            sub.reach_ids = np.asarray(whole.reach_ids)[rows].tolist()
            sub.dx = whole.dx[rows]
            for key in ("K", "X", "alpha", "beta", "chi", "gamma", "o_t_prev", "i_t_prev",
                        "o_t_next", "i_t_next"):
                setattr(sub, key, getattr(whole, key)[rows])
            sub.A = np.zeros((sub.n, sub.n))
            sub.B = np.zeros((sub.n, sub.n))
            sub.paths = [whole.paths[i] for i in rows]
            if create_state_space:
                sub.create_state_space()
            sub.save_state()
            components[k] = {"model": sub, "node_map": node_map}
        for k in range(n_components):
            down, cut, entry = links[k]
            up_c, down_c = components[k], components[down]
            up_c["exit_node"] = cut
            up_c["entry_node"] = entry
            if cut >= 0 and entry >= 0:
                upstream, downstream = up_c["model"], down_c["model"]
                u = up_c["node_map"][cut]
                d = down_c["node_map"][entry]
                downstream.indegree[d] -= 1
                downstream.i_t_next[d] -= upstream.o_t_next[u]
                connection = Connection(upstream, downstream, u, d)
                upstream.sinks.append(connection)
                downstream.sources.append(connection)
        return ModelCollection([components[k]["model"] for k in components], name=name)


def _large_arrays(model):
    """Per-reach arrays ``split`` replaces in every sub-model: shared, not deep-copied, while
    the sub-model is cloned (the reference deep-copies them once per component)."""
    keys = ("startnodes", "endnodes", "indegree", "K", "X", "o_t_next", "i_t_next", "o_t_prev",
            "i_t_prev", "alpha", "beta", "chi", "gamma", "dx", "paths", "reach_ids", "_A", "_B")
    arrays = [getattr(model, key, None) for key in keys]
    arrays += [model.saved_states.get(key) for key in ("i_t_next", "o_t_next")]
    return [a for a in arrays if a is not None]


class Connection:
    """Outlet reach ``upstream_index`` of ``upstream_model`` feeds reach ``downstream_index`` of
    ``downstream_model`` (reference :716-726)."""

    def __init__(self, upstream_model, downstream_model, upstream_index, downstream_index,
                 name=None):
        self.upstream_model = upstream_model
        self.downstream_model = downstream_model
        self.upstream_index = upstream_index
        self.downstream_index = downstream_index
        self.name = str(uuid.uuid4()) if name is None else name


class ModelCollection:
    """Named sub-basin models (reference :728-836)."""

    def __init__(self, models, name=None):
        self.models = {model.name: model for model in models}
        self.name = str(uuid.uuid4()) if name is None else name

    @property
    def info(self):
        return {}

    def _common(self, attr, convert, what):
        values = {getattr(model, attr) for model in self.models.values()}
        if len(values) != 1:
            raise ValueError(f"Models must all have the same {what}")
        return convert(values.pop())

    @property
    def datetime(self):
        return self._common("datetime", pd.to_datetime, "datetime")

    @property
    def timedelta(self):
        # (the reference's message says "datetime" here too)
        return self._common("timedelta", pd.to_timedelta, "timedelta")

    def load_states(self):
        for model in self.models.values():
            model.load_state()

    def save_states(self):
        for model in self.models.values():
            model.save_state()

    def set_datetime(self, timestamp):
        for model in self.models.values():
            model.datetime = timestamp

    def init_states(self, streamflow):
        for model in self.models.values():
            model.init_states(o_t_next=streamflow[model.reach_ids])

    def dump_model_collection(self, file_path, model_file_paths={}, dump_optional=True):  # noqa: B006
        connections = {}
        for model in self.models.values():
            for link in list(model.sinks) + list(model.sources):
                connections.setdefault(link.name, {
                    "upstream_model": link.upstream_model.name,
                    "downstream_model": link.downstream_model.name,
                    "upstream_index": int(link.upstream_index),
                    "downstream_index": int(link.downstream_index),
                })
        models = {name: {"model": model.info,
                         "sinks": [link.name for link in model.sinks],
                         "sources": [link.name for link in model.sources]}
                  for name, model in self.models.items()}
        with open(file_path, "w") as f:
            json.dump({"models": models, "connections": connections}, f, cls=ModelEncoder)

    @classmethod
    def from_file(cls, file_path, load_optional=True, **kwargs):
        return cls(load_model_collection(file_path, load_optional=load_optional), **kwargs)


# -- model files (reference :839-944) ----------------------------------------------------------
def load_model_file(file_path, load_optional=True):
    with open(file_path, "r") as f:
        obj = json.load(f, cls=ModelDecoder)
    if not REQUIRED_FIELDS.issubset(obj.keys()):
        raise ValueError(f"Model field must contain fields {set(REQUIRED_FIELDS)}")
    for key, dtype in (("startnodes", np.int64), ("endnodes", np.int64), ("K", np.float64),
                       ("X", np.float64), ("o_t", np.float64)):
        obj[key] = np.asarray(obj[key], dtype=dtype)
    sizes = {obj[key].size for key in ("startnodes", "endnodes", "K", "X", "o_t")}
    if len(sizes) != 1:
        raise ValueError("Arrays are not the same length")
    obj["n"] = obj["startnodes"].size
    if load_optional:
        return obj
    # (reference behaviour: without optional fields, the REQUIRED ones are dropped)
    return {k: v for k, v in obj.items() if k not in REQUIRED_FIELDS}


def dump_model_file(obj, file_path, dump_optional=True):
    to_dump = obj if dump_optional else {k: v for k, v in obj.items() if k in REQUIRED_FIELDS}
    with open(file_path, "w") as f:
        json.dump(to_dump, f, cls=ModelEncoder)


def load_nhd_geojson(file_path):
    """NHD flowline export (features with COMID / toCOMID / Shape_Length attributes and path
    geometry) -> model description with the reference NHD defaults K = 3600 s, X = 0.29,
    o_t = 1e-3 (reference :879-917).  Reaches draining outside the file become outlets."""
    with open(file_path, "r") as f:
        features = json.load(f)["features"]
    comids = [feat["attributes"]["COMID"] for feat in features]
    to_comids = [feat["attributes"]["toCOMID"] for feat in features]
    paths = [np.asarray(feat["geometry"]["paths"]) for feat in features]
    dx = np.asarray([feat["attributes"]["Shape_Length"] for feat in features])
    position = pd.Series(np.arange(len(comids)), index=comids)
    startnodes = position.reindex(comids, fill_value=-1).values
    endnodes = position.reindex(to_comids, fill_value=-1).values
    outside = endnodes == -1
    endnodes[outside] = startnodes[outside]
    n = startnodes.size
    return {
        "name": str(uuid.uuid4()),
        "datetime": DEFAULT_START_TIME,
        "timedelta": DEFAULT_TIMEDELTA,
        "reach_ids": [str(c) for c in comids],
        "startnodes": startnodes,
        "endnodes": endnodes,
        "K": np.full(n, 3600.0),
        "X": np.full(n, 0.29),
        "o_t": np.full(n, 1e-3),
        "dx": dx,
        "paths": paths,
    }


def load_model_collection(file_path, load_optional=True):
    with open(file_path, "r") as f:
        info = json.load(f, cls=ModelDecoder)
    models = {}
    for entry in info["models"].values():
        model = Muskingum(entry["model"], load_optional=load_optional)
        models[model.name] = model
    for link_name, link in info["connections"].items():
        upstream = models[link["upstream_model"]]
        downstream = models[link["downstream_model"]]
        connection = Connection(upstream, downstream, link["upstream_index"],
                                link["downstream_index"], name=link_name)
        upstream.sinks.append(connection)
        downstream.sources.append(connection)
    return list(models.values())
