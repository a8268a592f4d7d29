"""Sub-basin simulation drivers (reference ``tx_fast_hydrology/simulation.py``).

``AsyncSimulation`` routes a ``ModelCollection`` (from ``Muskingum.split`` or a collection
file) in dependency order: every sub-basin whose upstream sub-basins are done is simulated (one
fused device horizon per sub-basin when it has no callbacks), then its outlet series is turned
into the lateral-inflow correction of the downstream entry reach,
``alpha * I / gamma + beta * I_prev / gamma`` (reference ``simulation.py:137-166``), which
makes the collection reproduce the routing of the whole network.

When no sub-basin has callbacks, the collection runs as a device DAG instead: every
sub-basin's horizon is launched on its own session stream in dependency order, each cut edge's
correction is added on the device into the downstream session's forcing
(``RoutingNet.add_lateral_correction``, ordered by stream events), and the outflows are fetched
only after every launch -- no host round trip between sub-basins, independent sub-basins run
concurrently.  The corrections are applied in the order the reference's task group applies them
(its FIFO schedule is replayed on the host), so results are bit-identical to the host driver.

``CheckPoint`` saves the model state once at a checkpoint time (reference :169-211).
"""
from __future__ import annotations

import asyncio
import datetime
import logging

import numpy as np
import pandas as pd

from .callbacks import BaseCallback
from .muskingum import _host_array, _upload_forcing

logger = logging.getLogger(__name__)


class _TaskGroup:
    """``asyncio.TaskGroup`` for Python < 3.11: waits for every task created inside it, tasks
    included that other tasks create; the first failure cancels the rest and is re-raised."""

    async def __aenter__(self):
        self._tasks = set()
        return self

    def create_task(self, coro):
        task = asyncio.get_running_loop().create_task(coro)
        self._tasks.add(task)
        return task

    async def __aexit__(self, exc_type, exc, tb):
        while self._tasks:
            done, _ = await asyncio.wait(self._tasks, return_when=asyncio.FIRST_EXCEPTION)
            self._tasks -= done
            failed = [t for t in done if not t.cancelled() and t.exception() is not None]
            if failed:
                for task in self._tasks:
                    task.cancel()
                if self._tasks:
                    await asyncio.wait(self._tasks)
                raise failed[0].exception()
        return False


TaskGroup = getattr(asyncio, "TaskGroup", _TaskGroup)


class Simulation:
    """A model collection plus its lateral-input frames, one per sub-basin (columns cropped to
    the sub-basin's reach ids)."""

    def __init__(self, model_collection, inputs):
        self.model_collection = model_collection
        self.models = model_collection.models
        self.inputs = self.load_inputs(inputs)
        self.outputs = {}

    def load_inputs(self, inputs):
        return {name: inputs[model.reach_ids].copy() for name, model in self.models.items()}

    def simulate(self):
        # the reference's synchronous driver is disabled (simulation.py:26-27)
        raise NotImplementedError

    @property
    def datetime(self):
        return self.model_collection.datetime

    def load_states(self):
        self.model_collection.load_states()

    def save_states(self):
        self.model_collection.save_states()

    def init_states(self, streamflow):
        self.model_collection.init_states(streamflow)

    def set_datetime(self, timestamp):
        self.model_collection.set_datetime(timestamp)


class AsyncSimulation(Simulation):
    """Dependency-ordered asyncio driver; ``outputs[name]`` is the outflow frame of each
    sub-basin (start time row included).

    Memory note (device DAG): the outflow frames of one ``simulate`` are views into ONE
    page-locked host block (so all fetches are asynchronous, full-speed copies).  Any frame kept
    alive keeps that whole block alive, and torch's caching host allocator keeps page-locked
    memory cached for reuse by later horizons rather than returning it to the OS.  Callers that
    keep results of large collections for long should copy the frames they keep
    (``frame.copy()``) and drop the rest."""

    async def simulate(self):
        try:
            asyncio.get_running_loop()
        except RuntimeError:
            asyncio.run(self._main())
        else:
            await self._main()
        return self.outputs

    async def _main(self):
        if _device_dag(self):
            return
        self._indegree = {model.name: len(model.sources)
                          for model in self.model_collection.models.values()}
        async with TaskGroup() as taskgroup:
            for name, pending in self._indegree.items():
                if pending == 0:
                    taskgroup.create_task(self._simulate(taskgroup, self.models[name],
                                                         self.inputs[name], name))

    async def _simulate(self, taskgroup, model, inputs, name):
        logger.debug(f"Started job for sub-watershed {name}")
        self.outputs[name] = _outflow_frame(model, inputs)
        taskgroup.create_task(self._accumulate(taskgroup, self.outputs[name], name))

    async def _accumulate(self, taskgroup, outputs, name):
        """Fold this sub-basin's outlet series into every downstream sub-basin's inputs and
        start each downstream sub-basin whose last upstream this was."""
        upstream = self.models[name]
        for link in upstream.sinks:
            target = link.downstream_model.name
            if target == name:
                continue
            frame = self.inputs[target]
            column = link.downstream_model.reach_ids[link.downstream_index]
            series = outputs[upstream.reach_ids[link.upstream_index]]
            frame.loc[:, column] += _lateral_correction(link.downstream_model,
                                                        link.downstream_index, series)
            self._indegree[target] -= 1
            if not self._indegree[target]:
                taskgroup.create_task(self._simulate(taskgroup, link.downstream_model, frame,
                                                     target))
        logger.debug(f"Finished job for sub-watershed {name}")


def _task_order(sim):
    """Replay of the reference task group's FIFO schedule (simulation.py:110-166): the order
    the sub-basins run in and, per downstream sub-basin, the order its corrections arrive."""
    from collections import deque
    indeg = {m.name: len(m.sources) for m in sim.models.values()}
    ready = deque(("sim", name) for name, k in indeg.items() if k == 0)
    runs, corrections = [], {name: [] for name in sim.models}
    while ready:
        kind, name = ready.popleft()
        if kind == "sim":
            runs.append(name)
            ready.append(("acc", name))
            continue
        for link in sim.models[name].sinks:
            target = link.downstream_model.name
            if target == name:
                continue
            corrections[target].append(link)
            indeg[target] -= 1
            if not indeg[target]:
                ready.append(("sim", target))
    return runs, corrections


def _step_ns(model, end_time):
    """Step times of simulate_iter's loop (``while t < end_time: t = t + timedelta``,
    muskingum.py:527-533) as int64 ns: Timestamp arithmetic is exact integer nanoseconds, so the
    k-th step is t0 + k * dt for k = 1 .. ceil((end - t0) / dt)."""
    t0 = int(model.datetime.value)
    dt = int(model.timedelta.value)
    end = int(pd.Timestamp(end_time).value)
    if dt <= 0:
        raise ValueError("the model timedelta must be positive")
    k = -(-(end - t0) // dt) if end > t0 else 0
    return t0 + dt * np.arange(1, k + 1, dtype=np.int64)


class _Phases:
    """Wall-clock breakdown of one device-DAG pass (``AsyncSimulation.dag_phases``)."""

    def __init__(self):
        import time
        self._clock = time.perf_counter
        self._t = self._clock()
        self.ms = {}

    def __call__(self, name):
        t = self._clock()
        self.ms[name] = self.ms.get(name, 0.0) + 1e3 * (t - self._t)
        self._t = t


def _device_dag(sim):
    """Route the collection as a device DAG (module docstring).  Returns False, having changed
    nothing, when the host driver must run it: callbacks bound, a session that is not a device
    session, an empty horizon, forcing rows that do not match the upstream horizon, or a
    sub-basin horizon that was re-routed after its dataflow waits gave up.  The wall-clock
    phases of the pass are left in ``sim.dag_phases`` (ms)."""
    ph = _Phases()
    models = sim.models
    if any(m.callbacks for m in models.values()):
        return False
    runs, corrections = _task_order(sim)
    if len(runs) != len(models):
        return False
    steps = {}
    for name in runs:
        inputs = sim.inputs[name]
        if not isinstance(inputs.index, pd.DatetimeIndex) or inputs.index.tz is None:
            return False
        steps[name] = _step_ns(models[name], inputs.index.max())
        if not steps[name].size:
            return False
    for name in runs:
        for link in corrections[name]:
            if len(sim.inputs[name]) != steps[link.upstream_model.name].size:
                return False
    nets = {}
    for name in runs:
        models[name]._settle_inflows()      # rows a fused horizon left on the session
        net = models[name]._device.session(models[name])
        if not hasattr(net, "add_lateral_correction"):
            return False
        nets[name] = net
    ph("sessions")
    before = {name: nets[name].reroutes() for name in runs}
    start = {name: (models[name].datetime, models[name].o_t_next, models[name].i_t_next)
             for name in runs}
    for name in runs:
        m, inputs, net = models[name], sim.inputs[name], nets[name]
        _upload_forcing(net, inputs.index.asi8.astype(float), inputs)
        net.set_state(m.o_t_next, m.i_t_next)
    ph("upload")
    # enqueue: corrections then the horizon of every sub-basin, in the reference's order
    for name in runs:
        m, net = models[name], nets[name]
        for link in corrections[name]:
            up = link.upstream_model
            j = link.downstream_index
            net.add_lateral_correction(j, nets[up.name], link.upstream_index,
                                       start[up.name][1][link.upstream_index], m.alpha[j],
                                       m.beta[j], m.gamma[j])
        net.run(steps[name].astype(float))
    ph("enqueue")
    # outflow series straight into the frames' arrays (row 0: the start state); of the inflows
    # only the last two steps (the final state) are needed.  All of them are views of two
    # pinned host blocks, so every copy is asynchronous and runs at full PCIe speed (pageable
    # destinations made each of the ~700 small copies a synchronous staged transfer)
    sizes = {name: ((steps[name].size + 1) * models[name].n,
                    min(steps[name].size, 2) * models[name].n) for name in runs}
    big_o = _host_array((max(sum(a for a, _ in sizes.values()), 1),), np.float64)
    big_i = _host_array((max(sum(b for _, b in sizes.values()), 1),), np.float64)
    series, last_i, tickets = {}, {}, []
    po = pi = 0
    for name in runs:
        T, n = steps[name].size, models[name].n
        k = min(T, 2)
        o = big_o[po:po + (T + 1) * n].reshape(T + 1, n)
        li = big_i[pi:pi + k * n].reshape(k, n)
        po += (T + 1) * n
        pi += k * n
        o[0] = start[name][1]
        tickets.append((nets[name], nets[name].fetch_outputs_async(0, T, o[1:], None)))
        tickets.append((nets[name], nets[name].fetch_outputs_async(T - k, T, None, li)))
        series[name], last_i[name] = o, li
    ph("fetch_enqueue")
    for net, tk in tickets:
        net.fetch_wait(tk)
    ph("fetch_wait")
    if any(nets[name].reroutes() != before[name] for name in runs):
        # a horizon whose dataflow waits gave up (the device was shared) was re-routed by its
        # own session at the fetch, but the corrections its downstream sub-basins took from it
        # on the device used incomplete outflows (mcroute.h mc_net_lateral_correction).  Nothing
        # of this pass has reached the models or the frames yet: route the collection with the
        # host driver instead, which reloads every session's forcing and state
        logger.warning("device DAG: a sub-basin horizon gave up waiting and was re-routed; "
                       "routing the collection with the host driver")
        sim.dag_phases = ph.ms
        return False
    indexes = {}
    for name in runs:
        m, inputs = models[name], sim.inputs[name]
        t0, o0, i0 = start[name]
        o, li = series[name], last_i[name]
        T = steps[name].size
        # the state simulate_iter leaves (muskingum.py:458-464 per step): arrays of its own
        m.o_t_prev, m.i_t_prev = (o[-2].copy(), li[-2].copy()) if T > 1 else (o0, i0)
        m.o_t_next, m.i_t_next = o[-1].copy(), li[-1].copy()
        m.datetime = pd.Timestamp(int(steps[name][-1]), tz="UTC")
        key = (int(t0.value), T, int(steps[name][0]), int(steps[name][-1]))
        index = indexes.get(key)
        if index is None:
            ns = np.concatenate([[int(t0.value)], steps[name]])
            index = indexes[key] = pd.DatetimeIndex(ns.view("datetime64[ns]")).tz_localize("UTC")
        sim.outputs[name] = pd.DataFrame(o, index=index, columns=inputs.columns, copy=False)
    ph("frames")
    # the corrected input frames, as the reference's += leaves them: the same arithmetic as
    # _lateral_correction, on the fetched arrays (no Series round trips)
    for name in runs:
        frame = sim.inputs[name]
        for link in corrections[name]:
            up = link.upstream_model
            I = series[up.name][:, link.upstream_index]
            k = frame.columns.get_loc(models[name].reach_ids[link.downstream_index])
            corr = _correction_values(models[name], link.downstream_index, I)
            frame.iloc[:, k] = frame.iloc[:, k].to_numpy() + corr
    ph("corrections")
    sim.dag_phases = ph.ms
    return True


def _outflow_frame(model, inputs):
    """Route ``model`` over its input frame; outflows per timestamp, start time included."""
    rows = {model.datetime: model.o_t_next}
    rows.update((state.datetime, state.o_t_next) for state in model.simulate_iter(inputs))
    frame = pd.DataFrame.from_dict(rows, orient="index")
    frame.index = pd.to_datetime(frame.index, utc=True)
    frame.columns = inputs.columns
    return frame


def _correction_values(model, j, I):
    """_lateral_correction on a plain array I (the outflow series, start row first): now =
    I[1:], before = I[:-1] with NaN -> 0 (shift(1).iloc[1:].fillna(0)), same expression."""
    now = I[1:]
    before = I[:-1]
    before = np.where(np.isnan(before), 0.0, before)
    return model.alpha[j] * now / model.gamma[j] + model.beta[j] * before / model.gamma[j]


def _lateral_correction(model, j, series):
    """Inflow of an upstream outlet series expressed as lateral input of entry reach j:
    alpha I(t) / gamma + beta I(t-1) / gamma with I(t0 - dt) = 0 (simulation.py:152-159, same
    expression and association)."""
    now = series.iloc[1:].values
    before = series.shift(1).iloc[1:].fillna(0.0).values
    return model.alpha[j] * now / model.gamma[j] + model.beta[j] * before / model.gamma[j]


class CheckPoint(BaseCallback):
    """Saves the model state once, at the first step end at or after the checkpoint time, and
    forwards save / load to every bound callback that keeps state (``save_state`` /
    ``load_state``).  ``timedelta`` (seconds) re-arms the checkpoint at each simulation start,
    relative to the model time then."""

    def __init__(self, model, checkpoint_time=None, timedelta=None):
        if checkpoint_time is None and timedelta is None:
            raise ValueError("Either `checkpoint_time` or `timedelta` must not be `None`.")
        self.model = model
        self.timedelta = timedelta
        self.checkpoint_time = (checkpoint_time if checkpoint_time is not None
                                else self._offset(timedelta))
        self.model_saved = False

    def _offset(self, seconds):
        return self.model.datetime + datetime.timedelta(seconds=seconds)

    def __on_simulation_start__(self):
        if self.timedelta is not None:
            self.set_checkpoint(self._offset(self.timedelta))

    def __on_step_end__(self):
        if not self.model_saved and self.model.datetime >= self.checkpoint_time:
            self.model.save_state()
            self.model_saved = True

    def _forward(self, method):
        for callback in self.model.callbacks.values():
            hook = getattr(callback, method, None)
            if hook is not None:
                hook()

    def __on_save_state__(self):
        self._forward("save_state")

    def __on_load_state__(self):
        self._forward("load_state")

    def __idle_steps__(self):
        return self.model_saved

    def set_checkpoint(self, checkpoint_time):
        logger.info(f"Setting checkpoint time to {checkpoint_time}")
        self.checkpoint_time = checkpoint_time
        self.model_saved = False
