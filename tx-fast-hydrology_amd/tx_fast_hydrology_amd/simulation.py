"""Sub-basin simulation drivers (reference ``tx_fast_hydrology/simulation.py``).

``AsyncSimulation`` routes a ``ModelCollection`` (from ``Muskingum.split`` or a collection
file) in dependency order: every sub-basin whose upstream sub-basins are done is simulated (one
fused device horizon per sub-basin when it has no callbacks), then its outlet series is turned
into the lateral-inflow correction of the downstream entry reach,
``alpha * I / gamma + beta * I_prev / gamma`` (reference ``simulation.py:137-166``), which
makes the collection reproduce the routing of the whole network.

``CheckPoint`` saves the model state once at a checkpoint time (reference :169-211).
"""
from __future__ import annotations

import asyncio
import datetime
import logging

import pandas as pd

from .callbacks import BaseCallback

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
    sub-basin (start time row included)."""

    async def simulate(self):
        try:
            asyncio.get_running_loop()
        except RuntimeError:
            asyncio.run(self._main())
        else:
            await self._main()
        return self.outputs

    async def _main(self):
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


def _outflow_frame(model, inputs):
    """Route ``model`` over its input frame; outflows per timestamp, start time included."""
    rows = {model.datetime: model.o_t_next}
    rows.update((state.datetime, state.o_t_next) for state in model.simulate_iter(inputs))
    frame = pd.DataFrame.from_dict(rows, orient="index")
    frame.index = pd.to_datetime(frame.index, utc=True)
    frame.columns = inputs.columns
    return frame


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
