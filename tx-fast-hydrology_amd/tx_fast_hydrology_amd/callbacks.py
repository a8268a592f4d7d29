"""Hook protocol of the routing models (reference ``tx_fast_hydrology/callbacks.py:1-20``).

A callback bound with ``Muskingum.bind_callback`` is notified at six points, with the model's
host-visible state (``o_t_next``, ``i_t_next``, ``datetime`` ...) readable and assignable:

=========================  ===================================================================
hook                       fired by (reference line it mirrors)
=========================  ===================================================================
``__on_step_start__``      ``Muskingum.step_iter`` before routing (muskingum.py:454-455)
``__on_step_end__``        ``Muskingum.step_iter`` after the state rotation (:463-464)
``__on_simulation_start__`` ``Muskingum.simulate_iter`` before the first step (:523-524)
``__on_simulation_end__``  ``Muskingum.simulate_iter`` after the last step (:535-536)
``__on_save_state__``      ``Muskingum.save_state`` (:579-580)
``__on_load_state__``      ``Muskingum.load_state`` (:587-588)
=========================  ===================================================================

Every hook is a no-op here; subclasses override the ones they need.  A model with at least one
bound callback routes step by step on the device, so hooks observe every timestep exactly as in
the reference; a model without callbacks may route a whole horizon in one device call.

Extension (not in the reference): ``__idle_steps__`` returns True when the callback's step hooks
will do nothing for the rest of the current simulation (a filter past its last observation, a
checkpoint already taken).  When every bound callback is idle, ``simulate_iter`` routes the
remaining steps as one fused device horizon; the simulation-end hook still fires.  The default
is False (always step by step).
"""


class BaseCallback:
    """Base class of everything ``Muskingum.bind_callback`` accepts."""

    def __init__(self, *args, **kwargs):
        pass

    def __on_step_start__(self):
        return None

    def __on_step_end__(self):
        return None

    def __on_save_state__(self):
        return None

    def __on_load_state__(self):
        return None

    def __on_simulation_start__(self):
        return None

    def __on_simulation_end__(self):
        return None

    def __idle_steps__(self):
        return False
