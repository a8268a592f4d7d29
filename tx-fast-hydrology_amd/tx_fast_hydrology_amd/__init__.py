"""MI355X-native Muskingum routing engine with the tx_fast_hydrology API.

The routing hot path (nutils._ax_bu driven by Muskingum.simulate_iter) runs as hand-written HIP
kernels for gfx950 behind the C ABI in include/mcroute.h; this package is the host-side mirror
of the reference's Python interface.
"""
from .engine import Plan, RoutingNet, ax_bu  # noqa: F401

__version__ = "0.1.0"
