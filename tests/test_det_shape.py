"""The default resident shape of a single-member session (engine._det_shape): host plans of both
shapes, the one whose schedule ticks a nominal horizon faster -- one compute wave of single-slot
lanes for HUC-8-sized networks, 192 lanes x 2 for larger ones (profiles/r05v_shapes.txt)."""
import numpy as np

from oracle import oracle as orc
from tx_fast_hydrology_amd import engine, synthetic


def _shape(end):
    start = np.arange(end.size)
    deg = orc.compute_indegree(start, end)
    return engine._det_shape(end, deg, start[deg == 0], 0)


def test_small_network_takes_one_wave_of_single_slots():
    assert _shape(synthetic.huc8(seed=0, n=1000, max_depth=100)) == (64, 1)


def test_larger_network_keeps_192_by_2():
    end = synthetic.river_network(30_000, 16, 1500, np.random.default_rng(0))
    assert _shape(end) == (192, 2)


def test_explicit_chain_and_big_networks_skip_the_estimate():
    end = synthetic.huc8(seed=0, n=1000, max_depth=100)
    start = np.arange(end.size)
    deg = orc.compute_indegree(start, end)
    assert engine._det_shape(end, deg, start[deg == 0], 3) == (192, 3)
    big = np.arange(1, engine._DET_SHAPE_MAX_N + 2, dtype=np.int64)
    big[-1] = big.size - 1
    assert engine._det_shape(big, np.ones(big.size, np.int64), np.array([0]), 0) == (192, 0)
