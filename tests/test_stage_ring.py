"""CPU model of the LDS-ring staging of the skewed member windows (flow.hip member_inputs_ring /
member_unpack_ring): per group of 16 slots, the rounds of 4 x kStageLoads members, the LDS ring
slots they land in, and the window rows stored after each round.  Driven by the C++ plan of the
Texas-size network (wide groups included), every (slot, member) cell must be stored exactly once,
from the ring slot its member was staged in and not yet overwritten; the unpack side must write
each member exactly once after all of its cells were read."""
import numpy as np
import pytest

from tx_fast_hydrology_amd import engine, synthetic

SLOTS, RING, CHUNK = 16, 32, 16            # kStageSlots, kStageRing, kStageChunk (flow.hip)


def _inputs_group(gs, real, E):
    """Returns {(s, e): row} stored by one wave, checking the ring at every read."""
    glo, ghi = gs[real].min(), gs[real].max()
    out = {}
    if ghi - glo > RING - CHUNK:                          # wide group: direct stores
        for s in np.flatnonzero(real):
            for e in range(E):
                out[(s, e)] = gs[s] + e
        return out, True
    ring = -np.ones((RING, SLOTS), int)                   # member held by each ring slot
    nxt, rend = glo, ghi + E
    for e0 in range(0, E, CHUNK):
        for e in range(e0, min(e0 + CHUNK, E)):
            ring[e % RING, real] = e
        staged = min(e0 + CHUNK, E)
        rstop = rend if staged >= E else glo + staged
        for r in range(nxt, rstop):
            for s in np.flatnonzero(real):
                e = r - gs[s]
                if 0 <= e < E:
                    assert ring[e % RING, s] == e, (r, s, e)
                    assert (s, e) not in out
                    out[(s, e)] = r
        nxt = max(nxt, rstop)
    return out, False


def _unpack_group(gs, real, E):
    """Members written by one wave (ring form): each once, after all its cells were read."""
    glo, ghi = gs[real].min(), gs[real].max()
    if ghi - glo > RING - CHUNK:
        return False
    ring = -np.ones((RING, SLOTS), int)
    rend, done, written = ghi + E, 0, []
    for r0 in range(glo, rend, CHUNK):
        for r in range(r0, min(r0 + CHUNK, rend)):
            for s in np.flatnonzero(real):
                e = r - gs[s]
                if 0 <= e < E:
                    ring[e % RING, s] = e
        upto = min(min(r0 + CHUNK, rend) - ghi, E)
        for e in range(done, upto):
            assert (ring[e % RING, real] == e).all(), e
            written.append(e)
        done = max(done, upto)
    assert written == list(range(E))
    return True


@pytest.mark.parametrize("E", [128, 137, 256])
def test_stage_ring_covers_every_cell_once(E):
    end = synthetic.river_network(40_000, 60, 600, np.random.default_rng(0))
    n = end.size
    start = np.arange(n)
    indeg = np.bincount(end, minlength=n) - (end == start)
    plan = engine.Plan(end, indeg, start[indeg == 0], slots=192, tile=16, chain=2)
    info = plan.info
    G = plan.export()["G"]
    flags = plan.export_links()["flags"]
    rs = info["chain"] * info["slots"]
    ns = info["nslots"]
    assert rs % SLOTS == 0 and ns % SLOTS == 0
    gmin = np.array([G[w * rs:(w + 1) * rs][flags[w * rs:(w + 1) * rs] != 0].min()
                     if (flags[w * rs:(w + 1) * rs] != 0).any() else 0
                     for w in range(info["nwg"])])
    wide = ring = 0
    rng = np.random.default_rng(E)
    groups = np.arange(ns // SLOTS)
    # every wide group plus a sample of the others (the full set takes minutes in Python)
    spreads = []
    for g in groups:
        sl = slice(g * SLOTS, (g + 1) * SLOTS)
        real = flags[sl] != 0
        spreads.append(np.ptp(G[sl][real]) if real.any() else -1)
    spreads = np.array(spreads)
    pick = np.union1d(np.flatnonzero(spreads > RING - CHUNK),
                      rng.choice(np.flatnonzero((spreads >= 0) & (spreads <= RING - CHUNK)),
                                 200, replace=False))
    for g in pick:
        d0 = g * SLOTS
        w = d0 // rs
        real = flags[d0:d0 + SLOTS] != 0
        gs = np.where(real, G[d0:d0 + SLOTS] - gmin[w], 0)
        cells, is_wide = _inputs_group(gs, real, E)
        assert len(cells) == real.sum() * E
        for (s, e), r in cells.items():
            assert r == gs[s] + e
        assert _unpack_group(gs, real, E) == (not is_wide)
        wide += is_wide
        ring += not is_wide
    assert wide > 0 and ring > 0
