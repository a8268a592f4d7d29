"""Synthetic river networks and forcing (bench / tests; no NHD data ships with the repo).

``river_network`` builds a forest of drainage basins with the "main stem + recursive
tributaries" structure of real networks: basin sizes are heavy-tailed, every chain's length
follows Hack's law (length ~ c * area^0.6) capped by a basin depth budget, and the reach indices
are randomly permuted so that index order is NOT topological order (as with NHD COMIDs).
Outlets are self loops, the reference's convention (muskingum.py:899-902).

Sizes follow SURVEY.md §8(d): HUC-8 ~1k reaches, Texas ~190k reaches / ~300 outlets, CONUS
~2.7M reaches.  Depth is a parameter (no real network is available to calibrate it).
"""
from __future__ import annotations

import numpy as np
import pandas as pd

HACK_EXPONENT = 0.6


def random_forest(n, n_outlets, rng, p_chain=0.0, window=4):
    """Simple random forest in topological order, then permuted.  Node k >= n_outlets drains to
    one of the `window` previous nodes with probability p_chain (long chains), otherwise to a
    uniformly random earlier node."""
    n_outlets = max(1, min(n_outlets, n))
    parent = np.empty(n, dtype=np.int64)
    parent[:n_outlets] = np.arange(n_outlets)
    k = np.arange(n_outlets, n)
    if k.size:
        chain = rng.random(k.size) < p_chain
        near = k - 1 - rng.integers(0, np.minimum(window, k))
        far = (rng.random(k.size) * k).astype(np.int64)
        parent[n_outlets:] = np.where(chain, near, far)
    return _permute(parent, rng)


def fan_in_forest(n, rng, hubs=6, max_fan=30):
    """random_forest plus a few hub reaches of large fan-in (5 .. max_fan upstreams): some
    headwaters are re-pointed at each hub (a headwater has no upstream, so no cycle forms)."""
    end = random_forest(n, 2, rng, p_chain=0.9)
    ids = np.arange(n)
    for hub in rng.choice(n, size=min(hubs, n), replace=False):
        deg = np.bincount(end[end != ids], minlength=n)
        cand = np.flatnonzero((deg == 0) & (ids != hub) & (ids != end[hub]))
        fan = min(int(rng.integers(5, max_fan + 1)), cand.size)
        end[rng.choice(cand, size=fan, replace=False)] = hub
    return end


def _permute(parent, rng):
    n = parent.size
    perm = rng.permutation(n)
    end = np.empty(n, dtype=np.int64)
    end[perm] = perm[parent]
    return end


def _basin_sizes(n, n_basins, rng, largest_frac):
    """Heavy-tailed basin sizes summing to n with the largest ~ largest_frac * n."""
    n_basins = max(1, min(n_basins, n))
    w = rng.pareto(1.1, size=n_basins) + 1.0
    w = np.sort(w)[::-1]
    w[0] = 0.0
    rest = n - max(1, int(round(largest_frac * n)))
    sizes = np.maximum(1, np.floor(w / max(w[1:].sum(), 1e-12) * rest)).astype(np.int64)
    sizes[0] = n - sizes[1:].sum()
    if sizes[0] < 1:  # tiny n: fall back to an even split
        sizes = np.full(n_basins, n // n_basins, dtype=np.int64)
        sizes[: n - sizes.sum()] += 1
    return sizes


def river_network(n, n_basins, max_depth, rng, largest_frac=0.2, hack_c=None):
    """Forest of `n` reaches in `n_basins` basins; the deepest flow path has ~max_depth reaches.

    Returns endnodes (int64, caller order, outlets are self loops)."""
    sizes = _basin_sizes(n, n_basins, rng, largest_frac)
    if hack_c is None:
        hack_c = max_depth / max(float(sizes.max()), 1.0) ** HACK_EXPONENT
    parent = np.empty(n, dtype=np.int64)
    nxt = 0
    for m in sizes:
        nxt = _build_basin(int(m), nxt, parent, max_depth, hack_c, rng)
    assert nxt == n
    return _permute(parent, rng)


def _build_basin(m, base, parent, max_depth, hack_c, rng):
    """Fill parent[base:base+m] with one basin; returns the next free index."""
    # work items: (size, downstream node or -1, distance of the chain's first reach to outlet)
    stack = [(m, -1, 0)]
    nxt = base
    while stack:
        size, down, dist0 = stack.pop()
        budget = max(1, max_depth - dist0)
        L = int(min(size, budget, max(1, round(hack_c * size ** HACK_EXPONENT))))
        chain = np.arange(nxt, nxt + L)
        parent[chain[0]] = down if down >= 0 else chain[0]
        parent[chain[1:]] = chain[:-1]
        nxt += L
        rest = size - L
        while rest > 0:
            s = int(min(rest, max(1, round(rest * rng.beta(0.6, 2.0)))))
            # stem reach the tributary drains into, leaving the tributary some depth budget
            at = int(rng.integers(0, max(1, min(L, max_depth - dist0 - 1))))
            d = dist0 + at + 1
            stack.append((s, int(chain[at]), d))
            rest -= s
    return nxt


def heights(endnodes):
    """Longest upstream path (in reaches) for every reach (0 = headwater)."""
    end = np.asarray(endnodes, dtype=np.int64)
    n = end.size
    indeg = np.bincount(end, minlength=n) - (end == np.arange(n))
    h = np.zeros(n, dtype=np.int64)
    deg = indeg.copy()
    frontier = np.flatnonzero(deg == 0)
    while frontier.size:
        e = end[frontier]
        ok = e != frontier
        e, src = e[ok], frontier[ok]
        np.maximum.at(h, e, h[src] + 1)
        np.subtract.at(deg, e, 1)
        cand = np.unique(e)
        frontier = cand[deg[cand] == 0]
    return h


def level_histogram(endnodes):
    h = heights(endnodes)
    return np.bincount(h)


def model_arrays(n, seed=0, kind="random"):
    """Muskingum parameters per SURVEY §8(d): kind 'nhd' (K=3600 s, X=0.29, muskingum.py:911-912)
    or 'random' (K~U(1800,7200) s, X~U(0.1,0.4)); initial outflow o~U(0.5,5) m3/s."""
    if kind == "nhd":
        K = np.full(n, 3600.0)
        X = np.full(n, 0.29)
    else:
        K = np.random.default_rng(seed + 2).uniform(1800.0, 7200.0, n)
        X = np.random.default_rng(seed + 3).uniform(0.1, 0.4, n)
    o0 = np.random.default_rng(seed + 4).uniform(0.5, 5.0, n)
    return K, X, o0


def forcing(n, rows=25, seed=1, start="2024-05-01T00:00:00", freq="1h"):
    """Hourly lateral inflow q ~ Gamma(k=2, theta=0.5) m3/s (qSfcLatRunoff + qBucket shape,
    download.py:176-197).  Returns (index_ns int64 [rows], values [rows][n])."""
    idx = pd.date_range(start, periods=rows, freq=freq, tz="UTC")
    vals = np.random.default_rng(seed).gamma(2.0, 0.5, size=(rows, n))
    return idx.asi8.copy(), vals


def ensemble(o0, fp, members, seed=5, cols=None):
    """Ensemble inputs: member forcing = base x lognormal(0, 0.3) multiplier per
    (reach, member), constant in time (seed 5); initial state the same way (seed 6).
    Returns (o0 [n][E], fp [rows][n][E]) in the member-innermost layout of mcroute.h; `cols`
    (a slice of the members) gives one rank's share of the same ensemble."""
    n = o0.size
    cols = slice(0, members) if cols is None else cols
    m_f = np.random.default_rng(seed).lognormal(0.0, 0.3, (n, members))[:, cols]
    m_o = np.random.default_rng(seed + 1).lognormal(0.0, 0.3, (n, members))[:, cols]
    fpe = np.ascontiguousarray(fp[:, :, None] * m_f[None, :, :])
    return np.ascontiguousarray(o0[:, None] * m_o), fpe


def texas(seed=0, n=190_000, n_basins=300, max_depth=1500):
    """Texas-scale synthetic network: ~190k reaches, ~300 outlets."""
    return river_network(n, n_basins, max_depth, np.random.default_rng(seed))


def huc8(seed=0, n=1000, max_depth=100):
    return river_network(n, 1, max_depth, np.random.default_rng(seed), largest_frac=1.0)
