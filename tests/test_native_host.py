"""Host-side checks of libmcroute.so that need no GPU: the library loads, exports every symbol
declared in include/mcroute.h, and the topology compiler (plan.cpp) honours its invariants."""
import os
import re

import numpy as np
import pytest

from oracle import oracle as orc
from tx_fast_hydrology_amd import _native as nat
from tx_fast_hydrology_amd.engine import Plan
from tx_fast_hydrology_amd import synthetic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    text = open(os.path.join(ROOT, "include", "mcroute.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mc_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_header_symbol():
    L = nat.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(nat.SIGNATURES), set(syms) ^ set(nat.SIGNATURES)
    assert L.mc_version() == 101


def _replay_rank(heads, endnodes, indegree):
    """Independent replay of nutils.py:72-88 recording the processing order."""
    deg = list(indegree)
    rank = [-1] * len(endnodes)
    r = 0
    for s in heads:
        while deg[s] == 0:
            rank[s] = r
            r += 1
            e = endnodes[s]
            deg[e] -= 1
            s = e
    return np.array(rank)


def _check_plan(endnodes, indegree, heads, **kw):
    """Plan invariants; returns (info, export)."""
    P = Plan(endnodes, indegree, heads, **kw)
    info = P.info
    ex = P.export()
    n = len(endnodes)
    assert np.array_equal(ex["rank"], _replay_rank(heads, endnodes, indegree))
    assert info["n_routed"] == int((ex["rank"] >= 0).sum())
    # every reach has exactly one slot, slots map back
    assert np.array_equal(ex["slot_reach"][ex["pos"]], np.arange(n))
    G = np.full(n, -1)
    G[ex["slot_reach"][ex["slot_reach"] >= 0]] = ex["G"][ex["slot_reach"] >= 0]
    slots = info["slots"]
    tile = info["tile"]
    # schedule: no consumer runs before its producer (same tick only inside a fused lane pair)
    rank = ex["rank"]
    for u in range(n):
        e = endnodes[u]
        if rank[u] >= 0 and e != u:
            assert G[e] - G[u] >= 0
    # node level (reaches and partial-sum slots): at most 4 inputs per slot; an input from
    # the same workgroup has unit slack, one from another workgroup slack >= tile
    ln = P.export_links()
    Gs = ex["G"].astype(np.int64)
    assert (ln["up_cnt"] <= 4).all()
    assert int((ln["flags"] == 3).sum()) == info["n_partial"]
    assert (ex["slot_reach"][ln["flags"] == 3] == -1).all()
    rs = info["chain"] * slots
    for d in np.flatnonzero(ln["up_cnt"]):
        w = d // rs
        for c in range(int(ln["up_cnt"][d])):
            code = int((ln["up4"][d] >> np.uint64(16 * c)) & np.uint64(0xFFFF))
            if code == 0x7FFF:                      # chained edge: the lane's previous position
                assert d % rs >= slots
                assert Gs[d] == Gs[d - slots] and ln["flags"][d - slots] != 0
            elif code & 0x8000:
                row = int(ln["ext_src"][ln["ext_off"][w] + (code & 0x7FFF)])
                src = ex["pos"][row] if row < n else row - n
                assert Gs[d] - Gs[src] >= tile, (d, src)
                assert ln["ext_g"][ln["ext_off"][w] + (code & 0x7FFF)] == Gs[d]
            else:
                src = w * rs + code
                assert code < rs and Gs[d] - Gs[src] == 1, (d, src)
    assert info["gmax"] == G.max() if n else True
    return info, ex


@pytest.mark.parametrize("slots,tile,chain", [(64, 1, 2), (64, 8, 2), (256, 32, 2), (512, 64, 2),
                                              (64, 8, 1), (64, 16, 3), (128, 16, 4),
                                              (256, 32, 4)])
def test_plan_invariants_random(slots, tile, chain):
    rng = np.random.default_rng(slots + tile)
    for trial in range(3):
        n = int(rng.integers(1, 3000))
        end = synthetic.random_forest(n, int(rng.integers(1, 5)), rng, p_chain=0.9)
        deg = orc.compute_indegree(np.arange(n), end)
        heads = np.flatnonzero(deg == 0)
        _check_plan(end, deg, heads, slots=slots, tile=tile, chain=chain)


@pytest.mark.parametrize("slots,tile,chain", [(64, 1, 2), (64, 8, 2), (128, 16, 2), (256, 32, 2),
                                              (64, 16, 3), (128, 16, 4)])
def test_plan_partial_sums_high_fan_in(slots, tile, chain):
    rng = np.random.default_rng(slots * 3 + tile)
    end = synthetic.fan_in_forest(2500, rng)
    deg = orc.compute_indegree(np.arange(end.size), end)
    assert deg.max() > 4
    info, ex = _check_plan(end, deg, np.flatnonzero(deg == 0), slots=slots, tile=tile,
                           chain=chain)
    assert info["n_partial"] > 0


def test_plan_golden_edge_topologies(golden):
    g = golden("g8_ax_bu_edge.npz")
    for name in g["names"]:
        _check_plan(g[f"{name}_endnodes"], g[f"{name}_indegree"], g[f"{name}_heads"])


@pytest.mark.parametrize("chain", [1, 2, 3, 4])
def test_plan_deep_chain_and_capacity(chain):
    n = 5000
    end = np.arange(1, n + 1)
    end[-1] = n - 1                       # one 5000-reach chain
    deg = orc.compute_indegree(np.arange(n), end)
    info, ex = _check_plan(end, deg, np.flatnonzero(deg == 0), slots=256, tile=16, chain=chain)
    assert info["max_height"] == n - 1 and info["chain"] == chain
    assert info["nwg"] >= n // (256 * chain)        # `chain` node slots per lane
    # lane chains divide the chain: one tick per lane, plus the cross-cluster slack
    assert info["n_pairs"] >= n - n // chain - chain * info["nwg"]
    assert (n - 1) // chain <= info["gmax"] < (n - 1) // chain + 16 * (info["nwg"] + 1)


def test_plan_chain_rejects_out_of_range():
    with pytest.raises(nat.TopologyError):
        Plan(np.array([0]), np.array([0]), np.array([0]), chain=5)


def test_plan_rejects_bad_input():
    with pytest.raises(nat.TopologyError):
        Plan(np.array([0, 5]), np.array([1, 0]), np.array([1]))       # endnode out of range
    with pytest.raises(nat.TopologyError):
        Plan(np.array([1, 1]), np.array([0, 0]), np.array([0, 0]))    # duplicate headwater
    with pytest.raises(nat.TopologyError):                            # indegree too small
        Plan(np.array([2, 2, 2]), np.array([0, 0, 1]), np.array([0, 1]))


def test_plan_empty_network():
    P = Plan(np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.int64))
    assert P.info["n"] == 0


@pytest.mark.parametrize("rows,n", [(1, 1), (1, 7), (3, 1000), (2, 190_001), (5, 0)])
def test_host_digest_matches_restatement(rows, n):
    """mc_host_digest (the edit detector of the drop-in API's fused horizons, also formed on the
    device for every fetched row) equals its NumPy restatement, with NaN / Inf / -0.0 rows."""
    from api_helpers import digest_rows
    from tx_fast_hydrology_amd import engine
    rng = np.random.default_rng(rows * 7 + n)
    a = rng.normal(0, 10, (rows, n))
    if n > 3:
        a[0, :3] = [np.nan, -np.inf, -0.0]
    got = engine.host_digest(a)
    assert got.dtype == np.uint64 and got.shape == (rows,)
    assert np.array_equal(got, digest_rows(a) if n else np.zeros(rows, np.uint64))
    if n:
        b = a.copy()
        b[-1, n // 2] = np.nextafter(b[-1, n // 2], np.inf)   # one ulp in one element
        assert engine.host_digest(b)[-1] != got[-1]
        assert np.array_equal(engine.host_digest(b)[:-1], got[:-1])


def test_library_needs_no_vendor_blas_or_solver():
    """Every dense kernel (EnKF analysis, full-covariance KF gain, RTS solve) is the library's
    own: libmcroute.so links the HIP runtime only (no rocBLAS / rocSOLVER)."""
    import shutil
    import subprocess

    from tx_fast_hydrology_amd import _native
    if shutil.which("ldd") is None:
        pytest.skip("ldd not available")
    out = subprocess.run(["ldd", _native.lib_path()], capture_output=True, text=True).stdout
    assert "libamdhip64" in out
    assert "rocblas" not in out and "rocsolver" not in out, out


def test_host_digest_pair_matches_rows():
    from api_helpers import digest_rows
    from tx_fast_hydrology_amd import engine
    rng = np.random.default_rng(3)
    a, b = rng.normal(size=70_001), rng.normal(size=70_001)
    rd = engine.RowDigest()
    assert rd(a, b) == (int(digest_rows(a)[0]), int(digest_rows(b)[0]))
    with pytest.raises(ValueError):
        rd(a[::2], b[::2])
