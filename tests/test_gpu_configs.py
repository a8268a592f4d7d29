"""GPU parity at the BASELINE.json config shapes, on exactly the workloads bench.py measures
(bench.build_workload: same synthetic network, plan shape, forcing, members, gauges).

* configs[0] one HUC-8 sub-basin (1000 reaches, one outlet), deterministic, 24 h on the bench
  plan: every step's outflows and inflows and the final state bit-identical to the oracle.
* configs[1] full Texas deterministic: tests/test_gpu_routing.py (bit-exact at full size).

* configs[2] Texas, 64 members, 24 h on the bench's ensemble plan (256 lanes, 64-tick
  launches): every member's final state bit-identical to its serial oracle run, and every step
  of 8 sampled members (nutils.py:64-89 per member).
* configs[3] Texas, 256 members, 500 gauges, R = 1e-2 I: one member step (member dataflow)
  bit-exact for all members, then one analysis through the bench's path
  (ensemble.distributed_analysis) against the NumPy restatement of the ensemble update
  G = A HA^T W / (E - 1), W = (HA HA^T / (E - 1) + R)^-1 (Y - HX) (da.py:112-126 with the
  sample covariance), increments within 1e-10 of max|G|, applied by _apply_gain
  (nutils.py:116-134).
* configs[4] CONUS (2.7M reaches), the bench's 16 members per GPU over the full 288-step
  horizon: sampled members' outputs at steps 0, 143 and 287 and their final states bit-exact.
"""
import numpy as np
import pytest

import bench
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

THREADS = 16


def _coef(wl):
    return wl.alpha, wl.beta, wl.chi, wl.gamma


def _member(a, e):
    return np.ascontiguousarray(a[..., e])


def test_config0_huc8_bench_plan():
    args = bench.parse(["--huc8"], world=1)
    net, wl = bench.build_workload(args)
    n, T = wl.n, wl.x.size
    assert (n, T) == (1000, 288) and int((wl.end == wl.start).sum()) == 1
    net.run(wl.x)
    oo, ii = net.fetch_outputs(0, T)
    so, si = net.get_state()
    want_o, want_i, fo, fi = orc.simulate(wl.start, wl.end, wl.indeg, *_coef(wl), wl.o0, wl.i0,
                                          wl.x, wl.xp, wl.fp)
    assert np.array_equal(oo, want_o) and np.array_equal(ii, want_i)
    assert np.array_equal(so, fo) and np.array_equal(si, fi)
    net.close()


def test_config2_texas_ens64_bench_plan():
    """The bench's ens64 horizon: the multi-launch kernel on the 256-lane / 64-tick plan."""
    args = bench.parse(["--members", "64"], world=1)
    net, wl = bench.build_workload(args)
    assert net.info["slots"] == 256 and net.info["tile"] == 64 and wl.E == 64
    n, T = wl.n, wl.x.size
    assert (n, T) == (190_000, 288)
    net.run(wl.x)
    assert net.mode()[1] == "launches"
    so, si = net.get_state()
    fo, fi = orc.simulate_members(wl.start, wl.end, wl.indeg, *_coef(wl), wl.o0, wl.i0, wl.x,
                                  wl.xp, wl.fp, threads=THREADS)
    assert np.array_equal(so, fo) and np.array_equal(si, fi)
    sample = [0, 9, 18, 27, 36, 45, 54, 63]
    got_o = np.empty((T, n, len(sample)))
    got_i = np.empty((T, n, len(sample)))
    for t0 in range(0, T, 32):
        t1 = min(T, t0 + 32)
        oo, ii = net.fetch_outputs(t0, t1)
        got_o[t0:t1] = oo[:, :, sample]
        got_i[t0:t1] = ii[:, :, sample]
        del oo, ii
    for k, e in enumerate(sample):
        want_o, want_i, _, _ = orc.simulate(wl.start, wl.end, wl.indeg, *_coef(wl),
                                            _member(wl.o0, e), _member(wl.i0, e), wl.x, wl.xp,
                                            _member(wl.fp, e))
        assert np.array_equal(got_o[:, :, k], want_o), e
        assert np.array_equal(got_i[:, :, k], want_i), e
    net.close()


def test_config3_texas_enkf256_member_step_and_analysis():
    from tx_fast_hydrology_amd import ensemble
    args = bench.parse(["--members", "256", "--enkf", "--one-plan"], world=1)
    net, wl = bench.build_workload(args)
    ek = wl.enkf
    E = wl.E
    assert E == 256 and ek.m == 500 and np.array_equal(ek.R, 1e-2 * np.eye(500))
    # one member step: all 256 members bit-exact (auto: the member-dataflow launch at 256)
    net.run(wl.x[0:1])
    assert net.mode()[1] == "dataflow"
    X, I = net.get_state()
    fo, fi = orc.simulate_members(wl.start, wl.end, wl.indeg, *_coef(wl), wl.o0, wl.i0,
                                  wl.x[0:1], wl.xp, wl.fp, threads=THREADS)
    assert np.array_equal(X, fo) and np.array_equal(I, fi)
    # one analysis through the bench's path
    ensemble.distributed_analysis(net, ek.gauges, ek.Y[0], ek.R)
    o, i = net.get_state()
    g = ek.gauges
    A = X - X.mean(1, keepdims=True)
    HA = A[g]
    W = np.linalg.solve(HA @ HA.T / (E - 1) + ek.R, ek.Y[0] - X[g])
    G = A @ (HA.T @ W) / (E - 1)
    scale = np.abs(G).max()
    assert scale > 1e-3                          # the observations move the ensemble
    heads = wl.start[wl.indeg == 0]
    for e in range(E):
        ig, og = orc.apply_gain(heads, wl.end, np.ascontiguousarray(G[:, e]), wl.indeg)
        np.testing.assert_allclose(o[:, e] - X[:, e], og, rtol=0, atol=1e-10 * scale)
        np.testing.assert_allclose(i[:, e] - I[:, e], ig, rtol=0, atol=1e-10 * scale * 8)
    net.close()


@pytest.mark.timeout(600)
def test_config3_eight_shards_emulated_bitexact():
    """configs[3] in its SHARDED form: 8 sessions of 32 members (the 8-GPU layout of the
    256-member EnKF) on one GPU, driven by ensemble.emulated_analysis -- every mc_ens_* stage
    with nranks = 8 exactly as on 8 GPUs, the all-gathers and all-to-alls as device copies.
    Two analyses: bit-identical to the one-session 256-member analysis, and within 1e-10 of
    max|G| of the NumPy restatement of da.py:112-126 with the sample covariance."""
    import torch

    from tx_fast_hydrology_amd import engine, ensemble
    N = 8
    args = bench.parse(["--members", "256", "--enkf", "--one-plan"], world=1)
    full, wl = bench.build_workload(args)
    ek = wl.enkf
    E, El = wl.E, wl.E // N
    heads = wl.start[wl.indeg == 0]
    info = full.info
    shards = []
    for r in range(N):
        s = engine.RoutingNet(wl.end, wl.indeg, heads, slots=info["slots"], tile=info["tile"],
                              members=El)
        s.set_coeffs(*_coef(wl))
        cols = slice(r * El, (r + 1) * El)
        s.set_state(np.ascontiguousarray(wl.o0[:, cols]), np.ascontiguousarray(wl.i0[:, cols]))
        shards.append(s)
    X, I = full.get_state()
    for k in range(2):
        Y = ek.Y[k]                                  # [m, 256]: shard r holds columns r*32..
        stage_ms = {}
        ensemble.emulated_analysis(shards, ek.gauges,
                                   [np.ascontiguousarray(Y[:, r * El:(r + 1) * El])
                                    for r in range(N)], ek.R, stage_ms=stage_ms)
        full.enkf_analysis(ek.gauges, Y, ek.R)
        o_full, i_full = full.get_state()
        parts = [s.get_state() for s in shards]
        o_sh = np.concatenate([p[0] for p in parts], axis=1)
        i_sh = np.concatenate([p[1] for p in parts], axis=1)
        assert np.array_equal(o_sh, o_full) and np.array_equal(i_sh, i_full), k
        # the NumPy restatement (sample covariance in da.py:119-126)
        g = ek.gauges
        A = X - X.mean(1, keepdims=True)
        HA = A[g]
        W = np.linalg.solve(HA @ HA.T / (E - 1) + ek.R, Y - X[g])
        G = A @ (HA.T @ W) / (E - 1)
        scale = np.abs(G).max()
        assert scale > 1e-3
        for e in range(0, E, 37):
            ig, og = orc.apply_gain(heads, wl.end, np.ascontiguousarray(G[:, e]), wl.indeg)
            np.testing.assert_allclose(o_full[:, e] - X[:, e], og, rtol=0, atol=1e-10 * scale)
            np.testing.assert_allclose(i_full[:, e] - I[:, e], ig, rtol=0,
                                       atol=1e-10 * scale * 8)
        print("per-shard stage ms", {kk: [round(v, 3) for v in vv]
                                     for kk, vv in stage_ms.items()})
        X, I = o_full, i_full
    torch.cuda.synchronize()
    for s in shards:
        s.close()
    full.close()


def test_config4_conus_16_members_full_horizon():
    args = bench.parse(["--conus"], world=1)
    net, wl = bench.build_workload(args)
    assert wl.n == 2_700_000 and wl.E == 16 and net.info["nwg"] > 1000
    T = wl.x.size
    assert T == 288
    net.run(wl.x)
    assert net.mode()[1] == "launches"
    so, si = net.get_state()
    checks = [0, 143, 287]
    got = {t: net.fetch_outputs(t, t + 1) for t in checks}
    sample = [0, 7, 15]
    o = np.ascontiguousarray(wl.o0[:, sample])
    i = np.ascontiguousarray(wl.i0[:, sample])
    fp = np.ascontiguousarray(wl.fp[:, :, sample])
    t_prev = 0
    for t in checks:                   # the oracle's state after step t = the outputs of step t
        o, i = orc.simulate_members(wl.start, wl.end, wl.indeg, *_coef(wl), o, i,
                                    wl.x[t_prev:t + 1], wl.xp, fp, threads=len(sample))
        t_prev = t + 1
        go, gi = got[t]
        assert np.array_equal(go[0][:, sample], o), t
        assert np.array_equal(gi[0][:, sample], i), t
    assert np.array_equal(so[:, sample], o) and np.array_equal(si[:, sample], i)
    net.close()
