"""The composed configs[3] EnKF horizon exactly as bench.py times it: 24
one-step member runs, each followed by the ensemble analysis (da.py:112-126 with the ensemble
sample covariance; the gain folded lazily into the next step's staging), the device hand-over to
the forecast plan and the 264 forecast steps -- on the full Texas network with the bench's 500
gauges and R = 1e-2 I, E reduced to 16 so that the host restatement fits the test budget.

Compared with bench.enkf_restatement (the C member loop, the observation-space NumPy analysis
and the C _apply_gain; the same code bench.py's cpu_baseline leg times).  The device solves the
analysis in ensemble space (push-through identity), so the increments differ in
the last bits; the routing that follows is linear and contractive.  Tolerance: 1e-9 x the
largest |state|, on the final state and on sampled forecast steps."""
import numpy as np
import pytest

import bench
from oracle import oracle as orc

pytestmark = pytest.mark.gpu

E = 16
SAMPLES = [24, 143, 287]          # forecast steps compared (the first, the middle, the last)


def _workloads(shards):
    args = bench.parse(["--enkf", "--members", str(E)], world=1)
    built = [bench.build_workload(args, r, shards) for r in range(shards)]
    return [b[0] for b in built], [b[1] for b in built]


def _check(wls, o, i, fo, fi):
    ek = wls[0].enkf
    o0 = np.concatenate([w.o0 for w in wls], axis=1)
    i0 = np.concatenate([w.i0 for w in wls], axis=1)
    fp = np.ascontiguousarray(np.concatenate([w.fp for w in wls], axis=2))
    Y = [np.concatenate([w.enkf.Y[k] for w in wls], axis=1) for k in range(ek.n_an)]
    want_o, want_i, outs = bench.enkf_restatement(wls[0], orc, o0, i0, fp, Y, cores=16,
                                                  x_out=[t + 1 for t in SAMPLES])
    scale = max(np.abs(want_o).max(), np.abs(want_i).max())
    tol = 1e-9 * scale
    assert np.abs(o - want_o).max() <= tol and np.abs(i - want_i).max() <= tol
    for t in SAMPLES:
        assert np.abs(fo[t] - outs[t][0]).max() <= tol, t
        assert np.abs(fi[t] - outs[t][1]).max() <= tol, t


def _forecast_outputs(wls):
    n_an = wls[0].enkf.n_an
    fo, fi = {}, {}
    for t in SAMPLES:
        parts = [w.enkf.fnet.fetch_outputs(t - n_an, t - n_an + 1) for w in wls]
        fo[t] = np.concatenate([p[0][0] for p in parts], axis=1)
        fi[t] = np.concatenate([p[1][0] for p in parts], axis=1)
    return fo, fi


def test_bench_enkf_horizon_matches_restatement():
    nets, wls = _workloads(1)
    bench.run_horizon(nets[0], wls[0])
    o, i = nets[0].get_state()
    fo, fi = _forecast_outputs(wls)
    _check(wls, o, i, fo, fi)


def test_bench_enkf_horizon_two_emulated_shards():
    """The same horizon as two member shards (bench --emulate-shards 2: ensemble.emulated_
    analysis, every mc_ens_* stage at nranks = 2, the collectives as device copies)."""
    import torch
    nets, wls = _workloads(2)
    stream = torch.cuda.Stream()
    for s in nets + [w.enkf.fnet for w in wls]:
        s.set_stream(stream.cuda_stream)
    with torch.cuda.stream(stream):
        bench.run_emulated_horizon(nets, wls, stream)
    stream.synchronize()
    states = [net.get_state() for net in nets]
    o = np.concatenate([s[0] for s in states], axis=1)
    i = np.concatenate([s[1] for s in states], axis=1)
    fo, fi = _forecast_outputs(wls)
    _check(wls, o, i, fo, fi)
