"""CPU (gloo, world_size 2) check of the member-sharded analysis orchestration (ensemble.py):
pack -> all-to-all -> slice update -> all-to-all back -> unpack, with all-gathered gauge data.
A NumPy model stands in for the device stages (same layouts as mcroute.h: [E][m] gauge blocks,
[N][E][S] slice blocks); the sharded result must equal the single-process ensemble update."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tx_fast_hydrology_amd import ensemble


class NumpyStages:
    """Host model of the mc_ens_* stages on a member state X [n][E] (no padding slots)."""

    def __init__(self, X):
        self.X = np.array(X, dtype=float)
        self.n, self.E = self.X.shape

    def slice_size(self, N):
        return (self.n + N - 1) // N

    def ens_gauges(self, gauges, y, HX, D):
        hx = self.X[np.asarray(gauges)].T                         # [E][m]
        HX.copy_(torch.from_numpy(np.ascontiguousarray(hx)))
        D.copy_(torch.from_numpy(np.ascontiguousarray(np.asarray(y).T - hx)))

    def ens_pack(self, N, send):
        S = self.slice_size(N)
        pad = np.zeros((N * S, self.E))
        pad[:self.n] = self.X
        blocks = pad.reshape(N, S, self.E).transpose(0, 2, 1)     # [N][E][S]
        send.copy_(torch.from_numpy(np.ascontiguousarray(blocks).ravel()))

    def ens_slice_update(self, N, m, Xs, HXall, Dall, R, Gs):
        self.ens_weights(N, m, HXall, Dall, R)
        self.ens_increments(N, Xs, Gs)

    def ens_weights(self, N, m, HXall, Dall, R):
        Et = self.E * N
        hx = HXall.numpy().T                                      # [m][Et]
        d = Dall.numpy().T
        ha = hx - hx.mean(1, keepdims=True)
        C = ha @ ha.T / (Et - 1) + np.asarray(R)
        W = np.linalg.solve(C, d)
        self.Z = ha.T @ W / (Et - 1)

    def ens_increments(self, N, Xs, Gs):
        Et = self.E * N
        S = self.slice_size(N)
        xs = Xs.numpy().reshape(Et, S).T                          # [S][Et]
        A = xs - xs.mean(1, keepdims=True)
        Gs.copy_(torch.from_numpy(np.ascontiguousarray((A @ self.Z).T).ravel()))

    def ens_unpack_apply(self, N, Grecv):
        S = self.slice_size(N)
        g = Grecv.numpy().reshape(N, self.E, S).transpose(0, 2, 1).reshape(N * S, self.E)
        self.X += g[:self.n]


class FusedStages(NumpyStages):
    """The same stages without the weights / increments split (one slice-update call)."""

    def __getattribute__(self, name):
        if name in ("ens_weights", "ens_increments"):
            raise AttributeError(name)
        return super().__getattribute__(name)

    def ens_slice_update(self, N, m, Xs, HXall, Dall, R, Gs):
        NumpyStages.ens_weights(self, N, m, HXall, Dall, R)
        NumpyStages.ens_increments(self, N, Xs, Gs)


def _case(seed=0, n=97, E=8, m=5):
    rng = np.random.default_rng(seed)
    X = rng.uniform(1, 5, (n, E))
    gauges = np.sort(rng.choice(n, m, replace=False))
    R = 0.05 * np.eye(m) + 0.01
    Y = rng.normal(3, 0.5, (m, E))
    return X, gauges, R, Y


def _reference(X, gauges, R, Y):
    E = X.shape[1]
    A = X - X.mean(1, keepdims=True)
    HA = A[gauges]
    W = np.linalg.solve(HA @ HA.T / (E - 1) + R, Y - X[gauges])
    return X + A @ (HA.T @ W) / (E - 1)


def _worker(rank, world, port, q, fused=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    X, gauges, R, Y = _case()
    E = X.shape[1] // world
    cols = slice(rank * E, (rank + 1) * E)                        # rank-major member blocks
    st = (FusedStages if fused else NumpyStages)(X[:, cols])
    ensemble.distributed_analysis(st, gauges, Y[:, cols], R, device=torch.device("cpu"))
    out = torch.from_numpy(np.ascontiguousarray(st.X))
    parts = [torch.empty_like(out) for _ in range(world)]
    dist.all_gather(parts, out)
    if rank == 0:
        q.put(np.concatenate([p.numpy() for p in parts], axis=1))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_single_rank_stages_equal_reference():
    X, gauges, R, Y = _case(seed=3)
    st = NumpyStages(X)
    ensemble.distributed_analysis(st, gauges, Y, R, device=torch.device("cpu"))
    np.testing.assert_allclose(st.X, _reference(X, gauges, R, Y), rtol=1e-13, atol=1e-13)


@pytest.mark.parametrize("world,fused", [(2, False), (4, False), (2, True)])
def test_sharded_analysis_equals_single_process(world, fused):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, fused)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    X, gauges, R, Y = _case()
    np.testing.assert_allclose(got, _reference(X, gauges, R, Y), rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("shards,fused", [(2, False), (4, False), (8, False), (4, True)])
def test_emulated_shards_equal_reference(shards, fused):
    """ensemble.emulated_analysis: the per-rank programs of N shards stepped in one process,
    collectives as copies -- the same result as the single-process update (and as gloo ranks)."""
    X, gauges, R, Y = _case(seed=5, n=101, E=16)
    E = X.shape[1] // shards
    cls = FusedStages if fused else NumpyStages
    parts = [cls(X[:, r * E:(r + 1) * E]) for r in range(shards)]
    ensemble.emulated_analysis(parts, gauges, [Y[:, r * E:(r + 1) * E] for r in range(shards)],
                               R, device=torch.device("cpu"))
    got = np.concatenate([p.X for p in parts], axis=1)
    np.testing.assert_allclose(got, _reference(X, gauges, R, Y), rtol=1e-12, atol=1e-12)
