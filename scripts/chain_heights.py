#!/usr/bin/env python3
"""Diagnostic: critical-path length (ticks) of the wavefront schedule when a lane computes a
chain of up to K consecutive reaches per tick (K = 2 is the fused lane pair of plan.cpp).
Ignores partial-sum nodes and cross-cluster slack: the lower bound the plan approaches.
    python scripts/chain_heights.py [n] [basins] [depth]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tx-fast-hydrology_amd"))
from tx_fast_hydrology_amd import synthetic  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 190_000
    basins = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    depth = int(sys.argv[3]) if len(sys.argv) > 3 else 1500
    end = synthetic.river_network(n, basins, depth, np.random.default_rng(0))
    n = end.size
    ups = [[] for _ in range(n)]
    for u in range(n):
        if end[u] != u:
            ups[end[u]].append(u)
    deg = np.array([len(x) for x in ups])
    order, stack = [], list(np.flatnonzero(deg == 0))
    while stack:
        x = stack.pop()
        order.append(x)
        e = end[x]
        if e != x:
            deg[e] -= 1
            if deg[e] == 0:
                stack.append(e)
    inf = 1 << 30
    for K in (1, 2, 3, 4, 5, 6, 8):
        F = [[inf] * K for _ in range(n)]
        best = [0] * n
        for x in order:
            U = ups[x]
            bu = [best[u] + 1 for u in U]
            F[x][0] = max(bu, default=0)
            for k in range(1, K):
                for q, c in enumerate(U):
                    m = F[c][k - 1]
                    if m >= inf:
                        continue
                    for r, v in enumerate(bu):
                        if r != q and v > m:
                            m = v
                    if m < F[x][k]:
                        F[x][k] = m
            best[x] = min(F[x])
        print(f"K={K}: critical path {max(best)} ticks (+ T)", flush=True)


if __name__ == "__main__":
    main()
