"""Index mapping of the two-pass reach-order gather (kernels.hip unskew_windows / permute_steps,
launch_gather_slots): every (step, reach) of a pass is written exactly once, for horizons and
networks that fill the grid only partly.  Pure-Python restatement of the kernels' block ->
(step, item) arithmetic; the device results themselves are checked against the oracle by
tests/test_gpu_routing.py::test_device_gather_reference_layout."""
import itertools

import numpy as np
import pytest

K_UNSKEW = 16      # kernels.hip kUnskewSteps
K_PERMUTE = 2      # kernels.hip kPermuteSteps


def passes(t0, t1, scratch_steps):
    c0 = t0
    while c0 < t1:
        c1 = min(t1, c0 + scratch_steps)
        yield c0, c1
        c0 = c1


def unskew_cells(ns, c0, c1):
    sb = (c1 - c0 + K_UNSKEW - 1) // K_UNSKEW
    out = []
    for bx, by in itertools.product(range((ns + 255) // 256), range(sb)):
        for tid in range(256):
            d = bx * 256 + tid
            if d >= ns:
                continue
            tb = c0 + by * K_UNSKEW
            nt = min(K_UNSKEW, c1 - tb)
            out += [(tb + q, d) for q in range(nt)]
    return out


def permute_cells(n, c0, c1):
    ntile = (n + 255) // 256
    blocks = 8 * ntile * ((c1 - c0 + 8 * K_PERMUTE - 1) // (8 * K_PERMUTE))
    out = []
    for b in range(blocks):
        x, q = b & 7, b >> 3
        tb = c0 + (q // ntile) * 8 * K_PERMUTE + x
        for tid in range(256):
            j = (q % ntile) * 256 + tid
            if tb >= c1 or j >= n:
                continue
            out += [(tb + 8 * h, j, b % 8) for h in range(K_PERMUTE) if tb + 8 * h < c1]
    return out


@pytest.mark.parametrize("n,ns,t0,t1,scratch", [(300, 384, 0, 288, 288), (1000, 1152, 0, 37, 37),
                                                 (257, 512, 5, 29, 7), (50, 64, 0, 1, 1)])
def test_two_pass_gather_covers_every_cell_once(n, ns, t0, t1, scratch):
    seen_s, seen_o = [], []
    for c0, c1 in passes(t0, t1, scratch):
        s = unskew_cells(ns, c0, c1)
        assert len(s) == len(set(s)) == ns * (c1 - c0)
        assert {t for t, _ in s} == set(range(c0, c1))
        o = permute_cells(n, c0, c1)
        cells = [(t, j) for t, j, _ in o]
        assert len(cells) == len(set(cells)) == n * (c1 - c0)
        # the steps of one XCD (workgroup id mod 8) are t0 + x + 8 k: a row is read by one L2
        assert all((t - c0) % 8 == x for t, _, x in o)
        seen_s += s
        seen_o += cells
    assert sorted(set(seen_o)) == [(t, j) for t in range(t0, t1) for j in range(n)]
    assert len(set(seen_s)) == ns * (t1 - t0)


def test_scratch_passes_partition_the_steps():
    for t0, t1, s in [(0, 288, 23), (3, 4, 1), (0, 100, 100)]:
        ps = list(passes(t0, t1, s))
        assert ps[0][0] == t0 and ps[-1][1] == t1
        assert all(a[1] == b[0] for a, b in zip(ps, ps[1:]))
        assert np.all(np.array([c1 - c0 for c0, c1 in ps]) <= s)
