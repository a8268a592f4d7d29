"""CPU model of the HIP wavefront kernel (kernels.hip `wavefront_det`) -- TEST INFRASTRUCTURE.

Executes the exact launch/tick protocol of the device code on the host with numpy, driven by the
plan the C++ topology compiler exports (slots, G, upstream codes, external inputs, the active
workgroup schedule).  It lets the CPU test-suite check the schedule + kernel protocol
bit-for-bit against the oracle without a GPU:

* global outputs start as NaN and every launch reads a snapshot taken at launch start, so a read
  of a value not produced by an EARLIER launch (a missing slack / intra-launch race) or of a
  never-written step shows up as a mismatch;
* the LDS double buffer half that is not initialised in the prologue starts as NaN too.
"""
import numpy as np

ROUTED, UNROUTED, PSUM = 1, 2, 3
WAVE_SLACK = 4
EXT = 0x8000
SELF = 0x7FFF


def step_tables(x, xp):
    """nutils.py:21-33 per step -> (row_lo, row_hi (-1 = copy), w_lo, w_hi) like capi.cpp."""
    T = len(x)
    lo = np.zeros(T, np.int64)
    hi = np.full(T, -1, np.int64)
    w0 = np.ones(T)
    w1 = np.zeros(T)
    for t, xt in enumerate(x):
        ix = int(np.searchsorted(xp, xt, side="left"))
        if ix == 0:
            lo[t] = 0
        elif ix >= len(xp):
            lo[t] = len(xp) - 1
        else:
            dx0 = xt - xp[ix - 1]
            dx1 = xp[ix] - xt
            frac = dx0 / (dx0 + dx1)
            lo[t], hi[t], w0[t], w1[t] = ix - 1, ix, 1 - frac, frac
    return lo, hi, w0, w1


def run(plan, alpha, beta, chi, gamma, o0, i0, x, xp, fp):
    """Route len(x) steps exactly as the device does.  Returns (O [n][T], I [n][T]).

    A workgroup has `slots` lanes and chain * slots node slots: lane l owns slots p * slots + l
    for positions p = 0 .. chain-1, computed in that order within a tick.  A node may read the
    output of its lane's previous position in the same tick (SELF code); every other
    in-workgroup code reads the previous tick."""
    info = plan.info
    ex = plan.export()
    ln = plan.export_links()
    C, tile, nslots = info["slots"], info["tile"], info["nslots"]
    K = info["chain"]
    RS = K * C
    n = info["n"]
    T = len(x)
    off, wlist = plan.schedule(T)
    sr = ex["slot_reach"]
    real = sr >= 0
    rowc = np.where(real, sr, 0)

    def slots(a):
        return np.where(real, np.asarray(a, dtype=float)[rowc], 0.0)

    al, be, ch, ga = slots(alpha), slots(beta), slots(chi), slots(gamma)
    st_o, st_i = slots(o0), slots(i0)
    F = np.where(real[None, :], np.asarray(fp, float)[:, rowc], 0.0)
    lo, hi, w0, w1 = step_tables(np.asarray(x, float), np.asarray(xp, float))
    G = ex["G"].astype(np.int64)
    fl = ln["flags"]
    cnt = ln["up_cnt"].astype(np.int64)
    codes = np.zeros((nslots, 4), np.int64)
    for c in range(4):
        codes[:, c] = (ln["up4"] >> np.uint64(16 * c)).astype(np.int64) & 0xFFFF
    # output rows: reaches, then one row per slot for partial-sum nodes (ext_src convention)
    orow = np.where(real, sr, n + np.arange(nslots))
    O = np.full((n + nslots, T), np.nan)
    I = np.full((n + nslots, T), np.nan)

    # chunk-synchronous plans: local inputs (external columns after a workgroup's granule
    # inputs) deliver at tick k the producer's output of tick k - WAVE_SLACK, written within the
    # same workgroup (plan.hpp kWaveSlack)
    loc = plan.export_local()
    lx_off, lx_src = loc["lx_off"], loc["lx_src"]

    for k in range(len(off) - 1):
        k0 = k * tile
        Os, Is = O.copy(), I.copy()          # reads see only earlier launches
        for w in wlist[off[k]:off[k + 1]]:
            d = w * RS + np.arange(RS)
            e0, e1 = ln["ext_off"][w], ln["ext_off"][w + 1]
            ne = e1 - e0
            lsrc = lx_src[lx_off[w]:lx_off[w + 1]]
            xe = np.zeros((max(ne + lsrc.size, 1), tile))
            for e in range(ne):
                tt = k0 + np.arange(tile) - ln["ext_g"][e0 + e]
                ok = (tt >= 0) & (tt < T)
                xe[e, ok] = Os[ln["ext_src"][e0 + e], tt[ok]]
            g, f = G[d], fl[d]
            row = orow[d]
            tf = k0 - g
            live = (f != 0) & (tf < T) & (tf + tile > 0)
            rest = (f != 0) & (tf <= T) & (tf + tile > 0)
            op = np.zeros(RS)
            ip = np.zeros(RS)
            init = rest & (tf <= 0)
            op[init], ip[init] = st_o[d[init]], st_i[d[init]]
            later = rest & (tf > 0)
            op[later] = Os[row[later], tf[later] - 1]
            ip[later] = Is[row[later], tf[later] - 1]
            xb = np.full((2, RS + 1), np.nan)
            xb[:, RS] = 0.0
            xb[(k0 - 1) & 1, :RS] = op
            cd = codes[d]
            cn = cnt[d]
            for i in range(tile):
                kk = k0 + i
                for li, src in enumerate(lsrc):
                    ts = kk - WAVE_SLACK - G[src]
                    xe[ne + li, i] = O[orow[src], ts] if 0 <= ts < T else 0.0
                t = kk - g
                act = live & (t >= 0) & (t < T)
                if not act.any():
                    continue
                tc = np.clip(t, 0, T - 1)
                qlo = F[lo[tc], d]
                qhi = F[np.maximum(hi[tc], 0), d]
                q = np.where(hi[tc] < 0, qlo, w0[tc] * qlo + w1[tc] * qhi)
                prev = xb[(kk - 1) & 1]
                cur = xb[kk & 1]
                for half in (slice(p * C, (p + 1) * C) for p in range(K)):
                    Iv = np.zeros(RS)
                    for c in range(4):
                        m = act & (c < cn)
                        m[:half.start] = False
                        m[half.stop:] = False
                        code = cd[:, c]
                        isx = (code & EXT) != 0
                        self_ = code == SELF
                        vi = prev[np.minimum(code, RS)]
                        vs = cur[(np.arange(RS) - C) % RS]
                        vx = xe[np.clip(code & 0x7FFF, 0, xe.shape[0] - 1), i]
                        v = np.where(isx, vx, np.where(self_, vs, vi))
                        Iv = np.where(m, Iv + v, Iv)
                    o = np.where(f == ROUTED, 0.0 + (((al[d] * Iv + be[d] * ip) + ch[d] * op)
                                                      + ga[d] * q), 0.0)
                    o = np.where(f == PSUM, Iv, o)
                    sel = np.zeros(RS, bool)
                    sel[half] = True
                    a_ = act & sel
                    cur[:RS][a_] = o[a_]
                    O[row[a_], t[a_]] = o[a_]
                    I[row[a_], t[a_]] = Iv[a_]
                    op = np.where(a_, o, op)
                    ip = np.where(a_, Iv, ip)
    return O[:n], I[:n]
