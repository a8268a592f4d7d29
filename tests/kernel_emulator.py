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
EXT = 0x8000


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
    """Route len(x) steps exactly as the device does.  Returns (O [n][T], I [n][T], state)."""
    info = plan.info
    ex = plan.export()
    ln = plan.export_links()
    C, tile, nslots = info["slots"], info["tile"], info["nslots"]
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
    n_rows = F.shape[0]
    lo, hi, w0, w1 = step_tables(np.asarray(x, float), np.asarray(xp, float))
    G = ex["G"].astype(np.int64)
    fl = ln["flags"]
    cnt = ln["up_cnt"].astype(np.int64)
    maxc = int(cnt.max()) if cnt.size else 0
    codes = np.zeros((nslots, max(maxc, 1)), np.int64)
    for c in range(min(maxc, 4)):
        codes[:, c] = (ln["up4"] >> np.uint64(16 * c)).astype(np.int64) & 0xFFFF
    # output rows: reaches, then one row per slot for partial-sum nodes (ext_src convention)
    orow = np.where(real, sr, n + np.arange(nslots))
    O = np.full((n + nslots, T), np.nan)
    I = np.full((n + nslots, T), np.nan)

    for k in range(len(off) - 1):
        k0 = k * tile
        Os, Is = O.copy(), I.copy()          # reads see only earlier launches
        for w in wlist[off[k]:off[k + 1]]:
            d = w * C + np.arange(C)
            e0, e1 = ln["ext_off"][w], ln["ext_off"][w + 1]
            ne = e1 - e0
            xe = np.zeros((max(ne, 1), tile))
            for e in range(ne):
                tt = k0 + np.arange(tile) - ln["ext_g"][e0 + e]
                ok = (tt >= 0) & (tt < T)
                xe[e, ok] = Os[ln["ext_src"][e0 + e], tt[ok]]
            g, f = G[d], fl[d]
            row = orow[d]
            tf = k0 - g
            live = (f != 0) & (tf < T) & (tf + tile > 0)
            rest = (f != 0) & (tf <= T) & (tf + tile > 0)
            op = np.zeros(C)
            ip = np.zeros(C)
            init = rest & (tf <= 0)
            op[init], ip[init] = st_o[d[init]], st_i[d[init]]
            later = rest & (tf > 0)
            op[later] = Os[row[later], tf[later] - 1]
            ip[later] = Is[row[later], tf[later] - 1]
            xb = np.full((2, C), np.nan)
            xb[(k0 - 1) & 1] = op
            r_lo = np.full(C, -1)
            r_hi = np.full(C, -1)
            r_nx = np.full(C, -1)
            f_lo = np.zeros(C)
            f_hi = np.zeros(C)
            f_nx = np.zeros(C)
            tc = np.clip(tf, 0, T - 1)
            rn_x = np.where(live, lo[tc], 0)
            rn_y = np.where(live, hi[tc], -1)
            wn0 = np.where(live, w0[tc], 0.0)
            wn1 = np.where(live, w1[tc], 0.0)
            cd = codes[d]
            cn = cnt[d]
            for i in range(tile):
                kk = k0 + i
                t = kk - g
                rx, ry, ww0, ww1 = rn_x.copy(), rn_y.copy(), wn0.copy(), wn1.copy()
                act = live & (t >= 0) & (t < T)
                if not act.any():
                    continue
                pf = act & (t + 1 < T)
                tn = np.clip(t + 1, 0, T - 1)
                rn_x = np.where(pf, lo[tn], rn_x)
                rn_y = np.where(pf, hi[tn], rn_y)
                wn0 = np.where(pf, w0[tn], wn0)
                wn1 = np.where(pf, w1[tn], wn1)
                prev = xb[(kk - 1) & 1]
                Iv = np.zeros(C)
                for c in range(maxc):
                    m = act & (c < cn)
                    code = cd[:, c]
                    isx = (code & EXT) != 0
                    vi = prev[np.minimum(code, C - 1)]
                    vx = xe[np.clip(code & 0x7FFF, 0, xe.shape[0] - 1), i]
                    v = np.where(isx, vx, vi)
                    Iv = np.where(m, Iv + v, Iv)
                m1 = act & (rx != r_lo)
                c_hi = m1 & (rx == r_hi)
                c_nx = m1 & ~c_hi & (rx == r_nx)
                c_ld = m1 & ~c_hi & ~c_nx
                f_lo = np.where(c_hi, f_hi, f_lo)
                f_lo = np.where(c_nx, f_nx, f_lo)
                f_lo = np.where(c_ld, F[np.clip(rx, 0, n_rows - 1), d], f_lo)
                r_lo = np.where(m1, rx, r_lo)
                cp = ry < 0
                m2 = act & ~cp & (ry != r_hi)
                ld = F[np.clip(ry, 0, n_rows - 1), d]
                f_hi = np.where(m2, np.where(ry == r_nx, f_nx, ld), f_hi)
                r_hi = np.where(m2, ry, r_hi)
                m3 = m2 & (r_hi + 1 < n_rows) & (r_nx != r_hi + 1)
                r_nx = np.where(m3, r_hi + 1, r_nx)
                f_nx = np.where(m3, F[np.clip(r_nx, 0, n_rows - 1), d], f_nx)
                q = np.where(cp, f_lo, ww0 * f_lo + ww1 * f_hi)
                o = np.where(f == ROUTED, 0.0 + (((al[d] * Iv + be[d] * ip) + ch[d] * op)
                                                  + ga[d] * q), 0.0)
                o = np.where(f == PSUM, Iv, o)
                xb[kk & 1] = np.where(act, o, xb[kk & 1])
                O[row[act], t[act]] = o[act]
                I[row[act], t[act]] = Iv[act]
                op = np.where(act, o, op)
                ip = np.where(act, Iv, ip)
    return O[:n], I[:n]
