// Device helpers shared by the wavefront kernels (kernels.hip, flow.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.hpp"
#include "plan.hpp"

namespace mcr {
namespace dev {

// Forcing rows a lane needs for the chunk starting at tick kc: [rb, rb + nr).  Rows are
// non-decreasing in t (step times are increasing), so the first step's row_lo and the last
// step's max(row_lo, row_hi) bound them.  nr = 0 when the lane has no step in the chunk.
__device__ __forceinline__ void chunk_rows(const int4* tab, int tw0, int kc, int G, int T,
                                           int& rb, int& nr) {
    int ta = kc - G, tb = kc + kChunk - 1 - G;
    if (tb < 0 || ta >= T) {
        rb = 0;
        nr = 0;
        return;
    }
    ta = ta < 0 ? 0 : ta;
    tb = tb >= T ? T - 1 : tb;
    const int4 ea = tab[ta - tw0];
    const int4 eb = tab[tb - tw0];
    rb = ea.x;
    nr = (eb.y > eb.x ? eb.y : eb.x) - rb + 1;
}

// forcing row index clamped into [0, n_rows): rows of inactive ticks may be arbitrary
__device__ __forceinline__ int clamp_row(int r, int n_rows) {
    return r < 0 ? 0 : (r < n_rows ? r : n_rows - 1);
}

__device__ __forceinline__ double lds_f64(const char* lds, unsigned byte) {
    return *reinterpret_cast<const double*>(lds + byte);
}

// One node slot of a lane: the registers of its reach (or partial sum) for one launch.
struct Slot {
    int64_t d;            // node slot
    int G;                // tick of step 0 (huge when the slot has no work in this launch)
    // psum: a partial sum, whose state is never updated -- it stays 0, so its update
    // 0 + (((1 I + 0 Ip) + 0 Op) + 0 q) is exactly I, also for non-finite I (0 Ip with
    // Ip = +-Inf would be NaN).  unr: never processed by the reference walk (o = 0)
    bool routed, psum, unr, xsrc;
    double al, be, ch, ga, op, ip;
    int cnt;
    unsigned ubase[kUpInline];  // LDS byte base of each input
    bool uext[kUpInline];       // input from another cluster (XE region)
    bool chained;          // the last input is the lane's previous position of this tick
    int64_t xs0;           // XS address of tick 0 when the slot feeds another cluster
};

// k0 / tile: the ticks this launch covers (the dataflow kernel passes its whole window)
__device__ __forceinline__ void load_slot(Slot& s, const WaveArgs& a, int64_t d, int64_t mem,
                                          int k0, int tile, int T) {
    const uint8_t fl = a.flags[d];
    const int Gr = a.G[d];
    const bool real = fl != kSlotPad;
    const int t_first = k0 - Gr;                        // step at this launch's first tick
    const bool live = real && (t_first < T) && (t_first + tile > 0);
    s.d = d;
    s.G = live ? Gr : (1 << 29);                        // never active when not live
    s.routed = fl == kSlotRouted;
    s.psum = fl == kSlotSum;
    s.unr = fl == kSlotUnrouted;
    // state after the last step this slot ran in an earlier launch (or the initial state)
    s.op = a.st_o[mem * a.mS + d];
    s.ip = a.st_i[mem * a.mS + d];
    s.al = a.alpha[d];
    s.be = a.beta[d];
    s.ch = a.chi[d];
    s.ga = a.gamma[d];
    s.cnt = live ? a.up_cnt[d] : 0;
    const int xsid = a.xid[d];
    s.xsrc = live && xsid >= 0;
    s.xs0 = s.xsrc ? (int64_t)xsid * T - Gr : 0;
}

// input codes -> LDS byte bases; unused codes read the zero slot (adding +0.0 to a sum that
// started as a published value is exact, so the sum needs no predicate).  xb_stride: bytes
// between consecutive node slots' outputs; ext_stride: between external inputs.
template <int RS>
__device__ __forceinline__ void decode_codes(Slot& s, uint64_t up4, unsigned XB,
                                             unsigned xb_stride, unsigned XE,
                                             unsigned ext_stride) {
#pragma unroll
    for (int u = 0; u < kUpInline; ++u) {
        unsigned code = u < s.cnt ? (unsigned)((up4 >> (16 * u)) & 0xffffu) : (unsigned)RS;
        if (u == 0) s.chained = false;
        if (code == kSelfCode) {      // the chained (last) input: read the zero slot, added last
            s.chained = true;
            code = RS;
        }
        const bool ext = (code & kExtBit) != 0;
        s.ubase[u] = ext ? XE + (code & 0x7fffu) * ext_stride : XB + code * xb_stride;
        s.uext[u] = ext;
    }
}

// The input values of one slot for this tick (byte offset `off` from the bases m).  A lane reads the inputs of ALL its
// positions before it writes any output: the compiler cannot prove that a position's LDS
// write does not alias the next position's reads, so reads issued after it would wait for it
// (one LDS round trip per position per tick).  any3 (wave-uniform): some slot of the wave has
// more than 2 inputs.
__device__ __forceinline__ void read_inputs(const char* lds, const unsigned* m, unsigned off,
                                            bool any3, double* v) {
    v[0] = lds_f64(lds, m[0] + off);
    v[1] = lds_f64(lds, m[1] + off);
    if (any3) {
        v[2] = lds_f64(lds, m[2] + off);
        v[3] = lds_f64(lds, m[3] + off);
    } else {
        v[2] = v[3] = 0.0;
    }
}

// inflow fold in reference finalisation order.  Every value a lane publishes is 0 + (...) or
// such a sum, never -0.0, so the reference's leading 0 + is exact without an add, and so is
// adding the zero slot's +0.0 for an unused code.  The chained input of a slot is its LAST
// input (plan.cpp); its code reads the zero slot and the value, the lane's previous position
// output of this tick (`prev`), is added after the others: the same left fold bit for bit.
// first: position 0 (compile-time at every call site), which has no previous position.
__device__ __forceinline__ double fold_values(const double* v, bool chained, bool any3,
                                              double prev, bool first) {
    double I = v[0];
    I = I + v[1];
    if (any3) {
        I = I + v[2];
        I = I + v[3];
    }
    if (!first) I = I + (chained ? prev : 0.0);
    return I;
}

// The reference update o = 0 + (((a I + b Ip) + c Op) + g q) (nutils.py:80-83), evaluated as
// ((a I + b Ip) + c Op) + (0 + g q).  Bit-identical for every input: a round-to-nearest sum is
// -0.0 only when both addends are -0.0, so the leading 0 + only ever turns a -0.0 into +0.0,
// and it does the same when applied to the last addend first (NaN and +-Inf propagate the same
// way through either order).  gq0 = 0 + g q does not depend on the inflow I, so the
// canonicalising add leaves the tick's dependent chain: alpha I, + b Ip, + c Op, + gq0.
__device__ __forceinline__ double gq_term(double g, double q) { return 0.0 + g * q; }
__device__ __forceinline__ double muskingum_update(double a, double I, double b, double ip,
                                                   double c, double op, double gq0) {
    return ((a * I + b * ip) + c * op) + gq0;
}

}  // namespace dev
}  // namespace mcr
