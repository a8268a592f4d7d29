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
__device__ __forceinline__ void chunk_rows(const StepEntry* tab, int tw0, int kc, int G, int T,
                                           int& rb, int& nr) {
    int ta = kc - G, tb = kc + kChunk - 1 - G;
    if (tb < 0 || ta >= T) {
        rb = 0;
        nr = 0;
        return;
    }
    ta = ta < 0 ? 0 : ta;
    tb = tb >= T ? T - 1 : tb;
    const int lo = tab[ta - tw0].lo;
    const int2 eb = *reinterpret_cast<const int2*>(&tab[tb - tw0]);
    rb = lo;
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
    bool real;            // not a padding slot (a real slot keeps its state when idle)
    bool routed, psum, xsrc;
    double al, be, ch, ga, op, ip;
    int cnt;
    unsigned ubase[kUpInline], uinc[kUpInline];
    bool self_last;        // last input = the lane's low output of this tick (fused pair)
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
    s.real = real;
    s.G = live ? Gr : (1 << 29);                        // never active when not live
    s.routed = fl == kSlotRouted;
    s.psum = fl == kSlotSum;
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

// input codes -> LDS byte bases.  Codes are positional (plan.cpp): the last input sits in
// position kUpInline - 1, unused positions name the zero slot RS.  A SELF code (only ever in the
// last position) also reads the zero slot and is replaced by the low output in `fold`.
template <int RS>
__device__ __forceinline__ void decode_codes(Slot& s, uint64_t up4, unsigned XB, unsigned XE,
                                             unsigned ext_stride) {
#pragma unroll
    for (int u = 0; u < kUpInline; ++u) {
        unsigned code = (unsigned)((up4 >> (16 * u)) & 0xffffu);
        if (s.cnt == 0) code = RS;                      // idle / padding slot: read zeros
        if (u == kUpInline - 1) s.self_last = code == kSelfCode;
        if (code == kSelfCode) code = RS;
        const bool ext = (code & kExtBit) != 0;
        s.ubase[u] = ext ? XE + (code & 0x7fffu) * ext_stride : XB + code * 16;
        s.uinc[u] = ext ? 16u : 0u;
    }
}

// The four input values of a slot at tick parity rd (issued together at the start of a tick).
__device__ __forceinline__ void load_inputs(const char* lds, const unsigned* m, unsigned rd,
                                            double (&v)[kUpInline]) {
#pragma unroll
    for (int u = 0; u < kUpInline; ++u) v[u] = lds_f64(lds, m[u] + rd);
}

// Inflow fold in reference finalisation order: ((v0 + v1) + v2) + last.  Every value a lane
// publishes is 0 + (...) or such a sum, never -0.0, so the reference's leading 0 + and the
// zero-slot padding are exact.  `last` is v3, or the lane's low output of this tick when the
// slot is the high node of a fused pair (one add after the low output is known).
__device__ __forceinline__ double prefix3(const double (&v)[kUpInline]) {
    return (v[0] + v[1]) + v[2];
}

}  // namespace dev
}  // namespace mcr
