// Muskingum routing kernels for CDNA4 (gfx950).
//
// Hot path: `wavefront_det` -- the time-skewed wavefront sweep that replaces the per-step
// serial walk of nutils.py:64-89 (`_ax_bu`) driven by muskingum.py:499-536 (`simulate_iter`).
// One workgroup owns up to SLOTS reaches (one per lane).  Reach j handles model step t at tick
// G[j] + t; an upstream reach in the same cluster runs one tick ahead, so its outflow is read
// from an LDS double buffer written in the previous tick.  Inputs from other clusters were
// produced in an earlier launch and are staged in LDS in the launch prologue, together with the
// window of the per-step interpolation table this workgroup needs.  The tick loop issues no
// global loads except the per-chunk forcing-row prefetch; each tick's outputs leave as one
// contiguous row per wave (workgroup windows, kernels.hpp).
//
// Arithmetic follows the reference exactly (FMA contraction is off for this file):
//   I = ((0 + o[u1]) + o[u2]) + ...          upstream reaches in reference finalisation order
//   o = 0 + (((alpha*I + beta*I_prev) + chi*o_prev) + gamma*q)            nutils.py:80-83
//   q = (1 - frac) * f[ix-1] + frac * f[ix]   (or a row copy at the ends)  nutils.py:23-33
#include "kernels.hpp"
#include "plan.hpp"
#include "device_common.hpp"

#pragma clang fp contract(off)

// Diagnostic builds only (scripts/exp_variants.sh): each MCR_EXP_* switch removes one part of the
// tick to measure its cost.  Results of such a build are wrong by construction.
#ifndef MCR_EXP_NO_STORES
#define MCR_EXP_NO_STORES 0
#endif
#ifndef MCR_EXP_NO_BARRIER
#define MCR_EXP_NO_BARRIER 0
#endif
#ifndef MCR_EXP_NO_Q
#define MCR_EXP_NO_Q 0
#endif

namespace mcr {

namespace {

using dev::chunk_rows;
using dev::clamp_row;
using dev::lds_f64;
constexpr int kHalf = kChunk;  // ticks whose lateral inflow is formed in one burst

// LDS layout of one workgroup (bytes):
//   XB  [SLOTS + 1][2] f64  outflow of each slot at tick parity 0/1; slot SLOTS stays 0.0
//   FR  [SLOTS][3]     f64  the lane's forcing rows rb .. rb + 2 of the current chunk
//   TAB [table_cap]    int4 step-table window {row_lo, row_hi, frac}
//   XE  [ext_cap][tile] f64 external inputs of this launch
// DENSE: some chunk needs more than 3 forcing rows (model step >= ~1/3 of the forcing interval);
// those lanes read the forcing straight from global memory.  A separate instantiation keeps the
// direct loads (and the waits they need) out of the common kernel.
template <int SLOTS, bool DENSE>
__global__ __launch_bounds__(SLOTS) __attribute__((amdgpu_waves_per_eu(4)))
void wavefront_det(WaveArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    const int tile = a.tile;
    constexpr unsigned XB = 0;
    constexpr unsigned FR = XB + (SLOTS + 1) * 16;
    constexpr unsigned TAB = FR + SLOTS * 24;
    const unsigned XE = TAB + (unsigned)a.table_cap * 16;
    double* xbp = reinterpret_cast<double*>(lds + XB);
    int4* tab = reinterpret_cast<int4*>(lds + TAB);
    double* xe = reinterpret_cast<double*>(lds + XE);

    const int tid = threadIdx.x;
    const int64_t t_start = a.trace ? wall_clock64() : 0;
    const int w = a.active[blockIdx.x];
    // ensemble member of this workgroup instance: member-major arrays (uniform bases)
    const int64_t mem = blockIdx.y;
    const double* Fm = a.F + mem * a.mF;
    double* Om = a.O + mem * a.mO;
    double* XSm = a.XS + mem * a.mX;
    double* dum = a.dummy + mem * kDummyPerMember;
    const int64_t d = (int64_t)w * SLOTS + tid;
    const int T = a.T;
    const int k0 = a.kappa0;
    const int64_t ns = a.nslots;
    const int nrow = a.n_rows;

    // ---- per-reach registers and state at step t_first - 1 (issued first: longest latency)
    const uint8_t fl = a.flags[d];
    const int Gr = a.G[d];
    const bool real = fl != kSlotPad;
    const bool routed = fl == kSlotRouted;
    const bool psum = fl == kSlotSum;                   // partial-sum node: outputs I
    const int t_first = k0 - Gr;                        // step at this launch's first tick
    const bool live = real && (t_first < T) && (t_first + tile > 0);
    const int G = live ? Gr : (1 << 29);                // never active when not live
    const int gminw = a.wg_gmin[w], gmaxw = a.wg_gmax[w];
    const int64_t wb = a.wbase[w];
    // the state after the last step this lane ran in an earlier launch (or the initial state)
    const double st_o = a.st_o[mem * a.mS + d], st_i = a.st_i[mem * a.mS + d];
    const double al = a.alpha[d], be = a.beta[d], ch = a.chi[d], ga = a.gamma[d];
    const int cnt = live ? a.up_cnt[d] : 0;
    const uint64_t up4 = a.up4[d];
    const int xsid = a.xid[d];

    // ---- step-table window of this workgroup -> LDS
    int tw0 = k0 - gmaxw, tw1 = k0 + tile - gminw;
    tw0 = tw0 < 0 ? 0 : (tw0 > T ? T : tw0);
    tw1 = tw1 < 0 ? 0 : (tw1 > T ? T : tw1);
    for (int idx = tid; idx < tw1 - tw0; idx += SLOTS) tab[idx] = a.stab[tw0 + idx];

    // ---- external inputs (produced by earlier launches) -> LDS, 8 loads in flight per lane
    const int e0 = a.ext_off[w];
    const int ntot = (a.ext_off[w + 1] - e0) * tile;
    for (int base = tid; base < ntot; base += 8 * SLOTS) {
        int ti[8], eg[8], ee[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {   // unconditional (clamped) loads: one wait per batch
            const int idx = min(base + k * SLOTS, ntot - 1);
            const int e = idx / tile;
            ti[k] = k0 + (idx - e * tile);
            ee[k] = e0 + e;
            eg[k] = a.ext_g[e0 + e];
        }
        double v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {   // consecutive lanes read consecutive steps of a stream
            const int t = ti[k] - eg[k];
            const bool ok = t >= 0 && t < T;
            v[k] = XSm[ok ? (int64_t)ee[k] * T + t : 0];
            v[k] = ok ? v[k] : 0.0;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (base + k * SLOTS < ntot) xe[base + k * SLOTS] = v[k];
    }
    double op = st_o;
    double ip = st_i;
    // the downstream reach (one tick behind) reads step t_first - 1 at the first tick
    xbp[tid * 2 + ((k0 - 1) & 1)] = op;
    if (tid < 2) xbp[SLOTS * 2 + tid] = 0.0;            // zero slot for unused upstream codes
    // drain every prologue load: otherwise the wait-count pass carries "pending" state into
    // the tick loop and waits for each chunk's stores at every tick
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();

    // upstream codes -> LDS byte bases; unused codes read the zero slot (adding +0.0 to a sum
    // that started as 0.0 + v is exact, so the sum needs no predicate)
    unsigned ubase[kUpInline], uinc[kUpInline];
#pragma unroll
    for (int u = 0; u < kUpInline; ++u) {
        const unsigned code = u < cnt ? (unsigned)((up4 >> (16 * u)) & 0xffffu) : (unsigned)SLOTS;
        const bool ext = (code & kExtBit) != 0;
        ubase[u] = ext ? XE + (code & 0x7fffu) * (unsigned)tile * 8 : XB + code * 16;
        uinc[u] = ext ? 16u : 0u;
    }
    const bool any3 = __any(cnt > 2);                   // wave-uniform
    const unsigned own = XB + (unsigned)tid * 16;

    // forcing rows of the first chunk
    int rb, nr;
    chunk_rows(tab, tw0, k0, G, T, rb, nr);
    double f0 = Fm[(int64_t)clamp_row(rb, nrow) * ns + d];
    double f1 = Fm[(int64_t)clamp_row(rb + 1, nrow) * ns + d];
    double f2 = Fm[(int64_t)clamp_row(rb + 2, nrow) * ns + d];
    __builtin_amdgcn_s_waitcnt(0);   // same reason: nothing pending may enter the loop
    const int64_t t_loop = a.trace ? wall_clock64() : 0;
    const int64_t c_loop = a.trace ? clock64() : 0;

    const int wend = gmaxw + T;                         // end of this workgroup's window
    // feeds another cluster: step t also goes to XS[xsid][t] (address at tick k: xs0 + k)
    const bool xsrc = live && xsid >= 0;
    const int64_t xs0 = xsrc ? (int64_t)xsid * T - Gr : 0;
    for (int c = 0; c < tile; c += kChunk) {
        const int kc = k0 + c;
        // this chunk's forcing rows -> the lane's LDS slots (private: no barrier needed)
        double* frl = reinterpret_cast<double*>(lds + FR) + tid * 3;
        frl[0] = f0;
        frl[1] = f1;
        frl[2] = f2;
        const bool slow = DENSE && __any(nr > 3);       // more rows than slots: load direct
        const unsigned frp = FR + (unsigned)tid * 24 - (unsigned)rb * 8;
        // prefetch the forcing rows of the next chunk (unconditional, clamped rows)
        int rbn, nrn;
        chunk_rows(tab, tw0, kc + kChunk, G, c + kChunk < tile ? T : 0, rbn, nrn);
        const double g0 = Fm[(int64_t)clamp_row(rbn, nrow) * ns + d];
        const double g1 = Fm[(int64_t)clamp_row(rbn + 1, nrow) * ns + d];
        const double g2 = Fm[(int64_t)clamp_row(rbn + 2, nrow) * ns + d];
        // per-chunk LDS cursors: upstream value of tick i at m[u] + 8 * ((i + 1) & 1)
        unsigned m[kUpInline];
#pragma unroll
        for (int u = 0; u < kUpInline; ++u) m[u] = uinc[u] ? ubase[u] + 8u * c - 8u : ubase[u];
        const unsigned tp = TAB + (unsigned)(kc - G - tw0) * 16u;
#pragma unroll
        for (int h = 0; h < kChunk; h += kHalf) {
            // lateral inflow of the next kHalf ticks, interpolate_sample (nutils.py:23-33); it
            // does not depend on the routing state, so it is formed off the tick's critical path
            double qv[kHalf];
#pragma unroll
            for (int j = 0; j < kHalf; ++j) {
                const int4 e = *reinterpret_cast<const int4*>(lds + tp + 16u * (h + j));
                double flo, fhi;
                if (DENSE && slow) {
                    flo = Fm[(int64_t)clamp_row(e.x < 0 ? 0 : e.x, nrow) * ns + d];
                    fhi = Fm[(int64_t)clamp_row(e.y < 0 ? 0 : e.y, nrow) * ns + d];
                } else {
                    flo = lds_f64(lds, frp + 8u * (unsigned)e.x);
                    fhi = lds_f64(lds, frp + 8u * (unsigned)e.y);
                }
                const double fr = __hiloint2double(e.w, e.z);
                const double qi = (1.0 - fr) * flo + fr * fhi;
                qv[j] = MCR_EXP_NO_Q ? 0.0 : (e.y < 0 ? flo : qi);
            }
            if (DENSE && slow) __builtin_amdgcn_s_waitcnt(0);  // settle the direct loads here
#pragma unroll
            for (int j = 0; j < kHalf; ++j) {
                const int i = h + j;
                if (i & 1) {
#pragma unroll
                    for (int u = 0; u < kUpInline; ++u) m[u] += uinc[u];
                }
                const unsigned rd = 8u * ((i + 1) & 1);     // parity of tick k - 1
                const int t = kc + i - G;
                const bool act = (unsigned)t < (unsigned)T;
                // inflow: upstream outflows in reference finalisation order.  Every value a
                // lane publishes is 0 + (...) or such a sum, never -0.0, so the reference's
                // leading 0 + is exact without an add
                double I = lds_f64(lds, m[0] + rd);
                I = I + lds_f64(lds, m[1] + rd);
                if (any3) {
                    I = I + lds_f64(lds, m[2] + rd);
                    I = I + lds_f64(lds, m[3] + rd);
                }
                const double rv = 0.0 + (((al * I + be * ip) + ch * op) + ga * qv[j]);
                const double ov = psum ? I : rv;
                // inactive ticks write garbage that no active reach reads (its consumer is
                // inactive one tick later); never-processed reaches (no consumer) output 0
                *reinterpret_cast<double*>(lds + own + 8u * (i & 1)) = ov;
                op = act ? ov : op;
                ip = act ? I : ip;
                // one contiguous row per wave; ticks outside the window go to the dummy row
                const int k = kc + i;
                const bool inwin = k >= gminw && k < wend;
                const int64_t row = inwin ? wb + (int64_t)(k - gminw) * SLOTS : 0;
                double* orow = inwin ? Om + row : dum;
                if (!MCR_EXP_NO_STORES) {
                    orow[tid] = routed ? ov : 0.0;
                    if (xsrc && act) XSm[xs0 + k] = ov;
                }
                if (!MCR_EXP_NO_BARRIER) __syncthreads();
            }
        }
        rb = rbn;
        nr = nrn;
        f0 = g0;
        f1 = g1;
        f2 = g2;
    }
    // state for the next launch (lanes that did not run keep theirs); never-processed reaches
    // hold o = 0 as in the reference's fresh o_t_next
    const int64_t ds = (int64_t)blockIdx.y * a.mS + (int64_t)w * SLOTS + threadIdx.x;
    a.st_o[ds] = routed || psum ? op : 0.0;
    a.st_i[ds] = ip;
    if (a.trace && tid == 0 && mem == 0) {
        const int64_t c_end = clock64();
        int64_t* rec = a.trace + kTraceWords * (int64_t)blockIdx.x;
        rec[0] = t_start;
        rec[1] = t_loop;
        rec[2] = wall_clock64();
        rec[3] = (int64_t)__smid();
        rec[4] = c_loop;
        rec[5] = c_end;
    }
}

__global__ void scatter_to_slots(const double* __restrict__ src, double* __restrict__ dst,
                                 const int64_t* __restrict__ slot_reach, int64_t nslots,
                                 int64_t E) {
    const int64_t total = nslots * E;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = x / nslots;
        const int64_t d = x - e * nslots;
        const int64_t j = slot_reach[d];
        dst[x] = j >= 0 ? src[j * E + e] : 0.0;
    }
}

__global__ void gather_from_slots(const double* __restrict__ src, double* __restrict__ dst,
                                  const int64_t* __restrict__ pos, int64_t n, int64_t nslots,
                                  int64_t E) {
    const int64_t total = n * E;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = x / E;
        const int64_t e = x - j * E;
        dst[x] = src[e * nslots + pos[j]];
    }
}

__global__ void forcing_to_slots(const double* __restrict__ fp, double* __restrict__ F,
                                 const int64_t* __restrict__ slot_reach, int64_t n,
                                 int64_t nslots, int64_t n_rows, int64_t E) {
    const int64_t total = nslots * n_rows * E;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t er = x / nslots;                  // e * n_rows + r
        const int64_t d = x - er * nslots;
        const int64_t e = er / n_rows;
        const int64_t r = er - e * n_rows;
        const int64_t j = slot_reach[d];
        F[x] = j >= 0 ? fp[(r * n + j) * E + e] : 0.0;
    }
}

__global__ void window_index(const int64_t* __restrict__ pos, const int32_t* __restrict__ G,
                             const int32_t* __restrict__ wg_gmin,
                             const int64_t* __restrict__ wbase, int slots, int64_t n,
                             int64_t* __restrict__ jbase) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n;
         j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t d = pos[j];
        const int64_t w = d / slots;
        jbase[j] = wbase[w] + (int64_t)(G[d] - wg_gmin[w]) * slots + (d - w * slots);
    }
}


// inflow of caller reach j at step t: ((0 + o[u1][t]) + o[u2][t]) + ...  (reference order)
__device__ __forceinline__ double inflow_at(const double* __restrict__ O,
                                            const int64_t* __restrict__ jbase,
                                            const int64_t* __restrict__ in_off,
                                            const int64_t* __restrict__ in_list, int64_t j,
                                            int64_t t, int slots) {
    double s = 0.0;
    for (int64_t k = in_off[j]; k < in_off[j + 1]; ++k) s = s + O[jbase[in_list[k]] + t * slots];
    return s;
}

// out[t - t0][j][e]: consecutive threads take consecutive (j, e) (coalesced writes)
__global__ void gather_steps(const double* __restrict__ O, int64_t mO,
                             const int64_t* __restrict__ jbase,
                             const int64_t* __restrict__ in_off,
                             const int64_t* __restrict__ in_list, bool inflow, int slots,
                             double* __restrict__ out, int64_t n, int64_t t0, int64_t t1,
                             int64_t E) {
    const int64_t total = n * (t1 - t0) * E;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t tj = x / E;
        const int64_t e = x - tj * E;
        const int64_t t = tj / n;
        const int64_t j = tj - t * n;
        const double* Oe = O + e * mO;
        out[x] = inflow ? inflow_at(Oe, jbase, in_off, in_list, j, t0 + t, slots)
                        : Oe[jbase[j] + (t0 + t) * slots];
    }
}

// out[j][t][e]
__global__ void gather_series(const double* __restrict__ O, int64_t mO,
                              const int64_t* __restrict__ jbase,
                              const int64_t* __restrict__ in_off,
                              const int64_t* __restrict__ in_list, bool inflow, int slots,
                              double* __restrict__ out, int64_t n, int64_t T, int64_t E) {
    const int64_t total = n * T * E;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t jt = x / E;
        const int64_t e = x - jt * E;
        const int64_t j = jt / T;
        const int64_t t = jt - j * T;
        const double* Oe = O + e * mO;
        out[x] = inflow ? inflow_at(Oe, jbase, in_off, in_list, j, t, slots)
                        : Oe[jbase[j] + t * slots];
    }
}

inline int grid_for(int64_t work, int block) {
    int64_t g = (work + block - 1) / block;
    if (g < 1) g = 1;
    if (g > 65536) g = 65536;
    return (int)g;
}

}  // namespace

template <bool DENSE>
hipError_t launch_wavefront_t(const WaveArgs& a, int grid, int slots, size_t lds, int members,
                              hipStream_t s) {
    const dim3 g(grid, members);
    switch (slots) {
#define MCR_CASE(S) \
    case S: hipLaunchKernelGGL((wavefront_det<S, DENSE>), g, S, lds, s, a); break;
        MCR_SLOT_LIST(MCR_CASE)
#undef MCR_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_wavefront(const WaveArgs& a, int grid, int slots, size_t lds, bool dense,
                            int members, hipStream_t s) {
    return dense ? launch_wavefront_t<true>(a, grid, slots, lds, members, s)
                 : launch_wavefront_t<false>(a, grid, slots, lds, members, s);
}

hipError_t launch_scatter_to_slots(const double* src, double* dst, const int64_t* slot_reach,
                                   int64_t nslots, int64_t E, hipStream_t s) {
    hipLaunchKernelGGL(scatter_to_slots, grid_for(nslots * E, 256), 256, 0, s, src, dst,
                       slot_reach, nslots, E);
    return hipGetLastError();
}

hipError_t launch_gather_from_slots(const double* src, double* dst, const int64_t* pos,
                                    int64_t n, int64_t nslots, int64_t E, hipStream_t s) {
    hipLaunchKernelGGL(gather_from_slots, grid_for(n * E, 256), 256, 0, s, src, dst, pos, n,
                       nslots, E);
    return hipGetLastError();
}

hipError_t launch_forcing_to_slots(const double* fp, double* F, const int64_t* slot_reach,
                                   int64_t n, int64_t nslots, int64_t n_rows, int64_t E,
                                   hipStream_t s) {
    hipLaunchKernelGGL(forcing_to_slots, grid_for(nslots * n_rows * E, 256), 256, 0, s, fp, F,
                       slot_reach, n, nslots, n_rows, E);
    return hipGetLastError();
}

hipError_t launch_window_index(const int64_t* pos, const int32_t* G, const int32_t* wg_gmin,
                               const int64_t* wbase, int slots, int64_t n, int64_t* jbase,
                               hipStream_t s) {
    if (n > 0)
        hipLaunchKernelGGL(window_index, grid_for(n, 256), 256, 0, s, pos, G, wg_gmin, wbase,
                           slots, n, jbase);
    return hipGetLastError();
}

hipError_t launch_gather_steps(const double* O, int64_t mO, const int64_t* jbase,
                               const int64_t* in_off, const int64_t* in_list, bool inflow,
                               int slots, double* out, int64_t n, int64_t t0, int64_t t1,
                               int64_t E, hipStream_t s) {
    if (n <= 0 || t1 <= t0) return hipSuccess;
    hipLaunchKernelGGL(gather_steps, grid_for(n * (t1 - t0) * E, 256), 256, 0, s, O, mO, jbase,
                       in_off, in_list, inflow, slots, out, n, t0, t1, E);
    return hipGetLastError();
}

hipError_t launch_gather_series(const double* O, int64_t mO, const int64_t* jbase,
                                const int64_t* in_off, const int64_t* in_list, bool inflow,
                                int slots, double* out, int64_t n, int64_t T, int64_t E,
                                hipStream_t s) {
    if (n <= 0 || T <= 0) return hipSuccess;
    hipLaunchKernelGGL(gather_series, grid_for(n * T * E, 256), 256, 0, s, O, mO, jbase, in_off,
                       in_list, inflow, slots, out, n, T, E);
    return hipGetLastError();
}

}  // namespace mcr
