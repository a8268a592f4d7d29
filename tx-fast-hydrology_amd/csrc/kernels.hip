// Muskingum routing kernels for CDNA4 (gfx950).
//
// Hot path: `wavefront_det` -- the time-skewed wavefront sweep that replaces the per-step
// serial walk of nutils.py:64-89 (`_ax_bu`) driven by muskingum.py:499-536 (`simulate_iter`).
// One workgroup owns up to SLOTS reaches (one per lane).  Reach j handles model step t at tick
// G[j] + t; an upstream reach in the same cluster runs one tick ahead, so its outflow is read
// from an LDS double buffer written in the previous tick.  Inputs from other clusters were
// produced in an earlier launch and are staged in LDS in the launch prologue.
//
// Arithmetic follows the reference exactly (FMA contraction is off for this file):
//   I = ((0 + o[u1]) + o[u2]) + ...          upstream reaches in reference finalisation order
//   o = 0 + (((alpha*I + beta*I_prev) + chi*o_prev) + gamma*q)            nutils.py:80-83
//   q = (1 - frac) * f[ix-1] + frac * f[ix]   (or a row copy at the ends)  nutils.py:23-33
#include "kernels.hpp"
#include "plan.hpp"

#pragma clang fp contract(off)

namespace mcr {

namespace {

template <int SLOTS>
__global__ __launch_bounds__(SLOTS) void wavefront_det(WaveArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    double* xb = smem;                  // [2][SLOTS] outflow of the previous / current tick
    double* xe = smem + 2 * SLOTS;      // [n_ext][tile] external inputs of this launch

    const int tid = threadIdx.x;
    const int w = a.active[blockIdx.x];
    const int64_t d = (int64_t)w * SLOTS + tid;
    const int tile = a.tile;
    const int T = a.T;
    const int k0 = a.kappa0;

    // ---- prologue: external inputs (produced by earlier launches) -> LDS
    const int e0 = a.ext_off[w];
    const int ne = a.ext_off[w + 1] - e0;
    for (int idx = tid; idx < ne * tile; idx += SLOTS) {
        const int e = idx / tile;
        const int i = idx - e * tile;
        const int t = k0 + i - a.ext_g[e0 + e];
        double v = 0.0;
        if (t >= 0 && t < T) v = a.O[a.ext_src[e0 + e] * (int64_t)T + t];
        xe[idx] = v;
    }

    // ---- per-reach registers
    const uint8_t fl = a.flags[d];
    const int G = a.G[d];
    const int64_t row = a.slot_reach[d];
    const int t_first = k0 - G;               // model step at the first tick of this launch
    double al = 0.0, be = 0.0, ch = 0.0, ga = 0.0, op = 0.0, ip = 0.0;
    int cnt = 0, more = 0;
    uint64_t up4 = 0;
    // live: the reach has at least one model step inside this launch's ticks
    const bool live = (fl != kSlotPad) && (t_first < T) && (t_first + tile > 0);
    if (live) {
        al = a.alpha[d];
        be = a.beta[d];
        ch = a.chi[d];
        ga = a.gamma[d];
        cnt = a.up_cnt[d];
        up4 = a.up4[d];
        more = a.up_more_off[d];
    }
    // state at step t_first - 1: initial state, or this reach's output from an earlier launch
    if (fl != kSlotPad && t_first <= T && t_first + tile > 0) {
        if (t_first <= 0) {
            op = a.st_o[d];
            ip = a.st_i[d];
        } else {
            op = a.O[row * T + (t_first - 1)];
            ip = a.I[row * T + (t_first - 1)];
        }
    }
    // the downstream reach (one tick behind) reads this reach's step t_first - 1 outflow at the
    // first tick of the launch
    xb[((k0 - 1) & 1) * SLOTS + tid] = op;

    // forcing bracket kept in registers; step table prefetched one tick ahead
    int r_lo = -1, r_hi = -1, r_nx = -1;
    double f_lo = 0.0, f_hi = 0.0, f_nx = 0.0;
    int tc = t_first < 0 ? 0 : (t_first >= T ? T - 1 : t_first);
    int2 rr_n = make_int2(0, -1);
    double2 ww_n = make_double2(0.0, 0.0);
    if (live) {
        rr_n = a.srow[tc];
        ww_n = a.sw[tc];
    }
    __syncthreads();

    for (int i = 0; i < tile; ++i) {
        const int k = k0 + i;
        const int t = k - G;
        const int2 rr = rr_n;
        const double2 ww = ww_n;
        if (live && t >= 0 && t < T) {
            if (t + 1 < T) {                  // prefetch next tick's step table entry
                rr_n = a.srow[t + 1];
                ww_n = a.sw[t + 1];
            }
            // inflow: upstream outflows in reference finalisation order
            double I = 0.0;
            const double* prev = xb + ((k - 1) & 1) * SLOTS;
            for (int u = 0; u < cnt; ++u) {
                const unsigned code = u < kUpInline ? (unsigned)((up4 >> (16 * u)) & 0xffffu)
                                                    : (unsigned)a.up_more[more + u - kUpInline];
                const double v = (code & kExtBit) ? xe[(code & 0x7fffu) * tile + i] : prev[code];
                I = I + v;
            }
            // lateral inflow (interpolate_sample, linear)
            if (rr.x != r_lo) {
                if (rr.x == r_hi) f_lo = f_hi;
                else if (rr.x == r_nx) f_lo = f_nx;
                else f_lo = a.F[(int64_t)rr.x * a.nslots + d];
                r_lo = rr.x;
            }
            double q;
            if (rr.y < 0) {
                q = f_lo;
            } else {
                if (rr.y != r_hi) {
                    f_hi = (rr.y == r_nx) ? f_nx : a.F[(int64_t)rr.y * a.nslots + d];
                    r_hi = rr.y;
                    if (r_hi + 1 < a.n_rows && r_nx != r_hi + 1) {   // next row, ~1 bracket ahead
                        r_nx = r_hi + 1;
                        f_nx = a.F[(int64_t)r_nx * a.nslots + d];
                    }
                }
                q = ww.x * f_lo + ww.y * f_hi;
            }
            double o = 0.0;
            if (fl == kSlotRouted) o = 0.0 + (((al * I + be * ip) + ch * op) + ga * q);
            xb[(k & 1) * SLOTS + tid] = o;
            a.O[row * T + t] = o;
            a.I[row * T + t] = I;
            op = o;
            ip = I;
        }
        __syncthreads();
    }
}

__global__ void scatter_to_slots(const double* __restrict__ src, double* __restrict__ dst,
                                 const int64_t* __restrict__ slot_reach, int64_t nslots) {
    for (int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; d < nslots;
         d += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = slot_reach[d];
        dst[d] = j >= 0 ? src[j] : 0.0;
    }
}

__global__ void gather_from_slots(const double* __restrict__ src, double* __restrict__ dst,
                                  const int64_t* __restrict__ pos, int64_t n) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n;
         j += (int64_t)gridDim.x * blockDim.x)
        dst[j] = src[pos[j]];
}

__global__ void forcing_to_slots(const double* __restrict__ fp, double* __restrict__ F,
                                 const int64_t* __restrict__ slot_reach, int64_t n,
                                 int64_t nslots, int64_t n_rows) {
    const int64_t total = nslots * n_rows;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = x / nslots;
        const int64_t d = x - r * nslots;
        const int64_t j = slot_reach[d];
        F[x] = j >= 0 ? fp[r * n + j] : 0.0;
    }
}

__global__ void final_state(const double* __restrict__ O, const double* __restrict__ I,
                            double* __restrict__ st_o, double* __restrict__ st_i,
                            const int64_t* __restrict__ slot_reach, int64_t nslots, int64_t T) {
    for (int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; d < nslots;
         d += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = slot_reach[d];
        if (j >= 0) {
            st_o[d] = O[j * T + (T - 1)];
            st_i[d] = I[j * T + (T - 1)];
        }
    }
}

// 64 x 64 tile transpose through LDS: reads 512-B row segments of O, writes 512-B rows of out.
__global__ __launch_bounds__(256) void transpose_rt(const double* __restrict__ O,
                                                    double* __restrict__ out, int64_t n,
                                                    int64_t T, int64_t t0, int64_t t1) {
    __shared__ double tileb[64][65];
    const int64_t j0 = (int64_t)blockIdx.x * 64;
    const int64_t tb = t0 + (int64_t)blockIdx.y * 64;
    const int lx = threadIdx.x & 63;
    const int ly = threadIdx.x >> 6;  // 0..3
    for (int r = ly; r < 64; r += 4) {
        const int64_t j = j0 + r;
        const int64_t t = tb + lx;
        tileb[r][lx] = (j < n && t < t1) ? O[j * T + t] : 0.0;
    }
    __syncthreads();
    for (int r = ly; r < 64; r += 4) {
        const int64_t t = tb + r;
        const int64_t j = j0 + lx;
        if (t < t1 && j < n) out[(t - t0) * n + j] = tileb[lx][r];
    }
}

inline int grid_for(int64_t work, int block) {
    int64_t g = (work + block - 1) / block;
    if (g < 1) g = 1;
    if (g > 65536) g = 65536;
    return (int)g;
}

}  // namespace

hipError_t launch_wavefront(const WaveArgs& a, int grid, int slots, size_t lds, hipStream_t s) {
    switch (slots) {
        case 64: hipLaunchKernelGGL(wavefront_det<64>, grid, 64, lds, s, a); break;
        case 128: hipLaunchKernelGGL(wavefront_det<128>, grid, 128, lds, s, a); break;
        case 256: hipLaunchKernelGGL(wavefront_det<256>, grid, 256, lds, s, a); break;
        case 512: hipLaunchKernelGGL(wavefront_det<512>, grid, 512, lds, s, a); break;
        case 1024: hipLaunchKernelGGL(wavefront_det<1024>, grid, 1024, lds, s, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_scatter_to_slots(const double* src, double* dst, const int64_t* slot_reach,
                                   int64_t nslots, hipStream_t s) {
    hipLaunchKernelGGL(scatter_to_slots, grid_for(nslots, 256), 256, 0, s, src, dst, slot_reach,
                       nslots);
    return hipGetLastError();
}

hipError_t launch_gather_from_slots(const double* src, double* dst, const int64_t* pos,
                                    int64_t n, hipStream_t s) {
    hipLaunchKernelGGL(gather_from_slots, grid_for(n, 256), 256, 0, s, src, dst, pos, n);
    return hipGetLastError();
}

hipError_t launch_forcing_to_slots(const double* fp, double* F, const int64_t* slot_reach,
                                   int64_t n, int64_t nslots, int64_t n_rows, hipStream_t s) {
    hipLaunchKernelGGL(forcing_to_slots, grid_for(nslots * n_rows, 256), 256, 0, s, fp, F,
                       slot_reach, n, nslots, n_rows);
    return hipGetLastError();
}

hipError_t launch_final_state(const double* O, const double* I, double* st_o, double* st_i,
                              const int64_t* slot_reach, int64_t nslots, int64_t T,
                              hipStream_t s) {
    hipLaunchKernelGGL(final_state, grid_for(nslots, 256), 256, 0, s, O, I, st_o, st_i,
                       slot_reach, nslots, T);
    return hipGetLastError();
}

hipError_t launch_transpose(const double* O, double* out, int64_t n, int64_t T, int64_t t0,
                            int64_t t1, hipStream_t s) {
    if (n <= 0 || t1 <= t0) return hipSuccess;
    dim3 grid((unsigned)((n + 63) / 64), (unsigned)((t1 - t0 + 63) / 64));
    hipLaunchKernelGGL(transpose_rt, grid, 256, 0, s, O, out, n, T, t0, t1);
    return hipGetLastError();
}

}  // namespace mcr
