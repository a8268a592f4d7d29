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

// Loads/stores of one 16-tick chunk (128 B): 8 x 16-byte accesses, addresses 16-B aligned.
__device__ __forceinline__ void load_chunk(double (&v)[kChunk], const double* p) {
    const double2* q = reinterpret_cast<const double2*>(p);
#pragma unroll
    for (int k = 0; k < kChunk / 2; ++k) {
        const double2 x = q[k];
        v[2 * k] = x.x;
        v[2 * k + 1] = x.y;
    }
}

__device__ __forceinline__ void store_chunk(double* p, const double (&v)[kChunk]) {
    double2* q = reinterpret_cast<double2*>(p);
#pragma unroll
    for (int k = 0; k < kChunk / 2; ++k) q[k] = make_double2(v[2 * k], v[2 * k + 1]);
}

template <int SLOTS>
__global__ __launch_bounds__(SLOTS) void wavefront_det(WaveArgs a) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int tile = a.tile;
    double* xb = smem;                                  // [2][SLOTS] outflows, tick parity
    double* xe = smem + 2 * SLOTS;                      // [ext_cap][tile] external inputs
    unsigned* xm = reinterpret_cast<unsigned*>(xe + (size_t)a.ext_cap * tile);  // overflow codes

    const int tid = threadIdx.x;
    const int w = a.active[blockIdx.x];
    const int64_t d = (int64_t)w * SLOTS + tid;
    const int T = a.T;
    const int64_t Tp = a.Tp;
    const int k0 = a.kappa0;

    // ---- prologue 1: external inputs (produced by earlier launches) -> LDS
    const int e0 = a.ext_off[w];
    const int ne = a.ext_off[w + 1] - e0;
    for (int idx = tid; idx < ne * tile; idx += SLOTS) {
        const int e = idx / tile;
        const int i = idx - e * tile;
        const int t = k0 + i - a.ext_g[e0 + e];
        const int64_t code = a.ext_src[e0 + e];          // caller row * 16 + pad
        const bool ok = t >= 0 && t < T;
        const double v = a.O[ok ? (code >> 4) * Tp + (code & 15) + t : 0];
        xe[idx] = ok ? v : 0.0;
    }
    // ---- prologue 2: overflow upstream codes of this workgroup -> LDS
    const int m0 = a.up_more_off[(int64_t)w * SLOTS];
    const int nm = a.up_more_off[(int64_t)w * SLOTS + SLOTS] - m0;
    for (int idx = tid; idx < nm; idx += SLOTS) xm[idx] = a.up_more[m0 + idx];

    // ---- per-reach registers
    const uint8_t fl = a.flags[d];
    const int G = a.G[d];
    const int gq = G & ~(kChunk - 1);                   // padded position p = tick - gq
    const int64_t row = a.slot_reach[d];
    const bool real = fl != kSlotPad;
    const int t_first = k0 - G;                         // step at this launch's first tick
    const bool live = real && (t_first < T) && (t_first + tile > 0);
    const double al = a.alpha[d], be = a.beta[d], ch = a.chi[d], ga = a.gamma[d];
    const int cnt = a.up_cnt[d];
    const uint64_t up4 = a.up4[d];
    const int more = a.up_more_off[d] - m0;
    // state at step t_first - 1: initial state or this reach's output from an earlier launch
    const bool from_out = real && t_first >= 1 && t_first <= T;
    const int64_t obase = real ? row * Tp : 0;
    const double o_ld = a.O[from_out ? obase + (k0 - gq) - 1 : 0];
    const double i_ld = a.I[from_out ? obase + (k0 - gq) - 1 : 0];
    double op = from_out ? o_ld : a.st_o[d];
    double ip = from_out ? i_ld : a.st_i[d];
    const double* qrow = a.Q + d * Tp;

    // first chunk of lateral inflow
    double qn[kChunk];
    {
        const int p = k0 - gq;
        load_chunk(qn, (real && p >= 0 && p < Tp) ? qrow + p : a.dummy);
    }
    // the downstream reach (one tick behind) reads step t_first - 1 at the first tick
    xb[((k0 - 1) & 1) * SLOTS + tid] = op;
    // drain every prologue load here: otherwise the wait-count pass carries "pending" state for
    // op/ip into the tick loop and waits for each chunk's stores at every tick
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();

    for (int c = 0; c < tile; c += kChunk) {
        const int kc = k0 + c;
        const int pc = kc - gq;                         // multiple of kChunk
        double qc[kChunk];
#pragma unroll
        for (int i = 0; i < kChunk; ++i) qc[i] = qn[i];
        {                                               // prefetch the next chunk
            const int p = pc + kChunk;
            load_chunk(qn, (real && p >= 0 && p < Tp) ? qrow + p : a.dummy);
        }
        double ob[kChunk], ib[kChunk];
#pragma unroll
        for (int i = 0; i < kChunk; ++i) {
            const int k = kc + i;
            const int t = k - G;
            const bool act = live && t >= 0 && t < T;
            double I = 0.0, o = 0.0;
            if (act) {
                // inflow: upstream outflows in reference finalisation order
                const double* prev = xb + ((k - 1) & 1) * SLOTS;
                const int col = c + i;
                double v[kUpInline];
#pragma unroll
                for (int u = 0; u < kUpInline; ++u) {
                    const unsigned code = (unsigned)((up4 >> (16 * u)) & 0xffffu);
                    const double* src = (code & kExtBit) ? xe + (code & 0x7fffu) * tile + col
                                                         : prev + (code & (SLOTS - 1));
                    v[u] = *src;
                }
#pragma unroll
                for (int u = 0; u < kUpInline; ++u)
                    if (u < cnt) I = I + v[u];
                for (int u = kUpInline; u < cnt; ++u) {
                    const unsigned code = xm[more + u - kUpInline];
                    const double* src = (code & kExtBit) ? xe + (code & 0x7fffu) * tile + col
                                                         : prev + (code & (SLOTS - 1));
                    I = I + *src;
                }
                if (fl == kSlotRouted) o = 0.0 + (((al * I + be * ip) + ch * op) + ga * qc[i]);
                xb[(k & 1) * SLOTS + tid] = o;
                op = o;
                ip = I;
            }
            ob[i] = o;
            ib[i] = I;
            __syncthreads();
        }
        // whole aligned line per row and array; out-of-row chunks go to the dummy line
        const bool in_row = real && pc >= 0 && pc < Tp;
        store_chunk(in_row ? a.O + obase + pc : a.dummy, ob);
        store_chunk(in_row ? a.I + obase + pc : a.dummy + kChunk, ib);
    }
}

// Q[d][t + pad] = interpolated lateral inflow of step t; whole aligned chunks per slot.
__global__ __launch_bounds__(256) void interp_q(InterpArgs a) {
    const int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (d >= a.nslots) return;
    const int pad = a.G[d] & (kChunk - 1);
    double* qrow = a.Q + d * (int64_t)a.Tp;
    for (int p0 = 0; p0 < a.Tp; p0 += kChunk) {
        double v[kChunk];
#pragma unroll
        for (int i = 0; i < kChunk; ++i) {
            const int t = p0 + i - pad;
            double q = 0.0;
            if (t >= 0 && t < a.T) {
                const int2 rr = a.srow[t];
                const double flo = a.F[(int64_t)rr.x * a.nslots + d];
                if (rr.y < 0) {
                    q = flo;
                } else {
                    const double fr = a.sfrac[t];
                    const double fhi = a.F[(int64_t)rr.y * a.nslots + d];
                    q = (1.0 - fr) * flo + fr * fhi;
                }
            }
            v[i] = q;
        }
        store_chunk(qrow + p0, v);
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
                            const int64_t* __restrict__ slot_reach, const int32_t* __restrict__ G,
                            int64_t nslots, int64_t Tp, int64_t T) {
    for (int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; d < nslots;
         d += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = slot_reach[d];
        if (j >= 0) {
            const int64_t at = j * Tp + (G[d] & (kChunk - 1)) + (T - 1);
            st_o[d] = O[at];
            st_i[d] = I[at];
        }
    }
}

// 64 x 64 tile transpose through LDS: reads row segments of S, writes 512-B rows of out.
__global__ __launch_bounds__(256) void transpose_rt(const double* __restrict__ S,
                                                    const uint8_t* __restrict__ rpad,
                                                    double* __restrict__ out, int64_t n,
                                                    int64_t Tp, int64_t t0, int64_t t1) {
    __shared__ double tileb[64][65];
    const int64_t j0 = (int64_t)blockIdx.x * 64;
    const int64_t tb = t0 + (int64_t)blockIdx.y * 64;
    const int lx = threadIdx.x & 63;
    const int ly = threadIdx.x >> 6;  // 0..3
    for (int r = ly; r < 64; r += 4) {
        const int64_t j = j0 + r;
        const int64_t t = tb + lx;
        tileb[r][lx] = (j < n && t < t1) ? S[j * Tp + rpad[j] + t] : 0.0;
    }
    __syncthreads();
    for (int r = ly; r < 64; r += 4) {
        const int64_t t = tb + r;
        const int64_t j = j0 + lx;
        if (t < t1 && j < n) out[(t - t0) * n + j] = tileb[lx][r];
    }
}

__global__ void compact_rows(const double* __restrict__ S, const uint8_t* __restrict__ rpad,
                             double* __restrict__ out, int64_t n, int64_t Tp, int64_t T) {
    const int64_t total = n * T;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = x / T;
        const int64_t t = x - j * T;
        out[x] = S[j * Tp + rpad[j] + t];
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

hipError_t launch_interp(const InterpArgs& a, hipStream_t s) {
    if (a.nslots <= 0) return hipSuccess;
    hipLaunchKernelGGL(interp_q, (unsigned)((a.nslots + 255) / 256), 256, 0, s, a);
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
                              const int64_t* slot_reach, const int32_t* G, int64_t nslots,
                              int64_t Tp, int64_t T, hipStream_t s) {
    hipLaunchKernelGGL(final_state, grid_for(nslots, 256), 256, 0, s, O, I, st_o, st_i,
                       slot_reach, G, nslots, Tp, T);
    return hipGetLastError();
}

hipError_t launch_transpose(const double* S, const uint8_t* rpad, double* out, int64_t n,
                            int64_t Tp, int64_t t0, int64_t t1, hipStream_t s) {
    if (n <= 0 || t1 <= t0) return hipSuccess;
    dim3 grid((unsigned)((n + 63) / 64), (unsigned)((t1 - t0 + 63) / 64));
    hipLaunchKernelGGL(transpose_rt, grid, 256, 0, s, S, rpad, out, n, Tp, t0, t1);
    return hipGetLastError();
}

hipError_t launch_compact(const double* S, const uint8_t* rpad, double* out, int64_t n,
                          int64_t Tp, int64_t T, hipStream_t s) {
    if (n <= 0 || T <= 0) return hipSuccess;
    hipLaunchKernelGGL(compact_rows, grid_for(n * T, 256), 256, 0, s, S, rpad, out, n, Tp, T);
    return hipGetLastError();
}

}  // namespace mcr
