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
// row per wave, active cells only (workgroup windows, kernels.hpp).
//
// Arithmetic follows the reference exactly (FMA contraction is off for this file):
//   I = ((0 + o[u1]) + o[u2]) + ...          upstream reaches in reference finalisation order
//   o = 0 + (((alpha*I + beta*I_prev) + chi*o_prev) + gamma*q)            nutils.py:80-83
//   q = (1 - frac) * f[ix-1] + frac * f[ix]   (or a row copy at the ends)  nutils.py:23-33
#include "kernels.hpp"

#include <algorithm>
#include "plan.hpp"
#include "device_common.hpp"

#pragma clang fp contract(off)

namespace mcr {

namespace {

using dev::chunk_rows;
using dev::clamp_row;
using dev::lds_f64;
using dev::Slot;
using dev::load_slot;
using dev::decode_codes;
using dev::fold_values;
using dev::read_inputs;

// LDS layout of one workgroup (bytes), RS = K * SLOTS node slots (lane l: slots p * SLOTS + l
// for positions p < K):
//   XB  [RS + 1][2] f64   output of each node slot at tick parity 0/1; slot RS stays 0.0
//   FR  [RS][3]     f64   each slot's forcing rows rb .. rb + 2 of the current chunk
//   TAB [table_cap] int4  step-table window {row_lo, row_hi, frac}
//   XE  [ext_cap][tile] f64 external inputs of this launch
// Each tick a lane routes its K positions in order; position p may take the output of position
// p - 1 of the same tick from a register (SELF code), so a chained edge costs no tick.
// DENSE: some chunk needs more than 3 forcing rows (model step >= ~1/3 of the forcing interval);
// those lanes read the forcing straight from global memory.  A separate instantiation keeps the
// direct loads (and the waits they need) out of the common kernel.
template <int SLOTS, int K, bool DENSE>
__global__ __launch_bounds__(SLOTS)
__attribute__((amdgpu_waves_per_eu(K >= 4 ? 1 : 2, K >= 4 ? 1 : 2)))
void wavefront_det(WaveArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int RS = K * SLOTS;
    const int tile = a.tile;
    constexpr unsigned XB = 0;
    constexpr unsigned FR = XB + (RS + 1) * 16;
    constexpr unsigned TAB = FR + RS * 24;
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
    const int T = a.T;
    const int k0 = a.kappa0;
    const int64_t ns = a.nslots;
    const int nrow = a.n_rows;
    const int gminw = a.wg_gmin[w], gmaxw = a.wg_gmax[w];
    const int64_t wb = a.wbase[w];

    // ---- per-slot registers (issued first: longest latency)
    Slot S[K];
    uint64_t up[K];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        load_slot(S[p], a, (int64_t)w * RS + p * SLOTS + tid, mem, k0, tile, T);
        up[p] = a.up4[S[p].d];
    }

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
    // the consumer (one tick behind) reads step t_first - 1 at the first tick: the producer's
    // state o, or for a partial sum (whose state stays 0, Slot::Ga) its output of tick k0 - 1,
    // stored by the previous launch in the output window.  (S.G is huge for a slot with no step
    // in THIS launch -- e.g. a partial sum whose last step was tick k0 - 1 -- so the plan's G.)
#pragma unroll
    for (int p = 0; p < K; ++p) {
        double carry = S[p].op;
        if (S[p].psum && (unsigned)(k0 - 1 - a.G[S[p].d]) < (unsigned)T)
            carry = Om[wb + (int64_t)(k0 - 1 - gminw) * RS + p * SLOTS + tid];
        xbp[(p * SLOTS + tid) * 2 + ((k0 - 1) & 1)] = carry;
    }
    // sync plans (plan.hpp): local inputs, XE columns next .. next + nloc - 1 of this
    // workgroup, deliver at tick k the producer's output of tick k - kWaveSlack.  The first
    // kWaveSlack ticks of the launch take them from the previous launch's output window (active
    // cells only: an inactive producer tick feeds an inactive consumer tick); the producers
    // write the rest during this launch (tick loop below, one tick barrier apart at least).
    const int next = a.ext_off[w + 1] - e0;
    int lx_col[K];
#pragma unroll
    for (int p = 0; p < K; ++p) lx_col[p] = -1;
    if (a.lx_off) {
        const int l0 = a.lx_off[w], nloc = a.lx_off[w + 1] - l0;
        for (int idx = tid; idx < nloc * kWaveSlack; idx += SLOTS) {
            const int li = idx / kWaveSlack, q = idx - li * kWaveSlack;
            const int64_t src = a.lx_src[l0 + li];
            const int kk = k0 - kWaveSlack + q;
            const bool act = (unsigned)(kk - a.G[src]) < (unsigned)T;
            xe[(next + li) * tile + q] =
                act ? Om[wb + (int64_t)(kk - gminw) * RS + (src - (int64_t)w * RS)] : 0.0;
        }
#pragma unroll
        for (int p = 0; p < K; ++p) lx_col[p] = a.lx[S[p].d];
    }
    bool lx_any = false;                                // wave-uniform: skip the writes below
#pragma unroll
    for (int p = 0; p < K; ++p) lx_any = lx_any || lx_col[p] >= 0;
    lx_any = __any(lx_any);
    if (tid < 2) xbp[RS * 2 + tid] = 0.0;               // zero slot for unused codes
    // drain every prologue load: otherwise the wait-count pass carries "pending" state into
    // the tick loop and waits for each chunk's stores at every tick
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();

    bool any3[K];
    unsigned own[K];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        decode_codes<RS>(S[p], up[p], XB, 16u, XE, (unsigned)tile * 8);
        any3[p] = __any(S[p].cnt > 2);                  // wave-uniform
        own[p] = XB + (unsigned)(p * SLOTS + tid) * 16;
    }

    // forcing rows of the first chunk
    int rb[K], nr[K];
    double f0[K], f1[K], f2[K];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        chunk_rows(tab, tw0, k0, S[p].G, T, rb[p], nr[p]);
        f0[p] = Fm[(int64_t)clamp_row(rb[p], nrow) * ns + S[p].d];
        f1[p] = Fm[(int64_t)clamp_row(rb[p] + 1, nrow) * ns + S[p].d];
        f2[p] = Fm[(int64_t)clamp_row(rb[p] + 2, nrow) * ns + S[p].d];
    }
    __builtin_amdgcn_s_waitcnt(0);   // same reason: nothing pending may enter the loop
    const int64_t t_loop = a.trace ? wall_clock64() : 0;
    const int64_t c_loop = a.trace ? clock64() : 0;

    constexpr bool kBatchQ = K <= 2;                    // lateral inflows per chunk (registers)
    const bool maskq = a.nf == nullptr ||               // non-finite forcing (device flag)
                       __hip_atomic_load(a.nff, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    bool anyps = false;                                 // a partial sum in this wave
#pragma unroll
    for (int p = 0; p < K; ++p) anyps = anyps || S[p].psum;
    anyps = __any(anyps);
    for (int c = 0; c < tile; c += kChunk) {
        const int kc = k0 + c;
        // this chunk's forcing rows -> the slots' LDS rows (private: no barrier needed)
        unsigned frp[K], tp[K];
        bool slow = false;
#pragma unroll
        for (int p = 0; p < K; ++p) {
            double* fr = reinterpret_cast<double*>(lds + FR) + (p * SLOTS + tid) * 3;
            fr[0] = f0[p];
            fr[1] = f1[p];
            fr[2] = f2[p];
            slow = slow || (DENSE && __any(nr[p] > 3));
            frp[p] = FR + (unsigned)(p * SLOTS + tid) * 24 - (unsigned)rb[p] * 8;
            tp[p] = TAB + (unsigned)(kc - S[p].G - tw0) * 16u;
        }
        // prefetch the forcing rows of the next chunk (clamped rows), only for slots that run a
        // step in it (the rows of the others would feed ticks whose outputs are not kept)
        const int Tn = c + kChunk < tile ? T : 0;
        const int kn = kc + kChunk;
        int rbn[K], nrn[K];
        double g0[K], g1[K], g2[K];
#pragma unroll
        for (int p = 0; p < K; ++p) {
            chunk_rows(tab, tw0, kn, S[p].G, Tn, rbn[p], nrn[p]);
            g0[p] = g1[p] = g2[p] = 0.0;
            if (Tn > 0 && kn + kChunk > S[p].G && kn < S[p].G + T) {
                g0[p] = Fm[(int64_t)clamp_row(rbn[p], nrow) * ns + S[p].d];
                g1[p] = Fm[(int64_t)clamp_row(rbn[p] + 1, nrow) * ns + S[p].d];
                g2[p] = Fm[(int64_t)clamp_row(rbn[p] + 2, nrow) * ns + S[p].d];
            }
        }
        // per-chunk LDS cursors: input value of tick i at m[u] + 8 * ((i + 1) & 1)
        unsigned m[K][kUpInline];
#pragma unroll
        for (int p = 0; p < K; ++p)
#pragma unroll
            for (int u = 0; u < kUpInline; ++u)
                m[p][u] = S[p].uext[u] ? S[p].ubase[u] + 8u * c - 8u : S[p].ubase[u];
        // the masked high row of clamped steps only for non-finite forcing (for finite forcing
        // (1 - 0) lo + 0 lo is lo exactly), the frozen state of partial sums only in waves that
        // hold one: four straight-line forms of the chunk, the common one inline (flow.hip)
        auto run_chunk = [&](auto mtag, auto ptag) {
            constexpr bool MASKQ = decltype(mtag)::value, PSUM = decltype(ptag)::value;
            // lateral inflow of position p at tick j of the chunk, interpolate_sample
            // (nutils.py:23-33); it does not depend on the routing state (off the tick's chain)
            auto q_of = [&](int p, int j) -> double {
                const int4 e = *reinterpret_cast<const int4*>(lds + tp[p] + 16u * j);
                double lo, hi;
                if (DENSE && slow) {
                    lo = Fm[(int64_t)clamp_row(e.x < 0 ? 0 : e.x, nrow) * ns + S[p].d];
                    hi = Fm[(int64_t)clamp_row(e.y < 0 ? 0 : e.y, nrow) * ns + S[p].d];
                } else {
                    lo = lds_f64(lds, frp[p] + 8u * (unsigned)e.x);
                    hi = lds_f64(lds, frp[p] + 8u * (unsigned)e.y);
                }
                const double f = __hiloint2double(e.w, e.z);
                // clamped steps (frac = 0, row_lo == row_hi): lo + 0 * 0 -- the row itself as the
                // reference copies it (nutils.py:24-27), also for +-Inf / NaN rows, where
                // (1 - 0) f + 0 f is not (the sign of a zero q cannot reach the outflow, whose
                // update ends in 0 + ...).  (A select of lo instead costs the dataflow kernel 32
                // VGPRs in its batched q.)
                if constexpr (MASKQ) hi = f == 0.0 ? 0.0 : hi;
                const double qq = (1.0 - f) * lo + f * hi;
                return qq;
            };
            double qb[kBatchQ ? K : 1][kBatchQ ? kChunk : 1];
            if constexpr (kBatchQ) {
#pragma unroll
                for (int j = 0; j < kChunk; ++j)
#pragma unroll
                    for (int p = 0; p < K; ++p) qb[p][j] = q_of(p, j);
                if (DENSE && slow) __builtin_amdgcn_s_waitcnt(0);  // settle the direct loads here
            }
#pragma unroll
            for (int i = 0; i < kChunk; ++i) {
                if (i & 1) {
#pragma unroll
                    for (int p = 0; p < K; ++p)
#pragma unroll
                        for (int u = 0; u < kUpInline; ++u) m[p][u] += S[p].uext[u] ? 16u : 0u;
                }
                const unsigned rd = 8u * ((i + 1) & 1);     // parity of tick k - 1
                const int k = kc + i;
                double qv[K];
#pragma unroll
                for (int p = 0; p < K; ++p) {
                    if constexpr (kBatchQ) qv[p] = qb[p][i];
                    else qv[p] = q_of(p, i);
                }
                double vin[K][kUpInline];
#pragma unroll
                for (int p = 0; p < K; ++p) read_inputs(lds, m[p], rd, any3[p], vin[p]);
                double ov[K];
                bool act[K];
                double prev = 0.0;
#pragma unroll
                for (int p = 0; p < K; ++p) {
                    act[p] = (unsigned)(k - S[p].G) < (unsigned)T;
                    bool upd = act[p];
                    if constexpr (PSUM) upd = upd && !S[p].psum;   // partial sums: zero state
                    const double I = fold_values(vin[p], S[p].chained, any3[p], prev, p == 0);
                    const double rr = dev::muskingum_update(S[p].al, I, S[p].be, S[p].ip,
                                                            S[p].ch, S[p].op,
                                                            dev::gq_term(S[p].ga, qv[p]));
                    const double o = rr;   // psum / unrouted / pad: coefficients set_slot_coeffs
                    S[p].op = upd ? o : S[p].op;
                    S[p].ip = upd ? I : S[p].ip;
                    ov[p] = o;
                    prev = o;
                }
                // inactive ticks write garbage that no active node reads (its consumer is inactive
                // one tick later); never-processed reaches (no consumer) output 0
#pragma unroll
                for (int p = 0; p < K; ++p)
                    *reinterpret_cast<double*>(lds + own[p] + 8u * (i & 1)) = ov[p];
                // row k - gmin of the workgroup's window; only active (slot, tick) cells are stored
                // (slots are sorted by G, so a wave's active lanes are a contiguous run and the
                // masked rows stay whole 32-B sectors except at the run's ends): the window cells a
                // slot does not run in are never read (window_index), so they are not written
                {
                    double* orow = Om + wb + (int64_t)(k - gminw) * RS;
#pragma unroll
                    for (int p = 0; p < K; ++p) {
                        // non-temporal: rows are written once and read only by later fetches
                        if (act[p]) {
                            __builtin_nontemporal_store(ov[p], orow + p * SLOTS + tid);
                            if (S[p].xsrc) XSm[S[p].xs0 + k] = ov[p];
                        }
                    }
                }
                // local edges of sync plans: the consumer's input of tick k + kWaveSlack
                if (lx_any) {
#pragma unroll
                    for (int p = 0; p < K; ++p)
                        if (lx_col[p] >= 0 && c + i + kWaveSlack < tile)
                            xe[lx_col[p] * tile + c + i + kWaveSlack] = ov[p];
                }
                __syncthreads();
            }
        };
        using yes = std::true_type;
        using no = std::false_type;
        if (__builtin_expect(!maskq && !anyps, 1)) [[likely]] {
            run_chunk(no{}, no{});
        } else if (maskq) {
            if (anyps) run_chunk(yes{}, yes{});
            else run_chunk(yes{}, no{});
        } else {
            run_chunk(no{}, yes{});
        }
#pragma unroll
        for (int p = 0; p < K; ++p) {
            rb[p] = rbn[p];
            nr[p] = nrn[p];
            f0[p] = g0[p];
            f1[p] = g1[p];
            f2[p] = g2[p];
        }
    }
    // state for the next launch; never-processed reaches hold o = 0 as in the reference's fresh
    // o_t_next.  Slots that did not run in this launch (load_slot: G = 1 << 29) keep theirs
    // unchanged, so only the live ones are stored
    const int64_t sb = (int64_t)blockIdx.y * a.mS;
    bool nonfin = false;
#pragma unroll
    for (int p = 0; p < K; ++p) {
        if (S[p].G != (1 << 29)) {
            const double so = S[p].unr ? 0.0 : S[p].op;        // unrouted: o stays 0
            a.st_o[sb + S[p].d] = so;
            a.st_i[sb + S[p].d] = S[p].ip;
            nonfin = nonfin || !__builtin_isfinite(so) || !__builtin_isfinite(S[p].ip);
        }
    }
    if (a.nf && __any(nonfin) && (tid & 63) == 0)          // the dataflow kernel's fast form
        __hip_atomic_store(a.nf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

// Device coefficients by slot kind, so that the tick needs no per-slot selects: a partial-sum
// node computes 0 + (((1 I + 0 Ip) + 0 Op) + 0 q) = I, an unrouted reach (never processed by
// the reference walk) and a padding slot 0 + (((0 I + 0 Ip) + 0 Op) + 0 q) = +0 -- exact for
// finite values (the reference keeps o = 0 for unrouted reaches, nutils.py:68)
__global__ void set_slot_coeffs(const uint8_t* __restrict__ flags, double* __restrict__ alpha,
                                double* __restrict__ beta, double* __restrict__ chi,
                                double* __restrict__ gamma, int64_t ns) {
    for (int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; d < ns;
         d += (int64_t)gridDim.x * blockDim.x) {
        const uint8_t f = flags[d];
        if (f == kSlotRouted) continue;
        alpha[d] = f == kSlotSum ? 1.0 : 0.0;
        beta[d] = 0.0;
        chi[d] = 0.0;
        gamma[d] = 0.0;
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

// F [e][r][slot] from the caller's forcing: step-major fp [r][j][e] or, reach_major, the
// series layout fp [j][r][e] (a pandas frame's own block, no host transpose)
__global__ void forcing_to_slots(const double* __restrict__ fp, double* __restrict__ F,
                                 const int64_t* __restrict__ slot_reach, int64_t n,
                                 int64_t nslots, int64_t n_rows, int64_t E, bool reach_major) {
    const int64_t total = nslots * n_rows * E;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t er = x / nslots;                  // e * n_rows + r
        const int64_t d = x - er * nslots;
        const int64_t e = er / n_rows;
        const int64_t r = er - e * n_rows;
        const int64_t j = slot_reach[d];
        F[x] = j >= 0 ? fp[(reach_major ? j * n_rows + r : r * n + j) * E + e] : 0.0;
    }
}

__global__ void window_index(const int64_t* __restrict__ pos, const int32_t* __restrict__ G,
                             const uint8_t* __restrict__ flags,
                             const int32_t* __restrict__ wg_gmin,
                             const int64_t* __restrict__ wbase, int slots, int64_t n,
                             int64_t* __restrict__ jbase) {
    for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < n;
         j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t d = pos[j];
        const int64_t w = d / slots;
        // never-processed reaches: -1, their outflow reads as 0 (nutils.py:68); the kernels'
        // own value for them (0 q + ...) is NaN for non-finite inputs
        jbase[j] = flags[d] == kSlotUnrouted
                       ? -1
                       : wbase[w] + (int64_t)(G[d] - wg_gmin[w]) * slots + (d - w * slots);
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
        const int64_t jb = jbase[j];
        out[x] = inflow ? inflow_at(Oe, jbase, in_off, in_list, j, t0 + t, slots)
                        : (jb < 0 ? 0.0 : Oe[jb + (t0 + t) * slots]);
    }
}

// Both series of a step block in reach order from the output windows (E = 1), in two passes
// (kernels.hpp launch_gather_slots).  Reading the windows in reach order loads one random
// 8-byte cell per (reach, step) from all over the windows (0.6 GB for Texas, more than the
// Infinity cache): 1.63 ms per Texas horizon for o + i, ~0.8 TB/s.  Here
//   1. unskew_windows: thread per slot, kUnskewSteps steps each -> S[t][slot] (slot order).  A
//      wave's 64 slots read their window column pieces (slots of equal schedule offset share
//      lines, a line is re-read at the neighbouring slots' steps from L2) and store whole rows;
//   2. permute_steps: S[t] -> reach order, out_o[t][j] = S[t][pos[j]] and the inflow fold
//      ((0 + S[t][pos[u1]]) + ...) over j's rank-ordered inflow list.  The random reads stay in
//      one step's row (nslots doubles, 1.6 MB for Texas): workgroup b runs on XCD b % 8
//      (round-robin dispatch), so XCD x takes the steps t0 + x, t0 + x + 8, ... one after the
//      other and each row is read from HBM once, into that XCD's L2.
// Same values as reading the windows directly (pass 1 copies the cells; never-processed and
// padding slots read 0).
constexpr int kUnskewSteps = 16;
__global__ __launch_bounds__(256) void unskew_windows(const double* __restrict__ O,
                                                      const int64_t* __restrict__ sjb,
                                                      int64_t stride, double* __restrict__ S,
                                                      int64_t ns, int64_t t0, int64_t t1) {
    const int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (d >= ns) return;
    const int64_t tb = t0 + (int64_t)blockIdx.y * kUnskewSteps;
    const int nt = (int)(t1 - tb < kUnskewSteps ? t1 - tb : kUnskewSteps);
    const int64_t jb = sjb[d];
    double v[kUnskewSteps];
#pragma unroll
    for (int q = 0; q < kUnskewSteps; ++q)
        v[q] = (jb < 0 || q >= nt) ? 0.0 : O[jb + (tb + q) * stride];
#pragma unroll
    for (int q = 0; q < kUnskewSteps; ++q)
        if (q < nt) S[(tb + q - t0) * ns + d] = v[q];
}

// kPermuteSteps steps per thread (t, t + 8, ...: all on the thread's XCD), so the index loads
// are shared, and non-temporal series stores (they pass the L2 that holds the steps' rows):
// 0.97 ms for both Texas series (same box: plain stores 1.04, one step per thread 1.04-1.07,
// four 1.27, non-temporal index loads too 1.26; non-temporal scratch stores in the first pass
// within noise)
constexpr int kPermuteSteps = 2;
__global__ __launch_bounds__(256) void permute_steps(
        const double* __restrict__ S, const int32_t* __restrict__ pos,
        const int32_t* __restrict__ in_off, const int32_t* __restrict__ upos,
        double* __restrict__ out_o, double* __restrict__ out_i, int64_t n, int64_t ns,
        int64_t t0, int64_t t1, int ntile) {
    constexpr int P = kPermuteSteps;
    auto st = [](double v, double* p) { __builtin_nontemporal_store(v, p); };
    const int x = (int)(blockIdx.x & 7);
    const int64_t q = blockIdx.x >> 3;
    const int64_t tb = t0 + (q / ntile) * 8 * P + x;     // steps tb, tb + 8, ... (P of them)
    const int64_t j = (q % ntile) * 256 + threadIdx.x;
    if (tb >= t1 || j >= n) return;
    if (out_o) {
        const int64_t d = pos[j];
        double v[P];
#pragma unroll
        for (int h = 0; h < P; ++h) {
            const int64_t t = tb + 8 * h;
            v[h] = t < t1 ? S[(t - t0) * ns + d] : 0.0;
        }
#pragma unroll
        for (int h = 0; h < P; ++h) {
            const int64_t t = tb + 8 * h;
            if (t < t1) st(v[h], out_o + (t - t0) * n + j);
        }
    }
    if (out_i) {
        const int32_t k0 = in_off[j], k1 = in_off[j + 1];
        double sm[P];
#pragma unroll
        for (int h = 0; h < P; ++h) sm[h] = 0.0;
        for (int32_t k = k0; k < k1; ++k) {
            const int64_t u = upos[k];
#pragma unroll
            for (int h = 0; h < P; ++h) {
                const int64_t t = tb + 8 * h;
                if (t < t1) sm[h] = sm[h] + S[(t - t0) * ns + u];
            }
        }
#pragma unroll
        for (int h = 0; h < P; ++h) {
            const int64_t t = tb + 8 * h;
            if (t < t1) st(sm[h], out_i + (t - t0) * n + j);
        }
    }
}

// window index of step 0 of every node slot (-1: padding and never-processed slots)
__global__ void slot_window_index(const int32_t* __restrict__ G, const uint8_t* __restrict__ flags,
                                  const int32_t* __restrict__ wg_gmin,
                                  const int64_t* __restrict__ wbase, int slots, int64_t ns,
                                  int64_t* __restrict__ sjb) {
    for (int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; d < ns;
         d += (int64_t)gridDim.x * blockDim.x) {
        const int64_t w = d / slots;
        const uint8_t fl = flags[d];
        sjb[d] = fl == kSlotUnrouted || fl == kSlotPad
                     ? -1
                     : wbase[w] + (int64_t)(G[d] - wg_gmin[w]) * slots + (d - w * slots);
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
        const int64_t jb = jbase[j];
        out[x] = inflow ? inflow_at(Oe, jbase, in_off, in_list, j, t, slots)
                        : (jb < 0 ? 0.0 : Oe[jb + t * slots]);
    }
}

// Lateral-inflow correction of a sub-basin entry reach from the upstream sub-basin's outlet
// series (simulation.py:152-159, AsyncSimulation._accumulate): forcing row r of slot `dslot`
//   F[r][dslot] += alpha * I(r + 1) / gamma + beta * I(r) / gamma,  r < T,
// I(t) = the outlet's outflow after step t - 1 of the upstream run (I(0) = o_start, the outflow
// the run started from), in the reference's association.
__global__ void lateral_correction(const double* __restrict__ O, const int64_t* __restrict__ jbase,
                                   int64_t j, int slots, double o_start, double alpha,
                                   double beta, double gamma, double* __restrict__ F,
                                   int64_t ns, int64_t dslot, int64_t T) {
    for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < T;
         r += (int64_t)gridDim.x * blockDim.x) {
        const int64_t jb = jbase[j];                  // < 0: an unrouted outlet, o = 0
        const double inext = jb < 0 ? 0.0 : O[jb + r * slots];
        const double iprev = r == 0 ? o_start : (jb < 0 ? 0.0 : O[jb + (r - 1) * slots]);
        double* f = F + r * ns + dslot;
        *f = *f + (alpha * inext / gamma + beta * iprev / gamma);
    }
}

inline int grid_for(int64_t work, int block) {
    int64_t g = (work + block - 1) / block;
    if (g < 1) g = 1;
    if (g > 65536) g = 65536;
    return (int)g;
}

}  // namespace

hipError_t launch_lateral_correction(const double* O, const int64_t* jbase, int64_t j, int slots,
                                     double o_start, double alpha, double beta, double gamma,
                                     double* F, int64_t ns, int64_t dslot, int64_t T,
                                     hipStream_t s) {
    if (T <= 0) return hipSuccess;
    hipLaunchKernelGGL(lateral_correction, grid_for(T, 256), 256, 0, s, O, jbase, j, slots,
                       o_start, alpha, beta, gamma, F, ns, dslot, T);
    return hipGetLastError();
}

template <bool DENSE>
hipError_t launch_wavefront_t(const WaveArgs& a, int grid, int slots, int chain, size_t lds,
                              int members, hipStream_t s) {
    const dim3 g(grid, members);
#define MCR_CASE(S, K)                                                              \
    if (slots == S && chain == K) {                                                 \
        hipLaunchKernelGGL((wavefront_det<S, K, DENSE>), g, S, lds, s, a);          \
        return hipGetLastError();                                                   \
    }
    MCR_SLOT_SHAPES(MCR_CASE)
#undef MCR_CASE
    return hipErrorInvalidValue;
}

bool wavefront_shape_ok(int slots, int chain) {
#define MCR_CASE(S, K) if (slots == S && chain == K) return true;
    MCR_SLOT_SHAPES(MCR_CASE)
#undef MCR_CASE
    return false;
}

hipError_t launch_wavefront(const WaveArgs& a, int grid, int slots, int chain, size_t lds,
                            bool dense, int members, hipStream_t s) {
    return dense ? launch_wavefront_t<true>(a, grid, slots, chain, lds, members, s)
                 : launch_wavefront_t<false>(a, grid, slots, chain, lds, members, s);
}

namespace {
__global__ __launch_bounds__(256) void flag_nonfinite(const double* __restrict__ src, int64_t n,
                                                      int32_t* __restrict__ flag) {
    bool bad = false;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x)
        bad = bad || !__builtin_isfinite(src[x]);
    if (__any(bad) && (threadIdx.x & 63) == 0)
        __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
}  // namespace

hipError_t launch_flag_nonfinite(const double* src, int64_t n, int32_t* flag, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 2048);
    hipLaunchKernelGGL(flag_nonfinite, dim3((unsigned)blocks), 256, 0, s, src, n, flag);
    return hipGetLastError();
}

hipError_t launch_set_slot_coeffs(const uint8_t* flags, double* alpha, double* beta, double* chi,
                                  double* gamma, int64_t nslots, hipStream_t s) {
    if (nslots > 0)
        hipLaunchKernelGGL(set_slot_coeffs, grid_for(nslots, 256), 256, 0, s, flags, alpha, beta,
                           chi, gamma, nslots);
    return hipGetLastError();
}

hipError_t launch_scatter_to_slots(const double* src, double* dst, const int64_t* slot_reach,
                                   int64_t nslots, int64_t E, hipStream_t s) {
    hipLaunchKernelGGL(scatter_to_slots, grid_for(nslots * E, 256), 256, 0, s, src, dst,
                       slot_reach, nslots, E);
    return hipGetLastError();
}

// State hand-over between two plans of one network (mc_net_copy_state): dst[e][d] =
// src[e][map[d]] (map: the source slot of dst slot d's reach, -1 = no reach -> 0).  Member-major
// rows, a 2-D grid (slot blocks x members): a block's writes are one contiguous run of a member
// row and its gathers stay inside the same member's source row (1.5 MB at Texas: L2-resident).
__global__ __launch_bounds__(256) void permute_slots(const double* __restrict__ src,
                                                     double* __restrict__ dst,
                                                     const int32_t* __restrict__ map,
                                                     int64_t ns_src, int64_t ns_dst) {
    const int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (d >= ns_dst) return;
    const int64_t e = blockIdx.y;
    const int32_t k = map[d];
    dst[e * ns_dst + d] = k >= 0 ? src[e * ns_src + k] : 0.0;
}

hipError_t launch_permute_slots(const double* src, double* dst, const int32_t* map,
                                int64_t ns_src, int64_t ns_dst, int64_t E, hipStream_t s) {
    if (ns_dst <= 0 || E <= 0) return hipSuccess;
    if (E > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(permute_slots, dim3((unsigned)((ns_dst + 255) / 256), (unsigned)E), 256,
                       0, s, src, dst, map, ns_src, ns_dst);
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
                                   hipStream_t s, bool reach_major) {
    hipLaunchKernelGGL(forcing_to_slots, grid_for(nslots * n_rows * E, 256), 256, 0, s, fp, F,
                       slot_reach, n, nslots, n_rows, E, reach_major);
    return hipGetLastError();
}

hipError_t launch_window_index(const int64_t* pos, const int32_t* G, const uint8_t* flags,
                               const int32_t* wg_gmin, const int64_t* wbase, int slots, int64_t n,
                               int64_t* jbase, hipStream_t s) {
    if (n > 0)
        hipLaunchKernelGGL(window_index, grid_for(n, 256), 256, 0, s, pos, G, flags, wg_gmin,
                           wbase, slots, n, jbase);
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

hipError_t launch_slot_window_index(const int32_t* G, const uint8_t* flags, const int32_t* wg_gmin,
                                    const int64_t* wbase, int slots, int64_t ns, int64_t* sjb,
                                    hipStream_t s) {
    if (ns > 0)
        hipLaunchKernelGGL(slot_window_index, grid_for(ns, 256), 256, 0, s, G, flags, wg_gmin,
                           wbase, slots, ns, sjb);
    return hipGetLastError();
}

hipError_t launch_gather_slots(const double* O, const int64_t* sjb, int64_t stride,
                               const int32_t* pos, const int32_t* in_off, const int32_t* upos,
                               double* out_o, double* out_i, int64_t n, int64_t ns, int64_t t0,
                               int64_t t1, double* scratch, int64_t scratch_steps,
                               hipStream_t s) {
    if (n <= 0 || t1 <= t0 || (!out_o && !out_i)) return hipSuccess;
    if (!scratch || scratch_steps < 1) return hipErrorInvalidValue;
    const int64_t ntile = (n + 255) / 256;
    for (int64_t c0 = t0; c0 < t1; c0 += scratch_steps) {
        const int64_t c1 = std::min(t1, c0 + scratch_steps);
        const int64_t sb = (c1 - c0 + kUnskewSteps - 1) / kUnskewSteps;
        constexpr int P = kPermuteSteps;
        const int64_t blocks = 8 * ntile * ((c1 - c0 + 8 * P - 1) / (8 * P));
        if ((ns + 255) / 256 > 0x7fffffff || sb > 65535 || blocks > 0x7fffffff)
            return hipErrorInvalidValue;
        hipLaunchKernelGGL(unskew_windows, dim3((unsigned)((ns + 255) / 256), (unsigned)sb), 256,
                           0, s, O, sjb, stride, scratch, ns, c0, c1);
        hipLaunchKernelGGL(permute_steps, dim3((unsigned)blocks), 256, 0, s, scratch, pos, in_off,
                           upos, out_o ? out_o + (c0 - t0) * n : nullptr,
                           out_i ? out_i + (c0 - t0) * n : nullptr, n, ns, c0, c1, (int)ntile);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// one workgroup per row: strided partial sums, then an LDS tree (sums mod 2^64 are exact, so
// the order does not matter)
__global__ __launch_bounds__(256) void row_digests(const double* __restrict__ rows, int64_t n,
                                                   uint64_t* __restrict__ out) {
    __shared__ uint64_t part[256];
    const double* row = rows + (int64_t)blockIdx.x * n;
    uint64_t h = 0;
    for (int64_t j = threadIdx.x; j < n; j += 256)
        h += digest_term_dev((uint64_t)__double_as_longlong(row[j]), (uint64_t)j);
    part[threadIdx.x] = h;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = part[0];
}

hipError_t launch_row_digests(const double* rows, int64_t nrows, int64_t n, uint64_t* out,
                              hipStream_t s) {
    if (nrows <= 0) return hipSuccess;
    if (nrows > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(row_digests, dim3((unsigned)nrows), 256, 0, s, rows, n, out);
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
