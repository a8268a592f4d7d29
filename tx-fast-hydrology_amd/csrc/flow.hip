// Dataflow form of the wavefront sweep (gfx950): ONE launch routes the whole horizon.
//
// Same space-time schedule as `wavefront_det` (kernels.hip): reach j does model step t at tick
// G[j] + t, in-cluster upstreams one tick ahead through the LDS double buffer.  Instead of
// cutting the horizon into launches of `tile` ticks, every workgroup of the network is resident
// at once and walks its own tick window [gmin, gmax + T) chunk by chunk; registers and the LDS
// double buffer persist across the horizon.  Inputs from other clusters (slack >= 2 chunks,
// plan.hpp) travel as data-tagged granules: the producing lane writes {outflow, epoch} with a
// write-through (sc1) 16-byte store, and a helper wave of the consuming workgroup prefetches the
// next chunk's granules with sc1 loads, checks every tag and stages the values in an LDS ring
// (MI355X_MICROARCH.md, inter-workgroup visibility, granule form R2: no flag, no fence).  A tag
// that is not yet current means the producer is behind: the helper polls that granule until it
// is (bounded; on give-up it sets the status word and the run reports an error).
//
// Residency: the host launches this kernel only when every workgroup fits on the device at once
// (capi.cpp, occupancy check); otherwise the multi-launch `wavefront_det` path runs.
#include "device_common.hpp"
#include "kernels.hpp"
#include "plan.hpp"

#include <algorithm>

#pragma clang fp contract(off)

#ifndef MCR_EXP_NO_STORES
#define MCR_EXP_NO_STORES 0
#endif
#ifndef MCR_EXP_PAIR_STORES
#define MCR_EXP_PAIR_STORES 0
#endif
#ifndef MCR_EXP_NO_Q
#define MCR_EXP_NO_Q 0
#endif

namespace mcr {

namespace {

using dev::chunk_rows;
using dev::clamp_row;
using dev::lds_f64;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kHelperLanes = 64;                      // one helper wave per workgroup
// dataflow instantiations: compute waves + the helper fill whole wave slots on the SIMDs
#define MCR_SLOT_LIST_FLOW(X) X(64) X(128) X(192) X(256) X(384) X(448)
constexpr int kBatch = 8;                             // granules per helper lane per batch
constexpr int kBatchItems = kHelperLanes * kBatch;    // (external input, tick) items per batch
constexpr int64_t kGiveUpTicks = 200000000;           // 2 s of the 100 MHz wall clock
static_assert(kFlowMaxExt * kChunk == 2 * kBatchItems, "two helper batches per chunk");

__device__ __forceinline__ void sleep_backoff(int& sl) {
    // exponential back-off between polls of a granule that is not current yet
    for (int r = 0; r < sl; ++r) __builtin_amdgcn_s_sleep(32);
    sl = sl < 16 ? sl * 2 : 16;
}

// Helper wave: stage the external inputs of the chunk starting at tick kn in ring slot `slot`.
// Items idx = e * kChunk + i (external input e of this workgroup, tick kn + i) map one-to-one to
// the ring's LDS layout, and consecutive lanes read consecutive steps of one producer's stream.
struct Helper {
    const char* lds;
    __amdgpu_buffer_rsrc_t xg;
    unsigned XE, XSLOT, EG;
    int lane, e0, nitems, T;
    unsigned epoch;
    int32_t* status;
    bool dead;

    __device__ __forceinline__ bool item(int idx, int kn, unsigned& voff) const {
        const int e = idx >> 3;                          // < kFlowMaxExt: EG is that long
        const int t = kn + (idx & 7) - reinterpret_cast<const int*>(lds + EG)[e];
        const bool need = idx < nitems && t >= 0 && t < T;
        voff = need ? (unsigned)(((int64_t)(e0 + e) * T + t) * 16) : 0u;
        return need;
    }
    __device__ __forceinline__ int index(int b, int k, int ln) const {
        return b * kBatchItems + k * kHelperLanes + ln;
    }
    __device__ __forceinline__ void issue(int b, int kn, u32x4 (&g)[kBatch]) const {
#pragma unroll
        for (int k = 0; k < kBatch; ++k) {
            unsigned voff;
            item(index(b, k, lane), kn, voff);
            g[k] = __builtin_amdgcn_raw_buffer_load_b128(xg, voff, 0, 16);   // sc1
        }
    }
    // write the batch to LDS; returns the first (lane-local) item whose tag is stale, or -1
    __device__ __forceinline__ int consume(int b, int kn, unsigned slot,
                                           const u32x4 (&g)[kBatch]) const {
        int bad = -1;
#pragma unroll
        for (int k = 0; k < kBatch; ++k) {
            unsigned voff;
            const int idx = index(b, k, lane);
            const bool need = item(idx, kn, voff);
            const bool cur = g[k].y == epoch && g[k].w == epoch;
            const uint64_t bits = ((uint64_t)g[k].z << 32) | g[k].x;
            const double v = need ? __longlong_as_double((long long)bits) : 0.0;
            if (idx < nitems)
                *reinterpret_cast<double*>(const_cast<char*>(lds) + XE + slot * XSLOT + idx * 8) = v;
            if (need && !cur && bad < 0) bad = k;
        }
        return bad;
    }
    // slow path: poll one stale granule until current, then re-read the batch; repeat
    __device__ void settle(int b, int kn, unsigned slot, int bad) {
        const int64_t t0 = wall_clock64();
        int sl = 1;
        while (__any(bad >= 0) && !dead) {
            // poll the first stale granule of the wave (one sc1 load) with back-off
            const int src = __ffsll((long long)__ballot(bad >= 0)) - 1;
            const int kk = __shfl(bad, src);
            unsigned voff = 0;
            item(index(b, kk, src), kn, voff);
            for (;;) {
                const u32x4 p = __builtin_amdgcn_raw_buffer_load_b128(xg, voff, 0, 16);
                if (p.y == epoch && p.w == epoch) break;
                const int st = __hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (st != 0 || wall_clock64() - t0 > kGiveUpTicks) {
                    if (st == 0 && lane == 0)
                        __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    dead = true;
                    break;
                }
                sleep_backoff(sl);
            }
            u32x4 g[kBatch];
            issue(b, kn, g);
            bad = consume(b, kn, slot, g);
        }
    }
    __device__ __forceinline__ void fetch_now(int b, int kn, unsigned slot) {
        u32x4 g[kBatch];
        issue(b, kn, g);
        const int bad = consume(b, kn, slot, g);
        if (__any(bad >= 0)) settle(b, kn, slot, bad);
    }
};

// LDS layout (bytes): XB [SLOTS + 1][2] f64 | FR [SLOTS][3] f64 | TAB [T] int4 (whole step table)
//   | XE [2][ext_cap][kChunk] f64 (ring of external inputs, one slot per chunk parity)
//   | EG [kFlowMaxExt] i32 (consumer G)
template <int SLOTS, bool DENSE>
__global__ __launch_bounds__(SLOTS + kHelperLanes) __attribute__((amdgpu_waves_per_eu(4)))
void wavefront_flow(WaveArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr unsigned XB = 0;
    constexpr unsigned FR = XB + (SLOTS + 1) * 16;
    constexpr unsigned TAB = FR + SLOTS * 24;
    const int T = a.T;
    const unsigned XE = TAB + (unsigned)a.table_cap * 16;
    const unsigned XSLOT = (unsigned)a.ext_cap * kChunk * 8;
    const unsigned EG = XE + 2 * XSLOT;
    double* xbp = reinterpret_cast<double*>(lds + XB);
    int4* tab = reinterpret_cast<int4*>(lds + TAB);

    const int tid = threadIdx.x;
    const int nthr = SLOTS + kHelperLanes;
    const int64_t t_start = a.trace ? wall_clock64() : 0;
    const int w = a.active[blockIdx.x];
    const int gminw = a.wg_gmin[w], gmaxw = a.wg_gmax[w];
    const int kb = gminw & ~(kChunk - 1);               // first chunk of this workgroup
    const int wend = gmaxw + T;                         // end of its tick window
    const int e0 = a.ext_off[w];
    const int next = a.ext_off[w + 1] - e0;
    const auto xg = __builtin_amdgcn_make_buffer_rsrc(a.XG, (short)0, (int)a.xg_bytes, 0x00020000);

    // ---- shared prologue: step table, consumer ticks of external inputs
    for (int idx = tid; idx < T; idx += nthr) tab[idx] = a.stab[idx];
    for (int idx = tid; idx < next; idx += nthr)
        reinterpret_cast<int*>(lds + EG)[idx] = a.ext_g[e0 + idx];
    if (tid < 2) xbp[SLOTS * 2 + tid] = 0.0;

    if (tid >= SLOTS) {
        // ================================ helper wave ================================
        Helper h{lds, xg, XE, XSLOT, EG, tid - SLOTS, e0, next * kChunk, T, a.epoch, a.status,
                 false};
        const int nb = (h.nitems + kBatchItems - 1) / kBatchItems;   // <= 2 (host-checked)
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();                     // EG staged (LDS) before the helper reads it
        for (int b = 0; b < nb; ++b) h.fetch_now(b, kb, (unsigned)((kb >> 3) & 1));
        __syncthreads();                     // prologue barrier (matches the compute waves)
        for (int kc = kb; kc < wend; kc += kChunk) {
            const int kn = kc + kChunk;
            const bool pre = kn < wend && nb > 0;
            const unsigned slot = (unsigned)((kn >> 3) & 1);
            u32x4 g[kBatch];
            if (pre) h.issue(0, kn, g);
            __syncthreads();                 // tick 0
            __syncthreads();                 // tick 1
            __syncthreads();                 // tick 2
            if (pre) {
                const int bad = h.consume(0, kn, slot, g);
                if (__any(bad >= 0)) h.settle(0, kn, slot, bad);
                if (nb > 1) h.issue(1, kn, g);
            }
            __syncthreads();                 // tick 3
            __syncthreads();                 // tick 4
            __syncthreads();                 // tick 5
            if (pre && nb > 1) {
                const int bad = h.consume(1, kn, slot, g);
                if (__any(bad >= 0)) h.settle(1, kn, slot, bad);
            }
            __syncthreads();                 // tick 6
            __syncthreads();                 // tick 7
        }
        return;
    }

    // ================================ compute waves ================================
    const int64_t d = (int64_t)w * SLOTS + tid;
    const int64_t ns = a.nslots;
    const int nrow = a.n_rows;
    const uint8_t fl = a.flags[d];
    const int Gr = a.G[d];
    const bool real = fl != kSlotPad;
    const bool routed = fl == kSlotRouted;
    const bool psum = fl == kSlotSum;                   // partial-sum node: outputs I
    const int G = real ? Gr : (1 << 29);                // padding lanes are never active
    const double st_o = a.st_o[d], st_i = a.st_i[d];
    const double al = a.alpha[d], be = a.beta[d], ch = a.chi[d], ga = a.gamma[d];
    const int cnt = real ? a.up_cnt[d] : 0;
    const uint64_t up4 = a.up4[d];
    const int xsid = a.xid[d];
    const int64_t wb = a.wbase[w];

    double op = st_o;                                   // every lane starts at step 0 here
    double ip = st_i;
    xbp[tid * 2 + ((kb - 1) & 1)] = op;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();                                    // LDS tables staged

    unsigned ubase[kUpInline], uinc[kUpInline];
#pragma unroll
    for (int u = 0; u < kUpInline; ++u) {
        const unsigned code = u < cnt ? (unsigned)((up4 >> (16 * u)) & 0xffffu) : (unsigned)SLOTS;
        const bool ext = (code & kExtBit) != 0;
        ubase[u] = ext ? XE + (code & 0x7fffu) * kChunk * 8 : XB + code * 16;
        uinc[u] = ext ? 16u : 0u;
    }
    const bool any3 = __any(cnt > 2);
    const unsigned own = XB + (unsigned)tid * 16;

    int rb, nr;
    chunk_rows(tab, 0, kb, G, T, rb, nr);
    double f0 = a.F[(int64_t)clamp_row(rb, nrow) * ns + d];
    double f1 = a.F[(int64_t)clamp_row(rb + 1, nrow) * ns + d];
    double f2 = a.F[(int64_t)clamp_row(rb + 2, nrow) * ns + d];
    const bool xsrc = real && xsid >= 0;
    const int64_t xs0 = xsrc ? (int64_t)xsid * T - Gr : 0;
    const unsigned epoch = a.epoch;
    __builtin_amdgcn_s_waitcnt(0);                      // nothing pending may enter the loop
    __syncthreads();                                    // prologue barrier (helper staged XE)
    const int64_t t_loop = a.trace ? wall_clock64() : 0;
    const int64_t c_loop = a.trace ? clock64() : 0;

    double pv = 0.0;                                    // MCR_EXP_PAIR_STORES only
    for (int kc = kb; kc < wend; kc += kChunk) {
        const unsigned sb = (unsigned)((kc >> 3) & 1) * XSLOT;   // this chunk's ring slot
        double* frl = reinterpret_cast<double*>(lds + FR) + tid * 3;
        frl[0] = f0;
        frl[1] = f1;
        frl[2] = f2;
        const bool slow = DENSE && __any(nr > 3);
        const unsigned frp = FR + (unsigned)tid * 24 - (unsigned)rb * 8;
        int rbn, nrn;
        chunk_rows(tab, 0, kc + kChunk, G, kc + kChunk < wend ? T : 0, rbn, nrn);
        const double g0 = a.F[(int64_t)clamp_row(rbn, nrow) * ns + d];
        const double g1 = a.F[(int64_t)clamp_row(rbn + 1, nrow) * ns + d];
        const double g2 = a.F[(int64_t)clamp_row(rbn + 2, nrow) * ns + d];
        unsigned m[kUpInline];
#pragma unroll
        for (int u = 0; u < kUpInline; ++u) m[u] = uinc[u] ? ubase[u] + sb - 8u : ubase[u];
        const unsigned tp = TAB + (unsigned)(kc - G) * 16u;
        double qv[kChunk];
#pragma unroll
        for (int j = 0; j < kChunk; ++j) {
            const int4 e = *reinterpret_cast<const int4*>(lds + tp + 16u * j);
            double flo, fhi;
            if (DENSE && slow) {
                flo = a.F[(int64_t)clamp_row(e.x < 0 ? 0 : e.x, nrow) * ns + d];
                fhi = a.F[(int64_t)clamp_row(e.y < 0 ? 0 : e.y, nrow) * ns + d];
            } else {
                flo = lds_f64(lds, frp + 8u * (unsigned)e.x);
                fhi = lds_f64(lds, frp + 8u * (unsigned)e.y);
            }
            const double fr = __hiloint2double(e.w, e.z);
            const double qi = (1.0 - fr) * flo + fr * fhi;
            qv[j] = MCR_EXP_NO_Q ? 0.0 : (e.y < 0 ? flo : qi);
        }
        if (DENSE && slow) __builtin_amdgcn_s_waitcnt(0);
#pragma unroll
        for (int i = 0; i < kChunk; ++i) {
            if (i & 1) {
#pragma unroll
                for (int u = 0; u < kUpInline; ++u) m[u] += uinc[u];
            }
            const unsigned rd = 8u * ((i + 1) & 1);
            const int k = kc + i;
            const int t = k - G;
            const bool act = (unsigned)t < (unsigned)T;
            double I = lds_f64(lds, m[0] + rd);   // published values are never -0.0
            I = I + lds_f64(lds, m[1] + rd);
            if (any3) {
                I = I + lds_f64(lds, m[2] + rd);
                I = I + lds_f64(lds, m[3] + rd);
            }
            const double rv = 0.0 + (((al * I + be * ip) + ch * op) + ga * qv[i]);
            const double ov = psum ? I : rv;
            *reinterpret_cast<double*>(lds + own + 8u * (i & 1)) = ov;
            op = act ? ov : op;
            ip = act ? I : ip;
            const bool inwin = k >= gminw && k < wend;
            const int64_t row = inwin ? wb + (int64_t)(k - gminw) * SLOTS : 0;
            double* orow = inwin ? a.O + row : a.dummy;
            if (MCR_EXP_PAIR_STORES) {
                // timing experiment only: one 16-byte store per lane every second tick
                const double sv = routed ? ov : 0.0;
                if (i & 1) {
                    const int kp = k - 1 >= gminw ? k - 1 : gminw;
                    const int r0 = (kp - gminw) & ~1;
                    const bool fits = inwin && r0 + 2 <= wend - gminw;
                    const int64_t prow = wb + (int64_t)r0 * SLOTS;
                    double2* pr = reinterpret_cast<double2*>(fits ? a.O + prow : a.dummy);
                    pr[tid] = make_double2(pv, sv);
                }
                pv = sv;
            } else if (!MCR_EXP_NO_STORES) {
                orow[tid] = routed ? ov : 0.0;
            }
            if (xsrc && act) {
                const uint64_t bits = (uint64_t)__double_as_longlong(ov);
                const u32x4 gv = {(unsigned)bits, epoch, (unsigned)(bits >> 32), epoch};
                __builtin_amdgcn_raw_buffer_store_b128(gv, xg, (unsigned)((xs0 + k) * 16), 0, 16);
            }
            __syncthreads();
        }
        rb = rbn;
        nr = nrn;
        f0 = g0;
        f1 = g1;
        f2 = g2;
    }
    a.st_o[d] = routed || psum ? op : 0.0;              // session state after the horizon
    a.st_i[d] = ip;
    if (a.trace && tid == 0) {
        int64_t* rec = a.trace + kTraceWords * (int64_t)blockIdx.x;
        rec[0] = t_start;
        rec[1] = t_loop;
        rec[2] = wall_clock64();
        rec[3] = (int64_t)__smid();
        rec[4] = c_loop;
        rec[5] = clock64();
    }
}

template <bool DENSE>
const void* flow_fn(int slots) {
    switch (slots) {
#define MCR_CASE(S) \
    case S: return reinterpret_cast<const void*>(&wavefront_flow<S, DENSE>);
        MCR_SLOT_LIST_FLOW(MCR_CASE)
#undef MCR_CASE
        default: return nullptr;
    }
}

}  // namespace

hipError_t flow_occupancy(int slots, bool dense, size_t lds, int* blocks_per_cu) {
    const void* fn = dense ? flow_fn<true>(slots) : flow_fn<false>(slots);
    if (!fn) return hipErrorInvalidValue;
    const int threads = slots + kHelperLanes;
    int api = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, fn, threads, lds);
    if (e != hipSuccess) return e;
    hipFuncAttributes attr;
    e = hipFuncGetAttributes(&attr, fn);
    if (e != hipSuccess) return e;
    // Measured on gfx950 (launch trace, 5-wave workgroups at 128 VGPRs): a workgroup of W waves
    // takes ceil(W / 4) wave slots on EVERY SIMD, so the API's answer can be too high.
    const int vgpr = ((attr.numRegs > 0 ? attr.numRegs : 512) + 7) / 8 * 8;
    const int per_simd = std::min(8, 512 / vgpr);
    const int waves = (threads + 63) / 64;
    const int by_waves = per_simd / ((waves + 3) / 4);
    const int by_lds = lds ? (int)((160 * 1024) / lds) : 8;
    *blocks_per_cu = std::min(api, std::min(by_waves, by_lds));
    return hipSuccess;
}

hipError_t launch_flow(const WaveArgs& a, int grid, int slots, size_t lds, bool dense,
                       hipStream_t s) {
    const void* fn = dense ? flow_fn<true>(slots) : flow_fn<false>(slots);
    if (!fn) return hipErrorInvalidValue;
    void* args[] = {const_cast<WaveArgs*>(&a)};
    return hipLaunchKernel(fn, dim3(grid), dim3(slots + kHelperLanes), args, lds, s);
}

}  // namespace mcr
