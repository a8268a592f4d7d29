// Dataflow form of the wavefront sweep (gfx950): ONE launch routes the whole horizon.
//
// Same space-time schedule as `wavefront_det` (kernels.hip): reach j does model step t at tick
// G[j] + t, in-cluster upstreams one tick ahead through the LDS double buffer.  Instead of
// cutting the horizon into launches of `tile` ticks, every workgroup of the network is resident
// at once and walks its own tick window [gmin, gmax + T) chunk by chunk; registers and the LDS
// tick planes persist across the horizon; the workgroup's helper wave copies the plane of the
// tick that just ended to the output window.  Inputs from other clusters (slack >= 2 chunks,
// plan.hpp) travel as data-tagged granules: the producing lane writes {outflow, epoch} with a
// write-through (sc1) 16-byte store, and the helper wave of the consuming workgroup prefetches
// the next chunk's granules with sc1 loads, checks every tag and stages the values in an LDS ring
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

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

constexpr int kHelperLanes = 64;                      // one helper wave per workgroup
constexpr int kBatch = 8;                             // granules per helper lane per batch
constexpr int kBatchItems = kHelperLanes * kBatch;    // (external input, tick) items per batch
static_assert(kFlowMaxExt * kChunk == 2 * kBatchItems, "two helper batches per chunk");

// poll back-off: s_sleep 32 (x 64 clocks) per unit, at most 16 units (1-64 clocks per unit
// measured the same)
constexpr int kSleepUnit = 32;
constexpr int kSleepCap = 16;
__device__ __forceinline__ void sleep_backoff(int& sl) {
    // exponential back-off between polls of a granule that is not current yet
    for (int r = 0; r < sl; ++r) __builtin_amdgcn_s_sleep(kSleepUnit);
    sl = sl < kSleepCap ? sl * 2 : kSleepCap;
}

// Helper wave: stage the external inputs of the chunk starting at tick kn in ring slot `slot`.
// Items idx = e * kChunk + i (external input e of this workgroup, tick kn + i) map one-to-one to
// the ring's LDS layout, and consecutive lanes read consecutive steps of one producer's stream.
struct Helper {
    const char* lds;
    __amdgpu_buffer_rsrc_t xg;
    unsigned XE, XSLOT, EG, PL;   // XE: first external column byte; XSLOT: one ring slot's columns
    int lane, e0, nitems, T;
    unsigned epoch;
    int32_t* status;
    int64_t patience;             // wall-clock ticks a stale granule is polled before giving up
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
    // item idx = (external input e = idx / kChunk, chunk tick j = idx % kChunk) is staged in
    // tick plane (j + 7) & 7, column e of the ring slot (tick planes, see wavefront_flow)
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
                *reinterpret_cast<double*>(const_cast<char*>(lds) + XE + slot * XSLOT +
                                           (unsigned)(idx >> 3) * 8u +
                                           (unsigned)(((idx & 7) + 7) & 7) * PL) = v;
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
                if (st != 0 || wall_clock64() - t0 > patience) {
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

// LDS layout (bytes), RS = K * SLOTS node slots (lane l: slots p * SLOTS + l, p < K):
//   PLANES [8][RS + 1 + 2 * kFlowMaxExt] f64 | FR [RS][3] f64 | TAB [T] int4 (whole step
//   table) | EG [kFlowMaxExt] i32 (consumer G)
// Tick planes: plane k & 7 holds every node slot's output of tick k (column d; column RS is
// the zero slot) and, in columns RS + 1 + s * kFlowMaxExt + e, the value external input e
// delivers at chunk tick i (plane (i + 7) & 7) for chunk ring slot s (chunk parity).  At chunk
// tick i a slot reads plane (i + 7) & 7 of EVERY input: one compile-time LDS offset per
// unrolled tick, no per-tick address arithmetic, and consecutive node slots are consecutive
// 8-byte words (bank-conflict-free neighbour reads).
//   | EG [kFlowMaxExt] i32 (consumer G)
// Each tick a lane routes its K positions in order; position p may take the output of position
// p - 1 of the same tick (a chained edge, plan.hpp "lane chains").
// MEMB: member dataflow (kernels.hpp, launch_flow_members): T = E members in place of steps;
// SKEW: its staging cells are tick-major member windows (else member-major), a compile-time
// choice so that the tick computes one kind of cell address without branches.
// Register budget: two waves per SIMD (256 VGPRs) up to 3 positions per lane; lanes of 4
// positions need more (one wave per SIMD, so at most 3 compute waves + the helper).
// SYNC (chunk-synchronous plans, plan.hpp): 0 = one workgroup barrier per tick (classic
// plans); kWaveSlack = one per kWaveSlack ticks: a unit-slack edge stays inside one wave (its
// LDS accesses are processed in order, so the wave needs no barrier), an edge between two waves
// of the workgroup has slack kWaveSlack and its producer writes the value straight into the
// consumer's external column for tick k + kWaveSlack, which the consumer reads after the next
// barrier.  The helper copies the tick planes of one barrier period during the next one.
template <int SLOTS, int K, bool DENSE, bool MEMB, bool SKEW = false, int SYNC = 0>
__global__ __launch_bounds__(SLOTS + kHelperLanes)
__attribute__((amdgpu_waves_per_eu(K >= 4 ? 1 : 2, K >= 4 ? 1 : 2)))
void wavefront_flow(WaveArgs a) {
    static_assert(SYNC == 0 || (SYNC == kWaveSlack && kChunk == 2 * kWaveSlack),
                  "sync kernels: two barrier periods of kWaveSlack ticks per chunk");
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int RS = K * SLOTS;
    constexpr unsigned PL = flow_plane_bytes(RS);
    static_assert(7 * PL < 65536, "tick-plane offsets must fit the 16-bit LDS immediate");
    constexpr unsigned XB = 0;                          // node-slot columns of plane 0
    constexpr unsigned XE = XB + (RS + 1) * 8;          // external columns of plane 0
    constexpr unsigned XSLOT = kFlowMaxExt * 8;         // one chunk ring slot of them
    constexpr unsigned FR = 8 * PL;
    constexpr unsigned TAB = FR + RS * 24;
    const int T = a.T;
    const unsigned EG = TAB + (unsigned)a.table_cap * 16;
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
    const double* __restrict__ Fm = a.F;
    double* __restrict__ Om = a.O;
    const auto xg = __builtin_amdgcn_make_buffer_rsrc(a.XG, (short)0, (int)a.xg_bytes,
                                                      0x00020000);

    // ---- shared prologue: step table, consumer ticks of external inputs
    if (!MEMB)
        for (int idx = tid; idx < T; idx += nthr) tab[idx] = a.stab[idx];
    for (int idx = tid; idx < next; idx += nthr)
        reinterpret_cast<int*>(lds + EG)[idx] = a.ext_g[e0 + idx];
    if (tid < 8) xbp[(tid * PL) / 8 + RS] = 0.0;       // zero slot of every plane

    const int wave = tid >> 6;
    constexpr int kHW = SLOTS / 64;                     // the helper is the last wave
    if (wave == kHW) {
        // ================================ helper wave ================================
        Helper h{lds, xg, XE, XSLOT, EG, PL, tid & 63, e0, next * kChunk, T, a.epoch, a.status,
                 a.patience, false};
        const int nb = (h.nitems + kBatchItems - 1) / kBatchItems;   // <= 2 (host-checked)
        // the outputs of tick k (plane k & 7, written by the compute waves before the barrier
        // that ends tick k, overwritten at tick k + 8) -> row k of the workgroup's output window,
        // 16 bytes per lane: the compute waves' tick loop issues no output stores
        const int hl = tid & 63;
        const int64_t wbh = a.wbase[w];
        auto copy_row = [&](int k) {
            if (MEMB || k < gminw || k >= wend) return;   // wave-uniform
            const char* src = lds + XB + (unsigned)(k & 7) * PL;
            double* dst = Om + wbh + (int64_t)(k - gminw) * RS;
#pragma unroll
            for (int c = 2 * hl; c < RS; c += 128)
                __builtin_nontemporal_store(*reinterpret_cast<const f64x2*>(src + (unsigned)c * 8u),
                                            reinterpret_cast<f64x2*>(dst + c));
        };
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();                     // EG staged (LDS) before the helper reads it
        for (int b = 0; b < nb; ++b) h.fetch_now(b, kb, (unsigned)((kb >> 3) & 1));
        __syncthreads();                     // prologue barrier (matches the compute waves)
        if constexpr (SYNC != 0) {
            // two barrier periods per chunk: the planes of the period that just ended are
            // copied during the next one (the compute waves overwrite them a period later)
            int kc = kb;
            for (; kc < wend; kc += kChunk) {
                const int kn = kc + kChunk;
                const bool pre = kn < wend && nb > 0;
                const unsigned slot = (unsigned)((kn >> 3) & 1);
                u32x4 g[kBatch], g1[kBatch];
                if (pre) h.issue(0, kn, g);
                if (pre && nb > 1) h.issue(1, kn, g1);
#pragma unroll
                for (int q = SYNC; q > 0; --q) copy_row(kc - q);
                __syncthreads();   // ticks kc .. kc + SYNC - 1
                if (pre) {
                    const int bad = h.consume(0, kn, slot, g);
                    if (__any(bad >= 0)) h.settle(0, kn, slot, bad);
                }
                if (pre && nb > 1) {
                    const int bad = h.consume(1, kn, slot, g1);
                    if (__any(bad >= 0)) h.settle(1, kn, slot, bad);
                }
#pragma unroll
                for (int q = 0; q < SYNC; ++q) copy_row(kc + q);
                __syncthreads();   // ticks kc + SYNC .. kc + kChunk - 1
            }
#pragma unroll
            for (int q = SYNC; q > 0; --q) copy_row(kc - q);
            return;
        }
        for (int kc = kb; kc < wend; kc += kChunk) {
            const int kn = kc + kChunk;
            const bool pre = kn < wend && nb > 0;
            const unsigned slot = (unsigned)((kn >> 3) & 1);
            // both batches issued at the chunk start and consumed after ticks 4 and 5 (the
            // sc1 loads cross the XCDs: consuming at tick 3 stalled the group, -1.6% measured)
            u32x4 g[kBatch], g1[kBatch];
            if (pre) h.issue(0, kn, g);
            if (pre && nb > 1) h.issue(1, kn, g1);
            __syncthreads();   // tick 0
            copy_row(kc);
            __syncthreads();   // tick 1
            copy_row(kc + 1);
            __syncthreads();   // tick 2
            copy_row(kc + 2);
            __syncthreads();   // tick 3
            copy_row(kc + 3);
            __syncthreads();   // tick 4
            if (pre) {
                const int bad = h.consume(0, kn, slot, g);
                if (__any(bad >= 0)) h.settle(0, kn, slot, bad);
            }
            copy_row(kc + 4);
            __syncthreads();   // tick 5
            if (pre && nb > 1) {
                const int bad = h.consume(1, kn, slot, g1);
                if (__any(bad >= 0)) h.settle(1, kn, slot, bad);
            }
            copy_row(kc + 5);
            __syncthreads();   // tick 6
            copy_row(kc + 6);
            __syncthreads();                 // tick 7
            copy_row(kc + 7);
        }
        return;
    }

    // ================================ compute waves ================================
    const int lid = tid;                                // lane id over the compute waves
    const int64_t ns = a.nslots;
    const int nrow = a.n_rows;
    Slot S[K];                                          // every real slot runs steps 0 .. T-1
    uint64_t up[K];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        load_slot(S[p], a, (int64_t)w * RS + p * SLOTS + lid, 0, kb, wend - kb, T);
        up[p] = a.up4[S[p].d];
        xbp[(((kb - 1) & 7) * PL) / 8 + p * SLOTS + lid] = S[p].op;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();                                    // LDS tables staged

    bool any3[K];
    unsigned own[K];
    // sync plans: the XE column this slot's output feeds kWaveSlack ticks later (local edge)
    bool lxo[K];
    unsigned lxc[K];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        decode_codes<RS>(S[p], up[p], XB, 8u, XE, 8u);
        // every slot folds four inputs (codes beyond its count read the zero slot: adding +0.0
        // to a published value is exact): no wave-uniform test and no selects of the 2- and
        // 4-input sums (same box: det 0.467 -> 0.462 ms, EnKF32 21.9 -> 21.6 ms per horizon)
        any3[p] = true;
        own[p] = XB + (unsigned)(p * SLOTS + lid) * 8u;
        const int l = SYNC ? (int)a.lx[S[p].d] : -1;
        lxo[p] = l >= 0;
        lxc[p] = XE + (unsigned)(l < 0 ? 0 : l) * 8u;
    }
    // end of tick i of a chunk: the workgroup barrier (every tick, or every SYNC ticks); between
    // the ticks of a period only the compiler is kept from moving LDS accesses across
    auto tick_end = [&](int i) {
        if (SYNC == 0 || i % (SYNC ? SYNC : 1) == SYNC - 1) __syncthreads();
        else __asm__ __volatile__("" ::: "memory");
    };
    // local edges: the value of tick kc + i feeds the consumer's tick kc + i + SYNC: chunk tick
    // (i + SYNC) & 7 (plane (i + SYNC + 7) & 7) of this chunk's ring slot, or of the next one's
    auto write_local = [&](int i, unsigned sb, const double* ov) {
        if constexpr (SYNC != 0) {
            const unsigned rs = i + SYNC < kChunk ? sb : XSLOT - sb;
            const unsigned pl = (unsigned)((i + SYNC + 7) & 7) * PL;
#pragma unroll
            for (int p = 0; p < K; ++p)
                if (lxo[p]) *reinterpret_cast<double*>(lds + lxc[p] + rs + pl) = ov[p];
        }
    };

    const unsigned epoch = a.epoch;
    int64_t t_loop = 0, c_loop = 0;
    if constexpr (MEMB) {
        // ---- member dataflow: tick k runs member e = k - G of each slot.  Per-member inputs
        // (state, lateral inflow) are prefetched kRing ticks ahead into a register ring.  Large
        // ensembles stage them TICK-major in the workgroup's member window
        // (launch_member_inputs, a.mskew): the (slot, member) processed at tick k is in row
        // k - gmin, so every load and store of a tick is one contiguous row per wave; member-
        // major staging ([E][nslots]) scatters a wave's 64 lanes over ~19 member rows (lanes
        // rarely share G) but is cheaper to stage, which wins for small ensembles.
        const double* __restrict__ Qm = a.Qm;
        double2* __restrict__ IO = reinterpret_cast<double2*>(const_cast<double*>(a.IO));
        constexpr bool skew = SKEW;
        const int64_t mwb = skew ? a.wbase[w] : 0;      // member window of this workgroup
        const int rows = wend - gminw;                  // its rows: ticks gmin .. gmax + E - 1
        const int64_t mS = a.mS;
        constexpr int kRing = 4;          // (8: EnKF32 21.45 vs 21.49 ms per horizon, not kept)
        static_assert(kChunk % kRing == 0, "ring slots must be static in the unrolled chunk");
        // tick-major windows (SKEW): the staging cell of tick k (row clamped, wave-uniform)
        auto cell = [&](int k, int p) -> int64_t {
            int r = k - gminw;
            r = r < 0 ? 0 : (r >= rows ? rows - 1 : r);
            return mwb + (int64_t)(r * RS + p * SLOTS + lid);
        };
        // member-major cells (!SKEW): bounds-checked buffer accesses at 32-bit byte offsets that
        // advance one member row (mS cells) per tick -- no clamp and no 64-bit index per access.
        // An offset outside the buffer (ticks before / after the lane's members, modular
        // arithmetic) reads 0 and is never used; the offsets of active ticks are exact
        // (members_fit: nslots x E x 16 B < 2^31).
        const int ioRec = SKEW ? 0 : (int)(mS * T * 16), qmRec = SKEW ? 0 : (int)(mS * T * 8);
        const auto io_r = __builtin_amdgcn_make_buffer_rsrc(IO, (short)0, ioRec, 0x00020000);
        const auto qm_r = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(Qm), (short)0,
                                                            qmRec, 0x00020000);
        const unsigned ioStep = (unsigned)mS * 16u, qmStep = (unsigned)mS * 8u;
        unsigned ioB[K], qmB[K];                        // byte offsets of this tick's cells
#pragma unroll
        for (int p = 0; p < K; ++p) {
            const unsigned idx = (unsigned)(kb - S[p].G) * (unsigned)mS + (unsigned)S[p].d;
            ioB[p] = idx * 16u;
            qmB[p] = idx * 8u;
        }
        auto load_io = [&](unsigned off) -> double2 {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(io_r, off, 0, 0);
            return make_double2(__hiloint2double((int)v.y, (int)v.x),
                                __hiloint2double((int)v.w, (int)v.z));
        };
        auto load_q = [&](unsigned off) -> double {
            const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(qm_r, off, 0, 0);
            return __hiloint2double((int)v.y, (int)v.x);
        };
        double2 rIO[K][kRing];
        double rQ[K][kRing];
#pragma unroll
        for (int r = 0; r < kRing; ++r)
#pragma unroll
            for (int p = 0; p < K; ++p) {
                if constexpr (SKEW) {
                    const int64_t pa = cell(kb + r, p);
                    rIO[p][r] = IO[pa];
                    rQ[p][r] = Qm[pa];
                } else {
                    rIO[p][r] = load_io(ioB[p] + (unsigned)r * ioStep);
                    rQ[p][r] = load_q(qmB[p] + (unsigned)r * qmStep);
                }
            }
        __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();                                // prologue barrier (helper staged XE)
        t_loop = a.trace ? wall_clock64() : 0;
        c_loop = a.trace ? clock64() : 0;
        for (int kc = kb; kc < wend; kc += kChunk) {
            const unsigned sb = (unsigned)((kc >> 3) & 1) * XSLOT;
            unsigned m[K][kUpInline];
#pragma unroll
            for (int p = 0; p < K; ++p)
#pragma unroll
                for (int u = 0; u < kUpInline; ++u)
                    m[p][u] = S[p].uext[u] ? S[p].ubase[u] + sb : S[p].ubase[u];
#pragma unroll
            for (int i = 0; i < kChunk; ++i) {
                const unsigned rd = (unsigned)((i + 7) & 7) * PL;   // plane of tick k - 1
                const int k = kc + i;
                const int r = i % kRing;
                double vin[K][kUpInline];
#pragma unroll
                for (int p = 0; p < K; ++p) read_inputs(lds, m[p], rd, any3[p], vin[p]);
                double ov[K], Iv[K];
                double prev = 0.0;
#pragma unroll
                for (int p = 0; p < K; ++p) {
                    const double I = fold_values(vin[p], S[p].chained, any3[p], prev, p == 0);
                    const double rr = dev::muskingum_update(S[p].al, I, S[p].be, rIO[p][r].y,
                                                            S[p].ch, rIO[p][r].x,
                                                            dev::gq_term(S[p].ga, rQ[p][r]));
                    const double o = rr;   // psum / unrouted / pad: coefficients set_slot_coeffs
                    ov[p] = o;
                    Iv[p] = I;
                    prev = o;
                }
#pragma unroll
                for (int p = 0; p < K; ++p)
                    *reinterpret_cast<double*>(lds + own[p] + (unsigned)i * PL) = ov[p];
#pragma unroll
                for (int p = 0; p < K; ++p) {   // refill this ring slot with tick k + kRing
                    if constexpr (SKEW) {
                        const int64_t pa = cell(k + kRing, p);
                        rIO[p][r] = IO[pa];
                        rQ[p][r] = Qm[pa];
                    } else {
                        rIO[p][r] = load_io(ioB[p] + (unsigned)kRing * ioStep);
                        rQ[p][r] = load_q(qmB[p] + (unsigned)kRing * qmStep);
                    }
                }
                // the member's new state, in place of its inputs (read kRing ticks ago by this
                // lane); launch_member_unpack forms the session state
#pragma unroll
                for (int p = 0; p < K; ++p) {
                    const int e = k - S[p].G;
                    const bool act = (unsigned)e < (unsigned)T;
                    if constexpr (SKEW) {
                        if (act) IO[cell(k, p)] = make_double2(ov[p], Iv[p]);
                    } else {
                        const u32x4 v = {(unsigned)__double2loint(ov[p]),
                                         (unsigned)__double2hiint(ov[p]),
                                         (unsigned)__double2loint(Iv[p]),
                                         (unsigned)__double2hiint(Iv[p])};
                        if (act) __builtin_amdgcn_raw_buffer_store_b128(v, io_r, ioB[p], 0, 0);
                        ioB[p] += ioStep;
                        qmB[p] += qmStep;
                    }
                    if (S[p].xsrc && act) {
                        const uint64_t bits = (uint64_t)__double_as_longlong(ov[p]);
                        const u32x4 gv = {(unsigned)bits, epoch, (unsigned)(bits >> 32), epoch};
                        __builtin_amdgcn_raw_buffer_store_b128(
                            gv, xg, (unsigned)((S[p].xs0 + k) * 16), 0, 16);
                    }
                }
                write_local(i, sb, ov);
                tick_end(i);
            }
        }
    } else {
        int rb[K], nr[K];
        double f0[K], f1[K], f2[K];
#pragma unroll
        for (int p = 0; p < K; ++p) {
            chunk_rows(tab, 0, kb, S[p].G, T, rb[p], nr[p]);
            f0[p] = Fm[(int64_t)clamp_row(rb[p], nrow) * ns + S[p].d];
            f1[p] = Fm[(int64_t)clamp_row(rb[p] + 1, nrow) * ns + S[p].d];
            f2[p] = Fm[(int64_t)clamp_row(rb[p] + 2, nrow) * ns + S[p].d];
        }
        __builtin_amdgcn_s_waitcnt(0);                      // nothing pending may enter the loop
        __syncthreads();                                    // prologue barrier (helper staged XE)
        t_loop = a.trace ? wall_clock64() : 0;
        c_loop = a.trace ? clock64() : 0;

        // lateral inflow of a position at tick i of the chunk, interpolate_sample
        // (nutils.py:23-33); it does not depend on the routing state (off the tick's chain).
        // K <= 2 forms the whole chunk's values up front; longer lanes form them per tick
        // (register budget)
        constexpr bool kBatchQ = K <= 2;
        // the exact form only when a non-finite value may occur (device flags of the session's
        // state and forcing): partial sums then keep a zero state (their update 0 + (((1 I +
        // 0 Ip) + 0 Op) + 0 q) is I for a non-finite I too) and clamped steps mask their high
        // row.  Both selects cost the common form ~6 % (same box), and neither is needed for
        // finite values.  A partial sum that meets a non-finite value in the fast form anyway
        // (an overflow of finite inputs) reports it, and the host re-routes the horizon with
        // the exact launches (sync()).
        const bool exact = a.nf == nullptr ||
                           __hip_atomic_load(a.nf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
                           __hip_atomic_load(a.nff, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        for (int kc = kb; kc < wend; kc += kChunk) {
            const unsigned sb = (unsigned)((kc >> 3) & 1) * XSLOT;   // this chunk's ring slot
            unsigned frp[K], tp[K];
            bool slow = false;
#pragma unroll
            for (int p = 0; p < K; ++p) {
                double* fr = reinterpret_cast<double*>(lds + FR) + (p * SLOTS + lid) * 3;
                fr[0] = f0[p];
                fr[1] = f1[p];
                fr[2] = f2[p];
                slow = slow || (DENSE && __any(nr[p] > 3));
                frp[p] = FR + (unsigned)(p * SLOTS + lid) * 24 - (unsigned)rb[p] * 8;
                tp[p] = TAB + (unsigned)(kc - S[p].G) * 16u;
            }
            const int Tn = kc + kChunk < wend ? T : 0;
            int rbn[K], nrn[K];
            double g0[K], g1[K], g2[K];
#pragma unroll
            for (int p = 0; p < K; ++p) {
                chunk_rows(tab, 0, kc + kChunk, S[p].G, Tn, rbn[p], nrn[p]);
                g0[p] = Fm[(int64_t)clamp_row(rbn[p], nrow) * ns + S[p].d];
                g1[p] = Fm[(int64_t)clamp_row(rbn[p] + 1, nrow) * ns + S[p].d];
                g2[p] = Fm[(int64_t)clamp_row(rbn[p] + 2, nrow) * ns + S[p].d];
            }
            unsigned m[K][kUpInline];
#pragma unroll
            for (int p = 0; p < K; ++p)
#pragma unroll
                for (int u = 0; u < kUpInline; ++u)
                    m[p][u] = S[p].uext[u] ? S[p].ubase[u] + sb : S[p].ubase[u];
            // two straight-line forms of the chunk (EXACT: the session's state or forcing holds a
            // non-finite value): the masked high row of clamped steps and the frozen state of
            // partial sums are needed only then -- for finite forcing (1 - 0) lo + 0 lo is lo
            // exactly, and a partial sum's update is I exactly for any finite state
            auto run_chunk = [&](auto mtag, auto ptag) {
                constexpr bool MASKQ = decltype(mtag)::value, PSUM = decltype(ptag)::value;
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
                    // clamped steps (frac = 0, row_lo == row_hi): lo + 0 * 0 -- the row itself
                    // (nutils.py:24-27) also for +-Inf / NaN rows (0 * hi would be NaN); the
                    // sign of a zero q cannot reach the outflow (its update ends in 0 + ...)
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
                    if (DENSE && slow) __builtin_amdgcn_s_waitcnt(0);
                }
#pragma unroll
                for (int i = 0; i < kChunk; ++i) {
                    const unsigned rd = (unsigned)((i + 7) & 7) * PL;   // plane of tick k - 1
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
                    double prev = 0.0;
#pragma unroll
                    for (int p = 0; p < K; ++p) {
                        bool act = (unsigned)(k - S[p].G) < (unsigned)T;
                        if constexpr (PSUM) act = act && !S[p].psum;   // zero state (Slot::psum)
                        const double I = fold_values(vin[p], S[p].chained, any3[p], prev, p == 0);
                        const double rr = dev::muskingum_update(S[p].al, I, S[p].be, S[p].ip,
                                                                S[p].ch, S[p].op,
                                                                dev::gq_term(S[p].ga, qv[p]));
                        const double o = rr;   // psum / unrouted / pad: set_slot_coeffs
                        S[p].op = act ? o : S[p].op;
                        S[p].ip = act ? I : S[p].ip;
                        ov[p] = o;
                        prev = o;
                    }
#pragma unroll
                    for (int p = 0; p < K; ++p)
                        *reinterpret_cast<double*>(lds + own[p] + (unsigned)i * PL) = ov[p];
                    // the tick's outputs reach the output window through the helper wave (plane
                    // k & 7 -> window row, copy_row; Texas det 0.515 -> 0.502 ms); the
                    // cross-cluster values leave from here (moving them to the helper too: 0.524,
                    // the helper's tick got longer than the compute waves')
#pragma unroll
                    for (int p = 0; p < K; ++p) {
                        if (S[p].xsrc && (unsigned)(k - S[p].G) < (unsigned)T) {
                            const uint64_t bits = (uint64_t)__double_as_longlong(ov[p]);
                            const u32x4 gv = {(unsigned)bits, epoch, (unsigned)(bits >> 32),
                                              epoch};
                            __builtin_amdgcn_raw_buffer_store_b128(
                                gv, xg, (unsigned)((S[p].xs0 + k) * 16), 0, 16);
                        }
                    }
                    write_local(i, sb, ov);
                    tick_end(i);
                }
            };
            using yes = std::true_type;
            using no = std::false_type;
            // the fast form is the fall-through path and the exact one out of line (inline, the
            // unexecuted forms cost the executed one ~3 %, same box)
            if (__builtin_expect(!exact, 1)) [[likely]] run_chunk(no{}, no{});
            else run_chunk(yes{}, yes{});
#pragma unroll
            for (int p = 0; p < K; ++p) {
                rb[p] = rbn[p];
                nr[p] = nrn[p];
                f0[p] = g0[p];
                f1[p] = g1[p];
                f2[p] = g2[p];
            }
        }
        // session state after the horizon; never-processed reaches hold o = 0 (nutils.py:68:
        // the kernel's own value for them, 0 q + ..., is NaN for non-finite inputs)
        bool nonfin = false, psum_hit = false;
#pragma unroll
        for (int p = 0; p < K; ++p) {
            const double so = S[p].unr ? 0.0 : S[p].op;
            a.st_o_out[S[p].d] = so;
            a.st_i_out[S[p].d] = S[p].ip;
            const bool bad = !__builtin_isfinite(so) || !__builtin_isfinite(S[p].ip);
            nonfin = nonfin || bad;
            // fast form: a partial sum's state that went non-finite stays non-finite (0 x it is
            // NaN from then on), so the end of the horizon sees every such case
            psum_hit = psum_hit || (!exact && S[p].psum && bad);
        }
        if (a.nf && __any(nonfin) && (lid & 63) == 0)
            __hip_atomic_store(a.nf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (__any(psum_hit) && (lid & 63) == 0)
            __hip_atomic_fetch_or(a.status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
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

template <bool DENSE, bool MEMB, bool SKEW = false>
const void* flow_fn(int slots, int chain, bool sync);

}  // namespace

bool flow_shape_ok(int slots, int chain, bool sync) {
#define MCR_CASE(S, K) if (slots == S && chain == K) return true;
    if (sync) {
        MCR_SYNC_SHAPES(MCR_CASE)
    } else {
        MCR_FLOW_SHAPES(MCR_CASE)
    }
#undef MCR_CASE
    return false;
}

namespace {

template <bool DENSE, bool MEMB, bool SKEW>
const void* flow_fn(int slots, int chain, bool sync) {
#define MCR_CASE(S, K)                 \
    if (slots == S && chain == K)      \
        return reinterpret_cast<const void*>(&wavefront_flow<S, K, DENSE, MEMB, SKEW>);
#define MCR_SCASE(S, K)                \
    if (slots == S && chain == K)      \
        return reinterpret_cast<const void*>(                                          \
            &wavefront_flow<S, K, DENSE, MEMB, SKEW, kWaveSlack>);
    if (sync) {
        MCR_SYNC_SHAPES(MCR_SCASE)
    } else {
        MCR_FLOW_SHAPES(MCR_CASE)
    }
#undef MCR_CASE
#undef MCR_SCASE
    return nullptr;
}

hipError_t occupancy_of(const void* fn, int slots, size_t lds, int* blocks_per_cu) {
    if (!fn) return hipErrorInvalidValue;
    const int threads = slots + kHelperLanes;
    int api = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&api, fn, threads, lds);
    if (e != hipSuccess) return e;
    hipFuncAttributes attr;
    e = hipFuncGetAttributes(&attr, fn);
    if (e != hipSuccess) return e;
    // Measured on gfx950 (launch trace, 5-wave workgroups at 128 VGPRs): a workgroup of W waves
    // takes ceil(W / 4) wave slots on EVERY SIMD, so the API's answer can be too high.  A SIMD
    // holds 512 VGPRs per lane.
    const int vgpr = ((attr.numRegs > 0 ? attr.numRegs : 512) + 7) / 8 * 8;
    const int per_simd = std::min(8, 512 / vgpr);
    const int waves = (threads + 63) / 64;
    const int by_waves = per_simd / ((waves + 3) / 4);
    const int by_lds = lds ? (int)((160 * 1024) / lds) : 8;
    *blocks_per_cu = std::min(api, std::min(by_waves, by_lds));
    return hipSuccess;
}

// staging cell of (slot d, member e) in the tick-major member windows (kernels.hpp MemberWin)
__device__ __forceinline__ int64_t member_cell(const MemberWin& mw, int64_t d, int64_t e) {
    if (!mw.skew) return e * mw.ns + d;
    const int64_t w = d / mw.rs;
    return mw.wbase[w] + (mw.G[d] + e - mw.gmin[w]) * mw.rs + (d - w * mw.rs);
}

// Member staging runs: thread per slot d, kMemberRun consecutive members per thread.  The
// member-major side ([E][nslots]) is one contiguous row per member over a wave's slots; the
// staging cell of (d, e) walks the lane's window column down consecutive rows (tick G[d] + e),
// so every window line is completed within one wave's loop (merged in L2) by the few lanes of
// the wave that share it.  Cell order (thread per (e, d)) completed a line only across far-apart
// waves, window order scattered the loads: 1.06 / 1.17 ms per EnKF256 input pass.
constexpr int kMemberRun = 16;

struct RunCells {
    int64_t c0, cs;     // cell of (d, e0) and the stride between consecutive members
};
__device__ __forceinline__ RunCells member_run(const MemberWin& mw, int64_t d, int64_t e0) {
    if (!mw.skew) return {e0 * mw.ns + d, mw.ns};
    const int64_t w = d / mw.rs;
    return {mw.wbase[w] + (mw.G[d] + e0 - mw.gmin[w]) * mw.rs + (d - w * mw.rs), mw.rs};
}

// IO = {o, i} of the session state, Qm = the lateral inflow of member e at the step (same
// expression as the tick loop), both at the staging cell of (d, e); padding slots skipped
// gain.G: pending analysis increments, applied as apply_gain (analysis.hip) would have applied
// them to st_o / st_i first -- the same operations in the same order, so bit-identical.
// GAIN walks runs of 4 members per thread (RUN): the upstream gathers of the one-hop fold need
// more threads in flight than the plain copy's runs of kMemberRun
template <bool GAIN, int RUN>
__global__ __launch_bounds__(256) void member_inputs(
        const double* __restrict__ F, int64_t mF, int64_t ns, int n_rows, int4 ent,
        const double* __restrict__ st_o, const double* __restrict__ st_i,
        double2* __restrict__ IO, double* __restrict__ Qm, int64_t E, MemberWin mw,
        PendingGain gain) {
    const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= ns) return;
    const uint8_t fl = mw.flags[d];
    if (fl == kSlotPad) return;
    const int64_t e0 = (int64_t)blockIdx.y * RUN;
    const int ne = (int)(E - e0 < RUN ? E - e0 : RUN);
    const RunCells rc = member_run(mw, d, e0);
    const double f = __hiloint2double(ent.w, ent.z);
    const int64_t rlo = (int64_t)clamp_row(ent.x, n_rows) * ns + d;
    const int64_t rhi = (int64_t)clamp_row(ent.y < 0 ? ent.x : ent.y, n_rows) * ns + d;
    // partial sums keep their state; unrouted reaches get no outflow gain (nutils.py:116-134)
    const bool gained = GAIN && (fl == kSlotRouted || fl == kSlotUnrouted);
    const int32_t u0 = GAIN ? gain.up_off[d] : 0, u1 = GAIN ? gain.up_off[d + 1] : 0;
#pragma unroll 4
    for (int k = 0; k < ne; ++k) {
        const int64_t e = e0 + k;
        const int64_t idx = e * ns + d;
        const double* Fe = F + e * mF;
        const double lo = Fe[rlo];
        const double hi = Fe[rhi];
        const int64_t c = rc.c0 + k * rc.cs;
        double o = st_o[idx], i = st_i[idx];
        if (gained) {
            const double* Ge = gain.G + e * ns;
            const double og = fl == kSlotRouted ? 0.0 + Ge[d] : 0.0;
            double ig = 0.0;
#pragma unroll 4
            for (int32_t q = u0; q < u1; ++q) ig = ig + (0.0 + Ge[gain.up[q]]);
            o = o + og;
            i = i + ig;
        }
        IO[c] = make_double2(o, i);
        Qm[c] = ent.x == ent.y ? lo : (1.0 - f) * lo + f * hi;   // clamped: row copy
    }
}

// The one-hop inflow increments of a pending gain, GI[e][d] = the left fold from 0 of
// (0 + G[e][u]) over the routed upstream slots u of d in rank order -- exactly the sum
// apply_gain adds to the inflow state (analysis.hip).  Thread per slot, kGiRun members per
// thread: the upstream list is read once, and a wave's upstream reads stay within a few lines
// of each member row (upstream slots sit mostly one lane position away in the plan's order).
constexpr int kGiRun = 8;
__global__ __launch_bounds__(256) void inflow_increments(
        const double* __restrict__ G, const int32_t* __restrict__ up_off,
        const int32_t* __restrict__ up, double* __restrict__ GI, int64_t ns, int64_t E) {
    const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= ns) return;
    const int64_t e0 = (int64_t)blockIdx.y * kGiRun;
    const int ne = (int)(E - e0 < kGiRun ? E - e0 : kGiRun);
    const int32_t u0 = up_off[d], u1 = up_off[d + 1];
    int32_t upr[kUpInline];
#pragma unroll
    for (int k = 0; k < kUpInline; ++k) upr[k] = u0 + k < u1 ? up[u0 + k] : (int32_t)d;
#pragma unroll 2
    for (int k = 0; k < ne; ++k) {
        const double* Ge = G + (e0 + k) * ns;
        double gu[kUpInline];
#pragma unroll
        for (int q = 0; q < kUpInline; ++q) gu[q] = Ge[upr[q]];      // unconditional (dummy d)
        double ig = 0.0;
#pragma unroll
        for (int q = 0; q < kUpInline; ++q) ig = u0 + q < u1 ? ig + (0.0 + gu[q]) : ig;
        for (int32_t q = u0 + kUpInline; q < u1; ++q) ig = ig + (0.0 + Ge[up[q]]);
        GI[(e0 + k) * ns + d] = ig;
    }
}

// Member staging of the skewed windows through LDS (E >= kSkewMembers): one wave per group of
// kStageSlots consecutive slots (one 256-B IO segment of a window row).  The per-lane form above
// writes cell (d, e) at row G[d] + e, so a wave's store touches a different window line in
// almost every lane (~3.7 TB/s at EnKF256); here the wave reads the member-major side a whole
// 128-B line per 16 lanes (4 members per load), keeps the staged {o, i, q} of the last
// kStageRing members in an LDS ring, and writes the window rows whose members are all staged,
// 4 rows x 16 slots per store: both sides move whole lines.  A group whose G spread exceeds what
// the ring can hold (spread > kStageRing - kStageChunk) stores directly, as the per-lane form.
// Same operations per (d, e) as member_inputs, so bit-identical.
#ifndef MCR_STAGE_RING
#define MCR_STAGE_RING 1
#endif
constexpr int kStageSlots = 16;
constexpr int kStageRing = 32;
#ifndef MCR_STAGE_CHUNK
#define MCR_STAGE_CHUNK 16
#endif
constexpr int kStageChunk = MCR_STAGE_CHUNK;     // members staged per round (4 per load)
constexpr int kStageLoads = kStageChunk / 4;
template <bool GAIN>
__global__ __launch_bounds__(256) void member_inputs_ring(
        const double* __restrict__ F, int64_t mF, int64_t ns, int n_rows, int4 ent,
        const double* __restrict__ st_o, const double* __restrict__ st_i,
        double2* __restrict__ IO, double* __restrict__ Qm, int64_t E, MemberWin mw,
        PendingGain gain) {
    __shared__ double ring[4][3][kStageRing * kStageSlots];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int s = lane & (kStageSlots - 1), sub = lane >> 4;
    const int64_t d0 = ((int64_t)blockIdx.x * 4 + wv) * kStageSlots;
    if (d0 >= ns) return;                                  // wave-uniform
    const int64_t d = d0 + s;
    const uint8_t fl = mw.flags[d];
    const bool real = fl != kSlotPad;
    const int64_t w = d0 / mw.rs;
    const int gs = real ? mw.G[d] - mw.gmin[w] : 0;       // window row of member 0
    int glo = real ? gs : 0x7fffffff, ghi = real ? gs : -1;
#pragma unroll
    for (int o = kStageSlots / 2; o >= 1; o >>= 1) {
        glo = min(glo, __shfl_xor(glo, o, kStageSlots));
        ghi = max(ghi, __shfl_xor(ghi, o, kStageSlots));
    }
    if (ghi < 0) return;                                   // padding only (wave-uniform)
    const int64_t rs = mw.rs;
    const int64_t cell0 = mw.wbase[w] + (d - w * rs);
    const double f = __hiloint2double(ent.w, ent.z);
    const int64_t rlo = (int64_t)clamp_row(ent.x, n_rows) * ns + d;
    const int64_t rhi = (int64_t)clamp_row(ent.y < 0 ? ent.x : ent.y, n_rows) * ns + d;
    const bool gained = GAIN && (fl == kSlotRouted || fl == kSlotUnrouted);
    const bool pre = GAIN && gain.gi != nullptr;           // one-hop fold formed beforehand
    const int32_t u0 = GAIN && !pre ? gain.up_off[d] : 0;
    const int32_t u1 = GAIN && !pre ? gain.up_off[d + 1] : 0;
    // the first kUpInline upstream slots in registers: their increments are loaded together
    // (independent loads) and folded in rank order; longer lists continue in a loop
    int32_t upr[kUpInline];
#pragma unroll
    for (int k = 0; k < kUpInline; ++k) upr[k] = u0 + k < u1 ? gain.up[u0 + k] : (int32_t)d;
    auto value = [&](int64_t e, double& o, double& i, double& q) {
        const int64_t idx = e * ns + d;
        const double* Fe = F + e * mF;
        const double lo = Fe[rlo];
        const double hi = Fe[rhi];
        o = st_o[idx];
        i = st_i[idx];
        if (gained) {
            const double* Ge = gain.G + e * ns;
            const double og = fl == kSlotRouted ? 0.0 + Ge[d] : 0.0;
            double ig = 0.0;
            if (pre) {
                ig = gain.gi[idx];
            } else {
                double gu[kUpInline];
#pragma unroll
                for (int k = 0; k < kUpInline; ++k) gu[k] = Ge[upr[k]];   // unconditional (dummy d)
#pragma unroll
                for (int k = 0; k < kUpInline; ++k) ig = u0 + k < u1 ? ig + (0.0 + gu[k]) : ig;
                for (int32_t u = u0 + kUpInline; u < u1; ++u) ig = ig + (0.0 + Ge[gain.up[u]]);
            }
            o = o + og;
            i = i + ig;
        }
        q = ent.x == ent.y ? lo : (1.0 - f) * lo + f * hi;       // clamped: row copy
    };
    if (ghi - glo > kStageRing - kStageChunk) {            // wide group (wave-uniform)
        if (real)
            for (int64_t e0 = 0; e0 < E; e0 += kStageChunk) {
                double o[kStageLoads], i[kStageLoads], q[kStageLoads];
#pragma unroll
                for (int h = 0; h < kStageLoads; ++h)
                    if (e0 + 4 * h + sub < E) value(e0 + 4 * h + sub, o[h], i[h], q[h]);
#pragma unroll
                for (int h = 0; h < kStageLoads; ++h) {
                    const int64_t e = e0 + 4 * h + sub;
                    if (e < E) {
                        const int64_t c = cell0 + ((int64_t)gs + e) * rs;
                        IO[c] = make_double2(o[h], i[h]);
                        Qm[c] = q[h];
                    }
                }
            }
        return;
    }
    double* Ro = ring[wv][0];
    double* Ri = ring[wv][1];
    double* Rq = ring[wv][2];
    const int rend = ghi + (int)E;                         // rows glo .. rend - 1
    int next = glo;                                        // first row not yet stored
    for (int e0 = 0; e0 < (int)E; e0 += kStageChunk) {
        double o[kStageLoads], i[kStageLoads], q[kStageLoads];
#pragma unroll
        for (int h = 0; h < kStageLoads; ++h) {
            const int e = e0 + 4 * h + sub;
            if (real && e < (int)E) value(e, o[h], i[h], q[h]);
        }
#pragma unroll
        for (int h = 0; h < kStageLoads; ++h) {
            const int e = e0 + 4 * h + sub;
            if (real && e < (int)E) {
                const int k = (e & (kStageRing - 1)) * kStageSlots + s;
                Ro[k] = o[h];
                Ri[k] = i[h];
                Rq[k] = q[h];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // rows whose members are all staged: row r takes member r - gs <= r - glo
        const int staged = min(e0 + kStageChunk, (int)E);
        const int rstop = staged >= (int)E ? rend : glo + staged;
        if (next < rstop) {
            for (int r0 = next; r0 < rstop; r0 += 4) {
                const int r = r0 + sub;
                const int e = r - gs;
                if (real && r < rstop && e >= 0 && e < (int)E) {
                    const int k = (e & (kStageRing - 1)) * kStageSlots + s;
                    const int64_t c = cell0 + (int64_t)r * rs;
                    IO[c] = make_double2(Ro[k], Ri[k]);
                    Qm[c] = Rq[k];
                }
            }
            next = rstop;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// The reverse of member_inputs_ring for member_unpack: a wave per group of kStageSlots slots
// reads the group's window rows in order (4 rows x 16 slots per load: whole lines), parks the
// cells in an LDS ring by member, and writes each member's {o, i} once every slot's cell of it
// has been read (member e is complete after row ghi + e), 4 members x 16 slots per store.
template <int UNUSED = 0>
__global__ __launch_bounds__(256) void member_unpack_ring(
        const double2* __restrict__ IO, double* __restrict__ st_o, double* __restrict__ st_i,
        int64_t ns, int64_t E, MemberWin mw) {
    __shared__ double ring[4][2][kStageRing * kStageSlots];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int s = lane & (kStageSlots - 1), sub = lane >> 4;
    const int64_t d0 = ((int64_t)blockIdx.x * 4 + wv) * kStageSlots;
    if (d0 >= ns) return;                                  // wave-uniform
    const int64_t d = d0 + s;
    const uint8_t fl = mw.flags[d];
    const bool real = fl != kSlotPad;
    // never-processed reaches keep o = 0 (nutils.py:68; their cell holds the kernel's 0 q + ...),
    // partial sums a zero state (device_common.hpp Slot::Ga)
    const bool zo = fl == kSlotUnrouted || fl == kSlotSum, zi = fl == kSlotSum;
    const int64_t w = d0 / mw.rs;
    const int gs = real ? mw.G[d] - mw.gmin[w] : 0;
    int glo = real ? gs : 0x7fffffff, ghi = real ? gs : -1;
#pragma unroll
    for (int o = kStageSlots / 2; o >= 1; o >>= 1) {
        glo = min(glo, __shfl_xor(glo, o, kStageSlots));
        ghi = max(ghi, __shfl_xor(ghi, o, kStageSlots));
    }
    if (ghi < 0) return;
    const int64_t rs = mw.rs;
    const int64_t cell0 = mw.wbase[w] + (d - w * rs);
    if (ghi - glo > kStageRing - kStageChunk) {            // wide group: direct, per lane
        if (real)
            for (int64_t e0 = 0; e0 < E; e0 += kStageChunk) {
                double2 v[kStageLoads];
#pragma unroll
                for (int h = 0; h < kStageLoads; ++h) {
                    const int64_t e = e0 + 4 * h + sub;
                    if (e < E) v[h] = IO[cell0 + ((int64_t)gs + e) * rs];
                }
#pragma unroll
                for (int h = 0; h < kStageLoads; ++h) {
                    const int64_t e = e0 + 4 * h + sub;
                    if (e < E) {
                        st_o[e * ns + d] = zo ? 0.0 : v[h].x;
                        st_i[e * ns + d] = zi ? 0.0 : v[h].y;
                    }
                }
            }
        return;
    }
    double* Ro = ring[wv][0];
    double* Ri = ring[wv][1];
    const int rend = ghi + (int)E;
    int done = 0;                                          // members [0, done) written
    for (int r0 = glo; r0 < rend; r0 += kStageChunk) {
        double2 v[kStageLoads];
#pragma unroll
        for (int h = 0; h < kStageLoads; ++h) {
            const int r = r0 + 4 * h + sub, e = r - gs;
            if (real && r < rend && e >= 0 && e < (int)E) v[h] = IO[cell0 + (int64_t)r * rs];
        }
#pragma unroll
        for (int h = 0; h < kStageLoads; ++h) {
            const int r = r0 + 4 * h + sub, e = r - gs;
            if (real && r < rend && e >= 0 && e < (int)E) {
                const int k = (e & (kStageRing - 1)) * kStageSlots + s;
                Ro[k] = v[h].x;
                Ri[k] = v[h].y;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int upto = min(min(r0 + kStageChunk, rend) - ghi, (int)E);
        if (done < upto) {
            for (int e0 = done; e0 < upto; e0 += 4) {
                const int e = e0 + sub;
                if (real && e < upto) {
                    const int k = (e & (kStageRing - 1)) * kStageSlots + s;
                    st_o[(int64_t)e * ns + d] = zo ? 0.0 : Ro[k];
                    st_i[(int64_t)e * ns + d] = zi ? 0.0 : Ri[k];
                }
            }
            done = upto;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

}  // namespace

hipError_t flow_occupancy(int slots, int chain, bool dense, bool sync, size_t lds,
                          int* blocks_per_cu) {
    return occupancy_of(dense ? flow_fn<true, false>(slots, chain, sync)
                              : flow_fn<false, false>(slots, chain, sync),
                        slots, lds, blocks_per_cu);
}

hipError_t flow_members_occupancy(int slots, int chain, bool sync, size_t lds,
                                  int* blocks_per_cu) {
    int a = 0, b = 0;                        // both staging layouts must be resident
    hipError_t e = occupancy_of(flow_fn<false, true, false>(slots, chain, sync), slots, lds, &a);
    if (e == hipSuccess)
        e = occupancy_of(flow_fn<false, true, true>(slots, chain, sync), slots, lds, &b);
    *blocks_per_cu = std::min(a, b);
    return e;
}

hipError_t launch_flow(const WaveArgs& a, int grid, int slots, int chain, size_t lds, bool dense,
                       bool sync, hipStream_t s) {
    const void* fn = dense ? flow_fn<true, false>(slots, chain, sync)
                           : flow_fn<false, false>(slots, chain, sync);
    if (!fn) return hipErrorInvalidValue;
    void* args[] = {const_cast<WaveArgs*>(&a)};
    return hipLaunchKernel(fn, dim3(grid), dim3(slots + kHelperLanes), args, lds, s);
}

hipError_t launch_flow_members(const WaveArgs& a, int grid, int slots, int chain, size_t lds,
                               bool sync, hipStream_t s) {
    const void* fn = a.mskew ? flow_fn<false, true, true>(slots, chain, sync)
                             : flow_fn<false, true, false>(slots, chain, sync);
    if (!fn) return hipErrorInvalidValue;
    void* args[] = {const_cast<WaveArgs*>(&a)};
    return hipLaunchKernel(fn, dim3(grid), dim3(slots + kHelperLanes), args, lds, s);
}

// After a member-dataflow step: the session state from the IO pairs.  The IO pairs themselves
// stay the step's outputs (o, and the inflow fold i) until the next run: the fetches read them
// there (launch_gather_io) instead of scattering them into the T = 1 output windows.
__global__ __launch_bounds__(256) void member_unpack(
        const double2* __restrict__ IO, double* __restrict__ st_o, double* __restrict__ st_i,
        int64_t ns, int64_t E, MemberWin mw) {
    const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= ns || mw.flags[d] == kSlotPad) return;
    // never-processed reaches: o stays 0 (nutils.py:68); partial sums: zero state (Slot::Ga)
    const bool zo = mw.flags[d] == kSlotUnrouted || mw.flags[d] == kSlotSum;
    const bool zi = mw.flags[d] == kSlotSum;
    const int64_t e0 = (int64_t)blockIdx.y * kMemberRun;
    const int ne = (int)(E - e0 < kMemberRun ? E - e0 : kMemberRun);
    const RunCells rc = member_run(mw, d, e0);
#pragma unroll 4
    for (int k = 0; k < ne; ++k) {
        const double2 v = IO[rc.c0 + k * rc.cs];
        st_o[(e0 + k) * ns + d] = zo ? 0.0 : v.x;
        st_i[(e0 + k) * ns + d] = zi ? 0.0 : v.y;
    }
}

// out[j][e] = IO[e][pos[j]].x (outflow) or .y (inflow): the outputs of a member-dataflow step in
// caller order, member innermost
__global__ void gather_io(const double2* __restrict__ IO, const int64_t* __restrict__ pos,
                          bool inflow, double* __restrict__ out, int64_t n, int64_t E,
                          MemberWin mw) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= n * E) return;
    const int64_t j = x / E, e = x - j * E;
    const int64_t d = pos[j];
    const double2 v = IO[member_cell(mw, d, e)];
    out[x] = inflow ? v.y : (mw.flags[d] == kSlotUnrouted ? 0.0 : v.x);   // unrouted: o = 0
}

static dim3 member_grid(int64_t ns, int64_t E) {
    return dim3((unsigned)((ns + 255) / 256), (unsigned)((E + kMemberRun - 1) / kMemberRun));
}

hipError_t launch_member_unpack(const double* IO, const MemberWin& mw, double* st_o,
                                double* st_i, int64_t ns, int64_t E, hipStream_t s) {
    if (ns * E == 0) return hipSuccess;
    if (mw.skew && MCR_STAGE_RING && mw.rs % kStageSlots == 0 && ns % kStageSlots == 0) {
        hipLaunchKernelGGL(member_unpack_ring<>, dim3((unsigned)((ns / kStageSlots + 3) / 4)), 256,
                           0, s, reinterpret_cast<const double2*>(IO), st_o, st_i, ns, E, mw);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(member_unpack, member_grid(ns, E), 256, 0, s,
                       reinterpret_cast<const double2*>(IO), st_o, st_i, ns, E, mw);
    return hipGetLastError();
}

hipError_t launch_gather_io(const double* IO, const MemberWin& mw, const int64_t* pos,
                            bool inflow, double* out, int64_t n, int64_t E, hipStream_t s) {
    if (n * E == 0) return hipSuccess;
    hipLaunchKernelGGL(gather_io, dim3((unsigned)((n * E + 255) / 256)), 256, 0, s,
                       reinterpret_cast<const double2*>(IO), pos, inflow, out, n, E, mw);
    return hipGetLastError();
}

hipError_t launch_member_inputs(const double* F, int64_t mF, int64_t ns, int n_rows, int4 ent,
                                const double* st_o, const double* st_i, double* IO, double* Qm,
                                int64_t E, const MemberWin& mw, hipStream_t s,
                                const PendingGain& gain) {
    if (ns * E == 0) return hipSuccess;
    if ((E + kMemberRun - 1) / kMemberRun > 65535) return hipErrorInvalidValue;
    const bool ring = mw.skew && MCR_STAGE_RING && mw.rs % kStageSlots == 0 &&
                      ns % kStageSlots == 0;
    // the one-hop fold formed first for the LDS-ring staging (EnKF256 115.2 -> 112.8 ms per
    // horizon, same box); the per-lane runs of small ensembles gather it in place (EnKF32 21.7
    // vs 22.5 ms with the extra pass)
    PendingGain g = gain;
    if (!ring) g.gi = nullptr;
    if (g.G && g.gi) {
        if ((E + kGiRun - 1) / kGiRun > 65535) return hipErrorInvalidValue;
        hipLaunchKernelGGL(inflow_increments,
                           dim3((unsigned)((ns + 255) / 256), (unsigned)((E + kGiRun - 1) / kGiRun)),
                           256, 0, s, g.G, g.up_off, g.up, g.gi, ns, E);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (ring) {
        const dim3 grid((unsigned)((ns / kStageSlots + 3) / 4));
        if (gain.G)
            hipLaunchKernelGGL((member_inputs_ring<true>), grid, 256, 0, s, F, mF, ns, n_rows,
                               ent, st_o, st_i, reinterpret_cast<double2*>(IO), Qm, E, mw, g);
        else
            hipLaunchKernelGGL((member_inputs_ring<false>), grid, 256, 0, s, F, mF, ns, n_rows,
                               ent, st_o, st_i, reinterpret_cast<double2*>(IO), Qm, E, mw, g);
        return hipGetLastError();
    }
    constexpr int kGainRun = 4;
    if (gain.G) {
        if ((E + kGainRun - 1) / kGainRun > 65535) return hipErrorInvalidValue;
        hipLaunchKernelGGL((member_inputs<true, kGainRun>),
                           dim3((unsigned)((ns + 255) / 256),
                                (unsigned)((E + kGainRun - 1) / kGainRun)),
                           256, 0, s, F, mF, ns, n_rows, ent, st_o, st_i,
                           reinterpret_cast<double2*>(IO), Qm, E, mw, g);
    } else {
        hipLaunchKernelGGL((member_inputs<false, kMemberRun>), member_grid(ns, E), 256, 0, s, F,
                           mF, ns, n_rows, ent, st_o, st_i, reinterpret_cast<double2*>(IO), Qm,
                           E, mw, g);
    }
    return hipGetLastError();
}

// ---- latency floor of the dataflow tick (diagnostic, mc_probe_tick_floor) -------------------
// The irreducible per-tick chain of wavefront_flow<SLOTS, K> with no memory traffic: every lane
// reads two inputs of each position from the previous tick plane (LDS), folds them, runs its K
// chained Muskingum updates, writes the outputs to the current plane and joins the workgroup's
// tick barrier (with the helper wave, which here only joins the barriers).  Same block shape,
// waves-per-EU bound and LDS request as the real kernel, two workgroups per CU: ticks x this
// kernel's time per tick is the schedule's latency floor (bench.py roofline.latency).
template <int SLOTS, int K>
__global__ __launch_bounds__(SLOTS + kHelperLanes)
__attribute__((amdgpu_waves_per_eu(2, 2)))
void tick_floor(int ticks, double* __restrict__ out) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int RS = K * SLOTS;
    constexpr unsigned PL = flow_plane_bytes(RS);
    const int tid = threadIdx.x;
    if ((tid >> 6) == SLOTS / 64) {
        __syncthreads();
        for (int k = 0; k < ticks; ++k) __syncthreads();
        return;
    }
    unsigned m[K][2], own[K];
    double op[K], ip[K];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        m[p][0] = (unsigned)((p * SLOTS + tid + 1) % RS) * 8u;
        m[p][1] = (unsigned)((p * SLOTS + tid + 65) % RS) * 8u;
        own[p] = (unsigned)(p * SLOTS + tid) * 8u;
        op[p] = 1.0 + tid;
        ip[p] = 2.0;
        for (int k = 0; k < kChunk; ++k)
            *reinterpret_cast<double*>(lds + own[p] + (unsigned)k * PL) = 1.0;
    }
    const double al = 0.1, be = 0.1, ch = 0.2, ga = 0.5, q = 1.0 + 1e-3 * tid;
    __syncthreads();
    for (int kc = 0; kc < ticks; kc += kChunk) {
#pragma unroll
        for (int i = 0; i < kChunk; ++i) {
            const unsigned rd = (unsigned)((i + 7) & 7) * PL;
            double v[K][2];
#pragma unroll
            for (int p = 0; p < K; ++p) {
                v[p][0] = lds_f64(lds, m[p][0] + rd);
                v[p][1] = lds_f64(lds, m[p][1] + rd);
            }
            double prev = 0.0;
#pragma unroll
            for (int p = 0; p < K; ++p) {
                double I = v[p][0] + v[p][1];
                if (p > 0) I = I + prev;
                const double o = dev::muskingum_update(al, I, be, ip[p], ch, op[p],
                                                       dev::gq_term(ga, q));
                op[p] = o;
                ip[p] = I;
                prev = o;
            }
#pragma unroll
            for (int p = 0; p < K; ++p)
                *reinterpret_cast<double*>(lds + own[p] + (unsigned)i * PL) = op[p];
            __syncthreads();
        }
    }
    out[(int64_t)blockIdx.x * SLOTS + tid] = op[K - 1];
}

hipError_t probe_tick_floor(int slots, int chain, int grid, int ticks, hipStream_t s,
                            double* out) {
    if (ticks <= 0 || ticks % kChunk != 0 || grid <= 0) return hipErrorInvalidValue;
    const size_t lds = flow_lds_bytes(slots, chain, 288, kFlowMaxExt);
    if (slots == 192 && chain == 2)
        hipLaunchKernelGGL((tick_floor<192, 2>), dim3(grid), dim3(192 + kHelperLanes), lds, s,
                           ticks, out);
    else if (slots == 384 && chain == 2)
        hipLaunchKernelGGL((tick_floor<384, 2>), dim3(grid), dim3(384 + kHelperLanes), lds, s,
                           ticks, out);
    else if (slots == 64 && chain == 1)
        hipLaunchKernelGGL((tick_floor<64, 1>), dim3(grid), dim3(64 + kHelperLanes), lds, s,
                           ticks, out);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

}  // namespace mcr
