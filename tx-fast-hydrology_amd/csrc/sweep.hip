// Member sweep (sweep.hpp): the ensemble forecast with the members on the lanes.
//
// One workgroup = kSweepNW compute waves (+ a store wave) = the kSweepSlots node slots of one
// member-plan workgroup.  The member plan has kSweepNW "lanes" of kSweepNPW positions (plan.hpp
// lane chains): wave v routes the chain of plan lane v, positions p = 0 .. NPW - 1 in order
// within a tick (a chained input is the previous position's output of the same tick, from a
// register), for 64 members (lane = member, blockIdx.y = member group).  Per node everything that decides control flow or addresses is wave-uniform (the
// node's step at this tick, its inputs, coefficients and forcing rows), so the tick is scalar
// control plus f64 arithmetic on 64 members, and every global access is one 512-byte row.
//
// Tick k (node d runs step t = k - G[d] when 0 <= t < T):
//   reads   the inputs' outputs of tick k - 1: in-cluster inputs (unit slack) from the LDS buffer
//           of parity (k - 1) & 1, inputs of other workgroups (produced in earlier launches:
//           tile slack) from ring slot k % 4, which the loader wave filled by LDS-DMA three
//           ticks ahead; the table entry of each node's step (row pair, frac);
//   routes  I = ((0 + x1) + x2) + ...,  o = 0 + (((alpha I + beta I_prev) + chi o_prev) + gamma q),
//           q = (1 - frac) f[lo] + frac f[hi]   (nutils.py:23-33, 80-83; FMA contraction off),
//           the NPW nodes of a wave in position order (a chained input from a register);
//   writes  o to the LDS buffer of parity k & 1;
//   then one workgroup barrier; the store wave copies the rows of tick k to O[t][d][.] during
//   tick k + 1.
// Roles keep the wait counts apart: compute waves issue no stores (their only loads are
// forcing rows), the store wave never waits for its stores, the loader waits only for its own
// loads.  Forcing: a node keeps f[lo], f[hi] of its current step's row pair and f[hi + 1];
// when its step moves to the next pair (host-checked: rows advance by at most one per step)
// they shift and the next row is loaded.
#include "sweep.hpp"


#include "kernels.hpp"
#include "plan.hpp"

#pragma clang fp contract(off)

// minimum waves per SIMD the register allocation targets (4: two workgroups per CU at <= 128
// VGPRs, with some spilling; 1: the compiler's choice, 134 VGPRs = 3 waves per SIMD)
#ifndef MCR_SWEEP_MIN_WAVES
#define MCR_SWEEP_MIN_WAVES 1
#endif

namespace mcr {

namespace {

typedef unsigned u32x2_t __attribute__((ext_vector_type(2)));

constexpr unsigned kRow = 512;   // LDS / global row: 64 members x f64
constexpr int kRing = 4;         // external-input ring slots (ticks; a power of two)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rec(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes,
                                             0x00020000);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rec_at(uintptr_t p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(p), (short)0, (int)bytes,
                                             0x00020000);
}
__device__ __forceinline__ double bld(__amdgpu_buffer_rsrc_t r, unsigned off) {
    const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    return __hiloint2double((int)v.y, (int)v.x);
}
template <int AUX>
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, unsigned off, double x) {
    u32x2_t v;
    v.x = (unsigned)__double2loint(x);
    v.y = (unsigned)__double2hiint(x);
    __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, AUX);
}
__device__ __forceinline__ double lds_ld(const char* lds, unsigned byte) {
    return *reinterpret_cast<const double*>(lds + byte);
}
__device__ __forceinline__ void lds_st(char* lds, unsigned byte, double x) {
    *reinterpret_cast<double*>(lds + byte) = x;
}
__device__ __forceinline__ int clamp_t(int t, int T) { return t < 0 ? 0 : (t < T ? t : T - 1); }

// NPW node slots per compute wave, NW compute waves, a store wave and a loader wave; XMAX
// external inputs per workgroup.  LDS: the step-table window of the launch, the workgroup's
// coefficients and G, two parity buffers of node rows (+ a zero row), and a ring of kRing tick
// slots of external-input rows.
template <int NPW, int NW, int XMAX>
__global__ __launch_bounds__(64 * (NW + 2), MCR_SWEEP_MIN_WAVES)
void member_sweep(SweepArgs a) {
    constexpr int RS = NPW * NW;
    // the parity buffers first, so that their offsets fit a DS instruction's immediate
    constexpr unsigned XB = 0;                                    // [2][RS + 1 + XMAX] rows
    constexpr unsigned BUF = (RS + 1 + XMAX) * kRow;
    constexpr unsigned XE = XB + 2 * BUF;                         // [kRing][XMAX] rows
    constexpr unsigned XSLOT = XMAX * kRow;
    constexpr unsigned TAB = XE + kRing * XSLOT;                  // int4 [kSweepTabCap]
    constexpr unsigned COEF = TAB + 16u * kSweepTabCap;           // double [RS][4]
    constexpr unsigned GT = COEF + 32u * RS;                      // int [RS]
    static_assert(2 * BUF <= 65536, "parity buffers must be addressable by DS immediates");
    extern __shared__ __attribute__((aligned(16))) char lds[];

    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int w = a.active[blockIdx.x];
    const int T = a.T, k0 = a.k0, tile = a.tile, nrow = a.n_rows, E = a.E;
    const uint32_t rowB = a.rowB;
    const int e = (int)blockIdx.y * 64 + lane;
    const unsigned eo = e < E ? (unsigned)e * 8u : 0x80000000u;   // beyond E: out of range
    const unsigned l8 = (unsigned)lane * 8u;
    const uintptr_t Fb = reinterpret_cast<uintptr_t>(a.F);
    const uintptr_t Ob = reinterpret_cast<uintptr_t>(a.O);
    const bool tr = a.trace != nullptr && blockIdx.y == 0 && threadIdx.x == 0;
    const int64_t t_start = tr ? wall_clock64() : 0;

    // ---- step-table window: every (clamped) step a node of this workgroup looks up in the
    // launch, [tw0, tw1]; lookups outside it are clamped into it (non-live slots only)
    const int gmin = a.wg_gmin[w], gmax = a.wg_gmax[w];
    const int tw0 = clamp_t(k0 - gmax, T), tw1 = clamp_t(k0 + tile + kChunk - gmin, T);
    // entries {pair = 2 row_lo + (row_hi - row_lo), -, frac}: row_hi - row_lo is 0 or 1
    // (host-checked), so a step's row pair is one uniform word
    for (int i = threadIdx.x; i <= tw1 - tw0; i += 64 * (NW + 2)) {
        const int4 en = a.stab[tw0 + i];
        reinterpret_cast<int4*>(lds + TAB)[i] = make_int4(2 * en.x + (en.y - en.x), 0, en.z, en.w);
    }

    if (wv == NW + 1) {
        // ================= loader wave: the rows of the workgroup's external inputs (outputs of
        // other workgroups, produced in earlier launches) for consumer tick k go to ring slot
        // k % kRing by LDS-DMA, kRing - 1 ticks ahead, two rows per instruction (lanes 0-31 row
        // 2m, 32-63 row 2m + 1; 16 B = two members per lane).  Its wait counts cover only its
        // own loads, so it uses raw barriers (no drain at a __syncthreads).
        const int x0 = a.ext_off[w], nx = a.ext_off[w + 1] - x0;
        const int nin = (nx + 1) >> 1;                   // instructions per tick
        const int half = lane >> 5;
        const int em = (int)blockIdx.y * 64 + 2 * (lane & 31);
        const int64_t nsE = (int64_t)(rowB / 8u);
        int xg[XMAX / 2];
        int64_t xs[XMAX / 2];
#pragma unroll
        for (int m = 0; m < XMAX / 2; ++m) {
            const int x = 2 * m + half;
            const bool ok = x < nx;
            xg[m] = ok ? a.ext_g[x0 + x] : 0;
            xs[m] = ok ? (int64_t)a.ext_slot[x0 + x] * E : 0;
        }
        auto issue = [&](int k) {                        // the rows of consumer tick k
            const unsigned slot = XE + (unsigned)(k & (kRing - 1)) * XSLOT;
#pragma unroll
            for (int m = 0; m < XMAX / 2; ++m) {
                if (m < nin) {
                    const int t = clamp_t(k - xg[m], T);    // (other steps are never read)
                    const double* src = a.O + ((int64_t)t * nsE + xs[m] + em);
                    __builtin_amdgcn_global_load_lds(
                        src, (__attribute__((address_space(3))) void*)(lds + slot + 1024u * m),
                        16, 0, 0);
                }
            }
        };
        // wait until at most 2 ticks of loads are in flight (those of ticks k + 1, k + 2 issued
        // after the rows of tick k)
        auto wait_two = [&]() {
            switch (nin) {
#define MCR_SWEEP_W(n)                                                 \
    case n:                                                            \
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * n) : "memory");   \
        break;
                MCR_SWEEP_W(0) MCR_SWEEP_W(1) MCR_SWEEP_W(2) MCR_SWEEP_W(3) MCR_SWEEP_W(4)
                MCR_SWEEP_W(5) MCR_SWEEP_W(6) MCR_SWEEP_W(7) MCR_SWEEP_W(8) MCR_SWEEP_W(9)
                MCR_SWEEP_W(10) MCR_SWEEP_W(11) MCR_SWEEP_W(12)
#undef MCR_SWEEP_W
                default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
        };
        auto barrier = [&]() {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
        };
        // ring slot of consumer tick j -> the ext rows of parity buffer (j - 1) & 1, which the
        // consumers of tick j read (two rows per 16-B lane access)
        auto stage = [&](int j) {
            const unsigned src = XE + (unsigned)(j & (kRing - 1)) * XSLOT;
            const unsigned dst = XB + (unsigned)((j - 1) & 1) * BUF + (unsigned)(RS + 1) * kRow;
            const unsigned l16 = (unsigned)lane * 16u;
            for (int m = 0; m < nin; ++m) {
                typedef double d2 __attribute__((ext_vector_type(2)));
                const d2 v = *reinterpret_cast<const d2*>(lds + src + 1024u * m + l16);
                *reinterpret_cast<d2*>(lds + dst + 1024u * m + l16) = v;
            }
        };
        barrier();                                       // table window, G
        issue(k0);
        issue(k0 + 1);
        issue(k0 + 2);
        wait_two();                                      // tick k0's rows have landed
        stage(k0);
        barrier();                                       // prologue of the compute waves
        for (int k = k0; k < k0 + tile; ++k) {
            issue(k + kRing - 1);
            wait_two();                                  // the rows of tick k + 1
            stage(k + 1);
            barrier();
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        return;
    }
    if (wv == NW) {
        // ================= store wave: during tick k it copies the rows of tick k - 1 (stable
        // until the barrier that ends tick k) to O, two node rows per instruction (16 B = two
        // members per lane; E is even); it never waits for its stores
        __syncthreads();                                 // table window, G of every slot
        const int half = lane >> 5;
        const unsigned m2 = (unsigned)(lane & 31) * 16u;
        const int em = (int)blockIdx.y * 64 + 2 * (lane & 31);
        const bool mok = em < E;                         // member pair inside the ensemble
        int Gl[RS / 2];
#pragma unroll
        for (int m = 0; m < RS / 2; ++m)
            Gl[m] = *reinterpret_cast<const int*>(lds + GT + 4u * (unsigned)(2 * m + half));
        const int64_t nsE = (int64_t)(rowB / 8u);        // ns * E
        auto copy_rows = [&](int k) {                    // outputs of tick k
            const unsigned buf = XB + (unsigned)(k & 1) * BUF;
#pragma unroll
            for (int m = 0; m < RS / 2; ++m) {
                const int c = 2 * m + half;
                const int t = k - Gl[m];
                if ((unsigned)t < (unsigned)T && mok) {
                    typedef double d2 __attribute__((ext_vector_type(2)));
                    const d2 v = *reinterpret_cast<const d2*>(lds + buf + (unsigned)c * kRow + m2);
                    const int64_t d = (int64_t)w * RS + c;
                    d2* dst = reinterpret_cast<d2*>(Ob + (uintptr_t)(((int64_t)t * nsE +
                                                                      d * E + em) * 8));
                    __builtin_nontemporal_store(v, dst);
                }
            }
        };
        __syncthreads();                                 // prologue of the compute waves
        for (int k = k0; k < k0 + tile; ++k) {
            if (k > k0) copy_rows(k - 1);
            __syncthreads();
        }
        copy_rows(k0 + tile - 1);
        return;
    }

    // ================= compute waves
    // table entry of step t (clamped into [0, T) and the window): the row pair (uniform) and
    // frac (a broadcast VGPR operand)
    auto tab_raw = [&](int t) -> int4 {
        int c = clamp_t(t, T);
        c = c < tw0 ? tw0 : (c > tw1 ? tw1 : c);
        return *reinterpret_cast<const int4*>(lds + TAB + 16u * (unsigned)(c - tw0));
    };
    int G[NPW], cnt[NPW];
    uint64_t up[NPW];
    unsigned vo[NPW];
    double op[NPW], ip[NPW];
    // forcing: the rows of the pair of the node's current step, fA = f[lo], fB = f[hi]
    // (cur = the pair's table word), and the next row fN = f[hi + 1].  Host-checked: from one
    // step to the next, lo and hi advance by at most one row, so a new pair is made of these.
    double fA[NPW], fB[NPW], fN[NPW];
    int cur[NPW];
    const auto so = rec(a.So, rowB), si = rec(a.Si, rowB);
    auto frow = [&](int r, unsigned off) -> double {
        r = r < 0 ? 0 : (r < nrow ? r : nrow - 1);
        return bld(rec_at(Fb + (uintptr_t)r * rowB, rowB), off);
    };
#pragma unroll
    for (int p = 0; p < NPW; ++p) {
        const int c = p * NW + wv;       // plan lane = this wave, position p
        const int64_t d = (int64_t)w * RS + c;
        const uint8_t fl = a.flags[d];
        const int Gd = a.G[d];
        const bool live = fl != kSlotPad && k0 - Gd < T && k0 + tile - Gd > 0;
        G[p] = live ? Gd : (1 << 29);
        cnt[p] = live ? (int)a.up_cnt[d] : 0;
        up[p] = a.up4[d];
        vo[p] = eo + (unsigned)d * (unsigned)E * 8u;
        if (lane < 4)
            reinterpret_cast<double*>(lds + COEF)[4 * c + lane] = a.coef[4 * d + lane];
        if (lane == 0) *reinterpret_cast<int*>(lds + GT + 4u * (unsigned)c) = G[p];
        op[p] = bld(so, vo[p]);
        ip[p] = bld(si, vo[p]);
    }
    __syncthreads();                 // the table window, G
#pragma unroll
    for (int p = 0; p < NPW; ++p) {
        cur[p] = __builtin_amdgcn_readfirstlane(tab_raw(k0 - G[p]).x);
        const int lo = cur[p] >> 1, hi = lo + (cur[p] & 1);
        fA[p] = frow(lo, vo[p]);
        fB[p] = frow(hi, vo[p]);
        fN[p] = frow(hi + 1, vo[p]);
    }
    // LDS byte offset (lane included) of input u of node p inside a parity buffer: its node
    // row, an external input's row, or the zero row (unused inputs, and a chained input -- the
    // previous position's output of the same tick, always the last input of the fold, added
    // from a register)
    unsigned va[NPW][4];
#pragma unroll
    for (int p = 0; p < NPW; ++p) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            unsigned code =
                u < cnt[p] ? (unsigned)((up[p] >> (16 * u)) & 0xffffu) : (unsigned)RS;
            if (code == kSelfCode) code = RS;
            const unsigned row = (code & kExtBit) ? (unsigned)(RS + 1) + (code & 0x7fffu) : code;
            va[p][u] = row * kRow + l8;
        }
    }
    bool chained[NPW];
#pragma unroll
    for (int p = 0; p < NPW; ++p) {
        chained[p] = false;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            chained[p] = chained[p] ||
                         (u < cnt[p] && ((up[p] >> (16 * u)) & 0xffffu) == kSelfCode);
    }

    // ---- buffer of tick k0 - 1: the outputs of that tick are the state's o; the zero rows
    const unsigned b_prev = XB + (unsigned)((k0 - 1) & 1) * BUF;
#pragma unroll
    for (int p = 0; p < NPW; ++p) lds_st(lds, b_prev + (unsigned)(p * NW + wv) * kRow + l8, op[p]);
    if (wv == 0) {
        lds_st(lds, XB + (unsigned)RS * kRow + l8, 0.0);
        lds_st(lds, XB + BUF + (unsigned)RS * kRow + l8, 0.0);
    }
    __builtin_amdgcn_s_waitcnt(0);   // nothing pending may enter the tick loop
    __syncthreads();
    const int64_t t_loop = tr ? wall_clock64() : 0;
    const int64_t c_loop = tr ? clock64() : 0;

    for (int kc = k0; kc < k0 + tile; kc += kChunk) {
        {
#pragma unroll 2
            for (int i = 0; i < kChunk; ++i) {
                const int k = kc + i;
                const unsigned brd = XB + (unsigned)((i + 1) & 1) * BUF;   // tick k - 1
                const unsigned bwr = XB + (unsigned)(i & 1) * BUF;
                // every node's inputs and table entry first, then the updates without branches,
                // so the NPW dependency chains of the tick interleave (a node that does not run
                // this tick computes a value nobody reads: its consumers do not run at k + 1)
                double v[NPW][4], fr[NPW];
                int pr[NPW];
                bool chg = false;
#pragma unroll
                for (int p = 0; p < NPW; ++p) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) v[p][u] = lds_ld(lds, brd + va[p][u]);
                    const int4 tv = tab_raw(k - G[p]);
                    pr[p] = __builtin_amdgcn_readfirstlane(tv.x);
                    fr[p] = __hiloint2double(tv.w, tv.z);
                    chg = chg || pr[p] != cur[p];
                }
                if (chg) {                  // a node's step moved to another row pair (rare)
#pragma unroll
                    for (int p = 0; p < NPW; ++p) {
                        if (pr[p] != cur[p]) {
                            const int lo = cur[p] >> 1, hi = lo + (cur[p] & 1);
                            const int lo2 = pr[p] >> 1, hi2 = lo2 + (pr[p] & 1);
                            const double a0 = fA[p], b0 = fB[p], n0 = fN[p];
                            fA[p] = lo2 == lo ? a0 : (lo2 == hi ? b0 : n0);
                            fB[p] = hi2 == hi ? b0 : (hi2 == lo ? a0 : n0);
                            if (hi2 != hi) fN[p] = frow(hi2 + 1, vo[p]);
                            cur[p] = pr[p];
                        }
                    }
                }
                double prev = 0.0;          // output of the previous position (chained input)
#pragma unroll
                for (int p = 0; p < NPW; ++p) {
                    const double q = (1.0 - fr[p]) * fA[p] + fr[p] * fB[p];
                    // unused inputs read the zero row: adding +0.0 to a sum of published values
                    // (never -0.0) is exact, so the fold over 4 terms is the reference's fold
                    double I = v[p][0];
                    I = I + v[p][1];
                    I = I + v[p][2];
                    I = I + v[p][3];
                    if (p > 0 && chained[p]) I = I + prev;
                    const double* cf =
                        reinterpret_cast<const double*>(lds + COEF) + 4 * (p * NW + wv);
                    const double o = 0.0 + (((cf[0] * I + cf[1] * ip[p]) + cf[2] * op[p]) +
                                            cf[3] * q);
                    const bool act = (unsigned)(k - G[p]) < (unsigned)T;
                    op[p] = act ? o : op[p];
                    ip[p] = act ? I : ip[p];
                    prev = o;
                    lds_st(lds, bwr + (unsigned)(p * NW + wv) * kRow + l8, o);
                }
                __syncthreads();
            }
        }
    }
    if (tr) {
        const int64_t c_end = clock64();
        int64_t* r = a.trace + kTraceWords * (int64_t)blockIdx.x;
        r[0] = t_start;
        r[1] = t_loop;
        r[2] = wall_clock64();
        r[3] = (int64_t)__smid();
        r[4] = c_loop;
        r[5] = c_end;
    }
    // state for the next launch (slots that ran in this one)
#pragma unroll
    for (int p = 0; p < NPW; ++p) {
        const bool live = G[p] != (1 << 29);
        bst<0>(rec(a.So, live ? rowB : 0u), vo[p], op[p]);
        bst<0>(rec(a.Si, live ? rowB : 0u), vo[p], ip[p]);
    }
}

// ---- layout conversions ----------------------------------------------------------------------
// one workgroup: 64 main slots x 64 members of one row r, through an LDS tile
__global__ __launch_bounds__(256) void to_sweep(const double* __restrict__ src, int64_t sstride,
                                                int64_t nsm, const int32_t* __restrict__ map,
                                                double* __restrict__ dst, int64_t nss,
                                                int64_t E) {
    __shared__ double tile[64][65];
    const int64_t d0 = (int64_t)blockIdx.x * 64, e0 = (int64_t)blockIdx.y * 64;
    const int64_t r = blockIdx.z;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int i = ty; i < 64; i += 4) {          // member e0 + i: 64 consecutive slots
        const int64_t e = e0 + i, d = d0 + tx;
        tile[i][tx] = (e < E && d < nsm) ? src[e * sstride + r * nsm + d] : 0.0;
    }
    __syncthreads();
    for (int i = ty; i < 64; i += 4) {          // slot d0 + i: 64 consecutive members
        const int64_t d = d0 + i, e = e0 + tx;
        if (d >= nsm || e >= E) continue;
        const int32_t m = map[d];
        if (m >= 0) dst[(r * nss + m) * E + e] = tile[tx][i];
    }
}

__global__ __launch_bounds__(256) void from_sweep(const double* __restrict__ src, int64_t nss,
                                                  const int32_t* __restrict__ map,
                                                  double* __restrict__ dst, int64_t nsm,
                                                  int64_t E) {
    __shared__ double tile[64][65];
    const int64_t d0 = (int64_t)blockIdx.x * 64, e0 = (int64_t)blockIdx.y * 64;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int i = ty; i < 64; i += 4) {          // slot d0 + i: its members' row
        const int64_t d = d0 + i, e = e0 + tx;
        const int32_t m = d < nsm ? map[d] : -1;
        tile[i][tx] = (m >= 0 && e < E) ? src[(int64_t)m * E + e] : 0.0;
    }
    __syncthreads();
    for (int i = ty; i < 64; i += 4) {          // member e0 + i: 64 consecutive slots
        const int64_t e = e0 + i, d = d0 + tx;
        if (d >= nsm || e >= E || map[d] < 0) continue;
        dst[e * nsm + d] = tile[tx][i];
    }
}

__global__ void sweep_coeffs(const double* __restrict__ alpha, const double* __restrict__ beta,
                             const double* __restrict__ chi, const double* __restrict__ gamma,
                             const int32_t* __restrict__ rmap, const uint8_t* __restrict__ flags,
                             double* __restrict__ coef, int64_t nss) {
    for (int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; d < nss;
         d += (int64_t)gridDim.x * blockDim.x) {
        const int32_t m = rmap[d];
        double c[4] = {0.0, 0.0, 0.0, 0.0};
        if (m >= 0) {
            c[0] = alpha[m];
            c[1] = beta[m];
            c[2] = chi[m];
            c[3] = gamma[m];
        } else if (flags[d] == kSlotSum) {
            c[0] = 1.0;
        }
        for (int k = 0; k < 4; ++k) coef[4 * d + k] = c[k];
    }
}

__global__ void sweep_zero_free(const int32_t* __restrict__ rmap, double* __restrict__ So,
                                double* __restrict__ Si, int64_t nss, int64_t E) {
    const int64_t total = nss * E;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        if (rmap[x / E] < 0) {
            So[x] = 0.0;
            Si[x] = 0.0;
        }
    }
}

inline int grid_for(int64_t work, int block) {
    int64_t g = (work + block - 1) / block;
    return (int)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

}  // namespace

hipError_t launch_member_sweep(const SweepArgs& a, int grid, int member_groups, hipStream_t s) {
    if (grid <= 0) return hipSuccess;
    hipLaunchKernelGGL((member_sweep<kSweepNPW, kSweepNW, kSweepMaxExt>),
                       dim3(grid, member_groups), dim3(64 * (kSweepNW + 2)), sweep_lds_bytes(), s,
                       a);
    return hipGetLastError();
}

hipError_t launch_to_sweep(const double* src, int64_t src_stride, int64_t nsm, int64_t R,
                           const int32_t* map, double* dst, int64_t nss, int64_t E,
                           hipStream_t s) {
    if (nsm <= 0 || E <= 0 || R <= 0) return hipSuccess;
    hipLaunchKernelGGL(to_sweep, dim3((unsigned)((nsm + 63) / 64), (unsigned)((E + 63) / 64),
                                      (unsigned)R),
                       dim3(256), 0, s, src, src_stride, nsm, map, dst, nss, E);
    return hipGetLastError();
}

hipError_t launch_from_sweep(const double* src, int64_t nss, const int32_t* map, double* dst,
                             int64_t nsm, int64_t E, hipStream_t s) {
    if (nsm <= 0 || E <= 0) return hipSuccess;
    hipLaunchKernelGGL(from_sweep, dim3((unsigned)((nsm + 63) / 64), (unsigned)((E + 63) / 64)),
                       dim3(256), 0, s, src, nss, map, dst, nsm, E);
    return hipGetLastError();
}

hipError_t launch_sweep_coeffs(const double* alpha, const double* beta, const double* chi,
                               const double* gamma, const int32_t* rmap, const uint8_t* flags,
                               double* coef, int64_t nss, hipStream_t s) {
    hipLaunchKernelGGL(sweep_coeffs, grid_for(nss, 256), 256, 0, s, alpha, beta, chi, gamma,
                       rmap, flags, coef, nss);
    return hipGetLastError();
}

hipError_t launch_sweep_zero_free(const int32_t* rmap, double* So, double* Si, int64_t nss,
                                  int64_t E, hipStream_t s) {
    hipLaunchKernelGGL(sweep_zero_free, grid_for(nss * E, 256), 256, 0, s, rmap, So, Si, nss, E);
    return hipGetLastError();
}

}  // namespace mcr
