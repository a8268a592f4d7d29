// Ensemble sweep with several members per workgroup instance (gfx950): the multi-launch
// wavefront of kernels.hip `wavefront_det`, one instance routing MB members of the same
// workgroup window together.
//
// An ensemble horizon (BASELINE configs[2] / [4], the EnKF forecast) is E independent copies of
// the deterministic recurrence over one plan.  `wavefront_det` runs them as E
// instances (grid y = member) that each repeat the per-tick work that does not depend on the
// member: the tick loop, the workgroup barrier, the activity tests, the step-table lookup and
// every LDS address.  Here one instance carries MB members: a lane's inputs of all MB members
// sit side by side in LDS (one 16-byte read for MB = 2), the lateral-inflow weights and rows
// are looked up once, and the barrier is shared; only the floating-point work is per member.
// Same operations in the same order per member, so every member is bit-identical to its serial
// run (tests/test_gpu_configs.py, tests/test_gpu_ensemble.py).
//
// LDS (bytes), RS = K * SLOTS node slots:
//   XB  [RS + 1][2][MB] f64  outputs at tick parity 0 / 1 (slot RS: the zero slot)
//   FR  [RS][3][MB]     f64  forcing rows rb .. rb + 2 of the current chunk
//   TAB [table_cap]     int4 step-table window
//   XE  [ext_cap][16][MB] f64 external inputs of two chunks (a ring: ticks k & 15), staged one
//                            chunk ahead from the step-contiguous streams XS of earlier
//                            launches (slack >= tile), so the ring is 16 ticks deep whatever the
//                            launch length -- `wavefront_det` stages the whole launch, which at
//                            MB = 2 would not leave room for two workgroups per CU.
#include "device_common.hpp"
#include "kernels.hpp"
#include "plan.hpp"

#pragma clang fp contract(off)

namespace mcr {

namespace {

using dev::chunk_rows;
using dev::clamp_row;
using dev::lds_f64;
using dev::Slot;
using dev::load_slot;
using dev::decode_codes;

constexpr int kRing = 16;          // external-input ring: two chunks of ticks

template <int MB>
struct Vec {
    double v[MB];
};

template <int MB>
__device__ __forceinline__ Vec<MB> lds_vec(const char* lds, unsigned byte) {
    Vec<MB> r;
    if constexpr (MB == 2) {
        typedef double f64x2 __attribute__((ext_vector_type(2)));
        const f64x2 x = *reinterpret_cast<const f64x2*>(lds + byte);
        r.v[0] = x.x;
        r.v[1] = x.y;
    } else {
#pragma unroll
        for (int m = 0; m < MB; ++m) r.v[m] = lds_f64(lds, byte + 8u * m);
    }
    return r;
}

template <int MB>
__device__ __forceinline__ void lds_store_vec(char* lds, unsigned byte, const double* v) {
    if constexpr (MB == 2) {
        typedef double f64x2 __attribute__((ext_vector_type(2)));
        *reinterpret_cast<f64x2*>(lds + byte) = f64x2{v[0], v[1]};
    } else {
#pragma unroll
        for (int m = 0; m < MB; ++m) *reinterpret_cast<double*>(lds + byte + 8u * m) = v[m];
    }
}

// members e0 .. e0 + MB - 1 of workgroup a.active[blockIdx.x], e0 = blockIdx.y * MB (the host
// launches this kernel only for E % MB == 0, a step table of at most 3 forcing rows per chunk
// (not DENSE) and a classic plan)
template <int SLOTS, int K, int MB>
__global__ __launch_bounds__(SLOTS)
__attribute__((amdgpu_waves_per_eu(2, 2)))
void wavefront_members(WaveArgs a) {
    extern __shared__ __attribute__((aligned(16))) char lds[];
    constexpr int RS = K * SLOTS;
    constexpr unsigned VB = 8u * MB;                    // bytes of one member vector
    constexpr unsigned XB = 0;
    constexpr unsigned FR = XB + (unsigned)(RS + 1) * 2u * VB;
    constexpr unsigned TAB = FR + (unsigned)RS * 3u * VB;
    const unsigned XE = TAB + (unsigned)a.table_cap * 16u;
    const int tile = a.tile;
    int4* tab = reinterpret_cast<int4*>(lds + TAB);

    const int tid = threadIdx.x;
    const int w = a.active[blockIdx.x];
    const int64_t e0m = (int64_t)blockIdx.y * MB;
    const int T = a.T;
    const int k0 = a.kappa0;
    const int64_t ns = a.nslots;
    const int nrow = a.n_rows;
    const int gminw = a.wg_gmin[w], gmaxw = a.wg_gmax[w];
    const int64_t wb = a.wbase[w];

    // ---- per-slot registers: shared fields once, the state per member
    Slot S[K];
    uint64_t up[K];
    double op[K][MB], ip[K][MB];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        load_slot(S[p], a, (int64_t)w * RS + p * SLOTS + tid, e0m, k0, tile, T);
        up[p] = a.up4[S[p].d];
        op[p][0] = S[p].op;
        ip[p][0] = S[p].ip;
#pragma unroll
        for (int m = 1; m < MB; ++m) {
            op[p][m] = a.st_o[(e0m + m) * a.mS + S[p].d];
            ip[p][m] = a.st_i[(e0m + m) * a.mS + S[p].d];
        }
    }

    // ---- step-table window of this workgroup -> LDS
    int tw0 = k0 - gmaxw, tw1 = k0 + tile - gminw;
    tw0 = tw0 < 0 ? 0 : (tw0 > T ? T : tw0);
    tw1 = tw1 < 0 ? 0 : (tw1 > T ? T : tw1);
    for (int idx = tid; idx < tw1 - tw0; idx += SLOTS) tab[idx] = a.stab[tw0 + idx];

    // ---- external inputs: chunk c of the launch lives in ring half c & 1 (ticks k & 15); item
    // idx = (e, tick i of the chunk, member m).  Consecutive lanes read consecutive steps of
    // one producer stream.
    const int e0 = a.ext_off[w];
    const int next = a.ext_off[w + 1] - e0;
    const int nitem = next * kChunk * MB;
    constexpr int kExtLoads = 4;                        // items per lane and chunk (bounded)
    auto ext_item = [&](int idx, int kc, unsigned& lds_off, int64_t& src) -> bool {
        lds_off = XE;
        src = -1;
        if (idx >= nitem) return false;
        const int m = idx % MB;
        const int r = idx / MB;
        const int i = r % kChunk, e = r / kChunk;
        const int k = kc + i;
        const int t = k - a.ext_g[e0 + e];
        lds_off = XE + ((unsigned)e * kRing + (unsigned)(k & (kRing - 1))) * VB + 8u * m;
        const bool ok = t >= 0 && t < T;
        src = ok ? (e0m + m) * a.mX + (int64_t)(e0 + e) * T + t : -1;
        return true;
    };
    // first chunk (the launch's tick k0): staged directly
    for (int idx = tid; idx < nitem; idx += SLOTS) {
        unsigned off;
        int64_t src;
        ext_item(idx, k0, off, src);
        *reinterpret_cast<double*>(lds + off) = src >= 0 ? a.XS[src] : 0.0;
    }
    // the consumer (one tick behind) reads step t_first - 1 at the first tick: the producer's
    // state, or for a partial sum its output of tick k0 - 1 in the previous launch's window
    double* Om = a.O;
#pragma unroll
    for (int p = 0; p < K; ++p) {
        double carry[MB];
        const bool ps = S[p].psum && (unsigned)(k0 - 1 - a.G[S[p].d]) < (unsigned)T;
#pragma unroll
        for (int m = 0; m < MB; ++m) {
            carry[m] = op[p][m];
            if (ps) carry[m] = Om[(e0m + m) * a.mO + wb + (int64_t)(k0 - 1 - gminw) * RS +
                                  p * SLOTS + tid];
        }
        lds_store_vec<MB>(lds, XB + ((unsigned)(p * SLOTS + tid) * 2u +
                                     (unsigned)((k0 - 1) & 1)) * VB, carry);
    }
    if (tid < 2 * MB)
        *reinterpret_cast<double*>(lds + XB + (unsigned)RS * 2u * VB + 8u * tid) = 0.0;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();

    // input codes -> LDS bases: a node slot's outputs (2 parities x MB members), an external
    // input's ring row (kRing ticks x MB members)
    bool any3[K];
    unsigned own[K];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        decode_codes<RS>(S[p], up[p], XB, 2u * VB, XE, (unsigned)kRing * VB);
        any3[p] = __any(S[p].cnt > 2);
        own[p] = XB + (unsigned)(p * SLOTS + tid) * 2u * VB;
    }

    // forcing rows of the first chunk, per member
    int rb[K], nr[K];
    double f[K][3][MB];
#pragma unroll
    for (int p = 0; p < K; ++p) {
        chunk_rows(tab, tw0, k0, S[p].G, T, rb[p], nr[p]);
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int m = 0; m < MB; ++m)
                f[p][r][m] = a.F[(e0m + m) * a.mF + (int64_t)clamp_row(rb[p] + r, nrow) * ns +
                                 S[p].d];
    }
    __builtin_amdgcn_s_waitcnt(0);

    const bool maskq = a.nf == nullptr ||
                       __hip_atomic_load(a.nff, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    bool anyps = false;
#pragma unroll
    for (int p = 0; p < K; ++p) anyps = anyps || S[p].psum;
    anyps = __any(anyps);
    for (int c = 0; c < tile; c += kChunk) {
        const int kc = k0 + c;
        // this chunk's forcing rows -> the slot's LDS rows (private: no barrier needed)
        unsigned frp[K], tp[K];
#pragma unroll
        for (int p = 0; p < K; ++p) {
#pragma unroll
            for (int r = 0; r < 3; ++r)
                lds_store_vec<MB>(lds, FR + ((unsigned)(p * SLOTS + tid) * 3u + r) * VB,
                                  f[p][r]);
            frp[p] = FR + (unsigned)(p * SLOTS + tid) * 3u * VB - (unsigned)rb[p] * VB;
            tp[p] = TAB + (unsigned)(kc - S[p].G - tw0) * 16u;
        }
        // prefetch: the next chunk's forcing rows (slots that run a step in it) and external
        // inputs (ring half of the next chunk, read by no one since the previous chunk's end)
        const int Tn = c + kChunk < tile ? T : 0;
        const int kn = kc + kChunk;
        int rbn[K], nrn[K];
        double g[K][3][MB];
#pragma unroll
        for (int p = 0; p < K; ++p) {
            chunk_rows(tab, tw0, kn, S[p].G, Tn, rbn[p], nrn[p]);
            const bool need = Tn > 0 && kn + kChunk > S[p].G && kn < S[p].G + T;
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int m = 0; m < MB; ++m)
                    g[p][r][m] = need ? a.F[(e0m + m) * a.mF +
                                            (int64_t)clamp_row(rbn[p] + r, nrow) * ns + S[p].d]
                                      : 0.0;
        }
        double xv[kExtLoads];
        unsigned xo[kExtLoads];
        bool xw[kExtLoads];
        int xmore = 0;                    // items beyond kExtLoads per lane: staged late
#pragma unroll
        for (int q = 0; q < kExtLoads; ++q) {
            const int idx = tid + q * SLOTS;
            int64_t src;
            xw[q] = Tn > 0 && ext_item(idx, kn, xo[q], src);
            xv[q] = xw[q] && src >= 0 ? a.XS[src] : 0.0;
        }
        if (Tn > 0 && nitem > kExtLoads * SLOTS) xmore = 1;
        unsigned m_[K][kUpInline];
#pragma unroll
        for (int p = 0; p < K; ++p)
#pragma unroll
            for (int u = 0; u < kUpInline; ++u) m_[p][u] = S[p].ubase[u];

        // ALL: every live slot of this wave runs a step at every tick of the chunk (wave-
        // uniform; most chunks of an ensemble horizon): no per-tick activity tests and no state
        // selects -- the output stores keep the slot's liveness in this launch as their mask
        auto run_chunk = [&](auto mtag, auto ptag, auto atag) {
            constexpr bool MASKQ = decltype(mtag)::value, PSUM = decltype(ptag)::value;
            constexpr bool ALL = decltype(atag)::value;
#pragma unroll
            for (int i = 0; i < kChunk; ++i) {
                const int k = kc + i;
                const unsigned rdx = (unsigned)((k - 1) & 1) * VB;            // node inputs
                const unsigned rde = (unsigned)(k & (kRing - 1)) * VB;        // ring inputs
                // lateral inflow of every member: interpolate_sample (nutils.py:23-33), one
                // table lookup for all members
                double qv[K][MB];
#pragma unroll
                for (int p = 0; p < K; ++p) {
                    const int4 e = *reinterpret_cast<const int4*>(lds + tp[p] + 16u * i);
                    const Vec<MB> lo = lds_vec<MB>(lds, frp[p] + VB * (unsigned)e.x);
                    Vec<MB> hi = lds_vec<MB>(lds, frp[p] + VB * (unsigned)e.y);
                    const double fr = __hiloint2double(e.w, e.z);
#pragma unroll
                    for (int m = 0; m < MB; ++m) {
                        double h = hi.v[m];
                        if constexpr (MASKQ) h = fr == 0.0 ? 0.0 : h;
                        qv[p][m] = (1.0 - fr) * lo.v[m] + fr * h;
                    }
                }
                // inputs of all positions before any output is written (kernels.hip)
                Vec<MB> vin[K][kUpInline];
#pragma unroll
                for (int p = 0; p < K; ++p) {
#pragma unroll
                    for (int u = 0; u < kUpInline; ++u) {
                        if (u >= 2 && !any3[p]) {
#pragma unroll
                            for (int m = 0; m < MB; ++m) vin[p][u].v[m] = 0.0;
                            continue;
                        }
                        vin[p][u] = lds_vec<MB>(lds, m_[p][u] + (S[p].uext[u] ? rde : rdx));
                    }
                }
                double ov[K][MB];
                bool act[K];
                double prev[MB];
#pragma unroll
                for (int m = 0; m < MB; ++m) prev[m] = 0.0;
#pragma unroll
                for (int p = 0; p < K; ++p) {
                    act[p] = ALL ? S[p].G != (1 << 29) : (unsigned)(k - S[p].G) < (unsigned)T;
                    bool upd = act[p];
                    if constexpr (PSUM) upd = upd && !S[p].psum;
#pragma unroll
                    for (int m = 0; m < MB; ++m) {
                        // the reference's left fold (device_common.hpp fold_values)
                        double I = vin[p][0].v[m];
                        I = I + vin[p][1].v[m];
                        if (any3[p]) {
                            I = I + vin[p][2].v[m];
                            I = I + vin[p][3].v[m];
                        }
                        if (p > 0) I = I + (S[p].chained ? prev[m] : 0.0);
                        const double o = dev::muskingum_update(
                            S[p].al, I, S[p].be, ip[p][m], S[p].ch, op[p][m],
                            dev::gq_term(S[p].ga, qv[p][m]));
                        if constexpr (ALL && !PSUM) {
                            op[p][m] = o;        // (a slot that is not live is not written back)
                            ip[p][m] = I;
                        } else {
                            op[p][m] = upd ? o : op[p][m];
                            ip[p][m] = upd ? I : ip[p][m];
                        }
                        ov[p][m] = o;
                        prev[m] = o;
                    }
                }
#pragma unroll
                for (int p = 0; p < K; ++p)
                    lds_store_vec<MB>(lds, own[p] + (unsigned)(k & 1) * VB, ov[p]);
                // active cells of row k - gmin of every member's window, and the external
                // streams this slot feeds
#pragma unroll
                for (int p = 0; p < K; ++p) {
                    if (act[p]) {
#pragma unroll
                        for (int m = 0; m < MB; ++m) {
                            __builtin_nontemporal_store(
                                ov[p][m], Om + (e0m + m) * a.mO + wb +
                                              (int64_t)(k - gminw) * RS + p * SLOTS + tid);
                            if (S[p].xsrc) a.XS[(e0m + m) * a.mX + S[p].xs0 + k] = ov[p][m];
                        }
                    }
                }
                if (i == 3) {
                    // the next chunk's external inputs -> their ring half (its last readers
                    // finished before the previous chunk's final barrier)
#pragma unroll
                    for (int q = 0; q < kExtLoads; ++q)
                        if (xw[q]) *reinterpret_cast<double*>(lds + xo[q]) = xv[q];
                    if (xmore) {
                        for (int idx = tid + kExtLoads * SLOTS; idx < nitem; idx += SLOTS) {
                            unsigned off;
                            int64_t src;
                            ext_item(idx, kn, off, src);
                            *reinterpret_cast<double*>(lds + off) = src >= 0 ? a.XS[src] : 0.0;
                        }
                    }
                }
                __syncthreads();
            }
        };
        using yes = std::true_type;
        using no = std::false_type;
        bool all = true;
#pragma unroll
        for (int p = 0; p < K; ++p)
            all = all && (S[p].G == (1 << 29) ||
                          (unsigned)(kc - S[p].G) <= (unsigned)(T - kChunk));
        all = T >= kChunk && __all(all);
        if (__builtin_expect(!maskq && !anyps, 1)) [[likely]] {
            if (all) run_chunk(no{}, no{}, yes{});
            else run_chunk(no{}, no{}, no{});
        } else if (maskq) {
            if (anyps) run_chunk(yes{}, yes{}, no{});
            else run_chunk(yes{}, no{}, no{});
        } else {
            run_chunk(no{}, yes{}, no{});
        }
#pragma unroll
        for (int p = 0; p < K; ++p) {
            rb[p] = rbn[p];
            nr[p] = nrn[p];
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int m = 0; m < MB; ++m) f[p][r][m] = g[p][r][m];
        }
    }
    // state for the next launch (live slots only; never-processed reaches hold o = 0)
    bool nonfin = false;
#pragma unroll
    for (int p = 0; p < K; ++p) {
        if (S[p].G != (1 << 29)) {
#pragma unroll
            for (int m = 0; m < MB; ++m) {
                const double so = S[p].unr ? 0.0 : op[p][m];
                a.st_o[(e0m + m) * a.mS + S[p].d] = so;
                a.st_i[(e0m + m) * a.mS + S[p].d] = ip[p][m];
                nonfin = nonfin || !__builtin_isfinite(so) || !__builtin_isfinite(ip[p][m]);
            }
        }
    }
    if (a.nf && __any(nonfin) && (tid & 63) == 0)
        __hip_atomic_store(a.nf, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

size_t members_lds_bytes(int slots, int chain, int table_cap, int ext_cap, int mb) {
    const size_t rs = (size_t)chain * slots, vb = 8 * (size_t)mb;
    return (rs + 1) * 2 * vb + rs * 3 * vb + 16 * (size_t)table_cap +
           (size_t)ext_cap * kRing * vb;
}

bool members_shape_ok(int slots, int chain, int mb) {
    return mb == 2 && chain == 2 && (slots == 256 || slots == 192 || slots == 128);
}

hipError_t launch_members(const WaveArgs& a, int grid, int slots, int chain, size_t lds,
                          int members, int mb, hipStream_t s) {
    if (!members_shape_ok(slots, chain, mb) || members % mb) return hipErrorInvalidValue;
    const dim3 g(grid, members / mb);
#define MCR_CASE(S)                                                                      \
    if (slots == S) {                                                                    \
        hipLaunchKernelGGL((wavefront_members<S, 2, 2>), g, S, lds, s, a);               \
        return hipGetLastError();                                                        \
    }
    MCR_CASE(256)
    MCR_CASE(192)
    MCR_CASE(128)
#undef MCR_CASE
    return hipErrorInvalidValue;
}

}  // namespace mcr
