// One model step of E ensemble members swept along flow paths, members on the lanes (paths.hpp
// has the decomposition).  Replaces, for the one-step runs of the EnKF cycle (da.py:91-136 per
// member; nutils.py:64-89 per step), the member-dataflow launch whose critical path is the tick
// schedule's fill: here a wave walks a heavy path node after node, so the step's critical path is
// the longest heavy path at the latency of the update itself.
//
// Two launches per step:
//   * path_prep: per (node, member) the three inflow-independent terms beta i', chi o', gamma q of
//     0 + (((alpha I + beta i') + chi o') + gamma q)  (nutils.py:80-83; o', i' the state with the
//     pending analysis increments applied, q the interpolated lateral inflow, nutils.py:23-33),
//     read from the member-major session arrays in slot blocks (whole lines) and written in
//     sequence order, members innermost (one 512-B row per term and node);
//   * member_paths: a persistent grid of one-wave workgroups taking (task, member group)
//     tickets; per node: the inflow fold I in rank order from the chain register, the previous
//     node's register, the LDS ring of this task's earlier outputs or another task's granule,
//     then o = 0 + (((alpha I + c1) + c2) + c3), written in place to the session state.
// Arithmetic is the reference's: the same products, the same association and fold order as the
// wavefront kernels (FMA contraction off), so every member is bit-identical to its serial run.
#include "paths.hpp"
#include "device_common.hpp"
#include "kernels.hpp"

#pragma clang fp contract(off)

namespace mcr {

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kPrepSlots = 64;      // slots per prep block (one wave-wide run per member row)
constexpr int kPrepMembers = 32;    // members staged in LDS per pass of a prep block

// P[(g * n + s) * 192 + k * 64 + lane]
__global__ __launch_bounds__(256) void path_prep(
        const double* __restrict__ F, int64_t mF, int n_rows, int4 ent,
        const double* __restrict__ st_o, const double* __restrict__ st_i,
        const double* __restrict__ beta, const double* __restrict__ chi,
        const double* __restrict__ gamma, const uint8_t* __restrict__ flags,
        const int32_t* __restrict__ seq_of_slot, const double* __restrict__ G,
        const int32_t* __restrict__ up_off, const int32_t* __restrict__ up,
        double* __restrict__ P, int64_t ns, int64_t n, int64_t E) {
    __shared__ double T[kPrepSlots][3][kPrepMembers];
    __shared__ int32_t sq[kPrepSlots];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t d0 = (int64_t)blockIdx.x * kPrepSlots;
    const int64_t d = d0 + lane;
    const bool real = d < ns && seq_of_slot[d] >= 0;     // a reach (not padding / partial sum)
    if (threadIdx.x < kPrepSlots) sq[threadIdx.x] = d0 + threadIdx.x < ns ? seq_of_slot[d0 + threadIdx.x] : -1;
    const uint8_t fl = real ? flags[d] : (uint8_t)kSlotPad;
    const double b = real ? beta[d] : 0.0, c = real ? chi[d] : 0.0, gm = real ? gamma[d] : 0.0;
    const double f = __hiloint2double(ent.w, ent.z);
    const int64_t rlo = (int64_t)dev::clamp_row(ent.x, n_rows) * ns + d;
    const int64_t rhi = (int64_t)dev::clamp_row(ent.y < 0 ? ent.x : ent.y, n_rows) * ns + d;
    const bool gained = G != nullptr && (fl == kSlotRouted || fl == kSlotUnrouted);
    const int32_t u0 = G != nullptr && real ? up_off[d] : 0;
    const int32_t u1 = G != nullptr && real ? up_off[d + 1] : 0;
    const int64_t gbase = (int64_t)blockIdx.y * kPathLanes;     // member group
    for (int h = 0; h < kPathLanes; h += kPrepMembers) {
        const int64_t eb = gbase + h;
        if (eb >= E) break;
        __syncthreads();                                 // T free (previous pass written out)
        for (int m = wv; m < kPrepMembers; m += 4) {
            const int64_t e = eb + m;
            if (!real || e >= E) continue;
            const int64_t idx = e * ns + d;
            const double* Fe = F + e * mF;
            const double lo = Fe[rlo];
            const double hi = Fe[rhi];
            double o = st_o[idx], i = st_i[idx];
            if (gained) {                                // apply_gain's operations, in order
                const double* Ge = G + e * ns;
                const double og = fl == kSlotRouted ? 0.0 + Ge[d] : 0.0;
                double ig = 0.0;
                for (int32_t q = u0; q < u1; ++q) ig = ig + (0.0 + Ge[up[q]]);
                o = o + og;
                i = i + ig;
            }
            const double q = ent.x == ent.y ? lo : (1.0 - f) * lo + f * hi;   // clamped: row copy
            T[lane][0][m] = b * i;
            T[lane][1][m] = c * o;
            T[lane][2][m] = gm * q;
        }
        __syncthreads();
        // write out: per slot of the block, its three 32-member row segments (256 B each)
        const int mcount = (int)(E - eb < kPrepMembers ? E - eb : kPrepMembers);
        for (int x = threadIdx.x; x < kPrepSlots * 3 * kPrepMembers; x += 256) {
            const int m = x & (kPrepMembers - 1);
            const int k = (x / kPrepMembers) % 3;
            const int sl = x / (3 * kPrepMembers);
            const int32_t s = sq[sl];
            if (s < 0 || m >= mcount) continue;
            P[((int64_t)blockIdx.y * n + s) * 192 + k * 64 + h + m] = T[sl][k][m];
        }
    }
}

__global__ void path_alpha(int32_t* __restrict__ rec, const double* __restrict__ alpha,
                           int64_t n) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= n) return;
    int32_t* r = rec + s * kPathRecWords;
    const double a = alpha[r[1]];
    r[2] = __double2loint(a);
    r[3] = __double2hiint(a);
}

constexpr int kPathPrefetch = 8;    // nodes whose P rows are in flight ahead of the current one
constexpr int kPathChunk = 64;      // node records staged per LDS chunk (one per lane)
constexpr int kSleepUnit = 32;

__global__ __launch_bounds__(64) void member_paths(PathArgs a) {
    __shared__ double ring[kPathRing][kPathLanes];
    __shared__ int4 recs[2][kPathChunk][kPathRecWords / 4];
    const int lane = threadIdx.x;
    const auto gr = __builtin_amdgcn_make_buffer_rsrc(a.GR, (short)0, (int)a.gr_bytes, 0x00020000);
    const uint32_t epoch = a.epoch;
    const int32_t groups = a.groups;
    const int64_t nticket = (int64_t)a.n_tasks * groups;
    bool dead = false;
    for (;;) {
        int tk = 0;
        if (lane == 0) tk = __hip_atomic_fetch_add(a.queue, 1, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
        tk = __shfl(tk, 0);
        if ((int64_t)tk >= nticket) break;
        const int32_t task = tk / groups, g = tk - task * groups;
        const int64_t e = (int64_t)g * kPathLanes + lane;
        const bool act = e < a.E;
        const int64_t s0 = a.task_off[task], s1 = a.task_off[task + 1];
        const double* __restrict__ Pg = a.P + (int64_t)g * a.n * 192 + lane;
        // records: lane l holds the record of node cbase + l of the NEXT chunk in registers
        auto load_rec = [&](int64_t cbase, int4 (&r)[4]) {
            int64_t s = cbase + lane;
            s = s < s1 ? s : s1 - 1;
            const int4* src = reinterpret_cast<const int4*>(a.rec + s * kPathRecWords);
#pragma unroll
            for (int q = 0; q < 4; ++q) r[q] = src[q];
        };
        int4 rn[4];
        load_rec(s0, rn);
#pragma unroll
        for (int q = 0; q < 4; ++q) recs[0][lane][q] = rn[q];
        if (s0 + kPathChunk < s1) load_rec(s0 + kPathChunk, rn);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // P rows of the next kPathPrefetch nodes
        double pa[kPathPrefetch], pb[kPathPrefetch], pc[kPathPrefetch];
#pragma unroll
        for (int j = 0; j < kPathPrefetch; ++j) {
            const int64_t s = s0 + j < s1 ? s0 + j : s1 - 1;
            pa[j] = Pg[s * 192];
            pb[j] = Pg[s * 192 + 64];
            pc[j] = Pg[s * 192 + 128];
        }
        double prevv = 0.0, chainv = 0.0;
        for (int64_t base = s0; base < s1; base += kPathPrefetch) {
#pragma unroll
            for (int j = 0; j < kPathPrefetch; ++j) {
                const int64_t s = base + j;
                if (s >= s1) break;
                const int64_t rel = s - s0;
                if (rel > 0 && (rel & (kPathChunk - 1)) == 0) {
                    // next record chunk: the registers loaded one chunk ago -> LDS, then the
                    // chunk after it into the registers
                    const int buf = (int)((rel / kPathChunk) & 1);
#pragma unroll
                    for (int q = 0; q < 4; ++q) recs[buf][lane][q] = rn[q];
                    if (s + kPathChunk < s1) load_rec(s + kPathChunk, rn);
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                }
                const double c1 = pa[j], c2 = pb[j], c3 = pc[j];
                {
                    const int64_t sn = s + kPathPrefetch < s1 ? s + kPathPrefetch : s1 - 1;
                    pa[j] = Pg[sn * 192];
                    pb[j] = Pg[sn * 192 + 64];
                    pc[j] = Pg[sn * 192 + 128];
                }
                const int4* R = recs[(rel / kPathChunk) & 1][rel & (kPathChunk - 1)];
                const int4 r0 = R[0];
                const uint32_t meta = (uint32_t)__builtin_amdgcn_readfirstlane(r0.x);
                const int64_t d = __builtin_amdgcn_readfirstlane(r0.y);
                const double alpha = __hiloint2double(__builtin_amdgcn_readfirstlane(r0.w),
                                                      __builtin_amdgcn_readfirstlane(r0.z));
                const int n_in = (int)(meta & 0xffffu);
                double I = 0.0;
                for (int q = 0; q < n_in; ++q) {
                    uint32_t code;
                    if (q < kPathInline) {
                        const int4 w = R[1 + q / 4];
                        const int c = (q & 3) == 0 ? w.x : (q & 3) == 1 ? w.y : (q & 3) == 2 ? w.z : w.w;
                        code = (uint32_t)__builtin_amdgcn_readfirstlane(c);
                    } else {
                        const int4 w = R[3];
                        const int32_t off = __builtin_amdgcn_readfirstlane(w.x);
                        code = (uint32_t)__builtin_amdgcn_readfirstlane(a.ovf[off + q - kPathInline]);
                    }
                    const uint32_t kind = code & ~kInPayload, pay = code & kInPayload;
                    double v;
                    if (kind == kInChain) {
                        v = chainv;
                    } else if (kind == kInPrev) {
                        v = prevv;
                    } else if (kind == kInLocal) {
                        v = ring[pay & (kPathRing - 1)][lane];
                    } else {
                        // another task's bottom node: its granule {lo, epoch, hi, epoch}
                        const unsigned off =
                            (unsigned)(((int64_t)pay * groups + g) * kPathLanes + lane) * 16u;
                        u32x4 gv = __builtin_amdgcn_raw_buffer_load_b128(gr, off, 0, 16);
                        if (!__all(gv.y == epoch && gv.w == epoch) && !dead) {
                            const int64_t t0 = wall_clock64();
                            int sl = 1;
                            for (;;) {
                                for (int r = 0; r < sl; ++r) __builtin_amdgcn_s_sleep(kSleepUnit);
                                sl = sl < 16 ? sl * 2 : 16;
                                gv = __builtin_amdgcn_raw_buffer_load_b128(gr, off, 0, 16);
                                if (__all(gv.y == epoch && gv.w == epoch)) break;
                                if (wall_clock64() - t0 > a.patience ||
                                    __hip_atomic_load(a.status, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT) != 0) {
                                    if (lane == 0)
                                        __hip_atomic_store(a.status, 1, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
                                    dead = true;
                                    break;
                                }
                            }
                        }
                        v = __longlong_as_double((long long)(((uint64_t)gv.z << 32) | gv.x));
                    }
                    // reference fold ((0 + v1) + v2) + ...: every published value is 0 + (...),
                    // never -0, so 0 + v1 is v1 exactly
                    I = q == 0 ? v : I + v;
                }
                const bool routed = (meta & kRecRouted) != 0;
                double o = 0.0 + (((alpha * I + c1) + c2) + c3);
                o = routed ? o : 0.0;              // never-processed reaches keep o = 0
                if (act) {
                    a.st_o[e * a.ns + d] = o;
                    a.st_i[e * a.ns + d] = I;
                }
                prevv = o;
                if (meta & kRecChain) chainv = o;
                if (meta & kRecKeep) ring[s & (kPathRing - 1)][lane] = o;
                if (meta & kRecPublish) {
                    const uint64_t bits = (uint64_t)__double_as_longlong(o);
                    const u32x4 gv = {(unsigned)bits, epoch, (unsigned)(bits >> 32), epoch};
                    const unsigned off =
                        (unsigned)(((int64_t)task * groups + g) * kPathLanes + lane) * 16u;
                    __builtin_amdgcn_raw_buffer_store_b128(gv, gr, off, 0, 16);
                }
            }
        }
        // LDS ring / record buffers are reused by the next ticket's task: its own writes come
        // after these in program order (one wave), so no barrier is needed
    }
}

}  // namespace

hipError_t launch_path_prep(const double* F, int64_t mF, int n_rows, int4 ent, const double* st_o,
                            const double* st_i, const double* beta, const double* chi,
                            const double* gamma, const uint8_t* flags, const int32_t* seq_of_slot,
                            const double* G, const int32_t* up_off, const int32_t* up, double* P,
                            int64_t ns, int64_t n, int64_t E, hipStream_t s) {
    if (ns <= 0 || E <= 0) return hipSuccess;
    const dim3 grid((unsigned)((ns + kPrepSlots - 1) / kPrepSlots),
                    (unsigned)((E + kPathLanes - 1) / kPathLanes));
    hipLaunchKernelGGL(path_prep, grid, 256, 0, s, F, mF, n_rows, ent, st_o, st_i, beta, chi,
                       gamma, flags, seq_of_slot, G, up_off, up, P, ns, n, E);
    return hipGetLastError();
}

hipError_t launch_path_alpha(int32_t* rec, const double* alpha, int64_t n, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(path_alpha, dim3((unsigned)((n + 255) / 256)), 256, 0, s, rec, alpha, n);
    return hipGetLastError();
}

hipError_t launch_member_paths(const PathArgs& a, int grid, hipStream_t s) {
    if (a.n <= 0 || a.n_tasks <= 0) return hipSuccess;
    hipLaunchKernelGGL(member_paths, dim3((unsigned)grid), kPathLanes, 0, s, a);
    return hipGetLastError();
}

}  // namespace mcr
