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

constexpr int kStage = 32;          // staged nodes (LDS ring slots)
constexpr int kLag = 12;            // nodes the loader keeps in flight before publishing one
constexpr int kSlotBytes = 1600;    // one staged node: P (3 x 64 doubles) + its record (64 B)
constexpr int kTickLog = 64;        // tickets a loader announced, ring (> kStage + 1)
constexpr int kSleepUnit = 2;

// wait until at most N vector-memory operations of this wave are outstanding (in order)
template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

struct PathsLds {
    char stage[kStage * kSlotBytes];                   // 50 KB: P rows + record per slot
    int4 tlog[kTickLog];                                // per ticket: task, group, s0, s1
    double ring[kPathRing][kPathLanes];                 // 16 KB: outputs local inputs read
    int ready;                                          // stream entries [0, ready) are staged
    int consumed;                                       // slots of entries [0, consumed) are free
    int done;                                           // the loader took its last ticket
};

__device__ __forceinline__ int lds_ld(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(int* p, int v) {
    // LDS operations of one wave are performed in order, so everything this wave read from the
    // slot before is done when the loader sees this value; the compiler must not move LDS
    // accesses across it
    asm volatile("" ::: "memory");
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The loader wave's own LDS accesses, as inline asm: the compiler's waitcnt pass cannot tell an
// LDS-DMA target from any other LDS address, so it would drain every DMA in flight (vmcnt(0))
// before a plain LDS access of the loader -- the whole pipeline.  These wait for themselves.
typedef int v4i __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)const_cast<void*>(p);
}
__device__ __forceinline__ int lds_ld_asm(const int* p) {
    int v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
    return v;
}
__device__ __forceinline__ void lds_st_asm(int* p, int v) {
    asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
__device__ __forceinline__ void lds_st4_asm(void* p, v4i v) {
    asm volatile("ds_write_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(lds_addr(p)), "v"(v) : "memory");
}

// one staged node in the compute wave's registers: its three P terms and record words 0..7
// (meta, slot, alpha, the first four input codes); words 8..12 are read from the slot when a
// node has more than four inputs
struct Staged {
    double c1, c2, c3;
    int4 r0, r1;
};

// One workgroup = a compute wave + a loader wave.  The loader takes the tickets, announces each
// in the ticket log, and streams the nodes' P rows and records into the LDS ring by LDS-DMA
// (global_load_lds: no registers, kLag nodes in flight, explicit in-order waits), then publishes
// `ready`.  The compute wave walks the stream in order -- within a ticket the sequence numbers
// are consecutive, at a ticket boundary it reads the log -- and reads node k + 1's slot while
// node k computes, so neither global nor LDS latency is on the node chain: per node a few scalar
// decisions (two readfirstlanes: the meta word and the first input code), the update's own f64
// operations and the stores.  (A single wave that issued the LDS-DMA itself got a vmcnt(0)
// before every LDS read: the compiler cannot tell the DMA target from the slot being read.)
__global__ __launch_bounds__(2 * kPathLanes) void member_paths(PathArgs a) {
    __shared__ __attribute__((aligned(16))) PathsLds L;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int32_t groups = a.groups;
    const int64_t nticket = (int64_t)a.n_tasks * groups;
    if (threadIdx.x == 0) {
        L.ready = 0;
        L.consumed = 0;
        L.done = 0;
    }
    __syncthreads();
    if (wave == 1) {
        // ================================ loader wave ================================
        int k = 0, published = 0, j = 0;
        for (;;) {
            int tk = 0;
            if (lane == 0) tk = __hip_atomic_fetch_add(a.queue, 1, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
            tk = __shfl(tk, 0);                          // (waits for every load: drains)
            if ((int64_t)tk >= nticket) break;
            const int32_t task = tk / groups, g = tk - task * groups;
            const int32_t s0 = a.task_off[task], s1 = a.task_off[task + 1];
            const char* Pg = reinterpret_cast<const char*>(a.P + (int64_t)g * a.n * 192);
            // the ticket log entry is written before any of the ticket's nodes is published
            if (lane == 0) lds_st4_asm(&L.tlog[j & (kTickLog - 1)], v4i{task, g, s0, s1});
            ++j;
            published = k;                               // the drain above landed them all
            lds_st_asm(&L.ready, k);
            for (int32_t s = s0; s < s1; ++s) {
                int sl = 1;
                while (k - lds_ld_asm(&L.consumed) >= kStage) {
                    for (int r = 0; r < sl; ++r) __builtin_amdgcn_s_sleep(1);
                    sl = sl < 8 ? sl * 2 : 8;
                }
                char* dst = L.stage + (k & (kStage - 1)) * kSlotBytes;
                const char* p = Pg + (int64_t)s * 1536;
                __builtin_amdgcn_global_load_lds(p + lane * 16,
                                                 (__attribute__((address_space(3))) void*)dst, 16,
                                                 0, 0);
                const char* src2 = lane < 32 ? p + 1024 + lane * 16
                                             : reinterpret_cast<const char*>(a.rec + (int64_t)s * kPathRecWords) +
                                                   (lane & 3) * 16;
                if (lane < 36)
                    __builtin_amdgcn_global_load_lds(
                        src2, (__attribute__((address_space(3))) void*)(dst + 1024), 16, 0, 0);
                ++k;
                if (k - published > kLag) {
                    wait_vm<2 * kLag>();                 // all but the kLag newest have landed
                    published = k - kLag;
                    lds_st_asm(&L.ready, published);
                }
            }
        }
        wait_vm<0>();
        lds_st_asm(&L.ready, k);
        lds_st_asm(&L.done, 1);
        return;
    }
    // ================================ compute wave ================================
    const auto gr = __builtin_amdgcn_make_buffer_rsrc(a.GR, (short)0, (int)a.gr_bytes, 0x00020000);
    const uint32_t epoch = a.epoch;
    bool dead = false;
    double prevv = 0.0, chainv = 0.0;
    int rdy = 0;                                         // cached `ready` (wave-uniform)
    // is entry k staged?  Blocks until it is, or the stream ended (false)
    auto await = [&](int k) -> bool {
        int sl = 1;
        while (rdy <= k) {
            rdy = __builtin_amdgcn_readfirstlane(lds_ld(&L.ready));
            if (rdy > k) break;
            if (lds_ld(&L.done)) {
                rdy = __builtin_amdgcn_readfirstlane(lds_ld(&L.ready));
                return rdy > k;
            }
            for (int r = 0; r < sl; ++r) __builtin_amdgcn_s_sleep(1);
            sl = sl < 4 ? sl * 2 : 4;
        }
        return true;
    };
    auto read = [&](int k, Staged& x) {
        const char* b = L.stage + (k & (kStage - 1)) * kSlotBytes;
        x.c1 = reinterpret_cast<const double*>(b)[lane];
        x.c2 = reinterpret_cast<const double*>(b + 512)[lane];
        x.c3 = reinterpret_cast<const double*>(b + 1024)[lane];
        x.r0 = reinterpret_cast<const int4*>(b + 1536)[0];
        x.r1 = reinterpret_cast<const int4*>(b + 1536)[1];
    };
    // another task's bottom node: its granule {lo, epoch, hi, epoch}, polled until tagged
    auto granule = [&](uint32_t t, int32_t g) -> double {
        const unsigned off = (unsigned)(((int64_t)t * groups + g) * kPathLanes + lane) * 16u;
        u32x4 gv = __builtin_amdgcn_raw_buffer_load_b128(gr, off, 0, 16);
        if (!__all(gv.y == epoch && gv.w == epoch) && !dead) {
            const int64_t t0 = wall_clock64();
            int sw = 1;
            for (;;) {
                for (int r = 0; r < sw; ++r) __builtin_amdgcn_s_sleep(kSleepUnit);
                sw = sw < 4 ? sw * 2 : 4;
                gv = __builtin_amdgcn_raw_buffer_load_b128(gr, off, 0, 16);
                if (__all(gv.y == epoch && gv.w == epoch)) break;
                if (wall_clock64() - t0 > a.patience ||
                    __hip_atomic_load(a.status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
                    if (lane == 0)
                        __hip_atomic_store(a.status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    dead = true;
                    break;
                }
            }
        }
        return __longlong_as_double((long long)(((uint64_t)gv.z << 32) | gv.x));
    };
    if (!await(0)) return;
    // stream position: entry k is node s of ticket (task, g), whose sequence ends at s1
    int j = 0;
    int4 tl = L.tlog[0];
    int32_t task = __builtin_amdgcn_readfirstlane(tl.x), g = __builtin_amdgcn_readfirstlane(tl.y),
            s = __builtin_amdgcn_readfirstlane(tl.z), s1 = __builtin_amdgcn_readfirstlane(tl.w);
    Staged A, B;
    read(0, A);
    // a real waitcnt instruction (the compiler's waitcnt pass sees it): with node 0's reads done
    // before the loop, a node's own prefetch is the only LDS read in flight at its top
    __builtin_amdgcn_s_waitcnt(0xc07f);                 // lgkmcnt(0)
    int k = 0;
    // node k from `cur`; prefetches node k + 1 into `nxt`; false when the stream has ended
    auto node = [&](const Staged& cur, Staged& nxt) -> bool {
        // node k - 1 is done with its slot (node k reads record words 8..12 from its own slot
        // when it has more than four inputs): free it, and fetch node k + 1's while k computes
        lds_st(&L.consumed, k);
        const bool boundary = s + 1 >= s1;
        bool more = rdy > k + 1;
        if (!more) {
            rdy = __builtin_amdgcn_readfirstlane(lds_ld(&L.ready));
            more = rdy > k + 1;
        }
        if (more) read(k + 1, nxt);
        const uint32_t meta = (uint32_t)__builtin_amdgcn_readfirstlane(cur.r0.x);
        const int n_in = (int)(meta & 0xffffu);
        const double alpha = __hiloint2double(cur.r0.w, cur.r0.z);
        // the inflow fold in the reference's order ((0 + v1) + v2) + ...: every published value
        // is 0 + (...), never -0, so 0 + v1 is v1 exactly
        double I = 0.0;
        if (n_in > 0) {
            auto value = [&](uint32_t code) -> double {
                if (code < (uint32_t)kInLocal) return code < (uint32_t)kInPrev ? chainv : prevv;
                const uint32_t pay = code & kInPayload;
                if (code < (uint32_t)kInExt) return L.ring[pay & (kPathRing - 1)][lane];
                return granule(pay, g);
            };
            I = value((uint32_t)__builtin_amdgcn_readfirstlane(cur.r1.x));
            if (n_in > 1) {
                I = I + value((uint32_t)__builtin_amdgcn_readfirstlane(cur.r1.y));
                if (n_in > 2) {
                    I = I + value((uint32_t)__builtin_amdgcn_readfirstlane(cur.r1.z));
                    if (n_in > 3) {
                        I = I + value((uint32_t)__builtin_amdgcn_readfirstlane(cur.r1.w));
                        // the rest: record words 8..11 from the slot (still staged: `consumed`
                        // is k), then overflow
                        const int32_t* rw = reinterpret_cast<const int32_t*>(
                            L.stage + (k & (kStage - 1)) * kSlotBytes + 1536);
                        const int32_t ovf_off = __builtin_amdgcn_readfirstlane(rw[12]);
                        for (int q = 4; q < n_in; ++q) {
                            int32_t code;
                            if (q < kPathInline)
                                code = rw[4 + q];
                            else
                                code = a.ovf[ovf_off + q - kPathInline];
                            I = I + value((uint32_t)__builtin_amdgcn_readfirstlane(code));
                        }
                    }
                }
            }
        }
        double o = 0.0 + (((alpha * I + cur.c1) + cur.c2) + cur.c3);
        o = (meta & kRecRouted) ? o : 0.0;             // never-processed reaches keep o = 0
        const int64_t e = (int64_t)g * kPathLanes + lane;
        if (e < a.E) {
            const int64_t at = e * a.ns + cur.r0.y;
            a.st_o[at] = o;
            a.st_i[at] = I;
        }
        prevv = o;
        chainv = (meta & kRecChain) ? o : chainv;
        if (meta & kRecKeep) L.ring[s & (kPathRing - 1)][lane] = o;
        if (meta & kRecPublish) {
            const uint64_t bits = (uint64_t)__double_as_longlong(o);
            const u32x4 gv = {(unsigned)bits, epoch, (unsigned)(bits >> 32), epoch};
            const unsigned off = (unsigned)(((int64_t)task * groups + g) * kPathLanes + lane) * 16u;
            __builtin_amdgcn_raw_buffer_store_b128(gv, gr, off, 0, 16);
        }
        if (!more) {
            if (!await(k + 1)) return false;
            read(k + 1, nxt);
            // complete here, so the next node's first use of it waits for nothing newer
            __builtin_amdgcn_s_waitcnt(0xc07f);         // lgkmcnt(0)
        }
        ++k;
        if (boundary) {                                  // the next ticket (logged before k)
            ++j;
            tl = L.tlog[j & (kTickLog - 1)];
            task = __builtin_amdgcn_readfirstlane(tl.x);
            g = __builtin_amdgcn_readfirstlane(tl.y);
            s = __builtin_amdgcn_readfirstlane(tl.z);
            s1 = __builtin_amdgcn_readfirstlane(tl.w);
        } else {
            ++s;
        }
        return true;
    };
    for (;;) {
        if (!node(A, B)) break;
        if (!node(B, A)) break;
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
    hipLaunchKernelGGL(member_paths, dim3((unsigned)grid), 2 * kPathLanes, 0, s, a);
    return hipGetLastError();
}

}  // namespace mcr
