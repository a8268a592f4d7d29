// C ABI of the routing engine (include/mcroute.h): sessions, device buffers, launch sequencing.
#include "mcroute.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <new>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "analysis.hpp"
#include "capi_common.hpp"
#include "digest.hpp"
#include "kernels.hpp"
#include "plan.hpp"

#pragma clang fp contract(off)

namespace {

using namespace mcr::capi;

mcr::PlanParams to_params(const mc_plan_params* pp) {
    mcr::PlanParams p;
    if (pp) {
        if (pp->slots) p.slots = pp->slots;
        if (pp->tile) p.tile = pp->tile;
        if (pp->ext_cap) p.ext_cap = pp->ext_cap;
        if (pp->chain) p.chain = pp->chain;
        p.sync = pp->sync;
    }
    return p;
}

void fill_info(const mcr::Plan& P, mc_plan_info* info) {
    info->n = P.n;
    info->n_routed = P.n_routed;
    info->n_clusters = P.n_clusters;
    info->n_cross = P.n_cross;
    info->nslots = P.nslots;
    info->nwg = P.nwg;
    info->slots = P.p.slots;
    info->tile = P.p.tile;
    info->gmax = P.gmax;
    info->max_height = P.max_height;
    info->max_ext_wg = P.max_ext_wg;
    info->n_partial = P.n_partial;
    info->n_ext = (int64_t)P.ext_src.size();
    info->n_pairs = P.n_pairs;
    info->chain = P.p.chain;
    info->n_local = (int32_t)P.n_local;
}

void check_topology_args(int64_t n, const int64_t* endnodes, const int64_t* indegree,
                         const int64_t* heads, int64_t n_head) {
    REQUIRE(n >= 0, "n must be >= 0");
    REQUIRE(n == 0 || (endnodes && indegree), "endnodes/indegree must not be NULL");
    REQUIRE(n_head >= 0 && (n_head == 0 || heads), "bad headwater list");
}

// numpy.searchsorted(xp, x, side='left')
int64_t searchsorted_left(const double* xp, int64_t n, double x) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = lo + ((hi - lo) >> 1);
        if (xp[mid] < x) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// {row_lo, row_hi, frac as two 32-bit halves (lo, hi)}; a step clamped to the first / last
// forcing row (nutils.py:24-27 copies that row) is {row, row, 0}: (1 - 0) f + 0 f = f exactly
// for finite forcing
int4 step_entry(int lo, int hi, double frac) {
    uint64_t bits;
    std::memcpy(&bits, &frac, sizeof(bits));
    return make_int4(lo, hi, (int)(uint32_t)(bits & 0xffffffffu), (int)(uint32_t)(bits >> 32));
}

struct Net {
    mcr::Plan plan;
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;

    // static schedule
    DBuf<int32_t> G, sup_off, sup, ext_off, ext_g, wg_gmin, wg_gmax, xid, lx_off, lx_src;
    DBuf<int32_t> pos32, in_off32, upos32;   // reach -> slot, inflow lists in slot space
    DBuf<int16_t> lx;
    DBuf<uint8_t> flags, up_cnt;
    DBuf<uint64_t> up4;
    DBuf<int64_t> slot_reach, pos;
    // coefficients / state (slot order)
    DBuf<double> alpha, beta, chi, gamma, st_o, st_i;
    DBuf<double> st_o2, st_i2;     // input state of the last dataflow horizon (re-run source)
    // forcing (slot order) and single-step forcing
    DBuf<double> F, Fstep, stage, Qm;   // Qm: member lateral inflows of a member-dataflow step
    int64_t n_rows = 0;
    std::vector<double> xp;
    // per-step interpolation table {row_lo, row_hi, frac}
    DBuf<int4> stab;
    // outputs in workgroup windows (kernels.hpp), their per-horizon index (window base of each
    // workgroup, step-0 index of each reach and of each external input) and a scratch for fetches
    DBuf<double> O, outT;
    DBuf<double> gsc;                  // reach-order gathers: steps of a pass in slot order
    DBuf<int64_t> in_off, in_list;   // inflow lists (plan.hpp), caller order
    // per-horizon schedules (active workgroups per launch, output windows), cached per T
    struct Sched {
        int64_t T = -1;
        std::vector<int64_t> off;      // launch k runs list[off[k] .. off[k+1])
        std::vector<int32_t> list;
        DBuf<int32_t> active;
        DBuf<int64_t> wbase, jbase;    // window base per workgroup, step-0 cell per reach
        DBuf<int64_t> sjb;             // window index of step 0 of every node slot
        int64_t Otot = 0;              // output cells of one member
        uint64_t used = 0;
    };
    std::vector<std::unique_ptr<Sched>> scheds;
    Sched* cur = nullptr;              // schedule of the last run (its outputs are in O)
    uint64_t use_clock = 0;
    DBuf<double> XS;               // external-input streams [n_ext][T]
    int64_t T_out = 0;
    bool coeffs_set = false;

    // active-workgroup schedule cache

    // timing
    bool timing = false;
    double kernel_ms = 0.0, run_ms = 0.0;
    int64_t launches = 0;
    std::vector<hipEvent_t> events;
    // ensemble members (mc_net_set_members): per-member arrays are member-major on the device
    int64_t E = 1;

    // ensemble analysis (analysis.hip): anomalies, gauge operators, dense products, solver
    DBuf<double> An, HA, Zn, Gn, GIn, Yb, HXb, Db, Rd, Rb, Ub, EE, Wk;   // Wk: split-K slices
    // SPD solves (dense.hip block LDL^T): padded matrix, unit block factor and its transpose,
    // inverted diagonal blocks, solve scratch, padded right-hand sides
    DBuf<double> Pf, Sd, Rhs;
    DBuf<int64_t> gslot;
    DBuf<int32_t> info;
    // pinned copies of the factorisation status of every analysis since the last sync(), one
    // word each (a later successful analysis must not hide an earlier failure)
    static constexpr int kInfoRing = 256;
    int32_t* info_host = nullptr;
    int info_count = 0;

    // pinned staging ring for asynchronous host -> device uploads (no stream sync per call)
    struct PinSlot {
        void* p = nullptr;
        size_t cap = 0;
        hipEvent_t ev = nullptr;
    };
    PinSlot pins[8];
    int pin_next = 0;

    // dataflow kernel (flow.hip): mode 0 = automatic, 1 = multi-launch only, 2 = dataflow only
    int mode = 0;
    int last_path = 0;             // 1 multi-launch, 2 dataflow (path of the last run)
    int cu_count = 0;
    DBuf<int32_t> all_wg;          // every workgroup, in plan order (the dataflow grid)
    DBuf<uint32_t> XG;             // granules [n_ext][T][4 words]
    size_t xg_words = 0;
    uint32_t epoch = 0;
    DBuf<int32_t> status;
    // non-finite flags of the state, the forcing F and the step row Fstep (WaveArgs::nf, nff):
    // set by the flag kernels
    // when either is loaded, by a kernel epilogue that leaves a non-finite state, and
    // conservatively by every other state writer (mark_state)
    DBuf<int32_t> nf;
    void mark_state() { HIPC(hipMemsetAsync(nf.p, 1, 1, stream)); }
    // a flag from the caller's host arrays when they are small (one memset instead of a memset
    // and a flag kernel per array: sub-basin sessions reload state and forcing every horizon)
    static constexpr size_t kHostFlagMax = (size_t)1 << 16;
    static bool host_nonfinite(const double* a, size_t k) {
        for (size_t x = 0; x < k; ++x)
            if (!std::isfinite(a[x])) return true;
        return false;
    }
    void set_flag(int32_t* f, bool bad) {
        HIPC(hipMemsetAsync(f, 0, sizeof(int32_t), stream));
        if (bad) HIPC(hipMemsetAsync(f, 1, 1, stream));
    }
    int32_t* status_host = nullptr;  // pinned mirror, read at sync()
    int flow_runs = 0;               // dataflow launches since the status word was last read
    // the last dataflow horizon of one member, re-routed with launches when its waits gave up
    // (st_o2 / st_i2 hold its input state until the next dataflow run)
    struct FlowRun {
        bool valid = false;
        int64_t T = 0, rows = 0;
        const double* F = nullptr;
        std::vector<int4> tab;
    } last_flow;
    std::vector<int4> stab_host;     // step table last uploaded to stab
    int force_mode = -1;             // >= 0: mode override during a re-run
    // members per instance of the ensemble sweep (members.hip): 0 = default (2), 1 = the
    // one-member kernel (MCR_MEMBERS_MB for A/B runs)
    int members_mb = getenv("MCR_MEMBERS_MB") ? atoi(getenv("MCR_MEMBERS_MB")) : 0;
    int64_t patience = mcr::kFlowPatience;   // dataflow waits (mc_set_flow_patience)
    int64_t reroutes = 0;            // horizons re-routed after a give-up (mc_net_reroutes)

    // outputs of the last run are the {o, i} pairs of a member-dataflow step (IOb, member windows)
    bool out_io = false;


    // tick-major member windows of the member-dataflow step (kernels.hpp MemberWin), for E
    DBuf<int64_t> mwbase;
    int64_t mw_E = 0, mw_cells = 0;
    DBuf<double> IOb;                // staged {o, i} pairs, 2 doubles per member-window cell
    // tick-major staging pays for large ensembles (EnKF256 member step 2.01 -> 0.92 ms, its
    // staging kernels 0.73 -> 1.15 ms); at 32 members the two are within run-to-run noise
    // (26.5-27.3 ms per EnKF32 horizon either way) and member-major cells are kept
    static constexpr int64_t kSkewMembers = 128;
    bool member_skew() const { return E >= kSkewMembers; }
    mcr::MemberWin member_win() const {
        return mcr::MemberWin{mwbase.p, G.p, wg_gmin.p, flags.p, (int64_t)row_width(),
                              plan.nslots, member_skew()};
    }
    void ensure_member_windows() {
        if (mw_E == E) return;
        if (!member_skew()) {
            mw_E = E;
            mw_cells = plan.nslots * E;
            return;
        }
        std::vector<int64_t> wb(std::max<int32_t>(plan.nwg, 1), 0);
        int64_t total = 0;
        for (int32_t w = 0; w < plan.nwg; ++w) {
            wb[w] = total;
            total += ((int64_t)plan.wg_gmax[w] - plan.wg_gmin[w] + E) * row_width();
        }
        mwbase.upload(wb.data(), wb.size(), stream);
        sync();
        mw_E = E;
        mw_cells = total;
    }

    // identity of this session (slot maps of state hand-overs are cached per source session)
    const uint64_t uid = next_uid();
    static uint64_t next_uid() {
        static std::atomic<uint64_t> c{1};
        return c.fetch_add(1);
    }
    struct SlotMap {
        uint64_t src_uid = 0;
        DBuf<int32_t> map;
    };
    std::vector<std::unique_ptr<SlotMap>> slot_maps;
    // map[d] = the slot of the source plan holding the reach of this plan's slot d (-1: none)
    const int32_t* slot_map_from(const Net& S) {
        for (auto& m : slot_maps)
            if (m->src_uid == S.uid) return m->map.p;
        std::vector<int32_t> mp((size_t)std::max<int64_t>(plan.nslots, 1), -1);
        for (int64_t d = 0; d < plan.nslots; ++d) {
            const int64_t j = plan.slot_reach[d];
            if (j >= 0) mp[d] = (int32_t)S.plan.pos[j];
        }
        if (slot_maps.size() >= 4) slot_maps.erase(slot_maps.begin());
        slot_maps.push_back(std::make_unique<SlotMap>());
        slot_maps.back()->src_uid = S.uid;
        slot_maps.back()->map.upload(mp.data(), mp.size(), stream);
        return slot_maps.back()->map.p;
    }

    // launch trace (mc_set_trace)
    bool trace = false;
    DBuf<int64_t> trace_buf;
    std::vector<int64_t> trace_launch;   // launch index of each traced workgroup record
    std::vector<int32_t> trace_wg;       // workgroup of each record

    ~Net() {
        if (status_host) (void)hipHostFree(status_host);
        if (info_host) (void)hipHostFree(info_host);
        for (PinSlot& ps : pins) {
            if (ps.ev) (void)hipEventSynchronize(ps.ev);
            if (ps.p) (void)hipHostFree(ps.p);
            if (ps.ev) (void)hipEventDestroy(ps.ev);
        }
        for (hipEvent_t e : events) (void)hipEventDestroy(e);
        if (fetch_pending > 0 && stream) (void)hipStreamSynchronize(stream);
        if (cstream) (void)hipStreamSynchronize(cstream);
        for (hipEvent_t e : fetch_ev) (void)hipEventDestroy(e);
        for (int r = 0; r < 2; ++r) {
            if (a_ready[r]) (void)hipEventDestroy(a_ready[r]);
            if (a_copied[r]) (void)hipEventDestroy(a_copied[r]);
        }
        if (cstream) (void)hipStreamDestroy(cstream);
        if (own) (void)hipStreamDestroy(own);
    }

    void init(int64_t n, const int64_t* endnodes, const int64_t* indegree, const int64_t* heads,
              int64_t n_head, const mcr::PlanParams& p) {
        const std::string err = mcr::build_plan(n, endnodes, indegree, heads, n_head, p, plan);
        if (!err.empty()) throw Fail(MC_E_TOPOLOGY, err);
        if (plan.p.tile % mcr::kChunk != 0)
            throw Fail(MC_E_INVALID, "tile must be a multiple of 8 (the kernels' tick chunk)");
        if (!mcr::wavefront_shape_ok(plan.p.slots, plan.p.chain))
            throw Fail(MC_E_INVALID, "no device kernel for this (slots, chain): chain 1 takes "
                                     "slots 64, chain 2 slots 64..512 (multiples of 64 up to "
                                     "448, and 512), chain 3 slots 64/192/256, chain 4 slots "
                                     "64/128/192/256");
        HIPC(hipGetDevice(&device));
        HIPC(hipStreamCreateWithFlags(&own, hipStreamNonBlocking));
        stream = own;
        const size_t ns = (size_t)plan.nslots;
        G.upload(plan.G.data(), ns, stream);
        flags.upload(plan.flags.data(), ns, stream);
        up_cnt.upload(plan.up_cnt.data(), ns, stream);
        up4.upload(plan.up4.data(), ns, stream);
        slot_reach.upload(plan.slot_reach.data(), ns, stream);
        ext_off.upload(plan.ext_off.data(), plan.ext_off.size(), stream);
        ext_g.upload(plan.ext_g.data(), plan.ext_g.size(), stream);
        pos.upload(plan.pos.data(), plan.pos.size(), stream);
        xid.upload(plan.xid.data(), plan.xid.size(), stream);

        lx.upload(plan.lx.data(), plan.lx.size(), stream);
        lx_off.upload(plan.lx_off.data(), plan.lx_off.size(), stream);
        lx_src.upload(plan.lx_src.data(), plan.lx_src.size(), stream);
        lx_src.reserve(1);
        in_off.upload(plan.in_off.data(), plan.in_off.size(), stream);
        in_list.upload(plan.in_list.data(), plan.in_list.size(), stream);
        in_list.reserve(1);
        {   // int32 copies for the reach-order permutation (kernels.hip permute_steps)
            std::vector<int32_t> rp(plan.n), ro(plan.n + 1), ru(plan.in_list.size());
            for (int64_t j = 0; j < plan.n; ++j) rp[j] = (int32_t)plan.pos[j];
            for (int64_t j = 0; j <= plan.n; ++j) ro[j] = (int32_t)plan.in_off[j];
            for (size_t k = 0; k < plan.in_list.size(); ++k)
                ru[k] = (int32_t)plan.pos[plan.in_list[k]];
            pos32.upload(rp.data(), rp.size(), stream);
            pos32.reserve(1);
            in_off32.upload(ro.data(), ro.size(), stream);
            upos32.upload(ru.data(), ru.size(), stream);
            upos32.reserve(1);
        }
        {   // inflow lists in slot space (int32) for the gain scatter
            REQUIRE(ns < ((size_t)1 << 31), "network too large (node slots must fit int32)");
            std::vector<int32_t> so(ns + 1, 0), sl;
            sl.reserve(plan.in_list.size());
            for (size_t d = 0; d < ns; ++d) {
                const int64_t j = plan.slot_reach[d];
                if (j >= 0)
                    for (int64_t k = plan.in_off[j]; k < plan.in_off[j + 1]; ++k)
                        sl.push_back((int32_t)plan.pos[plan.in_list[k]]);
                so[d + 1] = (int32_t)sl.size();
            }
            sup_off.upload(so.data(), so.size(), stream);
            sup.upload(sl.data(), sl.size(), stream);
            sup.reserve(1);
        }
        wg_gmin.upload(plan.wg_gmin.data(), plan.wg_gmin.size(), stream);
        wg_gmax.upload(plan.wg_gmax.data(), plan.wg_gmax.size(), stream);
        for (DBuf<double>* b : {&alpha, &beta, &chi, &gamma, &st_o, &st_i}) {
            b->reserve(ns);
            HIPC(hipMemsetAsync(b->p, 0, ns * sizeof(double), stream));
        }
        stage.reserve(std::max<int64_t>(plan.n, 1));
        HIPC(hipDeviceGetAttribute(&cu_count, hipDeviceAttributeMultiprocessorCount, device));
        {
            std::vector<int32_t> ids(std::max<int32_t>(plan.nwg, 1));
            for (size_t w = 0; w < ids.size(); ++w) ids[w] = (int32_t)w;
            all_wg.upload(ids.data(), ids.size(), stream);
        }
        status.reserve(1);
        HIPC(hipMemsetAsync(status.p, 0, sizeof(int32_t), stream));
        nf.reserve(3);                   // {state, forcing F, step row}: a zero state, no forcing
        HIPC(hipMemsetAsync(nf.p, 0, 3 * sizeof(int32_t), stream));
        HIPC(hipHostMalloc(reinterpret_cast<void**>(&status_host), sizeof(int32_t),
                           hipHostMallocDefault));
        *status_host = 0;
        sync();
    }

    // Copy k elements host -> device without waiting for the stream: the source is staged in a
    // pinned slot whose previous copy (8 uploads ago) must have completed.
    template <class T>
    void upload_async(DBuf<T>& dst, const T* src, size_t k) {
        dst.reserve(k);
        if (k == 0) return;
        PinSlot& ps = pins[pin_next];
        pin_next = (pin_next + 1) % 8;
        if (!ps.ev) HIPC(hipEventCreateWithFlags(&ps.ev, hipEventDisableTiming));
        HIPC(hipEventSynchronize(ps.ev));
        const size_t bytes = k * sizeof(T);
        if (ps.cap < bytes) {
            if (ps.p) HIPC(hipHostFree(ps.p));
            ps.p = nullptr;
            HIPC(hipHostMalloc(&ps.p, bytes, hipHostMallocDefault));
            ps.cap = bytes;
        }
        std::memcpy(ps.p, src, bytes);
        HIPC(hipMemcpyAsync(dst.p, ps.p, bytes, hipMemcpyHostToDevice, stream));
        HIPC(hipEventRecord(ps.ev, stream));
    }

    // Wait for the stream; report a dataflow run whose waits gave up.
    void sync() {
        HIPC(hipStreamSynchronize(stream));
        if (info_count > 0) {
            int32_t bad = 0;
            for (int k = 0; k < info_count; ++k) {
                if (info_host[k] != 0 && bad == 0) bad = info_host[k];
                info_host[k] = 0;
            }
            info_count = 0;
            if (bad != 0) {
                throw Fail(MC_E_INVALID, "ensemble analysis: the analysis matrix (HPH^T + R, or "
                                         "its ensemble-space form) is not positive definite; "
                                         "the increment was zeroed, the member states are "
                                         "unchanged by that analysis");
            }
        }
        if (flow_runs > 0) {
            // the status word is sticky: read once per sync, not once per run
            const int runs = flow_runs;
            flow_runs = 0;
            HIPC(hipMemcpy(status_host, status.p, sizeof(int32_t), hipMemcpyDeviceToHost));
            const int32_t why = *status_host;
            if (why != 0) {
                *status_host = 0;
                HIPC(hipMemsetAsync(status.p, 0, sizeof(int32_t), stream));
                if (runs == 1 && last_flow.valid) {
                    // bit 0: the device was shared (another stream held CUs the resident launch
                    // needed); bit 1: a partial sum met a non-finite value in the fast form.
                    // Route the same horizon again from its input state with launches (exact)
                    st_o.swap(st_o2);
                    st_i.swap(st_i2);
                    last_flow.valid = false;
                    ++reroutes;
                    if (why & 1)
                        std::fprintf(stderr, "[mcroute] dataflow launch gave up waiting for "
                                             "upstream workgroups; the horizon was re-routed "
                                             "with launches\n");
                    mark_state();
                    force_mode = 1;
                    try {
                        run_tables(last_flow.T, last_flow.F, last_flow.rows, last_flow.tab);
                    } catch (...) {
                        force_mode = -1;
                        throw;
                    }
                    force_mode = -1;
                    HIPC(hipStreamSynchronize(stream));
                    flow_runs = 0;           // (the launches report nothing)
                    return;
                }
                if (why & 1)
                    throw Fail(MC_E_HIP, "dataflow kernel: a wait for upstream results gave up "
                                         "(outputs of the runs since the last synchronisation "
                                         "are invalid)");
                mark_state();
                throw Fail(MC_E_STATE, "dataflow kernel: a partial sum met a non-finite value "
                                       "produced from finite inputs (an overflow) in the fast "
                                       "form; the outputs of the runs since the last "
                                       "synchronisation may differ from the reference's there "
                                       "(the session's next run takes the exact form: set the "
                                       "state again and re-run)");
            }
        }
    }

    // Can the whole horizon run as one dataflow launch?  Every workgroup must be resident.
    bool flow_fits(int64_t T, bool dense, size_t& lds) {
        if (mode == 1 || force_mode == 1) return false;
        const int S = plan.p.slots, Kc = plan.p.chain;
        const size_t xg = plan.ext_src.size() * (size_t)T * 16;
        lds = mcr::flow_lds_bytes(S, Kc, (int)T, plan.max_xe_wg);
        bool ok = mcr::flow_shape_ok(S, Kc, plan.p.sync != 0) &&
                  plan.p.tile >= mcr::kFlowMinSlack && plan.max_xe_wg <= mcr::kFlowMaxExt &&
                  T <= mcr::kFlowMaxT && xg < (size_t(1) << 31) && lds <= 160 * 1024;
        if (ok) {
            int bpc = 0;
            HIPC(mcr::flow_occupancy(S, Kc, dense, plan.p.sync != 0, lds, &bpc));
            ok = (int64_t)bpc * cu_count >= plan.nwg;
        }
        if (mode == 2 && !ok)
            throw Fail(MC_E_STATE, "dataflow mode requested but this network/horizon does not fit "
                                   "one resident launch");
        return ok;
    }

    bool members_fit(size_t& lds) {
        if (mode == 1 || force_mode == 1) return false;
        const int S = plan.p.slots, Kc = plan.p.chain;
        const size_t xg = plan.ext_src.size() * (size_t)E * 16;
        lds = mcr::flow_lds_bytes(S, Kc, 0, plan.max_xe_wg);
        bool ok = mcr::flow_shape_ok(S, Kc, plan.p.sync != 0) &&
                  plan.p.tile >= mcr::kFlowMinSlack && plan.max_xe_wg <= mcr::kFlowMaxExt &&
                  E < (1 << 24) && xg < (size_t(1) << 31) && lds <= 160 * 1024 &&
                  // member-major cells are addressed by 32-bit buffer offsets (flow.hip MEMB)
                  (member_skew() || plan.nslots * E * 16 < (1ll << 31));
        if (ok) {
            int bpc = 0;
            HIPC(mcr::flow_members_occupancy(S, Kc, plan.p.sync != 0, lds, &bpc));
            ok = (int64_t)bpc * cu_count >= plan.nwg;
        }
        return ok;
    }

    // caller-order host array [n][m] -> member-major slot-order device array [m][nslots]
    void to_slots(const double* host, DBuf<double>& dst, int64_t m = 1,
                  DBuf<double>* via = nullptr) {
        const int64_t n = plan.n;
        if (n == 0) return;
        DBuf<double>& sb = via ? *via : stage;
        sb.reserve((size_t)(n * m));
        HIPC(hipMemcpyAsync(sb.p, host, n * m * sizeof(double), hipMemcpyHostToDevice, stream));
        HIPC(mcr::launch_scatter_to_slots(sb.p, dst.p, slot_reach.p, plan.nslots, m, stream));
        // a copy from pageable memory has read the caller's array when it returns; one from
        // page-locked memory (e.g. a yielded pinned output row) is truly asynchronous, so wait
        // for it: the C ABI promises that the caller may reuse its arrays on return
        if (host_pinned(host)) HIPC(hipStreamSynchronize(stream));
    }
    static bool host_pinned(const void* p) {
        hipPointerAttribute_t at{};
        if (hipPointerGetAttributes(&at, p) != hipSuccess) {
            (void)hipGetLastError();                    // unregistered pageable memory
            return false;
        }
        return at.type == hipMemoryTypeHost;
    }
    // Resolve pending dataflow runs (status word, re-run on give-up) before results are read.
    void settle() {
        if (flow_runs > 0) sync();
    }
    // Before a call changes the state, coefficients or forcing: a pending dataflow horizon that
    // could still be re-routed on give-up (sync) is resolved first, so the re-run can never
    // replay it over the caller's change or from a freed forcing buffer.  Member
    // steps are never re-routed (last_flow.valid is false), so the EnKF cycle does not sync here.
    void settle_state() {
        if (flow_runs > 0 && last_flow.valid) sync();
    }

    void from_slots(const DBuf<double>& src, double* host, int64_t m = 1) {
        const int64_t n = plan.n;
        if (n == 0) return;
        settle();
        settle_gain();
        stage.reserve((size_t)(n * m));
        HIPC(mcr::launch_gather_from_slots(src.p, stage.p, pos.p, n, plan.nslots, m, stream));
        HIPC(hipMemcpyAsync(host, stage.p, n * m * sizeof(double), hipMemcpyDeviceToHost,
                            stream));
        sync();
    }

    // ---- ensemble analysis ----------------------------------------------
    // The increments of the last analysis (Gn) are applied lazily: the EnKF cycle's next call
    // is the one-step member run, whose input staging applies them on the way
    // (launch_member_inputs, PendingGain); anything else that reads the state settles them
    // first with the apply_gain kernel (same arithmetic, bit-identical).
    bool gain_pending = false;
    void settle_gain() {
        if (!gain_pending) return;
        gain_pending = false;
        HIPC(mcr::launch_apply_gain(Gn.p, st_o.p, st_i.p, flags.p, sup_off.p, sup.p, plan.nslots,
                                    E, stream));
        mark_state();
    }

    void apply_gain(const double* gain) {
        REQUIRE(plan.n == 0 || gain, "gain must not be NULL");
        if (plan.n == 0) return;
        settle_state();
        settle_gain();
        const size_t ns = (size_t)plan.nslots;
        Gn.reserve(ns * E);
        to_slots(gain, Gn, E);
        HIPC(mcr::launch_apply_gain(Gn.p, st_o.p, st_i.p, flags.p, sup_off.p, sup.p,
                                    plan.nslots, E, stream));
        mark_state();
        sync();
    }

    // R diagonal with a positive diagonal?  (its diagonal into rd)
    static bool diagonal_R(const double* R, int64_t m, std::vector<double>& rd) {
        rd.resize(m);
        for (int64_t i = 0; i < m; ++i) {
            const double* row = R + i * m;
            for (int64_t j = 0; j < m; ++j)
                if (j != i && row[j] != 0.0) return false;
            if (!(row[i] > 0.0)) return false;
            rd[i] = row[i];
        }
        return true;
    }

    // B (kp x nrhs, leading dimension kp, padding rows 0) := P^-1 B for the padded SPD P
    // (kp x kp, overwritten); the status in `info` (device): B = 0 if P is not positive definite
    void spd_solve(double* P, int64_t kp, double* B, int64_t nrhs) {
        Sd.reserve((size_t)(kp * 32));
        info.reserve(1);
        HIPC(mcr::launch_spd_solve(P, kp, B, nrhs, Sd.p, info.p, stream));
    }
    // the factorisation status, read back asynchronously and reported at the next sync()
    void info_async() {
        if (!info_host) {
            HIPC(hipHostMalloc(reinterpret_cast<void**>(&info_host), kInfoRing * sizeof(int32_t),
                               hipHostMallocDefault));
            std::memset(info_host, 0, kInfoRing * sizeof(int32_t));
        }
        if (info_count == kInfoRing) sync();      // report (and free) the ring before reuse
        HIPC(hipMemcpyAsync(info_host + info_count, info.p, sizeof(int32_t),
                            hipMemcpyDeviceToHost, stream));
        ++info_count;
    }

    // C = HA HA^T / (E-1) + R (m x m) from the current member state (padded to
    // mp = spd_padded(m) in Pf); anomalies in An, gauge anomalies in HA
    void analysis_setup(int64_t m, const int64_t* gauges, const double* R) {
        REQUIRE(E >= 2, "the ensemble analysis needs at least 2 members");
        REQUIRE(m >= 1 && m < (1ll << 31) && gauges && R, "bad gauge arguments");
        settle_state();
        settle_gain();
        const int64_t n = plan.n, ns = plan.nslots;
        std::vector<int64_t> gs(m);
        for (int64_t g = 0; g < m; ++g) {
            REQUIRE(gauges[g] >= 0 && gauges[g] < n, "gauge index out of range");
            gs[g] = plan.pos[gauges[g]];
        }
        gslot.upload(gs.data(), gs.size(), stream);
        An.reserve((size_t)(ns * E));
        HA.reserve((size_t)(m * E));
        Rb.upload(R, (size_t)(m * m), stream);     // symmetric: row-major == column-major
        HIPC(mcr::launch_mean_anomalies(st_o.p, An.p, ns, E, stream));
        HIPC(mcr::launch_gauge_gather(An.p, st_o.p, gslot.p, nullptr, HA.p, nullptr, m, ns, E,
                                      stream));
        const double inv = 1.0 / (double)(E - 1);
        const int64_t mp = mcr::spd_padded(m);
        Pf.reserve((size_t)(mp * mp));
        HIPC(mcr::launch_pad_matrix(Rb.p, m, m, m, Pf.p, mp, 1.0, mp, stream));
        HIPC(mcr::launch_dgemm(false, true, m, m, E, inv, HA.p, m, HA.p, m, 1.0, Pf.p, mp,
                               stream));
    }

    // ---- staged ensemble analysis: the member-sharded form (several ranks, one per GPU; the
    // collectives between the stages run in the caller, ensemble.py) and, with N = 1, the
    // single-GPU mc_enkf_analysis.  Stage buffers are device pointers owned by the caller.
    int64_t slice_size(int64_t N) const { return (plan.nslots + N - 1) / N; }
    // values per tick row of an output window: the node slots of a workgroup
    int row_width() const { return plan.p.chain * plan.p.slots; }

    void upload_gauges(int64_t m, const int64_t* gauges) {
        REQUIRE(m >= 1 && m < (1ll << 31) && gauges, "bad gauge arguments");
        std::vector<int64_t> gs(m);
        for (int64_t g = 0; g < m; ++g) {
            REQUIRE(gauges[g] >= 0 && gauges[g] < plan.n, "gauge index out of range");
            gs[g] = plan.pos[gauges[g]];
        }
        upload_async(gslot, gs.data(), gs.size());
    }

    // local members: HX [E][m] (gauge outflows), D [E][m] = y[g][e] - HX
    void ens_gauges(int64_t m, const int64_t* gauges, const double* y, double* HX, double* D) {
        REQUIRE(y && HX && D, "null argument");
        settle_state();
        settle_gain();
        upload_gauges(m, gauges);
        upload_async(Yb, y, (size_t)(m * E));
        HIPC(mcr::launch_gauge_values(st_o.p, gslot.p, Yb.p, HX, D, m, plan.nslots, E, stream));
    }

    // local member states -> reach slices for every rank: send [N][E][S]
    void ens_pack(int64_t N, double* send) {
        REQUIRE(N >= 1 && send, "bad pack arguments");
        settle_state();
        settle_gain();
        HIPC(mcr::launch_pack_slices(st_o.p, send, plan.nslots, E, slice_size(N), N, stream));
    }

    // this rank's reach slice of ALL members (Xs [Et][S]) + all members' gauge values / innovations
    // ([Et][m]) -> the slice of the increments G = A Z (Gs [Et][S]);  Et = E * N.  Two halves:
    // the weights Z need only the gathered gauge data, so a caller can form them while the
    // member -> slice all-to-all of Xs is still in flight (ensemble.py)
    void ens_slice_update(int64_t N, int64_t m, const double* Xs, const double* HXall,
                          const double* Dall, const double* R, double* Gs) {
        ens_weights(N, m, HXall, Dall, R);
        ens_increments(N, Xs, Gs);
    }
    // the analysis weights Z [Et][Et] (kept in the session's buffers for ens_increments)
    const double* Zw = nullptr;
    int64_t Zld = 0, Zet = 0;
    void ens_weights(int64_t N, int64_t m, const double* HXall, const double* Dall,
                     const double* R) {
        REQUIRE(N >= 1 && m >= 1 && HXall && Dall && R, "bad weight arguments");
        const int64_t Et = E * N;
        REQUIRE(Et >= 2, "the ensemble analysis needs at least 2 members");
        const double inv = 1.0 / (double)(Et - 1);
        // gauge anomalies HA = HX - mean over members
        HA.reserve((size_t)(m * Et));
        HIPC(mcr::launch_mean_anomalies(HXall, HA.p, m, Et, stream));
        const double* Z = nullptr;
        int64_t ldz = Et;
        std::vector<double> rd;
        if (Et <= m && diagonal_R(R, m, rd)) {
            // ensemble space (diagonal R): with S = HA / sqrt(Et-1),
            //   S^T (S S^T + R)^-1 D = (I + S^T R^-1 S)^-1 S^T R^-1 D   (push-through identity)
            // so Z = HA^T C^-1 D / (Et-1) = M^-1 V with M = I + HA^T R^-1 HA / (Et-1) (Et x Et,
            // SPD, eigenvalues >= 1) and V = (R^-1 HA)^T D / (Et-1): an Et x Et solve instead
            // of m x m.  [M | V] = [I | 0] + U^T [HA | D] / (Et-1) (U = R^-1 HA) is ONE split-K
            // MFMA launch into the padded system buffer EE = [M (kp x kp) | V (kp x Et)]
            upload_async(Rd, rd.data(), rd.size());
            Ub.reserve((size_t)(m * Et));
            HIPC(mcr::launch_scale_rows(HA.p, Rd.p, Ub.p, m, Et, stream));
            const int64_t kp = mcr::spd_padded(Et);
            EE.reserve((size_t)(kp * (kp + Et)));
            HIPC(mcr::launch_pad_matrix(nullptr, 0, 0, 0, EE.p, kp, 1.0, kp + Et, stream));
            Wk.reserve((size_t)(64 * Et * 2 * Et));
            double* V = EE.p + kp * kp;
            HIPC(mcr::launch_dgemm(true, false, Et, 2 * Et, m, inv, Ub.p, m, HA.p, m, 1.0, EE.p,
                                   kp, stream, Wk.p, Wk.cap, Dall, Et, V));
            spd_solve(EE.p, kp, V, Et);
            info_async();
            Z = V;
            ldz = kp;
        } else {
            // observation space: C = HA HA^T / (Et-1) + R (m x m), W = C^-1 D,
            // Z = HA^T W / (Et-1)
            const int64_t mp = mcr::spd_padded(m);
            upload_async(Rb, R, (size_t)(m * m));      // symmetric: row-major == column-major
            Pf.reserve((size_t)(mp * mp));
            HIPC(mcr::launch_pad_matrix(Rb.p, m, m, m, Pf.p, mp, 1.0, mp, stream));
            HIPC(mcr::launch_dgemm(false, true, m, m, Et, inv, HA.p, m, HA.p, m, 1.0, Pf.p, mp,
                                   stream));
            Rhs.reserve((size_t)(mp * Et));
            HIPC(mcr::launch_pad_matrix(Dall, m, Et, m, Rhs.p, mp, 0.0, Et, stream));
            spd_solve(Pf.p, mp, Rhs.p, Et);
            info_async();
            Zn.reserve((size_t)(Et * Et));
            Wk.reserve((size_t)(64 * Et * Et));
            HIPC(mcr::launch_dgemm(true, false, Et, Et, m, inv, HA.p, m, Rhs.p, mp, 0.0, Zn.p, Et,
                                   stream, Wk.p, Wk.cap));
            Z = Zn.p;
            ldz = Et;
        }
        Zw = Z;
        Zld = ldz;
        Zet = Et;
    }
    void ens_increments(int64_t N, const double* Xs, double* Gs) {
        REQUIRE(N >= 1 && Xs && Gs, "bad increment arguments");
        const int64_t Et = E * N, S = slice_size(N);
        REQUIRE(Zw != nullptr && Zet == Et,
                "mc_ens_increments: no analysis weights of this ensemble (mc_ens_weights first)");
        const double* Z = Zw;
        const int64_t ldz = Zld;
        // slice increments G = A Z (= K D per member): one fused pass for the per-GPU ensemble
        // sizes, the 128 x 128 MFMA tile with the member mean folded in beyond (dense.hip)
        if (Et <= mcr::kFusedIncrementsMax)
            HIPC(mcr::launch_anomaly_increments(Xs, Z, ldz, Gs, S, Et, stream));
        else
            HIPC(mcr::launch_slice_increments(Xs, Z, ldz, Gs, S, Et, stream));
    }

    // increments of the local members from every rank's slice (Grecv [N][E][S]) -> _apply_gain
    void ens_unpack_apply(int64_t N, const double* Grecv) {
        REQUIRE(N >= 1 && Grecv, "bad unpack arguments");
        settle_state();
        const int64_t ns = plan.nslots;
        Gn.reserve((size_t)(ns * E));
        settle_gain();
        HIPC(mcr::launch_unpack_slices(Grecv, Gn.p, ns, E, slice_size(N), N, stream));
        gain_pending = true;             // applied by the next state reader (settle_gain)
    }

    void enkf_analysis(int64_t m, const int64_t* gauges, const double* y, const double* R) {
        REQUIRE(y && R, "observations / R must not be NULL");
        if (plan.n == 0) return;
        REQUIRE(E >= 2, "the ensemble analysis needs at least 2 members");
        const int64_t ns = plan.nslots;
        HXb.reserve((size_t)(m * E));
        Db.reserve((size_t)(m * E));
        Gn.reserve((size_t)(ns * E));
        ens_gauges(m, gauges, y, HXb.p, Db.p);
        // one rank: the slice of every member IS the member-major state (slice_size(1) = ns),
        // so the pack / unpack stages are identities
        ens_slice_update(1, m, st_o.p, HXb.p, Db.p, R, Gn.p);
        gain_pending = true;             // applied by the next state reader (settle_gain)
    }

    // K = (A HA^T / (E-1)) C2^-1  as [n][m] in caller order
    void enkf_gain(int64_t m, const int64_t* gauges, const double* R, double* K_out) {
        REQUIRE(K_out, "K_out must not be NULL");
        if (plan.n == 0) return;
        REQUIRE(plan.nslots < (1ll << 31), "network too large for the explicit gain");
        analysis_setup(m, gauges, R);
        const int64_t ns = plan.nslots, mp = mcr::spd_padded(m);
        const double inv = 1.0 / (double)(E - 1);
        Gn.reserve((size_t)(mp * ns));              // K^T (mp x ns, padding rows 0), solved in place
        HIPC(hipMemsetAsync(Gn.p, 0, (size_t)(mp * ns) * sizeof(double), stream));
        HIPC(mcr::launch_dgemm(false, true, m, ns, E, inv, HA.p, m, An.p, ns, 0.0, Gn.p, mp,
                               stream));
        spd_solve(Pf.p, mp, Gn.p, ns);
        int32_t ih = 0;
        HIPC(hipMemcpyAsync(&ih, info.p, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
        sync();
        if (ih != 0) throw Fail(MC_E_INVALID, "HPH^T + R is not positive definite");
        outT.reserve((size_t)(plan.n * m));
        HIPC(mcr::launch_gain_to_caller(Gn.p, mp, outT.p, pos.p, m, plan.n, stream));
        HIPC(hipMemcpyAsync(K_out, outT.p, (size_t)(plan.n * m) * sizeof(double),
                            hipMemcpyDeviceToHost, stream));
        sync();
    }

    void set_members(int64_t m) {
        REQUIRE(m >= 1 && m <= 65535, "members must be in [1, 65535]");
        settle_state();
        sync();
        gain_pending = false;            // the state is zeroed
        E = m;
        const size_t ns = (size_t)std::max<int64_t>(plan.nslots, 1);
        for (DBuf<double>* b : {&st_o, &st_i}) {
            b->reserve(ns * m);
            HIPC(hipMemsetAsync(b->p, 0, ns * m * sizeof(double), stream));
        }
        HIPC(hipMemsetAsync(nf.p, 0, sizeof(int32_t), stream));   // a zero state
        n_rows = 0;                    // forcing and outputs are per member: load again
        T_out = 0;
        sync();
    }

    void set_coeffs(const double* a, const double* b, const double* c, const double* g) {
        REQUIRE(plan.n == 0 || (a && b && c && g), "coefficient arrays must not be NULL");
        settle_state();
        to_slots(a, alpha);
        to_slots(b, beta);
        to_slots(c, chi);
        to_slots(g, gamma);
        // partial sums pass their fold through, unrouted reaches and padding output 0
        HIPC(mcr::launch_set_slot_coeffs(flags.p, alpha.p, beta.p, chi.p, gamma.p, plan.nslots,
                                         stream));
        sync();  // `stage` is reused by the next call
        coeffs_set = true;
    }

    void set_state(const double* o, const double* i) {
        REQUIRE(plan.n == 0 || (o && i), "state arrays must not be NULL");
        settle_state();
        gain_pending = false;            // replaced
        to_slots(o, st_o, E);
        to_slots(i, st_i, E, &stage2);   // its own staging (stream-ordered reuse, no sync)
        const size_t cells = (size_t)(plan.n * E);
        if (cells <= kHostFlagMax) {
            set_flag(nf.p, host_nonfinite(o, cells) || host_nonfinite(i, cells));
        } else {
            HIPC(hipMemsetAsync(nf.p, 0, sizeof(int32_t), stream));
            HIPC(mcr::launch_flag_nonfinite(st_o.p, plan.nslots * E, nf.p, stream));
            HIPC(mcr::launch_flag_nonfinite(st_i.p, plan.nslots * E, nf.p, stream));
        }
    }

    // Per-horizon layout: active workgroups of every launch and the output windows (cached
    // for the last few horizon lengths: assimilation alternates 1-step and long runs).
    void ensure_schedule(int64_t T) {
        Sched* hit = nullptr;
        for (auto& sc : scheds)
            if (sc->T == T) hit = sc.get();
        if (!hit) {
            if (scheds.size() >= 4) {
                auto old = std::min_element(scheds.begin(), scheds.end(),
                                            [](const auto& a, const auto& b) {
                                                return a->used < b->used;
                                            });
                scheds.erase(old);
            }
            scheds.push_back(std::make_unique<Sched>());
            hit = scheds.back().get();
            hit->T = T;
            mcr::active_schedule(plan, T, hit->list, hit->off);
            hit->active.upload(hit->list.data(), hit->list.size(), stream);
            std::vector<int64_t> wb(plan.nwg);
            int64_t total = 0;
            for (int32_t w = 0; w < plan.nwg; ++w) {
                wb[w] = total;
                total += ((int64_t)plan.wg_gmax[w] - plan.wg_gmin[w] + T) * row_width();
            }
            hit->wbase.upload(wb.data(), wb.size(), stream);
            hit->Otot = total;
            hit->jbase.reserve((size_t)std::max<int64_t>(plan.n, 1));
            HIPC(mcr::launch_window_index(pos.p, G.p, flags.p, wg_gmin.p, hit->wbase.p,
                                          row_width(), plan.n, hit->jbase.p, stream));
            hit->sjb.reserve((size_t)std::max<int64_t>(plan.nslots, 1));
            HIPC(mcr::launch_slot_window_index(G.p, flags.p, wg_gmin.p, hit->wbase.p, row_width(),
                                               plan.nslots, hit->sjb.p, stream));
            sync();
        }
        hit->used = ++use_clock;
        cur = hit;
        O.reserve((size_t)(cur->Otot * E));
        XS.reserve(std::max<size_t>(plan.ext_src.size() * (size_t)T * E, 1));
    }

    void ensure_events(size_t k) {
        while (events.size() < k) {
            hipEvent_t e;
            HIPC(hipEventCreate(&e));
            events.push_back(e);
        }
    }

    // the outputs of the last run, as the gather kernels address them
    struct OutView {
        const double* O;
        int64_t mO;
        const int64_t* jbase;
        int64_t stride;
    };
    OutView out_view() const {
        return {O.p, cur->Otot, cur->jbase.p, (int64_t)row_width()};
    }
    // steps [t0, t1) of the last run's outflows / inflows, reach order, step-major, into device
    // buffers (either may be NULL), on the session stream
    void gather_block(int64_t t0, int64_t t1, double* o_dst, double* i_dst) {
        const int64_t n = plan.n;
        if (out_io) {                      // T = 1: t0 = 0, t1 = 1
            if (o_dst) HIPC(mcr::launch_gather_io(IOb.p, member_win(), pos.p, false, o_dst, n, E,
                                                  stream));
            if (i_dst) HIPC(mcr::launch_gather_io(IOb.p, member_win(), pos.p, true, i_dst, n, E,
                                                  stream));
            return;
        }
        const OutView ov = out_view();
        if (E == 1) {                      // both series, slot order first (kernels.hip)
            // scratch of at most 512 MB (the whole Texas horizon; CONUS in passes of ~24 steps)
            const int64_t steps = std::max<int64_t>(
                1, std::min<int64_t>(t1 - t0, (512ll << 20) / (8 * std::max<int64_t>(plan.nslots, 1))));
            gsc.reserve((size_t)std::max<int64_t>(steps * plan.nslots, 1));
            HIPC(mcr::launch_gather_slots(ov.O, cur->sjb.p, ov.stride, pos32.p, in_off32.p,
                                          upos32.p, o_dst, i_dst, n, plan.nslots, t0, t1,
                                          gsc.p, steps, stream));
            return;
        }
        for (int c = 0; c < 2; ++c) {
            double* dst = c == 0 ? o_dst : i_dst;
            if (dst)
                HIPC(mcr::launch_gather_steps(ov.O, ov.mO, ov.jbase, in_off.p, in_list.p, c == 1,
                                              (int)ov.stride, dst, n, t0, t1, E, stream));
        }
    }

    // Run T steps using forcing buffer `Fsrc` with `rows` rows and the host step table.
    void run_tables(int64_t T, const double* Fsrc, int64_t rows, const std::vector<int4>& tabh) {
        REQUIRE(coeffs_set, "mc_set_coeffs must be called before running");
        REQUIRE(T >= 1 && T < (1ll << 30), "T out of range");
        // a second run before the first was synchronised: the first can no longer be re-routed
        // on give-up (its input state is about to be overwritten), so a give-up of either is
        // reported as an error, never replayed over this run
        if (flow_runs > 0) last_flow.valid = false;
        const int64_t n = plan.n;
        T_out = 0;
        if (n == 0) {
            T_out = T;
            return;
        }
        // dense forcing: some window of kChunk consecutive steps spans more than 3 rows
        bool dense = false;
        for (int64_t t = 0; t < T && !dense; ++t) {
            const int64_t t2 = std::min<int64_t>(t + mcr::kChunk - 1, T - 1);
            const int last = std::max(tabh[t2].x, tabh[t2].y);
            dense = last - tabh[t].x + 1 > 3;
        }
        if (tabh != stab_host) {           // repeated horizons reuse the uploaded table
            upload_async(stab, tabh.data(), tabh.size());
            stab_host = tabh;
        }
        last_path = 0;
        out_io = false;
        ensure_schedule(T);
        const int64_t nl = (int64_t)cur->off.size() - 1;
        if (timing) ensure_events(2 * (size_t)nl + 2);
        if (timing) HIPC(hipEventRecord(events[2 * nl], stream));

        mcr::WaveArgs a{};
        a.status = status.p;
        a.G = G.p;
        a.flags = flags.p;
        a.up_cnt = up_cnt.p;
        a.up4 = up4.p;
        a.ext_off = ext_off.p;
        a.xid = xid.p;
        a.lx = lx.p;
        a.lx_off = plan.p.sync ? lx_off.p : nullptr;
        a.lx_src = lx_src.p;
        a.XS = XS.p;
        a.ext_g = ext_g.p;
        a.alpha = alpha.p;
        a.beta = beta.p;
        a.chi = chi.p;
        a.gamma = gamma.p;
        a.st_o = st_o.p;
        a.st_i = st_i.p;
        a.F = Fsrc;
        a.stab = stab.p;
        a.nf = nf.p;
        a.nff = nf.p + (Fsrc == Fstep.p ? 2 : 1);
        a.wg_gmin = wg_gmin.p;
        a.wg_gmax = wg_gmax.p;
        a.wbase = cur->wbase.p;
        a.O = O.p;
        a.nslots = plan.nslots;
        a.n_rows = (int32_t)rows;
        a.T = (int32_t)T;
        a.tile = plan.p.tile;
        a.ext_cap = plan.max_xe_wg;
        a.mF = rows * plan.nslots;
        a.mO = cur->Otot;
        a.mX = (int64_t)plan.ext_src.size() * T;
        a.mS = plan.nslots;
        int64_t launched = 0;
        trace_launch.clear();
        trace_wg.clear();
        out_io = false;
        size_t flds = 0;
        {
            if (E > 1 && mode == 2 && T != 1)
                throw Fail(MC_E_STATE, "dataflow mode routes one member, or one step of an ensemble");
            const bool memb = E > 1 && T == 1 && members_fit(flds);
            if (!memb) settle_gain();
            if (memb) {
                // ---- one step of all members as one dataflow launch (flow.hip, MEMB): member e
                // of slot d at tick G[d] + e
                const size_t words = plan.ext_src.size() * (size_t)E * 4;
                if (words > xg_words || epoch == 0xffffffffu) {
                    XG.reserve(std::max<size_t>(words, 4));
                    HIPC(hipMemsetAsync(XG.p, 0, std::max<size_t>(words, 4) * 4, stream));
                    xg_words = std::max(xg_words, words);
                    epoch = 0;
                }
                ++epoch;
                ensure_member_windows();
                Qm.reserve((size_t)std::max<int64_t>(mw_cells, 1));
                IOb.reserve((size_t)std::max<int64_t>(2 * mw_cells, 2));
                double* IOp = IOb.p;
                const mcr::MemberWin mw = member_win();
                mcr::PendingGain pg;
                if (gain_pending) {
                    GIn.reserve((size_t)(plan.nslots * E));
                    pg = mcr::PendingGain{Gn.p, sup_off.p, sup.p, GIn.p};
                }
                HIPC(mcr::launch_member_inputs(Fsrc, a.mF, plan.nslots, (int)rows, tabh[0], st_o.p,
                                               st_i.p, IOp, Qm.p, E, mw, stream, pg));
                gain_pending = false;
                a.Qm = Qm.p;
                a.IO = IOp;
                a.wbase = mwbase.p;          // member windows (the launch stores no output rows)
                a.mskew = member_skew() ? 1 : 0;
                a.T = (int32_t)E;
                a.XG = XG.p;
                a.xg_bytes = (uint32_t)std::max<size_t>(words * 4, 16);
                a.epoch = epoch;
                a.status = status.p;
                a.patience = patience;
                a.table_cap = 0;
                a.active = all_wg.p;
                if (trace) {
                    trace_buf.reserve(mcr::kTraceWords * (size_t)std::max<int32_t>(plan.nwg, 1));
                    a.trace = trace_buf.p;
                    trace_launch.assign(plan.nwg, 0);
                    for (int32_t w = 0; w < plan.nwg; ++w) trace_wg.push_back(w);
                }
                if (timing) HIPC(hipEventRecord(events[0], stream));
                HIPC(mcr::launch_flow_members(a, plan.nwg, plan.p.slots, plan.p.chain, flds,
                                              plan.p.sync != 0, stream));
                if (timing) HIPC(hipEventRecord(events[1], stream));
                HIPC(mcr::launch_member_unpack(IOp, mw, st_o.p, st_i.p, plan.nslots, E, stream));
                mark_state();
                out_io = true;             // the step's outputs stay in IO (fetch)
                ++flow_runs;
                last_flow.valid = false;       // member runs update the state in place
                launched = 1;
                last_path = 2;
                a.T = (int32_t)T;
            } else if (E > 1 && mode == 2) {
                throw Fail(MC_E_STATE, "member dataflow requested but the network does not fit one "
                                       "resident launch");
            }
            if (E == 1 && flow_fits(T, dense, flds)) {
                // ---- one dataflow launch for the whole horizon (flow.hip)
                const size_t words = plan.ext_src.size() * (size_t)T * 4;
                if (words > xg_words || epoch == 0xffffffffu) {
                    XG.reserve(std::max<size_t>(words, 4));
                    HIPC(hipMemsetAsync(XG.p, 0, std::max<size_t>(words, 4) * 4, stream));
                    xg_words = std::max(xg_words, words);
                    epoch = 0;                 // granules of earlier runs can never match again
                }
                ++epoch;
                a.XG = XG.p;
                a.xg_bytes = (uint32_t)std::max<size_t>(words * 4, 16);
                a.epoch = epoch;
                a.status = status.p;
                a.patience = patience;
                a.table_cap = (int32_t)T;
                a.active = all_wg.p;
                if (trace) {
                    trace_buf.reserve(mcr::kTraceWords * (size_t)std::max<int32_t>(plan.nwg, 1));
                    a.trace = trace_buf.p;
                    trace_launch.assign(plan.nwg, 0);
                    for (int32_t w = 0; w < plan.nwg; ++w) trace_wg.push_back(w);
                }
                // the horizon's final state goes to the spare buffers, which then become the
                // session state; the input state stays in the old ones (re-run source, sync())
                st_o2.reserve(st_o.cap);
                st_i2.reserve(st_i.cap);
                a.st_o_out = st_o2.p;
                a.st_i_out = st_i2.p;
                if (timing) HIPC(hipEventRecord(events[0], stream));
                HIPC(mcr::launch_flow(a, plan.nwg, plan.p.slots, plan.p.chain, flds, dense,
                                      plan.p.sync != 0, stream));
                if (timing) HIPC(hipEventRecord(events[1], stream));
                st_o.swap(st_o2);
                st_i.swap(st_i2);
                ++flow_runs;
                last_flow.valid = true;
                last_flow.T = T;
                last_flow.F = Fsrc;
                last_flow.rows = rows;
                last_flow.tab = tabh;
                launched = 1;
                last_path = 2;
            }
            a.table_cap = (int32_t)mcr::table_entries(plan.p.slots, plan.p.tile);
            // ensembles: two members per workgroup instance (members.hip) where it applies
            const int mb = members_mb > 0 ? members_mb : 2;
            const bool memb2 = E >= 2 && E % mb == 0 && mb > 1 && !dense && !plan.p.sync &&
                               mcr::members_shape_ok(plan.p.slots, plan.p.chain, mb);
            const size_t lds = memb2 ? mcr::members_lds_bytes(plan.p.slots, plan.p.chain,
                                                              a.table_cap, a.ext_cap, mb)
                                     : mcr::wavefront_lds_bytes(plan.p.slots, plan.p.chain,
                                                                a.table_cap, a.ext_cap, a.tile);
            if (launched == 0 && trace) {
                trace_buf.reserve(mcr::kTraceWords * (size_t)std::max<int64_t>(cur->off[nl], 1));
                trace_wg = cur->list;
            }
            for (int64_t k = 0; k < nl && last_path != 2; ++k) {
                const int64_t grid = cur->off[k + 1] - cur->off[k];
                if (grid == 0) continue;
                a.active = cur->active.p + cur->off[k];
                if (trace) {
                    a.trace = trace_buf.p + mcr::kTraceWords * cur->off[k];
                    trace_launch.resize(cur->off[k + 1], k);
                }
                a.kappa0 = (int32_t)(k * plan.p.tile);
                if (timing) HIPC(hipEventRecord(events[2 * launched], stream));
                if (memb2)
                    HIPC(mcr::launch_members(a, (int)grid, plan.p.slots, plan.p.chain, lds,
                                             (int)E, mb, stream));
                else
                    HIPC(mcr::launch_wavefront(a, (int)grid, plan.p.slots, plan.p.chain, lds,
                                               dense, (int)E, stream));
                if (timing) HIPC(hipEventRecord(events[2 * launched + 1], stream));
                ++launched;
                last_path = 1;
            }
        }
        if (timing) {
            HIPC(hipEventRecord(events[2 * nl + 1], stream));
            HIPC(hipEventSynchronize(events[2 * nl + 1]));
            for (int64_t k = 0; k < launched; ++k) {
                float ms = 0.f;
                HIPC(hipEventElapsedTime(&ms, events[2 * k], events[2 * k + 1]));
                kernel_ms += ms;
            }
            float ms = 0.f;
            HIPC(hipEventElapsedTime(&ms, events[2 * nl], events[2 * nl + 1]));
            run_ms += ms;
            launches += launched;
        }
        T_out = T;
    }

    void load_forcing(int64_t rows, const double* xps, const double* fp,
                      bool reach_major = false) {
        REQUIRE(rows >= 1 && rows < (1ll << 31), "n_rows must be >= 1");
        REQUIRE(xps && (plan.n == 0 || fp), "xp/fp must not be NULL");
        for (int64_t r = 1; r < rows; ++r)
            REQUIRE(!(xps[r] < xps[r - 1]), "xp must be sorted ascending");
        settle_state();
        const int64_t n = plan.n;
        xp.assign(xps, xps + rows);
        n_rows = rows;
        F.reserve((size_t)(rows * plan.nslots * E));
        if (n == 0) return;
        // caller-order staging: kept between calls when small (sub-basin sessions reload their
        // forcing every horizon; a device allocation per call cost more than the copy)
        const size_t cells = (size_t)(rows * n * E);
        DBuf<double> tmp;
        DBuf<double>& st = cells <= kKeepStage ? fstage : tmp;
        st.upload(fp, cells, stream);
        HIPC(mcr::launch_forcing_to_slots(st.p, F.p, slot_reach.p, n, plan.nslots, rows, E,
                                          stream, reach_major));
        if (cells <= kHostFlagMax) {
            set_flag(nf.p + 1, host_nonfinite(fp, cells));
        } else {
            HIPC(hipMemsetAsync(nf.p + 1, 0, sizeof(int32_t), stream));
            HIPC(mcr::launch_flag_nonfinite(F.p, rows * plan.nslots * E, nf.p + 1, stream));
        }
        // a copy from pageable host memory has read the caller's array when it returns, and the
        // persistent staging is reused stream-ordered: only the temporary staging must be
        // drained before it is freed, and a page-locked source (an asynchronous copy) read
        if (&st == &tmp || host_pinned(fp)) sync();
    }
    static constexpr size_t kKeepStage = (size_t)1 << 23;   // 64 MiB
    DBuf<double> fstage, stage2;

    void run(int64_t T, const double* x) {
        REQUIRE(n_rows > 0, "mc_load_forcing must be called before mc_run");
        REQUIRE(x != nullptr, "x must not be NULL");
        for (int64_t t = 1; t < T; ++t)
            REQUIRE(!(x[t] < x[t - 1]), "step times x must be non-decreasing");
        std::vector<int4> tab(T);
        for (int64_t t = 0; t < T; ++t) {  // nutils.py:21-33
            const double xt = x[t];
            const int64_t ix = searchsorted_left(xp.data(), n_rows, xt);
            if (ix == 0) {
                tab[t] = step_entry(0, 0, 0.0);
            } else if (ix >= n_rows) {
                tab[t] = step_entry((int)(n_rows - 1), (int)(n_rows - 1), 0.0);
            } else {
                // the device forms (1 - frac) * f[ix-1] + frac * f[ix] exactly as numpy does
                const double dx0 = xt - xp[ix - 1];
                const double dx1 = xp[ix] - xt;
                tab[t] = step_entry((int)(ix - 1), (int)ix, dx0 / (dx0 + dx1));
            }
        }
        run_tables(T, F.p, n_rows, tab);
    }

    void step(const double* q, double* i_out, double* o_out) {
        REQUIRE(plan.n == 0 || (q && i_out && o_out), "q/outputs must not be NULL");
        const int64_t n = plan.n;
        Fstep.reserve((size_t)(std::max<int64_t>(plan.nslots, 1) * E));
        if (n) {
            to_slots(q, Fstep, E);
            HIPC(hipMemsetAsync(nf.p + 2, 0, sizeof(int32_t), stream));
            HIPC(mcr::launch_flag_nonfinite(Fstep.p, plan.nslots * E, nf.p + 2, stream));
        }
        run_tables(1, Fstep.p, 1, std::vector<int4>(1, step_entry(0, 0, 0.0)));
        if (n) {  // the new state is the output of the step
            from_slots(st_o, o_out, E);
            from_slots(st_i, i_out, E);
        }
        sync();
    }

    void fetch(int64_t t0, int64_t t1, double* oo, double* io) {
        settle();
        REQUIRE(T_out > 0, "no outputs: call mc_run first");
        REQUIRE(0 <= t0 && t0 <= t1 && t1 <= T_out, "step range out of bounds");
        const int64_t n = plan.n;
        const int64_t k = t1 - t0;
        if (n == 0 || k == 0) return;
        outT.reserve((size_t)(n * k * E));
        for (int c = 0; c < 2; ++c) {
            double* dst = c == 0 ? oo : io;
            if (!dst) continue;
            gather_block(t0, t1, c == 0 ? outT.p : nullptr, c == 1 ? outT.p : nullptr);
            HIPC(hipMemcpyAsync(dst, outT.p, n * k * E * sizeof(double), hipMemcpyDeviceToHost,
                                stream));
            sync();
        }
    }

    // ---- asynchronous fetches (mc_fetch_outputs_async / mc_fetch_wait): the drop-in API yields
    // the steps of a block while the next blocks are still being copied.  Each call gathers the
    // block's outflows and inflows into a staging pair of a two-slot ring, forms their row
    // digests, and queues the copies on a copy stream of their own; a ticket (an event on the
    // copy stream) marks the end.  The gathers of block b + 1 run while block b is copied (one
    // stream serialised them: 36 GB/s over PCIe against ~50 for back-to-back copies); a slot is
    // gathered into again only after its previous copy (event).
    DBuf<double> aO[2], aI[2];
    DBuf<uint64_t> aDg[2];
    hipStream_t cstream = nullptr;
    hipEvent_t a_ready[2] = {nullptr, nullptr}, a_copied[2] = {nullptr, nullptr};
    bool a_used[2] = {false, false};
    int64_t a_seq = 0;
    std::vector<hipEvent_t> fetch_ev;     // ticket -> event
    std::vector<char> fetch_live;
    int64_t fetch_pending = 0;
    int64_t fetch_async(int64_t t0, int64_t t1, double* oo, double* io, uint64_t* dgo,
                        uint64_t* dgi) {
        settle();
        REQUIRE(T_out > 0, "no outputs: call mc_run first");
        REQUIRE(0 <= t0 && t0 <= t1 && t1 <= T_out, "step range out of bounds");
        const int64_t n = plan.n, k = t1 - t0;
        const size_t cells = (size_t)std::max<int64_t>(n * k * E, 1);
        // small blocks (sub-basin sessions) gain nothing from the overlap: slot 0, the session
        // stream, no copy stream of their own
        const bool ring = cells * sizeof(double) >= ((size_t)4 << 20);
        if (ring && !cstream) {
            HIPC(hipStreamCreateWithFlags(&cstream, hipStreamNonBlocking));
            for (int q = 0; q < 2; ++q) {
                HIPC(hipEventCreateWithFlags(&a_ready[q], hipEventDisableTiming));
                HIPC(hipEventCreateWithFlags(&a_copied[q], hipEventDisableTiming));
            }
        }
        const int r = ring ? (int)(a_seq++ & 1) : 0;
        if (!ring && fetch_pending > 0 &&
            (aO[0].cap < cells || aI[0].cap < cells || aDg[0].cap < (size_t)(2 * k)))
            HIPC(hipStreamSynchronize(stream));   // a pending direct copy may read the old slot
        if (a_used[r]) {
            // the slot's previous copy must be done before it is gathered into (stream order),
            // and before its buffers are replaced (host order)
            if (aO[r].cap < cells || aI[r].cap < cells || aDg[r].cap < (size_t)(2 * k))
                HIPC(hipEventSynchronize(a_copied[r]));
            else
                HIPC(hipStreamWaitEvent(stream, a_copied[r], 0));
        }
        aO[r].reserve(cells);
        aI[r].reserve(cells);
        aDg[r].reserve((size_t)std::max<int64_t>(2 * k, 1));
        bool any = false;
        const bool want_o = oo || dgo, want_i = io || dgi;
        if (n > 0 && k > 0 && (want_o || want_i)) {
            gather_block(t0, t1, want_o ? aO[r].p : nullptr, want_i ? aI[r].p : nullptr);
            any = true;
        }
        for (int c = 0; c < 2 && any; ++c) {
            uint64_t* dg = c == 0 ? dgo : dgi;
            if (dg)
                HIPC(mcr::launch_row_digests(c == 0 ? aO[r].p : aI[r].p, k, n * E,
                                             aDg[r].p + c * k, stream));
        }
        hipStream_t cs = stream;
        if (ring) {
            HIPC(hipEventRecord(a_ready[r], stream));
            HIPC(hipStreamWaitEvent(cstream, a_ready[r], 0));
            cs = cstream;
        }
        for (int c = 0; c < 2 && any; ++c) {
            double* dst = c == 0 ? oo : io;
            uint64_t* dg = c == 0 ? dgo : dgi;
            if (dg)
                HIPC(hipMemcpyAsync(dg, aDg[r].p + c * k, (size_t)k * sizeof(uint64_t),
                                    hipMemcpyDeviceToHost, cs));
            if (dst)
                HIPC(hipMemcpyAsync(dst, c == 0 ? aO[r].p : aI[r].p,
                                    (size_t)(n * k * E) * sizeof(double), hipMemcpyDeviceToHost,
                                    cs));
        }
        if (ring) {
            HIPC(hipEventRecord(a_copied[r], cstream));
            a_used[r] = true;
        }
        int64_t t = 0;
        while (t < (int64_t)fetch_ev.size() && fetch_live[t]) ++t;
        if (t == (int64_t)fetch_ev.size()) {
            hipEvent_t e;
            HIPC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            fetch_ev.push_back(e);
            fetch_live.push_back(0);
        }
        HIPC(hipEventRecord(fetch_ev[t], cs));
        fetch_live[t] = 1;
        ++fetch_pending;
        return t;
    }
    void fetch_wait(int64_t t) {
        REQUIRE(t >= 0 && t < (int64_t)fetch_ev.size() && fetch_live[t], "unknown fetch ticket");
        fetch_live[t] = 0;
        --fetch_pending;
        HIPC(hipEventSynchronize(fetch_ev[t]));
    }

    void fetch_series(double* oo, double* io) {
        settle();
        REQUIRE(T_out > 0, "no outputs: call mc_run first");
        const int64_t n = plan.n;
        if (n == 0) return;
        outT.reserve((size_t)(n * T_out * E));
        const size_t bytes = (size_t)(n * T_out * E) * sizeof(double);
        for (int k = 0; k < 2; ++k) {
            double* dst = k == 0 ? oo : io;
            if (!dst) continue;
            if (out_io)                    // T = 1: [j][0][e] is the step layout
                HIPC(mcr::launch_gather_io(IOb.p, member_win(), pos.p, k == 1, outT.p, n, E,
                                           stream));
            else {
                const OutView ov = out_view();
                HIPC(mcr::launch_gather_series(ov.O, ov.mO, ov.jbase, in_off.p, in_list.p, k == 1,
                                               (int)ov.stride, outT.p, n, T_out, E, stream));
            }
            HIPC(hipMemcpyAsync(dst, outT.p, bytes, hipMemcpyDeviceToHost, stream));
            sync();
        }
    }
};

// ---- C-level communicator: RCCL loaded at first use (no link-time dependency) ---------------
struct Rccl {
    bool tried = false;
    void* h = nullptr;
    decltype(&ncclGetUniqueId) get_id = nullptr;
    decltype(&ncclCommInitRank) init = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclAllToAll) all_to_all = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) err = nullptr;
};
Rccl& rccl() {
    static Rccl R;
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    if (!R.tried) {
        R.tried = true;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            R.h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
            if (R.h) break;
        }
        if (R.h) {
            auto sym = [&](auto& f, const char* n) {
                f = reinterpret_cast<std::remove_reference_t<decltype(f)>>(dlsym(R.h, n));
            };
            sym(R.get_id, "ncclGetUniqueId");
            sym(R.init, "ncclCommInitRank");
            sym(R.destroy, "ncclCommDestroy");
            sym(R.all_gather, "ncclAllGather");
            sym(R.all_to_all, "ncclAllToAll");
            sym(R.group_start, "ncclGroupStart");
            sym(R.group_end, "ncclGroupEnd");
            sym(R.err, "ncclGetErrorString");
        }
    }
    if (!R.h || !R.get_id || !R.init || !R.destroy || !R.all_gather || !R.all_to_all ||
        !R.group_start || !R.group_end || !R.err)
        throw Fail(MC_E_STATE, "RCCL (librccl.so.1) could not be loaded");
    return R;
}
#define NCCLC(call)                                                                    \
    do {                                                                               \
        const ncclResult_t r_ = (call);                                                \
        if (r_ != ncclSuccess) throw Fail(MC_E_HIP, std::string("RCCL: ") + rccl().err(r_)); \
    } while (0)

struct Comm {
    ncclComm_t c = nullptr;
    int nranks = 1, rank = 0;
    hipStream_t side = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    DBuf<double> HX, D, HXall, Dall, send, Xs, Gs, Grecv;
    ~Comm() {
        if (side) (void)hipStreamSynchronize(side);
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
        if (side) (void)hipStreamDestroy(side);
        if (c) (void)rccl().destroy(c);
    }
};
Comm* as_comm(void* h) {
    if (!h) throw Fail(MC_E_INVALID, "null communicator handle");
    return static_cast<Comm*>(h);
}

Net* as_net(void* h) {
    if (!h) throw Fail(MC_E_INVALID, "null session handle");
    return static_cast<Net*>(h);
}

// cache for the stateless mc_ax_bu_f64 mirror: recompiled only when the topology changes
struct AxBuCache {
    std::mutex mu;
    std::unique_ptr<Net> net;
    std::vector<int64_t> endnodes, indegree, heads;
    int device = -1;
};
AxBuCache& axbu_cache() {
    static AxBuCache c;
    return c;
}

}  // namespace

extern "C" {

const char* mc_last_error(void) { return g_err.c_str(); }

int mc_version(void) { return 101; }

int mc_plan_create(int64_t n, const int64_t* endnodes, const int64_t* indegree,
                   const int64_t* headwaters, int64_t n_head, const mc_plan_params* params,
                   void** plan_out) {
    return guarded([&] {
        REQUIRE(plan_out, "plan_out must not be NULL");
        check_topology_args(n, endnodes, indegree, headwaters, n_head);
        auto p = std::make_unique<mcr::Plan>();
        const std::string err =
            mcr::build_plan(n, endnodes, indegree, headwaters, n_head, to_params(params), *p);
        if (!err.empty()) throw Fail(MC_E_TOPOLOGY, err);
        *plan_out = p.release();
    });
}

int mc_plan_get_info(const void* plan, mc_plan_info* info) {
    return guarded([&] {
        REQUIRE(plan && info, "null argument");
        fill_info(*static_cast<const mcr::Plan*>(plan), info);
    });
}

int mc_plan_export(const void* plan, int64_t* rank, int64_t* pos, int32_t* G,
                   int64_t* slot_reach) {
    return guarded([&] {
        REQUIRE(plan, "null plan");
        const mcr::Plan& P = *static_cast<const mcr::Plan*>(plan);
        if (rank) std::memcpy(rank, P.rank.data(), P.rank.size() * sizeof(int64_t));
        if (pos) std::memcpy(pos, P.pos.data(), P.pos.size() * sizeof(int64_t));
        if (G) std::memcpy(G, P.G.data(), P.G.size() * sizeof(int32_t));
        if (slot_reach)
            std::memcpy(slot_reach, P.slot_reach.data(), P.slot_reach.size() * sizeof(int64_t));
    });
}

int mc_plan_export_links(const void* plan, uint8_t* flags, uint8_t* up_cnt, uint64_t* up4,
                         int32_t* ext_off, int64_t* ext_src, int32_t* ext_g) {
    return guarded([&] {
        REQUIRE(plan, "null plan");
        const mcr::Plan& P = *static_cast<const mcr::Plan*>(plan);
        auto cp = [](auto* dst, const auto& v) {
            if (dst && !v.empty()) std::memcpy(dst, v.data(), v.size() * sizeof(v[0]));
        };
        cp(flags, P.flags);
        cp(up_cnt, P.up_cnt);
        cp(up4, P.up4);
        cp(ext_off, P.ext_off);
        cp(ext_src, P.ext_src);
        cp(ext_g, P.ext_g);
    });
}

int mc_plan_export_local(const void* plan, int32_t* lx_off, int32_t* lx_src) {
    return guarded([&] {
        REQUIRE(plan, "null plan");
        const mcr::Plan& P = *static_cast<const mcr::Plan*>(plan);
        if (lx_off && !P.lx_off.empty())
            std::memcpy(lx_off, P.lx_off.data(), P.lx_off.size() * sizeof(int32_t));
        if (lx_src && !P.lx_src.empty())
            std::memcpy(lx_src, P.lx_src.data(), P.lx_src.size() * sizeof(int32_t));
    });
}

int mc_plan_schedule(const void* plan, int64_t T, int64_t* n_launch, int64_t* n_list,
                     int64_t* off, int32_t* list) {
    return guarded([&] {
        REQUIRE(plan && n_launch && n_list, "null argument");
        REQUIRE(T >= 1, "T must be >= 1");
        std::vector<int32_t> l;
        std::vector<int64_t> o;
        const int64_t nl = mcr::active_schedule(*static_cast<const mcr::Plan*>(plan), T, l, o);
        *n_launch = nl;
        *n_list = (int64_t)l.size();
        if (off) std::memcpy(off, o.data(), o.size() * sizeof(int64_t));
        if (list && !l.empty()) std::memcpy(list, l.data(), l.size() * sizeof(int32_t));
    });
}

int mc_plan_destroy(void* plan) {
    return guarded([&] { delete static_cast<mcr::Plan*>(plan); });
}

int mc_net_create(int64_t n, const int64_t* endnodes, const int64_t* indegree,
                  const int64_t* headwaters, int64_t n_head, const mc_plan_params* params,
                  void** net_out) {
    return guarded([&] {
        REQUIRE(net_out, "net_out must not be NULL");
        check_topology_args(n, endnodes, indegree, headwaters, n_head);
        auto net = std::make_unique<Net>();
        net->init(n, endnodes, indegree, headwaters, n_head, to_params(params));
        *net_out = net.release();
    });
}

int mc_net_destroy(void* net) {
    return guarded([&] { delete static_cast<Net*>(net); });
}

int mc_net_get_info(const void* net, mc_plan_info* info) {
    return guarded([&] {
        REQUIRE(net && info, "null argument");
        fill_info(static_cast<const Net*>(net)->plan, info);
    });
}

int mc_net_set_stream(void* net, void* s) {
    return guarded([&] {
        Net* N = as_net(net);
        N->sync();
        N->stream = s ? static_cast<hipStream_t>(s) : N->own;
    });
}

int mc_net_set_members(void* net, int64_t members) {
    return guarded([&] { as_net(net)->set_members(members); });
}

int mc_net_get_members(const void* net, int64_t* members) {
    return guarded([&] {
        REQUIRE(net && members, "null argument");
        *members = static_cast<const Net*>(net)->E;
    });
}

int mc_apply_gain(void* net, const double* gain) {
    return guarded([&] { as_net(net)->apply_gain(gain); });
}

int mc_enkf_analysis(void* net, int64_t m, const int64_t* gauges, const double* y,
                     const double* R) {
    return guarded([&] { as_net(net)->enkf_analysis(m, gauges, y, R); });
}

int mc_ens_slice_size(const void* net, int64_t nranks, int64_t* S) {
    return guarded([&] {
        REQUIRE(net && S && nranks >= 1, "bad argument");
        *S = static_cast<const Net*>(net)->slice_size(nranks);
    });
}

int mc_ens_gauges(void* net, int64_t m, const int64_t* gauges, const double* y, double* HX,
                  double* D) {
    return guarded([&] { as_net(net)->ens_gauges(m, gauges, y, HX, D); });
}

int mc_ens_pack(void* net, int64_t nranks, double* send) {
    return guarded([&] { as_net(net)->ens_pack(nranks, send); });
}

int mc_ens_slice_update(void* net, int64_t nranks, int64_t m, const double* Xs,
                        const double* HXall, const double* Dall, const double* R, double* Gs) {
    return guarded([&] { as_net(net)->ens_slice_update(nranks, m, Xs, HXall, Dall, R, Gs); });
}

int mc_ens_weights(void* net, int64_t nranks, int64_t m, const double* HXall,
                   const double* Dall, const double* R) {
    return guarded([&] { as_net(net)->ens_weights(nranks, m, HXall, Dall, R); });
}

int mc_ens_increments(void* net, int64_t nranks, const double* Xs, double* Gs) {
    return guarded([&] { as_net(net)->ens_increments(nranks, Xs, Gs); });
}

int mc_ens_unpack_apply(void* net, int64_t nranks, const double* Grecv) {
    return guarded([&] { as_net(net)->ens_unpack_apply(nranks, Grecv); });
}

int mc_comm_unique_id(uint8_t* id128) {
    return guarded([&] {
        REQUIRE(id128, "id must not be NULL");
        static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
        ncclUniqueId id;
        NCCLC(rccl().get_id(&id));
        std::memcpy(id128, &id, sizeof(id));
    });
}

int mc_comm_init(int32_t nranks, int32_t rank, const uint8_t* id128, void** comm) {
    return guarded([&] {
        REQUIRE(comm && id128, "null argument");
        REQUIRE(nranks >= 1 && 0 <= rank && rank < nranks, "rank out of range");
        *comm = nullptr;
        auto C = std::make_unique<Comm>();
        C->nranks = nranks;
        C->rank = rank;
        ncclUniqueId id;
        std::memcpy(&id, id128, sizeof(id));
        NCCLC(rccl().init(&C->c, nranks, id, rank));
        HIPC(hipStreamCreateWithFlags(&C->side, hipStreamNonBlocking));
        for (hipEvent_t& e : C->ev) HIPC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        *comm = C.release();
    });
}

int mc_comm_destroy(void* comm) {
    return guarded([&] { delete static_cast<Comm*>(comm); });
}

int mc_ens_analysis_dist(void* net, void* comm, int64_t m, const int64_t* gauges,
                         const double* y_local, const double* R) {
    return guarded([&] {
        Net& N = *as_net(net);
        Comm& C = *as_comm(comm);
        REQUIRE(m >= 1 && gauges && y_local && R, "bad analysis arguments");
        if (N.plan.n == 0) return;
        const int64_t P = C.nranks, E = N.E, S = N.slice_size(P), Et = E * P;
        REQUIRE(Et >= 2, "the ensemble analysis needs at least 2 members");
        const hipStream_t st = N.stream;
        Rccl& R_ = rccl();
        C.HX.reserve((size_t)(E * m));
        C.D.reserve((size_t)(E * m));
        C.send.reserve((size_t)(P * E * S));
        C.HXall.reserve((size_t)(Et * m));
        C.Dall.reserve((size_t)(Et * m));
        C.Xs.reserve((size_t)(P * E * S));
        C.Gs.reserve((size_t)(Et * S));
        C.Grecv.reserve((size_t)(Et * S));
        N.ens_gauges(m, gauges, y_local, C.HX.p, C.D.p);
        N.ens_pack(P, C.send.p);
        // (one rank: the collectives are copies; the program is the same)
        NCCLC(R_.group_start());
        NCCLC(R_.all_gather(C.HX.p, C.HXall.p, (size_t)(E * m), ncclDouble, C.c, st));
        NCCLC(R_.all_gather(C.D.p, C.Dall.p, (size_t)(E * m), ncclDouble, C.c, st));
        NCCLC(R_.group_end());
        // the member -> slice all-to-all travels on the side stream while the weights form
        HIPC(hipEventRecord(C.ev[0], st));
        HIPC(hipStreamWaitEvent(C.side, C.ev[0], 0));
        NCCLC(R_.all_to_all(C.send.p, C.Xs.p, (size_t)(E * S), ncclDouble, C.c, C.side));
        HIPC(hipEventRecord(C.ev[1], C.side));
        N.ens_weights(P, m, C.HXall.p, C.Dall.p, R);
        HIPC(hipStreamWaitEvent(st, C.ev[1], 0));
        N.ens_increments(P, C.Xs.p, C.Gs.p);
        NCCLC(R_.all_to_all(C.Gs.p, C.Grecv.p, (size_t)(E * S), ncclDouble, C.c, st));
        N.ens_unpack_apply(P, C.Grecv.p);
    });
}

int mc_enkf_gain(void* net, int64_t m, const int64_t* gauges, const double* R, double* K_out) {
    return guarded([&] { as_net(net)->enkf_gain(m, gauges, R, K_out); });
}

int mc_set_coeffs(void* net, const double* a, const double* b, const double* c,
                  const double* g) {
    return guarded([&] { as_net(net)->set_coeffs(a, b, c, g); });
}

int mc_set_state(void* net, const double* o, const double* i) {
    return guarded([&] { as_net(net)->set_state(o, i); });
}

int mc_get_state(void* net, double* o, double* i) {
    return guarded([&] {
        Net* N = as_net(net);
        REQUIRE(N->plan.n == 0 || (o && i), "state arrays must not be NULL");
        N->from_slots(N->st_o, o, N->E);
        N->from_slots(N->st_i, i, N->E);
    });
}

int mc_net_copy_state(void* dst_net, const void* src_net) {
    return guarded([&] {
        Net* D = as_net(dst_net);
        Net* S = as_net(const_cast<void*>(src_net));
        REQUIRE(D != S, "source and destination must be different sessions");
        REQUIRE(D->plan.n == S->plan.n, "sessions route different networks (reach counts differ)");
        REQUIRE(D->E == S->E, "sessions hold different member counts");
        const int64_t n = D->plan.n, E = D->E;
        if (n == 0) return;
        S->settle();
        S->settle_gain();
        D->settle_state();
        D->gain_pending = false;         // its state is replaced
        // order: after the source's pending work, on the destination's stream; the source waits
        // for the copy before it may overwrite its state again
        hipEvent_t ev;
        HIPC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        struct EvGuard {
            hipEvent_t e;
            ~EvGuard() { (void)hipEventDestroy(e); }
        } guard{ev};
        HIPC(hipEventRecord(ev, S->stream));
        HIPC(hipStreamWaitEvent(D->stream, ev, 0));
        // one direct slot -> slot permutation per array (the map of this pair of plans is
        // built once and cached on the destination): was a gather into reach order and a
        // scatter, each a full pass (EnKF256: 8.4 ms of hand-overs per horizon)
        const int32_t* map = D->slot_map_from(*S);
        for (int k = 0; k < 2; ++k) {
            const DBuf<double>& from = k ? S->st_i : S->st_o;
            DBuf<double>& to = k ? D->st_i : D->st_o;
            HIPC(mcr::launch_permute_slots(from.p, to.p, map, S->plan.nslots, D->plan.nslots, E,
                                           D->stream));
        }
        D->mark_state();
        HIPC(hipEventRecord(ev, D->stream));
        HIPC(hipStreamWaitEvent(S->stream, ev, 0));
    });
}

int mc_net_lateral_correction(void* dst_net, int64_t dst_reach, const void* src_net,
                              int64_t src_reach, double o_start, double alpha, double beta,
                              double gamma) {
    return guarded([&] {
        Net* D = as_net(dst_net);
        Net* S = as_net(const_cast<void*>(src_net));
        REQUIRE(D != S, "source and destination must be different sessions");
        REQUIRE(D->E == 1 && S->E == 1, "lateral corrections route single-member sessions");
        REQUIRE(0 <= dst_reach && dst_reach < D->plan.n && 0 <= src_reach && src_reach < S->plan.n,
                "reach index out of range");
        REQUIRE(S->T_out > 0 && S->cur && !S->out_io,
                "the source session has no horizon outputs");
        REQUIRE(D->n_rows == S->T_out,
                "the destination's forcing rows must be the source horizon's steps (one input "
                "row per step, as the reference's positional add requires)");
        D->settle_state();
        // order: after the source's run, on the destination's stream; the source waits for the
        // read before it may overwrite its outputs (no host synchronisation)
        hipEvent_t ev;
        HIPC(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        struct EvGuard {
            hipEvent_t e;
            ~EvGuard() { (void)hipEventDestroy(e); }
        } guard{ev};
        HIPC(hipEventRecord(ev, S->stream));
        HIPC(hipStreamWaitEvent(D->stream, ev, 0));
        const auto ov = S->out_view();
        HIPC(mcr::launch_lateral_correction(ov.O, ov.jbase, src_reach, (int)ov.stride,
                                            o_start, alpha, beta, gamma, D->F.p, D->plan.nslots,
                                            D->plan.pos[dst_reach], S->T_out, D->stream));
        HIPC(mcr::launch_flag_nonfinite(D->F.p, D->n_rows * D->plan.nslots, D->nf.p + 1,
                                        D->stream));
        HIPC(hipEventRecord(ev, D->stream));
        HIPC(hipStreamWaitEvent(S->stream, ev, 0));
    });
}

int mc_net_reroutes(const void* net, int64_t* count) {
    return guarded([&] {
        REQUIRE(net && count, "null argument");
        *count = static_cast<const Net*>(net)->reroutes;
    });
}

int mc_step(void* net, const double* o_prev, const double* i_prev, const double* q,
            double* i_out, double* o_out) {
    return guarded([&] {
        Net* N = as_net(net);
        if (o_prev || i_prev) N->set_state(o_prev, i_prev);
        N->step(q, i_out, o_out);
    });
}

int mc_load_forcing(void* net, int64_t n_rows, const double* xp, const double* fp) {
    return guarded([&] { as_net(net)->load_forcing(n_rows, xp, fp); });
}

int mc_load_forcing_series(void* net, int64_t n_rows, const double* xp, const double* fp) {
    return guarded([&] { as_net(net)->load_forcing(n_rows, xp, fp, true); });
}

int mc_run(void* net, int64_t T, const double* x) {
    return guarded([&] { as_net(net)->run(T, x); });
}

int mc_fetch_outputs(void* net, int64_t t0, int64_t t1, double* out_o, double* out_i) {
    return guarded([&] { as_net(net)->fetch(t0, t1, out_o, out_i); });
}

int mc_gather_outputs(void* net, int64_t t0, int64_t t1, double* dev_o, double* dev_i) {
    return guarded([&] {
        Net* N = as_net(net);
        N->settle();
        REQUIRE(N->T_out > 0, "no outputs: call mc_run first");
        REQUIRE(0 <= t0 && t0 <= t1 && t1 <= N->T_out, "step range out of bounds");
        if (N->plan.n == 0 || t1 == t0) return;
        N->gather_block(t0, t1, dev_o, dev_i);
    });
}

int mc_fetch_outputs_async(void* net, int64_t t0, int64_t t1, double* out_o, double* out_i,
                           uint64_t* digest_o, uint64_t* digest_i, int64_t* ticket) {
    return guarded([&] {
        REQUIRE(ticket, "ticket must not be NULL");
        *ticket = as_net(net)->fetch_async(t0, t1, out_o, out_i, digest_o, digest_i);
    });
}

int mc_fetch_wait(void* net, int64_t ticket) {
    return guarded([&] { as_net(net)->fetch_wait(ticket); });
}

int mc_host_digest(const double* rows, int64_t nrows, int64_t n, uint64_t* out) {
    return guarded([&] {
        REQUIRE(nrows >= 0 && n >= 0 && (nrows == 0 || (out && (n == 0 || rows))),
                "bad digest arguments");
        if (nrows == 0) return;
        if (n == 0) {
            std::fill(out, out + nrows, 0);
            return;
        }
        std::vector<const double*> ptrs((size_t)nrows);
        for (int64_t r = 0; r < nrows; ++r) ptrs[(size_t)r] = rows + r * n;
        mcr::host_digest_rows(ptrs.data(), nrows, n, out);
    });
}

int mc_host_digest2(const double* a, const double* b, int64_t n, uint64_t* out2) {
    return guarded([&] {
        REQUIRE(n >= 0 && out2 && (n == 0 || (a && b)), "bad digest arguments");
        if (n == 0) {
            out2[0] = out2[1] = 0;
            return;
        }
        const double* rows[2] = {a, b};
        mcr::host_digest_rows(rows, 2, n, out2);
    });
}

int mc_fetch_series(void* net, double* out_o, double* out_i) {
    return guarded([&] { as_net(net)->fetch_series(out_o, out_i); });
}

int mc_simulate(void* net, int64_t T, const double* x, int64_t n_rows, const double* xp,
                const double* fp, double* out_o, double* out_i) {
    return guarded([&] {
        Net* N = as_net(net);
        N->load_forcing(n_rows, xp, fp);
        N->run(T, x);
        N->fetch(0, T, out_o, out_i);
    });
}

int mc_synchronize(void* net) {
    return guarded([&] { as_net(net)->sync(); });
}

int mc_set_timing(void* net, int enable) {
    return guarded([&] { as_net(net)->timing = enable != 0; });
}

int mc_get_timing(void* net, double* kernel_ms, int64_t* launches, double* run_ms) {
    return guarded([&] {
        Net* N = as_net(net);
        if (kernel_ms) *kernel_ms = N->kernel_ms;
        if (launches) *launches = N->launches;
        if (run_ms) *run_ms = N->run_ms;
    });
}

int mc_reset_timing(void* net) {
    return guarded([&] {
        Net* N = as_net(net);
        N->kernel_ms = N->run_ms = 0.0;
        N->launches = 0;
    });
}

int mc_set_mode(void* net, int mode) {
    return guarded([&] {
        REQUIRE(mode >= 0 && mode <= 2,
                "mode must be 0 (auto), 1 (multi-launch) or 2 (dataflow; one-step ensemble runs "
                "as member-dataflow launches)");
        as_net(net)->mode = mode;
    });
}

int mc_set_flow_patience(void* net, int64_t wall_ticks) {
    return guarded([&] {
        Net* N = as_net(net);
        N->patience = wall_ticks == 0 ? mcr::kFlowPatience : std::max<int64_t>(wall_ticks, 0);
    });
}

int mc_probe_tick_floor(int32_t slots, int32_t chain, int64_t ticks, double* ns_per_tick) {
    return guarded([&] {
        REQUIRE(ns_per_tick && ticks > 0 && ticks % mcr::kChunk == 0 && ticks < (1ll << 30),
                "ticks must be a positive multiple of 8");
        REQUIRE(((slots == 192 || slots == 384) && chain == 2) || (slots == 64 && chain == 1),
                "instantiated: (192, 2), (384, 2), (64, 1)");
        int dev = 0, cus = 0;
        HIPC(hipGetDevice(&dev));
        HIPC(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        // two workgroups per CU as the Texas launch runs them; the small-network shape (64, 1)
        // one per CU (its launches hold a few workgroups)
        const int grid = (slots == 192 ? 2 : 1) * cus;
        hipStream_t s = nullptr;
        HIPC(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        struct Guard {
            hipStream_t s;
            hipEvent_t e0 = nullptr, e1 = nullptr;
            ~Guard() {
                if (e0) (void)hipEventDestroy(e0);
                if (e1) (void)hipEventDestroy(e1);
                (void)hipStreamSynchronize(s);
                (void)hipStreamDestroy(s);
            }
        } g{s};
        DBuf<double> out;
        out.reserve((size_t)grid * slots);
        HIPC(hipEventCreate(&g.e0));
        HIPC(hipEventCreate(&g.e1));
        HIPC(mcr::probe_tick_floor(slots, chain, grid, 64, s, out.p));     // warm-up
        HIPC(hipEventRecord(g.e0, s));
        HIPC(mcr::probe_tick_floor(slots, chain, grid, (int)ticks, s, out.p));
        HIPC(hipEventRecord(g.e1, s));
        HIPC(hipEventSynchronize(g.e1));
        float ms = 0.f;
        HIPC(hipEventElapsedTime(&ms, g.e0, g.e1));
        *ns_per_tick = (double)ms * 1e6 / (double)ticks;
    });
}

int mc_get_mode(void* net, int* mode, int* last_path) {
    return guarded([&] {
        Net* N = as_net(net);
        if (mode) *mode = N->mode;
        if (last_path) *last_path = N->last_path;
    });
}

int mc_set_trace(void* net, int enable) {
    return guarded([&] { as_net(net)->trace = enable != 0; });
}

int mc_get_trace(void* net, int64_t* out, int64_t cap, int64_t* n_records, int64_t* clock_khz) {
    return guarded([&] {
        Net* N = as_net(net);
        const int64_t m = (int64_t)N->trace_launch.size();
        if (n_records) *n_records = m;
        if (clock_khz) {
            int khz = 0;
            HIPC(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, N->device));
            *clock_khz = khz;
        }
        if (!out || cap <= 0 || m == 0) return;
        const int W = mcr::kTraceWords;
        std::vector<int64_t> raw(W * (size_t)m);
        N->sync();
        HIPC(hipMemcpy(raw.data(), N->trace_buf.p, raw.size() * sizeof(int64_t),
                       hipMemcpyDeviceToHost));
        const std::vector<int32_t>& list = N->trace_wg;
        for (int64_t r = 0; r < std::min(cap, m); ++r) {
            int64_t* o = out + 8 * r;
            const int64_t* q = raw.data() + W * r;
            o[0] = N->trace_launch[r];
            o[1] = list[r];
            o[2] = q[0];
            o[3] = q[1];
            o[4] = q[2];
            o[5] = q[3];
            o[6] = q[4];
            o[7] = q[5];
        }
    });
}

int mc_ax_bu_f64(int64_t n, const int64_t* heads, int64_t n_head, const int64_t* endnodes,
                 const double* alpha, const double* beta, const double* chi, const double* gamma,
                 const double* i_prev, const double* o_prev, const double* q,
                 const int64_t* indegree, double* i_out, double* o_out) {
    return guarded([&] {
        check_topology_args(n, endnodes, indegree, heads, n_head);
        REQUIRE(n == 0 || (alpha && beta && chi && gamma && i_prev && o_prev && q && i_out &&
                           o_out),
                "null array argument");
        AxBuCache& c = axbu_cache();
        std::lock_guard<std::mutex> lock(c.mu);
        int dev = 0;
        HIPC(hipGetDevice(&dev));
        const bool same = c.net && c.device == dev && (int64_t)c.endnodes.size() == n &&
                          (int64_t)c.heads.size() == n_head &&
                          std::equal(endnodes, endnodes + n, c.endnodes.begin()) &&
                          std::equal(indegree, indegree + n, c.indegree.begin()) &&
                          std::equal(heads, heads + n_head, c.heads.begin());
        if (!same) {
            c.net.reset();
            auto net = std::make_unique<Net>();
            net->init(n, endnodes, indegree, heads, n_head, mcr::PlanParams());
            c.net = std::move(net);
            c.endnodes.assign(endnodes, endnodes + n);
            c.indegree.assign(indegree, indegree + n);
            c.heads.assign(heads, heads + n_head);
            c.device = dev;
        }
        Net* N = c.net.get();
        N->set_coeffs(alpha, beta, chi, gamma);
        N->set_state(o_prev, i_prev);
        N->step(q, i_out, o_out);
    });
}

}  // extern "C"
