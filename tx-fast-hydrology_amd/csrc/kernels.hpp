// Device-side entry points of the Muskingum routing engine (gfx950).  Launchers are plain host
// functions so the C-ABI layer (capi.cpp) stays free of kernel syntax.
//
// Output layout ("workgroup windows").  Workgroup w owns the ticks [gmin[w], gmax[w] + T) of the
// space-time schedule; its outputs are stored tick-major inside that window:
//     O[wbase[w] + (tick - gmin[w]) * RS + slot - w * RS]      (RS = chain * slots)
// so the 64 lanes of a wave write one contiguous 512-byte row per tick.  Only the cells of
// slots active at the tick are stored (the multi-launch kernel masks the rest: ens64 writes
// -23 %, 5 % faster); the dataflow kernel's helper copies whole rows (masking its copies cost
// 3 %).  (Per-wave "segment" windows wrote 10 % (det) / 30 % (ens64) fewer bytes but ran
// 1-2 % / 4-6 % slower: DESIGN.md §6, round 3.)  Inflows are not stored:
// i[j][t] = ((0 + o[u1][t]) + o[u2][t]) + ... over j's inflow list (plan.hpp) is recomputed
// bit-exactly wherever it is needed (fetches, final state).  A reach that feeds a
// reach of another cluster (an "external input" of the consumer's workgroup) also writes its
// outflow to a step-contiguous stream XS[e][t], which the consumer reads coalesced.  Step t of
// the reach in slot d lives at tick G[d] + t, i.e. at  jbase[j] + t * RS  for its caller index j
// (jbase is computed per horizon by launch_window_index).
#pragma once


#include <hip/hip_runtime.h>

#include <cstdint>

#include "digest.hpp"

namespace mcr {

// (lanes, node slots per lane) the kernels are instantiated for (plan slots, chain).
// Multi-launch sweep:
#define MCR_SLOT_SHAPES(X)                                                             \
    X(64, 1) X(64, 2) X(128, 2) X(192, 2) X(256, 2) X(384, 2) X(448, 2) X(512, 2) X(64, 3) X(128, 3) \
    X(192, 3) X(256, 3) X(64, 4) X(128, 4) X(192, 4) X(256, 4)
// Dataflow kernels (compute waves + the helper wave fill whole wave slots on the SIMDs):
// (4 positions per lane take one wave per SIMD: at most 192 lanes + the helper)
#define MCR_FLOW_SHAPES(X)                                                             \
    X(64, 1) X(64, 2) X(128, 2) X(192, 2) X(256, 2) X(384, 2) X(448, 2) X(64, 3) X(128, 3) X(192, 3) \
    X(256, 3) X(64, 4) X(128, 4) X(192, 4)
// ... of which these also run chunk-synchronous plans (plan.hpp sync: one workgroup barrier per
// kWaveSlack ticks)
#define MCR_SYNC_SHAPES(X) X(64, 1) X(64, 2) X(128, 2) X(192, 2) X(256, 2) X(192, 3)

// Ticks whose lateral inflow is formed in one burst (and whose forcing rows are prefetched
// together).  Launch lengths (`tile`) are multiples of it.
constexpr int kChunk = 8;


// Dataflow kernel (flow.hip): external inputs per workgroup it supports, longest step table it
// keeps in LDS, minimum cross-cluster slack (the helper stages the next chunk, so producers must
// be more than one chunk ahead of it).
constexpr int kFlowMaxExt = 128;
constexpr int kFlowMaxT = 1024;
constexpr int kFlowMinSlack = 2 * kChunk;
constexpr int64_t kFlowPatience = 200000000;   // default: 2 s of the 100 MHz wall clock

// launch trace record of one workgroup: wall clock at start / loop start / end, hw id, shader
// clock at loop start / end
constexpr int kTraceWords = 6;

// Everything the wavefront kernel reads, by value.  Per-slot arrays are in device-slot order
// (plan.hpp).
struct WaveArgs {
    const int32_t* active;        // workgroup ids of this launch
    const int32_t* G;             // [nslots]
    const uint8_t* flags;         // [nslots]
    const uint8_t* up_cnt;        // [nslots]
    const uint64_t* up4;          // [nslots]
    const int32_t* ext_off;       // [nwg + 1]
    const int32_t* xid;           // [nslots] external input fed by the slot's reach, -1 if none
    const int16_t* lx;            // [nslots] sync plans: local external input (XE column of the
                                  // slot's own workgroup) fed kWaveSlack ticks later, -1 if none
    const int32_t* lx_off;        // [nwg + 1] sync plans: local inputs of each workgroup (their
    const int32_t* lx_src;        // XE columns follow its granule inputs) and producer slots
    const int32_t* ext_g;         // G of the consuming reach
    const double* alpha;          // [nslots]
    const double* beta;
    const double* chi;
    const double* gamma;
    // routing state {o_t_next, i_t_next} [nslots]: read at a workgroup's first tick of a
    // launch, written back at its last, so it holds step t_last of the previous launch and the
    // final state after the horizon (the session state, no separate gather)
    double* st_o;
    double* st_i;
    // dataflow horizon (flow.hip, one member): the state after the horizon goes here (the
    // session keeps its input state until the run is known to have completed)
    double* st_o_out;
    double* st_i_out;
    const double* F;              // forcing rows in slot order [n_rows][nslots]
    const int4* stab;             // per step {row_lo, row_hi, frac (f64)}; clamped: {r, r, 0}
    const int32_t* wg_gmin;       // [nwg] tick range of each workgroup
    const int32_t* wg_gmax;
    const int64_t* wbase;         // [nwg] window base of each workgroup in O (member dataflow:
                                  // of its member window, MemberWin)
    double* O;                    // workgroup windows of outflows (see above)
    // ensemble members (grid y; multi-launch kernel): element strides between members of the
    // member-major arrays F, O, XS and of st_o / st_i (in slots)
    int64_t mF, mO, mX, mS;
    double* XS;                   // external-input streams [n_ext][T]: step t of each source
    int64_t* trace;               // optional launch trace, kTraceWords per workgroup (NULL = off)
    // dataflow kernel (flow.hip) only
    uint32_t* XG;                 // external-input granules [n_ext][T] x {lo, epoch, hi, epoch}
    uint32_t xg_bytes;            // size of XG in bytes (< 2^31)
    uint32_t epoch;               // tag of this run's granules (never 0)
    int32_t* status;              // bit 0: a wait gave up; bit 1: a partial sum met a non-finite
                                  // value in the fast form (the horizon is re-routed exactly)
    // non-finite flags {state, forcing} (device, stream-ordered): when both are 0 the dataflow
    // kernel runs its fast form, which lets partial sums carry a state (exact for finite values);
    // its epilogue sets the state flag when the new state holds a non-finite value
    int32_t* nf;                  // the state flag
    const int32_t* nff;           // the flag of the forcing buffer this run reads
    int64_t patience;             // wall-clock (100 MHz) ticks a wait polls before giving up
    const double* Qm;             // member dataflow: lateral inflow [E][nslots] of the step
    const double* IO;             // member dataflow: state {o, i} (staging cells, MemberWin)
    int32_t mskew;                // member dataflow: tick-major member windows (in wbase)
    int64_t nslots;
    int32_t n_rows;
    int32_t T;
    int32_t kappa0;               // first tick of this launch (multiple of kChunk)
    int32_t tile;                 // ticks in this launch (multiple of kChunk)
    int32_t table_cap;            // LDS entries reserved for the step-table window
    int32_t ext_cap;              // LDS rows reserved for external inputs
};

// LDS bytes of the multi-launch kernel for `slots` lanes (chain * slots node slots): the
// parity double buffer XB [RS + 1][2] f64, forcing rows FR [RS][3] f64, the step-table window
// and the external inputs of the launch (kernels.hip).  Over-allocating it costs resident
// workgroups: 64 B per slot here (the flow kernel's tick planes) made Texas ens64 18.8 ms
// instead of 12.7.
inline size_t wavefront_lds_bytes(int slots, int chain, int table_cap, int ext_cap, int tile) {
    const size_t rs = (size_t)chain * slots;
    return 16 * (rs + 1) + 24 * rs + 16 * (size_t)table_cap + 8 * (size_t)ext_cap * tile;
}

// dataflow kernel tick plane (flow.hip): every node slot, the zero slot and two chunk ring
// slots of external inputs, 8 bytes each, padded to 16 bytes (the helper wave copies the node
// slots of a plane to the output window with 16-byte LDS reads)
constexpr unsigned flow_plane_bytes(int rs) {
    return ((unsigned)(rs + 1 + 2 * kFlowMaxExt) * 8u + 15u) & ~15u;
}

inline size_t flow_lds_bytes(int slots, int chain, int T, int ext_cap) {
    (void)ext_cap;                               // external columns are sized for kFlowMaxExt
    const size_t rs = (size_t)chain * slots;
    return 8 * (size_t)flow_plane_bytes((int)rs) + 24 * rs + 16 * (size_t)T + 4 * kFlowMaxExt;
}

// One launch for the whole horizon; grid = every workgroup (all must be co-resident).
// sync: the plan is chunk-synchronous (plan.hpp; shapes MCR_SYNC_SHAPES)
hipError_t launch_flow(const WaveArgs& a, int grid, int slots, int chain, size_t lds_bytes,
                       bool dense, bool sync, hipStream_t s);
// Resident workgroups per CU of the dataflow kernel at this LDS size.
hipError_t flow_occupancy(int slots, int chain, bool dense, bool sync, size_t lds_bytes,
                          int* blocks_per_cu);

// Member dataflow (flow.hip): ONE step of E ensemble members as one resident launch.  Member e
// of node slot d runs at tick G[d] + e (the members take the place of the steps of a horizon;
// a.T = E), reading its state from a.IO and its lateral inflow from a.Qm (launch_member_inputs)
// and writing the member's new {o, i} in their place; launch_member_unpack then forms the
// session state from them.
hipError_t launch_flow_members(const WaveArgs& a, int grid, int slots, int chain,
                               size_t lds_bytes, bool sync, hipStream_t s);
hipError_t flow_members_occupancy(int slots, int chain, bool sync, size_t lds_bytes,
                                  int* blocks_per_cu);
// Tick-major member windows of a member-dataflow step: workgroup w stages the (slot d, member
// e) it processes at tick k = G[d] + e in row k - gmin[w] of its window, wbase[w] + row * rs +
// (d - w rs) (rs = chain * slots node slots per row; rows gmin[w] .. gmax[w] + E - 1), so every
// load and store of a tick in the member kernel is one contiguous row.
// skew = false: member-major cells e * ns + d instead (small ensembles).
struct MemberWin {
    const int64_t* wbase;      // [nwg] window base (cells)
    const int32_t* G;          // [nslots]
    const int32_t* gmin;       // [nwg]
    const uint8_t* flags;      // [nslots] (padding slots are not staged)
    int64_t rs;
    int64_t ns;
    bool skew;
};
// Inputs of a member-dataflow step at the member-window cells: IO = {o, i} of the session
// state (16 B per cell, one load per slot and tick) and Qm = the step's interpolated lateral
// inflow of the member (the kernels' formula: (1 - frac) F[e][lo][d] + frac F[e][hi][d]).
// With gain.G non-NULL the pending analysis increments are applied on the way, exactly as
// launch_apply_gain would have applied them to the state first (o + (0 + G), i + the one-hop
// fold of the routed upstreams' 0 + G): the EnKF cycle's apply_gain pass is folded in here.
struct PendingGain {
    const double* G = nullptr;       // [E][nslots] increments (NULL: none)
    const int32_t* up_off = nullptr; // routed upstream slots of each slot, rank order (CSR)
    const int32_t* up = nullptr;
    // scratch [E][nslots] (may be NULL; used by the LDS-ring staging): the one-hop inflow
    // increments of every (slot, member)
    // are formed into it first by a slot-parallel pass (coalesced upstream reads), so the
    // staging kernel reads one value per cell instead of gathering the upstream increments
    double* gi = nullptr;
};
hipError_t launch_member_inputs(const double* F, int64_t mF, int64_t nslots, int n_rows,
                                int4 ent, const double* st_o, const double* st_i, double* IO,
                                double* Qm, int64_t E, const MemberWin& mw, hipStream_t s,
                                const PendingGain& gain = PendingGain());
// After a member-dataflow step (which leaves each member's new {o, i} in IO): the session state
// st_o / st_i.  IO keeps the step's outputs until the next run; launch_gather_io reads them in
// caller order (out[j][e], the outflow or the inflow).
hipError_t launch_member_unpack(const double* IO, const MemberWin& mw, double* st_o,
                                double* st_i, int64_t nslots, int64_t E, hipStream_t s);
hipError_t launch_gather_io(const double* IO, const MemberWin& mw, const int64_t* pos,
                            bool inflow, double* out, int64_t n, int64_t E, hipStream_t s);

// Latency floor of the dataflow tick (flow.hip tick_floor): `ticks` ticks of the bare per-tick
// chain (LDS inputs, chained updates, LDS outputs, barrier) on `grid` workgroups of the
// (slots, chain) shape; out: grid * slots doubles.  (192, 2) and (384, 2) are instantiated.
hipError_t probe_tick_floor(int slots, int chain, int grid, int ticks, hipStream_t s,
                            double* out);

// dense: the step table has a kChunk-step window spanning more than 3 forcing rows.
// members: ensemble members (grid y); member strides are in `a`.
hipError_t launch_wavefront(const WaveArgs& a, int grid, int slots, int chain, size_t lds_bytes,
                            bool dense, int members, hipStream_t s);
// Ensemble sweep with mb members per workgroup instance (members.hip): the multi-launch
// protocol of launch_wavefront for classic plans, non-dense step tables and E % mb == 0.
size_t members_lds_bytes(int slots, int chain, int table_cap, int ext_cap, int mb);
bool members_shape_ok(int slots, int chain, int mb);
hipError_t launch_members(const WaveArgs& a, int grid, int slots, int chain, size_t lds_bytes,
                          int members, int mb, hipStream_t s);
// Is (slots, chain) instantiated for the multi-launch sweep / the dataflow kernels?
bool wavefront_shape_ok(int slots, int chain);
bool flow_shape_ok(int slots, int chain, bool sync = false);

// Device coefficients by slot kind (partial sums alpha = 1, unrouted reaches and padding 0;
// kernels.hip set_slot_coeffs), applied after every coefficient upload
// flag = 1 when some src[0 .. n) is NaN or +-Inf (otherwise the flag is left as it is)
hipError_t launch_flag_nonfinite(const double* src, int64_t n, int32_t* flag, hipStream_t s);
hipError_t launch_set_slot_coeffs(const uint8_t* flags, double* alpha, double* beta, double* chi,
                                  double* gamma, int64_t nslots, hipStream_t s);
// Layout conversions between the caller (reach order, member innermost: [n][E]) and the device
// (slot order, member-major: [E][nslots]).  E = 1 is the deterministic case.
// dst[e][d] = src[slot_reach[d]][e]  (0 for padding slots)
hipError_t launch_scatter_to_slots(const double* src, double* dst, const int64_t* slot_reach,
                                   int64_t nslots, int64_t E, hipStream_t s);
// dst[j][e] = src[e][pos[j]]
hipError_t launch_permute_slots(const double* src, double* dst, const int32_t* map,
                                int64_t ns_src, int64_t ns_dst, int64_t E, hipStream_t s);
hipError_t launch_gather_from_slots(const double* src, double* dst, const int64_t* pos,
                                    int64_t n, int64_t nslots, int64_t E, hipStream_t s);
// F[e][r][d] = fp[r][slot_reach[d]][e]  (forcing table to slot order; 0 for padding slots)
hipError_t launch_forcing_to_slots(const double* fp, double* F, const int64_t* slot_reach,
                                   int64_t n, int64_t nslots, int64_t n_rows, int64_t E,
                                   hipStream_t s, bool reach_major = false);
// jbase[j] = window index of step 0 of caller reach j
// (-1 for never-processed reaches: their outflow reads as 0)
hipError_t launch_window_index(const int64_t* pos, const int32_t* G, const uint8_t* flags,
                               const int32_t* wg_gmin, const int64_t* wbase, int slots, int64_t n,
                               int64_t* jbase, hipStream_t s);
// Output gathers (caller order, member innermost).  inflow = false: outflow O; true: the inflow
// of reach j, summed from O over its inflow list.
// step-major out[t - t0][j][e] for t in [t0, t1)
hipError_t launch_gather_steps(const double* O, int64_t mO, const int64_t* jbase,
                               const int64_t* in_off, const int64_t* in_list, bool inflow,
                               int slots, double* out, int64_t n, int64_t t0, int64_t t1,
                               int64_t E, hipStream_t s);
// reach-major out[j][t][e] for t in [0, T)
// Row digest of fetched outputs (digest.hpp: definition, constants, the host side): the device
// form of its term
__device__ inline uint64_t digest_term_dev(uint64_t bits, uint64_t j) {
    uint64_t t = (bits ^ (j * kDigestK1)) * kDigestK2;
    return t ^ (t >> 29);
}
// out[r] = digest of row r of rows [nrows][n] (row stride n)
hipError_t launch_row_digests(const double* rows, int64_t nrows, int64_t n, uint64_t* out,
                              hipStream_t s);

// Both series of steps [t0, t1) in reach order, step-major, from the output windows (E = 1):
// out_o[t - t0][j] = O[sjb[pos[j]] + t stride] (0 for a never-processed reach, nutils.py:68),
// out_i[t - t0][j] = ((0 + o[t][u1]) + ...) over j's inflow list (in_off, rank order; upos[k] =
// pos[in_list[k]]).  Either output may be NULL.  Two passes through `scratch` (scratch_steps x
// ns doubles: the steps of a pass in slot order, kernels.hip unskew_windows / permute_steps).
// sjb: launch_slot_window_index.
hipError_t launch_gather_slots(const double* O, const int64_t* sjb, int64_t stride,
                               const int32_t* pos, const int32_t* in_off, const int32_t* upos,
                               double* out_o, double* out_i, int64_t n, int64_t ns, int64_t t0,
                               int64_t t1, double* scratch, int64_t scratch_steps,
                               hipStream_t s);
// sjb[d] = window index of step 0 of node slot d (-1: padding / never-processed slots)
hipError_t launch_slot_window_index(const int32_t* G, const uint8_t* flags, const int32_t* wg_gmin,
                                    const int64_t* wbase, int slots, int64_t ns, int64_t* sjb,
                                    hipStream_t s);

hipError_t launch_gather_series(const double* O, int64_t mO, const int64_t* jbase,
                                const int64_t* in_off, const int64_t* in_list, bool inflow,
                                int slots, double* out, int64_t n, int64_t T, int64_t E,
                                hipStream_t s);

// F[r][dslot] += alpha * I(r + 1) / gamma + beta * I(r) / gamma for r < T, I(t) = the outflow of
// caller reach j after step t - 1 in the output windows O / jbase (I(0) = o_start): the
// sub-basin lateral correction of simulation.py:152-159
hipError_t launch_lateral_correction(const double* O, const int64_t* jbase, int64_t j, int slots,
                                     double o_start, double alpha, double beta, double gamma,
                                     double* F, int64_t ns, int64_t dslot, int64_t T,
                                     hipStream_t s);

}  // namespace mcr
