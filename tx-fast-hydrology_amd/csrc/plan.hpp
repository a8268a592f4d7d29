// Host-side topology compiler for the Muskingum wavefront sweep.
//
// The reference walks the forest once per timestep from every headwater, processing a reach as
// soon as its indegree countdown reaches zero (nutils.py:64-89).  This compiler replays that walk
// ONCE on the host (integer work only), records which reaches it processes and in which order,
// and turns the result into a static space-time schedule for the GPU:
//
//   * every reach j gets an upstream list sorted by the reference's finalisation rank, so the
//     inflow sum  i_next[j] = ((0 + o[u1]) + o[u2]) + ...  is formed in exactly the reference's
//     order (bitwise identical for >= 3-way confluences); a reach with more than kUpInline
//     upstreams reads a chain of partial-sum nodes (extra lanes that output a prefix of the
//     same left fold), so every lane reads at most kUpInline values per tick;
//   * reaches are grouped into clusters (connected sub-trees of at most `slots` reaches); a
//     cluster is swept by one workgroup with a time-skewed wavefront: reach j handles model step
//     t at global tick  G[j] + t.  Inside a cluster G[j] = G[down(j)] - 1, so every upstream
//     value is consumed exactly one tick after it is produced (one LDS double buffer);
//   * edges between clusters get slack  G[j] >= G[u] + tile,  so a value crossing clusters is
//     always produced in an earlier launch of `tile` ticks (the kernel boundary is the only
//     inter-workgroup synchronisation; no in-kernel hand-offs);
//   * clusters are packed into workgroups of `slots` threads.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace mcr {

struct PlanParams {
    int32_t slots = 256;       // lanes (threads) per workgroup
    int32_t tile = 32;         // ticks per launch; also the slack of a cross-cluster edge
    int32_t ext_cap = 64;      // preferred max cross-cluster inputs per workgroup (soft)
    int32_t chain = 2;         // node slots per lane (positions 0 .. chain-1, see "lane chains")
    int32_t sync = 0;          // 1: chunk-synchronous plan ("wave clusters" below)
};

// Chunk-synchronous plans (sync = 1, the dataflow kernel's default for one member): the kernel
// joins its waves with ONE workgroup barrier per kWaveSlack ticks (two per chunk of kChunk)
// instead of one per tick.  A unit-slack edge (value of tick k read at tick k + 1) must then stay
// inside one wave (LDS accesses of one wave are processed in order), so the clustering is
// two-level:
//   * a WAVE CLUSTER is a connected sub-tree that fits one wave's lanes; inside it
//     G[u] = G[down] - 1 (or a chained edge);
//   * a GROUP is a connected tree of wave clusters placed in one workgroup; an edge between two
//     of its wave clusters has slack exactly kWaveSlack: the producer writes its tick-k output
//     straight into the consumer's external-input column for tick k + kWaveSlack (this chunk's
//     or the next chunk's ring slot; the consumer reads it after the next barrier) -- a "local"
//     external input.  (Slack 8 with one barrier per chunk: a 1212-tick Texas schedule against
//     1168 at slack 4 and 1141 for the classic plan.)
//   * edges between groups are cross-workgroup (slack >= tile, granules), as before.
constexpr int kWaveSlack = 4;
constexpr int kWaveLanes = 64;

// Lane chains: a lane owns `chain` node slots (positions), computed in order within one tick;
// a node at position p >= 1 may take the output of position p - 1 of the SAME tick (a chained
// edge, no tick), so a run of up to `chain` consecutive reaches along a flow path costs one
// tick.  Node slot of (workgroup w, position p, lane l) = w * chain * slots + p * slots + l.
constexpr int kMaxChain = 4;

// LDS of one workgroup (bytes): outflow double buffer, step-table window, external inputs.
constexpr int64_t kLdsBudget = 160 * 1024;
inline int64_t span_cap(int64_t slots) { return slots < 256 ? 255 : slots - 1; }
inline int64_t table_entries(int64_t slots, int64_t tile) { return tile + span_cap(slots); }
constexpr int64_t kTableEntryBytes = 16;    // {int32 row_lo, int32 row_hi, f64 frac}

// upstream code: bit 15 set -> index into the workgroup's external-input list, else the
// workgroup-local slot of the upstream reach.
constexpr uint16_t kExtBit = 0x8000;
// code of a chained input: the output of the lane's previous position in the same tick
constexpr uint16_t kSelfCode = 0x7fff;
constexpr int kUpInline = 4;  // upstream values one lane reads per tick (codes in registers)

enum SlotFlags : uint8_t {
    kSlotPad = 0,        // unused thread slot
    kSlotRouted = 1,     // reach processed by the reference walk: o = 0 + (((a I + b Ip) + c Op) + g q)
    kSlotUnrouted = 2,   // reach never processed (cycle / unreachable): o stays 0, I = sum of inflows
    kSlotSum = 3,        // partial-sum node: outputs I (a prefix of a reach's inflow fold)
};

struct Plan {
    int64_t n = 0;
    PlanParams p;
    int32_t nwg = 0;
    int64_t nslots = 0;            // nwg * slots
    int32_t gmax = 0;              // max G over real reaches
    int64_t n_routed = 0;
    int64_t n_clusters = 0;
    int64_t n_cross = 0;           // cross-cluster edges
    int32_t max_height = 0;        // longest upstream path (levels - 1, partial sums included)
    int64_t n_partial = 0;         // partial-sum nodes
    int64_t n_pairs = 0;           // chained edges (chain = 2: fused lane pairs)
    int32_t max_ext_wg = 0;
    int32_t ext_hard = 0;          // LDS-derived hard cap of cross-cluster inputs per workgroup
    int32_t max_span = 0;          // max G span inside one workgroup

    // replay of the reference walk (original reach order)
    std::vector<int64_t> rank;     // -1 if never processed
    // inflow lists: routed upstream reaches of each reach in finalisation (rank) order, i.e.
    // i[j] = ((0 + o[in_list[in_off[j]]]) + ...) exactly as the reference accumulates it
    std::vector<int64_t> in_off, in_list;

    // per device slot d in [0, nslots)
    std::vector<int64_t> slot_reach;   // original reach index, -1 for padding / partial sums
    std::vector<int32_t> G;            // tick of model step 0
    std::vector<uint8_t> flags;
    std::vector<uint8_t> up_cnt;
    std::vector<uint64_t> up4;         // first kUpInline codes, 16 bits each
    std::vector<int32_t> xid;          // external input this slot feeds (index into ext_*), -1
    // sync plans: the workgroup-local external input (XE column of the slot's own workgroup,
    // after its ext_off range of granule inputs) this slot's output feeds kWaveSlack ticks
    // later, -1 if none
    std::vector<int16_t> lx;
    int64_t n_local = 0;               // sync plans: local (slack kWaveSlack) edges
    int32_t max_xe_wg = 0;             // external columns of a workgroup: granule + local

    // per workgroup
    std::vector<int32_t> wg_gmin, wg_gmax;  // G range of the workgroup's real reaches
    std::vector<int32_t> ext_off;           // [nwg + 1] granule (cross-workgroup) inputs
    std::vector<int32_t> lx_off;            // [nwg + 1] local inputs (sync plans)
    std::vector<int32_t> lx_src;            // producer slot of each local input
    std::vector<int64_t> ext_src;           // source row: reach index, or n + slot (partial sum)
    std::vector<int32_t> ext_g;             // G of the consuming reach

    // original reach -> device slot
    std::vector<int64_t> pos;
};

// Build the plan.  Returns an empty string on success, otherwise an error message.
std::string build_plan(int64_t n, const int64_t* endnodes, const int64_t* indegree,
                       const int64_t* heads, int64_t n_heads, const PlanParams& params,
                       Plan& out);

// Workgroups with work in launch k (ticks [k*tile, (k+1)*tile)) for a horizon of T steps.
// Fills `list` (concatenated) and `off` ([n_launch + 1]); returns the number of launches.
int64_t active_schedule(const Plan& plan, int64_t T, std::vector<int32_t>& list,
                        std::vector<int64_t>& off);

}  // namespace mcr
