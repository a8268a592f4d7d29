// Member paths: ONE model step of E ensemble members as a sweep along flow paths, members on
// the lanes (paths.hip).  The EnKF cycle routes one step between analyses (da.py:91-136 per
// member); in the tick schedule of the wavefront kernels that step costs the whole schedule fill
// (~850 ticks at ~0.44 us) whatever E is.  Here the step is decomposed along heavy paths instead:
//
//   * every reach is a node; its inputs are its routed upstream reaches in the reference's
//     finalisation (rank) order (nutils.py:72-88), so the inflow fold is the reference's;
//   * heavy-path decomposition: each node's heavy input is the upstream with the largest
//     subtree; a chain follows heavy inputs from a headwater down to the node where it joins
//     another chain as a light input (or to the outlet);
//   * a light input whose subtree has at most kPathAbsorb nodes is absorbed into the chain's
//     task (processed just before the node it feeds, in rank order); bigger light inputs are
//     tasks of their own, handed over through data-tagged granules;
//   * a task is processed by ONE wave, node after node, the members on the lanes: the chain
//     value stays in a register, absorbed values in an LDS ring, so the dependent chain per node
//     is the update itself (no barrier, no tick) and the step's critical path is the longest
//     heavy path plus a few hand-overs (O(log n) light edges on any path).
//
// Tasks are numbered in ticket order: a topological order of the task graph (producers first,
// longest remaining path first), so a wave only ever waits for tasks taken earlier by running
// waves -- deadlock-free without co-residency.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "plan.hpp"

namespace mcr {

constexpr int kPathAbsorb = 16;     // light subtrees up to this many nodes join the chain's task
constexpr int kPathRing = 32;       // LDS ring of node outputs a task keeps (local inputs)
constexpr int kPathInline = 8;      // inputs a node record holds; more go to the overflow list
constexpr int kPathRecWords = 16;   // int32 words per node record (64 B)

// input codes (record words): kind in bits 30..31, payload below
enum PathInput : uint32_t {
    kInChain = 0u << 30,    // the last chain node's output (register)
    kInPrev = 1u << 30,     // the previous node's output (register)
    kInLocal = 2u << 30,    // an earlier node of the same task: payload = its sequence number
    kInExt = 3u << 30,      // another task's bottom node: payload = that task's id
};
constexpr uint32_t kInPayload = (1u << 30) - 1;

// record word 0 (meta): bits 0..15 input count, 16 routed, 17 chain node, 18 publish (the task
// bottom feeds another task), 19 keep (a later node reads it from the ring)
constexpr uint32_t kRecRouted = 1u << 16, kRecChain = 1u << 17, kRecPublish = 1u << 18,
                   kRecKeep = 1u << 19;

struct PathPlan {
    int64_t n = 0;                     // nodes (reaches)
    int32_t n_tasks = 0;
    int32_t max_task = 0;              // longest task (nodes)
    int32_t crit = 0;                  // nodes on the longest path (the step's critical path)
    int64_t n_ext = 0;                 // cross-task edges
    std::vector<int32_t> task_off;     // [n_tasks + 1]: task t = sequence [task_off[t], task_off[t+1])
    std::vector<int64_t> seq_reach;    // [n] caller reach of each sequence position
    // [n * kPathRecWords]: meta, slot (session device slot of the reach), alpha (2 words: filled
    // on the device from the session's coefficients, launch_path_alpha), kPathInline input codes,
    // overflow offset into `ovf`, padding
    std::vector<int32_t> rec;
    std::vector<int32_t> ovf;          // input codes beyond kPathInline
};

// Build the path plan from a compiled schedule plan (its walk replay: rank, inflow lists, slot
// of each reach).  Host integer work, once per network.
std::string build_path_plan(const Plan& plan, PathPlan& out);

}  // namespace mcr

// ---- device side (paths.hip) -------------------------------------------------------------
#include <hip/hip_runtime.h>

namespace mcr {

constexpr int kPathLanes = 64;      // members per wave (a member group); E > 64: several groups

// Everything the one-step member sweep reads, by value.
struct PathArgs {
    const int32_t* rec;        // [n * kPathRecWords] node records (alpha filled, path_alpha)
    const int32_t* ovf;        // overflow input codes
    const int32_t* task_off;   // [n_tasks + 1]
    const double* P;           // [(g * n + s) * 3 * 64 + k * 64 + lane]: beta i', chi o', gamma q
    double* st_o;              // session state, member-major [E][ns] (updated in place)
    double* st_i;
    uint32_t* GR;              // task-bottom granules [(task * groups + g) * 64 + lane] x 16 B
    int32_t* queue;            // ticket counter, zeroed before the launch
    int32_t* status;           // set to 1 when a wait gave up
    int64_t patience;          // wall-clock (100 MHz) ticks a wait polls before giving up
    int64_t ns;
    int64_t n;
    int32_t n_tasks;
    int32_t groups;
    int32_t E;
    uint32_t gr_bytes;         // size of GR (< 2^31)
    uint32_t epoch;            // tag of this step's granules (never 0)
};

// Pre-pass: per (node, member) the three terms of the update that do not depend on the inflow,
// beta * i', chi * o', gamma * q (o', i' = the state with the pending analysis increments
// applied exactly as apply_gain would; q = the step's interpolated lateral inflow), into P in
// sequence order, members innermost.  seq_of_slot: the node's sequence position, -1 for
// padding / partial-sum slots.
hipError_t launch_path_prep(const double* F, int64_t mF, int n_rows, int4 ent,
                            const double* st_o, const double* st_i, const double* beta,
                            const double* chi, const double* gamma, const uint8_t* flags,
                            const int32_t* seq_of_slot, const double* G, const int32_t* up_off,
                            const int32_t* up, double* P, int64_t ns, int64_t n, int64_t E,
                            hipStream_t s);
// alpha of every node record from the session's per-slot coefficients
hipError_t launch_path_alpha(int32_t* rec, const double* alpha, int64_t n, hipStream_t s);
// The sweep: a persistent grid of waves taking (task, member group) tickets.
hipError_t launch_member_paths(const PathArgs& a, int grid, hipStream_t s);

}  // namespace mcr
