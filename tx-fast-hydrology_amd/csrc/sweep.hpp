// Member sweep: the ensemble forecast with the members on the lanes (sweep.hip).
//
// The multi-launch kernel (kernels.hip wavefront_det) puts one node slot on each lane and runs
// the members as grid instances: every lane walks its own reach's topology, forcing rows and
// state, and a 64-lane output row mixes 64 reaches.  In the member sweep a wave holds NPW node
// slots of a member plan (plan.hpp, chain 1) for 64 members at once: everything about a node
// (its step at a tick, inputs, coefficients, forcing rows, the output row it writes) is uniform
// over the wave, and every per-member access is one contiguous 512-byte row:
//
//   F [n_rows][ns][E]   forcing in member-plan slot order, members innermost
//   S {o, i} [ns][E]    state between launches (So / Si)
//   O [T][ns][E]        outflow of step t of slot d, member e at (t * ns + d) * E + e
//
// Node d handles step t at global tick G[d] + t as in the other kernels: in-cluster inputs come
// from the previous tick through an LDS double buffer (rows of 64 members), inputs of other
// clusters from earlier launches (tile slack) through O, staged in the same buffer by the wave
// that owns them.  A launch covers `tile` ticks of the workgroups active in them.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mcr {

// node slots per wave and waves per workgroup; the member plan has NPW * NW slots per
// workgroup (plan: kSweepNW lanes x kSweepNPW positions)
#ifndef MCR_SWEEP_NW
#define MCR_SWEEP_NW 8
#endif
constexpr int kSweepNPW = 4;
constexpr int kSweepNW = MCR_SWEEP_NW;
constexpr int kSweepSlots = kSweepNPW * kSweepNW;
// external inputs (inputs from other workgroups) per workgroup (even: two rows per LDS-DMA)
constexpr int kSweepMaxExt = 24;

struct SweepArgs {
    const int32_t* active;     // workgroups of this launch
    const int32_t* wg_gmin;    // [nwg] G range of each workgroup
    const int32_t* wg_gmax;
    const int32_t* G;          // [ns] member-plan slot arrays
    const uint8_t* flags;
    const uint8_t* up_cnt;
    const uint64_t* up4;
    const int32_t* ext_off;    // [nwg + 1]
    const int32_t* ext_slot;   // [n_ext] member-plan slot of the producing node
    const int32_t* ext_g;      // [n_ext] G of the consuming node
    const double* coef;        // [ns][4] alpha, beta, chi, gamma (slot kinds applied)
    double* So;                // [ns][E]
    double* Si;
    const double* F;           // [n_rows][ns][E]
    const int4* stab;          // [T] {row_lo, row_hi, frac}
    double* O;                 // [T][ns][E]
    uint32_t rowB;             // ns * E * 8 bytes (< 2^31)
    int32_t E;
    int32_t T;
    int32_t n_rows;
    int32_t k0;                // first tick of the launch (multiple of kChunk)
    int32_t tile;              // ticks of the launch (multiple of kChunk)
    // optional launch trace (kernels.hpp kTraceWords per workgroup of member group 0): wall
    // clock at start / loop start / end, hw id, shader clock at loop start / end
    int64_t* trace;
};

// member plan of the sweep: tile (launch ticks, cross-workgroup slack); step-table entries a
// launch keeps in LDS (tile + kChunk + 1 + the workgroup's G span must fit)
#ifndef MCR_SWEEP_TILE
#define MCR_SWEEP_TILE 32
#endif
constexpr int kSweepTile = MCR_SWEEP_TILE;
constexpr int kSweepTabCap = 352;
inline size_t sweep_lds_bytes() {
    return 16u * kSweepTabCap + 36u * kSweepSlots + 2u * (kSweepSlots + 1 + kSweepMaxExt) * 512u +
           4u * kSweepMaxExt * 512u;
}

hipError_t launch_member_sweep(const SweepArgs& a, int grid, int member_groups, hipStream_t s);

// dst[r][map[d]][e] = src[e * src_stride + r * nsm + d] for main-plan slots d with map[d] >= 0
// (e < E, r < R): member-major main-plan arrays (state: R = 1; forcing: R = n_rows,
// src_stride = n_rows * nsm) to the member plan's member-innermost layout.  Tiled through LDS
// (64 slots x 64 members), so both sides are read and written in whole rows.
hipError_t launch_to_sweep(const double* src, int64_t src_stride, int64_t nsm, int64_t R,
                           const int32_t* map, double* dst, int64_t nss, int64_t E,
                           hipStream_t s);
// the reverse for the state: dst[e * nsm + d] = src[map[d]][e] for d with map[d] >= 0
hipError_t launch_from_sweep(const double* src, int64_t nss, const int32_t* map, double* dst,
                             int64_t nsm, int64_t E, hipStream_t s);
// member-plan coefficients [ns][4] from the main plan's slot arrays (slot kinds applied there):
// member slot d' of a reach takes main slot rmap[d'] (>= 0); partial sums {1, 0, 0, 0};
// padding {0, 0, 0, 0}
hipError_t launch_sweep_coeffs(const double* alpha, const double* beta, const double* chi,
                               const double* gamma, const int32_t* rmap, const uint8_t* flags,
                               double* coef, int64_t nss, hipStream_t s);
// zero the state of member slots without a reach (partial sums, padding): rmap[d'] < 0
hipError_t launch_sweep_zero_free(const int32_t* rmap, double* So, double* Si, int64_t nss,
                                  int64_t E, hipStream_t s);

}  // namespace mcr
