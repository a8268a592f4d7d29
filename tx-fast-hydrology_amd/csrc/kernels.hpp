// Device-side entry points of the Muskingum routing engine (gfx950).  Launchers are plain host
// functions so the C-ABI layer (capi.cpp) stays free of kernel syntax.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mcr {

// Ticks per register chunk.  Series rows are padded so that a chunk always covers one aligned
// 64-byte segment: step t of reach j lives at  row(j) * Tp + t + (G[j] & (kChunk - 1)).
constexpr int kChunk = 8;

inline int64_t padded_steps(int64_t T) {  // Tp: room for the pad and a full trailing chunk
    return ((T + 2 * kChunk - 1) / kChunk) * kChunk;
}

// Everything the wavefront kernel reads, by value.  Per-slot arrays are in device-slot order
// (plan.hpp); the output series are reach-major in the CALLER's order, padded as above.
struct WaveArgs {
    const int32_t* active;        // workgroup ids of this launch
    const int32_t* G;             // [nslots]
    const uint8_t* flags;         // [nslots]
    const uint8_t* up_cnt;        // [nslots]
    const uint64_t* up4;          // [nslots]
    const int32_t* up_more_off;   // [nslots + 1]
    const uint16_t* up_more;
    const int64_t* slot_reach;    // [nslots] caller reach index or -1
    const int32_t* ext_off;       // [nwg + 1]
    const int64_t* ext_src;       // caller index of the upstream reach
    const int32_t* ext_g;         // G of the consuming reach
    const uint8_t* rpad;          // [n] pad of each caller reach (G & 15)
    const double* alpha;          // [nslots]
    const double* beta;
    const double* chi;
    const double* gamma;
    const double* st_o;           // state at step -1 (o_t_next before the horizon) [nslots]
    const double* st_i;
    const double* F;              // forcing rows in slot order [n_rows][nslots]
    const int4* stab;             // per step {row_lo, row_hi (-1 = copy row_lo), frac (f64)}
    const int32_t* wg_gmin;       // [nwg] G range of each workgroup (step-table window)
    const int32_t* wg_gmax;
    double* O;                    // [n][Tp]
    double* I;                    // [n][Tp]
    double* dummy;                // >= 2 * kChunk doubles: target of out-of-range chunks
    int64_t nslots;
    int32_t n_rows;
    int32_t T;
    int32_t Tp;
    int32_t kappa0;               // first tick of this launch (multiple of kChunk)
    int32_t tile;                 // ticks in this launch (multiple of kChunk)
    int32_t table_cap;            // LDS entries reserved for the step-table window
    int32_t ext_cap;              // LDS rows reserved for external inputs
    int32_t more_cap;             // LDS words reserved for overflow upstream codes
};

inline size_t wavefront_lds_bytes(int slots, int table_cap, int ext_cap, int tile,
                                  int more_cap) {
    return 16 * ((size_t)slots + 1) + 24 * (size_t)slots + 16 * (size_t)table_cap +
           8 * (size_t)ext_cap * tile + 4 * (size_t)more_cap;
}

// dense: the step table has an 8-step window spanning more than 3 forcing rows
hipError_t launch_wavefront(const WaveArgs& a, int grid, int slots, size_t lds_bytes, bool dense,
                            hipStream_t s);

// st[d] = src[slot_reach[d]] for real slots (caller order -> slot order)
hipError_t launch_scatter_to_slots(const double* src, double* dst, const int64_t* slot_reach,
                                   int64_t nslots, hipStream_t s);
// dst[j] = src[pos[j]] (slot order -> caller order)
hipError_t launch_gather_from_slots(const double* src, double* dst, const int64_t* pos,
                                    int64_t n, hipStream_t s);
// F[r][d] = fp[r][slot_reach[d]]  (forcing table to slot order; 0 for padding slots)
hipError_t launch_forcing_to_slots(const double* fp, double* F, const int64_t* slot_reach,
                                   int64_t n, int64_t nslots, int64_t n_rows, hipStream_t s);
// state after the last step: st[d] = O[row(d)][T - 1]
hipError_t launch_final_state(const double* O, const double* I, double* st_o, double* st_i,
                              const int64_t* slot_reach, const int32_t* G, int64_t nslots,
                              int64_t Tp, int64_t T, hipStream_t s);
// out[t - t0][j] = S[j][t]  for t in [t0, t1)   (padded reach-major -> step-major)
hipError_t launch_transpose(const double* S, const uint8_t* rpad, double* out, int64_t n,
                            int64_t Tp, int64_t t0, int64_t t1, hipStream_t s);
// out[j][t] = S[j][t] for t in [0, T)   (drop the padding)
hipError_t launch_compact(const double* S, const uint8_t* rpad, double* out, int64_t n,
                          int64_t Tp, int64_t T, hipStream_t s);

}  // namespace mcr
