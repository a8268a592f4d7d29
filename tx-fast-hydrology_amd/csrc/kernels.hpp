// Device-side entry points of the Muskingum routing engine (gfx950).  Launchers are plain host
// functions so the C-ABI layer (capi.cpp) stays free of kernel syntax.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mcr {

// Everything the wavefront kernel reads, by value.  Per-slot arrays are in device-slot order
// (plan.hpp), outputs are reach-major in the caller's reach order: O[j * T + t].
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
    const int64_t* ext_src;       // caller reach index of the upstream reach
    const int32_t* ext_g;         // G of the consuming reach
    const double* alpha;          // [nslots]
    const double* beta;
    const double* chi;
    const double* gamma;
    const double* st_o;           // state at step -1 (o_t_next before the horizon) [nslots]
    const double* st_i;
    const double* F;              // forcing rows, device-slot order [n_rows][nslots]
    const int2* srow;             // per step: (row_lo, row_hi) or (row, -1) = copy row
    const double2* sw;            // per step: (1 - frac, frac)
    double* O;                    // [n][T]
    double* I;                    // [n][T]
    int64_t nslots;
    int32_t n_rows;
    int32_t T;
    int32_t kappa0;               // first tick of this launch
    int32_t tile;                 // ticks in this launch
};

// One launch: `grid` workgroups of `slots` threads sweep ticks [kappa0, kappa0 + tile).
hipError_t launch_wavefront(const WaveArgs& a, int grid, int slots, size_t lds_bytes,
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
// st[d] = O[slot_reach[d] * T + (T - 1)]   (state after the last step)
hipError_t launch_final_state(const double* O, const double* I, double* st_o, double* st_i,
                              const int64_t* slot_reach, int64_t nslots, int64_t T,
                              hipStream_t s);
// out[t - t0][j] = O[j * T + t]  for t in [t0, t1), j in [0, n)   (reach-major -> step-major)
hipError_t launch_transpose(const double* O, double* out, int64_t n, int64_t T, int64_t t0,
                            int64_t t1, hipStream_t s);

}  // namespace mcr
