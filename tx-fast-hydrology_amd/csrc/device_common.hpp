// Device helpers shared by the wavefront kernels (kernels.hip, flow.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "kernels.hpp"

namespace mcr {
namespace dev {

// Forcing rows a lane needs for the chunk starting at tick kc: [rb, rb + nr).  Rows are
// non-decreasing in t (step times are increasing), so the first step's row_lo and the last
// step's max(row_lo, row_hi) bound them.  nr = 0 when the lane has no step in the chunk.
__device__ __forceinline__ void chunk_rows(const int4* tab, int tw0, int kc, int G, int T,
                                           int& rb, int& nr) {
    int ta = kc - G, tb = kc + kChunk - 1 - G;
    if (tb < 0 || ta >= T) {
        rb = 0;
        nr = 0;
        return;
    }
    ta = ta < 0 ? 0 : ta;
    tb = tb >= T ? T - 1 : tb;
    const int4 ea = tab[ta - tw0];
    const int4 eb = tab[tb - tw0];
    rb = ea.x;
    nr = (eb.y > eb.x ? eb.y : eb.x) - rb + 1;
}

// forcing row index clamped into [0, n_rows): rows of inactive ticks may be arbitrary
__device__ __forceinline__ int clamp_row(int r, int n_rows) {
    return r < 0 ? 0 : (r < n_rows ? r : n_rows - 1);
}

__device__ __forceinline__ double lds_f64(const char* lds, unsigned byte) {
    return *reinterpret_cast<const double*>(lds + byte);
}

}  // namespace dev
}  // namespace mcr
