// Ensemble analysis building blocks (analysis.hip): f64 MFMA GEMM and the element kernels of the
// ensemble Kalman update.  Matrices are column-major with explicit leading dimensions.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mcr {

// C = alpha op(A) op(B) + beta C  (op = transpose when ta / tb; op(A) M x K, op(B) K x N)
// work (optional, work_elems doubles): lets a GEMM with few output tiles and a deep K split K
// over workgroups (partial products in work, reduced in slice order: deterministic).
// Two-part operands (optional): columns j >= n1 of op(B) come from B2 (column j - n1, same
// leading dimension) and land in C2 (column j - n1, leading dimension ldc): one launch for
// [C | C2] = op(A) [op(B) | op(B2)].
hipError_t launch_dgemm(bool ta, bool tb, int64_t M, int64_t N, int64_t K, double alpha,
                        const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                        double* C, int64_t ldc, hipStream_t s, double* work = nullptr,
                        size_t work_elems = 0, const double* B2 = nullptr, int64_t n1 = -1,
                        double* C2 = nullptr);

// ---- dense.hip: hand-written f64 MFMA kernels of the large-ensemble analysis -------------
// G = (X - mean_e X) Z: member-major slice X [Et][S], Z (Et x Et, leading dimension ldz),
// G [Et][S]; 128 x 128 MFMA tiles, member mean as a rank-1 epilogue correction
hipError_t launch_slice_increments(const double* X, const double* Z, int64_t ldz, double* G,
                                   int64_t S, int64_t Et, hipStream_t s);
// SPD systems B := P^-1 B by block Gauss-Jordan elimination (32 x 32 pivot blocks) on a padded
// copy (kp = spd_padded(k)):
//   launch_pad_matrix: dst (kp x ncols, ld kp) = src where i < rows and j < cols, `diag` on the
//     other diagonal entries, 0 elsewhere (the padded SPD matrix: diag 1; right-hand sides: 0)
//   launch_spd_solve: P (kp x kp, full symmetric, overwritten) and B (kp x nrhs, ld kp,
//     padding rows 0) := P^-1 B; Sd: kp x 32 doubles of pivot-block inverses; info = 0, or the
//     1-based index of the first non-positive pivot (then B = 0).  kp / 32 + 2 launches.
int64_t spd_padded(int64_t k);
hipError_t launch_pad_matrix(const double* src, int64_t rows, int64_t cols, int64_t lds,
                             double* dst, int64_t kp, double diag, int64_t ncols, hipStream_t s);
hipError_t launch_spd_solve(double* P, int64_t kp, double* B, int64_t nrhs, double* Sd,
                            int32_t* info, hipStream_t s);
// U = R^-1 HA for a diagonal R (r = its diagonal), column-major m x E
hipError_t launch_scale_rows(const double* HA, const double* r, double* U, int64_t m, int64_t E,
                             hipStream_t s);
hipError_t launch_mean_anomalies(const double* X, double* A, int64_t ns, int64_t E,
                                 hipStream_t s);
// G = (X - mean) Z for a member-major slice X [Et][S] and Z (Et x Et, column-major): the
// increments of the slice in one pass (Et <= kFusedIncrementsMax)
constexpr int64_t kFusedIncrementsMax = 64;
hipError_t launch_anomaly_increments(const double* X, const double* Z, int64_t ldz, double* G,
                                     int64_t S, int64_t Et, hipStream_t s);
// HA (m x E) = A at the gauge slots; D (m x E) = Y[g][e] - X at the gauge slots (D may be NULL)
hipError_t launch_gauge_gather(const double* A, const double* X, const int64_t* gslot,
                               const double* Y, double* HA, double* D, int64_t m, int64_t ns,
                               int64_t E, hipStream_t s);
// local gauge values HX (m x E, column-major) and innovations D = Y[g][e] - HX
hipError_t launch_gauge_values(const double* X, const int64_t* gslot, const double* Y,
                               double* HX, double* D, int64_t m, int64_t ns, int64_t E,
                               hipStream_t s);
// member-major [E][ns] <-> per-rank reach slices [N][E][S] (S = ceil(ns / N), zero padded)
hipError_t launch_pack_slices(const double* X, double* out, int64_t ns, int64_t E, int64_t S,
                              int64_t N, hipStream_t s);
hipError_t launch_unpack_slices(const double* in, double* G, int64_t ns, int64_t E, int64_t S,
                                int64_t N, hipStream_t s);
// _apply_gain per member: o += 0 + G (routed reaches), i += rank-ordered one-hop sums;
// up_off / up: each slot's routed upstream slots in rank order (int32 CSR over slots)
hipError_t launch_apply_gain(const double* G, double* st_o, double* st_i, const uint8_t* flags,
                             const int32_t* up_off, const int32_t* up, int64_t ns, int64_t E,
                             hipStream_t s);
// Kt (m x nslots, column-major, leading dimension ldk) -> K_out[j][g] in caller reach order
hipError_t launch_gain_to_caller(const double* Kt, int64_t ldk, double* out, const int64_t* pos,
                                 int64_t m, int64_t n, hipStream_t s);

}  // namespace mcr
