// Ensemble analysis building blocks (analysis.hip): f64 MFMA GEMM and the element kernels of the
// ensemble Kalman update.  Matrices are column-major with explicit leading dimensions.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace mcr {

// C = alpha op(A) op(B) + beta C  (op = transpose when ta / tb; op(A) M x K, op(B) K x N)
// work (optional, work_elems doubles): lets a GEMM with few output tiles and a deep K split K
// over workgroups (partial products in work, reduced in slice order: deterministic)
hipError_t launch_dgemm(bool ta, bool tb, int64_t M, int64_t N, int64_t K, double alpha,
                        const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                        double* C, int64_t ldc, hipStream_t s, double* work = nullptr,
                        size_t work_elems = 0);
// ensemble mean over members and anomalies A = X - mean (both [E][ns])
// U = R^-1 HA for a diagonal R (r = its diagonal), column-major m x E
hipError_t launch_scale_rows(const double* HA, const double* r, double* U, int64_t m, int64_t E,
                             hipStream_t s);
// M = I (k x k)
hipError_t launch_set_identity(double* M, int64_t k, hipStream_t s);
// V := M^-1 V for SPD M (k x k, column-major, k <= 64) in one workgroup; info = 0, or j + 1 when
// the j-th leading minor is not positive definite (V then zeroed)
hipError_t launch_spd_solve_small(const double* M, double* V, int64_t k, int32_t* info,
                                  hipStream_t s);
constexpr int64_t kSpdSolveMax = 64;
// X[0 .. cnt) := 0 when *info != 0 (device-side gate after a rocSOLVER potrf / potrs pair)
hipError_t launch_zero_if_failed(double* X, int64_t cnt, const int32_t* info, hipStream_t s);
hipError_t launch_mean_anomalies(const double* X, double* A, int64_t ns, int64_t E,
                                 hipStream_t s);
// G = (X - mean) Z for a member-major slice X [Et][S] and Z (Et x Et, column-major): the
// increments of the slice in one pass (Et <= kFusedIncrementsMax)
constexpr int64_t kFusedIncrementsMax = 64;
hipError_t launch_anomaly_increments(const double* X, const double* Z, double* G, int64_t S,
                                     int64_t Et, hipStream_t s);
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
// Kt (m x nslots, column-major) -> K_out[j][g] in caller reach order
hipError_t launch_gain_to_caller(const double* Kt, double* out, const int64_t* pos, int64_t m,
                                 int64_t n, hipStream_t s);

}  // namespace mcr
