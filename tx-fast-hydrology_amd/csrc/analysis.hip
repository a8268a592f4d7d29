// Ensemble analysis kernels (gfx950): the da.py-style Kalman update with the forecast
// covariance replaced by the ensemble sample covariance.
//
//   reference (da.py:110-126, KalmanFilter.filter):  K = P[:, s] (P[s, s] + R)^-1,
//       gain = K dz,  o += gain,  i += one-hop(gain)  (_apply_gain, nutils.py:116-134)
//   here, with anomalies A = X - mean(X) over E members and HA = A[s]:
//       P H^T = A HA^T / (E-1),  H P H^T = HA HA^T / (E-1)
//       W = (HA HA^T / (E-1) + R)^-1 D,   D = Y - HX  (per-member innovations)
//       G = A (HA^T W) / (E-1)             (per-member increments, = K D)
//       o += 0 + G,  i += one-hop(G)       (rank-ordered sums, as _apply_gain)
// The dense products run on f64 MFMA (v_mfma_f64_16x16x4f64); the SPD solves and the large
// slice product are dense.hip.
// Device arrays are member-major slot order ([E][nslots]) like the routing session.
#include "analysis.hpp"
#include "plan.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>

namespace mcr {

namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kTile = 64;   // C tile per workgroup (4 waves, 32 x 32 each)
constexpr int kBK = 16;     // K slice staged in LDS
constexpr int kPad = 1;     // LDS row padding (f64)

// C = alpha op(A) op(B) + beta C, column-major, op = transpose when TA / TB.
// op(A) is M x K, op(B) is K x N.  beta == 0 never reads C.
// Split-K (gridDim.z > 1): slice z covers k in [z * kc, (z + 1) * kc) and writes its raw
// partial product to C + z * ldc * N (alpha = 1, beta = 0 passed by the launcher); splitk_reduce
// sums the slices in order (deterministic).
// Columns j >= n1 of op(B) come from B2 (column j - n1) and go to C2 (column j - n1): two
// products sharing op(A) in one launch.
template <bool TA, bool TB>
__global__ __launch_bounds__(256) void dgemm_mfma(int64_t M, int64_t N, int64_t K, double alpha,
                                                  const double* __restrict__ A, int64_t lda,
                                                  const double* __restrict__ B, int64_t ldb,
                                                  double beta, double* __restrict__ C,
                                                  int64_t ldc, int64_t kc,
                                                  const double* __restrict__ B2, int64_t n1,
                                                  double* __restrict__ C2) {
    __shared__ double As[kBK][kTile + kPad];   // As[k][i] = op(A)(row0 + i, k0 + k)
    __shared__ double Bs[kBK][kTile + kPad];   // Bs[k][j] = op(B)(k0 + k, col0 + j)
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int64_t row0 = (int64_t)blockIdx.x * kTile;
    const int64_t col0 = (int64_t)blockIdx.y * kTile;
    const int wr = (wave & 1) * 32, wc = (wave >> 1) * 32;
    f64x4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f64x4{0.0, 0.0, 0.0, 0.0};

    const int64_t kbeg = (int64_t)blockIdx.z * kc;
    const int64_t kend = kbeg + kc < K ? kbeg + kc : K;
    C += (int64_t)blockIdx.z * ldc * N;
    if (C2) C2 += (int64_t)blockIdx.z * ldc * N;
    // one K slice of both operands per thread (kTile * kBK / 256 elements each), read into
    // registers one slice ahead: the next slice's loads are in flight during this slice's MFMAs
    // (EnKF256 A Z 1.0 -> 0.72 ms per analysis)
    constexpr int kPer = (kTile * kBK) / 256;
    double ra[kPer], rb[kPer];
    auto load_slice = [&](int64_t k0) {
#pragma unroll
        for (int r = 0; r < kPer; ++r) {
            const int idx = tid + 256 * r;
            // coalesced along the contiguous dimension of each operand
            int i, k;
            if (TA) { k = idx % kBK; i = idx / kBK; } else { i = idx % kTile; k = idx / kTile; }
            const int64_t gi = row0 + i, gk = k0 + k;
            ra[r] = (gi < M && gk < kend) ? (TA ? A[gk + gi * lda] : A[gi + gk * lda]) : 0.0;
            int j;
            if (TB) { j = idx % kTile; k = idx / kTile; } else { k = idx % kBK; j = idx / kBK; }
            const int64_t gj = col0 + j, gk2 = k0 + k;
            const double* Bp = gj < n1 ? B : B2;
            const int64_t bj = gj < n1 ? gj : gj - n1;
            rb[r] = (gj < N && gk2 < kend) ? (TB ? Bp[bj + gk2 * ldb] : Bp[gk2 + bj * ldb]) : 0.0;
        }
    };
    if (kbeg < kend) load_slice(kbeg);
    for (int64_t k0 = kbeg; k0 < kend; k0 += kBK) {
#pragma unroll
        for (int r = 0; r < kPer; ++r) {
            const int idx = tid + 256 * r;
            int i, k;
            if (TA) { k = idx % kBK; i = idx / kBK; } else { i = idx % kTile; k = idx / kTile; }
            As[k][i] = ra[r];
            int j;
            if (TB) { j = idx % kTile; k = idx / kTile; } else { k = idx % kBK; j = idx / kBK; }
            Bs[k][j] = rb[r];
        }
        __syncthreads();
        if (k0 + kBK < kend) load_slice(k0 + kBK);
#pragma unroll
        for (int kk = 0; kk < kBK; kk += 4) {
            // f64 16x16x4: A lane l holds A[l & 15][k = l >> 4], B lane l holds B[k = l >> 4][l & 15]
            const int ka = kk + (lane >> 4);
            const double a0 = As[ka][wr + (lane & 15)];
            const double a1 = As[ka][wr + 16 + (lane & 15)];
            const double b0 = Bs[ka][wc + (lane & 15)];
            const double b1 = Bs[ka][wc + 16 + (lane & 15)];
            acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
            acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
            acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
            acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
        }
        __syncthreads();
    }
    // C/D of f64 16x16x4: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int64_t gi = row0 + wr + 16 * i + (lane >> 4) + 4 * r;
                const int64_t gj = col0 + wc + 16 * j + (lane & 15);
                if (gi < M && gj < N) {
                    double* c = gj < n1 ? C + gi + gj * ldc : C2 + gi + (gj - n1) * ldc;
                    *c = beta == 0.0 ? alpha * acc[i][j][r] : alpha * acc[i][j][r] + beta * *c;
                }
            }
}

// C = alpha * (W[0] + W[1] + ... + W[splits-1]) + beta * C  (W[z]: M x N, leading dim M;
// columns j >= n1 go to C2)
__global__ void splitk_reduce(const double* __restrict__ W, int splits, int64_t M, int64_t N,
                              double alpha, double beta, double* __restrict__ C, int64_t ldc,
                              int64_t n1, double* __restrict__ C2) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= M * N) return;
    const int64_t i = idx % M, j = idx / M;
    double acc = W[idx];
    for (int z = 1; z < splits; ++z) acc += W[(int64_t)z * M * N + idx];
    double* c = j < n1 ? C + i + j * ldc : C2 + i + (j - n1) * ldc;
    *c = beta == 0.0 ? alpha * acc : alpha * acc + beta * *c;
}

// U[g + e m] = HA[g + e m] / r[g]  (R^-1 HA for a diagonal R)
__global__ void scale_rows(const double* __restrict__ HA, const double* __restrict__ r,
                           double* __restrict__ U, int64_t m, int64_t E) {
    const int64_t total = m * E;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x)
        U[x] = HA[x] / r[x % m];
}

// xbar[d] = (sum_e X[e][d]) / E ;  A[e][d] = X[e][d] - xbar[d]
__global__ void mean_anomalies(const double* __restrict__ X, double* __restrict__ A,
                               int64_t ns, int64_t E) {
    for (int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; d < ns;
         d += (int64_t)gridDim.x * blockDim.x) {
        double s = 0.0;
#pragma unroll 8
        for (int64_t e = 0; e < E; ++e) s += X[e * ns + d];
        const double xbar = s / (double)E;
#pragma unroll 8
        for (int64_t e = 0; e < E; ++e) A[e * ns + d] = X[e * ns + d] - xbar;
    }
}

// The same for few rows of many members (the gauge anomalies HA of the ensemble-space weights:
// 500 rows x 256 members): a wave per row loads all of the row's members at once into LDS and
// every lane folds them in member order from there, so the sum is mean_anomalies' left fold
// and the loads are not serialised behind it (a thread per row walked 256 dependent adds with
// its loads 8 at a time: 28 us per EnKF256 analysis)
constexpr int kRowMaxE = 1024;
__global__ __launch_bounds__(256) void mean_anomalies_rows(const double* __restrict__ X,
                                                           double* __restrict__ A, int64_t ns,
                                                           int64_t E) {
    __shared__ double buf[4][kRowMaxE];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t d = (int64_t)blockIdx.x * 4 + wv;
    if (d >= ns) return;                                   // wave-uniform
    double* b = buf[wv];
    for (int64_t e = lane; e < E; e += 64) b[e] = X[e * ns + d];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    double s = 0.0;
#pragma unroll 8
    for (int64_t e = 0; e < E; ++e) s += b[e];
    const double xbar = s / (double)E;
    for (int64_t e = lane; e < E; e += 64) A[e * ns + d] = b[e] - xbar;
}

// Increments of a reach slice in one pass, for ensembles of at most MAXE members (the per-GPU
// shares of the sharded EnKF): per slot d the member mean (mean_anomalies' order), the
// anomalies A[e] = X[e][d] - mean in registers, and G[e][d] = sum_f A[f] Z[f][e] with Z (Et x Et,
// column-major) staged in LDS (every lane reads the same coefficient: broadcast).  Replaces
// mean_anomalies + the skinny (S x Et) x (Et x Et) GEMM, whose anomaly round trip through HBM
// was most of their time.  One slot per thread.
template <int MAXE>
__global__ __launch_bounds__(256) void anomaly_increments(const double* __restrict__ X,
                                                          const double* __restrict__ Z,
                                                          int64_t ldz,
                                                          double* __restrict__ G, int64_t S,
                                                          int Et) {
    // Zt[f][e] = Z[f + e Et]: the 8 coefficients of one anomaly for 8 consecutive outputs are
    // contiguous (two 32-byte LDS reads), and 8 independent FMA chains run side by side
    constexpr int EG = 8;
    __shared__ __attribute__((aligned(16))) double Zt[MAXE * MAXE];
    const int Ep = (Et + EG - 1) / EG * EG;               // padded row (zero columns)
    for (int i = threadIdx.x; i < MAXE * Ep && i < MAXE * MAXE; i += 256) {
        const int f = i / Ep, e = i - f * Ep;
        Zt[i] = (f < Et && e < Et) ? Z[f + (int64_t)e * ldz] : 0.0;
    }
    __syncthreads();
    const int64_t d = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (d >= S) return;
    double a[MAXE];
    double s = 0.0;
#pragma unroll
    for (int e = 0; e < MAXE; ++e)
        if (e < Et) {
            a[e] = X[e * S + d];
            s += a[e];
        }
    const double xbar = s / (double)Et;
#pragma unroll
    for (int e = 0; e < MAXE; ++e)
        if (e < Et) a[e] = a[e] - xbar;
    for (int e0 = 0; e0 < Et; e0 += EG) {
        double acc[EG];
#pragma unroll
        for (int j = 0; j < EG; ++j) acc[j] = 0.0;
#pragma unroll
        for (int f = 0; f < MAXE; ++f)
            if (f < Et) {
                const double* z = Zt + f * Ep + e0;
#pragma unroll
                for (int j = 0; j < EG; ++j) acc[j] = __builtin_fma(a[f], z[j], acc[j]);
            }
#pragma unroll
        for (int j = 0; j < EG; ++j)
            if (e0 + j < Et) G[(e0 + j) * S + d] = acc[j];
    }
}

// HA[g + e m] = A[e][gslot[g]],  D[g + e m] = Y[g][e] - X[e][gslot[g]]
__global__ void gauge_gather(const double* __restrict__ A, const double* __restrict__ X,
                             const int64_t* __restrict__ gslot, const double* __restrict__ Y,
                             double* __restrict__ HA, double* __restrict__ D, int64_t m,
                             int64_t ns, int64_t E) {
    const int64_t total = m * E;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = x / m;
        const int64_t g = x - e * m;
        const int64_t d = gslot[g];
        HA[x] = A[e * ns + d];
        if (D) D[x] = Y[g * E + e] - X[e * ns + d];
    }
}

// HX[e m + g] = X[e][gslot[g]],  D[e m + g] = Y[g][e] - HX  (local members)
__global__ void gauge_values(const double* __restrict__ X, const int64_t* __restrict__ gslot,
                             const double* __restrict__ Y, double* __restrict__ HX,
                             double* __restrict__ D, int64_t m, int64_t ns, int64_t E) {
    const int64_t total = m * E;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = x / m;
        const int64_t g = x - e * m;
        const double v = X[e * ns + gslot[g]];
        HX[x] = v;
        D[x] = Y[g * E + e] - v;
    }
}

// member-major state [E][ns] -> reach slices for every rank: out[(r E + e) S + k] = X[e][r S + k]
__global__ void pack_slices(const double* __restrict__ X, double* __restrict__ out, int64_t ns,
                            int64_t E, int64_t S, int64_t N) {
    const int64_t total = N * E * S;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t re = x / S;
        const int64_t k = x - re * S;
        const int64_t r = re / E;
        const int64_t e = re - r * E;
        const int64_t d = r * S + k;
        out[x] = d < ns ? X[e * ns + d] : 0.0;
    }
}

// inverse: G[e][r S + k] = in[(r E + e) S + k]
__global__ void unpack_slices(const double* __restrict__ in, double* __restrict__ G, int64_t ns,
                              int64_t E, int64_t S, int64_t N) {
    const int64_t total = N * E * S;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t re = x / S;
        const int64_t k = x - re * S;
        const int64_t r = re / E;
        const int64_t e = re - r * E;
        const int64_t d = r * S + k;
        if (d < ns) G[e * ns + d] = in[x];
    }
}

// _apply_gain (nutils.py:116-134) per member on slot-order state:
//   o_gain[j] = 0 + G[j] for reaches the reference walk processes, 0 otherwise;
//   i_gain[j] = ((0 + o_gain[u1]) + o_gain[u2]) + ...  over j's routed upstreams in rank order;
//   o += o_gain,  i += i_gain   (da.py:124-126)
constexpr int kGainMembers = 4;   // members per thread in apply_gain
__global__ __launch_bounds__(256) void apply_gain(const double* __restrict__ G,
                                                  double* __restrict__ st_o,
                                                  double* __restrict__ st_i,
                                                  const uint8_t* __restrict__ flags,
                                                  const int32_t* __restrict__ up_off,
                                                  const int32_t* __restrict__ up, int64_t ns,
                                                  int64_t E) {
    // one slot (x) and kGainMembers members (y) per thread: the slot's upstream list is read
    // once and the members' loads are independent (a grid-stride loop over [E][ns] with one
    // element per iteration ran a 4-deep dependent load chain per element)
    const int64_t d = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= ns) return;
    const uint8_t f = flags[d];
    if (f != kSlotRouted && f != kSlotUnrouted) return;   // padding / partial sums
    const int32_t u0 = up_off[d], u1 = up_off[d + 1];
    const int64_t eb = (int64_t)blockIdx.y * kGainMembers;
    double og[kGainMembers], ig[kGainMembers];
#pragma unroll
    for (int j = 0; j < kGainMembers; ++j) {
        const int64_t e = eb + j < E ? eb + j : E - 1;
        og[j] = f == kSlotRouted ? 0.0 + G[e * ns + d] : 0.0;
        ig[j] = 0.0;
    }
    for (int32_t k = u0; k < u1; ++k) {
        const int64_t u = up[k];
#pragma unroll
        for (int j = 0; j < kGainMembers; ++j) {
            const int64_t e = eb + j < E ? eb + j : E - 1;
            ig[j] = ig[j] + (0.0 + G[e * ns + u]);
        }
    }
#pragma unroll
    for (int j = 0; j < kGainMembers; ++j) {
        if (eb + j >= E) break;
        const int64_t x = (eb + j) * ns + d;
        st_o[x] = st_o[x] + og[j];
        st_i[x] = st_i[x] + ig[j];
    }
}

// Kt[g + j ldk] (m x n, solved in place) -> K_out[j][g] in caller order: K_out[j * m + g]
__global__ void gain_to_caller(const double* __restrict__ Kt, int64_t ldk, double* __restrict__ out,
                               const int64_t* __restrict__ pos, int64_t m, int64_t n) {
    const int64_t total = n * m;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t j = x / m;
        const int64_t g = x - j * m;
        out[x] = Kt[g + pos[j] * ldk];
    }
}

inline int grid_for(int64_t work, int block) {
    int64_t g = (work + block - 1) / block;
    if (g < 1) g = 1;
    if (g > 65536) g = 65536;
    return (int)g;
}

}  // namespace

namespace {

struct Second {
    const double* B2;
    int64_t n1;
    double* C2;
};

template <bool TA, bool TB>
void dgemm_go(dim3 grid, hipStream_t s, int64_t M, int64_t N, int64_t K, double alpha,
              const double* A, int64_t lda, const double* B, int64_t ldb, double beta, double* C,
              int64_t ldc, int64_t kc, Second t) {
    hipLaunchKernelGGL((dgemm_mfma<TA, TB>), grid, 256, 0, s, M, N, K, alpha, A, lda, B, ldb,
                       beta, C, ldc, kc, t.B2, t.n1, t.C2);
}

}  // namespace

hipError_t launch_dgemm(bool ta, bool tb, int64_t M, int64_t N, int64_t K, double alpha,
                        const double* A, int64_t lda, const double* B, int64_t ldb, double beta,
                        double* C, int64_t ldc, hipStream_t s, double* work, size_t work_elems,
                        const double* B2, int64_t n1, double* C2) {
    if (M <= 0 || N <= 0) return hipSuccess;
    if (n1 < 0 || n1 > N) n1 = N;
    if (n1 < N && (!B2 || !C2)) return hipErrorInvalidValue;
    const int64_t gm = (M + kTile - 1) / kTile, gn = (N + kTile - 1) / kTile;
    if (gm > 0x7fffffff || gn > 65535) return hipErrorInvalidValue;
    // few output tiles and a deep reduction (the E x E products of the analysis, K = gauges):
    // split K over workgroups into the workspace, then reduce the slices in order
    int splits = 1;
    if (work && gm * gn < 64 && K >= 8 * kBK) {
        splits = (int)std::min<int64_t>(std::min<int64_t>(256 / (gm * gn), K / (4 * kBK)), 64);
        while (splits > 1 && (size_t)splits * M * N > work_elems) --splits;
    }
    const int64_t kc = splits > 1 ? ((K + splits - 1) / splits + kBK - 1) / kBK * kBK : K;
    if (splits > 1) splits = (int)((K + kc - 1) / kc);
    const dim3 grid((unsigned)gm, (unsigned)gn, (unsigned)splits);
    double* out = splits > 1 ? work : C;
    const double a = splits > 1 ? 1.0 : alpha, b = splits > 1 ? 0.0 : beta;
    const int64_t ld = splits > 1 ? M : ldc;
    // split-K slices are contiguous M x N panels: the second part stays in them until the reduce
    const Second t = splits > 1 ? Second{B2, n1, work + n1 * M} : Second{B2, n1, C2};
    if (!ta && !tb) dgemm_go<false, false>(grid, s, M, N, K, a, A, lda, B, ldb, b, out, ld, kc, t);
    else if (!ta && tb) dgemm_go<false, true>(grid, s, M, N, K, a, A, lda, B, ldb, b, out, ld, kc, t);
    else if (ta && !tb) dgemm_go<true, false>(grid, s, M, N, K, a, A, lda, B, ldb, b, out, ld, kc, t);
    else dgemm_go<true, true>(grid, s, M, N, K, a, A, lda, B, ldb, b, out, ld, kc, t);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || splits == 1) return e;
    hipLaunchKernelGGL(splitk_reduce, dim3((unsigned)((M * N + 255) / 256)), 256, 0, s, work,
                       splits, M, N, alpha, beta, C, ldc, n1, C2);
    return hipGetLastError();
}

hipError_t launch_scale_rows(const double* HA, const double* r, double* U, int64_t m, int64_t E,
                             hipStream_t s) {
    if (m * E > 0)
        hipLaunchKernelGGL(scale_rows, grid_for(m * E, 256), 256, 0, s, HA, r, U, m, E);
    return hipGetLastError();
}

hipError_t launch_mean_anomalies(const double* X, double* A, int64_t ns, int64_t E,
                                 hipStream_t s) {
    if (ns <= 8192 && E >= 32 && E <= kRowMaxE)
        hipLaunchKernelGGL(mean_anomalies_rows, dim3((unsigned)((ns + 3) / 4)), 256, 0, s, X, A,
                           ns, E);
    else
        hipLaunchKernelGGL(mean_anomalies, grid_for(ns, 256), 256, 0, s, X, A, ns, E);
    return hipGetLastError();
}

hipError_t launch_anomaly_increments(const double* X, const double* Z, int64_t ldz, double* G,
                                     int64_t S, int64_t Et, hipStream_t s) {
    if (S <= 0) return hipSuccess;
    if (Et < 2 || Et > kFusedIncrementsMax) return hipErrorInvalidValue;
    const unsigned g = (unsigned)((S + 255) / 256);
    if (Et <= 16)
        hipLaunchKernelGGL(anomaly_increments<16>, g, 256, 0, s, X, Z, ldz, G, S, (int)Et);
    else if (Et <= 32)
        hipLaunchKernelGGL(anomaly_increments<32>, g, 256, 0, s, X, Z, ldz, G, S, (int)Et);
    else
        hipLaunchKernelGGL(anomaly_increments<64>, g, 256, 0, s, X, Z, ldz, G, S, (int)Et);
    return hipGetLastError();
}

hipError_t launch_gauge_gather(const double* A, const double* X, const int64_t* gslot,
                               const double* Y, double* HA, double* D, int64_t m, int64_t ns,
                               int64_t E, hipStream_t s) {
    if (m <= 0) return hipSuccess;
    hipLaunchKernelGGL(gauge_gather, grid_for(m * E, 256), 256, 0, s, A, X, gslot, Y, HA, D, m,
                       ns, E);
    return hipGetLastError();
}

hipError_t launch_gauge_values(const double* X, const int64_t* gslot, const double* Y,
                               double* HX, double* D, int64_t m, int64_t ns, int64_t E,
                               hipStream_t s) {
    if (m <= 0) return hipSuccess;
    hipLaunchKernelGGL(gauge_values, grid_for(m * E, 256), 256, 0, s, X, gslot, Y, HX, D, m, ns,
                       E);
    return hipGetLastError();
}

hipError_t launch_pack_slices(const double* X, double* out, int64_t ns, int64_t E, int64_t S,
                              int64_t N, hipStream_t s) {
    hipLaunchKernelGGL(pack_slices, grid_for(N * E * S, 256), 256, 0, s, X, out, ns, E, S, N);
    return hipGetLastError();
}

hipError_t launch_unpack_slices(const double* in, double* G, int64_t ns, int64_t E, int64_t S,
                                int64_t N, hipStream_t s) {
    hipLaunchKernelGGL(unpack_slices, grid_for(N * E * S, 256), 256, 0, s, in, G, ns, E, S, N);
    return hipGetLastError();
}

hipError_t launch_apply_gain(const double* G, double* st_o, double* st_i, const uint8_t* flags,
                             const int32_t* up_off, const int32_t* up, int64_t ns, int64_t E,
                             hipStream_t s) {
    if (ns * E == 0) return hipSuccess;
    const int64_t gy = (E + kGainMembers - 1) / kGainMembers;
    if (gy > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(apply_gain, dim3((unsigned)((ns + 255) / 256), (unsigned)gy), 256, 0, s, G,
                       st_o, st_i, flags, up_off, up, ns, E);
    return hipGetLastError();
}

hipError_t launch_gain_to_caller(const double* Kt, int64_t ldk, double* out, const int64_t* pos,
                                 int64_t m, int64_t n, hipStream_t s) {
    if (n <= 0 || m <= 0) return hipSuccess;
    hipLaunchKernelGGL(gain_to_caller, grid_for(n * m, 256), 256, 0, s, Kt, ldk, out, pos, m, n);
    return hipGetLastError();
}

}  // namespace mcr
