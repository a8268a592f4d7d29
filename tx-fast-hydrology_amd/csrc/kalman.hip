// Full-covariance Kalman filter on the device: the da.py KalmanFilter and
// KalmanSmoother products, with the covariance resident in HBM.
//
//   _ap_par   (nutils.py:157-170):  out = A P            one _ax sweep per column of P
//   _aqat_par (nutils.py:194-214):  out = A (A P)^T      = A P A^T for symmetric P
//   filter    (da.py:91-136):       P- = A P A^T + Q,  K = P-[:, s] (P-[s, s] + R)^-1,
//                                   gain = K dz,  P+ = P- - K P-[s, :]
//   _apply_gain (nutils.py:116-134) as a stateless gather
//
// A is never formed.  Applying it to a column is the reference walk _ax (nutils.py:91-114):
//   o[j] = 0 + ((alpha_j I[j] + beta_j Ip[j]) + chi_j x[j])
//   I[j]  = ((0 + o[u1]) + o[u2]) + ...   routed upstreams in the walk's finalisation order
//   Ip[j] = ((0 + x[i1]) + x[i2]) + ...   every i with endnodes[i] == j, in index order, self-loops
//                                         included (numba_init_inflows, nutils.py:136-141)
// Columns are independent, so they map to lanes (16 per workgroup, coalesced 128-B row
// segments); reaches are swept level by level (a level's reaches depend only on lower levels),
// 16 reach lanes per workgroup, one barrier per level.  Networks up to ~1300 reaches take the
// staged form (ax_columns_staged: everything a level reads is in LDS).
// Results are bit-identical to the reference walk: same operations, same association, same
// summation order, FMA contraction off.  The dense update products run on the f64 MFMA GEMM
// (analysis.hip); the m x m gain system P-[s, s] + R and the n x n RTS system P_p1 are SPD and
// are solved by the library's block Gauss-Jordan elimination (dense.hip, launch_spd_solve; no
// vendor solver).  numpy's inv / solve are LU: results agree to rounding (g5 / g11 tests).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "analysis.hpp"
#include "capi_common.hpp"
#include "mcroute.h"

#pragma clang fp contract(off)

namespace mcr {
namespace {

using namespace capi;

constexpr int kCB = 16;                  // columns per workgroup
constexpr int kRL = 256 / kCB;           // reach lanes per workgroup
constexpr size_t kLdsLimit = 160 * 1024; // LDS of one workgroup

struct GraphArgs {
    const int32_t* lv_off;   // [n_levels + 1] into lv_reach
    const int32_t* lv_reach; // routed reaches, level by level
    const int32_t* up_off;   // [n + 1] routed upstreams in finalisation order
    const int32_t* up;
    const int32_t* in_off;   // [n + 1] every upstream (index order, self-loops) for Ip
    const int32_t* in_src;
    const int32_t* unrouted; // reaches the walk never finalises (cycles): o = 0
    const double* alpha;
    const double* beta;
    const double* chi;
    int32_t n_levels;
    int32_t n_unrouted;
};

// Y[:, c] = A X[:, c] for the columns c of this workgroup; X, Y row-major n x ld (networks
// too large for the staged sweep below).
__global__ __launch_bounds__(256) void ax_columns(GraphArgs a, const double* __restrict__ X,
                                                  double* __restrict__ Y, int64_t ld,
                                                  int64_t C) {
    const int cl = threadIdx.x % kCB;
    const int rl = threadIdx.x / kCB;
    const int64_t c = (int64_t)blockIdx.x * kCB + cl;
    const bool col = c < C;
    const int64_t cs = col ? c : 0;  // keep loads in bounds for idle lanes
    for (int k = rl; k < a.n_unrouted; k += kRL)
        if (col) Y[(int64_t)a.unrouted[k] * ld + c] = 0.0;
    for (int lv = 0; lv < a.n_levels; ++lv) {
        const int e = a.lv_off[lv + 1];
        for (int k = a.lv_off[lv] + rl; k < e; k += kRL) {
            const int j = a.lv_reach[k];
            double ip = 0.0;
            for (int q = a.in_off[j], qe = a.in_off[j + 1]; q < qe; ++q)
                ip += X[(int64_t)a.in_src[q] * ld + cs];
            double in = 0.0;
            for (int q = a.up_off[j], qe = a.up_off[j + 1]; q < qe; ++q) {
                const int u = a.up[q];
                in += Y[(int64_t)u * ld + cs];
            }
            const double o = 0.0 + ((a.alpha[j] * in + a.beta[j] * ip) +
                                    a.chi[j] * X[(int64_t)j * ld + cs]);
            if (col) Y[(int64_t)j * ld + c] = o;
        }
        __syncthreads();
    }
}

// Staged sweep (n small enough that a workgroup keeps all it reads in LDS).  The level chain of
// ax_columns waits at every level on dependent global loads (the reach index, its upstream
// lists, x and the inflow-list terms: ~1.5 us per level).  Here the chain-independent terms
// are formed by one parallel pass (ax_terms) and every workgroup stages its kCS columns of
// them, the coefficients and the level / upstream lists in LDS before the sweep, so a level
// costs LDS round trips and one barrier.  Same operations and association:
//   o = 0 + ((alpha * I + t1) + t2),  t1 = beta * Ip,  t2 = chi * x  (products as before).
constexpr int kCS = 4;                   // columns per workgroup (staged sweep)
constexpr int kRS = 256 / kCS;           // reach lanes per workgroup (staged sweep)

// Tm[j * C + c] = {beta_j Ip[j][c], chi_j X[j][c]}  for routed and unrouted reaches alike
__global__ __launch_bounds__(256) void ax_terms(GraphArgs a, const double* __restrict__ X,
                                                double2* __restrict__ Tm, int64_t ld, int64_t n,
                                                int64_t C) {
    const int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= n * C) return;
    const int64_t j = x / C, c = x - j * C;
    double ip = 0.0;
    for (int q = a.in_off[j], qe = a.in_off[j + 1]; q < qe; ++q)
        ip += X[(int64_t)a.in_src[q] * ld + c];
    Tm[x] = make_double2(a.beta[j] * ip, a.chi[j] * X[j * ld + c]);
}

// LDS bytes of the staged sweep: outputs [n][kCS] f64, terms [n][kCS] double2, alpha [n],
// level entries [n_routed] int4 {reach, first, end of its upstream list, first upstream},
// upstreams [n_up], level offsets [L + 1]
inline size_t staged_lds_bytes(int64_t n, int64_t L, int64_t n_routed, int64_t n_up) {
    return (size_t)n * kCS * 8 + (size_t)n * kCS * 16 + (size_t)n * 8 + 16 * (size_t)n_routed +
           4 * (size_t)(n_up + L + 1);
}

__global__ __launch_bounds__(256) void ax_columns_staged(GraphArgs a,
                                                         const int4* __restrict__ lvx,
                                                         const double2* __restrict__ Tm,
                                                         double* __restrict__ Y, int64_t ld,
                                                         int64_t n, int64_t C, int32_t n_routed,
                                                         int32_t n_up) {
    extern __shared__ double lsm[];
    double* ys = lsm;                                            // [n][kCS]
    double2* tt = reinterpret_cast<double2*>(ys + n * kCS);      // [n][kCS]
    int4* lx = reinterpret_cast<int4*>(tt + n * kCS);            // [n_routed] (16-B aligned)
    double* al = reinterpret_cast<double*>(lx + n_routed);       // [n]
    int32_t* ul = reinterpret_cast<int32_t*>(al + n);            // [n_up]
    int32_t* lo = ul + n_up;                                     // [L + 1]
    const int cl = threadIdx.x % kCS;
    const int rl = threadIdx.x / kCS;
    const int64_t c0 = (int64_t)blockIdx.x * kCS;
    const int64_t c = c0 + cl;
    const bool col = c < C;
    // staging: 8 independent loads in flight per lane (one latency per batch, not per item)
    for (int64_t x0 = threadIdx.x; x0 < n * kCS; x0 += 8 * 256) {
        double2 v[8];
#pragma unroll
        for (int b = 0; b < 8; ++b) {
            const int64_t x = x0 + b * 256;
            const int64_t j = x / kCS, cc = c0 + (x - j * kCS);
            v[b] = x < n * kCS && cc < C ? Tm[j * C + cc] : make_double2(0.0, 0.0);
        }
#pragma unroll
        for (int b = 0; b < 8; ++b)
            if (x0 + b * 256 < n * kCS) tt[x0 + b * 256] = v[b];
    }
    for (int64_t j = threadIdx.x; j < n; j += 256) al[j] = a.alpha[j];
    for (int k = threadIdx.x; k <= a.n_levels; k += 256) lo[k] = a.lv_off[k];
    for (int k = threadIdx.x; k < n_routed; k += 256) lx[k] = lvx[k];
    for (int k = threadIdx.x; k < n_up; k += 256) ul[k] = a.up[k];
    for (int k = rl; k < a.n_unrouted; k += kRS)
        if (col) Y[(int64_t)a.unrouted[k] * ld + c] = 0.0;
    __syncthreads();
    int b = a.n_levels > 0 ? lo[0] : 0, e = a.n_levels > 0 ? lo[1] : 0;
    for (int lv = 0; lv < a.n_levels; ++lv) {
        const int ne = lv + 2 <= a.n_levels ? lo[lv + 2] : 0;   // next level's end, early
        for (int k = b + rl; k < e; k += kRS) {
            const int4 x = lx[k];                 // {j, q0, q1, ul[q0]}: one LDS hop
            const int j = x.x;
            const double alj = al[j];             // independent of the fold: read first
            const double2 t = tt[j * kCS + cl];
            double in = 0.0;
            if (x.y < x.z) in += ys[x.w * kCS + cl];
            for (int q = x.y + 1; q < x.z; ++q) in += ys[ul[q] * kCS + cl];
            const double o = 0.0 + ((alj * in + t.x) + t.y);
            ys[j * kCS + cl] = o;
            if (col) Y[(int64_t)j * ld + c] = o;
        }
        b = e;
        e = ne;
        __syncthreads();
    }
}

// out = in^T (n x n row-major), 32 x 32 tiles through LDS
__global__ __launch_bounds__(256) void transpose(const double* __restrict__ in,
                                                 double* __restrict__ out, int64_t n) {
    __shared__ double t[32][33];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
    const int64_t r0 = (int64_t)blockIdx.y * 32, c0 = (int64_t)blockIdx.x * 32;
    for (int k = ty; k < 32; k += 8)
        if (r0 + k < n && c0 + tx < n) t[k][tx] = in[(r0 + k) * n + c0 + tx];
    __syncthreads();
    for (int k = ty; k < 32; k += 8)
        if (c0 + k < n && r0 + tx < n) out[(c0 + k) * n + r0 + tx] = t[tx][k];
}

__global__ void add_into(double* __restrict__ y, const double* __restrict__ q, int64_t cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cnt) y[i] = y[i] + q[i];
}

__global__ void sub_into(double* __restrict__ y, const double* __restrict__ a,
                         const double* __restrict__ b, int64_t cnt) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cnt) y[i] = a[i] - b[i];
}

// _apply_gain: o[j] = 0 + g[j] (routed), i[j] = fold of the routed upstream o in walk order
__global__ void apply_gain_gather(GraphArgs a, const uint8_t* __restrict__ routed,
                                  const double* __restrict__ g, double* __restrict__ io,
                                  double* __restrict__ oo, int64_t n) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    double in = 0.0;
    for (int q = a.up_off[j], qe = a.up_off[j + 1]; q < qe; ++q) in += 0.0 + g[a.up[q]];
    io[j] = in;
    oo[j] = routed[j] ? 0.0 + g[j] : 0.0;
}

// S (column-major m x m) = P[s][:, s] + R (R row-major, as numpy);
// Bt (column-major m x n) = P[:, s]^T;  Ps (column-major m x n) = P[s, :]
// Gathers of the KF update for the padded SPD solve (kp = spd_padded(m), column-major):
//   St (kp x kp) = (P[s, s] + R)^T with an identity block beyond m  (getrs(transpose) of the
//                  reference's K = P[:, s] inv(P[s, s] + R): K^T solves St Y = P[s, :])
//   Bt (kp x n)  = P[:, s]^T, padding rows 0;   Ps (m x n) = P[s, :]
__global__ void kf_gather(const double* __restrict__ P, const int64_t* __restrict__ s,
                          const double* __restrict__ R, double* __restrict__ St,
                          double* __restrict__ Bt, double* __restrict__ Ps, int64_t n,
                          int64_t m, int64_t kp) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx < kp * n) {
        const int64_t g = idx % kp, j = idx / kp;
        Bt[idx] = g < m ? P[j * n + s[g]] : 0.0;
    }
    if (idx < m * n) {
        const int64_t g = idx % m, j = idx / m;
        Ps[idx] = P[s[g] * n + j];
    }
    if (idx < kp * kp) {
        const int64_t a = idx % kp, b = idx / kp;
        St[idx] = (a < m && b < m) ? P[s[b] * n + s[a]] + R[b * m + a] : (a == b ? 1.0 : 0.0);
    }
}

// dst (kp x ncols, column-major, ld kp) = the column-major form of the row-major n x n src
// (dst[i + j kp] = src[i n + j]), `diag` on the diagonal beyond n and 0 elsewhere; 32 x 32
// tiles through LDS (coalesced on both sides)
__global__ __launch_bounds__(256) void colmajor_padded(const double* __restrict__ src, int64_t n,
                                                       double* __restrict__ dst, int64_t kp,
                                                       int64_t ncols, double diag) {
    __shared__ double t[32][33];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 32 x 8
    const int64_t i0 = (int64_t)blockIdx.x * 32, j0 = (int64_t)blockIdx.y * 32;
    for (int k = ty; k < 32; k += 8) {                       // rows i0 + k of src, columns j0..
        const int64_t i = i0 + k, j = j0 + tx;
        t[k][tx] = (i < n && j < n) ? src[i * n + j] : 0.0;
    }
    __syncthreads();
    for (int k = ty; k < 32; k += 8) {                       // column j0 + k of dst, rows i0..
        const int64_t j = j0 + k, i = i0 + tx;
        if (i < kp && j < ncols)
            dst[i + j * kp] = (i < n && j < n) ? t[tx][k] : (i == j ? diag : 0.0);
    }
}

dim3 blocks_for(int64_t cnt, int threads) {
    return dim3((unsigned)((cnt + threads - 1) / threads));
}

template <class T>
void upload_vec(DBuf<T>& d, const std::vector<T>& v, hipStream_t s) {
    d.upload(v.data(), v.size(), s);
}

}  // namespace

// Reach graph of one network for the covariance sweeps (walk replay of nutils._ax).
struct Cov {
    int64_t n = 0;
    hipStream_t own = nullptr, stream = nullptr;
    int32_t n_levels = 0, n_unrouted = 0, n_routed = 0, n_up = 0;
    DBuf<int32_t> lv_off, lv_reach, up_off, up, in_off, in_src, unrouted;
    DBuf<uint8_t> routed;
    DBuf<double> alpha, beta, chi;
    bool coeffs_set = false;
    // scratch: A P, the transposed product, KF gathers, gain / dz / R / gauges, LU state
    DBuf<double> T1, T2, T3, S, Bt, Ps, gdev, ddev, Rdev;
    DBuf<double2> Tm;                  // chain-independent terms of the staged sweep
    DBuf<int4> lvx;                    // staged sweep: {reach, q0, q1, up[q0]} per level slot
    DBuf<int64_t> sdev;
    DBuf<double> Sd;                   // pivot-block inverses of the Gauss-Jordan solve
    DBuf<int32_t> info;

    ~Cov() {
        if (own) (void)hipStreamDestroy(own);
    }

    void build(int64_t n_, const int64_t* end, const int64_t* indeg, const int64_t* heads,
               int64_t n_head) {
        n = n_;
        REQUIRE(n < (int64_t)INT32_MAX, "network too large for the covariance sweep");
        for (int64_t j = 0; j < n; ++j)
            if (end[j] < 0 || end[j] >= n)
                throw Fail(MC_E_TOPOLOGY, "endnodes index out of range");
        // walk replay (nutils.py:98-113): finalisation order, levels, routed upstream lists
        std::vector<int64_t> left(indeg, indeg + n);
        std::vector<int32_t> level(n, 0), rank(n, -1);
        std::vector<std::vector<int32_t>> ups(n);
        int32_t r = 0;
        for (int64_t k = 0; k < n_head; ++k) {
            int64_t j = heads[k];
            if (j < 0 || j >= n) throw Fail(MC_E_TOPOLOGY, "headwater index out of range");
            while (left[j] == 0) {
                if (rank[j] >= 0)
                    throw Fail(MC_E_TOPOLOGY,
                               "a reach would be finalised twice (inconsistent indegree)");
                rank[j] = r++;
                const int64_t d = end[j];
                if (d != j) {
                    ups[d].push_back((int32_t)j);
                    level[d] = std::max(level[d], level[j] + 1);
                }
                left[d] -= 1;
                j = d;
            }
        }
        std::vector<int32_t> uo(n + 1, 0), ul, io(n + 1, 0), il, un;
        for (int64_t j = 0; j < n; ++j) {
            uo[j + 1] = uo[j] + (int32_t)ups[j].size();
            ul.insert(ul.end(), ups[j].begin(), ups[j].end());
        }
        std::vector<std::vector<int32_t>> ins(n);
        for (int64_t i = 0; i < n; ++i) ins[end[i]].push_back((int32_t)i);
        for (int64_t j = 0; j < n; ++j) {
            io[j + 1] = io[j] + (int32_t)ins[j].size();
            il.insert(il.end(), ins[j].begin(), ins[j].end());
        }
        int32_t L = 0;
        std::vector<uint8_t> rt(n, 0);
        for (int64_t j = 0; j < n; ++j) {
            if (rank[j] >= 0) {
                rt[j] = 1;
                L = std::max(L, level[j] + 1);
            } else {
                un.push_back((int32_t)j);
            }
        }
        std::vector<int32_t> lo(L + 1, 0), lr(r);
        for (int64_t j = 0; j < n; ++j)
            if (rt[j]) lo[level[j] + 1]++;
        for (int32_t l = 0; l < L; ++l) lo[l + 1] += lo[l];
        std::vector<int32_t> fill(lo.begin(), lo.end() - 1);
        for (int64_t j = 0; j < n; ++j)
            if (rt[j]) lr[fill[level[j]]++] = (int32_t)j;
        n_levels = L;
        n_unrouted = (int32_t)un.size();
        n_routed = r;
        n_up = (int32_t)ul.size();
        HIPC(hipStreamCreateWithFlags(&own, hipStreamNonBlocking));
        stream = own;
        upload_vec(lv_off, lo, stream);
        upload_vec(lv_reach, lr, stream);
        {
            std::vector<int4> lx(lr.size());
            for (size_t k = 0; k < lr.size(); ++k) {
                const int32_t j = lr[k], q0 = uo[j], q1 = uo[j + 1];
                lx[k] = make_int4(j, q0, q1, q1 > q0 ? ul[q0] : 0);
            }
            upload_vec(lvx, lx, stream);
        }
        upload_vec(up_off, uo, stream);
        upload_vec(up, ul, stream);
        upload_vec(in_off, io, stream);
        upload_vec(in_src, il, stream);
        upload_vec(unrouted, un, stream);
        upload_vec(routed, rt, stream);
        HIPC(hipStreamSynchronize(stream));
    }

    GraphArgs args() const {
        GraphArgs a;
        a.lv_off = lv_off.p;
        a.lv_reach = lv_reach.p;
        a.up_off = up_off.p;
        a.up = up.p;
        a.in_off = in_off.p;
        a.in_src = in_src.p;
        a.unrouted = unrouted.p;
        a.alpha = alpha.p;
        a.beta = beta.p;
        a.chi = chi.p;
        a.n_levels = n_levels;
        a.n_unrouted = n_unrouted;
        return a;
    }

    // Y = A X (square n x n, row-major); X and Y must not alias
    void ax(const double* X, double* Y) {
        REQUIRE(coeffs_set, "mc_cov_set_coeffs has not been called");
        if (n == 0) return;
        const size_t slds = staged_lds_bytes(n, n_levels, n_routed, n_up);
        if (slds <= kLdsLimit) {
            Tm.reserve((size_t)n * n);
            hipLaunchKernelGGL(ax_terms, blocks_for(n * n, 256), 256, 0, stream, args(), X, Tm.p,
                               n, n, n);
            HIPC(hipGetLastError());
            HIPC(hipFuncSetAttribute((const void*)ax_columns_staged,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)slds));
            hipLaunchKernelGGL(ax_columns_staged, dim3((unsigned)((n + kCS - 1) / kCS)), 256,
                               slds, stream, args(), lvx.p, Tm.p, Y, n, n, n, n_routed, n_up);
            HIPC(hipGetLastError());
            return;
        }
        const dim3 grid((unsigned)((n + kCB - 1) / kCB));
        hipLaunchKernelGGL(ax_columns, grid, 256, 0, stream, args(), X, Y, n, n);
        HIPC(hipGetLastError());
    }

    void aqat(const double* P, const double* Q, double* out) {
        if (n == 0) return;
        T1.reserve((size_t)n * n);
        T2.reserve((size_t)n * n);
        ax(P, T1.p);                                      // A P
        const dim3 tg((unsigned)((n + 31) / 32), (unsigned)((n + 31) / 32));
        hipLaunchKernelGGL(transpose, tg, 256, 0, stream, T1.p, T2.p, n);
        HIPC(hipGetLastError());
        ax(T2.p, out);                                    // A (A P)^T
        if (Q) {
            hipLaunchKernelGGL(add_into, blocks_for(n * n, 256), 256, 0, stream, out, Q, n * n);
            HIPC(hipGetLastError());
        }
    }

    void apply_gain(const double* g, double* io, double* oo) {
        if (n == 0) return;
        gdev.reserve(3 * (size_t)n);
        HIPC(hipMemcpyAsync(gdev.p, g, n * sizeof(double), hipMemcpyHostToDevice, stream));
        hipLaunchKernelGGL(apply_gain_gather, blocks_for(n, 256), 256, 0, stream, args(),
                           routed.p, gdev.p, gdev.p + n, gdev.p + 2 * n, n);
        HIPC(hipGetLastError());
        HIPC(hipMemcpyAsync(io, gdev.p + n, n * sizeof(double), hipMemcpyDeviceToHost, stream));
        HIPC(hipMemcpyAsync(oo, gdev.p + 2 * n, n * sizeof(double), hipMemcpyDeviceToHost,
                            stream));
        HIPC(hipStreamSynchronize(stream));
    }

    // da.py:118-122 on the prior P-: K (n x m) = P-[:, s] (P-[s, s] + R)^-1, gain = K dz,
    // P+ = P- - K P-[s, :].  P_post may alias P_prior (in-place posterior).
    void kf_update(int64_t m, const int64_t* s, const double* R, const double* dz,
                   const double* Pp, double* Pq, double* K_out, double* gain_out) {
        REQUIRE(m >= 1 && m <= n, "need 1 <= m <= n gauges");
        for (int64_t g = 0; g < m; ++g)
            REQUIRE(s[g] >= 0 && s[g] < n, "gauge index out of range");
        const int64_t kp = spd_padded(m);
        S.reserve((size_t)(kp * kp));
        Bt.reserve((size_t)(kp * n));
        Ps.reserve((size_t)m * n);
        Sd.reserve((size_t)(kp * 32));
        Rdev.upload(R, (size_t)m * m, stream);
        ddev.upload(dz, (size_t)m, stream);
        sdev.upload(s, (size_t)m, stream);
        gdev.reserve((size_t)std::max<int64_t>(3 * n, 1));
        info.reserve(1);
        hipLaunchKernelGGL(kf_gather, blocks_for(std::max(kp * n, kp * kp), 256), 256, 0,
                           stream, Pp, sdev.p, Rdev.p, S.p, Bt.p, Ps.p, n, m, kp);
        HIPC(hipGetLastError());
        // St Y = P-[s, :]  ->  Y = K^T (column-major m x n, leading dimension kp)
        HIPC(launch_spd_solve(S.p, kp, Bt.p, n, Sd.p, info.p, stream));
        HIPC(launch_dgemm(true, false, n, 1, m, 1.0, Bt.p, kp, ddev.p, m, 0.0, gdev.p, n,
                          stream));
        if (Pq != Pp)
            HIPC(hipMemcpyAsync(Pq, Pp, (size_t)n * n * sizeof(double), hipMemcpyDeviceToDevice,
                                stream));
        // column-major view Pc = P^T:  Pc+ = Pc - Ps^T Y
        HIPC(launch_dgemm(true, false, n, n, m, -1.0, Ps.p, m, Bt.p, kp, 1.0, Pq, n, stream));
        int32_t info_h = 0;
        HIPC(hipMemcpyAsync(&info_h, info.p, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
        HIPC(hipMemcpyAsync(gain_out, gdev.p, n * sizeof(double), hipMemcpyDeviceToHost,
                            stream));
        if (K_out)      // K row-major n x m = Y column-major m x n: drop the padding rows
            HIPC(hipMemcpy2DAsync(K_out, (size_t)m * sizeof(double), Bt.p,
                                  (size_t)kp * sizeof(double), (size_t)m * sizeof(double),
                                  (size_t)n, hipMemcpyDeviceToHost, stream));
        HIPC(hipStreamSynchronize(stream));
        if (info_h != 0)
            throw Fail(MC_E_STATE, "P-[s, s] + R is not positive definite (elimination pivot " +
                                       std::to_string(info_h) + ")");
    }

    // RTS step (da.py:241-251): J = (P_p1^-1 A P_f)^T, P_s = P_f + J (P_s1 - P_p1),
    // x_s = x_f + J d for nvec host vectors d = x_s1 - x_p1.  Row-major buffers are read as
    // column-major transposes: X = P_p1^-1 (A P_f) in column-major form (padded to kp, SPD block
    // Gauss-Jordan) is a buffer whose row-major view is J.
    void ks_step(const double* Pf, const double* Pp1, const double* Ps1, double* Ps_out,
                 int64_t nvec, const double* xf, const double* d, double* xs_out) {
        if (n == 0) return;
        REQUIRE(nvec >= 0 && (nvec == 0 || (xf && d && xs_out)), "bad vector arguments");
        const size_t nn = (size_t)n * n;
        const int64_t kp = spd_padded(n);
        T1.reserve(nn);
        T2.reserve((size_t)(kp * n));
        T3.reserve((size_t)(kp * kp));
        Sd.reserve((size_t)(kp * 32));
        info.reserve(1);
        ax(Pf, T1.p);                                               // A P_f (row-major)
        const dim3 tp((unsigned)((kp + 31) / 32), (unsigned)((kp + 31) / 32));
        const dim3 tb((unsigned)((kp + 31) / 32), (unsigned)((n + 31) / 32));
        hipLaunchKernelGGL(colmajor_padded, tp, 256, 0, stream, Pp1, n, T3.p, kp, kp, 1.0);
        HIPC(hipGetLastError());
        hipLaunchKernelGGL(colmajor_padded, tb, 256, 0, stream, T1.p, n, T2.p, kp, n, 0.0);
        HIPC(hipGetLastError());
        HIPC(launch_spd_solve(T3.p, kp, T2.p, n, Sd.p, info.p, stream));   // T2 := X (ld kp)
        hipLaunchKernelGGL(sub_into, blocks_for((int64_t)nn, 256), 256, 0, stream, T1.p, Ps1,
                           Pp1, (int64_t)nn);                      // D = P_s1 - P_p1
        HIPC(hipGetLastError());
        if (Ps_out != Pf)
            HIPC(hipMemcpyAsync(Ps_out, Pf, nn * sizeof(double), hipMemcpyDeviceToDevice,
                                stream));
        HIPC(launch_dgemm(false, false, n, n, n, 1.0, T1.p, n, T2.p, kp, 1.0, Ps_out, n,
                          stream));
        if (nvec > 0) {
            gdev.reserve((size_t)std::max<int64_t>(2 * nvec * n, 3 * n));
            HIPC(hipMemcpyAsync(gdev.p, d, nvec * n * sizeof(double), hipMemcpyHostToDevice,
                                stream));
            HIPC(hipMemcpyAsync(gdev.p + nvec * n, xf, nvec * n * sizeof(double),
                                hipMemcpyHostToDevice, stream));
            HIPC(launch_dgemm(true, false, n, nvec, n, 1.0, T2.p, kp, gdev.p, n, 1.0,
                              gdev.p + nvec * n, n, stream));
            HIPC(hipMemcpyAsync(xs_out, gdev.p + nvec * n, nvec * n * sizeof(double),
                                hipMemcpyDeviceToHost, stream));
        }
        int32_t info_h = 0;
        HIPC(hipMemcpyAsync(&info_h, info.p, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
        HIPC(hipStreamSynchronize(stream));
        if (info_h != 0)
            throw Fail(MC_E_STATE, "the predicted covariance is not positive definite "
                                   "(elimination pivot " + std::to_string(info_h) + ")");
    }
};

}  // namespace mcr

using mcr::Cov;
using namespace mcr::capi;

static Cov* as_cov(void* h) {
    REQUIRE(h, "NULL covariance handle");
    return static_cast<Cov*>(h);
}

extern "C" {

int mc_cov_create(int64_t n, const int64_t* endnodes, const int64_t* indegree,
                  const int64_t* headwaters, int64_t n_head, void** cov) {
    return guarded([&] {
        REQUIRE(cov, "cov must not be NULL");
        REQUIRE(n >= 0 && (n == 0 || (endnodes && indegree)), "bad network arrays");
        REQUIRE(n_head >= 0 && (n_head == 0 || headwaters), "bad headwater list");
        auto c = std::make_unique<Cov>();
        c->build(n, endnodes, indegree, headwaters, n_head);
        *cov = c.release();
    });
}

int mc_cov_destroy(void* cov) {
    return guarded([&] { delete static_cast<Cov*>(cov); });
}

int mc_cov_set_stream(void* cov, void* hip_stream) {
    return guarded([&] {
        Cov* c = as_cov(cov);
        c->stream = hip_stream ? static_cast<hipStream_t>(hip_stream) : c->own;
    });
}

int mc_cov_set_coeffs(void* cov, const double* alpha, const double* beta, const double* chi) {
    return guarded([&] {
        Cov* c = as_cov(cov);
        REQUIRE(c->n == 0 || (alpha && beta && chi), "coefficient arrays must not be NULL");
        c->alpha.upload(alpha, c->n, c->stream);
        c->beta.upload(beta, c->n, c->stream);
        c->chi.upload(chi, c->n, c->stream);
        HIPC(hipStreamSynchronize(c->stream));
        c->coeffs_set = true;
    });
}

int mc_cov_ap(void* cov, const double* P, double* out) {
    return guarded([&] {
        Cov* c = as_cov(cov);
        REQUIRE(c->n == 0 || (P && out && P != out), "P / out must be distinct device buffers");
        c->ax(P, out);
    });
}

int mc_cov_aqat(void* cov, const double* P, const double* Q, double* out) {
    return guarded([&] {
        Cov* c = as_cov(cov);
        REQUIRE(c->n == 0 || (P && out), "P / out must not be NULL");
        c->aqat(P, Q, out);
    });
}

int mc_cov_apply_gain(void* cov, const double* gain, double* i_gain, double* o_gain) {
    return guarded([&] {
        Cov* c = as_cov(cov);
        REQUIRE(c->n == 0 || (gain && i_gain && o_gain), "gain arrays must not be NULL");
        c->apply_gain(gain, i_gain, o_gain);
    });
}

int mc_kf_update(void* cov, int64_t m, const int64_t* s, const double* R, const double* dz,
                 const double* P_prior, double* P_post, double* K_out, double* gain_out) {
    return guarded([&] {
        Cov* c = as_cov(cov);
        REQUIRE(s && R && dz && P_prior && P_post && gain_out, "NULL argument");
        c->kf_update(m, s, R, dz, P_prior, P_post, K_out, gain_out);
    });
}

int mc_ks_step(void* cov, const double* P_f, const double* P_p1, const double* P_s1,
               double* P_s_out, int64_t nvec, const double* x_f, const double* d,
               double* x_s_out) {
    return guarded([&] {
        Cov* c = as_cov(cov);
        REQUIRE(c->n == 0 || (P_f && P_p1 && P_s1 && P_s_out), "NULL matrix");
        c->ks_step(P_f, P_p1, P_s1, P_s_out, nvec, x_f, d, x_s_out);
    });
}

int mc_cov_synchronize(void* cov) {
    return guarded([&] { HIPC(hipStreamSynchronize(as_cov(cov)->stream)); });
}

}  // extern "C"
