// Dense f64 linear algebra of the ensemble analysis on CDNA4 (gfx950), hand-written on
// v_mfma_f64_16x16x4f64 (da.py:119-122 K = P H^T (H P H^T + R)^-1 in its
// ensemble-space form):
//
//  * slice_increments: G = (X - mean_e X) Z for a member-major reach slice X [Et][S] and the
//    Et x Et analysis weights Z -- the largest product of the analysis (S x Et x Et,
//    2 S Et^2 flops).  128 x 128 output tiles, 4 waves of 64 x 64, K slices double-buffered in
//    LDS, the member mean folded in as a rank-1 epilogue correction (G = X' Z - xbar' zs^T with
//    X' = X shifted by member 0 of each slot, so the products are spread-sized) so X is read once
//    and no anomaly array is materialised.
//  * SPD solves B := A^-1 B by block Gauss-Jordan elimination with 32 x 32 pivot blocks on the
//    augmented system [A | B]: step J eliminates block column J from every other block row
//    (A_IC -= A_IJ S_J A_JC, B_I -= A_IJ S_J B_J, S_J = D_J^-1 the inverse of the pivot block),
//    and a last launch scales B_I := S_I B_I.  Every step is one launch whose workgroups each
//    update one block; the workgroup that updates the next pivot block inverts it (Gauss-Jordan
//    on [D | I] in one wave, which also detects a matrix that is not positive definite).  The
//    sequential chain is k / 32 + 2 launches and no separate substitution passes (a blocked
//    LDL^T + forward / backward substitution took ~250 us at k = 256: ~20 dependent cross-XCD
//    round trips).
// Matrices are column-major; the elimination works on a copy padded to kp = 32 * ceil(k / 32)
// with an identity block (pad_matrix), so every block is full.
#include "analysis.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>

namespace mcr {

namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f64x4 mfma4(double a, double b, f64x4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// =============================================================================================
// slice increments  G[e][d] = sum_f (X[f][d] - xbar[d]) Z[f][e]
// MFMA rows = members e (A operand = Z^T), columns = slots d (B operand = X), k = member f.
// MW wave rows of 64 members x 2 wave columns of 64 slots: a 64 MW x 128 tile, 128 MW threads
// (launched with MW = 2; MW = 4 reads X once at Et = 256 but was slower, launcher).
constexpr int kGN = 128;          // slots per tile
constexpr int kGK = 16;           // K slice
template <int MW>
constexpr int slice_stage() { return kGK * (64 * MW + kGN); }   // doubles per LDS stage

template <int MW>
__global__ __launch_bounds__(128 * MW, MW == 2 ? 2 : 1) void slice_increments(
        const double* __restrict__ X, const double* __restrict__ Z, int64_t ldz,
        double* __restrict__ G, int64_t S, int Et, int n_slot_tiles, int n_member_tiles) {
    constexpr int kGM = 64 * MW;           // members per tile
    constexpr int XF = 2 * MW;             // X rows (f) staged per pass
    constexpr int NXP = kGK / XF;          // X passes per K slice
    constexpr int kStage = slice_stage<MW>();
    extern __shared__ __attribute__((aligned(16))) double sm[];
    // XCD-aware tile order: the member tiles of one slot tile share its X rows; consecutive
    // workgroups go to consecutive XCDs, so blocks b, b + 8, ... (same XCD) take them
    const int b = blockIdx.x;
    const int xcd = b & 7;
    const int rest = b >> 3;
    const int mt = rest % n_member_tiles;
    const int st = (rest / n_member_tiles) * 8 + xcd;
    if (st >= n_slot_tiles) return;
    const int64_t d0 = (int64_t)st * kGN;
    const int e0 = mt * kGM;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = (wave >> 1) * 64, wc = (wave & 1) * 64;

    // global -> register staging of one K slice: Z^T (kGM members x 16 f) and X (16 f x 128 d)
    // Z: thread -> member e = tid >> 1, f = (tid & 1) * 8 + p (p < 8)
    // X: thread -> f = (tid >> 6) + XF p (p < NXP), slot pair 2 (tid & 63)
    // Two slices are in flight in registers (slice f + 2 loads while slice f's MFMAs run and
    // slice f + 1 is staged); the loads are unconditional at clamped addresses and masked after
    // (no branches, so the wait before staging counts only the older slice's loads).
    const int ze = tid >> 1, zf = (tid & 1) * 8;
    const int xf = __builtin_amdgcn_readfirstlane(tid >> 6), xd = 2 * (tid & 63);
    const bool zrow = e0 + ze < Et;
    const int64_t zcol = zrow ? (int64_t)(e0 + ze) * ldz : 0;
    const int64_t gd = d0 + xd;
    struct Slice {
        double z[8], x[2 * NXP];
    };
    double zsum = 0.0, xs0 = 0.0, xs1 = 0.0;     // partial sums for zs[e] and the mean of X
    // X is staged shifted by member 0's value of its slot (X - x0 1^T): the rank-1 mean
    // correction then works on spread-sized numbers, so reaches whose members agree get
    // increments of exactly 0 and a large mean with a small spread loses no digits (ADVICE r3;
    // the increments are (X - x0 1^T) Z - (xbar - x0) zs^T = (X - xbar 1^T) Z exactly in reals)
    const auto x0r = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(X), (short)0,
                                                       (int)(S * 8), 0x00020000);
    const double x0a = __builtin_bit_cast(
        double, __builtin_amdgcn_raw_buffer_load_b64(x0r, (unsigned)(gd * 8), 0, 0));
    const double x0b = __builtin_bit_cast(
        double, __builtin_amdgcn_raw_buffer_load_b64(x0r, (unsigned)(gd * 8 + 8), 0, 0));
    // buffer loads: an out-of-range offset (or an empty record) reads 0, so the edge masks are
    // offsets, not branches around the loads
    const int zrec = (int)(ldz * (int64_t)Et * 8);          // < 2^31 (launcher)
    const auto zr = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(Z), (short)0, zrec,
                                                      0x00020000);
    auto load = [&](Slice& r, int f0) {
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            const int f = f0 + zf + p;
            const bool ok = zrow && f < Et;
            const unsigned off = ok ? (unsigned)((f + zcol) * 8) : (unsigned)zrec;
            r.z[p] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(zr, off, 0, 0));
        }
#pragma unroll
        for (int p = 0; p < NXP; ++p) {
            const int f = f0 + xf + XF * p;     // wave-uniform: one X row per wave and pass
            const auto xr = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<double*>(X + (int64_t)(f < Et ? f : 0) * S), (short)0,
                f < Et ? (int)(S * 8) : 0, 0x00020000);
            r.x[2 * p] = __builtin_bit_cast(
                double, __builtin_amdgcn_raw_buffer_load_b64(xr, (unsigned)(gd * 8), 0, 0));
            r.x[2 * p + 1] = __builtin_bit_cast(
                double, __builtin_amdgcn_raw_buffer_load_b64(xr, (unsigned)(gd * 8 + 8), 0, 0));
        }
    };
    auto stage = [&](const Slice& r, int buf, int fb) {
        double* As = sm + buf * kStage;           // As[f][e]
        double* Bs = As + kGK * kGM;              // Bs[f][d]
#pragma unroll
        for (int p = 0; p < 8; ++p) {
            As[(zf + p) * kGM + ze] = r.z[p];
            zsum += r.z[p];
        }
#pragma unroll
        for (int p = 0; p < NXP; ++p) {
            const int f = xf + XF * p;
            const bool live = fb + f < Et;          // wave-uniform; rows past Et stage 0
            const double v0 = live ? r.x[2 * p] - x0a : 0.0;
            const double v1 = live ? r.x[2 * p + 1] - x0b : 0.0;
            *reinterpret_cast<double2*>(Bs + f * kGN + xd) = make_double2(v0, v1);
            xs0 += v0;
            xs1 += v1;
        }
    };

    f64x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f64x4{0.0, 0.0, 0.0, 0.0};

    // one K slice: slice f0 from LDS buffer `buf`; `next` holds slice f0 + kGK (staged into the
    // other buffer after the MFMAs), `fut` receives slice f0 + 2 kGK
    auto step = [&](int f0, int buf, Slice& next, Slice& fut) {
        load(fut, f0 + 2 * kGK);     // unconditional (past the end: out of range, reads 0), so
                                     // the wait before the staging below is a count, not 0
        const double* As = sm + buf * kStage;
        const double* Bs = As + kGK * kGM;
#pragma unroll
        for (int kk = 0; kk < kGK; kk += 4) {
            const int k = kk + (lane >> 4);
            double a[4], bb[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) a[i] = As[k * kGM + wr + 16 * i + (lane & 15)];
#pragma unroll
            for (int j = 0; j < 4; ++j) bb[j] = Bs[k * kGN + wc + 16 * j + (lane & 15)];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = mfma4(a[i], bb[j], acc[i][j]);
        }
        if (f0 + kGK < Et) stage(next, buf ^ 1, f0 + kGK);
        __syncthreads();
    };
    Slice ra, rb;
    load(ra, 0);
    stage(ra, 0, 0);
    __syncthreads();
    load(ra, kGK);
    for (int f0 = 0; f0 < Et; f0 += 2 * kGK) {
        step(f0, 0, ra, rb);
        if (f0 + kGK < Et) step(f0 + kGK, 1, rb, ra);
    }
    // member sums of X (XF partials per slot pair) and column sums of Z (2 partials per member)
    double* red = sm;                              // the K loop is over: reuse stage 0
    red[xf * kGN + xd] = xs0;
    red[xf * kGN + xd + 1] = xs1;
    const double zs_all = zsum + __shfl_xor(zsum, 1);
    if ((tid & 1) == 0) red[XF * kGN + ze] = zs_all;
    __syncthreads();
    const double inv = 1.0 / (double)Et;
    // C/D of f64 16x16x4: col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int dl = wc + 16 * j + (lane & 15);
        double xsum = red[dl];
#pragma unroll
        for (int q = 1; q < XF; ++q) xsum += red[q * kGN + dl];
        const double xbar = xsum * inv;
        const int64_t d = d0 + dl;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int el = wr + 16 * i + (lane >> 4) + 4 * r;
                const int e = e0 + el;
                if (e < Et && d < S) G[(int64_t)e * S + d] = acc[i][j][r] - red[XF * kGN + el] * xbar;
            }
    }
}

// =============================================================================================
// block LDL^T (32 x 32 blocks) and its solve
constexpr int kB = 32;
constexpr int kL = kB + 1;        // LDS row stride of a block (conflict-free column reads)

// One 16 x 16 output block per wave of a 32 x 32 x 32 product: wave w owns rows
// 16 (w >> 1) .. and columns 16 (w & 1) ..; a(i, k), b(k, j) read the operands
template <class FA, class FB>
__device__ __forceinline__ f64x4 mma32(FA a, FB b, f64x4 acc, int wave, int lane) {
    const int i = (wave >> 1) * 16 + (lane & 15);
    const int j = (wave & 1) * 16 + (lane & 15);
#pragma unroll
    for (int kk = 0; kk < kB; kk += 4) {
        const int k = kk + (lane >> 4);
        acc = mfma4(a(i, k), b(k, j), acc);
    }
    return acc;
}
__device__ __forceinline__ int blk_row(int wave, int lane, int r) {
    return (wave >> 1) * 16 + (lane >> 4) + 4 * r;
}
__device__ __forceinline__ int blk_col(int wave, int lane) {
    return (wave & 1) * 16 + (lane & 15);
}

// S = D^-1 for the SPD pivot block D (LDS, row stride kL) by Gauss-Jordan elimination on [D | I]
// inside ONE wave, without workgroup barriers: lane j holds column j of the 32 x 64 augmented
// matrix in registers; pivot k's column is broadcast through LDS (written by lane k, read by
// every lane at one address; LDS operations of one wave complete in order).  S goes to dst
// column-major (leading dimension kB) from lanes 32..63.  Returns 0, or k + 1 when pivot k is
// not positive (D not SPD).  Called by wave 0 only; col: 32 doubles of LDS scratch.
// Measured per EnKF256 elimination step (MI355X): 21.2 us vs 23.7 us for the 256-thread LDS
// elimination with one barrier per pivot and S = T^T T on MFMA; earlier one-wave forms with
// cross-lane permutes (~21 us per block) or scalar reads of the pivot lane in a runtime loop
// (~43 us) were no faster -- the 32-pivot chain is latency-bound in every form.
__device__ __forceinline__ int wave_block_inverse(const double* a, double* __restrict__ dst,
                                                  double* col) {
    const int lane = threadIdx.x & 63;
    double x[kB];
#pragma unroll
    for (int i = 0; i < kB; ++i)
        x[i] = lane < kB ? a[i * kL + lane] : (i == lane - kB ? 1.0 : 0.0);
#pragma unroll
    for (int k = 0; k < kB; ++k) {
        if (lane == k) {
#pragma unroll
            for (int i = 0; i < kB; i += 2)
                *reinterpret_cast<double2*>(col + i) = make_double2(x[i], x[i + 1]);
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);      // keep the write before the reads
        double c[kB];
#pragma unroll
        for (int i = 0; i < kB; i += 2) {
            const double2 v = *reinterpret_cast<const double2*>(col + i);
            c[i] = v.x;
            c[i + 1] = v.y;
        }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);      // and the reads before the next write
        const double piv = c[k];
        if (!(piv > 0.0)) return k + 1;               // the same value in every lane
        const double xk = x[k] / piv;
#pragma unroll
        for (int i = 0; i < kB; ++i)
            if (i != k) x[i] = x[i] - c[i] * xk;
        x[k] = xk;
    }
    if (lane >= kB) {
#pragma unroll
        for (int i = 0; i < kB; i += 2)
            *reinterpret_cast<double2*>(dst + (int64_t)(lane - kB) * kB + i) =
                make_double2(x[i], x[i + 1]);
    }
    return 0;
}

__device__ __forceinline__ void load_block(const double* src, int64_t ld, double* dst) {
    for (int x = threadIdx.x; x < kB * kB; x += 256) {
        const int i = x % kB, c = x / kB;
        dst[i * kL + c] = src[i + (int64_t)c * ld];
    }
}

// dst (kp x ncols, leading dimension kp) = src (rows x cols valid, leading dimension lds),
// `diag` on the diagonal outside it and 0 elsewhere
__global__ void pad_matrix(const double* __restrict__ src, int64_t rows, int64_t cols,
                           int64_t lds, double* __restrict__ dst, int64_t kp, double diag,
                           int64_t ncols) {
    const int64_t total = kp * ncols;
    for (int64_t x = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = x % kp, j = x / kp;
        dst[x] = (i < rows && j < cols) ? src[i + j * lds] : (i == j ? diag : 0.0);
    }
}

// first diagonal block: S_0 = A_00^-1
__global__ __launch_bounds__(256) void ldl_first(const double* __restrict__ P, int64_t kp,
                                                 double* __restrict__ Sd,
                                                 int32_t* __restrict__ info) {
    __shared__ double a[kB * kL], col[kB];
    if (threadIdx.x == 0) *info = 0;
    load_block(P, kp, a);
    __syncthreads();
    if (threadIdx.x >= 64) return;
    const int bad = wave_block_inverse(a, Sd, col);
    if (bad && threadIdx.x == 0) *info = bad;
}

// Block Gauss-Jordan step J on [P | B] (P kp x kp, B kp x nrhs, both column-major with
// leading dimension kp): every workgroup updates one block X_IC' of a row I != J, where C' is a
// matrix block column C > J or a right-hand-side block r (32 columns):
//   X_IC' -= (A_IJ S_J) X_JC'
// Row J and column J are read only, so the blocks of one step are independent.  The workgroup
// of block (J + 1, J + 1) inverts it into S_{J+1} after its update.
__global__ __launch_bounds__(256) void gj_step(double* __restrict__ P, int64_t kp, int J,
                                               int nbk, double* __restrict__ B, int64_t nrhs,
                                               int nrb, double* __restrict__ Sd,
                                               int32_t* __restrict__ info) {
    __shared__ double sS[kB * kL], sA[kB * kL], sX[kB * kL], sL[kB * kL];
    if (*info != 0) return;                          // an earlier pivot block was not SPD
    const int per_row = (nbk - 1 - J) + nrb;         // blocks C' of one row I
    const int ii = blockIdx.x / per_row, cc = blockIdx.x - ii * per_row;
    const int I = ii < J ? ii : ii + 1;              // every row but J
    const bool mat = cc < nbk - 1 - J;
    const int C = mat ? J + 1 + cc : cc - (nbk - 1 - J);   // matrix block column / RHS block
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t ro = (int64_t)I * kB, jo = (int64_t)J * kB;
    double* X = mat ? P : B;                         // the operand this block belongs to
    const int64_t co = (int64_t)C * kB;
    const int64_t ncol = mat ? kp : nrhs;            // columns of X
    load_block(Sd + (int64_t)J * kB * kB, kB, sS);
    load_block(P + ro + jo * kp, kp, sA);            // A_IJ
    for (int x = tid; x < kB * kB; x += 256) {       // X_JC' (row J)
        const int i = x % kB, c = x / kB;
        sX[i * kL + c] = co + c < ncol ? X[jo + i + (co + c) * kp] : 0.0;
    }
    f64x4 acc;                                       // X_IC' in the MFMA layout
    const int64_t mycol = co + blk_col(wave, lane);
    const bool colok = mycol < ncol;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = colok ? X[ro + blk_row(wave, lane, r) + mycol * kp] : 0.0;
    __syncthreads();
    f64x4 l = {0.0, 0.0, 0.0, 0.0};
    l = mma32([&](int i, int k) { return sA[i * kL + k]; },
              [&](int k, int j) { return sS[k * kL + j]; }, l, wave, lane);
#pragma unroll
    for (int r = 0; r < 4; ++r) sL[blk_row(wave, lane, r) * kL + blk_col(wave, lane)] = l[r];
    __syncthreads();
    acc = mma32([&](int i, int k) { return -sL[i * kL + k]; },
                [&](int k, int j) { return sX[k * kL + j]; }, acc, wave, lane);
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (colok) X[ro + blk_row(wave, lane, r) + mycol * kp] = acc[r];
    if (mat && I == J + 1 && C == J + 1) {
        // the next pivot block: fully updated now; invert it (after every wave's read of sA)
        __syncthreads();
#pragma unroll
        for (int r = 0; r < 4; ++r) sA[blk_row(wave, lane, r) * kL + blk_col(wave, lane)] = acc[r];
        __syncthreads();
        if (wave != 0) return;
        const int bad = wave_block_inverse(sA, Sd + (int64_t)C * kB * kB, sX);
        if (bad && tid == 0) *info = (int32_t)(co + bad);
    }
}

// Last launch of the Gauss-Jordan solve: B_I := S_I B_I for every block row I and right-hand
// side block (the rows are decoupled now); B := 0 when a pivot block was not SPD.
__global__ __launch_bounds__(256) void gj_scale(const double* __restrict__ Sd, int64_t kp,
                                                double* __restrict__ B, int64_t nrhs, int nrb,
                                                const int32_t* __restrict__ info) {
    __shared__ double sS[kB * kL], sX[kB * kL];
    const int I = blockIdx.x / nrb, rbk = blockIdx.x - (blockIdx.x / nrb) * nrb;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t ro = (int64_t)I * kB, co = (int64_t)rbk * kB;
    const bool failed = *info != 0;
    if (!failed) {
        load_block(Sd + (int64_t)I * kB * kB, kB, sS);
        for (int x = tid; x < kB * kB; x += 256) {
            const int i = x % kB, c = x / kB;
            sX[i * kL + c] = co + c < nrhs ? B[ro + i + (co + c) * kp] : 0.0;
        }
    }
    __syncthreads();
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    if (!failed)
        acc = mma32([&](int i, int k) { return sS[i * kL + k]; },
                    [&](int k, int j) { return sX[k * kL + j]; }, acc, wave, lane);
    const int64_t mycol = co + blk_col(wave, lane);
#pragma unroll
    for (int r = 0; r < 4; ++r)
        if (mycol < nrhs) B[ro + blk_row(wave, lane, r) + mycol * kp] = acc[r];
}

inline int grid_of(int64_t work, int block) {
    int64_t g = (work + block - 1) / block;
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, 65536));
}

}  // namespace

int64_t spd_padded(int64_t k) { return (k + kB - 1) / kB * kB; }

hipError_t launch_pad_matrix(const double* src, int64_t rows, int64_t cols, int64_t lds,
                             double* dst, int64_t kp, double diag, int64_t ncols, hipStream_t s) {
    if (kp <= 0 || ncols <= 0) return hipSuccess;
    if (rows > 0 && cols > 0 && !src) return hipErrorInvalidValue;
    hipLaunchKernelGGL(pad_matrix, grid_of(kp * ncols, 256), 256, 0, s, src, rows, cols, lds, dst,
                       kp, diag, ncols);
    return hipGetLastError();
}

hipError_t launch_spd_solve(double* P, int64_t kp, double* B, int64_t nrhs, double* Sd,
                            int32_t* info, hipStream_t s) {
    if (kp <= 0 || kp % kB || nrhs < 0) return hipErrorInvalidValue;
    const int nbk = (int)(kp / kB);
    const int64_t nrb = (nrhs + kB - 1) / kB;
    if (nrb * nbk > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(ldl_first, 1, 256, 0, s, P, kp, Sd, info);
    hipError_t e = hipGetLastError();
    for (int J = 0; J < nbk && e == hipSuccess; ++J) {
        const int64_t blocks = (int64_t)(nbk - 1) * ((nbk - 1 - J) + nrb);
        if (blocks == 0) continue;
        hipLaunchKernelGGL(gj_step, dim3((unsigned)blocks), 256, 0, s, P, kp, J, nbk, B, nrhs,
                           (int)nrb, Sd, info);
        e = hipGetLastError();
    }
    if (e != hipSuccess || nrb == 0) return e;
    hipLaunchKernelGGL(gj_scale, dim3((unsigned)(nbk * nrb)), 256, 0, s, Sd, kp, B, nrhs,
                       (int)nrb, info);
    return hipGetLastError();
}

hipError_t launch_slice_increments(const double* X, const double* Z, int64_t ldz, double* G,
                                   int64_t S, int64_t Et, hipStream_t s) {
    if (S <= 0) return hipSuccess;
    if (Et < 2 || Et > (1 << 20)) return hipErrorInvalidValue;
    // buffer records: one X row, and all of Z (their byte offsets are 32-bit)
    if (S * 8 >= 0x7fffffff || ldz * Et * 8 >= 0x7fffffff) return hipErrorInvalidValue;
    // 128-member tiles at every Et: 256-member tiles (slice_increments<4>, X read once at
    // Et = 256) measured 559 vs 528 us per EnKF256 analysis (profiles/r03i_*)
    constexpr int MW = 2;
    constexpr int kGM = 64 * MW;
    const int64_t nst = (S + kGN - 1) / kGN;
    const int nmt = (int)((Et + kGM - 1) / kGM);
    const int64_t grid = (nst + 7) / 8 * 8 * nmt;
    if (grid > 0x7fffffff || nst > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(slice_increments<MW>, dim3((unsigned)grid), 128 * MW,
                       2 * slice_stage<MW>() * sizeof(double), s, X, Z, ldz, G, S, (int)Et,
                       (int)nst, nmt);
    return hipGetLastError();
}

}  // namespace mcr
