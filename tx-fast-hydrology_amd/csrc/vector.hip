// Member-vector wavefront sweep for ensembles (gfx950): the lanes of a wave are MEMBERS.
//
// The deterministic kernels map one node slot to one lane and run ensembles as E copies of that
// schedule (grid y).  Every member then repeats the per-slot work that does not depend on the
// member: coefficient and topology registers, step-table and forcing-row bookkeeping, activity
// selects, and a row of outputs for every tick of the workgroup window, active or not.  Here a
// wave holds Ew = 64 / H members of H node slots at once (H = 1: one node, 64 members), so
//   * a node's coefficients, input codes, activity and step-table entry are wave-uniform
//     (scalar loads and branches when H = 1) and are paid once for 64 members;
//   * every load and store is a contiguous member vector (512 B for H = 1): the forcing rows,
//     the cross-cluster inputs and the outputs, which are written only for active ticks.
// Layouts are node-major with members innermost: forcing FM[d][r][e], state SM[d][e], outputs
// OM[d][t][e] (capi.cpp converts the session's member-major arrays in and out).  The H node
// slots of a wave instruction are consecutive, so the forcing and output vectors of one
// instruction lie in one buffer whose base is wave-uniform (built once per launch) and the
// per-tick addressing is a 32-bit lane offset; idle nodes store to an out-of-range offset, which
// the hardware drops.
//
// Schedule: the multi-launch plan of kernels.hip (plan.hpp), node slot d does model step t at
// tick G[d] + t.  A launch covers `tile` ticks; in-cluster values move through an LDS double
// buffer of tick planes (one member vector per node slot and per external input); values from
// other clusters were written to OM by earlier launches (slack >= tile); they and the forcing rows
// are loaded kVecPrefetch ticks ahead (register rings) and the external values are staged in
// the external columns of the plane one tick before they are read.
//
// Arithmetic is the reference's (FMA contraction off):
//   I = ((0 + o[u1]) + o[u2]) + ...       o = 0 + (((alpha I + beta I_prev) + chi o_prev) + gamma q)
//   q = (1 - frac) f[lo] + frac f[hi]     (nutils.py:23-33, 64-89)
#include "device_common.hpp"
#include "kernels.hpp"
#include "plan.hpp"

#pragma clang fp contract(off)

// Diagnostic builds only (scripts/exp_vec.sh; results are wrong by construction): each
// MCR_VEXP_* switch removes one part of the tick to measure its cost.
#ifndef MCR_VEXP_NO_STORES
#define MCR_VEXP_NO_STORES 0
#endif
#ifndef MCR_VEXP_NO_LOADS
#define MCR_VEXP_NO_LOADS 0
#endif
#ifndef MCR_VEXP_NO_BARRIER
#define MCR_VEXP_NO_BARRIER 0
#endif

namespace mcr {

namespace {

constexpr int kVecLanes = 64;     // plan lanes (node slots at chain 1) per workgroup
constexpr int kNT = 2;            // buffer-instruction cache policy: non-temporal
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// Forcing-row reuse.  With hourly forcing and 5-minute steps a node's two forcing rows change
// once every 12 steps, so the lateral-inflow loads of step t are issued only for rows that step
// t - 1 did not use; the other loads of the ring slot get an out-of-range offset (dropped by the
// hardware, no memory traffic) and the value is taken from the previous step's registers.
enum : int { kFromLoad = 0, kFromPrevLo = 1, kFromPrevHi = 2 };

// 4 nodes per instruction: two workgroups per CU, W / 2 waves per SIMD (the tick is latency
// bound; the second workgroup fills the first one's waits).  Wider member vectors need more
// registers per node and keep one.
template <int K, int W, int H>
__global__ __launch_bounds__(W * 64)
__attribute__((amdgpu_waves_per_eu(H == 4 && K == 1 ? W / 2 : 1, H == 4 && K == 1 ? W / 2 : 8)))
void wavefront_vec(VecArgs a) {
    constexpr int SL = kVecLanes;
    constexpr int RS = K * SL;                  // node slots of the plan workgroup
    constexpr int Ew = 64 / H;                  // members per node in a wave
    constexpr int L = SL / (W * H);             // lane groups of a wave
    static_assert(L * W * H == SL, "lanes must split evenly over the waves");
    constexpr int XW = (kVecMaxExt + W * H - 1) / (W * H);   // external inputs per lane
    constexpr int COLS = RS + 1 + kVecMaxExt;   // plane columns: slots, zero, external inputs
    constexpr int D = kVecPrefetch;             // ticks between a load's issue and its use
    constexpr unsigned kOOB = 0x80000000u;      // buffer offset past every buffer: dropped
    extern __shared__ __attribute__((aligned(16))) double plane[];   // [2][COLS][Ew]
    VecMeta* lrec = reinterpret_cast<VecMeta*>(plane + 2 * COLS * Ew);   // [RS]
    int4* ltab = reinterpret_cast<int4*>(lrec + RS);                     // step-table window

    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int h = lane / Ew, e = lane - h * Ew;
    const int w = a.active[blockIdx.x];
    const int64_t E = a.E;
    const int mb = (int)blockIdx.y * Ew;        // first member of this block
    const int T = a.T;
    const int nrow = a.n_rows;
    const int gminw = a.wg_gmin[w], gmaxw = a.wg_gmax[w];
    // ticks of this launch that fall inside the workgroup's window (block-uniform)
    const int kst = max(a.kappa0, gminw);
    const int ken = min(a.kappa0 + a.tile, gmaxw + T);
    if (kst >= ken) return;
    // the workgroup's node records and the step-table window it can touch -> LDS
    const int t_lo = max(0, kst - 1 - gmaxw);
    const int t_hi = min(T, ken + D - gminw);
    for (int i = tid; i < RS; i += W * 64) lrec[i] = a.meta[(int64_t)w * RS + i];
    for (int i = tid; i < t_hi - t_lo; i += W * 64) ltab[i] = a.stab[t_lo + i];
    __syncthreads();
    // step-table entry of step t (clamped into [0, T) and into the staged window)
    auto tab = [&](int t) -> int4 {
        int i = (t < 0 ? 0 : (t >= T ? T - 1 : t)) - t_lo;
        i = i < 0 ? 0 : (i >= t_hi - t_lo ? t_hi - t_lo - 1 : i);
        return ltab[i];
    };
    // lane offsets (bytes) inside a node group's forcing / output buffer
    const unsigned fh = (unsigned)((h * nrow) * E + e) * 8u;    // + row * E * 8
    const unsigned oh = (unsigned)((h * T) * E + e) * 8u;       // + t * E * 8
    const unsigned rowb = (unsigned)E * 8u;                     // one row / step of a node

    // ---- per node group: buffers of its forcing rows and outputs; the lane's node record
    // (static for the launch: registers) and state
    double op[L][K], ip[L][K];
    int cs[L][K], G[L][K], in[L][K][4];
    bool chn[L][K];
    __amdgpu_buffer_rsrc_t fbuf[L][K], obuf[L][K];
#pragma unroll
    for (int g = 0; g < L; ++g)
#pragma unroll
        for (int p = 0; p < K; ++p) {
            const int c0 = p * SL + (wave * L + g) * H;         // first slot of the group
            const int c = c0 + h;
            cs[g][p] = c;
            const VecMeta m = lrec[c];
            G[g][p] = m.G;
            chn[g][p] = m.chained != 0;
#pragma unroll
            for (int u = 0; u < 4; ++u) in[g][p][u] = m.in[u] * Ew + e;
            const int64_t d0 = (int64_t)w * RS + c0;
            fbuf[g][p] = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<double*>(a.FM) + d0 * nrow * E + mb, (short)0, H * nrow * (int)E * 8,
                0x00020000);
            obuf[g][p] = __builtin_amdgcn_make_buffer_rsrc(
                a.OM + d0 * T * E + mb, (short)0, H * T * (int)E * 8, 0x00020000);
            const int64_t sidx = (d0 + h) * E + mb + e;
            op[g][p] = a.SM_o[sidx];
            ip[g][p] = a.SM_i[sidx];
            // the consumer one tick behind reads the output of tick kst - 1 at the first tick
            plane[(((kst - 1) & 1) * COLS + c) * Ew + e] = op[g][p];
        }
    if (tid < Ew) {
        plane[(0 * COLS + RS) * Ew + tid] = 0.0;
        plane[(1 * COLS + RS) * Ew + tid] = 0.0;
    }

    // ---- external inputs: x = (i * W + wave) * H + h, consumed at tick k from plane (k-1)&1
    const int x0 = a.ext_off[w];
    const int nx = a.ext_off[w + 1] - x0;
    const double* xptr[XW];
    int xg[XW];
#pragma unroll
    for (int i = 0; i < XW; ++i) {
        const int x = (i * W + wave) * H + h;
        const bool ok = x < nx;
        const int64_t src = ok ? a.ext_slot[x0 + x] : 0;
        xptr[i] = a.OM + src * T * E + mb + e;
        xg[i] = ok ? a.ext_g[x0 + x] : 0;
    }
    auto ext_load = [&](int i, int k) -> double {
        // value external input i delivers at tick k: its producer's output at the consumer's
        // step k - G (clamped: ticks where the consumer is idle read any valid cell)
        int t = k - xg[i];
        t = t < 0 ? 0 : (t >= T ? T - 1 : t);
        return xptr[i][(int64_t)t * E];
    };
    // lateral inflow of the node's step at tick k: rows, interpolation weight and where each
    // row's value comes from (a load, or the previous step's registers; first = the first
    // step of the launch, every row loaded).  A clamped step t - 1 = t has the same rows.
    struct QSrc {
        int rl, rh, sl, sh;
        double fr;
    };
    auto q_src = [&](int g, int p, int k, bool first) -> QSrc {
        const int t = k - G[g][p];
        const int4 en = tab(t);
        const int4 pv = tab(t - 1);
        QSrc q;
        q.rl = dev::clamp_row(en.x, nrow);
        q.rh = dev::clamp_row(en.y, nrow);
        const int pl = dev::clamp_row(pv.x, nrow), ph = dev::clamp_row(pv.y, nrow);
        q.sl = first ? kFromLoad : (q.rl == pl ? kFromPrevLo : (q.rl == ph ? kFromPrevHi : kFromLoad));
        q.sh = first ? kFromLoad : (q.rh == ph ? kFromPrevHi : (q.rh == pl ? kFromPrevLo : kFromLoad));
        q.fr = __hiloint2double(en.w, en.z);
        return q;
    };
    // issue the row loads the step needs (the others: an out-of-range offset, no traffic)
    auto q_issue = [&](int g, int p, int k, bool first, double& lo, double& hi) {
        const QSrc q = q_src(g, p, k, first);
        lo = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                 fbuf[g][p], q.sl == kFromLoad ? fh + (unsigned)q.rl * rowb : kOOB, 0, 0));
        hi = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(
                 fbuf[g][p], q.sh == kFromLoad ? fh + (unsigned)q.rh * rowb : kOOB, 0, 0));
    };
    // prefetch rings, D deep: slot j serves the ticks k with (k - kst) % D == j
    double xv[D][XW];
    double qlo[D][L][K], qhi[D][L][K];
    double plo[L][K], phi[L][K];               // forcing rows of the node's previous tick
#pragma unroll
    for (int i = 0; i < XW; ++i) {
        const double v = ext_load(i, kst);
        const int x = (i * W + wave) * H + h;
        if (x < nx) plane[(((kst - 1) & 1) * COLS + RS + 1 + x) * Ew + e] = v;
    }
#pragma unroll
    for (int j = 0; j < D; ++j) {
#pragma unroll
        for (int i = 0; i < XW; ++i) xv[j][i] = ext_load(i, kst + 1 + j);
#pragma unroll
        for (int g = 0; g < L; ++g)
#pragma unroll
            for (int p = 0; p < K; ++p)
                q_issue(g, p, kst + j, j == 0, qlo[j][g][p], qhi[j][g][p]);
    }
#pragma unroll
    for (int g = 0; g < L; ++g)
#pragma unroll
        for (int p = 0; p < K; ++p) plo[g][p] = phi[g][p] = 0.0;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();

    for (int k0 = kst; k0 < ken; k0 += D) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
            // ticks past ken (the last group's remainder) change nothing: no state update,
            // no output; their plane writes are never read
            const int k = k0 + j;
            const bool live = k < ken;
            const int rd = ((k - 1) & 1) * COLS * Ew;   // plane of tick k - 1 (read)
            const int wr = (k & 1) * COLS * Ew;         // plane of tick k (written)
            // external values for tick k + 1 -> this tick's plane
#pragma unroll
            for (int i = 0; i < XW; ++i) {
                const int x = (i * W + wave) * H + h;
                if (x < nx) plane[wr + (RS + 1 + x) * Ew + e] = xv[j][i];
            }
            double qv[L][K];
#pragma unroll
            for (int g = 0; g < L; ++g)
#pragma unroll
                for (int p = 0; p < K; ++p) {
                    const QSrc q = q_src(g, p, k, k == kst);
                    const double lo = q.sl == kFromLoad ? qlo[j][g][p]
                                    : (q.sl == kFromPrevLo ? plo[g][p] : phi[g][p]);
                    const double hi = q.sh == kFromLoad ? qhi[j][g][p]
                                    : (q.sh == kFromPrevLo ? plo[g][p] : phi[g][p]);
                    plo[g][p] = lo;
                    phi[g][p] = hi;
                    qv[g][p] = (1.0 - q.fr) * lo + q.fr * hi;
                }
            // refill the ring slot D ticks ahead.  Unconditional loads and stores only (an
            // idle one gets an out-of-range offset): with every memory instruction on the
            // straight-line path the wait counts stay exact across ticks (a store in a branch
            // makes the next use of a load wait for ALL stores, vmcnt(0)); the scheduling
            // barrier keeps the loads at the top of the tick
            if (!MCR_VEXP_NO_LOADS) {
#pragma unroll
                for (int g = 0; g < L; ++g)
#pragma unroll
                    for (int p = 0; p < K; ++p)
                        q_issue(g, p, k + D, false, qlo[j][g][p], qhi[j][g][p]);
#pragma unroll
                for (int i = 0; i < XW; ++i) xv[j][i] = ext_load(i, k + 1 + D);
            }
            __builtin_amdgcn_sched_barrier(0);
            // every node of the lane, branch-free; inputs of tick k - 1 in the reference's fold
            // order, unused codes read the zero column, the chained input (the previous
            // position's output of this tick) is added last
            double ov[L][K];
            unsigned oo[L][K];
#pragma unroll
            for (int g = 0; g < L; ++g) {
                double prev = 0.0;
#pragma unroll
                for (int p = 0; p < K; ++p) {
                    const int t = k - G[g][p];
                    const bool act = live && (unsigned)t < (unsigned)T;
                    const VecMeta& m = lrec[cs[g][p]];   // coefficients: LDS, read each tick
                    double I = plane[rd + in[g][p][0]];
                    I = I + plane[rd + in[g][p][1]];
                    I = I + plane[rd + in[g][p][2]];
                    I = I + plane[rd + in[g][p][3]];
                    if (p > 0) I = chn[g][p] ? I + prev : I;
                    const double o = 0.0 + (((m.al * I + m.be * ip[g][p]) + m.ch * op[g][p]) +
                                            m.ga * qv[g][p]);
                    op[g][p] = act ? o : op[g][p];
                    ip[g][p] = act ? I : ip[g][p];
                    prev = o;
                    ov[g][p] = o;
                    oo[g][p] = act ? oh + (unsigned)t * rowb : kOOB;
                }
            }
#pragma unroll
            for (int g = 0; g < L; ++g)
#pragma unroll
                for (int p = 0; p < K; ++p) plane[wr + cs[g][p] * Ew + e] = ov[g][p];
            // outputs of the active nodes, one member vector each
            if (!MCR_VEXP_NO_STORES) {
#pragma unroll
                for (int g = 0; g < L; ++g)
#pragma unroll
                    for (int p = 0; p < K; ++p)
                        __builtin_amdgcn_raw_buffer_store_b64(
                            __builtin_bit_cast(u32x2, ov[g][p]), obuf[g][p], oo[g][p], 0, kNT);
            }
            if (!MCR_VEXP_NO_BARRIER) __syncthreads();
        }
    }
    // state for the next launch / after the horizon
#pragma unroll
    for (int g = 0; g < L; ++g)
#pragma unroll
        for (int p = 0; p < K; ++p) {
            const int64_t sidx = ((int64_t)w * RS + cs[g][p]) * E + mb + e;
            a.SM_o[sidx] = op[g][p];
            a.SM_i[sidx] = ip[g][p];
        }
}

// dst[c * dst_ld + r] = src[r * src_ld + c] for r < rows, c < cols through 32 x 32 LDS tiles
// (coalesced both ways); a 1-D grid of tiles (either dimension may exceed 65535 tiles)
__global__ void transpose_f64(const double* __restrict__ src, int64_t src_ld,
                              double* __restrict__ dst, int64_t dst_ld, int64_t rows,
                              int64_t cols, int64_t tiles_c, int64_t tiles) {
    __shared__ double tile[32][33];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 256 threads: 8 rows per pass
    for (int64_t q = blockIdx.x; q < tiles; q += gridDim.x) {
        const int64_t r0 = (q / tiles_c) * 32, c0 = (q % tiles_c) * 32;
        __syncthreads();
        for (int i = ty; i < 32; i += 8) {
            const int64_t r = r0 + i, c = c0 + tx;
            if (r < rows && c < cols) tile[i][tx] = src[r * src_ld + c];
        }
        __syncthreads();
        for (int i = ty; i < 32; i += 8) {
            const int64_t c = c0 + i, r = r0 + tx;
            if (r < rows && c < cols) dst[c * dst_ld + r] = tile[tx][i];
        }
    }
}

// coefficients of each node slot into its metadata record (after every coefficient upload)
__global__ void vec_meta_coeffs(const double* __restrict__ alpha, const double* __restrict__ beta,
                                const double* __restrict__ chi, const double* __restrict__ gamma,
                                VecMeta* __restrict__ meta, int64_t ns) {
    for (int64_t d = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; d < ns;
         d += (int64_t)gridDim.x * blockDim.x) {
        meta[d].al = alpha[d];
        meta[d].be = beta[d];
        meta[d].ch = chi[d];
        meta[d].ga = gamma[d];
    }
}

template <int K, int W, int H>
const void* vec_fn_t() {
    return reinterpret_cast<const void*>(&wavefront_vec<K, W, H>);
}

const void* vec_fn(int chain, int waves, int H) {
#define MCR_CASE(K_, W_, H_) \
    if (chain == K_ && waves == W_ && H == H_) return vec_fn_t<K_, W_, H_>();
    MCR_VEC_SHAPES(MCR_CASE)
#undef MCR_CASE
    return nullptr;
}

inline int grid_1d(int64_t work, int block) {
    int64_t g = (work + block - 1) / block;
    return (int)std::min<int64_t>(std::max<int64_t>(g, 1), 65536);
}

}  // namespace

bool vec_shape_ok(int slots, int chain, int waves, int H) {
    return slots == kVecLanes && vec_fn(chain, waves, H) != nullptr;
}

size_t vec_lds_bytes(int chain, int H, int tile) {
    const size_t rs = (size_t)chain * kVecLanes;
    const size_t cols = rs + 1 + kVecMaxExt;
    size_t b = 2 * cols * (size_t)(64 / H) * sizeof(double);
    // node records + the step-table window (tile + span + prefetch + 1 ticks)
    b += rs * sizeof(VecMeta) + ((size_t)tile + 257 + kVecPrefetch) * sizeof(int4);
    return b;
}

hipError_t launch_vec(const VecArgs& a, int grid, int member_blocks, int chain, int waves, int H,
                      hipStream_t s) {
    const void* fn = vec_fn(chain, waves, H);
    if (!fn) return hipErrorInvalidValue;
    void* args[] = {const_cast<VecArgs*>(&a)};
    return hipLaunchKernel(fn, dim3(grid, member_blocks), dim3(waves * 64), args,
                           vec_lds_bytes(chain, H, a.tile), s);
}

hipError_t vec_occupancy(int chain, int waves, int H, int tile, int* blocks_per_cu) {
    const void* fn = vec_fn(chain, waves, H);
    if (!fn) return hipErrorInvalidValue;
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, fn, waves * 64,
                                                        vec_lds_bytes(chain, H, tile));
}

hipError_t launch_transpose_ld(const double* src, int64_t src_ld, double* dst, int64_t dst_ld,
                               int64_t rows, int64_t cols, hipStream_t s) {
    if (rows * cols == 0) return hipSuccess;
    const int64_t tc = (cols + 31) / 32, tiles = tc * ((rows + 31) / 32);
    hipLaunchKernelGGL(transpose_f64, (unsigned)std::min<int64_t>(tiles, 1 << 20), 256, 0, s, src,
                       src_ld, dst, dst_ld, rows, cols, tc, tiles);
    return hipGetLastError();
}

hipError_t launch_transpose(const double* src, double* dst, int64_t rows, int64_t cols,
                            int64_t batch, hipStream_t s) {
    for (int64_t b = 0; b < batch; ++b) {
        const hipError_t e = launch_transpose_ld(src + b * rows * cols, cols,
                                                 dst + b * rows * cols, rows, rows, cols, s);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_vec_meta_coeffs(const double* alpha, const double* beta, const double* chi,
                                  const double* gamma, VecMeta* meta, int64_t ns, hipStream_t s) {
    if (ns == 0) return hipSuccess;
    hipLaunchKernelGGL(vec_meta_coeffs, grid_1d(ns, 256), 256, 0, s, alpha, beta, chi, gamma,
                       meta, ns);
    return hipGetLastError();
}

}  // namespace mcr
