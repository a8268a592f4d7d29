/*
 * mcroute -- MI355X (gfx950) Muskingum routing engine, C ABI.
 *
 * Drop-in boundary for the hot path of future-water/tx-fast-hydrology.  The reference calls a
 * module-level numba kernel positionally (muskingum.py:10 import, muskingum.py:456-457 call):
 *
 *     i_t_next, o_t_next = _ax_bu(sub_startnodes, endnodes, alpha, beta, chi, gamma,
 *                                 i_t_prev, o_t_prev, p_t_next, indegree)   # nutils.py:64-89
 *
 * and drives it once per timestep from Muskingum.step_iter / simulate_iter
 * (muskingum.py:435-465, 499-536).  This library replaces that call: `mc_ax_bu_f64` is the
 * stateless mirror of `_ax_bu`; the `mc_net_*` session keeps topology, coefficients, state,
 * forcing and outputs resident in HBM and runs whole horizons (`mc_run`).
 *
 * Conventions
 *   - plain pointers and sizes; all arrays are C-contiguous, int64 indices, float64 values, in
 *     the CALLER's reach order (the order of `endnodes`), exactly like the reference arrays;
 *   - every function returns MC_OK (0) or a negative MC_E_* code; `mc_last_error()` returns a
 *     thread-local message for the last failure.  No C++ exception crosses the ABI;
 *   - the library never retains a caller pointer past the call;
 *   - a session handle is not thread-safe: use one thread per handle (or lock externally);
 *   - results are bit-identical to the reference's float64 arithmetic (same association, no
 *     FMA contraction, inflows summed in the reference's finalisation order), non-finite inputs
 *     included: a step beyond the forcing index copies the clamped row (nutils.py:24-27), a
 *     reach the reference walk never processes keeps o = 0 whatever its state and forcing hold
 *     (nutils.py:68-88), and an overflow inside a partial-sum fold gives the reference's Inf /
 *     NaN (tests/test_gpu_edges.py, single-member and ensemble sessions, every execution mode).  The
 *     kernels run a fast form while the state and forcing in use are finite (device flags set
 *     by every upload) and the exact form otherwise; a fast-form horizon whose partial sum
 *     overflowed is re-routed from its input state at the next synchronising call.
 */
#ifndef MCROUTE_H
#define MCROUTE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MC_OK 0
#define MC_E_INVALID (-1)   /* bad argument (null pointer, size, range) */
#define MC_E_TOPOLOGY (-2)  /* topology cannot be scheduled (see mc_last_error) */
#define MC_E_HIP (-3)       /* HIP runtime error (no device, launch failure, ...) */
#define MC_E_NOMEM (-4)     /* host or device allocation failed */
#define MC_E_STATE (-5)     /* call out of order (e.g. mc_run before mc_load_forcing) */

typedef struct mc_plan_params {
    int32_t slots;    /* lanes (threads) per workgroup (multiple of 64, <= 512); 0 = default */
    int32_t tile;     /* ticks per launch = slack of a cross-cluster edge; 0 = default.
                         Device sessions need a multiple of 16. */
    int32_t ext_cap;  /* max cross-cluster inputs per workgroup; 0 = default */
    int32_t chain;    /* node slots per lane, 1..4 (0 = default 2): a run of up to `chain`
                         consecutive reaches along a flow path shares one lane and one tick */
    int32_t sync;     /* 1: chunk-synchronous plan (plan.hpp: unit-slack edges inside one wave,
                         8-tick local edges between the waves of a workgroup), so the dataflow
                         kernel joins its waves once per 8 ticks; 0: classic plan */
} mc_plan_params;

typedef struct mc_plan_info {
    int64_t n;            /* reaches */
    int64_t n_routed;     /* reaches the reference walk processes (others keep o = 0) */
    int64_t n_clusters;
    int64_t n_cross;      /* cross-cluster edges */
    int64_t nslots;       /* node slots: nwg * chain * slots */
    int32_t nwg;          /* workgroups */
    int32_t slots;
    int32_t tile;
    int32_t gmax;         /* schedule length without the horizon: ticks = gmax + T */
    int32_t max_height;   /* longest upstream path (network depth - 1) */
    int32_t max_ext_wg;
    int64_t n_partial;    /* partial-sum nodes (reaches with more than 4 routed upstreams) */
    int64_t n_ext;        /* cross-cluster inputs over all workgroups */
    int64_t n_pairs;      /* chained edges (a node and its consumer in one lane and tick) */
    int32_t chain;        /* node slots per lane */
    int32_t n_local;      /* sync plans: 8-tick local edges between the waves of a workgroup */
} mc_plan_info;

/* Thread-local description of the last error (never NULL). */
const char* mc_last_error(void);
/* ABI version (major * 100 + minor). */
int mc_version(void);

/* ---- host-only topology compiler (no GPU needed) --------------------------------------- */
/* Replays the reference walk (nutils.py:72-88) and builds the space-time schedule.
 * headwaters = the reference's sub_startnodes = startnodes[indegree == 0] (muskingum.py:444). */
int mc_plan_create(int64_t n, const int64_t* endnodes, const int64_t* indegree,
                   const int64_t* headwaters, int64_t n_head, const mc_plan_params* params,
                   void** plan_out);
int mc_plan_get_info(const void* plan, mc_plan_info* info);
/* Any output pointer may be NULL.  rank/pos: [n]; G/slot_reach: [nslots]. */
int mc_plan_export(const void* plan, int64_t* rank, int64_t* pos, int32_t* G,
                   int64_t* slot_reach);
/* Schedule links (test / inspection): flags, up_cnt, up4 [nslots] (at most 4 input codes per
 * slot: workgroup-local slot, 0x8000 | external input, or 0x7fff = the lane's previous position
 * in the same tick (chained edge); flags 3 = partial-sum slot); ext_off [nwg+1]; ext_src, ext_g
 * [n_ext] (ext_src is the source's output row: its reach index, or n + slot for a partial-sum
 * slot).  Node slot d of workgroup w, lane l, position p = w * chain * slots + p * slots + l.
 * Any pointer may be NULL. */
int mc_plan_export_links(const void* plan, uint8_t* flags, uint8_t* up_cnt, uint64_t* up4,
                         int32_t* ext_off, int64_t* ext_src, int32_t* ext_g);
/* Local edges of a chunk-synchronous plan (mc_plan_params.sync): lx_off [nwg+1] (the local
 * inputs of workgroup w are its external columns ext_off[w+1]-ext_off[w] + 0 .. after its
 * cross-workgroup ones) and lx_src [n_local] (the producing node slot of each).  A local input
 * delivers at tick k the producer's output of tick k - 4.  Any pointer may be NULL. */
int mc_plan_export_local(const void* plan, int32_t* lx_off, int32_t* lx_src);
/* Launch schedule for a horizon of T steps: launch k covers ticks [k*tile, (k+1)*tile) and
 * runs workgroups list[off[k] .. off[k+1]).  Call with off/list NULL to get the sizes
 * (*n_launch, *n_list); then with arrays of at least n_launch+1 / n_list entries. */
int mc_plan_schedule(const void* plan, int64_t T, int64_t* n_launch, int64_t* n_list,
                     int64_t* off, int32_t* list);
int mc_plan_destroy(void* plan);

/* ---- stateless mirror of nutils._ax_bu (nutils.py:64-89) -------------------------------- */
/* One timestep.  Same arguments and meaning as the reference; outputs are caller-allocated
 * (the reference returns fresh arrays).  The compiled topology is cached between calls. */
int mc_ax_bu_f64(int64_t n, const int64_t* headwaters, int64_t n_head, const int64_t* endnodes,
                 const double* alpha, const double* beta, const double* chi, const double* gamma,
                 const double* i_t_prev, const double* o_t_prev, const double* q_t_next,
                 const int64_t* indegree, double* i_t_next_out, double* o_t_next_out);

/* ---- device-resident session ------------------------------------------------------------ */
/* Creates a session on the calling thread's current HIP device.  params may be NULL. */
int mc_net_create(int64_t n, const int64_t* endnodes, const int64_t* indegree,
                  const int64_t* headwaters, int64_t n_head, const mc_plan_params* params,
                  void** net_out);
int mc_net_destroy(void* net);
int mc_net_get_info(const void* net, mc_plan_info* info);
/* Use an external hipStream_t (e.g. torch's current stream); NULL = the session's own. */
int mc_net_set_stream(void* net, void* hip_stream);
/* Ensemble members (default 1).  With E > 1 every per-reach array passed to or returned by
 * mc_set_state, mc_get_state, mc_step (o/i/q) is [n][E] (member innermost), the forcing of
 * mc_load_forcing / mc_simulate is [n_rows][n][E], mc_fetch_outputs returns [t][n][E] and
 * mc_fetch_series [n][T][E].  Members share topology and coefficients (each member
 * is an independent deterministic run with its own forcing and initial state).  Setting the
 * member count zeroes the state and drops loaded forcing and outputs.  Ensemble horizons run the
 * multi-launch path; a one-step ensemble run (the assimilation cycle) is one member-dataflow
 * launch when it fits the device (mc_set_mode). */
int mc_net_set_members(void* net, int64_t members);
int mc_net_get_members(const void* net, int64_t* members);

/* _apply_gain (nutils.py:116-134, applied as da.py:124-126) on the session state:
 * o += 0 + gain for reaches the reference walk processes; i += one-hop sums of those gains in
 * the reference's finalisation order.  gain: [n] (or [n][E] for an ensemble session). */
int mc_apply_gain(void* net, const double* gain);

/* Ensemble Kalman analysis on the session's E >= 2 member states: the update of
 * da.py:110-126 (KalmanFilter.filter) with the forecast covariance replaced by the ensemble
 * sample covariance, P H^T = X'(HX')^T / (E-1), H P H^T = HX'(HX')^T / (E-1):
 *     o_e += K (y_e - o_e[gauges]),  K = P H^T (H P H^T + R)^-1,   i_e += one-hop(gain_e)
 * gauges [m]: reach indices (caller order; H selects their outflow); y [m][E]: observations per
 * member (identical columns = no perturbation); R [m][m] SPD.  Every dense step runs on the
 * library's f64 MFMA kernels: for diagonal R and E <= m the E x E ensemble-space system
 * (I + HA^T R^-1 HA / (E-1)), else the m x m one, solved by block Gauss-Jordan.  A system that is
 * not positive definite zeroes that analysis's increment (the members stay unchanged) and is
 * reported by the next synchronising call (MC_E_INVALID), also when later analyses succeeded.
 * mc_enkf_gain returns K as [n][m] (diagnostics / tests). */
int mc_enkf_analysis(void* net, int64_t m, const int64_t* gauges, const double* y,
                     const double* R);
int mc_enkf_gain(void* net, int64_t m, const int64_t* gauges, const double* R, double* K_out);

/* The analysis in stages, for an ensemble sharded over N ranks (one GPU each, E local members,
 * Et = N E in all).  Pointers named *_dev are DEVICE buffers owned by the caller, who runs the
 * collectives between the stages (torch.distributed / RCCL; tx_fast_hydrology_amd/ensemble.py):
 *   1. mc_ens_gauges: local gauge outflows HX_dev [E][m] and innovations D_dev [E][m] from
 *      y [m][E] (host);                      -> all-gather both into [Et][m]
 *   2. mc_ens_pack: local states as reach slices send_dev [N][E][S] (S = mc_ens_slice_size);
 *                                            -> all-to-all into Xs_dev [Et][S] (this rank's slice)
 *   3. mc_ens_slice_update: anomalies, C = HA HA^T/(Et-1) + R, W = C^-1 D, Z = HA^T W/(Et-1),
 *      increments of the slice Gs_dev = A Z [Et][S];    -> all-to-all back into [N][E][S]
 *   4. mc_ens_unpack_apply: local increments -> _apply_gain on the local members.
 * Stage 3 in two halves: mc_ens_weights forms Z from the gathered gauge data only (kept in the
 * session), mc_ens_increments the slice increments from Xs_dev and that Z, so the weights can be
 * computed while the member -> slice all-to-all is in flight.  mc_ens_slice_update = both.
 * With N = 1 the stages are exactly mc_enkf_analysis.  Stages run on the session's stream. */
int mc_ens_slice_size(const void* net, int64_t nranks, int64_t* S);
int mc_ens_gauges(void* net, int64_t m, const int64_t* gauges, const double* y, double* HX_dev,
                  double* D_dev);
int mc_ens_pack(void* net, int64_t nranks, double* send_dev);
int mc_ens_slice_update(void* net, int64_t nranks, int64_t m, const double* Xs_dev,
                        const double* HXall_dev, const double* Dall_dev, const double* R,
                        double* Gs_dev);
int mc_ens_weights(void* net, int64_t nranks, int64_t m, const double* HXall_dev,
                   const double* Dall_dev, const double* R);
int mc_ens_increments(void* net, int64_t nranks, const double* Xs_dev, double* Gs_dev);
int mc_ens_unpack_apply(void* net, int64_t nranks, const double* Grecv_dev);

/* The member-sharded analysis for callers without torch.distributed: a
 * communicator of nranks processes, one GPU each, over RCCL (xGMI), which the library loads at
 * first use (librccl.so.1; a process that already holds one -- e.g. PyTorch's -- shares it).
 *   mc_comm_unique_id: rank 0 makes the 128-byte id and hands it to the other ranks (any
 *                      channel: MPI, a file, a socket);
 *   mc_comm_init:      every rank, with the same id (collective: blocks until all ranks join);
 *   mc_ens_analysis_dist: one analysis of this rank's E members (y_local [m][E]; gauges and R
 *                      identical on every rank): the stages above with the all-gathers and
 *                      all-to-alls on the session's stream, the member -> slice all-to-all on a
 *                      side stream while the Et x Et weights are formed.  With one rank it is
 *                      bit-identical to mc_enkf_analysis (tested); the same stages with N ranks
 *                      are bit-identical to the one-session analysis when driven by
 *                      ensemble.emulated_analysis (8 shards, tested), but the multi-rank RCCL run
 *                      itself is UNVERIFIED until tests/test_gpu_dist.py's multi-GPU test runs
 *                      on a node with two or more GPUs (it is skipped on one).
 * MC_E_STATE when no RCCL library can be loaded. */
int mc_comm_unique_id(uint8_t* id128);
int mc_comm_init(int32_t nranks, int32_t rank, const uint8_t* id128, void** comm);
int mc_comm_destroy(void* comm);
int mc_ens_analysis_dist(void* net, void* comm, int64_t m, const int64_t* gauges,
                         const double* y_local, const double* R);

/* Coefficients alpha, beta, chi, gamma (muskingum.py:332-360), caller order. */
int mc_set_coeffs(void* net, const double* alpha, const double* beta, const double* chi,
                  const double* gamma);
/* State (o_t_next, i_t_next) of the model, caller order.  Like every upload of this ABI it
 * has read the caller's arrays when it returns (page-locked sources are waited for). */
int mc_set_state(void* net, const double* o_t_next, const double* i_t_next);
int mc_get_state(void* net, double* o_t_next, double* i_t_next);
/* Device-to-device state hand-over between two sessions of the SAME network (e.g. plans with
 * different lane / launch shapes for different run lengths): dst's (o, i) := src's, member by
 * member, reach by reach (bit copy).  Ordered after src's pending work on dst's stream; src's
 * later work waits for the copy.  Replaces mc_get_state + mc_set_state through the host. */
int mc_net_copy_state(void* dst_net, const void* src_net);

/* One timestep with lateral inflow q (muskingum.py:435-465 -> nutils.py:64-89).  If o_prev and
 * i_prev are non-NULL they replace the session state first.  Writes the new (i, o) and keeps
 * them as the session state. */
int mc_step(void* net, const double* o_prev, const double* i_prev, const double* q_t_next,
            double* i_t_next_out, double* o_t_next_out);

/* Forcing table for mc_run: n_rows timestamps xp (float64 ns, sorted) and values fp
 * [n_rows][n] (the simulate_iter DataFrame, muskingum.py:526-531). */
int mc_load_forcing(void* net, int64_t n_rows, const double* xp, const double* fp);
/* Same, with the forcing in series layout fp [n][n_rows] ([n][n_rows][E]): the block a pandas
 * frame of the sub-basin's inputs already holds (simulation.py uploads it without a transpose). */
int mc_load_forcing_series(void* net, int64_t n_rows, const double* xp, const double* fp);
/* Horizon of T steps from the session state, all on the device: step t interpolates the
 * forcing at x[t] = float(next_timestep.value) (muskingum.py:528-531) and routes the network.
 * Outputs stay resident (reach-major); the session state becomes the state after step T-1. */
int mc_run(void* net, int64_t T, const double* x);
/* Copy steps [t0, t1) of the last mc_run to the host, step-major: out_o[t - t0][j]. */
int mc_fetch_outputs(void* net, int64_t t0, int64_t t1, double* out_o, double* out_i);
/* Device-side form of mc_fetch_outputs: the outflows / inflows of steps [t0, t1) of the last
 * run in the reference's layout (reach order, step-major: what _ax_bu returns at every step,
 * nutils.py:64-89, and simulate_iter yields, muskingum.py:527-533) written into caller-owned
 * DEVICE buffers dev_o / dev_i ([t1 - t0][n](E) float64; either may be NULL), enqueued on the
 * session stream and returning at once (stream-ordered: a consumer on that stream, or after
 * mc_synchronize, sees them).  Nothing crosses PCIe. */
int mc_gather_outputs(void* net, int64_t t0, int64_t t1, double* dev_o, double* dev_i);
/* Asynchronous form of mc_fetch_outputs for the drop-in API's fused horizons (muskingum.py
 * simulate_iter, :499-536, yields every step's fresh arrays): queues the copy of steps [t0, t1)
 * into out_o / out_i (host, [t1 - t0][n]; pinned memory makes the copy asynchronous and full
 * speed) and, when digest_o / digest_i are non-NULL, the row digest of every copied step
 * (mc_host_digest of the same row) -- the caller detects an in-place edit of a yielded array by
 * recomputing it on the host.  Returns at once with *ticket; the buffers are complete after
 * mc_fetch_wait(ticket) (every ticket must be waited for once).  Any pointer but ticket may be
 * NULL. */
int mc_fetch_outputs_async(void* net, int64_t t0, int64_t t1, double* out_o, double* out_i,
                           uint64_t* digest_o, uint64_t* digest_i, int64_t* ticket);
int mc_fetch_wait(void* net, int64_t ticket);
/* Row digests of a host array [nrows][n]: out[r] = sum mod 2^64 over j of
 * t ^ (t >> 29), t = (bits(rows[r][j]) ^ (j * 0x9E3779B97F4A7C15)) * 0xD6E8FEB86659FD93.  Changing
 * any single element changes it.  Host code (no device needed), a few threads. */
int mc_host_digest(const double* rows, int64_t nrows, int64_t n, uint64_t* out);
/* The digests of two rows of n values each (a step's outflows and inflows): out2[0], out2[1]. */
int mc_host_digest2(const double* a, const double* b, int64_t n, uint64_t* out2);
/* Copy the full series of the last mc_run, reach-major: out_o[j][t] (either may be NULL). */
int mc_fetch_series(void* net, double* out_o, double* out_i);
/* Convenience: mc_load_forcing + mc_run + mc_fetch_outputs(0, T). */
int mc_simulate(void* net, int64_t T, const double* x, int64_t n_rows, const double* xp,
                const double* fp, double* out_o, double* out_i);

/* Blocks until the session's stream is idle. */
int mc_synchronize(void* net);

/* Per-launch HIP-event timing of the wavefront kernel (off by default).  kernel_ms is the sum
 * of the wavefront launches of all mc_run calls since the last reset, run_ms the sum of whole
 * mc_run device times. */
int mc_set_timing(void* net, int enable);
int mc_get_timing(void* net, double* kernel_ms, int64_t* launches, double* run_ms);
int mc_reset_timing(void* net);

/* Execution path of mc_run / mc_step.  mode 0 (default): one resident dataflow launch for the
 * whole horizon when the network fits the device at once, else launches of `tile` ticks;
 * 1: always launches of `tile` ticks; 2: dataflow only (MC_E_STATE when it does not fit; a
 * one-step ensemble run is a member-dataflow launch).
 * last_path: 1 launches, 2 dataflow (0 before any run). */
int mc_set_mode(void* net, int mode);
int mc_get_mode(void* net, int* mode, int* last_path);

/* How long a dataflow wait polls a stale upstream value before it gives up, in ticks of the
 * device's 100 MHz wall clock (0 = the default 2 s; < 0 = give up at once, for tests).  A run
 * whose wait gave up is detected at the next synchronising call: when it was the only
 * dataflow run since the previous one, the library routes the same horizon again from its
 * input state with launches (last_path then reads 1); otherwise that call fails (MC_E_HIP). */
int mc_set_flow_patience(void* net, int64_t wall_ticks);

/* Sub-basin coupling on the device (reference AsyncSimulation._accumulate, simulation.py:
 * 137-166): adds the inflow correction of the upstream session's outlet reach `src_reach`
 * (its outflow series of the last horizon, o_start = the outflow before that horizon) to the
 * lateral-inflow forcing of reach `dst_reach` of the downstream session, row r:
 *   F[r] += alpha * I(r + 1) / gamma + beta * I(r) / gamma   (I(0) = o_start),
 * alpha / beta / gamma being the downstream reach's coefficients.  The destination's forcing
 * must have one row per source step.  Ordered on the streams (after the source's run, before
 * the destination's next call), no host synchronisation.  Single-member sessions.
 * The correction reads the source's outputs as its stream produced them.  If that horizon's
 * dataflow waits gave up (mc_set_flow_patience), the source re-routes it at its next
 * synchronising call and mc_net_reroutes(src) grows, but corrections already taken from it are
 * not redone: a caller that chains sessions checks the sources' reroute counts after
 * synchronising and re-routes the dependent horizons (simulation.py falls back to its host
 * driver). */
int mc_net_lateral_correction(void* dst_net, int64_t dst_reach, const void* src_net,
                              int64_t src_reach, double o_start, double alpha, double beta,
                              double gamma);
/* Horizons this session re-routed with launches after a dataflow wait gave up. */
int mc_net_reroutes(const void* net, int64_t* count);

/* Diagnostic (bench.py roofline): device time per tick of the bare dataflow tick chain -- LDS
 * inputs of the previous tick, `chain` chained Muskingum updates per lane, LDS outputs, the
 * workgroup barrier -- for the (slots, chain) = (192, 2) / (384, 2) kernel shape (two / one
 * resident workgroups per CU) or the small-network shape (64, 1) (one per CU), on the current
 * device, no global memory traffic.  Schedule ticks x *ns_per_tick is the latency floor of a
 * horizon.  ticks: a multiple of 8. */
int mc_probe_tick_floor(int32_t slots, int32_t chain, int64_t ticks, double* ns_per_tick);

/* Launch trace of the last mc_run (off by default; diagnostic).  One record of 8 int64 per
 * workgroup per launch: {launch, workgroup, t_start, t_loop, t_end, hw_id, c_loop, c_end}.
 * t_* are ticks of the device's constant wall clock (clock_khz); t_loop is the end of the launch
 * prologue; hw_id is the XCC/SE/CU id of the workgroup's first wave; c_loop / c_end are its
 * shader-clock counter at the start / end of the tick loop.  n_records receives the record
 * count; at most `cap` records are copied to `out` (which may be NULL). */
int mc_set_trace(void* net, int enable);
int mc_get_trace(void* net, int64_t* out, int64_t cap, int64_t* n_records, int64_t* clock_khz);

/* ---- Full-covariance Kalman filter (da.py KalmanFilter / KalmanSmoother) ----
 * A covariance handle compiles the reach graph of one network once (walk replay of nutils._ax,
 * nutils.py:91-114).  Matrices P, Q, out, P_prior, P_post are row-major n x n float64 DEVICE
 * buffers owned by the caller (numpy layout, e.g. torch tensors); everything else is host
 * memory.  Calls are stream-ordered on the handle's stream; host outputs are complete when the
 * call returns.  Sweeps are bit-identical to the reference walk. */
int mc_cov_create(int64_t n, const int64_t* endnodes, const int64_t* indegree,
                  const int64_t* headwaters, int64_t n_head, void** cov);
int mc_cov_destroy(void* cov);
int mc_cov_set_stream(void* cov, void* hip_stream);
/* alpha, beta, chi [n] (gamma does not enter the state transition). */
int mc_cov_set_coeffs(void* cov, const double* alpha, const double* beta, const double* chi);
/* out = A P: _ap_par (nutils.py:157-170); P and out must be distinct. */
int mc_cov_ap(void* cov, const double* P, double* out);
/* out = A (A P)^T (+ Q when Q != NULL): _aqat_par (nutils.py:194-214) then da.py:117. */
int mc_cov_aqat(void* cov, const double* P, const double* Q, double* out);
/* _apply_gain (nutils.py:116-134), stateless: host gain [n] -> host i_gain, o_gain [n]. */
int mc_cov_apply_gain(void* cov, const double* gain, double* i_gain, double* o_gain);
/* da.py:118-122 on the prior: K = P_prior[:, s] (P_prior[s, s] + R)^-1 (LU, as np.linalg.inv),
 * gain = K dz, P_post = P_prior - K P_prior[s, :].  s [m] gauge reach indices (the sorted mask
 * order of da.py:31-44), R [m][m], dz [m] host; K_out [n][m] host (may be NULL), gain_out [n]
 * host.  P_post may equal P_prior (in-place posterior). */
int mc_kf_update(void* cov, int64_t m, const int64_t* s, const double* R, const double* dz,
                 const double* P_prior, double* P_post, double* K_out, double* gain_out);
/* One backward step of the RTS smoother (da.py:241-251): J = solve(P_p1, A P_f)^T,
 * P_s_out = P_f + J (P_s1 - P_p1), and for nvec host vectors x_s_out[v] = x_f[v] + J d[v]
 * (d = x_s(t+1) - x_p(t+1); [nvec][n] each).  P_s_out may equal P_f. */
int mc_ks_step(void* cov, const double* P_f, const double* P_p1, const double* P_s1,
               double* P_s_out, int64_t nvec, const double* x_f, const double* d,
               double* x_s_out);
int mc_cov_synchronize(void* cov);

#ifdef __cplusplus
}
#endif

#endif /* MCROUTE_H */
