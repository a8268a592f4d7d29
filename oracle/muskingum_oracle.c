/*
 * CPU restatement of the reference's Muskingum kernels -- TEST INFRASTRUCTURE ONLY.
 *
 * This file is the parity oracle and the `cpu_baseline` of bench.py ("kind": "port").  It is
 * never linked into, loaded by, or called from the product library (libmcroute.so); only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the checker.
 *
 * Every function is a plain serial transliteration of the reference numba kernel it names, with
 * the reference's evaluation order.  Build with -ffp-contract=off so gcc keeps the separate
 * multiply/add roundings (numba without fastmath does the same).
 *
 * Pinned against the golden vectors in tests/golden/ (generated from the reference by
 * tests/golden/make_golden.py) by tests/test_oracle.py.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#pragma STDC FP_CONTRACT OFF

/* nutils.py:64-89 `_ax_bu`.  `indeg_work` is caller scratch of n int64 (the reference copies
 * `indegree` each call, nutils.py:70).  Outputs are zeroed here (nutils.py:68-69). */
void oracle_ax_bu(int64_t n, const int64_t *startnodes, int64_t m, const int64_t *endnodes,
                  const double *alpha, const double *beta, const double *chi,
                  const double *gamma, const double *i_t_prev, const double *o_t_prev,
                  const double *q_t_next, const int64_t *indegree, double *i_t_next,
                  double *o_t_next, int64_t *indeg_work)
{
    memset(i_t_next, 0, (size_t)n * sizeof(double));
    memset(o_t_next, 0, (size_t)n * sizeof(double));
    memcpy(indeg_work, indegree, (size_t)n * sizeof(int64_t));
    for (int64_t k = 0; k < m; ++k) {
        int64_t s = startnodes[k];
        int64_t e = endnodes[s];
        while (indeg_work[s] == 0) {
            o_t_next[s] += (alpha[s] * i_t_next[s] + beta[s] * i_t_prev[s]
                            + chi[s] * o_t_prev[s] + gamma[s] * q_t_next[s]);
            if (s != e)
                i_t_next[e] += o_t_next[s];
            indeg_work[e] -= 1;
            s = e;
            e = endnodes[s];
        }
    }
}

/* nutils.py:91-114 `_ax` (homogeneous step, no lateral term). */
void oracle_ax(int64_t n, const int64_t *startnodes, int64_t m, const int64_t *endnodes,
               const double *alpha, const double *beta, const double *chi,
               const double *i_t_prev, const double *o_t_prev, const int64_t *indegree,
               double *i_t_next, double *o_t_next, int64_t *indeg_work)
{
    memset(i_t_next, 0, (size_t)n * sizeof(double));
    memset(o_t_next, 0, (size_t)n * sizeof(double));
    memcpy(indeg_work, indegree, (size_t)n * sizeof(int64_t));
    for (int64_t k = 0; k < m; ++k) {
        int64_t s = startnodes[k];
        int64_t e = endnodes[s];
        while (indeg_work[s] == 0) {
            o_t_next[s] += (alpha[s] * i_t_next[s] + beta[s] * i_t_prev[s]
                            + chi[s] * o_t_prev[s]);
            if (s != e)
                i_t_next[e] += o_t_next[s];
            indeg_work[e] -= 1;
            s = e;
            e = endnodes[s];
        }
    }
}

/* nutils.py:116-134 `_apply_gain`. */
void oracle_apply_gain(int64_t n, const int64_t *startnodes, int64_t m, const int64_t *endnodes,
                       const double *gain, const int64_t *indegree, double *i_t_next,
                       double *o_t_next, int64_t *indeg_work)
{
    memset(i_t_next, 0, (size_t)n * sizeof(double));
    memset(o_t_next, 0, (size_t)n * sizeof(double));
    memcpy(indeg_work, indegree, (size_t)n * sizeof(int64_t));
    for (int64_t k = 0; k < m; ++k) {
        int64_t s = startnodes[k];
        int64_t e = endnodes[s];
        while (indeg_work[s] == 0) {
            o_t_next[s] += gain[s];
            if (s != e)
                i_t_next[e] += o_t_next[s];
            indeg_work[e] -= 1;
            s = e;
            e = endnodes[s];
        }
    }
}

/* nutils.py:136-141 `numba_init_inflows` (self loops included, as in muskingum.py:417). */
void oracle_init_inflows(double *a, const int64_t *indices, const double *b, int64_t n)
{
    for (int64_t i = 0; i < n; ++i)
        a[indices[i]] += b[i];
}

/* numpy.searchsorted(xp, x, side='left') on a sorted float64 array. */
static int64_t searchsorted_left(const double *xp, int64_t n, double x)
{
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        int64_t mid = lo + ((hi - lo) >> 1);
        if (xp[mid] < x)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

/* nutils.py:5-39 `interpolate_sample`: fp is [n_xp][m] row-major; out has m entries. */
void oracle_interpolate_sample(double x, const double *xp, int64_t n_xp, const double *fp,
                               int64_t m, int method, double *out)
{
    int64_t ix = searchsorted_left(xp, n_xp, x);
    if (ix == 0) {
        memcpy(out, fp, (size_t)m * sizeof(double));
    } else if (ix >= n_xp) {
        memcpy(out, fp + (n_xp - 1) * m, (size_t)m * sizeof(double));
    } else {
        double dx0 = x - xp[ix - 1];
        double dx1 = xp[ix] - x;
        const double *lo = fp + (ix - 1) * m, *hi = fp + ix * m;
        if (method == 1) {
            double frac = dx0 / (dx0 + dx1);
            double w0 = 1 - frac;
            for (int64_t j = 0; j < m; ++j)
                out[j] = w0 * lo[j] + frac * hi[j];
        } else {
            const double *src = (dx0 < 0 ? -dx0 : dx0) <= (dx1 < 0 ? -dx1 : dx1) ? lo : hi;
            memcpy(out, src, (size_t)m * sizeof(double));
        }
    }
}

/*
 * Deterministic horizon: muskingum.py:499-536 `simulate_iter` loop (interpolate_sample, then
 * step_iter -> _ax_bu) for T steps.  x[T] are the step times float(next_timestep.value).
 * o_state/i_state hold the initial (o_t_next, i_t_next) and are overwritten with the final
 * state.  out_o/out_i ([T][n]) may be NULL.  Returns 0, or -1 on allocation failure.
 */
int oracle_simulate(int64_t n, const int64_t *startnodes, int64_t m, const int64_t *endnodes,
                    const int64_t *indegree, const double *alpha, const double *beta,
                    const double *chi, const double *gamma, double *o_state, double *i_state,
                    int64_t T, const double *x, const double *xp, int64_t n_xp,
                    const double *fp, double *out_o, double *out_i)
{
    double *q = (double *)malloc((size_t)n * sizeof(double));
    double *o_new = (double *)malloc((size_t)n * sizeof(double));
    double *i_new = (double *)malloc((size_t)n * sizeof(double));
    int64_t *work = (int64_t *)malloc((size_t)n * sizeof(int64_t));
    if (!q || !o_new || !i_new || !work) {
        free(q); free(o_new); free(i_new); free(work);
        return -1;
    }
    for (int64_t t = 0; t < T; ++t) {
        oracle_interpolate_sample(x[t], xp, n_xp, fp, n, 1, q);
        oracle_ax_bu(n, startnodes, m, endnodes, alpha, beta, chi, gamma, i_state, o_state, q,
                     indegree, i_new, o_new, work);
        memcpy(o_state, o_new, (size_t)n * sizeof(double));
        memcpy(i_state, i_new, (size_t)n * sizeof(double));
        if (out_o)
            memcpy(out_o + t * n, o_new, (size_t)n * sizeof(double));
        if (out_i)
            memcpy(out_i + t * n, i_new, (size_t)n * sizeof(double));
    }
    free(q); free(o_new); free(i_new); free(work);
    return 0;
}

/*
 * Ensemble baseline: E independent member runs (the reference's equivalent is E
 * `Muskingum.copy()` runs, muskingum.py:604-605).  State and forcing are member-minor:
 * o_state[n][E], fp[n_xp][n][E].  Members are spread over `threads` OpenMP threads.
 */
int oracle_simulate_members(int64_t n, int64_t E, const int64_t *startnodes, int64_t m,
                            const int64_t *endnodes, const int64_t *indegree,
                            const double *alpha, const double *beta, const double *chi,
                            const double *gamma, double *o_state, double *i_state, int64_t T,
                            const double *x, const double *xp, int64_t n_xp, const double *fp,
                            int threads)
{
    int status = 0;
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1) reduction(| : status)
    for (int64_t e = 0; e < E; ++e) {
        double *o = (double *)malloc((size_t)n * sizeof(double));
        double *i = (double *)malloc((size_t)n * sizeof(double));
        double *f = (double *)malloc((size_t)(n_xp * n) * sizeof(double));
        if (!o || !i || !f) {
            status |= 1;
        } else {
            for (int64_t j = 0; j < n; ++j) {
                o[j] = o_state[j * E + e];
                i[j] = i_state[j * E + e];
            }
            for (int64_t r = 0; r < n_xp; ++r)
                for (int64_t j = 0; j < n; ++j)
                    f[r * n + j] = fp[(r * n + j) * E + e];
            if (oracle_simulate(n, startnodes, m, endnodes, indegree, alpha, beta, chi, gamma,
                                o, i, T, x, xp, n_xp, f, NULL, NULL) != 0)
                status |= 1;
            for (int64_t j = 0; j < n; ++j) {
                o_state[j * E + e] = o[j];
                i_state[j * E + e] = i[j];
            }
        }
        free(o); free(i); free(f);
    }
    return status ? -1 : 0;
}
