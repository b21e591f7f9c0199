/* TEST INFRASTRUCTURE ONLY (oracle): batched, multi-threaded drivers of the oracle's per-item
 * functions, for bench.py's CPU baselines (configs[2] pipeline: ConvexHullHelper over every phase
 * polygon, the phase expansion of every window, the swing-foot splines).  Each item is the same
 * call as the single-item entry point (orc_hull2d_hrep, orc_dcm_phase_expand, orc_quintic_fit /
 * orc_quintic_eval), items are handed to `threads` POSIX threads from an atomic counter, so a
 * CPU baseline uses the host's cores without Python in the loop. */
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>

#include "blf_oracle.h"

typedef struct par_job {
    void (*fn)(const struct par_job*, int64_t);
    int64_t count;
    atomic_llong next;
    const void* a[10];
    void* o[6];
    int64_t iv[8];
    double dv[2];
} par_job;

static void* par_worker(void* arg)
{
    par_job* J = (par_job*)arg;
    for (;;) {
        const long long i = atomic_fetch_add(&J->next, 1);
        if (i >= J->count) break;
        J->fn(J, i);
    }
    return NULL;
}

static void par_run(par_job* J, int threads)
{
    atomic_store(&J->next, 0);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    int started = 0;
    for (int t = 1; t < threads; ++t)
        if (pthread_create(&th[started], NULL, par_worker, J) == 0) ++started;
    par_worker(J);
    for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
}

/* ---- hulls: pts [count][P][2], npts [count] -> A [count][M][2], b [count][M], nf [count] ---- */
static void hull_item(const par_job* J, int64_t i)
{
    const int P = (int)J->iv[0], M = (int)J->iv[1];
    const double* pts = (const double*)J->a[0] + i * 2 * P;
    const int32_t* npts = (const int32_t*)J->a[1];
    ((int32_t*)J->o[2])[i] = orc_hull2d_hrep(pts, npts[i], M, (double*)J->o[0] + i * 2 * M,
                                             (double*)J->o[1] + i * M);
}

void orc_hull2d_hrep_batch(int64_t count, int P, int M, const double* pts, const int32_t* npts,
                           double* A, double* b, int32_t* nf, int threads)
{
    par_job J = {0};
    J.fn = hull_item;
    J.count = count;
    J.a[0] = pts; J.a[1] = npts;
    J.o[0] = A; J.o[1] = b; J.o[2] = nf;
    J.iv[0] = P; J.iv[1] = M;
    par_run(&J, threads);
}

/* ---- phase expansion of B windows (per-problem tables as orc_dcm_phase_expand) ---- */
static void expand_item(const par_job* J, int64_t q)
{
    const int P = (int)J->iv[0], M = (int)J->iv[1], N = (int)J->iv[2];
    const int64_t start = J->iv[3];
    const double dt = J->dv[0];
    orc_dcm_phase_expand(P, M, ((const int32_t*)J->a[0])[q], (const double*)J->a[1] + q * P,
                         (const double*)J->a[2] + q * P, (const double*)J->a[3] + q * P * M * 2,
                         (const double*)J->a[4] + q * P * M, (const int32_t*)J->a[5] + q * P,
                         (const double*)J->a[6] + q * P * 2, start, dt, N,
                         (double*)J->o[0] + q * N * M * 2, (double*)J->o[1] + q * N * M,
                         (int32_t*)J->o[2] + q * N, (double*)J->o[3] + q * (N + 1) * 2,
                         (double*)J->o[4] + q * N * 2);
}

void orc_dcm_phase_expand_batch(int64_t B, int P, int M, const int32_t* nphases, const double* begin,
                                const double* end, const double* pA, const double* pb,
                                const int32_t* pnf, const double* pref, int64_t start, double dt,
                                int N, double* A, double* b, int32_t* nfacets, double* xi_ref,
                                double* vrp_ref, int threads)
{
    par_job J = {0};
    J.fn = expand_item;
    J.count = B;
    J.a[0] = nphases; J.a[1] = begin; J.a[2] = end; J.a[3] = pA; J.a[4] = pb; J.a[5] = pnf;
    J.a[6] = pref;
    J.o[0] = A; J.o[1] = b; J.o[2] = nfacets; J.o[3] = xi_ref; J.o[4] = vrp_ref;
    J.iv[0] = P; J.iv[1] = M; J.iv[2] = N; J.iv[3] = start;
    J.dv[0] = dt;
    par_run(&J, threads);
}

/* ---- swing splines: fit S quintic splines (K1 knots, dim) and evaluate Q queries each ---- */
static void spline_item(const par_job* J, int64_t s)
{
    const int K1 = (int)J->iv[0], D = (int)J->iv[1], Q = (int)J->iv[2];
    const double* kt = (const double*)J->a[0] + s * K1;
    const double* kp = (const double*)J->a[1] + s * K1 * 3 * D;
    const double* tq = (const double*)J->a[2] + s * Q;
    double* co = (double*)J->o[0] + s * (K1 - 1) * D * 6;
    orc_quintic_fit(kt, kp, K1, D, co);
    orc_quintic_eval(kt, co, K1, D, tq, Q, (double*)J->o[1] + s * Q * 3 * D, (int32_t*)J->o[2] + s * Q);
}

void orc_quintic_batch(int64_t S, int K1, int dim, int Q, const double* knots_t,
                       const double* knots_pva, const double* tq, double* coeffs, double* pva,
                       int32_t* idx, int threads)
{
    par_job J = {0};
    J.fn = spline_item;
    J.count = S;
    J.a[0] = knots_t; J.a[1] = knots_pva; J.a[2] = tq;
    J.o[0] = coeffs; J.o[1] = pva; J.o[2] = idx;
    J.iv[0] = K1; J.iv[1] = dim; J.iv[2] = Q;
    par_run(&J, threads);
}
