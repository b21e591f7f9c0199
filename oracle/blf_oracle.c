/*
 * blf_oracle.c — TEST INFRASTRUCTURE ONLY (see blf_oracle.h).  CPU restatement of the reference
 * semantics, fp64, compiled with -ffp-contract=off so that every expression is evaluated exactly
 * in the order written (the device kernels follow the same order).
 */
#include "blf_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* ForwardEuler<LinearTimeInvariantSystem>::integrate — FixedStepIntegrator.tpp:21-72          */
/* ------------------------------------------------------------------------------------------ */
static void lti_step(int n, int m, const double* A, const double* B, const double* u, double* x,
                     double dT)
{
    /* LinearTimeInvariantSystem.cpp:71  dx = A x + B u ;  ForwardEuler.tpp:36-38  x += dx*dT */
    double dx[8];
    for (int r = 0; r < n; ++r) {
        double ax = A[r * n + 0] * x[0];
        for (int c = 1; c < n; ++c) ax = ax + A[r * n + c] * x[c];
        double bu = B[r * m + 0] * u[0];
        for (int c = 1; c < m; ++c) bu = bu + B[r * m + c] * u[c];
        dx[r] = ax + bu;
    }
    for (int r = 0; r < n; ++r) x[r] = x[r] + dx[r] * dT;
}

int orc_lti_euler_integrate(int n, int m, const double* A, const double* B, const double* u,
                            double* x, double t0, double t1, double dT, int64_t* nsteps_out)
{
    if (n < 1 || n > 8 || m < 1 || m > 8) return 1;
    if (t0 > t1 || !(dT > 0)) return 4;           /* FixedStepIntegrator.tpp:28-46            */
    if (t0 == t1) return 5;                       /* reference: size_t(i) < -1 -> never ends   */
    double q = ceil((t1 - t0) / dT);
    if (!(q < 2.0e9)) return 3;
    int iterations = (int)q;                      /* FixedStepIntegrator.tpp:48               */
    double currentTime = t0;
    int64_t steps = 0;
    for (int64_t i = 0; i < (int64_t)iterations - 1; ++i) {   /* :51-61                      */
        currentTime = t0 + dT * (double)i;
        lti_step(n, m, A, B, u, x, dT);
        ++steps;
    }
    double last = t1 - currentTime;               /* :63-70 stale currentTime                 */
    lti_step(n, m, A, B, u, x, last);
    ++steps;
    if (nsteps_out) *nsteps_out = steps;
    return 0;
}

void orc_dcm_euler_rollout(const double* xi0, const double* omega, const double* vrp, int N,
                           double dt, double* xi_out)
{
    xi_out[0] = xi0[0];
    xi_out[1] = xi0[1];
    for (int k = 0; k < N; ++k) {
        const double w = omega[k];
        for (int j = 0; j < 2; ++j) {
            const double x = xi_out[2 * k + j];
            /* dx = (w*x) + ((-w)*r);  x + dx*dt */
            const double dx = w * x + (-w) * vrp[2 * k + j];
            xi_out[2 * (k + 1) + j] = x + dx * dt;
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* ContactPhaseList::createPhases — ContactPhaseList.cpp:16-84 (quirks reproduced)            */
/* ------------------------------------------------------------------------------------------ */
typedef struct { double t; int l, c; } ev_t;
static int ev_cmp(const void* a, const void* b)
{
    const ev_t* x = (const ev_t*)a;
    const ev_t* y = (const ev_t*)b;
    if (x->t < y->t) return -1;
    if (x->t > y->t) return 1;
    return (x->l < y->l) ? -1 : (x->l > y->l);
}

int orc_contact_phases(int L, int C, const double* act, const double* deact,
                       const int32_t* ncontacts, int max_phases, double* begin, double* end,
                       int32_t* active)
{
    int total = 0;
    for (int l = 0; l < L; ++l) total += ncontacts[l];
    if (total == 0) return 0;                    /* :32-35                                    */
    ev_t* a = (ev_t*)malloc(sizeof(ev_t) * total);
    ev_t* d = (ev_t*)malloc(sizeof(ev_t) * total);
    int n = 0;
    for (int l = 0; l < L; ++l)
        for (int c = 0; c < ncontacts[l]; ++c) {
            a[n].t = act[l * C + c]; a[n].l = l; a[n].c = c;
            d[n].t = deact[l * C + c]; d[n].l = l; d[n].c = c;
            ++n;
        }
    qsort(a, n, sizeof(ev_t), ev_cmp);
    qsort(d, n, sizeof(ev_t), ev_cmp);
    /* group boundaries: the std::map keys are the distinct times */
    int* ga = (int*)malloc(sizeof(int) * (n + 1));
    int* gd = (int*)malloc(sizeof(int) * (n + 1));
    int na = 0, nd = 0;
    for (int i = 0; i < n; ++i) if (i == 0 || a[i].t != a[i - 1].t) ga[na++] = i;
    ga[na] = n;
    for (int i = 0; i < n; ++i) if (i == 0 || d[i].t != d[i - 1].t) gd[nd++] = i;
    gd[nd] = n;

    int32_t cur[64];
    int np = 0, ok = 1;
    if (L > 64) { free(a); free(d); free(ga); free(gd); return -1; }
    for (int l = 0; l < L; ++l) cur[l] = -1;
    double cbegin = a[ga[0]].t;
    for (int i = ga[0]; i < ga[1]; ++i) cur[a[i].l] = a[i].c;   /* :38-39 */
    int ia = 1, id = 0;

#define PUSH(e)                                                                             \
    do {                                                                                    \
        if (np >= max_phases) { ok = 0; break; }                                            \
        begin[np] = cbegin; end[np] = (e);                                                  \
        for (int l_ = 0; l_ < L; ++l_) active[np * L + l_] = cur[l_];                       \
        ++np;                                                                               \
    } while (0)

    while (ok && (na - ia) + (nd - id) > 1) {     /* :43                                      */
        if (ia == na || d[gd[id]].t <= a[ga[ia]].t) {
            double t = d[gd[id]].t;
            PUSH(t);
            cbegin = t;
            for (int i = gd[id]; i < gd[id + 1]; ++i) cur[d[i].l] = -1;   /* erase by key  */
            ++id;
            /* :60 compares the NEXT deactivation time with the next activation time */
            if (ia < na && id < nd && d[gd[id]].t == a[ga[ia]].t) {
                for (int i = ga[ia]; i < ga[ia + 1]; ++i)
                    if (cur[a[i].l] < 0) cur[a[i].l] = a[i].c;   /* insert keeps old keys */
                ++ia;
            }
        } else {
            double t = a[ga[ia]].t;
            PUSH(t);
            cbegin = t;
            for (int i = ga[ia]; i < ga[ia + 1]; ++i)
                if (cur[a[i].l] < 0) cur[a[i].l] = a[i].c;
            ++ia;
        }
    }
    if (ok && nd - id == 1) PUSH(d[gd[id]].t);   /* :81-83                                    */
#undef PUSH
    free(a); free(d); free(ga); free(gd);
    return ok ? np : -1;
}

int orc_present_index(const double* activation_times, int n, double t)
{
    for (int i = n - 1; i >= 0; --i)              /* reverse find_if, `activationTime <= time` */
        if (activation_times[i] <= t) return i;
    return -1;
}

/* ------------------------------------------------------------------------------------------ */
/* ConvexHullHelper (2-D): hull -> H-rep                                                       */
/* ------------------------------------------------------------------------------------------ */
static double cross3(const double* o, const double* a, const double* b)
{
    return (a[0] - o[0]) * (b[1] - o[1]) - (a[1] - o[1]) * (b[0] - o[0]);
}

int orc_hull2d_hrep(const double* pts, int npts, int max_facets, double* A, double* b)
{
    for (int i = 0; i < max_facets; ++i) { A[2 * i] = 0.0; A[2 * i + 1] = 0.0; b[i] = 0.0; }
    if (npts < 3 || npts > 16) return -1;
    /* insertion sort of indices by (x, y) — same comparator as the device kernel */
    int idx[16];
    for (int i = 0; i < npts; ++i) idx[i] = i;
    for (int i = 1; i < npts; ++i) {
        int v = idx[i], j = i - 1;
        while (j >= 0 && (pts[2 * idx[j]] > pts[2 * v] ||
                          (pts[2 * idx[j]] == pts[2 * v] && pts[2 * idx[j] + 1] > pts[2 * v + 1]))) {
            idx[j + 1] = idx[j];
            --j;
        }
        idx[j + 1] = v;
    }
    /* Andrew's monotone chain; cross <= 0 pops collinear and duplicate points */
    int H[34];
    int k = 0;
    for (int i = 0; i < npts; ++i) {
        const double* p = pts + 2 * idx[i];
        while (k >= 2 && cross3(pts + 2 * H[k - 2], pts + 2 * H[k - 1], p) <= 0.0) --k;
        H[k++] = idx[i];
    }
    for (int i = npts - 2, t = k + 1; i >= 0; --i) {
        const double* p = pts + 2 * idx[i];
        while (k >= t && cross3(pts + 2 * H[k - 2], pts + 2 * H[k - 1], p) <= 0.0) --k;
        H[k++] = idx[i];
    }
    const int nv = k - 1;  /* last point repeats the first */
    if (nv < 3) return -1;
    if (nv > max_facets) return -1;
    for (int j = 0; j < nv; ++j) {
        const double* v0 = pts + 2 * H[j];
        const double* v1 = pts + 2 * H[j + 1];
        const double ex = v1[0] - v0[0];
        const double ey = v1[1] - v0[1];
        const double len = sqrt(ex * ex + ey * ey);
        const double nx = ey / len;
        const double ny = (-ex) / len;
        A[2 * j] = nx;
        A[2 * j + 1] = ny;
        b[j] = nx * v0[0] + ny * v0[1];
    }
    return nv;
}

int orc_hull2d_contains(const double* A, const double* b, int nfacets, const double* p)
{
    if (nfacets < 0) return 0;
    for (int i = 0; i < nfacets; ++i)
        if (A[2 * i] * p[0] + A[2 * i + 1] * p[1] > b[i]) return 0;   /* :113 strict */
    return 1;
}

/* ------------------------------------------------------------------------------------------ */
/* Quintic spline (build-defined)                                              */
/* ------------------------------------------------------------------------------------------ */
void orc_quintic_fit(const double* knots_t, const double* knots_pva, int nknots, int dim,
                     double* coeffs)
{
    const int K = nknots - 1;
    for (int j = 0; j < K; ++j) {
        const double T = knots_t[j + 1] - knots_t[j];
        const double T2 = T * T;
        const double T3 = T2 * T;
        const double T4 = T3 * T;
        const double T5 = T4 * T;
        for (int d = 0; d < dim; ++d) {
            const double p0 = knots_pva[(j * 3 + 0) * dim + d];
            const double v0 = knots_pva[(j * 3 + 1) * dim + d];
            const double a0 = knots_pva[(j * 3 + 2) * dim + d];
            const double p1 = knots_pva[((j + 1) * 3 + 0) * dim + d];
            const double v1 = knots_pva[((j + 1) * 3 + 1) * dim + d];
            const double a1 = knots_pva[((j + 1) * 3 + 2) * dim + d];
            const double c2 = 0.5 * a0;
            const double h = p1 - ((p0 + v0 * T) + c2 * T2);
            const double hv = v1 - (v0 + a0 * T);
            const double ha = a1 - a0;
            double* c = coeffs + (j * dim + d) * 6;
            c[0] = p0;
            c[1] = v0;
            c[2] = c2;
            c[3] = ((10.0 * h - 4.0 * (hv * T)) + 0.5 * (ha * T2)) / T3;
            c[4] = ((-15.0 * h + 7.0 * (hv * T)) - ha * T2) / T4;
            c[5] = ((6.0 * h - 3.0 * (hv * T)) + 0.5 * (ha * T2)) / T5;
        }
    }
}

void orc_quintic_eval(const double* knots_t, const double* coeffs, int nknots, int dim,
                      const double* tq, int nq, double* pva, int32_t* knot_idx)
{
    const int K = nknots - 1;
    for (int q = 0; q < nq; ++q) {
        const double t = tq[q];
        const int raw = orc_present_index(knots_t, nknots, t);
        knot_idx[q] = raw;
        int seg = raw < 0 ? 0 : (raw > K - 1 ? K - 1 : raw);
        const double tau = t - knots_t[seg];
        for (int d = 0; d < dim; ++d) {
            const double* c = coeffs + (seg * dim + d) * 6;
            const double p = c[0] + tau * (c[1] + tau * (c[2] + tau * (c[3] + tau * (c[4] + tau * c[5]))));
            const double v = c[1] + tau * (2.0 * c[2] + tau * (3.0 * c[3] + tau * (4.0 * c[4] + tau * (5.0 * c[5]))));
            const double a = 2.0 * c[2] + tau * (6.0 * c[3] + tau * (12.0 * c[4] + tau * (20.0 * c[5])));
            pva[(q * 3 + 0) * dim + d] = p;
            pva[(q * 3 + 1) * dim + d] = v;
            pva[(q * 3 + 2) * dim + d] = a;
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* DCM-MPC QP: Mehrotra primal-dual IPM + Riccati                        */
/* ------------------------------------------------------------------------------------------ */
double orc_wave_tree_sum(const double* c, int n)
{
    const int nblk = (n + 63) / 64;
    double total = 0.0;
    for (int w = 0; w < nblk; ++w) {
        double v[64], t[64];
        for (int l = 0; l < 64; ++l) v[l] = (64 * w + l < n) ? c[64 * w + l] : 0.0;
        for (int off = 32; off >= 1; off >>= 1) {
            for (int l = 0; l < 64; ++l) t[l] = v[l] + v[l ^ off];
            memcpy(v, t, sizeof(v));
        }
        total = (w == 0) ? v[0] : total + v[0];
    }
    return total;
}

#define MF 8

/* Working state of one QP solve (all arrays owned by the caller of dcm_ws_alloc). */
typedef struct {
    int N, M, ntot;
    double dt, Qw0, Qw1, Rw0, Rw1, Pw0, Pw1;
    const double *omega, *xi_ref, *vrp_ref, *A, *b;
    const int32_t* nf;
    double *al, *be, *a2, *b2;          /* [N] */
    double *s, *lam, *rp, *prod;        /* [N][MF] */
    double *W;                          /* [N][4]  A^T diag(lam/s) A (3), det of it (1) */
    double *Hi, *Pn;                    /* [N][3] */
    double *g, *d, *rho, *kff, *dr, *qx; /* [N][2] */
    double *c;                          /* [N] */
    double *dxi, *nu;                   /* [N+1][2] */
    double *xi, *vrp;                   /* outputs, updated in place */
} dcm_ws;

/* Stage-parallel residual pass (the device runs one thread per knot): primal residuals
 * rp = A r + s - b, complementarity partials c_k, rho = R (r - r_ref) + A^T lam, Euler defects
 * d_k (reference step order) and Q (xi_k - xi_ref_k).  Returns max |rp|, |d| (NaN-propagating). */
static double dcm_residuals(dcm_ws* w)
{
    const int N = w->N, M = w->M;
    double pres = 0.0;
    for (int k = 0; k < N; ++k) {
        const int m = w->nf[k];
        const double r0 = w->vrp[2 * k], r1 = w->vrp[2 * k + 1];
        double ck = 0.0;
        double rh0 = w->Rw0 * (r0 - w->vrp_ref[2 * k]);
        double rh1 = w->Rw1 * (r1 - w->vrp_ref[2 * k + 1]);
        for (int i = 0; i < m; ++i) {
            const double* a = w->A + (k * M + i) * 2;
            const double si = w->s[k * MF + i], li = w->lam[k * MF + i];
            const double gr = a[0] * r0 + a[1] * r1;
            const double rpi = (gr + si) - w->b[k * M + i];
            w->rp[k * MF + i] = rpi;
            const double e = fabs(rpi);
            if (e > pres || e != e) pres = e;
            ck = ck + si * li;
            rh0 = rh0 + a[0] * li;
            rh1 = rh1 + a[1] * li;
        }
        w->c[k] = ck;
        w->rho[2 * k] = rh0;
        w->rho[2 * k + 1] = rh1;
        const double om = w->omega[k];
        for (int j = 0; j < 2; ++j) {
            const double x = w->xi[2 * k + j];
            const double dx = om * x + (-om) * w->vrp[2 * k + j];
            const double dk = (x + dx * w->dt) - w->xi[2 * (k + 1) + j];
            w->d[2 * k + j] = dk;
            const double e = fabs(dk);
            if (e > pres || e != e) pres = e;
        }
        if (k >= 1) {
            w->qx[2 * k] = w->Qw0 * (w->xi[2 * k] - w->xi_ref[2 * k]);
            w->qx[2 * k + 1] = w->Qw1 * (w->xi[2 * k + 1] - w->xi_ref[2 * k + 1]);
        }
    }
    return pres;
}

/* Backward Riccati sweep (sequential over knots).  factor != 0: builds Hi_k = H_k^{-1},
 * Pn_k = P_{k+1} (returns 0 if some H_k is not positive definite); factor == 0: reuses them.
 * Either way solves for the feed-forward kff with right-hand side g. */
static int dcm_backward(dcm_ws* w, int factor)
{
    const int N = w->N;
    int ok = 1;
    double P00 = w->Pw0, P01 = 0.0, P11 = w->Pw1;
    double pv0 = w->Pw0 * (w->xi[2 * N] - w->xi_ref[2 * N]);
    double pv1 = w->Pw1 * (w->xi[2 * N + 1] - w->xi_ref[2 * N + 1]);
    for (int k = N - 1; k >= 0; --k) {
        double h00, h01, h11;
        const double b2 = w->b2[k];
        if (factor) {
            /* H = B + W, B = R + b2 P_{k+1} (SPD, well conditioned), W PSD:
             * det H = det B + tr(adj(B) W) + det W, every term >= 0 — no cancellation when
             * the barrier weights inside W are huge */
            const double B00 = w->Rw0 + b2 * P00;
            const double B01 = b2 * P01;
            const double B11 = w->Rw1 + b2 * P11;
            const double W00 = w->W[4 * k], W01 = w->W[4 * k + 1], W11 = w->W[4 * k + 2];
            const double H00 = B00 + W00;
            const double H01 = B01 + W01;
            const double H11 = B11 + W11;
            const double detB = B00 * B11 - B01 * B01;
            const double trW = (B11 * W00 + B00 * W11) - 2.0 * (B01 * W01);
            const double det = (detB + trW) + w->W[4 * k + 3];
            if (!(det > 0.0) || isinf(det)) ok = 0;
            const double idet = 1.0 / det;
            h00 = H11 * idet;
            h01 = -(H01 * idet);
            h11 = H00 * idet;
            w->Hi[3 * k] = h00; w->Hi[3 * k + 1] = h01; w->Hi[3 * k + 2] = h11;
            w->Pn[3 * k] = P00; w->Pn[3 * k + 1] = P01; w->Pn[3 * k + 2] = P11;
        } else {
            h00 = w->Hi[3 * k]; h01 = w->Hi[3 * k + 1]; h11 = w->Hi[3 * k + 2];
            P00 = w->Pn[3 * k]; P01 = w->Pn[3 * k + 1]; P11 = w->Pn[3 * k + 2];
        }
        const double be = w->be[k];
        const double d0 = w->d[2 * k], d1 = w->d[2 * k + 1];
        const double t0 = (P00 * d0 + P01 * d1) + pv0;
        const double t1 = (P01 * d0 + P11 * d1) + pv1;
        const double hu0 = w->g[2 * k] - be * t0;
        const double hu1 = w->g[2 * k + 1] - be * t1;
        const double k0 = -(h00 * hu0 + h01 * hu1);
        const double k1 = -(h01 * hu0 + h11 * hu1);
        w->kff[2 * k] = k0;
        w->kff[2 * k + 1] = k1;
        if (k > 0) {
            const double al = w->al[k];
            const double pk0 = P00 * k0 + P01 * k1;
            const double pk1 = P01 * k0 + P11 * k1;
            const double npv0 = w->qx[2 * k] + al * (t0 - be * pk0);
            const double npv1 = w->qx[2 * k + 1] + al * (t1 - be * pk1);
            if (factor) {
                /* P_k = Q + a^2 (P - b^2 P H^-1 P)  (never multiplies by the huge W) */
                const double a2 = w->a2[k];
                const double M00 = P00 * h00 + P01 * h01;
                const double M01 = P00 * h01 + P01 * h11;
                const double M10 = P01 * h00 + P11 * h01;
                const double M11 = P01 * h01 + P11 * h11;
                const double S00 = M00 * P00 + M01 * P01;
                const double S01 = M00 * P01 + M01 * P11;
                const double S10 = M10 * P00 + M11 * P01;
                const double S11 = M10 * P01 + M11 * P11;
                const double n00 = w->Qw0 + a2 * (P00 - b2 * S00);
                const double n11 = w->Qw1 + a2 * (P11 - b2 * S11);
                const double n01 = a2 * (P01 - b2 * (0.5 * (S01 + S10)));
                P00 = n00;
                P01 = n01;
                P11 = n11;
            }
            pv0 = npv0;
            pv1 = npv1;
        }
    }
    return ok;
}

/* Forward sweep: dr_k = (alpha beta) Hi_k (P_{k+1} dxi_k) + kff_k,
 * dxi_{k+1} = (alpha dxi_k - beta dr_k) + d_k, dxi_0 = 0. */
static void dcm_forward(dcm_ws* w)
{
    double x0 = 0.0, x1 = 0.0;
    w->dxi[0] = 0.0;
    w->dxi[1] = 0.0;
    for (int k = 0; k < w->N; ++k) {
        const double q00 = w->Pn[3 * k], q01 = w->Pn[3 * k + 1], q11 = w->Pn[3 * k + 2];
        const double u0 = q00 * x0 + q01 * x1;
        const double u1 = q01 * x0 + q11 * x1;
        const double v0 = w->Hi[3 * k] * u0 + w->Hi[3 * k + 1] * u1;
        const double v1 = w->Hi[3 * k + 1] * u0 + w->Hi[3 * k + 2] * u1;
        const double al = w->al[k], be = w->be[k];
        const double ab = al * be;
        const double r0 = ab * v0 + w->kff[2 * k];
        const double r1 = ab * v1 + w->kff[2 * k + 1];
        w->dr[2 * k] = r0;
        w->dr[2 * k + 1] = r1;
        const double n0 = (al * x0 - be * r0) + w->d[2 * k];
        const double n1 = (al * x1 - be * r1) + w->d[2 * k + 1];
        w->dxi[2 * (k + 1)] = n0;
        w->dxi[2 * (k + 1) + 1] = n1;
        x0 = n0;
        x1 = n1;
    }
}

int orc_dcm_mpc_solve(const orc_dcm_params* prm, const double* xi_init, const double* omega,
                      const double* xi_ref, const double* vrp_ref, const double* Ain,
                      const double* bin, const int32_t* nfacets, double* xi, double* vrp,
                      int32_t* iters_out)
{
    const int N = prm->horizon;
    const int M = prm->max_facets;
    dcm_ws ws;
    dcm_ws* w = &ws;
    w->N = N; w->M = M; w->dt = prm->dt;
    w->Qw0 = prm->w_xi[0]; w->Qw1 = prm->w_xi[1];
    w->Rw0 = prm->w_vrp[0]; w->Rw1 = prm->w_vrp[1];
    w->Pw0 = prm->w_terminal[0]; w->Pw1 = prm->w_terminal[1];
    w->omega = omega; w->xi_ref = xi_ref; w->vrp_ref = vrp_ref; w->A = Ain; w->b = bin;
    w->nf = nfacets; w->xi = xi; w->vrp = vrp;
    double* mem = (double*)malloc(sizeof(double) * ((size_t)N * (4 + 4 * MF + 4 + 6 + 12 + 1) +
                                                    4 * (size_t)(N + 1)));
    double* q = mem;
    w->al = q; q += N; w->be = q; q += N; w->a2 = q; q += N; w->b2 = q; q += N;
    w->s = q; q += N * MF; w->lam = q; q += N * MF; w->rp = q; q += N * MF; w->prod = q; q += N * MF;
    w->W = q; q += 4 * N;
    w->Hi = q; q += 3 * N; w->Pn = q; q += 3 * N;
    w->g = q; q += 2 * N; w->d = q; q += 2 * N; w->rho = q; q += 2 * N; w->kff = q; q += 2 * N;
    w->dr = q; q += 2 * N; w->qx = q; q += 2 * N;
    w->c = q; q += N;
    w->dxi = q; q += 2 * (N + 1); w->nu = q; q += 2 * (N + 1);

    int status = 0, it = 0;
    int ntot = 0;
    for (int k = 0; k < N; ++k) {
        if (nfacets[k] < 0 || nfacets[k] > M) status = 3;
        else ntot += nfacets[k];
    }
    w->ntot = ntot;

    /* ---- initial point ----
     * 1. vrp = vrp_ref, xi = reference Euler rollout from xi_init;
     * 2. one full Newton step of the QP WITHOUT the polygon constraints (the unconstrained LQ
     *    optimum; W = 0, lam = 0): for the unstable DCM the open-loop rollout is far from
     *    dual feasible (costates grow like alpha^N), this step makes the linear residuals O(1);
     * 3. s = max(b - A r, 1e-2), lam = 1. */
    for (int k = 0; k < N; ++k) {
        w->be[k] = w->dt * omega[k];
        w->al[k] = 1.0 + w->be[k];
        w->a2[k] = w->al[k] * w->al[k];
        w->b2[k] = w->be[k] * w->be[k];
        vrp[2 * k] = vrp_ref[2 * k];
        vrp[2 * k + 1] = vrp_ref[2 * k + 1];
    }
    orc_dcm_euler_rollout(xi_init, omega, vrp, N, w->dt, xi);
    if (status == 3) {
        if (iters_out) *iters_out = 0;
        free(mem);
        return 3;
    }
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < MF; ++i) { w->s[k * MF + i] = 1.0; w->lam[k * MF + i] = 0.0; }
    {
        const int nf_saved = w->ntot;
        int32_t* zero = (int32_t*)calloc(N, sizeof(int32_t));
        w->nf = zero;                      /* no facets: rho = R (r - r_ref), W = 0 */
        dcm_residuals(w);
        w->nf = nfacets;
        w->ntot = nf_saved;
        free(zero);
        for (int k = 0; k < N; ++k) {
            w->W[4 * k] = 0.0; w->W[4 * k + 1] = 0.0; w->W[4 * k + 2] = 0.0; w->W[4 * k + 3] = 0.0;
            w->g[2 * k] = w->rho[2 * k];
            w->g[2 * k + 1] = w->rho[2 * k + 1];
        }
        if (!dcm_backward(w, 1)) status = 2;
        dcm_forward(w);
        for (int k = 0; k < N; ++k) {
            vrp[2 * k] = vrp[2 * k] + w->dr[2 * k];
            vrp[2 * k + 1] = vrp[2 * k + 1] + w->dr[2 * k + 1];
            xi[2 * (k + 1)] = xi[2 * (k + 1)] + w->dxi[2 * (k + 1)];
            xi[2 * (k + 1) + 1] = xi[2 * (k + 1) + 1] + w->dxi[2 * (k + 1) + 1];
        }
    }
    for (int k = 0; k < N; ++k) {
        const int m = nfacets[k];
        for (int i = 0; i < MF; ++i) {
            if (i < m) {
                const double* a = Ain + (k * M + i) * 2;
                const double gr = a[0] * vrp[2 * k] + a[1] * vrp[2 * k + 1];
                double sl = bin[k * M + i] - gr;
                w->s[k * MF + i] = sl > 1e-2 ? sl : 1e-2;
                w->lam[k * MF + i] = 1.0;
            }
        }
    }

    /* initial dual residual (single-shooting costates): dres0 = max |rho_k - beta_k nu_{k+1}|;
     * it then contracts by (1 - a) with every damped Newton step (the QP's linear residuals). */
    double dres = 0.0;
    {
        double* nu = w->nu;
        nu[2 * N] = w->Pw0 * (xi[2 * N] - xi_ref[2 * N]);
        nu[2 * N + 1] = w->Pw1 * (xi[2 * N + 1] - xi_ref[2 * N + 1]);
        for (int k = N - 1; k >= 1; --k) {
            nu[2 * k] = w->Qw0 * (xi[2 * k] - xi_ref[2 * k]) + w->al[k] * nu[2 * (k + 1)];
            nu[2 * k + 1] = w->Qw1 * (xi[2 * k + 1] - xi_ref[2 * k + 1]) + w->al[k] * nu[2 * (k + 1) + 1];
        }
        for (int k = 0; k < N; ++k) {
            const int m = nfacets[k];
            for (int j = 0; j < 2; ++j) {
                double rj = (j == 0 ? w->Rw0 : w->Rw1) * (vrp[2 * k + j] - vrp_ref[2 * k + j]);
                for (int i = 0; i < m; ++i) rj = rj + Ain[(k * M + i) * 2 + j] * w->lam[k * MF + i];
                const double e = fabs(rj - w->be[k] * nu[2 * (k + 1) + j]);
                if (e > dres || e != e) dres = e;
            }
        }
    }
    if (status == 2) {
        if (iters_out) *iters_out = 0;
        free(mem);
        return 2;
    }

    for (it = 0;; ++it) {
        const double pres = dcm_residuals(w);
        const double mu = ntot > 0 ? orc_wave_tree_sum(w->c, N) / (double)ntot : 0.0;
        if (!(mu == mu) || !(pres == pres) || !(dres == dres) || isinf(mu)) { status = 2; break; }
        if (mu <= prm->tol_mu && pres <= prm->tol_primal && dres <= prm->tol_dual) { status = 0; break; }
        if (it >= prm->max_iter) { status = 1; break; }

        /* ---- W = A^T diag(lam/s) A, det(W) as a sum of non-negative terms, affine rhs g
         *      (stage-parallel) ---- */
        for (int k = 0; k < N; ++k) {
            const int m = nfacets[k];
            double W00 = 0.0, W01 = 0.0, W11 = 0.0, dW = 0.0;
            double g0 = w->rho[2 * k], g1 = w->rho[2 * k + 1];
            double sgv[MF];
            for (int i = 0; i < m; ++i) {
                const double* a = Ain + (k * M + i) * 2;
                const double si = w->s[k * MF + i], li = w->lam[k * MF + i];
                const double sg = li / si;
                sgv[i] = sg;
                const double t0 = sg * a[0];
                const double t1 = sg * a[1];
                W00 = W00 + t0 * a[0];
                W01 = W01 + t0 * a[1];
                W11 = W11 + t1 * a[1];
                const double rc = si * li;
                const double e = (li * w->rp[k * MF + i] - rc) / si;
                g0 = g0 + a[0] * e;
                g1 = g1 + a[1] * e;
            }
            /* det(sum_i sg_i a_i a_i^T) = sum_{i<j} sg_i sg_j (a_i x a_j)^2 */
            for (int i = 1; i < m; ++i) {
                const double* ai = Ain + (k * M + i) * 2;
                for (int j = 0; j < i; ++j) {
                    const double* aj = Ain + (k * M + j) * 2;
                    const double cr = ai[0] * aj[1] - ai[1] * aj[0];
                    dW = dW + (sgv[i] * sgv[j]) * (cr * cr);
                }
            }
            w->W[4 * k] = W00; w->W[4 * k + 1] = W01; w->W[4 * k + 2] = W11; w->W[4 * k + 3] = dW;
            w->g[2 * k] = g0; w->g[2 * k + 1] = g1;
        }

        /* ---- affine (predictor) step ---- */
        if (!dcm_backward(w, 1)) status = 2;
        dcm_forward(w);
        double smax = INFINITY;
        for (int k = 0; k < N; ++k) {
            const int m = nfacets[k];
            for (int i = 0; i < m; ++i) {
                const double* a = Ain + (k * M + i) * 2;
                const double si = w->s[k * MF + i], li = w->lam[k * MF + i];
                const double rc = si * li;
                const double ds = (-w->rp[k * MF + i]) - (a[0] * w->dr[2 * k] + a[1] * w->dr[2 * k + 1]);
                const double dl = ((-rc) - li * ds) / si;
                if (ds < 0.0) { const double qq = (-si) / ds; if (qq < smax) smax = qq; }
                if (dl < 0.0) { const double qq = (-li) / dl; if (qq < smax) smax = qq; }
                w->prod[k * MF + i] = ds * dl;
            }
        }
        const double a_aff = smax < 1.0 ? smax : 1.0;
        for (int k = 0; k < N; ++k) {
            const int m = nfacets[k];
            double ck = 0.0;
            for (int i = 0; i < m; ++i) {
                const double* a = Ain + (k * M + i) * 2;
                const double si = w->s[k * MF + i], li = w->lam[k * MF + i];
                const double rc = si * li;
                const double ds = (-w->rp[k * MF + i]) - (a[0] * w->dr[2 * k] + a[1] * w->dr[2 * k + 1]);
                const double dl = ((-rc) - li * ds) / si;
                ck = ck + (si + a_aff * ds) * (li + a_aff * dl);
            }
            w->c[k] = ck;
        }
        const double mu_aff = ntot > 0 ? orc_wave_tree_sum(w->c, N) / (double)ntot : 0.0;
        double sigma = 0.0;
        if (mu > 0.0) {
            const double qq = mu_aff / mu;
            sigma = (qq * qq) * qq;
        }
        const double sigma_mu = sigma * mu;

        /* ---- corrector: rhs (stage-parallel), solve reusing the factorization ---- */
        for (int k = 0; k < N; ++k) {
            const int m = nfacets[k];
            double g0 = w->rho[2 * k], g1 = w->rho[2 * k + 1];
            for (int i = 0; i < m; ++i) {
                const double* a = Ain + (k * M + i) * 2;
                const double si = w->s[k * MF + i], li = w->lam[k * MF + i];
                const double rc = (si * li + w->prod[k * MF + i]) - sigma_mu;
                const double e = (li * w->rp[k * MF + i] - rc) / si;
                g0 = g0 + a[0] * e;
                g1 = g1 + a[1] * e;
            }
            w->g[2 * k] = g0; w->g[2 * k + 1] = g1;
        }
        dcm_backward(w, 0);
        dcm_forward(w);
        smax = INFINITY;
        for (int k = 0; k < N; ++k) {
            const int m = nfacets[k];
            for (int i = 0; i < m; ++i) {
                const double* a = Ain + (k * M + i) * 2;
                const double si = w->s[k * MF + i], li = w->lam[k * MF + i];
                const double rc = (si * li + w->prod[k * MF + i]) - sigma_mu;
                const double ds = (-w->rp[k * MF + i]) - (a[0] * w->dr[2 * k] + a[1] * w->dr[2 * k + 1]);
                const double dl = ((-rc) - li * ds) / si;
                if (ds < 0.0) { const double qq = (-si) / ds; if (qq < smax) smax = qq; }
                if (dl < 0.0) { const double qq = (-li) / dl; if (qq < smax) smax = qq; }
                w->rp[k * MF + i] = ds;      /* keep the step for the update */
                w->prod[k * MF + i] = dl;
            }
        }
        if (status == 2) break;
        const double step = 0.99 * smax;
        const double a = step < 1.0 ? step : 1.0;
        for (int k = 0; k < N; ++k) {
            vrp[2 * k] = vrp[2 * k] + a * w->dr[2 * k];
            vrp[2 * k + 1] = vrp[2 * k + 1] + a * w->dr[2 * k + 1];
            xi[2 * (k + 1)] = xi[2 * (k + 1)] + a * w->dxi[2 * (k + 1)];
            xi[2 * (k + 1) + 1] = xi[2 * (k + 1) + 1] + a * w->dxi[2 * (k + 1) + 1];
            const int m = nfacets[k];
            for (int i = 0; i < m; ++i) {
                w->s[k * MF + i] = w->s[k * MF + i] + a * w->rp[k * MF + i];
                w->lam[k * MF + i] = w->lam[k * MF + i] + a * w->prod[k * MF + i];
            }
        }
        dres = dres * (1.0 - a);
    }
    if (iters_out) *iters_out = it;
    free(mem);
    return status;
}

/* ---- batch driver with POSIX threads (CPU baseline) ---- */
typedef struct {
    const orc_dcm_params* prm;
    int64_t batch;
    const double *xi_init, *omega, *xi_ref, *vrp_ref, *A, *b;
    const int32_t* nfacets;
    double *xi, *vrp;
    int32_t *status, *iters;
    atomic_llong next;
} batch_job;

static void* batch_worker(void* arg)
{
    batch_job* J = (batch_job*)arg;
    const int N = J->prm->horizon, M = J->prm->max_facets;
    for (;;) {
        const long long p = atomic_fetch_add(&J->next, 1);
        if (p >= J->batch) break;
        J->status[p] = orc_dcm_mpc_solve(J->prm, J->xi_init + 2 * p, J->omega + (int64_t)N * p,
                                         J->xi_ref + (int64_t)2 * (N + 1) * p,
                                         J->vrp_ref + (int64_t)2 * N * p,
                                         J->A + (int64_t)2 * N * M * p, J->b + (int64_t)N * M * p,
                                         J->nfacets + (int64_t)N * p,
                                         J->xi + (int64_t)2 * (N + 1) * p,
                                         J->vrp + (int64_t)2 * N * p, J->iters + p);
    }
    return NULL;
}

void orc_dcm_mpc_solve_batch(const orc_dcm_params* prm, int64_t batch, int threads,
                             const double* xi_init, const double* omega, const double* xi_ref,
                             const double* vrp_ref, const double* A, const double* b,
                             const int32_t* nfacets, double* xi, double* vrp, int32_t* status,
                             int32_t* iters)
{
    batch_job J = {.prm = prm, .batch = batch, .xi_init = xi_init, .omega = omega,
                   .xi_ref = xi_ref, .vrp_ref = vrp_ref, .A = A, .b = b, .nfacets = nfacets,
                   .xi = xi, .vrp = vrp, .status = status, .iters = iters};
    atomic_init(&J.next, 0);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int t = 1; t < threads; ++t) pthread_create(&th[t], NULL, batch_worker, &J);
    batch_worker(&J);
    for (int t = 1; t < threads; ++t) pthread_join(th[t], NULL);
}
