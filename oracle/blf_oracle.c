/*
 * blf_oracle.c — TEST INFRASTRUCTURE ONLY (see blf_oracle.h).  CPU restatement of the reference
 * semantics, fp64, compiled with -ffp-contract=off so that every expression is evaluated exactly
 * in the order written (the device kernels follow the same order).
 */
#include "blf_oracle.h"

#include <math.h>
#include <stdio.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------------ */
/* ForwardEuler<LinearTimeInvariantSystem>::integrate — FixedStepIntegrator.tpp:21-72          */
/* ------------------------------------------------------------------------------------------ */
static void lti_step(int n, int m, const double* A, const double* B, const double* u, double* x,
                     double dT, double* dx)
{
    /* LinearTimeInvariantSystem.cpp:71  dx = A x + B u ;  ForwardEuler.tpp:36-38  x += dx*dT */
    for (int r = 0; r < n; ++r) {
        const double* Ar = A + (int64_t)r * n;
        const double* Br = B + (int64_t)r * m;
        double ax = Ar[0] * x[0];
        for (int c = 1; c < n; ++c) ax = ax + Ar[c] * x[c];
        double bu = Br[0] * u[0];
        for (int c = 1; c < m; ++c) bu = bu + Br[c] * u[c];
        dx[r] = ax + bu;
    }
    for (int r = 0; r < n; ++r) x[r] = x[r] + dx[r] * dT;
}

int orc_lti_euler_integrate(int n, int m, const double* A, const double* B, const double* u,
                            double* x, double t0, double t1, double dT, int64_t* nsteps_out)
{
    if (n < 1 || m < 1) return 1;                 /* any size (the C ABI's n, m >= 1)          */
    if (t0 > t1 || !(dT > 0)) return 4;           /* FixedStepIntegrator.tpp:28-46            */
    if (t0 == t1) return 5;                       /* reference: size_t(i) < -1 -> never ends   */
    double q = ceil((t1 - t0) / dT);
    if (!(q < 2.0e9)) return 3;
    double* dx = (double*)malloc(sizeof(double) * (size_t)n);
    if (!dx) return 2;
    int iterations = (int)q;                      /* FixedStepIntegrator.tpp:48               */
    double currentTime = t0;
    int64_t steps = 0;
    for (int64_t i = 0; i < (int64_t)iterations - 1; ++i) {   /* :51-61                      */
        currentTime = t0 + dT * (double)i;
        lti_step(n, m, A, B, u, x, dT, dx);
        ++steps;
    }
    double last = t1 - currentTime;               /* :63-70 stale currentTime                 */
    lti_step(n, m, A, B, u, x, last, dx);
    ++steps;
    free(dx);
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

/* Test switch (tests/test_oracle.py): 1 forces Andrew's monotone chain for every point count, so
 * the all-triples rule the device uses for up to 8 finite points can be compared with it. */
static int g_hull_force_andrew = 0;
void orc_hull2d_force_andrew(int on) { g_hull_force_andrew = on; }

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
    int finite = 1;
    for (int i = 0; i < 2 * npts; ++i) finite = finite && isfinite(pts[i]);
    int H[34];
    int k = 0;
    if (npts <= 8 && finite && !g_hull_force_andrew) {
        /* Up to 8 finite points (the device's register path, hull2d_kernel): sorted point j
         * (0 < j < n - 1) is a lower-chain vertex iff cross3(p_i, p_j, p_k) > 0 for every
         * i < j < k < n, an upper-chain vertex iff cross3(p_k, p_j, p_i) > 0 for every such pair:
         * the triples Andrew's pops test, in the same argument order; in exact arithmetic exactly
         * the chain's vertices (strictly convex ones; collinear and duplicate points dropped). */
        int bl[8] = {0}, bu[8] = {0};
        const double* p0 = pts + 2 * idx[0];
        const double* pn = pts + 2 * idx[npts - 1];
        for (int kk = 2; kk < npts; ++kk)
            for (int j = 1; j < kk; ++j)
                for (int i = 0; i < j; ++i) {
                    const double* pi = pts + 2 * idx[i];
                    const double* pj = pts + 2 * idx[j];
                    const double* pk = pts + 2 * idx[kk];
                    /* duplicates: Andrew's lower pass keeps the last copy of a repeated point
                     * (the first at the left end), its upper pass the first copy (none at the
                     * right end), so a copy's own duplicates do not reject it there */
                    const int li = !(pi[0] == pj[0] && pi[1] == pj[1]) || (pj[0] == p0[0] && pj[1] == p0[1]);
                    const int ui = !(pk[0] == pj[0] && pk[1] == pj[1]) || (pj[0] == pn[0] && pj[1] == pn[1]);
                    if (li && !(cross3(pi, pj, pk) > 0.0)) bl[j] = 1;
                    if (ui && !(cross3(pk, pj, pi) > 0.0)) bu[j] = 1;
                }
        for (int s = 0; s < npts; ++s)
            if (s == 0 || s == npts - 1 || !bl[s]) H[k++] = idx[s];
        for (int s = npts - 2; s >= 1; --s)
            if (!bu[s]) H[k++] = idx[s];
        H[k++] = idx[0];
    } else {
        /* Andrew's monotone chain; cross <= 0 pops collinear and duplicate points */
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
    }
    const int nv = k - 1;  /* last point repeats the first */
    if (nv < 3) return -1;
    if (nv > max_facets) return -1;
    for (int j = 0; j < nv; ++j) {
        const double* v0 = pts + 2 * H[j];
        const double* v1 = pts + 2 * H[j + 1];
        const double ex = v1[0] - v0[0];
        const double ey = v1[1] - v0[1];
        /* one reciprocal of the edge length per facet (the device's instruction count, DESIGN.md
         * 3.0); within the Qhull fixture's 1e-12 of the two quotients it replaced */
        const double il = 1.0 / sqrt(ex * ex + ey * ey);
        const double nx = ey * il;
        const double ny = (-ex) * il;
        A[2 * j] = nx;
        A[2 * j + 1] = ny;
        b[j] = nx * v0[0] + ny * v0[1];
    }
    return nv;
}

/* 3-D H-representation (ConvexHullHelper::buildConvexHull on a 3 x p matrix,
 * ConvexHullHelper.cpp:35-99; the reference's own test is 3-D, ConvexHullHelperTest.cpp:15-63).
 * The facets are the distinct supporting planes through three input points: for i < j < k in
 * lexicographic order, c = (p_j - p_i) x (p_k - p_i), n = c / |c|, d_l = n . (p_l - p_i); the plane
 * supports the set when no d_l exceeds tol on one side (tol = 1e-12 (1 + max |coordinate|)); its
 * outward normal is n when no d_l > tol, else -n; b = max_l n . p_l, so every input point satisfies
 * A p <= b exactly (the reference test's membership checks).  A plane within 1e-9 (normal,
 * infinity norm) and 1e-9 (1 + scale) (offset) of an earlier one is the same facet (Qhull "Qt"
 * triangulates a face into several facets with one plane; compare as sets of planes).  Returns
 * -1 for fewer than 4 points, a flat set (every triple has all points within tol of its plane),
 * or more than max_facets planes.  The kernel (hull3d_kernel) runs these operations in this order
 * (-ffp-contract=off), so the two agree bit for bit. */
int orc_hull3d_hrep(const double* pts, int npts, int max_facets, double* A, double* b)
{
    for (int e = 0; e < 3 * max_facets; ++e) A[e] = 0.0;
    for (int e = 0; e < max_facets; ++e) b[e] = 0.0;
    if (npts < 4) return -1;
    double scale = 0.0;
    for (int e = 0; e < 3 * npts; ++e) {
        const double a = fabs(pts[e]);
        if (a > scale) scale = a;
    }
    const double tol = 1e-12 * (1.0 + scale);
    const double btol = 1e-9 * (1.0 + scale);
    int count = 0, overflow = 0;
    for (int i = 0; i < npts; ++i)
        for (int j = i + 1; j < npts; ++j)
            for (int k = j + 1; k < npts; ++k) {
                const double* pi = pts + 3 * i;
                const double* pj = pts + 3 * j;
                const double* pk = pts + 3 * k;
                const double ux = pj[0] - pi[0], uy = pj[1] - pi[1], uz = pj[2] - pi[2];
                const double vx = pk[0] - pi[0], vy = pk[1] - pi[1], vz = pk[2] - pi[2];
                const double cx = uy * vz - uz * vy;
                const double cy = uz * vx - ux * vz;
                const double cz = ux * vy - uy * vx;
                const double len = sqrt(cx * cx + cy * cy + cz * cz);
                if (!(len > 0.0)) continue;
                double nx = cx / len, ny = cy / len, nz = cz / len;
                int pos = 0, neg = 0;
                for (int l = 0; l < npts; ++l) {
                    const double* q = pts + 3 * l;
                    const double d = nx * (q[0] - pi[0]) + ny * (q[1] - pi[1]) + nz * (q[2] - pi[2]);
                    if (d > tol) pos = 1;
                    if (d < -tol) neg = 1;
                }
                if ((pos && neg) || !(pos || neg)) continue;
                if (pos) {
                    nx = -nx;
                    ny = -ny;
                    nz = -nz;
                }
                double bm = -INFINITY;
                for (int l = 0; l < npts; ++l) {
                    const double* q = pts + 3 * l;
                    const double v = nx * q[0] + ny * q[1] + nz * q[2];
                    if (v > bm) bm = v;
                }
                int dup = 0;
                for (int e = 0; e < count && e < max_facets; ++e)
                    if (fabs(A[3 * e] - nx) <= 1e-9 && fabs(A[3 * e + 1] - ny) <= 1e-9 &&
                        fabs(A[3 * e + 2] - nz) <= 1e-9 && fabs(b[e] - bm) <= btol)
                        dup = 1;
                if (dup) continue;
                if (count < max_facets) {
                    A[3 * count] = nx;
                    A[3 * count + 1] = ny;
                    A[3 * count + 2] = nz;
                    b[count] = bm;
                } else {
                    overflow = 1;
                }
                ++count;
            }
    if (overflow || count < 4) {
        for (int e = 0; e < 3 * max_facets; ++e) A[e] = 0.0;
        for (int e = 0; e < max_facets; ++e) b[e] = 0.0;
        return -1;
    }
    return count;
}

/* ConvexHullHelper::buildConvexHull on dim x p points, any dim (ConvexHullHelper.cpp:35-99; the
 * reference hands the n x p matrix to Qhull).  Every dim-subset of the points in lexicographic
 * order spans a candidate hyperplane; its normal is the null vector of the (dim-1) x dim matrix of
 * differences p_j - p_i0 (Gaussian elimination with full pivoting, first maximum in row-major
 * order, then back substitution with the last permuted column free), normalised; a plane with
 * every point on one side (tolerance tol) is a supporting plane, oriented outward, with b = the
 * largest n . p over the points; planes equal to a stored one (1e-9 on the normal, btol on b) are
 * dropped -- the rule of orc_hull3d_hrep in any dimension.  dim = 1: the rows +1 / -1 at the
 * largest / smallest coordinate.  Returns the row count, or -1 for fewer than dim + 1 points, a
 * set that spans less than dim dimensions, more than max_facets planes, or dim outside
 * [1, ORC_HULLND_MAX_DIM]. */
#define ORC_HULLND_MAX_DIM 8
static int64_t orc_binom(int a, int b)
{
    if (b < 0 || a < b) return 0;
    int64_t r = 1;
    for (int k = 1; k <= b; ++k) r = r * (a - b + k) / k;
    return r;
}

int orc_hullnd_hrep(int dim, const double* pts, int npts, int max_facets, double* A, double* b)
{
    for (int e = 0; e < dim * max_facets; ++e) A[e] = 0.0;
    for (int e = 0; e < max_facets; ++e) b[e] = 0.0;
    if (dim < 1 || dim > ORC_HULLND_MAX_DIM || npts < dim + 1) return -1;
    double scale = 0.0;
    for (int e = 0; e < dim * npts; ++e) {
        const double a = fabs(pts[e]);
        if (a > scale) scale = a;
    }
    const double tol = 1e-12 * (1.0 + scale);
    const double btol = 1e-9 * (1.0 + scale);
    if (dim == 1) {
        double mn = pts[0], mx = pts[0];
        for (int l = 1; l < npts; ++l) {
            if (pts[l] < mn) mn = pts[l];
            if (pts[l] > mx) mx = pts[l];
        }
        if (!(mx - mn > tol) || max_facets < 2) return -1;
        A[0] = 1.0, b[0] = mx, A[1] = -1.0, b[1] = -mn;
        return 2;
    }
    const int R = dim - 1;
    int idx[ORC_HULLND_MAX_DIM];
    for (int i = 0; i < dim; ++i) idx[i] = i;
    const int64_t total = orc_binom(npts, dim);
    int count = 0, overflow = 0;
    for (int64_t t = 0; t < total; ++t) {
        if (t > 0) {   /* next combination in lexicographic order */
            int i = dim - 1;
            while (idx[i] == npts - dim + i) --i;
            ++idx[i];
            for (int k = i + 1; k < dim; ++k) idx[k] = idx[k - 1] + 1;
        }
        const double* p0 = pts + (int64_t)idx[0] * dim;
        double W[ORC_HULLND_MAX_DIM - 1][ORC_HULLND_MAX_DIM];
        int perm[ORC_HULLND_MAX_DIM];
        for (int r = 0; r < R; ++r)
            for (int c = 0; c < dim; ++c) W[r][c] = pts[(int64_t)idx[r + 1] * dim + c] - p0[c];
        for (int c = 0; c < dim; ++c) perm[c] = c;
        int ok = 1;
        for (int k = 0; k < R && ok; ++k) {
            double best = -1.0;
            int pr = k, pc = k;
            for (int r = k; r < R; ++r)
                for (int c = k; c < dim; ++c) {
                    const double a = fabs(W[r][c]);
                    if (a > best) best = a, pr = r, pc = c;
                }
            if (!(best > tol)) { ok = 0; break; }
            for (int c = 0; c < dim; ++c) { const double x = W[k][c]; W[k][c] = W[pr][c]; W[pr][c] = x; }
            for (int r = 0; r < R; ++r) { const double x = W[r][k]; W[r][k] = W[r][pc]; W[r][pc] = x; }
            { const int x = perm[k]; perm[k] = perm[pc]; perm[pc] = x; }
            for (int r = k + 1; r < R; ++r) {
                const double f = W[r][k] / W[k][k];
                for (int c = k + 1; c < dim; ++c) W[r][c] = W[r][c] - f * W[k][c];
            }
        }
        if (!ok) continue;
        double x[ORC_HULLND_MAX_DIM], nrm[ORC_HULLND_MAX_DIM];
        x[dim - 1] = 1.0;
        for (int k = R - 1; k >= 0; --k) {
            double sum = W[k][dim - 1];
            for (int c = k + 1; c < R; ++c) sum = sum + W[k][c] * x[c];
            x[k] = -sum / W[k][k];
        }
        for (int c = 0; c < dim; ++c) nrm[perm[c]] = x[c];
        double len = nrm[0] * nrm[0];
        for (int c = 1; c < dim; ++c) len = len + nrm[c] * nrm[c];
        len = sqrt(len);
        if (!(len > 0.0)) continue;
        for (int c = 0; c < dim; ++c) nrm[c] = nrm[c] / len;
        int pos = 0, neg = 0;
        for (int l = 0; l < npts; ++l) {
            const double* q = pts + (int64_t)l * dim;
            double d = nrm[0] * (q[0] - p0[0]);
            for (int c = 1; c < dim; ++c) d = d + nrm[c] * (q[c] - p0[c]);
            if (d > tol) pos = 1;
            if (d < -tol) neg = 1;
        }
        if ((pos && neg) || !(pos || neg)) continue;
        if (pos)
            for (int c = 0; c < dim; ++c) nrm[c] = -nrm[c];
        double bm = -INFINITY;
        for (int l = 0; l < npts; ++l) {
            const double* q = pts + (int64_t)l * dim;
            double v = nrm[0] * q[0];
            for (int c = 1; c < dim; ++c) v = v + nrm[c] * q[c];
            if (v > bm) bm = v;
        }
        int dup = 0;
        for (int e = 0; e < count && e < max_facets && !dup; ++e) {
            int same = fabs(b[e] - bm) <= btol;
            for (int c = 0; c < dim; ++c) same = same && fabs(A[e * dim + c] - nrm[c]) <= 1e-9;
            dup = same;
        }
        if (dup) continue;
        if (count < max_facets) {
            for (int c = 0; c < dim; ++c) A[count * dim + c] = nrm[c];
            b[count] = bm;
        } else {
            overflow = 1;
        }
        ++count;
    }
    if (overflow || count < dim + 1) {
        for (int e = 0; e < dim * max_facets; ++e) A[e] = 0.0;
        for (int e = 0; e < max_facets; ++e) b[e] = 0.0;
        return -1;
    }
    return count;
}

/* doesPointBelongToConvexHull in any dimension (ConvexHullHelper.cpp:101-117): strict `>` rejects. */
int orc_halfspace_contains(const double* A, const double* b, int nfacets, int dim, const double* p)
{
    if (nfacets < 0) return 0;
    for (int i = 0; i < nfacets; ++i) {
        double v = 0.0;
        for (int c = 0; c < dim; ++c) v = v + A[i * dim + c] * p[c];
        if (v > b[i]) return 0;
    }
    return 1;
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

/* Knot -> contact-phase expansion of one problem (blf_dcm_phase_expand): knot k at
 * t = (start + k) dt belongs to p = the last phase with begin_p <= t (binary search, the
 * getPresentContact rule of Planners/src/ContactList.cpp:190-202) if t < end_p. */
static int phase_of(const double* begin, const double* end, int n, double t)
{
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (begin[mid] <= t) lo = mid + 1;
        else hi = mid;
    }
    const int p = lo - 1;
    return (p >= 0 && t < end[p]) ? p : -1;
}

void orc_dcm_phase_expand(int P, int M, int nphases, const double* begin, const double* end,
                          const double* pA, const double* pb, const int32_t* pnf,
                          const double* pref, int64_t start, double dt, int N, double* A,
                          double* b, int32_t* nfacets, double* xi_ref, double* vrp_ref)
{
    const int np = nphases < 0 ? 0 : (nphases > P ? P : nphases);
    for (int k = 0; k <= N; ++k) {
        const double t = (double)(start + k) * dt;
        const int p = phase_of(begin, end, np, t);
        const double r0 = p >= 0 ? pref[2 * p] : 0.0, r1 = p >= 0 ? pref[2 * p + 1] : 0.0;
        xi_ref[2 * k] = r0;
        xi_ref[2 * k + 1] = r1;
        if (k == N) break;
        vrp_ref[2 * k] = r0;
        vrp_ref[2 * k + 1] = r1;
        nfacets[k] = p >= 0 ? pnf[p] : -1;
        for (int i = 0; i < M; ++i) {
            A[(k * M + i) * 2] = p >= 0 ? pA[(p * M + i) * 2] : 0.0;
            A[(k * M + i) * 2 + 1] = p >= 0 ? pA[(p * M + i) * 2 + 1] : 0.0;
            b[k * M + i] = p >= 0 ? pb[p * M + i] : 0.0;
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
        for (int off = 1; off <= 32; off <<= 1) {      /* the device's DPP / permlane order */
            for (int l = 0; l < 64; ++l) t[l] = v[l] + v[l ^ off];
            memcpy(v, t, sizeof(v));
        }
        total = (w == 0) ? v[0] : total + v[0];
    }
    return total;
}

#define MF 16   /* facet slots (max_facets <= 16) */
#ifndef ORC_GUESS_PASSES
#define ORC_GUESS_PASSES 8    /* active-set start: drop/add passes (kernel: kGuessPasses) */
#endif
#define ORC_TOL_DUAL_REL 1e-3   /* the certificate's relative dual tolerance (kernel kTolDualRel) */
#define ORC_LAM_REL 1e-8        /* the IPM polish's guess: lam_i >= this x the knot's largest (kernel kLamRel) */
#define ORC_LAM_REL_CROSS 0.3   /* ... among facets this close to parallel to the largest one's (kernel kLamRelCross) */
#define ORC_ADD_REL 1e-2        /* the IPM polish adds facets violated by >= this x the largest (kernel kAddRel) */
#define ORC_GUESS_SLACK 1e-5  /* the fp64 passes' guess after the fp32 search (kernel: kGuessSlack) */
/* round 6: the IPM polish also runs after a stalled step (a < ORC_STALL_STEP) once mu <= ORC_STALL_MU
 * (kernel kStallStep / kStallMu), and a certified optimum whose largest multiplier exceeds
 * ORC_REFINE_LAM takes one refinement step with double-double residuals (kernel kRefineLam) */
#define ORC_STALL_STEP 0.2
#define ORC_STALL_MU 1.0
#define ORC_REFINE_LAM 1e4
#define ORC_REFINE_STEPS 2   /* refinement steps (kernel kRefineSteps) */
/* round 6: the active-set kernels' fp64 passes (the cold kernel's phase B and the warm kernel) run
 * up to ORC_AS_PASSES drop/add passes under the anti-cycling rule of dcm_polish (kernel kAsPasses) */
#define ORC_AS_PASSES 12
#define WV 64

/* Fused forms, used in exactly the places the kernel uses them (csrc/dcm_mpc_ipm.hip):
 *   FD2(a, b, c, d) = a b + c d as fma(a, b, c d);  FD3(a, b, c, d, e) = fma(a, b, fma(c, d, e)).
 * C fma() is correctly rounded like v_fma_f64, so oracle and kernel stay bit-identical. */
#define FD2(a, b, c, d) fma((a), (b), (c) * (d))
#define FD3(a, b, c, d, e) fma((a), (b), fma((c), (d), (e)))

/* Working state of one QP solve.  Per-knot arrays are indexed by the knot k = 64 w + lane: the
 * device runs one thread per knot, NW = ceil(N / 64) wavefronts per QP. */
typedef struct {
    int N, M, NW, ntot;
    int scans;                             /* 1: device-order Kogge-Stone scans, 0: sequential */
    int pairs;                             /* 1: the active-set kernel's pair tree (64 < N <= 128) */
    int dpp;                               /* 1: the active-set kernels' DPP tree (N <= 128) */
    double dt, Qw0, Qw1, Rw0, Rw1, Pw0, Pw1;
    const double *omega, *xi_ref, *vrp_ref, *A, *b;
    const int32_t* nf;
    double *al, *be, *a2, *b2, *ab;        /* [N] */
    double *s, *lam, *is, *cds, *cdl;      /* [N][MF] slacks, multipliers, 1/s, step */
    double *W;                             /* [N][4] A^T diag(lam/s) A (3), its determinant (1) */
    double *E, *Pn, *h;                    /* [N][3] */
    double *G, *Mm;                        /* [N][4]: G_k, M_k = P_{k+1} h_k */
    double *rh, *g, *d, *qx, *dr, *dra;    /* [N][2] */
    double *c, *q;                         /* [N] reduction partials */
    double *sc, *sg;                       /* [N][2], [N][4] scan elements */
    double *v, *x;                         /* [N+1][2] scan results */
    double *xi, *vrp;                      /* outputs, updated in place */
    int npass;   /* dcm_polish passes run since the solve began */
} dcm_ws;

static double keepmax(double q, double x) { return x > q ? x : q; }
static double nanmax(double q, double x) { return (x > q || x != x) ? x : q; }

/* ---- the active-set kernel's scan tree (csrc/dcm_mpc_as.hip, 64 < N <= 128): lane l of ONE
 * wavefront owns the knot pair (2l, 2l + 1); the pair's element is composed in the lane, a
 * Kogge-Stone scan runs over the 64 lanes, and the pair's inner knot is applied in the lane.
 * Knots >= N carry the zero element (affine scans) or the identity (Riccati), as in the wavefront
 * tree above. ---- */

/* 2x2 affine compose: (a, e) <- (a b, a c + e), the COMPOSE of the device */
static void aff_compose(double* a, double* e, const double* b, const double* c)
{
    const double n0 = FD2(a[0], b[0], a[1], b[2]);
    const double n1 = FD2(a[0], b[1], a[1], b[3]);
    const double n2 = FD2(a[2], b[0], a[3], b[2]);
    const double n3 = FD2(a[2], b[1], a[3], b[3]);
    const double m0 = FD3(a[0], c[0], a[1], c[1], e[0]);
    const double m1 = FD3(a[2], c[0], a[3], c[1], e[1]);
    a[0] = n0; a[1] = n1; a[2] = n2; a[3] = n3; e[0] = m0; e[1] = m1;
}

static void scan_backward_pairs(dcm_ws* w, const double* G, const double* c)
{
    const int N = w->N;
    double g[WV][4], e[WV][2], ng[WV][4], ne[WV][2];
    for (int l = 0; l < WV; ++l) {
        const int k0 = 2 * l, k1 = 2 * l + 1;
        for (int j = 0; j < 4; ++j) g[l][j] = k0 < N ? G[4 * k0 + j] : 0.0;
        for (int j = 0; j < 2; ++j) e[l][j] = k0 < N ? c[2 * k0 + j] : 0.0;
        double b[4], cc[2];
        for (int j = 0; j < 4; ++j) b[j] = k1 < N ? G[4 * k1 + j] : 0.0;
        for (int j = 0; j < 2; ++j) cc[j] = k1 < N ? c[2 * k1 + j] : 0.0;
        aff_compose(g[l], e[l], b, cc);            /* knot 2l after knot 2l + 1 */
    }
    const int pad = N <= 2 * WV - 2;   /* lane WV - 1 holds no knot: its zero element (kernel as_pad) */
    for (int dd = 1; dd < WV; dd <<= 1) {
        for (int l = 0; l < WV; ++l) {
            memcpy(ng[l], g[l], sizeof(ng[l]));
            memcpy(ne[l], e[l], sizeof(ne[l]));
            if (l + dd < WV) aff_compose(ng[l], ne[l], g[l + dd], e[l + dd]);
            else if (pad) aff_compose(ng[l], ne[l], g[WV - 1], e[WV - 1]);
        }
        memcpy(g, ng, sizeof(g));
        memcpy(e, ne, sizeof(e));
    }
    for (int l = 0; l < WV; ++l) {               /* v_{2l} = e_l; v_{2l+1} = G v_{2l+2} + c */
        const int k0 = 2 * l, k1 = 2 * l + 1;
        if (k0 < N) { w->v[2 * k0] = e[l][0]; w->v[2 * k0 + 1] = e[l][1]; }
        if (k1 < N) {
            const double vb0 = l + 1 < WV ? e[l + 1][0] : 0.0, vb1 = l + 1 < WV ? e[l + 1][1] : 0.0;
            const double* Gk = G + 4 * k1;
            w->v[2 * k1] = FD3(Gk[0], vb0, Gk[1], vb1, c[2 * k1]);
            w->v[2 * k1 + 1] = FD3(Gk[2], vb0, Gk[3], vb1, c[2 * k1 + 1]);
        }
    }
}

static void scan_forward_pairs(dcm_ws* w, const double* F, int transpose, const double* f)
{
    const int N = w->N;
    double g[WV][4], e[WV][2], ng[WV][4], ne[WV][2];
    double F0[WV][4], f0[WV][2];
    for (int l = 0; l < WV; ++l) {
        const int ks[2] = {2 * l, 2 * l + 1};
        double Fk[2][4], fk[2][2];
        for (int q = 0; q < 2; ++q) {
            const int k = ks[q];
            if (k < N) {
                const double* Fp = F + 4 * k;
                Fk[q][0] = Fp[0];
                Fk[q][1] = transpose ? Fp[2] : Fp[1];
                Fk[q][2] = transpose ? Fp[1] : Fp[2];
                Fk[q][3] = Fp[3];
                fk[q][0] = f[2 * k];
                fk[q][1] = f[2 * k + 1];
            } else {
                Fk[q][0] = Fk[q][1] = Fk[q][2] = Fk[q][3] = 0.0;
                fk[q][0] = fk[q][1] = 0.0;
            }
        }
        memcpy(F0[l], Fk[0], sizeof(F0[l]));
        memcpy(f0[l], fk[0], sizeof(f0[l]));
        memcpy(g[l], Fk[1], sizeof(g[l]));
        memcpy(e[l], fk[1], sizeof(e[l]));
        aff_compose(g[l], e[l], Fk[0], fk[0]);     /* knot 2l + 1 after knot 2l */
    }
    const int pad = N <= 2 * WV - 2;   /* lanes before their partner take lane WV - 1's zero element */
    for (int dd = 1; dd < WV; dd <<= 1) {
        for (int l = 0; l < WV; ++l) {
            memcpy(ng[l], g[l], sizeof(ng[l]));
            memcpy(ne[l], e[l], sizeof(ne[l]));
            if (l - dd >= 0) aff_compose(ng[l], ne[l], g[l - dd], e[l - dd]);
            else if (pad) aff_compose(ng[l], ne[l], g[WV - 1], e[WV - 1]);
        }
        memcpy(g, ng, sizeof(g));
        memcpy(e, ne, sizeof(e));
    }
    for (int l = 0; l < WV; ++l) {               /* x_{2l+2} = e_l; x_{2l+1} = F x_{2l} + f */
        const int k0 = 2 * l, k1 = 2 * l + 1;
        const double xb0 = l > 0 ? e[l - 1][0] : 0.0, xb1 = l > 0 ? e[l - 1][1] : 0.0;
        if (k0 < N) {
            w->x[2 * (k0 + 1)] = FD3(F0[l][0], xb0, F0[l][1], xb1, f0[l][0]);
            w->x[2 * (k0 + 1) + 1] = FD3(F0[l][2], xb0, F0[l][3], xb1, f0[l][1]);
        }
        if (k1 < N) {
            w->x[2 * (k1 + 1)] = e[l][0];
            w->x[2 * (k1 + 1) + 1] = e[l][1];
        }
    }
}

/* ---- the active-set kernels' DPP tree (csrc/dcm_qp_common.h tree_fwd / tree_bwd; batches of at
 * most BLF_DPP_TREE_MAX_BATCH QPs, orc_dcm_params.as_tree = 1): lane l of ONE wavefront owns KPL
 * knots (knot l for N <= 64, the pair 2l, 2l + 1 for 64 < N <= 128); a pair's element is composed
 * in the lane, the 64 lane elements are scanned Kogge-Stone inside each row of 16 lanes, then in
 * two row-level steps (orc_lane_src), and a pair's inner knot is applied in the lane. ---- */
int orc_lane_src(int L, int fwd, int l)
{
    const int r = l >> 4, d = 1 << L;
    if (fwd) {
        if (L < 4) return (l & 15) >= d ? l - d : -1;   /* row_shr:d */
        if (L == 4) return (r & 1) ? 16 * r - 1 : -1;    /* row_bcast:15, rows 1 and 3 */
        return r >= 2 ? 31 : -1;                         /* row_bcast:31, rows 2 and 3 */
    }
    if (L < 4) return (l & 15) + d <= 15 ? l + d : -1;   /* row_shl:d */
    if (L == 4) return (r & 1) ? -1 : 16 * r + 16;       /* row_newbcast:0 + permlane16_swap */
    return r < 2 ? 32 : -1;                              /* v_readlane 32, rows 0 and 1 */
}

#define AS_LEVELS 6

/* the DPP tree over the 64 lane elements (g, e): a lane combines with its level's source lane's
 * element when it has one (orc_lane_src >= 0), and keeps its element otherwise */
static void aff_tree(double (*g)[4], double (*e)[2], int fwd)
{
    double ng[WV][4], ne[WV][2];
    for (int L = 0; L < AS_LEVELS; ++L) {
        for (int l = 0; l < WV; ++l) {
            const int s = orc_lane_src(L, fwd, l);
            memcpy(ng[l], g[l], sizeof(ng[l]));
            memcpy(ne[l], e[l], sizeof(ne[l]));
            if (s >= 0) aff_compose(ng[l], ne[l], g[s], e[s]);
        }
        memcpy(g, ng, sizeof(ng));
        memcpy(e, ne, sizeof(ne));
    }
}

static void scan_backward_dpp(dcm_ws* w, const double* G, const double* c)
{
    const int N = w->N, KPL = N > WV ? 2 : 1;
    double g[WV][4], e[WV][2];
    for (int l = 0; l < WV; ++l) {
        const int k0 = KPL * l, k1 = KPL * l + 1;
        for (int j = 0; j < 4; ++j) g[l][j] = k0 < N ? G[4 * k0 + j] : 0.0;
        for (int j = 0; j < 2; ++j) e[l][j] = k0 < N ? c[2 * k0 + j] : 0.0;
        if (KPL == 2) {
            double b[4], cc[2];
            for (int j = 0; j < 4; ++j) b[j] = k1 < N ? G[4 * k1 + j] : 0.0;
            for (int j = 0; j < 2; ++j) cc[j] = k1 < N ? c[2 * k1 + j] : 0.0;
            aff_compose(g[l], e[l], b, cc);            /* knot 2l after knot 2l + 1 */
        }
    }
    aff_tree(g, e, 0);
    for (int l = 0; l < WV; ++l) {               /* v_{KPL l} = e_l; v_{2l+1} = G v_{2l+2} + c */
        const int k0 = KPL * l, k1 = KPL * l + 1;
        if (k0 < N) { w->v[2 * k0] = e[l][0]; w->v[2 * k0 + 1] = e[l][1]; }
        if (KPL == 2 && k1 < N) {
            const double vb0 = l + 1 < WV ? e[l + 1][0] : 0.0, vb1 = l + 1 < WV ? e[l + 1][1] : 0.0;
            const double* Gk = G + 4 * k1;
            w->v[2 * k1] = FD3(Gk[0], vb0, Gk[1], vb1, c[2 * k1]);
            w->v[2 * k1 + 1] = FD3(Gk[2], vb0, Gk[3], vb1, c[2 * k1 + 1]);
        }
    }
}

static void scan_forward_dpp(dcm_ws* w, const double* F, int transpose, const double* f)
{
    const int N = w->N, KPL = N > WV ? 2 : 1;
    double g[WV][4], e[WV][2];
    double F0[WV][4], f0[WV][2];
    for (int l = 0; l < WV; ++l) {
        double Fk[2][4], fk[2][2];
        for (int q = 0; q < KPL; ++q) {
            const int k = KPL * l + q;
            if (k < N) {
                const double* Fp = F + 4 * k;
                Fk[q][0] = Fp[0];
                Fk[q][1] = transpose ? Fp[2] : Fp[1];
                Fk[q][2] = transpose ? Fp[1] : Fp[2];
                Fk[q][3] = Fp[3];
                fk[q][0] = f[2 * k];
                fk[q][1] = f[2 * k + 1];
            } else {
                Fk[q][0] = Fk[q][1] = Fk[q][2] = Fk[q][3] = 0.0;
                fk[q][0] = fk[q][1] = 0.0;
            }
        }
        memcpy(F0[l], Fk[0], sizeof(F0[l]));
        memcpy(f0[l], fk[0], sizeof(f0[l]));
        memcpy(g[l], Fk[KPL - 1], sizeof(g[l]));
        memcpy(e[l], fk[KPL - 1], sizeof(e[l]));
        if (KPL == 2) aff_compose(g[l], e[l], Fk[0], fk[0]);   /* knot 2l + 1 after knot 2l */
    }
    aff_tree(g, e, 1);
    for (int l = 0; l < WV; ++l) {               /* x past the lane's last knot = e_l */
        const int k0 = KPL * l, kl = KPL * l + KPL - 1;
        if (KPL == 2 && k0 < N) {                /* x_{2l+1} = F x_{2l} + f */
            const double xb0 = l > 0 ? e[l - 1][0] : 0.0, xb1 = l > 0 ? e[l - 1][1] : 0.0;
            w->x[2 * (k0 + 1)] = FD3(F0[l][0], xb0, F0[l][1], xb1, f0[l][0]);
            w->x[2 * (k0 + 1) + 1] = FD3(F0[l][2], xb0, F0[l][3], xb1, f0[l][1]);
        }
        if (kl < N) {
            w->x[2 * (kl + 1)] = e[l][0];
            w->x[2 * (kl + 1) + 1] = e[l][1];
        }
    }
}

/* Backward affine recursion v_k = G_k v_{k+1} + c_k (v_N = 0) the way the device evaluates it:
 * a Kogge-Stone scan over the 64 lanes of each wavefront (lane l combines with lane l + d from
 * the previous level, d = 1, 2, ..., 32; lanes past the last knot hold the zero element), then
 * the wavefronts from last to first apply the first knot's value of the next wavefront.
 * Result: w->v[k] = v_k for k < N, w->v[N] = 0. */
static void scan_backward(dcm_ws* w, const double* G, const double* c)
{
    const int N = w->N;
    w->v[2 * N] = 0.0;
    w->v[2 * N + 1] = 0.0;
    if (!w->scans) {   /* CPU-efficient sequential recursion (cpu_baseline timing only) */
        for (int k = N - 1; k >= 0; --k) {
            const double* g = G + 4 * k;
            const double vn0 = w->v[2 * (k + 1)], vn1 = w->v[2 * (k + 1) + 1];
            w->v[2 * k] = FD3(g[0], vn0, g[1], vn1, c[2 * k]);
            w->v[2 * k + 1] = FD3(g[2], vn0, g[3], vn1, c[2 * k + 1]);
        }
        return;
    }
    if (w->dpp) { scan_backward_dpp(w, G, c); return; }
    if (w->pairs) { scan_backward_pairs(w, G, c); return; }
    for (int wv = w->NW - 1; wv >= 0; --wv) {
        double g[WV][4], e[WV][2], ng[WV][4], ne[WV][2];
        for (int l = 0; l < WV; ++l) {
            const int k = WV * wv + l;
            for (int j = 0; j < 4; ++j) g[l][j] = k < N ? G[4 * k + j] : 0.0;
            for (int j = 0; j < 2; ++j) e[l][j] = k < N ? c[2 * k + j] : 0.0;
        }
        for (int dd = 1; dd < WV; dd <<= 1) {
            for (int l = 0; l < WV; ++l) {
                if (l + dd < WV) {
                    const double* a = g[l];
                    const double* bq = g[l + dd];
                    const double* ce = e[l + dd];
                    ng[l][0] = FD2(a[0], bq[0], a[1], bq[2]);
                    ng[l][1] = FD2(a[0], bq[1], a[1], bq[3]);
                    ng[l][2] = FD2(a[2], bq[0], a[3], bq[2]);
                    ng[l][3] = FD2(a[2], bq[1], a[3], bq[3]);
                    ne[l][0] = FD3(a[0], ce[0], a[1], ce[1], e[l][0]);
                    ne[l][1] = FD3(a[2], ce[0], a[3], ce[1], e[l][1]);
                } else {
                    memcpy(ng[l], g[l], sizeof(ng[l]));
                    memcpy(ne[l], e[l], sizeof(ne[l]));
                }
            }
            memcpy(g, ng, sizeof(g));
            memcpy(e, ne, sizeof(e));
        }
        for (int l = 0; l < WV; ++l) {
            const int k = WV * wv + l;
            if (k >= N) break;
            if (wv == w->NW - 1) {
                w->v[2 * k] = e[l][0];
                w->v[2 * k + 1] = e[l][1];
            } else {
                const double vn0 = w->v[2 * WV * (wv + 1)], vn1 = w->v[2 * WV * (wv + 1) + 1];
                w->v[2 * k] = FD3(g[l][0], vn0, g[l][1], vn1, e[l][0]);
                w->v[2 * k + 1] = FD3(g[l][2], vn0, g[l][3], vn1, e[l][1]);
            }
        }
    }
}

/* Forward affine recursion x_{k+1} = F_k x_k + f_k (x_0 = 0): Kogge-Stone per wavefront (lane l
 * combines with lane l - d), then the wavefronts from first to last apply the last value of the
 * previous wavefront.  F is given as [N][4] row-major; `transpose` uses F_k = G_k^T.
 * Result: w->x[k + 1] for k < N, w->x[0] = 0. */
static void scan_forward(dcm_ws* w, const double* F, int transpose, const double* f)
{
    const int N = w->N;
    w->x[0] = 0.0;
    w->x[1] = 0.0;
    if (!w->scans) {   /* CPU-efficient sequential recursion (cpu_baseline timing only) */
        for (int k = 0; k < N; ++k) {
            const double* F_ = F + 4 * k;
            const double f01 = transpose ? F_[2] : F_[1], f10 = transpose ? F_[1] : F_[2];
            const double x0 = w->x[2 * k], x1 = w->x[2 * k + 1];
            w->x[2 * (k + 1)] = FD3(F_[0], x0, f01, x1, f[2 * k]);
            w->x[2 * (k + 1) + 1] = FD3(f10, x0, F_[3], x1, f[2 * k + 1]);
        }
        return;
    }
    if (w->dpp) { scan_forward_dpp(w, F, transpose, f); return; }
    if (w->pairs) { scan_forward_pairs(w, F, transpose, f); return; }
    for (int wv = 0; wv < w->NW; ++wv) {
        double g[WV][4], e[WV][2], ng[WV][4], ne[WV][2];
        for (int l = 0; l < WV; ++l) {
            const int k = WV * wv + l;
            if (k < N) {
                const double* Fk = F + 4 * k;
                g[l][0] = Fk[0];
                g[l][1] = transpose ? Fk[2] : Fk[1];
                g[l][2] = transpose ? Fk[1] : Fk[2];
                g[l][3] = Fk[3];
                e[l][0] = f[2 * k];
                e[l][1] = f[2 * k + 1];
            } else {
                g[l][0] = g[l][1] = g[l][2] = g[l][3] = 0.0;
                e[l][0] = e[l][1] = 0.0;
            }
        }
        for (int dd = 1; dd < WV; dd <<= 1) {
            for (int l = 0; l < WV; ++l) {
                if (l - dd >= 0) {
                    const double* a = g[l];
                    const double* bq = g[l - dd];
                    const double* ce = e[l - dd];
                    ng[l][0] = FD2(a[0], bq[0], a[1], bq[2]);
                    ng[l][1] = FD2(a[0], bq[1], a[1], bq[3]);
                    ng[l][2] = FD2(a[2], bq[0], a[3], bq[2]);
                    ng[l][3] = FD2(a[2], bq[1], a[3], bq[3]);
                    ne[l][0] = FD3(a[0], ce[0], a[1], ce[1], e[l][0]);
                    ne[l][1] = FD3(a[2], ce[0], a[3], ce[1], e[l][1]);
                } else {
                    memcpy(ng[l], g[l], sizeof(ng[l]));
                    memcpy(ne[l], e[l], sizeof(ne[l]));
                }
            }
            memcpy(g, ng, sizeof(g));
            memcpy(e, ne, sizeof(e));
        }
        for (int l = 0; l < WV; ++l) {
            const int k = WV * wv + l;
            if (k >= N) break;
            if (wv == 0) {
                w->x[2 * (k + 1)] = e[l][0];
                w->x[2 * (k + 1) + 1] = e[l][1];
            } else {
                const double x0 = w->x[2 * WV * wv], x1 = w->x[2 * WV * wv + 1];
                w->x[2 * (k + 1)] = FD3(g[l][0], x0, g[l][1], x1, e[l][0]);
                w->x[2 * (k + 1) + 1] = FD3(g[l][2], x0, g[l][3], x1, e[l][1]);
            }
        }
    }
}

/* Stage-parallel residual pass (one device thread per knot): rp = A r + s - b is recomputed
 * where needed; here complementarity partials c_k, rh = R (r - r_ref) + A^T lam, the Euler
 * defects d_k (reference step order, ForwardEuler.tpp:37-45 over LinearTimeInvariantSystem.cpp:71)
 * and qx_k = Q (xi_{k+1} - xi_ref_{k+1}) (knot N-1: the terminal gradient P (xi_N - xi_ref_N)).
 * use_facets = 0: no facets (the warm start).  Returns max |rp|, |d| (NaN-propagating). */
static double dcm_residuals(dcm_ws* w, int use_facets)
{
    const int N = w->N, M = w->M;
    double pres = 0.0;
    for (int k = 0; k < N; ++k) {
        const int m = use_facets ? w->nf[k] : 0;
        const double r0 = w->vrp[2 * k], r1 = w->vrp[2 * k + 1];
        double ck = 0.0;
        double rh0 = w->Rw0 * (r0 - w->vrp_ref[2 * k]);
        double rh1 = w->Rw1 * (r1 - w->vrp_ref[2 * k + 1]);
        for (int i = 0; i < m; ++i) {
            const double* a = w->A + (k * M + i) * 2;
            const double si = w->s[k * MF + i], li = w->lam[k * MF + i];
            const double gr = FD2(a[0], r0, a[1], r1);
            const double rpi = (gr + si) - w->b[k * M + i];
            pres = nanmax(pres, fabs(rpi));
            ck = fma(si, li, ck);
            rh0 = fma(a[0], li, rh0);
            rh1 = fma(a[1], li, rh1);
        }
        w->c[k] = ck;
        w->rh[2 * k] = rh0;
        w->rh[2 * k + 1] = rh1;
        const double om = w->omega[k];
        {
            const double x0 = w->xi[2 * k], x1 = w->xi[2 * k + 1];
            const double y0 = w->xi[2 * (k + 1)], y1 = w->xi[2 * (k + 1) + 1];
            const double dx0 = FD2(om, x0, -om, r0);
            const double dk0 = fma(dx0, w->dt, x0) - y0;
            const double dx1 = FD2(om, x1, -om, r1);
            const double dk1 = fma(dx1, w->dt, x1) - y1;
            w->d[2 * k] = dk0;
            w->d[2 * k + 1] = dk1;
            pres = nanmax(pres, fabs(dk0));
            pres = nanmax(pres, fabs(dk1));
            if (k + 1 < N) {
                w->qx[2 * k] = w->Qw0 * (y0 - w->xi_ref[2 * (k + 1)]);
                w->qx[2 * k + 1] = w->Qw1 * (y1 - w->xi_ref[2 * (k + 1) + 1]);
            } else {
                w->qx[2 * k] = w->Pw0 * (y0 - w->xi_ref[2 * (k + 1)]);
                w->qx[2 * k + 1] = w->Pw1 * (y1 - w->xi_ref[2 * (k + 1) + 1]);
            }
        }
    }
    return pres;
}

/* Riccati map element f(P) = H + A^T P (I + G P)^{-1} A (A 2x2 row-major, G and H symmetric).
 * Knot k: A = alpha_k I, G = E_k = beta_k^2 (R + W_k)^{-1}, H = Q, so P_k = f_k(P_{k+1}).
 * rc_combine(e1, e2) = e1 o e2 (e1 the earlier knot):
 *   T = I + G1 H2,  U = T^{-1} A1,  A = A2 U,  G = (A2 T^{-1}) G1 A2^T + G2,  H = U^T (H2 A1) + H1
 * (the structure-preserving doubling composition: only (I + G H)^{-1}, eigenvalues >= 1). */
typedef struct { double a[4], g[3], h[3]; } rc_el;

/* the kernel's BLF_RC_FORM (dcm_qp_common.h): where 1 / det(I + G H) enters the products */
#ifndef ORC_RC_FORM
#define ORC_RC_FORM 2
#endif

static int rc_combine(rc_el* e1, const rc_el* e2)
{
    const double* A1 = e1->a; const double* G1 = e1->g; const double* H1 = e1->h;
    const double* A2 = e2->a; const double* G2 = e2->g; const double* H2 = e2->h;
    const double T00 = FD3(G1[0], H2[0], G1[1], H2[1], 1.0);
    const double T01 = FD2(G1[0], H2[1], G1[1], H2[2]);
    const double T10 = FD2(G1[1], H2[0], G1[2], H2[1]);
    const double T11 = FD3(G1[1], H2[1], G1[2], H2[2], 1.0);
    const double detT = fma(T00, T11, -(T01 * T10));
    const int ok = (detT > 0.0) && !isinf(detT);
    const double it = 1.0 / detT;
#if ORC_RC_FORM >= 2
    {
        /* adj(T) = [T11, -T01; -T10, T00]: the products run beside the division (rc_combine of
         * dcm_qp_common.h, BLF_RC_FORM) */
        const double Up00 = FD2(T11, A1[0], -T01, A1[2]);
        const double Up01 = FD2(T11, A1[1], -T01, A1[3]);
        const double Up10 = FD2(-T10, A1[0], T00, A1[2]);
        const double Up11 = FD2(-T10, A1[1], T00, A1[3]);
        const double Vp00 = FD2(A2[0], T11, A2[1], -T10);
        const double Vp01 = FD2(A2[0], -T01, A2[1], T00);
        const double Vp10 = FD2(A2[2], T11, A2[3], -T10);
        const double Vp11 = FD2(A2[2], -T01, A2[3], T00);
        const double Xp00 = FD2(Vp00, G1[0], Vp01, G1[1]);
        const double Xp01 = FD2(Vp00, G1[1], Vp01, G1[2]);
        const double Xp10 = FD2(Vp10, G1[0], Vp11, G1[1]);
        const double Xp11 = FD2(Vp10, G1[1], Vp11, G1[2]);
        const double Y00 = FD2(H2[0], A1[0], H2[1], A1[2]);
        const double Y01 = FD2(H2[0], A1[1], H2[1], A1[3]);
        const double Y10 = FD2(H2[1], A1[0], H2[2], A1[2]);
        const double Y11 = FD2(H2[1], A1[1], H2[2], A1[3]);
        const double gp0 = FD2(Xp00, A2[0], Xp01, A2[1]);
        const double gp1 = FD2(Xp00, A2[2], Xp01, A2[3]);
        const double gp2 = FD2(Xp10, A2[2], Xp11, A2[3]);
        rc_el r;
#if ORC_RC_FORM == 2
        const double U00 = Up00 * it, U01 = Up01 * it, U10 = Up10 * it, U11 = Up11 * it;
        r.a[0] = FD2(A2[0], U00, A2[1], U10);
        r.a[1] = FD2(A2[0], U01, A2[1], U11);
        r.a[2] = FD2(A2[2], U00, A2[3], U10);
        r.a[3] = FD2(A2[2], U01, A2[3], U11);
        r.h[0] = FD3(U00, Y00, U10, Y10, H1[0]);
        r.h[1] = FD3(U00, Y01, U10, Y11, H1[1]);
        r.h[2] = FD3(U01, Y01, U11, Y11, H1[2]);
#else
        r.a[0] = FD2(A2[0], Up00, A2[1], Up10) * it;
        r.a[1] = FD2(A2[0], Up01, A2[1], Up11) * it;
        r.a[2] = FD2(A2[2], Up00, A2[3], Up10) * it;
        r.a[3] = FD2(A2[2], Up01, A2[3], Up11) * it;
        r.h[0] = fma(FD2(Up00, Y00, Up10, Y10), it, H1[0]);
        r.h[1] = fma(FD2(Up00, Y01, Up10, Y11), it, H1[1]);
        r.h[2] = fma(FD2(Up01, Y01, Up11, Y11), it, H1[2]);
#endif
        r.g[0] = fma(gp0, it, G2[0]);
        r.g[1] = fma(gp1, it, G2[1]);
        r.g[2] = fma(gp2, it, G2[2]);
        *e1 = r;
        return ok;
    }
#endif
    const double Ti00 = T11 * it, Ti01 = -(T01 * it), Ti10 = -(T10 * it), Ti11 = T00 * it;
    const double U00 = FD2(Ti00, A1[0], Ti01, A1[2]);
    const double U01 = FD2(Ti00, A1[1], Ti01, A1[3]);
    const double U10 = FD2(Ti10, A1[0], Ti11, A1[2]);
    const double U11 = FD2(Ti10, A1[1], Ti11, A1[3]);
    const double V00 = FD2(A2[0], Ti00, A2[1], Ti10);
    const double V01 = FD2(A2[0], Ti01, A2[1], Ti11);
    const double V10 = FD2(A2[2], Ti00, A2[3], Ti10);
    const double V11 = FD2(A2[2], Ti01, A2[3], Ti11);
    const double X00 = FD2(V00, G1[0], V01, G1[1]);
    const double X01 = FD2(V00, G1[1], V01, G1[2]);
    const double X10 = FD2(V10, G1[0], V11, G1[1]);
    const double X11 = FD2(V10, G1[1], V11, G1[2]);
    const double Y00 = FD2(H2[0], A1[0], H2[1], A1[2]);
    const double Y01 = FD2(H2[0], A1[1], H2[1], A1[3]);
    const double Y10 = FD2(H2[1], A1[0], H2[2], A1[2]);
    const double Y11 = FD2(H2[1], A1[1], H2[2], A1[3]);
    rc_el r;
    r.a[0] = FD2(A2[0], U00, A2[1], U10);
    r.a[1] = FD2(A2[0], U01, A2[1], U11);
    r.a[2] = FD2(A2[2], U00, A2[3], U10);
    r.a[3] = FD2(A2[2], U01, A2[3], U11);
    r.g[0] = FD3(X00, A2[0], X01, A2[1], G2[0]);
    r.g[1] = FD3(X00, A2[2], X01, A2[3], G2[1]);
    r.g[2] = FD3(X10, A2[2], X11, A2[3], G2[2]);
    r.h[0] = FD3(U00, Y00, U10, Y10, H1[0]);
    r.h[1] = FD3(U00, Y01, U10, Y11, H1[1]);
    r.h[2] = FD3(U01, Y01, U11, Y11, H1[2]);
    *e1 = r;
    return ok;
}

/* P_out = f(e, P) */
static int rc_apply(const rc_el* e, double P00, double P01, double P11, double* out)
{
    const double* A = e->a; const double* G = e->g; const double* H = e->h;
    const double S00 = FD3(G[0], P00, G[1], P01, 1.0);
    const double S01 = FD2(G[0], P01, G[1], P11);
    const double S10 = FD2(G[1], P00, G[2], P01);
    const double S11 = FD3(G[1], P01, G[2], P11, 1.0);
    const double detS = fma(S00, S11, -(S01 * S10));
    const int ok = (detS > 0.0) && !isinf(detS);
    const double is = 1.0 / detS;
#if ORC_RC_FORM >= 1
    {
        /* W' = P adj(S), Z' = W' A, out = (A^T Z') / det(S) + H (rc_apply, BLF_RC_FORM) */
        const double Wp00 = FD2(P00, S11, P01, -S10);
        const double Wp01 = FD2(P00, -S01, P01, S00);
        const double Wp10 = FD2(P01, S11, P11, -S10);
        const double Wp11 = FD2(P01, -S01, P11, S00);
        const double Zp00 = FD2(Wp00, A[0], Wp01, A[2]);
        const double Zp01 = FD2(Wp00, A[1], Wp01, A[3]);
        const double Zp10 = FD2(Wp10, A[0], Wp11, A[2]);
        const double Zp11 = FD2(Wp10, A[1], Wp11, A[3]);
        out[0] = fma(FD2(A[0], Zp00, A[2], Zp10), is, H[0]);
        out[1] = fma(FD2(A[0], Zp01, A[2], Zp11), is, H[1]);
        out[2] = fma(FD2(A[1], Zp01, A[3], Zp11), is, H[2]);
        return ok;
    }
#endif
    const double Si00 = S11 * is, Si01 = -(S01 * is), Si10 = -(S10 * is), Si11 = S00 * is;
    const double W00 = FD2(P00, Si00, P01, Si10);
    const double W01 = FD2(P00, Si01, P01, Si11);
    const double W10 = FD2(P01, Si00, P11, Si10);
    const double W11 = FD2(P01, Si01, P11, Si11);
    const double Z00 = FD2(W00, A[0], W01, A[2]);
    const double Z01 = FD2(W00, A[1], W01, A[3]);
    const double Z10 = FD2(W10, A[0], W11, A[2]);
    const double Z11 = FD2(W10, A[1], W11, A[3]);
    out[0] = FD3(A[0], Z00, A[2], Z10, H[0]);
    out[1] = FD3(A[0], Z01, A[2], Z11, H[1]);
    out[2] = FD3(A[1], Z01, A[3], Z11, H[2]);
    return ok;
}

/* The Riccati map element of knot k (identity for k >= N). */
static void rc_knot(const dcm_ws* w, int k, rc_el* e)
{
    if (k < w->N) {
        e->a[0] = w->al[k]; e->a[1] = 0.0; e->a[2] = 0.0; e->a[3] = w->al[k];
        e->g[0] = w->E[3 * k]; e->g[1] = w->E[3 * k + 1]; e->g[2] = w->E[3 * k + 2];
        e->h[0] = w->Qw0; e->h[1] = 0.0; e->h[2] = w->Qw1;
    } else {
        e->a[0] = 1.0; e->a[1] = 0.0; e->a[2] = 0.0; e->a[3] = 1.0;
        e->g[0] = e->g[1] = e->g[2] = 0.0;
        e->h[0] = e->h[1] = e->h[2] = 0.0;
    }
}

/* riccati_sweep in the active-set kernel's pair tree (lane l: knots 2l, 2l + 1; see
 * scan_backward_pairs): the pair element e_{2l} o e_{2l+1}, Kogge-Stone over the 64 lanes,
 * P_{2l} = f(P_N), then P_{2l+1} = f_{2l+1}(P_{2l+2}) in the lane (P_{2l+2} from lane l + 1). */
static int riccati_sweep_pairs(dcm_ws* w)
{
    const int N = w->N;
    int ok = 1;
    rc_el e[WV], ne[WV];
    for (int l = 0; l < WV; ++l) {
        rc_el e1;
        rc_knot(w, 2 * l, &e[l]);
        rc_knot(w, 2 * l + 1, &e1);
        if (!rc_combine(&e[l], &e1)) ok = 0;
    }
    const int pad = N <= 2 * WV - 2;   /* lane WV - 1 holds no knot: the identity (kernel as_pad) */
    for (int dd = 1; dd < WV; dd <<= 1) {
        for (int l = 0; l < WV; ++l) {
            ne[l] = e[l];
            if (l + dd < WV) {
                if (!rc_combine(&ne[l], &e[l + dd])) ok = 0;
            } else if (pad && !rc_combine(&ne[l], &e[WV - 1])) {
                ok = 0;
            }
        }
        memcpy(e, ne, sizeof(e));
    }
    double P0[WV][3];
    for (int l = 0; l < WV; ++l)
        if (!rc_apply(&e[l], w->Pw0, 0.0, w->Pw1, P0[l])) ok = 0;
    for (int l = 0; l < WV; ++l) {
        const int k0 = 2 * l, k1 = 2 * l + 1;
        rc_el e1;
        rc_knot(w, k1, &e1);
        double Pn[3] = {w->Pw0, 0.0, w->Pw1};
        if (l + 1 < WV) { Pn[0] = P0[l + 1][0]; Pn[1] = P0[l + 1][1]; Pn[2] = P0[l + 1][2]; }
        double P1[3];
        if (!rc_apply(&e1, Pn[0], Pn[1], Pn[2], P1)) ok = 0;
        /* P_{k+1} of knot k: knot 2l takes P_{2l+1}, knot 2l + 1 takes P_{2l+2} */
        if (k0 < N) { w->Pn[3 * k0] = P1[0]; w->Pn[3 * k0 + 1] = P1[1]; w->Pn[3 * k0 + 2] = P1[2]; }
        if (k1 < N) { w->Pn[3 * k1] = Pn[0]; w->Pn[3 * k1 + 1] = Pn[1]; w->Pn[3 * k1 + 2] = Pn[2]; }
    }
    w->Pn[3 * (N - 1)] = w->Pw0;
    w->Pn[3 * (N - 1) + 1] = 0.0;
    w->Pn[3 * (N - 1) + 2] = w->Pw1;
    return ok;
}

/* riccati_sweep in the active-set kernels' DPP tree (see scan_backward_dpp): the lane element
 * (the pair e_{2l} o e_{2l+1} for KPL = 2), the DPP tree, P at the lane's first knot
 * = f(P_N); a knot's P_{k+1} from the next lane (P_{2l+1} = f_{2l+1}(P_{2l+2}) in the lane). */
static int riccati_sweep_dpp(dcm_ws* w)
{
    const int N = w->N, KPL = N > WV ? 2 : 1;
    int ok = 1;
    rc_el e[WV], ne[WV];
    for (int l = 0; l < WV; ++l) {
        rc_knot(w, KPL * l, &e[l]);
        if (KPL == 2) {
            rc_el e1;
            rc_knot(w, 2 * l + 1, &e1);
            if (!rc_combine(&e[l], &e1)) ok = 0;
        }
    }
    for (int L = 0; L < AS_LEVELS; ++L) {
        for (int l = 0; l < WV; ++l) {
            const int src = orc_lane_src(L, 0, l);
            ne[l] = e[l];
            if (src >= 0 && !rc_combine(&ne[l], &e[src])) ok = 0;
        }
        memcpy(e, ne, sizeof(e));
    }
    double P0[WV][3];
    for (int l = 0; l < WV; ++l)
        if (!rc_apply(&e[l], w->Pw0, 0.0, w->Pw1, P0[l])) ok = 0;
    for (int l = 0; l < WV; ++l) {
        double Pn[3] = {w->Pw0, 0.0, w->Pw1};
        if (l + 1 < WV) { Pn[0] = P0[l + 1][0]; Pn[1] = P0[l + 1][1]; Pn[2] = P0[l + 1][2]; }
        const int kl = KPL * l + KPL - 1;   /* the lane's last knot takes P from the next lane */
        if (kl < N) { w->Pn[3 * kl] = Pn[0]; w->Pn[3 * kl + 1] = Pn[1]; w->Pn[3 * kl + 2] = Pn[2]; }
        if (KPL == 2) {
            const int k0 = 2 * l;
            rc_el e1;
            rc_knot(w, 2 * l + 1, &e1);
            double P1[3];
            if (!rc_apply(&e1, Pn[0], Pn[1], Pn[2], P1)) ok = 0;
            if (k0 < N) { w->Pn[3 * k0] = P1[0]; w->Pn[3 * k0 + 1] = P1[1]; w->Pn[3 * k0 + 2] = P1[2]; }
        }
    }
    w->Pn[3 * (N - 1)] = w->Pw0;
    w->Pn[3 * (N - 1) + 1] = 0.0;
    w->Pn[3 * (N - 1) + 2] = w->Pw1;
    return ok;
}

/* Riccati sweep for the per-knot E_k = w->E: P_k for every knot by a Kogge-Stone
 * scan of Riccati map elements over the 64 lanes of each wavefront (lane l composes with lane
 * l + d), then P_k = f_{k..}(P at the next wavefront's first knot, or P_N = diag(Pw)), wavefronts
 * from last to first.  Leaves P_{k+1} in w->Pn[k].  Returns 0 if some (I + G H) or (I + G P) is
 * not positive definite. */
static int riccati_sweep(dcm_ws* w)
{
    const int N = w->N;
    int ok = 1;
    double Pb0 = w->Pw0, Pb1 = 0.0, Pb2 = w->Pw1;      /* P at the next wavefront's first knot */
    if (!w->scans) {   /* CPU-efficient sequential recursion P_k = f_k(P_{k+1}) (cpu_baseline only) */
        for (int k = N - 1; k >= 1; --k) {
            rc_el e;
            e.a[0] = w->al[k]; e.a[1] = 0.0; e.a[2] = 0.0; e.a[3] = w->al[k];
            e.g[0] = w->E[3 * k]; e.g[1] = w->E[3 * k + 1]; e.g[2] = w->E[3 * k + 2];
            e.h[0] = w->Qw0; e.h[1] = 0.0; e.h[2] = w->Qw1;
            double out[3];
            if (!rc_apply(&e, Pb0, Pb1, Pb2, out)) ok = 0;
            w->Pn[3 * (k - 1)] = out[0]; w->Pn[3 * (k - 1) + 1] = out[1]; w->Pn[3 * (k - 1) + 2] = out[2];
            Pb0 = out[0]; Pb1 = out[1]; Pb2 = out[2];
        }
    }
    if (w->scans && w->dpp) return riccati_sweep_dpp(w);
    if (w->scans && w->pairs) return riccati_sweep_pairs(w);
    for (int wv = w->scans ? w->NW - 1 : -1; wv >= 0; --wv) {
        rc_el e[WV], ne[WV];
        for (int l = 0; l < WV; ++l) {
            const int k = WV * wv + l;
            if (k < N) {
                e[l].a[0] = w->al[k]; e[l].a[1] = 0.0; e[l].a[2] = 0.0; e[l].a[3] = w->al[k];
                e[l].g[0] = w->E[3 * k]; e[l].g[1] = w->E[3 * k + 1]; e[l].g[2] = w->E[3 * k + 2];
                e[l].h[0] = w->Qw0; e[l].h[1] = 0.0; e[l].h[2] = w->Qw1;
            } else {
                e[l].a[0] = 1.0; e[l].a[1] = 0.0; e[l].a[2] = 0.0; e[l].a[3] = 1.0;
                e[l].g[0] = e[l].g[1] = e[l].g[2] = 0.0;
                e[l].h[0] = e[l].h[1] = e[l].h[2] = 0.0;
            }
        }
        for (int dd = 1; dd < WV; dd <<= 1) {
            for (int l = 0; l < WV; ++l) {
                ne[l] = e[l];
                if (l + dd < WV && !rc_combine(&ne[l], &e[l + dd])) ok = 0;
            }
            memcpy(e, ne, sizeof(e));
        }
        double Pw0v = 0.0, Pw1v = 0.0, Pw2v = 0.0;
        for (int l = 0; l < WV; ++l) {
            const int k = WV * wv + l;
            double out[3];
            if (!rc_apply(&e[l], Pb0, Pb1, Pb2, out)) ok = 0;
            if (l == 0) { Pw0v = out[0]; Pw1v = out[1]; Pw2v = out[2]; }
            if (k >= 1 && k < N) {
                w->Pn[3 * (k - 1)] = out[0];        /* P_k, needed by knot k - 1 */
                w->Pn[3 * (k - 1) + 1] = out[1];
                w->Pn[3 * (k - 1) + 2] = out[2];
            }
        }
        Pb0 = Pw0v; Pb1 = Pw1v; Pb2 = Pw2v;
    }
    w->Pn[3 * (N - 1)] = w->Pw0;
    w->Pn[3 * (N - 1) + 1] = 0.0;
    w->Pn[3 * (N - 1) + 2] = w->Pw1;
    return ok;
}

/* M_k = P_{k+1} h_k and G_k = alpha_k (I - beta_k^2 M_k) from w->h[k] (knot-parallel). */
static void mg_from_h(dcm_ws* w, int k)
{
    const double P00 = w->Pn[3 * k], P01 = w->Pn[3 * k + 1], P11 = w->Pn[3 * k + 2];
    const double h00 = w->h[3 * k], h01 = w->h[3 * k + 1], h11 = w->h[3 * k + 2];
    const double b2 = w->b2[k];
    const double M00 = FD2(P00, h00, P01, h01);
    const double M01 = FD2(P00, h01, P01, h11);
    const double M10 = FD2(P01, h00, P11, h01);
    const double M11 = FD2(P01, h01, P11, h11);
    double* Mk = w->Mm + 4 * k;
    Mk[0] = M00; Mk[1] = M01; Mk[2] = M10; Mk[3] = M11;
    const double al = w->al[k];
    double* G = w->G + 4 * k;
    G[0] = al * fma(-b2, M00, 1.0);
    G[1] = -(al * (b2 * M01));
    G[2] = -(al * (b2 * M10));
    G[3] = al * fma(-b2, M11, 1.0);
}

/* Factorization of the Newton system for the barrier Hessian blocks W_k.
 * 1. E_k = beta_k^2 (R + W_k)^{-1}                                           (knot-parallel)
 * 2. P_k for every knot by the Riccati sweep (riccati_sweep)
 * 3. H_k = R + W_k + beta_k^2 P_{k+1}, h_k = H_k^{-1}, M_k = P_{k+1} h_k,
 *    G_k = alpha_k (I - beta_k^2 M_k)                                         (knot-parallel)
 * Returns 0 if some (I + G H), (I + G P) or H_k is not positive definite (status NUMERICAL). */
static int dcm_factor(dcm_ws* w)
{
    const int N = w->N;
    for (int k = 0; k < N; ++k) {
        const double* Wk = w->W + 4 * k;
        const double detRW = fma(w->Rw0, w->Rw1, FD2(w->Rw1, Wk[0], w->Rw0, Wk[2])) + Wk[3];
        const double ie = w->b2[k] / detRW;
        w->E[3 * k] = (w->Rw1 + Wk[2]) * ie;
        w->E[3 * k + 1] = -(Wk[1] * ie);
        w->E[3 * k + 2] = (w->Rw0 + Wk[0]) * ie;
    }
    int ok = riccati_sweep(w);
    for (int k = 0; k < N; ++k) {
        const double P00 = w->Pn[3 * k], P01 = w->Pn[3 * k + 1], P11 = w->Pn[3 * k + 2];
        const double* Wk = w->W + 4 * k;
        const double b2 = w->b2[k];
        /* det H = det B + tr(adj(B) W) + det W, B = R + b2 P: no cancellation for huge W */
        const double B00 = fma(b2, P00, w->Rw0);
        const double B01 = b2 * P01;
        const double B11 = fma(b2, P11, w->Rw1);
        const double H00 = B00 + Wk[0];
        const double H01 = B01 + Wk[1];
        const double H11 = B11 + Wk[2];
        const double detB = fma(B00, B11, -(B01 * B01));
        const double trW = FD2(B11, Wk[0], B00, Wk[2]) - 2.0 * (B01 * Wk[1]);
        const double det = (detB + trW) + Wk[3];
        if (!(det > 0.0) || isinf(det)) ok = 0;
        const double idet = 1.0 / det;
        w->h[3 * k] = H11 * idet; w->h[3 * k + 1] = -(H01 * idet); w->h[3 * k + 2] = H00 * idet;
        mg_from_h(w, k);
    }
    return ok;
}

/* Solve the factored Newton system for the right-hand side g:
 *   c_k = G_k (qx_k + P_{k+1} d_k) + alpha beta M_k g_k;  v: backward scan;
 *   t = (qx + P d) + v_{k+1};  kff = -h (g - beta t);  f = d - beta kff;
 *   dxi_{k+1} = G_k^T dxi_k + f_k: forward scan;  dr_k = alpha beta M_k^T dxi_k + kff_k. */
static void dcm_solve(dcm_ws* w)
{
    const int N = w->N;
    for (int k = 0; k < N; ++k) {
        const double P00 = w->Pn[3 * k], P01 = w->Pn[3 * k + 1], P11 = w->Pn[3 * k + 2];
        const double d0 = w->d[2 * k], d1 = w->d[2 * k + 1];
        const double y0 = FD3(P00, d0, P01, d1, w->qx[2 * k]);
        const double y1 = FD3(P01, d0, P11, d1, w->qx[2 * k + 1]);
        const double* Mk = w->Mm + 4 * k;
        const double M00 = Mk[0], M01 = Mk[1], M10 = Mk[2], M11 = Mk[3];
        const double g0 = w->g[2 * k], g1 = w->g[2 * k + 1];
        const double Mg0 = FD2(M00, g0, M01, g1);
        const double Mg1 = FD2(M10, g0, M11, g1);
        const double* G = w->G + 4 * k;
        w->sc[2 * k] = FD3(G[0], y0, G[1], y1, w->ab[k] * Mg0);
        w->sc[2 * k + 1] = FD3(G[2], y0, G[3], y1, w->ab[k] * Mg1);
    }
    scan_backward(w, w->G, w->sc);
    for (int k = 0; k < N; ++k) {
        const double P00 = w->Pn[3 * k], P01 = w->Pn[3 * k + 1], P11 = w->Pn[3 * k + 2];
        const double d0 = w->d[2 * k], d1 = w->d[2 * k + 1];
        const double y0 = FD3(P00, d0, P01, d1, w->qx[2 * k]);
        const double y1 = FD3(P01, d0, P11, d1, w->qx[2 * k + 1]);
        const double t0 = y0 + w->v[2 * (k + 1)];
        const double t1 = y1 + w->v[2 * (k + 1) + 1];
        const double be = w->be[k];
        const double hu0 = fma(-be, t0, w->g[2 * k]);
        const double hu1 = fma(-be, t1, w->g[2 * k + 1]);
        const double h00 = w->h[3 * k], h01 = w->h[3 * k + 1], h11 = w->h[3 * k + 2];
        const double k0 = -FD2(h00, hu0, h01, hu1);
        const double k1 = -FD2(h01, hu0, h11, hu1);
        w->dr[2 * k] = k0;                        /* kff until the forward scan is done */
        w->dr[2 * k + 1] = k1;
        w->sc[2 * k] = fma(-be, k0, d0);
        w->sc[2 * k + 1] = fma(-be, k1, d1);
    }
    scan_forward(w, w->G, 1, w->sc);
    for (int k = 0; k < N; ++k) {
        const double* Mk = w->Mm + 4 * k;
        const double M00 = Mk[0], M01 = Mk[1], M10 = Mk[2], M11 = Mk[3];
        const double x0 = w->x[2 * k], x1 = w->x[2 * k + 1];
        const double ab = w->ab[k];
        w->dr[2 * k] = fma(ab, FD2(M00, x0, M10, x1), w->dr[2 * k]);
        w->dr[2 * k + 1] = fma(ab, FD2(M01, x0, M11, x1), w->dr[2 * k + 1]);
    }
}

/* W-phase (knot-parallel): 1/s, W = A^T diag(lam/s) A, det W = sum_{i<j} sg_i sg_j (a_i x a_j)^2
 * (a sum of non-negative terms), and the predictor right-hand side g = rh + A^T e,
 * e_i = (lam_i rp_i - s_i lam_i) / s_i. */
static void dcm_wphase(dcm_ws* w)
{
    const int N = w->N, M = w->M;
    for (int k = 0; k < N; ++k) {
        const int m = w->nf[k];
        const double r0 = w->vrp[2 * k], r1 = w->vrp[2 * k + 1];
        double W00 = 0.0, W01 = 0.0, W11 = 0.0, dW = 0.0;
        double g0 = w->rh[2 * k], g1 = w->rh[2 * k + 1];
        double sgv[MF];
        for (int i = 0; i < m; ++i) {
            const double* a = w->A + (k * M + i) * 2;
            const double si = w->s[k * MF + i], li = w->lam[k * MF + i];
            const double is = 1.0 / si;
            w->is[k * MF + i] = is;
            const double sg = li * is;
            sgv[i] = sg;
            const double t0 = sg * a[0];
            const double t1 = sg * a[1];
            W00 = fma(t0, a[0], W00);
            W01 = fma(t0, a[1], W01);
            W11 = fma(t1, a[1], W11);
            const double rpi = (FD2(a[0], r0, a[1], r1) + si) - w->b[k * M + i];
            const double e = fma(li, rpi, -(si * li)) * is;
            g0 = fma(a[0], e, g0);
            g1 = fma(a[1], e, g1);
        }
        for (int i = 1; i < m; ++i) {
            const double* ai = w->A + (k * M + i) * 2;
            for (int j = 0; j < i; ++j) {
                const double* aj = w->A + (k * M + j) * 2;
                const double cr = fma(ai[0], aj[1], -(ai[1] * aj[0]));
                dW = fma(sgv[i] * sgv[j], cr * cr, dW);
            }
        }
        double* Wk = w->W + 4 * k;
        Wk[0] = W00; Wk[1] = W01; Wk[2] = W11; Wk[3] = dW;
        w->g[2 * k] = g0;
        w->g[2 * k + 1] = g1;
    }
}

/* The affine (predictor) slack / multiplier step of facet i of knot k for the VRP step dra:
 * ds = -rp - a . dra,  dl = -(lam (s + ds)) / s  (= (-s lam - lam ds) / s). */
static void affine_step(const dcm_ws* w, int k, int i, double* ds, double* dl)
{
    const double* a = w->A + (k * w->M + i) * 2;
    const double r0 = w->vrp[2 * k], r1 = w->vrp[2 * k + 1];
    const double si = w->s[k * MF + i], li = w->lam[k * MF + i];
    const double rpi = (FD2(a[0], r0, a[1], r1) + si) - w->b[k * w->M + i];
    const double dsv = (-rpi) - FD2(a[0], w->dra[2 * k], a[1], w->dra[2 * k + 1]);
    *ds = dsv;
    *dl = -((li * (si + dsv)) * w->is[k * MF + i]);
}

/* Active-set polish ("Polish"; the kernel's polish block mirrors it term for term).
 * From an interior iterate, guess the active set (facet i of knot k is active iff lam_i > s_i; at
 * most two per knot), move each r_k onto its active lines, and take ONE Newton step of the
 * equality-constrained QP, where knot k's VRP moves only along the active lines:
 *   c_k = 0: E_k = beta^2 R^{-1},                 h_k = B^{-1}
 *   c_k = 1: E_k = beta^2 t t^T / (t^T R t),      h_k = t t^T / (t^T B t),  t = (-a_y, a_x)
 *   c_k = 2: E_k = 0,                             h_k = 0                   (r_k is the vertex)
 * with B = R + beta^2 P_{k+1} — the W -> infinity limits of the barrier blocks.  The QP is
 * quadratic, so the step lands on the equality-constrained optimum up to rounding.  It is then
 * certified as the optimum of the inequality QP: every inactive facet satisfied (a r - b <= tol_p),
 * stationarity R (r - r_ref) + A_act^T lam = beta nu_k (the solve's costates of the new point)
 * solved for the active multipliers with residual <= tol_d, and lam >= -tol_d.  Accepted: xi, vrp hold
 * the polished optimum, lam its multipliers (max(lam, 0) on the active facets, 0 on the others)
 * and 1 is returned.  Rejected: xi, vrp are restored, 0 is returned. */
/* Facet i of knot k is in a polish pass's active set: guessed (the active-set start's guess bits,
 * or an IPM iterate's lam_i > s_i) and not dropped, or added. */
/* An IPM iterate's guess: lam_i > s_i, and not faint: lam_i below ORC_LAM_REL (1e-8) of the knot's
 * largest multiplier while facet i is within |a_i x a_max| < ORC_LAM_REL_CROSS (0.3, 17 degrees) of
 * parallel to that multiplier's facet.  The rule only matters where multipliers reach ~1e7 (the
 * uncapturable-state windows, tests/golden/c5_hard_windows.npz): on an edge that meets a nearly
 * parallel neighbour (support polygons of slightly rotated feet, facets 0.1 degree apart) the
 * neighbour's slack is ~1e-5 while its multiplier is ~0.1, rounding-level against the edge's
 * 1e6, and lam > s alone would put the knot on their ill-conditioned vertex.  Round 6: only near
 * parallel facets are faint — on the pushed-robot windows (tests/golden/c5_pushed_windows.npz) a
 * well-conditioned vertex's second multiplier is below 1e-8 of the first (1e8 against 0.5) and
 * excluding it made every pass of the polish fail. */
static int cand_bit(const dcm_ws* w, const int* guess, const int* drop, const int* add, int k, int i)
{
    double lmx = 0.0;
    int jm = 0;   /* the knot's largest multiplier (the first of equal ones) */
    for (int j = 0; j < w->nf[k]; ++j) {
        if (w->lam[k * MF + j] > lmx) jm = j;
        lmx = keepmax(lmx, w->lam[k * MF + j]);
    }
    const double* ai = w->A + (k * w->M + i) * 2;
    const double* am = w->A + (k * w->M + jm) * 2;
    const double cr = fabs(fma(ai[0], am[1], -(ai[1] * am[0])));
    const int faint = w->lam[k * MF + i] < ORC_LAM_REL * lmx && cr < ORC_LAM_REL_CROSS;
    const int base = guess ? ((guess[k] >> i) & 1) : (w->lam[k * MF + i] > w->s[k * MF + i] && !faint);
    return (base && !((drop[k] >> i) & 1)) || ((add[k] >> i) & 1);
}

/* ---- the refinement of a certified optimum (round 6; the kernels' refine_rhs, dcm_qp_common.h).
 * Where the multipliers reach 1e6-1e9 (uncapturable DCM states, tests/golden/c5_*_windows.npz)
 * the costates are ~1e8-1e10 and a fp64 solve determines the VRPs only to ~1e-14 x the largest
 * multiplier: the step's own right-hand side (q_k = Q (xi - xi_ref), the costate scan) rounds at
 * that scale.  The refinement takes ORC_REFINE_STEPS (2) more Newton steps of the same equality-constrained QP with
 * the same factorization, written in the Lagrangian-shifted form: with the certified costates nu
 * (nu_k = the costate of xi_{k+1}),
 *   d_k  = xi_k + dt (om_k xi_k - om_k r_k) - xi_{k+1}                    (the Euler defect)
 *   qx_k = W_k (xi_{k+1} - xi_ref_{k+1}) - nu_k + (1 + dt om_{k+1}) nu_{k+1}   (0 past knot N - 1)
 *   g_k  = R (r_k - r_ref_k) - dt om_k nu_k, projected onto the active line (c = 1), 0 at a vertex
 * — the stationarity residuals at (xi, r, nu), which are small, so the step's costates are small
 * and its rounding is small.  Each is evaluated in double-double (exact TwoSum / TwoProd by fma,
 * the exact alpha_k = 1 + dt om_k and beta_k = dt om_k) and rounded once.  Measured: every window of
 * the three c5 fixtures from <= 5.7e-4 to <= 1.6e-11 m against the extended-precision solve
 * (tests/test_c5_windows.py). */
typedef struct { double hi, lo; } ddv;
static ddv dd_two_sum(double a, double b)
{
    const double s = a + b;
    const double bb = s - a;
    ddv r = { s, (a - (s - bb)) + (b - bb) };
    return r;
}
static ddv dd_fast(double a, double b)
{
    const double s = a + b;
    ddv r = { s, b - (s - a) };
    return r;
}
static ddv dd_prod(double a, double b)
{
    const double p = a * b;
    ddv r = { p, fma(a, b, -p) };
    return r;
}
static ddv dd_add(ddv x, ddv y)
{
    const ddv s = dd_two_sum(x.hi, y.hi);
    return dd_fast(s.hi, s.lo + (x.lo + y.lo));
}
static ddv dd_add_d(ddv x, double y)
{
    const ddv s = dd_two_sum(x.hi, y);
    return dd_fast(s.hi, s.lo + x.lo);
}
static ddv dd_mul_d(ddv x, double y)
{
    const ddv p = dd_prod(x.hi, y);
    return dd_fast(p.hi, fma(x.lo, y, p.lo));
}
static ddv dd_neg(ddv x)
{
    ddv r = { -x.hi, -x.lo };
    return r;
}

/* The refinement's right-hand side of knot k (active count c, active row a = facet pi1). */
static void refine_rhs(const dcm_ws* w, int k, int c, const double* a, const double* nu, double* d,
                       double* qx, double* g)
{
    const int N = w->N;
    const double om = w->omega[k];
    const int last = k == N - 1;
    for (int j = 0; j < 2; ++j) {
        const double xk = w->xi[2 * k + j], xn = w->xi[2 * (k + 1) + j], r = w->vrp[2 * k + j];
        ddv e = dd_add(dd_prod(om, xk), dd_neg(dd_prod(om, r)));
        e = dd_mul_d(e, w->dt);
        e = dd_add_d(e, xk);
        e = dd_add_d(e, -xn);
        d[j] = e.hi;
        const double Wq = last ? (j ? w->Pw1 : w->Pw0) : (j ? w->Qw1 : w->Qw0);
        ddv q = dd_mul_d(dd_two_sum(xn, -w->xi_ref[2 * (k + 1) + j]), Wq);
        q = dd_add_d(q, -nu[2 * k + j]);
        if (!last) {
            q = dd_add(q, dd_mul_d(dd_prod(w->dt, w->omega[k + 1]), nu[2 * (k + 1) + j]));
            q = dd_add_d(q, nu[2 * (k + 1) + j]);
        }
        qx[j] = q.hi;
    }
    const ddv bk = dd_prod(w->dt, om);
    const ddv g0 = dd_add(dd_mul_d(dd_two_sum(w->vrp[2 * k], -w->vrp_ref[2 * k]), w->Rw0), dd_neg(dd_mul_d(bk, nu[2 * k])));
    const ddv g1 = dd_add(dd_mul_d(dd_two_sum(w->vrp[2 * k + 1], -w->vrp_ref[2 * k + 1]), w->Rw1),
                          dd_neg(dd_mul_d(bk, nu[2 * k + 1])));
    if (c == 0) {
        g[0] = g0.hi;
        g[1] = g1.hi;
    } else if (c == 1) {   /* t = (-a_y, a_x): g <- t (t . g) / |a|^2 */
        const ddv tg = dd_add(dd_mul_d(g0, -a[1]), dd_mul_d(g1, a[0]));
        const double tau = tg.hi / FD2(a[0], a[0], a[1], a[1]);
        g[0] = -(a[1] * tau);
        g[1] = a[0] * tau;
    } else {
        g[0] = 0.0;
        g[1] = 0.0;
    }
}

/* r_k back onto its active line after a step (c = 1): the step moves r along the line in exact
 * arithmetic, but its rounding scales with the step's terms (costates up to 1e10 on the pushed-robot
 * windows, tests/golden/c5_pushed_windows.npz), and a drift of 1e-10 off the line failed the
 * certificate's primal check there pass after pass (round 6; the kernels' project_line). */
static void project_line(dcm_ws* w, int k, const double* a, double b)
{
    const double aa = FD2(a[0], a[0], a[1], a[1]);
    const double t = (FD2(a[0], w->vrp[2 * k], a[1], w->vrp[2 * k + 1]) - b) / aa;
    w->vrp[2 * k] = fma(-t, a[0], w->vrp[2 * k]);
    w->vrp[2 * k + 1] = fma(-t, a[1], w->vrp[2 * k + 1]);
}

/* The anti-cycling rule of the active-set kernels' fp64 passes (anti_cycle = 1; round 6).  The
 * drop/add moves change every knot at once, and on degenerate vertices of three-contact polygons
 * they cycle: e.g. knot 0 on the vertex of facets 1 and 2 with multipliers -150 / 150, facet 1
 * dropped, then facet 2, then both added back (bench.py --workload mc: 3 of 4096 cold windows
 * went to the interior point method after 8 passes, 0.45 of the window's 0.57 ms).  From pass
 * ORC_GUESS_PASSES (8) on, up to ORC_AS_PASSES (12), every pass changes ONE facet: at the lowest
 * knot whose sets the certificate changed, the lowest-index facet it dropped (negative
 * multiplier), else the lowest-index facet it added (violated) -- Bland's rule, which cannot
 * cycle the way the simultaneous moves do.  (A hash of the passes' candidate sets that switched
 * on repetition certified the same windows, cost the kernel's pass loop 1.5 % on configs[1]
 * and is not kept.) */
static int dcm_polish(dcm_ws* w, double tol_p, double tol_dd, const int* guess, int max_pass, int anti_cycle)
{
    const int N = w->N, M = w->M;
    int ok = 1;
    double* nuv = (double*)malloc(sizeof(double) * 2 * (size_t)N);   /* [N][2] the certified costates */
    int* pc = (int*)malloc(sizeof(int) * 4 * (size_t)N);
    int* pi1 = pc + N;
    int* pi2 = pc + 2 * N;
    int* drop = pc + 3 * N;   /* facets taken out of the guessed active set (bit i: facet i) */
    int* add = (int*)calloc((size_t)N, sizeof(int));   /* facets put into it */
    double* bak = (double*)malloc(sizeof(double) * (6 * (size_t)N + 2));
    double* lm = bak + 4 * (size_t)N + 2;   /* [N][2] multipliers of the active facets */
    memcpy(bak, w->vrp, sizeof(double) * 2 * N);
    memcpy(bak + 2 * N, w->xi, sizeof(double) * (2 * (size_t)N + 2));
    for (int k = 0; k < N; ++k) drop[k] = 0;
    /* pass 0: the guessed active set; every further pass drops the facets whose multiplier came
     * out negative and adds the facets left violated (a facet's drop and add bits are exclusive,
     * the later event wins), up to max_pass passes.  Every pass starts from the same iterate.
     * (Until round 3 the IPM's polish ran at most three passes: pass 1 only dropping, pass 2 only
     * adding; the uncapturable-state windows of tests/golden/c5_hard_windows.npz need the
     * alternating moves of the active-set start there too.) */
    int* sdr = (int*)malloc(sizeof(int) * 2 * (size_t)N);   /* drop / add before the certificate */
    int* sad = sdr + N;
    for (int pass = 0; pass < max_pass; ++pass) {
    ++w->npass;
    ok = 1;
    const int bland = anti_cycle && pass >= ORC_GUESS_PASSES;   /* Bland's rule from pass 8 on */
    memcpy(sdr, drop, sizeof(int) * N);
    memcpy(sad, add, sizeof(int) * N);
    int neg = 0, viol = 0;
    double vmax = 0.0;   /* the pass's largest violation (the IPM polish's add threshold) */
    /* 1. active sets, projection onto the active lines, E_k (knot-parallel) */
    for (int k = 0; k < N; ++k) {
        const int m = w->nf[k];
        int c = 0, i1 = 0, i2 = 0;
        for (int i = 0; i < m; ++i) {
            if (cand_bit(w, guess, drop, add, k, i)) {
                if (c == 0) i1 = i;
                else if (c == 1) i2 = i;
                ++c;
            }
        }
        if (c > 2) {
            /* more than two candidate lines (the drop/add moves can add two facets at once): the
             * first pair in facet order whose vertex satisfies every facet of the knot (a vertex
             * of the support polygon) becomes the active pair; none: the pass fails */
            int found = 0;
            for (int x = 0; x < m && !found; ++x) {
                if (!cand_bit(w, guess, drop, add, k, x)) continue;
                for (int y = x + 1; y < m && !found; ++y) {
                    if (!cand_bit(w, guess, drop, add, k, y)) continue;
                    const double* a = w->A + (k * M + x) * 2;
                    const double* e = w->A + (k * M + y) * 2;
                    const double ba = w->b[k * M + x], be = w->b[k * M + y];
                    const double det = fma(a[0], e[1], -(a[1] * e[0]));
                    const double aa = FD2(a[0], a[0], a[1], a[1]), ee = FD2(e[0], e[0], e[1], e[1]);
                    if (!(det * det > 1e-18 * (aa * ee))) continue;
                    const double idet = 1.0 / det;
                    const double v0 = fma(ba, e[1], -(a[1] * be)) * idet;
                    const double v1 = fma(a[0], be, -(ba * e[0])) * idet;
                    int feas = 1;
                    for (int l = 0; l < m; ++l) {
                        const double* f = w->A + (k * M + l) * 2;
                        if (!(FD2(f[0], v0, f[1], v1) - w->b[k * M + l] <= tol_p)) feas = 0;
                    }
                    if (feas) { found = 1; i1 = x; i2 = y; }
                }
            }
            if (found) c = 2;
            else ok = 0;
        }
        pc[k] = c; pi1[k] = i1; pi2[k] = i2;
        const double r0 = w->vrp[2 * k], r1 = w->vrp[2 * k + 1];
        const double b2 = w->b2[k];
        double* E = w->E + 3 * k;
        if (c == 0) {
            E[0] = b2 / w->Rw0; E[1] = 0.0; E[2] = b2 / w->Rw1;
        } else if (c == 1) {
            const double* a = w->A + (k * M + i1) * 2;
            const double aa = FD2(a[0], a[0], a[1], a[1]);
            const double t = (FD2(a[0], r0, a[1], r1) - w->b[k * M + i1]) / aa;
            w->vrp[2 * k] = fma(-t, a[0], r0);
            w->vrp[2 * k + 1] = fma(-t, a[1], r1);
            const double u = a[1] * a[1], v = a[0] * a[0], q = a[0] * a[1];
            const double ie = b2 / FD2(w->Rw0, u, w->Rw1, v);
            E[0] = u * ie; E[1] = -(q * ie); E[2] = v * ie;
        } else {
            const double* a = w->A + (k * M + i1) * 2;
            const double* e = w->A + (k * M + i2) * 2;
            const double ba = w->b[k * M + i1], be = w->b[k * M + i2];
            const double det = fma(a[0], e[1], -(a[1] * e[0]));
            const double aa = FD2(a[0], a[0], a[1], a[1]), ee = FD2(e[0], e[0], e[1], e[1]);
            if (!(det * det > 1e-18 * (aa * ee))) ok = 0;      /* (nearly) parallel active facets */
            const double idet = 1.0 / det;
            w->vrp[2 * k] = fma(ba, e[1], -(a[1] * be)) * idet;
            w->vrp[2 * k + 1] = fma(a[0], be, -(ba * e[0])) * idet;
            E[0] = 0.0; E[1] = 0.0; E[2] = 0.0;
        }
    }
    /* 2. residuals at (xi, projected r): gradient, Euler defects */
    dcm_residuals(w, 0);
    /* 3. Riccati sweep; 4. h_k of the active subspace (knot-parallel) */
    if (!riccati_sweep(w)) ok = 0;
    for (int k = 0; k < N; ++k) {
        const double P00 = w->Pn[3 * k], P01 = w->Pn[3 * k + 1], P11 = w->Pn[3 * k + 2];
        const double b2 = w->b2[k];
        const double B00 = fma(b2, P00, w->Rw0);
        const double B01 = b2 * P01;
        const double B11 = fma(b2, P11, w->Rw1);
        double* h = w->h + 3 * k;
        if (pc[k] == 0) {
            const double det = fma(B00, B11, -(B01 * B01));
            if (!(det > 0.0) || isinf(det)) ok = 0;
            const double idet = 1.0 / det;
            h[0] = B11 * idet; h[1] = -(B01 * idet); h[2] = B00 * idet;
        } else if (pc[k] == 1) {
            const double* a = w->A + (k * M + pi1[k]) * 2;
            const double u = a[1] * a[1], v = a[0] * a[0], q = a[0] * a[1];
            const double tbt = FD3(B00, u, B11, v, -2.0 * (B01 * q));
            if (!(tbt > 0.0) || isinf(tbt)) ok = 0;
            const double it = 1.0 / tbt;
            h[0] = u * it; h[1] = -(q * it); h[2] = v * it;
        } else {
            h[0] = 0.0; h[1] = 0.0; h[2] = 0.0;
        }
        mg_from_h(w, k);
    }
    /* 5. the Newton step for g = R (r - r_ref) */
    for (int k = 0; k < N; ++k) {
        w->g[2 * k] = w->rh[2 * k];
        w->g[2 * k + 1] = w->rh[2 * k + 1];
    }
    dcm_solve(w);
    for (int k = 0; k < N; ++k) {
        w->vrp[2 * k] = w->vrp[2 * k] + w->dr[2 * k];
        w->vrp[2 * k + 1] = w->vrp[2 * k + 1] + w->dr[2 * k + 1];
        w->xi[2 * (k + 1)] = w->xi[2 * (k + 1)] + w->x[2 * (k + 1)];
        w->xi[2 * (k + 1) + 1] = w->xi[2 * (k + 1) + 1] + w->x[2 * (k + 1) + 1];
        if (pc[k] == 1) project_line(w, k, w->A + (k * M + pi1[k]) * 2, w->b[k * M + pi1[k]]);
    }
    /* 6. certificate: primal feasibility, stationarity, dual feasibility (knot-parallel).  The
     *    costates of the new point are the value-function gradients of the Riccati solve,
     *    nu_k = P_{k+1} dxi_{k+1} + (qx_k + v_{k+1}) — through the closed loop, which contracts;
     *    single shooting (nu_k = qx_k + alpha nu_{k+1}) would amplify rounding by alpha^N. */
    for (int k = 0; k < N; ++k) {
        const double P00 = w->Pn[3 * k], P01 = w->Pn[3 * k + 1], P11 = w->Pn[3 * k + 2];
        const double dx0 = w->x[2 * (k + 1)], dx1 = w->x[2 * (k + 1) + 1];
        const double s0 = w->qx[2 * k] + w->v[2 * (k + 1)];
        const double s1 = w->qx[2 * k + 1] + w->v[2 * (k + 1) + 1];
        const double nu0 = FD3(P00, dx0, P01, dx1, s0);
        const double nu1 = FD3(P01, dx0, P11, dx1, s1);
        nuv[2 * k] = nu0;
        nuv[2 * k + 1] = nu1;
        const double rh0 = w->Rw0 * (w->vrp[2 * k] - w->vrp_ref[2 * k]);
        const double rh1 = w->Rw1 * (w->vrp[2 * k + 1] - w->vrp_ref[2 * k + 1]);
        const double g0 = fma(w->be[k], nu0, -rh0);
        const double g1 = fma(w->be[k], nu1, -rh1);
        /* the dual tolerance grows with the knot's costate force beta nu once it exceeds
         * 1 / ORC_TOL_DUAL_REL (1e3; a planned walk's |beta nu| stays below ~2): the rounding of
         * nu grows with it, and the QPs of uncapturable DCM states carry |beta nu| and multipliers
         * up to ~1e8 (tests/golden/c5_hard_windows.npz) */
        const double tol_d = tol_dd * fmax(1.0, ORC_TOL_DUAL_REL * fmax(fabs(w->be[k] * nu0), fabs(w->be[k] * nu1)));
        const int c = pc[k];
        double l1 = 0.0, l2 = 0.0;
        if (c == 0) {
            if (!(fabs(g0) <= tol_d) || !(fabs(g1) <= tol_d)) ok = 0;
        } else if (c == 1) {
            const double* a = w->A + (k * M + pi1[k]) * 2;
            l1 = FD2(a[0], g0, a[1], g1) / FD2(a[0], a[0], a[1], a[1]);
            if (!(l1 >= -tol_d)) { ok = 0; neg = 1; drop[k] |= 1 << pi1[k]; add[k] &= ~(1 << pi1[k]); }
            if (!(fabs(fma(-l1, a[0], g0)) <= tol_d) || !(fabs(fma(-l1, a[1], g1)) <= tol_d)) ok = 0;
        } else {
            const double* a = w->A + (k * M + pi1[k]) * 2;
            const double* e = w->A + (k * M + pi2[k]) * 2;
            const double idet = 1.0 / fma(a[0], e[1], -(a[1] * e[0]));
            l1 = fma(g0, e[1], -(e[0] * g1)) * idet;
            l2 = fma(a[0], g1, -(g0 * a[1])) * idet;
            if (!(l1 >= -tol_d)) { ok = 0; neg = 1; drop[k] |= 1 << pi1[k]; add[k] &= ~(1 << pi1[k]); }
            if (!(l2 >= -tol_d)) { ok = 0; neg = 1; drop[k] |= 1 << pi2[k]; add[k] &= ~(1 << pi2[k]); }
#ifdef ORC_TRACE
            if (!(l1 >= -tol_d) || !(l2 >= -tol_d)) fprintf(stderr, "  k %d pair %d %d l1 %.3g l2 %.3g tol %.3g\n", k, pi1[k], pi2[k], l1, l2, tol_d);
#endif
        }
        lm[2 * k] = l1 > 0.0 ? l1 : 0.0;
        lm[2 * k + 1] = l2 > 0.0 ? l2 : 0.0;
        const double r0 = w->vrp[2 * k], r1 = w->vrp[2 * k + 1];
        for (int i = 0; i < w->nf[k]; ++i) {
            const double* a = w->A + (k * M + i) * 2;
            const double vi = FD2(a[0], r0, a[1], r1) - w->b[k * M + i];
            if (!(vi <= tol_p)) {
#ifdef ORC_TRACE
                fprintf(stderr, "  k %d facet %d viol %.3g c %d\n", k, i, vi, c);
#endif
                ok = 0;
                viol = 1;
                vmax = nanmax(vmax, vi);
                if (guess) { add[k] |= 1 << i; drop[k] &= ~(1 << i); }
            }
        }
    }
#ifdef ORC_TRACE
    {
        int n0 = 0, n1 = 0, n2 = 0, nd = 0, na = 0;
        for (int k = 0; k < N; ++k) { n0 += pc[k] == 0; n1 += pc[k] == 1; n2 += pc[k] == 2;
                                      nd += __builtin_popcount(drop[k]); na += __builtin_popcount(add[k]); }
        fprintf(stderr, "pass %d guess %d ok %d neg %d viol %d c0 %d c1 %d c2 %d drop %d add %d\n", pass,
                guess != 0, ok, neg, viol, n0, n1, n2, nd, na);
    }
#endif
    /* the IPM polish adds only the facets violated by at least ORC_ADD_REL of the pass's largest
     * violation: the knots next to a misidentified one are pushed over their own facets by
     * rounding-level amounts that the next pass removes (adding them as well made the passes
     * alternate on the uncapturable-state windows); the active-set start adds every one */
    if (!guess && viol) {
        const double thr = ORC_ADD_REL * vmax;
        for (int k = 0; k < N; ++k) {
            const double r0 = w->vrp[2 * k], r1 = w->vrp[2 * k + 1];
            for (int i = 0; i < w->nf[k]; ++i) {
                const double* a = w->A + (k * M + i) * 2;
                const double vi = FD2(a[0], r0, a[1], r1) - w->b[k * M + i];
                if (vi > tol_p && vi >= thr) { add[k] |= 1 << i; drop[k] &= ~(1 << i); }
            }
        }
    }
    if (bland && !ok) {   /* Bland: one change, at the lowest knot the certificate changed */
        int ks = -1;
        for (int k = 0; k < N && ks < 0; ++k)
            if (drop[k] != sdr[k] || add[k] != sad[k]) ks = k;
        for (int k = 0; k < N; ++k)
            if (k != ks) { drop[k] = sdr[k]; add[k] = sad[k]; }
        if (ks >= 0) {
            const int dn = drop[ks] & ~sdr[ks], an = add[ks] & ~sad[ks];
            const int bt = dn ? (dn & -dn) : (an & -an);
            drop[ks] = dn ? (sdr[ks] | bt) : (sdr[ks] & ~bt);
            add[ks] = dn ? (sad[ks] & ~bt) : (sad[ks] | bt);
        }
    }
    if (ok) break;
    if (!(neg || viol)) break;
    memcpy(w->vrp, bak, sizeof(double) * 2 * N);   /* pass 1 starts from the same iterate */
    memcpy(w->xi, bak + 2 * N, sizeof(double) * (2 * (size_t)N + 2));
    }
    if (!ok) {
        memcpy(w->vrp, bak, sizeof(double) * 2 * N);
        memcpy(w->xi, bak + 2 * N, sizeof(double) * (2 * (size_t)N + 2));
    } else {
        /* the refinement step (refine_rhs) where the largest multiplier exceeds ORC_REFINE_LAM */
        double lmx = 0.0;
        for (int k = 0; k < 2 * N; ++k) lmx = keepmax(lmx, lm[k]);
        for (int rs = 0; rs < ORC_REFINE_STEPS && lmx > ORC_REFINE_LAM; ++rs) {
            for (int k = 0; k < N; ++k)
                refine_rhs(w, k, pc[k], w->A + (k * M + pi1[k]) * 2, nuv, w->d + 2 * k, w->qx + 2 * k, w->g + 2 * k);
            dcm_solve(w);
            for (int k = 0; k < N; ++k) {
                /* the costates of the refined point: nu + the step's own (Lagrangian-shifted) costate */
                const double P00 = w->Pn[3 * k], P01 = w->Pn[3 * k + 1], P11 = w->Pn[3 * k + 2];
                const double dx0 = w->x[2 * (k + 1)], dx1 = w->x[2 * (k + 1) + 1];
                nuv[2 * k] = nuv[2 * k] + FD3(P00, dx0, P01, dx1, w->qx[2 * k] + w->v[2 * (k + 1)]);
                nuv[2 * k + 1] = nuv[2 * k + 1] + FD3(P01, dx0, P11, dx1, w->qx[2 * k + 1] + w->v[2 * (k + 1) + 1]);
                w->vrp[2 * k] = w->vrp[2 * k] + w->dr[2 * k];
                w->vrp[2 * k + 1] = w->vrp[2 * k + 1] + w->dr[2 * k + 1];
                w->xi[2 * (k + 1)] = w->xi[2 * (k + 1)] + w->x[2 * (k + 1)];
                w->xi[2 * (k + 1) + 1] = w->xi[2 * (k + 1) + 1] + w->x[2 * (k + 1) + 1];
                if (pc[k] == 1) project_line(w, k, w->A + (k * M + pi1[k]) * 2, w->b[k * M + pi1[k]]);
            }
        }
        /* the multipliers of the certified optimum: lam of the active facets, 0 elsewhere */
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < w->nf[k]; ++i)
                w->lam[k * MF + i] = (pc[k] >= 1 && i == pi1[k]) ? lm[2 * k]
                                     : (pc[k] == 2 && i == pi2[k]) ? lm[2 * k + 1] : 0.0;
    }
    free(pc);
    free(bak);
    free(add);
    free(nuv);
    free(sdr);
    return ok;
}

/* B-metric projection of rs onto the polygon {r : a_i . r <= b_i, i < m} of knot k (the saturated
 * start's one-step problem, see dcm_saturated_start): rs itself if no facet is violated; else the
 * candidate of least (r - rs)^T B (r - rs) among the projections onto single facet lines (valid
 * when the facet is violated and the point is feasible) and the vertices of facet pairs (valid
 * when feasible), candidates in the order: facets 0..m-1, then pairs (i, j), i < j < m,
 * lexicographic (the kernel: rounds of 64 candidates, one per lane);
 * the first of equal distances wins (the kernel: one candidate per lane, the lowest lane of the
 * minimum).  None valid (rounding): rs.  Returns the active count (0, 1, 2), facets in *i1, *i2. */
static int sat_project(const dcm_ws* w, int k, double rs0, double rs1, double B00, double B01,
                       double B11, double tol_p, double* r0, double* r1, int* i1, int* i2)
{
    const int M = w->M, m = w->nf[k];
    const double* A = w->A + (size_t)k * M * 2;
    const double* b = w->b + (size_t)k * M;
    *r0 = rs0; *r1 = rs1; *i1 = 0; *i2 = 0;
    int inside = 1;
    for (int i = 0; i < m; ++i)
        if (!(FD2(A[2 * i], rs0, A[2 * i + 1], rs1) - b[i] <= 0.0)) inside = 0;
    if (inside) return 0;
    const double detB = fma(B00, B11, -(B01 * B01));
    double best = 0.0;
    int bc = -1;
    const int nc = m + m * (m - 1) / 2;
    for (int c = 0; c < nc; ++c) {
        double v0, v1, dist;
        int x, y;
        if (c < m) {
            x = c; y = c;
            const double a0 = A[2 * x], a1 = A[2 * x + 1];
            const double u0 = fma(B11, a0, -(B01 * a1));       /* adj(B) a = det(B) B^{-1} a */
            const double u1 = fma(B00, a1, -(B01 * a0));
            const double aua = FD2(a0, u0, a1, u1);
            const double viol = FD2(a0, rs0, a1, rs1) - b[x];
            const double t = viol / aua;
            v0 = fma(-t, u0, rs0);
            v1 = fma(-t, u1, rs1);
            if (!(viol > 0.0)) continue;
            dist = (t * viol) * detB;
        } else {
            /* pair q = c - m of (0,1), (0,2), .., (0,m-1), (1,2), .. (m-2,m-1) */
            int q = c - m;
            x = 0;
            while (q >= m - 1 - x) { q -= m - 1 - x; ++x; }
            y = x + 1 + q;
            const double a0 = A[2 * x], a1 = A[2 * x + 1], e0 = A[2 * y], e1 = A[2 * y + 1];
            const double det = fma(a0, e1, -(a1 * e0));
            const double aa = FD2(a0, a0, a1, a1), ee = FD2(e0, e0, e1, e1);
            if (!(det * det > 1e-18 * (aa * ee))) continue;
            const double idet = 1.0 / det;
            v0 = fma(b[x], e1, -(a1 * b[y])) * idet;
            v1 = fma(a0, b[y], -(b[x] * e0)) * idet;
            const double d0 = v0 - rs0, d1 = v1 - rs1;
            dist = fma(d0, fma(B00, d0, 2.0 * (B01 * d1)), (B11 * d1) * d1);
        }
        int feas = 1;
        for (int l = 0; l < m; ++l)
            if (!(FD2(A[2 * l], v0, A[2 * l + 1], v1) - b[l] <= tol_p)) feas = 0;
        if (!feas || !(dist == dist)) continue;
        if (bc < 0 || dist < best) { best = dist; bc = c; *r0 = v0; *r1 = v1; *i1 = x; *i2 = y; }
    }
    if (bc < 0) { *r0 = rs0; *r1 = rs1; return 0; }
    return bc < m ? 1 : 2;
}

/* The saturated LQ start of the interior point method: when the active-set
 * start does not certify, the IPM starts from the closed-loop rollout of the unconstrained LQ
 * policy with every VRP projected onto its support polygon, instead of from the LQ optimum with
 * centred multipliers.  The QPs that get here are those of uncapturable DCM states
 * (tests/golden/c5_hard_windows.npz): the optimal VRPs sit on polygon vertices at nearly every
 * knot and the multipliers reach ~1e7, which an IPM started at lam ~ 1 takes 30-60 iterations to
 * reach.  The rollout puts the trajectory on the escaping side, and its costates give the
 * multipliers their scale:
 *   1. the LQ policy around the current iterate (one Newton step of the QP without facets):
 *      r_k(xi) = r*_k + alpha_k beta_k M_k^T (xi - xi*_k), with the one-step Hessian
 *      B_k = R + beta_k^2 P_{k+1};
 *   2. the rollout xi_0 = xi_init, r_k = the B_k-metric projection of r_k(xi_k) onto polygon k
 *      (sat_project), xi_{k+1} = xi_k + (omega xi_k - omega r_k) dt (the dynamics' own form: no
 *      defects);
 *   3. costates by single shooting over the rollout, nu_k = qx_k + alpha_k nu_{k+1}, and at each
 *      knot the multipliers of its projected facets from stationarity beta nu - R (r - r_ref) =
 *      A_act^T lam (clamped at 0);
 *   4. s = max(b - A r, 1e-2), lam = max(estimate, 1e-2 / s).
 * Returns 0 if the factorization fails; *dres receives max |R (r - r_ref) + A^T lam - beta nu|. */
static int dcm_saturated_start(dcm_ws* w, const double* xi_init, double tol_p, double* dres_out)
{
    const int N = w->N, M = w->M;
    int* act = (int*)malloc(sizeof(int) * 3 * (size_t)N);
    for (int k = 0; k < N; ++k) { w->W[4 * k] = w->W[4 * k + 1] = w->W[4 * k + 2] = w->W[4 * k + 3] = 0.0; }
    dcm_residuals(w, 0);
    for (int k = 0; k < N; ++k) { w->g[2 * k] = w->rh[2 * k]; w->g[2 * k + 1] = w->rh[2 * k + 1]; }
    const int ok = dcm_factor(w);
    dcm_solve(w);
    /* the LQ optimum: r*_k, xi*_k (knot k's own state; xi*_0 = xi_init) */
    for (int k = 0; k < N; ++k) {
        double* S = w->sg + 4 * k;
        S[0] = w->vrp[2 * k] + w->dr[2 * k];
        S[1] = w->vrp[2 * k + 1] + w->dr[2 * k + 1];
        S[2] = (k ? w->xi[2 * k] : xi_init[0]) + (k ? w->x[2 * k] : 0.0);
        S[3] = (k ? w->xi[2 * k + 1] : xi_init[1]) + (k ? w->x[2 * k + 1] : 0.0);
    }
    double x0 = xi_init[0], x1 = xi_init[1];
    for (int k = 0; k < N; ++k) {
        const double* S = w->sg + 4 * k;
        const double* Mk = w->Mm + 4 * k;
        const double d0 = x0 - S[2], d1 = x1 - S[3];
        const double rs0 = fma(w->ab[k], FD2(Mk[0], d0, Mk[2], d1), S[0]);
        const double rs1 = fma(w->ab[k], FD2(Mk[1], d0, Mk[3], d1), S[1]);
        const double b2 = w->b2[k];
        const double B00 = fma(b2, w->Pn[3 * k], w->Rw0);
        const double B01 = b2 * w->Pn[3 * k + 1];
        const double B11 = fma(b2, w->Pn[3 * k + 2], w->Rw1);
        double r0, r1;
        act[3 * k] = sat_project(w, k, rs0, rs1, B00, B01, B11, tol_p, &r0, &r1, &act[3 * k + 1], &act[3 * k + 2]);
        const double om = w->omega[k];
        const double dx0 = FD2(om, x0, -om, r0);
        const double dx1 = FD2(om, x1, -om, r1);
        x0 = fma(dx0, w->dt, x0);
        x1 = fma(dx1, w->dt, x1);
        w->vrp[2 * k] = r0;
        w->vrp[2 * k + 1] = r1;
        w->xi[2 * (k + 1)] = x0;
        w->xi[2 * (k + 1) + 1] = x1;
    }
    /* costates of the rollout (the warm start's backward scan) */
    dcm_residuals(w, 0);
    for (int k = 0; k < N; ++k) {
        double* G = w->sg + 4 * k;
        G[0] = w->al[k]; G[1] = 0.0; G[2] = 0.0; G[3] = w->al[k];
        w->sc[2 * k] = w->al[k] * w->qx[2 * k];
        w->sc[2 * k + 1] = w->al[k] * w->qx[2 * k + 1];
    }
    scan_backward(w, w->sg, w->sc);
    double dres = 0.0;
    for (int k = 0; k < N; ++k) {
        const double nu0 = w->qx[2 * k] + w->v[2 * (k + 1)];
        const double nu1 = w->qx[2 * k + 1] + w->v[2 * (k + 1) + 1];
        const double g0 = fma(w->be[k], nu0, -w->rh[2 * k]);
        const double g1 = fma(w->be[k], nu1, -w->rh[2 * k + 1]);
        const int c = act[3 * k], x = act[3 * k + 1], y = act[3 * k + 2];
        double l1 = 0.0, l2 = 0.0;
        if (c == 1) {
            const double* a = w->A + (k * M + x) * 2;
            l1 = FD2(a[0], g0, a[1], g1) / FD2(a[0], a[0], a[1], a[1]);
        } else if (c == 2) {
            const double* a = w->A + (k * M + x) * 2;
            const double* e = w->A + (k * M + y) * 2;
            const double idet = 1.0 / fma(a[0], e[1], -(a[1] * e[0]));
            l1 = fma(g0, e[1], -(e[0] * g1)) * idet;
            l2 = fma(a[0], g1, -(g0 * a[1])) * idet;
        }
        double al0 = 0.0, al1 = 0.0;   /* A^T lam */
        for (int i = 0; i < w->nf[k]; ++i) {
            const double* a = w->A + (k * M + i) * 2;
            const double sl = w->b[k * M + i] - FD2(a[0], w->vrp[2 * k], a[1], w->vrp[2 * k + 1]);
            const double si = sl > 1e-2 ? sl : 1e-2;
            const double est = (c >= 1 && i == x) ? l1 : (c == 2 && i == y) ? l2 : 0.0;
            const double lc = 1e-2 / si;
            w->s[k * MF + i] = si;
            w->lam[k * MF + i] = est > lc ? est : lc;
            al0 = fma(a[0], w->lam[k * MF + i], al0);
            al1 = fma(a[1], w->lam[k * MF + i], al1);
        }
        dres = nanmax(dres, fabs(al0 - g0));
        dres = nanmax(dres, fabs(al1 - g1));
    }
    free(act);
    *dres_out = dres;
    return ok;
}

int orc_dcm_mpc_solve(const orc_dcm_params* prm, const double* xi_init, const double* omega,
                      const double* xi_ref, const double* vrp_ref, const double* Ain,
                      const double* bin, const int32_t* nfacets, double* xi, double* vrp,
                      int32_t* iters_out)
{
    return orc_dcm_mpc_solve_warm(prm, xi_init, omega, xi_ref, vrp_ref, Ain, bin, nfacets, NULL,
                                  xi, vrp, NULL, iters_out, NULL, NULL);
}

#ifndef ORC_WARM_RETRY
#define ORC_WARM_RETRY 1   /* BLF_WARM_RETRY */
#endif
int orc_dcm_mpc_solve_warm(const orc_dcm_params* prm, const double* xi_init, const double* omega,
                           const double* xi_ref, const double* vrp_ref, const double* Ain,
                           const double* bin, const int32_t* nfacets, const orc_dcm_warm* warm,
                           double* xi, double* vrp, double* lam_out, int32_t* iters_out,
                           int32_t* polished_out, int32_t* passes_out)
{
    const int N = prm->horizon;
    const int M = prm->max_facets;
    dcm_ws ws;
    dcm_ws* w = &ws;
    w->N = N; w->M = M; w->NW = (N + WV - 1) / WV; w->dt = prm->dt;
    w->scans = prm->sequential ? 0 : 1;
    /* the start point and the active-set start are evaluated as the device's active-set kernel
     * evaluates them (one wavefront, knot pairs per lane) when that kernel runs: 64 < N <= 128
     * with the start enabled (csrc/dcm_mpc_ipm.hip launch_dcm_mpc); the IPM iterations always in
     * the wavefront tree of the IPM kernel */
    /* the active-set kernels run for N <= 128 with the polish on (8 or 16 facet slots) */
    const int as_kernel = prm->tol_polish > 0.0 && N <= 2 * WV && !prm->single_kernel && M <= MF;
    w->pairs = (as_kernel && N > WV) ? 1 : 0;
    /* small batches, one knot per lane: the active-set kernels' DPP tree (prm->as_tree) */
    w->dpp = (as_kernel && N <= WV && prm->as_tree) ? 1 : 0;
    w->Qw0 = prm->w_xi[0]; w->Qw1 = prm->w_xi[1];
    w->Rw0 = prm->w_vrp[0]; w->Rw1 = prm->w_vrp[1];
    w->Pw0 = prm->w_terminal[0]; w->Pw1 = prm->w_terminal[1];
    w->omega = omega; w->xi_ref = xi_ref; w->vrp_ref = vrp_ref; w->A = Ain; w->b = bin;
    w->nf = nfacets; w->xi = xi; w->vrp = vrp;
    const size_t per_knot = 5 + 5 * MF + 4 + 3 * 3 + 8 + 6 * 2 + 2 + 2 + 4;
    double* mem = (double*)calloc((size_t)N * per_knot + 4 * (size_t)(N + 1), sizeof(double));
    double* p = mem;
    w->al = p; p += N; w->be = p; p += N; w->a2 = p; p += N; w->b2 = p; p += N; w->ab = p; p += N;
    w->s = p; p += N * MF; w->lam = p; p += N * MF; w->is = p; p += N * MF;
    w->cds = p; p += N * MF; w->cdl = p; p += N * MF;
    w->W = p; p += 4 * N;
    w->E = p; p += 3 * N; w->Pn = p; p += 3 * N; w->h = p; p += 3 * N;
    w->G = p; p += 4 * N; w->Mm = p; p += 4 * N;
    w->rh = p; p += 2 * N; w->g = p; p += 2 * N; w->d = p; p += 2 * N; w->qx = p; p += 2 * N;
    w->dr = p; p += 2 * N; w->dra = p; p += 2 * N;
    w->c = p; p += N; w->q = p; p += N;
    w->sc = p; p += 2 * N; w->sg = p; p += 4 * N;
    w->v = p; p += 2 * (N + 1); w->x = p; p += 2 * (N + 1);

    int status = 0, it = 0, ntot = 0, polished = 0;
    int as_passes = 0;   /* the active-set kernels' drop/add passes (blf_dcm_mpc_solution.passes) */
    w->npass = 0;
    for (int k = 0; k < N; ++k) {
        if (nfacets[k] < 0 || nfacets[k] > M) status = 3;
        else ntot += nfacets[k];
    }
    w->ntot = ntot;
    for (int k = 0; k < N; ++k) {
        w->be[k] = w->dt * omega[k];
        w->al[k] = 1.0 + w->be[k];
        w->a2[k] = w->al[k] * w->al[k];
        w->b2[k] = w->be[k] * w->be[k];
        w->ab[k] = w->al[k] * w->be[k];
        /* start VRP: the warm start's knot k + shift, or (cold start, or a knot new to the
         * window) the reference VRP */
        const int ws = warm && k + warm->shift < N;
        const double* r0 = ws ? warm->vrp + 2 * warm->shift : vrp_ref;
        vrp[2 * k] = r0[2 * k];
        vrp[2 * k + 1] = r0[2 * k + 1];
        for (int i = 0; i < MF; ++i) { w->s[k * MF + i] = 1.0; w->lam[k * MF + i] = 0.0; }
    }
    /* ---- initial point 1: a warm start rolls xi out from its VRPs by the affine forward scan
     *      xi_{k+1} = alpha_k xi_k - beta_k r_k (xi_0 folded into knot 0's element); a cold start
     *      begins at xi = xi_ref (the LQ step below is exact from any trajectory) ---- */
    xi[0] = xi_init[0];
    xi[1] = xi_init[1];
    if (warm) {
        for (int k = 0; k < N; ++k) {
            double* G = w->sg + 4 * k;
            G[0] = w->al[k]; G[1] = 0.0; G[2] = 0.0; G[3] = w->al[k];
            if (k == 0) {
                w->sc[0] = fma(w->al[0], xi_init[0], -(w->be[0] * vrp[0]));
                w->sc[1] = fma(w->al[0], xi_init[1], -(w->be[0] * vrp[1]));
            } else {
                w->sc[2 * k] = -(w->be[k] * vrp[2 * k]);
                w->sc[2 * k + 1] = -(w->be[k] * vrp[2 * k + 1]);
            }
        }
        scan_forward(w, w->sg, 0, w->sc);
        for (int k = 1; k <= N; ++k) { xi[2 * k] = w->x[2 * k]; xi[2 * k + 1] = w->x[2 * k + 1]; }
    } else {
        for (int k = 1; k <= N; ++k) { xi[2 * k] = xi_ref[2 * k]; xi[2 * k + 1] = xi_ref[2 * k + 1]; }
    }
    if (status == 3) goto done;
    /* ---- the active-set kernel's cold start (csrc/dcm_mpc_as.hip): the active
     *      set searched in fp32 (blf_oracle_as32.c, kernel A: float LQ optimum, guess, drop/add
     *      passes), then the fp64 passes (kernel B) from the float point with the facets active
     *      there as the guess;
     *      when they do not certify, the IPM's start from the fp64 LQ optimum below ---- */
    if (!warm && as_kernel) {
        double* r32 = (double*)malloc(sizeof(double) * 4 * (size_t)N);
        double* x32 = r32 + 2 * N;
        int* g32 = (int*)malloc(sizeof(int) * (size_t)N);
        int32_t np32 = 0;
        const int cert32 = orc_as32_search(prm, prm->sequential, xi_init, omega, xi_ref, vrp_ref, Ain,
                                           bin, nfacets, r32, x32, g32, &np32);
        for (int k = 0; k < N; ++k) {
            vrp[2 * k] = r32[2 * k];
            vrp[2 * k + 1] = r32[2 * k + 1];
            xi[2 * (k + 1)] = x32[2 * k];
            xi[2 * (k + 1) + 1] = x32[2 * k + 1];
        }
        /* the fp64 passes' guess: the facets whose slack at a certified float point is below
         * ORC_GUESS_SLACK (kernel kGuessSlack); when the search stopped uncertified (its hand-over,
         * or the pass cap), its next candidate sets as returned in g32 */
        for (int k = 0; k < N && cert32; ++k) {
            int gk = 0;
            for (int i = 0; i < nfacets[k]; ++i) {
                const double* a = Ain + (k * M + i) * 2;
                const double sl = bin[k * M + i] - FD2(a[0], vrp[2 * k], a[1], vrp[2 * k + 1]);
                if (sl < ORC_GUESS_SLACK) gk |= 1 << i;
            }
            g32[k] = gk;
        }
        const int okg = dcm_polish(w, prm->tol_primal, prm->tol_dual, g32, ORC_AS_PASSES, 1);
        as_passes = np32 + w->npass;
        free(r32);
        free(g32);
        if (okg) { polished = 1; status = 0; it = 0; goto done; }
        for (int k = 0; k < N; ++k) {
            vrp[2 * k] = vrp_ref[2 * k];
            vrp[2 * k + 1] = vrp_ref[2 * k + 1];
            xi[2 * (k + 1)] = xi_ref[2 * (k + 1)];
            xi[2 * (k + 1) + 1] = xi_ref[2 * (k + 1) + 1];
        }
    }
    /* ---- initial point 2: one full Newton step of the QP without the polygon constraints
     *      (W = 0, lam = 0): the unconstrained LQ optimum.  For the unstable DCM the rollout is far
     *      from dual feasible (costates grow like alpha^N); this step makes the linear residuals
     *      vanish up to rounding. ---- */
    /*      A warm start skips it: its VRP is a previous optimum, already close. */
    if (!warm) {
        dcm_residuals(w, 0);
        for (int k = 0; k < N; ++k) {
            w->W[4 * k] = 0.0; w->W[4 * k + 1] = 0.0; w->W[4 * k + 2] = 0.0; w->W[4 * k + 3] = 0.0;
            w->g[2 * k] = w->rh[2 * k];
            w->g[2 * k + 1] = w->rh[2 * k + 1];
        }
        if (!dcm_factor(w)) status = 2;
        dcm_solve(w);
        for (int k = 0; k < N; ++k) {
            vrp[2 * k] = vrp[2 * k] + w->dr[2 * k];
            vrp[2 * k + 1] = vrp[2 * k + 1] + w->dr[2 * k + 1];
            xi[2 * (k + 1)] = xi[2 * (k + 1)] + w->x[2 * (k + 1)];
            xi[2 * (k + 1) + 1] = xi[2 * (k + 1) + 1] + w->x[2 * (k + 1) + 1];
        }
    }
    if (status == 2) goto done;
    /* ---- active-set start (DESIGN.md 4 "Polish"): before any IPM iteration, the polish from the
     *      guess "facets the start point violates" (a warm start: also the facets whose previous
     *      multiplier exceeds the floor), with up to ORC_GUESS_PASSES drop/add passes (the cold
     *      starts of the active-set kernel already ran theirs above) ---- */
    if (prm->tol_polish > 0.0 && (warm || !as_kernel)) {
        int* gm = (int*)calloc((size_t)N, sizeof(int));
        for (int k = 0; k < N; ++k) {
            const int ws = warm && k + warm->shift < N;
            for (int i = 0; i < nfacets[k]; ++i) {
                const double* a = Ain + (k * M + i) * 2;
                const double sl = bin[k * M + i] - FD2(a[0], vrp[2 * k], a[1], vrp[2 * k + 1]);
                if (sl < 0.0) gm[k] |= 1 << i;
                if (ws && warm->lambda[(k + warm->shift) * M + i] > warm->floor) gm[k] |= 1 << i;
            }
        }
        const int okg = dcm_polish(w, prm->tol_primal, prm->tol_dual, gm, as_kernel ? ORC_AS_PASSES : ORC_GUESS_PASSES,
                                   as_kernel);
        if (as_kernel) as_passes = w->npass;   /* the warm kernel's passes */
        free(gm);
        if (okg) { polished = 1; status = 0; it = 0; goto done; }
        if (ORC_WARM_RETRY && warm && as_kernel) {
            /* the warm kernel's cold re-solve (csrc/dcm_mpc_as.hip, BLF_WARM_RETRY): a QP its warm
             * passes do not certify is solved again from a cold start (fp32 search, fp64 passes),
             * and the interior point method, if it still needs it, starts cold (kPendingCold) */
            free(mem);
            return orc_dcm_mpc_solve_warm(prm, xi_init, omega, xi_ref, vrp_ref, Ain, bin, nfacets, NULL, xi,
                                          vrp, lam_out, iters_out, polished_out, passes_out);
        }
    }
    /* the interior point method's own start (only when the active-set start did not certify):
     * the start point was restored exactly */

    w->pairs = 0;   /* the IPM kernel's tree from here on */
    w->dpp = 0;
    double dres = 0.0;
    /* ---- after a failed active-set start: the saturated LQ start (dcm_saturated_start) ---- */
    const int sat = prm->tol_polish > 0.0;
    if (sat && !dcm_saturated_start(w, xi_init, prm->tol_primal, &dres)) { status = 2; goto done; }
    /* ---- initial point 3 (the interior point method alone, tol_polish = 0): s = max(b - A r,
     *      1e-2), lam = 1e-2 / s; warm: s = max(b - A r, floor), lam = max(lam_warm[src], floor)
     *      with the same source knot as the VRP ---- */
    for (int k = 0; k < N && !sat; ++k) {
        const int m = nfacets[k];
        const int ws = warm && k + warm->shift < N;
        const double sfloor = ws ? warm->floor : 1e-2;
        double al0 = 0.0, al1 = 0.0;   /* A^T lam */
        for (int i = 0; i < m; ++i) {
            const double* a = Ain + (k * M + i) * 2;
            const double gr = FD2(a[0], vrp[2 * k], a[1], vrp[2 * k + 1]);
            const double sl = bin[k * M + i] - gr;
            w->s[k * MF + i] = sl > sfloor ? sl : sfloor;
            if (ws) {
                const double lw = warm->lambda[(k + warm->shift) * M + i];
                w->lam[k * MF + i] = lw > sfloor ? lw : sfloor;
            } else {
                w->lam[k * MF + i] = 1e-2 / w->s[k * MF + i];   /* centred: s lam = 1e-2 */
            }
            al0 = fma(a[0], w->lam[k * MF + i], al0);
            al1 = fma(a[1], w->lam[k * MF + i], al1);
        }
        /* a cold start sits at the unconstrained optimum, R (r - r_ref) = beta nu: its dual
         * residual is A^T lam exactly */
        if (!warm) dres = nanmax(dres, nanmax(nanmax(0.0, fabs(al0)), fabs(al1)));
    }
    /* ---- initial mu, primal residual, dual residual (a warm start: single-shooting costates
     *      nu_k = qx_k + alpha_k nu_{k+1}, backward scan of v_k = alpha_k nu_{k+1}); each step then
     *      carries them (the QP's linear residuals contract by (1 - a)) ---- */
    double pres = dcm_residuals(w, 1);
    double mu = ntot > 0 ? orc_wave_tree_sum(w->c, N) / (double)ntot : 0.0;
    if (warm && !sat) {
        for (int k = 0; k < N; ++k) {
            double* G = w->sg + 4 * k;
            G[0] = w->al[k]; G[1] = 0.0; G[2] = 0.0; G[3] = w->al[k];
            w->sc[2 * k] = w->al[k] * w->qx[2 * k];
            w->sc[2 * k + 1] = w->al[k] * w->qx[2 * k + 1];
        }
        scan_backward(w, w->sg, w->sc);
        for (int k = 0; k < N; ++k) {
            const double nu0 = w->qx[2 * k] + w->v[2 * (k + 1)];
            const double nu1 = w->qx[2 * k + 1] + w->v[2 * (k + 1) + 1];
            dres = nanmax(dres, fabs(fma(-w->be[k], nu0, w->rh[2 * k])));
            dres = nanmax(dres, fabs(fma(-w->be[k], nu1, w->rh[2 * k + 1])));
        }
    }
    /* mu, pres and dres are known at the top of every iteration without a reduction there: the
     * start computes them, and each step updates them from sums gathered with the step-length
     * maxima (mu: the exact quadratic in the step length; pres, dres: the linear residuals of an
     * exact Newton step contract by (1 - a)) */
    double last_a = 1.0;   /* the previous step length (the stalled-step polish) */
    for (it = 0;; ++it) {
        if (it > 0) dcm_residuals(w, 1);   /* the iterate's gradient, defects, Q (xi - xi_ref) */
        if (!(mu == mu) || !(pres == pres) || !(dres == dres) || isinf(mu)) { status = 2; break; }
        /* the polish at mu <= tol_polish, and (round 6) after a stalled step once mu <= ORC_STALL_MU:
         * on the pushed-robot windows (tests/golden/c5_pushed_windows.npz, multipliers up to 1e9)
         * the iterates stall at mu ~1e-3 with steps of 1e-8..1e-100 while lam > s already names the
         * optimal active set */
        if (prm->tol_polish > 0.0 && (mu <= prm->tol_polish || (last_a < ORC_STALL_STEP && mu <= ORC_STALL_MU))) {
            if (dcm_polish(w, prm->tol_primal, prm->tol_dual, NULL, ORC_GUESS_PASSES, 0)) { polished = 1; status = 0; break; }
            dcm_residuals(w, 1);   /* the iterate's gradient and defects again (the polish reused them) */
        }
        if (mu <= prm->tol_mu && pres <= prm->tol_primal && dres <= prm->tol_dual) { status = 0; break; }
        if (it >= prm->max_iter) { status = 1; break; }

        dcm_wphase(w);
        const int fok = dcm_factor(w);

        /* ---- predictor ---- */
        dcm_solve(w);
        /* affine ratio test with the complementarity sums U0 = sum s lam, U2 = sum ds dl: then
         * mu_aff = ((1 - a) U0 + a^2 U2) / ntot, since s dl + lam ds = -s lam for this step */
        double qmax = 0.0;
        for (int k = 0; k < N; ++k) {
            w->dra[2 * k] = w->dr[2 * k];
            w->dra[2 * k + 1] = w->dr[2 * k + 1];
            const int m = nfacets[k];
            double u0 = 0.0, u2 = 0.0;
            for (int i = 0; i < m; ++i) {
                double ds, dl;
                affine_step(w, k, i, &ds, &dl);
                const double is = w->is[k * MF + i];
                if (ds < 0.0) qmax = keepmax(qmax, (-ds) * is);
                if (dl < 0.0) qmax = keepmax(qmax, (w->s[k * MF + i] + ds) * is);
                u0 = fma(w->s[k * MF + i], w->lam[k * MF + i], u0);
                u2 = fma(ds, dl, u2);
            }
            w->c[k] = u0;
            w->q[k] = u2;
        }
        const double U0 = orc_wave_tree_sum(w->c, N), U2 = orc_wave_tree_sum(w->q, N);
        if (!fok || !(U0 == U0) || !(U2 == U2)) { status = 2; break; }
        const double a_aff = qmax > 1.0 ? 1.0 / qmax : 1.0;
        const double mu_aff = ntot > 0 ? fma(a_aff * a_aff, U2, (1.0 - a_aff) * U0) / (double)ntot : 0.0;
        double sigma = 0.0;
        if (mu > 0.0) {
            const double qq = mu_aff / mu;
            sigma = (qq * qq) * qq;
        }
        const double sigma_mu = sigma * mu;

        /* ---- corrector: rhs (knot-parallel), solve with the same factorization ---- */
        for (int k = 0; k < N; ++k) {
            const int m = nfacets[k];
            const double r0 = vrp[2 * k], r1 = vrp[2 * k + 1];
            double g0 = w->rh[2 * k], g1 = w->rh[2 * k + 1];
            for (int i = 0; i < m; ++i) {
                const double* a = Ain + (k * M + i) * 2;
                const double si = w->s[k * MF + i], li = w->lam[k * MF + i];
                double ds, dl;
                affine_step(w, k, i, &ds, &dl);
                const double rc = FD2(si, li, ds, dl) - sigma_mu;
                const double rpi = (FD2(a[0], r0, a[1], r1) + si) - bin[k * M + i];
                const double e = fma(li, rpi, -rc) * w->is[k * MF + i];
                g0 = fma(a[0], e, g0);
                g1 = fma(a[1], e, g1);
            }
            w->g[2 * k] = g0;
            w->g[2 * k + 1] = g1;
        }
        dcm_solve(w);
        qmax = 0.0;
        for (int k = 0; k < N; ++k) {
            const int m = nfacets[k];
            const double r0 = vrp[2 * k], r1 = vrp[2 * k + 1];
            double t2 = 0.0;
            for (int i = 0; i < m; ++i) {
                const double* a = Ain + (k * M + i) * 2;
                const double si = w->s[k * MF + i], li = w->lam[k * MF + i];
                double ads, adl;
                affine_step(w, k, i, &ads, &adl);
                const double rc = FD2(si, li, ads, adl) - sigma_mu;
                const double rpi = (FD2(a[0], r0, a[1], r1) + si) - bin[k * M + i];
                const double ds = (-rpi) - FD2(a[0], w->dr[2 * k], a[1], w->dr[2 * k + 1]);
                const double dl = fma(-li, ds, -rc) * w->is[k * MF + i];
                if (ds < 0.0) qmax = keepmax(qmax, (-ds) * w->is[k * MF + i]);
                if (dl < 0.0) qmax = keepmax(qmax, (-dl) / li);
                w->cds[k * MF + i] = ds;
                w->cdl[k * MF + i] = dl;
                t2 = fma(ds, dl, t2);
            }
            w->q[k] = t2;
        }
        const double T2 = orc_wave_tree_sum(w->q, N);
        const double step = qmax > 0.0 ? 0.99 / qmax : 1.0;
        const double a = step < 1.0 ? step : 1.0;
        for (int k = 0; k < N; ++k) {
            vrp[2 * k] = fma(a, w->dr[2 * k], vrp[2 * k]);
            vrp[2 * k + 1] = fma(a, w->dr[2 * k + 1], vrp[2 * k + 1]);
            xi[2 * (k + 1)] = fma(a, w->x[2 * (k + 1)], xi[2 * (k + 1)]);
            xi[2 * (k + 1) + 1] = fma(a, w->x[2 * (k + 1) + 1], xi[2 * (k + 1) + 1]);
            const int m = nfacets[k];
            for (int i = 0; i < m; ++i) {
                w->s[k * MF + i] = fma(a, w->cds[k * MF + i], w->s[k * MF + i]);
                w->lam[k * MF + i] = fma(a, w->cdl[k * MF + i], w->lam[k * MF + i]);
            }
        }
#ifdef ORC_TRACE
        {
            int nact = 0; double lmax = 0.0;
            for (int k = 0; k < N; ++k) for (int i = 0; i < nfacets[k]; ++i) {
                nact += w->lam[k * MF + i] > w->s[k * MF + i];
                lmax = fmax(lmax, w->lam[k * MF + i]); }
            fprintf(stderr, "it %d mu %.3g a_aff %.3g a %.3g sigma %.3g pres %.3g dres %.3g nact %d lmax %.3g\n",
                    it, mu, a_aff, a, sigma, pres, dres, nact, lmax);
        }
#endif
        dres = dres * (1.0 - a);
        pres = pres * (1.0 - a);
        last_a = a;
        /* sum (s + a ds)(lam + a dl) = U0 + a T1 + a^2 T2 with T1 = sum (s dl + lam ds) = -sum rc
         * = -(U0 + U2 - ntot sigma mu) for the corrector step */
        if (ntot > 0) {
            const double nt = (double)ntot;
            mu = fma(a * a, T2, fma(a, fma(nt, sigma_mu, -U2), (1.0 - a) * U0)) / nt;
        }
    }
done:
    if (iters_out) *iters_out = it;
    if (polished_out) *polished_out = polished;
    if (passes_out) *passes_out = as_passes;
#ifdef ORC_STATS   /* diagnostic builds only: the solve's IPM iterations and all polish passes */
    fprintf(stderr, "ORC_STATS it %d as_passes %d all_polish_passes %d status %d\n", it, as_passes, w->npass, status);
#endif
    if (lam_out) {   /* final multipliers, [N][M], zero in unused facet slots */
        for (int k = 0; k < N; ++k)
            for (int i = 0; i < M; ++i)
                lam_out[k * M + i] = (i < nfacets[k] && nfacets[k] <= M) ? w->lam[k * MF + i] : 0.0;
    }
    free(mem);
    return status;
}

/* ---- batch driver with POSIX threads (CPU baseline) ---- */
typedef struct {
    const orc_dcm_params* prm;
    int64_t batch;
    const double *xi_init, *omega, *xi_ref, *vrp_ref, *A, *b;
    const int32_t* nfacets;
    const double *vrp_ws, *lam_ws;
    const int32_t* prev_status;
    int32_t shift;
    double floor;
    double *xi, *vrp, *lam_out;
    int32_t *status, *iters, *polished, *passes;
    atomic_llong next;
} batch_job;

static void* batch_worker(void* arg)
{
    batch_job* J = (batch_job*)arg;
    const int N = J->prm->horizon, M = J->prm->max_facets;
    for (;;) {
        const long long p = atomic_fetch_add(&J->next, 1);
        if (p >= J->batch) break;
        orc_dcm_warm wm;
        const orc_dcm_warm* wp = NULL;
        /* a problem whose previous solve failed starts cold (blf_dcm_mpc_warm_start.prev_status) */
        if (J->vrp_ws && !(J->prev_status && J->prev_status[p] != 0)) {
            wm.vrp = J->vrp_ws + (int64_t)2 * N * p;
            wm.lambda = J->lam_ws + (int64_t)N * M * p;
            wm.shift = J->shift;
            wm.reserved = 0;
            wm.floor = J->floor;
            wp = &wm;
        }
        J->status[p] = orc_dcm_mpc_solve_warm(
            J->prm, J->xi_init + 2 * p, J->omega + (int64_t)N * p,
            J->xi_ref + (int64_t)2 * (N + 1) * p, J->vrp_ref + (int64_t)2 * N * p,
            J->A + (int64_t)2 * N * M * p, J->b + (int64_t)N * M * p, J->nfacets + (int64_t)N * p,
            wp, J->xi + (int64_t)2 * (N + 1) * p, J->vrp + (int64_t)2 * N * p,
            J->lam_out ? J->lam_out + (int64_t)N * M * p : NULL, J->iters + p,
            J->polished ? J->polished + p : NULL, J->passes ? J->passes + p : NULL);
    }
    return NULL;
}

static void run_batch(batch_job* J, int threads)
{
    atomic_init(&J->next, 0);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    for (int t = 1; t < threads; ++t) pthread_create(&th[t], NULL, batch_worker, J);
    batch_worker(J);
    for (int t = 1; t < threads; ++t) pthread_join(th[t], NULL);
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
    run_batch(&J, threads);
}

void orc_dcm_mpc_solve_batch_warm(const orc_dcm_params* prm, int64_t batch, int threads,
                                  const double* xi_init, const double* omega, const double* xi_ref,
                                  const double* vrp_ref, const double* A, const double* b,
                                  const int32_t* nfacets, const double* vrp_ws,
                                  const double* lam_ws, const int32_t* prev_status, int32_t shift,
                                  double floor, double* xi, double* vrp, double* lam_out,
                                  int32_t* status, int32_t* iters, int32_t* polished, int32_t* passes)
{
    batch_job J = {.prm = prm, .batch = batch, .xi_init = xi_init, .omega = omega,
                   .xi_ref = xi_ref, .vrp_ref = vrp_ref, .A = A, .b = b, .nfacets = nfacets,
                   .vrp_ws = vrp_ws, .lam_ws = lam_ws, .prev_status = prev_status, .shift = shift,
                   .floor = floor,
                   .xi = xi, .vrp = vrp, .lam_out = lam_out, .status = status, .iters = iters,
                   .polished = polished, .passes = passes};
    run_batch(&J, threads);
}
