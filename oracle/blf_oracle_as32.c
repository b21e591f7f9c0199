/* TEST INFRASTRUCTURE ONLY (oracle): the fp32 active-set search of a cold start, as the device's
 * active-set kernel evaluates it (bipedal-locomotion-framework_amd/csrc/dcm_mpc_as.hip, phase A;
 * DESIGN.md section 4, item 7).  Build-defined algorithm (A1 of SURVEY.md 8(a) is absent from the
 * reference, so this is a restatement of this build's own kernel, not of reference code).
 *
 * The search runs the LQ optimum, the guess (the facets it violates) and up to ORC_GUESS_PASSES
 * drop/add passes entirely in float, with the kernel's operations in the kernel's order: every
 * expression below is the float instance of the templated device code, lane by lane (lane l owns
 * knot l for N <= 64, the knot pair 2l, 2l + 1 for 64 < N <= 128), the scans in the same
 * tree (Kogge-Stone, or the DPP tree for small batches).  C float arithmetic with fmaf and IEEE division rounds exactly like the
 * device's v_fma_f32 / correctly rounded division, and the fp64 -> fp32 conversions round to
 * nearest on both sides, so the search's outputs are bit-identical to the kernel's.
 * `sequential` = 1 evaluates the same search with plain recursions (CPU baseline only). */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "blf_oracle.h"

#define WV 64
#ifndef ORC_GUESS_PASSES
#define ORC_GUESS_PASSES 8
#endif
#define PASSES ORC_GUESS_PASSES   /* kernel kGuessPasses */
#define SEARCH_TOL_P 1e-5f       /* kernel kSearchTolP */
#define SEARCH_TOL_D 1e-4f       /* kernel kSearchTolD */
#define F2(a, b, c, d) fmaf((a), (b), (c) * (d))
#define F3(a, b, c, d, e) fmaf((a), (b), fmaf((c), (d), (e)))

typedef struct { float dt, Qw0, Qw1, Rw0, Rw1, Pw0, Pw1, tol_p, tol_d; } pf_t;
typedef struct { float a0, a1, a2, a3, g0, g1, g2, h0, h1, h2; } rcf;

#ifndef ORC_RC_FORM   /* the kernel's BLF_RC_FORM (dcm_qp_common.h) */
#define ORC_RC_FORM 2
#endif

typedef struct {
    int N, M, KPL, seq, dpp;   /* dpp: the DPP scan tree (orc_dcm_params.as_tree) */
    pf_t P;
    const double *A, *b;
    int m[2 * WV], gm[2 * WV], drop[2 * WV], add[2 * WV];
    float r0[2 * WV], r1[2 * WV], x0[2 * WV], x1[2 * WV], w[2 * WV], al[2 * WV], be[2 * WV];
    float rh0[2 * WV], rh1[2 * WV], d0[2 * WV], d1[2 * WV], qx0[2 * WV], qx1[2 * WV];
    float P00[2 * WV], P01[2 * WV], P11[2 * WV], h00[2 * WV], h01[2 * WV], h11[2 * WV];
    float rr0[2 * WV], rr1[2 * WV], xr0[2 * WV], xr1[2 * WV];
    float xi00, xi01;
    int npass;   /* the passes run (the kernel's as_passes npass) */
} s32;

/* facet row i of knot k, rounded to float */
static void rowf(const s32* s, int k, int i, float* ax, float* ay, float* bb)
{
    const double* a = s->A + ((size_t)k * s->M + i) * 2;
    *ax = (float)a[0];
    *ay = (float)a[1];
    *bb = (float)s->b[(size_t)k * s->M + i];
}

/* ---- the Riccati map elements (rc_combine / rc_apply of dcm_qp_common.h, float) ---- */
static int rcf_combine(rcf* e, const rcf* q)
{
    const float one = 1.0f;
    const float T00 = F3(e->g0, q->h0, e->g1, q->h1, one);
    const float T01 = F2(e->g0, q->h1, e->g1, q->h2);
    const float T10 = F2(e->g1, q->h0, e->g2, q->h1);
    const float T11 = F3(e->g1, q->h1, e->g2, q->h2, one);
    const float detT = fmaf(T00, T11, -(T01 * T10));
    const int ok = (detT > 0.0f) && !isinf(detT);
    const float it = one / detT;
#if ORC_RC_FORM >= 2
    {
        /* adj(T) = [T11, -T01; -T10, T00]: the products run beside the division (rc_combine of
         * dcm_qp_common.h, BLF_RC_FORM) */
        const float Up00 = F2(T11, e->a0, -T01, e->a2);
        const float Up01 = F2(T11, e->a1, -T01, e->a3);
        const float Up10 = F2(-T10, e->a0, T00, e->a2);
        const float Up11 = F2(-T10, e->a1, T00, e->a3);
        const float Vp00 = F2(q->a0, T11, q->a1, -T10);
        const float Vp01 = F2(q->a0, -T01, q->a1, T00);
        const float Vp10 = F2(q->a2, T11, q->a3, -T10);
        const float Vp11 = F2(q->a2, -T01, q->a3, T00);
        const float Xp00 = F2(Vp00, e->g0, Vp01, e->g1);
        const float Xp01 = F2(Vp00, e->g1, Vp01, e->g2);
        const float Xp10 = F2(Vp10, e->g0, Vp11, e->g1);
        const float Xp11 = F2(Vp10, e->g1, Vp11, e->g2);
        const float Y00 = F2(q->h0, e->a0, q->h1, e->a2);
        const float Y01 = F2(q->h0, e->a1, q->h1, e->a3);
        const float Y10 = F2(q->h1, e->a0, q->h2, e->a2);
        const float Y11 = F2(q->h1, e->a1, q->h2, e->a3);
        const float gp0 = F2(Xp00, q->a0, Xp01, q->a1);
        const float gp1 = F2(Xp00, q->a2, Xp01, q->a3);
        const float gp2 = F2(Xp10, q->a2, Xp11, q->a3);
        rcf r;
#if ORC_RC_FORM == 2
        const float U00 = Up00 * it, U01 = Up01 * it, U10 = Up10 * it, U11 = Up11 * it;
        r.a0 = F2(q->a0, U00, q->a1, U10);
        r.a1 = F2(q->a0, U01, q->a1, U11);
        r.a2 = F2(q->a2, U00, q->a3, U10);
        r.a3 = F2(q->a2, U01, q->a3, U11);
        r.h0 = F3(U00, Y00, U10, Y10, e->h0);
        r.h1 = F3(U00, Y01, U10, Y11, e->h1);
        r.h2 = F3(U01, Y01, U11, Y11, e->h2);
#else
        r.a0 = F2(q->a0, Up00, q->a1, Up10) * it;
        r.a1 = F2(q->a0, Up01, q->a1, Up11) * it;
        r.a2 = F2(q->a2, Up00, q->a3, Up10) * it;
        r.a3 = F2(q->a2, Up01, q->a3, Up11) * it;
        r.h0 = fmaf(F2(Up00, Y00, Up10, Y10), it, e->h0);
        r.h1 = fmaf(F2(Up00, Y01, Up10, Y11), it, e->h1);
        r.h2 = fmaf(F2(Up01, Y01, Up11, Y11), it, e->h2);
#endif
        r.g0 = fmaf(gp0, it, q->g0);
        r.g1 = fmaf(gp1, it, q->g1);
        r.g2 = fmaf(gp2, it, q->g2);
        *e = r;
        return ok;
    }
#endif
    const float Ti00 = T11 * it, Ti01 = -(T01 * it), Ti10 = -(T10 * it), Ti11 = T00 * it;
    const float U00 = F2(Ti00, e->a0, Ti01, e->a2);
    const float U01 = F2(Ti00, e->a1, Ti01, e->a3);
    const float U10 = F2(Ti10, e->a0, Ti11, e->a2);
    const float U11 = F2(Ti10, e->a1, Ti11, e->a3);
    const float V00 = F2(q->a0, Ti00, q->a1, Ti10);
    const float V01 = F2(q->a0, Ti01, q->a1, Ti11);
    const float V10 = F2(q->a2, Ti00, q->a3, Ti10);
    const float V11 = F2(q->a2, Ti01, q->a3, Ti11);
    const float X00 = F2(V00, e->g0, V01, e->g1);
    const float X01 = F2(V00, e->g1, V01, e->g2);
    const float X10 = F2(V10, e->g0, V11, e->g1);
    const float X11 = F2(V10, e->g1, V11, e->g2);
    const float Y00 = F2(q->h0, e->a0, q->h1, e->a2);
    const float Y01 = F2(q->h0, e->a1, q->h1, e->a3);
    const float Y10 = F2(q->h1, e->a0, q->h2, e->a2);
    const float Y11 = F2(q->h1, e->a1, q->h2, e->a3);
    rcf r;
    r.a0 = F2(q->a0, U00, q->a1, U10);
    r.a1 = F2(q->a0, U01, q->a1, U11);
    r.a2 = F2(q->a2, U00, q->a3, U10);
    r.a3 = F2(q->a2, U01, q->a3, U11);
    r.g0 = F3(X00, q->a0, X01, q->a1, q->g0);
    r.g1 = F3(X00, q->a2, X01, q->a3, q->g1);
    r.g2 = F3(X10, q->a2, X11, q->a3, q->g2);
    r.h0 = F3(U00, Y00, U10, Y10, e->h0);
    r.h1 = F3(U00, Y01, U10, Y11, e->h1);
    r.h2 = F3(U01, Y01, U11, Y11, e->h2);
    *e = r;
    return ok;
}

static int rcf_apply(const rcf* e, float P00, float P01, float P11, float* o)
{
    const float one = 1.0f;
    const float S00 = F3(e->g0, P00, e->g1, P01, one);
    const float S01 = F2(e->g0, P01, e->g1, P11);
    const float S10 = F2(e->g1, P00, e->g2, P01);
    const float S11 = F3(e->g1, P01, e->g2, P11, one);
    const float detS = fmaf(S00, S11, -(S01 * S10));
    const int ok = (detS > 0.0f) && !isinf(detS);
    const float is = one / detS;
#if ORC_RC_FORM >= 1
    {
        /* W' = P adj(S), Z' = W' A, out = (A^T Z') / det(S) + H (rc_apply, BLF_RC_FORM) */
        const float Wp00 = F2(P00, S11, P01, -S10);
        const float Wp01 = F2(P00, -S01, P01, S00);
        const float Wp10 = F2(P01, S11, P11, -S10);
        const float Wp11 = F2(P01, -S01, P11, S00);
        const float Zp00 = F2(Wp00, e->a0, Wp01, e->a2);
        const float Zp01 = F2(Wp00, e->a1, Wp01, e->a3);
        const float Zp10 = F2(Wp10, e->a0, Wp11, e->a2);
        const float Zp11 = F2(Wp10, e->a1, Wp11, e->a3);
        o[0] = fmaf(F2(e->a0, Zp00, e->a2, Zp10), is, e->h0);
        o[1] = fmaf(F2(e->a0, Zp01, e->a2, Zp11), is, e->h1);
        o[2] = fmaf(F2(e->a1, Zp01, e->a3, Zp11), is, e->h2);
        return ok;
    }
#endif
    const float Si00 = S11 * is, Si01 = -(S01 * is), Si10 = -(S10 * is), Si11 = S00 * is;
    const float W00 = F2(P00, Si00, P01, Si10);
    const float W01 = F2(P00, Si01, P01, Si11);
    const float W10 = F2(P01, Si00, P11, Si10);
    const float W11 = F2(P01, Si01, P11, Si11);
    const float Z00 = F2(W00, e->a0, W01, e->a2);
    const float Z01 = F2(W00, e->a1, W01, e->a3);
    const float Z10 = F2(W10, e->a0, W11, e->a2);
    const float Z11 = F2(W10, e->a1, W11, e->a3);
    o[0] = F3(e->a0, Z00, e->a2, Z10, e->h0);
    o[1] = F3(e->a0, Z01, e->a2, Z11, e->h1);
    o[2] = F3(e->a1, Z01, e->a3, Z11, e->h2);
    return ok;
}

static void rcf_knot(const s32* s, int k, const float (*E)[3], rcf* e)
{
    if (k < s->N) {
        e->a0 = s->al[k]; e->a1 = 0.0f; e->a2 = 0.0f; e->a3 = s->al[k];
        e->g0 = E[k][0]; e->g1 = E[k][1]; e->g2 = E[k][2];
        e->h0 = s->P.Qw0; e->h1 = 0.0f; e->h2 = s->P.Qw1;
    } else {
        e->a0 = 1.0f; e->a1 = 0.0f; e->a2 = 0.0f; e->a3 = 1.0f;
        e->g0 = e->g1 = e->g2 = 0.0f;
        e->h0 = e->h1 = e->h2 = 0.0f;
    }
}

/* as_riccati: P_{k+1} of every knot into s->P..; returns 0 when some pivot is not positive */
static int riccati32(s32* s, const float (*E)[3])
{
    const int N = s->N, KPL = s->KPL;
    int ok = 1;
    if (s->seq) {
        float Pn[3] = {s->P.Pw0, 0.0f, s->P.Pw1};
        s->P00[N - 1] = Pn[0]; s->P01[N - 1] = Pn[1]; s->P11[N - 1] = Pn[2];
        for (int k = N - 1; k >= 1; --k) {
            rcf e;
            rcf_knot(s, k, E, &e);
            float o[3];
            if (!rcf_apply(&e, Pn[0], Pn[1], Pn[2], o)) ok = 0;
            s->P00[k - 1] = o[0]; s->P01[k - 1] = o[1]; s->P11[k - 1] = o[2];
            Pn[0] = o[0]; Pn[1] = o[1]; Pn[2] = o[2];
        }
        return ok;
    }
    rcf e[WV], ne[WV];
    for (int l = 0; l < WV; ++l) {
        rcf_knot(s, KPL * l, E, &e[l]);
        if (KPL == 2) {
            rcf e1;
            rcf_knot(s, 2 * l + 1, E, &e1);
            if (!rcf_combine(&e[l], &e1)) ok = 0;
        }
    }
    const int pad = KPL == 2 && N <= 2 * WV - 2;   /* the kernel's as_pad: lane WV - 1's identity */
    for (int L = 0; s->dpp && L < 6; ++L) {   /* the DPP tree (orc_lane_src) */
        for (int l = 0; l < WV; ++l) {
            const int src = orc_lane_src(L, 0, l);
            ne[l] = e[l];
            if (src >= 0 && !rcf_combine(&ne[l], &e[src])) ok = 0;
        }
        memcpy(e, ne, sizeof(e));
    }
    for (int d = 1; !s->dpp && d < WV; d <<= 1) {
        for (int l = 0; l < WV; ++l) {
            ne[l] = e[l];
            if (l + d < WV) {
                if (!rcf_combine(&ne[l], &e[l + d])) ok = 0;
            } else if (pad && !rcf_combine(&ne[l], &e[WV - 1])) {
                ok = 0;
            }
        }
        memcpy(e, ne, sizeof(e));
    }
    float P0[WV][3];
    for (int l = 0; l < WV; ++l)
        if (!rcf_apply(&e[l], s->P.Pw0, 0.0f, s->P.Pw1, P0[l])) ok = 0;
    for (int l = 0; l < WV; ++l) {
        float Pn[3] = {s->P.Pw0, 0.0f, s->P.Pw1};
        if (l + 1 < WV) { Pn[0] = P0[l + 1][0]; Pn[1] = P0[l + 1][1]; Pn[2] = P0[l + 1][2]; }
        const int kl = KPL * l + KPL - 1;   /* the lane's last knot takes P from the next lane */
        s->P00[kl] = Pn[0]; s->P01[kl] = Pn[1]; s->P11[kl] = Pn[2];
        if (KPL == 2) {
            rcf e1;
            rcf_knot(s, 2 * l + 1, E, &e1);
            float o[3];
            if (!rcf_apply(&e1, Pn[0], Pn[1], Pn[2], o)) ok = 0;
            s->P00[2 * l] = o[0]; s->P01[2 * l] = o[1]; s->P11[2 * l] = o[2];
        }
    }
    s->P00[N - 1] = s->P.Pw0; s->P01[N - 1] = 0.0f; s->P11[N - 1] = s->P.Pw1;
    return ok;
}

/* (a, e) <- (a b, a c + e): the device's COMPOSE */
static void compose(float* a, float* e, const float* b, const float* c)
{
    const float n0 = F2(a[0], b[0], a[1], b[2]);
    const float n1 = F2(a[0], b[1], a[1], b[3]);
    const float n2 = F2(a[2], b[0], a[3], b[2]);
    const float n3 = F2(a[2], b[1], a[3], b[3]);
    const float m0 = F3(a[0], c[0], a[1], c[1], e[0]);
    const float m1 = F3(a[2], c[0], a[3], c[1], e[1]);
    a[0] = n0; a[1] = n1; a[2] = n2; a[3] = n3; e[0] = m0; e[1] = m1;
}

/* the DPP tree over the 64 lane elements (g, e): a lane combines with its level's source lane's
 * element when it has one (orc_lane_src >= 0) */
static void aff_tree32(float (*g)[4], float (*e)[2], int fwd)
{
    float ng[WV][4], ne[WV][2];
    for (int L = 0; L < 6; ++L) {
        for (int l = 0; l < WV; ++l) {
            const int src = orc_lane_src(L, fwd, l);
            memcpy(ng[l], g[l], sizeof(ng[l]));
            memcpy(ne[l], e[l], sizeof(ne[l]));
            if (src >= 0) compose(ng[l], ne[l], g[src], e[src]);
        }
        memcpy(g, ng, sizeof(ng));
        memcpy(e, ne, sizeof(ne));
    }
}

/* as_scan_backward: vn[k] = v_{k+1} for v_k = G_k v_{k+1} + c_k, v_N = 0 (every knot < 2 WV) */
static void scan_backward32(const s32* s, float (*G)[4], float (*c)[2], float (*vn)[2])
{
    const int N = s->N, KPL = s->KPL;
    if (s->seq) {
        float v0 = 0.0f, v1 = 0.0f;
        for (int k = N - 1; k >= 0; --k) {
            vn[k][0] = v0; vn[k][1] = v1;
            const float n0 = F3(G[k][0], v0, G[k][1], v1, c[k][0]);
            const float n1 = F3(G[k][2], v0, G[k][3], v1, c[k][1]);
            v0 = n0; v1 = n1;
        }
        return;
    }
    float g[WV][4], e[WV][2], ng[WV][4], ne[WV][2];
    for (int l = 0; l < WV; ++l) {
        memcpy(g[l], G[KPL * l], sizeof(g[l]));
        memcpy(e[l], c[KPL * l], sizeof(e[l]));
        if (KPL == 2) compose(g[l], e[l], G[2 * l + 1], c[2 * l + 1]);
    }
    const int pad = KPL == 2 && N <= 2 * WV - 2;   /* lane WV - 1's zero element (kernel as_pad) */
    if (s->dpp) aff_tree32(g, e, 0);
    for (int d = 1; !s->dpp && d < WV; d <<= 1) {
        for (int l = 0; l < WV; ++l) {
            memcpy(ng[l], g[l], sizeof(ng[l]));
            memcpy(ne[l], e[l], sizeof(ne[l]));
            if (l + d < WV) compose(ng[l], ne[l], g[l + d], e[l + d]);
            else if (pad) compose(ng[l], ne[l], g[WV - 1], e[WV - 1]);
        }
        memcpy(g, ng, sizeof(g));
        memcpy(e, ne, sizeof(e));
    }
    for (int l = 0; l < WV; ++l) {
        const float vb0 = l + 1 < WV ? e[l + 1][0] : 0.0f, vb1 = l + 1 < WV ? e[l + 1][1] : 0.0f;
        if (KPL == 2) {
            const int k1 = 2 * l + 1;
            vn[2 * l][0] = F3(G[k1][0], vb0, G[k1][1], vb1, c[k1][0]);
            vn[2 * l][1] = F3(G[k1][2], vb0, G[k1][3], vb1, c[k1][1]);
            vn[k1][0] = vb0;
            vn[k1][1] = vb1;
        } else {
            vn[l][0] = vb0;
            vn[l][1] = vb1;
        }
    }
}

/* as_scan_forward: x[k] = x_{k+1}, xk[k] = x_k of x_{k+1} = F_k x_k + f_k, x_0 = 0 */
static void scan_forward32(const s32* s, float (*F)[4], float (*f)[2], float (*x)[2], float (*xk)[2])
{
    const int N = s->N, KPL = s->KPL;
    if (s->seq) {
        float v0 = 0.0f, v1 = 0.0f;
        for (int k = 0; k < N; ++k) {
            xk[k][0] = v0; xk[k][1] = v1;
            const float n0 = F3(F[k][0], v0, F[k][1], v1, f[k][0]);
            const float n1 = F3(F[k][2], v0, F[k][3], v1, f[k][1]);
            v0 = n0; v1 = n1;
            x[k][0] = v0; x[k][1] = v1;
        }
        return;
    }
    float g[WV][4], e[WV][2], ng[WV][4], ne[WV][2];
    const int L = KPL - 1;
    for (int l = 0; l < WV; ++l) {
        memcpy(g[l], F[KPL * l + L], sizeof(g[l]));
        memcpy(e[l], f[KPL * l + L], sizeof(e[l]));
        if (KPL == 2) compose(g[l], e[l], F[2 * l], f[2 * l]);
    }
    const int pad = KPL == 2 && N <= 2 * WV - 2;   /* lane WV - 1's zero element (kernel as_pad) */
    if (s->dpp) aff_tree32(g, e, 1);
    for (int d = 1; !s->dpp && d < WV; d <<= 1) {
        for (int l = 0; l < WV; ++l) {
            memcpy(ng[l], g[l], sizeof(ng[l]));
            memcpy(ne[l], e[l], sizeof(ne[l]));
            if (l >= d) compose(ng[l], ne[l], g[l - d], e[l - d]);
            else if (pad) compose(ng[l], ne[l], g[WV - 1], e[WV - 1]);
        }
        memcpy(g, ng, sizeof(g));
        memcpy(e, ne, sizeof(e));
    }
    for (int l = 0; l < WV; ++l) {
        const float xb0 = l > 0 ? e[l - 1][0] : 0.0f, xb1 = l > 0 ? e[l - 1][1] : 0.0f;
        xk[KPL * l][0] = xb0;
        xk[KPL * l][1] = xb1;
        if (KPL == 2) {
            const int k0 = 2 * l;
            const float x10 = F3(F[k0][0], xb0, F[k0][1], xb1, f[k0][0]);
            const float x11 = F3(F[k0][2], xb0, F[k0][3], xb1, f[k0][1]);
            x[k0][0] = x10; x[k0][1] = x11;
            xk[k0 + 1][0] = x10; xk[k0 + 1][1] = x11;
        }
        x[KPL * l + L][0] = e[l][0];
        x[KPL * l + L][1] = e[l][1];
    }
}

/* as_residuals */
static void residuals32(s32* s, int k, float xk0, float xk1)
{
    const pf_t* P = &s->P;
    s->rh0[k] = P->Rw0 * (s->r0[k] - s->rr0[k]);
    s->rh1[k] = P->Rw1 * (s->r1[k] - s->rr1[k]);
    const float dx0 = F2(s->w[k], xk0, -s->w[k], s->r0[k]);
    s->d0[k] = fmaf(dx0, P->dt, xk0) - s->x0[k];
    const float dx1 = F2(s->w[k], xk1, -s->w[k], s->r1[k]);
    s->d1[k] = fmaf(dx1, P->dt, xk1) - s->x1[k];
    const int last = k == s->N - 1;
    const float q0 = last ? P->Pw0 : P->Qw0;
    const float q1 = last ? P->Pw1 : P->Qw1;
    s->qx0[k] = q0 * (s->x0[k] - s->xr0[k]);
    s->qx1[k] = q1 * (s->x1[k] - s->xr1[k]);
}

static void xi_prev32(const s32* s, float (*xk)[2])
{
    for (int k = 0; k < s->N; ++k) {
        xk[k][0] = k == 0 ? s->xi00 : s->x0[k - 1];
        xk[k][1] = k == 0 ? s->xi01 : s->x1[k - 1];
    }
}

/* as_solve for g = rh: dr, dx (xi_{k+1} step), vn (v_{k+1}) of every knot */
static void solve32(const s32* s, float (*dr)[2], float (*dx)[2], float (*vn)[2])
{
    const int N = s->N;
    static __thread float G[2 * WV][4], Gt[2 * WV][4], c[2 * WV][2], y[2 * WV][2], kf[2 * WV][2],
        f[2 * WV][2], xk[2 * WV][2];
    for (int k = 0; k < 2 * WV; ++k) {
        G[k][0] = G[k][1] = G[k][2] = G[k][3] = 0.0f;
        c[k][0] = c[k][1] = y[k][0] = y[k][1] = 0.0f;
        if (k < N) {
            const float b2 = s->be[k] * s->be[k];
            const float ab = s->al[k] * s->be[k];
            const float m00 = F2(s->P00[k], s->h00[k], s->P01[k], s->h01[k]);
            const float m01 = F2(s->P00[k], s->h01[k], s->P01[k], s->h11[k]);
            const float m10 = F2(s->P01[k], s->h00[k], s->P11[k], s->h01[k]);
            const float m11 = F2(s->P01[k], s->h01[k], s->P11[k], s->h11[k]);
            y[k][0] = F3(s->P00[k], s->d0[k], s->P01[k], s->d1[k], s->qx0[k]);
            y[k][1] = F3(s->P01[k], s->d0[k], s->P11[k], s->d1[k], s->qx1[k]);
            const float Mg0 = F2(m00, s->rh0[k], m01, s->rh1[k]);
            const float Mg1 = F2(m10, s->rh0[k], m11, s->rh1[k]);
            G[k][0] = s->al[k] * fmaf(-b2, m00, 1.0f);
            G[k][1] = -(s->al[k] * (b2 * m01));
            G[k][2] = -(s->al[k] * (b2 * m10));
            G[k][3] = s->al[k] * fmaf(-b2, m11, 1.0f);
            c[k][0] = F3(G[k][0], y[k][0], G[k][1], y[k][1], ab * Mg0);
            c[k][1] = F3(G[k][2], y[k][0], G[k][3], y[k][1], ab * Mg1);
        }
        Gt[k][0] = G[k][0]; Gt[k][1] = G[k][2]; Gt[k][2] = G[k][1]; Gt[k][3] = G[k][3];
    }
    scan_backward32(s, G, c, vn);
    for (int k = 0; k < 2 * WV; ++k) {
        kf[k][0] = kf[k][1] = f[k][0] = f[k][1] = 0.0f;
        if (k < N) {
            const float t0 = y[k][0] + vn[k][0];
            const float t1 = y[k][1] + vn[k][1];
            const float hu0 = fmaf(-s->be[k], t0, s->rh0[k]);
            const float hu1 = fmaf(-s->be[k], t1, s->rh1[k]);
            kf[k][0] = -F2(s->h00[k], hu0, s->h01[k], hu1);
            kf[k][1] = -F2(s->h01[k], hu0, s->h11[k], hu1);
            f[k][0] = fmaf(-s->be[k], kf[k][0], s->d0[k]);
            f[k][1] = fmaf(-s->be[k], kf[k][1], s->d1[k]);
        }
    }
    scan_forward32(s, Gt, f, dx, xk);
    for (int k = 0; k < N; ++k) {
        const float ab = s->al[k] * s->be[k];
        const float m00 = F2(s->P00[k], s->h00[k], s->P01[k], s->h01[k]);
        const float m01 = F2(s->P00[k], s->h01[k], s->P01[k], s->h11[k]);
        const float m10 = F2(s->P01[k], s->h00[k], s->P11[k], s->h01[k]);
        const float m11 = F2(s->P01[k], s->h01[k], s->P11[k], s->h11[k]);
        dr[k][0] = fmaf(ab, F2(m00, xk[k][0], m10, xk[k][1]), kf[k][0]);
        dr[k][1] = fmaf(ab, F2(m01, xk[k][0], m11, xk[k][1]), kf[k][1]);
    }
}

/* as_lq_step (the numerical flag is not used by the search) */
static void lq_step32(s32* s)
{
    const int N = s->N;
    const pf_t* P = &s->P;
    static __thread float xk[2 * WV][2], E[2 * WV][3], dr[2 * WV][2], dx[2 * WV][2], vn[2 * WV][2];
    xi_prev32(s, xk);
    for (int k = 0; k < N; ++k) residuals32(s, k, xk[k][0], xk[k][1]);
    for (int k = 0; k < 2 * WV; ++k) {
        E[k][0] = E[k][1] = E[k][2] = 0.0f;
        if (k < N) {
            const float b2 = s->be[k] * s->be[k];
            const float W00 = 0.0f, W01 = 0.0f, W11 = 0.0f, dW = 0.0f;
            const float detRW = fmaf(P->Rw0, P->Rw1, F2(P->Rw1, W00, P->Rw0, W11)) + dW;
            const float ie = b2 / detRW;
            E[k][0] = (P->Rw1 + W11) * ie;
            E[k][1] = -(W01 * ie);
            E[k][2] = (P->Rw0 + W00) * ie;
        }
    }
    riccati32(s, (const float (*)[3])E);
    for (int k = 0; k < N; ++k) {
        const float b2 = s->be[k] * s->be[k];
        const float W00 = 0.0f, W01 = 0.0f, W11 = 0.0f, dW = 0.0f;
        const float B00 = fmaf(b2, s->P00[k], P->Rw0);
        const float B01 = b2 * s->P01[k];
        const float B11 = fmaf(b2, s->P11[k], P->Rw1);
        const float H00 = B00 + W00, H01 = B01 + W01, H11 = B11 + W11;
        const float detB = fmaf(B00, B11, -(B01 * B01));
        const float trW = F2(B11, W00, B00, W11) - 2.0f * (B01 * W01);
        const float det = (detB + trW) + dW;
        const float idet = 1.0f / det;
        s->h00[k] = H11 * idet;
        s->h01[k] = -(H01 * idet);
        s->h11[k] = H00 * idet;
    }
    solve32(s, dr, dx, vn);
    for (int k = 0; k < N; ++k) {
        s->r0[k] = s->r0[k] + dr[k][0];
        s->r1[k] = s->r1[k] + dr[k][1];
        s->x0[k] = s->x0[k] + dx[k][0];
        s->x1[k] = s->x1[k] + dx[k][1];
    }
}

/* as_vertex_pair (float) */
static int vertex_pair32(const s32* s, int k, int km, int cm, int* pi1, int* pi2)
{
    for (int x = 0; x < km; ++x) {
        if (!((cm >> x) & 1)) continue;
        for (int y = x + 1; y < km; ++y) {
            if (!((cm >> y) & 1)) continue;
            float ax, ay, ab, ex, ey, eb;
            rowf(s, k, x, &ax, &ay, &ab);
            rowf(s, k, y, &ex, &ey, &eb);
            const float det = fmaf(ax, ey, -(ay * ex));
            const float aa = F2(ax, ax, ay, ay), ee = F2(ex, ex, ey, ey);
            if (!(det * det > 1e-18f * (aa * ee))) continue;
            const float idet = 1.0f / det;
            const float v0 = fmaf(ab, ey, -(ay * eb)) * idet;
            const float v1 = fmaf(ax, eb, -(ab * ex)) * idet;
            int feas = 1;
            for (int l = 0; l < km; ++l) {
                float fx, fy, fb;
                rowf(s, k, l, &fx, &fy, &fb);
                if (!(F2(fx, v0, fy, v1) - fb <= s->P.tol_p)) feas = 0;
            }
            if (feas) { *pi1 = x; *pi2 = y; return 2; }
        }
    }
    return 3;
}

static int popc(int x) { int n = 0; while (x) { n += x & 1; x >>= 1; } return n; }
static int ctz(int x) { int n = 0; while (!(x & 1)) { ++n; x >>= 1; } return n; }

/* as_passes (float): returns 1 when a pass certifies.  A failed pass that changed the candidate
 * sets of at most N / ORC_HANDOVER_DIV knots ends the search (the kernel's handover): its next
 * candidate sets go to the fp64 passes (orc_dcm_mpc_solve_warm) instead of another float pass. */
#ifndef ORC_HANDOVER_DIV
#define ORC_HANDOVER_DIV 16   /* kernel kHandoverDiv */
#endif
static int passes32(s32* s)
{
    const int N = s->N;
    const pf_t* P = &s->P;
    static __thread float xk[2 * WV][2], sv[2 * WV][4], E[2 * WV][3], dr[2 * WV][2], dx[2 * WV][2],
        vn[2 * WV][2];
    static __thread int pk[2 * WV];
    xi_prev32(s, xk);
    static __thread int cand0[2 * WV];
    for (int pass = 0; pass < PASSES; ++pass) {
        s->npass = pass + 1;
        int okp = 1, neg = 0, viol = 0;
        for (int k = 0; k < 2 * WV; ++k) { E[k][0] = E[k][1] = E[k][2] = 0.0f; pk[k] = 0; }
        /* setup + residuals */
        for (int k = 0; k < N; ++k) {
            sv[k][0] = s->r0[k]; sv[k][1] = s->r1[k]; sv[k][2] = s->x0[k]; sv[k][3] = s->x1[k];
            const int km = s->m[k];
            const int cm = ((s->gm[k] & ~s->drop[k]) | s->add[k]) & ((1 << km) - 1);
            cand0[k] = cm;
            int pc = popc(cm);
            const int cm2 = cm & (cm - 1);
            int pi1 = cm ? ctz(cm) : 0;
            int pi2 = cm2 ? ctz(cm2) : 0;
            if (pc > 2) pc = vertex_pair32(s, k, km, cm, &pi1, &pi2);
            if (pc > 2) okp = 0;
            const int c = pc < 3 ? pc : 2;
            pk[k] = c | (pi1 << 2) | (pi2 << 6);
            const float b2 = s->be[k] * s->be[k];
            float ax, ay, ab, ex, ey, eb;
            rowf(s, k, pi1, &ax, &ay, &ab);
            rowf(s, k, pi2, &ex, &ey, &eb);
            const float sr0 = sv[k][0], sr1 = sv[k][1];
            const float aa = F2(ax, ax, ay, ay);
            const float u = ay * ay, v = ax * ax, q = ax * ay;
            const float det = fmaf(ax, ey, -(ay * ex));
            const float n1 = c == 0 ? b2 : c == 1 ? F2(ax, sr0, ay, sr1) - ab : 1.0f;
            const float d1 = c == 0 ? P->Rw0 : c == 1 ? aa : det;
            const float d2 = c == 0 ? P->Rw1 : c == 1 ? F2(P->Rw0, u, P->Rw1, v) : 1.0f;
            const float q1 = n1 / d1;
            const float q2 = b2 / d2;
            if (c == 2) {
                const float ee = F2(ex, ex, ey, ey);
                if (!(det * det > 1e-18f * (aa * ee))) okp = 0;
            }
            const float p0 = c == 1 ? fmaf(-q1, ax, sr0) : fmaf(ab, ey, -(ay * eb)) * q1;
            const float p1 = c == 1 ? fmaf(-q1, ay, sr1) : fmaf(ax, eb, -(ab * ex)) * q1;
            s->r0[k] = c == 0 ? s->r0[k] : p0;
            s->r1[k] = c == 0 ? s->r1[k] : p1;
            E[k][0] = c == 0 ? q1 : c == 1 ? u * q2 : 0.0f;
            E[k][1] = c == 1 ? -(q * q2) : 0.0f;
            E[k][2] = c == 0 ? q2 : c == 1 ? v * q2 : 0.0f;
            residuals32(s, k, xk[k][0], xk[k][1]);
        }
        if (!riccati32(s, (const float (*)[3])E)) okp = 0;
        /* h */
        for (int k = 0; k < N; ++k) {
            const int pc = pk[k] & 3, pi1 = (pk[k] >> 2) & 15;
            const float b2 = s->be[k] * s->be[k];
            const float B00 = fmaf(b2, s->P00[k], P->Rw0);
            const float B01 = b2 * s->P01[k];
            const float B11 = fmaf(b2, s->P11[k], P->Rw1);
            float ax, ay, ab;
            rowf(s, k, pi1, &ax, &ay, &ab);
            const float u = ay * ay, v = ax * ax, q = ax * ay;
            const float detB = fmaf(B00, B11, -(B01 * B01));
            const float tbt = F3(B00, u, B11, v, -2.0f * (B01 * q));
            const float den = pc == 0 ? detB : pc == 1 ? tbt : 1.0f;
            if (pc < 2 && (!(den > 0.0f) || isinf(den))) okp = 0;
            const float id = 1.0f / den;
            s->h00[k] = pc == 0 ? B11 * id : pc == 1 ? u * id : 0.0f;
            s->h01[k] = pc == 0 ? -(B01 * id) : pc == 1 ? -(q * id) : 0.0f;
            s->h11[k] = pc == 0 ? B00 * id : pc == 1 ? v * id : 0.0f;
        }
        solve32(s, dr, dx, vn);
        /* step, certificate */
        for (int k = 0; k < N; ++k) {
            s->r0[k] = s->r0[k] + dr[k][0];
            s->r1[k] = s->r1[k] + dr[k][1];
            s->x0[k] = s->x0[k] + dx[k][0];
            s->x1[k] = s->x1[k] + dx[k][1];
            const int pc = pk[k] & 3, pi1 = (pk[k] >> 2) & 15, pi2 = (pk[k] >> 6) & 15;
            const float s0 = s->qx0[k] + vn[k][0];
            const float s1 = s->qx1[k] + vn[k][1];
            const float nu0 = F3(s->P00[k], dx[k][0], s->P01[k], dx[k][1], s0);
            const float nu1 = F3(s->P01[k], dx[k][0], s->P11[k], dx[k][1], s1);
            const float rh0 = P->Rw0 * (s->r0[k] - s->rr0[k]);
            const float rh1 = P->Rw1 * (s->r1[k] - s->rr1[k]);
            const float g0 = fmaf(s->be[k], nu0, -rh0);
            const float g1 = fmaf(s->be[k], nu1, -rh1);
            float ax, ay, ab, ex, ey, eb;
            rowf(s, k, pi1, &ax, &ay, &ab);
            rowf(s, k, pi2, &ex, &ey, &eb);
            const float n = pc == 1 ? F2(ax, g0, ay, g1) : 1.0f;
            const float d = pc == 1 ? F2(ax, ax, ay, ay) : fmaf(ax, ey, -(ay * ex));
            const float qd = n / d;
            const float l1 = pc == 1 ? qd : pc == 2 ? fmaf(g0, ey, -(ex * g1)) * qd : 0.0f;
            const float l2 = pc == 2 ? fmaf(ax, g1, -(g0 * ay)) * qd : 0.0f;
            int bad = 0;
            if (pc == 0) bad = !(fabsf(g0) <= P->tol_d) || !(fabsf(g1) <= P->tol_d);
            if (pc == 1) bad = !(fabsf(fmaf(-l1, ax, g0)) <= P->tol_d) || !(fabsf(fmaf(-l1, ay, g1)) <= P->tol_d);
            const int n1 = pc >= 1 && !(l1 >= -P->tol_d);
            const int n2 = pc == 2 && !(l2 >= -P->tol_d);
            const int dm = (n1 ? 1 << pi1 : 0) | (n2 ? 1 << pi2 : 0);
            if (bad || dm) okp = 0;
            if (dm) neg = 1;
            s->drop[k] |= dm;
            s->add[k] &= ~dm;
            int vm = 0;
            for (int i = 0; i < s->m[k]; ++i) {
                float fx, fy, fb;
                rowf(s, k, i, &fx, &fy, &fb);
                if (!(F2(fx, s->r0[k], fy, s->r1[k]) - fb <= P->tol_p)) vm |= 1 << i;
            }
            if (vm) {
                okp = 0;
                viol = 1;
                s->add[k] |= vm;
                s->drop[k] &= ~vm;
            }
        }
        if (okp) return 1;
        for (int k = 0; k < N; ++k) {
            s->r0[k] = sv[k][0]; s->r1[k] = sv[k][1]; s->x0[k] = sv[k][2]; s->x1[k] = sv[k][3];
        }
        if (!(neg || viol)) break;
        int ch = 0;
        for (int k = 0; k < N; ++k)
            ch += (((s->gm[k] & ~s->drop[k]) | s->add[k]) & ((1 << s->m[k]) - 1)) != cand0[k];
        if (ch <= N / ORC_HANDOVER_DIV) break;
    }
    return 0;
}

int orc_as32_search(const orc_dcm_params* prm, int sequential, const double* xi_init,
                     const double* omega, const double* xi_ref, const double* vrp_ref,
                     const double* A, const double* b, const int32_t* nfacets, double* r_out,
                     double* x_out, int32_t* guess, int32_t* npass)
{
    static __thread s32 st;
    s32* s = &st;
    const int N = prm->horizon;
    memset(s, 0, sizeof(*s));
    s->N = N;
    s->M = prm->max_facets;
    s->KPL = N <= WV ? 1 : 2;
    s->seq = sequential;
    s->dpp = (prm->as_tree && s->KPL == 1) ? 1 : 0;
    s->A = A;
    s->b = b;
    s->P.dt = (float)prm->dt;
    s->P.Qw0 = (float)prm->w_xi[0]; s->P.Qw1 = (float)prm->w_xi[1];
    s->P.Rw0 = (float)prm->w_vrp[0]; s->P.Rw1 = (float)prm->w_vrp[1];
    s->P.Pw0 = (float)prm->w_terminal[0]; s->P.Pw1 = (float)prm->w_terminal[1];
    s->P.tol_p = SEARCH_TOL_P;
    s->P.tol_d = SEARCH_TOL_D;
    for (int k = 0; k < 2 * WV; ++k) s->al[k] = 1.0f;   /* knots >= N: be = 0, al = 1 */
    for (int k = 0; k < N; ++k) {
        s->m[k] = nfacets[k];
        s->w[k] = (float)omega[k];
        s->be[k] = s->P.dt * s->w[k];
        s->al[k] = 1.0f + s->be[k];
        s->rr0[k] = (float)vrp_ref[2 * k]; s->rr1[k] = (float)vrp_ref[2 * k + 1];
        s->xr0[k] = (float)xi_ref[2 * (k + 1)]; s->xr1[k] = (float)xi_ref[2 * (k + 1) + 1];
        s->r0[k] = s->rr0[k]; s->r1[k] = s->rr1[k];
        s->x0[k] = s->xr0[k]; s->x1[k] = s->xr1[k];
    }
    s->xi00 = (float)xi_init[0];
    s->xi01 = (float)xi_init[1];
    lq_step32(s);
    /* the guess: facets the float LQ optimum violates */
    for (int k = 0; k < N; ++k) {
        int gm = 0;
        for (int i = 0; i < s->m[k]; ++i) {
            float ax, ay, ab;
            rowf(s, k, i, &ax, &ay, &ab);
            const float gr = F2(ax, s->r0[k], ay, s->r1[k]);
            const float sl = ab - gr;
            if (sl < 0.0f) gm |= 1 << i;
        }
        s->gm[k] = gm;
    }
    const int cert = passes32(s);
    if (npass) *npass = s->npass;
    for (int k = 0; k < N; ++k) {
        r_out[2 * k] = (double)s->r0[k];
        r_out[2 * k + 1] = (double)s->r1[k];
        x_out[2 * k] = (double)s->x0[k];
        x_out[2 * k + 1] = (double)s->x1[k];
        guess[k] = ((s->gm[k] & ~s->drop[k]) | s->add[k]) & ((1 << s->m[k]) - 1);
    }
    return cert;
}
