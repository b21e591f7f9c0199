// dcm_mpc_as.hip — batched time-varying DCM MPC QP, active-set start on ONE wavefront per QP
// (TimeVaryingDCMPlanner).
//
// Almost every QP of a batch is solved by the active-set start: the LQ
// optimum, then up to kGuessPasses exact equality-constrained solves, each certified or corrected
// by drop/add moves.  This kernel runs exactly that part, and nothing of the interior point
// method, so a knot carries no slacks or multipliers:
//   * one 64-lane wavefront per QP; lane l owns knot l (N <= 64) or the knot pair (2l, 2l + 1)
//     (N <= 128).  A scan composes the pair in the lane, runs Kogge-Stone over the 64 lanes on one
//     element per lane and applies the pair's inner knot in the lane: 7 compositions per scan
//     instead of 12 for two knots per lane on separate wavefronts, and no barrier at all.  The
//     oracle evaluates the start in the same tree (oracle scan_backward_pairs etc.), bit for bit;
//   * the facet rows are staged once in LDS from coalesced loads of the QP's contiguous A / b
//     slabs (consecutive lanes on consecutive 16 B), [M][slot][lane].
// A QP whose start does not certify is left with status kPending and its start point (the LQ
// optimum, or the warm start's rollout) in the output arrays; the IPM kernel's stage 2
// (dcm_mpc_ipm.hip) continues from there exactly as the oracle does after a failed start.
#include "dcm_qp_common.h"

namespace blf {
namespace {
using namespace qp;

#ifdef BLF_STAMPS
// Diagnostic build only (make stamps): per-phase cycle sums of lane 0 for the first 64 QPs.
// [0] whole kernel, [1] slab staging + knot loads, [2] LQ step, [3] guess, [4] pass: setup +
// residuals, [5] pass: Riccati sweep, [6] pass: h, [7] pass: solve, [8] pass: certificate,
// [9] pass: vote + restore, [10] passes (count), [11] outputs.
__device__ unsigned long long g_as_stamps[16];
#define AS_STAMP(t) unsigned long long t = __builtin_amdgcn_s_memtime()
#define AS_STAMP_ADD(slot, t0) \
    do { if (blockIdx.x < 64 && threadIdx.x == 0) atomicAdd(&g_as_stamps[slot], __builtin_amdgcn_s_memtime() - (t0)); } while (0)
#define AS_COUNT(slot) \
    do { if (blockIdx.x < 64 && threadIdx.x == 0) atomicAdd(&g_as_stamps[slot], 1ull); } while (0)
#else
#define AS_STAMP(t)
#define AS_STAMP_ADD(slot, t0)
#define AS_COUNT(slot)
#endif

// Per-knot state of the active-set passes.
struct AKnot {
    int m;                          // facet count
    int gm;                         // the start's guess (bit i: facet i)
    int drop, add;                  // facets taken out of / put into the guess by earlier passes
    double r0, r1;                  // VRP
    double x0, x1;                  // xi_{k+1}
    double w, al, be;               // omega_k, 1 + dt omega_k, dt omega_k
    double rh0, rh1, d0, d1, qx0, qx1;
    double P00, P01, P11;           // P_{k+1}
    double h00, h01, h11;           // H_k^{-1} of the active subspace
    double rr0, rr1, xr0, xr1;      // vrp_ref_k, xi_ref_{k+1}
};

// The scan tree (oracle scan_backward_pairs / scan_forward_pairs / riccati_sweep_pairs):
//   KPL = 1 (N <= 64): lane l owns knot l; Kogge-Stone over the 64 lanes (the IPM kernel's tree
//            for one wavefront);
//   KPL = 2 (N <= 128): lane l owns the knot pair (2l, 2l + 1): the pair's element is composed in
//            the lane, Kogge-Stone runs over the 64 lanes on one element per lane, and the pair's
//            inner knot is applied in the lane afterwards.
// Slot j of a lane is knot KPL lane + j.  Knots >= N carry the zero element (affine scans) or the
// identity (Riccati).

// Backward affine scan v_k = G_k v_{k+1} + c_k, v_N = 0.  Returns v_{k+1} per slot.
template <int KPL>
__device__ __forceinline__ void as_scan_backward(const double (&G)[KPL][4], const double (&c)[KPL][2], int lane,
                                                 double (&vn)[KPL][2])
{
    double g0 = G[0][0], g1 = G[0][1], g2 = G[0][2], g3 = G[0][3], e0 = c[0][0], e1 = c[0][1];
    if constexpr (KPL == 2)   // knot 2l after knot 2l + 1
        COMPOSE(g0, g1, g2, g3, G[1][0], G[1][1], G[1][2], G[1][3], c[1][0], c[1][1], e0, e1);
    const int ln = opaque(lane);
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const int ad = ((ln + d) & (kWave - 1)) << 2;
        const double p0 = bperm(ad, g0), p1 = bperm(ad, g1), p2 = bperm(ad, g2), p3 = bperm(ad, g3);
        const double q0 = bperm(ad, e0), q1 = bperm(ad, e1);
        if (ln + d < kWave) COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, e0, e1);
    }
    // e = v at this lane's first knot; the next lane's = v past this lane's last knot
    const int a1 = ((ln + 1) & (kWave - 1)) << 2;
    double vb0 = bperm(a1, e0), vb1 = bperm(a1, e1);
    if (lane == kWave - 1) {
        vb0 = 0.0;
        vb1 = 0.0;
    }
    if constexpr (KPL == 2) {
        vn[0][0] = FD3(G[1][0], vb0, G[1][1], vb1, c[1][0]);   // v_{2l+1}
        vn[0][1] = FD3(G[1][2], vb0, G[1][3], vb1, c[1][1]);
        vn[1][0] = vb0;                                       // v_{2l+2}
        vn[1][1] = vb1;
    } else {
        vn[0][0] = vb0;
        vn[0][1] = vb1;
    }
}

// Forward affine scan x_{k+1} = F_k x_k + f_k, x_0 = 0.  Returns x_{k+1} and x_k per slot.
template <int KPL>
__device__ __forceinline__ void as_scan_forward(const double (&F)[KPL][4], const double (&f)[KPL][2], int lane,
                                                double (&x)[KPL][2], double (&xk)[KPL][2])
{
    constexpr int L = KPL - 1;   // the lane's last knot
    double g0 = F[L][0], g1 = F[L][1], g2 = F[L][2], g3 = F[L][3], e0 = f[L][0], e1 = f[L][1];
    if constexpr (KPL == 2)   // knot 2l + 1 after knot 2l
        COMPOSE(g0, g1, g2, g3, F[0][0], F[0][1], F[0][2], F[0][3], f[0][0], f[0][1], e0, e1);
    const int ln = opaque(lane);
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const int ad = ((ln - d) & (kWave - 1)) << 2;
        const double p0 = bperm(ad, g0), p1 = bperm(ad, g1), p2 = bperm(ad, g2), p3 = bperm(ad, g3);
        const double q0 = bperm(ad, e0), q1 = bperm(ad, e1);
        if (ln >= d) COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, e0, e1);
    }
    // e = x past this lane's last knot; the previous lane's = x at this lane's first knot
    const int a1 = ((ln - 1) & (kWave - 1)) << 2;
    double xb0 = bperm(a1, e0), xb1 = bperm(a1, e1);
    if (lane == 0) {
        xb0 = 0.0;
        xb1 = 0.0;
    }
    xk[0][0] = xb0;
    xk[0][1] = xb1;
    if constexpr (KPL == 2) {
        const double x10 = FD3(F[0][0], xb0, F[0][1], xb1, f[0][0]);   // x_{2l+1}
        const double x11 = FD3(F[0][2], xb0, F[0][3], xb1, f[0][1]);
        x[0][0] = x10;
        x[0][1] = x11;
        xk[1][0] = x10;
        xk[1][1] = x11;
    }
    x[L][0] = e0;
    x[L][1] = e1;
}

// xi_k of every slot: the previous knot's xi_{k+1} (lane 0, slot 0: xi_init).
template <int KPL>
__device__ __forceinline__ void as_xi_prev(const AKnot (&K)[KPL], int lane, double xi00, double xi01,
                                           double (&xk)[KPL][2])
{
    constexpr int L = KPL - 1;
    xk[0][0] = __shfl_up(K[L].x0, 1, kWave);
    xk[0][1] = __shfl_up(K[L].x1, 1, kWave);
    if (lane == 0) {
        xk[0][0] = xi00;
        xk[0][1] = xi01;
    }
    if constexpr (KPL == 2) {
        xk[1][0] = K[0].x0;
        xk[1][1] = K[0].x1;
    }
}

// Gradient, Euler defect and Q (xi - xi_ref) of one knot without facet terms (IPM kernel
// residuals(facets = false)).
__device__ __forceinline__ void as_residuals(AKnot& K, const KParams& P, bool last, double xk0, double xk1)
{
    K.rh0 = P.Rw0 * (K.r0 - K.rr0);
    K.rh1 = P.Rw1 * (K.r1 - K.rr1);
    const double dx0 = FD2(K.w, xk0, -K.w, K.r0);
    K.d0 = fma(dx0, P.dt, xk0) - K.x0;
    const double dx1 = FD2(K.w, xk1, -K.w, K.r1);
    K.d1 = fma(dx1, P.dt, xk1) - K.x1;
    const double q0 = last ? P.Pw0 : P.Qw0;
    const double q1 = last ? P.Pw1 : P.Qw1;
    K.qx0 = q0 * (K.x0 - K.xr0);
    K.qx1 = q1 * (K.x1 - K.xr1);
}

// Riccati sweep (oracle riccati_sweep_pairs; KPL = 1: riccati_sweep on one wavefront): leaves
// P_{k+1} in K; false on a lane where some (I + G H) or (I + G P) is not positive definite.
__device__ __forceinline__ void rc_knot(Rc& e, bool own, double al, const double (&E)[3], const KParams& P)
{
    if (own) {
        e.a0 = al; e.a1 = 0.0; e.a2 = 0.0; e.a3 = al;
        e.g0 = E[0]; e.g1 = E[1]; e.g2 = E[2];
        e.h0 = P.Qw0; e.h1 = 0.0; e.h2 = P.Qw1;
    } else {
        e.a0 = 1.0; e.a1 = 0.0; e.a2 = 0.0; e.a3 = 1.0;
        e.g0 = e.g1 = e.g2 = 0.0;
        e.h0 = e.h1 = e.h2 = 0.0;
    }
}

template <int KPL>
__device__ __forceinline__ bool as_riccati(AKnot (&K)[KPL], const KParams& P, const double (&E)[KPL][3],
                                           int N, int lane)
{
    bool ok = true;
    Rc e;
    rc_knot(e, KPL * lane < N, K[0].al, E[0], P);
    if constexpr (KPL == 2) {
        Rc e1;
        rc_knot(e1, KPL * lane + 1 < N, K[1].al, E[1], P);
        ok = rc_combine(e, e1) && ok;
    }
    const int ln = opaque(lane);
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const int ad = ((ln + d) & (kWave - 1)) << 2;
        Rc q;
        q.a0 = bperm(ad, e.a0); q.a1 = bperm(ad, e.a1); q.a2 = bperm(ad, e.a2); q.a3 = bperm(ad, e.a3);
        q.g0 = bperm(ad, e.g0); q.g1 = bperm(ad, e.g1); q.g2 = bperm(ad, e.g2);
        q.h0 = bperm(ad, e.h0); q.h1 = bperm(ad, e.h1); q.h2 = bperm(ad, e.h2);
        if (ln + d < kWave) ok = rc_combine(e, q) && ok;
    }
    // P at this lane's first knot; the next lane's (terminal past the last lane)
    double P00, P01, P11;
    ok = rc_apply(e, P.Pw0, 0.0, P.Pw1, P00, P01, P11) && ok;
    const int a1 = ((ln + 1) & (kWave - 1)) << 2;
    double Pn00 = bperm(a1, P00), Pn01 = bperm(a1, P01), Pn11 = bperm(a1, P11);
    if (lane == kWave - 1) {
        Pn00 = P.Pw0;
        Pn01 = 0.0;
        Pn11 = P.Pw1;
    }
    constexpr int L = KPL - 1;
    K[L].P00 = Pn00;
    K[L].P01 = Pn01;
    K[L].P11 = Pn11;
    if constexpr (KPL == 2) {   // P_{2l+1} = f_{2l+1}(P_{2l+2}), the first knot's P_{k+1}
        Rc e1;
        rc_knot(e1, KPL * lane + 1 < N, K[1].al, E[1], P);
        double o00, o01, o11;
        ok = rc_apply(e1, Pn00, Pn01, Pn11, o00, o01, o11) && ok;
        K[0].P00 = o00;
        K[0].P01 = o01;
        K[0].P11 = o11;
    }
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        if (KPL * lane + j == N - 1) {
            K[j].P00 = P.Pw0;
            K[j].P01 = 0.0;
            K[j].P11 = P.Pw1;
        }
    }
    return ok;
}

// Solve the factored Newton system for the right-hand side g (IPM kernel solve) over every slot.
template <int KPL>
__device__ __forceinline__ void as_solve(const AKnot (&K)[KPL], const double (&g)[KPL][2], int N, int lane,
                                         double (&dr)[KPL][2], double (&dx)[KPL][2], double (&vn)[KPL][2])
{
    double G[KPL][4], c[KPL][2], y[KPL][2];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        G[j][0] = G[j][1] = G[j][2] = G[j][3] = 0.0;
        c[j][0] = c[j][1] = y[j][0] = y[j][1] = 0.0;
        if (KPL * lane + j < N) {
            const AKnot& Kj = K[j];
            const double b2 = Kj.be * Kj.be;
            const double ab = Kj.al * Kj.be;
            const double m00 = FD2(Kj.P00, Kj.h00, Kj.P01, Kj.h01);
            const double m01 = FD2(Kj.P00, Kj.h01, Kj.P01, Kj.h11);
            const double m10 = FD2(Kj.P01, Kj.h00, Kj.P11, Kj.h01);
            const double m11 = FD2(Kj.P01, Kj.h01, Kj.P11, Kj.h11);
            y[j][0] = FD3(Kj.P00, Kj.d0, Kj.P01, Kj.d1, Kj.qx0);
            y[j][1] = FD3(Kj.P01, Kj.d0, Kj.P11, Kj.d1, Kj.qx1);
            const double Mg0 = FD2(m00, g[j][0], m01, g[j][1]);
            const double Mg1 = FD2(m10, g[j][0], m11, g[j][1]);
            G[j][0] = Kj.al * fma(-b2, m00, 1.0);
            G[j][1] = -(Kj.al * (b2 * m01));
            G[j][2] = -(Kj.al * (b2 * m10));
            G[j][3] = Kj.al * fma(-b2, m11, 1.0);
            c[j][0] = FD3(G[j][0], y[j][0], G[j][1], y[j][1], ab * Mg0);
            c[j][1] = FD3(G[j][2], y[j][0], G[j][3], y[j][1], ab * Mg1);
        }
    }
    double Gt[KPL][4];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        Gt[j][0] = G[j][0]; Gt[j][1] = G[j][2]; Gt[j][2] = G[j][1]; Gt[j][3] = G[j][3];
    }
    as_scan_backward<KPL>(G, c, lane, vn);
    double k[KPL][2], f[KPL][2];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        k[j][0] = k[j][1] = f[j][0] = f[j][1] = 0.0;
        if (KPL * lane + j < N) {
            const AKnot& Kj = K[j];
            const double t0 = y[j][0] + vn[j][0];
            const double t1 = y[j][1] + vn[j][1];
            const double hu0 = fma(-Kj.be, t0, g[j][0]);
            const double hu1 = fma(-Kj.be, t1, g[j][1]);
            k[j][0] = -FD2(Kj.h00, hu0, Kj.h01, hu1);
            k[j][1] = -FD2(Kj.h01, hu0, Kj.h11, hu1);
            f[j][0] = fma(-Kj.be, k[j][0], Kj.d0);
            f[j][1] = fma(-Kj.be, k[j][1], Kj.d1);
        }
    }
    double xk[KPL][2];
    as_scan_forward<KPL>(Gt, f, lane, dx, xk);
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const AKnot& Kj = K[j];
        const double ab = Kj.al * Kj.be;
        const double m00 = FD2(Kj.P00, Kj.h00, Kj.P01, Kj.h01);
        const double m01 = FD2(Kj.P00, Kj.h01, Kj.P01, Kj.h11);
        const double m10 = FD2(Kj.P01, Kj.h00, Kj.P11, Kj.h01);
        const double m11 = FD2(Kj.P01, Kj.h01, Kj.P11, Kj.h11);
        dr[j][0] = fma(ab, FD2(m00, xk[j][0], m10, xk[j][1]), k[j][0]);
        dr[j][1] = fma(ab, FD2(m01, xk[j][0], m11, xk[j][1]), k[j][1]);
    }
}

// Candidate facets of a pass -> (pc, pi1, pi2) packed as pc | pi1 << 2 | pi2 << 5, the VRP moved
// onto the active lines and E_k (IPM kernel polish block, "active sets, projection").
// Branch-free: the two knots of a lane, and the lanes of a wavefront, have every mix of 0, 1 and 2
// active lines, so per-case branches serialised all three bodies and their divisions.  Each knot
// instead evaluates exactly two quotients whose operands its case selects (c = 0: b2 / Rw0,
// b2 / Rw1; c = 1: (a r - b) / |a|^2, b2 / (Rw0 a_y^2 + Rw1 a_x^2); c = 2: 1 / det) — the same
// operations as the per-case form of the oracle, so the results are bit-identical.
__device__ __forceinline__ void as_pass_setup(AKnot& K, const KParams& P, const double2* A2, const double* Bv,
                                              int S, int col, double sr0, double sr1, int& pk, double (&E)[3],
                                              bool& okp)
{
    const int cx = opaque(col);
    const int km = opaque(K.m);
    // candidates: guessed and not dropped, or added (bit i, i < m); the first two in facet order
    const int cm = ((K.gm & ~K.drop) | K.add) & ((1 << km) - 1);
    int pc = __builtin_popcount(cm);
    const int cm2 = cm & (cm - 1);
    int pi1 = cm ? __builtin_ctz(cm) : 0;
    int pi2 = cm2 ? __builtin_ctz(cm2) : 0;
    if (pc > 2) pc = vertex_pair(A2, Bv, 1, S, cx, km, cm, P.tol_p, pi1, pi2);
    if (pc > 2) okp = false;
    const int c = pc < 3 ? pc : 2;
    pk = c | (pi1 << 2) | (pi2 << 5);
    const double b2 = K.be * K.be;
    const double2 a = A2[pi1 * S + cx];
    const double2 e = A2[pi2 * S + cx];
    const double ba = Bv[pi1 * S + cx], be = Bv[pi2 * S + cx];
    const double aa = FD2(a.x, a.x, a.y, a.y);
    const double u = a.y * a.y, v = a.x * a.x, q = a.x * a.y;
    const double det = fma(a.x, e.y, -(a.y * e.x));
    const double n1 = c == 0 ? b2 : c == 1 ? FD2(a.x, sr0, a.y, sr1) - ba : 1.0;
    const double d1 = c == 0 ? P.Rw0 : c == 1 ? aa : det;
    const double d2 = c == 0 ? P.Rw1 : c == 1 ? FD2(P.Rw0, u, P.Rw1, v) : 1.0;
    const double q1 = n1 / d1;   // c = 0: E00; c = 1: t; c = 2: 1 / det
    const double q2 = b2 / d2;   // c = 0: E11; c = 1: ie
    if (c == 2) {
        const double ee = FD2(e.x, e.x, e.y, e.y);
        if (!(det * det > 1e-18 * (aa * ee))) okp = false;   // (nearly) parallel active facets
    }
    const double p0 = c == 1 ? fma(-q1, a.x, sr0) : fma(ba, e.y, -(a.y * be)) * q1;
    const double p1 = c == 1 ? fma(-q1, a.y, sr1) : fma(a.x, be, -(ba * e.x)) * q1;
    K.r0 = c == 0 ? K.r0 : p0;
    K.r1 = c == 0 ? K.r1 : p1;
    E[0] = c == 0 ? q1 : c == 1 ? u * q2 : 0.0;
    E[1] = c == 1 ? -(q * q2) : 0.0;
    E[2] = c == 0 ? q2 : c == 1 ? v * q2 : 0.0;
}

// h_k = H_k^{-1} of the knot's active subspace after the Riccati sweep (IPM kernel polish block):
// c = 0: B^{-1}; c = 1: t t^T / (t^T B t), t = (-a_y, a_x); c = 2: 0.  One quotient per knot,
// operands selected by the case (bit-identical to the per-case form).
__device__ __forceinline__ void as_pass_h(AKnot& K, const KParams& P, const double2* A2, int S, int col, int pk,
                                          bool& okp)
{
    const int pc = pk & 3, pi1 = (pk >> 2) & 7;
    const double b2 = K.be * K.be;
    const double B00 = fma(b2, K.P00, P.Rw0);
    const double B01 = b2 * K.P01;
    const double B11 = fma(b2, K.P11, P.Rw1);
    const double2 a = A2[pi1 * S + opaque(col)];
    const double u = a.y * a.y, v = a.x * a.x, q = a.x * a.y;
    const double detB = fma(B00, B11, -(B01 * B01));
    const double tbt = FD3(B00, u, B11, v, -2.0 * (B01 * q));
    const double den = pc == 0 ? detB : pc == 1 ? tbt : 1.0;
    if (pc < 2 && (!(den > 0.0) || __builtin_isinf(den))) okp = false;
    const double id = 1.0 / den;
    K.h00 = pc == 0 ? B11 * id : pc == 1 ? u * id : 0.0;
    K.h01 = pc == 0 ? -(B01 * id) : pc == 1 ? -(q * id) : 0.0;
    K.h11 = pc == 0 ? B00 * id : pc == 1 ? v * id : 0.0;
}

// The certificate of one knot after the step (IPM kernel polish block): stationarity with the
// solve's costates, multiplier signs, primal feasibility of every facet; drop / add bookkeeping.
// One quotient per knot (c = 1: (a g) / |a|^2; c = 2: 1 / det), operands selected by the case.
__device__ __forceinline__ void as_certify(AKnot& K, const KParams& P, const double2* A2, const double* Bv,
                                           int S, int col, int pk, double dx0, double dx1, double vn0,
                                           double vn1, double& l1o, double& l2o, bool& okp, bool& neg,
                                           bool& viol)
{
    const int cx = opaque(col);
    const int pc = pk & 3, pi1 = (pk >> 2) & 7, pi2 = (pk >> 5) & 7;
    const double s0 = K.qx0 + vn0;
    const double s1 = K.qx1 + vn1;
    const double nu0 = FD3(K.P00, dx0, K.P01, dx1, s0);
    const double nu1 = FD3(K.P01, dx0, K.P11, dx1, s1);
    const double rh0 = P.Rw0 * (K.r0 - K.rr0);
    const double rh1 = P.Rw1 * (K.r1 - K.rr1);
    const double g0 = fma(K.be, nu0, -rh0);
    const double g1 = fma(K.be, nu1, -rh1);
    const double2 a = A2[pi1 * S + cx];
    const double2 e = A2[pi2 * S + cx];
    const double n = pc == 1 ? FD2(a.x, g0, a.y, g1) : 1.0;
    const double d = pc == 1 ? FD2(a.x, a.x, a.y, a.y) : fma(a.x, e.y, -(a.y * e.x));
    const double qd = n / d;
    const double l1 = pc == 1 ? qd : pc == 2 ? fma(g0, e.y, -(e.x * g1)) * qd : 0.0;
    const double l2 = pc == 2 ? fma(a.x, g1, -(g0 * a.y)) * qd : 0.0;
    l1o = l1;
    l2o = l2;
    bool bad = false;
    if (pc == 0) bad = !(fabs(g0) <= P.tol_d) || !(fabs(g1) <= P.tol_d);
    if (pc == 1) bad = !(fabs(fma(-l1, a.x, g0)) <= P.tol_d) || !(fabs(fma(-l1, a.y, g1)) <= P.tol_d);
    const bool n1 = pc >= 1 && !(l1 >= -P.tol_d);
    const bool n2 = pc == 2 && !(l2 >= -P.tol_d);
    const int dm = (n1 ? 1 << pi1 : 0) | (n2 ? 1 << pi2 : 0);
    if (bad || dm) okp = false;
    if (dm) neg = true;
    K.drop |= dm;
    K.add &= ~dm;
    // primal feasibility of every facet, rows read four at a time
    const int km = opaque(K.m);
    int vm = 0;
#pragma unroll
    for (int i0 = 0; i0 < kMaxFacets; i0 += 4) {
        if (i0 >= km) break;
        double2 av[4];
        double bv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = i0 + q < km ? i0 + q : 0;
            av[q] = A2[i * S + cx];
            bv[q] = Bv[i * S + cx];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (!(FD2(av[q].x, K.r0, av[q].y, K.r1) - bv[q] <= P.tol_p)) vm |= 1 << (i0 + q);
    }
    vm &= (1 << km) - 1;
    if (vm) {
        okp = false;
        viol = true;
        K.add |= vm;
        K.drop &= ~vm;
    }
}

template <int KPL, bool WARM, bool LAMOUT>
__global__ __launch_bounds__(kWave, 2) void dcm_mpc_as_kernel(
    KParams P, const double* __restrict__ xi_init, const double* __restrict__ omega,
    const double* __restrict__ xi_ref, const double* __restrict__ vrp_ref,
    const double* __restrict__ Ain, const double* __restrict__ bin,
    const int32_t* __restrict__ nfacets, const double* __restrict__ ws_vrp,
    const double* __restrict__ ws_lam, double* __restrict__ xi_out,
    double* __restrict__ vrp_out, int32_t* __restrict__ status_out,
    int32_t* __restrict__ iters_out, int32_t* __restrict__ polished_out, double* __restrict__ lam_out)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int N = P.N, M = P.M;
    const int NH = (N + KPL - 1) / KPL;   // lanes holding knots
    const int S = KPL * NH;               // LDS row stride: facet i of slot j, lane l at i S + j NH + l
    double2* A2 = reinterpret_cast<double2*>(smem);   // [M][S] facet normals
    double* Bv = smem + 2 * (size_t)M * S;              // [M][S] offsets
    const int lane = threadIdx.x;
    const int64_t p = blockIdx.x;
    AS_STAMP(t_start);

    // ---- the QP's facet slabs A [N][M][2], b [N][M] into LDS: coalesced (consecutive lanes on
    //      consecutive 16 B).  Every load of the start-up is issued before the first wait: the
    //      slab loads (one round, U per lane covers N M <= 128 x 8), then the knots' own loads,
    //      then the LDS stores, which wait for the slab loads only. ----
    const int nA = N * M;
    constexpr int U = (2 * kWave * kMaxFacets) / kWave;   // 16: nA <= 1024 in one round
    double2 va[U];
    double vb[U];
    {
        const double2* As = reinterpret_cast<const double2*>(Ain) + p * nA;
        const double* bs = bin + p * nA;
#pragma unroll
        for (int u = 0; u < U; ++u) {   // clamped, so every load is unconditional
            const int t = min(u * kWave + lane, nA - 1);
            va[u] = As[t];
            vb[u] = bs[t];
        }
    }

    // ---- the knots this lane owns ----
    constexpr bool warm = WARM;
    AKnot K[KPL];
    bool bad = false;
    const double xi00 = xi_init[2 * p], xi01 = xi_init[2 * p + 1];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const int k = KPL * lane + j;
        AKnot& Kj = K[j];
        Kj.m = 0;
        Kj.gm = Kj.drop = Kj.add = 0;
        Kj.r0 = Kj.r1 = Kj.x0 = Kj.x1 = Kj.w = Kj.be = 0.0;
        Kj.rh0 = Kj.rh1 = Kj.d0 = Kj.d1 = Kj.qx0 = Kj.qx1 = 0.0;
        Kj.P00 = Kj.P01 = Kj.P11 = Kj.h00 = Kj.h01 = Kj.h11 = 0.0;
        Kj.rr0 = Kj.rr1 = Kj.xr0 = Kj.xr1 = 0.0;
        if (k < N) {
            const int64_t st = p * N + k;
            Kj.m = nfacets[st];
            Kj.w = omega[st];
            const bool ws = warm && k + P.ws_shift < N;
            const double* r0 = ws ? ws_vrp + 2 * P.ws_shift : vrp_ref;
            Kj.r0 = r0[2 * st];
            Kj.r1 = r0[2 * st + 1];
            Kj.rr0 = vrp_ref[2 * st];
            Kj.rr1 = vrp_ref[2 * st + 1];
            const int64_t sx = p * (N + 1) + (k + 1);
            Kj.xr0 = xi_ref[2 * sx];
            Kj.xr1 = xi_ref[2 * sx + 1];
        }
    }
    {
        const bool pow2 = (M & (M - 1)) == 0;
        const int sh = __builtin_ctz(M);
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int t = u * kWave + lane;
            if (t < nA) {
                const int k = pow2 ? t >> sh : t / M, i = t - k * M;
                const int o = i * S + (k % KPL) * NH + k / KPL;
                A2[o] = va[u];
                Bv[o] = vb[u];
            }
        }
    }
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        AKnot& Kj = K[j];
        if (KPL * lane + j < N) {
            if (Kj.m < 0 || Kj.m > M) {
                bad = true;
                Kj.m = 0;
            }
            Kj.be = P.dt * Kj.w;
        }
        Kj.al = 1.0 + Kj.be;
    }
    const bool any_bad = __ballot(bad) != 0;
    __syncthreads();   // the LDS slabs (one wavefront: a wait for the stores)
    AS_STAMP_ADD(1, t_start);
    AS_STAMP(t_lq);

    // ---- initial point: a warm start rolls xi out from its VRPs (forward scan of
    //      xi_{k+1} = alpha_k xi_k - beta_k r_k); a cold start takes xi_ref, then the LQ step ----
    if (warm) {
        double g[KPL][4], f[KPL][2], xk[KPL][2], x[KPL][2];
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            const int k = KPL * lane + j;
            f[j][0] = f[j][1] = 0.0;
            if (k < N) {
                if (k == 0) {
                    f[j][0] = fma(K[j].al, xi00, -(K[j].be * K[j].r0));
                    f[j][1] = fma(K[j].al, xi01, -(K[j].be * K[j].r1));
                } else {
                    f[j][0] = -(K[j].be * K[j].r0);
                    f[j][1] = -(K[j].be * K[j].r1);
                }
            }
            const double ga = k < N ? K[j].al : 0.0;
            g[j][0] = ga; g[j][1] = 0.0; g[j][2] = 0.0; g[j][3] = ga;
        }
        as_scan_forward<KPL>(g, f, lane, x, xk);
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            K[j].x0 = x[j][0];
            K[j].x1 = x[j][1];
        }
    } else {
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            if (KPL * lane + j < N) {
                K[j].x0 = K[j].xr0;
                K[j].x1 = K[j].xr1;
            }
        }
    }
    int status = 0;
    bool certified = false;
    double pl[KPL][2];
    int pk[KPL];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        pl[j][0] = pl[j][1] = 0.0;
        pk[j] = 0;
    }
    if (any_bad) {
        status = BLF_QP_BAD_FACETS;
    } else {
        if (!warm) {   // full Newton step of the unconstrained QP (W = 0, lambda = 0): the LQ optimum
            double xk[KPL][2];
            as_xi_prev<KPL>(K, lane, xi00, xi01, xk);
#pragma unroll
            for (int j = 0; j < KPL; ++j) {
                const int k = KPL * lane + j;
                if (k < N) as_residuals(K[j], P, k == N - 1, xk[j][0], xk[j][1]);
            }
            double E[KPL][3];
#pragma unroll
            for (int j = 0; j < KPL; ++j) {
                E[j][0] = E[j][1] = E[j][2] = 0.0;
                if (KPL * lane + j < N) {
                    const double b2 = K[j].be * K[j].be;
                    const double W00 = 0.0, W01 = 0.0, W11 = 0.0, dW = 0.0;
                    const double detRW = fma(P.Rw0, P.Rw1, FD2(P.Rw1, W00, P.Rw0, W11)) + dW;
                    const double ie = b2 / detRW;
                    E[j][0] = (P.Rw1 + W11) * ie;
                    E[j][1] = -(W01 * ie);
                    E[j][2] = (P.Rw0 + W00) * ie;
                }
            }
            bool ok = as_riccati<KPL>(K, P, E, N, lane);
#pragma unroll
            for (int j = 0; j < KPL; ++j) {
                if (KPL * lane + j < N) {
                    AKnot& Kj = K[j];
                    const double b2 = Kj.be * Kj.be;
                    const double W00 = 0.0, W01 = 0.0, W11 = 0.0, dW = 0.0;
                    const double B00 = fma(b2, Kj.P00, P.Rw0);
                    const double B01 = b2 * Kj.P01;
                    const double B11 = fma(b2, Kj.P11, P.Rw1);
                    const double H00 = B00 + W00;
                    const double H01 = B01 + W01;
                    const double H11 = B11 + W11;
                    const double detB = fma(B00, B11, -(B01 * B01));
                    const double trW = FD2(B11, W00, B00, W11) - 2.0 * (B01 * W01);
                    const double det = (detB + trW) + dW;
                    if (!(det > 0.0) || __builtin_isinf(det)) ok = false;
                    const double idet = 1.0 / det;
                    Kj.h00 = H11 * idet;
                    Kj.h01 = -(H01 * idet);
                    Kj.h11 = H00 * idet;
                }
            }
            if (__ballot(!ok) != 0) status = BLF_QP_NUMERICAL;   // still takes the step (oracle)
            double g[KPL][2], dr[KPL][2], dx[KPL][2], vn[KPL][2];
#pragma unroll
            for (int j = 0; j < KPL; ++j) {
                g[j][0] = K[j].rh0;
                g[j][1] = K[j].rh1;
            }
            as_solve<KPL>(K, g, N, lane, dr, dx, vn);
#pragma unroll
            for (int j = 0; j < KPL; ++j) {
                if (KPL * lane + j < N) {
                    K[j].r0 = K[j].r0 + dr[j][0];
                    K[j].r1 = K[j].r1 + dr[j][1];
                    K[j].x0 = K[j].x0 + dx[j][0];
                    K[j].x1 = K[j].x1 + dx[j][1];
                }
            }
        }
    }

    AS_STAMP_ADD(2, t_lq);
    if (status == 0) {
        AS_STAMP(t_g);
        // ---- the guess: facets the start point violates (warm: also those whose previous
        //      multiplier exceeds the floor) ----
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            const int k = KPL * lane + j;
            if (k < N) {
                const int col = j * NH + lane;
                const bool ws = warm && k + P.ws_shift < N;
                const double* lw = ws_lam + (ws ? (p * N + k + P.ws_shift) * M : 0);
                int gm = 0;
                for (int i = 0; i < K[j].m; ++i) {
                    const double2 a = A2[i * S + col];
                    const double gr = FD2(a.x, K[j].r0, a.y, K[j].r1);
                    const double sl = Bv[i * S + col] - gr;
                    if (sl < 0.0) gm |= 1 << i;
                    if (ws && lw[i] > P.ws_floor) gm |= 1 << i;
                }
                K[j].gm = gm;
            }
        }

        // ---- active-set passes (oracle dcm_polish with the guess) ----
        double xk[KPL][2];
        as_xi_prev<KPL>(K, lane, xi00, xi01, xk);
        AS_STAMP_ADD(3, t_g);
        for (int pass = 0; pass < kGuessPasses; ++pass) {
            AS_COUNT(10);
            AS_STAMP(t_s);
            double sv[KPL][4];
            double E[KPL][3];
            bool okp = true;
#pragma unroll
            for (int j = 0; j < KPL; ++j) {
                const int k = KPL * lane + j;
                sv[j][0] = K[j].r0; sv[j][1] = K[j].r1; sv[j][2] = K[j].x0; sv[j][3] = K[j].x1;
                E[j][0] = E[j][1] = E[j][2] = 0.0;
                pk[j] = 0;
                if (k < N) {
                    as_pass_setup(K[j], P, A2, Bv, S, j * NH + lane, sv[j][0], sv[j][1], pk[j], E[j], okp);
                    as_residuals(K[j], P, k == N - 1, xk[j][0], xk[j][1]);
                }
            }
            AS_STAMP_ADD(4, t_s);
            AS_STAMP(t_r);
            okp = as_riccati<KPL>(K, P, E, N, lane) && okp;
            AS_STAMP_ADD(5, t_r);
            AS_STAMP(t_h);
#pragma unroll
            for (int j = 0; j < KPL; ++j)
                if (KPL * lane + j < N) as_pass_h(K[j], P, A2, S, j * NH + lane, opaque(pk[j]), okp);
            AS_STAMP_ADD(6, t_h);
            // the Newton step, then the certificate (costates of the new point from the solve)
            bool neg = false, viol = false;
            {
                double g[KPL][2], dr[KPL][2], dx[KPL][2], vn[KPL][2];
#pragma unroll
                for (int j = 0; j < KPL; ++j) {
                    g[j][0] = K[j].rh0;
                    g[j][1] = K[j].rh1;
                }
                AS_STAMP(t_v);
                as_solve<KPL>(K, g, N, lane, dr, dx, vn);
                AS_STAMP_ADD(7, t_v);
                AS_STAMP(t_c);
#pragma unroll
                for (int j = 0; j < KPL; ++j) {
                    pl[j][0] = pl[j][1] = 0.0;
                    if (KPL * lane + j < N) {
                        K[j].r0 = K[j].r0 + dr[j][0];
                        K[j].r1 = K[j].r1 + dr[j][1];
                        K[j].x0 = K[j].x0 + dx[j][0];
                        K[j].x1 = K[j].x1 + dx[j][1];
                        as_certify(K[j], P, A2, Bv, S, j * NH + lane, opaque(pk[j]), dx[j][0], dx[j][1],
                                   vn[j][0], vn[j][1], pl[j][0], pl[j][1], okp, neg, viol);
                    }
                }
                AS_STAMP_ADD(8, t_c);
            }
            AS_STAMP(t_o);
            if (__ballot(!okp) == 0) {
                certified = true;
                AS_STAMP_ADD(9, t_o);
                break;
            }
            const bool more = __ballot(neg || viol) != 0;
#pragma unroll
            for (int j = 0; j < KPL; ++j) {
                K[j].r0 = sv[j][0];
                K[j].r1 = sv[j][1];
                K[j].x0 = sv[j][2];
                K[j].x1 = sv[j][3];
            }
            AS_STAMP_ADD(9, t_o);
            if (!more) break;
        }
    }
    AS_STAMP(t_out);

    // ---- outputs: the solution (certified), the oracle's outputs of a bad or failed start
    //      (status 3 / 2), or the start point for the IPM kernel's stage 2 (kPending) ----
    const bool done = certified || status != 0;
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const int k = KPL * lane + j;
        if (k < N) {
            const int64_t st = p * N + k;
            vrp_out[2 * st] = K[j].r0;
            vrp_out[2 * st + 1] = K[j].r1;
            const int64_t sx = p * (N + 1) + (k + 1);
            xi_out[2 * sx] = K[j].x0;
            xi_out[2 * sx + 1] = K[j].x1;
            if (LAMOUT && done) {   // the optimum's multipliers: active facets, 0 elsewhere
                const int pc = certified ? (pk[j] & 3) : 0, pi1 = (pk[j] >> 2) & 7, pi2 = (pk[j] >> 5) & 7;
                const double l1 = pl[j][0] > 0.0 ? pl[j][0] : 0.0;
                const double l2 = pl[j][1] > 0.0 ? pl[j][1] : 0.0;
                double* lo = lam_out + st * M;
                for (int i = 0; i < M; ++i)
                    lo[i] = (i < K[j].m && pc >= 1 && i == pi1) ? l1 : (i < K[j].m && pc == 2 && i == pi2) ? l2 : 0.0;
            }
        }
    }
    if (lane == 0) {
        xi_out[2 * p * (N + 1)] = xi00;
        xi_out[2 * p * (N + 1) + 1] = xi01;
        status_out[p] = done ? status : kPending;
        if (done) {
            iters_out[p] = 0;
            if (polished_out) polished_out[p] = certified ? 1 : 0;
        }
    }
    AS_STAMP_ADD(11, t_out);
    AS_STAMP_ADD(0, t_start);
}

template <int KPL>
blf_status launch_kpl(const KParams& kp, const blf_dcm_mpc_problem* pb, const blf_dcm_mpc_warm_start* warm,
                      int64_t batch, const blf_dcm_mpc_solution* sol, double* lam_out, hipStream_t s)
{
    const size_t lds = 3 * sizeof(double) * (size_t)kp.M * (KPL * ((kp.N + KPL - 1) / KPL));
    auto kern = (warm != nullptr)
                    ? (lam_out ? dcm_mpc_as_kernel<KPL, true, true> : dcm_mpc_as_kernel<KPL, true, false>)
                    : (lam_out ? dcm_mpc_as_kernel<KPL, false, true> : dcm_mpc_as_kernel<KPL, false, false>);
    hipLaunchKernelGGL(kern, dim3((unsigned)batch), dim3(kWave), lds, s, kp, pb->xi_init, pb->omega,
                       pb->xi_ref, pb->vrp_ref, pb->A, pb->b, pb->nfacets, warm ? warm->vrp : nullptr,
                       warm ? warm->lambda : nullptr, sol->xi, sol->vrp, sol->status, sol->iters,
                       sol->polished, lam_out);
    return check_hip(hipGetLastError(), "dcm_mpc_as_kernel launch");
}

}  // namespace

#ifdef BLF_STAMPS
extern "C" int blf_debug_as_stamps(unsigned long long* out, int reset)
{
    unsigned long long h[16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_as_stamps), sizeof(h)) != hipSuccess) return -1;
    for (int i = 0; i < 16; ++i) out[i] = h[i];
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_as_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

// Active-set kernel of a launch_dcm_mpc call (N <= 128, tol_polish > 0): every QP either solved
// (status 0, polished) or marked kPending for the IPM kernel's stage 2.
blf_status launch_dcm_mpc_as(const qp::KParams& kp, const blf_dcm_mpc_problem* pb,
                             const blf_dcm_mpc_warm_start* warm, int64_t batch,
                             const blf_dcm_mpc_solution* sol, double* lam_out, hipStream_t s)
{
    if (kp.N <= kWave) return launch_kpl<1>(kp, pb, warm, batch, sol, lam_out, s);
    if (kp.N <= 2 * kWave) return launch_kpl<2>(kp, pb, warm, batch, sol, lam_out, s);
    return set_error(BLF_ERR_UNSUPPORTED, "active-set kernel: horizon %d > 128", kp.N);
}

}  // namespace blf
