// dcm_mpc_as.hip — batched time-varying DCM MPC QP, active-set start on ONE wavefront per QP
// (TimeVaryingDCMPlanner).
//
// Almost every QP of a batch is solved by the active-set start: exact
// equality-constrained solves, each certified or corrected by drop/add moves.  This kernel runs
// exactly that part, and nothing of the interior point method, so a knot carries no slacks or
// multipliers:
//   * one 64-lane wavefront per QP; lane l owns knot l (N <= 64) or the knot pair (2l, 2l + 1)
//     (N <= 128).  A scan composes the pair in the lane, runs Kogge-Stone over the 64 lanes on one
//     element per lane and applies the pair's inner knot in the lane: 7 compositions per scan
//     instead of 12 for two knots per lane on separate wavefronts, and no barrier at all.  The
//     oracle evaluates the start in the same tree (oracle scan_backward_pairs etc.), bit for bit;
//   * the facet rows are staged once in LDS from coalesced loads of the QP's contiguous A / b
//     slabs (consecutive lanes on consecutive 16 B), [M][slot][lane].
// The pass loop is bound by fp64 VALU issue, so a cold start searches for the
// active set in fp32 first: the LQ optimum and the drop/add passes in float
// (half the issue cycles, half the lane shuffles), then the fp64 passes start from the float
// solution with the float search's active set as their guess and certify it, in 1.01 passes on
// average instead of 4.7.  Every arithmetic step is templated on the scalar type and mirrored by
// the oracle (oracle/blf_oracle_as32.c for the float search), so the results stay bit-identical.
// A QP whose fp64 passes do not certify gets the fp64 LQ optimum as its start point, status
// kPending, and the IPM kernel's stage 2 (dcm_mpc_ipm.hip) continues from there exactly as the
// oracle does after a failed start.  Small batches with N <= 64 (configs[0]) run that stage 2 in
// the same workgroup instead (dcm_mpc_cold_fused_kernel): one launch for the whole solve.
#include "dcm_qp_common.h"
#include "dcm_mpc_ipm_body.h"

#include <stdlib.h>

namespace blf {
namespace {
using namespace qp;

#ifdef BLF_STAMPS
// Diagnostic build only (make stamps): per-phase cycle sums of lane 0 for the first 64 QPs.
// [0] whole kernel, [1] slab staging + knot loads, [2] LQ step (fp32 for cold starts), [3] guess,
// [4] pass: setup + residuals, [5] pass: Riccati sweep, [6] pass: h, [7] pass: solve,
// [8] pass: certificate, [9] pass: vote + restore, [10] fp64 passes (count), [11] outputs,
// [12] fp32 passes (count), [13] fp32 passes (cycles), [14] fp64 passes (cycles), [15] kernel B
// (cycles); [16..21] the fp32 passes' phases as [4..9].  Kernel A: [0] [1] [2] [3] [12] [13] [16..21].
__device__ unsigned long long g_as_stamps[32];
// per-workgroup timeline of the first 65536 QPs: s_memrealtime (100 MHz) at start and end, and
// s_memtime at start and end (shader clock), for the clock and the residency over the launch
__device__ unsigned long long g_as_timeline[65536 * 4];
__device__ unsigned long long g_as32_timeline[65536 * 4];   // the same for the cold-start kernel
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

// Parameters of the pass arithmetic in the scalar type T: the QP's own for the fp64 passes, their
// float roundings and the search tolerances for the fp32 search.
template <class T>
struct PT {
    T dt, Qw0, Qw1, Rw0, Rw1, Pw0, Pw1, tol_p, tol_d;
};

__device__ __forceinline__ PT<double> params_d(const KParams& P)
{
    return {P.dt, P.Qw0, P.Qw1, P.Rw0, P.Rw1, P.Pw0, P.Pw1, P.tol_p, P.tol_d};
}

__device__ __forceinline__ PT<float> params_f(const KParams& P)
{
    return {P.f_dt, P.f_Qw0, P.f_Qw1, P.f_Rw0, P.f_Rw1, P.f_Pw0, P.f_Pw1, P.f_tol_p, P.f_tol_d};
}

// Per-knot state of the active-set passes.
template <class T>
struct AKnotT {
    int m;                          // facet count
    int gm;                         // the start's guess (bit i: facet i)
    int drop, add;                  // facets taken out of / put into the guess by earlier passes
    T r0, r1;                       // VRP
    T x0, x1;                       // xi_{k+1}
    T w, al, be;                    // omega_k, 1 + dt omega_k, dt omega_k
    T rh0, rh1, d0, d1, qx0, qx1;
    T P00, P01, P11;                // P_{k+1}
    T h00, h01, h11;                // H_k^{-1} of the active subspace
    T rr0, rr1, xr0, xr1;           // vrp_ref_k, xi_ref_{k+1}
};
using AKnot = AKnotT<double>;

// The QP's facet rows in LDS, [M][S] normals and [M][S] offsets (facet i of column col at
// i S + col), fp64 (rounded to float as the fp32 search reads them).
template <class V, int MF = kMaxFacets>
struct LdsRows;
// at(): a 24-bit multiply (v_mul_u32_u24, full rate; i < 8, S <= 128) for the per-lane facet
// indices of the passes, which v_mul_lo_u32 (quarter rate) took before.
template <int MF>
struct LdsRows<double, MF> {
    static constexpr int kMF = MF;   // facet slots (8, or 16 for phases of three or four contacts)
    using V2 = double2;
    const double2* A2;
    const double* Bv;
    int S, NH;
    __device__ int col(int j, int lane) const { return j * NH + lane; }
    __device__ int at(int i, int col) const { return (int)__umul24((unsigned)i, (unsigned)S) + col; }
};
template <int MF>
struct LdsRows<float, MF> {
    static constexpr int kMF = MF;
    using V2 = float2;
    const float2* A2;
    const float* Bv;
    int S, NH;
    __device__ int col(int j, int lane) const { return j * NH + lane; }
    __device__ int at(int i, int col) const { return (int)__umul24((unsigned)i, (unsigned)S) + col; }
};

// BLF_AS_MINWAVES: the fused cold kernel's __launch_bounds__ waves per SIMD (A/B builds);
#ifndef BLF_AS_MINWAVES
#define BLF_AS_MINWAVES 2
#endif
#ifndef BLF_AS_OVERLAP
#define BLF_AS_OVERLAP 1
#endif
#ifndef BLF_AS_KEEPIN
#define BLF_AS_KEEPIN 1
#endif
// A/B builds only (the oracle restates the product, 1 / 1): the anti-cycling rule of the fp64
// passes and the refinement of multiplier-1e4+ optima
#ifndef BLF_AS_ANTICYCLE
#define BLF_AS_ANTICYCLE 1
#endif
#ifndef BLF_AS_REFINE
#define BLF_AS_REFINE 1
#endif

// One facet row (normal, offset) in the scalar type of the pass.
template <class T>
struct Row {
    T x, y, b;
};

template <class T, class RS>
__device__ __forceinline__ Row<T> row(const RS& R, int i, int col)
{
    const int o = R.at(i, col);
    const auto a = R.A2[o];
    return {T(a.x), T(a.y), T(R.Bv[o])};
}

template <class T, class RS>
__device__ __forceinline__ Row<T> normal(const RS& R, int i, int col)
{
    const auto a = R.A2[R.at(i, col)];
    return {T(a.x), T(a.y), T(0)};
}

// The knots of a lane (oracle scan_backward_as / scan_forward_as / riccati_sweep_as):
//   KPL = 1 (N <= 64): lane l owns knot l; the tree (TR, below) runs over the 64 lanes (kTreeKS is
//            the IPM kernel's tree for one wavefront);
//   KPL = 2 (N <= 128): lane l owns the knot pair (2l, 2l + 1): the pair's element is composed in
//            the lane, the tree runs over the 64 lanes on one element per lane, and the pair's
//            inner knot is applied in the lane afterwards.
// Slot j of a lane is knot KPL lane + j.  Knots >= N carry the zero element (affine scans) or the
// identity (Riccati).

// kTreePad (KPL = 2, N <= 126): lane 63 holds no knot, so it carries the zero element (affine scans) or
// the identity (Riccati) at every level.  A lane whose partner would lie past the wavefront then
// combines with lane 63 instead of being masked: the combine leaves its vector part unchanged
// (signed zeros aside; the oracle's pair tree does the same), and the level needs no exec mask,
// no branch and no write-back of temporaries (0.141 -> 0.133 ms at B = 4096).

// The scan tree of a launch (template parameter TR of the kernels and the scans):
//   kTreeKS:  Kogge-Stone over the 64 lanes, distance 1 by DPP, 2..32 by ds_bpermute; a lane whose
//             partner lies past the wavefront does not combine;
//   kTreePad: the same for KPL = 2 with N <= 126 (as_pad): lane 63 holds no knot and carries the
//             zero element / identity, and a lane whose partner lies past the wavefront combines
//             with lane 63 instead, so no level needs an exec mask (0.141 -> 0.133 ms at B = 4096);
//   kTreeDpp: every level a VALU move, no LDS round trip (tree_fwd / tree_bwd of dcm_qp_common.h:
//             Kogge-Stone inside each row of 16 lanes by DPP row shifts, then two row-level steps).
//             It issues more VALU than the ds_bpermute levels, which move data through the LDS
//             pipe, but shortens the dependency chain: with one knot per lane (N <= 64) it is
//             4-8 % faster up to 1024 QPs and even at 2048-4096; with knot pairs it is slower at
//             every batch size (3-8 %), and so is a fully DPP tree at B = 4096.
//             So it serves N <= 64 at up to kDppTreeMaxBatch QPs (the oracle's as_tree rule).
// The pad kernels tell the compiler which as_pad value holds, so every scan's pad test folds.
enum : int { kTreeKS = 0, kTreePad = 1, kTreeDpp = 2 };

template <int KPL, int TR>
__device__ __forceinline__ void assume_pad(int N)
{
    if (KPL == 2 && TR != kTreeDpp) __builtin_assume((TR == kTreePad) == (N <= 2 * kWave - 2));
}

// One level L of the DPP tree for the affine scans: (g, e) <- (g, e) o the element of the level's
// source lane, on the lanes that have one (tree_has); the others keep their element.
template <int L, bool FWD, class T>
__device__ __forceinline__ void aff_level(T& g0, T& g1, T& g2, T& g3, T& e0, T& e1, int lane)
{
    T p0, p1, p2, p3, q0, q1;
    if constexpr (FWD) {
        p0 = tree_fwd<L>(g0); p1 = tree_fwd<L>(g1); p2 = tree_fwd<L>(g2);
        p3 = tree_fwd<L>(g3); q0 = tree_fwd<L>(e0); q1 = tree_fwd<L>(e1);
    } else {
        p0 = tree_bwd<L>(g0); p1 = tree_bwd<L>(g1); p2 = tree_bwd<L>(g2);
        p3 = tree_bwd<L>(g3); q0 = tree_bwd<L>(e0); q1 = tree_bwd<L>(e1);
    }
    if (tree_has<L, FWD>(lane)) COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, e0, e1);
}

template <bool FWD, class T>
__device__ __forceinline__ void aff_tree(T& g0, T& g1, T& g2, T& g3, T& e0, T& e1, int lane)
{
    aff_level<0, FWD>(g0, g1, g2, g3, e0, e1, lane);
    aff_level<1, FWD>(g0, g1, g2, g3, e0, e1, lane);
    aff_level<2, FWD>(g0, g1, g2, g3, e0, e1, lane);
    aff_level<3, FWD>(g0, g1, g2, g3, e0, e1, lane);
    aff_level<4, FWD>(g0, g1, g2, g3, e0, e1, lane);
    aff_level<5, FWD>(g0, g1, g2, g3, e0, e1, lane);
}

// One level of the Riccati scan in the DPP tree (backward): e <- e o the source lane's element.
template <int L, class T>
__device__ __forceinline__ void rc_tree(RcT<T>& e, bool& ok, int lane)
{
    RcT<T> q;
    q.a0 = tree_bwd<L>(e.a0); q.a1 = tree_bwd<L>(e.a1); q.a2 = tree_bwd<L>(e.a2); q.a3 = tree_bwd<L>(e.a3);
    q.g0 = tree_bwd<L>(e.g0); q.g1 = tree_bwd<L>(e.g1); q.g2 = tree_bwd<L>(e.g2);
    q.h0 = tree_bwd<L>(e.h0); q.h1 = tree_bwd<L>(e.h1); q.h2 = tree_bwd<L>(e.h2);
    if (tree_has<L, false>(lane)) ok = rc_combine(e, q) && ok;
}

// Backward affine scan v_k = G_k v_{k+1} + c_k, v_N = 0.  Returns v_{k+1} per slot.
template <int KPL, int TR, class T>
__device__ __forceinline__ void as_scan_backward(const T (&G)[KPL][4], const T (&c)[KPL][2], int lane,
                                                 T (&vn)[KPL][2])
{
    T g0 = G[0][0], g1 = G[0][1], g2 = G[0][2], g3 = G[0][3], e0 = c[0][0], e1 = c[0][1];
    if constexpr (KPL == 2)   // knot 2l after knot 2l + 1
        COMPOSE(g0, g1, g2, g3, G[1][0], G[1][1], G[1][2], G[1][3], c[1][0], c[1][1], e0, e1);
    const int ln = opaque(lane);
    if constexpr (TR == kTreeDpp) {
        aff_tree<false>(g0, g1, g2, g3, e0, e1, lane);
    } else if (KPL == 2 && TR == kTreePad) {
        {   // d = 1 (DPP)
            const T p0 = dpp1<kNextKeep>(g0), p1 = dpp1<kNextKeep>(g1), p2 = dpp1<kNextKeep>(g2);
            const T p3 = dpp1<kNextKeep>(g3), q0 = dpp1<kNextKeep>(e0), q1 = dpp1<kNextKeep>(e1);
            COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, e0, e1);
        }
#pragma unroll
        for (int d = 2; d < kWave; d <<= 1) {
            const int ad = min(ln + d, kWave - 1) << 2;
            const T p0 = bperm(ad, g0), p1 = bperm(ad, g1), p2 = bperm(ad, g2), p3 = bperm(ad, g3);
            const T q0 = bperm(ad, e0), q1 = bperm(ad, e1);
            COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, e0, e1);
        }
    } else {
        {
            const T p0 = dpp1<kNextWrap>(g0), p1 = dpp1<kNextWrap>(g1), p2 = dpp1<kNextWrap>(g2);
            const T p3 = dpp1<kNextWrap>(g3), q0 = dpp1<kNextWrap>(e0), q1 = dpp1<kNextWrap>(e1);
            if (ln + 1 < kWave) COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, e0, e1);
        }
#pragma unroll
        for (int d = 2; d < kWave; d <<= 1) {
            const int ad = ((ln + d) & (kWave - 1)) << 2;
            const T p0 = bperm(ad, g0), p1 = bperm(ad, g1), p2 = bperm(ad, g2), p3 = bperm(ad, g3);
            const T q0 = bperm(ad, e0), q1 = bperm(ad, e1);
            if (ln + d < kWave) COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, e0, e1);
        }
    }
    // e = v at this lane's first knot; the next lane's = v past this lane's last knot
    T vb0 = dpp1<kNextWrap>(e0), vb1 = dpp1<kNextWrap>(e1);
    if (lane == kWave - 1) {
        vb0 = T(0);
        vb1 = T(0);
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
template <int KPL, int TR, class T>
__device__ __forceinline__ void as_scan_forward(const T (&F)[KPL][4], const T (&f)[KPL][2], int lane,
                                                T (&x)[KPL][2], T (&xk)[KPL][2])
{
    constexpr int L = KPL - 1;   // the lane's last knot
    T g0 = F[L][0], g1 = F[L][1], g2 = F[L][2], g3 = F[L][3], e0 = f[L][0], e1 = f[L][1];
    if constexpr (KPL == 2)   // knot 2l + 1 after knot 2l
        COMPOSE(g0, g1, g2, g3, F[0][0], F[0][1], F[0][2], F[0][3], f[0][0], f[0][1], e0, e1);
    const int ln = opaque(lane);
    if constexpr (TR == kTreeDpp) {
        aff_tree<true>(g0, g1, g2, g3, e0, e1, lane);
    } else if (KPL == 2 && TR == kTreePad) {   // lanes before the first partner take lane 63's zero element (as_pad)
        {   // d = 1 (DPP; lane 0 takes lane 63's)
            const T p0 = dpp1<kPrevWrap>(g0), p1 = dpp1<kPrevWrap>(g1), p2 = dpp1<kPrevWrap>(g2);
            const T p3 = dpp1<kPrevWrap>(g3), q0 = dpp1<kPrevWrap>(e0), q1 = dpp1<kPrevWrap>(e1);
            COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, e0, e1);
        }
#pragma unroll
        for (int d = 2; d < kWave; d <<= 1) {
            const int ad = (ln >= d ? ln - d : kWave - 1) << 2;
            const T p0 = bperm(ad, g0), p1 = bperm(ad, g1), p2 = bperm(ad, g2), p3 = bperm(ad, g3);
            const T q0 = bperm(ad, e0), q1 = bperm(ad, e1);
            COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, e0, e1);
        }
    } else {
        {
            const T p0 = dpp1<kPrevWrap>(g0), p1 = dpp1<kPrevWrap>(g1), p2 = dpp1<kPrevWrap>(g2);
            const T p3 = dpp1<kPrevWrap>(g3), q0 = dpp1<kPrevWrap>(e0), q1 = dpp1<kPrevWrap>(e1);
            if (ln >= 1) COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, e0, e1);
        }
#pragma unroll
        for (int d = 2; d < kWave; d <<= 1) {
            const int ad = ((ln - d) & (kWave - 1)) << 2;
            const T p0 = bperm(ad, g0), p1 = bperm(ad, g1), p2 = bperm(ad, g2), p3 = bperm(ad, g3);
            const T q0 = bperm(ad, e0), q1 = bperm(ad, e1);
            if (ln >= d) COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, e0, e1);
        }
    }
    // e = x past this lane's last knot; the previous lane's = x at this lane's first knot
    T xb0 = dpp1<kPrevWrap>(e0), xb1 = dpp1<kPrevWrap>(e1);
    if (lane == 0) {
        xb0 = T(0);
        xb1 = T(0);
    }
    xk[0][0] = xb0;
    xk[0][1] = xb1;
    if constexpr (KPL == 2) {
        const T x10 = FD3(F[0][0], xb0, F[0][1], xb1, f[0][0]);   // x_{2l+1}
        const T x11 = FD3(F[0][2], xb0, F[0][3], xb1, f[0][1]);
        x[0][0] = x10;
        x[0][1] = x11;
        xk[1][0] = x10;
        xk[1][1] = x11;
    }
    x[L][0] = e0;
    x[L][1] = e1;
}

// xi_k of every slot: the previous knot's xi_{k+1} (lane 0, slot 0: xi_init).
template <int KPL, class T>
__device__ __forceinline__ void as_xi_prev(const AKnotT<T> (&K)[KPL], int lane, T xi00, T xi01, T (&xk)[KPL][2])
{
    constexpr int L = KPL - 1;
    xk[0][0] = dpp1<kPrevWrap>(K[L].x0);
    xk[0][1] = dpp1<kPrevWrap>(K[L].x1);
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
template <class T>
__device__ __forceinline__ void as_residuals(AKnotT<T>& K, const PT<T>& P, bool last, T xk0, T xk1)
{
    K.rh0 = P.Rw0 * (K.r0 - K.rr0);
    K.rh1 = P.Rw1 * (K.r1 - K.rr1);
    const T dx0 = FD2(K.w, xk0, -K.w, K.r0);
    K.d0 = fma(dx0, P.dt, xk0) - K.x0;
    const T dx1 = FD2(K.w, xk1, -K.w, K.r1);
    K.d1 = fma(dx1, P.dt, xk1) - K.x1;
    const T q0 = last ? P.Pw0 : P.Qw0;
    const T q1 = last ? P.Pw1 : P.Qw1;
    K.qx0 = q0 * (K.x0 - K.xr0);
    K.qx1 = q1 * (K.x1 - K.xr1);
}

// Riccati sweep (oracle riccati_sweep_pairs; KPL = 1: riccati_sweep on one wavefront): leaves
// P_{k+1} in K; false on a lane where some (I + G H) or (I + G P) is not positive definite.
template <class T>
__device__ __forceinline__ void rc_knot(RcT<T>& e, bool own, T al, const T (&E)[3], const PT<T>& P)
{
    if (own) {
        e.a0 = al; e.a1 = T(0); e.a2 = T(0); e.a3 = al;
        e.g0 = E[0]; e.g1 = E[1]; e.g2 = E[2];
        e.h0 = P.Qw0; e.h1 = T(0); e.h2 = P.Qw1;
    } else {
        e.a0 = T(1); e.a1 = T(0); e.a2 = T(0); e.a3 = T(1);
        e.g0 = e.g1 = e.g2 = T(0);
        e.h0 = e.h1 = e.h2 = T(0);
    }
}

template <int KPL, int TR, class T>
__device__ __forceinline__ bool as_riccati(AKnotT<T> (&K)[KPL], const PT<T>& P, const T (&E)[KPL][3], int N,
                                           int lane)
{
    bool ok = true;
    RcT<T> e;
    rc_knot(e, KPL * lane < N, K[0].al, E[0], P);
    if constexpr (KPL == 2) {
        RcT<T> e1;
        rc_knot(e1, KPL * lane + 1 < N, K[1].al, E[1], P);
        ok = rc_combine(e, e1) && ok;
    }
    const int ln = opaque(lane);
    constexpr bool pad = KPL == 2 && TR == kTreePad;
    auto level = [&](int ad, RcT<T>& q) {
        q.a0 = bperm(ad, e.a0); q.a1 = bperm(ad, e.a1); q.a2 = bperm(ad, e.a2); q.a3 = bperm(ad, e.a3);
        q.g0 = bperm(ad, e.g0); q.g1 = bperm(ad, e.g1); q.g2 = bperm(ad, e.g2);
        q.h0 = bperm(ad, e.h0); q.h1 = bperm(ad, e.h1); q.h2 = bperm(ad, e.h2);
    };
    auto level1 = [&](RcT<T>& q) {   // d = 1 (DPP; as_pad: lane 63 keeps its own identity)
        if (pad) {
            q.a0 = dpp1<kNextKeep>(e.a0); q.a1 = dpp1<kNextKeep>(e.a1);
            q.a2 = dpp1<kNextKeep>(e.a2); q.a3 = dpp1<kNextKeep>(e.a3);
            q.g0 = dpp1<kNextKeep>(e.g0); q.g1 = dpp1<kNextKeep>(e.g1); q.g2 = dpp1<kNextKeep>(e.g2);
            q.h0 = dpp1<kNextKeep>(e.h0); q.h1 = dpp1<kNextKeep>(e.h1); q.h2 = dpp1<kNextKeep>(e.h2);
        } else {
            q.a0 = dpp1<kNextWrap>(e.a0); q.a1 = dpp1<kNextWrap>(e.a1);
            q.a2 = dpp1<kNextWrap>(e.a2); q.a3 = dpp1<kNextWrap>(e.a3);
            q.g0 = dpp1<kNextWrap>(e.g0); q.g1 = dpp1<kNextWrap>(e.g1); q.g2 = dpp1<kNextWrap>(e.g2);
            q.h0 = dpp1<kNextWrap>(e.h0); q.h1 = dpp1<kNextWrap>(e.h1); q.h2 = dpp1<kNextWrap>(e.h2);
        }
    };
    if constexpr (TR == kTreeDpp) {
        rc_tree<0>(e, ok, lane);
        rc_tree<1>(e, ok, lane);
        rc_tree<2>(e, ok, lane);
        rc_tree<3>(e, ok, lane);
        rc_tree<4>(e, ok, lane);
        rc_tree<5>(e, ok, lane);
    } else if (pad) {   // past the wavefront: lane 63's identity (as_pad)
        {
            RcT<T> q;
            level1(q);
            ok = rc_combine(e, q) && ok;
        }
#pragma unroll
        for (int d = 2; d < kWave; d <<= 1) {
            RcT<T> q;
            level(min(ln + d, kWave - 1) << 2, q);
            ok = rc_combine(e, q) && ok;
        }
    } else {
        {
            RcT<T> q;
            level1(q);
            if (ln + 1 < kWave) ok = rc_combine(e, q) && ok;
        }
#pragma unroll
        for (int d = 2; d < kWave; d <<= 1) {
            RcT<T> q;
            level(((ln + d) & (kWave - 1)) << 2, q);
            if (ln + d < kWave) ok = rc_combine(e, q) && ok;
        }
    }
    // P at this lane's first knot; the next lane's (terminal past the last lane)
    T P00, P01, P11;
    ok = rc_apply(e, P.Pw0, T(0), P.Pw1, P00, P01, P11) && ok;
    T Pn00 = dpp1<kNextWrap>(P00), Pn01 = dpp1<kNextWrap>(P01), Pn11 = dpp1<kNextWrap>(P11);
    if (lane == kWave - 1) {
        Pn00 = P.Pw0;
        Pn01 = T(0);
        Pn11 = P.Pw1;
    }
    constexpr int L = KPL - 1;
    K[L].P00 = Pn00;
    K[L].P01 = Pn01;
    K[L].P11 = Pn11;
    if constexpr (KPL == 2) {   // P_{2l+1} = f_{2l+1}(P_{2l+2}), the first knot's P_{k+1}
        RcT<T> e1;
        rc_knot(e1, KPL * lane + 1 < N, K[1].al, E[1], P);
        T o00, o01, o11;
        ok = rc_apply(e1, Pn00, Pn01, Pn11, o00, o01, o11) && ok;
        K[0].P00 = o00;
        K[0].P01 = o01;
        K[0].P11 = o11;
    }
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        if (KPL * lane + j == N - 1) {
            K[j].P00 = P.Pw0;
            K[j].P01 = T(0);
            K[j].P11 = P.Pw1;
        }
    }
    return ok;
}

// Solve the factored Newton system for the right-hand side g (IPM kernel solve) over every slot.
template <int KPL, int TR, class T>
__device__ __forceinline__ void as_solve(const AKnotT<T> (&K)[KPL], const T (&g)[KPL][2], int N, int lane,
                                         T (&dr)[KPL][2], T (&dx)[KPL][2], T (&vn)[KPL][2])
{
    T G[KPL][4], c[KPL][2], y[KPL][2];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        G[j][0] = G[j][1] = G[j][2] = G[j][3] = T(0);
        c[j][0] = c[j][1] = y[j][0] = y[j][1] = T(0);
        if (KPL * lane + j < N) {
            const AKnotT<T>& Kj = K[j];
            const T b2 = Kj.be * Kj.be;
            const T ab = Kj.al * Kj.be;
            const T m00 = FD2(Kj.P00, Kj.h00, Kj.P01, Kj.h01);
            const T m01 = FD2(Kj.P00, Kj.h01, Kj.P01, Kj.h11);
            const T m10 = FD2(Kj.P01, Kj.h00, Kj.P11, Kj.h01);
            const T m11 = FD2(Kj.P01, Kj.h01, Kj.P11, Kj.h11);
            y[j][0] = FD3(Kj.P00, Kj.d0, Kj.P01, Kj.d1, Kj.qx0);
            y[j][1] = FD3(Kj.P01, Kj.d0, Kj.P11, Kj.d1, Kj.qx1);
            const T Mg0 = FD2(m00, g[j][0], m01, g[j][1]);
            const T Mg1 = FD2(m10, g[j][0], m11, g[j][1]);
            G[j][0] = Kj.al * fma(-b2, m00, T(1));
            G[j][1] = -(Kj.al * (b2 * m01));
            G[j][2] = -(Kj.al * (b2 * m10));
            G[j][3] = Kj.al * fma(-b2, m11, T(1));
            c[j][0] = FD3(G[j][0], y[j][0], G[j][1], y[j][1], ab * Mg0);
            c[j][1] = FD3(G[j][2], y[j][0], G[j][3], y[j][1], ab * Mg1);
        }
    }
    T Gt[KPL][4];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        Gt[j][0] = G[j][0]; Gt[j][1] = G[j][2]; Gt[j][2] = G[j][1]; Gt[j][3] = G[j][3];
    }
    as_scan_backward<KPL, TR, T>(G, c, lane, vn);
    T k[KPL][2], f[KPL][2];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        k[j][0] = k[j][1] = f[j][0] = f[j][1] = T(0);
        if (KPL * lane + j < N) {
            const AKnotT<T>& Kj = K[j];
            const T t0 = y[j][0] + vn[j][0];
            const T t1 = y[j][1] + vn[j][1];
            const T hu0 = fma(-Kj.be, t0, g[j][0]);
            const T hu1 = fma(-Kj.be, t1, g[j][1]);
            k[j][0] = -FD2(Kj.h00, hu0, Kj.h01, hu1);
            k[j][1] = -FD2(Kj.h01, hu0, Kj.h11, hu1);
            f[j][0] = fma(-Kj.be, k[j][0], Kj.d0);
            f[j][1] = fma(-Kj.be, k[j][1], Kj.d1);
        }
    }
    T xk[KPL][2];
    as_scan_forward<KPL, TR, T>(Gt, f, lane, dx, xk);
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const AKnotT<T>& Kj = K[j];
        const T ab = Kj.al * Kj.be;
        const T m00 = FD2(Kj.P00, Kj.h00, Kj.P01, Kj.h01);
        const T m01 = FD2(Kj.P00, Kj.h01, Kj.P01, Kj.h11);
        const T m10 = FD2(Kj.P01, Kj.h00, Kj.P11, Kj.h01);
        const T m11 = FD2(Kj.P01, Kj.h01, Kj.P11, Kj.h11);
        dr[j][0] = fma(ab, FD2(m00, xk[j][0], m10, xk[j][1]), k[j][0]);
        dr[j][1] = fma(ab, FD2(m01, xk[j][0], m11, xk[j][1]), k[j][1]);
    }
}

// The unconstrained LQ optimum: one full Newton step of the QP without the polygon constraints
// (W = 0, lambda = 0) from the current (r, xi) (oracle: dcm_residuals(0), dcm_factor, dcm_solve).
// Returns false when some factorization pivot is not positive definite (status NUMERICAL; the
// step is still taken, as in the oracle).
template <int KPL, int TR, class T>
__device__ __forceinline__ bool as_lq_step(AKnotT<T> (&K)[KPL], const PT<T>& P, int N, int lane, T xi00, T xi01)
{
    T E[KPL][3];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        E[j][0] = E[j][1] = E[j][2] = T(0);
        if (KPL * lane + j < N) {
            const T b2 = K[j].be * K[j].be;
            const T W00 = T(0), W01 = T(0), W11 = T(0), dW = T(0);
            const T detRW = fma(P.Rw0, P.Rw1, FD2(P.Rw1, W00, P.Rw0, W11)) + dW;
            const T ie = b2 / detRW;
            E[j][0] = (P.Rw1 + W11) * ie;
            E[j][1] = -(W01 * ie);
            E[j][2] = (P.Rw0 + W00) * ie;
        }
    }
    bool ok = as_riccati<KPL, TR, T>(K, P, E, N, lane);
    // the residuals after the sweep, which does not read them (their registers stay free across it)
    {
        T xk[KPL][2];
        as_xi_prev<KPL, T>(K, lane, xi00, xi01, xk);
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            const int k = KPL * lane + j;
            if (k < N) as_residuals(K[j], P, k == N - 1, xk[j][0], xk[j][1]);
        }
    }
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        if (KPL * lane + j < N) {
            AKnotT<T>& Kj = K[j];
            const T b2 = Kj.be * Kj.be;
            const T W00 = T(0), W01 = T(0), W11 = T(0), dW = T(0);
            const T B00 = fma(b2, Kj.P00, P.Rw0);
            const T B01 = b2 * Kj.P01;
            const T B11 = fma(b2, Kj.P11, P.Rw1);
            const T H00 = B00 + W00;
            const T H01 = B01 + W01;
            const T H11 = B11 + W11;
            const T detB = fma(B00, B11, -(B01 * B01));
            const T trW = FD2(B11, W00, B00, W11) - T(2) * (B01 * W01);
            const T det = (detB + trW) + dW;
            if (!(det > T(0)) || __builtin_isinf(det)) ok = false;
            const T idet = T(1) / det;
            Kj.h00 = H11 * idet;
            Kj.h01 = -(H01 * idet);
            Kj.h11 = H00 * idet;
        }
    }
    T g[KPL][2], dr[KPL][2], dx[KPL][2], vn[KPL][2];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        g[j][0] = K[j].rh0;
        g[j][1] = K[j].rh1;
    }
    as_solve<KPL, TR, T>(K, g, N, lane, dr, dx, vn);
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        if (KPL * lane + j < N) {
            K[j].r0 = K[j].r0 + dr[j][0];
            K[j].r1 = K[j].r1 + dr[j][1];
            K[j].x0 = K[j].x0 + dx[j][0];
            K[j].x1 = K[j].x1 + dx[j][1];
        }
    }
    return __ballot(!ok) == 0;
}

// More than two candidate lines in a pass: the first pair (i < j in facet order) whose vertex
// satisfies every facet of the knot — a vertex of the support polygon — is the active pair
// (oracle dcm_polish; the double instance is qp::vertex_pair's arithmetic).  Returns 2 with pi1,
// pi2 set, or 3 (no such pair: the pass fails).  Rare, so it reads the rows straight from LDS.
template <class T, class RS>
__device__ __forceinline__ int as_vertex_pair(const RS& R, int kx, int km, int cm, T tol_p, int& pi1,
                                              int& pi2)
{
    for (int x = 0; x < km; ++x) {
        if (!((cm >> x) & 1)) continue;
        for (int y = x + 1; y < km; ++y) {
            if (!((cm >> y) & 1)) continue;
            const Row<T> a = row<T>(R, x, kx);
            const Row<T> e = row<T>(R, y, kx);
            const T det = fma(a.x, e.y, -(a.y * e.x));
            const T aa = FD2(a.x, a.x, a.y, a.y), ee = FD2(e.x, e.x, e.y, e.y);
            if (!(det * det > T(1e-18) * (aa * ee))) continue;
            const T idet = T(1) / det;
            const T v0 = fma(a.b, e.y, -(a.y * e.b)) * idet;
            const T v1 = fma(a.x, e.b, -(a.b * e.x)) * idet;
            bool feas = true;
            for (int l = 0; l < km; ++l) {
                const Row<T> f = row<T>(R, l, kx);
                if (!(FD2(f.x, v0, f.y, v1) - f.b <= tol_p)) feas = false;
            }
            if (feas) {
                pi1 = x;
                pi2 = y;
                return 2;
            }
        }
    }
    return 3;
}

// Candidate facets of a pass -> (pc, pi1, pi2) packed as pc | pi1 << 2 | pi2 << 6, the VRP moved
// onto the active lines and E_k (IPM kernel polish block, "active sets, projection").
// Branch-free: the two knots of a lane, and the lanes of a wavefront, have every mix of 0, 1 and 2
// active lines, so per-case branches serialised all three bodies and their divisions.  Each knot
// instead evaluates exactly two quotients whose operands its case selects (c = 0: b2 / Rw0,
// b2 / Rw1; c = 1: (a r - b) / |a|^2, b2 / (Rw0 a_y^2 + Rw1 a_x^2); c = 2: 1 / det) — the same
// operations as the per-case form of the oracle, so the results are bit-identical.
template <class T, class RS>
__device__ __forceinline__ void as_pass_setup(AKnotT<T>& K, const PT<T>& P, const RS& R, int col, T sr0,
                                              T sr1, int& pk, T (&E)[3], bool& okp)
{
    const int cx = opaque(col);
    const int km = opaque(K.m);
    // candidates: guessed and not dropped, or added (bit i, i < m); the first two in facet order
    const int cm = ((K.gm & ~K.drop) | K.add) & ((1 << km) - 1);
    int pc = __builtin_popcount(cm);
    const int cm2 = cm & (cm - 1);
    int pi1 = cm ? __builtin_ctz(cm) : 0;
    int pi2 = cm2 ? __builtin_ctz(cm2) : 0;
    if (pc > 2) pc = as_vertex_pair<T>(R, cx, km, cm, P.tol_p, pi1, pi2);
    if (pc > 2) okp = false;
    const int c = pc < 3 ? pc : 2;
    pk = c | (pi1 << 2) | (pi2 << 6);
    const T b2 = K.be * K.be;
    const Row<T> a = row<T>(R, pi1, cx);
    const Row<T> e = row<T>(R, pi2, cx);
    const T aa = FD2(a.x, a.x, a.y, a.y);
    const T u = a.y * a.y, v = a.x * a.x, q = a.x * a.y;
    const T det = fma(a.x, e.y, -(a.y * e.x));
    const T n1 = c == 0 ? b2 : c == 1 ? FD2(a.x, sr0, a.y, sr1) - a.b : T(1);
    const T d1 = c == 0 ? P.Rw0 : c == 1 ? aa : det;
    const T d2 = c == 0 ? P.Rw1 : c == 1 ? FD2(P.Rw0, u, P.Rw1, v) : T(1);
    const T q1 = n1 / d1;   // c = 0: E00; c = 1: t; c = 2: 1 / det
    const T q2 = b2 / d2;   // c = 0: E11; c = 1: ie
    if (c == 2) {
        const T ee = FD2(e.x, e.x, e.y, e.y);
        if (!(det * det > T(1e-18) * (aa * ee))) okp = false;   // (nearly) parallel active facets
    }
    const T p0 = c == 1 ? fma(-q1, a.x, sr0) : fma(a.b, e.y, -(a.y * e.b)) * q1;
    const T p1 = c == 1 ? fma(-q1, a.y, sr1) : fma(a.x, e.b, -(a.b * e.x)) * q1;
    K.r0 = c == 0 ? K.r0 : p0;
    K.r1 = c == 0 ? K.r1 : p1;
    E[0] = c == 0 ? q1 : c == 1 ? u * q2 : T(0);
    E[1] = c == 1 ? -(q * q2) : T(0);
    E[2] = c == 0 ? q2 : c == 1 ? v * q2 : T(0);
}

// h_k = H_k^{-1} of the knot's active subspace after the Riccati sweep (IPM kernel polish block):
// c = 0: B^{-1}; c = 1: t t^T / (t^T B t), t = (-a_y, a_x); c = 2: 0.  One quotient per knot,
// operands selected by the case (bit-identical to the per-case form).
template <class T, class RS>
__device__ __forceinline__ void as_pass_h(AKnotT<T>& K, const PT<T>& P, const RS& R, int col, int pk,
                                          bool& okp)
{
    const int pc = pk & 3, pi1 = (pk >> 2) & 15;
    const T b2 = K.be * K.be;
    const T B00 = fma(b2, K.P00, P.Rw0);
    const T B01 = b2 * K.P01;
    const T B11 = fma(b2, K.P11, P.Rw1);
    const Row<T> a = normal<T>(R, pi1, opaque(col));
    const T u = a.y * a.y, v = a.x * a.x, q = a.x * a.y;
    const T detB = fma(B00, B11, -(B01 * B01));
    const T tbt = FD3(B00, u, B11, v, T(-2) * (B01 * q));
    const T den = pc == 0 ? detB : pc == 1 ? tbt : T(1);
    if (pc < 2 && (!(den > T(0)) || __builtin_isinf(den))) okp = false;
    const T id = T(1) / den;
    K.h00 = pc == 0 ? B11 * id : pc == 1 ? u * id : T(0);
    K.h01 = pc == 0 ? -(B01 * id) : pc == 1 ? -(q * id) : T(0);
    K.h11 = pc == 0 ? B00 * id : pc == 1 ? v * id : T(0);
}

// The certificate of one knot after the step (IPM kernel polish block): stationarity with the
// solve's costates, multiplier signs, primal feasibility of every facet; drop / add bookkeeping.
// One quotient per knot (c = 1: (a g) / |a|^2; c = 2: 1 / det), operands selected by the case.
template <class T, class RS>
__device__ __forceinline__ void as_certify(AKnotT<T>& K, const PT<T>& P, const RS& R, int col, int pk,
                                           T dx0, T dx1, T vn0, T vn1, T& l1o, T& l2o, bool& okp, bool& neg,
                                           bool& viol, bool bland, int& ndrop, int& nadd)
{
    const int cx = opaque(col);
    const int pc = pk & 3, pi1 = (pk >> 2) & 15, pi2 = (pk >> 6) & 15;
    const T s0 = K.qx0 + vn0;
    const T s1 = K.qx1 + vn1;
    const T nu0 = FD3(K.P00, dx0, K.P01, dx1, s0);
    const T nu1 = FD3(K.P01, dx0, K.P11, dx1, s1);
    const T rh0 = P.Rw0 * (K.r0 - K.rr0);
    const T rh1 = P.Rw1 * (K.r1 - K.rr1);
    // the costates of the new point (K.rh is free after the solve): the refinement's nu (as_refine)
    K.rh0 = nu0;
    K.rh1 = nu1;
    const T g0 = fma(K.be, nu0, -rh0);
    const T g1 = fma(K.be, nu1, -rh1);
    const Row<T> a = normal<T>(R, pi1, cx);
    const Row<T> e = normal<T>(R, pi2, cx);
    const T n = pc == 1 ? FD2(a.x, g0, a.y, g1) : T(1);
    const T d = pc == 1 ? FD2(a.x, a.x, a.y, a.y) : fma(a.x, e.y, -(a.y * e.x));
    const T qd = n / d;
    const T l1 = pc == 1 ? qd : pc == 2 ? fma(g0, e.y, -(e.x * g1)) * qd : T(0);
    const T l2 = pc == 2 ? fma(a.x, g1, -(g0 * a.y)) * qd : T(0);
    l1o = l1;
    l2o = l2;
    // fp64: the dual tolerance relative to |beta nu| beyond 1 / kTolDualRel (oracle dcm_polish);
    // the fp32 search keeps its absolute kSearchTolD
    T tol_d = P.tol_d;
    if constexpr (sizeof(T) == 8) tol_d = P.tol_d * fmax(1.0, kTolDualRel * fmax(fabs(K.be * nu0), fabs(K.be * nu1)));
    bool bad = false;
    if (pc == 0) bad = !(fabs(g0) <= tol_d) || !(fabs(g1) <= tol_d);
    if (pc == 1) bad = !(fabs(fma(-l1, a.x, g0)) <= tol_d) || !(fabs(fma(-l1, a.y, g1)) <= tol_d);
    const bool n1 = pc >= 1 && !(l1 >= -tol_d);
    const bool n2 = pc == 2 && !(l2 >= -tol_d);
    const int dm = (n1 ? 1 << pi1 : 0) | (n2 ? 1 << pi2 : 0);
    if (bad || dm) okp = false;
    if (dm) neg = true;
    // Bland mode (the anti-cycling rule): the new sets go to ndrop / nadd, applied by as_passes
    int dr = K.drop | dm, ad = K.add & ~dm;
    // primal feasibility of every facet, rows read four at a time
    const int km = opaque(K.m);
    int vm = 0;
#pragma unroll
    for (int i0 = 0; i0 < RS::kMF; i0 += 4) {
        if (i0 >= km) break;
        Row<T> rv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = i0 + q < km ? i0 + q : 0;
            rv[q] = row<T>(R, i, cx);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (!(FD2(rv[q].x, K.r0, rv[q].y, K.r1) - rv[q].b <= P.tol_p)) vm |= 1 << (i0 + q);
    }
    vm &= (1 << km) - 1;
    if (vm) {
        okp = false;
        viol = true;
        ad |= vm;
        dr &= ~vm;
    }
    ndrop = dr;
    nadd = ad;
    if (!bland) {
        K.drop = dr;
        K.add = ad;
    }
}

// r_k back onto its active line after a fp64 step (c = 1; oracle project_line): the step moves r
// along the line in exact arithmetic, but its rounding scales with the step's terms (costates up to
// 1e10 on the pushed-robot windows), and a drift of 1e-10 off the line failed the certificate's
// primal check pass after pass.  One quotient per knot, the result selected by the case.
template <class T, class RS>
__device__ __forceinline__ void as_project(AKnotT<T>& K, const RS& R, int col, int pk)
{
    const int pc = pk & 3, pi1 = (pk >> 2) & 15;
    const Row<T> a = row<T>(R, pi1, opaque(col));
    const T aa = FD2(a.x, a.x, a.y, a.y);
    const T t = (FD2(a.x, K.r0, a.y, K.r1) - a.b) / aa;
    const T p0 = fma(-t, a.x, K.r0);
    const T p1 = fma(-t, a.y, K.r1);
    K.r0 = pc == 1 ? p0 : K.r0;
    K.r1 = pc == 1 ? p1 : K.r1;
}

// The refinement of a certified fp64 optimum (oracle dcm_polish, refine_rhs; dcm_qp_common.h): the
// stationarity residuals at (xi, r, nu) in double-double drive one more Newton step with the
// certified pass's factorization (K.P, K.h).  K.rh holds the certificate's costates nu_k.
template <int KPL, int TR, class RS>
__device__ __forceinline__ void as_refine(AKnot (&K)[KPL], const PT<double>& P, const RS& R, int N, int lane,
                                          double xi00, double xi01, const int (&pk)[KPL])
{
    constexpr int L = KPL - 1;
    for (int rs = 0; rs < kRefineSteps; ++rs) {
    double xk[KPL][2];
    as_xi_prev<KPL, double>(K, lane, xi00, xi01, xk);
    // the next knot's costate and omega: the lane's next slot, or the next lane's first
    double nn0[KPL], nn1[KPL], wn[KPL];
    if constexpr (KPL == 2) {
        nn0[0] = K[1].rh0;
        nn1[0] = K[1].rh1;
        wn[0] = K[1].w;
    }
    nn0[L] = dpp1<kNextWrap>(K[0].rh0);
    nn1[L] = dpp1<kNextWrap>(K[0].rh1);
    wn[L] = dpp1<kNextWrap>(K[0].w);
    double g[KPL][2], dr[KPL][2], dx[KPL][2], vn[KPL][2];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const int k = KPL * lane + j;
        g[j][0] = g[j][1] = 0.0;
        if (k < N) {
            const bool last = k == N - 1;
            const Row<double> a = normal<double>(R, (pk[j] >> 2) & 15, opaque(R.col(j, lane)));
            refine_rhs(xk[j][0], xk[j][1], K[j].x0, K[j].x1, K[j].r0, K[j].r1, K[j].rr0, K[j].rr1, K[j].xr0,
                       K[j].xr1, K[j].w, wn[j], K[j].rh0, K[j].rh1, nn0[j], nn1[j], last, P.dt,
                       last ? P.Pw0 : P.Qw0, last ? P.Pw1 : P.Qw1, P.Rw0, P.Rw1, pk[j] & 3, a.x, a.y, K[j].d0,
                       K[j].d1, K[j].qx0, K[j].qx1, g[j][0], g[j][1]);
        }
    }
    as_solve<KPL, TR, double>(K, g, N, lane, dr, dx, vn);
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        if (KPL * lane + j < N) {
            // the refined point's costates: nu + the step's own (Lagrangian-shifted) costate
            K[j].rh0 = K[j].rh0 + FD3(K[j].P00, dx[j][0], K[j].P01, dx[j][1], K[j].qx0 + vn[j][0]);
            K[j].rh1 = K[j].rh1 + FD3(K[j].P01, dx[j][0], K[j].P11, dx[j][1], K[j].qx1 + vn[j][1]);
            K[j].r0 = K[j].r0 + dr[j][0];
            K[j].r1 = K[j].r1 + dr[j][1];
            K[j].x0 = K[j].x0 + dx[j][0];
            K[j].x1 = K[j].x1 + dx[j][1];
            as_project<double>(K[j], R, R.col(j, lane), pk[j]);
        }
    }
    }
}

// The start's guess: the facets whose slack at the current point is below `thr` (0: the facets it
// violates; the fp64 passes after the fp32 search: kGuessSlack, the facets active at the float
// point); warm starts add those whose previous multiplier exceeds the floor (lw = that knot's
// previous multipliers, or nullptr).
template <int KPL, class T, class RS>
__device__ __forceinline__ void as_guess(AKnotT<T> (&K)[KPL], const RS& R, int NH, int N, int lane,
                                         const double* const (&lw)[KPL], double ws_floor, T thr)
{
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const int k = KPL * lane + j;
        if (k < N) {
            const int col = R.col(j, lane);
            int gm = 0;
            for (int i = 0; i < K[j].m; ++i) {
                const Row<T> a = row<T>(R, i, col);
                const T gr = FD2(a.x, K[j].r0, a.y, K[j].r1);
                const T sl = a.b - gr;
                if (sl < thr) gm |= 1 << i;
                if (lw[j] && lw[j][i] > ws_floor) gm |= 1 << i;
            }
            K[j].gm = gm;
        }
    }
}

// The drop/add passes from the current point and guess (oracle dcm_polish with a guess): each
// pass projects r onto its candidate lines, takes the exact equality-constrained Newton step and
// certifies it; a failed pass drops the facets with negative multipliers, adds the violated ones
// and restores the start point.  Returns true when a pass is certified (the point is then the
// optimum, pk / pl its active facets and multipliers).
// The candidate set of a knot's next pass: guessed and not dropped, or added (bit i, i < m).
template <class T>
__device__ __forceinline__ int as_cand(const AKnotT<T>& K)
{
    return ((K.gm & ~K.drop) | K.add) & ((1 << K.m) - 1);
}

// handover >= 0 (the fp32 search): a failed pass that changed the candidate sets of at most
// `handover` knots ends the search, its next candidate sets going to the fp64 passes instead of
// another float pass (oracle passes32): the last float pass before the
// certifying one changes a few knots, and the fp64 passes certify that set.  -1: never.
#ifndef BLF_AS_OPQLANE   // A/B: 1 (VGPRs 228 -> 221, SGPR spills 36 -> 44) took 0.127 / 0.128 against 0.125 /
#define BLF_AS_OPQLANE 0   // 0.126 ms at B = 4096 (profiles/r04_cstage_asopq_ab.log), so 0
#endif

template <int KPL, int TR, class T, class RS>
__device__ __forceinline__ bool as_passes(AKnotT<T> (&K)[KPL], const PT<T>& P, const RS& R, int NH, int N,
                                          int lane, T xi00, T xi01, int (&pk)[KPL],
                                          T (&pl)[KPL][2], int count_slot, int sb, int handover, int& npass)
{
    T xk[KPL][2];
    as_xi_prev<KPL, T>(K, lane, xi00, xi01, xk);
    bool certified = false;
    const int lane0 = lane;
    // the fp64 passes: up to kAsPasses, the last ones under the anti-cycling rule (oracle
    // dcm_polish anti_cycle: Bland's rule from pass kGuessPasses on); the fp32 search: kGuessPasses
    constexpr bool kAnti = sizeof(T) == 8 && BLF_AS_ANTICYCLE;
    constexpr int kMaxPass = kAnti ? kAsPasses : kGuessPasses;
    int pass = 0;
    for (; pass < kMaxPass; ++pass) {
        const bool bland = kAnti && pass >= kGuessPasses;   // Bland's rule from pass 8 on
        // BLF_AS_OPQLANE: the lane index opaque per pass, so its masks are recomputed inside the
        // pass instead of hoisted out of the loop into SGPRs (which spill)
        int lane = lane0;
        if constexpr (BLF_AS_OPQLANE) asm volatile("" : "+v"(lane));
        AS_COUNT(count_slot);
        AS_STAMP(t_s);
        T sv[KPL][4];
        T E[KPL][3];
        int c0[KPL];
        bool okp = true;
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            const int k = KPL * lane + j;
            c0[j] = as_cand(K[j]);
            sv[j][0] = K[j].r0; sv[j][1] = K[j].r1; sv[j][2] = K[j].x0; sv[j][3] = K[j].x1;
            E[j][0] = E[j][1] = E[j][2] = T(0);
            pk[j] = 0;
            if (k < N) as_pass_setup<T>(K[j], P, R, R.col(j, lane), sv[j][0], sv[j][1], pk[j], E[j], okp);
        }
        AS_STAMP_ADD(sb + 0, t_s);
        AS_STAMP(t_r);
        okp = as_riccati<KPL, TR, T>(K, P, E, N, lane) && okp;
        AS_STAMP_ADD(sb + 1, t_r);
        AS_STAMP(t_h);
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            const int k = KPL * lane + j;
            if (k < N) {
                as_pass_h<T>(K[j], P, R, R.col(j, lane), opaque(pk[j]), okp);
                // the residuals at the projected point (after the sweep, which does not read them)
                as_residuals(K[j], P, k == N - 1, xk[j][0], xk[j][1]);
            }
        }
        AS_STAMP_ADD(sb + 2, t_h);
        // the Newton step, then the certificate (costates of the new point from the solve)
        bool neg = false, viol = false;
        int ndr[KPL], nad[KPL];   // the certificate's new drop / add sets (Bland mode: applied below)
        {
            T g[KPL][2], dr[KPL][2], dx[KPL][2], vn[KPL][2];
#pragma unroll
            for (int j = 0; j < KPL; ++j) {
                g[j][0] = K[j].rh0;
                g[j][1] = K[j].rh1;
            }
            AS_STAMP(t_v);
            as_solve<KPL, TR, T>(K, g, N, lane, dr, dx, vn);
            AS_STAMP_ADD(sb + 3, t_v);
            AS_STAMP(t_c);
#pragma unroll
            for (int j = 0; j < KPL; ++j) {
                pl[j][0] = pl[j][1] = T(0);
                ndr[j] = K[j].drop;
                nad[j] = K[j].add;
                if (KPL * lane + j < N) {
                    K[j].r0 = K[j].r0 + dr[j][0];
                    K[j].r1 = K[j].r1 + dr[j][1];
                    K[j].x0 = K[j].x0 + dx[j][0];
                    K[j].x1 = K[j].x1 + dx[j][1];
                    if constexpr (sizeof(T) == 8) as_project<T>(K[j], R, R.col(j, lane), opaque(pk[j]));
                    as_certify<T>(K[j], P, R, R.col(j, lane), opaque(pk[j]), dx[j][0], dx[j][1], vn[j][0], vn[j][1],
                                  pl[j][0], pl[j][1], okp, neg, viol, kAnti && bland, ndr[j], nad[j]);
                }
            }
            AS_STAMP_ADD(sb + 4, t_c);
        }
        AS_STAMP(t_o);
        if (__ballot(!okp) == 0) {
            certified = true;
            AS_STAMP_ADD(sb + 5, t_o);
            break;
        }
        if constexpr (kAnti) {
            if (bland) {   // Bland: one change, at the lowest knot the certificate changed
                bool ch[KPL];
#pragma unroll
                for (int j = 0; j < KPL; ++j) ch[j] = ndr[j] != K[j].drop || nad[j] != K[j].add;
                bool any = false;
#pragma unroll
                for (int j = 0; j < KPL; ++j) any = any || ch[j];
                const unsigned long long bl = __ballot(any);
                const int ls = bl ? __builtin_ctzll(bl) : -1;
                bool first = true;   // the lane's lowest changed slot is the one kept (lane ls only)
#pragma unroll
                for (int j = 0; j < KPL; ++j) {
                    const bool star = lane == ls && ch[j] && first;
                    if (ch[j]) first = false;
                    const int sd = K[j].drop, sa = K[j].add;
                    const int dn = ndr[j] & ~sd, an = nad[j] & ~sa;
                    const int bt = dn ? (dn & -dn) : (an & -an);
                    K[j].drop = star ? (dn ? (sd | bt) : (sd & ~bt)) : sd;
                    K[j].add = star ? (dn ? (sa & ~bt) : (sa | bt)) : sa;
                }
            }
        }
        const bool more = __ballot(neg || viol) != 0;
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            K[j].r0 = sv[j][0];
            K[j].r1 = sv[j][1];
            K[j].x0 = sv[j][2];
            K[j].x1 = sv[j][3];
        }
        AS_STAMP_ADD(sb + 5, t_o);
        if (!more) break;
        if (handover >= 0) {
            int ch = 0;
#pragma unroll
            for (int j = 0; j < KPL; ++j) ch += __builtin_popcountll(__ballot(as_cand(K[j]) != c0[j]));
            if (ch <= handover) break;
        }
    }
    npass = pass < kMaxPass ? pass + 1 : kMaxPass;   // the passes run (wave-uniform)
    if constexpr (sizeof(T) == 8) {
        // the refinement where the largest multiplier exceeds kRefineLam (oracle ORC_REFINE_LAM)
        bool big = false;
#pragma unroll
        for (int j = 0; j < KPL; ++j) big = big || pl[j][0] > kRefineLam || pl[j][1] > kRefineLam;
        if (BLF_AS_REFINE && certified && __ballot(big) != 0)
            as_refine<KPL, TR>(K, P, R, N, lane0, xi00, xi01, pk);
    }
    return certified;
}

// Stages the QP's facet slabs A [N][M][2], b [N][M] into LDS ([M][S] normals, [M][S] offsets,
// facet i of knot k at i S + (k % KPL) NH + k / KPL), in the scalar type V: coalesced loads
// (consecutive lanes on consecutive 16 B), U per lane in flight before the LDS stores.
template <int U>
__device__ __forceinline__ void stage_rows_issue(const double* Ain, const double* bin, int64_t p, int lane,
                                                 int t0, int nA, double2 (&va)[U], double (&vb)[U])
{
    const double2* As = reinterpret_cast<const double2*>(Ain) + p * nA;
    const double* bs = bin + p * nA;
#pragma unroll
    for (int u = 0; u < U; ++u) {   // clamped, so every load is unconditional
        const int t = min(t0 + u * kWave + lane, nA - 1);
        // read once into LDS: non-temporal, so the streamed rows do not push the problem's knot
        // data (re-read by the fp64 phase) out of L2 (FETCH x 2 per launch 115 -> 100 MB)
        typedef double d2v __attribute__((ext_vector_type(2)));
        const d2v w = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(As + t));
        va[u] = make_double2(w.x, w.y);
        vb[u] = __builtin_nontemporal_load(bs + t);
    }
}

template <int KPL, int U, class V>
__device__ __forceinline__ void stage_rows_commit(const double2 (&va)[U], const double (&vb)[U], int M, int S,
                                                  int NH, int lane, int t0, int nA, V* A2v, V* Bv)
{
    const bool pow2 = (M & (M - 1)) == 0;
    const int sh = __builtin_ctz(M);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int t = t0 + u * kWave + lane;
        if (t < nA) {
            const int k = pow2 ? t >> sh : t / M, i = t - k * M;
            const int o = i * S + (k % KPL) * NH + k / KPL;
            A2v[2 * o] = V(va[u].x);
            A2v[2 * o + 1] = V(va[u].y);
            Bv[o] = V(vb[u]);
        }
    }
}

template <int KPL, int U, class V>
__device__ __forceinline__ void stage_rows(const double* Ain, const double* bin, int64_t p, int N, int M, int S,
                                           int NH, int lane, int t0, int nA, V* A2v, V* Bv)
{
    double2 va[U];
    double vb[U];
    stage_rows_issue<U>(Ain, bin, p, lane, t0, nA, va, vb);
    stage_rows_commit<KPL, U, V>(va, vb, M, S, NH, lane, t0, nA, A2v, Bv);
}

// ---- the phase-indexed input (blf_dcm_mpc_solve_phased) ----
// The window is expanded from the plan's phase table straight into the kernel's LDS, as
// phase_expand_kernel would write it to HBM: the same knot -> phase rule (phase_of), the phase's
// rows verbatim, nfacets = -1 and zero rows / references outside every phase.  LDS after the
// facet rows: the problem's phase begin / end times [2][P] doubles, the knot phases [N+1] int32.
__host__ __device__ inline size_t ph_lds_bytes(int P, int N)
{
    return sizeof(double) * 2 * (size_t)P + sizeof(int32_t) * (size_t)(N + 1);
}

__device__ __forceinline__ void ph_stage_phases(const PhaseSrc& ps, int64_t p, int N, double dt, int lane,
                                                double* sBE, int32_t* sPh)
{
    int np = ps.nphases[p];
    np = np < 0 ? 0 : (np > ps.P ? ps.P : np);
    for (int j = lane; j < np; j += kWave) {
        sBE[j] = ps.begin[p * ps.P + j];
        sBE[ps.P + j] = ps.end[p * ps.P + j];
    }
    __syncthreads();
    for (int k = lane; k <= N; k += kWave)
        sPh[k] = phase_of(sBE, sBE + ps.P, np, (double)(ps.start + k) * dt);
    __syncthreads();
}

// stage_rows from the phase table: slot (k, i) = row i of knot k's phase (zeros outside every
// phase).  The table rows are a few KB per problem, read through the caches.
template <int U>
__device__ __forceinline__ void stage_rows_ph_issue(const PhaseSrc& ps, const int32_t* sPh, int64_t p, int N, int M,
                                                    int lane, double2 (&va)[U], double (&vb)[U], int t0 = 0)
{
    const int nA = N * M;
    const double2* As = reinterpret_cast<const double2*>(ps.A) + p * ps.P * M;
    const double* bs = ps.b + p * ps.P * M;
    const bool pow2 = (M & (M - 1)) == 0;
    const int sh = __builtin_ctz(M);
#pragma unroll
    for (int u = 0; u < U; ++u) {   // clamped, so every load is unconditional
        const int t = min(t0 + u * kWave + lane, nA - 1);
        const int k = pow2 ? t >> sh : t / M, i = t - k * M;
        const int ph = sPh[k];
        const int src = (ph < 0 ? 0 : ph) * M + i;
        const double2 a = As[src];
        const double b = bs[src];
        va[u] = ph < 0 ? make_double2(0.0, 0.0) : a;
        vb[u] = ph < 0 ? 0.0 : b;
    }
}

// ROUNDS = false: one round of U loads per lane covers the rows (M <= kMaxFacets); true: as many
// rounds as N M needs (the 16-slot instantiations)
template <int KPL, int U, bool ROUNDS = false>
__device__ __forceinline__ void stage_rows_ph(const PhaseSrc& ps, const int32_t* sPh, int64_t p, int N, int M,
                                              int S, int NH, int lane, double* A2v, double* Bv)
{
    double2 va[U];
    double vb[U];
    if constexpr (ROUNDS) {
        for (int t0 = 0; t0 < N * M; t0 += U * kWave) {
            stage_rows_ph_issue<U>(ps, sPh, p, N, M, lane, va, vb, t0);
            stage_rows_commit<KPL, U, double>(va, vb, M, S, NH, lane, t0, N * M, A2v, Bv);
        }
    } else {
        stage_rows_ph_issue<U>(ps, sPh, p, N, M, lane, va, vb);
        stage_rows_commit<KPL, U, double>(va, vb, M, S, NH, lane, 0, N * M, A2v, Bv);
    }
}

// The QP's rows into LDS in rounds of U loads per lane (the 16-slot instantiations).
template <int KPL, int U>
__device__ __forceinline__ void stage_rows_rounds(const double* Ain, const double* bin, int64_t p, int N, int M,
                                                  int S, int NH, int lane, double* A2v, double* Bv)
{
    for (int t0 = 0; t0 < N * M; t0 += U * kWave)
        stage_rows<KPL, U, double>(Ain, bin, p, N, M, S, NH, lane, t0, N * M, A2v, Bv);
}

// A knot's own inputs: facet count, omega, references (vrp_ref_k, xi_ref_{k+1}).
struct KnotIn {
    int m;
    double w, rr0, rr1, xr0, xr1;
};

template <bool PH>
__device__ __forceinline__ KnotIn knot_in(int64_t p, int k, int N, const double* omega, const double* xi_ref,
                                          const double* vrp_ref, const int32_t* nfacets, const PhaseSrc& ps,
                                          const int32_t* sPh)
{
    KnotIn r;
    if (PH) {
        const int ph = sPh[k], ph1 = sPh[k + 1];
        const int64_t t0 = p * ps.P + (ph < 0 ? 0 : ph), t1 = p * ps.P + (ph1 < 0 ? 0 : ph1);
        const int m = ps.nf[t0];
        const double a0 = ps.ref[2 * t0], a1 = ps.ref[2 * t0 + 1];
        const double c0 = ps.ref[2 * t1], c1 = ps.ref[2 * t1 + 1];
        r.m = ph < 0 ? -1 : m;
        r.w = omega[p * ps.ostride + k];
        r.rr0 = ph < 0 ? 0.0 : a0;
        r.rr1 = ph < 0 ? 0.0 : a1;
        r.xr0 = ph1 < 0 ? 0.0 : c0;
        r.xr1 = ph1 < 0 ? 0.0 : c1;
    } else {
        const int64_t st = p * N + k, sx = p * (N + 1) + (k + 1);
        r.m = nfacets[st];
        r.w = omega[st];
        r.rr0 = vrp_ref[2 * st];
        r.rr1 = vrp_ref[2 * st + 1];
        r.xr0 = xi_ref[2 * sx];
        r.xr1 = xi_ref[2 * sx + 1];
    }
    return r;
}

// A QP handed to the IPM kernel (status kPending) under the phase-indexed input: its expanded
// window into the caller's scratch, which stage 2 reads as a blf_dcm_mpc_problem.
template <int KPL>
__device__ void ph_write_window(const PhaseSrc& ps, const int32_t* sPh, const double* omega, const double* A2v,
                                const double* Bv, int64_t p, int N, int M, int S, int NH, int lane)
{
    const int nA = N * M;
    for (int t = lane; t < nA; t += kWave) {
        const int k = t / M, i = t - k * M;
        const int o = i * S + (k % KPL) * NH + k / KPL;
        ps.wA[2 * (p * nA + t)] = A2v[2 * o];
        ps.wA[2 * (p * nA + t) + 1] = A2v[2 * o + 1];
        ps.wb[p * nA + t] = Bv[o];
    }
    for (int k = lane; k <= N; k += kWave) {
        const int ph = sPh[k];
        const int64_t tp = p * ps.P + (ph < 0 ? 0 : ph);
        const double r0 = ph < 0 ? 0.0 : ps.ref[2 * tp], r1 = ph < 0 ? 0.0 : ps.ref[2 * tp + 1];
        ps.wxr[2 * (p * (N + 1) + k)] = r0;
        ps.wxr[2 * (p * (N + 1) + k) + 1] = r1;
        if (k < N) {
            ps.wrr[2 * (p * N + k)] = r0;
            ps.wrr[2 * (p * N + k) + 1] = r1;
            ps.wnf[p * N + k] = ph < 0 ? -1 : ps.nf[tp];
            ps.wom[p * N + k] = omega[p * ps.ostride + k];
        }
    }
}

// Outputs of one QP: the solution (certified), the oracle's outputs of a bad start or a failed LQ
// factorization (status 3 / 2), or the start point for the IPM kernel's stage 2 (kPending).
template <int KPL, bool LAMOUT>
__device__ __forceinline__ void as_write_outputs(const AKnot (&K)[KPL], const int (&pk)[KPL], const double (&pl)[KPL][2],
                                                 bool certified, int status, int64_t p, int N, int M, int lane,
                                                 double xi00, double xi01, double* xi_out, double* vrp_out,
                                                 int32_t* status_out, int32_t* iters_out, int32_t* polished_out,
                                                 double* lam_out, int32_t* list, int list_slot, int list_cap,
                                                 int32_t* passes_out, int npass, int pend = kPending)
{
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
                const int pc = certified ? (pk[j] & 3) : 0, pi1 = (pk[j] >> 2) & 15, pi2 = (pk[j] >> 6) & 15;
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
        status_out[p] = done ? status : pend;
        if (passes_out) passes_out[p] = npass;
        if (done) {
            iters_out[p] = 0;
            if (polished_out) polished_out[p] = certified ? 1 : 0;
        } else if (list != nullptr) {
            // stage 2's work list: its kernel loops over the listed QPs only, so a batch with none
            // pending costs one tiny launch (order is irrelevant: each QP is solved on its own)
            // (bounded by the list's capacity: stage 2 reads at most list_cap entries)
            const int at = atomicAdd(&list[list_slot], 1);
            if (at < list_cap) list[2 + at] = (int32_t)p;
        }
    }
}

// ---- the cold-start kernel ----
// One wavefront per QP, the fp64 facet rows in LDS.  Phase A, in float (rows rounded as they are
// read): from (xi_ref, vrp_ref) the LQ optimum, the facets it violates, up to kGuessPasses drop/add
// passes.  Phase B, in fp64: from the float point (the certified one, or the float LQ optimum when
// no pass certified), guess = the facets active there (slack < kGuessSlack), the fp64 passes;
// when none certifies, the fp64 LQ optimum from (xi_ref, vrp_ref) becomes the IPM's start point.
// The cold solve of one QP (the cold kernel's body; the warm kernel runs it for the problems whose
// previous solve failed, blf_dcm_mpc_warm_start.prev_status).
template <int KPL, bool LAMOUT, bool PH, int TR, int MF = kMaxFacets>
__device__ __forceinline__ void cold_solve(
    const KParams& P, const double* __restrict__ xi_init, const double* __restrict__ omega,
    const double* __restrict__ xi_ref, const double* __restrict__ vrp_ref,
    const double* __restrict__ Ain, const double* __restrict__ bin,
    const int32_t* __restrict__ nfacets, double* __restrict__ xi_out, double* __restrict__ vrp_out,
    int32_t* __restrict__ status_out, int32_t* __restrict__ iters_out, int32_t* __restrict__ polished_out,
    double* __restrict__ lam_out, const PhaseSrc& ps, int pend = kPending)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int N = P.N, M = P.M;
    assume_pad<KPL, TR>(N);
    const int NH = (N + KPL - 1) / KPL;
    const int S = KPL * NH;
    double* A2d = smem;                               // [M][S] double2 normals
    double* Bv = smem + 2 * (size_t)M * S;            // [M][S] offsets
    const int lane = threadIdx.x;
    const int64_t p = blockIdx.x;
    const PT<float> Pf = params_f(P);
    AS_STAMP(t_start);
#ifdef BLF_STAMPS
    const unsigned long long t_rt0 = __builtin_amdgcn_s_memrealtime();
#endif

    const int nA = N * M;
    constexpr bool kWide = MF > kMaxFacets;   // 16 slots: the rows staged in rounds
    constexpr int U = KPL == 2 ? 2 * kMaxFacets : kMaxFacets;   // one round covers N M <= 1024 / 512
    double* sBE = smem + 3 * (size_t)M * S;                            // PH: [2][P]
    int32_t* sPh = reinterpret_cast<int32_t*>(sBE + 2 * (size_t)ps.P);  // PH: [N+1]
    // The facet rows' loads are issued first and land in LDS only after the float LQ step, which
    // does not read them: the step's arithmetic runs under the loads' latency (at launch every
    // wave of the first round stages its rows at once).
    // (The phase-indexed input keeps its gathers before the LQ step: issued after the knot loads
    // and committed after the step like the slab loads, it measured 1 % slower on the c3 pipeline,
    // 1.900 / 1.893 against 1.882 / 1.874 ms per step, profiles/r03_ph_overlap_ab.log.)
    constexpr bool kOverlap = !PH && BLF_AS_OVERLAP && !kWide;
    double2 va[U];
    double vb[U];
    if (PH) {
        ph_stage_phases(ps, p, N, P.dt, lane, sBE, sPh);
        stage_rows_ph<KPL, U, kWide>(ps, sPh, p, N, M, S, NH, lane, A2d, Bv);
    } else if (kOverlap) {
        // issued below, after the knot loads: a wait for those (vmcnt counts in issue order) then
        // leaves the younger row loads in flight
    } else if (kWide) {
        stage_rows_rounds<KPL, U>(Ain, bin, p, N, M, S, NH, lane, A2d, Bv);
    } else {
        stage_rows<KPL, U, double>(Ain, bin, p, N, M, S, NH, lane, 0, nA, A2d, Bv);
    }
    const LdsRows<double, MF> R{reinterpret_cast<const typename LdsRows<double, MF>::V2*>(smem),
                                smem + 2 * (size_t)M * S, S, NH};

    AKnotT<float> F[KPL];
    // BLF_AS_KEEPIN: the knots' fp64 inputs kept from phase A's loads for phase B (instead of
    // reading them from global memory again after the float search)
    KnotIn kin[KPL];
    int cand[KPL];         // the float search's next candidate sets (phase B's guess when uncertified)
    bool cert32 = false;   // the float search certified its point
    int npass32 = 0;       // its passes
    const double xi00 = xi_init[2 * p], xi01 = xi_init[2 * p + 1];
    // ---- phase A: the float search (facet counts clamped; a bad count is reported below) ----
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const int k = KPL * lane + j;
        AKnotT<float>& Fj = F[j];
        Fj.m = 0;
        Fj.gm = Fj.drop = Fj.add = 0;
        Fj.w = Fj.be = 0.0f;
        Fj.rr0 = Fj.rr1 = Fj.xr0 = Fj.xr1 = 0.0f;
        Fj.rh0 = Fj.rh1 = Fj.d0 = Fj.d1 = Fj.qx0 = Fj.qx1 = 0.0f;
        Fj.P00 = Fj.P01 = Fj.P11 = Fj.h00 = Fj.h01 = Fj.h11 = 0.0f;
        kin[j] = KnotIn{0, 0.0, 0.0, 0.0, 0.0, 0.0};
        if (k < N) {
            const KnotIn in = knot_in<PH>(p, k, N, omega, xi_ref, vrp_ref, nfacets, ps, sPh);
            if (BLF_AS_KEEPIN) kin[j] = in;
            Fj.m = in.m < 0 ? 0 : in.m > M ? M : in.m;
            Fj.w = float(in.w);
            Fj.be = Pf.dt * Fj.w;
            Fj.rr0 = float(in.rr0);
            Fj.rr1 = float(in.rr1);
            Fj.xr0 = float(in.xr0);
            Fj.xr1 = float(in.xr1);
        }
        Fj.al = 1.0f + Fj.be;
        Fj.r0 = Fj.rr0; Fj.r1 = Fj.rr1;
        Fj.x0 = Fj.xr0; Fj.x1 = Fj.xr1;
    }
    const float xf00 = float(xi00), xf01 = float(xi01);
    if (kOverlap) stage_rows_issue<U>(Ain, bin, p, lane, 0, nA, va, vb);
    AS_STAMP_ADD(1, t_start);
    {
        AS_STAMP(t_q);
        as_lq_step<KPL, TR, float>(F, Pf, N, lane, xf00, xf01);
        if (kOverlap) stage_rows_commit<KPL, U, double>(va, vb, M, S, NH, lane, 0, nA, A2d, Bv);
        __syncthreads();   // the LDS rows (one wavefront: a wait for the stores)
        AS_STAMP_ADD(2, t_q);
        AS_STAMP(t_g);
        const double* const lw0[KPL] = {};
        as_guess<KPL, float>(F, R, NH, N, lane, lw0, 0.0, 0.0f);
        AS_STAMP_ADD(3, t_g);
        AS_STAMP(t_a);
        int pkf[KPL];
        float plf[KPL][2];
        cert32 = as_passes<KPL, TR, float>(F, Pf, R, NH, N, lane, xf00, xf01, pkf, plf, 12, 16, N / kHandoverDiv,
                                           npass32);
        AS_STAMP_ADD(13, t_a);
    }
#pragma unroll
    for (int j = 0; j < KPL; ++j) cand[j] = as_cand(F[j]);

    // ---- phase B: the fp64 passes from the float point ----
    AS_STAMP(t_b);
    const PT<double> Pd = params_d(P);
    AKnot K[KPL];
    bool bad = false;
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
            const KnotIn in = BLF_AS_KEEPIN ? kin[j] : knot_in<PH>(p, k, N, omega, xi_ref, vrp_ref, nfacets, ps, sPh);
            Kj.m = in.m;
            Kj.w = in.w;
            Kj.rr0 = in.rr0;
            Kj.rr1 = in.rr1;
            Kj.xr0 = in.xr0;
            Kj.xr1 = in.xr1;
            if (Kj.m < 0 || Kj.m > M) {
                bad = true;
                Kj.m = 0;
            }
            Kj.be = Pd.dt * Kj.w;
            Kj.r0 = double(F[j].r0);
            Kj.r1 = double(F[j].r1);
            Kj.x0 = double(F[j].x0);
            Kj.x1 = double(F[j].x1);
        }
        Kj.al = 1.0 + Kj.be;
    }
    int status = 0;
    int npass = npass32;   // active-set passes run (float + fp64), blf_dcm_mpc_solution.passes
    bool certified = false;
    double pl[KPL][2];
    int pk[KPL];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        pl[j][0] = pl[j][1] = 0.0;
        pk[j] = 0;
    }
    if (__ballot(bad) != 0) {
        status = BLF_QP_BAD_FACETS;   // outputs (xi_ref, vrp_ref), as the oracle
        npass = 0;                    // (and no passes reported)
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            K[j].r0 = K[j].rr0;
            K[j].r1 = K[j].rr1;
            K[j].x0 = K[j].xr0;
            K[j].x1 = K[j].xr1;
        }
    } else {
        // the fp64 passes' guess: the facets active at a certified float point (slack below
        // kGuessSlack); when the search stopped uncertified, its next candidate sets
        const double* const lw0[KPL] = {};
        as_guess<KPL, double>(K, R, NH, N, lane, lw0, 0.0, kGuessSlack);
        if (!cert32) {
#pragma unroll
            for (int j = 0; j < KPL; ++j) K[j].gm = KPL * lane + j < N ? cand[j] : 0;
        }
        int npass64 = 0;
        certified = as_passes<KPL, TR, double>(K, Pd, R, NH, N, lane, xi00, xi01, pk, pl, 10, 4, -1, npass64);
        npass += npass64;
        if (!certified) {
            // ---- the IPM's start point: the fp64 LQ optimum from (xi_ref, vrp_ref) ----
#pragma unroll
            for (int j = 0; j < KPL; ++j) {
                if (KPL * lane + j < N) {
                    K[j].r0 = K[j].rr0;
                    K[j].r1 = K[j].rr1;
                    K[j].x0 = K[j].xr0;
                    K[j].x1 = K[j].xr1;
                }
            }
            if (!as_lq_step<KPL, TR, double>(K, Pd, N, lane, xi00, xi01)) status = BLF_QP_NUMERICAL;
        }
    }
    AS_STAMP_ADD(14, t_b);
    as_write_outputs<KPL, LAMOUT>(K, pk, pl, certified, status, p, N, M, lane, xi00, xi01, xi_out, vrp_out,
                                  status_out, iters_out, polished_out, lam_out, P.list, P.list_slot, P.list_cap,
                                  P.passes_out, npass, pend);
    if (PH && !certified && status == 0) ph_write_window<KPL>(ps, sPh, omega, A2d, Bv, p, N, M, S, NH, lane);
    AS_STAMP_ADD(0, t_start);
#ifdef BLF_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < 65536) {
        g_as32_timeline[4 * blockIdx.x + 0] = t_rt0;
        g_as32_timeline[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        g_as32_timeline[4 * blockIdx.x + 2] = t_start;
        g_as32_timeline[4 * blockIdx.x + 3] = __builtin_amdgcn_s_memtime();
    }
#endif
}

template <int KPL, bool LAMOUT, bool PH, int TR, int MF>
__global__ __launch_bounds__(kWave, BLF_AS_MINWAVES) void dcm_mpc_cold_kernel(
    KParams P, const double* __restrict__ xi_init, const double* __restrict__ omega,
    const double* __restrict__ xi_ref, const double* __restrict__ vrp_ref,
    const double* __restrict__ Ain, const double* __restrict__ bin,
    const int32_t* __restrict__ nfacets, double* __restrict__ xi_out, double* __restrict__ vrp_out,
    int32_t* __restrict__ status_out, int32_t* __restrict__ iters_out, int32_t* __restrict__ polished_out,
    double* __restrict__ lam_out, PhaseSrc ps)
{
    cold_solve<KPL, LAMOUT, PH, TR, MF>(P, xi_init, omega, xi_ref, vrp_ref, Ain, bin, nfacets, xi_out, vrp_out,
                                         status_out, iters_out, polished_out, lam_out, ps);
}

// Small batches, N <= 64 (configs[0], one TimeVaryingDCMPlanner solve): the QP the active-set
// start hands over continues in the same workgroup, the IPM kernel's stage 2 run by the
// wavefront's 64 lanes (ipm_solve<64>: one thread per knot, exactly the stage-2 workgroup), so the
// solve is one launch instead of two (the second one's dispatch was 4 us of a 28 us solve, and
// the host's second enqueue).  Same code, same inputs, so the same bits as the two launches.
template <bool LAMOUT>
__global__ __launch_bounds__(kWave, BLF_AS_MINWAVES) void dcm_mpc_cold_fused_kernel(
    KParams P, const double* __restrict__ xi_init, const double* __restrict__ omega,
    const double* __restrict__ xi_ref, const double* __restrict__ vrp_ref,
    const double* __restrict__ Ain, const double* __restrict__ bin,
    const int32_t* __restrict__ nfacets, double* __restrict__ xi_out, double* __restrict__ vrp_out,
    int32_t* __restrict__ status_out, int32_t* __restrict__ iters_out, int32_t* __restrict__ polished_out,
    double* __restrict__ lam_out)
{
    cold_solve<1, LAMOUT, false, kTreeDpp>(P, xi_init, omega, xi_ref, vrp_ref, Ain, bin, nfacets, xi_out, vrp_out,
                                        status_out, iters_out, polished_out, lam_out, PhaseSrc{});
    // the outputs just written are stage 2's start point and its status gate; the LDS is reused
    __syncthreads();
    KParams P2 = P;
    P2.stage2 = 1;
    ipm_solve<kWave, false, LAMOUT>(P2, blockIdx.x, xi_init, omega, xi_ref, vrp_ref, Ain, bin, nfacets,
                                    nullptr, nullptr, xi_out, vrp_out, status_out, iters_out, polished_out,
                                    lam_out);
}

#ifndef BLF_WARM_RETRY
#define BLF_WARM_RETRY 1
#endif
// ---- the warm-start kernel ("Warm start") ----
// One wavefront per QP, fp64 facet rows in LDS.  From the shifted previous solution (xi rolled
// out from its VRPs), guess = the facets the rollout violates plus those whose previous multiplier
// exceeds the floor, then the fp64 passes (1.7 per window on average: no float search first).
template <int KPL, bool LAMOUT, bool PH, int TR, int MF>
__global__ __launch_bounds__(kWave, 2) void dcm_mpc_warm_kernel(
    KParams P, const double* __restrict__ xi_init, const double* __restrict__ omega,
    const double* __restrict__ xi_ref, const double* __restrict__ vrp_ref,
    const double* __restrict__ Ain, const double* __restrict__ bin,
    const int32_t* __restrict__ nfacets, const double* __restrict__ ws_vrp,
    const double* __restrict__ ws_lam, double* __restrict__ xi_out, double* __restrict__ vrp_out,
    int32_t* __restrict__ status_out,
    int32_t* __restrict__ iters_out, int32_t* __restrict__ polished_out, double* __restrict__ lam_out,
    PhaseSrc ps)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    // a problem whose previous solve failed (prev_status != 0) is not warm-started from it: it is
    // solved exactly as a cold launch solves it (the IPM's stage 2 treats it as cold too)
    int pend = kPending;
    if (P.ws_status != nullptr && P.ws_status[blockIdx.x] != 0) goto cold;
    {
    const int N = P.N, M = P.M;
    assume_pad<KPL, TR>(N);
    const int NH = (N + KPL - 1) / KPL;   // lanes holding knots
    const int S = KPL * NH;               // LDS row stride: facet i of slot j, lane l at i S + j NH + l
    double2* A2 = reinterpret_cast<double2*>(smem);   // [M][S] facet normals
    double* Bv = smem + 2 * (size_t)M * S;              // [M][S] offsets
    const int lane = threadIdx.x;
    const int64_t p = blockIdx.x;
    const PT<double> Pd = params_d(P);
    AS_STAMP(t_start);
#ifdef BLF_STAMPS
    const unsigned long long t_rt0 = __builtin_amdgcn_s_memrealtime();
#endif

    // ---- the QP's facet slabs into LDS, every start-up load issued before the first wait: the
    //      slab loads (one round, U per lane covers N M <= 128 x 8), then the knots' own loads,
    //      then the LDS stores, which wait for the slab loads only ----
    const int nA = N * M;
    constexpr bool kWide = MF > kMaxFacets;   // 16 slots: the rows staged in rounds, up front
    constexpr int U = KPL == 2 ? 2 * kMaxFacets : kMaxFacets;   // one round: nA <= 1024 / 512
    double* sBE = smem + 3 * (size_t)M * S;                            // PH: [2][P]
    int32_t* sPh = reinterpret_cast<int32_t*>(sBE + 2 * (size_t)ps.P);  // PH: [N+1]
    if (PH) ph_stage_phases(ps, p, N, P.dt, lane, sBE, sPh);
    if constexpr (kWide) {
        if (PH) stage_rows_ph<KPL, U, true>(ps, sPh, p, N, M, S, NH, lane, reinterpret_cast<double*>(A2), Bv);
        else stage_rows_rounds<KPL, U>(Ain, bin, p, N, M, S, NH, lane, reinterpret_cast<double*>(A2), Bv);
    }
    // the rows' loads are issued after the knots' loads (vmcnt counts in issue order) and land in
    // LDS after the warm start's rollout, which does not read them
    double2 va[U];
    double vb[U];

    // ---- the knots this lane owns ----
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
            const KnotIn in = knot_in<PH>(p, k, N, omega, xi_ref, vrp_ref, nfacets, ps, sPh);
            Kj.m = in.m;
            Kj.w = in.w;
            const bool ws = k + P.ws_shift < N;
            Kj.r0 = ws ? ws_vrp[2 * (st + P.ws_shift)] : in.rr0;
            Kj.r1 = ws ? ws_vrp[2 * (st + P.ws_shift) + 1] : in.rr1;
            Kj.rr0 = in.rr0;
            Kj.rr1 = in.rr1;
            Kj.xr0 = in.xr0;
            Kj.xr1 = in.xr1;
        }
    }
    if constexpr (!kWide) {
        if (PH) stage_rows_ph_issue<U>(ps, sPh, p, N, M, lane, va, vb);
        else stage_rows_issue<U>(Ain, bin, p, lane, 0, nA, va, vb);
    }
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        AKnot& Kj = K[j];
        if (KPL * lane + j < N) {
            if (Kj.m < 0 || Kj.m > M) {
                bad = true;
                Kj.m = 0;
            }
            Kj.be = Pd.dt * Kj.w;
        }
        Kj.al = 1.0 + Kj.be;
    }
    const bool any_bad = __ballot(bad) != 0;
    AS_STAMP_ADD(1, t_start);
    const LdsRows<double, MF> R{A2, Bv, S, NH};

    int status = 0;
    int npass = 0;   // active-set passes run (float + fp64), blf_dcm_mpc_solution.passes
    bool certified = false;
    double pl[KPL][2];
    int pk[KPL];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        pl[j][0] = pl[j][1] = 0.0;
        pk[j] = 0;
    }
    // ---- initial point: xi rolled out from the VRPs (forward scan of
    //      xi_{k+1} = alpha_k xi_k - beta_k r_k) ----
    AS_STAMP(t_lq);
    {
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
        as_scan_forward<KPL, TR, double>(g, f, lane, x, xk);
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            K[j].x0 = x[j][0];
            K[j].x1 = x[j][1];
        }
    }
    if constexpr (!kWide) stage_rows_commit<KPL, U, double>(va, vb, M, S, NH, lane, 0, nA, reinterpret_cast<double*>(A2), Bv);
    __syncthreads();   // the LDS slabs (one wavefront: a wait for the stores)
    AS_STAMP_ADD(2, t_lq);
    if (any_bad) {
        status = BLF_QP_BAD_FACETS;
    } else {
        AS_STAMP(t_g);
        const double* lw[KPL];
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            const int k = KPL * lane + j;
            lw[j] = (k < N && k + P.ws_shift < N) ? ws_lam + (p * N + k + P.ws_shift) * M : nullptr;
        }
        as_guess<KPL, double>(K, R, NH, N, lane, lw, P.ws_floor, 0.0);
        AS_STAMP_ADD(3, t_g);
        AS_STAMP(t_b);
        certified = as_passes<KPL, TR, double>(K, Pd, R, NH, N, lane, xi00, xi01, pk, pl, 10, 4, -1, npass);
        AS_STAMP_ADD(14, t_b);
    }
#if BLF_WARM_RETRY
    // the warm passes did not certify: the QP is solved again from a cold start (fp32 search,
    // fp64 passes), and if that hands it over, stage 2 starts it cold (kPendingCold)
    if (!certified && status == 0) {
        pend = kPendingCold;
        __syncthreads();   // the LDS is the cold solve's
        goto cold;
    }
#endif
    AS_STAMP(t_out);

    as_write_outputs<KPL, LAMOUT>(K, pk, pl, certified, status, p, N, M, lane, xi00, xi01, xi_out, vrp_out,
                                  status_out, iters_out, polished_out, lam_out, P.list, P.list_slot, P.list_cap,
                                  P.passes_out, npass);
    if (PH && !certified && status == 0)
        ph_write_window<KPL>(ps, sPh, omega, reinterpret_cast<const double*>(A2), Bv, p, N, M, S, NH, lane);
    AS_STAMP_ADD(11, t_out);
    AS_STAMP_ADD(15, t_start);
#ifdef BLF_STAMPS
    if (threadIdx.x == 0 && blockIdx.x < 65536) {
        g_as_timeline[4 * blockIdx.x + 0] = t_rt0;
        g_as_timeline[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
        g_as_timeline[4 * blockIdx.x + 2] = t_start;
        g_as_timeline[4 * blockIdx.x + 3] = __builtin_amdgcn_s_memtime();
    }
#endif
    return;
    }
cold:
    cold_solve<KPL, LAMOUT, PH, TR, MF>(P, xi_init, omega, xi_ref, vrp_ref, Ain, bin, nfacets, xi_out, vrp_out,
                                         status_out, iters_out, polished_out, lam_out, ps, pend);
}

// Batches up to this size take the fused kernel (N <= 64, cold, per-knot input): they fill at
// most 4 of a CU's wavefront slots, so its larger LDS / register footprint costs nothing.  They
// also take the DPP scan tree (kTreeDpp): at most one wavefront per SIMD, so the dependency chain
// of a wavefront, not the SIMD's VALU issue, sets the time.
constexpr int64_t kFusedMaxBatch = 1024;
constexpr int64_t kDppTreeMaxBatch = BLF_DPP_TREE_MAX_BATCH;

template <int KPL, int MF>
blf_status launch_kpl(const KParams& kp, const blf_dcm_mpc_problem* pb, const blf_dcm_mpc_warm_start* warm,
                      int64_t batch, const blf_dcm_mpc_solution* sol, double* lam_out, hipStream_t s,
                      const PhaseSrc* ps, bool* stage2_done)
{
#ifndef AS_EXTRA_LDS
#define AS_EXTRA_LDS 0
#endif
    const size_t slots = (size_t)kp.M * (KPL * ((kp.N + KPL - 1) / KPL));
    const PhaseSrc none{};
    const PhaseSrc& src = ps ? *ps : none;
    const size_t lds = 3 * sizeof(double) * slots +
                       (ps ? ph_lds_bytes(ps->P, kp.N) : 0) + AS_EXTRA_LDS;
    if (lds > 64 * 1024)
        return set_error(BLF_ERR_UNSUPPORTED, "active-set kernel: %zu B of LDS (%d phases)", lds, ps ? ps->P : 0);
    // the scan tree: DPP for small batches with one knot per lane (the oracle's as_tree follows the
    // same rule); knot pairs always take the ds_bpermute tree
    constexpr int kAltTree = KPL == 2 ? kTreePad : kTreeDpp;   // the instantiated trees: this, kTreeKS
    const int tr = (KPL == 1 && batch <= kDppTreeMaxBatch) ? kTreeDpp
                   : (KPL == 2 && kp.N <= 2 * kWave - 2) ? kTreePad : kTreeKS;
    if (KPL == 1 && MF == kMaxFacets && warm == nullptr && ps == nullptr && batch <= kFusedMaxBatch &&
        qp_launch_mode().fuse_stage2.load(std::memory_order_relaxed)) {
        const size_t lds_f = std::max(lds, sizeof(double) * Lds(nullptr, kp.N, kp.M, 1).total);
        auto kern = lam_out ? dcm_mpc_cold_fused_kernel<true> : dcm_mpc_cold_fused_kernel<false>;
        KParams kf = kp;
        kf.list = nullptr;   // its own stage 2 follows in the workgroup: nothing to list
        hipLaunchKernelGGL(kern, dim3((unsigned)batch), dim3(kWave), lds_f, s, kf,
                           pb->xi_init, pb->omega, pb->xi_ref, pb->vrp_ref, pb->A, pb->b, pb->nfacets, sol->xi,
                           sol->vrp, sol->status, sol->iters, sol->polished, lam_out);
        *stage2_done = true;
        return check_hip(hipGetLastError(), "dcm_mpc_cold_fused_kernel launch");
    }
    if (warm == nullptr) {
#define AS_COLD(L, H, D) dcm_mpc_cold_kernel<KPL, L, H, D, MF>
#define AS_COLD_TR(D) (ps ? (lam_out ? AS_COLD(true, true, D) : AS_COLD(false, true, D)) \
                          : (lam_out ? AS_COLD(true, false, D) : AS_COLD(false, false, D)))
        auto kern = tr == kAltTree ? AS_COLD_TR(kAltTree) : AS_COLD_TR(kTreeKS);
#undef AS_COLD_TR
#undef AS_COLD
        hipLaunchKernelGGL(kern, dim3((unsigned)batch), dim3(kWave), lds, s, kp,
                           pb->xi_init, pb->omega, pb->xi_ref, pb->vrp_ref, pb->A, pb->b, pb->nfacets, sol->xi,
                           sol->vrp, sol->status, sol->iters, sol->polished, lam_out, src);
        return check_hip(hipGetLastError(), "dcm_mpc_cold_kernel launch");
    }
#define AS_WARM(L, H, D) dcm_mpc_warm_kernel<KPL, L, H, D, MF>
#define AS_WARM_TR(D) (ps ? (lam_out ? AS_WARM(true, true, D) : AS_WARM(false, true, D)) \
                          : (lam_out ? AS_WARM(true, false, D) : AS_WARM(false, false, D)))
    auto kern = tr == kAltTree ? AS_WARM_TR(kAltTree) : AS_WARM_TR(kTreeKS);
#undef AS_WARM_TR
#undef AS_WARM
    hipLaunchKernelGGL(kern, dim3((unsigned)batch), dim3(kWave), lds, s, kp,
                       pb->xi_init, pb->omega, pb->xi_ref, pb->vrp_ref, pb->A, pb->b, pb->nfacets, warm->vrp,
                       warm->lambda, sol->xi, sol->vrp, sol->status, sol->iters, sol->polished, lam_out, src);
    return check_hip(hipGetLastError(), "dcm_mpc_warm_kernel launch");
}

}  // namespace

#ifdef BLF_STAMPS
extern "C" int blf_debug_as_timeline(unsigned long long* out, int n)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_as_timeline), sizeof(unsigned long long) * 4 * (size_t)n) == hipSuccess ? 0 : -1;
}

extern "C" int blf_debug_as32_timeline(unsigned long long* out, int n)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_as32_timeline), sizeof(unsigned long long) * 4 * (size_t)n) == hipSuccess ? 0 : -1;
}

extern "C" int blf_debug_as_stamps(unsigned long long* out, int reset)
{
    unsigned long long h[32];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_as_stamps), sizeof(h)) != hipSuccess) return -1;
    for (int i = 0; i < 32; ++i) out[i] = h[i];
    if (reset) {
        unsigned long long z[32] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_as_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

// Active-set kernel of a launch_dcm_mpc call (N <= 128, tol_polish > 0): every QP either solved
// (status 0, polished) or marked kPending for the IPM kernel's stage 2.
blf_status launch_dcm_mpc_as(const qp::KParams& kp, const blf_dcm_mpc_problem* pb,
                             const blf_dcm_mpc_warm_start* warm, int64_t batch,
                             const blf_dcm_mpc_solution* sol, double* lam_out, hipStream_t s,
                             const qp::PhaseSrc* ps, bool* stage2_done)
{
    bool none = false;
    bool* done = stage2_done ? stage2_done : &none;
    *done = false;
    // facet slots: 8, or 16 for phases of three or four contacts (twice the LDS per QP)
    if (kp.M <= kMaxFacets) {
        if (kp.N <= kWave) return launch_kpl<1, kMaxFacets>(kp, pb, warm, batch, sol, lam_out, s, ps, done);
        if (kp.N <= 2 * kWave) return launch_kpl<2, kMaxFacets>(kp, pb, warm, batch, sol, lam_out, s, ps, done);
    } else if (kp.M <= kMaxFacetsWide) {
        if (kp.N <= kWave) return launch_kpl<1, kMaxFacetsWide>(kp, pb, warm, batch, sol, lam_out, s, ps, done);
        if (kp.N <= 2 * kWave) return launch_kpl<2, kMaxFacetsWide>(kp, pb, warm, batch, sol, lam_out, s, ps, done);
    } else {
        return set_error(BLF_ERR_UNSUPPORTED, "active-set kernel: %d facet slots > %d", kp.M, kMaxFacetsWide);
    }
    return set_error(BLF_ERR_UNSUPPORTED, "active-set kernel: horizon %d > 128", kp.N);
}

}  // namespace blf
