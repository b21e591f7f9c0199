// dcm_qp_common.h — device pieces shared by the DCM-MPC QP kernels (dcm_mpc_ipm.hip: the
// general interior point kernel; dcm_mpc_as.hip: the one-wavefront active-set kernel).  Both
// mirror oracle/blf_oracle.c term for term (same fused forms, same scan combine order), so their
// results agree with the oracle and with each other bit for bit.
#pragma once
#include "blf_internal.h"

namespace blf {
namespace qp {

constexpr int kGuessPasses = 8;   // active-set start: drop/add passes (oracle: ORC_GUESS_PASSES)
constexpr int kAsPasses = 12;     // the active-set kernels' fp64 passes, anti-cycling (oracle: ORC_AS_PASSES)


constexpr int kPending = -1;      // status of a QP the active-set kernel hands to the IPM kernel
constexpr int kPendingCold = -2;  // handed over by the warm kernel after its cold re-solve: stage 2 starts cold

struct KParams {
    int N, M, max_iter;
    int ws_shift;        // warm start: knot k starts from knot k + ws_shift (ws_vrp != nullptr)
    const int32_t* ws_status;   // warm start: [B] status of the previous solve, or nullptr; a
                                // problem with ws_status != 0 starts cold (no warm start)
    double dt, Qw0, Qw1, Rw0, Rw1, Pw0, Pw1, tol_mu, tol_p, tol_d;
    double tol_polish;   // > 0: try the active-set polish once mu <= tol_polish
    double ws_floor;     // warm start: s, lambda >= ws_floor
    int stage2;          // IPM kernel after the active-set kernel: only QPs with status kPending,
                         // and no active-set start (it already failed for them)
    int32_t* list;       // the pending list of stage 2 (or nullptr): [list_slot] = count, [2..] =
                         // the problems the active-set kernel handed over.  The active-set
                         // kernels append to it; stage 2's small grid loops over it.
    int list_slot;       // 0 or 1
    int list_cap;        // entries the list holds (appends beyond it are dropped; stage 2 reads at most this many)
    int32_t* passes_out; // [B] or nullptr: the active-set kernels' passes per QP (float + fp64);
                         // the IPM kernel writes 0 for the problems it solves alone
    // The active-set kernel's fp32 search (cold starts): the parameters rounded to float, and the
    // search's own certificate tolerances (kSearchTolP / kSearchTolD)
    float f_dt, f_Qw0, f_Qw1, f_Rw0, f_Rw1, f_Pw0, f_Pw1, f_tol_p, f_tol_d;
};

// Tolerances of the fp32 active-set search (oracle ORC_SEARCH_TOL_P / _D): the search only
// proposes the active set that the fp64 passes then certify at tol_primal / tol_dual.
constexpr float kSearchTolP = 1e-5f;
constexpr float kSearchTolD = 1e-4f;
// The fp64 passes' guess after the search: the facets whose slack at the float point is below
// this (oracle ORC_GUESS_SLACK).
constexpr double kGuessSlack = 1e-5;
// The fp32 search hands over to the fp64 passes after a failed pass that changed the candidate
// sets of at most N / kHandoverDiv knots (oracle ORC_HANDOVER_DIV).
#ifndef BLF_HANDOVER_DIV   // (A/B builds; the oracle's ORC_HANDOVER_DIV must match)
#define BLF_HANDOVER_DIV 16
#endif
constexpr int kHandoverDiv = BLF_HANDOVER_DIV;
// The fp64 certificate's dual tolerance grows with the knot's costate force once
// |beta nu| > 1 / kTolDualRel: tol_d max(1, kTolDualRel max |beta nu|) (oracle ORC_TOL_DUAL_REL).
// A planned walk keeps |beta nu| below ~2, so only the QPs of uncapturable DCM states (|beta nu|
// and the multipliers up to ~1e8, tests/golden/c5_hard_windows.npz) see a larger tolerance.
constexpr double kTolDualRel = 1e-3;
// The IPM polish's guess from an iterate: lam_i > s_i and lam_i >= kLamRel x the knot's largest
// multiplier (oracle ORC_LAM_REL); it adds only the facets violated by >= kAddRel x the pass's
// largest violation (oracle ORC_ADD_REL).
constexpr double kLamRel = 1e-8;
constexpr double kAddRel = 1e-2;
// Round 6 (oracle ORC_LAM_REL_CROSS, ORC_STALL_STEP / ORC_STALL_MU, ORC_REFINE_LAM; DESIGN.md 4,
// item 11): the kLamRel rule only drops a facet within |a_i x a_max| < kLamRelCross of parallel to
// the knot's largest multiplier's facet; the IPM polish also runs after a step shorter than
// kStallStep once mu <= kStallMu; a certified optimum whose largest multiplier exceeds kRefineLam
// takes one refinement step with double-double residuals (refine_rhs below).
constexpr double kLamRelCross = 0.3;
constexpr double kStallStep = 0.2;
constexpr double kStallMu = 1.0;
constexpr double kRefineLam = 1e4;
constexpr int kRefineSteps = 2;   // oracle ORC_REFINE_STEPS

// ---- double-double arithmetic of the refinement (exact TwoSum / TwoProd by fma; the oracle's
//      dd_* restate these operation for operation) ----
struct DD {
    double hi, lo;
};
__device__ __forceinline__ DD dd_two_sum(double a, double b)
{
    const double s = a + b;
    const double bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
__device__ __forceinline__ DD dd_fast(double a, double b)
{
    const double s = a + b;
    return {s, b - (s - a)};
}
__device__ __forceinline__ DD dd_prod(double a, double b)
{
    const double p = a * b;
    return {p, fma(a, b, -p)};
}
__device__ __forceinline__ DD dd_add(DD x, DD y)
{
    const DD s = dd_two_sum(x.hi, y.hi);
    return dd_fast(s.hi, s.lo + (x.lo + y.lo));
}
__device__ __forceinline__ DD dd_add_d(DD x, double y)
{
    const DD s = dd_two_sum(x.hi, y);
    return dd_fast(s.hi, s.lo + x.lo);
}
__device__ __forceinline__ DD dd_mul_d(DD x, double y)
{
    const DD p = dd_prod(x.hi, y);
    return dd_fast(p.hi, fma(x.lo, y, p.lo));
}
__device__ __forceinline__ DD dd_neg(DD x)
{
    return {-x.hi, -x.lo};
}

// The refinement's right-hand side of one knot k (oracle refine_rhs): with the certified costates
// nu_k (of xi_{k+1}) and nu_{k+1},
//   d_k  = xi_k + dt (om_k xi_k - om_k r_k) - xi_{k+1},
//   qx_k = W (xi_{k+1} - xi_ref_{k+1}) - nu_k + (1 + dt om_{k+1}) nu_{k+1}   (no last term at N - 1),
//   g_k  = R (r_k - r_ref_k) - dt om_k nu_k, onto the active line's tangent (c = 1), 0 at a vertex,
// each in double-double, rounded once.  The stationarity residuals of the certified point are
// small, so the Newton step they drive (the same factorization) is small and accurate: it brings
// the multiplier-1e6..1e9 windows from ~1e-14 x lambda_max to ~1e-11 m (tests/test_c5_windows.py).
// One component j of d_k and qx_k.
__device__ __forceinline__ void refine_comp(double xk, double xn, double r, double xr, double om, double omn,
                                            double nu, double nun, bool last, double dt, double Wq, double& d,
                                            double& q)
{
    DD e = dd_add(dd_prod(om, xk), dd_neg(dd_prod(om, r)));
    e = dd_mul_d(e, dt);
    e = dd_add_d(e, xk);
    e = dd_add_d(e, -xn);
    d = e.hi;
    DD s = dd_mul_d(dd_two_sum(xn, -xr), Wq);
    s = dd_add_d(s, -nu);
    if (!last) {
        s = dd_add(s, dd_mul_d(dd_prod(dt, omn), nun));
        s = dd_add_d(s, nun);
    }
    q = s.hi;
}

__device__ __forceinline__ void refine_rhs(double xk0, double xk1, double xn0, double xn1, double r0, double r1,
                                           double rr0, double rr1, double xr0, double xr1, double om, double omn,
                                           double nu0, double nu1, double nun0, double nun1, bool last, double dt,
                                           double Wq0, double Wq1, double Rw0, double Rw1, int c, double ax,
                                           double ay, double& d0, double& d1, double& q0, double& q1, double& g0,
                                           double& g1)
{
    refine_comp(xk0, xn0, r0, xr0, om, omn, nu0, nun0, last, dt, Wq0, d0, q0);
    refine_comp(xk1, xn1, r1, xr1, om, omn, nu1, nun1, last, dt, Wq1, d1, q1);
    const DD bk = dd_prod(dt, om);
    const DD e0 = dd_add(dd_mul_d(dd_two_sum(r0, -rr0), Rw0), dd_neg(dd_mul_d(bk, nu0)));
    const DD e1 = dd_add(dd_mul_d(dd_two_sum(r1, -rr1), Rw1), dd_neg(dd_mul_d(bk, nu1)));
    if (c == 0) {
        g0 = e0.hi;
        g1 = e1.hi;
    } else if (c == 1) {   // t = (-a_y, a_x): g <- t (t . g) / |a|^2
        const DD tg = dd_add(dd_mul_d(e0, -ay), dd_mul_d(e1, ax));
        const double tau = tg.hi / fma(ax, ax, ay * ay);   // FD2(ax, ax, ay, ay)
        g0 = -(ay * tau);
        g1 = ax * tau;
    } else {
        g0 = 0.0;
        g1 = 0.0;
    }
}

// v_readlane of a double (lane l uniform)
__device__ __forceinline__ double readlane_f64(double v, int l)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)b, l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// The facet rows never change during a solve, so the compiler would hoist every phase's row loads
// out of the IPM loop and keep 8 facets x 4 doubles live in VGPRs across it (spilling).  Each phase
// indexes the rows through an opaque copy of the knot index instead, so they are re-read from LDS.
__device__ __forceinline__ int opaque(int k)
{
    asm volatile("" : "+v"(k));
    return k;
}

// The facet-count predicates (i < m_k per lane, i < mmax per QP) never change during a solve, so
// the compiler would hoist all 8 of each out of the IPM loop as 64-bit lane masks and spill them
// to VGPR lanes (46 SGPRs; every use then costs two v_readlane).  Each facet loop reads the counts
// through these opaque copies instead, so the masks are recomputed per phase (one v_cmp each).
__device__ __forceinline__ int opaque_s(int k)
{
    asm volatile("" : "+s"(k));
    return k;
}

// Lane shuffles for the scans.  The source-lane address is recomputed from an opaque lane id
// at every call: hoisted out of the IPM loop, the twelve shift addresses would stay live in
// VGPRs for the whole kernel.  Out-of-range sources wrap; the scans never use those values.
__device__ __forceinline__ double bperm(int addr, double x)
{
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_ds_bpermute(addr, (int)b);
    const int hi = __builtin_amdgcn_ds_bpermute(addr, (int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ float bperm(int addr, float x)
{
    return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(x)));
}

// One-lane shifts across the wavefront through DPP (a VALU move, no LDS round trip), for the
// scans' distance-1 level and their final hand-over to the neighbour lane.  They return exactly
// what bperm returns at the addresses they replace:
//   kNextKeep (wave_shl:1): lane l takes lane l + 1's value, lane 63 keeps its own (min(l + 1, 63));
//   kNextWrap (wave_rol:1): lane l takes lane (l + 1) mod 64's;
//   kPrevWrap (wave_ror:1): lane l takes lane (l - 1) mod 64's.
// update_dpp's "old" operand is the lane's own value and bound_ctrl is off, so the lane with no
// source (wave_shl's lane 63) keeps it.
enum : int { kNextKeep = 0x130, kNextWrap = 0x134, kPrevWrap = 0x13C };

template <int CTRL>
__device__ __forceinline__ int dpp1(int x)
{
    return __builtin_amdgcn_update_dpp(x, x, CTRL, 0xF, 0xF, false);
}

template <int CTRL>
__device__ __forceinline__ double dpp1(double x)
{
    const long long b = __double_as_longlong(x);
    const int lo = dpp1<CTRL>((int)b);
    const int hi = dpp1<CTRL>((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

template <int CTRL>
__device__ __forceinline__ float dpp1(float x)
{
    return __int_as_float(dpp1<CTRL>(__float_as_int(x)));
}

// ---- the DPP scan tree of the active-set kernels (small batches): every level a VALU move ----
// Kogge-Stone inside each row of 16 lanes by DPP row shifts (4 levels), then two row-level steps
// (oracle orc_lane_src):
//   forward (a lane combines with lower lanes): row_shr:1,2,4,8, then rows 1 and 3 take lane 15 of
//     the row before (row_bcast:15), then rows 2 and 3 take lane 31 (row_bcast:31);
//   backward (a lane combines with higher lanes): row_shl:1,2,4,8, then rows 0 and 2 take the first
//     lane of the row after (row_newbcast:0, then v_permlane16_swap moves rows 1 / 3 onto rows
//     0 / 2), then rows 0 and 1 take lane 32 (v_readlane).
// tree_fwd / tree_bwd return the level's source value (undefined on a lane without a source);
// tree_has says whether the lane has one — only those lanes combine (the others keep their
// element), and the oracle combines at exactly the same lanes.
enum : int { kRowShr = 0x110, kRowShl = 0x100, kRowBcast15 = 0x142, kRowBcast31 = 0x143, kRowNewBcast0 = 0x150 };

template <int CTRL, int RM>
__device__ __forceinline__ int dpp_mov(int x)
{
    return __builtin_amdgcn_mov_dpp(x, CTRL, RM, 0xF, true);
}

// rows 0 and 2 <- the first lane of rows 1 and 3
__device__ __forceinline__ int next_row_first(int x)
{
    const int t = dpp_mov<kRowNewBcast0, 0xF>(x);
    return (int)__builtin_amdgcn_permlane16_swap((unsigned)t, (unsigned)t, false, false)[1];
}

template <int L, bool FWD>
__device__ __forceinline__ int tree_src(int x)
{
    if constexpr (FWD) {
        if constexpr (L < 4) return dpp_mov<kRowShr + (1 << L), 0xF>(x);
        else if constexpr (L == 4) return dpp_mov<kRowBcast15, 0xA>(x);
        else return dpp_mov<kRowBcast31, 0xC>(x);
    } else {
        if constexpr (L < 4) return dpp_mov<kRowShl + (1 << L), 0xF>(x);
        else if constexpr (L == 4) return next_row_first(x);
        else return __builtin_amdgcn_readlane(x, 32);
    }
}

template <int L, bool FWD>
__device__ __forceinline__ float tree_src(float x)
{
    return __int_as_float(tree_src<L, FWD>(__float_as_int(x)));
}

template <int L, bool FWD>
__device__ __forceinline__ double tree_src(double x)
{
    const long long b = __double_as_longlong(x);
    const int lo = tree_src<L, FWD>((int)b);
    const int hi = tree_src<L, FWD>((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

template <int L, class T>
__device__ __forceinline__ T tree_fwd(T x)
{
    return tree_src<L, true>(x);
}

template <int L, class T>
__device__ __forceinline__ T tree_bwd(T x)
{
    return tree_src<L, false>(x);
}

template <int L, bool FWD>
__device__ __forceinline__ bool tree_has(int lane)
{
    const int r = lane >> 4;
    if constexpr (FWD) {
        if constexpr (L < 4) return (lane & 15) >= (1 << L);
        else if constexpr (L == 4) return (r & 1) != 0;
        else return r >= 2;
    } else {
        if constexpr (L < 4) return (lane & 15) + (1 << L) <= 15;
        else if constexpr (L == 4) return (r & 1) == 0;
        else return r < 2;
    }
}

// Fused forms used throughout (and in the same places by oracle/blf_oracle.c):
//   FD2(a, b, c, d)    = a b + c d      as fma(a, b, c d)
//   FD3(a, b, c, d, e) = a b + c d + e  as fma(a, b, fma(c, d, e))
// fma is correctly rounded on both sides, so kernel and oracle stay bit-identical; it saves one
// VALU op per product pair (the kernel is VALU-issue bound).
#define FD2(a, b, c, d) fma((a), (b), (c) * (d))
#define FD3(a, b, c, d, e) fma((a), (b), fma((c), (d), (e)))

// More than two candidate lines in a polish pass (the drop/add moves can add two facets at once):
// the first pair (i < j in facet order) whose vertex satisfies every facet of the knot — a vertex
// of the support polygon — is the active pair (oracle dcm_polish).  Returns 2 with pi1, pi2 set,
// or 3 (no such pair: the pass fails).  Rare, so it reads the rows straight from LDS.
// The offsets are read as Bo[(i N + kx) * bs] (bs = 2: the IPM kernel's (b, 1/s) pairs).
static __device__ __forceinline__ int vertex_pair(const double2* A2, const double* Bo, int bs, int N,
                                                            int kx, int km, int cm, double tol_p, int& pi1,
                                                            int& pi2)
{
    for (int x = 0; x < km; ++x) {
        if (!((cm >> x) & 1)) continue;
        for (int y = x + 1; y < km; ++y) {
            if (!((cm >> y) & 1)) continue;
            const double2 a = A2[x * N + kx];
            const double2 e = A2[y * N + kx];
            const double ba = Bo[(x * N + kx) * bs], be = Bo[(y * N + kx) * bs];
            const double det = fma(a.x, e.y, -(a.y * e.x));
            const double aa = FD2(a.x, a.x, a.y, a.y), ee = FD2(e.x, e.x, e.y, e.y);
            if (!(det * det > 1e-18 * (aa * ee))) continue;
            const double idet = 1.0 / det;
            const double v0 = fma(ba, e.y, -(a.y * be)) * idet;
            const double v1 = fma(a.x, be, -(ba * e.x)) * idet;
            bool feas = true;
            for (int l = 0; l < km; ++l) {
                const double2 f = A2[l * N + kx];
                if (!(FD2(f.x, v0, f.y, v1) - Bo[(l * N + kx) * bs] <= tol_p)) feas = false;
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

// 2x2 compose (row-major): n = a * b;  nc = a * c + e.
#define COMPOSE(a0, a1, a2, a3, b0, b1, b2, b3, c0, c1, e0, e1)                 \
    do {                                                                         \
        const double n0_ = FD2(a0, b0, a1, b2);                                  \
        const double n1_ = FD2(a0, b1, a1, b3);                                  \
        const double n2_ = FD2(a2, b0, a3, b2);                                  \
        const double n3_ = FD2(a2, b1, a3, b3);                                  \
        const double m0_ = FD3(a0, c0, a1, c1, e0);                              \
        const double m1_ = FD3(a2, c0, a3, c1, e1);                              \
        a0 = n0_; a1 = n1_; a2 = n2_; a3 = n3_; e0 = m0_; e1 = m1_;               \
    } while (0)

// Riccati map element f(P) = H + A^T P (I + G P)^{-1} A (oracle rc_el); knot k: A = alpha_k I,
// G = E_k, H = Q.  rc_combine(e, q): e <- e o q (q the later knots), the structure-preserving
// doubling composition — it inverts only I + G H (eigenvalues >= 1).
// Templated on the scalar type: double everywhere, float in the active-set kernel's fp32 search
// (the same operations in the same order, so oracle/blf_oracle_as32.c restates them bit for bit).
template <class T>
struct RcT {
    T a0, a1, a2, a3, g0, g1, g2, h0, h1, h2;
};
using Rc = RcT<double>;

// BLF_RC_FORM selects where the reciprocal of det(I + G H) enters (the oracle's ORC_RC_FORM must
// match):  0: T^{-1} = adj(T) / det first (the reciprocal heads the chain of products);
// 1: rc_apply deferred only; 2: rc_apply deferred, rc_combine scales U = adj(T) A_e and the G
// block at the end; 3: both scale their outputs at the end, so the products of adj(T) run
// beside the division (the division no longer heads the dependent chain).
#ifndef BLF_RC_FORM
#define BLF_RC_FORM 2
#endif

template <class T>
__device__ __forceinline__ bool rc_combine(RcT<T>& e, const RcT<T>& q)
{
    const T one = T(1);
    const T T00 = FD3(e.g0, q.h0, e.g1, q.h1, one);
    const T T01 = FD2(e.g0, q.h1, e.g1, q.h2);
    const T T10 = FD2(e.g1, q.h0, e.g2, q.h1);
    const T T11 = FD3(e.g1, q.h1, e.g2, q.h2, one);
    const T detT = fma(T00, T11, -(T01 * T10));
    const bool ok = (detT > T(0)) && !__builtin_isinf(detT);
    const T it = one / detT;
    if constexpr (BLF_RC_FORM >= 2) {
        // adj(T) = [T11, -T01; -T10, T00]; U' = adj(T) A_e, V' = A_q adj(T), X' = V' G_e
        const T Up00 = FD2(T11, e.a0, -T01, e.a2);
        const T Up01 = FD2(T11, e.a1, -T01, e.a3);
        const T Up10 = FD2(-T10, e.a0, T00, e.a2);
        const T Up11 = FD2(-T10, e.a1, T00, e.a3);
        const T Vp00 = FD2(q.a0, T11, q.a1, -T10);
        const T Vp01 = FD2(q.a0, -T01, q.a1, T00);
        const T Vp10 = FD2(q.a2, T11, q.a3, -T10);
        const T Vp11 = FD2(q.a2, -T01, q.a3, T00);
        const T Xp00 = FD2(Vp00, e.g0, Vp01, e.g1);
        const T Xp01 = FD2(Vp00, e.g1, Vp01, e.g2);
        const T Xp10 = FD2(Vp10, e.g0, Vp11, e.g1);
        const T Xp11 = FD2(Vp10, e.g1, Vp11, e.g2);
        const T Y00 = FD2(q.h0, e.a0, q.h1, e.a2);
        const T Y01 = FD2(q.h0, e.a1, q.h1, e.a3);
        const T Y10 = FD2(q.h1, e.a0, q.h2, e.a2);
        const T Y11 = FD2(q.h1, e.a1, q.h2, e.a3);
        const T gp0 = FD2(Xp00, q.a0, Xp01, q.a1);
        const T gp1 = FD2(Xp00, q.a2, Xp01, q.a3);
        const T gp2 = FD2(Xp10, q.a2, Xp11, q.a3);
        RcT<T> r;
        if constexpr (BLF_RC_FORM == 2) {
            const T U00 = Up00 * it, U01 = Up01 * it, U10 = Up10 * it, U11 = Up11 * it;
            r.a0 = FD2(q.a0, U00, q.a1, U10);
            r.a1 = FD2(q.a0, U01, q.a1, U11);
            r.a2 = FD2(q.a2, U00, q.a3, U10);
            r.a3 = FD2(q.a2, U01, q.a3, U11);
            r.h0 = FD3(U00, Y00, U10, Y10, e.h0);
            r.h1 = FD3(U00, Y01, U10, Y11, e.h1);
            r.h2 = FD3(U01, Y01, U11, Y11, e.h2);
        } else {
            r.a0 = FD2(q.a0, Up00, q.a1, Up10) * it;
            r.a1 = FD2(q.a0, Up01, q.a1, Up11) * it;
            r.a2 = FD2(q.a2, Up00, q.a3, Up10) * it;
            r.a3 = FD2(q.a2, Up01, q.a3, Up11) * it;
            r.h0 = fma(FD2(Up00, Y00, Up10, Y10), it, e.h0);
            r.h1 = fma(FD2(Up00, Y01, Up10, Y11), it, e.h1);
            r.h2 = fma(FD2(Up01, Y01, Up11, Y11), it, e.h2);
        }
        r.g0 = fma(gp0, it, q.g0);
        r.g1 = fma(gp1, it, q.g1);
        r.g2 = fma(gp2, it, q.g2);
        e = r;
        return ok;
    }
    const T Ti00 = T11 * it, Ti01 = -(T01 * it), Ti10 = -(T10 * it), Ti11 = T00 * it;
    const T U00 = FD2(Ti00, e.a0, Ti01, e.a2);
    const T U01 = FD2(Ti00, e.a1, Ti01, e.a3);
    const T U10 = FD2(Ti10, e.a0, Ti11, e.a2);
    const T U11 = FD2(Ti10, e.a1, Ti11, e.a3);
    const T V00 = FD2(q.a0, Ti00, q.a1, Ti10);
    const T V01 = FD2(q.a0, Ti01, q.a1, Ti11);
    const T V10 = FD2(q.a2, Ti00, q.a3, Ti10);
    const T V11 = FD2(q.a2, Ti01, q.a3, Ti11);
    const T X00 = FD2(V00, e.g0, V01, e.g1);
    const T X01 = FD2(V00, e.g1, V01, e.g2);
    const T X10 = FD2(V10, e.g0, V11, e.g1);
    const T X11 = FD2(V10, e.g1, V11, e.g2);
    const T Y00 = FD2(q.h0, e.a0, q.h1, e.a2);
    const T Y01 = FD2(q.h0, e.a1, q.h1, e.a3);
    const T Y10 = FD2(q.h1, e.a0, q.h2, e.a2);
    const T Y11 = FD2(q.h1, e.a1, q.h2, e.a3);
    RcT<T> r;
    r.a0 = FD2(q.a0, U00, q.a1, U10);
    r.a1 = FD2(q.a0, U01, q.a1, U11);
    r.a2 = FD2(q.a2, U00, q.a3, U10);
    r.a3 = FD2(q.a2, U01, q.a3, U11);
    r.g0 = FD3(X00, q.a0, X01, q.a1, q.g0);
    r.g1 = FD3(X00, q.a2, X01, q.a3, q.g1);
    r.g2 = FD3(X10, q.a2, X11, q.a3, q.g2);
    r.h0 = FD3(U00, Y00, U10, Y10, e.h0);
    r.h1 = FD3(U00, Y01, U10, Y11, e.h1);
    r.h2 = FD3(U01, Y01, U11, Y11, e.h2);
    e = r;
    return ok;
}

template <class T>
__device__ __forceinline__ bool rc_apply(const RcT<T>& e, T P00, T P01, T P11, T& o00, T& o01, T& o11)
{
    const T one = T(1);
    const T S00 = FD3(e.g0, P00, e.g1, P01, one);
    const T S01 = FD2(e.g0, P01, e.g1, P11);
    const T S10 = FD2(e.g1, P00, e.g2, P01);
    const T S11 = FD3(e.g1, P01, e.g2, P11, one);
    const T detS = fma(S00, S11, -(S01 * S10));
    const bool ok = (detS > T(0)) && !__builtin_isinf(detS);
    const T is = one / detS;
    if constexpr (BLF_RC_FORM >= 1) {
        // W' = P adj(S), Z' = W' A, out = (A^T Z') / det(S) + H
        const T Wp00 = FD2(P00, S11, P01, -S10);
        const T Wp01 = FD2(P00, -S01, P01, S00);
        const T Wp10 = FD2(P01, S11, P11, -S10);
        const T Wp11 = FD2(P01, -S01, P11, S00);
        const T Zp00 = FD2(Wp00, e.a0, Wp01, e.a2);
        const T Zp01 = FD2(Wp00, e.a1, Wp01, e.a3);
        const T Zp10 = FD2(Wp10, e.a0, Wp11, e.a2);
        const T Zp11 = FD2(Wp10, e.a1, Wp11, e.a3);
        o00 = fma(FD2(e.a0, Zp00, e.a2, Zp10), is, e.h0);
        o01 = fma(FD2(e.a0, Zp01, e.a2, Zp11), is, e.h1);
        o11 = fma(FD2(e.a1, Zp01, e.a3, Zp11), is, e.h2);
        return ok;
    }
    const T Si00 = S11 * is, Si01 = -(S01 * is), Si10 = -(S10 * is), Si11 = S00 * is;
    const T W00 = FD2(P00, Si00, P01, Si10);
    const T W01 = FD2(P00, Si01, P01, Si11);
    const T W10 = FD2(P01, Si00, P11, Si10);
    const T W11 = FD2(P01, Si01, P11, Si11);
    const T Z00 = FD2(W00, e.a0, W01, e.a2);
    const T Z01 = FD2(W00, e.a1, W01, e.a3);
    const T Z10 = FD2(W10, e.a0, W11, e.a2);
    const T Z11 = FD2(W10, e.a1, W11, e.a3);
    o00 = FD3(e.a0, Z00, e.a2, Z10, e.h0);
    o01 = FD3(e.a0, Z01, e.a2, Z11, e.h1);
    o11 = FD3(e.a1, Z01, e.a3, Z11, e.h2);
    return ok;
}

// The phase-indexed input of blf_dcm_mpc_solve_phased: the plan's phase table (blf_phase_table)
// in place of the window's per-knot arrays, and the window scratch a QP handed to the IPM kernel
// is expanded into (blf_dcm_mpc_window).
struct PhaseSrc {
    int32_t P;                         // phases per problem (table stride)
    const int32_t* nphases;            // [B]
    const double *begin, *end;         // [B][P]
    const double *A, *b;               // [B][P][M][2], [B][P][M]
    const int32_t* nf;                 // [B][P]
    const double* ref;                 // [B][P][2]
    int64_t start;                     // window start knot: t_k = (start + k) dt
    int64_t ostride;                   // omega row stride of the window
    double *wom, *wxr, *wrr, *wA, *wb; // window scratch (stage 2)
    int32_t* wnf;
};

}  // namespace qp

// The knot -> phase rule of blf_dcm_phase_expand (phase_expand.hip and the fused phase-indexed
// solve share it, so both expand a window identically): p = the last phase with begin_p <= t, by
// this binary search over the phases in table order; the knot is in p iff t < end_p, else -1.
__device__ __forceinline__ int phase_of(const double* begin, const double* end, int n, double t)
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

// dcm_mpc_as.hip: the one-wavefront active-set kernel (N <= 128); QPs it does not certify are left
// with status qp::kPending for the IPM kernel's stage 2.  ps != nullptr: the phase-indexed input
// (pb->xi_init and pb->omega are used, the other per-knot arrays are not).  *stage2_done: the
// launch already ran stage 2 (the fused small-batch kernel), so the IPM launch is skipped.
blf_status launch_dcm_mpc_as(const qp::KParams& kp, const blf_dcm_mpc_problem* pb,
                             const blf_dcm_mpc_warm_start* warm, int64_t batch,
                             const blf_dcm_mpc_solution* sol, double* lam_out, hipStream_t s,
                             const qp::PhaseSrc* ps = nullptr, bool* stage2_done = nullptr);
}  // namespace blf
