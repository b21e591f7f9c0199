// dcm_mpc_ipm_body.h — the interior point solve of one QP by one workgroup (dcm_mpc_ipm.hip's
// kernel; included by dcm_mpc_as.hip for the fused stage 2).  See dcm_mpc_ipm.hip for the
// algorithm notes.
#pragma once
#include "dcm_qp_common.h"

#include <stdlib.h>

#include <stdlib.h>

namespace blf {
namespace {
using namespace qp;

#ifdef BLF_STAMPS
// Diagnostic build only (make stamps): per-phase cycle sums of thread 0 for the first 64 QPs.
// [0] whole kernel, [1] factorization, [2] predictor solve .. corrector solve, [3] iterations,
// [4] residuals + reduction, [5] W-phase, [6] predictor solve, [7] corrector step + update,
// [8] polish attempts (cycles), [9] polish attempts (count), [10] load phase, [11] LQ start step,
// [12] initial slacks / multipliers / dual residual, [13] polish: projection + residuals,
// [14] polish: Riccati sweep, [15] polish: solve.
__device__ unsigned long long g_blf_stamps[16];
#define STAMP(t) unsigned long long t = __builtin_amdgcn_s_memtime()
#define STAMP_ADD(slot, t0) \
    do { if (blockIdx.x < 64 && threadIdx.x == 0) atomicAdd(&g_blf_stamps[slot], __builtin_amdgcn_s_memtime() - (t0)); } while (0)
#else
#define STAMP(t)
#define STAMP_ADD(slot, t0)
#endif


// LDS carve-up (doubles).  The host sizes the launch with the same code (Lds(nullptr, ...)).
//   A2  [M][N] double2  facet normals, knot-contiguous per facet (conflict-free b128 reads)
//   BI  [M][N] double2  (b, 1/s) of every facet: the offsets, and 1/s refreshed once per
//                       iteration (W-phase), overwritten by the corrector's multiplier step;
//                       one address and one b128 read serve both
//   bnd [NW][16]        per-wavefront boundary values (see the kB* slots)
//   red [4][NW][4]      reduction scratch, four rotating slots (no second barrier needed)
constexpr int kBP = 4;    // P_{64w} (3): the first knot's P, read by lane 63 of wavefront w-1
constexpr int kBV = 8;    // v_{64w} (2): backward-scan value at the first knot of wavefront w
constexpr int kBX = 10;   // x_{64w+64} (2): forward-scan value past the last knot of wavefront w
constexpr int kBN = 0;    // (nu_{64w}, omega_{64w}) (3): the refinement's next-knot costate, read by
                          // lane 63 of wavefront w-1
constexpr int kBnd = 16;
struct Lds {
    double2 *A2, *BI;   // facet rows: normal (a_x, a_y); (b, 1/s), 1/s later the multiplier step
    double *bnd, *red, *flag;
    size_t total;
    __host__ __device__ Lds(double* base, int N, int M, int NW)
    {
        size_t o = 0;
        auto take = [&](size_t n) {
            double* p = base ? base + o : nullptr;
            o += (n + 1) & ~size_t(1);
            return p;
        };
        A2 = reinterpret_cast<double2*>(take(2 * (size_t)M * N));
        BI = reinterpret_cast<double2*>(take(2 * (size_t)M * N));
        bnd = take((size_t)kBnd * NW);
        red = take(16 * (size_t)NW);
        flag = take(2);
        total = o;
    }
};

// Block reductions: xor-butterfly per wavefront, then the wavefronts' values in order (the
// oracle's orc_wave_tree_sum).  `slot` rotates over 4 scratch rows so that a row is never
// rewritten before every wavefront has read it (each reduction ends with one barrier).
template <int NW>
struct Reduce {
    double* red;
    int nwa;      // wavefronts that own knots (ceil(N/64)); the rest hold no data
    int slot = 0;
    __device__ double* row() { double* r = red + 4 * NW * slot; slot = (slot + 1) & 3; return r; }
    __device__ void sum_nanmax(double& s, double& m)
    {
        s = wave_sum(s);
        m = wave_nanmax(m);
        if constexpr (NW > 1) {
            double* r = row();
            const int w = threadIdx.x >> 6;
            if ((threadIdx.x & 63) == 0) { r[4 * w] = s; r[4 * w + 1] = m; }
            __syncthreads();
            s = r[0];
            m = r[1];
#pragma unroll
            for (int i = 1; i < NW; ++i) if (i < nwa) { s = s + r[4 * i]; m = nanmax(m, r[4 * i + 1]); }
        }
    }
    // Two sums and two NaN-propagating maxima in one exchange (the start-up statistics).
    __device__ void sums_nanmaxes(double& s1, double& s2, double& m1, double& m2)
    {
        s1 = wave_sum(s1);
        s2 = wave_sum(s2);
        m1 = wave_nanmax(m1);
        m2 = wave_nanmax(m2);
        if constexpr (NW > 1) {
            double* r = row();
            const int w = threadIdx.x >> 6;
            if ((threadIdx.x & 63) == 0) {
                r[4 * w] = s1;
                r[4 * w + 1] = s2;
                r[4 * w + 2] = m1;
                r[4 * w + 3] = m2;
            }
            __syncthreads();
            s1 = r[0];
            s2 = r[1];
            m1 = r[2];
            m2 = r[3];
#pragma unroll
            for (int i = 1; i < NW; ++i) {
                if (i < nwa) {
                    s1 = s1 + r[4 * i];
                    s2 = s2 + r[4 * i + 1];
                    m1 = nanmax(m1, r[4 * i + 2]);
                    m2 = nanmax(m2, r[4 * i + 3]);
                }
            }
        }
    }
    // A step-length maximum and up to two sums in one exchange (one barrier).
    template <int NS>
    __device__ void max_sums(double& q, double& s1, double& s2)
    {
        q = wave_keepmax(q);
        s1 = wave_sum(s1);
        if constexpr (NS > 1) s2 = wave_sum(s2);
        if constexpr (NW > 1) {
            double* r = row();
            const int w = threadIdx.x >> 6;
            if ((threadIdx.x & 63) == 0) {
                r[4 * w] = q;
                r[4 * w + 1] = s1;
                if constexpr (NS > 1) r[4 * w + 2] = s2;
            }
            __syncthreads();
            q = r[0];
            s1 = r[1];
            if constexpr (NS > 1) s2 = r[2];
#pragma unroll
            for (int i = 1; i < NW; ++i) {
                if (i < nwa) {
                    q = ::blf::keepmax(q, r[4 * i]);
                    s1 = s1 + r[4 * i + 1];
                    if constexpr (NS > 1) s2 = s2 + r[4 * i + 2];
                }
            }
        }
    }
    __device__ double sum(double s)
    {
        s = wave_sum(s);
        if constexpr (NW > 1) {
            double* r = row();
            const int w = threadIdx.x >> 6;
            if ((threadIdx.x & 63) == 0) r[4 * w] = s;
            __syncthreads();
            s = r[0];
#pragma unroll
            for (int i = 1; i < NW; ++i) if (i < nwa) s = s + r[4 * i];
        }
        return s;
    }
    __device__ double keepmax(double q)
    {
        q = wave_keepmax(q);
        if constexpr (NW > 1) {
            double* r = row();
            const int w = threadIdx.x >> 6;
            if ((threadIdx.x & 63) == 0) r[4 * w] = q;
            __syncthreads();
            q = r[0];
#pragma unroll
            for (int i = 1; i < NW; ++i) if (i < nwa) q = ::blf::keepmax(q, r[4 * i]);
        }
        return q;
    }
    // OR of a few flag bits over the workgroup in one exchange (__syncthreads_or costs a
    // reduction and two barriers per flag).
    template <int NB>
    __device__ int or_bits(int f)
    {
        int b = 0;
#pragma unroll
        for (int j = 0; j < NB; ++j) if (__ballot((f >> j) & 1) != 0) b |= 1 << j;
        if constexpr (NW > 1) {
            double* r = row();
            const int w = threadIdx.x >> 6;
            if ((threadIdx.x & 63) == 0) r[4 * w] = (double)b;
            __syncthreads();
            b = (int)r[0];
#pragma unroll
            for (int i = 1; i < NW; ++i) b |= (int)r[4 * i];
        }
        return b;
    }
    __device__ double nanmax_(double q)
    {
        q = wave_nanmax(q);
        if constexpr (NW > 1) {
            double* r = row();
            const int w = threadIdx.x >> 6;
            if ((threadIdx.x & 63) == 0) r[4 * w] = q;
            __syncthreads();
            q = r[0];
#pragma unroll
            for (int i = 1; i < NW; ++i) if (i < nwa) q = nanmax(q, r[4 * i]);
        }
        return q;
    }
};

// Backward affine recursion v_k = G_k v_{k+1} + c_k, v_N = 0 (oracle scan_backward).  Lanes past
// the last knot carry the zero element.  Returns v_{k+1} for this lane's knot.
template <int NW>
__device__ __forceinline__ void scan_backward(double g0, double g1, double g2, double g3, double c0,
                                              double c1, double* bnd, int nwa, int wv, int lane,
                                              double& vn0, double& vn1)
{
    const int ln = opaque(lane);
    {   // d = 1 through DPP (dcm_qp_common.h)
        const double p0 = dpp1<kNextWrap>(g0), p1 = dpp1<kNextWrap>(g1);
        const double p2 = dpp1<kNextWrap>(g2), p3 = dpp1<kNextWrap>(g3);
        const double q0 = dpp1<kNextWrap>(c0), q1 = dpp1<kNextWrap>(c1);
        if (ln + 1 < kWave) COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, c0, c1);
    }
#pragma unroll
    for (int d = 2; d < kWave; d <<= 1) {
        const int ad = ((ln + d) & (kWave - 1)) << 2;
        const double p0 = bperm(ad, g0), p1 = bperm(ad, g1);
        const double p2 = bperm(ad, g2), p3 = bperm(ad, g3);
        const double q0 = bperm(ad, c0), q1 = bperm(ad, c1);
        if (ln + d < kWave) COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, c0, c1);
    }
    double v0 = c0, v1 = c1;
    if constexpr (NW > 1) {
        for (int w = nwa - 1; w >= 0; --w) {
            if (wv == w) {
                if (w < nwa - 1) {
                    const double b0 = bnd[kBnd * (w + 1) + kBV], b1 = bnd[kBnd * (w + 1) + kBV + 1];
                    v0 = FD3(g0, b0, g1, b1, c0);
                    v1 = FD3(g2, b0, g3, b1, c1);
                }
                if (lane == 0) { bnd[kBnd * w + kBV] = v0; bnd[kBnd * w + kBV + 1] = v1; }
            }
            if (w > 0) __syncthreads();
        }
    }
    vn0 = dpp1<kNextWrap>(v0);
    vn1 = dpp1<kNextWrap>(v1);
    if (lane == kWave - 1) {
        vn0 = 0.0;
        vn1 = 0.0;
        if (NW > 1 && wv < nwa - 1) {
            vn0 = bnd[kBnd * (wv + 1) + kBV];
            vn1 = bnd[kBnd * (wv + 1) + kBV + 1];
        }
    }
}

// Forward affine recursion x_{k+1} = F_k x_k + f_k, x_0 = 0 (oracle scan_forward).  Returns
// x_{k+1} (this lane's result) and x_k (its input).
template <int NW>
__device__ __forceinline__ void scan_forward(double g0, double g1, double g2, double g3, double c0,
                                             double c1, double* bnd, int nwa, int wv, int lane, double& x0,
                                             double& x1, double& xk0, double& xk1)
{
    const int ln = opaque(lane);
    {   // d = 1 through DPP
        const double p0 = dpp1<kPrevWrap>(g0), p1 = dpp1<kPrevWrap>(g1);
        const double p2 = dpp1<kPrevWrap>(g2), p3 = dpp1<kPrevWrap>(g3);
        const double q0 = dpp1<kPrevWrap>(c0), q1 = dpp1<kPrevWrap>(c1);
        if (ln >= 1) COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, c0, c1);
    }
#pragma unroll
    for (int d = 2; d < kWave; d <<= 1) {
        const int ad = ((ln - d) & (kWave - 1)) << 2;
        const double p0 = bperm(ad, g0), p1 = bperm(ad, g1);
        const double p2 = bperm(ad, g2), p3 = bperm(ad, g3);
        const double q0 = bperm(ad, c0), q1 = bperm(ad, c1);
        if (ln >= d) COMPOSE(g0, g1, g2, g3, p0, p1, p2, p3, q0, q1, c0, c1);
    }
    x0 = c0;
    x1 = c1;
    if constexpr (NW > 1) {
        for (int w = 0; w < nwa; ++w) {
            if (wv == w) {
                if (w > 0) {
                    const double b0 = bnd[kBnd * (w - 1) + kBX], b1 = bnd[kBnd * (w - 1) + kBX + 1];
                    x0 = FD3(g0, b0, g1, b1, c0);
                    x1 = FD3(g2, b0, g3, b1, c1);
                }
                if (lane == kWave - 1) { bnd[kBnd * w + kBX] = x0; bnd[kBnd * w + kBX + 1] = x1; }
            }
            if (w < nwa - 1) __syncthreads();
        }
    }
    xk0 = dpp1<kPrevWrap>(x0);
    xk1 = dpp1<kPrevWrap>(x1);
    if (lane == 0) {
        xk0 = 0.0;
        xk1 = 0.0;
        if (NW > 1 && wv > 0) {
            xk0 = bnd[kBnd * (wv - 1) + kBX];
            xk1 = bnd[kBnd * (wv - 1) + kBX + 1];
        }
    }
}

// Per-knot state (registers of the knot's thread); MF facet slots (8, or 16 for phases of up to
// four contacts, max_facets > 8).
template <int MF>
struct KnotT {
    static constexpr int kMF = MF;
    int m;                                      // facet count
    double s[MF], lam[MF];
    double r0, r1;                              // VRP
    double x0, x1;                              // xi_{k+1}
    double w, al, be;                           // omega_k, 1 + dt omega_k, dt omega_k
    double rh0, rh1, d0, d1, qx0, qx1;          // dual residual part, Euler defect, Q(xi - xi_ref)
    double P00, P01, P11;                       // P_{k+1}
    double h00, h01, h11;                       // H_k^{-1}
};

// M = P_{k+1} H_k^{-1} (recomputed where needed: cheaper than 8 live VGPRs).
struct Mmat {
    double m00, m01, m10, m11;
    template <class KN>
    __device__ __forceinline__ explicit Mmat(const KN& K)
    {
        m00 = FD2(K.P00, K.h00, K.P01, K.h01);
        m01 = FD2(K.P00, K.h01, K.P01, K.h11);
        m10 = FD2(K.P01, K.h00, K.P11, K.h01);
        m11 = FD2(K.P01, K.h01, K.P11, K.h11);
    }
};

// Facet residual rp_i = (a . r + s_i) - b_i.
template <class KN>
__device__ __forceinline__ double facet_rp(const KN& K, double2 a, double bi, int i)
{
    return (FD2(a.x, K.r0, a.y, K.r1) + K.s[i]) - bi;
}

// r back onto its active line after a polish step (c = 1; oracle project_line): the step moves r
// along the line in exact arithmetic, but its rounding scales with the step's terms (costates up
// to 1e10 on the pushed-robot windows), and a drift of 1e-10 off the line failed the certificate.
template <class KN>
__device__ __forceinline__ void project_line(KN& K, double2 a, double bi)
{
    const double aa = FD2(a.x, a.x, a.y, a.y);
    const double t = (FD2(a.x, K.r0, a.y, K.r1) - bi) / aa;
    K.r0 = fma(-t, a.x, K.r0);
    K.r1 = fma(-t, a.y, K.r1);
}

// The affine slack / multiplier step of facet i for the VRP step (dra0, dra1) (oracle affine_step).
template <class KN>
__device__ __forceinline__ void affine_step(const KN& K, double2 a, double bi, double is, int i,
                                            double dra0, double dra1, double& ds, double& dl)
{
    const double rpi = facet_rp(K, a, bi, i);
    ds = (-rpi) - FD2(a.x, dra0, a.y, dra1);
    dl = -((K.lam[i] * (K.s[i] + ds)) * is);
}

// Residual pass (oracle dcm_residuals) for this lane's knot; xk = xi_k.  Returns pres, ck.
template <class KN>
__device__ __forceinline__ void residuals(KN& K, bool facets, const KParams& P, bool last,
                                          const double2* A2, const double2* BI, int N, int k,
                                          int mmax, double xk0, double xk1, const double* rref,
                                          const double* xref, double& pres, double& ck)
{
    pres = 0.0;
    ck = 0.0;
    double rh0 = P.Rw0 * (K.r0 - rref[0]);
    double rh1 = P.Rw1 * (K.r1 - rref[1]);
    if (facets) {
        const int kx = opaque(k);
        const int km = opaque(K.m), mm = opaque_s(mmax);
#pragma unroll
        for (int i = 0; i < KN::kMF; ++i) {
            if (KN::kMF <= kMaxFacets && i >= mm) break;   // 16 slots: no early exit, so the loop unrolls fully
            if (i < km) {
                const double2 a = A2[i * N + kx];
                const double gr = FD2(a.x, K.r0, a.y, K.r1);
                const double rpi = (gr + K.s[i]) - BI[i * N + kx].x;
                pres = nanmax(pres, fabs(rpi));
                ck = fma(K.s[i], K.lam[i], ck);
                rh0 = fma(a.x, K.lam[i], rh0);
                rh1 = fma(a.y, K.lam[i], rh1);
            }
        }
    }
    K.rh0 = rh0;
    K.rh1 = rh1;
    const double dx0 = FD2(K.w, xk0, -K.w, K.r0);
    const double dk0 = fma(dx0, P.dt, xk0) - K.x0;
    const double dx1 = FD2(K.w, xk1, -K.w, K.r1);
    const double dk1 = fma(dx1, P.dt, xk1) - K.x1;
    K.d0 = dk0;
    K.d1 = dk1;
    pres = nanmax(pres, fabs(dk0));
    pres = nanmax(pres, fabs(dk1));
    const double q0 = last ? P.Pw0 : P.Qw0;
    const double q1 = last ? P.Pw1 : P.Qw1;
    K.qx0 = q0 * (K.x0 - xref[0]);
    K.qx1 = q1 * (K.x1 - xref[1]);
}

// xi_k of this lane's knot: xi_{k+1} of the previous lane; lane 0 takes the wavefront's left boundary
// xb = xi_{64 w}, which every wavefront tracks itself (from the forward scans' boundary values, with
// the same arithmetic as the previous wavefront's last lane), so no barrier publishes it.
template <class KN>
__device__ __forceinline__ void xi_prev(const KN& K, int lane, double xb0, double xb1, double& xk0,
                                        double& xk1)
{
    xk0 = dpp1<kPrevWrap>(K.x0);
    xk1 = dpp1<kPrevWrap>(K.x1);
    if (lane == 0) {
        xk0 = xb0;
        xk1 = xb1;
    }
}

// Riccati sweep (oracle riccati_sweep) for this lane's E_k.  Leaves P_{k+1} in K.  Returns false
// on this lane if some (I + G H) or (I + G P) is not positive definite.
template <int NW, class KN>
__device__ __forceinline__ bool riccati(KN& K, const KParams& P, double E00, double E01,
                                        double E11, double* bnd, int N, int nwa, int k, int wv,
                                        int lane, bool own)
{
    bool ok = true;
    // P_k for every knot: Kogge-Stone scan of Riccati map elements over the wavefront's lanes
    // (oracle dcm_factor / rc_combine), then P_k = f_{k..}(P at the next wavefront's first knot)
    Rc e;
    if (own) {
        e.a0 = K.al; e.a1 = 0.0; e.a2 = 0.0; e.a3 = K.al;
        e.g0 = E00; e.g1 = E01; e.g2 = E11;
        e.h0 = P.Qw0; e.h1 = 0.0; e.h2 = P.Qw1;
    } else {
        e.a0 = 1.0; e.a1 = 0.0; e.a2 = 0.0; e.a3 = 1.0;
        e.g0 = e.g1 = e.g2 = 0.0;
        e.h0 = e.h1 = e.h2 = 0.0;
    }
    const int ln = opaque(lane);
    {   // d = 1 through DPP
        Rc q;
        q.a0 = dpp1<kNextWrap>(e.a0); q.a1 = dpp1<kNextWrap>(e.a1);
        q.a2 = dpp1<kNextWrap>(e.a2); q.a3 = dpp1<kNextWrap>(e.a3);
        q.g0 = dpp1<kNextWrap>(e.g0); q.g1 = dpp1<kNextWrap>(e.g1); q.g2 = dpp1<kNextWrap>(e.g2);
        q.h0 = dpp1<kNextWrap>(e.h0); q.h1 = dpp1<kNextWrap>(e.h1); q.h2 = dpp1<kNextWrap>(e.h2);
        if (ln + 1 < kWave) ok = rc_combine(e, q) && ok;
    }
#pragma unroll
    for (int d = 2; d < kWave; d <<= 1) {
        const int ad = ((ln + d) & (kWave - 1)) << 2;
        Rc q;
        q.a0 = bperm(ad, e.a0); q.a1 = bperm(ad, e.a1); q.a2 = bperm(ad, e.a2); q.a3 = bperm(ad, e.a3);
        q.g0 = bperm(ad, e.g0); q.g1 = bperm(ad, e.g1); q.g2 = bperm(ad, e.g2);
        q.h0 = bperm(ad, e.h0); q.h1 = bperm(ad, e.h1); q.h2 = bperm(ad, e.h2);
        if (ln + d < kWave) ok = rc_combine(e, q) && ok;
    }
    double Pk00 = 0.0, Pk01 = 0.0, Pk11 = 0.0;
    for (int w = nwa - 1; w >= 0; --w) {
        if (wv == w) {
            double b0 = P.Pw0, b1 = 0.0, b2v = P.Pw1;
            if (w < nwa - 1) {
                b0 = bnd[kBnd * (w + 1) + kBP];
                b1 = bnd[kBnd * (w + 1) + kBP + 1];
                b2v = bnd[kBnd * (w + 1) + kBP + 2];
            }
            ok = rc_apply(e, b0, b1, b2v, Pk00, Pk01, Pk11) && ok;
            if (lane == 0 && w > 0) {
                bnd[kBnd * w + kBP] = Pk00;
                bnd[kBnd * w + kBP + 1] = Pk01;
                bnd[kBnd * w + kBP + 2] = Pk11;
            }
        }
        if (w > 0) __syncthreads();
    }
    // lane k takes P_{k+1} from lane k+1
    double P00 = dpp1<kNextWrap>(Pk00);
    double P01 = dpp1<kNextWrap>(Pk01);
    double P11 = dpp1<kNextWrap>(Pk11);
    if (lane == kWave - 1 && NW > 1 && wv < nwa - 1) {
        P00 = bnd[kBnd * (wv + 1) + kBP];
        P01 = bnd[kBnd * (wv + 1) + kBP + 1];
        P11 = bnd[kBnd * (wv + 1) + kBP + 2];
    }
    if (k == N - 1) {
        P00 = P.Pw0;
        P01 = 0.0;
        P11 = P.Pw1;
    }
    K.P00 = P00;
    K.P01 = P01;
    K.P11 = P11;
    return ok;
}

// Factorization (oracle dcm_factor) from W = (W00, W01, W11, detW).  Leaves P_{k+1}, h, M in K.
// Returns false on this lane if its K or H block is not positive definite.
template <int NW, class KN>
__device__ __forceinline__ bool factor(KN& K, const KParams& P, double W00, double W01,
                                       double W11, double dW, double* bnd, int N, int nwa, int k,
                                       int wv, int lane, bool own)
{
    const double b2 = K.be * K.be;
    double E00 = 0.0, E01 = 0.0, E11 = 0.0;
    if (own) {
        const double detRW = fma(P.Rw0, P.Rw1, FD2(P.Rw1, W00, P.Rw0, W11)) + dW;
        const double ie = b2 / detRW;
        E00 = (P.Rw1 + W11) * ie;
        E01 = -(W01 * ie);
        E11 = (P.Rw0 + W00) * ie;
    }
    bool ok = riccati<NW>(K, P, E00, E01, E11, bnd, N, nwa, k, wv, lane, own);
    if (own) {
        const double B00 = fma(b2, K.P00, P.Rw0);
        const double B01 = b2 * K.P01;
        const double B11 = fma(b2, K.P11, P.Rw1);
        const double H00 = B00 + W00;
        const double H01 = B01 + W01;
        const double H11 = B11 + W11;
        const double detB = fma(B00, B11, -(B01 * B01));
        const double trW = FD2(B11, W00, B00, W11) - 2.0 * (B01 * W01);
        const double det = (detB + trW) + dW;
        if (!(det > 0.0) || __builtin_isinf(det)) ok = false;
        const double idet = 1.0 / det;
        K.h00 = H11 * idet;
        K.h01 = -(H01 * idet);
        K.h11 = H00 * idet;
    }
    return ok;
}

// Solve the factored Newton system for the right-hand side g (oracle dcm_solve).  Returns
// dr (the VRP step of this knot), dx (the DCM step of xi_{k+1}), v_{k+1} of the backward scan and
// the DCM step of xi_k (lane 0 of a wavefront: its left boundary, from the previous wavefront).
template <int NW, class KN>
__device__ __forceinline__ void solve(const KN& K, double g0, double g1, double* bnd, int nwa,
                                      int wv, int lane, bool own, double& dr0, double& dr1, double& dx0,
                                      double& dx1, double& vn0, double& vn1, double& xk0, double& xk1)
{
    const double b2 = K.be * K.be;
    const double ab = K.al * K.be;
    double G00 = 0.0, G01 = 0.0, G10 = 0.0, G11 = 0.0, c0 = 0.0, c1 = 0.0, y0 = 0.0, y1 = 0.0;
    if (own) {
        const Mmat Mm(K);
        y0 = FD3(K.P00, K.d0, K.P01, K.d1, K.qx0);
        y1 = FD3(K.P01, K.d0, K.P11, K.d1, K.qx1);
        const double Mg0 = FD2(Mm.m00, g0, Mm.m01, g1);
        const double Mg1 = FD2(Mm.m10, g0, Mm.m11, g1);
        G00 = K.al * fma(-b2, Mm.m00, 1.0);
        G01 = -(K.al * (b2 * Mm.m01));
        G10 = -(K.al * (b2 * Mm.m10));
        G11 = K.al * fma(-b2, Mm.m11, 1.0);
        c0 = FD3(G00, y0, G01, y1, ab * Mg0);
        c1 = FD3(G10, y0, G11, y1, ab * Mg1);
    }
    scan_backward<NW>(G00, G01, G10, G11, c0, c1, bnd, nwa, wv, lane, vn0, vn1);
    double k0 = 0.0, k1 = 0.0, f0 = 0.0, f1 = 0.0;
    if (own) {
        const double t0 = y0 + vn0;
        const double t1 = y1 + vn1;
        const double hu0 = fma(-K.be, t0, g0);
        const double hu1 = fma(-K.be, t1, g1);
        k0 = -FD2(K.h00, hu0, K.h01, hu1);
        k1 = -FD2(K.h01, hu0, K.h11, hu1);
        f0 = fma(-K.be, k0, K.d0);
        f1 = fma(-K.be, k1, K.d1);
    }
    scan_forward<NW>(G00, G10, G01, G11, f0, f1, bnd, nwa, wv, lane, dx0, dx1, xk0, xk1);
    const Mmat Mm(K);
    dr0 = fma(ab, FD2(Mm.m00, xk0, Mm.m10, xk1), k0);
    dr1 = fma(ab, FD2(Mm.m01, xk0, Mm.m11, xk1), k1);
}

// The saturated LQ start of the interior point method (oracle dcm_saturated_start, DESIGN.md 4
// item 9), run when the active-set start did not certify (tol_polish > 0): the LQ policy around the
// current iterate, rolled out from xi_init with every VRP projected onto its support polygon in the
// one-step Hessian's metric, costates of the rollout by single shooting, multipliers of the
// projected facets from stationarity, s = max(b - A r, 1e-2), lam = max(estimate, 1e-2 / s).
// The rollout is sequential over the knots: wavefront w takes its 64 knots in turn (the others
// wait at a barrier), each knot's policy data broadcast from its lane by v_readlane and its
// projection candidates (8 single facets, 28 facet pairs) evaluated one per lane, the lowest lane
// of the least B-distance winning (oracle sat_project's candidate order).  Leaves r, xi, s, lam,
// the residuals and xb in place; returns mu, pres, dres, and false on a lane whose LQ factorization
// failed.
#ifndef BLF_SAT_ON
#define BLF_SAT_ON 1
#endif
constexpr int kBS = 12;   // bnd slot: the rollout's xi at the end of wavefront w
template <int NW, class KN>
__device__ __forceinline__ bool sat_start(KN& K, const KParams& P, const Lds& L, Reduce<NW>& R, double* bnd,
                                          int N, int nwa, int k, int wv, int lane, bool own, bool last,
                                          int mmax, double xi00, double xi01, const double* rref,
                                          const double* xref, double& xb0, double& xb1, double& mu,
                                          double& pres, double& dres)
{
    // 1. the LQ step around the current iterate: the LQ optimum (r*, xi*) and its policy
    double xk0, xk1, pd, cd;
    xi_prev(K, lane, xb0, xb1, xk0, xk1);
    if (own) residuals(K, false, P, last, L.A2, L.BI, N, k, mmax, xk0, xk1, rref, xref, pd, cd);
    const bool ok = factor<NW>(K, P, 0.0, 0.0, 0.0, 0.0, bnd, N, nwa, k, wv, lane, own);
    double dr0, dr1, dx0, dx1, vn0, vn1, dxk0, dxk1;
    solve<NW>(K, K.rh0, K.rh1, bnd, nwa, wv, lane, own, dr0, dr1, dx0, dx1, vn0, vn1, dxk0, dxk1);
    const double rs0 = K.r0 + dr0, rs1 = K.r1 + dr1;       // r*_k
    const double xs0 = xk0 + dxk0, xs1 = xk1 + dxk1;       // xi*_k
    const Mmat Mm(K);
    const double ab = K.al * K.be;
    const double b2 = K.be * K.be;
    const double B00 = fma(b2, K.P00, P.Rw0);
    const double B01 = b2 * K.P01;
    const double B11 = fma(b2, K.P11, P.Rw1);
    // 2. the rollout
    int sc = 0, s1 = 0, s2 = 0;   // this knot's projected facets
    for (int w = 0; w < nwa; ++w) {
        if (wv == w) {
            double x0 = xi00, x1 = xi01;
            if (w > 0) {
                x0 = bnd[kBnd * (w - 1) + kBS];
                x1 = bnd[kBnd * (w - 1) + kBS + 1];
            }
            xb0 = x0;
            xb1 = x1;
            const int jn = N - kWave * w < kWave ? N - kWave * w : kWave;
            for (int j = 0; j < jn; ++j) {
                const int kk = kWave * w + j;
                const int m = __builtin_amdgcn_readlane(K.m, j);
                const double d0 = x0 - readlane_f64(xs0, j), d1 = x1 - readlane_f64(xs1, j);
                const double abj = readlane_f64(ab, j);
                const double t0 = fma(abj, FD2(readlane_f64(Mm.m00, j), d0, readlane_f64(Mm.m10, j), d1),
                                      readlane_f64(rs0, j));
                const double t1 = fma(abj, FD2(readlane_f64(Mm.m01, j), d0, readlane_f64(Mm.m11, j), d1),
                                      readlane_f64(rs1, j));
                const double c00 = readlane_f64(B00, j), c01 = readlane_f64(B01, j), c11 = readlane_f64(B11, j);
                // (the facet loops below are unrolled over the slots and predicated on i < m, so
                // every row's LDS read issues at once; the same comparisons as a loop to m)
                bool inside = true;
#pragma unroll
                for (int i = 0; i < KN::kMF; ++i) {
                    const int ii = i < m ? i : 0;
                    const double2 a = L.A2[ii * N + kk];
                    const double bi = L.BI[ii * N + kk].x;
                    if (i < m && !(FD2(a.x, t0, a.y, t1) - bi <= 0.0)) inside = false;
                }
                double r0 = t0, r1 = t1;
                int c = 0, i1 = 0, i2 = 0;
                if (!inside) {
                    // the candidates, one per lane in rounds of 64: c < m facet c; c >= m the
                    // facet pair q = c - m of (x, y), x < y < m, in lexicographic order
                    const int nc = m + (m * (m - 1)) / 2;
                    bool have = false;
                    double best = 0.0;
                    for (int c0 = 0; c0 < nc; c0 += kWave) {
                        const int cc = c0 + lane;
                        int cx = cc, cy = cc;
                        if (cc >= m) {
                            int q = cc - m;
                            cx = 0;
                            while (cx < m - 1 && q >= m - 1 - cx) { q -= m - 1 - cx; ++cx; }
                            cy = cx + 1 + q;
                        }
                        bool valid = false;
                        double v0 = 0.0, v1 = 0.0, dist = 0.0;
                        if (cc < m) {
                            const double2 a = L.A2[cx * N + kk];
                            const double u0 = fma(c11, a.x, -(c01 * a.y));
                            const double u1 = fma(c00, a.y, -(c01 * a.x));
                            const double aua = FD2(a.x, u0, a.y, u1);
                            const double viol = FD2(a.x, t0, a.y, t1) - L.BI[cx * N + kk].x;
                            const double t = viol / aua;
                            v0 = fma(-t, u0, t0);
                            v1 = fma(-t, u1, t1);
                            valid = viol > 0.0;
                            dist = (t * viol) * fma(c00, c11, -(c01 * c01));
                        } else if (cc < nc) {
                            const double2 a = L.A2[cx * N + kk];
                            const double2 e = L.A2[cy * N + kk];
                            const double ba = L.BI[cx * N + kk].x, be = L.BI[cy * N + kk].x;
                            const double det = fma(a.x, e.y, -(a.y * e.x));
                            const double aa = FD2(a.x, a.x, a.y, a.y), ee = FD2(e.x, e.x, e.y, e.y);
                            valid = det * det > 1e-18 * (aa * ee);
                            const double idet = 1.0 / det;
                            v0 = fma(ba, e.y, -(a.y * be)) * idet;
                            v1 = fma(a.x, be, -(ba * e.x)) * idet;
                            const double e0 = v0 - t0, e1 = v1 - t1;
                            dist = fma(e0, fma(c00, e0, 2.0 * (c01 * e1)), (c11 * e1) * e1);
                        }
#pragma unroll
                        for (int l = 0; l < KN::kMF; ++l) {
                            const int ll = l < m ? l : 0;
                            const double2 f = L.A2[ll * N + kk];
                            const double bl = L.BI[ll * N + kk].x;
                            if (l < m && !(FD2(f.x, v0, f.y, v1) - bl <= P.tol_p)) valid = false;
                        }
                        if (!(dist == dist)) valid = false;
                        const double key = valid ? dist : __builtin_inf();
                        const double kmin = wave_keepmin(key);
                        const unsigned long long win = __ballot(valid && key == kmin);
                        // the first of equal distances wins: a later round only with a smaller one
                        if (win != 0ull && (!have || kmin < best)) {
                            const int f = __builtin_ctzll(win);
                            have = true;
                            best = kmin;
                            r0 = readlane_f64(v0, f);
                            r1 = readlane_f64(v1, f);
                            i1 = __builtin_amdgcn_readlane(cx, f);
                            i2 = __builtin_amdgcn_readlane(cy, f);
                            c = c0 + f < m ? 1 : 2;
                        }
                    }
                }
                const double om = readlane_f64(K.w, j);
                const double y0 = fma(FD2(om, x0, -om, r0), P.dt, x0);
                const double y1 = fma(FD2(om, x1, -om, r1), P.dt, x1);
                if (lane == j) {
                    K.r0 = r0;
                    K.r1 = r1;
                    K.x0 = y0;
                    K.x1 = y1;
                    sc = c;
                    s1 = i1;
                    s2 = i2;
                }
                x0 = y0;
                x1 = y1;
            }
            if (lane == 0) {
                bnd[kBnd * w + kBS] = x0;
                bnd[kBnd * w + kBS + 1] = x1;
            }
        }
        if (w < nwa - 1) __syncthreads();
    }
    // 3. costates of the rollout (the warm start's backward scan), multiplier estimates, s, lam
    xi_prev(K, lane, xb0, xb1, xk0, xk1);
    if (own) residuals(K, false, P, last, L.A2, L.BI, N, k, mmax, xk0, xk1, rref, xref, pd, cd);
    {
        const double ga = own ? K.al : 0.0;
        const double c0 = own ? K.al * K.qx0 : 0.0, c1 = own ? K.al * K.qx1 : 0.0;
        scan_backward<NW>(ga, 0.0, 0.0, ga, c0, c1, bnd, nwa, wv, lane, vn0, vn1);
    }
    dres = 0.0;
    if (own) {
        const int kx = opaque(k);
        const double nu0 = K.qx0 + vn0;
        const double nu1 = K.qx1 + vn1;
        const double g0 = fma(K.be, nu0, -K.rh0);
        const double g1 = fma(K.be, nu1, -K.rh1);
        double l1 = 0.0, l2 = 0.0;
        if (sc == 1) {
            const double2 a = L.A2[s1 * N + kx];
            l1 = FD2(a.x, g0, a.y, g1) / FD2(a.x, a.x, a.y, a.y);
        } else if (sc == 2) {
            const double2 a = L.A2[s1 * N + kx];
            const double2 e = L.A2[s2 * N + kx];
            const double idet = 1.0 / fma(a.x, e.y, -(a.y * e.x));
            l1 = fma(g0, e.y, -(e.x * g1)) * idet;
            l2 = fma(a.x, g1, -(g0 * a.y)) * idet;
        }
        double al0 = 0.0, al1 = 0.0;
        const int km = opaque(K.m);
        // every slot written (the unused ones to their initial 1 / 0), so the old values are dead
        // during the rollout
#pragma unroll
        for (int i = 0; i < KN::kMF; ++i) {
            K.s[i] = 1.0;
            K.lam[i] = 0.0;
            if (i < km) {
                const double2 a = L.A2[i * N + kx];
                const double sl = L.BI[i * N + kx].x - FD2(a.x, K.r0, a.y, K.r1);
                const double si = sl > 1e-2 ? sl : 1e-2;
                const double est = (sc >= 1 && i == s1) ? l1 : (sc == 2 && i == s2) ? l2 : 0.0;
                const double lc = 1e-2 / si;
                K.s[i] = si;
                K.lam[i] = est > lc ? est : lc;
                al0 = fma(a.x, K.lam[i], al0);
                al1 = fma(a.y, K.lam[i], al1);
            }
        }
        dres = nanmax(nanmax(0.0, fabs(al0 - g0)), fabs(al1 - g1));
    }
    // 4. mu and the primal residual at the new point, in one reduction with dres
    pres = 0.0;
    double ck = 0.0;
    if (own) residuals(K, true, P, last, L.A2, L.BI, N, k, mmax, xk0, xk1, rref, xref, pres, ck);
    double mcount = (double)K.m;
    R.sums_nanmaxes(mcount, ck, pres, dres);
    const int ntot = (int)mcount;
    mu = ntot > 0 ? ck / (double)ntot : 0.0;
    return ok;
}

#ifndef BLF_MIN_WAVES
// waves per SIMD the register allocation must allow: 2 (<= 256 VGPRs).  At 3 (<= 168) the polish
// and the saturated start spill 89-118 VGPRs and ~210 B of scratch per lane (round 4).
#define BLF_MIN_WAVES 2
#endif
// The solve of QP p by one workgroup of NT threads (the kernel below; the active-set kernel's
// fused stage 2 for N <= 64, dcm_mpc_as.hip, calls it from its own 64-thread workgroup).
template <int NT, bool WARM, bool LAMOUT, int MF = kMaxFacets>
__device__ __forceinline__ void ipm_solve(
    const KParams P, const int64_t p, const double* __restrict__ xi_init, const double* __restrict__ omega,
    const double* __restrict__ xi_ref, const double* __restrict__ vrp_ref,
    const double* __restrict__ Ain, const double* __restrict__ bin,
    const int32_t* __restrict__ nfacets, const double* __restrict__ ws_vrp,
    const double* __restrict__ ws_lam, double* __restrict__ xi_out,
    double* __restrict__ vrp_out, int32_t* __restrict__ status_out,
    int32_t* __restrict__ iters_out, int32_t* __restrict__ polished_out, double* __restrict__ lam_out)
{
    constexpr int NW = NT / kWave;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int N = P.N, M = P.M;
    const Lds L(smem, N, M, NW);
    double* bnd = L.bnd;
    const int nwa = (N + kWave - 1) / kWave;
    Reduce<NW> R{L.red, nwa};

    const int k = threadIdx.x;
    const int lane = k & (kWave - 1);
    const int wv = __builtin_amdgcn_readfirstlane(k >> 6);
    const bool own = k < N;
    const bool last = k == N - 1;
    // after the active-set kernel (dcm_mpc_as.hip): only the QPs it handed over
    const int st0 = P.stage2 ? status_out[p] : 0;
    if (P.stage2 && st0 != kPending && st0 != kPendingCold) return;
    // solved here alone (no active-set kernel before): no active-set kernel passes
    if (!P.stage2 && P.passes_out != nullptr && threadIdx.x == 0) P.passes_out[p] = 0;
    // a separate instantiation each way; in the warm one, a problem whose previous solve failed
    // (KParams::ws_status) starts cold, as the cold instantiation would start it
    // (and one the warm kernel re-solved cold and still handed over, kPendingCold)
    const bool warm = WARM && !(P.ws_status != nullptr && P.ws_status[p] != 0) && st0 != kPendingCold;
    const bool ws = warm && k + P.ws_shift < N;           // this knot starts from the warm start
    STAMP(t_start);

    // ---- load the knot this thread owns ----
    KnotT<MF> K;
    K.m = 0;
    K.r0 = K.r1 = K.x0 = K.x1 = K.w = K.be = 0.0;
    K.rh0 = K.rh1 = K.d0 = K.d1 = K.qx0 = K.qx1 = 0.0;
    K.P00 = K.P01 = K.P11 = K.h00 = K.h01 = K.h11 = 0.0;
#pragma unroll
    for (int i = 0; i < MF; ++i) { K.s[i] = 1.0; K.lam[i] = 0.0; }
    bool bad = false;
    const double xi00 = xi_init[2 * p], xi01 = xi_init[2 * p + 1];
    if (own) {
        const int64_t st = p * N + k;
        K.m = nfacets[st];
        bad = (K.m < 0 || K.m > M);
        if (bad) K.m = 0;
        K.w = omega[st];
        K.be = P.dt * K.w;
        // stage 2: the start point the active-set kernel left in the outputs
        const double* r0 = P.stage2 ? vrp_out : ws ? ws_vrp + 2 * P.ws_shift : vrp_ref;
        K.r0 = r0[2 * st];
        K.r1 = r0[2 * st + 1];
        const double* Ak = Ain + st * M * 2;
        const double* bk = bin + st * M;
        for (int i = 0; i < K.m; ++i) {
            L.A2[i * N + k] = make_double2(Ak[2 * i], Ak[2 * i + 1]);
            L.BI[i * N + k].x = bk[i];
        }
    }
    K.al = 1.0 + K.be;
    // this knot's references (re-read from global memory in every residual pass)
    const int64_t kk_ = own ? p * N + k : 0;
    const double* rref = vrp_ref + 2 * kk_;
    const double* xref = xi_ref + 2 * (own ? p * (N + 1) + (k + 1) : 0);
    int mmax = K.m;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const int o = __shfl_xor(mmax, off, kWave);
        mmax = o > mmax ? o : mmax;
    }
    mmax = __builtin_amdgcn_readfirstlane(mmax);
    const bool any_bad = __syncthreads_or(bad);
    STAMP_ADD(10, t_start);

    // ---- initial point 1: a warm start rolls xi out from its VRPs, xi_{k+1} = alpha_k xi_k -
    //      beta_k r_k; a cold start begins at xi = xi_ref (its LQ step is exact from any
    //      trajectory) ----
    // xb = xi_{64 wv}, the left boundary of this wavefront (lane 0 uses it; wavefront 0: xi_init)
    double xb0 = xi00, xb1 = xi01;
    if (P.stage2) {   // the start point (the LQ optimum or the warm rollout) from the outputs
        const double* xo = xi_out + 2 * p * (N + 1);
        if (own) {
            K.x0 = xo[2 * (k + 1)];
            K.x1 = xo[2 * (k + 1) + 1];
        }
        if (wv > 0) {
            xb0 = xo[2 * kWave * wv];
            xb1 = xo[2 * kWave * wv + 1];
        }
    } else if (!warm) {
        if (own) {
            K.x0 = xref[0];
            K.x1 = xref[1];
            if (wv > 0) {   // xi_ref_{64 wv}: the previous wavefront's last xi_{k+1}
                xb0 = xref[-2];
                xb1 = xref[-1];
            }
        }
    } else {
        double f0 = 0.0, f1 = 0.0;
        if (own) {
            if (k == 0) {
                f0 = fma(K.al, xi00, -(K.be * K.r0));
                f1 = fma(K.al, xi01, -(K.be * K.r1));
            } else {
                f0 = -(K.be * K.r0);
                f1 = -(K.be * K.r1);
            }
        }
        const double ga = own ? K.al : 0.0;
        double xk0, xk1;
        scan_forward<NW>(ga, 0.0, 0.0, ga, f0, f1, bnd, nwa, wv, lane, K.x0, K.x1, xk0, xk1);
        if (wv > 0) {
            xb0 = xk0;
            xb1 = xk1;
        }
    }

    int status = 0, it = 0, polished = 0;
    if (any_bad) {
        status = BLF_QP_BAD_FACETS;
    } else {
        double xk0, xk1, pres, ck;
        bool ok, init_bad = false;
        // ---- initial point 2: full Newton step of the unconstrained QP (W = 0, lam = 0);
        //      a warm start skips it ----
        STAMP(t_lq);
        if (!warm && !P.stage2) {
            xi_prev(K, lane, xb0, xb1, xk0, xk1);
            if (own) residuals(K, false, P, last, L.A2, L.BI, N, k, mmax, xk0, xk1, rref, xref, pres, ck);
            ok = factor<NW>(K, P, 0.0, 0.0, 0.0, 0.0, bnd, N, nwa, k, wv, lane, own);
            init_bad = __syncthreads_or(!ok);
            {
                double dr0, dr1, dx0, dx1, vn0, vn1, dxk0, dxk1;
                solve<NW>(K, K.rh0, K.rh1, bnd, nwa, wv, lane, own, dr0, dr1, dx0, dx1, vn0, vn1, dxk0,
                          dxk1);
                if (own) {
                    K.r0 = K.r0 + dr0;
                    K.r1 = K.r1 + dr1;
                    K.x0 = K.x0 + dx0;
                    K.x1 = K.x1 + dx1;
                }
                if (wv > 0) {
                    xb0 = xb0 + dxk0;
                    xb1 = xb1 + dxk1;
                }
            }
        }
        STAMP_ADD(11, t_lq);
        STAMP(t_in);
        // ---- initial point 3: s = max(b - A r, 1e-2), lam = 1e-2 / s;
        //      warm knots: s = max(b - A r, floor), lam = max(lam_warm, floor) ----
        double dres = 0.0;
        int gm = 0;   // the active-set start's guess (bit i: facet i), see below
        if (own) {
            const double sfloor = ws ? P.ws_floor : 1e-2;
            const double* lw = ws_lam + (ws ? (p * N + k + P.ws_shift) * M : 0);
            double al0 = 0.0, al1 = 0.0;   // A^T lam
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                if (MF <= kMaxFacets && i >= mmax) break;
                if (i < K.m) {
                    const double2 a = L.A2[i * N + k];
                    const double gr = FD2(a.x, K.r0, a.y, K.r1);
                    const double sl = L.BI[i * N + k].x - gr;
                    K.s[i] = sl > sfloor ? sl : sfloor;
                    if (sl < 0.0) gm |= 1 << i;   // violated by the start point
                    if (ws) {
                        const double l = lw[i];
                        K.lam[i] = l > sfloor ? l : sfloor;
                        if (l > sfloor) gm |= 1 << i;   // active in the previous solution
                    } else {
                        K.lam[i] = 1e-2 / K.s[i];   // centred: s lam = 1e-2
                    }
                    al0 = fma(a.x, K.lam[i], al0);
                    al1 = fma(a.y, K.lam[i], al1);
                }
            }
            // a cold start sits at the unconstrained optimum, R (r - r_ref) = beta nu: its dual
            // residual is A^T lam exactly (single-shooting costates would only add rounding
            // amplified by alpha^N)
            if (!warm) dres = nanmax(nanmax(0.0, fabs(al0)), fabs(al1));
        }
        // ---- initial mu, primal residual and dual residual (warm start: costates nu_k = qx_k +
        //      alpha_k nu_{k+1} by a backward scan), in one reduction with the facet count;
        //      afterwards every step updates them (mu, pres and dres are known at the top of
        //      every iteration) ----
        xi_prev(K, lane, xb0, xb1, xk0, xk1);
        pres = 0.0;
        ck = 0.0;
        if (own) residuals(K, true, P, last, L.A2, L.BI, N, k, mmax, xk0, xk1, rref, xref, pres, ck);
        if (warm) {
            const double ga = own ? K.al : 0.0;
            const double c0 = own ? K.al * K.qx0 : 0.0, c1 = own ? K.al * K.qx1 : 0.0;
            double vn0, vn1;
            scan_backward<NW>(ga, 0.0, 0.0, ga, c0, c1, bnd, nwa, wv, lane, vn0, vn1);
            if (own) {
                const double nu0 = K.qx0 + vn0;
                const double nu1 = K.qx1 + vn1;
                dres = nanmax(dres, fabs(fma(-K.be, nu0, K.rh0)));
                dres = nanmax(dres, fabs(fma(-K.be, nu1, K.rh1)));
            }
        }
        double mcount = (double)K.m;
        R.sums_nanmaxes(mcount, ck, pres, dres);
        const int ntot = (int)mcount;   // exact: small integers
        double mu = ntot > 0 ? ck / (double)ntot : 0.0;
        if (init_bad) status = BLF_QP_NUMERICAL;
        STAMP_ADD(12, t_in);

        int drop = 0;    // polish passes 1, 2: facets taken out of the guessed active set (bit i)
        int add = 0;     // polish pass 2: facets put into it
        int pass = 0;    // the polish pass the next loop top runs (uniform)
        // active-set start (oracle: before its IPM loop): the first polish runs before any IPM
        // iteration from the guess gm, with up to kGuessPasses drop/add passes
        bool guess = P.tol_polish > 0.0 && !P.stage2;
        // the interior point method starts from the saturated LQ start (sat_start) when an
        // active-set start failed: the kernel's own (guess), or the active-set kernel's (stage 2)
        bool sat_pending = P.tol_polish > 0.0 && P.stage2;
        double last_a = 1.0;   // the previous IPM step length (the stalled-step polish, kStallStep)
        for (it = 0; status == 0; ++it) {
            if (BLF_SAT_ON && sat_pending) {
                sat_pending = false;
                STAMP(t_sat);   // (stamp builds: the saturated start counts as start-up, slot 12)
                const bool oks = sat_start<NW>(K, P, L, R, bnd, N, nwa, k, wv, lane, own, last, mmax, xi00, xi01,
                                               rref, xref, xb0, xb1, mu, pres, dres);
                STAMP_ADD(12, t_sat);
                if (__syncthreads_or(!oks)) {
                    status = BLF_QP_NUMERICAL;
                    it = 0;
                    break;
                }
            }
            // ---- residuals (knot-parallel) ----
            STAMP(t_r);
            xi_prev(K, lane, xb0, xb1, xk0, xk1);
            if (it > 0 && own) {
                double pd, cd;
                residuals(K, true, P, last, L.A2, L.BI, N, k, mmax, xk0, xk1, rref, xref, pd, cd);
            }
            if (!(mu == mu) || !(pres == pres) || !(dres == dres) || __builtin_isinf(mu)) {
                status = BLF_QP_NUMERICAL;
                break;
            }
            STAMP_ADD(4, t_r);
            // the polish at mu <= tol_polish, and after a stalled step once mu <= kStallMu (oracle
            // ORC_STALL_STEP: the pushed-robot windows stall at mu ~1e-3 with steps of 1e-8..1e-100
            // while lam > s already names the optimal active set)
            if (guess || (P.tol_polish > 0.0 && (mu <= P.tol_polish || (last_a < kStallStep && mu <= kStallMu)))) {
                // ---- active-set polish (oracle dcm_polish, DESIGN.md 4 "Polish"): one Newton
                //      step of the QP with the guessed active facets as equalities, certified
                //      (primal, stationarity, multiplier signs) or undone; a failed pass is
                //      retried without the negative-multiplier facets, then with the violated
                //      facets added (oracle dcm_polish) ----
                STAMP(t_p);
                const double sr0 = K.r0, sr1 = K.r1, sx0 = K.x0, sx1 = K.x1;
                int pc = 0, pi1 = 0, pi2 = 0, pk = 0;
                double E00 = 0.0, E01 = 0.0, E11 = 0.0;
                bool okp = true, neg = false, viol = false;
                if (own) {
                    const int kx = opaque(k);
                    const int km = opaque(K.m), mm = opaque_s(mmax);
                    const int dm = opaque(drop), am = opaque(add), gk = opaque(gm);
                    int cm = 0;   // the pass's active-set candidates (bit i: facet i)
                    double lmx = 0.0;   // the knot's largest multiplier (the IPM guess's scale)
                    int jm = 0;         // its facet (the first of equal ones)
                    if (!guess) {
#pragma unroll
                        for (int i = 0; i < MF; ++i) {
                            if (MF <= kMaxFacets && i >= mm) break;   // 16 slots: no early exit, so the loop unrolls fully
                            if (i < km) {
                                if (K.lam[i] > lmx) jm = i;
                                lmx = keepmax(lmx, K.lam[i]);
                            }
                        }
                    }
                    const double2 amx = L.A2[jm * N + kx];
#pragma unroll
                    for (int i = 0; i < MF; ++i) {
                        if (MF <= kMaxFacets && i >= mm) break;   // 16 slots: no early exit, so the loop unrolls fully
                        // faint (oracle cand_bit): below kLamRel of the knot's largest multiplier and
                        // within kLamRelCross of parallel to its facet
                        bool faint = false;
                        if (!guess && i < km) {
                            const double2 ai = L.A2[i * N + kx];
                            const double cr = fabs(fma(ai.x, amx.y, -(ai.y * amx.x)));
                            faint = K.lam[i] < kLamRel * lmx && cr < kLamRelCross;
                        }
                        const bool base = guess ? ((gk >> i) & 1) != 0 : (K.lam[i] > K.s[i] && !faint);
                        if (i < km && ((base && !((dm >> i) & 1)) || ((am >> i) & 1))) {
                            if (pc == 0) pi1 = i;
                            else if (pc == 1) pi2 = i;
                            ++pc;
                            cm |= 1 << i;
                        }
                    }
                    if (pc > 2) pc = vertex_pair(L.A2, reinterpret_cast<const double*>(L.BI), 2, N, kx, km, cm, P.tol_p, pi1, pi2);
                    okp = pc <= 2;
                    pk = (pc < 3 ? pc : 2) | (pi1 << 2) | (pi2 << 6);
                    const double b2 = K.be * K.be;
                    if (pc == 0) {
                        E00 = b2 / P.Rw0;
                        E11 = b2 / P.Rw1;
                    } else if (pc == 1) {
                        const double2 a = L.A2[pi1 * N + kx];
                        const double aa = FD2(a.x, a.x, a.y, a.y);
                        const double t = (FD2(a.x, sr0, a.y, sr1) - L.BI[pi1 * N + kx].x) / aa;
                        K.r0 = fma(-t, a.x, sr0);
                        K.r1 = fma(-t, a.y, sr1);
                        const double u = a.y * a.y, v = a.x * a.x, q = a.x * a.y;
                        const double ie = b2 / FD2(P.Rw0, u, P.Rw1, v);
                        E00 = u * ie;
                        E01 = -(q * ie);
                        E11 = v * ie;
                    } else {
                        const double2 a = L.A2[pi1 * N + kx];
                        const double2 e = L.A2[pi2 * N + kx];
                        const double ba = L.BI[pi1 * N + kx].x, be = L.BI[pi2 * N + kx].x;
                        const double det = fma(a.x, e.y, -(a.y * e.x));
                        const double aa = FD2(a.x, a.x, a.y, a.y), ee = FD2(e.x, e.x, e.y, e.y);
                        if (!(det * det > 1e-18 * (aa * ee))) okp = false;
                        const double idet = 1.0 / det;
                        K.r0 = fma(ba, e.y, -(a.y * be)) * idet;
                        K.r1 = fma(a.x, be, -(ba * e.x)) * idet;
                    }
                    double pd, cd;
                    residuals(K, false, P, last, L.A2, L.BI, N, k, mmax, xk0, xk1, rref, xref, pd, cd);
                }
                STAMP_ADD(13, t_p);
                STAMP(t_pr);
                okp = riccati<NW>(K, P, E00, E01, E11, bnd, N, nwa, k, wv, lane, own) && okp;
                STAMP_ADD(14, t_pr);
                pk = opaque(pk);
                pc = pk & 3;
                pi1 = (pk >> 2) & 15;
                pi2 = (pk >> 6) & 15;
                if (own) {
                    const double b2 = K.be * K.be;
                    const double B00 = fma(b2, K.P00, P.Rw0);
                    const double B01 = b2 * K.P01;
                    const double B11 = fma(b2, K.P11, P.Rw1);
                    if (pc == 0) {
                        const double det = fma(B00, B11, -(B01 * B01));
                        if (!(det > 0.0) || __builtin_isinf(det)) okp = false;
                        const double idet = 1.0 / det;
                        K.h00 = B11 * idet;
                        K.h01 = -(B01 * idet);
                        K.h11 = B00 * idet;
                    } else if (pc == 1) {
                        const double2 a = L.A2[pi1 * N + opaque(k)];
                        const double u = a.y * a.y, v = a.x * a.x, q = a.x * a.y;
                        const double tbt = FD3(B00, u, B11, v, -2.0 * (B01 * q));
                        if (!(tbt > 0.0) || __builtin_isinf(tbt)) okp = false;
                        const double itb = 1.0 / tbt;
                        K.h00 = u * itb;
                        K.h01 = -(q * itb);
                        K.h11 = v * itb;
                    } else {
                        K.h00 = 0.0;
                        K.h01 = 0.0;
                        K.h11 = 0.0;
                    }
                }
                double pl1 = 0.0, pl2 = 0.0;
                double vmx = 0.0;   // this knot's largest violation (the IPM polish's add threshold)
                {
                    // the Newton step; then the certificate: costates of the new point from the
                    // solve, nu_k = P_{k+1} dxi_{k+1} + (qx_k + v_{k+1}) (oracle dcm_polish step 6)
                    double dr0, dr1, dx0, dx1, vn0, vn1, dxk0, dxk1;
                    STAMP(t_ps);
                    solve<NW>(K, K.rh0, K.rh1, bnd, nwa, wv, lane, own, dr0, dr1, dx0, dx1, vn0, vn1,
                              dxk0, dxk1);
                    STAMP_ADD(15, t_ps);
                    // K.rh and K.d are free after the solve: the refinement's nu_k (below) and the step
                    // of xi_{64 wv} (lane 0: the refinement's xi_k)
                    K.d0 = dxk0;
                    K.d1 = dxk1;
                    if (own) {
                        K.r0 = K.r0 + dr0;
                        K.r1 = K.r1 + dr1;
                        K.x0 = K.x0 + dx0;
                        K.x1 = K.x1 + dx1;
                        const int kx = opaque(k);
                        if (pc == 1) project_line(K, L.A2[pi1 * N + kx], L.BI[pi1 * N + kx].x);
                        const double s0 = K.qx0 + vn0;
                        const double s1 = K.qx1 + vn1;
                        const double nu0 = FD3(K.P00, dx0, K.P01, dx1, s0);
                        const double nu1 = FD3(K.P01, dx0, K.P11, dx1, s1);
                        K.rh0 = nu0;
                        K.rh1 = nu1;
                        const double rh0 = P.Rw0 * (K.r0 - rref[0]);
                        const double rh1 = P.Rw1 * (K.r1 - rref[1]);
                        const double g0 = fma(K.be, nu0, -rh0);
                        const double g1 = fma(K.be, nu1, -rh1);
                        // the dual tolerance relative to |beta nu| beyond 1 / kTolDualRel
                        const double tol_d =
                            P.tol_d * fmax(1.0, kTolDualRel * fmax(fabs(K.be * nu0), fabs(K.be * nu1)));
                        if (pc == 0) {
                            if (!(fabs(g0) <= tol_d) || !(fabs(g1) <= tol_d)) okp = false;
                        } else if (pc == 1) {
                            const double2 a = L.A2[pi1 * N + kx];
                            pl1 = FD2(a.x, g0, a.y, g1) / FD2(a.x, a.x, a.y, a.y);
                            if (!(pl1 >= -tol_d)) {
                                okp = false;
                                neg = true;
                                drop |= 1 << pi1;
                                add &= ~(1 << pi1);
                            }
                            if (!(fabs(fma(-pl1, a.x, g0)) <= tol_d) || !(fabs(fma(-pl1, a.y, g1)) <= tol_d))
                                okp = false;
                        } else {
                            const double2 a = L.A2[pi1 * N + kx];
                            const double2 e = L.A2[pi2 * N + kx];
                            const double idet = 1.0 / fma(a.x, e.y, -(a.y * e.x));
                            pl1 = fma(g0, e.y, -(e.x * g1)) * idet;
                            pl2 = fma(a.x, g1, -(g0 * a.y)) * idet;
                            if (!(pl1 >= -tol_d)) {
                                okp = false;
                                neg = true;
                                drop |= 1 << pi1;
                                add &= ~(1 << pi1);
                            }
                            if (!(pl2 >= -tol_d)) {
                                okp = false;
                                neg = true;
                                drop |= 1 << pi2;
                                add &= ~(1 << pi2);
                            }
                        }
                        // primal feasibility of every facet: the rows are read four at a time
                        // (all lanes, clamped to the staged slots) so the LDS reads overlap
                        const int km = opaque(K.m), mm = opaque_s(mmax);
                        int vm = 0;
#pragma unroll
                        for (int i0 = 0; i0 < MF; i0 += 4) {
                            if (i0 >= mm) break;
                            double2 av[4];
                            double bv[4];
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                const int i = i0 + j < mm ? i0 + j : 0;
                                av[j] = L.A2[i * N + kx];
                                bv[j] = L.BI[i * N + kx].x;
                            }
#pragma unroll
                            for (int j = 0; j < 4; ++j) {
                                const double vi = FD2(av[j].x, K.r0, av[j].y, K.r1) - bv[j];
                                if (!(vi <= P.tol_p) && i0 + j < km) {
                                    vm |= 1 << (i0 + j);
                                    vmx = nanmax(vmx, vi);
                                }
                            }
                        }
                        vm &= (1 << (km < mm ? km : mm)) - 1;
                        if (vm) {
                            okp = false;
                            viol = true;
                            if (guess) {
                                add |= vm;
                                drop &= ~vm;
                            }
                        }
                    }
                }
                const int fl = R.template or_bits<4>((okp ? 0 : 1) | (neg || viol ? 2 : 0) |
                                                     (neg ? 4 : 0) | (viol ? 8 : 0));
                const bool rejected = (fl & 1) != 0;
                if (!guess && (fl & 8) != 0) {
                    // the IPM polish adds only the facets violated by >= kAddRel x the pass's
                    // largest violation (oracle dcm_polish)
                    const double thr = kAddRel * R.nanmax_(vmx);
                    if (own) {
                        const int kx = opaque(k);
                        const int km = opaque(K.m), mm = opaque_s(mmax);
#pragma unroll
                        for (int i = 0; i < MF; ++i) {
                            if (MF <= kMaxFacets && i >= mm) break;   // 16 slots: no early exit, so the loop unrolls fully
                            if (i < km) {
                                const double2 a = L.A2[i * N + kx];
                                const double vi = FD2(a.x, K.r0, a.y, K.r1) - L.BI[i * N + kx].x;
                                if (vi > P.tol_p && vi >= thr) {
                                    add |= 1 << i;
                                    drop &= ~(1 << i);
                                }
                            }
                        }
                    }
                }
                STAMP_ADD(8, t_p);
#ifdef BLF_STAMPS
                if (blockIdx.x < 64 && threadIdx.x == 0) atomicAdd(&g_blf_stamps[9], 1ull);
#endif
                if (!rejected) {
                    if (LAMOUT && own) {   // the optimum's multipliers: active facets, 0 elsewhere
                        pl1 = pl1 > 0.0 ? pl1 : 0.0;
                        pl2 = pl2 > 0.0 ? pl2 : 0.0;
#pragma unroll
                        for (int i = 0; i < MF; ++i)
                            K.lam[i] = (pc >= 1 && i == pi1) ? pl1 : (pc == 2 && i == pi2) ? pl2 : 0.0;
                    }
                    // the refinement where the largest multiplier exceeds kRefineLam (oracle
                    // dcm_polish, refine_rhs): the certificate's costates, the same factorization
                    const double lq = R.keepmax(own ? keepmax(keepmax(0.0, pl1), pl2) : 0.0);
                    if (lq > kRefineLam) {
                        // xi_{64 wv} after the polish step (the previous wavefront's last lane did the same)
                        double xr0 = wv > 0 ? xb0 + K.d0 : xb0, xr1 = wv > 0 ? xb1 + K.d1 : xb1;
                        for (int rs = 0; rs < kRefineSteps; ++rs) {
                            const double nu0 = K.rh0, nu1 = K.rh1;
                            double xk0r, xk1r;
                            xi_prev(K, lane, xr0, xr1, xk0r, xk1r);
                            // the next knot's costate and omega: the next lane's, across a wavefront from LDS
                            if (lane == 0 && wv > 0) {
                                bnd[kBnd * wv + kBN] = nu0;
                                bnd[kBnd * wv + kBN + 1] = nu1;
                                bnd[kBnd * wv + kBN + 2] = K.w;
                            }
                            if constexpr (NW > 1) __syncthreads();
                            double nn0 = dpp1<kNextWrap>(nu0), nn1 = dpp1<kNextWrap>(nu1), wn = dpp1<kNextWrap>(K.w);
                            if (NW > 1 && lane == kWave - 1 && wv < nwa - 1) {
                                nn0 = bnd[kBnd * (wv + 1) + kBN];
                                nn1 = bnd[kBnd * (wv + 1) + kBN + 1];
                                wn = bnd[kBnd * (wv + 1) + kBN + 2];
                            }
                            double g0 = 0.0, g1 = 0.0;
                            if (own) {
                                const double2 a = L.A2[pi1 * N + opaque(k)];
                                refine_rhs(xk0r, xk1r, K.x0, K.x1, K.r0, K.r1, rref[0], rref[1], xref[0], xref[1], K.w,
                                           wn, nu0, nu1, nn0, nn1, last, P.dt, last ? P.Pw0 : P.Qw0,
                                           last ? P.Pw1 : P.Qw1, P.Rw0, P.Rw1, pc, a.x, a.y, K.d0, K.d1, K.qx0,
                                           K.qx1, g0, g1);
                            }
                            double dr0, dr1, dx0, dx1, vn0, vn1, ek0, ek1;
                            solve<NW>(K, g0, g1, bnd, nwa, wv, lane, own, dr0, dr1, dx0, dx1, vn0, vn1, ek0, ek1);
                            if (own) {
                                // the refined point's costates: nu + the step's own (Lagrangian-shifted) costate
                                K.rh0 = nu0 + FD3(K.P00, dx0, K.P01, dx1, K.qx0 + vn0);
                                K.rh1 = nu1 + FD3(K.P01, dx0, K.P11, dx1, K.qx1 + vn1);
                                K.r0 = K.r0 + dr0;
                                K.r1 = K.r1 + dr1;
                                K.x0 = K.x0 + dx0;
                                K.x1 = K.x1 + dx1;
                                if (pc == 1) project_line(K, L.A2[pi1 * N + opaque(k)], L.BI[pi1 * N + opaque(k)].x);
                            }
                            if (wv > 0) {   // the same update as the previous wavefront's last lane
                                xr0 = xr0 + ek0;
                                xr1 = xr1 + ek1;
                            }
                            if constexpr (NW > 1) __syncthreads();   // bnd's kBN slots are rewritten next step
                        }
                    }
                    polished = 1;
                    break;   // solved: the certified optimum
                }
                K.r0 = sr0;
                K.r1 = sr1;
                K.x0 = sx0;
                K.x1 = sx1;
                const bool more = pass + 1 < kGuessPasses && (fl & 2) != 0;
                if (more) {
                    // every further pass starts from the same iterate without the facets whose
                    // multiplier came out negative and with the violated ones (the IPM polish: those
                    // violated by >= kAddRel x the largest), up to kGuessPasses.  Each runs this
                    // block again from the top of the loop (one copy of the polish code) and does
                    // not count as an IPM iteration.
                    ++pass;
                    --it;
                    continue;
                }
                pass = 0;
                drop = 0;
                add = 0;
                // the iterate's gradient and defects again (the polish reused them); the wavefront
                // boundary values were not touched, so xi_k comes back without a barrier
                xi_prev(K, lane, xb0, xb1, xk0, xk1);
                if (own) {
                    double pd, cd;
                    residuals(K, true, P, last, L.A2, L.BI, N, k, mmax, xk0, xk1, rref, xref, pd, cd);
                }
                if (guess) {   // the active-set start failed: the IPM takes over from the top,
                    guess = false;   // from the saturated LQ start
                    sat_pending = true;
                    --it;
                    continue;
                }
            }
            if (mu <= P.tol_mu && pres <= P.tol_p && dres <= P.tol_d) break;   // solved
            if (it >= P.max_iter) {
                status = BLF_QP_MAX_ITER;
                break;
            }

            // ---- W-phase: 1/s, W = A^T diag(lam/s) A, det W, predictor rhs ----
            STAMP(t_w);
            double W00 = 0.0, W01 = 0.0, W11 = 0.0, dW = 0.0;
            double g0 = K.rh0, g1 = K.rh1;
            if (own) {
                const int kx = opaque(k);
                const int km = opaque(K.m), mm = opaque_s(mmax);
#pragma unroll
                for (int i = 0; i < MF; ++i) {
                    if (MF <= kMaxFacets && i >= mm) break;   // 16 slots: no early exit, so the loop unrolls fully
                    if (i < km) {
                        const double2 a = L.A2[i * N + kx];
                        const double is = 1.0 / K.s[i];
                        L.BI[i * N + kx].y = is;
                        const double sg = K.lam[i] * is;
                        const double t0 = sg * a.x;
                        const double t1 = sg * a.y;
                        W00 = fma(t0, a.x, W00);
                        W01 = fma(t0, a.y, W01);
                        W11 = fma(t1, a.y, W11);
                        const double rpi = facet_rp(K, a, L.BI[i * N + kx].x, i);
                        const double e = fma(K.lam[i], rpi, -(K.s[i] * K.lam[i])) * is;
                        g0 = fma(a.x, e, g0);
                        g1 = fma(a.y, e, g1);
                    }
                }
                // sg_i = lam_i / s_i is recomputed from the stored 1/s (bit-identical) rather than
                // kept in an 8-entry register array across the pair loop (which spilled)
#pragma unroll
                for (int i = 1; i < MF; ++i) {
                    if (MF <= kMaxFacets && i >= mm) break;   // 16 slots: no early exit, so the loop unrolls fully
                    if (i < km) {
                        const int ki = opaque(k);
                        const double2 ai = L.A2[i * N + ki];
                        const double sgi = K.lam[i] * L.BI[i * N + ki].y;
#pragma unroll
                        for (int j = 0; j < i; ++j) {
                            const double2 aj = L.A2[j * N + ki];
                            const double sgj = K.lam[j] * L.BI[j * N + ki].y;
                            const double cr = fma(ai.x, aj.y, -(ai.y * aj.x));
                            dW = fma(sgi * sgj, cr * cr, dW);
                        }
                    }
                }
            }
            STAMP_ADD(5, t_w);
            STAMP(t_f);
            ok = factor<NW>(K, P, W00, W01, W11, dW, bnd, N, nwa, k, wv, lane, own);
            STAMP_ADD(1, t_f);

            // ---- predictor ----
            STAMP(t_s);
            double dra0, dra1, dx0, dx1, vn0, vn1, dxk0, dxk1;
            solve<NW>(K, g0, g1, bnd, nwa, wv, lane, own, dra0, dra1, dx0, dx1, vn0, vn1, dxk0, dxk1);
            STAMP_ADD(6, t_s);
            // affine ratio test with U0 = sum s lam and U2 = sum ds dl in the same exchange:
            // mu_aff = ((1 - a) U0 + a^2 U2) / ntot; a failed factorization votes through U0 = NaN
            double q = 0.0, u0 = 0.0, u2 = 0.0;
            if (own) {
                const int kx = opaque(k);
                const int km = opaque(K.m), mm = opaque_s(mmax);
#pragma unroll
                for (int i = 0; i < MF; ++i) {
                    if (MF <= kMaxFacets && i >= mm) break;   // 16 slots: no early exit, so the loop unrolls fully
                    if (i < km) {
                        double ds, dl;
                        const double is = L.BI[i * N + kx].y;
                        affine_step(K, L.A2[i * N + kx], L.BI[i * N + kx].x, is, i, dra0, dra1, ds, dl);
                        if (ds < 0.0) q = keepmax(q, (-ds) * is);
                        if (dl < 0.0) q = keepmax(q, (K.s[i] + ds) * is);
                        u0 = fma(K.s[i], K.lam[i], u0);
                        u2 = fma(ds, dl, u2);
                    }
                }
            }
            if (!ok) u0 = __builtin_nan("");
            R.template max_sums<2>(q, u0, u2);
            if (!(u0 == u0) || !(u2 == u2)) {
                status = BLF_QP_NUMERICAL;
                break;
            }
            const double a_aff = q > 1.0 ? 1.0 / q : 1.0;
            const double mu_aff = ntot > 0 ? fma(a_aff * a_aff, u2, (1.0 - a_aff) * u0) / (double)ntot : 0.0;
            double sigma = 0.0;
            if (mu > 0.0) {
                const double qq = mu_aff / mu;
                sigma = (qq * qq) * qq;
            }
            const double sigma_mu = sigma * mu;

            // ---- corrector ----
            g0 = K.rh0;
            g1 = K.rh1;
            if (own) {
                const int kx = opaque(k);
                const int km = opaque(K.m), mm = opaque_s(mmax);
#pragma unroll
                for (int i = 0; i < MF; ++i) {
                    if (MF <= kMaxFacets && i >= mm) break;   // 16 slots: no early exit, so the loop unrolls fully
                    if (i < km) {
                        const double2 a = L.A2[i * N + kx];
                        const double bi = L.BI[i * N + kx].x;
                        const double is = L.BI[i * N + kx].y;
                        double ds, dl;
                        affine_step(K, a, bi, is, i, dra0, dra1, ds, dl);
                        const double rc = FD2(K.s[i], K.lam[i], ds, dl) - sigma_mu;
                        const double rpi = facet_rp(K, a, bi, i);
                        const double e = fma(K.lam[i], rpi, -rc) * is;
                        g0 = fma(a.x, e, g0);
                        g1 = fma(a.y, e, g1);
                    }
                }
            }
            double dr0, dr1;
            solve<NW>(K, g0, g1, bnd, nwa, wv, lane, own, dr0, dr1, dx0, dx1, vn0, vn1, dxk0, dxk1);
            STAMP_ADD(2, t_s);
            STAMP(t_c);
            q = 0.0;
            double t2 = 0.0;
            if (own) {
                const int kx = opaque(k);
                const int km = opaque(K.m), mm = opaque_s(mmax);
#pragma unroll
                for (int i = 0; i < MF; ++i) {
                    if (MF <= kMaxFacets && i >= mm) break;   // 16 slots: no early exit, so the loop unrolls fully
                    if (i < km) {
                        const double2 a = L.A2[i * N + kx];
                        const double bi = L.BI[i * N + kx].x;
                        const double is = L.BI[i * N + kx].y;
                        double ads, adl;
                        affine_step(K, a, bi, is, i, dra0, dra1, ads, adl);
                        const double rc = FD2(K.s[i], K.lam[i], ads, adl) - sigma_mu;
                        const double rpi = facet_rp(K, a, bi, i);
                        const double ds = (-rpi) - FD2(a.x, dr0, a.y, dr1);
                        const double dl = fma(-K.lam[i], ds, -rc) * is;
                        if (ds < 0.0) q = keepmax(q, (-ds) * is);
                        if (dl < 0.0) q = keepmax(q, (-dl) / K.lam[i]);
                        L.BI[i * N + kx].y = dl;   // 1/s is dead now: keep the multiplier step
                        t2 = fma(ds, dl, t2);
                    }
                }
            }
            R.template max_sums<1>(q, t2, t2);
            const double step = q > 0.0 ? 0.99 / q : 1.0;
            const double a = step < 1.0 ? step : 1.0;
            if (own) {
                const int kx = opaque(k);
                const int km = opaque(K.m), mm = opaque_s(mmax);
#pragma unroll
                for (int i = 0; i < MF; ++i) {
                    if (MF <= kMaxFacets && i >= mm) break;   // 16 slots: no early exit, so the loop unrolls fully
                    if (i < km) {
                        const double2 fa = L.A2[i * N + kx];
                        const double ds = (-facet_rp(K, fa, L.BI[i * N + kx].x, i)) - FD2(fa.x, dr0, fa.y, dr1);
                        K.s[i] = fma(a, ds, K.s[i]);
                        K.lam[i] = fma(a, L.BI[i * N + kx].y, K.lam[i]);
                    }
                }
                K.r0 = fma(a, dr0, K.r0);   // after the facet steps, which use the old r
                K.r1 = fma(a, dr1, K.r1);
                K.x0 = fma(a, dx0, K.x0);
                K.x1 = fma(a, dx1, K.x1);
            }
            if (wv > 0) {   // the same update as the previous wavefront's last lane
                xb0 = fma(a, dxk0, xb0);
                xb1 = fma(a, dxk1, xb1);
            }
            dres = dres * (1.0 - a);
            pres = pres * (1.0 - a);
            last_a = a;
            // sum (s + a ds)(lam + a dl) = U0 + a T1 + a^2 T2, T1 = -sum rc = -(U0 + U2 - ntot sigma mu)
            if (ntot > 0) {
                const double nt = (double)ntot;
                mu = fma(a * a, t2, fma(a, fma(nt, sigma_mu, -u2), (1.0 - a) * u0)) / nt;
            }
            STAMP_ADD(7, t_c);
        }
    }

    // ---- outputs ----
    if (own) {
        const int64_t st = p * N + k;
        vrp_out[2 * st] = K.r0;
        vrp_out[2 * st + 1] = K.r1;
        const int64_t sx = p * (N + 1) + (k + 1);
        xi_out[2 * sx] = K.x0;
        xi_out[2 * sx + 1] = K.x1;
        if (LAMOUT) {
            double* lo = lam_out + st * M;
#pragma unroll
            for (int i = 0; i < MF; ++i) {
                if constexpr (MF <= kMaxFacets) {
                    if (i >= M) break;
                } else {
                    if (i >= M) continue;
                }
                lo[i] = i < K.m ? K.lam[i] : 0.0;
            }
        }
    }
    if (k == 0) {
        xi_out[2 * p * (N + 1)] = xi00;
        xi_out[2 * p * (N + 1) + 1] = xi01;
        status_out[p] = status;
        iters_out[p] = it;
        if (polished_out) polished_out[p] = polished;
        STAMP_ADD(0, t_start);
#ifdef BLF_STAMPS
        if (blockIdx.x < 64) atomicAdd(&g_blf_stamps[3], (unsigned long long)it);
#endif
    }
}
}  // namespace
}  // namespace blf
