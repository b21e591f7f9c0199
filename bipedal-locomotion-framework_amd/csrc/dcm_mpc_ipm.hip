// dcm_mpc_ipm.hip — batched time-varying DCM MPC QP (TimeVaryingDCMPlanner).
//
// One workgroup per QP, one thread per knot ("stage") k < N, NT = 64*ceil(N/64) threads.
// Stage-parallel work (residuals, barrier Hessian R'_k = R + A_k^T diag(lam/s) A_k, Newton
// right-hand sides, per-facet step / update) runs on all lanes with the stage's facets held in
// registers; the Riccati recursion over the knots (backward factor/solve, forward rollout of the
// Newton step) is inherently sequential and runs on thread 0 out of LDS.  Reductions (mean
// complementarity, max residual, step length) are xor-butterflies over each wavefront plus an
// ordered sum over waves — the exact order the oracle's orc_wave_tree_sum restates.
//
// Every arithmetic expression mirrors oracle/blf_oracle.c:orc_dcm_mpc_solve term for term and
// the file is built with -ffp-contract=off, so device and oracle iterates agree bit for bit
// (verified by tests/test_gpu_dcm_mpc.py).  DESIGN.md section 4 is the algorithm statement.
#include "blf_internal.h"

namespace blf {
namespace {

#ifdef BLF_STAMPS
// Diagnostic build only (make stamps): per-phase cycle sums of thread 0 for the first 64 QPs.
// [0] whole kernel, [1] factor sweep + forward, [2] solve sweep + forward, [3] iterations.
__device__ unsigned long long g_blf_stamps[8];
#define STAMP(t) unsigned long long t = __builtin_amdgcn_s_memtime()
#define STAMP_ADD(slot, t0) \
    do { if (blockIdx.x < 64) atomicAdd(&g_blf_stamps[slot], __builtin_amdgcn_s_memtime() - (t0)); } while (0)
#else
#define STAMP(t)
#define STAMP_ADD(slot, t0)
#endif

struct KParams {
    int N, M, max_iter;
    double dt, Qw0, Qw1, Rw0, Rw1, Pw0, Pw1, tol_mu, tol_p, tol_d;
};

// LDS carve-up (in doubles), sized by N.  The same code computes the launch size on the host
// (Lds(nullptr, ...).total), so the allocation always covers every array.
//
// Everything the Riccati sweeps exchange with the knot threads lives in one 144-byte record per
// knot, so a sweep step addresses one base pointer and moves its data with ds_read_b128 /
// ds_write_b128 at immediate offsets.  144 B = 36 dwords: the knot threads' 16-byte accesses
// to their own records are bank-conflict free (36 k mod 32 = 4 k).
//   R[k]: 0-3 W00 W01 W11 detW | 4-5 g (rhs; the forward sweep overwrites it with dr)
//         6-7 d (Euler defect) | 8-9 Q (xi_k - xi_ref_k) | 10 alpha 11 beta 12 alpha^2 13 beta^2
//         14-15 kff | 16 omega | 17 pad
//   H[k]: 0-2 H_k^{-1} (00 01 11) | 3-5 P_{k+1} (00 01 11) | 6-7 pad
constexpr int kRec = 18;
constexpr int kHrec = 8;
struct Lds {
    double *R, *H, *xi, *dxi, *red;
    size_t total;   // doubles
    __host__ __device__ Lds(double* base, int N, int NW)
    {
        size_t o = 0;
        auto take = [&](size_t n) {
            double* p = base ? base + o : nullptr;
            o += (n + 1) & ~size_t(1);   // keep every array 16-byte aligned
            return p;
        };
        R = take((size_t)kRec * N);
        H = take((size_t)kHrec * N);
        xi = take(2 * (N + 1));   // [N+1][2]
        dxi = take(2 * (N + 1));  // [N+1][2] (also the costates nu at start-up)
        red = take(4 * NW + 8);   // [NW] reduction scratch + flags
        total = o;
    }
    __device__ double* rec(int k) const { return R + (size_t)kRec * k; }
    __device__ double& W(int k, int j) const { return R[kRec * k + j]; }
    __device__ double& g(int k, int j) const { return R[kRec * k + 4 + j]; }
    __device__ double& dr(int k, int j) const { return R[kRec * k + 4 + j]; }
    __device__ double& d(int k, int j) const { return R[kRec * k + 6 + j]; }
    __device__ double& qx(int k, int j) const { return R[kRec * k + 8 + j]; }
    __device__ double& al(int k) const { return R[kRec * k + 10]; }
    __device__ double& be(int k) const { return R[kRec * k + 11]; }
    __device__ double& a2(int k) const { return R[kRec * k + 12]; }
    __device__ double& b2(int k) const { return R[kRec * k + 13]; }
    __device__ double& kff(int k, int j) const { return R[kRec * k + 14 + j]; }
    __device__ double& om(int k) const { return R[kRec * k + 16]; }
    __device__ double& Hi(int k, int j) const { return H[kHrec * k + j]; }
    __device__ double& Pn(int k, int j) const { return H[kHrec * k + 3 + j]; }
};

inline size_t lds_doubles(int N, int NW) { return Lds(nullptr, N, NW).total; }

template <int NW>
__device__ __forceinline__ double block_sum(double v, double* red)
{
    v = wave_sum(v);
    if constexpr (NW == 1) return v;
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double t = red[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) t = t + red[i];
    __syncthreads();
    return t;
}
template <int NW>
__device__ __forceinline__ double block_nanmax(double v, double* red)
{
    v = wave_nanmax(v);
    if constexpr (NW == 1) return v;
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double t = red[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) t = nanmax(t, red[i]);
    __syncthreads();
    return t;
}
template <int NW>
__device__ __forceinline__ double block_keepmin(double v, double* red)
{
    v = wave_keepmin(v);
    if constexpr (NW == 1) return v;
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    double t = red[0];
#pragma unroll
    for (int i = 1; i < NW; ++i) t = keepmin(t, red[i]);
    __syncthreads();
    return t;
}

// Backward Riccati sweep (thread 0) = oracle dcm_backward.  FACTOR: builds H_k^{-1} and
// P_{k+1} (returns false if some H_k is not positive definite); otherwise reuses them.
template <bool FACTOR>
__device__ bool backward_sweep(const Lds& L, const KParams& k, double pv0, double pv1)
{
    bool ok = true;
    double P00 = k.Pw0, P01 = 0.0, P11 = k.Pw1;
    for (int s = k.N - 1; s >= 0; --s) {
        const double2* rc = reinterpret_cast<const double2*>(L.rec(s));
        double2* hr = reinterpret_cast<double2*>(L.H + (size_t)kHrec * s);
        const double2 gg = rc[2], dd = rc[3], qq = rc[4], ab = rc[5], sq = rc[6];
        const double be = ab.y, al = ab.x, a2 = sq.x, b2 = sq.y;
        double h00, h01, h11;
        if (FACTOR) {
            const double2 w0 = rc[0], w1 = rc[1];
            // H = B + W, B = R + b2 P_{k+1}: det H = det B + tr(adj(B) W) + det W (all >= 0)
            const double B00 = k.Rw0 + b2 * P00;
            const double B01 = b2 * P01;
            const double B11 = k.Rw1 + b2 * P11;
            const double H00 = B00 + w0.x;
            const double H01 = B01 + w0.y;
            const double H11 = B11 + w1.x;
            const double detB = B00 * B11 - B01 * B01;
            const double trW = (B11 * w0.x + B00 * w1.x) - 2.0 * (B01 * w0.y);
            const double det = (detB + trW) + w1.y;
            if (!(det > 0.0) || __builtin_isinf(det)) ok = false;
            const double idet = 1.0 / det;
            h00 = H11 * idet;
            h01 = -(H01 * idet);
            h11 = H00 * idet;
            hr[0] = make_double2(h00, h01);
            hr[1] = make_double2(h11, P00);
            hr[2] = make_double2(P01, P11);
        } else {
            const double2 x0 = hr[0], x1 = hr[1], x2 = hr[2];
            h00 = x0.x; h01 = x0.y; h11 = x1.x;
            P00 = x1.y; P01 = x2.x; P11 = x2.y;
        }
        const double t0 = (P00 * dd.x + P01 * dd.y) + pv0;
        const double t1 = (P01 * dd.x + P11 * dd.y) + pv1;
        const double hu0 = gg.x - be * t0;
        const double hu1 = gg.y - be * t1;
        const double k0 = -(h00 * hu0 + h01 * hu1);
        const double k1 = -(h01 * hu0 + h11 * hu1);
        reinterpret_cast<double2*>(L.rec(s))[7] = make_double2(k0, k1);
        if (s > 0) {
            const double pk0 = P00 * k0 + P01 * k1;
            const double pk1 = P01 * k0 + P11 * k1;
            const double npv0 = qq.x + al * (t0 - be * pk0);
            const double npv1 = qq.y + al * (t1 - be * pk1);
            if (FACTOR) {
                // P_k = Q + a^2 (P - b^2 P H^-1 P)
                const double M00 = P00 * h00 + P01 * h01;
                const double M01 = P00 * h01 + P01 * h11;
                const double M10 = P01 * h00 + P11 * h01;
                const double M11 = P01 * h01 + P11 * h11;
                const double S00 = M00 * P00 + M01 * P01;
                const double S01 = M00 * P01 + M01 * P11;
                const double S10 = M10 * P00 + M11 * P01;
                const double S11 = M10 * P01 + M11 * P11;
                const double n00 = k.Qw0 + a2 * (P00 - b2 * S00);
                const double n11 = k.Qw1 + a2 * (P11 - b2 * S11);
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

// Forward sweep (thread 0) = oracle dcm_forward.  dr_k overwrites g_k in the knot record.
__device__ void forward_sweep(const Lds& L, int N)
{
    double x0 = 0.0, x1 = 0.0;
    double2* dxi = reinterpret_cast<double2*>(L.dxi);
    dxi[0] = make_double2(0.0, 0.0);
    for (int s = 0; s < N; ++s) {
        double2* rc = reinterpret_cast<double2*>(L.rec(s));
        const double2* hr = reinterpret_cast<const double2*>(L.H + (size_t)kHrec * s);
        const double2 h0 = hr[0], h1 = hr[1], h2 = hr[2];
        const double2 dd = rc[3], ab = rc[5], kf = rc[7];
        const double u0 = h1.y * x0 + h2.x * x1;
        const double u1 = h2.x * x0 + h2.y * x1;
        const double v0 = h0.x * u0 + h0.y * u1;
        const double v1 = h0.y * u0 + h1.x * u1;
        const double al = ab.x, be = ab.y;
        const double abp = al * be;
        const double r0 = abp * v0 + kf.x;
        const double r1 = abp * v1 + kf.y;
        rc[2] = make_double2(r0, r1);
        const double n0 = (al * x0 - be * r0) + dd.x;
        const double n1 = (al * x1 - be * r1) + dd.y;
        dxi[s + 1] = make_double2(n0, n1);
        x0 = n0;
        x1 = n1;
    }
}

// The knot a thread owns: slacks, multipliers, residual scratch and the knot's VRP in registers.
struct Stage {
    double s[kMaxFacets], lam[kMaxFacets];
    int m;
    double r0, r1, rr0, rr1, xr0, xr1, w, be;
    double dra0, dra1;  // the affine (predictor) VRP step of this knot
    const double* Ak;   // this knot's facet rows A_k [M][2] and offsets b_k [M] (global memory)
    const double* bk;
};

// The facet rows are constant for the whole solve.  They are re-read (L2-resident) at the start
// of every stage-parallel phase instead of being held in VGPRs across the IPM loop: that keeps the
// stage threads' register footprint small enough for the software-pipelined Riccati sweeps to
// run at two waves per SIMD.  The empty asm launders the pointers so LICM cannot hoist the loads
// back out of the iteration loop.
struct Rows {
    double a0[kMaxFacets], a1[kMaxFacets], h[kMaxFacets];
};

__device__ __forceinline__ void load_rows(const Stage& S, Rows& F)
{
    const double* Ak = S.Ak;
    const double* bk = S.bk;
    asm volatile("" : "+v"(Ak), "+v"(bk));
#pragma unroll
    for (int i = 0; i < kMaxFacets; ++i) {
        if (i < S.m) {
            F.a0[i] = Ak[2 * i];
            F.a1[i] = Ak[2 * i + 1];
            F.h[i] = bk[i];
        } else {
            F.a0[i] = 0.0; F.a1[i] = 0.0; F.h[i] = 0.0;
        }
    }
}

// Per-facet quantities are recomputed from (r, s, lam, A, b) and the stored affine VRP step
// instead of being kept in registers across phases: the expressions are exactly the oracle's,
// so the recomputed values are bit-identical, and the knot threads stay at <= 168 VGPRs.
__device__ __forceinline__ double primal_res(const Stage& S, const Rows& F, int i)
{
    const double gr = F.a0[i] * S.r0 + F.a1[i] * S.r1;
    return (gr + S.s[i]) - F.h[i];
}

__device__ __forceinline__ void affine_step(const Stage& S, const Rows& F, int i, double& ds,
                                            double& dl)
{
    const double rc = S.s[i] * S.lam[i];
    ds = (-primal_res(S, F, i)) - (F.a0[i] * S.dra0 + F.a1[i] * S.dra1);
    dl = ((-rc) - S.lam[i] * ds) / S.s[i];
}

// Stage-parallel residual pass = the body of oracle dcm_residuals for one knot.  Writes the
// Euler defect and Q(xi_{k+1} - xi_ref_{k+1}) (or the terminal pv) to LDS; returns pres, ck,
// rho in registers.  mfac: the facet count to use (0 for the unconstrained warm start).
__device__ __forceinline__ void stage_residuals(Stage& S, int mfac, int k, int N, const KParams& P,
                                                const Lds& L, double* flag, double& pres,
                                                double& ck, double& rh0, double& rh1)
{
    rh0 = P.Rw0 * (S.r0 - S.rr0);
    rh1 = P.Rw1 * (S.r1 - S.rr1);
    Rows F;
    if (mfac > 0) load_rows(S, F);
#pragma unroll
    for (int i = 0; i < kMaxFacets; ++i) {
        if (i < mfac) {
            const double gr = F.a0[i] * S.r0 + F.a1[i] * S.r1;
            const double rpi = (gr + S.s[i]) - F.h[i];
            pres = nanmax(pres, fabs(rpi));
            ck = ck + S.s[i] * S.lam[i];
            rh0 = rh0 + F.a0[i] * S.lam[i];
            rh1 = rh1 + F.a1[i] * S.lam[i];
        }
    }
    const double x0 = L.xi[2 * k], x1 = L.xi[2 * k + 1];
    const double y0 = L.xi[2 * (k + 1)], y1 = L.xi[2 * (k + 1) + 1];
    const double dx0 = S.w * x0 + (-S.w) * S.r0;
    const double dk0 = (x0 + dx0 * P.dt) - y0;
    const double dx1 = S.w * x1 + (-S.w) * S.r1;
    const double dk1 = (x1 + dx1 * P.dt) - y1;
    L.d(k, 0) = dk0;
    L.d(k, 1) = dk1;
    pres = nanmax(pres, fabs(dk0));
    pres = nanmax(pres, fabs(dk1));
    if (k + 1 < N) {
        L.qx((k + 1), 0) = P.Qw0 * (y0 - S.xr0);
        L.qx((k + 1), 1) = P.Qw1 * (y1 - S.xr1);
    } else {
        flag[1] = P.Pw0 * (y0 - S.xr0);
        flag[2] = P.Pw1 * (y1 - S.xr1);
    }
}

template <int NT>
// 3 waves per SIMD (<= 168 VGPRs): with ~25 KB of LDS per QP that is 6 two-wave workgroups
// (6 QPs) per CU, and every SIMD keeps its own Riccati sweep streams in flight.
#ifndef BLF_MIN_WAVES
#define BLF_MIN_WAVES 3
#endif
__global__ __launch_bounds__(NT, (NT <= 256 ? BLF_MIN_WAVES : 1)) void dcm_mpc_ipm_kernel(
    KParams P, const double* __restrict__ xi_init, const double* __restrict__ omega,
    const double* __restrict__ xi_ref, const double* __restrict__ vrp_ref,
    const double* __restrict__ Ain, const double* __restrict__ bin,
    const int32_t* __restrict__ nfacets, double* __restrict__ xi_out,
    double* __restrict__ vrp_out, int32_t* __restrict__ status_out,
    int32_t* __restrict__ iters_out)
{
    constexpr int NW = NT / kWave;
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int N = P.N, M = P.M;
    Lds L(smem, N, NW);
    double* red = L.red;               // [NW] scratch for block reductions
    double* flag = L.red + 4 * NW;     // shared scalars: [0] factor failed, [1..2] terminal pv

    const int k = threadIdx.x;
    const bool own = k < N;
    const int64_t p = blockIdx.x;
    STAMP(t_start);

    // ---- load the knot this thread owns ----
    Stage S;
    S.m = 0;
    S.r0 = S.r1 = S.rr0 = S.rr1 = S.xr0 = S.xr1 = S.w = S.be = S.dra0 = S.dra1 = 0.0;
    S.Ak = Ain;
    S.bk = bin;
#pragma unroll
    for (int i = 0; i < kMaxFacets; ++i) {
        S.s[i] = 1.0; S.lam[i] = 0.0;
    }
    bool bad = false;
    if (own) {
        const int64_t st = p * N + k;
        S.m = nfacets[st];
        bad = (S.m < 0 || S.m > M);
        S.Ak = Ain + st * M * 2;
        S.bk = bin + st * M;
        S.w = omega[st];
        S.be = P.dt * S.w;
        const double al = 1.0 + S.be;
        L.al(k) = al;
        L.be(k) = S.be;
        L.a2(k) = al * al;
        L.b2(k) = S.be * S.be;
        L.om(k) = S.w;
        S.rr0 = vrp_ref[2 * st];
        S.rr1 = vrp_ref[2 * st + 1];
        S.r0 = S.rr0;
        S.r1 = S.rr1;
        L.dr(k, 0) = S.rr0;      // scratch: initial VRP for the rollout below
        L.dr(k, 1) = S.rr1;
        const int64_t sx = p * (N + 1) + (k + 1);
        S.xr0 = xi_ref[2 * sx];
        S.xr1 = xi_ref[2 * sx + 1];
    }
    if (k == 0) {
        L.xi[0] = xi_init[2 * p];
        L.xi[1] = xi_init[2 * p + 1];
    }
    const bool any_bad = __syncthreads_or(bad);

    // ---- initial state 1: reference Euler rollout of vrp_ref (thread 0) ----
    if (k == 0) {
        for (int q = 0; q < N; ++q) {
            const double wq = L.om(q);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const double x = L.xi[2 * q + j];
                const double dx = wq * x + (-wq) * L.dr(q, j);
                L.xi[2 * (q + 1) + j] = x + dx * P.dt;
            }
        }
    }
    __syncthreads();

    int status = 0, it = 0;
    if (any_bad) {
        status = BLF_QP_BAD_FACETS;
    } else {
        // ---- initial state 2: full Newton step of the unconstrained QP (W = 0, lam = 0) ----
        {
            double pres = 0.0, ck = 0.0, rh0 = 0.0, rh1 = 0.0;
            if (own) {
                stage_residuals(S, 0, k, N, P, L, flag, pres, ck, rh0, rh1);
                L.W(k, 0) = 0.0; L.W(k, 1) = 0.0; L.W(k, 2) = 0.0; L.W(k, 3) = 0.0;
                L.g(k, 0) = rh0;
                L.g(k, 1) = rh1;
            }
            __syncthreads();
            if (k == 0) {
                const bool ok = backward_sweep<true>(L, P, flag[1], flag[2]);
                flag[0] = ok ? 0.0 : 1.0;
                forward_sweep(L, N);
            }
            __syncthreads();
            if (own) {
                S.r0 = S.r0 + L.dr(k, 0);
                S.r1 = S.r1 + L.dr(k, 1);
                const double y0 = L.xi[2 * (k + 1)] + L.dxi[2 * (k + 1)];
                const double y1 = L.xi[2 * (k + 1) + 1] + L.dxi[2 * (k + 1) + 1];
                L.xi[2 * (k + 1)] = y0;
                L.xi[2 * (k + 1) + 1] = y1;
                // Q (xi - xi_ref) terms of the start-up costate pass below
                if (k + 1 < N) {
                    L.qx(k + 1, 0) = P.Qw0 * (y0 - S.xr0);
                    L.qx(k + 1, 1) = P.Qw1 * (y1 - S.xr1);
                } else {
                    flag[1] = P.Pw0 * (y0 - S.xr0);
                    flag[2] = P.Pw1 * (y1 - S.xr1);
                }
            }
        }
        const bool init_bad = flag[0] != 0.0;
        // ---- initial state 3: s = max(b - A r, 1e-2), lam = 1; ntot ----
        Rows F;
        load_rows(S, F);
#pragma unroll
        for (int i = 0; i < kMaxFacets; ++i) {
            if (i < S.m) {
                const double gr = F.a0[i] * S.r0 + F.a1[i] * S.r1;
                const double sl = F.h[i] - gr;
                S.s[i] = sl > 1e-2 ? sl : 1e-2;
                S.lam[i] = 1.0;
            }
        }
        int ntot = wave_isum(S.m);
        if constexpr (NW > 1) {
            if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = (double)ntot;
            __syncthreads();
            ntot = 0;
            for (int i = 0; i < NW; ++i) ntot += (int)red[i];
        }
        __syncthreads();
        // costates nu (single shooting) for the initial dual residual, thread 0 -> L.dxi
        if (k == 0) {
            double n0 = flag[1];
            double n1 = flag[2];
            L.dxi[2 * N] = n0;
            L.dxi[2 * N + 1] = n1;
            for (int q = N - 1; q >= 1; --q) {
                const double aq = L.al(q);
                n0 = L.qx(q, 0) + aq * n0;
                n1 = L.qx(q, 1) + aq * n1;
                L.dxi[2 * q] = n0;
                L.dxi[2 * q + 1] = n1;
            }
        }
        __syncthreads();
        double dres = 0.0;
        if (own) {
            double rj0 = P.Rw0 * (S.r0 - S.rr0);
            double rj1 = P.Rw1 * (S.r1 - S.rr1);
#pragma unroll
            for (int i = 0; i < kMaxFacets; ++i)
                if (i < S.m) {
                    rj0 = rj0 + F.a0[i] * S.lam[i];
                    rj1 = rj1 + F.a1[i] * S.lam[i];
                }
            dres = nanmax(dres, fabs(rj0 - S.be * L.dxi[2 * (k + 1)]));
            dres = nanmax(dres, fabs(rj1 - S.be * L.dxi[2 * (k + 1) + 1]));
        }
        dres = block_nanmax<NW>(dres, red);
        if (init_bad) status = BLF_QP_NUMERICAL;

        for (it = 0; status == 0; ++it) {
            // ---- residuals (stage-parallel) ----
            double pres = 0.0, ck = 0.0, rh0 = 0.0, rh1 = 0.0;
            if (own) stage_residuals(S, S.m, k, N, P, L, flag, pres, ck, rh0, rh1);
            const double csum = block_sum<NW>(ck, red);
            const double mu = ntot > 0 ? csum / (double)ntot : 0.0;
            pres = block_nanmax<NW>(pres, red);
            if (!(mu == mu) || !(pres == pres) || !(dres == dres) || __builtin_isinf(mu)) {
                status = BLF_QP_NUMERICAL;
                break;
            }
            if (mu <= P.tol_mu && pres <= P.tol_p && dres <= P.tol_d) break;   // solved
            if (it >= P.max_iter) {
                status = BLF_QP_MAX_ITER;
                break;
            }

            // ---- W = A^T diag(lam/s) A, det W, affine right-hand side (stage-parallel) ----
            if (own) {
                Rows F;
                load_rows(S, F);
                double W00 = 0.0, W01 = 0.0, W11 = 0.0, dW = 0.0;
                double g0 = rh0, g1 = rh1;
                double sg[kMaxFacets];
#pragma unroll
                for (int i = 0; i < kMaxFacets; ++i) {
                    sg[i] = 0.0;
                    if (i < S.m) {
                        sg[i] = S.lam[i] / S.s[i];
                        const double t0 = sg[i] * F.a0[i];
                        const double t1 = sg[i] * F.a1[i];
                        W00 = W00 + t0 * F.a0[i];
                        W01 = W01 + t0 * F.a1[i];
                        W11 = W11 + t1 * F.a1[i];
                        const double rc = S.s[i] * S.lam[i];
                        const double e = (S.lam[i] * primal_res(S, F, i) - rc) / S.s[i];
                        g0 = g0 + F.a0[i] * e;
                        g1 = g1 + F.a1[i] * e;
                    }
                }
#pragma unroll
                for (int i = 1; i < kMaxFacets; ++i) {
#pragma unroll
                    for (int j = 0; j < i; ++j) {
                        if (i < S.m) {
                            const double cr = F.a0[i] * F.a1[j] - F.a1[i] * F.a0[j];
                            dW = dW + (sg[i] * sg[j]) * (cr * cr);
                        }
                    }
                }
                L.W(k, 0) = W00;
                L.W(k, 1) = W01;
                L.W(k, 2) = W11;
                L.W(k, 3) = dW;
                L.g(k, 0) = g0;
                L.g(k, 1) = g1;
            }
            __syncthreads();

            // ---- affine (predictor) Newton step: factor + solve on thread 0 ----
            if (k == 0) {
                STAMP(t_f);
                const bool ok = backward_sweep<true>(L, P, flag[1], flag[2]);
                flag[0] = ok ? 0.0 : 1.0;
                forward_sweep(L, N);
                STAMP_ADD(1, t_f);
            }
            __syncthreads();
            const bool factor_bad = flag[0] != 0.0;

            double smax = __builtin_inf();
            if (own) {
                Rows F;
                load_rows(S, F);
                S.dra0 = L.dr(k, 0);
                S.dra1 = L.dr(k, 1);
#pragma unroll
                for (int i = 0; i < kMaxFacets; ++i) {
                    if (i < S.m) {
                        double ds, dl;
                        affine_step(S, F, i, ds, dl);
                        if (ds < 0.0) smax = keepmin(smax, (-S.s[i]) / ds);
                        if (dl < 0.0) smax = keepmin(smax, (-S.lam[i]) / dl);
                    }
                }
            }
            smax = block_keepmin<NW>(smax, red);
            const double a_aff = smax < 1.0 ? smax : 1.0;
            ck = 0.0;
            if (own) {
                Rows F;
                load_rows(S, F);
#pragma unroll
                for (int i = 0; i < kMaxFacets; ++i) {
                    if (i < S.m) {
                        double ds, dl;
                        affine_step(S, F, i, ds, dl);
                        ck = ck + (S.s[i] + a_aff * ds) * (S.lam[i] + a_aff * dl);
                    }
                }
            }
            const double caff = block_sum<NW>(ck, red);
            const double mu_aff = ntot > 0 ? caff / (double)ntot : 0.0;
            double sigma = 0.0;
            if (mu > 0.0) {
                const double q = mu_aff / mu;
                sigma = (q * q) * q;
            }
            const double sigma_mu = sigma * mu;

            // ---- corrector right-hand side (stage-parallel) + solve (thread 0) ----
            if (own) {
                Rows F;
                load_rows(S, F);
                double g0 = rh0, g1 = rh1;
#pragma unroll
                for (int i = 0; i < kMaxFacets; ++i) {
                    if (i < S.m) {
                        double ds, dl;
                        affine_step(S, F, i, ds, dl);
                        const double rc = (S.s[i] * S.lam[i] + ds * dl) - sigma_mu;
                        const double e = (S.lam[i] * primal_res(S, F, i) - rc) / S.s[i];
                        g0 = g0 + F.a0[i] * e;
                        g1 = g1 + F.a1[i] * e;
                    }
                }
                L.g(k, 0) = g0;
                L.g(k, 1) = g1;
            }
            __syncthreads();
            if (k == 0) {
                STAMP(t_s);
                backward_sweep<false>(L, P, flag[1], flag[2]);
                forward_sweep(L, N);
                STAMP_ADD(2, t_s);
            }
            __syncthreads();

            // ---- corrector step length and update ----
            smax = __builtin_inf();
            double dr0 = 0.0, dr1 = 0.0;
            double cds[kMaxFacets], cdl[kMaxFacets];
            if (own) {
                Rows F;
                load_rows(S, F);
                dr0 = L.dr(k, 0);
                dr1 = L.dr(k, 1);
#pragma unroll
                for (int i = 0; i < kMaxFacets; ++i) {
                    cds[i] = 0.0;
                    cdl[i] = 0.0;
                    if (i < S.m) {
                        double ads, adl;
                        affine_step(S, F, i, ads, adl);
                        const double rc = (S.s[i] * S.lam[i] + ads * adl) - sigma_mu;
                        const double ds = (-primal_res(S, F, i)) - (F.a0[i] * dr0 + F.a1[i] * dr1);
                        const double dl = ((-rc) - S.lam[i] * ds) / S.s[i];
                        if (ds < 0.0) smax = keepmin(smax, (-S.s[i]) / ds);
                        if (dl < 0.0) smax = keepmin(smax, (-S.lam[i]) / dl);
                        cds[i] = ds;
                        cdl[i] = dl;
                    }
                }
            }
            smax = block_keepmin<NW>(smax, red);
            if (factor_bad) {
                status = BLF_QP_NUMERICAL;
                break;
            }
            const double step = 0.99 * smax;
            const double a = step < 1.0 ? step : 1.0;
            if (own) {
                S.r0 = S.r0 + a * dr0;
                S.r1 = S.r1 + a * dr1;
                L.xi[2 * (k + 1)] = L.xi[2 * (k + 1)] + a * L.dxi[2 * (k + 1)];
                L.xi[2 * (k + 1) + 1] = L.xi[2 * (k + 1) + 1] + a * L.dxi[2 * (k + 1) + 1];
#pragma unroll
                for (int i = 0; i < kMaxFacets; ++i) {
                    if (i < S.m) {
                        S.s[i] = S.s[i] + a * cds[i];
                        S.lam[i] = S.lam[i] + a * cdl[i];
                    }
                }
            }
            dres = dres * (1.0 - a);
            __syncthreads();
        }
    }

    // ---- outputs ----
    __syncthreads();
    if (own) {
        const int64_t st = p * N + k;
        vrp_out[2 * st] = S.r0;
        vrp_out[2 * st + 1] = S.r1;
        const int64_t sx = p * (N + 1) + (k + 1);
        xi_out[2 * sx] = L.xi[2 * (k + 1)];
        xi_out[2 * sx + 1] = L.xi[2 * (k + 1) + 1];
    }
    if (k == 0) {
        xi_out[2 * p * (N + 1)] = L.xi[0];
        xi_out[2 * p * (N + 1) + 1] = L.xi[1];
        status_out[p] = status;
        iters_out[p] = it;
        STAMP_ADD(0, t_start);
#ifdef BLF_STAMPS
        if (blockIdx.x < 64) atomicAdd(&g_blf_stamps[3], (unsigned long long)it);
#endif
    }
}

template <int NT>
blf_status launch_nt(const KParams& kp, const blf_dcm_mpc_problem* pb, int64_t batch,
                     const blf_dcm_mpc_solution* sol, hipStream_t s)
{
    const size_t lds = sizeof(double) * lds_doubles(kp.N, NT / kWave);
    if (lds > 160 * 1024) return set_error(BLF_ERR_UNSUPPORTED, "horizon %d needs %zu B of LDS", kp.N, lds);
    hipLaunchKernelGGL(dcm_mpc_ipm_kernel<NT>, dim3((unsigned)batch), dim3(NT), lds, s, kp,
                       pb->xi_init, pb->omega, pb->xi_ref, pb->vrp_ref, pb->A, pb->b,
                       pb->nfacets, sol->xi, sol->vrp, sol->status, sol->iters);
    return check_hip(hipGetLastError(), "dcm_mpc_ipm_kernel launch");
}

}  // namespace

#ifdef BLF_STAMPS
extern "C" int blf_debug_stamps(unsigned long long* out, int reset)
{
    unsigned long long h[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_blf_stamps), sizeof(h)) != hipSuccess) return -1;
    for (int i = 0; i < 8; ++i) out[i] = h[i];
    if (reset) {
        unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_blf_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

blf_status launch_dcm_mpc(const blf_dcm_mpc_params* prm, const blf_dcm_mpc_problem* pb,
                          int64_t batch, const blf_dcm_mpc_solution* sol, hipStream_t s)
{
    KParams kp;
    kp.N = prm->horizon;
    kp.M = prm->max_facets;
    kp.max_iter = prm->max_iter;
    kp.dt = prm->dt;
    kp.Qw0 = prm->w_xi[0]; kp.Qw1 = prm->w_xi[1];
    kp.Rw0 = prm->w_vrp[0]; kp.Rw1 = prm->w_vrp[1];
    kp.Pw0 = prm->w_terminal[0]; kp.Pw1 = prm->w_terminal[1];
    kp.tol_mu = prm->tol_mu;
    kp.tol_p = prm->tol_primal;
    kp.tol_d = prm->tol_dual;
    if (batch == 0) return BLF_OK;
    if (batch > 0x7fffffffLL) return set_error(BLF_ERR_UNSUPPORTED, "batch %lld too large", (long long)batch);
    const int N = kp.N;
    if (N <= 64) return launch_nt<64>(kp, pb, batch, sol, s);
    if (N <= 128) return launch_nt<128>(kp, pb, batch, sol, s);
    if (N <= 256) return launch_nt<256>(kp, pb, batch, sol, s);
    if (N <= 512) return launch_nt<512>(kp, pb, batch, sol, s);
    if (N <= 1024) return launch_nt<1024>(kp, pb, batch, sol, s);
    return set_error(BLF_ERR_UNSUPPORTED, "horizon %d > 1024", N);
}

}  // namespace blf
