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

struct KParams {
    int N, M, max_iter;
    double dt, Qw0, Qw1, Rw0, Rw1, Pw0, Pw1, tol_mu, tol_p, tol_d;
};

// LDS carve-up (in doubles), sized by N.  The same code computes the launch size on the host
// (Lds(nullptr, ...).total), so the allocation always covers every array.
struct Lds {
    double *xi, *al, *be, *a2, *b2, *W, *Hi, *Pn, *g, *d, *qx, *kff, *dr, *dxi, *om, *xir, *red;
    size_t total;   // doubles
    __host__ __device__ Lds(double* base, int N, int NW)
    {
        size_t o = 0;
        auto take = [&](size_t n) {
            double* p = base ? base + o : nullptr;
            o += n;
            return p;
        };
        xi = take(2 * (N + 1));   // [N+1][2]
        al = take(N);             // [N]
        be = take(N);
        a2 = take(N);
        b2 = take(N);
        W = take(4 * N);          // [N][4]  A^T diag(lam/s) A (3) + its determinant
        Hi = take(3 * N);         // [N][3]
        Pn = take(3 * N);         // [N][3]
        g = take(2 * N);          // [N][2]
        d = take(2 * N);          // [N][2]
        qx = take(2 * N);         // [N][2]  Q (xi_k - xi_ref_k), k >= 1
        kff = take(2 * N);        // [N][2]
        dr = take(2 * N);         // [N][2]
        dxi = take(2 * (N + 1));  // [N+1][2] (also the costates nu at start-up)
        om = take(N);             // [N]
        xir = take(2 * (N + 1));  // [N+1][2]
        red = take(4 * NW + 8);   // [NW] reduction scratch + flags
        total = o;
    }
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

// Backward Riccati sweep (thread 0) = oracle dcm_backward.  factor: builds Hi_k = H_k^{-1} and
// Pn_k = P_{k+1}; otherwise reuses them.  Returns false if some H_k is not positive definite.
__device__ bool backward_sweep(const Lds& L, const KParams& k, bool factor, double pv0, double pv1)
{
    bool ok = true;
    double P00 = k.Pw0, P01 = 0.0, P11 = k.Pw1;
    for (int s = k.N - 1; s >= 0; --s) {
        double h00, h01, h11;
        const double b2 = L.b2[s];
        if (factor) {
            // H = B + W, B = R + b2 P_{k+1}: det H = det B + tr(adj(B) W) + det W (all >= 0)
            const double B00 = k.Rw0 + b2 * P00;
            const double B01 = b2 * P01;
            const double B11 = k.Rw1 + b2 * P11;
            const double W00 = L.W[4 * s], W01 = L.W[4 * s + 1], W11 = L.W[4 * s + 2];
            const double H00 = B00 + W00;
            const double H01 = B01 + W01;
            const double H11 = B11 + W11;
            const double detB = B00 * B11 - B01 * B01;
            const double trW = (B11 * W00 + B00 * W11) - 2.0 * (B01 * W01);
            const double det = (detB + trW) + L.W[4 * s + 3];
            if (!(det > 0.0) || __builtin_isinf(det)) ok = false;
            const double idet = 1.0 / det;
            h00 = H11 * idet;
            h01 = -(H01 * idet);
            h11 = H00 * idet;
            L.Hi[3 * s] = h00; L.Hi[3 * s + 1] = h01; L.Hi[3 * s + 2] = h11;
            L.Pn[3 * s] = P00; L.Pn[3 * s + 1] = P01; L.Pn[3 * s + 2] = P11;
        } else {
            h00 = L.Hi[3 * s]; h01 = L.Hi[3 * s + 1]; h11 = L.Hi[3 * s + 2];
            P00 = L.Pn[3 * s]; P01 = L.Pn[3 * s + 1]; P11 = L.Pn[3 * s + 2];
        }
        const double be = L.be[s];
        const double d0 = L.d[2 * s], d1 = L.d[2 * s + 1];
        const double t0 = (P00 * d0 + P01 * d1) + pv0;
        const double t1 = (P01 * d0 + P11 * d1) + pv1;
        const double hu0 = L.g[2 * s] - be * t0;
        const double hu1 = L.g[2 * s + 1] - be * t1;
        const double k0 = -(h00 * hu0 + h01 * hu1);
        const double k1 = -(h01 * hu0 + h11 * hu1);
        L.kff[2 * s] = k0;
        L.kff[2 * s + 1] = k1;
        if (s > 0) {
            const double al = L.al[s];
            const double pk0 = P00 * k0 + P01 * k1;
            const double pk1 = P01 * k0 + P11 * k1;
            const double npv0 = L.qx[2 * s] + al * (t0 - be * pk0);
            const double npv1 = L.qx[2 * s + 1] + al * (t1 - be * pk1);
            if (factor) {
                // P_k = Q + a^2 (P - b^2 P H^-1 P)
                const double a2 = L.a2[s];
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

// Forward sweep (thread 0) = oracle dcm_forward.
__device__ void forward_sweep(const Lds& L, int N)
{
    double x0 = 0.0, x1 = 0.0;
    L.dxi[0] = 0.0;
    L.dxi[1] = 0.0;
    for (int s = 0; s < N; ++s) {
        const double q00 = L.Pn[3 * s], q01 = L.Pn[3 * s + 1], q11 = L.Pn[3 * s + 2];
        const double u0 = q00 * x0 + q01 * x1;
        const double u1 = q01 * x0 + q11 * x1;
        const double v0 = L.Hi[3 * s] * u0 + L.Hi[3 * s + 1] * u1;
        const double v1 = L.Hi[3 * s + 1] * u0 + L.Hi[3 * s + 2] * u1;
        const double al = L.al[s], be = L.be[s];
        const double ab = al * be;
        const double r0 = ab * v0 + L.kff[2 * s];
        const double r1 = ab * v1 + L.kff[2 * s + 1];
        L.dr[2 * s] = r0;
        L.dr[2 * s + 1] = r1;
        const double n0 = (al * x0 - be * r0) + L.d[2 * s];
        const double n1 = (al * x1 - be * r1) + L.d[2 * s + 1];
        L.dxi[2 * (s + 1)] = n0;
        L.dxi[2 * (s + 1) + 1] = n1;
        x0 = n0;
        x1 = n1;
    }
}

// The knot a thread owns: facet rows, slacks, multipliers and the knot's VRP in registers.
struct Stage {
    double a0[kMaxFacets], a1[kMaxFacets], h[kMaxFacets], s[kMaxFacets], lam[kMaxFacets];
    double rp[kMaxFacets], pr[kMaxFacets];
    int m;
    double r0, r1, rr0, rr1, xr0, xr1, w, be;
};

// Stage-parallel residual pass = the body of oracle dcm_residuals for one knot.  Writes the
// Euler defect and Q(xi_{k+1} - xi_ref_{k+1}) (or the terminal pv) to LDS; returns pres, ck,
// rho in registers.  mfac: the facet count to use (0 for the unconstrained warm start).
__device__ __forceinline__ void stage_residuals(Stage& S, int mfac, int k, int N, const KParams& P,
                                                const Lds& L, double* flag, double& pres,
                                                double& ck, double& rh0, double& rh1)
{
    rh0 = P.Rw0 * (S.r0 - S.rr0);
    rh1 = P.Rw1 * (S.r1 - S.rr1);
#pragma unroll
    for (int i = 0; i < kMaxFacets; ++i) {
        if (i < mfac) {
            const double gr = S.a0[i] * S.r0 + S.a1[i] * S.r1;
            const double rpi = (gr + S.s[i]) - S.h[i];
            S.rp[i] = rpi;
            pres = nanmax(pres, fabs(rpi));
            ck = ck + S.s[i] * S.lam[i];
            rh0 = rh0 + S.a0[i] * S.lam[i];
            rh1 = rh1 + S.a1[i] * S.lam[i];
        }
    }
    const double x0 = L.xi[2 * k], x1 = L.xi[2 * k + 1];
    const double y0 = L.xi[2 * (k + 1)], y1 = L.xi[2 * (k + 1) + 1];
    const double dx0 = S.w * x0 + (-S.w) * S.r0;
    const double dk0 = (x0 + dx0 * P.dt) - y0;
    const double dx1 = S.w * x1 + (-S.w) * S.r1;
    const double dk1 = (x1 + dx1 * P.dt) - y1;
    L.d[2 * k] = dk0;
    L.d[2 * k + 1] = dk1;
    pres = nanmax(pres, fabs(dk0));
    pres = nanmax(pres, fabs(dk1));
    if (k + 1 < N) {
        L.qx[2 * (k + 1)] = P.Qw0 * (y0 - S.xr0);
        L.qx[2 * (k + 1) + 1] = P.Qw1 * (y1 - S.xr1);
    } else {
        flag[1] = P.Pw0 * (y0 - S.xr0);
        flag[2] = P.Pw1 * (y1 - S.xr1);
    }
}

template <int NT>
__global__ __launch_bounds__(NT) void dcm_mpc_ipm_kernel(
    KParams P, const double* __restrict__ xi_init, const double* __restrict__ omega,
    const double* __restrict__ xi_ref, const double* __restrict__ vrp_ref,
    const double* __restrict__ Ain, const double* __restrict__ bin,
    const int32_t* __restrict__ nfacets, double* __restrict__ xi_out,
    double* __restrict__ vrp_out, int32_t* __restrict__ status_out,
    int32_t* __restrict__ iters_out)
{
    constexpr int NW = NT / kWave;
    extern __shared__ double smem[];
    const int N = P.N, M = P.M;
    Lds L(smem, N, NW);
    double* red = L.red;               // [NW] scratch for block reductions
    double* flag = L.red + 4 * NW;     // shared scalars: [0] factor failed, [1..2] terminal pv

    const int k = threadIdx.x;
    const bool own = k < N;
    const int64_t p = blockIdx.x;

    // ---- load the knot this thread owns ----
    Stage S;
    S.m = 0;
    S.r0 = S.r1 = S.rr0 = S.rr1 = S.xr0 = S.xr1 = S.w = S.be = 0.0;
#pragma unroll
    for (int i = 0; i < kMaxFacets; ++i) {
        S.a0[i] = 0.0; S.a1[i] = 0.0; S.h[i] = 0.0;
        S.s[i] = 1.0; S.lam[i] = 0.0; S.rp[i] = 0.0; S.pr[i] = 0.0;
    }
    bool bad = false;
    if (own) {
        const int64_t st = p * N + k;
        S.m = nfacets[st];
        bad = (S.m < 0 || S.m > M);
        const double* Ak = Ain + st * M * 2;
        const double* bk = bin + st * M;
#pragma unroll
        for (int i = 0; i < kMaxFacets; ++i) {
            if (i < M) {
                S.a0[i] = Ak[2 * i];
                S.a1[i] = Ak[2 * i + 1];
                S.h[i] = bk[i];
            }
        }
        S.w = omega[st];
        S.be = P.dt * S.w;
        const double al = 1.0 + S.be;
        L.al[k] = al;
        L.be[k] = S.be;
        L.a2[k] = al * al;
        L.b2[k] = S.be * S.be;
        L.om[k] = S.w;
        S.rr0 = vrp_ref[2 * st];
        S.rr1 = vrp_ref[2 * st + 1];
        S.r0 = S.rr0;
        S.r1 = S.rr1;
        L.dr[2 * k] = S.rr0;      // scratch: initial VRP for the rollout below
        L.dr[2 * k + 1] = S.rr1;
        const int64_t sx = p * (N + 1) + (k + 1);
        S.xr0 = xi_ref[2 * sx];
        S.xr1 = xi_ref[2 * sx + 1];
        L.xir[2 * (k + 1)] = S.xr0;
        L.xir[2 * (k + 1) + 1] = S.xr1;
    }
    if (k == 0) {
        L.xi[0] = xi_init[2 * p];
        L.xi[1] = xi_init[2 * p + 1];
        L.xir[0] = xi_ref[2 * p * (N + 1)];
        L.xir[1] = xi_ref[2 * p * (N + 1) + 1];
    }
    const bool any_bad = __syncthreads_or(bad);

    // ---- initial state 1: reference Euler rollout of vrp_ref (thread 0) ----
    if (k == 0) {
        for (int q = 0; q < N; ++q) {
            const double wq = L.om[q];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const double x = L.xi[2 * q + j];
                const double dx = wq * x + (-wq) * L.dr[2 * q + j];
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
                L.W[4 * k] = 0.0; L.W[4 * k + 1] = 0.0; L.W[4 * k + 2] = 0.0; L.W[4 * k + 3] = 0.0;
                L.g[2 * k] = rh0;
                L.g[2 * k + 1] = rh1;
            }
            __syncthreads();
            if (k == 0) {
                const bool ok = backward_sweep(L, P, true, flag[1], flag[2]);
                flag[0] = ok ? 0.0 : 1.0;
                forward_sweep(L, N);
            }
            __syncthreads();
            if (own) {
                S.r0 = S.r0 + L.dr[2 * k];
                S.r1 = S.r1 + L.dr[2 * k + 1];
                L.xi[2 * (k + 1)] = L.xi[2 * (k + 1)] + L.dxi[2 * (k + 1)];
                L.xi[2 * (k + 1) + 1] = L.xi[2 * (k + 1) + 1] + L.dxi[2 * (k + 1) + 1];
            }
        }
        const bool init_bad = flag[0] != 0.0;
        // ---- initial state 3: s = max(b - A r, 1e-2), lam = 1; ntot ----
#pragma unroll
        for (int i = 0; i < kMaxFacets; ++i) {
            if (i < S.m) {
                const double gr = S.a0[i] * S.r0 + S.a1[i] * S.r1;
                const double sl = S.h[i] - gr;
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
            double n0 = P.Pw0 * (L.xi[2 * N] - L.xir[2 * N]);
            double n1 = P.Pw1 * (L.xi[2 * N + 1] - L.xir[2 * N + 1]);
            L.dxi[2 * N] = n0;
            L.dxi[2 * N + 1] = n1;
            for (int q = N - 1; q >= 1; --q) {
                const double aq = L.al[q];
                n0 = P.Qw0 * (L.xi[2 * q] - L.xir[2 * q]) + aq * n0;
                n1 = P.Qw1 * (L.xi[2 * q + 1] - L.xir[2 * q + 1]) + aq * n1;
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
                    rj0 = rj0 + S.a0[i] * S.lam[i];
                    rj1 = rj1 + S.a1[i] * S.lam[i];
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
                double W00 = 0.0, W01 = 0.0, W11 = 0.0, dW = 0.0;
                double g0 = rh0, g1 = rh1;
                double sg[kMaxFacets];
#pragma unroll
                for (int i = 0; i < kMaxFacets; ++i) {
                    sg[i] = 0.0;
                    if (i < S.m) {
                        sg[i] = S.lam[i] / S.s[i];
                        const double t0 = sg[i] * S.a0[i];
                        const double t1 = sg[i] * S.a1[i];
                        W00 = W00 + t0 * S.a0[i];
                        W01 = W01 + t0 * S.a1[i];
                        W11 = W11 + t1 * S.a1[i];
                        const double rc = S.s[i] * S.lam[i];
                        const double e = (S.lam[i] * S.rp[i] - rc) / S.s[i];
                        g0 = g0 + S.a0[i] * e;
                        g1 = g1 + S.a1[i] * e;
                    }
                }
#pragma unroll
                for (int i = 1; i < kMaxFacets; ++i) {
#pragma unroll
                    for (int j = 0; j < i; ++j) {
                        if (i < S.m) {
                            const double cr = S.a0[i] * S.a1[j] - S.a1[i] * S.a0[j];
                            dW = dW + (sg[i] * sg[j]) * (cr * cr);
                        }
                    }
                }
                L.W[4 * k] = W00;
                L.W[4 * k + 1] = W01;
                L.W[4 * k + 2] = W11;
                L.W[4 * k + 3] = dW;
                L.g[2 * k] = g0;
                L.g[2 * k + 1] = g1;
            }
            __syncthreads();

            // ---- affine (predictor) Newton step: factor + solve on thread 0 ----
            if (k == 0) {
                const bool ok = backward_sweep(L, P, true, flag[1], flag[2]);
                flag[0] = ok ? 0.0 : 1.0;
                forward_sweep(L, N);
            }
            __syncthreads();
            const bool factor_bad = flag[0] != 0.0;

            double smax = __builtin_inf();
            double dr0 = 0.0, dr1 = 0.0;
            if (own) {
                dr0 = L.dr[2 * k];
                dr1 = L.dr[2 * k + 1];
#pragma unroll
                for (int i = 0; i < kMaxFacets; ++i) {
                    if (i < S.m) {
                        const double rc = S.s[i] * S.lam[i];
                        const double ds = (-S.rp[i]) - (S.a0[i] * dr0 + S.a1[i] * dr1);
                        const double dl = ((-rc) - S.lam[i] * ds) / S.s[i];
                        if (ds < 0.0) smax = keepmin(smax, (-S.s[i]) / ds);
                        if (dl < 0.0) smax = keepmin(smax, (-S.lam[i]) / dl);
                        S.pr[i] = ds * dl;
                    }
                }
            }
            smax = block_keepmin<NW>(smax, red);
            const double a_aff = smax < 1.0 ? smax : 1.0;
            ck = 0.0;
            if (own) {
#pragma unroll
                for (int i = 0; i < kMaxFacets; ++i) {
                    if (i < S.m) {
                        const double rc = S.s[i] * S.lam[i];
                        const double ds = (-S.rp[i]) - (S.a0[i] * dr0 + S.a1[i] * dr1);
                        const double dl = ((-rc) - S.lam[i] * ds) / S.s[i];
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
                double g0 = rh0, g1 = rh1;
#pragma unroll
                for (int i = 0; i < kMaxFacets; ++i) {
                    if (i < S.m) {
                        const double rc = (S.s[i] * S.lam[i] + S.pr[i]) - sigma_mu;
                        const double e = (S.lam[i] * S.rp[i] - rc) / S.s[i];
                        g0 = g0 + S.a0[i] * e;
                        g1 = g1 + S.a1[i] * e;
                    }
                }
                L.g[2 * k] = g0;
                L.g[2 * k + 1] = g1;
            }
            __syncthreads();
            if (k == 0) {
                backward_sweep(L, P, false, flag[1], flag[2]);
                forward_sweep(L, N);
            }
            __syncthreads();

            // ---- corrector step length and update ----
            smax = __builtin_inf();
            if (own) {
                dr0 = L.dr[2 * k];
                dr1 = L.dr[2 * k + 1];
#pragma unroll
                for (int i = 0; i < kMaxFacets; ++i) {
                    if (i < S.m) {
                        const double rc = (S.s[i] * S.lam[i] + S.pr[i]) - sigma_mu;
                        const double ds = (-S.rp[i]) - (S.a0[i] * dr0 + S.a1[i] * dr1);
                        const double dl = ((-rc) - S.lam[i] * ds) / S.s[i];
                        if (ds < 0.0) smax = keepmin(smax, (-S.s[i]) / ds);
                        if (dl < 0.0) smax = keepmin(smax, (-S.lam[i]) / dl);
                        S.rp[i] = ds;
                        S.pr[i] = dl;
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
                        S.s[i] = S.s[i] + a * S.rp[i];
                        S.lam[i] = S.lam[i] + a * S.pr[i];
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
