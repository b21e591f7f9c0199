// euler_rollout.hip — ForwardEuler<LinearTimeInvariantSystem> on the device.
//
//  * lti_euler_kernel: FixedStepIntegrator::integrate(t0, T) for a batch of small LTI systems
//    (reference: src/System/include/BipedalLocomotion/System/FixedStepIntegrator.tpp:21-72,
//    ForwardEuler.tpp:18-49, src/System/src/LinearTimeInvariantSystem.cpp:71).  The step
//    schedule (count and the stale-time last step) is computed once on the host (blf_capi.hip)
//    and is identical for every system of the batch.  One lane per system.
//  * dcm_rollout_kernel: the DCM instance, one reference Euler step per knot with
//    A = omega_k I, B = -omega_k I.  One lane per problem; each workgroup stages its 64 problems'
//    omega / vrp rows through LDS in chunks of knots so that the HBM reads and the xi writes are
//    coalesced (problem-major layout).
// Built with -ffp-contract=off: bit-identical to oracle/blf_oracle.c.
#include "blf_internal.h"

namespace blf {
namespace {

constexpr int kNmax = 8;

__global__ __launch_bounds__(256) void lti_euler_kernel(int n, int m, const double* __restrict__ A,
                                                        const double* __restrict__ Bm, int shared,
                                                        const double* __restrict__ u,
                                                        double* __restrict__ x, int64_t batch,
                                                        int32_t nsteps, double dT, double dT_last)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= batch) return;
    const double* Aq = shared ? A : A + q * n * n;
    const double* Bq = shared ? Bm : Bm + q * n * m;
    double xr[kNmax], ur[kNmax], Ar[kNmax * kNmax], Br[kNmax * kNmax];
#pragma unroll
    for (int r = 0; r < kNmax; ++r) {
        xr[r] = r < n ? x[q * n + r] : 0.0;
        ur[r] = r < m ? u[q * m + r] : 0.0;
#pragma unroll
        for (int c = 0; c < kNmax; ++c) {
            Ar[r * kNmax + c] = (r < n && c < n) ? Aq[r * n + c] : 0.0;
            Br[r * kNmax + c] = (r < n && c < m) ? Bq[r * m + c] : 0.0;
        }
    }
    // B u is constant over the interval (setControlInput holds u), but the reference recomputes
    // it every step; the value is identical, so compute it once.
    double bu[kNmax];
#pragma unroll
    for (int r = 0; r < kNmax; ++r) {
        double acc = Br[r * kNmax + 0] * ur[0];
#pragma unroll
        for (int c = 1; c < kNmax; ++c)
            if (c < m) acc = acc + Br[r * kNmax + c] * ur[c];
        bu[r] = acc;
    }
    for (int32_t i = 0; i < nsteps; ++i) {
        const double h = (i == nsteps - 1) ? dT_last : dT;
        double dx[kNmax];
#pragma unroll
        for (int r = 0; r < kNmax; ++r) {
            double acc = Ar[r * kNmax + 0] * xr[0];
#pragma unroll
            for (int c = 1; c < kNmax; ++c)
                if (c < n) acc = acc + Ar[r * kNmax + c] * xr[c];
            dx[r] = acc + bu[r];
        }
#pragma unroll
        for (int r = 0; r < kNmax; ++r)
            if (r < n) xr[r] = xr[r] + dx[r] * h;
    }
#pragma unroll
    for (int r = 0; r < kNmax; ++r)
        if (r < n) x[q * n + r] = xr[r];
}

__global__ __launch_bounds__(256) void lti_dynamics_kernel(int n, int m,
                                                           const double* __restrict__ A,
                                                           const double* __restrict__ Bm,
                                                           int shared,
                                                           const double* __restrict__ u,
                                                           const double* __restrict__ x,
                                                           double* __restrict__ dx, int64_t batch)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= batch) return;
    const double* Aq = shared ? A : A + q * n * n;
    const double* Bq = shared ? Bm : Bm + q * n * m;
    for (int r = 0; r < n; ++r) {
        double ax = Aq[r * n] * x[q * n];
        for (int c = 1; c < n; ++c) ax = ax + Aq[r * n + c] * x[q * n + c];
        double bu = Bq[r * m] * u[q * m];
        for (int c = 1; c < m; ++c) bu = bu + Bq[r * m + c] * u[q * m + c];
        dx[q * n + r] = ax + bu;
    }
}

// 64 problems per workgroup (one wave), knots staged in chunks of KC.
constexpr int KC = 16;

__global__ __launch_bounds__(64) void dcm_rollout_kernel(const double* __restrict__ xi0,
                                                         const double* __restrict__ omega,
                                                         const double* __restrict__ vrp,
                                                         int32_t N, double dt,
                                                         double* __restrict__ xi_out,
                                                         int64_t batch)
{
    // per chunk: omega [64][KC], vrp [64][KC][2] (overwritten in place by xi) ; +1 padding per
    // row breaks the power-of-two stride between lanes (bank conflicts on the per-lane reads).
    __shared__ double s_om[64 * (KC + 1)];
    __shared__ double s_r[64 * (2 * KC + 1)];
    double* s_x = s_r;
    const int lane = threadIdx.x;
    const int64_t p0 = (int64_t)blockIdx.x * 64;
    const int64_t q = p0 + lane;
    const int nprob = (int)((batch - p0) < 64 ? (batch - p0) : 64);
    double x0 = 0.0, x1 = 0.0;
    if (q < batch) {
        x0 = xi0[2 * q];
        x1 = xi0[2 * q + 1];
        xi_out[2 * q * (N + 1)] = x0;
        xi_out[2 * q * (N + 1) + 1] = x1;
    }
    for (int kb = 0; kb < N; kb += KC) {
        const int kc = (N - kb) < KC ? (N - kb) : KC;
        // cooperative, coalesced loads of the chunk: row p of omega is contiguous
        for (int e = lane; e < nprob * kc; e += 64) {
            const int pr = e / kc, kk = e % kc;
            s_om[pr * (KC + 1) + kk] = omega[(p0 + pr) * N + kb + kk];
        }
        for (int e = lane; e < nprob * 2 * kc; e += 64) {
            const int pr = e / (2 * kc), kk = e % (2 * kc);
            s_r[pr * (2 * KC + 1) + kk] = vrp[(p0 + pr) * 2 * N + 2 * kb + kk];
        }
        __syncthreads();
        if (lane < nprob) {
            for (int kk = 0; kk < kc; ++kk) {
                const double w = s_om[lane * (KC + 1) + kk];
                const double dx0 = w * x0 + (-w) * s_r[lane * (2 * KC + 1) + 2 * kk];
                const double dx1 = w * x1 + (-w) * s_r[lane * (2 * KC + 1) + 2 * kk + 1];
                x0 = x0 + dx0 * dt;
                x1 = x1 + dx1 * dt;
                s_x[lane * (2 * KC + 1) + 2 * kk] = x0;
                s_x[lane * (2 * KC + 1) + 2 * kk + 1] = x1;
            }
        }
        __syncthreads();
        for (int e = lane; e < nprob * 2 * kc; e += 64) {
            const int pr = e / (2 * kc), kk = e % (2 * kc);
            xi_out[(p0 + pr) * 2 * (N + 1) + 2 * (kb + 1) + kk] = s_x[pr * (2 * KC + 1) + kk];
        }
        __syncthreads();
    }
}

}  // namespace

blf_status launch_lti_euler(int n, int m, const double* A, const double* Bm, int shared,
                            const double* u, double* x, int64_t batch, int32_t nsteps,
                            double dT, double dT_last, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    const int64_t blocks = ceil_div(batch, 256);
    hipLaunchKernelGGL(lti_euler_kernel, dim3((unsigned)blocks), dim3(256), 0, s, n, m, A, Bm,
                       shared, u, x, batch, nsteps, dT, dT_last);
    return check_hip(hipGetLastError(), "lti_euler_kernel launch");
}

blf_status launch_lti_dynamics(int n, int m, const double* A, const double* Bm, int shared,
                               const double* u, const double* x, double* dx, int64_t batch,
                               hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    hipLaunchKernelGGL(lti_dynamics_kernel, dim3((unsigned)ceil_div(batch, 256)), dim3(256), 0, s,
                       n, m, A, Bm, shared, u, x, dx, batch);
    return check_hip(hipGetLastError(), "lti_dynamics_kernel launch");
}

blf_status launch_dcm_rollout(const double* xi0, const double* omega, const double* vrp,
                              int32_t N, double dt, double* xi_out, int64_t batch,
                              hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    const int64_t blocks = ceil_div(batch, 64);
    hipLaunchKernelGGL(dcm_rollout_kernel, dim3((unsigned)blocks), dim3(64), 0, s, xi0, omega,
                       vrp, N, dt, xi_out, batch);
    return check_hip(hipGetLastError(), "dcm_rollout_kernel launch");
}

}  // namespace blf
