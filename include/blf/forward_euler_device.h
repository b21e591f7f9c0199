/* forward_euler_device.h — ForwardEuler<System>::integrate over a batch of USER dynamical
 * systems on the device (HIP, gfx950).  Header-only: the user's translation unit, compiled with
 * hipcc, instantiates the kernel for its own system type.
 *
 * Reference surface it replaces for user systems:
 *   src/System/include/BipedalLocomotion/System/DynamicalSystem.h:98   (dynamics(t, dx) override)
 *   src/System/include/BipedalLocomotion/System/ForwardEuler.tpp:18-49 (x = x + dT * dx)
 *   src/System/include/BipedalLocomotion/System/FixedStepIntegrator.tpp:21-72 (the step schedule)
 * The reference integrates any DynamicalSystem subclass that overrides dynamics(); a GPU cannot
 * call a host-side virtual, so here the user states the dynamics once as a __device__ function of
 * a System type and the integrator kernel is generated for it.  The schedule (validation, step
 * count, stale last-step time) comes from the library (blf_step_schedule), so user systems step
 * exactly like the built-in ones (blf_lti_euler_integrate, blf_fbk_euler_integrate, ...).
 *
 * A System provides:
 *   static constexpr int kStateSize;   // n >= 1 (state in registers: keep it small, <= ~64)
 *   static constexpr int kInputSize;   // m >= 0 (the control input, held over the interval as
 *                                      //         setControlInput holds it)
 *   struct Params;                     // trivially copyable parameters of one system
 *   __device__ static void dynamics(double t, const double* x, const double* u,
 *                                   const Params& p, double* dx);
 *       t: the step's currentTime (FixedStepIntegrator.tpp:53; the last step reuses the stale
 *          time of the step before it, :63-64), x: [n], u: [m], dx: [n] output.
 *
 * Layout: x [batch][n] (updated in place), u [batch][m], params [batch] (or one shared Params
 * when params_shared != 0).  One lane per system (states of up to 16 doubles staged through LDS,
 * so the batch's state is read and written coalesced); x_r <- x_r + dx_r * h after every step (no FMA
 * contraction: build the user TU with -ffp-contract=off for results that match a CPU restatement
 * bit for bit).  Returns the C ABI's status codes (blf_c.h): the schedule's errors (with
 * blf_last_error() set), BLF_ERR_INVALID_ARGUMENT for null buffers or a negative batch, and
 * BLF_ERR_HIP when the launch fails (hipGetLastError() holds the cause). */
#pragma once
#include <hip/hip_runtime.h>

#include "blf_c.h"

namespace blf {

template <class System>
__global__ __launch_bounds__(256) void forward_euler_user_kernel(
    const typename System::Params* __restrict__ params, int params_shared, const double* __restrict__ u,
    double* __restrict__ x, int64_t batch, double t0, double dT, int32_t iterations, double dT_last,
    double t_last)
{
    constexpr int n = System::kStateSize;
    constexpr int m = System::kInputSize > 0 ? System::kInputSize : 1;
    // States of up to 16 doubles move through LDS: the workgroup's contiguous [256][n] slab is read
    // and written with consecutive lanes on consecutive doubles (coalesced), and each lane takes its
    // own row from LDS (odd row stride: no bank conflicts).  Larger states are read lane by lane.
    constexpr bool kStage = n <= 16;
    constexpr int SW = n | 1;
    __shared__ double sx[kStage ? 256 * SW : 1];
    const int64_t q0 = (int64_t)blockIdx.x * blockDim.x;
    const int64_t q = q0 + threadIdx.x;
    const int rows = (int)(batch - q0 < (int64_t)blockDim.x ? batch - q0 : (int64_t)blockDim.x);
    double xr[n], ur[m], dx[n];
    if (kStage) {
        for (int e = threadIdx.x; e < rows * n; e += blockDim.x) {
            const int r = e / n;
            sx[r * SW + (e - r * n)] = x[q0 * n + e];
        }
        __syncthreads();
    }
    if (q < batch) {
        const typename System::Params p = params[params_shared ? 0 : q];
#pragma unroll
        for (int r = 0; r < n; ++r) xr[r] = kStage ? sx[threadIdx.x * SW + r] : x[q * n + r];
#pragma unroll
        for (int c = 0; c < m; ++c) ur[c] = System::kInputSize > 0 ? u[q * System::kInputSize + c] : 0.0;
        // steps 0 .. iterations-2 at currentTime = t0 + dT i, then the last one at the stale time
        for (int32_t i = 0; i < iterations; ++i) {
            const bool last = i == iterations - 1;
            const double t = last ? t_last : t0 + dT * (double)i;
            const double h = last ? dT_last : dT;
            System::dynamics(t, xr, ur, p, dx);
#pragma unroll
            for (int r = 0; r < n; ++r) xr[r] = xr[r] + dx[r] * h;
        }
#pragma unroll
        for (int r = 0; r < n; ++r) {
            if (kStage) sx[threadIdx.x * SW + r] = xr[r];
            else x[q * n + r] = xr[r];
        }
    }
    if (kStage) {
        __syncthreads();
        for (int e = threadIdx.x; e < rows * n; e += blockDim.x) {
            const int r = e / n;
            x[q0 * n + e] = sx[r * SW + (e - r * n)];
        }
    }
}

/* ForwardEuler<System>::integrate(initial_time, final_time) with sampling time dT, for `batch`
 * systems, stream-ordered on `stream`. */
template <class System>
blf_status forward_euler_integrate(const typename System::Params* params, int params_shared, const double* u,
                                   double* x, int64_t batch, double initial_time, double final_time, double dT,
                                   hipStream_t stream)
{
    static_assert(System::kStateSize >= 1, "kStateSize must be >= 1");
    static_assert(System::kInputSize >= 0, "kInputSize must be >= 0");
    int32_t iterations = 0;
    double dT_last = 0.0, t_last = 0.0;
    const blf_status st = blf_step_schedule(initial_time, final_time, dT, &iterations, &dT_last, &t_last);
    if (st != BLF_OK) return st;
    if (batch < 0 || (batch > 0 && (!params || !x || (System::kInputSize > 0 && !u))))
        return BLF_ERR_INVALID_ARGUMENT;
    if (batch == 0) return BLF_OK;
    const int64_t blocks = (batch + 255) / 256;
    if (blocks > 0x7fffffff) return BLF_ERR_UNSUPPORTED;
    hipLaunchKernelGGL(forward_euler_user_kernel<System>, dim3((unsigned)blocks), dim3(256), 0, stream, params,
                       params_shared, u, x, batch, initial_time, dT, iterations, dT_last, t_last);
    return hipGetLastError() == hipSuccess ? BLF_OK : BLF_ERR_HIP;
}

}  // namespace blf
