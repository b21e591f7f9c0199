// floating_base.hip — FloatingBaseSystemKinematics on the device.
//
//  * fbk_dynamics_kernel: FloatingBaseSystemKinematics::dynamics
//    (src/System/src/FloatingBaseSystemKinematics.cpp:36-73), one lane per system:
//      dp = v,  dR = -R.colwise().cross(w) + rho/2 ((R R^T)^{-1} - I) R,  ds = s_dot
//    (mixed velocity representation; (R R^T)^{-1} by cofactors, Baumgarte term included).
//  * fbk_euler_kernel: ForwardEuler<FloatingBaseSystemKinematics>::integrate over the
//    FixedStepIntegrator schedule (computed once on the host, blf_capi.hip): every step
//    x_i += dx_i dT for each state element (no re-projection onto SO(3), ForwardEuler.tpp:37-45).
//    The base pose lives in registers for the whole integration; the joint coordinates are
//    independent of it and are stepped one at a time.
// Layout: pos [B][3], rot [B][9] row-major, joints [B][n], twist [B][6], joint_vel [B][n].
// Built with -ffp-contract=off; same expression order as oracle/blf_oracle_contact.c.
#include "blf_internal.h"
#include "fbk_math.h"

namespace blf {
namespace {

__global__ __launch_bounds__(256) void fbk_dynamics_kernel(
    int n, double rho, const double* __restrict__ rot, const double* __restrict__ twist,
    const double* __restrict__ joint_vel, double* __restrict__ dpos, double* __restrict__ drot,
    double* __restrict__ djoints, int64_t batch)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= batch) return;
    double R[9], w[3], dR[9];
#pragma unroll
    for (int i = 0; i < 9; ++i) R[i] = rot[9 * q + i];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        w[i] = twist[6 * q + 3 + i];
        dpos[3 * q + i] = twist[6 * q + i];
    }
    fbk_rot_rate(rho, R, w, dR);
#pragma unroll
    for (int i = 0; i < 9; ++i) drot[9 * q + i] = dR[i];
    for (int i = 0; i < n; ++i) djoints[(int64_t)n * q + i] = joint_vel[(int64_t)n * q + i];
}

__global__ __launch_bounds__(256) void fbk_euler_kernel(
    int n, double rho, double* __restrict__ pos, double* __restrict__ rot,
    double* __restrict__ joints, const double* __restrict__ twist,
    const double* __restrict__ joint_vel, int64_t batch, int32_t nsteps, double dT,
    double dT_last)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= batch) return;
    double p[3], R[9], v[3], w[3], dR[9];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        p[i] = pos[3 * q + i];
        v[i] = twist[6 * q + i];
        w[i] = twist[6 * q + 3 + i];
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) R[i] = rot[9 * q + i];
    for (int32_t st = 0; st < nsteps; ++st) {
        const double h = st + 1 < nsteps ? dT : dT_last;
        fbk_rot_rate(rho, R, w, dR);
#pragma unroll
        for (int i = 0; i < 3; ++i) p[i] = p[i] + v[i] * h;
#pragma unroll
        for (int i = 0; i < 9; ++i) R[i] = R[i] + dR[i] * h;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) pos[3 * q + i] = p[i];
#pragma unroll
    for (int i = 0; i < 9; ++i) rot[9 * q + i] = R[i];
    for (int j = 0; j < n; ++j) {
        double s = joints[(int64_t)n * q + j];
        const double sd = joint_vel[(int64_t)n * q + j];
        for (int32_t st = 0; st < nsteps; ++st) s = s + sd * (st + 1 < nsteps ? dT : dT_last);
        joints[(int64_t)n * q + j] = s;
    }
}

}  // namespace

blf_status launch_fbk_dynamics(int n, double rho, const double* rot, const double* twist,
                               const double* joint_vel, double* dpos, double* drot,
                               double* djoints, int64_t batch, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    hipLaunchKernelGGL(fbk_dynamics_kernel, dim3((unsigned)ceil_div(batch, 256)), dim3(256), 0, s,
                       n, rho, rot, twist, joint_vel, dpos, drot, djoints, batch);
    return check_hip(hipGetLastError(), "fbk_dynamics_kernel launch");
}

blf_status launch_fbk_euler(int n, double rho, double* pos, double* rot, double* joints,
                            const double* twist, const double* joint_vel, int64_t batch,
                            int32_t nsteps, double dT, double dT_last, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    hipLaunchKernelGGL(fbk_euler_kernel, dim3((unsigned)ceil_div(batch, 256)), dim3(256), 0, s,
                       n, rho, pos, rot, joints, twist, joint_vel, batch, nsteps, dT, dT_last);
    return check_hip(hipGetLastError(), "fbk_euler_kernel launch");
}

}  // namespace blf
