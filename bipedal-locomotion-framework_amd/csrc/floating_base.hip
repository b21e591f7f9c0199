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
//    independent of it and are stepped element-parallel.
// Layout: pos [B][3], rot [B][9] row-major, joints [B][n], twist [B][6], joint_vel [B][n]; each
// workgroup stages its slab of these rows through LDS with coalesced loads and stores (slab.h).
// Built with -ffp-contract=off; same expression order as oracle/blf_oracle_contact.c.
#include "blf_internal.h"
#include "fbk_math.h"
#include "slab.h"

namespace blf {
namespace {

constexpr int kFbkBlock = 256;
constexpr int kFbkU = 4;

// one workgroup = 256 consecutive systems; rot / twist slabs staged through LDS (slab.h), the
// rotation rate written over the system's own rot row, dpos taken from the twist rows.
__global__ __launch_bounds__(kFbkBlock) void fbk_dynamics_kernel(
    int n, double rho, const double* __restrict__ rot, const double* __restrict__ twist,
    const double* __restrict__ joint_vel, double* __restrict__ dpos, double* __restrict__ drot,
    double* __restrict__ djoints, int64_t batch)
{
    __shared__ double s_rot[kFbkBlock * 9];
    __shared__ double s_tw[kFbkBlock * 7];
    const int t = threadIdx.x;
    const int64_t q0 = (int64_t)blockIdx.x * kFbkBlock;
    const int rows = (int)((batch - q0) < kFbkBlock ? (batch - q0) : kFbkBlock);
    slab_load<kFbkBlock, kFbkU>(s_rot, 9, rot + 9 * q0, 9, rows, 9);
    slab_load<kFbkBlock, kFbkU>(s_tw, 7, twist + 6 * q0, 6, rows, 6);
    if (n > 0) slab_copy<kFbkBlock, kFbkU>(djoints + n * q0, joint_vel + n * q0, rows * n);
    __syncthreads();
    if (t < rows) {
        double R[9], w[3], dR[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) R[i] = s_rot[9 * t + i];
#pragma unroll
        for (int i = 0; i < 3; ++i) w[i] = s_tw[7 * t + 3 + i];
        fbk_rot_rate(rho, R, w, dR);
#pragma unroll
        for (int i = 0; i < 9; ++i) s_rot[9 * t + i] = dR[i];
    }
    __syncthreads();
    slab_store<kFbkBlock, kFbkU>(drot + 9 * q0, 9, s_rot, 9, rows, 9);
    slab_store<kFbkBlock, kFbkU>(dpos + 3 * q0, 3, s_tw, 7, rows, 3);
}

// pos / rot / twist staged as above; the base pose stays in registers for the whole
// integration.  The joint coordinates are independent of the base: each lane steps consecutive
// elements of the workgroup's contiguous [rows][n] slab.
__global__ __launch_bounds__(kFbkBlock) void fbk_euler_kernel(
    int n, double rho, double* __restrict__ pos, double* __restrict__ rot,
    double* __restrict__ joints, const double* __restrict__ twist,
    const double* __restrict__ joint_vel, int64_t batch, int32_t nsteps, double dT,
    double dT_last)
{
    __shared__ double s_rot[kFbkBlock * 9];
    __shared__ double s_tw[kFbkBlock * 7];
    __shared__ double s_pos[kFbkBlock * 3];
    const int t = threadIdx.x;
    const int64_t q0 = (int64_t)blockIdx.x * kFbkBlock;
    const int rows = (int)((batch - q0) < kFbkBlock ? (batch - q0) : kFbkBlock);
    slab_load<kFbkBlock, kFbkU>(s_rot, 9, rot + 9 * q0, 9, rows, 9);
    slab_load<kFbkBlock, kFbkU>(s_tw, 7, twist + 6 * q0, 6, rows, 6);
    slab_load<kFbkBlock, kFbkU>(s_pos, 3, pos + 3 * q0, 3, rows, 3);
    __syncthreads();
    if (t < rows) {
        double p[3], R[9], v[3], w[3], dR[9];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            p[i] = s_pos[3 * t + i];
            v[i] = s_tw[7 * t + i];
            w[i] = s_tw[7 * t + 3 + i];
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) R[i] = s_rot[9 * t + i];
        for (int32_t st = 0; st < nsteps; ++st) {
            const double h = st + 1 < nsteps ? dT : dT_last;
            fbk_rot_rate(rho, R, w, dR);
#pragma unroll
            for (int i = 0; i < 3; ++i) p[i] = p[i] + v[i] * h;
#pragma unroll
            for (int i = 0; i < 9; ++i) R[i] = R[i] + dR[i] * h;
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) s_pos[3 * t + i] = p[i];
#pragma unroll
        for (int i = 0; i < 9; ++i) s_rot[9 * t + i] = R[i];
    }
    // joints: n * rows contiguous elements, kFbkU in flight per lane
    const int nj = n * rows;
    double* js = joints + n * q0;
    const double* jv = joint_vel + n * q0;
    for (int base = 0; base < nj; base += kFbkU * kFbkBlock) {
        double s[kFbkU], sd[kFbkU];
#pragma unroll
        for (int u = 0; u < kFbkU; ++u) {
            const int e = base + u * kFbkBlock + t;
            if (e < nj) {
                s[u] = js[e];
                sd[u] = jv[e];
            }
        }
#pragma unroll
        for (int u = 0; u < kFbkU; ++u) {
            const int e = base + u * kFbkBlock + t;
            if (e < nj) {
                double x = s[u];
                for (int32_t st = 0; st < nsteps; ++st) x = x + sd[u] * (st + 1 < nsteps ? dT : dT_last);
                js[e] = x;
            }
        }
    }
    __syncthreads();
    slab_store<kFbkBlock, kFbkU>(rot + 9 * q0, 9, s_rot, 9, rows, 9);
    slab_store<kFbkBlock, kFbkU>(pos + 3 * q0, 3, s_pos, 3, rows, 3);
}

}  // namespace

blf_status launch_fbk_dynamics(int n, double rho, const double* rot, const double* twist,
                               const double* joint_vel, double* dpos, double* drot,
                               double* djoints, int64_t batch, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    hipLaunchKernelGGL(fbk_dynamics_kernel, dim3((unsigned)ceil_div(batch, kFbkBlock)),
                       dim3(kFbkBlock), 0, s,
                       n, rho, rot, twist, joint_vel, dpos, drot, djoints, batch);
    return check_hip(hipGetLastError(), "fbk_dynamics_kernel launch");
}

blf_status launch_fbk_euler(int n, double rho, double* pos, double* rot, double* joints,
                            const double* twist, const double* joint_vel, int64_t batch,
                            int32_t nsteps, double dT, double dT_last, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    hipLaunchKernelGGL(fbk_euler_kernel, dim3((unsigned)ceil_div(batch, kFbkBlock)),
                       dim3(kFbkBlock), 0, s,
                       n, rho, pos, rot, joints, twist, joint_vel, batch, nsteps, dT, dT_last);
    return check_hip(hipGetLastError(), "fbk_euler_kernel launch");
}

}  // namespace blf
