// fbk_math.h — the FloatingBaseSystemKinematics rotation rate, shared by floating_base.hip and
// fb_dynamics.hip (FloatingBaseSystemKinematics.cpp:61-70 / FloatingBaseSystemDynamics.cpp:133-138):
//   dR = -R.colwise().cross(w) + rho/2 ((R R^T)^{-1} - I) R,  (R R^T)^{-1} by cofactors.
// Expression order of oracle/blf_oracle_contact.c:orc_fbk_dynamics.
#pragma once

#include <hip/hip_runtime.h>

namespace blf {

__device__ __forceinline__ void fbk_rot_rate(double rho, const double* R, const double* w,
                                             double* dR)
{
    double S[9], C[9], D[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
            S[3 * i + j] = (R[3 * i] * R[3 * j] + R[3 * i + 1] * R[3 * j + 1]) + R[3 * i + 2] * R[3 * j + 2];
    C[0] = S[4] * S[8] - S[5] * S[7];
    C[1] = S[5] * S[6] - S[3] * S[8];
    C[2] = S[3] * S[7] - S[4] * S[6];
    C[3] = S[2] * S[7] - S[1] * S[8];
    C[4] = S[0] * S[8] - S[2] * S[6];
    C[5] = S[1] * S[6] - S[0] * S[7];
    C[6] = S[1] * S[5] - S[2] * S[4];
    C[7] = S[2] * S[3] - S[0] * S[5];
    C[8] = S[0] * S[4] - S[1] * S[3];
    const double det = (S[0] * C[0] + S[1] * C[1]) + S[2] * C[2];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) D[3 * i + j] = C[3 * j + i] / det - (i == j ? 1.0 : 0.0);
    const double hr = rho / 2.0;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        const double c0 = R[j], c1 = R[3 + j], c2 = R[6 + j];
        const double cr[3] = {c1 * w[2] - c2 * w[1], c2 * w[0] - c0 * w[2], c0 * w[1] - c1 * w[0]};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            const double DR = (D[3 * i] * R[j] + D[3 * i + 1] * R[3 + j]) + D[3 * i + 2] * R[6 + j];
            dR[3 * i + j] = (-cr[i]) + hr * DR;
        }
    }
}

}  // namespace blf
