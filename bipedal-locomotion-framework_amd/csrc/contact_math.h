// contact_math.h — device helpers shared by the kernels that evaluate the ContinuousContactModel
// wrench (contact_model.hip, fb_dynamics.hip): ContinuousContactModel.cpp:79-108, expression order
// of oracle/blf_oracle_contact.c.
#pragma once

#include <hip/hip_runtime.h>

namespace blf {

struct V3 {
    double x, y, z;
};

__device__ __forceinline__ V3 cross(V3 a, V3 b)
{
    return V3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ double at(const V3& a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }

// pr = {L, W, k, b}; tw = {v, w} (mixed); ps, ns = {p, R row-major}; out = {force, torque}
__device__ __forceinline__ void contact_wrench(const double* pr, const double* tw, const double* ps,
                                               const double* ns, double* out)
{
    const double L = pr[0], W = pr[1], k = pr[2], b = pr[3];
    const double area = L * W;
    const double LL = L * L, WW = W * W;
    const double* R = ps + 3;
    const double* R0 = ns + 3;
    const V3 w{tw[3], tw[4], tw[5]};
    const V3 e1{R[0], R[3], R[6]}, e2{R[1], R[4], R[7]};
    const V3 r01{R0[0], R0[3], R0[6]}, r02{R0[1], R0[4], R0[7]};
    const double aR = fabs(R[8]);
    const V3 t1 = cross(e1, r01), t2 = cross(e2, r02);
    const V3 u1 = cross(e1, cross(e1, w)), u2 = cross(e2, cross(e2, w));
    const double cf = aR * area;
    const double ct = aR * area / 12.0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        out[i] = cf * (k * (ns[i] - ps[i]) - b * tw[i]);
        out[3 + i] = ct * (LL * (b * at(u1, i) + k * at(t1, i)) + WW * (b * at(u2, i) + k * at(t2, i)));
    }
}

}  // namespace blf
