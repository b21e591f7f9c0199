/*
 * blf_oracle_contact.c — TEST INFRASTRUCTURE ONLY (see blf_oracle.h).  CPU restatement of the
 * closed-loop rows of SURVEY.md 8(a) (config 5), fp64, -ffp-contract=off, in the expression order
 * the device kernels use (csrc/contact_model.hip, csrc/floating_base.hip):
 *
 *   orc_contact_eval         ContactModels/src/ContinuousContactModel.cpp:79-108 (wrench),
 *                            :110-146 (autonomous dynamics, R22 WITHOUT abs as in :127-144),
 *                            :148-171 (control matrix), :223-254 (regressor)
 *   orc_contact_point        ContinuousContactModel.cpp:173-221 (force / torque at a point)
 *   orc_fbk_dynamics         System/src/FloatingBaseSystemKinematics.cpp:36-73
 *   orc_fbk_euler_integrate  the same under ForwardEuler + the FixedStepIntegrator schedule
 *                            (FixedStepIntegrator.tpp:21-72, ForwardEuler.tpp:18-49)
 *
 * The reference cannot be built here (Eigen / iDynTree absent), so these are pinned by the
 * reference's own test properties (ContactModels/tests/ContinousContactModelTest.cpp: Monte Carlo
 * integral of the point forces, the regressor identity, finite-difference consistency of the
 * wrench rate) and by closed forms for the kinematics (orthonormal R: dR = skew(w) R).
 */
#include "blf_oracle.h"

#include <math.h>

static void cross(const double* a, const double* b, double* o)
{
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

/* skew(e)^2 = e e^T - |e|^2 I */
static void skew2(const double* e, double* S)
{
    const double n = (e[0] * e[0] + e[1] * e[1]) + e[2] * e[2];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) S[3 * i + j] = i == j ? e[i] * e[j] - n : e[i] * e[j];
}

void orc_contact_eval(const double* prm, const double* twist, const double* pose,
                      const double* null_pose, double* wrench, double* autonomous,
                      double* control, double* regressor)
{
    const double L = prm[0], W = prm[1], k = prm[2], b = prm[3];
    const double area = L * W;
    const double LL = L * L, WW = W * W;
    const double* v = twist;
    const double* w = twist + 3;
    const double* p = pose;
    const double* R = pose + 3;
    const double* p0 = null_pose;
    const double* R0 = null_pose + 3;
    const double e1[3] = {R[0], R[3], R[6]}, e2[3] = {R[1], R[4], R[7]};
    const double r01[3] = {R0[0], R0[3], R0[6]}, r02[3] = {R0[1], R0[4], R0[7]};
    const double R22 = R[8];
    const double aR = fabs(R22);
    double t1[3], t2[3], c1[3], c2[3], u1[3], u2[3];
    cross(e1, r01, t1);
    cross(e2, r02, t2);
    cross(e1, w, c1);
    cross(e2, w, c2);
    cross(e1, c1, u1);                     /* skew(e1) skew(e1) w */
    cross(e2, c2, u2);
    if (wrench) {
        const double cf = aR * area;
        const double ct = aR * area / 12.0;
        for (int i = 0; i < 3; ++i) {
            wrench[i] = cf * (k * (p0[i] - p[i]) - b * v[i]);
            wrench[3 + i] = ct * (LL * (b * u1[i] + k * t1[i]) + WW * (b * u2[i] + k * t2[i]));
        }
    }
    if (autonomous) {
        const double c2col[3] = {R[2], R[5], R[8]};
        double rd2[3], ed1[3], ed2[3];
        cross(w, c2col, rd2);                /* (skew(w) R) e3 */
        cross(w, e1, ed1);
        cross(w, e2, ed2);
        const double Rd22 = rd2[2];
        double q1[3], q2[3], g1[3], g2[3], h1[3], h2[3], tmp[3];
        cross(ed1, r01, q1);
        cross(ed2, r02, q2);
        cross(ed1, c1, g1);                  /* skew(ed1) skew(e1) w */
        cross(ed1, w, tmp);
        cross(e1, tmp, h1);                  /* skew(e1) skew(ed1) w */
        cross(ed2, c2, g2);
        cross(ed2, w, tmp);
        cross(e2, tmp, h2);
        for (int i = 0; i < 3; ++i) {
            autonomous[i] = area * (Rd22 * (k * (p0[i] - p[i]) - b * v[i]) - (R22 * k) * v[i]);
            const double X = LL * (b * u1[i] + k * t1[i]) + WW * (b * u2[i] + k * t2[i]);
            const double Y = LL * (k * q1[i] + b * (g1[i] + h1[i]))
                             + WW * (k * q2[i] + b * (g2[i] + h2[i]));
            autonomous[3 + i] = area / 12.0 * (Rd22 * X + R22 * Y);
        }
    }
    double S1[9], S2[9];
    skew2(e1, S1);
    skew2(e2, S2);
    if (control) {
        for (int i = 0; i < 36; ++i) control[i] = 0.0;
        const double d = -area * b * R22;
        const double s = area / 12.0 * R22 * b;
        for (int i = 0; i < 3; ++i) {
            control[6 * i + i] = d;
            for (int j = 0; j < 3; ++j)
                control[6 * (3 + i) + 3 + j] = s * (LL * S1[3 * i + j] + WW * S2[3 * i + j]);
        }
    }
    if (regressor) {
        const double cf = aR * area;
        const double cv = -aR * area;
        const double ct = area / 12.0 * aR;
        for (int i = 0; i < 3; ++i) {
            regressor[2 * i] = cf * (p0[i] - p[i]);
            regressor[2 * i + 1] = cv * v[i];
            regressor[2 * (3 + i)] = ct * (LL * t1[i] + WW * t2[i]);
            const double M0 = LL * S1[3 * i] + WW * S2[3 * i];
            const double M1 = LL * S1[3 * i + 1] + WW * S2[3 * i + 1];
            const double M2 = LL * S1[3 * i + 2] + WW * S2[3 * i + 2];
            regressor[2 * (3 + i) + 1] = ct * ((M0 * w[0] + M1 * w[1]) + M2 * w[2]);
        }
    }
}

void orc_contact_point(const double* prm, const double* twist, const double* pose,
                       const double* null_pose, double x, double y, double* force, double* torque)
{
    const double L = prm[0], W = prm[1], k = prm[2], b = prm[3];
    if (fabs(x) > L / 2 || fabs(y) > W / 2) {
        for (int i = 0; i < 3; ++i) { force[i] = 0.0; torque[i] = 0.0; }
        return;
    }
    const double* v = twist;
    const double* w = twist + 3;
    const double* p = pose;
    const double* R = pose + 3;
    const double* p0 = null_pose;
    const double* R0 = null_pose + 3;
    double rp[3], dp[3], vp[3], f[3];
    for (int i = 0; i < 3; ++i) {
        rp[i] = R[3 * i] * x + R[3 * i + 1] * y;                       /* R pt, pt = (x, y, 0) */
        dp[i] = (R0[3 * i] - R[3 * i]) * x + (R0[3 * i + 1] - R[3 * i + 1]) * y;
    }
    cross(w, rp, vp);                                                  /* skew(w) R pt */
    for (int i = 0; i < 3; ++i) f[i] = k * ((p0[i] - p[i]) + dp[i]) - b * (v[i] + vp[i]);
    cross(rp, f, torque);
    for (int i = 0; i < 3; ++i) force[i] = f[i];
}

void orc_fbk_dynamics(int n, double rho, const double* rot, const double* twist,
                      const double* joint_vel, double* dpos, double* drot, double* djoints)
{
    const double* R = rot;
    const double* w = twist + 3;
    for (int i = 0; i < 3; ++i) dpos[i] = twist[i];
    double S[9], C[9], D[9];
    for (int i = 0; i < 3; ++i)
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
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) D[3 * i + j] = C[3 * j + i] / det - (i == j ? 1.0 : 0.0);
    const double hr = rho / 2.0;
    for (int j = 0; j < 3; ++j) {
        const double col[3] = {R[j], R[3 + j], R[6 + j]};
        double cr[3];
        cross(col, w, cr);
        for (int i = 0; i < 3; ++i) {
            const double DR = (D[3 * i] * R[j] + D[3 * i + 1] * R[3 + j]) + D[3 * i + 2] * R[6 + j];
            drot[3 * i + j] = (-cr[i]) + hr * DR;
        }
    }
    for (int i = 0; i < n; ++i) djoints[i] = joint_vel[i];
}

static void fbk_step(int n, double rho, double* pos, double* rot, double* joints,
                     const double* twist, const double* joint_vel, double dT)
{
    double dp[3], dR[9], dq[64];
    orc_fbk_dynamics(n, rho, rot, twist, joint_vel, dp, dR, dq);
    for (int i = 0; i < 3; ++i) pos[i] = pos[i] + dp[i] * dT;
    for (int i = 0; i < 9; ++i) rot[i] = rot[i] + dR[i] * dT;
    for (int i = 0; i < n; ++i) joints[i] = joints[i] + dq[i] * dT;
}

int orc_fbk_euler_integrate(int n, double rho, double* pos, double* rot, double* joints,
                            const double* twist, const double* joint_vel, double t0, double t1,
                            double dT)
{
    if (n < 0 || n > 64) return 1;
    if (t0 > t1 || !(dT > 0)) return 4;
    if (t0 == t1) return 5;
    const double q = ceil((t1 - t0) / dT);
    if (!(q < 2.0e9)) return 3;
    const int iterations = (int)q;
    double currentTime = t0;
    for (int64_t i = 0; i < (int64_t)iterations - 1; ++i) {
        currentTime = t0 + dT * (double)i;
        fbk_step(n, rho, pos, rot, joints, twist, joint_vel, dT);
    }
    fbk_step(n, rho, pos, rot, joints, twist, joint_vel, t1 - currentTime);
    return 0;
}
