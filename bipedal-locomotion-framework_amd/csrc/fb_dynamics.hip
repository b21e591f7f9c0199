// fb_dynamics.hip — FloatingBaseDynamicalSystem on the device.
//
// FloatingBaseSystemDynamics.cpp:102-251 takes the free-floating mass matrix M, the generalized
// bias forces h and the contact-frame Jacobians from iDynTree KinDynComputations and then solves
//   nu_dot = LLT(M [+ reg]) \ (-h + sum_c J_c^T w_c + [0; tau]).
// Here the rigid-body terms are computed directly, in the mixed representation (base velocity
// (dp_B/dt, w_B), world coordinates), for a kinematic tree of revolute joints:
//   M = sum_l m_l Jv_l^T Jv_l + Jw_l^T I_l Jw_l            (Jv at the link COM, I_l = R Ic R^T)
//   h = sum_l Jv_l^T m_l (a_l - g) + Jw_l^T (I_l al_l + w_l x I_l w_l)   (accelerations at nu_dot=0)
// One 64-lane workgroup per system.  The tree recursion (poses, velocities, bias accelerations)
// runs on lane 0 with the per-joint rotations precomputed lane-parallel; the per-link terms, the
// mass-matrix entries (one lane per (i, j) of the lower triangle, a bitmask of each link's
// ancestor joints selecting the nonzero Jacobian columns), the bias forces and the contact
// Jacobians are lane-parallel; the Cholesky factorization is right-looking with the trailing
// update spread over the lanes.  Everything lives in LDS.  The ForwardEuler kernel keeps the
// state in LDS across its steps.  Checked against the numpy restatement oracle/fb_dynamics.py.
#include "blf_internal.h"
#include "contact_math.h"
#include "fbk_math.h"

namespace blf {
namespace {

constexpr int kLinkRec = 40;   // R 9 | p 3 | w 3 | v 3 | al 3 | a 3 | c 3 | Iw 6 (xx xy xz yy yz zz) | f 3 | tq 3 | pad 1
constexpr int kR = 0, kP = 9, kW = 12, kV = 15, kAl = 18, kA = 21, kC = 24, kIw = 27, kF = 33, kTq = 36;

struct Smem {
    double *link, *jrot, *jz, *jo, *M, *rhs, *cscr, *st;
    unsigned long long* anc;
    size_t total;
    __host__ __device__ Smem(double* base, int n, int C)
    {
        const int L = n + 1, NV = n + 6;
        size_t o = 0;
        auto take = [&](size_t k) {
            double* p = base ? base + o : nullptr;
            o += (k + 1) & ~size_t(1);
            return p;
        };
        link = take((size_t)kLinkRec * L);
        jrot = take(12 * (size_t)n);           // E_j Rot(a_j, s_j) (9) | E_j a_j (3)
        jz = take(3 * (size_t)n);
        jo = take(3 * (size_t)n);
        M = take((size_t)NV * NV);
        rhs = take((size_t)NV);
        cscr = take(16 * (size_t)(C > 0 ? C : 1));   // per contact: point (3) | wrench (6) | link (1)
        st = take(18 + 2 * (size_t)n + (size_t)NV + 9);   // Euler state (6 + n + 3 + 9 + n) + acc + dR
        anc = reinterpret_cast<unsigned long long*>(take((size_t)L));
        total = o;
    }
};

struct Model {
    int n, F;
    const int32_t* parent;
    const double *jorig, *jrot, *jaxis, *mass, *com, *inertia, *fpose;
    const int32_t* flink;
    double g0, g1, g2, rho;
};

struct Contacts {
    int C;
    const int32_t* frame;
    const double* params;
    const double* null_pose;   // [B][C][12]
};

__device__ __forceinline__ void cross3(const double* a, const double* b, double* o)
{
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

// Jacobian column `col` (mixed) of a point x rigidly attached to a link: linear jv, angular jw.
// Caller guarantees the column is visible from the link (base column or an ancestor joint).
__device__ __forceinline__ void jac_col(const Smem& S, int col, const double* x, const double* pB,
                                        double* jv, double* jw)
{
    if (col < 3) {
        jv[0] = col == 0 ? 1.0 : 0.0; jv[1] = col == 1 ? 1.0 : 0.0; jv[2] = col == 2 ? 1.0 : 0.0;
        jw[0] = jw[1] = jw[2] = 0.0;
    } else if (col < 6) {
        const int i = col - 3;
        const double e[3] = {i == 0 ? 1.0 : 0.0, i == 1 ? 1.0 : 0.0, i == 2 ? 1.0 : 0.0};
        const double d[3] = {x[0] - pB[0], x[1] - pB[1], x[2] - pB[2]};
        cross3(e, d, jv);                       // column i of -skew(x - p_B)
        jw[0] = e[0]; jw[1] = e[1]; jw[2] = e[2];
    } else {
        const int j = col - 6;
        const double* z = S.jz + 3 * j;
        const double d[3] = {x[0] - S.jo[3 * j], x[1] - S.jo[3 * j + 1], x[2] - S.jo[3 * j + 2]};
        cross3(z, d, jv);
        jw[0] = z[0]; jw[1] = z[1]; jw[2] = z[2];
    }
}

__device__ __forceinline__ bool visible(const Smem& S, int col, int link)
{
    return col < 6 || ((S.anc[link] >> (col - 6)) & 1ull);
}

// sym 3x3 (xx xy xz yy yz zz) times vector
__device__ __forceinline__ void sym_mv(const double* I, const double* x, double* y)
{
    y[0] = (I[0] * x[0] + I[1] * x[1]) + I[2] * x[2];
    y[1] = (I[1] * x[0] + I[3] * x[1]) + I[4] * x[2];
    y[2] = (I[2] * x[0] + I[4] * x[1]) + I[5] * x[2];
}

// One evaluation of the dynamics for the system whose state sits in LDS (bv, jv, bp, bR, jp).
// Leaves the generalized acceleration in S.rhs and returns false if the factorization failed.
__device__ bool fbd_eval(const Model& m, const Smem& S, const double* bv, const double* jvel,
                         const double* bp, const double* bR, const double* jp,
                         const double* tau, const Contacts& ct, int64_t sys, const double* reg)
{
    const int n = m.n, L = n + 1, NV = n + 6;
    const int lane = threadIdx.x;
    // 1. per-joint rotation E_j Rot(a_j, s_j) (Rodrigues) and E_j a_j, lane-parallel
    for (int j = lane; j < n; j += kWave) {
        const double* a = m.jaxis + 3 * j;
        const double* E = m.jrot + 9 * j;
        double sn, cs;
        sincos(jp[j], &sn, &cs);
        const double c1 = 1.0 - cs;
        const double K[9] = {0.0, -a[2], a[1], a[2], 0.0, -a[0], -a[1], a[0], 0.0};
        double Rr[9];
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const double K2 = (K[3 * r] * K[c] + K[3 * r + 1] * K[3 + c]) + K[3 * r + 2] * K[6 + c];
                Rr[3 * r + c] = ((r == c ? 1.0 : 0.0) + sn * K[3 * r + c]) + c1 * K2;
            }
        double* out = S.jrot + 12 * j;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
#pragma unroll
            for (int c = 0; c < 3; ++c)
                out[3 * r + c] = (E[3 * r] * Rr[c] + E[3 * r + 1] * Rr[3 + c]) + E[3 * r + 2] * Rr[6 + c];
            out[9 + r] = (E[3 * r] * a[0] + E[3 * r + 1] * a[1]) + E[3 * r + 2] * a[2];
        }
    }
    __syncthreads();
    // 2. tree recursion on lane 0: poses, mixed velocities, nu_dot = 0 accelerations
    if (lane == 0) {
        double* b = S.link;
        for (int i = 0; i < 9; ++i) b[kR + i] = bR[i];
        for (int i = 0; i < 3; ++i) {
            b[kP + i] = bp[i]; b[kV + i] = bv[i]; b[kW + i] = bv[3 + i];
            b[kAl + i] = 0.0; b[kA + i] = 0.0;
        }
        S.anc[0] = 0ull;
        for (int j = 0; j < n; ++j) {
            const int P = m.parent[j];
            const double* pr = S.link + kLinkRec * P;
            double* cr = S.link + kLinkRec * (j + 1);
            const double* Ej = S.jrot + 12 * j;
            const double* o = m.jorig + 3 * j;
            const double* RP = pr + kR;
            double r[3], z[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    cr[kR + 3 * a + c] = (RP[3 * a] * Ej[c] + RP[3 * a + 1] * Ej[3 + c]) + RP[3 * a + 2] * Ej[6 + c];
                r[a] = (RP[3 * a] * o[0] + RP[3 * a + 1] * o[1]) + RP[3 * a + 2] * o[2];
                z[a] = (RP[3 * a] * Ej[9] + RP[3 * a + 1] * Ej[10]) + RP[3 * a + 2] * Ej[11];
            }
            const double sd = jvel[j];
            const double zs[3] = {z[0] * sd, z[1] * sd, z[2] * sd};
            double t1[3], t2[3], t3[3];
            cross3(pr + kW, r, t1);            // w_P x r
            cross3(pr + kW, zs, t2);           // w_P x z sd
            for (int a = 0; a < 3; ++a) {
                cr[kP + a] = pr[kP + a] + r[a];
                S.jz[3 * j + a] = z[a];
                S.jo[3 * j + a] = cr[kP + a];
                cr[kW + a] = pr[kW + a] + zs[a];
                cr[kV + a] = pr[kV + a] + t1[a];
                cr[kAl + a] = pr[kAl + a] + t2[a];
            }
            cross3(pr + kAl, r, t2);           // al_P x r
            cross3(pr + kW, t1, t3);           // w_P x (w_P x r)
            for (int a = 0; a < 3; ++a) cr[kA + a] = (pr[kA + a] + t2[a]) + t3[a];
            S.anc[j + 1] = S.anc[P] | (1ull << j);
        }
    }
    __syncthreads();
    // 3. per-link COM, world inertia, Newton-Euler force / moment (lane-parallel)
    for (int l = lane; l < L; l += kWave) {
        double* k = S.link + kLinkRec * l;
        const double* R = k + kR;
        const double* cl = m.com + 3 * l;
        const double* Ic = m.inertia + 9 * l;
        double rc[3];
        for (int a = 0; a < 3; ++a) {
            rc[a] = (R[3 * a] * cl[0] + R[3 * a + 1] * cl[1]) + R[3 * a + 2] * cl[2];
            k[kC + a] = k[kP + a] + rc[a];
        }
        double RI[9];   // R Ic
        for (int a = 0; a < 3; ++a)
            for (int c = 0; c < 3; ++c)
                RI[3 * a + c] = (R[3 * a] * Ic[c] + R[3 * a + 1] * Ic[3 + c]) + R[3 * a + 2] * Ic[6 + c];
        const int ii[6] = {0, 0, 0, 1, 1, 2}, jj[6] = {0, 1, 2, 1, 2, 2};
        for (int e = 0; e < 6; ++e) {
            const int a = ii[e], c = jj[e];
            k[kIw + e] = (RI[3 * a] * R[3 * c] + RI[3 * a + 1] * R[3 * c + 1]) + RI[3 * a + 2] * R[3 * c + 2];
        }
        double t1[3], t2[3], t3[3];
        cross3(k + kAl, rc, t1);
        cross3(k + kW, rc, t2);
        cross3(k + kW, t2, t3);
        const double ms = m.mass[l];
        const double g[3] = {m.g0, m.g1, m.g2};
        for (int a = 0; a < 3; ++a) k[kF + a] = ms * (((k[kA + a] + t1[a]) + t3[a]) - g[a]);
        double Ia[3], Iw[3];
        sym_mv(k + kIw, k + kAl, Ia);
        sym_mv(k + kIw, k + kW, Iw);
        cross3(k + kW, Iw, t1);
        for (int a = 0; a < 3; ++a) k[kTq + a] = Ia[a] + t1[a];
    }
    __syncthreads();
    const double* pB = S.link + kP;
    // 4. mass matrix, lower triangle, one lane per entry
    const int ntri = NV * (NV + 1) / 2;
    for (int e = lane; e < ntri; e += kWave) {
        int i = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
        while ((i + 1) * (i + 2) / 2 <= e) ++i;
        while (i * (i + 1) / 2 > e) --i;
        const int j = e - i * (i + 1) / 2;
        double acc = 0.0;
        for (int l = 0; l < L; ++l) {
            if (!visible(S, i, l) || !visible(S, j, l)) continue;
            const double* k = S.link + kLinkRec * l;
            double vi[3], wi[3], vj[3], wj[3], Iwj[3];
            jac_col(S, i, k + kC, pB, vi, wi);
            jac_col(S, j, k + kC, pB, vj, wj);
            sym_mv(k + kIw, wj, Iwj);
            acc = acc + (m.mass[l] * ((vi[0] * vj[0] + vi[1] * vj[1]) + vi[2] * vj[2])
                         + ((wi[0] * Iwj[0] + wi[1] * Iwj[1]) + wi[2] * Iwj[2]));
        }
        S.M[NV * i + j] = acc + (reg ? reg[NV * i + j] : 0.0);
    }
    // 5. bias forces, one lane per generalized coordinate
    for (int c = lane; c < NV; c += kWave) {
        double h = 0.0;
        for (int l = 0; l < L; ++l) {
            if (!visible(S, c, l)) continue;
            const double* k = S.link + kLinkRec * l;
            double jv[3], jw[3];
            jac_col(S, c, k + kC, pB, jv, jw);
            h = h + (((jv[0] * k[kF] + jv[1] * k[kF + 1]) + jv[2] * k[kF + 2])
                     + ((jw[0] * k[kTq] + jw[1] * k[kTq + 1]) + jw[2] * k[kTq + 2]));
        }
        S.rhs[c] = (-h) + (c >= 6 ? tau[c - 6] : 0.0);
    }
    // 6. contacts: frame state + ContinuousContactModel wrench (lane c), then J_c^T w (lanes)
    for (int c = lane; c < ct.C; c += kWave) {
        const int f = ct.frame[c];
        const int l = m.flink[f];
        const double* k = S.link + kLinkRec * l;
        const double* fp = m.fpose + 12 * f;
        const double* R = k + kR;
        double pose[12], tw[6], d[3], t1[3];
        for (int a = 0; a < 3; ++a) {
            pose[a] = k[kP + a] + ((R[3 * a] * fp[0] + R[3 * a + 1] * fp[1]) + R[3 * a + 2] * fp[2]);
            for (int b = 0; b < 3; ++b)
                pose[3 + 3 * a + b] = (R[3 * a] * fp[3 + b] + R[3 * a + 1] * fp[6 + b]) + R[3 * a + 2] * fp[9 + b];
            d[a] = pose[a] - k[kP + a];
        }
        cross3(k + kW, d, t1);
        for (int a = 0; a < 3; ++a) {
            tw[a] = k[kV + a] + t1[a];
            tw[3 + a] = k[kW + a];
        }
        double* sc = S.cscr + 16 * c;
        contact_wrench(ct.params + 4 * c, tw, pose, ct.null_pose + (sys * ct.C + c) * 12, sc + 3);
        sc[0] = pose[0]; sc[1] = pose[1]; sc[2] = pose[2];
        sc[9] = (double)l;
    }
    __syncthreads();
    for (int col = lane; col < NV; col += kWave) {
        double add = 0.0;
        for (int c = 0; c < ct.C; ++c) {
            const double* sc = S.cscr + 16 * c;
            const int l = (int)sc[9];
            if (!visible(S, col, l)) continue;
            double jv[3], jw[3];
            jac_col(S, col, sc, pB, jv, jw);
            add = add + (((jv[0] * sc[3] + jv[1] * sc[4]) + jv[2] * sc[5])
                         + ((jw[0] * sc[6] + jw[1] * sc[7]) + jw[2] * sc[8]));
        }
        S.rhs[col] = S.rhs[col] + add;
    }
    __syncthreads();
    // 7. Cholesky M = L L^T (lower, in place), right-looking
    bool ok = true;
    for (int k = 0; k < NV; ++k) {
        const double piv = S.M[NV * k + k];
        ok = ok && (piv > 0.0);
        const double d = sqrt(piv);
        __syncthreads();
        for (int i = k + 1 + lane; i < NV; i += kWave) S.M[NV * i + k] = S.M[NV * i + k] / d;
        if (lane == 0) S.M[NV * k + k] = d;
        __syncthreads();
        const int rem = NV - k - 1;
        const int nup = rem * (rem + 1) / 2;
        for (int e = lane; e < nup; e += kWave) {
            int i = (int)((sqrt(8.0 * e + 1.0) - 1.0) * 0.5);
            while ((i + 1) * (i + 2) / 2 <= e) ++i;
            while (i * (i + 1) / 2 > e) --i;
            const int j = e - i * (i + 1) / 2;
            const int I = k + 1 + i, J = k + 1 + j;
            S.M[NV * I + J] = S.M[NV * I + J] - S.M[NV * I + k] * S.M[NV * J + k];
        }
        __syncthreads();
    }
    // 8. forward / back substitution on lane 0
    if (lane == 0) {
        for (int i = 0; i < NV; ++i) {
            double s = S.rhs[i];
            for (int k = 0; k < i; ++k) s = s - S.M[NV * i + k] * S.rhs[k];
            S.rhs[i] = s / S.M[NV * i + i];
        }
        for (int i = NV - 1; i >= 0; --i) {
            double s = S.rhs[i];
            for (int k = i + 1; k < NV; ++k) s = s - S.M[NV * k + i] * S.rhs[k];
            S.rhs[i] = s / S.M[NV * i + i];
        }
    }
    __syncthreads();
    return ok;
}

__global__ __launch_bounds__(64) void fbd_dynamics_kernel(Model m, blf_fb_state st,
                                                          const double* __restrict__ tau,
                                                          Contacts ct, const double* reg,
                                                          blf_fb_state out)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int n = m.n, NV = n + 6;
    const Smem S(smem, n, ct.C);
    const int64_t q = blockIdx.x;
    const int lane = threadIdx.x;
    double* loc = S.st;   // bv 6 | jv n | bp 3 | bR 9 | jp n
    for (int i = lane; i < 18 + 2 * n; i += kWave) {
        double v;
        if (i < 6) v = st.base_vel[6 * q + i];
        else if (i < 6 + n) v = st.joint_vel[(int64_t)n * q + (i - 6)];
        else if (i < 9 + n) v = st.base_pos[3 * q + (i - 6 - n)];
        else if (i < 18 + n) v = st.base_rot[9 * q + (i - 9 - n)];
        else v = st.joint_pos[(int64_t)n * q + (i - 18 - n)];
        loc[i] = v;
    }
    __syncthreads();
    const bool ok = fbd_eval(m, S, loc, loc + 6, loc + 6 + n, loc + 9 + n, loc + 18 + n,
                             tau + (int64_t)n * q, ct, q, reg);
    const double nan = __builtin_nan("");
    for (int c = lane; c < NV; c += kWave) {
        const double a = ok ? S.rhs[c] : nan;
        if (c < 6) out.base_vel[6 * q + c] = a;
        else out.joint_vel[(int64_t)n * q + (c - 6)] = a;
    }
    if (lane == 0) {
        double dR[9];
        fbk_rot_rate(m.rho, loc + 9 + n, loc + 3, dR);
        for (int i = 0; i < 3; ++i) out.base_pos[3 * q + i] = loc[i];
        for (int i = 0; i < 9; ++i) out.base_rot[9 * q + i] = dR[i];
    }
    for (int j = lane; j < n; j += kWave) out.joint_pos[(int64_t)n * q + j] = loc[6 + j];
}

__global__ __launch_bounds__(64) void fbd_euler_kernel(Model m, blf_fb_state st,
                                                       const double* __restrict__ tau,
                                                       Contacts ct, const double* reg,
                                                       int32_t nsteps, double dT, double dT_last)
{
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int n = m.n, NV = n + 6;
    const Smem S(smem, n, ct.C);
    const int64_t q = blockIdx.x;
    const int lane = threadIdx.x;
    double* loc = S.st;   // bv 6 | jv n | bp 3 | bR 9 | jp n | dR 9
    double* dR = loc + 18 + 2 * n;
    for (int i = lane; i < 18 + 2 * n; i += kWave) {
        double v;
        if (i < 6) v = st.base_vel[6 * q + i];
        else if (i < 6 + n) v = st.joint_vel[(int64_t)n * q + (i - 6)];
        else if (i < 9 + n) v = st.base_pos[3 * q + (i - 6 - n)];
        else if (i < 18 + n) v = st.base_rot[9 * q + (i - 9 - n)];
        else v = st.joint_pos[(int64_t)n * q + (i - 18 - n)];
        loc[i] = v;
    }
    __syncthreads();
    bool ok = true;
    for (int32_t step = 0; step < nsteps; ++step) {
        const double h = step + 1 < nsteps ? dT : dT_last;
        ok = fbd_eval(m, S, loc, loc + 6, loc + 6 + n, loc + 9 + n, loc + 18 + n,
                      tau + (int64_t)n * q, ct, q, reg) && ok;
        if (lane == 0) fbk_rot_rate(m.rho, loc + 9 + n, loc + 3, dR);
        __syncthreads();
        // every element moves by its derivative at the start of the step (ForwardEuler.tpp:37-45):
        // positions first (they read the old velocities), then the velocities
        for (int i = lane; i < 12 + n; i += kWave) {
            // base position (3), base rotation (9), joint positions (n)
            if (i < 3) loc[6 + n + i] = loc[6 + n + i] + loc[i] * h;
            else if (i < 12) loc[6 + n + i] = loc[6 + n + i] + dR[i - 3] * h;
            else loc[18 + n + (i - 12)] = loc[18 + n + (i - 12)] + loc[6 + (i - 12)] * h;
        }
        __syncthreads();
        for (int i = lane; i < NV; i += kWave) loc[i] = loc[i] + S.rhs[i] * h;
        __syncthreads();
    }
    const double nan = __builtin_nan("");
    for (int i = lane; i < 18 + 2 * n; i += kWave) {
        const double v = ok ? loc[i] : nan;
        if (i < 6) st.base_vel[6 * q + i] = v;
        else if (i < 6 + n) st.joint_vel[(int64_t)n * q + (i - 6)] = v;
        else if (i < 9 + n) st.base_pos[3 * q + (i - 6 - n)] = v;
        else if (i < 18 + n) st.base_rot[9 * q + (i - 9 - n)] = v;
        else st.joint_pos[(int64_t)n * q + (i - 18 - n)] = v;
    }
}

Model to_model(const blf_fb_model* md)
{
    Model m;
    m.n = md->ndof;
    m.F = md->nframes;
    m.parent = md->parent;
    m.jorig = md->joint_origin;
    m.jrot = md->joint_rot;
    m.jaxis = md->joint_axis;
    m.mass = md->link_mass;
    m.com = md->link_com;
    m.inertia = md->link_inertia;
    m.flink = md->frame_link;
    m.fpose = md->frame_pose;
    m.g0 = md->gravity[0];
    m.g1 = md->gravity[1];
    m.g2 = md->gravity[2];
    m.rho = md->rho;
    return m;
}

Contacts to_contacts(const blf_fb_contacts* c)
{
    Contacts o;
    o.C = c ? c->ncontacts : 0;
    o.frame = c ? c->frame : nullptr;
    o.params = c ? c->params : nullptr;
    o.null_pose = c ? c->null_pose : nullptr;
    return o;
}

}  // namespace

size_t fbd_lds_bytes(int n, int C) { return sizeof(double) * Smem(nullptr, n, C).total; }

blf_status launch_fbd_dynamics(const blf_fb_model* md, const blf_fb_state* st, const double* tau,
                               const blf_fb_contacts* ct, const double* reg, int64_t batch,
                               const blf_fb_state* out, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    const Contacts c = to_contacts(ct);
    hipLaunchKernelGGL(fbd_dynamics_kernel, dim3((unsigned)batch), dim3(kWave),
                       fbd_lds_bytes(md->ndof, c.C), s, to_model(md), *st, tau, c, reg, *out);
    return check_hip(hipGetLastError(), "fbd_dynamics_kernel launch");
}

blf_status launch_fbd_euler(const blf_fb_model* md, const blf_fb_state* st, const double* tau,
                            const blf_fb_contacts* ct, const double* reg, int64_t batch,
                            int32_t nsteps, double dT, double dT_last, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    const Contacts c = to_contacts(ct);
    hipLaunchKernelGGL(fbd_euler_kernel, dim3((unsigned)batch), dim3(kWave),
                       fbd_lds_bytes(md->ndof, c.C), s, to_model(md), *st, tau, c, reg, nsteps,
                       dT, dT_last);
    return check_hip(hipGetLastError(), "fbd_euler_kernel launch");
}

}  // namespace blf
