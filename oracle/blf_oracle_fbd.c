/* TEST INFRASTRUCTURE ONLY (oracle): plain-C restatement of FloatingBaseDynamicalSystem::dynamics
 * (reference src/System/src/FloatingBaseSystemDynamics.cpp:102-251) for the synthetic tree of
 * blf/robot.py, and of ForwardEuler<FloatingBaseDynamicalSystem>::integrate with the closed loop's
 * joint impedance set before every step (FixedStepIntegrator.tpp:21-72, ForwardEuler.tpp:18-49).
 * It is the same algorithm as oracle/fb_dynamics.py (the rigid-body terms in the Jacobian form of
 * the MIXED representation, then the reference's algebra: known = -h + sum_c J_c^T w_c,
 * known[6:] += tau, nu_dot = LLT(M) \ known), written in C so that bench.py's configs[4] CPU
 * baseline times a compiled port instead of numpy.  tests/test_oracle_closed_loop.py checks it
 * against the numpy restatement (parity against iDynTree stays unpinned).
 *
 * Model arrays (blf_fb_model's layout): parent[n] (link of joint j's parent; joint j moves link
 * j + 1), joint_origin[n][3], joint_rot[n][9], joint_axis[n][3], link_mass[n+1], link_com[n+1][3],
 * link_inertia[n+1][9], frame_link[F], frame_pose[F][12] (p, R row-major). */
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

#include "blf_oracle.h"

#define FB_MAXN 40
#define FB_NV (6 + FB_MAXN)

typedef struct {
    double R[FB_MAXN + 1][9], p[FB_MAXN + 1][3], w[FB_MAXN + 1][3], v[FB_MAXN + 1][3];
    double al[FB_MAXN + 1][3], a[FB_MAXN + 1][3], z[FB_MAXN][3], o[FB_MAXN][3];
} fb_kin;

static void mm3(const double* A, const double* B, double* C)
{
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) C[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
}

static void mv3(const double* A, const double* x, double* y)
{
    for (int i = 0; i < 3; ++i) y[i] = A[3 * i] * x[0] + A[3 * i + 1] * x[1] + A[3 * i + 2] * x[2];
}

static void cross3(const double* a, const double* b, double* c)
{
    const double c0 = a[1] * b[2] - a[2] * b[1], c1 = a[2] * b[0] - a[0] * b[2], c2 = a[0] * b[1] - a[1] * b[0];
    c[0] = c0; c[1] = c1; c[2] = c2;
}

/* Rodrigues: I + sin(q) K + (1 - cos(q)) K^2, K = skew(axis) */
static void rot_axis(const double* ax, double q, double* R)
{
    const double s = sin(q), c1 = 1.0 - cos(q);
    const double K[9] = {0, -ax[2], ax[1], ax[2], 0, -ax[0], -ax[1], ax[0], 0};
    double K2[9];
    mm3(K, K, K2);
    for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + s * K[i] + c1 * K2[i];
}

static void kinematics(const orc_fb_model* m, const double* bpos, const double* brot, const double* q,
                       const double* bvel, const double* qd, fb_kin* K)
{
    const int n = m->n;
    memcpy(K->R[0], brot, 9 * sizeof(double));
    memcpy(K->p[0], bpos, 3 * sizeof(double));
    memcpy(K->v[0], bvel, 3 * sizeof(double));
    memcpy(K->w[0], bvel + 3, 3 * sizeof(double));
    memset(K->al[0], 0, 3 * sizeof(double));
    memset(K->a[0], 0, 3 * sizeof(double));
    for (int j = 0; j < n; ++j) {
        const int P = m->parent[j], c = j + 1;
        double RE[9], Ra[9], r[3], t[3], zq[3], u[3];
        mm3(K->R[P], m->joint_rot + 9 * j, RE);
        if (m->joint_type && m->joint_type[j] == 1) {
            /* prismatic: the child slides along z = R_P E a by q (oracle/fb_dynamics.py) */
            memcpy(K->R[c], RE, 9 * sizeof(double));
            mv3(RE, m->joint_axis + 3 * j, K->z[j]);
            mv3(K->R[P], m->joint_origin + 3 * j, r);
            for (int i = 0; i < 3; ++i) {
                r[i] += K->z[j][i] * q[j];
                K->p[c][i] = K->p[P][i] + r[i];
                zq[i] = K->z[j][i] * qd[j];
                K->w[c][i] = K->w[P][i];
                K->al[c][i] = K->al[P][i];
            }
            memcpy(K->o[j], K->p[c], 3 * sizeof(double));
            cross3(K->w[P], r, t);
            for (int i = 0; i < 3; ++i) K->v[c][i] = K->v[P][i] + t[i] + zq[i];
            cross3(K->al[P], r, t);
            cross3(K->w[P], r, u);
            cross3(K->w[P], u, u);
            double wz[3];
            cross3(K->w[P], zq, wz);
            for (int i = 0; i < 3; ++i) K->a[c][i] = K->a[P][i] + t[i] + u[i] + 2.0 * wz[i];
            continue;
        }
        rot_axis(m->joint_axis + 3 * j, q[j], Ra);
        mm3(RE, Ra, K->R[c]);
        mv3(K->R[P], m->joint_origin + 3 * j, r);
        for (int i = 0; i < 3; ++i) K->p[c][i] = K->p[P][i] + r[i];
        mv3(RE, m->joint_axis + 3 * j, K->z[j]);
        memcpy(K->o[j], K->p[c], 3 * sizeof(double));
        for (int i = 0; i < 3; ++i) {
            zq[i] = K->z[j][i] * qd[j];
            K->w[c][i] = K->w[P][i] + zq[i];
        }
        cross3(K->w[P], r, t);
        for (int i = 0; i < 3; ++i) K->v[c][i] = K->v[P][i] + t[i];
        cross3(K->w[P], zq, t);
        for (int i = 0; i < 3; ++i) K->al[c][i] = K->al[P][i] + t[i];
        cross3(K->al[P], r, t);
        cross3(K->w[P], r, u);
        cross3(K->w[P], u, u);
        for (int i = 0; i < 3; ++i) K->a[c][i] = K->a[P][i] + t[i] + u[i];
    }
}

/* ancestor mask of link l: bit j set for the joints on the path base -> l */
static void ancestors(const orc_fb_model* m, unsigned long long* anc)
{
    anc[0] = 0;
    for (int j = 0; j < m->n; ++j) anc[j + 1] = anc[m->parent[j]] | (1ull << j);
}

/* mixed Jacobian (6 x NV, row-major with stride NV) of point x on link l */
static void point_jacobian(const orc_fb_model* m, const fb_kin* K, unsigned long long anc, const double* x,
                           double* J, int NV)
{
    memset(J, 0, sizeof(double) * 6 * NV);
    const double d[3] = {x[0] - K->p[0][0], x[1] - K->p[0][1], x[2] - K->p[0][2]};
    for (int i = 0; i < 3; ++i) {
        J[i * NV + i] = 1.0;
        J[(3 + i) * NV + 3 + i] = 1.0;
    }
    /* -skew(d) */
    J[0 * NV + 4] = d[2];  J[0 * NV + 5] = -d[1];
    J[1 * NV + 3] = -d[2]; J[1 * NV + 5] = d[0];
    J[2 * NV + 3] = d[1];  J[2 * NV + 4] = -d[0];
    for (int j = 0; j < m->n; ++j) {
        if (!((anc >> j) & 1)) continue;
        if (m->joint_type && m->joint_type[j] == 1) {   /* prismatic: (z; 0) */
            for (int i = 0; i < 3; ++i) J[i * NV + 6 + j] = K->z[j][i];
            continue;
        }
        const double e[3] = {x[0] - K->o[j][0], x[1] - K->o[j][1], x[2] - K->o[j][2]};
        double t[3];
        cross3(K->z[j], e, t);
        for (int i = 0; i < 3; ++i) {
            J[i * NV + 6 + j] = t[i];
            J[(3 + i) * NV + 6 + j] = K->z[j][i];
        }
    }
}

/* M (NV x NV) and h (NV) of the Jacobian form, nu_dot = 0 */
static void mass_and_bias(const orc_fb_model* m, const fb_kin* K, const unsigned long long* anc, double* M,
                          double* h)
{
    const int n = m->n, NV = 6 + n;
    double J[6 * FB_NV];
    memset(M, 0, sizeof(double) * NV * NV);
    memset(h, 0, sizeof(double) * NV);
    for (int l = 0; l <= n; ++l) {
        const double* Rl = K->R[l];
        double rc[3], c[3], Iw[9], T[9], RT[9], ac[3], f[3], tq[3], t[3], u[3];
        mv3(Rl, m->link_com + 3 * l, rc);
        for (int i = 0; i < 3; ++i) c[i] = K->p[l][i] + rc[i];
        point_jacobian(m, K, anc[l], c, J, NV);
        for (int i = 0; i < 3; ++i)
            for (int k = 0; k < 3; ++k) RT[3 * i + k] = Rl[3 * k + i];
        mm3(Rl, m->link_inertia + 9 * l, T);
        mm3(T, RT, Iw);
        const double ms = m->link_mass[l];
        /* M += m Jv^T Jv + Jw^T Iw Jw (columns of the link's support only) */
        int sup[FB_NV], ns = 0;   /* the nonzero columns: the base's six and the ancestor joints */
        for (int b = 0; b < 6; ++b) sup[ns++] = b;
        for (int j = 0; j < n; ++j)
            if ((anc[l] >> j) & 1) sup[ns++] = 6 + j;
        double IJ[3 * FB_NV];
        for (int i = 0; i < 3; ++i)
            for (int bb = 0; bb < ns; ++bb) {
                const int b = sup[bb];
                IJ[i * NV + b] = Iw[3 * i] * J[3 * NV + b] + Iw[3 * i + 1] * J[4 * NV + b] + Iw[3 * i + 2] * J[5 * NV + b];
            }
        for (int aa = 0; aa < ns; ++aa)
            for (int bb = 0; bb < ns; ++bb) {
                const int a = sup[aa], b = sup[bb];
                double s = 0.0;
                for (int i = 0; i < 3; ++i) s += ms * J[i * NV + a] * J[i * NV + b] + J[(3 + i) * NV + a] * IJ[i * NV + b];
                M[a * NV + b] += s;
            }
        cross3(K->al[l], rc, t);
        cross3(K->w[l], rc, u);
        cross3(K->w[l], u, u);
        for (int i = 0; i < 3; ++i) {
            ac[i] = K->a[l][i] + t[i] + u[i];
            f[i] = ms * (ac[i] - m->gravity[i]);
        }
        double Ia[3], Iww[3];
        mv3(Iw, K->al[l], Ia);
        mv3(Iw, K->w[l], Iww);
        cross3(K->w[l], Iww, t);
        for (int i = 0; i < 3; ++i) tq[i] = Ia[i] + t[i];
        for (int bb = 0; bb < ns; ++bb) {
            const int b = sup[bb];
            for (int i = 0; i < 3; ++i) h[b] += J[i * NV + b] * f[i] + J[(3 + i) * NV + b] * tq[i];
        }
    }
}

int orc_fbd_dynamics(const orc_fb_model* m, const double* bpos, const double* brot, const double* q,
                     const double* bvel, const double* qd, const double* tau, int ncontacts,
                     const double* cparams, const double* null_poses, double* base_acc, double* joint_acc,
                     double* dpos, double* drot, double* dq)
{
    const int n = m->n, NV = 6 + n;
    if (n > FB_MAXN || n < 0) return -1;
    fb_kin K;
    unsigned long long anc[FB_MAXN + 1];
    double M[FB_NV * FB_NV], h[FB_NV], known[FB_NV], J[6 * FB_NV];
    kinematics(m, bpos, brot, q, bvel, qd, &K);
    ancestors(m, anc);
    mass_and_bias(m, &K, anc, M, h);
    for (int a = 0; a < NV; ++a) known[a] = -h[a];
    for (int c = 0; c < ncontacts; ++c) {
        const int l = m->frame_link[c];
        const double* fp = m->frame_pose + 12 * c;
        double pose[12], vel[6], t[3], d[3], w6[6];
        mv3(K.R[l], fp, t);
        for (int i = 0; i < 3; ++i) pose[i] = K.p[l][i] + t[i];
        mm3(K.R[l], fp + 3, pose + 3);
        for (int i = 0; i < 3; ++i) d[i] = pose[i] - K.p[l][i];
        cross3(K.w[l], d, t);
        for (int i = 0; i < 3; ++i) {
            vel[i] = K.v[l][i] + t[i];
            vel[3 + i] = K.w[l][i];
        }
        point_jacobian(m, &K, anc[l], pose, J, NV);
        orc_contact_eval(cparams + 4 * c, vel, pose, null_poses + 12 * c, w6, NULL, NULL, NULL);
        for (int a = 0; a < NV; ++a)
            for (int i = 0; i < 6; ++i) known[a] += J[i * NV + a] * w6[i];
    }
    for (int j = 0; j < n; ++j) known[6 + j] += tau[j];
    /* Cholesky M = L L^T (lower, in place), then the two triangular solves */
    for (int j = 0; j < NV; ++j) {
        double s = M[j * NV + j];
        for (int k = 0; k < j; ++k) s -= M[j * NV + k] * M[j * NV + k];
        if (!(s > 0.0)) return -2;
        const double d = sqrt(s);
        M[j * NV + j] = d;
        for (int i = j + 1; i < NV; ++i) {
            double t = M[i * NV + j];
            for (int k = 0; k < j; ++k) t -= M[i * NV + k] * M[j * NV + k];
            M[i * NV + j] = t / d;
        }
    }
    for (int i = 0; i < NV; ++i) {
        double t = known[i];
        for (int k = 0; k < i; ++k) t -= M[i * NV + k] * known[k];
        known[i] = t / M[i * NV + i];
    }
    for (int i = NV - 1; i >= 0; --i) {
        double t = known[i];
        for (int k = i + 1; k < NV; ++k) t -= M[k * NV + i] * known[k];
        known[i] = t / M[i * NV + i];
    }
    memcpy(base_acc, known, 6 * sizeof(double));
    memcpy(joint_acc, known + 6, n * sizeof(double));
    orc_fbk_dynamics(n, m->rho, brot, bvel, qd, dpos, drot, dq);
    return 0;
}

int orc_fbd_euler_impedance(const orc_fb_model* m, double* bpos, double* brot, double* q, double* bvel,
                            double* qd, const double* q_ref, const double* kp, const double* kd,
                            int ncontacts, const double* cparams, const double* null_poses, double t0,
                            double t1, double dT)
{
    const int n = m->n;
    if (!(t1 > t0) || !(dT > 0)) return -3;
    const int iters = (int)ceil((t1 - t0) / dT);
    const double cur = iters >= 2 ? t0 + dT * (iters - 2) : t0;
    double tau[FB_MAXN], ba[6], ja[FB_MAXN], dp[3], dR[9], dqv[FB_MAXN];
    for (int it = 0; it < iters; ++it) {
        const double hs = it == iters - 1 ? t1 - cur : dT;
        for (int j = 0; j < n; ++j) tau[j] = kp[j] * (q_ref[j] - q[j]) - kd[j] * qd[j];
        const int rc = orc_fbd_dynamics(m, bpos, brot, q, bvel, qd, tau, ncontacts, cparams, null_poses,
                                        ba, ja, dp, dR, dqv);
        if (rc) return rc;
        for (int i = 0; i < 3; ++i) bpos[i] = bpos[i] + dp[i] * hs;
        for (int i = 0; i < 9; ++i) brot[i] = brot[i] + dR[i] * hs;
        for (int j = 0; j < n; ++j) q[j] = q[j] + dqv[j] * hs;
        for (int i = 0; i < 6; ++i) bvel[i] = bvel[i] + ba[i] * hs;
        for (int j = 0; j < n; ++j) qd[j] = qd[j] + ja[j] * hs;
    }
    return 0;
}

/* ---- batch driver: B robots, states [B][...], q_ref [B][n], null poses [B][C][12] ---- */
typedef struct {
    const orc_fb_model* m;
    double *bpos, *brot, *q, *bvel, *qd;
    const double *q_ref, *kp, *kd, *cparams, *null_poses;
    int ncontacts;
    double t0, t1, dT;
    int64_t count;
    atomic_llong next;
    atomic_int err;
} fbd_job;

static void* fbd_worker(void* arg)
{
    fbd_job* J = (fbd_job*)arg;
    const int n = J->m->n;
    for (;;) {
        const long long i = atomic_fetch_add(&J->next, 1);
        if (i >= J->count) break;
        const int rc = orc_fbd_euler_impedance(J->m, J->bpos + 3 * i, J->brot + 9 * i, J->q + n * i,
                                               J->bvel + 6 * i, J->qd + n * i, J->q_ref + n * i, J->kp,
                                               J->kd, J->ncontacts, J->cparams,
                                               J->null_poses + 12 * J->ncontacts * i, J->t0, J->t1, J->dT);
        if (rc) atomic_store(&J->err, rc);
    }
    return NULL;
}

int orc_fbd_euler_impedance_batch(const orc_fb_model* m, int64_t B, double* bpos, double* brot, double* q,
                                  double* bvel, double* qd, const double* q_ref, const double* kp,
                                  const double* kd, int ncontacts, const double* cparams,
                                  const double* null_poses, double t0, double t1, double dT, int threads)
{
    fbd_job J;
    J.m = m; J.bpos = bpos; J.brot = brot; J.q = q; J.bvel = bvel; J.qd = qd;
    J.q_ref = q_ref; J.kp = kp; J.kd = kd; J.cparams = cparams; J.null_poses = null_poses;
    J.ncontacts = ncontacts; J.t0 = t0; J.t1 = t1; J.dT = dT; J.count = B;
    atomic_store(&J.next, 0);
    atomic_store(&J.err, 0);
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    pthread_t th[256];
    int started = 0;
    for (int t = 1; t < threads; ++t)
        if (pthread_create(&th[started], NULL, fbd_worker, &J) == 0) ++started;
    fbd_worker(&J);
    for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
    return atomic_load(&J.err);
}

/* centre of mass and its velocity of B robots (closed_loop.com_state): com [B][6] = (c, cdot),
 * c = sum_l m_l (p_l + R_l com_l) / m, cdot = sum_l m_l (v_l + w_l x R_l com_l) / m */
void orc_fbd_com_batch(const orc_fb_model* m, int64_t B, const double* bpos, const double* brot,
                       const double* q, const double* bvel, const double* qd, double* com)
{
    const int n = m->n;
    fb_kin K;
    for (int64_t i = 0; i < B; ++i) {
        kinematics(m, bpos + 3 * i, brot + 9 * i, q + n * i, bvel + 6 * i, qd + n * i, &K);
        double c[3] = {0, 0, 0}, cd[3] = {0, 0, 0}, mt = 0.0;
        for (int l = 0; l <= n; ++l) {
            double rc[3], t[3];
            mv3(K.R[l], m->link_com + 3 * l, rc);
            cross3(K.w[l], rc, t);
            const double ms = m->link_mass[l];
            for (int k = 0; k < 3; ++k) {
                c[k] += ms * (K.p[l][k] + rc[k]);
                cd[k] += ms * (K.v[l][k] + t[k]);
            }
            mt += ms;
        }
        for (int k = 0; k < 3; ++k) {
            com[6 * i + k] = c[k] / mt;
            com[6 * i + 3 + k] = cd[k] / mt;
        }
    }
}
