/*
 * blf_oracle.h — TEST INFRASTRUCTURE ONLY.  CPU restatement (plain C, fp64, no FMA contraction)
 * of the reference semantics on the DCM-MPC path.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product path (the HIP library behind
 * include/blf/blf_c.h) never links or calls it.
 *
 * Parity anchors (reference paths relative to src/):
 *   orc_lti_euler_integrate  System/include/BipedalLocomotion/System/FixedStepIntegrator.tpp:21-72,
 *                            ForwardEuler.tpp:18-49, ForwardEuler.h:35-50,
 *                            System/src/LinearTimeInvariantSystem.cpp:40-74
 *                            pinned by System/tests/IntegratorTest.cpp:27-75 (closed form, tol 1e-3)
 *   orc_dcm_euler_rollout    the LTI step with A = omega I, B = -omega I (bit-exact by construction)
 *   orc_contact_phases       Planners/src/ContactPhaseList.cpp:16-84
 *                            pinned by Planners/tests/ContactPhaseListTest.cpp:15-153 (8 phases)
 *   orc_present_index        Planners/src/ContactList.cpp:190-202 (getPresentContact)
 *                            pinned by Planners/tests/ContactListTest.cpp:85-92
 *   orc_dcm_phase_expand     the phases of ContactPhaseList.cpp:16-84 per knot with the
 *                            getPresentContact rule (ContactList.cpp:190-202)
 *   orc_hull2d_hrep          Planners/src/ConvexHullHelper.cpp:35-99; arithmetic of the pinned
 *                            third-party dependency Qhull 8.0.0 ("Qt"), restated as a 2-D
 *                            monotone chain with collinear merge; pinned against scipy's bundled
 *                            Qhull 7.3.2 "Qt" fixtures (tests/golden/hull2d.json)
 *   orc_hull2d_contains      Planners/src/ConvexHullHelper.cpp:101-117
 *   orc_hull3d_hrep          ConvexHullHelper.cpp:35-99 on 3 x p points (the reference test's case,
 *                            ConvexHullHelperTest.cpp:15-63); checked as plane sets against scipy's
 *                            Qhull (tests/golden/hull3d.json)
 *   orc_hullnd_hrep          ConvexHullHelper.cpp:35-99 on n x p points, any n (dim-subset planes)
 *   orc_halfspace_contains   ConvexHullHelper.cpp:101-117 in any dimension
 *   orc_quintic_*            ABSENT in the reference: parity unpinned against the
 *                            reference; pinned by boundary-condition identities + sympy fixtures
 *   orc_contact_* / orc_fbk_* blf_oracle_contact.c: ContinuousContactModel.cpp:79-254 and
 *                            FloatingBaseSystemKinematics.cpp:36-73 (config 5 rows), pinned by the
 *                            properties of ContactModels/tests/ContinousContactModelTest.cpp
 *   orc_dcm_mpc_solve        ABSENT in the reference: parity unpinned against the
 *                            reference; pinned by an independent dense KKT solve (iteratively
 *                            refined) of the same QP in tests/test_oracle_dcm_mpc.py
 */
#ifndef BLF_ORACLE_H
#define BLF_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int orc_lti_euler_integrate(int n, int m, const double* A, const double* B, const double* u,
                            double* x, double t0, double t1, double dT, int64_t* nsteps_out);

void orc_dcm_euler_rollout(const double* xi0, const double* omega, const double* vrp, int N,
                           double dt, double* xi_out);

/* ContactPhaseList::createPhases over L lists of contact intervals.
 * act/deact: [L][C] (list l has ncontacts[l] valid entries, sorted, non-overlapping).
 * Output: up to max_phases phases: begin[p], end[p], active[p][L] = contact index of list l
 * active in phase p or -1.  Returns the number of phases (or -1 if max_phases too small). */
int orc_contact_phases(int L, int C, const double* act, const double* deact,
                       const int32_t* ncontacts, int max_phases, double* begin, double* end,
                       int32_t* active);

/* getPresentContact: index of the last element with activation_time <= t, or -1 (end()). */
int orc_present_index(const double* activation_times, int n, double t);

/* blf_dcm_phase_expand for one problem: phase table begin/end [P], pA [P][M][2], pb [P][M],
 * pnf [P], pref [P][2] (nphases valid) -> A [N][M][2], b [N][M], nfacets [N], xi_ref [N+1][2],
 * vrp_ref [N][2] of the window of knots (start + k) dt. */
void orc_dcm_phase_expand(int P, int M, int nphases, const double* begin, const double* end,
                          const double* pA, const double* pb, const int32_t* pnf,
                          const double* pref, int64_t start, double dt, int N, double* A,
                          double* b, int32_t* nfacets, double* xi_ref, double* vrp_ref);

void orc_hull2d_force_andrew(int on);
int orc_hull2d_hrep(const double* pts, int npts, int max_facets, double* A, double* b);
int orc_hull2d_contains(const double* A, const double* b, int nfacets, const double* p);
int orc_hull3d_hrep(const double* pts, int npts, int max_facets, double* A, double* b);
int orc_hullnd_hrep(int dim, const double* pts, int npts, int max_facets, double* A, double* b);
int orc_halfspace_contains(const double* A, const double* b, int nfacets, int dim, const double* p);

void orc_quintic_fit(const double* knots_t, const double* knots_pva, int nknots, int dim,
                     double* coeffs);
void orc_quintic_eval(const double* knots_t, const double* coeffs, int nknots, int dim,
                      const double* tq, int nq, double* pva, int32_t* knot_idx);

/* sequential != 0: evaluate the affine recursions as plain sequential loops (the CPU-efficient
 * form, used only for bench.py's cpu_baseline timing); 0: the device's Kogge-Stone scan order,
 * bit-identical to the kernel (every parity test). */
typedef struct orc_dcm_params {
    int32_t horizon, max_facets, max_iter, sequential;
    double dt, w_xi[2], w_vrp[2], w_terminal[2], tol_mu, tol_primal, tol_dual;
    double tol_polish;   /* > 0: try the active-set polish once mu <= tol_polish */
    int32_t single_kernel;   /* 1: the device's BLF_QP_SINGLE_KERNEL=1 path (IPM kernel alone) */
    int32_t as_tree;         /* 1: the active-set kernels' DPP scan tree, as the device evaluates
                              * horizons <= 64 in batches of at most BLF_DPP_TREE_MAX_BATCH QPs */
} orc_dcm_params;

/* Solve one problem (arrays for this problem only, same layout as blf_dcm_mpc_problem).
 * Returns the BLF_QP_* status; writes xi [N+1][2], vrp [N][2], *iters. */
int orc_dcm_mpc_solve(const orc_dcm_params* prm, const double* xi_init, const double* omega,
                      const double* xi_ref, const double* vrp_ref, const double* A,
                      const double* b, const int32_t* nfacets, double* xi, double* vrp,
                      int32_t* iters);

/* Batched, multi-threaded drivers (blf_oracle_batch.c; bench.py CPU baselines): the per-item
 * entry points above over `count` items on `threads` POSIX threads. */
void orc_hull2d_hrep_batch(int64_t count, int P, int M, const double* pts, const int32_t* npts,
                           double* A, double* b, int32_t* nf, int threads);
void orc_dcm_phase_expand_batch(int64_t B, int P, int M, const int32_t* nphases, const double* begin,
                                const double* end, const double* pA, const double* pb,
                                const int32_t* pnf, const double* pref, int64_t start, double dt,
                                int N, double* A, double* b, int32_t* nfacets, double* xi_ref,
                                double* vrp_ref, int threads);
void orc_quintic_batch(int64_t S, int K1, int dim, int Q, const double* knots_t,
                       const double* knots_pva, const double* tq, double* coeffs, double* pva,
                       int32_t* idx, int threads);

/* The fp32 active-set search of a cold start as the device's active-set kernel runs it
 * (blf_oracle_as32.c): returns 1 when a float pass certified, the float point
 * (r [N][2], xi_{k+1} [N][2], as doubles) and the search's next candidate sets (guess bits per
 * knot), which the fp64 passes start from when it did not certify; *npass (NULL: not written) the
 * float passes it ran.
 * sequential = 1: plain recursions instead of the kernel's scan tree (CPU baseline). */
int orc_as32_search(const orc_dcm_params* prm, int sequential, const double* xi_init,
                     const double* omega, const double* xi_ref, const double* vrp_ref,
                     const double* A, const double* b, const int32_t* nfacets, double* r_out,
                     double* x_out, int32_t* guess, int32_t* npass);

/* Warm start of a receding-horizon re-solve ("Warm start"): knot k
 * starts from knot src = min(k + shift, N - 1) of a previous solution: r_k = vrp[src],
 * s = max(b - A r, floor), lam = max(lambda[src], floor); the LQ start step is skipped. */
typedef struct orc_dcm_warm {
    const double* vrp;      /* [N][2]  */
    const double* lambda;   /* [N][M]  */
    int32_t shift;
    int32_t reserved;
    double floor;
} orc_dcm_warm;

/* As orc_dcm_mpc_solve, from the warm start `warm` (NULL: the cold start), also writing the final
 * multipliers to lam_out [N][M] (NULL: not written; zero in unused facet slots), whether the
 * active-set polish was accepted to *polished and the active-set kernels' drop/add passes (a cold
 * start's fp32 search plus its fp64 passes, a warm start's fp64 passes; 0 without the active-set
 * kernels) to *passes (NULL: not written; blf_dcm_mpc_solution.passes). */
int orc_dcm_mpc_solve_warm(const orc_dcm_params* prm, const double* xi_init, const double* omega,
                           const double* xi_ref, const double* vrp_ref, const double* A,
                           const double* b, const int32_t* nfacets, const orc_dcm_warm* warm,
                           double* xi, double* vrp, double* lam_out, int32_t* iters,
                           int32_t* polished, int32_t* passes);

/* Whole batch (problem-major arrays), split over `threads` POSIX threads (one problem per
 * thread at a time).  Used as bench.py's CPU baseline. */
void orc_dcm_mpc_solve_batch(const orc_dcm_params* prm, int64_t batch, int threads,
                             const double* xi_init, const double* omega, const double* xi_ref,
                             const double* vrp_ref, const double* A, const double* b,
                             const int32_t* nfacets, double* xi, double* vrp, int32_t* status,
                             int32_t* iters);
/* Batch with warm starts: vrp_ws [B][N][2] and lam_ws [B][N][M] (both NULL: cold starts),
 * prev_status [B] or NULL (a problem with prev_status != 0 is solved cold: the device's
 * blf_dcm_mpc_warm_start.prev_status), lam_out [B][N][M] or NULL, polished [B] or NULL, passes
 * [B] or NULL. */
void orc_dcm_mpc_solve_batch_warm(const orc_dcm_params* prm, int64_t batch, int threads,
                                  const double* xi_init, const double* omega, const double* xi_ref,
                                  const double* vrp_ref, const double* A, const double* b,
                                  const int32_t* nfacets, const double* vrp_ws,
                                  const double* lam_ws, const int32_t* prev_status, int32_t shift,
                                  double floor, double* xi, double* vrp, double* lam_out,
                                  int32_t* status, int32_t* iters, int32_t* polished, int32_t* passes);

/* Tree sum with the device's reduction order: c has n entries, padded with
 * zeros to 64*ceil(n/64); per 64-block xor-butterfly (distances 1, 2, 4, ..., 32), then block
 * sums left to right. */
double orc_wave_tree_sum(const double* c, int n);
/* The active-set kernels' scan tree (csrc/dcm_qp_common.h tree_fwd / tree_bwd): the lane whose
 * element lane l combines with at level L = 0..5 (fwd: lower lanes, else higher lanes), or -1 (the
 * identity element). */
int orc_lane_src(int level, int fwd, int l);

/* ContinuousContactModel (one contact).  prm = {length, width, spring_coeff, damper_coeff};
 * twist = {v[3], w[3]} (mixed); pose / null_pose = {p[3], R[9] row-major}.  Outputs (NULL to skip):
 * wrench[6] = {force, torque}, autonomous[6], control[36] (6x6 row-major), regressor[12] (6x2). */
void orc_contact_eval(const double* prm, const double* twist, const double* pose,
                      const double* null_pose, double* wrench, double* autonomous,
                      double* control, double* regressor);
/* getForceAtPoint / getTorqueGeneratedAtPoint at (x, y) of the contact surface. */
void orc_contact_point(const double* prm, const double* twist, const double* pose,
                       const double* null_pose, double x, double y, double* force, double* torque);
/* FloatingBaseSystemKinematics::dynamics: rot[9] row-major, twist[6] mixed, joint_vel[n];
 * outputs dpos[3], drot[9], djoints[n]. */
void orc_fbk_dynamics(int n, double rho, const double* rot, const double* twist,
                      const double* joint_vel, double* dpos, double* drot, double* djoints);
/* ForwardEuler<FloatingBaseSystemKinematics>::integrate(t0, t1) with constant inputs; the state
 * (pos[3], rot[9], joints[n], n <= 64) is updated in place.  Returns 0 or a BLF_ERR_* code. */
int orc_fbk_euler_integrate(int n, double rho, double* pos, double* rot, double* joints,
                            const double* twist, const double* joint_vel, double t0, double t1,
                            double dT);

/* FloatingBaseDynamicalSystem::dynamics and its ForwardEuler with a joint impedance
 * (blf_oracle_fbd.c; the C restatement of oracle/fb_dynamics.py).  n <= 40 joints. */
typedef struct orc_fb_model {
    int n;
    const int32_t* parent;
    const double* joint_origin;
    const double* joint_rot;
    const double* joint_axis;
    const double* link_mass;
    const double* link_com;
    const double* link_inertia;
    const int32_t* frame_link;
    const double* frame_pose;
    double gravity[3];
    double rho;
    const int32_t* joint_type;   /* [n] or NULL (all revolute): 1 = prismatic (blf_fb_model) */
} orc_fb_model;
int orc_fbd_dynamics(const orc_fb_model* m, const double* bpos, const double* brot, const double* q,
                     const double* bvel, const double* qd, const double* tau, int ncontacts,
                     const double* cparams, const double* null_poses, double* base_acc, double* joint_acc,
                     double* dpos, double* drot, double* dq);
int orc_fbd_euler_impedance(const orc_fb_model* m, double* bpos, double* brot, double* q, double* bvel,
                            double* qd, const double* q_ref, const double* kp, const double* kd,
                            int ncontacts, const double* cparams, const double* null_poses, double t0,
                            double t1, double dT);
int orc_fbd_euler_impedance_batch(const orc_fb_model* m, int64_t B, double* bpos, double* brot, double* q,
                                  double* bvel, double* qd, const double* q_ref, const double* kp,
                                  const double* kd, int ncontacts, const double* cparams,
                                  const double* null_poses, double t0, double t1, double dT, int threads);
void orc_fbd_com_batch(const orc_fb_model* m, int64_t B, const double* bpos, const double* brot,
                       const double* q, const double* bvel, const double* qd, double* com);

#ifdef __cplusplus
}
#endif
#endif
