/*
 * blf_c.h — C ABI of the MI355X-native batched DCM-MPC planning path.
 *
 * This is the drop-in boundary.  Every entry point takes plain pointers and sizes (no C++ or
 * torch types), returns a blf_status, and is stream-ordered on the hipStream_t passed in
 * (passed as `void*` so this header needs no HIP include; NULL = the default stream).
 * All device buffers are caller-owned and must be device-resident (hipMalloc'd or a torch CUDA
 * tensor's data_ptr()).  Layout convention: PROBLEM-MAJOR ("[B][...]", batch outermost, each
 * problem's arrays contiguous), innermost index = the spatial coordinate.  One workgroup (or one
 * lane for the rollout/eval kernels) serves one problem; see DESIGN.md for why.
 *
 * Which reference interface each entry point replaces (paths relative to the reference root,
 * src/...):
 *   blf_lti_euler_integrate   System/include/BipedalLocomotion/System/FixedStepIntegrator.tpp:21-72
 *                             + ForwardEuler.tpp:18-49 + System/src/LinearTimeInvariantSystem.cpp:40-74
 *                             (ForwardEuler<LinearTimeInvariantSystem>::integrate(t0, T))
 *   blf_dcm_euler_rollout     the same ForwardEuler<LTI> step applied per knot with
 *                             A = omega_k I, B = -omega_k I (LinearTimeInvariantSystem.cpp:13-38, :71)
 *   blf_hull2d_hrep           Planners/src/ConvexHullHelper.cpp:35-99 (buildConvexHull/getA/getB)
 *   blf_hull2d_contains       Planners/src/ConvexHullHelper.cpp:101-117 (doesPointBelongToConvexHull)
 *   blf_hullnd_hrep           ConvexHullHelper.cpp:35-99 on n x p points, any n
 *   blf_hull3d_hrep           ConvexHullHelper.cpp:35-99 on 3 x p points (Planners/tests/
 *                             ConvexHullHelperTest.cpp:15-63 is 3-D)
 *   blf_halfspace_contains    ConvexHullHelper.cpp:101-117 in any dimension
 *   blf_quintic_fit/_eval     ABSENT in the reference (QuinticSpline); knot rule
 *                             of Planners/src/ContactList.cpp:190-202 (getPresentContact, `<=`)
 *   blf_contact_model_eval    ContactModels/src/ContinuousContactModel.cpp:79-171, 223-254 behind the
 *                             lazy getters of ContactModels/src/ContactModel.cpp:12-92
 *                             (getContactWrench / getAutonomousDynamics / getControlMatrix /
 *                             getRegressor)
 *   blf_contact_point_wrench  ContinuousContactModel.cpp:173-221 (getForceAtPoint,
 *                             getTorqueGeneratedAtPoint)
 *   blf_fbk_dynamics          System/src/FloatingBaseSystemKinematics.cpp:36-73
 *   blf_fbk_euler_integrate   ForwardEuler<FloatingBaseSystemKinematics>::integrate
 *                             (FixedStepIntegrator.tpp:21-72 + ForwardEuler.tpp:18-49)
 *   blf_fbd_dynamics          System/src/FloatingBaseSystemDynamics.cpp:102-251
 *                             (FloatingBaseDynamicalSystem::dynamics; the rigid-body terms that the
 *                             reference takes from iDynTree KinDynComputations are computed here)
 *   blf_fbd_euler_integrate   ForwardEuler<FloatingBaseDynamicalSystem>::integrate
 *   blf_dcm_phase_expand      Planners/src/ContactPhaseList.cpp:16-84 phases looked up per knot with the
 *                             getPresentContact rule (ContactList.cpp:190-202), SURVEY.md 8(f) item 2
 *   blf_dcm_mpc_solve_phased  blf_dcm_phase_expand + blf_dcm_mpc_solve_warm fused: one
 *                             Advanceable::advance() (System/Advanceable.h:24-46) of the planner
 *   blf_fb_dcm / blf_dcm_posture_reference  the state -> plan and plan -> input maps a user
 *                             writes around Advanceable::advance() and ForwardEuler::integrate in a
 *                             closed loop (config 5); no reference counterpart
 *   blf_fbd_euler_integrate_impedance  blf_fbd_euler_integrate with a joint impedance as the
 *                             control input of every step (the user's per-step setControlInput)
 *   blf_dcm_mpc_solve[_warm]  ABSENT in the reference (TimeVaryingDCMPlanner QP),
 *                             driven through System/Advanceable.h:24-46 (advance()) by the C++ host
 *                             adapter blf::Planners::TimeVaryingDCMPlanner
 */
#ifndef BLF_C_H
#define BLF_C_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status ------------------------------------------------------------------------------- */
typedef int32_t blf_status;
#define BLF_OK                   0
#define BLF_ERR_INVALID_ARGUMENT 1  /* bad size / null pointer / bad parameter                   */
#define BLF_ERR_HIP              2  /* a HIP runtime call failed (see blf_last_error())          */
#define BLF_ERR_UNSUPPORTED      3  /* size outside what the kernels are built for               */
#define BLF_ERR_TIME_INTERVAL    4  /* reference rejects: initialTime > finalTime or dT <= 0     */
#define BLF_ERR_EMPTY_INTERVAL   5  /* initialTime == finalTime: the reference loops forever
                                       (FixedStepIntegrator.tpp:96-99, size_t vs -1); we refuse  */

/* per-problem solver status written by blf_dcm_mpc_solve */
#define BLF_QP_SOLVED        0
#define BLF_QP_MAX_ITER      1
#define BLF_QP_NUMERICAL     2   /* non-finite iterate or non-positive-definite KKT block        */
#define BLF_QP_BAD_FACETS    3   /* nfacets[k] outside [0, max_facets]                            */

typedef struct blf_handle blf_handle;

/* Create a handle bound to HIP device `device`.  Fails with BLF_ERR_HIP if no device.  A handle
 * keeps, per stream it solves QPs on, a small device work list (the problems the active-set
 * kernel hands to the interior point kernel; allocated at the first solve on the stream and grown,
 * after a synchronisation of that stream, when a batch outgrows it).  Solves on one handle and one
 * stream must be enqueued from one host thread at a time. */
blf_status blf_create(blf_handle** handle, int32_t device);
blf_status blf_destroy(blf_handle* handle);
/* Human-readable description of the last error on this thread (never NULL). */
const char* blf_last_error(void);
/* Version string of the library: "blf-mi355x <version> (abi <n>, ...) src <hash>".  ABI 2 (0.2.0)
 * added the optional pointer fields blf_dcm_mpc_solution.passes and blf_fb_contacts.law / .wrench:
 * a caller built against an older header must zero-initialise these structs (`= {0}`), since the
 * library reads every field as a device pointer or NULL.  Solves that use a stream's stage-2 list
 * (blf_dcm_mpc_solve*) are refused with BLF_ERR_UNSUPPORTED while that stream is being captured
 * into a graph: the list's slot is sequenced on the host. */
#define BLF_ABI_VERSION 2
const char* blf_version(void);
/* QP kernel routing for A/B and parity tests (no reference counterpart; the defaults are the
 * product's).  fuse_stage2 = 0: small cold batches with N <= 64 run the IPM's stage 2 as its own
 * launch instead of inside the active-set kernel; single_kernel = 1: every QP runs in the
 * interior point kernel alone (no active-set kernel).  -1 leaves a setting unchanged.  The initial
 * values come from BLF_QP_FUSE_STAGE2 / BLF_QP_SINGLE_KERNEL, read once at the first solve.  The
 * setting is process-wide (every handle and thread), not per handle. */
blf_status blf_set_qp_launch_mode(int32_t fuse_stage2, int32_t single_kernel);
/* ---- 0. FixedStepIntegrator::integrate's step schedule (FixedStepIntegrator.tpp:21-72) -------
 * The validation (in the reference's order) and schedule every batched integrator below uses:
 * iterations = (int)ceil((T - t0) / dT); steps i = 0..iterations-2 run at currentTime = t0 + dT*i
 * with step dT; the last step runs at the stale currentTime (t0 + dT*(iterations-2), or t0 when
 * iterations < 2), *t_last, with step *dT_last = T - *t_last.  Errors: BLF_ERR_TIME_INTERVAL
 * (t0 > T or dT <= 0), BLF_ERR_EMPTY_INTERVAL (t0 == T), BLF_ERR_UNSUPPORTED (>= 2e9 steps).
 * Host-only; used by include/blf/forward_euler_device.h to integrate user systems. */
blf_status blf_step_schedule(double initial_time, double final_time, double dT,
                             int32_t* iterations, double* dT_last, double* t_last);

/* ---- 1. ForwardEuler<LinearTimeInvariantSystem>::integrate(t0, T), batched ------------------
 * x_{i+1} = x_i + (A x_i + B u) * dT_i over the reference's step schedule:
 *   iters = (int)ceil((T - t0) / dT); steps i = 0..iters-2 advance by dT; the final step
 *   advances by (T - currentTime) with the stale currentTime = t0 + dT*(iters-2) (0 if iters<2).
 * A: [B][n][n] row-major, Bm: [B][n][m] (or a single shared matrix when `shared_matrices` != 0),
 * u: [B][m] (held constant, as setControlInput does), x: [B][n] updated in place.
 * n, m >= 1, any size (n, m <= 8: one lane per system, registers; up to 512: one 64-lane
 * workgroup per system, state in LDS; larger: one 256-thread workgroup per system, state in x and
 * a stream-ordered scratch — the same arithmetic order everywhere, so the same bits).  Arithmetic order (no FMA contraction): dx_r = (sum_c A_rc x_c) + (sum_c B_rc u_c),
 * each sum left to right; x_r = x_r + dx_r * dT_i.                                            */
blf_status blf_lti_euler_integrate(blf_handle* handle, int32_t n, int32_t m,
                                   const double* A, const double* Bm, int32_t shared_matrices,
                                   const double* u, double* x, int64_t batch,
                                   double initial_time, double final_time, double dT,
                                   void* stream);

/* LinearTimeInvariantSystem::dynamics (LinearTimeInvariantSystem.cpp:40-74), batched:
 * dx = A x + B u with the same summation order as blf_lti_euler_integrate; dx: [B][n]. */
blf_status blf_lti_dynamics(blf_handle* handle, int32_t n, int32_t m, const double* A,
                            const double* Bm, int32_t shared_matrices, const double* u,
                            const double* x, double* dx, int64_t batch, void* stream);

/* ---- 2. DCM rollout: one reference Euler step per knot -------------------------------------
 * xi_{k+1} = xi_k + ((omega_k * xi_k) + (-omega_k * r_k)) * dt,  k = 0..N-1
 * xi0: [B][2], omega: [B][N], vrp: [B][N][2], xi_out: [B][N+1][2] (xi_out[:,0] = xi0).       */
blf_status blf_dcm_euler_rollout(blf_handle* handle, const double* xi0, const double* omega,
                                 const double* vrp, int32_t horizon, double dt,
                                 double* xi_out, int64_t batch, void* stream);

/* ---- 3. Support polygon H-representation (ConvexHullHelper, 2-D) ---------------------------
 * pts: [B][P][2] (P <= BLF_HULL_MAX_POINTS), npts: [B] valid point count (<= P).
 * Output, padded to `max_facets` rows: A: [B][max_facets][2] unit outward normals,
 * b: [B][max_facets] offsets (inside: A x <= b), nfacets: [B] facet count (rows >= nfacets are
 * zero rows with b = 0).  Collinear boundary points are merged (Qhull "Qt" merges them too, see
 * ConvexHullHelper.cpp:54-58).  Facets are ordered counter-clockwise from the lowest-leftmost
 * vertex; Qhull's order is internal, so compare as sets.  If the hull needs more than
 * max_facets rows, or fewer than 3 distinct non-collinear points are given, nfacets = -1.     */
#define BLF_HULL_MAX_POINTS 16
blf_status blf_hull2d_hrep(blf_handle* handle, const double* pts, const int32_t* npts,
                           int32_t max_points, int32_t max_facets, int64_t batch,
                           double* A, double* b, int32_t* nfacets, void* stream);

/* doesPointBelongToConvexHull: inside[q] = 1 iff for all rows i < nfacets: (A p)_i <= b_i
 * (strict `>` rejects, no tolerance, ConvexHullHelper.cpp:110-114).  One query point per polygon:
 * query: [B][2], inside: [B] int32.  A polygon with nfacets < 0 or nfacets > max_facets gives 0
 * (a bad polygon: no row past its own max_facets is read).                                     */
blf_status blf_hull2d_contains(blf_handle* handle, const double* A, const double* b,
                               const int32_t* nfacets, int32_t max_facets, const double* query,
                               int64_t batch, int32_t* inside, void* stream);

/* 3-D H-representation (ConvexHullHelper on 3 x p points).  pts: [B][P][3] (P <=
 * BLF_HULL_MAX_POINTS), npts: [B].  Output padded to max_facets rows: A: [B][max_facets][3] unit
 * outward normals, b: [B][max_facets] (inside: A x <= b), nfacets: [B].  The rows are the distinct
 * supporting planes of the set (a face Qhull "Qt" splits into triangles is one row here; compare
 * as sets of planes), b = the largest n . p over the input points, so every input point is
 * inside exactly.  nfacets = -1 for fewer than 4 points, a flat set, or more than max_facets
 * planes.  Rule and tolerances: oracle orc_hull3d_hrep.                                       */
#define BLF_HULL3D_MAX_FACETS 64
blf_status blf_hull3d_hrep(blf_handle* handle, const double* pts, const int32_t* npts,
                           int32_t max_points, int32_t max_facets, int64_t batch,
                           double* A, double* b, int32_t* nfacets, void* stream);

/* n-D H-representation (ConvexHullHelper on n x p points, any n: ConvexHullHelper.cpp:35-99 hands
 * the matrix to Qhull).  pts: [B][P][dim] (1 <= dim <= BLF_HULLND_MAX_DIM, P <=
 * BLF_HULLND_MAX_POINTS, C(P, dim) <= BLF_HULLND_MAX_SUBSETS), npts: [B].  Output padded to
 * max_facets rows (<= BLF_HULLND_MAX_FACETS): A: [B][max_facets][dim] unit outward normals,
 * b: [B][max_facets] (inside: A x <= b), nfacets: [B].  The rows are the distinct supporting
 * hyperplanes through dim of the points (a facet Qhull "Qt" splits into simplices is one row;
 * compare as sets), b = the largest n . p over the points; dim = 1: the rows +1 / -1.
 * nfacets = -1 for fewer than dim + 1 points, a set spanning fewer than dim dimensions, or more
 * than max_facets planes.  One wavefront per set.  Rule and order: oracle orc_hullnd_hrep. */
#define BLF_HULLND_MAX_DIM 8
#define BLF_HULLND_MAX_POINTS 32
#define BLF_HULLND_MAX_FACETS 1024
#define BLF_HULLND_MAX_SUBSETS (1 << 20)
blf_status blf_hullnd_hrep(blf_handle* handle, int32_t dim, const double* pts, const int32_t* npts,
                           int32_t max_points, int32_t max_facets, int64_t batch, double* A,
                           double* b, int32_t* nfacets, void* stream);

/* doesPointBelongToConvexHull in `dim` dimensions: A: [B][max_facets][dim], b: [B][max_facets],
 * query: [B][dim]; inside[q] = 1 iff no row i < nfacets has (A p)_i > b_i (sum in column order
 * from 0.0).  nfacets < 0 or nfacets > max_facets gives 0.                                      */
blf_status blf_halfspace_contains(blf_handle* handle, const double* A, const double* b,
                                  const int32_t* nfacets, int32_t dim, int32_t max_facets,
                                  const double* query, int64_t batch, int32_t* inside,
                                  void* stream);

/* ---- 4. Quintic spline (swing foot) -------------------------------------------------------
 * A spline has K+1 knots t_0 < ... < t_K, and per knot and per axis (D axes, D <= 3) the
 * position, velocity and acceleration.  Segment j spans [t_j, t_{j+1}] and is the unique
 * quintic matching (p, v, a) at both ends.
 * fit:  knots_t: [S][K+1], knots_pva: [S][K+1][3 (p,v,a)][D]  ->  coeffs: [S][K][D][6]
 *       (c0..c5 of p(tau) = sum c_i tau^i, tau = t - t_j).
 * eval: query t: [S][Q]; segment = last knot j with t_j <= t, clamped to [0, K-1] (the
 *       getPresentContact rule, ContactList.cpp:190-202; t < t_0 -> segment 0); tau = t - t_j;
 *       pva out: [S][Q][3][D] (position, velocity, acceleration), knot_idx out: [S][Q].     */
blf_status blf_quintic_fit(blf_handle* handle, const double* knots_t, const double* knots_pva,
                           int32_t nknots, int32_t dim, int64_t nsplines, double* coeffs,
                           void* stream);
blf_status blf_quintic_eval(blf_handle* handle, const double* knots_t, const double* coeffs,
                            int32_t nknots, int32_t dim, int64_t nsplines, const double* tq,
                            int32_t nq, double* pva, int32_t* knot_idx, void* stream);

/* ---- 5. Time-varying DCM MPC QP (TimeVaryingDCMPlanner), batched ---------------------------
 * Per problem, with alpha_k = 1 + dt*omega_k, beta_k = dt*omega_k:
 *   min  sum_{k=0}^{N-1} 1/2|xi_k - xi_ref_k|^2_Q + 1/2|r_k - r_ref_k|^2_R + 1/2|xi_N - xi_ref_N|^2_P
 *   s.t. xi_0 = xi_init,  xi_{k+1} = xi_k + dt*omega_k*(xi_k - r_k)  (reference Euler step),
 *        A_k r_k <= b_k  (rows i < nfacets[k] of the support polygon H-rep)
 * Solved by a Mehrotra primal-dual interior point method whose Newton systems are factored by a
 * Riccati recursion over the knots (DESIGN.md section 4 gives the exact iteration).           */
typedef struct blf_dcm_mpc_params {
    int32_t horizon;       /* N >= 1                                                        */
    int32_t max_facets;    /* M, 1..16 (padded facet slots per knot; above 8 the interior     *
                            * point kernel alone: support polygons of three or four contacts) */
    int32_t max_iter;      /* IPM iteration cap (e.g. 50)                                   */
    int32_t reserved;      /* must be 0                                                     */
    double dt;             /* knot spacing [s]                                              */
    double w_xi[2];        /* Q diagonal                                                    */
    double w_vrp[2];       /* R diagonal                                                    */
    double w_terminal[2];  /* P diagonal                                                    */
    double tol_mu;         /* stop when mean complementarity <= tol_mu ...                   */
    double tol_primal;     /* ... and max |primal residual|, |dynamics defect| <= tol_primal */
    double tol_dual;       /* ... and the tracked dual residual bound <= tol_dual            */
    double tol_polish;     /* > 0: once mean complementarity <= tol_polish, try the active-set
                            * polish: one Newton step of the QP with the guessed
                            * active facets as equalities, accepted only if it certifies as the
                            * optimum (primal feasible, stationary, multipliers >= 0 to
                            * tol_primal / tol_dual); else the IPM goes on.  0: IPM only.     */
} blf_dcm_mpc_params;

typedef struct blf_dcm_mpc_problem {
    const double* xi_init;   /* [B][2]                                                      */
    const double* omega;     /* [B][N]      omega_k = sqrt(g / z_k)                          */
    const double* xi_ref;    /* [B][N+1][2]                                                 */
    const double* vrp_ref;   /* [B][N][2]   also the IPM's initial VRP guess                 */
    const double* A;         /* [B][N][M][2]                                                */
    const double* b;         /* [B][N][M]                                                   */
    const int32_t* nfacets;  /* [B][N]                                                      */
} blf_dcm_mpc_problem;

typedef struct blf_dcm_mpc_solution {
    double* xi;              /* [B][N+1][2]                                                 */
    double* vrp;             /* [B][N][2]                                                   */
    int32_t* status;         /* [B]  BLF_QP_*                                               */
    int32_t* iters;          /* [B]  IPM iterations taken                                   */
    int32_t* polished;       /* [B]  optional (NULL: not written): 1 if the solution is the
                              *      certified active-set polish, 0 if the IPM's own iterate    */
    int32_t* passes;         /* [B]  optional (NULL: not written): the drop/add passes the
                              *      active-set kernels ran (a cold start's fp32 search plus its
                              *      fp64 passes; a warm start's fp64 passes), what a warm start
                              *      saves; 0 for a problem the interior point kernel solves alone
                              *      (horizon > 128, max_facets > 8, tol_polish = 0)             */
} blf_dcm_mpc_solution;

/* Warm start of a receding-horizon re-solve (TimeVaryingDCMPlanner::advance()):
 * knot k of the new window starts from knot k + shift of a previous solution of the same plan
 * (shift = 1 after the window moved one knot):
 *   r_k = vrp[k + shift],  s_i = max(b_i - a_i r_k, floor),  lambda_i = max(lambda[k + shift][i], floor)
 * and the cold start's LQ step is skipped.  Knots with k + shift >= N are new to the window and
 * start cold (r_k = vrp_ref_k, s_i = max(b_i - a_i r_k, 1e-2), lambda_i = 1e-2 / s_i).
 * prev_status (optional): the status of the solve that produced vrp / lambda.  A problem whose
 * previous status is not BLF_QP_OK (e.g. BLF_QP_MAX_ITER) is not warm-started from that iterate:
 * it is solved exactly as the cold start (warm == NULL) solves it, so one failed window does not
 * poison the next (Advanceable::advance, System/include/BipedalLocomotion/System/Advanceable.h:24-46,
 * is called again after a failure with the planner's previous state).  A warm-started problem
 * (horizon <= 128, the active-set kernels' range) whose warm passes do not certify is solved
 * again from the cold start as well, the interior point method included (round 5; oracle
 * orc_dcm_mpc_solve_warm, ORC_WARM_RETRY): the same result as a cold solve of it.               */
typedef struct blf_dcm_mpc_warm_start {
    const double* vrp;       /* [B][N][2]  VRPs of the previous solve (must not alias the output) */
    const double* lambda;    /* [B][N][M]  its multipliers (blf_dcm_mpc_solve_warm's lambda_out)  */
    int32_t shift;           /* >= 0                                                          */
    int32_t reserved;        /* must be 0                                                     */
    double floor;            /* > 0, e.g. 1e-2                                                */
    const int32_t* prev_status; /* [B] or NULL (NULL: every problem warm-started)             */
} blf_dcm_mpc_warm_start;

/* Batches of at most this many QPs (horizon <= 64) evaluate the solver's recursions in a
 * different association order (the DPP scan tree), tuned for latency; larger
 * batches use the throughput tree.  Both return the certified optimum; the two orders can differ
 * in the last bits, so a problem is bit-reproducible within either size class (and bit-identical to
 * the oracle, which follows the same rule). */
#define BLF_DPP_TREE_MAX_BATCH 1024

/* Fill `p` with the defaults used by the benchmark (dt 0.02, Q 1e2, R 1, P 1e3, tol_mu 1e-16,
 * tol_primal 1e-10, tol_dual 1e-9, tol_polish 3e-4, max_iter 50, max_facets 8). */
void blf_dcm_mpc_default_params(blf_dcm_mpc_params* p, int32_t horizon);

blf_status blf_dcm_mpc_solve(blf_handle* handle, const blf_dcm_mpc_params* params,
                             const blf_dcm_mpc_problem* problem, int64_t batch,
                             const blf_dcm_mpc_solution* solution, void* stream);

/* blf_dcm_mpc_solve from the warm start `warm` (NULL: the cold start, identical to
 * blf_dcm_mpc_solve).  lambda_out [B][N][M] (or NULL) receives the final multipliers, zero in
 * facet slots >= nfacets[k]; it is the next advance()'s warm->lambda.                         */
blf_status blf_dcm_mpc_solve_warm(blf_handle* handle, const blf_dcm_mpc_params* params,
                                  const blf_dcm_mpc_problem* problem,
                                  const blf_dcm_mpc_warm_start* warm, int64_t batch,
                                  const blf_dcm_mpc_solution* solution, double* lambda_out,
                                  void* stream);

/* ---- 5b. Knot -> contact-phase expansion (receding-horizon windows on the device) -----------
 * The phases of each problem's plan (ContactPhaseList::createPhases, Planners/src/
 * ContactPhaseList.cpp:16-84), sorted by begin time, with the H-rep of each phase's support
 * polygon (blf_hull2d_hrep over the phase's active-contact corners) and its reference point:
 *   begin, end: [B][P];  A: [B][P][M][2];  b: [B][P][M];  nfacets: [B][P];  ref: [B][P][2];
 *   nphases: [B] (phases >= nphases[q] are ignored).
 * For the window of knots t_k = (start_knot + k) dt, k = 0..N, knot k belongs to phase
 *   p = the last phase with begin_p <= t_k (the getPresentContact rule, ContactList.cpp:190-202)
 * when t_k < end_p, else to no phase.  Outputs (the blf_dcm_mpc_problem arrays of the window):
 *   A [B][N][M][2], b [B][N][M] = phase p's rows verbatim; nfacets [B][N] = phase p's count;
 *   xi_ref [B][N+1][2] and vrp_ref [B][N][2] = phase p's reference point; a knot outside every
 *   phase gets nfacets = -1 (the QP reports BLF_QP_BAD_FACETS) and zero rows / references.   */
typedef struct blf_phase_table {
    int32_t max_phases;        /* P >= 1                                                     */
    int32_t max_facets;        /* M, 1..16                                                   */
    const int32_t* nphases;    /* [B]                                                        */
    const double* begin;       /* [B][P]                                                     */
    const double* end;         /* [B][P]                                                     */
    const double* A;           /* [B][P][M][2]                                               */
    const double* b;           /* [B][P][M]                                                  */
    const int32_t* nfacets;    /* [B][P]                                                     */
    const double* ref;         /* [B][P][2]                                                  */
} blf_phase_table;

blf_status blf_dcm_phase_expand(blf_handle* handle, const blf_phase_table* phases,
                                int64_t start_knot, double dt, int32_t horizon, int64_t batch,
                                double* A, double* b, int32_t* nfacets, double* xi_ref,
                                double* vrp_ref, void* stream);

/* ---- 5c. Phase-indexed solve: one advance() of the receding horizon in one call ---------------
 * blf_dcm_phase_expand(phases, start_knot, params->dt, params->horizon) followed by
 * blf_dcm_mpc_solve_warm on the expanded window, with the same results bit for bit, for horizons
 * up to 128 (larger: BLF_ERR_UNSUPPORTED; use the two calls).  The window's rows are expanded from
 * the phase table into the solver's on-chip memory instead of through HBM: a problem reads its
 * phase table (a few KB) instead of the window's per-knot arrays (~19 KB at N = 100, M = 8).
 * phases->max_facets must equal params->max_facets.  omega: row q (the window's N values) at
 * omega + q * omega_stride (omega_stride >= N; e.g. the plan's omega shifted by start_knot, no
 * copy).  xi_init, warm, solution and lambda_out as blf_dcm_mpc_solve_warm.
 * window: blf_dcm_phase_expand's output arrays plus the window's omega (omega [B][N]), used as
 * scratch: a problem the active-set passes do not certify continues in the interior point method,
 * which reads its expanded window from there.  Only such problems' rows are written (none, with
 * the default parameters, in every workload measured); the contents are unspecified otherwise. */
typedef struct blf_dcm_mpc_window {
    double* omega;             /* [B][N]                                                     */
    double* xi_ref;            /* [B][N+1][2]                                                */
    double* vrp_ref;           /* [B][N][2]                                                  */
    double* A;                 /* [B][N][M][2]                                               */
    double* b;                 /* [B][N][M]                                                  */
    int32_t* nfacets;          /* [B][N]                                                     */
} blf_dcm_mpc_window;

blf_status blf_dcm_mpc_solve_phased(blf_handle* handle, const blf_dcm_mpc_params* params,
                                    const blf_phase_table* phases, int64_t start_knot,
                                    const double* xi_init, const double* omega,
                                    int64_t omega_stride, const blf_dcm_mpc_warm_start* warm,
                                    int64_t batch, const blf_dcm_mpc_window* window,
                                    const blf_dcm_mpc_solution* solution, double* lambda_out,
                                    void* stream);
/* ---- 6. Contact model (ContinuousContactModel), batched ------------------------------------
 * Rectangular L x W patch, spring k, damper b (ContinuousContactModel.h:22-57).
 * params: [B][4] = {length, width, spring_coeff, damper_coeff} (or one shared [4] when
 * shared_params != 0); twist: [B][6] = {v, w} in mixed representation; pose, null_pose:
 * [B][12] = {p[3], R[9] row-major} (world_T_link and the null-force transform).
 * Outputs (NULL = not computed): wrench [B][6] = {force, torque}; autonomous [B][6] and
 * control [B][36] (6x6 row-major), with d(wrench)/dt = autonomous + control * (dv, dw);
 * regressor [B][12] (6x2 row-major), wrench = regressor * (k, b).
 * As the reference: the wrench and the regressor scale by |R22|, the autonomous dynamics and
 * the control matrix by R22 (no abs, ContinuousContactModel.cpp:127-170).                   */
blf_status blf_contact_model_eval(blf_handle* handle, const double* params, int32_t shared_params,
                                  const double* twist, const double* pose,
                                  const double* null_pose, int64_t batch, double* wrench,
                                  double* autonomous, double* control, double* regressor,
                                  void* stream);

/* Force and torque (about the contact frame origin) generated at Q points (x, y) of each contact
 * surface: points [B][Q][2] -> force, torque [B][Q][3]; zero outside the rectangle.           */
blf_status blf_contact_point_wrench(blf_handle* handle, const double* params,
                                    int32_t shared_params, const double* twist, const double* pose,
                                    const double* null_pose, int64_t batch, const double* points,
                                    int32_t npoints, double* force, double* torque, void* stream);

/* ---- 7. Floating-base kinematics (FloatingBaseSystemKinematics), batched -------------------
 * State (p [B][3], R [B][9] row-major, s [B][ndof]); input (twist [B][6] mixed, s_dot [B][ndof]):
 *   dp = v,  dR = -R.colwise().cross(w) + rho/2 ((R R^T)^{-1} - I) R,  ds = s_dot
 * (Baumgarte parameter rho, default 0.01 in the reference).  ndof <= BLF_FBK_MAX_DOFS.      */
#define BLF_FBK_MAX_DOFS 64
blf_status blf_fbk_dynamics(blf_handle* handle, int32_t ndof, double rho, const double* rot,
                            const double* twist, const double* joint_vel, double* dpos,
                            double* drot, double* djoints, int64_t batch, void* stream);

/* ForwardEuler<FloatingBaseSystemKinematics>::integrate(t0, T) with the inputs held constant:
 * the step schedule and error codes of blf_lti_euler_integrate; every step updates each state
 * element x += dx * dT_i (no re-projection onto SO(3), as ForwardEuler.tpp:37-45).
 * pos, rot, joints are updated in place.                                                      */
blf_status blf_fbk_euler_integrate(blf_handle* handle, int32_t ndof, double rho, double* pos,
                                   double* rot, double* joints, const double* twist,
                                   const double* joint_vel, int64_t batch, double initial_time,
                                   double final_time, double dT, void* stream);

/* ---- 8. Floating-base dynamics (FloatingBaseDynamicalSystem), batched ----------------------
 * A kinematic tree of ndof revolute joints on a 6-DoF floating base (the robot model the reference
 * loads into iDynTree KinDynComputations; blf/robot.py documents the layout).  All pointers are
 * device memory.  Link 0 is the base; joint j moves link j + 1, whose parent link is parent[j]
 * (<= j).  Velocities are in the MIXED representation (iDynTree's default): the base twist is
 * (dp_B/dt, omega_B) in world coordinates.                                                      */
#define BLF_FBD_MAX_DOFS 48
#define BLF_FBD_MAX_CONTACTS 8
typedef struct blf_fb_model {
    int32_t ndof;                 /* n, 1..BLF_FBD_MAX_DOFS                                 */
    int32_t nframes;              /* F, frames contacts may be attached to                  */
    const int32_t* parent;        /* [n]                                                     */
    const double* joint_origin;   /* [n][3]  joint origin in the parent link frame           */
    const double* joint_rot;      /* [n][9]  fixed rotation parent link -> joint frame        */
    const double* joint_axis;     /* [n][3]  unit axis in the joint frame                    */
    const double* link_mass;      /* [n+1]                                                   */
    const double* link_com;       /* [n+1][3] COM in the link frame                         */
    const double* link_inertia;   /* [n+1][9] inertia about the COM, link frame              */
    const int32_t* frame_link;    /* [F]                                                     */
    const double* frame_pose;     /* [F][12] (p, R) of the frame in its link frame           */
    double gravity[3];            /* (0, 0, -9.81) in the reference                          */
    double rho;                   /* Baumgarte parameter of the base rotation rate           */
    const int32_t* joint_type;    /* [n] or NULL (every joint revolute): BLF_JOINT_REVOLUTE /
                                     BLF_JOINT_PRISMATIC (the child link slides along the axis
                                     by q; URDF "prismatic"); any other value makes every
                                     output of every robot NaN (the wrappers refuse it up
                                     front: the C++ adapter's setRobotModel returns false,
                                     blf.native raises).  Fixed joints carry no DoF: merge
                                     them into their parent link first (the C++ adapter's
                                     blf::reduceFixedJoints)                                  */
} blf_fb_model;
#define BLF_JOINT_REVOLUTE  0
#define BLF_JOINT_PRISMATIC 1

/* The state tuple (FloatingBaseSystemDynamics.h: base velocity, joint velocities, base position,
 * base orientation, joint positions); the same struct carries the state derivative (base
 * acceleration, joint accelerations, base linear velocity, base rotation rate, joint velocities). */
typedef struct blf_fb_state {
    double* base_vel;   /* [B][6]  */
    double* joint_vel;  /* [B][n]  */
    double* base_pos;   /* [B][3]  */
    double* base_rot;   /* [B][9]  row-major */
    double* joint_pos;  /* [B][n]  */
} blf_fb_state;

/* Contacts of the control input (the reference's std::vector<ContactWrench>, each a frame index
 * and a std::weak_ptr<ContactModel>; FloatingBaseSystemDynamics.cpp:198-228 maps every contact's
 * getContactWrench() through the frame Jacobian).  Each contact follows one of two laws:
 *   BLF_CONTACT_CONTINUOUS  a ContinuousContactModel (params, null_pose), updated on the device
 *                           with the frame's world transform and mixed velocity at every
 *                           evaluation, as the reference's setState + getContactWrench;
 *   BLF_CONTACT_WRENCH      any other ContactModel: the caller evaluates it (its setState from
 *                           blf_fb_frame_state, then getContactWrench) and passes the wrench,
 *                           (force, torque) in the mixed representation at the frame; held
 *                           constant over one blf_fbd_euler_integrate call (the C++ adapter
 *                           integrates step by step when a contact has this law).
 * law == NULL: every contact BLF_CONTACT_CONTINUOUS; any law value other than BLF_CONTACT_WRENCH
 * is taken as continuous.  params and null_pose are required for every contact (ignored for
 * BLF_CONTACT_WRENCH ones), wrench whenever law is given. */
#define BLF_CONTACT_CONTINUOUS 0
#define BLF_CONTACT_WRENCH     1
typedef struct blf_fb_contacts {
    int32_t ncontacts;            /* 0..BLF_FBD_MAX_CONTACTS                                  */
    const int32_t* frame;         /* [C] frame indices                                       */
    const double* params;         /* [C][4] (length, width, spring_coeff, damper_coeff)      */
    const double* null_pose;      /* [B][C][12] null-force transforms                        */
    const int32_t* law;           /* [C] BLF_CONTACT_* or NULL (all continuous)              */
    const double* wrench;         /* [B][C][6] wrenches of the BLF_CONTACT_WRENCH contacts   */
} blf_fb_contacts;

/* The world transform pose [B][K][12] = (p, R row-major) and the mixed velocity twist [B][K][6]
 * = (v, w) of K frames of every system (either output may be NULL): what the reference hands a
 * contact model through kinDyn getWorldTransform / getFrameVel (FloatingBaseSystemDynamics.cpp:
 * 225-226) before it asks for the wrench, for the caller's BLF_CONTACT_WRENCH models.  A frame
 * index outside [0, model->nframes) yields NaN pose and twist for that frame (no read past the
 * model).                                                                                        */
blf_status blf_fb_frame_state(blf_handle* handle, const blf_fb_model* model,
                              const blf_fb_state* state, int32_t nframes, const int32_t* frames,
                              int64_t batch, double* pose, double* twist, void* stream);

/* FloatingBaseDynamicalSystem::dynamics for a batch:
 *   nu_dot = LLT(M [+ mass_reg]) \ (-h + sum_c J_c^T w_c + [0; tau]),  dp = v_B,
 *   dR = -R.colwise().cross(w_B) + rho/2 ((R R^T)^{-1} - I) R,  ds = s_dot
 * joint_torque [B][n]; mass_reg [(n+6)^2] row-major or NULL; out receives the derivative. */
blf_status blf_fbd_dynamics(blf_handle* handle, const blf_fb_model* model,
                            const blf_fb_state* state, const double* joint_torque,
                            const blf_fb_contacts* contacts, const double* mass_reg,
                            int64_t batch, const blf_fb_state* out, void* stream);

/* ForwardEuler<FloatingBaseDynamicalSystem>::integrate(t0, T): the schedule and errors of
 * blf_lti_euler_integrate; each step evaluates the dynamics at the current state (torques and
 * contact parameters held constant) and updates every state element x += dx * dT_i.           */
blf_status blf_fbd_euler_integrate(blf_handle* handle, const blf_fb_model* model,
                                   const blf_fb_state* state, const double* joint_torque,
                                   const blf_fb_contacts* contacts, const double* mass_reg,
                                   int64_t batch, double initial_time, double final_time,
                                   double dT, void* stream);

/* ---- 9. Closed loop (BASELINE.json configs[4]): the maps between the robot and the planner ----
 * The reference has no closed-loop API: a user drives TimeVaryingDCMPlanner::advance()
 * (System/Advanceable.h:24-46) and ForwardEuler<FloatingBaseDynamicalSystem>::integrate
 * (ForwardEuler.tpp:18-49 over FloatingBaseSystemDynamics.cpp:102-251) in turn and maps the robot
 * state to the plan's initial DCM and the plan to the robot's input.  These two entry points are
 * those maps:
 *
 * blf_fb_dcm: state -> centre of mass c, its velocity cdot and the DCM
 *   c = sum_l m_l (p_l + R_l com_l) / m,  cdot = sum_l m_l (v_l + w_l x R_l com_l) / m,
 *   xi = c_xy + cdot_xy / omega0[b * omega0_stride]  (the plan's first-knot omega).
 *   com [B][6] = (c, cdot); xi [B][2] (may be the next solve's xi_init) or NULL.            */
blf_status blf_fb_dcm(blf_handle* handle, const blf_fb_model* model, const blf_fb_state* state,
                      const double* omega0, int64_t omega0_stride, int64_t batch, double* com,
                      double* xi, void* stream);

/* blf_dcm_posture_reference: plan -> joint references, held over the control period:
 *   q_ref[b][j] = q_nominal_j + lean_j0 (r0_x - c_x) + lean_j1 (r0_y - c_y)
 *   with r0 = vrp[b * vrp_stride + (0, 1)] (the plan's first VRP) and c = com[b][0..1].  The joint
 *   impedance of blf_fbd_euler_integrate_impedance tracks them.                               */
typedef struct blf_posture_law {
    int32_t ndof;                 /* n                                                       */
    int32_t reserved;             /* must be 0                                               */
    const double* q_nominal;      /* [n]                                                     */
    const double* lean;           /* [n][2] joint offset per metre of (r0 - c)              */
} blf_posture_law;
blf_status blf_dcm_posture_reference(blf_handle* handle, const blf_posture_law* law,
                                     const double* com, const double* vrp, int64_t vrp_stride,
                                     int64_t batch, double* q_ref, void* stream);
/* blf_fbd_euler_integrate_impedance: ForwardEuler<FloatingBaseDynamicalSystem>::integrate(t0, T)
 * (the schedule of blf_fbd_euler_integrate) with the control input set before EVERY step from a
 * joint impedance, tau = kp (q_ref - q) - kd qdot at the step's start state: the reference loop
 * `system->setControlInput(tau(x)); integrator.integrate(t_i, t_i + dT_i)` a user writes for a
 * joint-level controller faster than the planner, in one launch.                             */
typedef struct blf_joint_impedance {
    int32_t ndof;                 /* n, must match the model                                 */
    int32_t reserved;             /* must be 0                                               */
    const double* kp;             /* [n]                                                     */
    const double* kd;             /* [n]                                                     */
    const double* q_ref;          /* [B][n]                                                  */
} blf_joint_impedance;
blf_status blf_fbd_euler_integrate_impedance(blf_handle* handle, const blf_fb_model* model,
                                             const blf_fb_state* state,
                                             const blf_joint_impedance* impedance,
                                             const blf_fb_contacts* contacts,
                                             const double* mass_reg, int64_t batch,
                                             double initial_time, double final_time, double dT,
                                             void* stream);
/* Algorithmic flop count of one IPM iteration of one problem (what the fp64 roofline field
 * of bench.py is computed from); `active_facets` = sum_k nfacets[k]. */
double blf_dcm_mpc_flops_per_iter(int32_t horizon, int64_t active_facets);

#ifdef __cplusplus
}
#endif

#endif /* BLF_C_H */
