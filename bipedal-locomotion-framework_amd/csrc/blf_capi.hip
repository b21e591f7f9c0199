// blf_capi.hip — the extern "C" boundary declared in include/blf/blf_c.h: argument validation,
// the reference's error semantics, and dispatch to the kernels' launchers.
#include <algorithm>
#include <cmath>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "blf_internal.h"

namespace blf {

static thread_local char g_err[512] = "no error";

QpLaunchMode& qp_launch_mode()
{
    static QpLaunchMode mode{{[] {
                                 const char* fz = getenv("BLF_QP_FUSE_STAGE2");
                                 return !(fz && fz[0] == '0') ? 1 : 0;
                             }()},
                             {[] {
                                 const char* sk = getenv("BLF_QP_SINGLE_KERNEL");
                                 return (sk && sk[0] == '1') ? 1 : 0;
                             }()},
                             [] {
                                 const char* lg = getenv("BLF_QP_LIST_GRID");
                                 const int v = lg ? atoi(lg) : 0;
                                 return v > 0 ? v : kListGrid;
                             }()};
    return mode;
}

blf_status set_error(blf_status code, const char* fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

blf_status check_hip(hipError_t e, const char* what)
{
    if (e == hipSuccess) return BLF_OK;
    return set_error(BLF_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

Handle::~Handle()
{
    for (auto& kv : lists) (void)hipFree(kv.second.buf);   // (hipFree waits for the device)
}

blf_status Handle::stage2_list(hipStream_t s, int64_t batch, Stage2List* out)
{
    // the list's slot toggles on the host between solves and may need a stream synchronisation to
    // grow: a captured graph would freeze one toggle and fail the synchronisation, so a solve under
    // stream capture is refused (the solve itself is capture-safe; its bookkeeping is not)
    hipStreamCaptureStatus cap_st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap_st) == hipSuccess && cap_st != hipStreamCaptureStatusNone)
        return set_error(BLF_ERR_UNSUPPORTED, "DCM-MPC solve under stream capture (the stage-2 list is host-sequenced)");
    std::lock_guard<std::mutex> lock(mu);
    List& l = lists[s];
    if (l.cap < batch) {
        // the old list may still be read by the stream's last solve: let it finish first
        blf_status st = check_hip(hipStreamSynchronize(s), "stage-2 list: hipStreamSynchronize");
        if (st != BLF_OK) return st;
        if (l.buf) (void)hipFree(l.buf);
        l.buf = nullptr;
        l.cap = 0;
        const int64_t cap = std::max<int64_t>(batch, 4096);
        st = check_hip(hipMalloc(&l.buf, sizeof(int32_t) * (size_t)(cap + 2)), "stage-2 list: hipMalloc");
        if (st != BLF_OK) return st;
        st = check_hip(hipMemset(l.buf, 0, sizeof(int32_t) * 2), "stage-2 list: hipMemset");
        if (st != BLF_OK) {
            (void)hipFree(l.buf);
            l.buf = nullptr;
            return st;
        }
        l.cap = cap;
        l.slot = 0;
    }
    *out = Stage2List{l.buf, &l.slot, l.cap};
    return BLF_OK;
}

}  // namespace blf

using namespace blf;

struct blf_handle {
    Handle h;
};

#define BLF_REQUIRE(cond, ...)                                                             \
    do {                                                                                   \
        if (!(cond)) return set_error(BLF_ERR_INVALID_ARGUMENT, __VA_ARGS__);              \
    } while (0)

// FixedStepIntegrator::integrate's step schedule (FixedStepIntegrator.tpp:21-72): validation in
// the reference's order, iterations = ceil((T - t0) / dT); steps 0..iterations-2 advance by dT and
// the last one by T - currentTime with the stale currentTime = t0 + dT (iterations - 2) (:48-64).
static blf_status step_schedule(double initial_time, double final_time, double dT,
                                int* iterations_out, double* dT_last_out)
{
    if (initial_time > final_time)                                                      // :26-30
        return set_error(BLF_ERR_TIME_INTERVAL,
                         "[FixedStepIntegrator::integrate] The final time has to be greater than "
                         "the initial one.");
    if (!(dT > 0))                                                                      // :40-46
        return set_error(BLF_ERR_TIME_INTERVAL,
                         "[FixedStepIntegrator::integrate] The sampling time must be a strictly "
                         "positive number.");
    if (initial_time == final_time)
        return set_error(BLF_ERR_EMPTY_INTERVAL,
                         "integrate(t, t): the reference loops forever here "
                         "(FixedStepIntegrator.tpp:51, size_t i < -1); refused");
    const double q = ceil((final_time - initial_time) / dT);                            // :48
    if (!(q < 2.0e9)) return set_error(BLF_ERR_UNSUPPORTED, "too many integration steps");
    const int iterations = (int)q;
    double currentTime = initial_time;
    if (iterations >= 2) currentTime = initial_time + dT * (double)(iterations - 2);   // :53
    *iterations_out = iterations;
    *dT_last_out = final_time - currentTime;                                            // :64
    return BLF_OK;
}

extern "C" {

blf_status blf_create(blf_handle** handle, int32_t device)
{
    BLF_REQUIRE(handle != nullptr, "blf_create: null handle pointer");
    int count = 0;
    blf_status st = check_hip(hipGetDeviceCount(&count), "hipGetDeviceCount");
    if (st != BLF_OK) return st;
    if (device < 0 || device >= count)
        return set_error(BLF_ERR_HIP, "blf_create: device %d not present (%d devices)", device, count);
    st = check_hip(hipSetDevice(device), "hipSetDevice");
    if (st != BLF_OK) return st;
    blf_handle* h = new blf_handle;
    h->h.device = device;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) h->h.num_cus = prop.multiProcessorCount;
    *handle = h;
    return BLF_OK;
}

blf_status blf_destroy(blf_handle* handle)
{
    delete handle;
    return BLF_OK;
}

const char* blf_last_error(void) { return g_err; }

blf_status blf_step_schedule(double initial_time, double final_time, double dT, int32_t* iterations,
                             double* dT_last, double* t_last)
{
    BLF_REQUIRE(iterations && dT_last && t_last, "blf_step_schedule: null output");
    int it = 0;
    double last = 0.0;
    const blf_status st = step_schedule(initial_time, final_time, dT, &it, &last);
    if (st != BLF_OK) return st;
    *iterations = it;
    *dT_last = last;
    *t_last = it >= 2 ? initial_time + dT * (double)(it - 2) : initial_time;   // :53, as step_schedule
    return BLF_OK;
}

#ifndef BLF_SRC_HASH
#define BLF_SRC_HASH "unknown"
#endif
// The sources' hash (Makefile SRC_HASH) makes the loaded library traceable to the tree it was
// built from (blf/native.py build_provenance).
const char* blf_version(void) { return "blf-mi355x 0.2.0 (abi 2, gfx950, fp64, -ffp-contract=off) src " BLF_SRC_HASH; }


blf_status blf_set_qp_launch_mode(int32_t fuse_stage2, int32_t single_kernel)
{
    BLF_REQUIRE(fuse_stage2 >= -1 && fuse_stage2 <= 1 && single_kernel >= -1 && single_kernel <= 1,
                "blf_set_qp_launch_mode: settings are -1, 0 or 1");
    QpLaunchMode& m = qp_launch_mode();
    if (fuse_stage2 >= 0) m.fuse_stage2.store(fuse_stage2, std::memory_order_relaxed);
    if (single_kernel >= 0) m.single_kernel.store(single_kernel, std::memory_order_relaxed);
    return BLF_OK;
}

blf_status blf_lti_euler_integrate(blf_handle* handle, int32_t n, int32_t m, const double* A,
                                   const double* Bm, int32_t shared_matrices, const double* u,
                                   double* x, int64_t batch, double initial_time,
                                   double final_time, double dT, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_lti_euler_integrate: null handle");
    BLF_REQUIRE(n >= 1 && m >= 1, "blf_lti_euler_integrate: n=%d m=%d, both must be >= 1", n, m);
    BLF_REQUIRE(batch >= 0, "blf_lti_euler_integrate: negative batch");
    BLF_REQUIRE(batch == 0 || (A && Bm && u && x), "blf_lti_euler_integrate: null buffer");
    int iterations = 0;
    double dT_last = 0.0;
    const blf_status st = step_schedule(initial_time, final_time, dT, &iterations, &dT_last);
    if (st != BLF_OK) return st;
    return launch_lti_euler(n, m, A, Bm, shared_matrices, u, x, batch, iterations, dT, dT_last,
                            (hipStream_t)stream);
}

blf_status blf_lti_dynamics(blf_handle* handle, int32_t n, int32_t m, const double* A,
                            const double* Bm, int32_t shared_matrices, const double* u,
                            const double* x, double* dx, int64_t batch, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_lti_dynamics: null handle");
    BLF_REQUIRE(n >= 1 && m >= 1, "blf_lti_dynamics: n=%d m=%d, both must be >= 1", n, m);
    BLF_REQUIRE(batch >= 0, "blf_lti_dynamics: negative batch");
    BLF_REQUIRE(batch == 0 || (A && Bm && u && x && dx), "blf_lti_dynamics: null buffer");
    return launch_lti_dynamics(n, m, A, Bm, shared_matrices, u, x, dx, batch, (hipStream_t)stream);
}

blf_status blf_dcm_euler_rollout(blf_handle* handle, const double* xi0, const double* omega,
                                 const double* vrp, int32_t horizon, double dt, double* xi_out,
                                 int64_t batch, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_dcm_euler_rollout: null handle");
    BLF_REQUIRE(horizon >= 1, "blf_dcm_euler_rollout: horizon %d < 1", horizon);
    BLF_REQUIRE(batch >= 0, "blf_dcm_euler_rollout: negative batch");
    BLF_REQUIRE(batch == 0 || (xi0 && omega && vrp && xi_out), "blf_dcm_euler_rollout: null buffer");
    return launch_dcm_rollout(xi0, omega, vrp, horizon, dt, xi_out, batch, (hipStream_t)stream);
}

blf_status blf_hull2d_hrep(blf_handle* handle, const double* pts, const int32_t* npts,
                           int32_t max_points, int32_t max_facets, int64_t batch, double* A,
                           double* b, int32_t* nfacets, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_hull2d_hrep: null handle");
    BLF_REQUIRE(max_points >= 1 && max_points <= BLF_HULL_MAX_POINTS,
                "blf_hull2d_hrep: max_points %d outside [1, %d]", max_points, BLF_HULL_MAX_POINTS);
    BLF_REQUIRE(max_facets >= 1 && max_facets <= 2 * BLF_HULL_MAX_POINTS,
                "blf_hull2d_hrep: max_facets %d", max_facets);
    BLF_REQUIRE(batch >= 0, "blf_hull2d_hrep: negative batch");
    BLF_REQUIRE(batch == 0 || (pts && npts && A && b && nfacets), "blf_hull2d_hrep: null buffer");
    return launch_hull2d(pts, npts, max_points, max_facets, batch, A, b, nfacets,
                         (hipStream_t)stream);
}

blf_status blf_hull2d_contains(blf_handle* handle, const double* A, const double* b,
                               const int32_t* nfacets, int32_t max_facets, const double* query,
                               int64_t batch, int32_t* inside, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_hull2d_contains: null handle");
    BLF_REQUIRE(max_facets >= 1, "blf_hull2d_contains: max_facets %d", max_facets);
    BLF_REQUIRE(batch >= 0, "blf_hull2d_contains: negative batch");
    BLF_REQUIRE(batch == 0 || (A && b && nfacets && query && inside),
                "blf_hull2d_contains: null buffer");
    return launch_hull2d_contains(A, b, nfacets, max_facets, query, batch, inside,
                                  (hipStream_t)stream);
}

blf_status blf_hull3d_hrep(blf_handle* handle, const double* pts, const int32_t* npts,
                           int32_t max_points, int32_t max_facets, int64_t batch, double* A,
                           double* b, int32_t* nfacets, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_hull3d_hrep: null handle");
    BLF_REQUIRE(max_points >= 1 && max_points <= BLF_HULL_MAX_POINTS,
                "blf_hull3d_hrep: max_points %d outside [1, %d]", max_points, BLF_HULL_MAX_POINTS);
    BLF_REQUIRE(max_facets >= 1 && max_facets <= BLF_HULL3D_MAX_FACETS,
                "blf_hull3d_hrep: max_facets %d outside [1, %d]", max_facets, BLF_HULL3D_MAX_FACETS);
    BLF_REQUIRE(batch >= 0, "blf_hull3d_hrep: negative batch");
    BLF_REQUIRE(batch == 0 || (pts && npts && A && b && nfacets), "blf_hull3d_hrep: null buffer");
    return launch_hull3d(pts, npts, max_points, max_facets, batch, A, b, nfacets,
                         (hipStream_t)stream);
}

blf_status blf_hullnd_hrep(blf_handle* handle, int32_t dim, const double* pts, const int32_t* npts,
                           int32_t max_points, int32_t max_facets, int64_t batch, double* A,
                           double* b, int32_t* nfacets, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_hullnd_hrep: null handle");
    BLF_REQUIRE(dim >= 1 && dim <= BLF_HULLND_MAX_DIM, "blf_hullnd_hrep: dim %d outside [1, %d]", dim,
                BLF_HULLND_MAX_DIM);
    BLF_REQUIRE(max_points >= 1 && max_points <= BLF_HULLND_MAX_POINTS,
                "blf_hullnd_hrep: max_points %d outside [1, %d]", max_points, BLF_HULLND_MAX_POINTS);
    BLF_REQUIRE(max_facets >= 1 && max_facets <= BLF_HULLND_MAX_FACETS,
                "blf_hullnd_hrep: max_facets %d outside [1, %d]", max_facets, BLF_HULLND_MAX_FACETS);
    BLF_REQUIRE(batch >= 0, "blf_hullnd_hrep: negative batch");
    BLF_REQUIRE(batch == 0 || (pts && npts && A && b && nfacets), "blf_hullnd_hrep: null buffer");
    int64_t subsets = 1;   // C(max_points, dim)
    for (int k = 1; k <= dim; ++k) subsets = subsets * (max_points - dim + k) / k;
    if (subsets > BLF_HULLND_MAX_SUBSETS)
        return set_error(BLF_ERR_UNSUPPORTED, "blf_hullnd_hrep: C(%d, %d) = %lld subsets above %d",
                         max_points, dim, (long long)subsets, BLF_HULLND_MAX_SUBSETS);
    return launch_hullnd(dim, pts, npts, max_points, max_facets, batch, A, b, nfacets,
                         (hipStream_t)stream);
}

blf_status blf_halfspace_contains(blf_handle* handle, const double* A, const double* b,
                                  const int32_t* nfacets, int32_t dim, int32_t max_facets,
                                  const double* query, int64_t batch, int32_t* inside, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_halfspace_contains: null handle");
    BLF_REQUIRE(dim >= 1, "blf_halfspace_contains: dim %d", dim);
    BLF_REQUIRE(max_facets >= 1, "blf_halfspace_contains: max_facets %d", max_facets);
    BLF_REQUIRE(batch >= 0, "blf_halfspace_contains: negative batch");
    BLF_REQUIRE(batch == 0 || (A && b && nfacets && query && inside),
                "blf_halfspace_contains: null buffer");
    return launch_halfspace_contains(A, b, nfacets, dim, max_facets, query, batch, inside,
                                     (hipStream_t)stream);
}

blf_status blf_quintic_fit(blf_handle* handle, const double* knots_t, const double* knots_pva,
                           int32_t nknots, int32_t dim, int64_t nsplines, double* coeffs,
                           void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_quintic_fit: null handle");
    BLF_REQUIRE(nknots >= 2, "blf_quintic_fit: nknots %d < 2", nknots);
    BLF_REQUIRE(dim >= 1 && dim <= 3, "blf_quintic_fit: dim %d outside [1, 3]", dim);
    BLF_REQUIRE(nsplines >= 0, "blf_quintic_fit: negative nsplines");
    BLF_REQUIRE(nsplines == 0 || (knots_t && knots_pva && coeffs), "blf_quintic_fit: null buffer");
    return launch_quintic_fit(knots_t, knots_pva, nknots, dim, nsplines, coeffs,
                              (hipStream_t)stream);
}

blf_status blf_quintic_eval(blf_handle* handle, const double* knots_t, const double* coeffs,
                            int32_t nknots, int32_t dim, int64_t nsplines, const double* tq,
                            int32_t nq, double* pva, int32_t* knot_idx, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_quintic_eval: null handle");
    BLF_REQUIRE(nknots >= 2, "blf_quintic_eval: nknots %d < 2", nknots);
    BLF_REQUIRE(dim >= 1 && dim <= 3, "blf_quintic_eval: dim %d outside [1, 3]", dim);
    BLF_REQUIRE(nsplines >= 0 && nq >= 0, "blf_quintic_eval: negative size");
    BLF_REQUIRE(nsplines == 0 || nq == 0 || (knots_t && coeffs && tq && pva && knot_idx),
                "blf_quintic_eval: null buffer");
    return launch_quintic_eval(knots_t, coeffs, nknots, dim, nsplines, tq, nq, pva, knot_idx,
                               (hipStream_t)stream);
}

void blf_dcm_mpc_default_params(blf_dcm_mpc_params* p, int32_t horizon)
{
    if (!p) return;
    memset(p, 0, sizeof(*p));
    p->horizon = horizon;
    p->max_facets = 8;
    p->max_iter = 50;
    p->dt = 0.02;
    p->w_xi[0] = p->w_xi[1] = 1e2;
    p->w_vrp[0] = p->w_vrp[1] = 1.0;
    p->w_terminal[0] = p->w_terminal[1] = 1e3;
    p->tol_mu = 1e-16;
    p->tol_primal = 1e-10;
    p->tol_dual = 1e-9;
    p->tol_polish = 3e-4;
}

blf_status blf_dcm_phase_expand(blf_handle* handle, const blf_phase_table* ph,
                                int64_t start_knot, double dt, int32_t horizon, int64_t batch,
                                double* A, double* b, int32_t* nfacets, double* xi_ref,
                                double* vrp_ref, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_dcm_phase_expand: null handle");
    BLF_REQUIRE(ph != nullptr, "blf_dcm_phase_expand: null phase table");
    BLF_REQUIRE(ph->max_phases >= 1, "blf_dcm_phase_expand: max_phases %d < 1", ph->max_phases);
    BLF_REQUIRE(ph->max_facets >= 1 && ph->max_facets <= kMaxFacetsWide,
                "blf_dcm_phase_expand: max_facets %d outside [1, %d]", ph->max_facets, kMaxFacetsWide);
    BLF_REQUIRE(horizon >= 1, "blf_dcm_phase_expand: horizon %d < 1", horizon);
    BLF_REQUIRE(dt > 0 && std::isfinite(dt), "blf_dcm_phase_expand: dt must be finite and > 0");
    BLF_REQUIRE(start_knot >= 0, "blf_dcm_phase_expand: start_knot < 0");
    BLF_REQUIRE(batch >= 0, "blf_dcm_phase_expand: negative batch");
    BLF_REQUIRE(batch == 0 || (ph->nphases && ph->begin && ph->end && ph->A && ph->b &&
                               ph->nfacets && ph->ref && A && b && nfacets && xi_ref && vrp_ref),
                "blf_dcm_phase_expand: null buffer");
    return launch_phase_expand(ph->max_phases, ph->nphases, ph->begin, ph->end, ph->A, ph->b,
                               ph->nfacets, ph->ref, ph->max_facets, start_knot, dt, horizon,
                               batch, A, b, nfacets, xi_ref, vrp_ref, (hipStream_t)stream);
}

// The warm-start argument checks of every QP entry point.
static blf_status check_warm(const char* fn, const blf_dcm_mpc_warm_start* warm, int64_t batch,
                             const blf_dcm_mpc_solution* solution, const double* lambda_out)
{
    if (!warm) return BLF_OK;
    BLF_REQUIRE(batch == 0 || (warm->vrp && warm->lambda), "%s: null warm-start buffer", fn);
    BLF_REQUIRE(warm->shift >= 0, "%s: shift %d < 0", fn, warm->shift);
    BLF_REQUIRE(warm->reserved == 0, "%s: reserved must be 0", fn);
    BLF_REQUIRE(warm->floor > 0 && std::isfinite(warm->floor), "%s: floor must be finite and > 0", fn);
    BLF_REQUIRE(warm->vrp != solution->vrp && warm->lambda != lambda_out &&
                    (warm->prev_status == nullptr || warm->prev_status != solution->status),
                "%s: warm-start buffers must not alias the outputs", fn);
    return BLF_OK;
}

blf_status blf_dcm_mpc_solve_warm(blf_handle* handle, const blf_dcm_mpc_params* params,
                                  const blf_dcm_mpc_problem* problem,
                                  const blf_dcm_mpc_warm_start* warm, int64_t batch,
                                  const blf_dcm_mpc_solution* solution, double* lambda_out,
                                  void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_dcm_mpc_solve: null handle");
    BLF_REQUIRE(params && problem && solution, "blf_dcm_mpc_solve: null argument");
    BLF_REQUIRE(params->horizon >= 1, "blf_dcm_mpc_solve: horizon %d < 1", params->horizon);
    BLF_REQUIRE(params->max_facets >= 1 && params->max_facets <= kMaxFacetsWide,
                "blf_dcm_mpc_solve: max_facets %d outside [1, %d]", params->max_facets, kMaxFacetsWide);
    BLF_REQUIRE(params->max_iter >= 0, "blf_dcm_mpc_solve: max_iter < 0");
    BLF_REQUIRE(params->reserved == 0, "blf_dcm_mpc_solve: reserved must be 0");
    BLF_REQUIRE(params->dt > 0, "blf_dcm_mpc_solve: dt must be > 0");
    BLF_REQUIRE(params->w_vrp[0] > 0 && params->w_vrp[1] > 0 && params->w_xi[0] >= 0 &&
                    params->w_xi[1] >= 0 && params->w_terminal[0] >= 0 && params->w_terminal[1] >= 0,
                "blf_dcm_mpc_solve: weights must be R > 0, Q >= 0, P >= 0");
    BLF_REQUIRE(batch >= 0, "blf_dcm_mpc_solve: negative batch");
    BLF_REQUIRE(batch == 0 || (problem->xi_init && problem->omega && problem->xi_ref &&
                               problem->vrp_ref && problem->A && problem->b && problem->nfacets &&
                               solution->xi && solution->vrp && solution->status && solution->iters),
                "blf_dcm_mpc_solve: null buffer");
    {
        const blf_status st = check_warm("blf_dcm_mpc_solve_warm", warm, batch, solution, lambda_out);
        if (st != BLF_OK) return st;
    }
    if (batch == 0) return BLF_OK;
    Stage2List list{};
    const blf_status st = handle->h.stage2_list((hipStream_t)stream, batch, &list);
    if (st != BLF_OK) return st;
    return launch_dcm_mpc(params, problem, warm, batch, solution, lambda_out, (hipStream_t)stream, list);
}

static blf_status phased_solve(const char* fn, blf_handle* handle,
                               const blf_dcm_mpc_params* params, const blf_phase_table* ph, int64_t start_knot,
                               const double* xi_init, const double* omega, int64_t omega_stride,
                               const blf_dcm_mpc_warm_start* warm, int64_t batch,
                               const blf_dcm_mpc_window* win, const blf_dcm_mpc_solution* solution,
                               double* lambda_out, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "%s: null handle", fn);
    BLF_REQUIRE(params && ph && win && solution, "%s: null argument", fn);
    BLF_REQUIRE(ph->max_phases >= 1, "%s: max_phases %d < 1", fn, ph->max_phases);
    BLF_REQUIRE(ph->max_facets == params->max_facets,
                "%s: phase table max_facets %d != params max_facets %d", fn,
                ph->max_facets, params->max_facets);
    BLF_REQUIRE(start_knot >= 0, "%s: start_knot < 0", fn);
    BLF_REQUIRE(omega_stride >= params->horizon, "%s: omega_stride %lld < horizon %d", fn,
                (long long)omega_stride, params->horizon);
    BLF_REQUIRE(batch == 0 || (ph->nphases && ph->begin && ph->end && ph->A && ph->b && ph->nfacets &&
                               ph->ref && win->omega && win->xi_ref && win->vrp_ref && win->A &&
                               win->b && win->nfacets),
                "%s: null buffer", fn);
    // the QP arguments as blf_dcm_mpc_solve_warm checks them (the window scratch stands in for the
    // per-knot arrays, which this call does not read)
    const blf_dcm_mpc_problem pb{xi_init, omega, win->xi_ref, win->vrp_ref, win->A, win->b, win->nfacets};
    if (batch > 0) {
        BLF_REQUIRE(params->horizon >= 1 && params->horizon <= 128,
                    "%s: horizon %d outside [1, 128]", fn, params->horizon);
        BLF_REQUIRE(params->tol_polish > 0, "%s: tol_polish must be > 0", fn);
    }
    BLF_REQUIRE(params->max_facets >= 1 && params->max_facets <= kMaxFacetsWide,
                "%s: max_facets %d outside [1, %d]", fn, params->max_facets, kMaxFacetsWide);
    BLF_REQUIRE(params->max_iter >= 0, "%s: max_iter < 0", fn);
    BLF_REQUIRE(params->reserved == 0, "%s: reserved must be 0", fn);
    BLF_REQUIRE(params->dt > 0 && std::isfinite(params->dt), "%s: dt must be finite and > 0", fn);
    BLF_REQUIRE(params->w_vrp[0] > 0 && params->w_vrp[1] > 0 && params->w_xi[0] >= 0 &&
                    params->w_xi[1] >= 0 && params->w_terminal[0] >= 0 && params->w_terminal[1] >= 0,
                "%s: weights must be R > 0, Q >= 0, P >= 0", fn);
    BLF_REQUIRE(batch >= 0, "%s: negative batch", fn);
    BLF_REQUIRE(batch == 0 || (pb.xi_init && pb.omega && solution->xi && solution->vrp &&
                               solution->status && solution->iters),
                "%s: null buffer", fn);
    blf_status st = check_warm(fn, warm, batch, solution, lambda_out);
    if (st != BLF_OK || batch == 0) return st;
    Stage2List list{};
    st = handle->h.stage2_list((hipStream_t)stream, batch, &list);
    if (st != BLF_OK) return st;
    return launch_dcm_mpc_phased(params, ph, start_knot, xi_init, omega, omega_stride, warm, batch,
                                 win, solution, lambda_out, (hipStream_t)stream, list);
}

blf_status blf_dcm_mpc_solve_phased(blf_handle* handle, const blf_dcm_mpc_params* params,
                                    const blf_phase_table* ph, int64_t start_knot,
                                    const double* xi_init, const double* omega,
                                    int64_t omega_stride, const blf_dcm_mpc_warm_start* warm,
                                    int64_t batch, const blf_dcm_mpc_window* win,
                                    const blf_dcm_mpc_solution* solution, double* lambda_out,
                                    void* stream)
{
    return phased_solve("blf_dcm_mpc_solve_phased", handle, params, ph, start_knot, xi_init, omega,
                        omega_stride, warm, batch, win, solution, lambda_out, stream);
}

blf_status blf_dcm_mpc_solve(blf_handle* handle, const blf_dcm_mpc_params* params,
                             const blf_dcm_mpc_problem* problem, int64_t batch,
                             const blf_dcm_mpc_solution* solution, void* stream)
{
    return blf_dcm_mpc_solve_warm(handle, params, problem, nullptr, batch, solution, nullptr,
                                  stream);
}

double blf_dcm_mpc_flops_per_iter(int32_t horizon, int64_t active_facets)
{
    // Algorithmic flops of one IPM iteration, counted on the sequential restatement of the
    // algorithm (fp64 add/sub/mul/div = 1 flop, negation / fabs / compares
    // not counted) — the device's lane scans do more arithmetic than this on purpose:
    //   per knot:  residuals 20, E 10, Riccati step 40, H^-1 / M / G 45, two solves 2 x 66,
    //              update 8                                                         = 255
    //   per facet: residual 11, W-phase 22, affine ratio 16, mu_aff 18, corrector rhs 27,
    //              corrector step 31, update 12                                     = 137
    //   per facet pair (det W): 6, i.e. 3 m(m-1) per knot; taken as 12 per facet (m ~ 5)
    return 149.0 * (double)active_facets + 255.0 * (double)horizon;
}

}  // extern "C"

extern "C" {

blf_status blf_contact_model_eval(blf_handle* handle, const double* params, int32_t shared_params,
                                  const double* twist, const double* pose,
                                  const double* null_pose, int64_t batch, double* wrench,
                                  double* autonomous, double* control, double* regressor,
                                  void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_contact_model_eval: null handle");
    BLF_REQUIRE(batch >= 0, "blf_contact_model_eval: negative batch");
    BLF_REQUIRE(batch == 0 || (params && twist && pose && null_pose),
                "blf_contact_model_eval: null input buffer");
    BLF_REQUIRE(wrench || autonomous || control || regressor,
                "blf_contact_model_eval: no output requested");
    return launch_contact_eval(params, shared_params, twist, pose, null_pose, batch, wrench,
                               autonomous, control, regressor, (hipStream_t)stream);
}

blf_status blf_contact_point_wrench(blf_handle* handle, const double* params,
                                    int32_t shared_params, const double* twist, const double* pose,
                                    const double* null_pose, int64_t batch, const double* points,
                                    int32_t npoints, double* force, double* torque, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_contact_point_wrench: null handle");
    BLF_REQUIRE(batch >= 0 && npoints >= 0, "blf_contact_point_wrench: negative size");
    BLF_REQUIRE(batch == 0 || npoints == 0 ||
                    (params && twist && pose && null_pose && points && force && torque),
                "blf_contact_point_wrench: null buffer");
    return launch_contact_point(params, shared_params, twist, pose, null_pose, batch, points,
                                npoints, force, torque, (hipStream_t)stream);
}

blf_status blf_fbk_dynamics(blf_handle* handle, int32_t ndof, double rho, const double* rot,
                            const double* twist, const double* joint_vel, double* dpos,
                            double* drot, double* djoints, int64_t batch, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_fbk_dynamics: null handle");
    BLF_REQUIRE(ndof >= 0 && ndof <= BLF_FBK_MAX_DOFS, "blf_fbk_dynamics: ndof=%d outside [0, %d]",
                ndof, BLF_FBK_MAX_DOFS);
    BLF_REQUIRE(batch >= 0, "blf_fbk_dynamics: negative batch");
    BLF_REQUIRE(batch == 0 || (rot && twist && dpos && drot && (ndof == 0 || (joint_vel && djoints))),
                "blf_fbk_dynamics: null buffer");
    return launch_fbk_dynamics(ndof, rho, rot, twist, joint_vel, dpos, drot, djoints, batch,
                               (hipStream_t)stream);
}

blf_status blf_fbk_euler_integrate(blf_handle* handle, int32_t ndof, double rho, double* pos,
                                   double* rot, double* joints, const double* twist,
                                   const double* joint_vel, int64_t batch, double initial_time,
                                   double final_time, double dT, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_fbk_euler_integrate: null handle");
    BLF_REQUIRE(ndof >= 0 && ndof <= BLF_FBK_MAX_DOFS,
                "blf_fbk_euler_integrate: ndof=%d outside [0, %d]", ndof, BLF_FBK_MAX_DOFS);
    BLF_REQUIRE(batch >= 0, "blf_fbk_euler_integrate: negative batch");
    BLF_REQUIRE(batch == 0 || (pos && rot && twist && (ndof == 0 || (joints && joint_vel))),
                "blf_fbk_euler_integrate: null buffer");
    int iterations = 0;
    double dT_last = 0.0;
    const blf_status st = step_schedule(initial_time, final_time, dT, &iterations, &dT_last);
    if (st != BLF_OK) return st;
    return launch_fbk_euler(ndof, rho, pos, rot, joints, twist, joint_vel, batch, iterations, dT,
                            dT_last, (hipStream_t)stream);
}

}  // extern "C"

static blf_status check_fbd(const char* fn, blf_handle* handle, const blf_fb_model* model,
                            const blf_fb_state* state, const double* tau,
                            const blf_fb_contacts* contacts, int64_t batch)
{
    BLF_REQUIRE(handle != nullptr, "%s: null handle", fn);
    BLF_REQUIRE(model != nullptr && state != nullptr, "%s: null model / state", fn);
    BLF_REQUIRE(model->ndof >= 1 && model->ndof <= BLF_FBD_MAX_DOFS, "%s: ndof=%d outside [1, %d]",
                fn, model->ndof, BLF_FBD_MAX_DOFS);
    BLF_REQUIRE(batch >= 0, "%s: negative batch", fn);
    BLF_REQUIRE(model->parent && model->joint_origin && model->joint_rot && model->joint_axis &&
                    model->link_mass && model->link_com && model->link_inertia,
                "%s: null model array", fn);
    BLF_REQUIRE(batch == 0 || (state->base_vel && state->joint_vel && state->base_pos &&
                               state->base_rot && state->joint_pos && tau),
                "%s: null state buffer", fn);
    const int C = contacts ? contacts->ncontacts : 0;
    BLF_REQUIRE(C >= 0 && C <= BLF_FBD_MAX_CONTACTS, "%s: %d contacts outside [0, %d]", fn, C,
                BLF_FBD_MAX_CONTACTS);
    BLF_REQUIRE(C == 0 || (contacts->frame && contacts->params && contacts->null_pose &&
                           model->frame_link && model->frame_pose && model->nframes > 0),
                "%s: null contact buffer", fn);
    BLF_REQUIRE(C == 0 || contacts->law == nullptr || batch == 0 || contacts->wrench != nullptr,
                "%s: contact laws given without the wrench buffer", fn);
    if (fbd_lds_bytes(model->ndof, C) > 160 * 1024)
        return set_error(BLF_ERR_UNSUPPORTED, "%s: model too large for one workgroup's LDS", fn);
    return BLF_OK;
}

extern "C" {

blf_status blf_fbd_dynamics(blf_handle* handle, const blf_fb_model* model,
                            const blf_fb_state* state, const double* joint_torque,
                            const blf_fb_contacts* contacts, const double* mass_reg,
                            int64_t batch, const blf_fb_state* out, void* stream)
{
    blf_status st = check_fbd("blf_fbd_dynamics", handle, model, state, joint_torque, contacts, batch);
    if (st != BLF_OK) return st;
    BLF_REQUIRE(out != nullptr && (batch == 0 || (out->base_vel && out->joint_vel && out->base_pos &&
                                                  out->base_rot && out->joint_pos)),
                "blf_fbd_dynamics: null output buffer");
    return launch_fbd_dynamics(model, state, joint_torque, contacts, mass_reg, batch, out,
                               (hipStream_t)stream);
}

blf_status blf_fb_dcm(blf_handle* handle, const blf_fb_model* model, const blf_fb_state* state,
                      const double* omega0, int64_t omega0_stride, int64_t batch, double* com,
                      double* xi, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_fb_dcm: null handle");
    BLF_REQUIRE(model != nullptr && state != nullptr, "blf_fb_dcm: null model / state");
    BLF_REQUIRE(model->ndof >= 1 && model->ndof <= BLF_FBD_MAX_DOFS, "blf_fb_dcm: ndof=%d outside [1, %d]",
                model->ndof, BLF_FBD_MAX_DOFS);
    BLF_REQUIRE(batch >= 0, "blf_fb_dcm: negative batch");
    BLF_REQUIRE(model->parent && model->joint_origin && model->joint_rot && model->joint_axis &&
                    model->link_mass && model->link_com && model->link_inertia,
                "blf_fb_dcm: null model array");
    BLF_REQUIRE(batch == 0 || (state->base_vel && state->joint_vel && state->base_pos &&
                               state->base_rot && state->joint_pos && com),
                "blf_fb_dcm: null state / output buffer");
    BLF_REQUIRE(xi == nullptr || omega0 != nullptr, "blf_fb_dcm: xi requested without omega0");
    BLF_REQUIRE(omega0_stride >= 0, "blf_fb_dcm: negative omega0 stride");
    return launch_fb_dcm(model, state, omega0, omega0_stride, batch, com, xi, (hipStream_t)stream);
}

blf_status blf_fb_frame_state(blf_handle* handle, const blf_fb_model* model,
                              const blf_fb_state* state, int32_t nframes, const int32_t* frames,
                              int64_t batch, double* pose, double* twist, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_fb_frame_state: null handle");
    BLF_REQUIRE(model != nullptr && state != nullptr, "blf_fb_frame_state: null model / state");
    BLF_REQUIRE(model->ndof >= 1 && model->ndof <= BLF_FBD_MAX_DOFS,
                "blf_fb_frame_state: ndof=%d outside [1, %d]", model->ndof, BLF_FBD_MAX_DOFS);
    BLF_REQUIRE(batch >= 0 && nframes >= 0, "blf_fb_frame_state: negative size");
    BLF_REQUIRE(model->parent && model->joint_origin && model->joint_rot && model->joint_axis &&
                    model->link_mass && model->link_com && model->link_inertia,
                "blf_fb_frame_state: null model array");
    BLF_REQUIRE(nframes == 0 || (frames && model->frame_link && model->frame_pose && model->nframes > 0),
                "blf_fb_frame_state: null frame buffer");
    BLF_REQUIRE(batch == 0 || nframes == 0 ||
                    ((pose || twist) && state->base_vel && state->joint_vel && state->base_pos &&
                     state->base_rot && state->joint_pos),
                "blf_fb_frame_state: null state / output buffer");
    return launch_fb_frame_state(model, state, nframes, frames, batch, pose, twist,
                                 (hipStream_t)stream);
}

blf_status blf_dcm_posture_reference(blf_handle* handle, const blf_posture_law* law,
                                     const double* com, const double* vrp, int64_t vrp_stride,
                                     int64_t batch, double* q_ref, void* stream)
{
    BLF_REQUIRE(handle != nullptr, "blf_dcm_posture_reference: null handle");
    BLF_REQUIRE(law != nullptr, "blf_dcm_posture_reference: null law");
    BLF_REQUIRE(law->reserved == 0, "blf_dcm_posture_reference: reserved must be 0");
    BLF_REQUIRE(law->ndof >= 1 && law->ndof <= BLF_FBD_MAX_DOFS,
                "blf_dcm_posture_reference: ndof=%d outside [1, %d]", law->ndof, BLF_FBD_MAX_DOFS);
    BLF_REQUIRE(law->q_nominal && law->lean, "blf_dcm_posture_reference: null law array");
    BLF_REQUIRE(batch >= 0 && vrp_stride >= 2, "blf_dcm_posture_reference: bad batch / vrp stride");
    BLF_REQUIRE(batch == 0 || (com && vrp && q_ref), "blf_dcm_posture_reference: null buffer");
    return launch_posture_reference(law, com, vrp, vrp_stride, batch, q_ref, (hipStream_t)stream);
}

blf_status blf_fbd_euler_integrate_impedance(blf_handle* handle, const blf_fb_model* model,
                                             const blf_fb_state* state,
                                             const blf_joint_impedance* impedance,
                                             const blf_fb_contacts* contacts,
                                             const double* mass_reg, int64_t batch,
                                             double initial_time, double final_time, double dT,
                                             void* stream)
{
    BLF_REQUIRE(impedance != nullptr, "blf_fbd_euler_integrate_impedance: null impedance");
    BLF_REQUIRE(impedance->reserved == 0, "blf_fbd_euler_integrate_impedance: reserved must be 0");
    BLF_REQUIRE(impedance->kp && impedance->kd && (batch == 0 || impedance->q_ref),
                "blf_fbd_euler_integrate_impedance: null impedance array");
    BLF_REQUIRE(model != nullptr && impedance->ndof == model->ndof,
                "blf_fbd_euler_integrate_impedance: impedance ndof %d != model ndof %d",
                impedance->ndof, model ? model->ndof : -1);
    // the constant-torque checks with a stand-in torque pointer (the impedance replaces it)
    blf_status st = check_fbd("blf_fbd_euler_integrate_impedance", handle, model, state,
                              impedance->kp, contacts, batch);
    if (st != BLF_OK) return st;
    int iterations = 0;
    double dT_last = 0.0;
    st = step_schedule(initial_time, final_time, dT, &iterations, &dT_last);
    if (st != BLF_OK) return st;
    return launch_fbd_euler(model, state, nullptr, contacts, mass_reg, batch, iterations, dT,
                            dT_last, (hipStream_t)stream, impedance);
}

blf_status blf_fbd_euler_integrate(blf_handle* handle, const blf_fb_model* model,
                                   const blf_fb_state* state, const double* joint_torque,
                                   const blf_fb_contacts* contacts, const double* mass_reg,
                                   int64_t batch, double initial_time, double final_time,
                                   double dT, void* stream)
{
    blf_status st = check_fbd("blf_fbd_euler_integrate", handle, model, state, joint_torque,
                              contacts, batch);
    if (st != BLF_OK) return st;
    int iterations = 0;
    double dT_last = 0.0;
    st = step_schedule(initial_time, final_time, dT, &iterations, &dT_last);
    if (st != BLF_OK) return st;
    return launch_fbd_euler(model, state, joint_torque, contacts, mass_reg, batch, iterations, dT,
                            dT_last, (hipStream_t)stream);
}

}  // extern "C"
