// dcm_mpc_ipm.hip — batched time-varying DCM MPC QP (TimeVaryingDCMPlanner).
//
// One workgroup per QP, one thread per knot k < N, NW = ceil(N/64) wavefronts.  Everything a knot
// owns — its slacks, multipliers, 1/s, VRP, DCM xi_{k+1}, the Newton-system blocks of the knot —
// lives in that thread's registers for the whole solve; LDS holds only the facet rows (read in
// every phase) and a few boundary values exchanged between wavefronts.
//
// The Newton system is block tridiagonal in time and is solved without any sequential loop over
// the knots: every recursion runs as a Kogge-Stone scan over the 64 lanes of a wavefront
// (6 levels of ds_bpermute + a compose), then one boundary value per wavefront through LDS.
//  * the Riccati recursion P_k = Q + alpha_k^2 P_{k+1} (I + E_k P_{k+1})^{-1} composes its
//    maps f(P) = H + A^T P (I + G P)^{-1} A in the structure-preserving doubling form (only
//    I + G H, eigenvalues >= 1, is ever inverted);
//  * the costate recursion and the forward rollout of the Newton step are affine maps.
// All remaining work (residuals, barrier Hessians, right-hand sides, step lengths, updates) is
// knot-parallel.
//
// Every expression mirrors oracle/blf_oracle.c:orc_dcm_mpc_solve term for term (the scans in the
// same combine order, the reductions in the same xor-butterfly order) and the file is built with
// -ffp-contract=off, so device and oracle iterates agree bit for bit (tests/test_gpu_dcm_mpc.py).
// DESIGN.md section 4 is the algorithm statement.
#include "dcm_mpc_ipm_body.h"

// The 16-slot instantiations (max_facets > 8) keep their facet loops rolled where the unroller
// gives up; that is expected, not a defect.
#pragma clang diagnostic ignored "-Wpass-failed"

namespace blf {
namespace {
using namespace qp;

template <int NT, bool WARM, bool LAMOUT, int MF>
__global__ __launch_bounds__(NT, (NT <= 256 ? BLF_MIN_WAVES : 1)) void dcm_mpc_ipm_kernel(
    KParams P, const double* __restrict__ xi_init, const double* __restrict__ omega,
    const double* __restrict__ xi_ref, const double* __restrict__ vrp_ref,
    const double* __restrict__ Ain, const double* __restrict__ bin,
    const int32_t* __restrict__ nfacets, const double* __restrict__ ws_vrp,
    const double* __restrict__ ws_lam, double* __restrict__ xi_out,
    double* __restrict__ vrp_out, int32_t* __restrict__ status_out,
    int32_t* __restrict__ iters_out, int32_t* __restrict__ polished_out, double* __restrict__ lam_out)
{
    // one problem per workgroup, or stage 2 over the pending list: a grid of a few workgroups,
    // each taking every gridDim-th listed problem (the whole batch's grid would have to be
    // dispatched beside whatever else holds the chip -- the closed loop's dynamics -- before the
    // launch could end).  One call site of the solve either way.
    const bool lst = P.list != nullptr;
    const int count = lst ? P.list[0] : (int)blockIdx.x + 1;
    for (int i = lst ? (int)blockIdx.x : (int)blockIdx.x; i < count; i += lst ? (int)gridDim.x : count) {
        const int64_t p = lst ? P.list[1 + i] : (int64_t)blockIdx.x;
        ipm_solve<NT, WARM, LAMOUT, MF>(P, p, xi_init, omega, xi_ref, vrp_ref, Ain, bin, nfacets, ws_vrp,
                                    ws_lam, xi_out, vrp_out, status_out, iters_out, polished_out, lam_out);
        if (lst) __syncthreads();   // the LDS is the next problem's
    }
}

// MF facet slots per knot in the registers: 8, or 16 when max_facets > 8 (support polygons of up
// to four contacts; those QPs run in this kernel alone, without the active-set kernel)
template <int NT, int MF = kMaxFacets>
blf_status launch_nt(const KParams& kp, const blf_dcm_mpc_problem* pb,
                     const blf_dcm_mpc_warm_start* warm, int64_t batch,
                     const blf_dcm_mpc_solution* sol, double* lam_out, hipStream_t s)
{
    const size_t lds = sizeof(double) * Lds(nullptr, kp.N, kp.M, NT / kWave).total;
    if (lds > 160 * 1024)
        return set_error(BLF_ERR_UNSUPPORTED, "horizon %d with %d facet slots needs %zu B of LDS",
                         kp.N, kp.M, lds);
    auto kern = (warm != nullptr)
                    ? (lam_out ? dcm_mpc_ipm_kernel<NT, true, true, MF> : dcm_mpc_ipm_kernel<NT, true, false, MF>)
                    : (lam_out ? dcm_mpc_ipm_kernel<NT, false, true, MF> : dcm_mpc_ipm_kernel<NT, false, false, MF>);
    // a pending list: at most kListGrid workgroups loop over it
    const unsigned grid = kp.list ? (unsigned)std::min<int64_t>(batch, kListGrid) : (unsigned)batch;
    hipLaunchKernelGGL(kern, dim3(grid), dim3(NT), lds, s, kp,
                       pb->xi_init, pb->omega, pb->xi_ref, pb->vrp_ref, pb->A, pb->b,
                       pb->nfacets, warm ? warm->vrp : nullptr, warm ? warm->lambda : nullptr,
                       sol->xi, sol->vrp, sol->status, sol->iters, sol->polished, lam_out);
    return check_hip(hipGetLastError(), "dcm_mpc_ipm_kernel launch");
}

}  // namespace

#ifdef BLF_STAMPS
extern "C" int blf_debug_stamps(unsigned long long* out, int reset)
{
    unsigned long long h[16];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_blf_stamps), sizeof(h)) != hipSuccess) return -1;
    for (int i = 0; i < 16; ++i) out[i] = h[i];
    if (reset) {
        unsigned long long z[16] = {};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_blf_stamps), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

namespace {
KParams make_kparams(const blf_dcm_mpc_params* prm, const blf_dcm_mpc_warm_start* warm)
{
    KParams kp;
    kp.N = prm->horizon;
    kp.M = prm->max_facets;
    kp.max_iter = prm->max_iter;
    kp.dt = prm->dt;
    kp.Qw0 = prm->w_xi[0]; kp.Qw1 = prm->w_xi[1];
    kp.Rw0 = prm->w_vrp[0]; kp.Rw1 = prm->w_vrp[1];
    kp.Pw0 = prm->w_terminal[0]; kp.Pw1 = prm->w_terminal[1];
    kp.tol_mu = prm->tol_mu;
    kp.tol_p = prm->tol_primal;
    kp.tol_d = prm->tol_dual;
    kp.tol_polish = prm->tol_polish;
    kp.ws_shift = warm ? warm->shift : 0;
    kp.ws_floor = warm ? warm->floor : 0.0;
    kp.ws_status = warm ? warm->prev_status : nullptr;
    kp.stage2 = 0;
    kp.list = nullptr;
    kp.f_dt = (float)kp.dt;
    kp.f_Qw0 = (float)kp.Qw0; kp.f_Qw1 = (float)kp.Qw1;
    kp.f_Rw0 = (float)kp.Rw0; kp.f_Rw1 = (float)kp.Rw1;
    kp.f_Pw0 = (float)kp.Pw0; kp.f_Pw1 = (float)kp.Pw1;
    kp.f_tol_p = kSearchTolP;
    kp.f_tol_d = kSearchTolD;
    return kp;
}

blf_status launch_ipm(const KParams& kp, const blf_dcm_mpc_problem* pb, const blf_dcm_mpc_warm_start* warm,
                      int64_t batch, const blf_dcm_mpc_solution* sol, double* lam_out, hipStream_t s)
{
    const int N = kp.N;
    if (kp.M > kMaxFacets) {
        if (N <= 64) return launch_nt<64, kMaxFacetsWide>(kp, pb, warm, batch, sol, lam_out, s);
        if (N <= 128) return launch_nt<128, kMaxFacetsWide>(kp, pb, warm, batch, sol, lam_out, s);
        if (N <= 256) return launch_nt<256, kMaxFacetsWide>(kp, pb, warm, batch, sol, lam_out, s);
        return set_error(BLF_ERR_UNSUPPORTED, "horizon %d > 256 with %d facet slots (> %d)", N, kp.M,
                         kMaxFacets);
    }
    if (N <= 64) return launch_nt<64>(kp, pb, warm, batch, sol, lam_out, s);
    if (N <= 128) return launch_nt<128>(kp, pb, warm, batch, sol, lam_out, s);
    if (N <= 256) return launch_nt<256>(kp, pb, warm, batch, sol, lam_out, s);
    if (N <= 512) return launch_nt<512>(kp, pb, warm, batch, sol, lam_out, s);
    if (N <= 1024) return launch_nt<1024>(kp, pb, warm, batch, sol, lam_out, s);
    return set_error(BLF_ERR_UNSUPPORTED, "horizon %d > 1024", N);
}

// pending[p] = 1 for the QPs the active-set kernel handed to stage 2 (status kPending), else 0;
// list (optional, list[0] zeroed before): their indices appended after the count, in no
// particular order (each problem is solved on its own, so the order changes no result)
__global__ __launch_bounds__(256) void pending_mask_kernel(const int32_t* __restrict__ status, int64_t batch,
                                                           int32_t* __restrict__ pending, int32_t* __restrict__ list)
{
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= batch) return;
    const bool pend = status[p] == kPending;
    pending[p] = pend ? 1 : 0;
    if (list && pend) list[1 + atomicAdd(&list[0], 1)] = (int32_t)p;
}
}  // namespace

blf_status launch_dcm_mpc(const blf_dcm_mpc_params* prm, const blf_dcm_mpc_problem* pb,
                          const blf_dcm_mpc_warm_start* warm, int64_t batch,
                          const blf_dcm_mpc_solution* sol, double* lam_out, hipStream_t s)
{
    KParams kp = make_kparams(prm, warm);
    if (batch == 0) return BLF_OK;
    if (batch > 0x7fffffffLL) return set_error(BLF_ERR_UNSUPPORTED, "batch %lld too large", (long long)batch);
    const int N = kp.N;
    // With the active-set start (tol_polish > 0) and N <= 128, the one-wavefront active-set kernel
    // solves the QPs its start certifies; this kernel then takes only the rest (stage 2), from
    // scratch and without the start.  BLF_QP_SINGLE_KERNEL=1 keeps everything in this kernel
    // (A/B and parity tests: both ways give the same bits).
    if (kp.tol_polish > 0.0 && N <= 2 * kWave && kp.M <= kMaxFacets && !qp_launch_mode().single_kernel) {
        bool stage2_done = false;
        const blf_status st = launch_dcm_mpc_as(kp, pb, warm, batch, sol, lam_out, s, nullptr, &stage2_done);
        if (st != BLF_OK || stage2_done) return st;
        kp.stage2 = 1;
    }
    return launch_ipm(kp, pb, warm, batch, sol, lam_out, s);
}

// blf_dcm_mpc_solve_phased: the active-set kernels read the window from the phase table (PhaseSrc);
// the QPs they hand over (kPending) leave their expanded window in the caller's scratch, from
// which the IPM kernel's stage 2 continues exactly as after blf_dcm_phase_expand + solve.
// part: 0 the whole solve; 1 the active-set part alone (stage 2's QPs left at kPending, their
// windows in the scratch, `pending` marking them); 2 stage 2 alone (blf_dcm_mpc_solve_phased_begin /
// _finish: parts 1 then 2 on one stream are part 0).  With more than 8 facet slots there is no
// active-set part: part 1 solves everything and marks nothing, part 2 does nothing.
blf_status launch_dcm_mpc_phased(const blf_dcm_mpc_params* prm, const blf_phase_table* ph,
                                 int64_t start_knot, const double* xi_init, const double* omega,
                                 int64_t omega_stride, const blf_dcm_mpc_warm_start* warm,
                                 int64_t batch, const blf_dcm_mpc_window* win,
                                 const blf_dcm_mpc_solution* sol, double* lam_out, hipStream_t s,
                                 int part, int32_t* pending, int32_t* list)
{
    KParams kp = make_kparams(prm, warm);
    if (batch == 0) return BLF_OK;
    if (part == 2) {
        if (kp.M > kMaxFacets) return BLF_OK;
        kp.stage2 = 1;
        kp.list = list;
        const blf_dcm_mpc_problem pw{xi_init, win->omega, win->xi_ref, win->vrp_ref, win->A, win->b, win->nfacets};
        return launch_ipm(kp, &pw, warm, batch, sol, lam_out, s);
    }
    if (pending && (kp.M > kMaxFacets || part == 0)) {
        blf_status st = check_hip(hipMemsetAsync(pending, 0, sizeof(int32_t) * (size_t)batch, s), "pending mask");
        if (st != BLF_OK) return st;
    }
    if (list) {   // the count; the kernel below (or nothing, M > 8) appends
        blf_status st = check_hip(hipMemsetAsync(list, 0, sizeof(int32_t), s), "pending list");
        if (st != BLF_OK) return st;
    }
    if (batch > 0x7fffffffLL) return set_error(BLF_ERR_UNSUPPORTED, "batch %lld too large", (long long)batch);
    if (kp.N > 2 * kWave || !(kp.tol_polish > 0.0))
        return set_error(BLF_ERR_UNSUPPORTED,
                         "phase-indexed solve: horizon %d > 128 or tol_polish = 0 (use blf_dcm_phase_expand "
                         "+ blf_dcm_mpc_solve_warm)", kp.N);
    if (kp.M > kMaxFacets) {
        // more facet slots than the active-set kernels hold (phases of up to four contacts): the
        // window expanded into the caller's scratch, then the interior point kernel's solve of it
        // (the same bits as blf_dcm_phase_expand + blf_dcm_mpc_solve_warm)
        blf_status st = launch_phase_expand(ph->max_phases, ph->nphases, ph->begin, ph->end, ph->A, ph->b,
                                            ph->nfacets, ph->ref, kp.M, start_knot, kp.dt, kp.N, batch, win->A,
                                            win->b, win->nfacets, win->xi_ref, win->vrp_ref, s);
        if (st != BLF_OK) return st;
        st = check_hip(hipMemcpy2DAsync(win->omega, sizeof(double) * kp.N, omega, sizeof(double) * omega_stride,
                                        sizeof(double) * kp.N, (size_t)batch, hipMemcpyDeviceToDevice, s),
                       "phase-indexed solve: omega copy");
        if (st != BLF_OK) return st;
        const blf_dcm_mpc_problem pw{xi_init, win->omega, win->xi_ref, win->vrp_ref, win->A, win->b, win->nfacets};
        return launch_dcm_mpc(prm, &pw, warm, batch, sol, lam_out, s);
    }
    PhaseSrc ps{};
    ps.P = ph->max_phases;
    ps.nphases = ph->nphases;
    ps.begin = ph->begin;
    ps.end = ph->end;
    ps.A = ph->A;
    ps.b = ph->b;
    ps.nf = ph->nfacets;
    ps.ref = ph->ref;
    ps.start = start_knot;
    ps.ostride = omega_stride;
    ps.wom = win->omega;
    ps.wxr = win->xi_ref;
    ps.wrr = win->vrp_ref;
    ps.wA = win->A;
    ps.wb = win->b;
    ps.wnf = win->nfacets;
    const blf_dcm_mpc_problem pin{xi_init, omega, nullptr, nullptr, nullptr, nullptr, nullptr};
    const blf_status st = launch_dcm_mpc_as(kp, &pin, warm, batch, sol, lam_out, s, &ps);
    if (st != BLF_OK) return st;
    if (part == 1) {
        if (!pending) return BLF_OK;
        hipLaunchKernelGGL(pending_mask_kernel, dim3((unsigned)ceil_div(batch, 256)), dim3(256), 0, s,
                           sol->status, batch, pending, list);
        return check_hip(hipGetLastError(), "pending_mask_kernel launch");
    }
    kp.stage2 = 1;
    const blf_dcm_mpc_problem pw{xi_init, win->omega, win->xi_ref, win->vrp_ref, win->A, win->b, win->nfacets};
    return launch_ipm(kp, &pw, warm, batch, sol, lam_out, s);
}

}  // namespace blf
