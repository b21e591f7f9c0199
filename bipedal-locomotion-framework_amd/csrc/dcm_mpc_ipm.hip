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
    ipm_solve<NT, WARM, LAMOUT, MF>(P, blockIdx.x, xi_init, omega, xi_ref, vrp_ref, Ain, bin, nfacets, ws_vrp,
                                    ws_lam, xi_out, vrp_out, status_out, iters_out, polished_out, lam_out);
}

// Stage 2 over the pending list the active-set kernel appended to (KParams::list): a grid of a
// few workgroups, each taking every gridDim-th listed problem.  With a budget of 256 VGPRs the
// solve needs no scratch, so a workgroup that finds nothing listed -- every workgroup of a batch
// the active-set kernel certified whole -- loads the count and leaves (round 4's batch-sized grid
// at 168 VGPRs stored 12.5 KB of register spills per QP on its way to the status check).
// Workgroup 0 zeroes the other count slot, the one the stream's next solve appends to.
template <int NT, bool WARM, bool LAMOUT, int MF>
__global__ __launch_bounds__(NT, (NT <= 256 ? BLF_MIN_WAVES : 1)) void dcm_mpc_ipm_list_kernel(
    KParams P, const double* __restrict__ xi_init, const double* __restrict__ omega,
    const double* __restrict__ xi_ref, const double* __restrict__ vrp_ref,
    const double* __restrict__ Ain, const double* __restrict__ bin,
    const int32_t* __restrict__ nfacets, const double* __restrict__ ws_vrp,
    const double* __restrict__ ws_lam, double* __restrict__ xi_out,
    double* __restrict__ vrp_out, int32_t* __restrict__ status_out,
    int32_t* __restrict__ iters_out, int32_t* __restrict__ polished_out, double* __restrict__ lam_out)
{
    const int32_t* idx = P.list + 2;
    const int listed = __builtin_amdgcn_readfirstlane(P.list[P.list_slot]);
    const int count = listed < P.list_cap ? listed : P.list_cap;
    if (blockIdx.x == 0 && threadIdx.x == 0) P.list[P.list_slot ^ 1] = 0;
    for (int i = (int)blockIdx.x; i < count; i += (int)gridDim.x) {
        ipm_solve<NT, WARM, LAMOUT, MF>(P, __builtin_amdgcn_readfirstlane(idx[i]), xi_init, omega, xi_ref, vrp_ref,
                                        Ain, bin, nfacets, ws_vrp, ws_lam, xi_out, vrp_out, status_out, iters_out,
                                        polished_out, lam_out);
        __syncthreads();   // the LDS is the next problem's
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
#define IPM_KERN(K) ((warm != nullptr) ? (lam_out ? K<NT, true, true, MF> : K<NT, true, false, MF>) \
                                       : (lam_out ? K<NT, false, true, MF> : K<NT, false, false, MF>))
    if (kp.list) {
        // stage 2 runs only after the active-set kernels (N <= 128); at most kListGrid
        // workgroups loop over the pending list
        if constexpr (NT <= 2 * kWave) {
            hipLaunchKernelGGL(IPM_KERN(dcm_mpc_ipm_list_kernel), dim3((unsigned)std::min<int64_t>(batch, qp_launch_mode().list_grid)),
                               dim3(NT), lds, s, kp, pb->xi_init, pb->omega, pb->xi_ref, pb->vrp_ref, pb->A, pb->b,
                               pb->nfacets, warm ? warm->vrp : nullptr, warm ? warm->lambda : nullptr, sol->xi,
                               sol->vrp, sol->status, sol->iters, sol->polished, lam_out);
            return check_hip(hipGetLastError(), "dcm_mpc_ipm_list_kernel launch");
        } else {
            return set_error(BLF_ERR_UNSUPPORTED, "stage 2 with %d threads, %d facet slots", NT, MF);
        }
    }
    hipLaunchKernelGGL(IPM_KERN(dcm_mpc_ipm_kernel), dim3((unsigned)batch), dim3(NT), lds, s, kp,
                       pb->xi_init, pb->omega, pb->xi_ref, pb->vrp_ref, pb->A, pb->b,
                       pb->nfacets, warm ? warm->vrp : nullptr, warm ? warm->lambda : nullptr,
                       sol->xi, sol->vrp, sol->status, sol->iters, sol->polished, lam_out);
#undef IPM_KERN
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
    kp.list_slot = 0;
    kp.list_cap = 0;
    kp.passes_out = nullptr;
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

}  // namespace

// The QPs the active-set kernel hands over go to stage 2 through the stream's pending list
// (Handle::stage2_list: [0], [1] two count slots, [2..] the QPs).  The active-set kernel appends
// to slot *slot, which is 0 when it starts; the IPM kernel's list instantiation loops over what it
// finds there with kListGrid workgroups and zeroes the other slot, and *slot flips to that one
// for the stream's next solve -- only once that launch is enqueued (finish_stage2).  When a launch
// fails after the active-set kernel may have appended, both count slots are zeroed on the stream,
// so the stream's next solve does not append on top of a stale count.
static void set_pend(KParams& kp, const Stage2List& l)
{
    kp.list = l.buf;
    kp.list_slot = *l.slot;
    kp.list_cap = (int)l.cap;
}
static void set_stage2(KParams& kp, const Stage2List& l)
{
    kp.stage2 = 1;
    kp.list = l.buf;
    kp.list_slot = *l.slot;
    kp.list_cap = (int)l.cap;
}
static blf_status finish_stage2(blf_status st, const Stage2List& l, hipStream_t s)
{
    if (st == BLF_OK) {
        *l.slot ^= 1;
        return st;
    }
    (void)hipMemsetAsync(l.buf, 0, sizeof(int32_t) * 2, s);
    *l.slot = 0;
    return st;
}

blf_status launch_dcm_mpc(const blf_dcm_mpc_params* prm, const blf_dcm_mpc_problem* pb,
                          const blf_dcm_mpc_warm_start* warm, int64_t batch,
                          const blf_dcm_mpc_solution* sol, double* lam_out, hipStream_t s,
                          const Stage2List& l)
{
    KParams kp = make_kparams(prm, warm);
    kp.passes_out = sol->passes;
    if (batch == 0) return BLF_OK;
    if (batch > 0x7fffffffLL) return set_error(BLF_ERR_UNSUPPORTED, "batch %lld too large", (long long)batch);
    const int N = kp.N;
    // With the active-set start (tol_polish > 0) and N <= 128, the one-wavefront active-set kernel
    // solves the QPs its start certifies; the IPM kernel then takes only the rest (stage 2), from
    // scratch and without the start.  BLF_QP_SINGLE_KERNEL=1 keeps everything in the IPM kernel
    // (A/B and parity tests: both ways give the same bits).
    if (kp.tol_polish > 0.0 && N <= 2 * kWave && kp.M <= kMaxFacetsWide &&
        !qp_launch_mode().single_kernel.load(std::memory_order_relaxed)) {
        bool stage2_done = false;
        set_pend(kp, l);
        const blf_status st = launch_dcm_mpc_as(kp, pb, warm, batch, sol, lam_out, s, nullptr, &stage2_done);
        kp.list = nullptr;
        if (st != BLF_OK) return finish_stage2(st, l, s);
        if (stage2_done) return st;
        set_stage2(kp, l);
        return finish_stage2(launch_ipm(kp, pb, warm, batch, sol, lam_out, s), l, s);
    }
    return launch_ipm(kp, pb, warm, batch, sol, lam_out, s);
}

// blf_dcm_mpc_solve_phased: the active-set kernels read the window from the phase table (PhaseSrc);
// the QPs they hand over (kPending) leave their expanded window in the caller's scratch, from
// which the IPM kernel's stage 2 continues exactly as after blf_dcm_phase_expand + solve.
blf_status launch_dcm_mpc_phased(const blf_dcm_mpc_params* prm, const blf_phase_table* ph,
                                 int64_t start_knot, const double* xi_init, const double* omega,
                                 int64_t omega_stride, const blf_dcm_mpc_warm_start* warm,
                                 int64_t batch, const blf_dcm_mpc_window* win,
                                 const blf_dcm_mpc_solution* sol, double* lam_out, hipStream_t s,
                                 const Stage2List& l)
{
    KParams kp = make_kparams(prm, warm);
    kp.passes_out = sol->passes;
    if (batch == 0) return BLF_OK;
    if (batch > 0x7fffffffLL) return set_error(BLF_ERR_UNSUPPORTED, "batch %lld too large", (long long)batch);
    if (kp.N > 2 * kWave || !(kp.tol_polish > 0.0))
        return set_error(BLF_ERR_UNSUPPORTED,
                         "phase-indexed solve: horizon %d > 128 or tol_polish = 0 (use blf_dcm_phase_expand "
                         "+ blf_dcm_mpc_solve_warm)", kp.N);
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
    set_pend(kp, l);
    const blf_status st = launch_dcm_mpc_as(kp, &pin, warm, batch, sol, lam_out, s, &ps);
    kp.list = nullptr;
    if (st != BLF_OK) return finish_stage2(st, l, s);
    set_stage2(kp, l);
    const blf_dcm_mpc_problem pw{xi_init, win->omega, win->xi_ref, win->vrp_ref, win->A, win->b, win->nfacets};
    return finish_stage2(launch_ipm(kp, &pw, warm, batch, sol, lam_out, s), l, s);
}

}  // namespace blf
