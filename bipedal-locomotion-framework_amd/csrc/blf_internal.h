// blf_internal.h — shared declarations of the HIP kernels' launchers and device helpers.
// Everything in csrc/ is compiled with -ffp-contract=off: every fp64 expression is evaluated
// exactly in source order, the same order as the CPU oracle (oracle/blf_oracle.c), so that
// device and oracle results can be compared bit for bit.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <mutex>
#include <unordered_map>

#include "blf/blf_c.h"

namespace blf {

constexpr int kWave = 64;   // CDNA wavefront width
constexpr int kMaxFacets = 8;       // facet slots per knot of the active-set kernels (and the default)
constexpr int kMaxFacetsWide = 16;  // max_facets up to this: the interior point kernel alone
// grid of the QP's stage 2, which loops over the pending list (one workgroup per CU)
constexpr int kListGrid = 256;

// ---- error plumbing (blf_capi.hip) ----
blf_status set_error(blf_status code, const char* fmt, ...);
blf_status check_hip(hipError_t e, const char* what);

// A stream's stage-2 work list (Handle::stage2_list; dcm_mpc_ipm.hip)
struct Stage2List {
    int32_t* buf;
    int* slot;
    int64_t cap;   // entries after the two count slots
};

struct Handle {
    int device = 0;
    int num_cus = 0;
    // The QP's stage-2 work list of each stream the handle solves on (dcm_mpc_ipm.hip): device
    // int32 [0], [1] two count slots, [2..] the QPs; grown (after a sync of the stream) when a
    // batch outgrows it.  `slot`: the count slot the stream's next solve appends to (0 there).
    struct List {
        int32_t* buf = nullptr;
        int64_t cap = 0;   // QPs it holds
        int slot = 0;
    };
    std::mutex mu;
    std::unordered_map<hipStream_t, List> lists;
    ~Handle();
    blf_status stage2_list(hipStream_t s, int64_t batch, Stage2List* out);
};

// ---- launchers (one per kernel file) ----
blf_status launch_lti_euler(int n, int m, const double* A, const double* Bm, int shared,
                            const double* u, double* x, int64_t batch, int32_t nsteps,
                            double dT, double dT_last, hipStream_t s);
blf_status launch_lti_dynamics(int n, int m, const double* A, const double* Bm, int shared,
                               const double* u, const double* x, double* dx, int64_t batch,
                               hipStream_t s);
blf_status launch_dcm_rollout(const double* xi0, const double* omega, const double* vrp,
                              int32_t N, double dt, double* xi_out, int64_t batch,
                              hipStream_t s);
blf_status launch_hull2d(const double* pts, const int32_t* npts, int32_t P, int32_t M,
                         int64_t batch, double* A, double* b, int32_t* nf, hipStream_t s);
blf_status launch_hullnd(int32_t D, const double* pts, const int32_t* npts, int32_t P, int32_t M,
                         int64_t batch, double* A, double* b, int32_t* nf, hipStream_t s);
size_t hullnd_lds_bytes(int D, int P, int M);
blf_status launch_hull3d(const double* pts, const int32_t* npts, int32_t P, int32_t M,
                         int64_t batch, double* A, double* b, int32_t* nf, hipStream_t s);
blf_status launch_halfspace_contains(const double* A, const double* b, const int32_t* nf,
                                     int32_t dim, int32_t M, const double* q, int64_t batch,
                                     int32_t* inside, hipStream_t s);
blf_status launch_hull2d_contains(const double* A, const double* b, const int32_t* nf, int32_t M,
                                  const double* q, int64_t batch, int32_t* inside,
                                  hipStream_t s);
blf_status launch_quintic_fit(const double* kt, const double* kp, int32_t K1, int32_t D,
                              int64_t S, double* coeffs, hipStream_t s);
blf_status launch_quintic_eval(const double* kt, const double* coeffs, int32_t K1, int32_t D,
                               int64_t S, const double* tq, int32_t Q, double* pva,
                               int32_t* idx, hipStream_t s);
blf_status launch_phase_expand(int32_t P, const int32_t* nphases, const double* begin,
                               const double* end, const double* pA, const double* pb,
                               const int32_t* pnf, const double* pref, int32_t M,
                               int64_t start_knot, double dt, int32_t N, int64_t batch, double* A,
                               double* b, int32_t* nfacets, double* xi_ref, double* vrp_ref,
                               hipStream_t s);
// The QP kernel routing (blf_set_qp_launch_mode): process-wide, not per handle; initialised once
// from the environment, read on every solve (relaxed atomics: a setting applies to the solves
// enqueued after it).
struct QpLaunchMode {
    std::atomic<int> fuse_stage2;     // 1 (default): stage 2 inside the small-batch active-set kernel
    std::atomic<int> single_kernel;   // 0 (default): active-set kernel first
    int list_grid;                    // stage 2's grid (kListGrid; BLF_QP_LIST_GRID, A/B only)
};
QpLaunchMode& qp_launch_mode();
// l: the stream's stage-2 work list (Handle::stage2_list)
blf_status launch_dcm_mpc(const blf_dcm_mpc_params* prm, const blf_dcm_mpc_problem* pb,
                          const blf_dcm_mpc_warm_start* warm, int64_t batch,
                          const blf_dcm_mpc_solution* sol, double* lambda_out, hipStream_t s,
                          const Stage2List& l);
blf_status launch_dcm_mpc_phased(const blf_dcm_mpc_params* prm, const blf_phase_table* ph,
                                 int64_t start_knot, const double* xi_init, const double* omega,
                                 int64_t omega_stride, const blf_dcm_mpc_warm_start* warm,
                                 int64_t batch, const blf_dcm_mpc_window* win,
                                 const blf_dcm_mpc_solution* sol, double* lambda_out, hipStream_t s,
                                 const Stage2List& l);

blf_status launch_contact_eval(const double* prm, int shared, const double* twist,
                               const double* pose, const double* null_pose, int64_t batch,
                               double* wrench, double* autonomous, double* control,
                               double* regressor, hipStream_t s);
blf_status launch_contact_point(const double* prm, int shared, const double* twist,
                                const double* pose, const double* null_pose, int64_t batch,
                                const double* points, int32_t Q, double* force, double* torque,
                                hipStream_t s);
blf_status launch_fbk_dynamics(int n, double rho, const double* rot, const double* twist,
                               const double* joint_vel, double* dpos, double* drot,
                               double* djoints, int64_t batch, hipStream_t s);
blf_status launch_fbd_dynamics(const blf_fb_model* md, const blf_fb_state* st, const double* tau,
                               const blf_fb_contacts* ct, const double* reg, int64_t batch,
                               const blf_fb_state* out, hipStream_t s);
blf_status launch_fbd_euler(const blf_fb_model* md, const blf_fb_state* st, const double* tau,
                            const blf_fb_contacts* ct, const double* reg, int64_t batch,
                            int32_t nsteps, double dT, double dT_last, hipStream_t s,
                            const blf_joint_impedance* impedance = nullptr);
size_t fbd_lds_bytes(int n, int C, bool aba = false);   // aba: the articulated-body layout
blf_status launch_fb_dcm(const blf_fb_model* md, const blf_fb_state* st, const double* omega0,
                         int64_t ostride, int64_t batch, double* com, double* xi, hipStream_t s);
blf_status launch_fb_frame_state(const blf_fb_model* md, const blf_fb_state* st, int32_t K,
                                 const int32_t* frames, int64_t batch, double* pose, double* twist,
                                 hipStream_t s);
blf_status launch_posture_reference(const blf_posture_law* law, const double* com, const double* vrp,
                                    int64_t vstride, int64_t batch, double* qref, hipStream_t s);
blf_status launch_fbk_euler(int n, double rho, double* pos, double* rot, double* joints,
                            const double* twist, const double* joint_vel, int64_t batch,
                            int32_t nsteps, double dT, double dT_last, hipStream_t s);

// ---- device helpers ----
// NaN-propagating max (matches the oracle's `if (e > m || e != e) m = e`).
__device__ __forceinline__ double nanmax(double a, double b) { return (b > a || b != b) ? b : a; }
// min that ignores NaN candidates (matches `if (q < m) m = q`).
__device__ __forceinline__ double keepmin(double a, double b) { return (b < a) ? b : a; }
// max that ignores NaN candidates (matches the oracle's keepmax).
__device__ __forceinline__ double keepmax(double a, double b) { return (b > a) ? b : a; }

// Cross-lane moves of a double that stay in the VALU (no LDS round trip): DPP quad permutes and
// row mirrors, and gfx950's v_permlane16_swap / v_permlane32_swap.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v)
{
    const long long b = __double_as_longlong(v);
    // every lane has a valid source for these patterns, so no "old" value (update_dpp's first
    // operand would cost a zeroing v_mov per half)
    const int lo = __builtin_amdgcn_mov_dpp((int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// v_permlane16_swap(x, x) returns (x with its odd rows replaced by the even rows, x with its even
// rows replaced by the odd rows); lane l takes its row partner (l ^ 16) from the half that moved
// into its own row.  v_permlane32_swap likewise for the two 32-lane halves (l ^ 32).
__device__ __forceinline__ double swap16_f64(double v)
{
    const long long b = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((int)b, (int)b, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((int)(b >> 32), (int)(b >> 32), false, false);
    const bool odd = (threadIdx.x >> 4) & 1;
    const int l = odd ? lo[0] : lo[1];
    const int h = odd ? hi[0] : hi[1];
    return __longlong_as_double(((long long)h << 32) | (unsigned int)l);
}
__device__ __forceinline__ double swap32_f64(double v)
{
    const long long b = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane32_swap((int)b, (int)b, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((int)(b >> 32), (int)(b >> 32), false, false);
    const bool upper = (threadIdx.x >> 5) & 1;
    const int l = upper ? lo[0] : lo[1];
    const int h = upper ? hi[0] : hi[1];
    return __longlong_as_double(((long long)h << 32) | (unsigned int)l);
}

// Butterfly over the 64 lanes, xor distances 1, 2, 4, 8, 16, 32 in that order (the oracle's
// orc_wave_tree_sum).  After the 1- and 2-steps every quad holds one value and after the 4-step
// every half-row does, so the half-row / row mirrors combine exactly the partners lane ^ 4 and
// lane ^ 8 would; every lane ends with the identical value (fp addition is commutative).
template <typename Op>
__device__ __forceinline__ double wave_reduce(double v, Op op)
{
    v = op(v, dpp_f64<0xB1>(v));    // quad_perm [1,0,3,2]: lane ^ 1
    v = op(v, dpp_f64<0x4E>(v));    // quad_perm [2,3,0,1]: lane ^ 2
    v = op(v, dpp_f64<0x141>(v));   // row_half_mirror
    v = op(v, dpp_f64<0x140>(v));   // row_mirror
    v = op(v, swap16_f64(v));       // lane ^ 16
    v = op(v, swap32_f64(v));       // lane ^ 32
    return v;
}
__device__ __forceinline__ double wave_sum(double v)
{
    return wave_reduce(v, [](double a, double b) { return a + b; });
}
__device__ __forceinline__ double wave_nanmax(double v)
{
    return wave_reduce(v, [](double a, double b) { return nanmax(a, b); });
}
__device__ __forceinline__ double wave_keepmin(double v)
{
    return wave_reduce(v, [](double a, double b) { return keepmin(a, b); });
}
__device__ __forceinline__ double wave_keepmax(double v)
{
    return wave_reduce(v, [](double a, double b) { return keepmax(a, b); });
}
__device__ __forceinline__ int wave_isum(int v)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

}  // namespace blf
