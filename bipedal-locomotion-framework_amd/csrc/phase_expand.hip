// phase_expand.hip — on-device knot -> contact-phase expansion of the receding-horizon DCM QP
// (rows 10-11 of 8(a)).
//
// The contact phases of a plan (ContactPhaseList::createPhases, src/Planners/src/
// ContactPhaseList.cpp:16-84) change only when the plan changes, so their support polygons are
// built once (blf_hull2d_hrep over the phases' corner sets) and stay resident.  Every advance()
// then expands them onto the knots of the current window:
//   t_k = (start_knot + k) * dt;  p = last phase with begin_p <= t_k (binary search, the
//   getPresentContact rule of ContactList.cpp:190-202);  knot k is in p iff t_k < end_p
// and copies phase p's H-rep rows, facet count and reference point to the knot.  A knot outside
// every phase gets nfacets = -1 (the QP then reports BLF_QP_BAD_FACETS) and zero rows/references.
//
// Mapping: one thread per (problem, knot 0..N, facet slot).  Consecutive threads write
// consecutive 16-B A rows and 8-B offsets; the facet-slot-0 thread of a knot also writes the
// knot's facet count and references.  The phase tables (a few hundred bytes per problem) are
// read through the cache by the (N+1) M threads of the problem.  HBM-bound: the bytes written
// are the per-knot arrays of the QP.
#include "blf_internal.h"

namespace blf {
namespace {

constexpr int kExpandBlock = 256;

__device__ __forceinline__ int phase_of(const double* __restrict__ begin,
                                        const double* __restrict__ end, int n, double t)
{
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (begin[mid] <= t) lo = mid + 1;
        else hi = mid;
    }
    const int p = lo - 1;
    return (p >= 0 && t < end[p]) ? p : -1;
}

__global__ __launch_bounds__(kExpandBlock) void phase_expand_kernel(
    int32_t P, const int32_t* __restrict__ nphases, const double* __restrict__ pbegin,
    const double* __restrict__ pend, const double* __restrict__ pA, const double* __restrict__ pb,
    const int32_t* __restrict__ pnf, const double* __restrict__ pref, int32_t M,
    int64_t start_knot, double dt, int32_t N, int64_t batch, double* __restrict__ A,
    double* __restrict__ b, int32_t* __restrict__ nfacets, double* __restrict__ xi_ref,
    double* __restrict__ vrp_ref)
{
    const int64_t t = (int64_t)blockIdx.x * kExpandBlock + threadIdx.x;
    const int64_t per = (int64_t)(N + 1) * M;
    if (t >= batch * per) return;
    const int64_t q = t / per;                 // problem
    const int r = (int)(t - q * per);
    const int k = r / M;                       // knot 0..N
    const int i = r - k * M;                   // facet slot
    int np = nphases[q];
    np = np < 0 ? 0 : (np > P ? P : np);
    const double tk = (double)(start_knot + k) * dt;
    const int ph = phase_of(pbegin + q * P, pend + q * P, np, tk);
    const int64_t src = q * P + ph;            // valid only if ph >= 0
    if (k < N) {
        const int64_t dst = (q * N + k) * M + i;
        double2 a = make_double2(0.0, 0.0);
        double bi = 0.0;
        if (ph >= 0) {
            a = reinterpret_cast<const double2*>(pA)[src * M + i];
            bi = pb[src * M + i];
        }
        reinterpret_cast<double2*>(A)[dst] = a;
        b[dst] = bi;
    }
    if (i == 0) {
        double2 ref = make_double2(0.0, 0.0);
        if (ph >= 0) ref = reinterpret_cast<const double2*>(pref)[src];
        reinterpret_cast<double2*>(xi_ref)[q * (N + 1) + k] = ref;
        if (k < N) {
            reinterpret_cast<double2*>(vrp_ref)[q * N + k] = ref;
            nfacets[q * N + k] = ph >= 0 ? pnf[src] : -1;
        }
    }
}

}  // namespace

blf_status launch_phase_expand(int32_t P, const int32_t* nphases, const double* begin,
                               const double* end, const double* pA, const double* pb,
                               const int32_t* pnf, const double* pref, int32_t M,
                               int64_t start_knot, double dt, int32_t N, int64_t batch, double* A,
                               double* b, int32_t* nfacets, double* xi_ref, double* vrp_ref,
                               hipStream_t s)
{
    const int64_t threads = batch * (int64_t)(N + 1) * M;
    if (threads == 0) return BLF_OK;
    const int64_t blocks = ceil_div(threads, kExpandBlock);
    if (blocks > 0x7fffffffLL)
        return set_error(BLF_ERR_UNSUPPORTED, "phase expansion of %lld knots too large",
                         (long long)(threads / M));
    hipLaunchKernelGGL(phase_expand_kernel, dim3((unsigned)blocks), dim3(kExpandBlock), 0, s, P,
                       nphases, begin, end, pA, pb, pnf, pref, M, start_knot, dt, N, batch, A, b,
                       nfacets, xi_ref, vrp_ref);
    return check_hip(hipGetLastError(), "phase_expand_kernel launch");
}

}  // namespace blf
