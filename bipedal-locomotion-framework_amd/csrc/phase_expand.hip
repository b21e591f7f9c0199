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
// Mapping: one workgroup per problem.  The problem's phase table (a few hundred bytes per phase)
// is staged into LDS with coalesced loads; one pass assigns every knot its phase (binary search
// in LDS); then the workgroup writes the window's arrays with consecutive threads on consecutive
// 16-B A rows, 8-B offsets, facet counts and 16-B references.  HBM-bound: the bytes written are
// the per-knot arrays of the QP.
#include "dcm_qp_common.h"   // phase_of
#include "slab.h"

namespace blf {
namespace {

constexpr int kExpandBlock = 256;

// Dynamic LDS (doubles first, 16-B aligned): A [P][M] double2, ref [P] double2, b [P][M],
// begin [P], end [P], then nf [P] and the knot phases [N+1] as int32.
__host__ __device__ inline size_t expand_lds_bytes(int P, int M, int N)
{
    return sizeof(double) * ((size_t)P * (3 * M + 4)) + sizeof(int32_t) * ((size_t)P + N + 1);
}

// The window is read straight back by the QP kernel.  A window set that fits the 256 MB
// Infinity Cache is stored plainly, so the solve reads it from there; a larger one streams past
// it non-temporally (measured on one box, two rounds: 4096 windows, 97 MB, plain stores 0.104 /
// 0.105 ms per expand + solve step against 0.108 / 0.109 ms non-temporal; 65 536 windows, 1.5 GB,
// non-temporal 2.07 ms per pipeline step against 2.19 ms plain; profiles/r03_expand_nt_ab.log).
constexpr size_t kExpandNtBytes = (size_t)128 << 20;

template <bool NT>
__global__ __launch_bounds__(kExpandBlock) void phase_expand_kernel(
    int32_t P, const int32_t* __restrict__ nphases, const double* __restrict__ pbegin,
    const double* __restrict__ pend, const double* __restrict__ pA, const double* __restrict__ pb,
    const int32_t* __restrict__ pnf, const double* __restrict__ pref, int32_t M,
    int64_t start_knot, double dt, int32_t N, double* __restrict__ A, double* __restrict__ b,
    int32_t* __restrict__ nfacets, double* __restrict__ xi_ref, double* __restrict__ vrp_ref)
{
    extern __shared__ __attribute__((aligned(16))) double xs[];
    double2* sA = reinterpret_cast<double2*>(xs);            // [P][M]
    double2* sRef = sA + (size_t)P * M;                       // [P]
    double* sB = reinterpret_cast<double*>(sRef + P);         // [P][M]
    double* sBeg = sB + (size_t)P * M;                        // [P]
    double* sEnd = sBeg + P;                                  // [P]
    int32_t* sNf = reinterpret_cast<int32_t*>(sEnd + P);      // [P]
    int32_t* sPh = sNf + P;                                   // [N+1]
    const int tid = threadIdx.x;
    const int64_t q = blockIdx.x;

    // 1. stage the phase table (coalesced, contiguous per problem)
    int np = nphases[q];
    np = np < 0 ? 0 : (np > P ? P : np);
    {
        const double2* gA = reinterpret_cast<const double2*>(pA) + q * P * M;
        for (int j = tid; j < np * M; j += kExpandBlock) sA[j] = gA[j];
        const double* gB = pb + q * P * M;
        for (int j = tid; j < np * M; j += kExpandBlock) sB[j] = gB[j];
        const double2* gR = reinterpret_cast<const double2*>(pref) + q * P;
        for (int j = tid; j < np; j += kExpandBlock) {
            sRef[j] = gR[j];
            sBeg[j] = pbegin[q * P + j];
            sEnd[j] = pend[q * P + j];
            sNf[j] = pnf[q * P + j];
        }
    }
    __syncthreads();
    // 2. knot -> phase
    for (int k = tid; k <= N; k += kExpandBlock)
        sPh[k] = phase_of(sBeg, sEnd, np, (double)(start_knot + k) * dt);
    __syncthreads();
    // 3. the window's arrays, consecutive threads on consecutive elements
    const int nm = N * M;
    double2* oA = reinterpret_cast<double2*>(A) + q * nm;
    double* oB = b + q * nm;
    const bool pow2 = (M & (M - 1)) == 0;
    const int sh = __builtin_ctz(M);
    for (int j = tid; j < nm; j += kExpandBlock) {
        const int k = pow2 ? j >> sh : j / M, i = j - k * M;
        const int ph = sPh[k];
        st_out<NT>(oA + j, ph >= 0 ? sA[ph * M + i] : make_double2(0.0, 0.0));
        st_out<NT>(oB + j, ph >= 0 ? sB[ph * M + i] : 0.0);
    }
    double2* oX = reinterpret_cast<double2*>(xi_ref) + q * (N + 1);
    double2* oR = reinterpret_cast<double2*>(vrp_ref) + q * N;
    int32_t* oN = nfacets + q * N;
    for (int k = tid; k <= N; k += kExpandBlock) {
        const int ph = sPh[k];
        const double2 ref = ph >= 0 ? sRef[ph] : make_double2(0.0, 0.0);
        st_out<NT>(oX + k, ref);
        if (k < N) {
            st_out<NT>(oR + k, ref);
            st_out<NT>(oN + k, ph >= 0 ? sNf[ph] : -1);
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
    if (batch == 0) return BLF_OK;
    if (batch > 0x7fffffffLL)
        return set_error(BLF_ERR_UNSUPPORTED, "phase expansion of %lld problems too large",
                         (long long)batch);
    const size_t lds = expand_lds_bytes(P, M, N);
    if (lds > 64 * 1024)
        return set_error(BLF_ERR_UNSUPPORTED,
                         "%d phases and a horizon of %d need %zu B of LDS (64 KiB at most)", P, N,
                         lds);
    const size_t out_bytes = (size_t)batch * ((size_t)N * M * 24 + (size_t)N * 20 + (size_t)(N + 1) * 16);
    auto kern = out_bytes > kExpandNtBytes ? phase_expand_kernel<true> : phase_expand_kernel<false>;
    hipLaunchKernelGGL(kern, dim3((unsigned)batch), dim3(kExpandBlock), lds, s, P,
                       nphases, begin, end, pA, pb, pnf, pref, M, start_knot, dt, N, A, b,
                       nfacets, xi_ref, vrp_ref);
    return check_hip(hipGetLastError(), "phase_expand_kernel launch");
}

}  // namespace blf
