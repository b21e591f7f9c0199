// hullnd.hip — ConvexHullHelper on n x p points, any n (blf_hullnd_hrep).
// Its own translation unit: the default scheduler (the iterative-ILP strategy the other planner
// kernels use crashes the compiler on the unrolled elimination).
// Built with -ffp-contract=off: bit-identical to oracle/blf_oracle.c orc_hullnd_hrep.
#include "blf_internal.h"

namespace blf {
namespace {

// n-D hull (ConvexHullHelper::buildConvexHull on D x p points, any D; the reference hands the
// matrix to Qhull): one wavefront per point set, its points in LDS, the D-subsets in
// lexicographic order 64 at a time, one per lane.  Each lane unranks its subset, takes the null
// vector of the (D-1) x D difference matrix (full pivoting, in registers: every index is a
// compile-time constant, the pivot's row / column swaps are selects), runs the one-side test and
// the offset over every point, and checks the stored planes; the chunk's survivors are then
// deduplicated among themselves in lane order (a lane is dropped when an earlier surviving lane
// carries the same plane) and appended in lane order.  That is the oracle's sequential rule
// (orc_hullnd_hrep: every subset in order, compared with the planes stored before it), with the
// same operations in the same order, so the rows are the same bits.
__device__ __forceinline__ int64_t hull_binom(int a, int b)
{
    if (b < 0 || a < b) return 0;
    int64_t r = 1;
    for (int k = 1; k <= b; ++k) r = r * (a - b + k) / k;
    return r;
}

template <int D>
__global__ __launch_bounds__(64) void hullnd_kernel(const double* __restrict__ pts,
                                                    const int32_t* __restrict__ npts, int32_t P,
                                                    int32_t M, double* __restrict__ Aout,
                                                    double* __restrict__ bout,
                                                    int32_t* __restrict__ nfout)
{
    constexpr int R = D - 1;
    extern __shared__ double hsm[];
    double* sp = hsm;            // [P][D] the set's points
    double* sA = sp + P * D;     // [M][D] stored planes
    double* sb = sA + M * D;     // [M]
    double* cA = sb + M;         // [64][D] this chunk's candidates
    double* cb = cA + 64 * D;    // [64]
    const int64_t s = blockIdx.x;
    const int lane = threadIdx.x;
    const int n = npts[s];
    double* A = Aout + s * D * M;
    double* b = bout + s * M;
    for (int e = lane; e < D * M; e += 64) A[e] = 0.0;
    for (int e = lane; e < M; e += 64) b[e] = 0.0;
    if (n < D + 1 || n > P) {
        if (lane == 0) nfout[s] = -1;
        return;
    }
    double scale = 0.0;
    for (int e = lane; e < D * n; e += 64) {
        const double v = pts[s * D * P + e];
        sp[e] = v;
        scale = fmax(scale, fabs(v));
    }
    for (int o = 32; o > 0; o >>= 1) scale = fmax(scale, __shfl_xor(scale, o));
    __syncthreads();
    const double tol = 1e-12 * (1.0 + scale);
    const double btol = 1e-9 * (1.0 + scale);
    const int64_t total = hull_binom(n, D);
    int count = 0;
    bool overflow = false;
    for (int64_t base = 0; base < total; base += 64) {
        const int64_t t = base + lane;
        bool cand = t < total;
        double nrm[D];
        double bm = -__builtin_inf();
        if (cand) {
            // the t-th D-subset in lexicographic order
            int idx[D];
            int64_t rr = t;
            int x = 0;
#pragma unroll
            for (int i = 0; i < D; ++i) {
                for (; x < n - 1; ++x) {   // bounded: every wave leaves the loop
                    const int64_t c = hull_binom(n - x - 1, D - i - 1);
                    if (rr < c) break;
                    rr -= c;
                }
                idx[i] = x++;
            }
            const double* p0 = sp + idx[0] * D;
            double W[R][D];
            int perm[D];
#pragma unroll
            for (int r = 0; r < R; ++r)
#pragma unroll
                for (int c = 0; c < D; ++c) W[r][c] = sp[idx[r + 1] * D + c] - p0[c];
#pragma unroll
            for (int c = 0; c < D; ++c) perm[c] = c;
#pragma unroll
            for (int k = 0; k < R; ++k) {
                double best = -1.0;
                int pr = k, pc = k;
#pragma unroll
                for (int r = k; r < R; ++r)
#pragma unroll
                    for (int c = k; c < D; ++c) {
                        const double a = fabs(W[r][c]);
                        if (a > best) best = a, pr = r, pc = c;
                    }
                cand = cand && best > tol;
                // swap rows k <-> pr, then columns k <-> pc (selects over constant indices)
#pragma unroll
                for (int r = k + 1; r < R; ++r)
#pragma unroll
                    for (int c = 0; c < D; ++c) {
                        const bool sw = r == pr;
                        const double a = W[k][c], z = W[r][c];
                        W[k][c] = sw ? z : a;
                        W[r][c] = sw ? a : z;
                    }
#pragma unroll
                for (int c = k + 1; c < D; ++c) {
                    const bool sw = c == pc;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const double a = W[r][k], z = W[r][c];
                        W[r][k] = sw ? z : a;
                        W[r][c] = sw ? a : z;
                    }
                    const int pa = perm[k], pz = perm[c];
                    perm[k] = sw ? pz : pa;
                    perm[c] = sw ? pa : pz;
                }
#pragma unroll
                for (int r = k + 1; r < R; ++r) {
                    const double f = W[r][k] / W[k][k];
#pragma unroll
                    for (int c = k + 1; c < D; ++c) W[r][c] = W[r][c] - f * W[k][c];
                }
            }
            double xs[D];
            xs[D - 1] = 1.0;
#pragma unroll
            for (int k = R - 1; k >= 0; --k) {
                double sum = W[k][D - 1];
#pragma unroll
                for (int c = k + 1; c < R; ++c) sum = sum + W[k][c] * xs[c];
                xs[k] = -sum / W[k][k];
            }
#pragma unroll
            for (int c = 0; c < D; ++c) {
                double v = 0.0;
#pragma unroll
                for (int k = 0; k < D; ++k) v = perm[k] == c ? xs[k] : v;
                nrm[c] = v;
            }
            double len = nrm[0] * nrm[0];
#pragma unroll
            for (int c = 1; c < D; ++c) len = len + nrm[c] * nrm[c];
            len = sqrt(len);
            cand = cand && len > 0.0;
#pragma unroll
            for (int c = 0; c < D; ++c) nrm[c] = nrm[c] / len;
            bool pos = false, neg = false;
            if (cand)
                for (int l = 0; l < n; ++l) {
                    const double* q = sp + l * D;
                    double d = nrm[0] * (q[0] - p0[0]);
#pragma unroll
                    for (int c = 1; c < D; ++c) d = d + nrm[c] * (q[c] - p0[c]);
                    pos = pos || d > tol;
                    neg = neg || d < -tol;
                }
            cand = cand && !((pos && neg) || !(pos || neg));
            if (cand) {
                if (pos)
#pragma unroll
                    for (int c = 0; c < D; ++c) nrm[c] = -nrm[c];
                for (int l = 0; l < n; ++l) {
                    const double* q = sp + l * D;
                    double v = nrm[0] * q[0];
#pragma unroll
                    for (int c = 1; c < D; ++c) v = v + nrm[c] * q[c];
                    if (v > bm) bm = v;
                }
                for (int e = 0; e < count && e < M && cand; ++e) {
                    bool same = fabs(sb[e] - bm) <= btol;
#pragma unroll
                    for (int c = 0; c < D; ++c) same = same && fabs(sA[e * D + c] - nrm[c]) <= 1e-9;
                    cand = !same;
                }
            }
        }
        if (cand) {
#pragma unroll
            for (int c = 0; c < D; ++c) cA[lane * D + c] = nrm[c];
            cb[lane] = bm;
        }
        __syncthreads();
        // duplicates inside the chunk: the earliest surviving lane keeps the plane
        uint64_t live = __ballot(cand);
        uint64_t todo = live;
        while (todo) {
            const int j = __builtin_ctzll(todo);
            if (cand && lane > j) {
                bool same = fabs(cb[j] - bm) <= btol;
#pragma unroll
                for (int c = 0; c < D; ++c) same = same && fabs(cA[j * D + c] - nrm[c]) <= 1e-9;
                cand = !same;
            }
            live = __ballot(cand);
            todo = live & ~((2ull << j) - 1ull);
        }
        const int pos = count + __builtin_popcountll(live & ((1ull << lane) - 1ull));
        if (cand && pos < M) {
#pragma unroll
            for (int c = 0; c < D; ++c) sA[pos * D + c] = nrm[c];
            sb[pos] = bm;
        }
        count += __builtin_popcountll(live);
        overflow = overflow || count > M;
        __syncthreads();
        if (overflow) break;   // the result is -1 already (count is wave-uniform)
    }
    if (overflow || count < D + 1) {
        if (lane == 0) nfout[s] = -1;
        return;
    }
    for (int e = lane; e < D * count; e += 64) A[e] = sA[e];
    for (int e = lane; e < count; e += 64) b[e] = sb[e];
    if (lane == 0) nfout[s] = count;
}

// D = 1: the largest and smallest coordinate (one lane per set).
__global__ __launch_bounds__(64) void hull1d_kernel(const double* __restrict__ pts,
                                                    const int32_t* __restrict__ npts, int32_t P,
                                                    int32_t M, int64_t batch,
                                                    double* __restrict__ A, double* __restrict__ b,
                                                    int32_t* __restrict__ nf)
{
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= batch) return;
    for (int e = 0; e < M; ++e) A[s * M + e] = 0.0, b[s * M + e] = 0.0;
    const int n = npts[s];
    const double* q = pts + s * P;
    if (n < 2 || n > P || M < 2) {
        nf[s] = -1;
        return;
    }
    double scale = 0.0, mn = q[0], mx = q[0];
    for (int e = 0; e < n; ++e) scale = fmax(scale, fabs(q[e]));
    for (int l = 1; l < n; ++l) {
        if (q[l] < mn) mn = q[l];
        if (q[l] > mx) mx = q[l];
    }
    if (!(mx - mn > 1e-12 * (1.0 + scale))) {
        nf[s] = -1;
        return;
    }
    A[s * M] = 1.0, b[s * M] = mx, A[s * M + 1] = -1.0, b[s * M + 1] = -mn;
    nf[s] = 2;
}

}  // namespace

size_t hullnd_lds_bytes(int D, int P, int M)
{
    return sizeof(double) * ((size_t)P * D + (size_t)M * (D + 1) + 64 * (size_t)(D + 1));
}

blf_status launch_hullnd(int32_t D, const double* pts, const int32_t* npts, int32_t P, int32_t M,
                         int64_t batch, double* A, double* b, int32_t* nf, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    if (D == 1) {
        hipLaunchKernelGGL(hull1d_kernel, dim3((unsigned)ceil_div(batch, 64)), dim3(64), 0, s, pts,
                           npts, P, M, batch, A, b, nf);
        return check_hip(hipGetLastError(), "hull1d_kernel launch");
    }
    if (batch > 0x7fffffffLL)
        return set_error(BLF_ERR_UNSUPPORTED, "hullnd: %lld point sets too many", (long long)batch);
    const size_t lds = hullnd_lds_bytes(D, P, M);
    using Kern = void (*)(const double*, const int32_t*, int32_t, int32_t, double*, double*, int32_t*);
    Kern kern = nullptr;
    switch (D) {
    case 2: kern = hullnd_kernel<2>; break;
    case 3: kern = hullnd_kernel<3>; break;
    case 4: kern = hullnd_kernel<4>; break;
    case 5: kern = hullnd_kernel<5>; break;
    case 6: kern = hullnd_kernel<6>; break;
    case 7: kern = hullnd_kernel<7>; break;
    case 8: kern = hullnd_kernel<8>; break;
    default:
        return set_error(BLF_ERR_INVALID_ARGUMENT, "hullnd: dim %d outside [1, %d]", D, BLF_HULLND_MAX_DIM);
    }
    if (lds > 65536) {   // above the default dynamic LDS limit (up to 80 KB at P = 32, M = 1024, D = 8)
        const blf_status st = check_hip(
            hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
            "hullnd_kernel LDS attribute");
        if (st != BLF_OK) return st;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)batch), dim3(64), lds, s, pts, npts, P, M, A, b, nf);
    return check_hip(hipGetLastError(), "hullnd_kernel launch");
}

}  // namespace blf
