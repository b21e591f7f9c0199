// planners.hip — support-polygon H-representation (ConvexHullHelper) and quintic swing-foot
// splines on the device.
//
//  * hull2d_kernel: one lane per polygon (ConvexHullHelper::buildConvexHull + getA/getB,
//    src/Planners/src/ConvexHullHelper.cpp:35-99).  The workgroup's contiguous slab of input
//    points is staged through LDS with coalesced loads (rows padded to an odd number of doubles so
//    the per-lane reads are bank-conflict free); each lane then sorts its points (insertion sort,
//    p <= 16) and runs Andrew's monotone chain with a `cross <= 0` pop, which merges collinear
//    boundary points the way Qhull's "Qt" facet merge does.  Output rows: unit outward normal,
//    b = n . v (inside: A x <= b), counter-clockwise from the leftmost-lowest vertex.
//  * hull2d_contains_kernel: doesPointBelongToConvexHull (ConvexHullHelper.cpp:101-117): strict
//    `(A p)_i > b_i` rejects, no tolerance.
//  * quintic_fit_kernel / quintic_eval_kernel: QuinticSpline (absent in the reference, SURVEY.md
//    8(a) A2).  Knot rule = getPresentContact (ContactList.cpp:190-202): the last knot with
//    t_j <= t, -1 if none; the evaluated segment is that index clamped to [0, K-1].
// Built with -ffp-contract=off; same expression order as oracle/blf_oracle.c.
#include "blf_internal.h"

namespace blf {
namespace {

constexpr int kHullBlock = 64;
constexpr int kPmax = BLF_HULL_MAX_POINTS;

__device__ __forceinline__ double cross3(double ox, double oy, double ax, double ay, double bx,
                                         double by)
{
    return (ax - ox) * (by - oy) - (ay - oy) * (bx - ox);
}

__global__ __launch_bounds__(kHullBlock) void hull2d_kernel(const double* __restrict__ pts,
                                                            const int32_t* __restrict__ npts,
                                                            int32_t P, int32_t M, int64_t batch,
                                                            double* __restrict__ Aout,
                                                            double* __restrict__ bout,
                                                            int32_t* __restrict__ nfout)
{
    __shared__ double s_pts[kHullBlock * (2 * kPmax + 1)];
    __shared__ unsigned char s_idx[kPmax][kHullBlock];
    __shared__ unsigned char s_H[2 * kPmax + 2][kHullBlock];
    const int t = threadIdx.x;
    const int64_t p0 = (int64_t)blockIdx.x * kHullBlock;
    const int nprob = (int)((batch - p0) < kHullBlock ? (batch - p0) : kHullBlock);
    const int row = 2 * P;            // doubles per polygon in global memory
    const int srow = 2 * P + 1;       // padded LDS row (odd stride)
    const double* src = pts + p0 * row;
    for (int e = t; e < nprob * row; e += kHullBlock) {
        const int r = e / row, c = e - r * row;
        s_pts[r * srow + c] = src[e];
    }
    __syncthreads();
    const int64_t q = p0 + t;
    if (t >= nprob) return;
    const double* X = s_pts + t * srow;   // X[2*i], X[2*i+1]
    double* Aq = Aout + q * M * 2;
    double* bq = bout + q * M;
    for (int i = 0; i < M; ++i) {
        Aq[2 * i] = 0.0;
        Aq[2 * i + 1] = 0.0;
        bq[i] = 0.0;
    }
    const int n = npts[q];
    if (n < 3 || n > P) {
        nfout[q] = -1;
        return;
    }
    // insertion sort by (x, y)
    for (int i = 0; i < n; ++i) s_idx[i][t] = (unsigned char)i;
    for (int i = 1; i < n; ++i) {
        const int v = s_idx[i][t];
        const double vx = X[2 * v], vy = X[2 * v + 1];
        int j = i - 1;
        while (j >= 0) {
            const int u = s_idx[j][t];
            const double ux = X[2 * u], uy = X[2 * u + 1];
            if (!(ux > vx || (ux == vx && uy > vy))) break;
            s_idx[j + 1][t] = (unsigned char)u;
            --j;
        }
        s_idx[j + 1][t] = (unsigned char)v;
    }
    // monotone chain
    int k = 0;
    for (int i = 0; i < n; ++i) {
        const int v = s_idx[i][t];
        const double px = X[2 * v], py = X[2 * v + 1];
        while (k >= 2) {
            const int a = s_H[k - 2][t], b = s_H[k - 1][t];
            if (cross3(X[2 * a], X[2 * a + 1], X[2 * b], X[2 * b + 1], px, py) <= 0.0) --k;
            else break;
        }
        s_H[k++][t] = (unsigned char)v;
    }
    const int lower = k + 1;
    for (int i = n - 2; i >= 0; --i) {
        const int v = s_idx[i][t];
        const double px = X[2 * v], py = X[2 * v + 1];
        while (k >= lower) {
            const int a = s_H[k - 2][t], b = s_H[k - 1][t];
            if (cross3(X[2 * a], X[2 * a + 1], X[2 * b], X[2 * b + 1], px, py) <= 0.0) --k;
            else break;
        }
        s_H[k++][t] = (unsigned char)v;
    }
    const int nv = k - 1;
    if (nv < 3 || nv > M) {
        nfout[q] = -1;
        return;
    }
    for (int j = 0; j < nv; ++j) {
        const int a = s_H[j][t], b = s_H[j + 1][t];
        const double v0x = X[2 * a], v0y = X[2 * a + 1];
        const double ex = X[2 * b] - v0x;
        const double ey = X[2 * b + 1] - v0y;
        const double len = sqrt(ex * ex + ey * ey);
        const double nx = ey / len;
        const double ny = (-ex) / len;
        Aq[2 * j] = nx;
        Aq[2 * j + 1] = ny;
        bq[j] = nx * v0x + ny * v0y;
    }
    nfout[q] = nv;
}

__global__ __launch_bounds__(256) void hull2d_contains_kernel(const double* __restrict__ A,
                                                              const double* __restrict__ b,
                                                              const int32_t* __restrict__ nf,
                                                              int32_t M,
                                                              const double* __restrict__ query,
                                                              int64_t batch,
                                                              int32_t* __restrict__ inside)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= batch) return;
    const int m = nf[q];
    int in = m >= 0 ? 1 : 0;
    const double px = query[2 * q], py = query[2 * q + 1];
    for (int i = 0; i < m; ++i)
        if (A[(q * M + i) * 2] * px + A[(q * M + i) * 2 + 1] * py > b[q * M + i]) in = 0;
    inside[q] = in;
}

// one lane per (spline, segment, axis)
__global__ __launch_bounds__(256) void quintic_fit_kernel(const double* __restrict__ kt,
                                                          const double* __restrict__ kp,
                                                          int32_t K1, int32_t D, int64_t S,
                                                          double* __restrict__ coeffs)
{
    const int K = K1 - 1;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= S * K * D) return;
    const int d = (int)(gid % D);
    const int j = (int)((gid / D) % K);
    const int64_t sp = gid / ((int64_t)D * K);
    const double* t = kt + sp * K1;
    const double* pva = kp + sp * K1 * 3 * D;
    const double T = t[j + 1] - t[j];
    const double T2 = T * T;
    const double T3 = T2 * T;
    const double T4 = T3 * T;
    const double T5 = T4 * T;
    const double p0 = pva[(j * 3 + 0) * D + d];
    const double v0 = pva[(j * 3 + 1) * D + d];
    const double a0 = pva[(j * 3 + 2) * D + d];
    const double p1 = pva[((j + 1) * 3 + 0) * D + d];
    const double v1 = pva[((j + 1) * 3 + 1) * D + d];
    const double a1 = pva[((j + 1) * 3 + 2) * D + d];
    const double c2 = 0.5 * a0;
    const double h = p1 - ((p0 + v0 * T) + c2 * T2);
    const double hv = v1 - (v0 + a0 * T);
    const double ha = a1 - a0;
    double* c = coeffs + ((sp * K + j) * D + d) * 6;
    c[0] = p0;
    c[1] = v0;
    c[2] = c2;
    c[3] = ((10.0 * h - 4.0 * (hv * T)) + 0.5 * (ha * T2)) / T3;
    c[4] = ((-15.0 * h + 7.0 * (hv * T)) - ha * T2) / T4;
    c[5] = ((6.0 * h - 3.0 * (hv * T)) + 0.5 * (ha * T2)) / T5;
}

// one lane per (spline, query)
__global__ __launch_bounds__(256) void quintic_eval_kernel(const double* __restrict__ kt,
                                                           const double* __restrict__ coeffs,
                                                           int32_t K1, int32_t D, int64_t S,
                                                           const double* __restrict__ tq,
                                                           int32_t Q, double* __restrict__ pva,
                                                           int32_t* __restrict__ idx)
{
    const int K = K1 - 1;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= S * Q) return;
    const int64_t sp = gid / Q;
    const double* t = kt + sp * K1;
    const double tt = tq[gid];
    int raw = -1;
    for (int j = K1 - 1; j >= 0; --j)
        if (t[j] <= tt) {
            raw = j;
            break;
        }
    idx[gid] = raw;
    const int seg = raw < 0 ? 0 : (raw > K - 1 ? K - 1 : raw);
    const double tau = tt - t[seg];
    for (int d = 0; d < D; ++d) {
        const double* c = coeffs + ((sp * K + seg) * D + d) * 6;
        const double c0 = c[0], c1 = c[1], c2 = c[2], c3 = c[3], c4 = c[4], c5 = c[5];
        const double p = c0 + tau * (c1 + tau * (c2 + tau * (c3 + tau * (c4 + tau * c5))));
        const double v = c1 + tau * (2.0 * c2 + tau * (3.0 * c3 + tau * (4.0 * c4 + tau * (5.0 * c5))));
        const double a = 2.0 * c2 + tau * (6.0 * c3 + tau * (12.0 * c4 + tau * (20.0 * c5)));
        pva[(gid * 3 + 0) * D + d] = p;
        pva[(gid * 3 + 1) * D + d] = v;
        pva[(gid * 3 + 2) * D + d] = a;
    }
}

}  // namespace

blf_status launch_hull2d(const double* pts, const int32_t* npts, int32_t P, int32_t M,
                         int64_t batch, double* A, double* b, int32_t* nf, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    const int64_t blocks = ceil_div(batch, kHullBlock);
    hipLaunchKernelGGL(hull2d_kernel, dim3((unsigned)blocks), dim3(kHullBlock), 0, s, pts, npts, P,
                       M, batch, A, b, nf);
    return check_hip(hipGetLastError(), "hull2d_kernel launch");
}

blf_status launch_hull2d_contains(const double* A, const double* b, const int32_t* nf, int32_t M,
                                  const double* q, int64_t batch, int32_t* inside, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    hipLaunchKernelGGL(hull2d_contains_kernel, dim3((unsigned)ceil_div(batch, 256)), dim3(256), 0,
                       s, A, b, nf, M, q, batch, inside);
    return check_hip(hipGetLastError(), "hull2d_contains_kernel launch");
}

blf_status launch_quintic_fit(const double* kt, const double* kp, int32_t K1, int32_t D,
                              int64_t S, double* coeffs, hipStream_t s)
{
    const int64_t n = S * (K1 - 1) * D;
    if (n == 0) return BLF_OK;
    hipLaunchKernelGGL(quintic_fit_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, kt,
                       kp, K1, D, S, coeffs);
    return check_hip(hipGetLastError(), "quintic_fit_kernel launch");
}

blf_status launch_quintic_eval(const double* kt, const double* coeffs, int32_t K1, int32_t D,
                               int64_t S, const double* tq, int32_t Q, double* pva, int32_t* idx,
                               hipStream_t s)
{
    const int64_t n = S * Q;
    if (n == 0) return BLF_OK;
    hipLaunchKernelGGL(quintic_eval_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s, kt,
                       coeffs, K1, D, S, tq, Q, pva, idx);
    return check_hip(hipGetLastError(), "quintic_eval_kernel launch");
}

}  // namespace blf
