// planners.hip — support-polygon H-representation (ConvexHullHelper) and quintic swing-foot
// splines on the device.
//
//  * hull2d_kernel: one lane per polygon (ConvexHullHelper::buildConvexHull + getA/getB,
//    src/Planners/src/ConvexHullHelper.cpp:35-99).  The workgroup's contiguous slab of input
//    points is loaded coalesced and transposed into lane-minor LDS arrays; each lane then sorts
//    its points in place (a sorting network for p <= 8 finite points, else insertion sort) and
//    chains them: for p <= 8 finite points by the all-triples rule (a point is a lower / upper
//    chain vertex iff every triple around it turns strictly; branch-free, in registers), else by
//    Andrew's monotone chain with a `cross <= 0` pop (chain stack packed in a register for
//    P <= 8).  Both drop collinear boundary points the way Qhull's "Qt" facet merge
//    does.  The facets are then computed and stored by (polygon, facet) pair, coalesced.  Output rows: unit outward normal,
//    b = n . v (inside: A x <= b), counter-clockwise from the leftmost-lowest vertex.
//  * hull2d_contains_kernel: doesPointBelongToConvexHull (ConvexHullHelper.cpp:101-117): strict
//    `(A p)_i > b_i` rejects, no tolerance.
//  * quintic_fit_kernel / quintic_eval_kernel: QuinticSpline (absent in the reference, SURVEY.md
//    8(a) A2).  Knot rule = getPresentContact (ContactList.cpp:190-202): the last knot with
//    t_j <= t, -1 if none; the evaluated segment is that index clamped to [0, K-1].
// Built with -ffp-contract=off; same expression order as oracle/blf_oracle.c.
#include "blf_internal.h"
#include "slab.h"

namespace blf {
namespace {

constexpr int kHullBlock = 64;
// LDS row stride of the X / Y arrays in doubles, and the Y array's extra offset.  A row is 64
// polygons; 68 = 64 + 4 puts vertex row a of polygon r on bank pair (8 a + 2 r) mod 64, so the
// eight facets of a polygon that phase 2 reads in one lane group hit distinct banks (a stride of
// 64 put all eight on one bank: 8-way), and the Y array's 2-double offset interleaves the
// staging stores of X and Y (16-way on one bank pair before: 13 % of the wave's cycles).
#ifndef BLF_HULL_PAD
#define BLF_HULL_PAD 1
#endif
constexpr int kHullStride = BLF_HULL_PAD ? 68 : 64;   // BLF_HULL_PAD=0: the unpadded layout (A/B)
constexpr int kHullYOff = BLF_HULL_PAD ? 2 : 0;
#ifndef BLF_HULL_U
#define BLF_HULL_U 8
#endif
constexpr int HU = BLF_HULL_U;   // facet pairs per lane in flight (phase 2)

__device__ __forceinline__ double cross3(double ox, double oy, double ax, double ay, double bx,
                                         double by)
{
    return (ax - ox) * (by - oy) - (ay - oy) * (bx - ox);
}

// Dynamic LDS of hull2d_kernel, per workgroup of 64 polygons (one per lane), lane-minor so that
// the data-dependent indices of the sort and the chain never conflict:
//   X, Y   [P][kHullStride] doubles (Y offset by kHullYOff): the points, sorted in place by the lane
//   stack  P <= 8: [64] uint64, the monotone chain packed 3 bits per entry (at most 2P + 2 = 18
//          entries), held in a register while the chain runs;
//          P > 8: [2P+2][64] int32, the chain as positions in the sorted arrays
//   nf     [64] int32
// The packed stack frees 4 KB per workgroup (8.8 KB instead of 12.8 KB at P = 8): LDS is what
// bounds the resident wavefronts of this latency-bound kernel.
__host__ __device__ inline bool hull2d_packed(int P) { return P <= 8; }
__host__ __device__ inline size_t hull2d_lds_bytes(int P, int /*M*/)
{
    const size_t xy = sizeof(double) * ((size_t)kHullStride * 2 * P + kHullYOff);
    if (hull2d_packed(P)) return xy + sizeof(uint64_t) * kHullBlock + sizeof(int32_t) * kHullBlock;
    return xy + sizeof(int32_t) * kHullBlock * (2 * P + 3);
}

__device__ __forceinline__ int hull2d_rows(int64_t batch, int64_t p0)
{
    return (int)((batch - p0) < kHullBlock ? (batch - p0) : kHullBlock);
}

// Phase 1 (lane per polygon): up to 8 finite points are sorted by a network and chained by the
// all-triples rule in registers; otherwise an insertion sort of the coordinates by (x, y) with the
// oracle's comparisons in the oracle's order (a stable sort, identical for any input including
// NaN), then Andrew's monotone chain with the top two stack points held in registers (LDS is read
// only on a pop).  Phase 2 (after a barrier): consecutive threads take consecutive (polygon, facet) pairs,
// compute the facet once and store A as 16-B and b as 8-B coalesced writes.
template <bool PK>
#ifndef BLF_HULL_MINWAVES   // waves per SIMD the register allocation must allow (A/B builds)
#define BLF_HULL_MINWAVES 1
#endif
__global__ __launch_bounds__(kHullBlock, BLF_HULL_MINWAVES) void hull2d_kernel(const double* __restrict__ pts,
                                                            const int32_t* __restrict__ npts,
                                                            int32_t P, int32_t M, int64_t batch,
                                                            double* __restrict__ Aout,
                                                            double* __restrict__ bout,
                                                            int32_t* __restrict__ nfout)
{
    extern __shared__ double hull_smem[];
    const int t = threadIdx.x;
    const int64_t p0 = (int64_t)blockIdx.x * kHullBlock;
    const int nprob = hull2d_rows(batch, p0);
    double* s_x = hull_smem;                                               // [P][68]
    double* s_y = s_x + kHullStride * P + kHullYOff;                       // [P][68]
    int32_t* s_stk = reinterpret_cast<int32_t*>(s_y + kHullStride * P);    // [2P+2][64] (!PK)
    uint64_t* s_pk = reinterpret_cast<uint64_t*>(s_y + kHullStride * P);   // [64] (PK)
    int32_t* s_nf = PK ? reinterpret_cast<int32_t*>(s_pk + kHullBlock) : s_stk + kHullBlock * (2 * P + 2);
    // the lane's point count, issued before the slab so its latency hides under the slab's
    const int n = t < nprob ? npts[p0 + t] : 0;
    {
        // coalesced load of the [64][P][2] slab, transposed into X / Y: every load of a lane in
        // flight before the first LDS store (P <= 8: 16 per lane, one memory round trip; larger
        // P: 8 at a time)
        constexpr int UL = PK ? 16 : 8;
        const double* src = pts + p0 * 2 * P;
        const int ne = nprob * 2 * P;
        const SlabIdx ix(2 * P);
        for (int base = 0; base < ne; base += UL * kHullBlock) {
            double v[UL];
#pragma unroll
            for (int u = 0; u < UL; ++u) {
                const int e = base + u * kHullBlock + t;
                if (e < ne) v[u] = src[e];
            }
#pragma unroll
            for (int u = 0; u < UL; ++u) {
                const int e = base + u * kHullBlock + t;
                if (e < ne) {
                    const int r = ix.row(e), c = e - r * 2 * P;
                    (c & 1 ? s_y : s_x)[(c >> 1) * kHullStride + r] = v[u];
                }
            }
        }
    }
    __syncthreads();
#define HX(i) s_x[(i) * kHullStride + t]
#define HY(i) s_y[(i) * kHullStride + t]
    // the chain stack: packed 3-bit entries in a register (PK), else lane-minor int32 in LDS
    uint64_t stk = 0;
#define STK_GET(i) (PK ? (int)((stk >> (3 * (i))) & 7) : s_stk[(i) * kHullBlock + t])
#define STK_SET(i, v)                                                                           \
    do {                                                                                        \
        if (PK) stk = (stk & ~(7ull << (3 * (i)))) | ((uint64_t)(v) << (3 * (i)));              \
        else s_stk[(i) * kHullBlock + t] = (v);                                                 \
    } while (0)
    int nf = -1;
    if (t < nprob && n >= 3 && n <= P) {
        // Up to 8 points with finite coordinates: a 19-comparator sorting network in registers,
        // branch-free, keyed (x, y, original index) -- for finite keys exactly the permutation of
        // the stable insertion sort below -- and the chain by the all-triples rule (below), also
        // branch-free and in registers.  Non-finite coordinates (NaN comparisons) or more than 8
        // points keep the insertion sort and Andrew's chain, so every input sorts and chains as
        // the oracle does (orc_hull2d_hrep takes the same two paths).
        bool done = false;
        int nv = 0;
        if (n <= 8) {
            double x[8], y[8];
            int id[8];
            bool clean = true;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const bool in = i < n;
                x[i] = in ? HX(i) : __builtin_inf();
                y[i] = in ? HY(i) : __builtin_inf();
                id[i] = i;
                clean = clean && (!in || (__builtin_isfinite(x[i]) && __builtin_isfinite(y[i])));
            }
            if (clean) {
#define HULL_CE(a, b)                                                                       \
    do {                                                                                    \
        const bool g = x[a] > x[b] || (x[a] == x[b] && (y[a] > y[b] || (y[a] == y[b] && id[a] > id[b]))); \
        const double xa = x[a], ya = y[a];                                                  \
        const int ia = id[a];                                                               \
        x[a] = g ? x[b] : xa; y[a] = g ? y[b] : ya; id[a] = g ? id[b] : ia;                 \
        x[b] = g ? xa : x[b]; y[b] = g ? ya : y[b]; id[b] = g ? ia : id[b];                 \
    } while (0)
                HULL_CE(0, 2); HULL_CE(1, 3); HULL_CE(4, 6); HULL_CE(5, 7);
                HULL_CE(0, 4); HULL_CE(1, 5); HULL_CE(2, 6); HULL_CE(3, 7);
                HULL_CE(0, 1); HULL_CE(2, 3); HULL_CE(4, 5); HULL_CE(6, 7);
                HULL_CE(2, 4); HULL_CE(3, 5);
                HULL_CE(1, 4); HULL_CE(3, 6);
                HULL_CE(1, 2); HULL_CE(3, 4); HULL_CE(5, 6);
#undef HULL_CE
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (i < n) {
                        HX(i) = x[i];
                        HY(i) = y[i];
                    }
                // The chain without a stack: sorted point j (0 < j < n - 1) is a lower-chain vertex
                // iff cross3(p_i, p_j, p_k) > 0 for every i < j < k < n, an upper-chain vertex iff
                // cross3(p_k, p_j, p_i) > 0 for every such pair -- the triples Andrew's pops test,
                // in the same argument order (in exact arithmetic exactly the chain's vertices:
                // strictly convex ones, collinear and duplicate points dropped).  56 triples, no
                // data-dependent loop, no LDS round trip.
                // Duplicates: Andrew's lower pass keeps the last copy of a repeated point (the first
                // at the left end), its upper pass the first copy (none at the right end), so a
                // copy's own duplicates do not reject it there.
                bool bl[8], bu[8], at0[8], atn[8];
                double xn = x[0], yn = y[0];
#pragma unroll
                for (int s = 1; s < 8; ++s) {
                    xn = s == n - 1 ? x[s] : xn;
                    yn = s == n - 1 ? y[s] : yn;
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    bl[j] = bu[j] = false;
                    at0[j] = x[j] == x[0] && y[j] == y[0];
                    atn[j] = x[j] == xn && y[j] == yn;
                }
#pragma unroll
                for (int k = 2; k < 8; ++k) {
                    const bool kin = k < n;
#pragma unroll
                    for (int j = 1; j < k; ++j) {
                        const bool ui = !(x[k] == x[j] && y[k] == y[j]) || atn[j];
#pragma unroll
                        for (int i = 0; i < j; ++i) {
                            const bool li = !(x[i] == x[j] && y[i] == y[j]) || at0[j];
                            const double cl = cross3(x[i], y[i], x[j], y[j], x[k], y[k]);
                            const double cu = cross3(x[k], y[k], x[j], y[j], x[i], y[i]);
                            bl[j] = bl[j] || (kin && li && !(cl > 0.0));
                            bu[j] = bu[j] || (kin && ui && !(cu > 0.0));
                        }
                    }
                }
                // H: the lower chain left to right (0 and n - 1 always), the upper chain right to
                // left, then 0 again -- Andrew's stack, 3 bits per entry
                uint64_t st = 0;
                int k = 0;
#pragma unroll
                for (int s = 0; s < 8; ++s)
                    if (s < n && (s == 0 || s == n - 1 || !bl[s])) {
                        st |= (uint64_t)s << (3 * k);
                        ++k;
                    }
#pragma unroll
                for (int s = 7; s >= 1; --s)
                    if (s < n - 1 && !bu[s]) {
                        st |= (uint64_t)s << (3 * k);
                        ++k;
                    }
                ++k;   // the closing 0
                if (PK) {
                    stk = st;
                } else {
                    for (int i = 0; i < k; ++i) s_stk[i * kHullBlock + t] = (int)((st >> (3 * i)) & 7);
                }
                nv = k - 1;
                done = true;
            }
        }
        if (!done) {
            for (int i = 1; i < n; ++i) {
                const double vx = HX(i), vy = HY(i);
                int j = i - 1;
                while (j >= 0) {
                    const double ux = HX(j), uy = HY(j);
                    if (!(ux > vx || (ux == vx && uy > vy))) break;
                    HX(j + 1) = ux;
                    HY(j + 1) = uy;
                    --j;
                }
                HX(j + 1) = vx;
                HY(j + 1) = vy;
            }
            // monotone chain; (ax, ay) = STK(k-2), (bx, by) = STK(k-1) when they exist
            int k = 0;
            double ax = 0.0, ay = 0.0, bx = 0.0, by = 0.0;
            for (int i = 0; i < n; ++i) {
                const double px = HX(i), py = HY(i);
                while (k >= 2) {
                    if (cross3(ax, ay, bx, by, px, py) <= 0.0) {
                        --k;
                        bx = ax;
                        by = ay;
                        if (k >= 2) {
                            const int a = STK_GET(k - 2);
                            ax = HX(a);
                            ay = HY(a);
                        }
                    } else {
                        break;
                    }
                }
                STK_SET(k, i);
                ++k;
                ax = bx;
                ay = by;
                bx = px;
                by = py;
            }
            const int lower = k + 1;
            for (int i = n - 2; i >= 0; --i) {
                const double px = HX(i), py = HY(i);
                while (k >= lower) {
                    if (cross3(ax, ay, bx, by, px, py) <= 0.0) {
                        --k;
                        bx = ax;
                        by = ay;
                        if (k >= 2) {
                            const int a = STK_GET(k - 2);
                            ax = HX(a);
                            ay = HY(a);
                        }
                    } else {
                        break;
                    }
                }
                STK_SET(k, i);
                ++k;
                ax = bx;
                ay = by;
                bx = px;
                by = py;
            }
            nv = k - 1;
        }
        if (nv >= 3 && nv <= M) nf = nv;
    }
#undef HX
#undef HY
#undef STK_GET
#undef STK_SET
    if (t < nprob) {
        s_nf[t] = nf;
        nfout[p0 + t] = nf;
        if (PK) s_pk[t] = stk;
    }
    __syncthreads();
    // phase 2: (polygon r, facet j) pairs in output order
    const int npair = nprob * M;
    double* Ab = Aout + p0 * 2 * M;
    double* bb = bout + p0 * M;
    const bool vecA = ((uintptr_t)Ab & 15) == 0;
    const SlabIdx im(M);
    auto facet = [&](int e, double& nx, double& ny, double& bj) {
        const int r = im.row(e), j = e - r * M;
        nx = 0.0;
        ny = 0.0;
        bj = 0.0;
        if (j < s_nf[r]) {
            int a, b;
            if (PK) {
                const uint64_t sk = s_pk[r];
                a = (int)((sk >> (3 * j)) & 7);
                b = (int)((sk >> (3 * (j + 1))) & 7);
            } else {
                a = s_stk[j * kHullBlock + r];
                b = s_stk[(j + 1) * kHullBlock + r];
            }
            const double v0x = s_x[a * kHullStride + r], v0y = s_y[a * kHullStride + r];
            const double ex = s_x[b * kHullStride + r] - v0x;
            const double ey = s_y[b * kHullStride + r] - v0y;
            // one reciprocal of the edge length instead of two quotients (oracle orc_hull2d_hrep)
            const double il = 1.0 / sqrt(ex * ex + ey * ey);
            nx = ey * il;
            ny = (-ex) * il;
            bj = nx * v0x + ny * v0y;
        }
    };
    auto put = [&](int e, double nx, double ny, double bj) {
        if (vecA) {
            *reinterpret_cast<double2*>(Ab + 2 * e) = make_double2(nx, ny);
        } else {
            Ab[2 * e] = nx;
            Ab[2 * e + 1] = ny;
        }
        bb[e] = bj;
    };
    int e = t;
    // HU pairs per lane at a time: their LDS reads, square roots and divisions are independent,
    // so they overlap instead of serialising one pair's latency chain after another
    for (; e + (HU - 1) * kHullBlock < npair; e += HU * kHullBlock) {
        double nx[HU], ny[HU], bj[HU];
#pragma unroll
        for (int u = 0; u < HU; ++u) facet(e + u * kHullBlock, nx[u], ny[u], bj[u]);
#pragma unroll
        for (int u = 0; u < HU; ++u) put(e + u * kHullBlock, nx[u], ny[u], bj[u]);
    }
    for (; e < npair; e += kHullBlock) {
        double nx, ny, bj;
        facet(e, nx, ny, bj);
        put(e, nx, ny, bj);
    }
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
    // a count outside [0, M] is a bad polygon: nothing belongs to it, and no row past the
    // problem's own M is read
    const int m0 = nf[q];
    const bool okm = m0 >= 0 && m0 <= M;
    const int m = okm ? m0 : 0;
    int in = okm ? 1 : 0;
    const double px = query[2 * q], py = query[2 * q + 1];
    for (int i = 0; i < m; ++i)
        if (A[(q * M + i) * 2] * px + A[(q * M + i) * 2 + 1] * py > b[q * M + i]) in = 0;
    inside[q] = in;
}

// 3-D hull (ConvexHullHelper::buildConvexHull on 3 x p points; the reference's own test,
// ConvexHullHelperTest.cpp:15-63, is 3-D): one lane per point set, the supporting planes through
// every triple in lexicographic order, deduplicated -- oracle orc_hull3d_hrep states the rule and
// runs the same operations in the same order.  Off the planning path (the support polygons are
// 2-D), so it stays a plain lane-per-set kernel reading its points through L1/L2.
__global__ __launch_bounds__(64) void hull3d_kernel(const double* __restrict__ pts,
                                                    const int32_t* __restrict__ npts, int32_t P,
                                                    int32_t M, int64_t batch,
                                                    double* __restrict__ Aout,
                                                    double* __restrict__ bout,
                                                    int32_t* __restrict__ nfout)
{
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= batch) return;
    const double* q = pts + s * 3 * P;
    double* A = Aout + s * 3 * M;
    double* b = bout + s * M;
    for (int e = 0; e < 3 * M; ++e) A[e] = 0.0;
    for (int e = 0; e < M; ++e) b[e] = 0.0;
    const int n = npts[s];
    if (n < 4 || n > P) {
        nfout[s] = -1;
        return;
    }
    double scale = 0.0;
    for (int e = 0; e < 3 * n; ++e) {
        const double a = fabs(q[e]);
        if (a > scale) scale = a;
    }
    const double tol = 1e-12 * (1.0 + scale);
    const double btol = 1e-9 * (1.0 + scale);
    int count = 0;
    bool overflow = false;
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j)
            for (int k = j + 1; k < n; ++k) {
                const double pix = q[3 * i], piy = q[3 * i + 1], piz = q[3 * i + 2];
                const double ux = q[3 * j] - pix, uy = q[3 * j + 1] - piy, uz = q[3 * j + 2] - piz;
                const double vx = q[3 * k] - pix, vy = q[3 * k + 1] - piy, vz = q[3 * k + 2] - piz;
                const double cx = uy * vz - uz * vy;
                const double cy = uz * vx - ux * vz;
                const double cz = ux * vy - uy * vx;
                const double len = sqrt(cx * cx + cy * cy + cz * cz);
                if (!(len > 0.0)) continue;
                double nx = cx / len, ny = cy / len, nz = cz / len;
                bool pos = false, neg = false;
                for (int l = 0; l < n; ++l) {
                    const double d = nx * (q[3 * l] - pix) + ny * (q[3 * l + 1] - piy) +
                                     nz * (q[3 * l + 2] - piz);
                    pos = pos || d > tol;
                    neg = neg || d < -tol;
                }
                if ((pos && neg) || !(pos || neg)) continue;
                if (pos) {
                    nx = -nx;
                    ny = -ny;
                    nz = -nz;
                }
                double bm = -__builtin_inf();
                for (int l = 0; l < n; ++l) {
                    const double v = nx * q[3 * l] + ny * q[3 * l + 1] + nz * q[3 * l + 2];
                    if (v > bm) bm = v;
                }
                bool dup = false;
                for (int e = 0; e < count && e < M; ++e)
                    dup = dup || (fabs(A[3 * e] - nx) <= 1e-9 && fabs(A[3 * e + 1] - ny) <= 1e-9 &&
                                  fabs(A[3 * e + 2] - nz) <= 1e-9 && fabs(b[e] - bm) <= btol);
                if (dup) continue;
                if (count < M) {
                    A[3 * count] = nx;
                    A[3 * count + 1] = ny;
                    A[3 * count + 2] = nz;
                    b[count] = bm;
                } else {
                    overflow = true;
                }
                ++count;
            }
    if (overflow || count < 4) {
        for (int e = 0; e < 3 * M; ++e) A[e] = 0.0;
        for (int e = 0; e < M; ++e) b[e] = 0.0;
        count = -1;
    }
    nfout[s] = count;
}

// doesPointBelongToConvexHull in any dimension (ConvexHullHelper.cpp:101-117): strict `>` rejects.
__global__ __launch_bounds__(256) void halfspace_contains_kernel(const double* __restrict__ A,
                                                                 const double* __restrict__ b,
                                                                 const int32_t* __restrict__ nf,
                                                                 int32_t dim, int32_t M,
                                                                 const double* __restrict__ query,
                                                                 int64_t batch,
                                                                 int32_t* __restrict__ inside)
{
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= batch) return;
    const int m0 = nf[s];   // outside [0, M]: a bad hull, nothing belongs to it (as above)
    const bool okm = m0 >= 0 && m0 <= M;
    const int m = okm ? m0 : 0;
    int in = okm ? 1 : 0;
    const double* p = query + s * dim;
    for (int i = 0; i < m; ++i) {
        double v = 0.0;
        for (int c = 0; c < dim; ++c) v = v + A[(s * M + i) * dim + c] * p[c];
        if (v > b[s * M + i]) in = 0;
    }
    inside[s] = in;
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

// one lane per (spline, query); the workgroup's [256][3][D] output slab is staged in LDS and
// written with coalesced 16-B stores (slab.h)
#ifndef BLF_Q_BLOCK   // queries per workgroup (A/B builds)
#define BLF_Q_BLOCK 256
#endif
constexpr int kEvalBlock = BLF_Q_BLOCK;
#ifndef BLF_Q_STAGE
#define BLF_Q_STAGE 512
#endif
constexpr int kEvalStage = BLF_Q_STAGE;
#ifndef BLF_Q_DIRECT
#define BLF_Q_DIRECT 0
#endif   // doubles of staged spline data per workgroup (4 KB)

template <bool VEC>
__global__ __launch_bounds__(kEvalBlock) void quintic_eval_kernel(const double* __restrict__ kt,
                                                                  const double* __restrict__ coeffs,
                                                                  int32_t K1, int32_t D, int64_t S,
                                                                  const double* __restrict__ tq,
                                                                  int32_t Q, double* __restrict__ pva,
                                                                  int32_t* __restrict__ idx)
{
    __shared__ __attribute__((aligned(16))) double s_out[kEvalBlock * 9];
    __shared__ __attribute__((aligned(16))) double s_spl[kEvalStage];   // the splines' knots + coefficients
    const int K = K1 - 1;
    const int W = 3 * D, SW = odd_stride(W);
    const int64_t g0 = (int64_t)blockIdx.x * kEvalBlock;
    const int64_t gid = g0 + threadIdx.x;
    const int rows = (int)((S * Q - g0) < kEvalBlock ? (S * Q - g0) : kEvalBlock);
    // 32-bit division when the launch fits (every bench / test shape): the 64-bit one is a long
    // VALU sequence per lane
    const bool small = S * Q < 0x7fffffffLL;
    auto spline_of = [&](int64_t g) { return small ? (int64_t)((uint32_t)g / (uint32_t)Q) : g / Q; };
    // The workgroup's queries belong to a few consecutive splines (8-9 at 32 queries each), whose
    // knots and coefficients are contiguous: staged once into LDS (coalesced, in flight together
    // with the query times) instead of every lane gathering its segment from L2 after its knot
    // search.  Larger spans read global memory as before.
    const int64_t sp0 = spline_of(g0);
    const int nsp = (int)(spline_of(g0 + rows - 1) - sp0 + 1);
    const int ncf = nsp * K * D * 6, nkt = nsp * K1;
    const bool staged = VEC && ncf + nkt <= kEvalStage;
    double tt = 0.0;
    if (gid < S * Q) tt = __builtin_nontemporal_load(tq + gid);   // streamed once
    if (staged) {
        const double2* gc = reinterpret_cast<const double2*>(coeffs + sp0 * K * D * 6);
        double2* sc = reinterpret_cast<double2*>(s_spl + nkt + (nkt & 1));
        for (int j = threadIdx.x; j < ncf / 2; j += kEvalBlock) sc[j] = gc[j];
        for (int j = threadIdx.x; j < nkt; j += kEvalBlock) s_spl[j] = kt[sp0 * K1 + j];
        __syncthreads();
    }
    if (gid < S * Q) {
        const int64_t sp = spline_of(gid);
        const double* t = staged ? s_spl + (sp - sp0) * K1 : kt + sp * K1;
        // last j with t_j <= t: a forward pass keeps the knot loads independent of each other
        // (up to 8 knots all issued before the first comparison)
        int raw = -1;
        if (K1 <= 8) {
            double tk[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) tk[j] = j < K1 ? t[j] : 0.0;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j < K1 && tk[j] <= tt) raw = j;
        } else {
            for (int j = 0; j < K1; ++j)
                if (t[j] <= tt) raw = j;
        }
        __builtin_nontemporal_store(raw, idx + gid);
        const int seg = raw < 0 ? 0 : (raw > K - 1 ? K - 1 : raw);
        const double tau = tt - t[seg];
        double* o = s_out + threadIdx.x * SW;
        const double* cbase = staged ? s_spl + nkt + (nkt & 1) + ((sp - sp0) * K + seg) * D * 6
                                     : coeffs + (sp * K + seg) * D * 6;
        for (int d = 0; d < D; ++d) {
            // the segment's 6 coefficients are 48 contiguous bytes: three 16-B loads when the
            // array is 16-B aligned (VEC), six 8-B loads otherwise
            const double* cp = cbase + d * 6;
            double c0, c1, c2, c3, c4, c5;
            if (VEC) {
                const double2* c = reinterpret_cast<const double2*>(cp);
                const double2 ca = c[0], cb = c[1], cc = c[2];
                c0 = ca.x; c1 = ca.y; c2 = cb.x; c3 = cb.y; c4 = cc.x; c5 = cc.y;
            } else {
                c0 = cp[0]; c1 = cp[1]; c2 = cp[2]; c3 = cp[3]; c4 = cp[4]; c5 = cp[5];
            }
            const double p = c0 + tau * (c1 + tau * (c2 + tau * (c3 + tau * (c4 + tau * c5))));
            const double v = c1 + tau * (2.0 * c2 + tau * (3.0 * c3 + tau * (4.0 * c4 + tau * (5.0 * c5))));
            const double a = 2.0 * c2 + tau * (6.0 * c3 + tau * (12.0 * c4 + tau * (20.0 * c5)));
            if (BLF_Q_DIRECT) {   // A/B: the lane's own row straight to HBM (plain stores)
                double* og = pva + gid * W;
                og[d] = p;
                og[D + d] = v;
                og[2 * D + d] = a;
            } else {
                o[d] = p;
                o[D + d] = v;
                o[2 * D + d] = a;
            }
        }
    }
    if (BLF_Q_DIRECT) return;
    __syncthreads();
    slab_store<kEvalBlock, 6>(pva + g0 * W, W, s_out, SW, rows, W);   // 9 doubles x 256: one batch
}

}  // namespace

blf_status launch_hull2d(const double* pts, const int32_t* npts, int32_t P, int32_t M,
                         int64_t batch, double* A, double* b, int32_t* nf, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    const int64_t blocks = ceil_div(batch, kHullBlock);
    const size_t lds = hull2d_lds_bytes(P, M);
    auto kern = hull2d_packed(P) ? hull2d_kernel<true> : hull2d_kernel<false>;
    if (lds > 65536) {
        const blf_status st = check_hip(
            hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds),
            "hull2d_kernel LDS attribute");
        if (st != BLF_OK) return st;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kHullBlock), lds, s, pts, npts, P, M,
                       batch, A, b, nf);
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

blf_status launch_hull3d(const double* pts, const int32_t* npts, int32_t P, int32_t M,
                         int64_t batch, double* A, double* b, int32_t* nf, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    hipLaunchKernelGGL(hull3d_kernel, dim3((unsigned)ceil_div(batch, 64)), dim3(64), 0, s, pts, npts,
                       P, M, batch, A, b, nf);
    return check_hip(hipGetLastError(), "hull3d_kernel launch");
}

blf_status launch_halfspace_contains(const double* A, const double* b, const int32_t* nf,
                                     int32_t dim, int32_t M, const double* q, int64_t batch,
                                     int32_t* inside, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    hipLaunchKernelGGL(halfspace_contains_kernel, dim3((unsigned)ceil_div(batch, 256)), dim3(256),
                       0, s, A, b, nf, dim, M, q, batch, inside);
    return check_hip(hipGetLastError(), "halfspace_contains_kernel launch");
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
    const bool vec = ((uintptr_t)coeffs & 15) == 0;
    const int64_t ntiles = ceil_div(n, kEvalBlock);
    auto kern = vec ? quintic_eval_kernel<true> : quintic_eval_kernel<false>;
    hipLaunchKernelGGL(kern, dim3((unsigned)ntiles), dim3(kEvalBlock), 0, s, kt,
                       coeffs, K1, D, S, tq, Q, pva, idx);
    return check_hip(hipGetLastError(), "quintic_eval_kernel launch");
}

}  // namespace blf
