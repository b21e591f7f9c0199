// euler_rollout.hip — ForwardEuler<LinearTimeInvariantSystem> on the device.
//
//  * lti_euler_kernel: FixedStepIntegrator::integrate(t0, T) for a batch of small LTI systems
//    (n, m <= 8; lti_euler_wg_kernel up to 512; lti_euler_big_kernel any size)
//    (reference: src/System/include/BipedalLocomotion/System/FixedStepIntegrator.tpp:21-72,
//    ForwardEuler.tpp:18-49, src/System/src/LinearTimeInvariantSystem.cpp:71).  The step
//    schedule (count and the stale-time last step) is computed once on the host (blf_capi.hip)
//    and is identical for every system of the batch.  One lane per system.
//  * dcm_rollout_rows_kernel / dcm_rollout_kernel: the DCM instance, one reference Euler step
//    per knot with A = omega_k I, B = -omega_k I.  Horizons up to 160: a wave takes 8 problems'
//    whole rows (contiguous in HBM) through LDS, two lanes per problem; longer horizons: one lane
//    per problem, 64 problems' rows staged in chunks of knots (problem-major layout, DESIGN.md
//    section 3).
// Built with -ffp-contract=off: bit-identical to oracle/blf_oracle.c.
#include "blf_internal.h"
#include "slab.h"

namespace blf {
namespace {

constexpr int kNmax = 8;

__global__ __launch_bounds__(256) void lti_euler_kernel(int n, int m, const double* __restrict__ A,
                                                        const double* __restrict__ Bm, int shared,
                                                        const double* __restrict__ u,
                                                        double* __restrict__ x, int64_t batch,
                                                        int32_t nsteps, double dT, double dT_last)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= batch) return;
    const double* Aq = shared ? A : A + q * n * n;
    const double* Bq = shared ? Bm : Bm + q * n * m;
    double xr[kNmax], ur[kNmax], Ar[kNmax * kNmax], Br[kNmax * kNmax];
#pragma unroll
    for (int r = 0; r < kNmax; ++r) {
        xr[r] = r < n ? x[q * n + r] : 0.0;
        ur[r] = r < m ? u[q * m + r] : 0.0;
#pragma unroll
        for (int c = 0; c < kNmax; ++c) {
            Ar[r * kNmax + c] = (r < n && c < n) ? Aq[r * n + c] : 0.0;
            Br[r * kNmax + c] = (r < n && c < m) ? Bq[r * m + c] : 0.0;
        }
    }
    // B u is constant over the interval (setControlInput holds u), but the reference recomputes
    // it every step; the value is identical, so compute it once.
    double bu[kNmax];
#pragma unroll
    for (int r = 0; r < kNmax; ++r) {
        double acc = Br[r * kNmax + 0] * ur[0];
#pragma unroll
        for (int c = 1; c < kNmax; ++c)
            if (c < m) acc = acc + Br[r * kNmax + c] * ur[c];
        bu[r] = acc;
    }
    for (int32_t i = 0; i < nsteps; ++i) {
        const double h = (i == nsteps - 1) ? dT_last : dT;
        double dx[kNmax];
#pragma unroll
        for (int r = 0; r < kNmax; ++r) {
            double acc = Ar[r * kNmax + 0] * xr[0];
#pragma unroll
            for (int c = 1; c < kNmax; ++c)
                if (c < n) acc = acc + Ar[r * kNmax + c] * xr[c];
            dx[r] = acc + bu[r];
        }
#pragma unroll
        for (int r = 0; r < kNmax; ++r)
            if (r < n) xr[r] = xr[r] + dx[r] * h;
    }
#pragma unroll
    for (int r = 0; r < kNmax; ++r)
        if (r < n) x[q * n + r] = xr[r];
}

// Systems with n or m above kNmax (up to kLtiWgMax): one 64-lane workgroup per system, x and
// B u in LDS, thread t owning rows t, t + 64, ...; each row's sums run left to right exactly as in
// lti_euler_kernel and the oracle, so the results are the same bits.  A and B are read from
// global memory (L2; one copy for every system when shared).
constexpr int kLtiWgMax = 512;   // lti_euler_wg_kernel's limit; above it, lti_euler_big_kernel
constexpr int kLtiRowsPerLane = (kLtiWgMax + 63) / 64;

__global__ __launch_bounds__(64) void lti_euler_wg_kernel(int n, int m, const double* __restrict__ A,
                                                          const double* __restrict__ Bm, int shared,
                                                          const double* __restrict__ u,
                                                          double* __restrict__ x, int32_t nsteps,
                                                          double dT, double dT_last)
{
    extern __shared__ double lti_s[];   // x [n], B u [n]
    const int64_t q = blockIdx.x;
    const int t = threadIdx.x;
    const double* Aq = shared ? A : A + q * n * n;
    const double* Bq = shared ? Bm : Bm + q * n * m;
    const double* uq = u + q * m;
    double* xs = lti_s;
    double* bs = lti_s + n;
    for (int r = t; r < n; r += 64) {
        xs[r] = x[q * n + r];
        double acc = Bq[(int64_t)r * m] * uq[0];
        for (int c = 1; c < m; ++c) acc = acc + Bq[(int64_t)r * m + c] * uq[c];
        bs[r] = acc;
    }
    __syncthreads();
    for (int32_t i = 0; i < nsteps; ++i) {
        const double h = (i == nsteps - 1) ? dT_last : dT;
        double dx[kLtiRowsPerLane];
#pragma unroll
        for (int j = 0; j < kLtiRowsPerLane; ++j) {
            const int r = t + 64 * j;
            dx[j] = 0.0;
            if (r < n) {
                const double* Ar = Aq + (int64_t)r * n;
                double acc = Ar[0] * xs[0];
                for (int c = 1; c < n; ++c) acc = acc + Ar[c] * xs[c];
                dx[j] = acc + bs[r];
            }
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kLtiRowsPerLane; ++j) {
            const int r = t + 64 * j;
            if (r < n) xs[r] = xs[r] + dx[j] * h;
        }
        __syncthreads();
    }
    for (int r = t; r < n; r += 64) x[q * n + r] = xs[r];
}

__global__ __launch_bounds__(256) void lti_dynamics_kernel(int n, int m,
                                                           const double* __restrict__ A,
                                                           const double* __restrict__ Bm,
                                                           int shared,
                                                           const double* __restrict__ u,
                                                           const double* __restrict__ x,
                                                           double* __restrict__ dx, int64_t batch)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= batch) return;
    const double* Aq = shared ? A : A + q * n * n;
    const double* Bq = shared ? Bm : Bm + q * n * m;
    for (int r = 0; r < n; ++r) {
        double ax = Aq[r * n] * x[q * n];
        for (int c = 1; c < n; ++c) ax = ax + Aq[r * n + c] * x[q * n + c];
        double bu = Bq[r * m] * u[q * m];
        for (int c = 1; c < m; ++c) bu = bu + Bq[r * m + c] * u[q * m + c];
        dx[q * n + r] = ax + bu;
    }
}

// Systems above kLtiWgMax (any size, round 5): one 256-thread workgroup per system, the state
// updated in place in x and B u / dx in a global scratch ([batch][n] each), thread t owning rows
// t, t + 256, ...  Each row's sums run left to right as in the kernels above and the oracle (the
// same bits).  A row of A is read once per step; the x it is dotted with stays in L1/L2.  The
// barriers order the reads of step i before the writes of x (__syncthreads is the workgroup-scope
// fence for global memory too).
__global__ __launch_bounds__(256) void lti_euler_big_kernel(int n, int m, const double* __restrict__ A,
                                                            const double* __restrict__ Bm, int shared,
                                                            const double* __restrict__ u, double* x,
                                                            double* scratch, int32_t nsteps,
                                                            double dT, double dT_last)
{
    const int64_t q = blockIdx.x;
    const int t = threadIdx.x;
    const int64_t nn = n;
    const double* Aq = shared ? A : A + q * nn * nn;
    const double* Bq = shared ? Bm : Bm + q * nn * m;
    const double* uq = u + q * m;
    double* xq = x + q * nn;
    double* bs = scratch + 2 * q * nn;
    double* dxs = bs + nn;
    for (int r = t; r < n; r += 256) {
        const double* Br = Bq + (int64_t)r * m;
        double acc = Br[0] * uq[0];
        for (int c = 1; c < m; ++c) acc = acc + Br[c] * uq[c];
        bs[r] = acc;
    }
    for (int32_t i = 0; i < nsteps; ++i) {
        const double h = (i == nsteps - 1) ? dT_last : dT;
        for (int r = t; r < n; r += 256) {
            const double* Ar = Aq + (int64_t)r * nn;
            double acc = Ar[0] * xq[0];
            for (int c = 1; c < n; ++c) acc = acc + Ar[c] * xq[c];
            dxs[r] = acc + bs[r];
        }
        __syncthreads();
        for (int r = t; r < n; r += 256) xq[r] = xq[r] + dxs[r] * h;
        __syncthreads();
    }
}

// dx = A x + B u for systems above kLtiWgMax: one thread per row, rblocks row blocks per system.
__global__ __launch_bounds__(256) void lti_dynamics_rows_kernel(int n, int m,
                                                                const double* __restrict__ A,
                                                                const double* __restrict__ Bm,
                                                                int shared,
                                                                const double* __restrict__ u,
                                                                const double* __restrict__ x,
                                                                double* __restrict__ dx, int rblocks)
{
    const int64_t q = blockIdx.x / rblocks;
    const int r = (int)(blockIdx.x % rblocks) * 256 + threadIdx.x;
    if (r >= n) return;
    const int64_t nn = n;
    const double* Ar = (shared ? A : A + q * nn * nn) + (int64_t)r * nn;
    const double* Br = (shared ? Bm : Bm + q * nn * m) + (int64_t)r * m;
    const double* xq = x + q * nn;
    const double* uq = u + q * m;
    double ax = Ar[0] * xq[0];
    for (int c = 1; c < n; ++c) ax = ax + Ar[c] * xq[c];
    double bu = Br[0] * uq[0];
    for (int c = 1; c < m; ++c) bu = bu + Br[c] * uq[c];
    dx[q * nn + r] = ax + bu;
}

// 64 problems per workgroup (one wave), knots staged in chunks of KC.  The chunk's omega and
// vrp rows are loaded by the whole wave with consecutive lanes on consecutive doubles (one batch
// of loads per lane, 16 B each on full aligned chunks), transposed through LDS; the recurrence
// runs lane-per-problem and the xi chunk leaves through LDS the same way.  (Prefetching the next
// chunk during the recurrence measured no faster and cost 96 VGPRs.)
#ifndef BLF_ROLL_KC
#define BLF_ROLL_KC 32
#endif
constexpr int KC = BLF_ROLL_KC;   // knots per chunk: 64 x 98 x 8 B of LDS per wave (16: 12 % slower,
                                  // per-chunk overhead; 50: the register chunk spills)
constexpr int kRollSw = 2 * KC + 1;   // padded LDS row of the vrp / xi chunk

struct RollChunk {
    double om[KC];       // omega [64][KC]   : double2 element u * 64 + lane
    double r[2 * KC];    // vrp   [64][2 KC] : double2 element u * 64 + lane
};

// Full chunks of a full tile (64 problems x KC knots) with 16-B aligned rows: the element ->
// (row, column) map is compile-time and every global access moves 16 B per lane.
//   omega chunk: 64 rows x KC/2 double2, vrp / xi chunk: 64 rows x KC double2.
__device__ __forceinline__ void roll_load_full(RollChunk& c, const double* __restrict__ omega,
                                               const double* __restrict__ vrp, int64_t p0, int N,
                                               int kb, int lane)
{
#pragma unroll
    for (int u = 0; u < KC / 2; ++u) {
        const int j = u * 64 + lane, r = j / (KC / 2), c2 = j % (KC / 2);
        const double2 v = *reinterpret_cast<const double2*>(omega + (p0 + r) * N + kb + 2 * c2);
        c.om[2 * u] = v.x;
        c.om[2 * u + 1] = v.y;
    }
#pragma unroll
    for (int u = 0; u < KC; ++u) {
        const int j = u * 64 + lane, r = j / KC, c2 = j % KC;
        const double2 v =
            *reinterpret_cast<const double2*>(vrp + (p0 + r) * 2 * N + 2 * kb + 2 * c2);
        c.r[2 * u] = v.x;
        c.r[2 * u + 1] = v.y;
    }
}

__device__ __forceinline__ void roll_to_lds_full(const RollChunk& c, double* s_om, double* s_r,
                                                 int lane)
{
#pragma unroll
    for (int u = 0; u < KC / 2; ++u) {
        const int j = u * 64 + lane, r = j / (KC / 2), c2 = j % (KC / 2);
        s_om[r * (KC + 1) + 2 * c2] = c.om[2 * u];
        s_om[r * (KC + 1) + 2 * c2 + 1] = c.om[2 * u + 1];
    }
#pragma unroll
    for (int u = 0; u < KC; ++u) {
        const int j = u * 64 + lane, r = j / KC, c2 = j % KC;
        s_r[r * kRollSw + 2 * c2] = c.r[2 * u];
        s_r[r * kRollSw + 2 * c2 + 1] = c.r[2 * u + 1];
    }
}

__device__ __forceinline__ void roll_store_full(double* __restrict__ xi_out, const double* s_x,
                                                int64_t p0, int N, int kb, int lane)
{
    double2 v[KC];
#pragma unroll
    for (int u = 0; u < KC; ++u) {
        const int j = u * 64 + lane, r = j / KC, c2 = j % KC;
        v[u].x = s_x[r * kRollSw + 2 * c2];
        v[u].y = s_x[r * kRollSw + 2 * c2 + 1];
    }
#pragma unroll
    for (int u = 0; u < KC; ++u) {
        const int j = u * 64 + lane, r = j / KC, c2 = j % KC;
        st_stream(reinterpret_cast<double2*>(xi_out + (p0 + r) * 2 * (N + 1) + 2 * (kb + 1) + 2 * c2), v[u]);
    }
}

template <bool VEC>
__global__ __launch_bounds__(64) void dcm_rollout_kernel(const double* __restrict__ xi0,
                                                         const double* __restrict__ omega,
                                                         const double* __restrict__ vrp,
                                                         int32_t N, double dt,
                                                         double* __restrict__ xi_out,
                                                         int64_t batch)
{
    // per chunk: omega [64][KC], vrp [64][KC][2] (overwritten in place by xi); rows padded to an
    // odd number of doubles so the per-lane row reads do not conflict.
    __shared__ double s_om[64 * (KC + 1)];
    __shared__ double s_r[64 * kRollSw];
    double* s_x = s_r;
    const int lane = threadIdx.x;
    const int64_t p0 = (int64_t)blockIdx.x * 64;
    const int64_t q = p0 + lane;
    const int nprob = (int)((batch - p0) < 64 ? (batch - p0) : 64);
    double x0 = 0.0, x1 = 0.0;
    if (q < batch) {
        x0 = xi0[2 * q];
        x1 = xi0[2 * q + 1];
        xi_out[2 * q * (N + 1)] = x0;
        xi_out[2 * q * (N + 1) + 1] = x1;
    }
    // VEC: omega / vrp / xi_out 16-B aligned and N even (every row of every array aligned)
    auto full = [&](int kb) { return VEC && nprob == 64 && kb + KC <= N; };
    for (int kb = 0; kb < N; kb += KC) {
        const int kc = (N - kb) < KC ? (N - kb) : KC;
        {
            RollChunk c;
            if (full(kb)) {
                roll_load_full(c, omega, vrp, p0, N, kb, lane);
                roll_to_lds_full(c, s_om, s_r, lane);
            } else {   // tail chunk, partial tile or unaligned rows
                slab_load<64, 8>(s_om, KC + 1, omega + p0 * N + kb, N, nprob, kc);
                slab_load<64, 8>(s_r, kRollSw, vrp + p0 * 2 * N + 2 * kb, 2 * N, nprob, 2 * kc);
            }
        }
        __syncthreads();
        if (lane < nprob) {
            for (int kk = 0; kk < kc; ++kk) {
                const double w = s_om[lane * (KC + 1) + kk];
                const double dx0 = w * x0 + (-w) * s_r[lane * kRollSw + 2 * kk];
                const double dx1 = w * x1 + (-w) * s_r[lane * kRollSw + 2 * kk + 1];
                x0 = x0 + dx0 * dt;
                x1 = x1 + dx1 * dt;
                s_x[lane * kRollSw + 2 * kk] = x0;
                s_x[lane * kRollSw + 2 * kk + 1] = x1;
            }
        }
        __syncthreads();
        if (full(kb)) roll_store_full(xi_out, s_x, p0, N, kb, lane);
        else slab_store<64, 8>(xi_out + p0 * 2 * (N + 1) + 2 * (kb + 1), 2 * (N + 1), s_x,
                               kRollSw, nprob, 2 * kc);
        __syncthreads();
    }
}

// Whole rows, PPW problems per wave (horizons up to kRollRowsMaxN).  The tile's omega, vrp and xi
// rows are contiguous regions of HBM, so the wave reads and writes them as plain 16-B streams
// with whole 128-B lines; chunks of knots across 64 problems (the kernel above) cut every row
// at chunk edges, which re-fetches the lines they split and writes partial lines (1.19x the
// algorithmic bytes fetched).  Two lanes per problem, one per component of xi (the components
// share omega and nothing else).  LDS: omega rows, and vrp rows shifted by one knot with xi0 in
// front, overwritten in place by xi_{k+1} (r_k is read just before xi_{k+1} replaces it), so the
// xi row leaves exactly as it is laid out in xi_out.
constexpr int kRollRowsMaxN = 160;

template <int PPW>
__global__ __launch_bounds__(64) void dcm_rollout_rows_kernel(const double* __restrict__ xi0,
                                                              const double* __restrict__ omega,
                                                              const double* __restrict__ vrp,
                                                              int32_t N, double dt,
                                                              double* __restrict__ xi_out,
                                                              int64_t batch)
{
    extern __shared__ double s_rows[];
    const int SWo = odd_stride(N), SWx = odd_stride(2 * (N + 1));
    double* s_om = s_rows;              // [PPW][SWo]
    double* s_x = s_rows + PPW * SWo;   // [PPW][SWx]: xi0, r_0 .. r_{N-1} -> xi0 .. xi_N
    const int lane = threadIdx.x;
    const int64_t p0 = (int64_t)blockIdx.x * PPW;
    const int np = (int)((batch - p0) < PPW ? (batch - p0) : PPW);
    const double* go = omega + p0 * N;
    const double* gr = vrp + p0 * 2 * N;
    const int no = np * N / 2, nr = np * N;   // 16-B pairs of the tile's omega / vrp regions
    if (lane < 2 * np) s_x[(lane >> 1) * SWx + (lane & 1)] = xi0[2 * p0 + lane];
    constexpr int UO = PPW, UR = 2 * PPW;   // N <= 128
    if (((N & 1) | (((uintptr_t)go | (uintptr_t)gr) & 15)) == 0 && no <= UO * 64 && nr <= UR * 64) {
        // both regions' loads in flight before the first LDS write
        double2 vo[UO], vr[UR];
#pragma unroll
        for (int u = 0; u < UO; ++u) {
            const int j = u * 64 + lane;
            if (j < no) vo[u] = reinterpret_cast<const double2*>(go)[j];
        }
#pragma unroll
        for (int u = 0; u < UR; ++u) {
            const int j = u * 64 + lane;
            if (j < nr) vr[u] = reinterpret_cast<const double2*>(gr)[j];
        }
        const SlabIdx io(N), ir(2 * N);
#pragma unroll
        for (int u = 0; u < UO; ++u) {
            const int e = 2 * (u * 64 + lane);
            if (e < 2 * no) {   // N even: a pair never straddles two rows
                const int r = io.row(e);
                s_om[r * SWo + e - r * N] = vo[u].x;
                s_om[r * SWo + e - r * N + 1] = vo[u].y;
            }
        }
#pragma unroll
        for (int u = 0; u < UR; ++u) {
            const int e = 2 * (u * 64 + lane);
            if (e < 2 * nr) {
                const int r = ir.row(e);
                s_x[2 + r * SWx + e - r * 2 * N] = vr[u].x;
                s_x[2 + r * SWx + e - r * 2 * N + 1] = vr[u].y;
            }
        }
    } else {
        slab_load<64, 8>(s_om, SWo, go, N, np, N);
        slab_load<64, 16>(s_x + 2, SWx, gr, 2 * N, np, 2 * N);
    }
    __syncthreads();
    if (lane < 2 * np) {
        const double* om = s_om + (lane >> 1) * SWo;
        double* xr = s_x + (lane >> 1) * SWx + (lane & 1);
        double x = xr[0];
        int k = 0;
        for (; k + 4 <= N; k += 4) {   // the LDS reads of four knots ahead of their recurrence
            double w[4], r[4];
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                w[g] = om[k + g];
                r[g] = xr[2 * (k + g + 1)];
            }
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const double dx = w[g] * x + (-w[g]) * r[g];
                x = x + dx * dt;
                xr[2 * (k + g + 1)] = x;
            }
        }
        for (; k < N; ++k) {
            const double w = om[k];
            const double dx = w * x + (-w) * xr[2 * (k + 1)];
            x = x + dx * dt;
            xr[2 * (k + 1)] = x;
        }
    }
    __syncthreads();
    slab_store<64, 16>(xi_out + p0 * 2 * (N + 1), 2 * (N + 1), s_x, SWx, np, 2 * (N + 1));
}

#ifndef BLF_ROLL_PPW
#define BLF_ROLL_PPW 8
#endif
constexpr int kRollPPW = BLF_ROLL_PPW;
inline int odd_stride_host(int w) { return w | 1; }

}  // namespace

blf_status launch_lti_euler(int n, int m, const double* A, const double* Bm, int shared,
                            const double* u, double* x, int64_t batch, int32_t nsteps,
                            double dT, double dT_last, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    if (n > kNmax || m > kNmax) {
        if (batch > 0x7fffffffLL)
            return set_error(BLF_ERR_UNSUPPORTED, "lti_euler: %lld systems of size %d too many",
                             (long long)batch, n);
        if (n <= kLtiWgMax && m <= kLtiWgMax) {
            hipLaunchKernelGGL(lti_euler_wg_kernel, dim3((unsigned)batch), dim3(64),
                               2 * sizeof(double) * (size_t)n, s, n, m, A, Bm, shared, u, x, nsteps,
                               dT, dT_last);
            return check_hip(hipGetLastError(), "lti_euler_wg_kernel launch");
        }
        // B u and dx scratch, stream-ordered: allocated, used and released on s.
        double* scratch = nullptr;
        const size_t bytes = 2 * sizeof(double) * (size_t)n * (size_t)batch;
        blf_status st = check_hip(hipMallocAsync((void**)&scratch, bytes, s), "lti_euler scratch");
        if (st != BLF_OK) return st;
        hipLaunchKernelGGL(lti_euler_big_kernel, dim3((unsigned)batch), dim3(256), 0, s, n, m, A, Bm,
                           shared, u, x, scratch, nsteps, dT, dT_last);
        st = check_hip(hipGetLastError(), "lti_euler_big_kernel launch");
        const blf_status fr = check_hip(hipFreeAsync(scratch, s), "lti_euler scratch free");
        return st != BLF_OK ? st : fr;
    }
    const int64_t blocks = ceil_div(batch, 256);
    hipLaunchKernelGGL(lti_euler_kernel, dim3((unsigned)blocks), dim3(256), 0, s, n, m, A, Bm,
                       shared, u, x, batch, nsteps, dT, dT_last);
    return check_hip(hipGetLastError(), "lti_euler_kernel launch");
}

blf_status launch_lti_dynamics(int n, int m, const double* A, const double* Bm, int shared,
                               const double* u, const double* x, double* dx, int64_t batch,
                               hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    if (n > kLtiWgMax || m > kLtiWgMax) {
        const int64_t rblocks = ceil_div(n, 256);
        if (batch * rblocks > 0x7fffffffLL)
            return set_error(BLF_ERR_UNSUPPORTED, "lti_dynamics: %lld systems of size %d too many",
                             (long long)batch, n);
        hipLaunchKernelGGL(lti_dynamics_rows_kernel, dim3((unsigned)(batch * rblocks)), dim3(256), 0,
                           s, n, m, A, Bm, shared, u, x, dx, (int)rblocks);
        return check_hip(hipGetLastError(), "lti_dynamics_rows_kernel launch");
    }
    hipLaunchKernelGGL(lti_dynamics_kernel, dim3((unsigned)ceil_div(batch, 256)), dim3(256), 0, s,
                       n, m, A, Bm, shared, u, x, dx, batch);
    return check_hip(hipGetLastError(), "lti_dynamics_kernel launch");
}

blf_status launch_dcm_rollout(const double* xi0, const double* omega, const double* vrp,
                              int32_t N, double dt, double* xi_out, int64_t batch,
                              hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    if (N <= kRollRowsMaxN) {
        const size_t lds = (size_t)kRollPPW * (odd_stride_host(N) + odd_stride_host(2 * (N + 1))) * 8;
        hipLaunchKernelGGL(dcm_rollout_rows_kernel<kRollPPW>, dim3((unsigned)ceil_div(batch, kRollPPW)),
                           dim3(64), lds, s, xi0, omega, vrp, N, dt, xi_out, batch);
        return check_hip(hipGetLastError(), "dcm_rollout_rows_kernel launch");
    }
    const int64_t blocks = ceil_div(batch, 64);
    const bool vec = (N % 2 == 0) && ((((uintptr_t)omega | (uintptr_t)vrp | (uintptr_t)xi_out) & 15) == 0);
    if (vec)
        hipLaunchKernelGGL(dcm_rollout_kernel<true>, dim3((unsigned)blocks), dim3(64), 0, s, xi0,
                           omega, vrp, N, dt, xi_out, batch);
    else
        hipLaunchKernelGGL(dcm_rollout_kernel<false>, dim3((unsigned)blocks), dim3(64), 0, s, xi0,
                           omega, vrp, N, dt, xi_out, batch);
    return check_hip(hipGetLastError(), "dcm_rollout_kernel launch");
}

}  // namespace blf
