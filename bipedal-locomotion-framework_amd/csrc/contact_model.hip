// contact_model.hip — ContinuousContactModel on the device.
//
//  * contact_eval_kernel: one lane per contact, 64 per wavefront, rows staged through LDS
//    both ways (coalesced 16-B loads and stores).  Computes any subset of the wrench
//    (ContinuousContactModel.cpp:79-108), the autonomous dynamics of the wrench rate (:110-146,
//    R22 without abs exactly as the reference), the control matrix (:148-171) and the regressor
//    (:223-254).  Inputs and outputs are contact-major ([B][6], [B][12], [B][36], [B][12]) so a
//    wavefront's 64 contacts read / write contiguous slabs.
//  * contact_point_kernel: getForceAtPoint / getTorqueGeneratedAtPoint (:173-221) for Q sample
//    points per contact, one lane per (contact, point).
// Built with -ffp-contract=off; every expression in the order of oracle/blf_oracle_contact.c.
#include "blf_internal.h"
#include "contact_math.h"
#include "slab.h"

namespace blf {
namespace {

// skew(e)^2 = e e^T - |e|^2 I, row-major
__device__ __forceinline__ void skew2(V3 e, double* S)
{
    const double n = (e.x * e.x + e.y * e.y) + e.z * e.z;
    const double ev[3] = {e.x, e.y, e.z};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) S[3 * i + j] = i == j ? ev[i] * ev[j] - n : ev[i] * ev[j];
}

// One wavefront per 64 contacts.  The tile's twist / pose / null-pose rows (6 + 12 + 12 doubles
// per contact) arrive as coalesced 16-B loads, all three arrays' loads in flight together, into
// one LDS slab (row stride 31); every lane then reads its own row.  Each requested output leaves
// the same way: the lanes write their rows into LDS and the wave stores the tile's contiguous
// [64][W] region with 16-B stores (slab.h), instead of 64 rows 48-288 B apart per instruction.
constexpr int kCT = 64;           // contacts per workgroup (one wavefront)
constexpr int kCIn = 31;          // LDS input row: twist 6 | pose 12 | null pose 12, odd stride
constexpr int kCOut = 37;         // LDS output row: up to 36 doubles, odd stride

__device__ __forceinline__ void contact_tile_load(double* s_in, const double* twist, const double* pose,
                                                  const double* null_pose, int64_t p0, int rows, int lane)
{
    const double* gt = twist + p0 * 6;
    const double* gp = pose + p0 * 12;
    const double* gn = null_pose + p0 * 12;
    if ((((uintptr_t)gt | (uintptr_t)gp | (uintptr_t)gn) & 15) == 0) {
        const int nt = rows * 3, np = rows * 6;   // 16-B pairs of the three regions
        double2 vt[3], vp[6], vn[6];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int j = u * kCT + lane;
            if (j < nt) vt[u] = reinterpret_cast<const double2*>(gt)[j];
        }
#pragma unroll
        for (int u = 0; u < 6; ++u) {
            const int j = u * kCT + lane;
            if (j < np) {
                vp[u] = reinterpret_cast<const double2*>(gp)[j];
                vn[u] = reinterpret_cast<const double2*>(gn)[j];
            }
        }
        // rows of even width: a pair never straddles two rows
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int j = u * kCT + lane;
            if (j < nt) {
                const int r = j / 3, c = 2 * (j - 3 * r);
                s_in[r * kCIn + c] = vt[u].x;
                s_in[r * kCIn + c + 1] = vt[u].y;
            }
        }
#pragma unroll
        for (int u = 0; u < 6; ++u) {
            const int j = u * kCT + lane;
            if (j < np) {
                const int r = j / 6, c = 2 * (j - 6 * r);
                s_in[r * kCIn + 6 + c] = vp[u].x;
                s_in[r * kCIn + 6 + c + 1] = vp[u].y;
                s_in[r * kCIn + 18 + c] = vn[u].x;
                s_in[r * kCIn + 18 + c + 1] = vn[u].y;
            }
        }
    } else {
        slab_load<kCT, 4>(s_in, kCIn, gt, 6, rows, 6);
        slab_load<kCT, 8>(s_in + 6, kCIn, gp, 12, rows, 12);
        slab_load<kCT, 8>(s_in + 18, kCIn, gn, 12, rows, 12);
    }
}

__global__ __launch_bounds__(kCT) void contact_eval_kernel(
    const double* __restrict__ prm, int shared, const double* __restrict__ twist,
    const double* __restrict__ pose, const double* __restrict__ null_pose, int64_t batch,
    double* __restrict__ wrench, double* __restrict__ autonomous, double* __restrict__ control,
    double* __restrict__ regressor)
{
    // one LDS slab: the input rows, then (after every lane holds its row in registers) the output
    // rows; 18.9 KB per 64 contacts
    __shared__ double s_io[kCT * kCOut];
    double* s_out = s_io;
    const int lane = threadIdx.x;
    const int64_t p0 = (int64_t)blockIdx.x * kCT;
    const int rows = (int)((batch - p0) < kCT ? (batch - p0) : kCT);
    const int64_t q = p0 + lane;
    const bool own = lane < rows;
    contact_tile_load(s_io, twist, pose, null_pose, p0, rows, lane);
    double prv[4] = {0.0, 0.0, 0.0, 0.0};
    if (own) {
        const double* pq = shared ? prm : prm + 4 * q;
#pragma unroll
        for (int i = 0; i < 4; ++i) prv[i] = pq[i];
    }
    __syncthreads();
    double in[30];
#pragma unroll
    for (int i = 0; i < 30; ++i) in[i] = s_io[lane * kCIn + i];
    __syncthreads();
    const double* tw = in;
    const double* ps = in + 6;
    const double* ns = in + 18;
    double* o = s_out + lane * kCOut;
    const double* pr = prv;
    const double L = pr[0], W = pr[1], k = pr[2], b = pr[3];
    const double area = L * W;
    const double LL = L * L, WW = W * W;
    const double v[3] = {tw[0], tw[1], tw[2]};
    const V3 w{tw[3], tw[4], tw[5]};
    const double p[3] = {ps[0], ps[1], ps[2]};
    const double* R = ps + 3;
    const double p0v[3] = {ns[0], ns[1], ns[2]};
    const double* R0 = ns + 3;
    const V3 e1{R[0], R[3], R[6]}, e2{R[1], R[4], R[7]};
    const V3 r01{R0[0], R0[3], R0[6]}, r02{R0[1], R0[4], R0[7]};
    const double R22 = R[8];
    const double aR = fabs(R22);
    const V3 t1 = cross(e1, r01), t2 = cross(e2, r02);
    const V3 c1 = cross(e1, w), c2 = cross(e2, w);
    const V3 u1 = cross(e1, c1), u2 = cross(e2, c2);   // skew(e) skew(e) w
    // the tile's [rows][Wd] output region from the lanes' LDS rows
    auto flush = [&](double* out, int Wd) {
        __syncthreads();
        slab_store<kCT, 12>(out + p0 * Wd, Wd, s_out, kCOut, rows, Wd);
        __syncthreads();
    };
    if (wrench) {
        if (own) contact_wrench(pr, tw, ps, ns, o);
        flush(wrench, 6);
    }
    if (autonomous) {
        if (own) {
            const V3 rd2 = cross(w, V3{R[2], R[5], R[8]});   // (skew(w) R) e3
            const V3 ed1 = cross(w, e1), ed2 = cross(w, e2);
            const double Rd22 = rd2.z;
            const V3 q1 = cross(ed1, r01), q2 = cross(ed2, r02);
            const V3 g1 = cross(ed1, c1), g2 = cross(ed2, c2);
            const V3 h1 = cross(e1, cross(ed1, w)), h2 = cross(e2, cross(ed2, w));
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                o[i] = area * (Rd22 * (k * (p0v[i] - p[i]) - b * v[i]) - (R22 * k) * v[i]);
                const double X = LL * (b * at(u1, i) + k * at(t1, i)) + WW * (b * at(u2, i) + k * at(t2, i));
                const double Y = LL * (k * at(q1, i) + b * (at(g1, i) + at(h1, i)))
                                 + WW * (k * at(q2, i) + b * (at(g2, i) + at(h2, i)));
                o[3 + i] = area / 12.0 * (Rd22 * X + R22 * Y);
            }
        }
        flush(autonomous, 6);
    }
    if (control || regressor) {
        double S1[9], S2[9];
        skew2(e1, S1);
        skew2(e2, S2);
        if (control) {
            if (own) {
                const double d = -area * b * R22;
                const double s = area / 12.0 * R22 * b;
#pragma unroll
                for (int i = 0; i < 6; ++i)
#pragma unroll
                    for (int j = 0; j < 6; ++j) {
                        double c = 0.0;
                        if (i < 3 && j == i) c = d;
                        if (i >= 3 && j >= 3)
                            c = s * (LL * S1[3 * (i - 3) + (j - 3)] + WW * S2[3 * (i - 3) + (j - 3)]);
                        o[6 * i + j] = c;
                    }
            }
            flush(control, 36);
        }
        if (regressor) {
            if (own) {
                const double cf = aR * area;
                const double cv = -aR * area;
                const double ct = area / 12.0 * aR;
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    o[2 * i] = cf * (p0v[i] - p[i]);
                    o[2 * i + 1] = cv * v[i];
                    o[2 * (3 + i)] = ct * (LL * at(t1, i) + WW * at(t2, i));
                    const double M0 = LL * S1[3 * i] + WW * S2[3 * i];
                    const double M1 = LL * S1[3 * i + 1] + WW * S2[3 * i + 1];
                    const double M2 = LL * S1[3 * i + 2] + WW * S2[3 * i + 2];
                    o[2 * (3 + i) + 1] = ct * ((M0 * w.x + M1 * w.y) + M2 * w.z);
                }
            }
            flush(regressor, 12);
        }
    }
}

__global__ __launch_bounds__(256) void contact_point_kernel(
    const double* __restrict__ prm, int shared, const double* __restrict__ twist,
    const double* __restrict__ pose, const double* __restrict__ null_pose, int64_t batch,
    const double* __restrict__ points, int32_t Q, double* __restrict__ force,
    double* __restrict__ torque)
{
    const int64_t id = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= batch * Q) return;
    const int64_t q = id / Q;
    const double* pr = shared ? prm : prm + 4 * q;
    const double L = pr[0], W = pr[1], k = pr[2], b = pr[3];
    const double x = points[2 * id], y = points[2 * id + 1];
    double* fo = force + 3 * id;
    double* to = torque + 3 * id;
    if (fabs(x) > L / 2 || fabs(y) > W / 2) {
#pragma unroll
        for (int i = 0; i < 3; ++i) { fo[i] = 0.0; to[i] = 0.0; }
        return;
    }
    const double* tw = twist + 6 * q;
    const double* ps = pose + 12 * q;
    const double* ns = null_pose + 12 * q;
    const double* R = ps + 3;
    const double* R0 = ns + 3;
    const V3 w{tw[3], tw[4], tw[5]};
    const V3 rp{R[0] * x + R[1] * y, R[3] * x + R[4] * y, R[6] * x + R[7] * y};   // R (x, y, 0)
    const double dp[3] = {(R0[0] - R[0]) * x + (R0[1] - R[1]) * y,
                          (R0[3] - R[3]) * x + (R0[4] - R[4]) * y,
                          (R0[6] - R[6]) * x + (R0[7] - R[7]) * y};
    const V3 vp = cross(w, rp);
    const V3 f{k * ((ns[0] - ps[0]) + dp[0]) - b * (tw[0] + vp.x),
               k * ((ns[1] - ps[1]) + dp[1]) - b * (tw[1] + vp.y),
               k * ((ns[2] - ps[2]) + dp[2]) - b * (tw[2] + vp.z)};
    const V3 t = cross(rp, f);
    fo[0] = f.x; fo[1] = f.y; fo[2] = f.z;
    to[0] = t.x; to[1] = t.y; to[2] = t.z;
}

}  // namespace

blf_status launch_contact_eval(const double* prm, int shared, const double* twist,
                               const double* pose, const double* null_pose, int64_t batch,
                               double* wrench, double* autonomous, double* control,
                               double* regressor, hipStream_t s)
{
    if (batch == 0) return BLF_OK;
    hipLaunchKernelGGL(contact_eval_kernel, dim3((unsigned)ceil_div(batch, kCT)), dim3(kCT), 0, s,
                       prm, shared, twist, pose, null_pose, batch, wrench, autonomous, control,
                       regressor);
    return check_hip(hipGetLastError(), "contact_eval_kernel launch");
}

blf_status launch_contact_point(const double* prm, int shared, const double* twist,
                                const double* pose, const double* null_pose, int64_t batch,
                                const double* points, int32_t Q, double* force, double* torque,
                                hipStream_t s)
{
    const int64_t n = batch * (int64_t)Q;
    if (n == 0) return BLF_OK;
    hipLaunchKernelGGL(contact_point_kernel, dim3((unsigned)ceil_div(n, 256)), dim3(256), 0, s,
                       prm, shared, twist, pose, null_pose, batch, points, Q, force, torque);
    return check_hip(hipGetLastError(), "contact_point_kernel launch");
}

}  // namespace blf
