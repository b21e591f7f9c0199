// Diagnostic (not the product): the SURVEY.md section 7 step-6 ablation the round-1 verdict asked
// for.  One LQ step of the DCM-MPC QP (the unconstrained Newton step: a Riccati sweep, then the
// backward costate and forward rollout scans; the core of every active-set pass) for B problems,
// two ways:
//   wave: one wavefront per QP, knot pairs per lane, Kogge-Stone scans (the product's
//         as_lq_step<2, double> from csrc/dcm_mpc_as.hip, included below);
//   lane: one lane per QP, sequential recursions over the knots, the per-knot Riccati and solve
//         state in a [knot][field][qp] global scratch (consecutive lanes on consecutive QPs, so
//         every access is coalesced).
// Both solve the same step from the same inputs (they agree to rounding, checked on the host).
//   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -I include -I <pkg>/csrc tools/ablation_lane_per_qp.hip
#include "../bipedal-locomotion-framework_amd/csrc/dcm_mpc_as.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace blf {
namespace {

__global__ __launch_bounds__(kWave, 2) void lq_wave_kernel(KParams P, const double* __restrict__ xi_init,
                                                           const double* __restrict__ omega,
                                                           const double* __restrict__ xi_ref,
                                                           const double* __restrict__ vrp_ref,
                                                           double* __restrict__ vrp_out)
{
    constexpr int KPL = 2;
    const int N = P.N;
    const int lane = threadIdx.x;
    const int64_t p = blockIdx.x;
    const PT<double> Pd = params_d(P);
    AKnot K[KPL];
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const int k = KPL * lane + j;
        AKnot& Kj = K[j];
        Kj.m = Kj.gm = Kj.drop = Kj.add = 0;
        Kj.r0 = Kj.r1 = Kj.x0 = Kj.x1 = Kj.w = Kj.be = 0.0;
        Kj.rh0 = Kj.rh1 = Kj.d0 = Kj.d1 = Kj.qx0 = Kj.qx1 = 0.0;
        Kj.P00 = Kj.P01 = Kj.P11 = Kj.h00 = Kj.h01 = Kj.h11 = 0.0;
        Kj.rr0 = Kj.rr1 = Kj.xr0 = Kj.xr1 = 0.0;
        if (k < N) {
            const int64_t st = p * N + k;
            Kj.w = omega[st];
            Kj.be = Pd.dt * Kj.w;
            Kj.rr0 = vrp_ref[2 * st];
            Kj.rr1 = vrp_ref[2 * st + 1];
            const int64_t sx = p * (N + 1) + (k + 1);
            Kj.xr0 = xi_ref[2 * sx];
            Kj.xr1 = xi_ref[2 * sx + 1];
            Kj.r0 = Kj.rr0; Kj.r1 = Kj.rr1;
            Kj.x0 = Kj.xr0; Kj.x1 = Kj.xr1;
        }
        Kj.al = 1.0 + Kj.be;
    }
    as_lq_step<KPL, double>(K, Pd, N, lane, xi_init[2 * p], xi_init[2 * p + 1]);
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const int k = KPL * lane + j;
        if (k < N) {
            vrp_out[2 * (p * N + k)] = K[j].r0;
            vrp_out[2 * (p * N + k) + 1] = K[j].r1;
        }
    }
}

// Scratch [N][F][B]: F = 8 doubles per knot (P_{k+1} 3, h 3, v_{k+1} 2).
constexpr int F = 8;

__global__ __launch_bounds__(256) void lq_lane_kernel(KParams P, const double* __restrict__ xi_init,
                                                      const double* __restrict__ omega,
                                                      const double* __restrict__ xi_ref,
                                                      const double* __restrict__ vrp_ref,
                                                      double* __restrict__ scratch, double* __restrict__ vrp_out,
                                                      int64_t B)
{
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= B) return;
    const int N = P.N;
    auto S = [&](int k, int f) -> double& { return scratch[((int64_t)k * F + f) * B + q]; };
    // inputs are problem-major; the lane reads its own rows (the Riccati needs only omega)
    // ---- backward Riccati sweep P_k = f_k(P_{k+1}), h_k = (R + b2 P_{k+1})^-1 ----
    double Pn0 = P.Pw0, Pn1 = 0.0, Pn2 = P.Pw1;
    for (int k = N - 1; k >= 0; --k) {
        const double w = omega[q * N + k];
        const double be = P.dt * w, al = 1.0 + be, b2 = be * be;
        S(k, 0) = Pn0; S(k, 1) = Pn1; S(k, 2) = Pn2;
        const double B00 = fma(b2, Pn0, P.Rw0), B01 = b2 * Pn1, B11 = fma(b2, Pn2, P.Rw1);
        const double idet = 1.0 / fma(B00, B11, -(B01 * B01));
        S(k, 3) = B11 * idet; S(k, 4) = -(B01 * idet); S(k, 5) = B00 * idet;
        if (k == 0) break;
        const double detRW = P.Rw0 * P.Rw1, ie = b2 / detRW;
        RcT<double> e;
        e.a0 = al; e.a1 = 0.0; e.a2 = 0.0; e.a3 = al;
        e.g0 = P.Rw1 * ie; e.g1 = 0.0; e.g2 = P.Rw0 * ie;
        e.h0 = P.Qw0; e.h1 = 0.0; e.h2 = P.Qw1;
        double o0, o1, o2;
        rc_apply(e, Pn0, Pn1, Pn2, o0, o1, o2);
        Pn0 = o0; Pn1 = o1; Pn2 = o2;
    }
    // ---- residuals at (xi_ref, vrp_ref) and the backward costate scan v_k = G_k v_{k+1} + c_k ----
    double v0 = 0.0, v1 = 0.0;
    for (int k = N - 1; k >= 0; --k) {
        const double w = omega[q * N + k], be = P.dt * w, al = 1.0 + be, b2 = be * be, ab = al * be;
        const double r0 = vrp_ref[2 * (q * N + k)], r1 = vrp_ref[2 * (q * N + k) + 1];
        const double xk0 = k == 0 ? xi_init[2 * q] : xi_ref[2 * (q * (N + 1) + k)];
        const double xk1 = k == 0 ? xi_init[2 * q + 1] : xi_ref[2 * (q * (N + 1) + k) + 1];
        const double y0_ = xi_ref[2 * (q * (N + 1) + k + 1)], y1_ = xi_ref[2 * (q * (N + 1) + k + 1) + 1];
        const double d0 = fma(FD2(w, xk0, -w, r0), P.dt, xk0) - y0_;
        const double d1 = fma(FD2(w, xk1, -w, r1), P.dt, xk1) - y1_;
        const double P00 = S(k, 0), P01 = S(k, 1), P11 = S(k, 2), h00 = S(k, 3), h01 = S(k, 4), h11 = S(k, 5);
        const double m00 = FD2(P00, h00, P01, h01), m01 = FD2(P00, h01, P01, h11);
        const double m10 = FD2(P01, h00, P11, h01), m11 = FD2(P01, h01, P11, h11);
        const double y0 = FD3(P00, d0, P01, d1, 0.0), y1 = FD3(P01, d0, P11, d1, 0.0);   // q_k = 0 at xi_ref
        const double G0 = al * fma(-b2, m00, 1.0), G1 = -(al * (b2 * m01));
        const double G2 = -(al * (b2 * m10)), G3 = al * fma(-b2, m11, 1.0);
        S(k, 6) = v0; S(k, 7) = v1;   // v_{k+1}
        const double c0 = FD3(G0, y0, G1, y1, 0.0), c1 = FD3(G2, y0, G3, y1, 0.0);   // g_k = 0 at vrp_ref
        const double n0 = FD3(G0, v0, G1, v1, c0), n1 = FD3(G2, v0, G3, v1, c1);
        v0 = n0; v1 = n1;
        (void)ab;
    }
    // ---- forward rollout of the step dxi_{k+1} = G_k^T dxi_k + f_k, dr_k ----
    double x0 = 0.0, x1 = 0.0;
    for (int k = 0; k < N; ++k) {
        const double w = omega[q * N + k], be = P.dt * w, al = 1.0 + be, b2 = be * be, ab = al * be;
        const double r0 = vrp_ref[2 * (q * N + k)], r1 = vrp_ref[2 * (q * N + k) + 1];
        const double xk0 = k == 0 ? xi_init[2 * q] : xi_ref[2 * (q * (N + 1) + k)];
        const double xk1 = k == 0 ? xi_init[2 * q + 1] : xi_ref[2 * (q * (N + 1) + k) + 1];
        const double y0_ = xi_ref[2 * (q * (N + 1) + k + 1)], y1_ = xi_ref[2 * (q * (N + 1) + k + 1) + 1];
        const double d0 = fma(FD2(w, xk0, -w, r0), P.dt, xk0) - y0_;
        const double d1 = fma(FD2(w, xk1, -w, r1), P.dt, xk1) - y1_;
        const double P00 = S(k, 0), P01 = S(k, 1), P11 = S(k, 2), h00 = S(k, 3), h01 = S(k, 4), h11 = S(k, 5);
        const double vn0 = S(k, 6), vn1 = S(k, 7);
        const double m00 = FD2(P00, h00, P01, h01), m01 = FD2(P00, h01, P01, h11);
        const double m10 = FD2(P01, h00, P11, h01), m11 = FD2(P01, h01, P11, h11);
        const double t0 = FD3(P00, d0, P01, d1, 0.0) + vn0, t1 = FD3(P01, d0, P11, d1, 0.0) + vn1;
        const double k0 = -FD2(h00, -be * t0, h01, -be * t1), k1 = -FD2(h01, -be * t0, h11, -be * t1);
        const double G0 = al * fma(-b2, m00, 1.0), G1 = -(al * (b2 * m01));
        const double G2 = -(al * (b2 * m10)), G3 = al * fma(-b2, m11, 1.0);
        const double dr0 = fma(ab, FD2(m00, x0, m10, x1), k0), dr1 = fma(ab, FD2(m01, x0, m11, x1), k1);
        vrp_out[2 * (q * N + k)] = r0 + dr0;
        vrp_out[2 * (q * N + k) + 1] = r1 + dr1;
        const double f0 = fma(-be, k0, d0), f1 = fma(-be, k1, d1);
        const double n0 = FD3(G0, x0, G2, x1, f0), n1 = FD3(G1, x0, G3, x1, f1);
        x0 = n0; x1 = n1;
    }
}

}  // namespace
}  // namespace blf

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main(int argc, char** argv)
{
    using namespace blf;
    const int N = 100;
    for (int64_t B : {(int64_t)4096, (int64_t)65536}) {
        std::vector<double> xi0(2 * B), om(B * N), xr(2 * B * (N + 1)), rr(2 * B * N);
        srand(1);
        auto U = [] { return rand() / (double)RAND_MAX; };
        for (auto& v : xi0) v = 0.05 * U();
        for (auto& v : om) v = 3.0 + 0.5 * U();
        for (auto& v : xr) v = 0.3 * U();
        for (auto& v : rr) v = 0.3 * U();
        double *d_xi0, *d_om, *d_xr, *d_rr, *d_a, *d_b, *d_s;
        CK(hipMalloc(&d_xi0, 8 * xi0.size())); CK(hipMalloc(&d_om, 8 * om.size()));
        CK(hipMalloc(&d_xr, 8 * xr.size())); CK(hipMalloc(&d_rr, 8 * rr.size()));
        CK(hipMalloc(&d_a, 8 * rr.size())); CK(hipMalloc(&d_b, 8 * rr.size()));
        CK(hipMalloc(&d_s, 8 * (size_t)N * F * B));
        CK(hipMemcpy(d_xi0, xi0.data(), 8 * xi0.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(d_om, om.data(), 8 * om.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(d_xr, xr.data(), 8 * xr.size(), hipMemcpyHostToDevice));
        CK(hipMemcpy(d_rr, rr.data(), 8 * rr.size(), hipMemcpyHostToDevice));
        KParams P{};
        P.N = N; P.M = 8; P.dt = 0.02; P.Qw0 = P.Qw1 = 1e2; P.Rw0 = P.Rw1 = 1.0; P.Pw0 = P.Pw1 = 1e3;
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        const int reps = 20;
        auto run_wave = [&] { hipLaunchKernelGGL(lq_wave_kernel, dim3((unsigned)B), dim3(kWave), 0, 0, P, d_xi0, d_om, d_xr, d_rr, d_a); };
        auto run_lane = [&] { hipLaunchKernelGGL(lq_lane_kernel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, 0, P, d_xi0, d_om, d_xr, d_rr, d_s, d_b, B); };
        float ms_w = 0, ms_l = 0;
        run_wave(); run_lane(); CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0)); for (int i = 0; i < reps; ++i) run_wave(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms_w, e0, e1));
        CK(hipEventRecord(e0)); for (int i = 0; i < reps; ++i) run_lane(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms_l, e0, e1));
        std::vector<double> a(rr.size()), b(rr.size());
        CK(hipMemcpy(a.data(), d_a, 8 * a.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), d_b, 8 * b.size(), hipMemcpyDeviceToHost));
        double diff = 0, mag = 0;
        for (size_t i = 0; i < a.size(); ++i) { diff = fmax(diff, fabs(a[i] - b[i])); mag = fmax(mag, fabs(a[i])); }
        printf("{\"B\": %lld, \"N\": %d, \"wave_per_qp_ms\": %.4f, \"lane_per_qp_ms\": %.4f, \"scratch_bytes\": %lld, "
               "\"max_abs_diff\": %.3e, \"max_abs\": %.3e}\n", (long long)B, N, ms_w / reps, ms_l / reps,
               (long long)(8LL * N * F * B), diff, mag);
        for (double* ptr : {d_xi0, d_om, d_xr, d_rr, d_a, d_b, d_s}) CK(hipFree(ptr));
    }
    return 0;
}
