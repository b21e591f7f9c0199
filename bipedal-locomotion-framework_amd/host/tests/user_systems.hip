// user_systems.hip — TEST INFRASTRUCTURE: user dynamical systems integrated on the device through
// include/blf/forward_euler_device.h (ForwardEuler<UserSystem>, the reference's
// DynamicalSystem::dynamics override, DynamicalSystem.h:98, ForwardEuler.tpp:18-49), exported for
// tests/test_gpu_user_systems.py:
//   * UserLti<N, M>: LinearTimeInvariantSystem restated as a user system, in the arithmetic order of
//     blf_lti_euler_integrate, so the two agree bit for bit;
//   * ForcedOscillator: a time-varying nonlinear system (forcing u t^2, a cubic spring), checked
//     against a plain-Python restatement of the reference schedule.
// Built with -ffp-contract=off, as the library.
#include <blf/forward_euler_device.h>

namespace {

template <int N, int M>
struct UserLti {
    static constexpr int kStateSize = N;
    static constexpr int kInputSize = M;
    struct Params {
        double A[N * N], B[N * M];
    };
    __device__ static void dynamics(double /*t*/, const double* x, const double* u, const Params& p, double* dx)
    {
        for (int r = 0; r < N; ++r) {
            double bu = p.B[r * M] * u[0];
            for (int c = 1; c < M; ++c) bu = bu + p.B[r * M + c] * u[c];
            double acc = p.A[r * N] * x[0];
            for (int c = 1; c < N; ++c) acc = acc + p.A[r * N + c] * x[c];
            dx[r] = acc + bu;
        }
    }
};

struct ForcedOscillator {
    static constexpr int kStateSize = 2;   // q, v
    static constexpr int kInputSize = 1;   // forcing amplitude
    struct Params {
        double k, c, k3;
    };
    __device__ static void dynamics(double t, const double* x, const double* u, const Params& p, double* dx)
    {
        dx[0] = x[1];
        dx[1] = ((u[0] * (t * t) - p.k * x[0]) - p.c * x[1]) - p.k3 * (x[0] * x[0] * x[0]);
    }
};

}  // namespace

extern "C" {

blf_status blf_test_user_lti3x2(const double* params, int32_t shared, const double* u, double* x, int64_t batch,
                                double t0, double T, double dT, void* stream)
{
    using S = UserLti<3, 2>;
    return blf::forward_euler_integrate<S>(reinterpret_cast<const S::Params*>(params), shared, u, x, batch, t0, T,
                                           dT, (hipStream_t)stream);
}

blf_status blf_test_user_lti8x8(const double* params, int32_t shared, const double* u, double* x, int64_t batch,
                                double t0, double T, double dT, void* stream)
{
    using S = UserLti<8, 8>;
    return blf::forward_euler_integrate<S>(reinterpret_cast<const S::Params*>(params), shared, u, x, batch, t0, T,
                                           dT, (hipStream_t)stream);
}

blf_status blf_test_user_forced_oscillator(const double* params, int32_t shared, const double* u, double* x,
                                           int64_t batch, double t0, double T, double dT, void* stream)
{
    using S = ForcedOscillator;
    return blf::forward_euler_integrate<S>(reinterpret_cast<const S::Params*>(params), shared, u, x, batch, t0, T,
                                           dT, (hipStream_t)stream);
}

}  // extern "C"
