/**
 * @file ForwardEuler.h
 * Drop-in for src/System/include/BipedalLocomotion/System/ForwardEuler.h:29-70 (+ .tpp:18-49).
 * x <- x + dx * dT per step.
 *
 * A system with a device hook
 *   bool forwardEulerIntegrate(double t0, double T, double dT);
 * (LinearTimeInvariantSystem, FloatingBaseSystemKinematics, FloatingBaseDynamicalSystem and
 * user systems built on include/blf/forward_euler_device.h) integrates the whole schedule on the
 * device in one call; the library's own systems always take this path.
 *
 * A system without one is a user's host-side DynamicalSystem subclass: its dynamics() is CPU
 * code, so it cannot run on the device, and it is integrated by the reference's host loop
 * (ForwardEuler.tpp:18-49 over FixedStepIntegrator.tpp:48-64): dynamics(t, dx), then
 * x = getState() + dx * dT element by element (addArea, ForwardEuler.h:35-50), then setState(x).
 * The schedule (step count, stale last-step time) comes from blf_step_schedule, the same one the
 * device integrators use.  No library system ever reaches this loop.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_SYSTEM_FORWARD_EULER_H
#define BLF_BIPEDAL_LOCOMOTION_SYSTEM_FORWARD_EULER_H

#include <cstddef>
#include <tuple>
#include <type_traits>
#include <utility>

#include <BipedalLocomotion/System/FixedStepIntegrator.h>
#include <blf/blf_c.h>

namespace BipedalLocomotion
{
namespace System
{

namespace detail
{
template <class S, class = void> struct HasDeviceEuler : std::false_type
{
};
template <class S>
struct HasDeviceEuler<S, std::void_t<decltype(std::declval<S&>().forwardEulerIntegrate(
                             0.0, 0.0, 0.0))>> : std::true_type
{
};

// x += dx * dT as the element type defines it (Eigen-like types, scalars) ...
template <class X, class D, class = void> struct HasScaledAdd : std::false_type
{
};
template <class X, class D>
struct HasScaledAdd<X, D, std::void_t<decltype(std::declval<X&>() += std::declval<const D&>() * 1.0)>>
    : std::true_type
{
};
// ... or entry by entry for the adapters' blf::VectorXd (size(), operator[]) ...
template <class X, class = void> struct IsIndexable : std::false_type
{
};
template <class X>
struct IsIndexable<X, std::void_t<decltype(std::declval<X&>().size()),
                                  decltype(std::declval<X&>()[std::size_t{0}])>> : std::true_type
{
};
// ... or blf::MatrixXd / blf::Matrix3 style (rows(), cols(), operator()(i, j)).
template <class X, class = void> struct IsMatrixLike : std::false_type
{
};
template <class X>
struct IsMatrixLike<X, std::void_t<decltype(std::declval<X&>().rows()), decltype(std::declval<X&>().cols()),
                                   decltype(std::declval<X&>()(std::size_t{0}, std::size_t{0}))>>
    : std::true_type
{
};

template <class X, class D> bool addScaled(X& x, const D& dx, double dT)
{
    if constexpr (HasScaledAdd<X, D>::value)
    {
        x += dx * dT;
        return true;
    } else if constexpr (IsIndexable<X>::value)
    {
        if (x.size() != dx.size()) return false;
        for (std::size_t i = 0; i < x.size(); ++i) x[i] = x[i] + dx[i] * dT;
        return true;
    } else if constexpr (IsMatrixLike<X>::value)
    {
        if (x.rows() != dx.rows() || x.cols() != dx.cols()) return false;
        for (std::size_t i = 0; i < std::size_t(x.rows()); ++i)
            for (std::size_t j = 0; j < std::size_t(x.cols()); ++j)
                x(i, j) = x(i, j) + dx(i, j) * dT;
        return true;
    } else
    {
        static_assert(HasScaledAdd<X, D>::value,
                      "ForwardEuler: the state element type needs x += dx * dT, size()/operator[] "
                      "or rows()/cols()/operator()(i, j)");
        return false;
    }
}

template <std::size_t I = 0, class... Tx, class... Td>
bool addArea(const std::tuple<Td...>& dx, double dT, std::tuple<Tx...>& x)
{
    static_assert(sizeof...(Tx) == sizeof...(Td),
                  "ForwardEuler: the state and its derivative must have the same number of elements");
    if constexpr (I == sizeof...(Tx))
        return true;
    else
        return addScaled(std::get<I>(x), std::get<I>(dx), dT) && addArea<I + 1>(dx, dT, x);
}
} // namespace detail

template <typename DynamicalSystemDerived>
class ForwardEuler : public FixedStepIntegrator<DynamicalSystemDerived>
{
    typename DynamicalSystemDerived::StateDerivativeType m_computationalBufferStateDerivative;
    typename DynamicalSystemDerived::StateType m_computationalBufferState;

    /** ForwardEuler.tpp:18-49, for a host-side system. */
    bool oneStepIntegration(double t0, double dT)
    {
        if (!this->m_dynamicalSystem->dynamics(t0, m_computationalBufferStateDerivative))
        {
            std::cerr << "[ForwardEuler::oneStepIntegration] Unable to compute the system dynamics."
                      << std::endl;
            return false;
        }
        m_computationalBufferState = this->m_dynamicalSystem->getState();
        if (!detail::addArea(m_computationalBufferStateDerivative, dT, m_computationalBufferState))
        {
            std::cerr << "[ForwardEuler::oneStepIntegration] The state and its derivative have "
                         "different sizes."
                      << std::endl;
            return false;
        }
        if (!this->m_dynamicalSystem->setState(m_computationalBufferState))
        {
            std::cerr << "[ForwardEuler::oneStepIntegration] Unable to set the new state in the "
                         "dynamical system."
                      << std::endl;
            return false;
        }
        return true;
    }

    bool integrateSchedule(double initialTime, double finalTime) final
    {
        if constexpr (detail::HasDeviceEuler<DynamicalSystemDerived>::value)
        {
            if (!this->m_dynamicalSystem->forwardEulerIntegrate(initialTime, finalTime, this->m_dT))
            {
                std::cerr << "[ForwardEuler::oneStepIntegration] Unable to compute the system "
                             "dynamics."
                          << std::endl;
                return false;
            }
            return true;
        } else
        {
            // FixedStepIntegrator.tpp:48-64 over the shared schedule.
            int32_t iterations = 0;
            double dTLast = 0.0, tLast = 0.0;
            if (blf_step_schedule(initialTime, finalTime, this->m_dT, &iterations, &dTLast, &tLast)
                != BLF_OK)
            {
                std::cerr << "[FixedStepIntegrator::integrate] Invalid integration interval."
                          << std::endl;
                return false;
            }
            for (int32_t i = 0; i + 1 < iterations; ++i)
            {
                const double currentTime = initialTime + this->m_dT * static_cast<double>(i);
                if (!oneStepIntegration(currentTime, this->m_dT))
                {
                    std::cerr << "[FixedStepIntegrator::integrate] Error while integrating at time: "
                              << currentTime << "." << std::endl;
                    return false;
                }
            }
            if (!oneStepIntegration(tLast, dTLast))
            {
                std::cerr << "[FixedStepIntegrator::integrate] Error while integrating the last "
                             "step."
                          << std::endl;
                return false;
            }
            return true;
        }
    }

public:
    explicit ForwardEuler(const double& dT) : FixedStepIntegrator<DynamicalSystemDerived>(dT) {}
};

} // namespace System
} // namespace BipedalLocomotion

#endif
