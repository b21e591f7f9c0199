/**
 * @file FixedStepIntegrator.h
 * Drop-in for src/System/include/BipedalLocomotion/System/FixedStepIntegrator.h:26-62 and
 * FixedStepIntegrator.tpp:21-72.  integrate(t0, T) validates its arguments exactly like the
 * reference (same messages, same `false` returns) and then hands the whole fixed-step schedule to
 * the system's device integrator in ONE call: the step count iters = ceil((T - t0)/dT) and the
 * stale-time final step (see include/blf/blf_c.h, blf_lti_euler_integrate) are reproduced
 * inside the C ABI, bit for bit.  integrate(t, t), which never returns in the reference
 * (size_t vs -1 at FixedStepIntegrator.tpp:99), is refused with an error instead.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_SYSTEM_FIXED_STEP_INTEGRATOR_H
#define BLF_BIPEDAL_LOCOMOTION_SYSTEM_FIXED_STEP_INTEGRATOR_H

#include <iostream>

#include <BipedalLocomotion/System/Integrator.h>

namespace BipedalLocomotion
{
namespace System
{

template <typename DynamicalSystemDerived>
class FixedStepIntegrator : public Integrator<DynamicalSystemDerived>
{
protected:
    double m_dT{0.0};

    /** Integrate the whole schedule on the device (implemented by each method). */
    virtual bool integrateSchedule(double initialTime, double finalTime) = 0;

public:
    explicit FixedStepIntegrator(const double& dT) : m_dT{dT} {}

    bool integrate(double initialTime, double finalTime) final
    {
        if (this->m_dynamicalSystem == nullptr)
        {
            std::cerr << "[FixedStepIntegrator::integrate] Please set the dynamical system before "
                         "call this function."
                      << std::endl;
            return false;
        }
        if (initialTime > finalTime)
        {
            std::cerr << "[FixedStepIntegrator::integrate] The final time has to be greater than "
                         "the initial one."
                      << std::endl;
            return false;
        }
        if (m_dT <= 0)
        {
            std::cerr << "[FixedStepIntegrator::integrate] The sampling time must be a strictly "
                         "positive number."
                      << std::endl;
            return false;
        }
        return integrateSchedule(initialTime, finalTime);
    }
};

} // namespace System
} // namespace BipedalLocomotion

#endif
