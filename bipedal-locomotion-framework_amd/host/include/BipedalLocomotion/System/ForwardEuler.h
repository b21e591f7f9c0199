/**
 * @file ForwardEuler.h
 * Drop-in for src/System/include/BipedalLocomotion/System/ForwardEuler.h:29-70 (+ .tpp:18-49).
 * x <- x + dx * dT per step, on the device.  The system type must provide the device hook
 *   bool forwardEulerIntegrate(double t0, double T, double dT);
 * (LinearTimeInvariantSystem does, through blf_lti_euler_integrate).  A system without a
 * device implementation does not compile with this integrator: the adapters never fall back to
 * host arithmetic on the path.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_SYSTEM_FORWARD_EULER_H
#define BLF_BIPEDAL_LOCOMOTION_SYSTEM_FORWARD_EULER_H

#include <BipedalLocomotion/System/FixedStepIntegrator.h>

namespace BipedalLocomotion
{
namespace System
{

template <typename DynamicalSystemDerived>
class ForwardEuler : public FixedStepIntegrator<DynamicalSystemDerived>
{
    bool integrateSchedule(double initialTime, double finalTime) final
    {
        if (!this->m_dynamicalSystem->forwardEulerIntegrate(initialTime, finalTime, this->m_dT))
        {
            std::cerr << "[ForwardEuler::oneStepIntegration] Unable to compute the system dynamics."
                      << std::endl;
            return false;
        }
        return true;
    }

public:
    explicit ForwardEuler(const double& dT) : FixedStepIntegrator<DynamicalSystemDerived>(dT) {}
};

} // namespace System
} // namespace BipedalLocomotion

#endif
