/**
 * @file Integrator.h
 * Drop-in for src/System/include/BipedalLocomotion/System/Integrator.h:28-74 (+ .tpp:18-54):
 * the dynamical system can be set once; getSolution() aliases the system's state.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_SYSTEM_INTEGRATOR_H
#define BLF_BIPEDAL_LOCOMOTION_SYSTEM_INTEGRATOR_H

#include <iostream>
#include <memory>

#include <BipedalLocomotion/System/DynamicalSystem.h>

namespace BipedalLocomotion
{
namespace System
{

template <typename DynamicalSystemDerived> class Integrator
{
protected:
    std::shared_ptr<DynamicalSystemDerived> m_dynamicalSystem;

public:
    bool setDynamicalSystem(std::shared_ptr<DynamicalSystemDerived> dynamicalSystem)
    {
        if (m_dynamicalSystem != nullptr)
        {
            std::cerr << "[Integrator::setDynamicalSystem] The dynamical system has been already "
                         "set."
                      << std::endl;
            return false;
        }
        if (dynamicalSystem == nullptr)
        {
            std::cerr << "[Integrator::setDynamicalSystem] The dynamical system passed to the "
                         "function is corrupted."
                      << std::endl;
            return false;
        }
        m_dynamicalSystem = dynamicalSystem;
        return true;
    }

    const std::weak_ptr<DynamicalSystemDerived> dynamicalSystem() const { return m_dynamicalSystem; }

    const typename DynamicalSystemDerived::StateType& getSolution() const
    {
        return m_dynamicalSystem->getState();
    }

    virtual bool integrate(double initialTime, double finalTime) = 0;
    virtual ~Integrator() = default;
};

} // namespace System
} // namespace BipedalLocomotion

#endif
