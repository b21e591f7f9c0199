/**
 * @file FloatingBaseSystemKinematics.h
 * Drop-in for src/System/include/BipedalLocomotion/System/FloatingBaseSystemKinematics.h:25-74
 * (src/System/src/FloatingBaseSystemKinematics.cpp:13-73):
 *   state  (base position p, base rotation R, joint positions s),
 *   input  (base twist in mixed representation, joint velocities s_dot),
 *   dp = v,  dR = -R.colwise().cross(w) + rho/2 ((R R^T)^{-1} - I) R,  ds = s_dot.
 * dynamics() runs blf_fbk_dynamics and ForwardEuler runs blf_fbk_euler_integrate (include/blf/
 * blf_c.h); the Baumgarte parameter comes from the key "rho" (default 0.01), read by the
 * reference-spelled initalize().
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_SYSTEM_FLOATING_BASE_SYSTEM_KINEMATICS_H
#define BLF_BIPEDAL_LOCOMOTION_SYSTEM_FLOATING_BASE_SYSTEM_KINEMATICS_H

#include <tuple>

#include <BipedalLocomotion/System/DynamicalSystem.h>
#include <blf/dense.h>
#include <blf/device.h>
#include <blf/spatial.h>

namespace BipedalLocomotion
{
namespace System
{

class FloatingBaseSystemKinematics
    : public DynamicalSystem<std::tuple<blf::Vector3, blf::Matrix3, blf::VectorXd>,
                             std::tuple<blf::Vector3, blf::Matrix3, blf::VectorXd>,
                             std::tuple<blf::Vector6, blf::VectorXd>>
{
    double m_rho{0.01}; /**< Baumgarte stabilization over SO(3) */
    blf::DeviceBuffer<double> m_dState, m_dInput, m_dOut;

    bool checkSizes(const char* where) const;
    bool uploadState();

public:
    bool initalize(std::weak_ptr<ParametersHandler::IParametersHandler> handler) final;
    bool dynamics(const double& time, StateDerivativeType& stateDerivative) final;

    /** Device hook used by ForwardEuler<FloatingBaseSystemKinematics>. */
    bool forwardEulerIntegrate(double initialTime, double finalTime, double dT);
};

} // namespace System
} // namespace BipedalLocomotion

#endif
