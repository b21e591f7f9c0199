/**
 * @file LinearTimeInvariantSystem.h
 * Drop-in for src/System/include/BipedalLocomotion/System/LinearTimeInvariantSystem.h:35-69
 * (src/System/src/LinearTimeInvariantSystem.cpp:13-74): dx = A x + B u.  The matrices, state and
 * input are mirrored to device memory; dynamics() runs blf_lti_dynamics and ForwardEuler runs
 * blf_lti_euler_integrate (any n, m >= 1).
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_SYSTEM_LTI_H
#define BLF_BIPEDAL_LOCOMOTION_SYSTEM_LTI_H

#include <tuple>

#include <BipedalLocomotion/System/DynamicalSystem.h>
#include <blf/dense.h>
#include <blf/device.h>

namespace BipedalLocomotion
{
namespace System
{

class LinearTimeInvariantSystem
    : public DynamicalSystem<std::tuple<blf::VectorXd>, std::tuple<blf::VectorXd>,
                             std::tuple<blf::VectorXd>>
{
    blf::MatrixXd m_A;
    blf::MatrixXd m_B;
    bool m_isInitialized{false};
    blf::DeviceBuffer<double> m_dA, m_dB, m_dx, m_du, m_ddx;

    bool checkSizes(const char* where) const;

public:
    /** Set A (n x n) and B (n x m).  Any matrix type with rows(), cols(), operator()(i, j). */
    template <class MatA, class MatB> bool setSystemMatrices(const MatA& A, const MatB& B)
    {
        return setSystemMatrices(blf::MatrixXd::from(A), blf::MatrixXd::from(B));
    }
    bool setSystemMatrices(const blf::MatrixXd& A, const blf::MatrixXd& B);

    bool dynamics(const double& time, StateDerivativeType& stateDerivative) final;

    /** Device hook used by ForwardEuler<LinearTimeInvariantSystem>. */
    bool forwardEulerIntegrate(double initialTime, double finalTime, double dT);
};

} // namespace System
} // namespace BipedalLocomotion

#endif
