/**
 * @file LinearTimeInvariantSystem.cpp
 * Argument checks and messages follow src/System/src/LinearTimeInvariantSystem.cpp:13-74; the
 * arithmetic runs on the device through the C ABI.
 */
#include <iostream>

#include <BipedalLocomotion/System/LinearTimeInvariantSystem.h>

using namespace BipedalLocomotion::System;

bool LinearTimeInvariantSystem::setSystemMatrices(const blf::MatrixXd& A, const blf::MatrixXd& B)
{
    if (A.rows() != B.rows())
    {
        std::cerr << "[LinearTimeInvariantSystem::setSystemMatrices] A and B must have the same "
                     "number of rows."
                  << std::endl;
        return false;
    }
    if (A.rows() != A.cols())
    {
        std::cerr << "[LinearTimeInvariantSystem::setSystemMatrices] The A matrix has to be a "
                     "square matrix."
                  << std::endl;
        return false;
    }
    m_A = A;
    m_B = B;
    // Any size, as the reference.  An input-free system (B with no columns) runs with one zero
    // column and a zero input: Eigen's B u is then a zero vector too, so dx = A x + 0 either way.
    // An empty system (n = 0) has nothing on the device.
    const std::size_t n = m_A.rows();
    if (n > 0)
    {
        const blf::VectorXd zero(n, 0.0);
        if (!m_dA.upload(m_A.data(), n * n) ||
            !(m_B.cols() > 0 ? m_dB.upload(m_B.data(), n * m_B.cols()) : m_dB.upload(zero.data(), n)))
            return false;
    }
    m_isInitialized = true;
    return true;
}

bool LinearTimeInvariantSystem::checkSizes(const char* where) const
{
    if (!m_isInitialized)
    {
        std::cerr << "[" << where << "] Please initialize the matrices." << std::endl;
        return false;
    }
    if (std::get<0>(m_state).size() != m_A.rows())
    {
        std::cerr << "[" << where << "] The size of the vector 'state' is not coherent with the "
                     "system matrices."
                  << std::endl;
        return false;
    }
    if (std::get<0>(m_controlInput).size() != m_B.cols())
    {
        std::cerr << "[" << where << "] The size of the vector 'control input' is not coherent "
                     "with the system matrices."
                  << std::endl;
        return false;
    }
    return true;
}

bool LinearTimeInvariantSystem::dynamics(const double& time, StateDerivativeType& stateDerivative)
{
    (void)time;
    if (!checkSizes("LinearTimeInvariantSystem::dynamics")) return false;
    const blf::VectorXd& x = std::get<0>(m_state);
    const blf::VectorXd& u = std::get<0>(m_controlInput);
    const int n = static_cast<int>(m_A.rows()), m = static_cast<int>(m_B.cols());
    blf::VectorXd& dx = std::get<0>(stateDerivative);
    dx.resize(n);
    if (n == 0) return true;
    blf_handle* h = blf::threadHandle();
    if (h == nullptr) return false;
    const double zero = 0.0;
    if (!m_dx.upload(x.data(), n) || !m_du.upload(m > 0 ? u.data() : &zero, m > 0 ? m : 1) ||
        !m_ddx.resize(n))
        return false;
    if (!blf::report(blf_lti_dynamics(h, n, m > 0 ? m : 1, m_dA.data(), m_dB.data(), 1,
                                      m_du.data(), m_dx.data(), m_ddx.data(), 1, nullptr),
                     "LinearTimeInvariantSystem::dynamics"))
        return false;
    return m_ddx.download(dx.data(), n);
}

bool LinearTimeInvariantSystem::forwardEulerIntegrate(double initialTime, double finalTime, double dT)
{
    if (!checkSizes("LinearTimeInvariantSystem::dynamics")) return false;
    blf::VectorXd& x = std::get<0>(m_state);
    const blf::VectorXd& u = std::get<0>(m_controlInput);
    const int n = static_cast<int>(m_A.rows()), m = static_cast<int>(m_B.cols());
    if (n == 0)   // nothing to integrate; the schedule's argument checks still apply
    {
        int32_t it = 0;
        double dTl = 0.0, tl = 0.0;
        return blf::report(blf_step_schedule(initialTime, finalTime, dT, &it, &dTl, &tl),
                           "FixedStepIntegrator::integrate");
    }
    blf_handle* h = blf::threadHandle();
    if (h == nullptr) return false;
    const double zero = 0.0;
    if (!m_dx.upload(x.data(), n) || !m_du.upload(m > 0 ? u.data() : &zero, m > 0 ? m : 1))
        return false;
    if (!blf::report(blf_lti_euler_integrate(h, n, m > 0 ? m : 1, m_dA.data(), m_dB.data(), 1, m_du.data(),
                                             m_dx.data(), 1, initialTime, finalTime, dT, nullptr),
                     "FixedStepIntegrator::integrate"))
        return false;
    return m_dx.download(x.data(), n);
}
