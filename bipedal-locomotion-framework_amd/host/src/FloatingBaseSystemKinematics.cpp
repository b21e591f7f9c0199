/**
 * @file FloatingBaseSystemKinematics.cpp
 * Messages and checks follow src/System/src/FloatingBaseSystemKinematics.cpp:13-73; the
 * arithmetic runs on the device through the C ABI.
 */
#include <iostream>

#include <BipedalLocomotion/System/FloatingBaseSystemKinematics.h>

using namespace BipedalLocomotion::System;
using namespace BipedalLocomotion::ParametersHandler;

bool FloatingBaseSystemKinematics::initalize(std::weak_ptr<IParametersHandler> handler)
{
    auto ptr = handler.lock();
    if (ptr == nullptr)
    {
        std::cerr << "[FloatingBaseSystemKinematics::initalize] The parameter handler is expired. "
                     "Please call the function passing a pointer pointing an already allocated "
                     "memory."
                  << std::endl;
        return false;
    }
    if (!ptr->getParameter("rho", m_rho))
    {
        std::cerr << "[FloatingBaseSystemKinematics::initalize] Unable to load the Baumgarte "
                     "stabilization parameter."
                  << std::endl;
        return false;
    }
    return true;
}

bool FloatingBaseSystemKinematics::checkSizes(const char* where) const
{
    const std::size_t n = std::get<2>(m_state).size();
    if (std::get<1>(m_controlInput).size() != n)
    {
        std::cerr << "[" << where << "] Wrong size of the vectors." << std::endl;
        return false;
    }
    if (n > BLF_FBK_MAX_DOFS)
    {
        std::cerr << "[" << where << "] The device kernels support up to " << BLF_FBK_MAX_DOFS
                  << " joints." << std::endl;
        return false;
    }
    return true;
}

// device layout: state = p 3 | R 9 | s n ; input = twist 6 | s_dot n
bool FloatingBaseSystemKinematics::uploadState()
{
    const auto& [p, R, s] = m_state;
    const auto& [twist, sd] = m_controlInput;
    const std::size_t n = s.size();
    std::vector<double> st(12 + n), in(6 + n);
    for (int i = 0; i < 3; ++i) st[i] = p[i];
    for (int i = 0; i < 9; ++i) st[3 + i] = R[i];
    for (std::size_t i = 0; i < n; ++i) st[12 + i] = s[i];
    for (int i = 0; i < 6; ++i) in[i] = twist[i];
    for (std::size_t i = 0; i < n; ++i) in[6 + i] = sd[i];
    return m_dState.upload(st) && m_dInput.upload(in);
}

bool FloatingBaseSystemKinematics::dynamics(const double& time, StateDerivativeType& stateDerivative)
{
    (void)time;
    if (!checkSizes("FloatingBaseSystemKinematics::dynamics")) return false;
    const int n = static_cast<int>(std::get<2>(m_state).size());
    blf_handle* h = blf::threadHandle();
    if (h == nullptr || !uploadState() || !m_dOut.resize(12 + n)) return false;
    double* o = m_dOut.data();
    if (!blf::report(blf_fbk_dynamics(h, n, m_rho, m_dState.data() + 3, m_dInput.data(),
                                      m_dInput.data() + 6, o, o + 3, o + 12, 1, nullptr),
                     "FloatingBaseSystemKinematics::dynamics"))
        return false;
    std::vector<double> host(12 + n);
    if (!m_dOut.download(host.data(), 12 + n)) return false;
    auto& [dp, dR, ds] = stateDerivative;
    for (int i = 0; i < 3; ++i) dp[i] = host[i];
    for (int i = 0; i < 9; ++i) dR[i] = host[3 + i];
    ds.resize(n);
    for (int i = 0; i < n; ++i) ds[i] = host[12 + i];
    return true;
}

bool FloatingBaseSystemKinematics::forwardEulerIntegrate(double initialTime, double finalTime,
                                                         double dT)
{
    if (!checkSizes("FloatingBaseSystemKinematics::dynamics")) return false;
    const int n = static_cast<int>(std::get<2>(m_state).size());
    blf_handle* h = blf::threadHandle();
    if (h == nullptr || !uploadState()) return false;
    double* st = m_dState.data();
    const double* in = m_dInput.data();
    if (!blf::report(blf_fbk_euler_integrate(h, n, m_rho, st, st + 3, st + 12, in, in + 6, 1,
                                             initialTime, finalTime, dT, nullptr),
                     "FixedStepIntegrator::integrate"))
        return false;
    std::vector<double> host(12 + n);
    if (!m_dState.download(host.data(), 12 + n)) return false;
    auto& [p, R, s] = m_state;
    for (int i = 0; i < 3; ++i) p[i] = host[i];
    for (int i = 0; i < 9; ++i) R[i] = host[3 + i];
    for (int i = 0; i < n; ++i) s[i] = host[12 + i];
    return true;
}
