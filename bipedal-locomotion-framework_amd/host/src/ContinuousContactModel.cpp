/**
 * @file ContinuousContactModel.cpp
 * Parameter handling and messages follow src/ContactModels/src/ContinuousContactModel.cpp:24-76;
 * the arithmetic of :79-254 runs on the device through the C ABI.
 */
#include <iostream>
#include <limits>

#include <BipedalLocomotion/ContactModels/ContinuousContactModel.h>

using namespace BipedalLocomotion::ContactModels;
using namespace BipedalLocomotion::ParametersHandler;

namespace
{
// device input block: params 4 | twist 6 | pose 12 | null pose 12
constexpr int kIn = 34;
enum Which { kWrench = 0, kAutonomous = 1, kControl = 2, kRegressor = 3 };
} // namespace

ContinuousContactModel::ContinuousContactModel()
{
    m_controlMatrix.fill(0.0);
    m_autonomousDynamics.fill(0.0);
    m_regressor.resize(6, 2);
}

bool ContinuousContactModel::initializePrivate(std::weak_ptr<IParametersHandler> weakHandler)
{
    auto handler = weakHandler.lock();
    if (handler == nullptr)
    {
        std::cerr << "[ContinuousContactModel::initialize] The parameter handler is corrupted. "
                     "Please make sure that the handler exists."
                  << std::endl;
        return false;
    }
    if (!handler->getParameter("length", m_length))
    {
        std::cerr << "[ContinuousContactModel::initialize] Unable to get the variable named length."
                  << std::endl;
        return false;
    }
    if (!handler->getParameter("width", m_width))
    {
        std::cerr << "[ContinuousContactModel::initialize] Unable to get the variable named width."
                  << std::endl;
        return false;
    }
    if (!handler->getParameter("spring_coeff", m_springCoeff))
    {
        std::cerr << "[ContinuousContactModel::initialize] Unable to get the variable named "
                     "spring_coeff."
                  << std::endl;
        return false;
    }
    if (!handler->getParameter("damper_coeff", m_damperCoeff))
    {
        std::cerr << "[ContinuousContactModel::initialize] Unable to get the variable named "
                     "damper_coeff."
                  << std::endl;
        return false;
    }
    return true;
}

void ContinuousContactModel::setNullForceTransformPrivate(const blf::Transform& transform)
{
    m_nullForceTransform = transform;
}

void ContinuousContactModel::setStatePrivate(const blf::Twist& twist, const blf::Transform& transform)
{
    m_twist = twist;
    m_frameTransform = transform;
}

bool ContinuousContactModel::upload()
{
    double in[kIn];
    in[0] = m_length;
    in[1] = m_width;
    in[2] = m_springCoeff;
    in[3] = m_damperCoeff;
    for (int i = 0; i < 6; ++i) in[4 + i] = m_twist[i];
    const auto pose = m_frameTransform.packed();
    const auto null = m_nullForceTransform.packed();
    for (int i = 0; i < 12; ++i)
    {
        in[10 + i] = pose[i];
        in[22 + i] = null[i];
    }
    return m_dIn.upload(in, kIn);
}

void ContinuousContactModel::evaluate(int which, double* host, int n, const char* where)
{
    blf_handle* h = blf::threadHandle();
    bool ok = h != nullptr && upload() && m_dOut.resize(n);
    if (ok)
    {
        const double* in = m_dIn.data();
        double* out[4] = {nullptr, nullptr, nullptr, nullptr};
        out[which] = m_dOut.data();
        ok = blf::report(blf_contact_model_eval(h, in, 1, in + 4, in + 10, in + 22, 1, out[0],
                                                out[1], out[2], out[3], nullptr),
                         where)
             && m_dOut.download(host, n);
    }
    if (!ok)
    {
        std::cerr << "[" << where << "] device evaluation failed" << std::endl;
        for (int i = 0; i < n; ++i) host[i] = std::numeric_limits<double>::quiet_NaN();
    }
}

void ContinuousContactModel::computeContactWrench()
{
    evaluate(kWrench, m_contactWrench.data(), 6, "ContinuousContactModel::computeContactWrench");
}

void ContinuousContactModel::computeAutonomousDynamics()
{
    evaluate(kAutonomous, m_autonomousDynamics.data(), 6,
             "ContinuousContactModel::computeAutonomousDynamics");
}

void ContinuousContactModel::computeControlMatrix()
{
    evaluate(kControl, m_controlMatrix.data(), 36, "ContinuousContactModel::computeControlMatrix");
}

void ContinuousContactModel::computeRegressor()
{
    m_regressor.resize(6, 2);
    evaluate(kRegressor, m_regressor.data(), 12, "ContinuousContactModel::computeRegressor");
}

bool ContinuousContactModel::getWrenchesAtPoints(const std::vector<double>& points,
                                                 std::vector<double>& force,
                                                 std::vector<double>& torque)
{
    const int q = static_cast<int>(points.size() / 2);
    force.assign(3 * q, 0.0);
    torque.assign(3 * q, 0.0);
    blf_handle* h = blf::threadHandle();
    blf::DeviceBuffer<double> dPts, dF, dT;
    if (h == nullptr || !upload() || !dPts.upload(points.data(), 2 * q) || !dF.resize(3 * q)
        || !dT.resize(3 * q))
        return false;
    const double* in = m_dIn.data();
    if (!blf::report(blf_contact_point_wrench(h, in, 1, in + 4, in + 10, in + 22, 1, dPts.data(),
                                              q, dF.data(), dT.data(), nullptr),
                     "ContinuousContactModel::getForceAtPoint"))
        return false;
    return dF.download(force.data(), 3 * q) && dT.download(torque.data(), 3 * q);
}

blf::Vector3 ContinuousContactModel::getForceAtPoint(const double& x, const double& y)
{
    std::vector<double> f, t;
    blf::Vector3 out{};
    if (!getWrenchesAtPoints({x, y}, f, t))
        out.fill(std::numeric_limits<double>::quiet_NaN());
    else
        out = {f[0], f[1], f[2]};
    return out;
}

blf::Vector3 ContinuousContactModel::getTorqueGeneratedAtPoint(const double& x, const double& y)
{
    std::vector<double> f, t;
    blf::Vector3 out{};
    if (!getWrenchesAtPoints({x, y}, f, t))
        out.fill(std::numeric_limits<double>::quiet_NaN());
    else
        out = {t[0], t[1], t[2]};
    return out;
}
