/**
 * @file QuinticSpline.cpp
 */
#include <iostream>

#include <BipedalLocomotion/Planners/QuinticSpline.h>

using namespace BipedalLocomotion::Planners;

bool QuinticSpline::setKnots(const std::vector<double>& times, int dim,
                             const std::vector<double>& position,
                             const std::vector<double>& velocity,
                             const std::vector<double>& acceleration)
{
    const std::size_t K1 = times.size();
    if (K1 < 2 || dim < 1 || dim > 3 || position.size() != K1 * dim || velocity.size() != K1 * dim ||
        acceleration.size() != K1 * dim)
    {
        std::cerr << "[QuinticSpline::setKnots] Need at least two knots, 1 <= dim <= 3 and "
                     "(knots x dim) values for position, velocity and acceleration."
                  << std::endl;
        return false;
    }
    for (std::size_t j = 1; j < K1; ++j)
        if (!(times[j] > times[j - 1]))
        {
            std::cerr << "[QuinticSpline::setKnots] Knot times must be strictly increasing."
                      << std::endl;
            return false;
        }
    blf_handle* h = blf::threadHandle();
    if (h == nullptr) return false;
    std::vector<double> pva(K1 * 3 * dim);
    for (std::size_t j = 0; j < K1; ++j)
        for (int d = 0; d < dim; ++d)
        {
            pva[(j * 3 + 0) * dim + d] = position[j * dim + d];
            pva[(j * 3 + 1) * dim + d] = velocity[j * dim + d];
            pva[(j * 3 + 2) * dim + d] = acceleration[j * dim + d];
        }
    if (!m_dT.upload(times) || !m_dPva.upload(pva) || !m_dCoeffs.resize((K1 - 1) * dim * 6))
        return false;
    if (!blf::report(blf_quintic_fit(h, m_dT.data(), m_dPva.data(), static_cast<int32_t>(K1), dim,
                                     1, m_dCoeffs.data(), nullptr),
                     "QuinticSpline::setKnots"))
        return false;
    m_knots = static_cast<int>(K1);
    m_dim = dim;
    m_times = times;
    return true;
}

bool QuinticSpline::evaluate(const std::vector<double>& queries, std::vector<double>& pva,
                             std::vector<int32_t>& knotIndex)
{
    if (m_knots < 2)
    {
        std::cerr << "[QuinticSpline::evaluate] Please call setKnots first." << std::endl;
        return false;
    }
    blf_handle* h = blf::threadHandle();
    if (h == nullptr) return false;
    const int32_t Q = static_cast<int32_t>(queries.size());
    if (!m_dQ.upload(queries) || !m_dOut.resize(static_cast<std::size_t>(Q) * 3 * m_dim) ||
        !m_dIdx.resize(Q))
        return false;
    if (!blf::report(blf_quintic_eval(h, m_dT.data(), m_dCoeffs.data(), m_knots, m_dim, 1,
                                      m_dQ.data(), Q, m_dOut.data(), m_dIdx.data(), nullptr),
                     "QuinticSpline::evaluate"))
        return false;
    return m_dOut.download(pva) && m_dIdx.download(knotIndex);
}

bool QuinticSpline::coefficients(std::vector<double>& coeffs) const
{
    return m_dCoeffs.download(coeffs);
}
