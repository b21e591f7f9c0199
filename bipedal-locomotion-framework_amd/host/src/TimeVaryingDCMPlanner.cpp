/**
 * @file TimeVaryingDCMPlanner.cpp
 * Host bookkeeping (knot -> phase -> active-contact corners) around the device pipeline
 * blf_hull2d_hrep -> blf_dcm_mpc_solve.
 */
#include <cmath>
#include <iostream>

#include <BipedalLocomotion/Planners/TimeVaryingDCMPlanner.h>

using namespace BipedalLocomotion::Planners;

namespace
{
constexpr int kCorners = 8;   // two rectangular feet at most per knot
}

TimeVaryingDCMPlanner::TimeVaryingDCMPlanner()
{
    blf_dcm_mpc_default_params(&m_params, 100);
}

bool TimeVaryingDCMPlanner::initialize(std::weak_ptr<ParametersHandler::IParametersHandler> handler)
{
    auto ptr = handler.lock();
    if (ptr == nullptr)
    {
        std::cerr << "[TimeVaryingDCMPlanner::initialize] The parameter handler is expired."
                  << std::endl;
        return false;
    }
    int horizon = m_params.horizon;
    ptr->getParameter("horizon", horizon);
    if (horizon < 1)
    {
        std::cerr << "[TimeVaryingDCMPlanner::initialize] horizon must be >= 1." << std::endl;
        return false;
    }
    blf_dcm_mpc_default_params(&m_params, horizon);
    ptr->getParameter("sampling_time", m_params.dt);
    ptr->getParameter("gravity", m_gravity);
    ptr->getParameter("foot_length", m_footLength);
    ptr->getParameter("foot_width", m_footWidth);
    ptr->getParameter("tolerance", m_params.tol_mu);
    int maxIter = m_params.max_iter;
    if (ptr->getParameter("max_iterations", maxIter)) m_params.max_iter = maxIter;
    auto weight = [&](const char* key, double* w) {
        std::vector<double> v;
        if (!ptr->getParameter(key, v)) return true;
        if (v.size() == 1) w[0] = w[1] = v[0];
        else if (v.size() == 2) { w[0] = v[0]; w[1] = v[1]; }
        else
        {
            std::cerr << "[TimeVaryingDCMPlanner::initialize] " << key
                      << " must be a scalar or a 2-vector." << std::endl;
            return false;
        }
        return true;
    };
    if (!weight("dcm_weight", m_params.w_xi) || !weight("vrp_weight", m_params.w_vrp) ||
        !weight("terminal_weight", m_params.w_terminal))
        return false;
    if (!(m_params.dt > 0) || !(m_params.w_vrp[0] > 0) || !(m_params.w_vrp[1] > 0))
    {
        std::cerr << "[TimeVaryingDCMPlanner::initialize] sampling_time and vrp_weight must be "
                     "positive."
                  << std::endl;
        return false;
    }
    m_start = 0;
    m_valid = false;
    return true;
}

bool TimeVaryingDCMPlanner::setContactPhaseLists(const std::vector<ContactPhaseList>& plans)
{
    if (plans.empty())
    {
        std::cerr << "[TimeVaryingDCMPlanner::setContactPhaseLists] Empty batch." << std::endl;
        return false;
    }
    m_plans = plans;
    m_start = 0;
    m_valid = false;
    return true;
}

bool TimeVaryingDCMPlanner::setInitialDCM(const std::vector<std::array<double, 2>>& xi0)
{
    m_xi0.resize(2 * xi0.size());
    for (std::size_t i = 0; i < xi0.size(); ++i)
    {
        m_xi0[2 * i] = xi0[i][0];
        m_xi0[2 * i + 1] = xi0[i][1];
    }
    return true;
}

bool TimeVaryingDCMPlanner::setCoMHeights(const std::vector<double>& heights)
{
    for (double z : heights)
        if (!(z > 0))
        {
            std::cerr << "[TimeVaryingDCMPlanner::setCoMHeights] Heights must be positive."
                      << std::endl;
            return false;
        }
    m_height = heights;
    return true;
}

bool TimeVaryingDCMPlanner::advance()
{
    m_valid = false;
    const int B = static_cast<int>(m_plans.size());
    const int N = m_params.horizon;
    if (B == 0 || static_cast<int>(m_xi0.size()) != 2 * B)
    {
        std::cerr << "[TimeVaryingDCMPlanner::advance] Set the contact phase lists and one "
                     "initial DCM per problem first."
                  << std::endl;
        return false;
    }
    if (!m_height.empty() && static_cast<int>(m_height.size()) != B * N)
    {
        std::cerr << "[TimeVaryingDCMPlanner::advance] CoM heights must be [batch][horizon]."
                  << std::endl;
        return false;
    }
    blf_handle* h = blf::threadHandle();
    if (h == nullptr) return false;

    // 1. knot -> phase -> corners of the active contacts (host bookkeeping)
    std::vector<double> corners(static_cast<std::size_t>(B) * (N + 1) * kCorners * 2, 0.0);
    std::vector<int32_t> ncorners(static_cast<std::size_t>(B) * (N + 1), 0);
    std::vector<double> xiRef(static_cast<std::size_t>(B) * (N + 1) * 2);
    std::vector<double> omega(static_cast<std::size_t>(B) * N);
    for (int b = 0; b < B; ++b)
    {
        for (int k = 0; k <= N; ++k)
        {
            const double t = static_cast<double>(m_start + k) * m_params.dt;
            const int phase = m_plans[b].phaseIndexAt(t);
            if (phase < 0)
            {
                std::cerr << "[TimeVaryingDCMPlanner::advance] Problem " << b << ": knot time " << t
                          << " is outside every contact phase." << std::endl;
                return false;
            }
            // deterministic corner order: active contacts sorted by list name
            std::map<std::string, ContactList::const_iterator> active(
                m_plans[b][phase].activeContacts.begin(), m_plans[b][phase].activeContacts.end());
            const std::size_t base = (static_cast<std::size_t>(b) * (N + 1) + k);
            int c = 0;
            double sx = 0.0, sy = 0.0;
            for (const auto& entry : active)
            {
                for (double ex : {0.5, -0.5})
                    for (double ey : {0.5, -0.5})
                    {
                        if (c >= kCorners) break;
                        const auto p = entry.second->pose.apply({{ex * m_footLength, ey * m_footWidth, 0.0}});
                        corners[(base * kCorners + c) * 2] = p[0];
                        corners[(base * kCorners + c) * 2 + 1] = p[1];
                        sx += p[0];
                        sy += p[1];
                        ++c;
                    }
            }
            if (c < 3)
            {
                std::cerr << "[TimeVaryingDCMPlanner::advance] Problem " << b
                          << ": no active contact at knot time " << t << "." << std::endl;
                return false;
            }
            ncorners[base] = c;
            xiRef[2 * base] = sx / c;
            xiRef[2 * base + 1] = sy / c;
            if (k < N)
            {
                const double z = m_height.empty() ? 0.53 : m_height[static_cast<std::size_t>(b) * N + k];
                omega[static_cast<std::size_t>(b) * N + k] = std::sqrt(m_gravity / z);
            }
        }
    }
    std::vector<double> vrpRef(static_cast<std::size_t>(B) * N * 2);
    for (int b = 0; b < B; ++b)
        for (int k = 0; k < N; ++k)
            for (int j = 0; j < 2; ++j)
                vrpRef[(static_cast<std::size_t>(b) * N + k) * 2 + j] =
                    xiRef[(static_cast<std::size_t>(b) * (N + 1) + k) * 2 + j];

    // 2. support polygons on the device: knots 0..N-1 of every problem
    const int M = m_params.max_facets;
    const std::size_t polys = static_cast<std::size_t>(B) * N;
    std::vector<double> cornersQP(polys * kCorners * 2);
    std::vector<int32_t> ncornersQP(polys);
    for (int b = 0; b < B; ++b)
        for (int k = 0; k < N; ++k)
        {
            const std::size_t src = static_cast<std::size_t>(b) * (N + 1) + k;
            const std::size_t dst = static_cast<std::size_t>(b) * N + k;
            for (int c = 0; c < kCorners * 2; ++c) cornersQP[dst * kCorners * 2 + c] = corners[src * kCorners * 2 + c];
            ncornersQP[dst] = ncorners[src];
        }
    if (!m_dCorners.upload(cornersQP) || !m_dNCorners.upload(ncornersQP) ||
        !m_dA.resize(polys * M * 2) || !m_dB.resize(polys * M) || !m_dNf.resize(polys))
        return false;
    if (!blf::report(blf_hull2d_hrep(h, m_dCorners.data(), m_dNCorners.data(), kCorners, M,
                                     static_cast<int64_t>(polys), m_dA.data(), m_dB.data(),
                                     m_dNf.data(), nullptr),
                     "TimeVaryingDCMPlanner::advance"))
        return false;

    // 3. the QPs
    if (!m_dXi0.upload(m_xi0) || !m_dOmega.upload(omega) || !m_dXiRef.upload(xiRef) ||
        !m_dVrpRef.upload(vrpRef) || !m_dXi.resize(static_cast<std::size_t>(B) * (N + 1) * 2) ||
        !m_dVrp.resize(static_cast<std::size_t>(B) * N * 2) || !m_dStatus.resize(B) ||
        !m_dIters.resize(B))
        return false;
    blf_dcm_mpc_problem prob{m_dXi0.data(), m_dOmega.data(), m_dXiRef.data(), m_dVrpRef.data(),
                             m_dA.data(),   m_dB.data(),     m_dNf.data()};
    blf_dcm_mpc_solution sol{m_dXi.data(), m_dVrp.data(), m_dStatus.data(), m_dIters.data()};
    if (!blf::report(blf_dcm_mpc_solve(h, &m_params, &prob, B, &sol, nullptr),
                     "TimeVaryingDCMPlanner::advance"))
        return false;

    // 4. publish, then shift the window
    m_output.batch = B;
    m_output.horizon = N;
    m_output.initialTime = static_cast<double>(m_start) * m_params.dt;
    if (!m_dXi.download(m_output.dcm) || !m_dVrp.download(m_output.vrp) ||
        !m_dStatus.download(m_output.status) || !m_dIters.download(m_output.iterations))
        return false;
    bool ok = true;
    for (int b = 0; b < B; ++b)
    {
        ok = ok && m_output.status[b] == BLF_QP_SOLVED;
        m_xi0[2 * b] = m_output.dcm[(static_cast<std::size_t>(b) * (N + 1) + 1) * 2];
        m_xi0[2 * b + 1] = m_output.dcm[(static_cast<std::size_t>(b) * (N + 1) + 1) * 2 + 1];
    }
    m_valid = ok;
    ++m_start;
    return true;
}
