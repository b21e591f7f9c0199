/**
 * @file TimeVaryingDCMPlanner.cpp
 * Host bookkeeping (phases -> active-contact corners, once per plan) around the device pipeline
 * blf_hull2d_hrep (once per plan) -> blf_dcm_mpc_solve_phased (per advance(); horizons above 128:
 * blf_dcm_phase_expand -> blf_dcm_mpc_solve_warm).
 */
#include <algorithm>
#include <cmath>
#include <iostream>
#include <limits>
#include <map>

#include <BipedalLocomotion/Planners/TimeVaryingDCMPlanner.h>

using namespace BipedalLocomotion::Planners;

namespace
{
constexpr int kCorners = 16;  // four rectangular contacts at most per phase (the hull kernel's limit)
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
    // warm-started windows start next to the optimum: a tighter polish trigger than the cold
    // default pays there (bench.py --workload rh: 0.19 ms per 4096-window solve at 1e-4, 0.26 ms
    // at the cold default 3e-4)
    m_params.tol_polish = 1e-4;
    ptr->getParameter("polish_tolerance", m_params.tol_polish);
    ptr->getParameter("warm_start", m_warmStart);
    ptr->getParameter("warm_start_floor", m_warmFloor);
    if (!(m_warmFloor > 0) || !std::isfinite(m_warmFloor))
    {
        std::cerr << "[TimeVaryingDCMPlanner::initialize] warm_start_floor must be positive."
                  << std::endl;
        return false;
    }
    int maxIter = m_params.max_iter;
    if (ptr->getParameter("max_iterations", maxIter)) m_params.max_iter = maxIter;
    // facet slots per knot: 8 (default) covers one or two feet; phases with three or four
    // contacts can need more (up to 16, then the interior point kernel alone)
    int maxFacets = m_params.max_facets;
    if (ptr->getParameter("max_facets", maxFacets))
    {
        if (maxFacets < 3 || maxFacets > 16)
        {
            std::cerr << "[TimeVaryingDCMPlanner::initialize] max_facets must be in [3, 16]."
                      << std::endl;
            return false;
        }
        m_params.max_facets = maxFacets;
    }
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
    // the QP's variable layout: the DCM knots, then the VRPs
    m_variables = System::VariablesHandler();
    if (!m_variables.addVariable("dcm", 2 * static_cast<std::size_t>(horizon + 1)) ||
        !m_variables.addVariable("vrp", 2 * static_cast<std::size_t>(horizon)))
        return false;
    m_start = 0;
    m_solved = false;
    m_haveWarm = false;
    m_tableDirty = m_omegaDirty = m_xi0Dirty = true;
    return true;
}

bool TimeVaryingDCMPlanner::setContactPhaseLists(const std::vector<ContactPhaseList>& plans)
{
    if (plans.empty())
    {
        std::cerr << "[TimeVaryingDCMPlanner::setContactPhaseLists] Empty batch." << std::endl;
        return false;
    }
    if (!m_plans.empty() && plans.size() != m_plans.size()) m_xi0Dirty = m_omegaDirty = true;
    m_plans = plans;
    m_start = 0;
    m_solved = false;
    m_haveWarm = false;   // the multipliers belong to the old plan's facets
    m_tableDirty = true;
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
    m_xi0Dirty = true;
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
    m_omegaDirty = true;
    return true;
}

bool TimeVaryingDCMPlanner::buildPhaseTable(blf_handle* h)
{
    const int B = static_cast<int>(m_plans.size());
    int P = 1;
    for (const auto& plan : m_plans) P = std::max(P, static_cast<int>(plan.size()));
    const std::size_t BP = static_cast<std::size_t>(B) * P;
    std::vector<int32_t> nphases(B), ncorners(BP, 0);
    std::vector<double> begin(BP, 0.0), end(BP, 0.0), corners(BP * kCorners * 2, 0.0),
        ref(BP * 2, 0.0);
    const double inf = std::numeric_limits<double>::infinity();
    m_planBegin.assign(B, inf);
    m_planEnd.assign(B, -inf);
    m_unsupported.assign(B, {});
    for (int b = 0; b < B; ++b)
    {
        const ContactPhaseList& plan = m_plans[b];
        nphases[b] = static_cast<int32_t>(plan.size());
        for (std::size_t p = 0; p < plan.size(); ++p)
        {
            const std::size_t row = static_cast<std::size_t>(b) * P + p;
            begin[row] = plan[p].beginTime;
            end[row] = plan[p].endTime;
            // deterministic corner order: active contacts sorted by list name
            std::map<std::string, ContactList::const_iterator> active(
                plan[p].activeContacts.begin(), plan[p].activeContacts.end());
            if (active.size() > static_cast<std::size_t>(kCorners / 4))
            {   // the support polygon holds four rectangular contacts (16 corners) at most
                std::cerr << "[TimeVaryingDCMPlanner::advance] Problem " << b << ": phase " << p
                          << " has " << active.size() << " active contacts; at most "
                          << kCorners / 4 << " are supported." << std::endl;
                return false;
            }
            int c = 0;
            double sx = 0.0, sy = 0.0;
            for (const auto& entry : active)
                for (double ex : {0.5, -0.5})
                    for (double ey : {0.5, -0.5})
                    {
                        if (c >= kCorners) break;
                        const auto q = entry.second->pose.apply(
                            {{ex * m_footLength, ey * m_footWidth, 0.0}});
                        corners[(row * kCorners + c) * 2] = q[0];
                        corners[(row * kCorners + c) * 2 + 1] = q[1];
                        sx += q[0];
                        sy += q[1];
                        ++c;
                    }
            ncorners[row] = c;
            if (c > 0)
            {
                ref[2 * row] = sx / c;
                ref[2 * row + 1] = sy / c;
            }
            else   // no support polygon: a window touching this phase cannot be planned
                m_unsupported[b].emplace_back(plan[p].beginTime, plan[p].endTime);
            if (p == 0) m_planBegin[b] = plan[p].beginTime;
            m_planEnd[b] = plan[p].endTime;
        }
    }
    const int M = m_params.max_facets;
    m_maxPhases = P;
    if (!m_dNPhases.upload(nphases) || !m_dPhBegin.upload(begin) || !m_dPhEnd.upload(end) ||
        !m_dPhCorners.upload(corners) || !m_dPhNCorners.upload(ncorners) ||
        !m_dPhRef.upload(ref) || !m_dPhA.resize(BP * M * 2) || !m_dPhB.resize(BP * M) ||
        !m_dPhNf.resize(BP))
        return false;
    if (!blf::report(blf_hull2d_hrep(h, m_dPhCorners.data(), m_dPhNCorners.data(), kCorners, M,
                                     static_cast<int64_t>(BP), m_dPhA.data(), m_dPhB.data(),
                                     m_dPhNf.data(), nullptr),
                     "TimeVaryingDCMPlanner::advance"))
        return false;
    // once per plan: every phase with contacts must have a support polygon that fits the QP's
    // facet slots (a hull of three or four contacts can need more than the default 8: set
    // max_facets up to 16)
    std::vector<int32_t> nf(BP);
    if (!m_dPhNf.download(nf)) return false;
    for (int b = 0; b < B; ++b)
        for (std::size_t p = 0; p < m_plans[b].size(); ++p)
        {
            const std::size_t row = static_cast<std::size_t>(b) * P + p;
            if (ncorners[row] > 0 && nf[row] < 0)
            {
                std::cerr << "[TimeVaryingDCMPlanner::advance] Problem " << b << ": the support "
                          << "polygon of phase " << p << " (" << ncorners[row] / 4
                          << " contacts) is degenerate or needs more than max_facets = " << M
                          << " facets (at most " << kCorners << ")." << std::endl;
                return false;
            }
        }
    return true;
}

bool TimeVaryingDCMPlanner::checkWindow() const
{
    // the plans' phases are contiguous (ContactPhaseList::createPhases), so every knot of the
    // window lies in some phase iff the window lies in [first begin, last end)
    const int N = m_params.horizon;
    const double t0 = static_cast<double>(m_start) * m_params.dt;
    const double t1 = static_cast<double>(m_start + N) * m_params.dt;
    for (std::size_t b = 0; b < m_plans.size(); ++b)
    {
        if (!(m_planBegin[b] <= t0 && t1 < m_planEnd[b]))
        {
            std::cerr << "[TimeVaryingDCMPlanner::advance] Problem " << b << ": the window ["
                      << t0 << ", " << t1 << "] leaves the contact phases." << std::endl;
            return false;
        }
        for (const auto& bad : m_unsupported[b])
            if (bad.first <= t1 && t0 < bad.second)
            {
                std::cerr << "[TimeVaryingDCMPlanner::advance] Problem " << b
                          << ": no active contact in a phase of the window." << std::endl;
                return false;
            }
    }
    return true;
}

bool TimeVaryingDCMPlanner::advance()
{
    const int B = static_cast<int>(m_plans.size());
    const int N = m_params.horizon;
    const int M = m_params.max_facets;
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

    // 1. once per plan: phase table and its support polygons on the device
    if (m_tableDirty)
    {
        if (!buildPhaseTable(h)) return false;
        m_tableDirty = false;
    }
    if (!checkWindow()) return false;
    const std::size_t BN = static_cast<std::size_t>(B) * N;
    if (m_omegaDirty)
    {
        std::vector<double> omega(BN);
        for (std::size_t i = 0; i < BN; ++i)
            omega[i] = std::sqrt(m_gravity / (m_height.empty() ? 0.53 : m_height[i]));
        if (!m_dOmega.upload(omega)) return false;
        m_omegaDirty = false;
    }
    if (m_xi0Dirty)
    {
        if (!m_dXi0.upload(m_xi0)) return false;
        m_xi0Dirty = false;
    }

    // 2. the window's QPs, warm-started from the previous solution shifted by one knot.  Horizons
    //    up to 128 read the window straight from the phase table (blf_dcm_mpc_solve_phased: the
    //    expansion happens in the solver's LDS; the per-knot arrays are only scratch for problems
    //    the interior point method finishes); longer ones expand the window through HBM first.
    if (!m_dA.resize(BN * M * 2) || !m_dB.resize(BN * M) || !m_dNf.resize(BN) ||
        !m_dXiRef.resize(static_cast<std::size_t>(B) * (N + 1) * 2) || !m_dVrpRef.resize(BN * 2))
        return false;
    blf_phase_table table{m_maxPhases,     M,             m_dNPhases.data(), m_dPhBegin.data(),
                          m_dPhEnd.data(), m_dPhA.data(), m_dPhB.data(),     m_dPhNf.data(),
                          m_dPhRef.data()};
    const int nxt = m_solved ? 1 - m_cur : m_cur;
    if (!m_dXi.resize(static_cast<std::size_t>(B) * (N + 1) * 2) ||
        !m_dVrp[nxt].resize(BN * 2) || !m_dLam[nxt].resize(BN * M) || !m_dStatus[nxt].resize(B) ||
        !m_dIters.resize(B) || !m_dPasses.resize(B))
        return false;
    blf_dcm_mpc_solution sol{m_dXi.data(), m_dVrp[nxt].data(), m_dStatus[nxt].data(), m_dIters.data(),
                             nullptr,      m_dPasses.data()};
    // the previous window's statuses ride along: a plan whose last window was not solved is
    // planned cold this time instead of from that failed iterate
    blf_dcm_mpc_warm_start warm{m_dVrp[m_cur].data(), m_dLam[m_cur].data(), 1, 0, m_warmFloor,
                                m_dStatus[m_cur].data()};
    const bool useWarm = m_warmStart && m_haveWarm && m_solved;
    if (N <= 128 && m_params.tol_polish > 0)
    {
        if (!m_dWinOmega.resize(BN)) return false;
        blf_dcm_mpc_window win{m_dWinOmega.data(), m_dXiRef.data(), m_dVrpRef.data(),
                               m_dA.data(),        m_dB.data(),     m_dNf.data()};
        if (!blf::report(blf_dcm_mpc_solve_phased(h, &m_params, &table, m_start, m_dXi0.data(),
                                                  m_dOmega.data(), N, useWarm ? &warm : nullptr,
                                                  B, &win, &sol, m_dLam[nxt].data(), nullptr),
                         "TimeVaryingDCMPlanner::advance"))
            return false;
    }
    else
    {
        if (!blf::report(blf_dcm_phase_expand(h, &table, m_start, m_params.dt, N, B, m_dA.data(),
                                              m_dB.data(), m_dNf.data(), m_dXiRef.data(),
                                              m_dVrpRef.data(), nullptr),
                         "TimeVaryingDCMPlanner::advance"))
            return false;
        blf_dcm_mpc_problem prob{m_dXi0.data(), m_dOmega.data(), m_dXiRef.data(), m_dVrpRef.data(),
                                 m_dA.data(),   m_dB.data(),     m_dNf.data()};
        if (!blf::report(blf_dcm_mpc_solve_warm(h, &m_params, &prob, useWarm ? &warm : nullptr, B,
                                                &sol, m_dLam[nxt].data(), nullptr),
                         "TimeVaryingDCMPlanner::advance"))
            return false;
    }

    // 4. the planned xi_1 is the next window's initial DCM; move the window
    if (!blf::copyRows(m_dXi0.data(), 2 * sizeof(double), m_dXi.data() + 2,
                       static_cast<std::size_t>(N + 1) * 2 * sizeof(double), 2 * sizeof(double),
                       static_cast<std::size_t>(B)))
        return false;
    m_cur = nxt;
    m_solved = true;
    m_haveWarm = true;
    m_outputDirty = true;
    m_output.initialTime = static_cast<double>(m_start) * m_params.dt;
    ++m_start;
    return true;
}

void TimeVaryingDCMPlanner::download() const
{
    if (!m_outputDirty) return;
    m_outputDirty = false;
    const int B = static_cast<int>(m_plans.size());
    m_output.batch = B;
    m_output.horizon = m_params.horizon;
    bool ok = m_dXi.download(m_output.dcm) && m_dVrp[m_cur].download(m_output.vrp) &&
              m_dStatus[m_cur].download(m_output.status) && m_dIters.download(m_output.iterations) &&
              m_dPasses.download(m_output.passes);
    if (ok)
    {
        for (int b = 0; b < B; ++b) ok = ok && m_output.status[b] == BLF_QP_SOLVED;
        // each problem's QP variables in the VariablesHandler layout
        const System::IndexRange dcm = m_variables.getVariable("dcm");
        const System::IndexRange vrp = m_variables.getVariable("vrp");
        const std::size_t n = m_variables.getNumberOfVariables();
        m_output.variables.assign(static_cast<std::size_t>(B) * n, 0.0);
        for (int b = 0; b < B; ++b)
        {
            double* row = m_output.variables.data() + static_cast<std::size_t>(b) * n;
            std::copy_n(m_output.dcm.data() + static_cast<std::size_t>(b) * dcm.size, dcm.size,
                        row + dcm.offset);
            std::copy_n(m_output.vrp.data() + static_cast<std::size_t>(b) * vrp.size, vrp.size,
                        row + vrp.offset);
        }
    }
    else
    {
        std::cerr << "[TimeVaryingDCMPlanner::get] Could not download the plan." << std::endl;
    }
    m_valid = ok;
}

const DCMPlanBatch& TimeVaryingDCMPlanner::get() const
{
    download();
    return m_output;
}

bool TimeVaryingDCMPlanner::isValid() const
{
    if (!m_solved) return false;
    download();
    return m_valid;
}

blf_dcm_mpc_solution TimeVaryingDCMPlanner::deviceSolution()
{
    return blf_dcm_mpc_solution{m_dXi.data(), m_dVrp[m_cur].data(), m_dStatus[m_cur].data(),
                                m_dIters.data(), nullptr, m_dPasses.data()};
}
