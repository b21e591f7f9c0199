/**
 * @file host_tests.cpp
 * The reference's Catch2 tests for the DCM path, restated against the C++ adapters:
 *   ContactListTest.cpp:28-118, ContactPhaseListTest.cpp:15-153, VariablesHandlerTest.cpp:15-35
 *   (host bookkeeping, run everywhere), IntegratorTest.cpp:27-75 (device), a 2-D
 *   ConvexHullHelperTest (device), the QuinticSpline and TimeVaryingDCMPlanner::advance (device),
 *   ContinousContactModelTest.cpp:30-214 (device) and FloatingBaseSystemKinematics under
 *   ForwardEuler (device), and ParametersHandlerYarpTest.cpp:30-140 on the reference's own
 *   config.ini (tests/golden/parameters_config.ini) read by StdImplementation::setFromFile.
 * usage: blf_host_tests [cpu|gpu|all]   (exit status = number of failed checks)
 */
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <iostream>
#include <memory>
#include <string>
#include <vector>

#include <random>

#include <BipedalLocomotion/ContactModels/ContinuousContactModel.h>
#include <BipedalLocomotion/ParametersHandler/IParametersHandler.h>
#include <BipedalLocomotion/Planners/ContactList.h>
#include <BipedalLocomotion/Planners/ContactPhaseList.h>
#include <BipedalLocomotion/Planners/ConvexHullHelper.h>
#include <BipedalLocomotion/Planners/QuinticSpline.h>
#include <BipedalLocomotion/Planners/TimeVaryingDCMPlanner.h>
#include <BipedalLocomotion/System/FloatingBaseSystemDynamics.h>
#include <BipedalLocomotion/System/FloatingBaseSystemKinematics.h>
#include <BipedalLocomotion/System/ForwardEuler.h>
#include <BipedalLocomotion/System/LinearTimeInvariantSystem.h>
#include <BipedalLocomotion/System/VariablesHandler.h>
#include <blf/urdf.h>

using namespace BipedalLocomotion;
using namespace BipedalLocomotion::Planners;
using namespace BipedalLocomotion::System;

static int g_failed = 0, g_checks = 0;
#define REQUIRE(cond)                                                                          \
    do {                                                                                       \
        ++g_checks;                                                                            \
        if (!(cond)) {                                                                         \
            ++g_failed;                                                                        \
            std::fprintf(stderr, "  FAILED %s:%d: %s\n", __FILE__, __LINE__, #cond);           \
        }                                                                                      \
    } while (0)
#define REQUIRE_FALSE(cond) REQUIRE(!(cond))

static bool sameContact(const Contact& a, const Contact& b)
{
    return a.type == b.type && a.name == b.name && a.activationTime == b.activationTime &&
           a.deactivationTime == b.deactivationTime && a.pose.position == b.pose.position &&
           a.pose.rotation == b.pose.rotation;
}

// ---- ContactListTest.cpp:28-118 ----------------------------------------------------------------
static void testContactList()
{
    auto fresh = [](Contact& p1, Contact& p2) {
        ContactList list;
        p1 = Contact{};
        p2 = Contact{};
        p1.activationTime = 0.1;
        p1.deactivationTime = 0.5;
        p2.activationTime = 1.0;
        p2.deactivationTime = 1.5;
        REQUIRE(list.addContact(p2));   // insertion out of order
        REQUIRE(list.addContact(p1));
        return list;
    };
    Contact p1, p2;
    {   // insertion order + size
        ContactList list = fresh(p1, p2);
        REQUIRE(sameContact(p1, *list.firstContact()));
        REQUIRE(sameContact(p2, *list.lastContact()));
        Contact p3;
        p3.activationTime = 0.6;
        p3.deactivationTime = 0.8;
        REQUIRE(list.addContact(p3));
        REQUIRE(list.size() == 3);
        REQUIRE(sameContact(p3, *(++list.begin())));
    }
    {   // invalid (overlapping) insertion; touching intervals are rejected too
        ContactList list = fresh(p1, p2);
        Contact p3;
        p3.activationTime = 0.9;
        p3.deactivationTime = 1.6;
        REQUIRE_FALSE(list.addContact(p3));
        Contact p4;
        p4.activationTime = 1.5;
        p4.deactivationTime = 2.0;
        REQUIRE_FALSE(list.addContact(p4));
        Contact bad;
        bad.activationTime = 3.0;
        bad.deactivationTime = 2.0;
        REQUIRE_FALSE(list.addContact(bad));
    }
    {   // edit
        ContactList list = fresh(p1, p2);
        Contact p2m = p2;
        p2m.type = ContactType::POINT;
        REQUIRE(list.editContact(list.lastContact(), p2m));
        REQUIRE(sameContact(p2m, *list.lastContact()));
    }
    {   // present step (`<=` rule)
        ContactList list = fresh(p1, p2);
        REQUIRE(sameContact(p2, *list.getPresentContact(1.2)));
        REQUIRE(sameContact(p2, *list.getPresentContact(1.6)));
        REQUIRE(sameContact(p1, *list.getPresentContact(0.6)));
        REQUIRE(list.getPresentContact(0.0) == list.end());
        REQUIRE(list.keepOnlyPresentContact(0.6));
        REQUIRE(list.size() == 1 && sameContact(p1, *list.begin()));
    }
    {   // clear
        ContactList list = fresh(p1, p2);
        list.clear();
        REQUIRE(list.size() == 0);
    }
    {   // accessor over 51 contacts
        ContactList list = fresh(p1, p2);
        bool ok = true;
        for (std::size_t i = 0; i < 49; ++i)
            ok = ok && list.addContact(Transform::Identity(), 2.0 + i, 2.5 + i);
        REQUIRE(ok);
        REQUIRE(list.size() == 51);
        auto it = list.begin();
        for (std::size_t i = 0; i < list.size(); ++i, ++it) ok = ok && sameContact(list[i], *it);
        REQUIRE(ok);
    }
}

// ---- ContactPhaseListTest.cpp:15-153 -----------------------------------------------------------
static void testContactPhaseList()
{
    ContactList left, right, additional;
    left.setDefaultName("left");
    right.setDefaultName("right");
    additional.setDefaultName("additional");
    REQUIRE(left.addContact(Transform::Identity(), 0.0, 1.0));
    REQUIRE(left.addContact(Transform::Identity(), 2.0, 5.0));
    REQUIRE(left.addContact(Transform::Identity(), 6.0, 7.0));
    REQUIRE(right.addContact(Transform::Identity(), 0.0, 3.0));
    REQUIRE(right.addContact(Transform::Identity(), 4.0, 7.0));
    REQUIRE(additional.addContact(Transform::Identity(), 4.0, 5.0));
    REQUIRE(additional.addContact(Transform::Identity(), 6.0, 7.5));

    ContactPhaseList phases;
    REQUIRE(phases.setLists({additional, left, right}));
    REQUIRE(phases.size() == 8);
    const ContactListMap& lists = phases.lists();
    auto L = lists.at("left").begin();
    auto R = lists.at("right").begin();
    auto A = lists.at("additional").begin();
    struct Expect { double b, e; std::vector<std::pair<std::string, ContactList::const_iterator*>> act; };
    auto check = [&](const ContactPhase& ph, double b, double e,
                     std::vector<std::pair<std::string, ContactList::const_iterator>> act) {
        REQUIRE(ph.beginTime == b);
        REQUIRE(ph.endTime == e);
        REQUIRE(ph.activeContacts.size() == act.size());
        for (auto& [name, it] : act) REQUIRE(ph.isListIncluded(name) && ph.activeContacts.at(name) == it);
    };
    auto ph = phases.begin();
    check(*ph++, 0.0, 1.0, {{"left", L}, {"right", R}});
    ++L;
    check(*ph++, 1.0, 2.0, {{"right", R}});
    check(*ph++, 2.0, 3.0, {{"left", L}, {"right", R}});
    ++R;
    check(*ph++, 3.0, 4.0, {{"left", L}});
    check(*ph++, 4.0, 5.0, {{"left", L}, {"right", R}, {"additional", A}});
    ++L;
    ++A;
    check(*ph++, 5.0, 6.0, {{"right", R}});
    check(*ph++, 6.0, 7.0, {{"left", L}, {"right", R}, {"additional", A}});
    ++L;
    ++R;
    check(*ph++, 7.0, 7.5, {{"additional", A}});
    ++A;
    REQUIRE(ph == phases.end());
    REQUIRE(L == lists.at("left").end());
    REQUIRE(R == lists.at("right").end());
    REQUIRE(A == lists.at("additional").end());
    REQUIRE(phases.phaseIndexAt(4.0) == 4 && phases.phaseIndexAt(7.5) == -1);

    ContactList dup;
    dup.setDefaultName("left");
    REQUIRE_FALSE(phases.setLists({left, dup}));
}

// ---- VariablesHandlerTest.cpp:15-35 ------------------------------------------------------------
static void testVariablesHandler()
{
    VariablesHandler handler;
    REQUIRE(handler.addVariable("variable_1", 42));
    REQUIRE(handler.addVariable("variable_2", 35));
    REQUIRE_FALSE(handler.addVariable("variable_1", 3));
    REQUIRE(handler.getVariable("variable_1").offset == 0);
    REQUIRE(handler.getVariable("variable_1").size == 42);
    REQUIRE(handler.getVariable("variable_2").offset == 42);
    REQUIRE(handler.getVariable("variable_2").size == 35);
    REQUIRE(handler.getNumberOfVariables() == 77);
    REQUIRE_FALSE(handler.getVariable("variable_3").isValid());
}

// ---- IntegratorTest.cpp:27-75 (device) --------------------------------------------------------
static void testIntegratorLTI()
{
    constexpr double dT = 0.0001;
    constexpr double tolerance = 1e-3;
    constexpr double simulationTime = 2;
    auto system = std::make_shared<LinearTimeInvariantSystem>();
    blf::MatrixXd A(2, 2, {0, 1, -2, -2});
    blf::MatrixXd b(2, 1, {0, 2});
    REQUIRE(system->setSystemMatrices(A, b));
    system->setControlInput({blf::VectorXd{1.0}});
    system->setState({blf::VectorXd{0.0, 0.0}});
    ForwardEuler<LinearTimeInvariantSystem> integrator(dT);
    REQUIRE(integrator.setDynamicalSystem(system));
    REQUIRE_FALSE(integrator.setDynamicalSystem(system));   // set once only
    bool ok = true;
    for (int i = 0; i < simulationTime / dT; i++)
    {
        const auto& [x] = integrator.getSolution();
        const double t = dT * i;
        const double e0 = 1 - std::exp(-t) * (std::cos(t) + std::sin(t));
        const double e1 = 2 * std::exp(-t) * std::sin(t);
        const double dn = std::hypot(x(0) - e0, x(1) - e1);
        ok = ok && dn <= tolerance * std::min(std::hypot(x(0), x(1)), std::hypot(e0, e1));
        ok = ok && integrator.integrate(0, dT);
        if (!ok) break;
    }
    REQUIRE(ok);
    // dynamics() on the device: dx = A x + B u
    std::tuple<blf::VectorXd> dx;
    REQUIRE(system->dynamics(0.0, dx));
    const auto& [xs] = integrator.getSolution();
    REQUIRE(std::get<0>(dx)(0) == 0.0 * xs(0) + 1.0 * xs(1) + 0.0 * 1.0);
    // error semantics: t0 > T, T == t0 (the reference never returns: refused here)
    REQUIRE_FALSE(integrator.integrate(1.0, 0.5));
    REQUIRE_FALSE(integrator.integrate(1.0, 1.0));
    ForwardEuler<LinearTimeInvariantSystem> bad(-1.0);
    REQUIRE(bad.setDynamicalSystem(system));
    REQUIRE_FALSE(bad.integrate(0.0, 1.0));
}

// ---- ConvexHullHelper on n x p points (device, blf_hullnd_hrep) ---------------------------------
static void testConvexHullN()
{
    ConvexHullHelper helper;
    // the 4-D unit hypercube: 16 points, 8 facets x_c <= 1, -x_c <= 0
    blf::MatrixXd cube(4, 16);
    for (int j = 0; j < 16; ++j)
        for (int c = 0; c < 4; ++c) cube(c, j) = (j >> c) & 1;
    REQUIRE(helper.buildConvexHull(cube));
    REQUIRE(helper.getA().rows() == 8 && helper.getA().cols() == 4);
    int unitRows = 0;
    for (std::size_t i = 0; i < helper.getA().rows(); ++i)
    {
        int nz = 0, which = -1;
        for (int c = 0; c < 4; ++c)
            if (std::abs(helper.getA()(i, c)) > 1e-12) ++nz, which = c;
        const double a = helper.getA()(i, which);
        unitRows += nz == 1 && std::abs(std::abs(a) - 1.0) < 1e-12
                    && std::abs(helper.getB()(i) - (a > 0 ? 1.0 : 0.0)) < 1e-12;
    }
    REQUIRE(unitRows == 8);
    REQUIRE(helper.doesPointBelongToConvexHull(blf::VectorXd{0.5, 0.5, 0.5, 0.5}));
    REQUIRE(helper.doesPointBelongToConvexHull(blf::VectorXd{1.0, 0.0, 1.0, 0.0}));
    REQUIRE_FALSE(helper.doesPointBelongToConvexHull(blf::VectorXd{0.5, 0.5, 0.5, 1.01}));
    // 1-D: an interval
    blf::MatrixXd line(1, 3, {0.3, -0.2, 0.9});
    REQUIRE(helper.buildConvexHull(line));
    REQUIRE(helper.getA().rows() == 2);
    REQUIRE(helper.doesPointBelongToConvexHull(blf::VectorXd{0.0}));
    REQUIRE_FALSE(helper.doesPointBelongToConvexHull(blf::VectorXd{1.0}));
    // 2-D with more points than the polygon kernel takes (20 on a circle)
    blf::MatrixXd ring(2, 20);
    for (int j = 0; j < 20; ++j) ring(0, j) = std::cos(0.1 * M_PI * j), ring(1, j) = std::sin(0.1 * M_PI * j);
    REQUIRE(helper.buildConvexHull(ring));
    REQUIRE(helper.getA().rows() == 20);
    // a flat 4-D set, too few points, too many dimensions
    blf::MatrixXd flat = cube;
    for (int j = 0; j < 16; ++j) flat(3, j) = 0.5;
    REQUIRE_FALSE(helper.buildConvexHull(flat));
    REQUIRE_FALSE(helper.doesPointBelongToConvexHull(blf::VectorXd{0.5, 0.5, 0.5, 0.5}));
    REQUIRE_FALSE(helper.buildConvexHull(blf::MatrixXd(4, 4)));
    REQUIRE_FALSE(helper.buildConvexHull(blf::MatrixXd(9, 12)));
}

// ---- ForwardEuler over a host-side DynamicalSystem subclass (ForwardEuler.tpp:18-49) ----------
// The reference's IntegratorTest system written as a user's CPU system: dx = A x + B u with the
// device kernel's summation order, so its trajectory is bit for bit blf_lti_euler_integrate's.
class HostLinearSystem
    : public DynamicalSystem<std::tuple<blf::VectorXd>, std::tuple<blf::VectorXd>,
                             std::tuple<blf::VectorXd>>
{
public:
    int calls = 0;
    bool dynamics(const double& time, StateDerivativeType& stateDerivative) final
    {
        (void)time;
        ++calls;
        const auto& x = std::get<0>(m_state);
        const auto& u = std::get<0>(m_controlInput);
        auto& dx = std::get<0>(stateDerivative);
        dx.resize(2);
        const double A[2][2] = {{0, 1}, {-2, -2}}, B[2] = {0, 2};
        for (int r = 0; r < 2; ++r)
        {
            double ax = 0.0;
            for (int c = 0; c < 2; ++c) ax = ax + A[r][c] * x[c];
            dx[r] = ax + B[r] * u[0];
        }
        return true;
    }
};

// A time-varying system with a two-element state (vector + scalar): the scalar uses `+=`, the
// vector the entry-wise path; the time argument of every step is recorded.
class HostClock
    : public DynamicalSystem<std::tuple<blf::VectorXd, double>, std::tuple<blf::VectorXd, double>,
                             std::tuple<double>>
{
public:
    std::vector<double> times;
    bool failAt = false;
    bool dynamics(const double& time, StateDerivativeType& stateDerivative) final
    {
        times.push_back(time);
        if (failAt && times.size() == 3) return false;
        auto& [dv, ds] = stateDerivative;
        dv = blf::VectorXd{std::cos(time), std::get<0>(m_controlInput)};
        ds = std::get<1>(m_state) * -0.5;
        return true;
    }
};

static void testIntegratorHostSystem()
{
    // IntegratorTest.cpp:27-75 on the host-side system: the analytic solution at 1e-3.
    constexpr double dT = 0.0001, tolerance = 1e-3, simulationTime = 2;
    auto system = std::make_shared<HostLinearSystem>();
    system->setControlInput({blf::VectorXd{1.0}});
    system->setState({blf::VectorXd{0.0, 0.0}});
    ForwardEuler<HostLinearSystem> integrator(dT);
    REQUIRE(integrator.setDynamicalSystem(system));
    bool ok = true;
    for (int i = 0; i < simulationTime / dT; i++)
    {
        const auto& [x] = integrator.getSolution();
        const double t = dT * i;
        const double e0 = 1 - std::exp(-t) * (std::cos(t) + std::sin(t));
        const double e1 = 2 * std::exp(-t) * std::sin(t);
        const double dn = std::hypot(x(0) - e0, x(1) - e1);
        ok = ok && dn <= tolerance * std::min(std::hypot(x(0), x(1)), std::hypot(e0, e1));
        ok = ok && integrator.integrate(0, dT);
        if (!ok) break;
    }
    REQUIRE(ok);
    REQUIRE(system->calls == int(simulationTime / dT));

    // The schedule, literally FixedStepIntegrator.tpp:48-64: ceil((T - t0)/dT) steps, the last at
    // the stale time with the remainder step.
    auto clock = std::make_shared<HostClock>();
    clock->setState({blf::VectorXd{0.0, 1.0}, 2.0});
    clock->setControlInput({0.25});
    ForwardEuler<HostClock> euler(0.3);
    REQUIRE(euler.setDynamicalSystem(clock));
    REQUIRE(euler.integrate(0.1, 1.0));
    const int iters = int(std::ceil((1.0 - 0.1) / 0.3));
    double v0 = 0.0, v1 = 1.0, s = 2.0, cur = 0.1;
    std::vector<double> expect;
    for (std::size_t i = 0; i < std::size_t(iters - 1); i++)
    {
        cur = 0.1 + 0.3 * i;
        expect.push_back(cur);
        const double d0 = std::cos(cur), d1 = 0.25, ds = s * -0.5;
        v0 = v0 + d0 * 0.3, v1 = v1 + d1 * 0.3, s += ds * 0.3;
    }
    const double last = 1.0 - cur;
    expect.push_back(cur);
    {
        const double d0 = std::cos(cur), d1 = 0.25, ds = s * -0.5;
        v0 = v0 + d0 * last, v1 = v1 + d1 * last, s += ds * last;
    }
    REQUIRE(clock->times == expect);
    const auto& [v, sc] = euler.getSolution();
    REQUIRE(v(0) == v0);
    REQUIRE(v(1) == v1);
    REQUIRE(sc == s);

    // Errors: the reference's argument checks, a failing dynamics() mid-schedule, a derivative of
    // the wrong size.
    REQUIRE_FALSE(euler.integrate(1.0, 0.5));
    REQUIRE_FALSE(euler.integrate(1.0, 1.0));
    clock->times.clear();
    clock->failAt = true;
    REQUIRE_FALSE(euler.integrate(0.0, 1.0));
    REQUIRE(clock->times.size() == 3);
    ForwardEuler<HostClock> negative(-0.1);
    REQUIRE(negative.setDynamicalSystem(clock));
    REQUIRE_FALSE(negative.integrate(0.0, 1.0));
    auto wrong = std::make_shared<HostLinearSystem>();
    wrong->setControlInput({blf::VectorXd{1.0}});
    wrong->setState({blf::VectorXd{0.0, 0.0, 0.0}});
    ForwardEuler<HostLinearSystem> mismatch(0.1);
    REQUIRE(mismatch.setDynamicalSystem(wrong));
    REQUIRE_FALSE(mismatch.integrate(0.0, 0.3));
}

// LinearTimeInvariantSystem of any size (LinearTimeInvariantSystem.cpp:13-38 takes any): a 600-state
// system against the host-side loop (same sums, same bits), an input-free system (B with no
// columns) and an empty one (device).
class HostLti
    : public DynamicalSystem<std::tuple<blf::VectorXd>, std::tuple<blf::VectorXd>,
                             std::tuple<blf::VectorXd>>
{
public:
    blf::MatrixXd A, B;
    bool dynamics(const double&, StateDerivativeType& stateDerivative) final
    {
        const auto& x = std::get<0>(m_state);
        const auto& u = std::get<0>(m_controlInput);
        auto& dx = std::get<0>(stateDerivative);
        dx.resize(A.rows());
        for (std::size_t r = 0; r < A.rows(); ++r)
        {
            double ax = A(r, 0) * x[0];
            for (std::size_t c = 1; c < A.cols(); ++c) ax = ax + A(r, c) * x[c];
            double bu = B.cols() ? B(r, 0) * u[0] : 0.0;
            for (std::size_t c = 1; c < B.cols(); ++c) bu = bu + B(r, c) * u[c];
            dx[r] = ax + bu;
        }
        return true;
    }
};

static void testIntegratorLTIAnySize()
{
    std::mt19937_64 rng(11);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    for (const auto& [n, m] : {std::pair<int, int>{600, 3}, std::pair<int, int>{70, 0}})
    {
        blf::MatrixXd A(n, n), B(n, m);
        for (int r = 0; r < n; ++r)
        {
            for (int c = 0; c < n; ++c) A(r, c) = U(rng) / n;
            for (int c = 0; c < m; ++c) B(r, c) = U(rng);
        }
        blf::VectorXd x0(n), u(m);
        for (int r = 0; r < n; ++r) x0[r] = U(rng);
        for (int c = 0; c < m; ++c) u[c] = U(rng);
        auto dev = std::make_shared<LinearTimeInvariantSystem>();
        auto host = std::make_shared<HostLti>();
        host->A = A, host->B = B;
        REQUIRE(dev->setSystemMatrices(A, B));
        dev->setState({x0}), host->setState({x0});
        dev->setControlInput({u}), host->setControlInput({u});
        ForwardEuler<LinearTimeInvariantSystem> di(0.01);
        ForwardEuler<HostLti> hi(0.01);
        REQUIRE(di.setDynamicalSystem(dev));
        REQUIRE(hi.setDynamicalSystem(host));
        REQUIRE(di.integrate(0.0, 0.045));
        REQUIRE(hi.integrate(0.0, 0.045));
        const auto& [xd] = di.getSolution();
        const auto& [xh] = hi.getSolution();
        bool same = xd.size() == std::size_t(n);
        for (int r = 0; same && r < n; ++r) same = xd[r] == xh[r];
        REQUIRE(same);
        std::tuple<blf::VectorXd> dd, dh;
        REQUIRE(dev->dynamics(0.0, dd));
        REQUIRE(host->dynamics(0.0, dh));
        same = std::get<0>(dd).size() == std::size_t(n);
        for (int r = 0; same && r < n; ++r) same = std::get<0>(dd)[r] == std::get<0>(dh)[r];
        REQUIRE(same);
    }
    auto empty = std::make_shared<LinearTimeInvariantSystem>();
    REQUIRE(empty->setSystemMatrices(blf::MatrixXd(0, 0), blf::MatrixXd(0, 0)));
    empty->setState({blf::VectorXd{}});
    empty->setControlInput({blf::VectorXd{}});
    ForwardEuler<LinearTimeInvariantSystem> ei(0.1);
    REQUIRE(ei.setDynamicalSystem(empty));
    REQUIRE(ei.integrate(0.0, 1.0));
    REQUIRE_FALSE(ei.integrate(1.0, 0.0));
    std::tuple<blf::VectorXd> de;
    REQUIRE(empty->dynamics(0.0, de));
    REQUIRE(std::get<0>(de).size() == 0);
}

// The host-side system and the device LTI integrator give the same bits (device).
static void testIntegratorHostSystemMatchesDevice()
{
    auto host = std::make_shared<HostLinearSystem>();
    auto dev = std::make_shared<LinearTimeInvariantSystem>();
    REQUIRE(dev->setSystemMatrices(blf::MatrixXd(2, 2, {0, 1, -2, -2}), blf::MatrixXd(2, 1, {0, 2})));
    host->setControlInput({blf::VectorXd{1.0}});
    dev->setControlInput({blf::VectorXd{1.0}});
    host->setState({blf::VectorXd{0.3, -0.2}});
    dev->setState({blf::VectorXd{0.3, -0.2}});
    ForwardEuler<HostLinearSystem> hi(0.001);
    ForwardEuler<LinearTimeInvariantSystem> di(0.001);
    REQUIRE(hi.setDynamicalSystem(host));
    REQUIRE(di.setDynamicalSystem(dev));
    REQUIRE(hi.integrate(0.0, 0.9995));
    REQUIRE(di.integrate(0.0, 0.9995));
    const auto& [xh] = hi.getSolution();
    const auto& [xd] = di.getSolution();
    REQUIRE(xh(0) == xd(0));
    REQUIRE(xh(1) == xd(1));
}

// ---- ConvexHullHelper (device, 2-D) -----------------------------------------------------------
static void testConvexHull()
{
    ConvexHullHelper helper;
    // two feet in staggered double support (the planners' polygons)
    blf::MatrixXd p(2, 8);
    const double xs[8] = {0.06, 0.06, -0.06, -0.06, 0.26, 0.26, 0.14, 0.14};
    const double ys[8] = {0.145, 0.055, 0.145, 0.055, -0.055, -0.145, -0.055, -0.145};
    for (int j = 0; j < 8; ++j) { p(0, j) = xs[j]; p(1, j) = ys[j]; }
    REQUIRE(helper.buildConvexHull(p));
    REQUIRE(helper.getA().rows() == 6 && helper.getA().cols() == 2);
    double cx = 0.0, cy = 0.0;
    for (int j = 0; j < 8; ++j) { cx += xs[j] / 8; cy += ys[j] / 8; }
    for (int j = 0; j < 8; ++j)   // every corner, pulled 0.1 % towards the centroid, is inside
        REQUIRE(helper.doesPointBelongToConvexHull(
            blf::VectorXd{cx + 0.999 * (xs[j] - cx), cy + 0.999 * (ys[j] - cy)}));
    REQUIRE_FALSE(helper.doesPointBelongToConvexHull(blf::VectorXd{0.0, 0.0 - 1.0}));
    REQUIRE(helper.doesPointBelongToConvexHull(blf::VectorXd{0.1, 0.0}));
    REQUIRE_FALSE(helper.doesPointBelongToConvexHull(blf::VectorXd{0.1, 0.0, 0.0}));   // wrong size
    // 4-D input is refused
    blf::MatrixXd p4(4, 8);
    REQUIRE_FALSE(helper.buildConvexHull(p4));
}

// ---- ConvexHullHelper (device, 3-D): the reference's own test, ConvexHullHelperTest.cpp:15-63 --
static void testConvexHull3()
{
    ConvexHullHelper helper;
    blf::MatrixXd p(3, 8);
    const double c[8][3] = {{0.6269, 0.7207, 0.3000}, {0.5538, 0.6526, 0.3000},
                            {0.6901, 0.5062, 0.3000}, {0.7633, 0.5744, 0.3000},
                            {0.8927, 0.7319, 0.2400}, {0.8101, 0.6754, 0.2400},
                            {0.9231, 0.5103, 0.2400}, {1.0056, 0.5668, 0.2400}};
    for (int j = 0; j < 8; ++j)
        for (int r = 0; r < 3; ++r) p(r, j) = c[j][r];
    REQUIRE(helper.buildConvexHull(p));
    // check if the points belong to convex hull
    for (int col = 0; col < 8; ++col)
        REQUIRE(helper.doesPointBelongToConvexHull(blf::VectorXd{p(0, col), p(1, col), p(2, col)}));
    // p = [0 0 0] does not belong to the convex hull
    REQUIRE_FALSE(helper.doesPointBelongToConvexHull(blf::VectorXd{0.0, 0.0, 0.0}));
    // Qhull's 12 facets (tests/golden/hull3d.json): 10 distinct planes, the two quadrilateral
    // faces (z = 0.3, z = 0.24) as two triangles each; unit normals
    REQUIRE(helper.getA().rows() == 12 && helper.getA().cols() == 3);
    for (std::size_t i = 0; i < helper.getA().rows(); ++i)
    {
        const double n2 = helper.getA()(i, 0) * helper.getA()(i, 0) +
                          helper.getA()(i, 1) * helper.getA()(i, 1) +
                          helper.getA()(i, 2) * helper.getA()(i, 2);
        REQUIRE(std::abs(n2 - 1.0) < 1e-12);
    }
    REQUIRE_FALSE(helper.doesPointBelongToConvexHull(blf::VectorXd{0.7, 0.6}));   // wrong size
    // the unit cube: 6 square faces, Qhull's 12 triangles; a tetrahedron: 4; a cube with face
    // centres and edge midpoints (coplanar points, not vertices): still 12
    {
        blf::MatrixXd cube(3, 8);
        for (int j = 0; j < 8; ++j) { cube(0, j) = j & 1; cube(1, j) = (j >> 1) & 1; cube(2, j) = (j >> 2) & 1; }
        REQUIRE(helper.buildConvexHull(cube));
        REQUIRE(helper.getA().rows() == 12);
        const blf::MatrixXd tet(3, 4, {0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1});
        REQUIRE(helper.buildConvexHull(tet));
        REQUIRE(helper.getA().rows() == 4);
        blf::MatrixXd dense(3, 16);
        for (int j = 0; j < 8; ++j) { dense(0, j) = j & 1; dense(1, j) = (j >> 1) & 1; dense(2, j) = (j >> 2) & 1; }
        const double extra[8][3] = {{0.5, 0.5, 0.0}, {0.5, 0.5, 1.0}, {0.5, 0.0, 0.5}, {0.5, 1.0, 0.5},
                                    {0.0, 0.5, 0.5}, {1.0, 0.5, 0.5}, {0.5, 0.0, 0.0}, {1.0, 1.0, 0.5}};
        for (int j = 0; j < 8; ++j)
            for (int r = 0; r < 3; ++r) dense(r, 8 + j) = extra[j][r];
        REQUIRE(helper.buildConvexHull(dense));
        REQUIRE(helper.getA().rows() == 12);
        REQUIRE(helper.buildConvexHull(p));   // back to the reference test's hull
    }
    // a flat set has no 3-D hull
    blf::MatrixXd flat(3, 4);
    for (int j = 0; j < 4; ++j) { flat(0, j) = j & 1; flat(1, j) = j >> 1; flat(2, j) = 0.5; }
    REQUIRE_FALSE(helper.buildConvexHull(flat));
    // ... and after the failed build no point belongs to the (absent) hull, not even one that was
    // inside the previous hull (no vacuous "inside" from an empty H-representation)
    REQUIRE_FALSE(helper.doesPointBelongToConvexHull(blf::VectorXd{p(0, 0), p(1, 0), p(2, 0)}));
    REQUIRE_FALSE(helper.doesPointBelongToConvexHull(blf::VectorXd{0.5, 0.5, 0.5}));
    // a never-built helper rejects too
    ConvexHullHelper fresh;
    REQUIRE_FALSE(fresh.doesPointBelongToConvexHull(blf::VectorXd{0.0, 0.0}));
}

// ---- QuinticSpline (device) -------------------------------------------------------------------
static void testQuinticSpline()
{
    QuinticSpline spline;
    // swing foot: lift at 0.2 s, apex at 0.5 s, land at 0.8 s; x: 0 -> 0.2, z: 0 -> 0.05 -> 0
    const std::vector<double> t = {0.2, 0.5, 0.8};
    const std::vector<double> pos = {0.0, 0.0, 0.1, 0.05, 0.2, 0.0};
    const std::vector<double> vel = {0.0, 0.0, 0.2 / 0.6, 0.0, 0.0, 0.0};
    const std::vector<double> acc = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    REQUIRE(spline.setKnots(t, 2, pos, vel, acc));
    std::vector<double> pva;
    std::vector<int32_t> idx;
    REQUIRE(spline.evaluate({0.1, 0.2, 0.5, 0.8, 0.9}, pva, idx));
    REQUIRE(idx.size() == 5 && idx[0] == -1 && idx[1] == 0 && idx[2] == 1 && idx[3] == 2 && idx[4] == 2);
    auto at = [&](int q, int k, int d) { return pva[(q * 3 + k) * 2 + d]; };
    REQUIRE(std::fabs(at(1, 0, 0) - 0.0) < 1e-15 && std::fabs(at(1, 1, 0)) < 1e-15);
    REQUIRE(std::fabs(at(2, 0, 1) - 0.05) < 1e-12 && std::fabs(at(2, 1, 1)) < 1e-12);
    REQUIRE(std::fabs(at(3, 0, 0) - 0.2) < 1e-12 && std::fabs(at(3, 1, 0)) < 1e-10);
    REQUIRE_FALSE(spline.setKnots({0.0, 0.0}, 1, {0, 0}, {0, 0}, {0, 0}));
}

// ---- TimeVaryingDCMPlanner::advance (device) ---------------------------------------------------
static ContactPhaseList walkingPlan(double stride, double yaw)
{
    ContactList left, right;
    left.setDefaultName("left");
    right.setDefaultName("right");
    const double dt = 0.02;
    left.addContact(Transform::fromPlanar(0.0, 0.1, yaw), 0 * dt, 50 * dt);
    left.addContact(Transform::fromPlanar(2 * stride, 0.1, -yaw), 80 * dt, 400 * dt);
    right.addContact(Transform::fromPlanar(0.0, -0.1, -yaw), 0 * dt, 10 * dt);
    right.addContact(Transform::fromPlanar(stride, -0.1, yaw), 40 * dt, 400 * dt);
    ContactPhaseList plan;
    plan.setLists({left, right});
    return plan;
}

static void testPlanner()
{
    auto handler = std::make_shared<ParametersHandler::StdImplementation>();
    handler->setParameter("horizon", 100);
    handler->setParameter("sampling_time", 0.02);
    handler->setParameter("dcm_weight", std::vector<double>{100.0});
    handler->setParameter("vrp_weight", std::vector<double>{1.0, 1.0});
    handler->setParameter("terminal_weight", std::vector<double>{1000.0});
    TimeVaryingDCMPlanner planner;
    REQUIRE(planner.initialize(handler));
    REQUIRE_FALSE(planner.isValid());
    REQUIRE_FALSE(planner.advance());   // no plans yet
    std::vector<ContactPhaseList> plans;
    std::vector<std::array<double, 2>> xi0;
    for (int b = 0; b < 16; ++b)
    {
        plans.push_back(walkingPlan(0.18 + 0.005 * b, 0.01 * (b - 8)));
        xi0.push_back({{0.0 + 0.001 * b, 0.0}});
    }
    REQUIRE(planner.setContactPhaseLists(plans));
    REQUIRE(planner.setInitialDCM(xi0));
    for (int step = 0; step < 5; ++step)
    {
        REQUIRE(planner.advance());
        REQUIRE(planner.isValid());
        const DCMPlanBatch& plan = planner.get();
        REQUIRE(plan.batch == 16 && plan.horizon == 100);
        REQUIRE(plan.initialTime == step * 0.02);
        // the plan starts at the previous plan's xi_1 and follows the Euler DCM step
        bool dyn = true;
        for (int b = 0; b < 16; ++b)
        {
            const double* xi = &plan.dcm[static_cast<std::size_t>(b) * 101 * 2];
            const double* r = &plan.vrp[static_cast<std::size_t>(b) * 100 * 2];
            for (int k = 0; k < 100; ++k)
            {
                const double w = std::sqrt(9.81 / 0.53);
                for (int j = 0; j < 2; ++j)
                {
                    const double nxt = xi[2 * k + j] + (w * xi[2 * k + j] + (-w) * r[2 * k + j]) * 0.02;
                    dyn = dyn && std::fabs(nxt - xi[2 * (k + 1) + j]) < 1e-12;
                }
            }
        }
        REQUIRE(dyn);
    }

    // warm-started receding horizon vs cold re-solves: the same plans (both certified optima of
    // the same QPs) for fewer active-set passes; the first advance is a cold solve either way
    auto cold = std::make_shared<ParametersHandler::StdImplementation>();
    cold->setParameter("horizon", 100);
    cold->setParameter("warm_start", false);
    TimeVaryingDCMPlanner warmPlanner, coldPlanner;
    REQUIRE(warmPlanner.initialize(handler));
    REQUIRE(coldPlanner.initialize(cold));
    REQUIRE(warmPlanner.setContactPhaseLists(plans) && coldPlanner.setContactPhaseLists(plans));
    REQUIRE(warmPlanner.setInitialDCM(xi0) && coldPlanner.setInitialDCM(xi0));
    double itWarm = 0, itCold = 0, pWarm = 0, pCold = 0, maxDiff = 0;
    for (int step = 0; step < 40; ++step)
    {
        REQUIRE(warmPlanner.advance() && coldPlanner.advance());
        REQUIRE(warmPlanner.isValid() && coldPlanner.isValid());
        const DCMPlanBatch& a = warmPlanner.get();
        const DCMPlanBatch& c = coldPlanner.get();
        for (int b = 0; b < 16; ++b)
        {
            if (step == 0)
            {
                REQUIRE(a.iterations[b] == c.iterations[b]);
                REQUIRE(a.passes[b] == c.passes[b]);
            }
            else
            {
                itWarm += a.iterations[b];
                itCold += c.iterations[b];
                pWarm += a.passes[b];
                pCold += c.passes[b];
            }
        }
        for (std::size_t i = 0; i < a.vrp.size(); ++i)
            maxDiff = std::max(maxDiff, std::fabs(a.vrp[i] - c.vrp[i]));
        // re-anchor both on the same initial DCM so the windows pose the same QPs
        std::vector<std::array<double, 2>> x1;
        for (int b = 0; b < 16; ++b)
            x1.push_back({{c.dcm[(static_cast<std::size_t>(b) * 101 + 1) * 2],
                           c.dcm[(static_cast<std::size_t>(b) * 101 + 1) * 2 + 1]}});
        REQUIRE(warmPlanner.setInitialDCM(x1) && coldPlanner.setInitialDCM(x1));
    }
    // the active-set kernels certify every window with no interior point iteration either way; a
    // warm start (the shifted previous optimum and multipliers, fp64 passes only) needs far fewer
    // active-set passes than a cold one (the fp32 search, then the fp64 passes), and both land on
    // the same optimum (north_star's fp64 bar, 1e-9)
    REQUIRE(itWarm <= itCold);
    REQUIRE(pCold > 0);
    REQUIRE(pWarm < 0.8 * pCold);
    REQUIRE(maxDiff <= 1e-9);
    // the QP layout contract (VariablesHandlerTest.cpp:15-35): "dcm" then
    // "vrp", and the plan's variable rows read through it equal the dcm / vrp arrays
    {
        const VariablesHandler& vh = warmPlanner.variablesHandler();
        const IndexRange dcm = vh.getVariable("dcm"), vrp = vh.getVariable("vrp");
        REQUIRE(dcm.offset == 0 && dcm.size == 2 * 101);
        REQUIRE(vrp.offset == 2 * 101 && vrp.size == 2 * 100);
        REQUIRE(vh.getNumberOfVariables() == 4 * 100 + 2);
        REQUIRE_FALSE(vh.getVariable("com").isValid());
        const DCMPlanBatch& a = warmPlanner.get();
        const std::size_t n = vh.getNumberOfVariables();
        REQUIRE(a.variables.size() == 16 * n);
        bool same = true;
        for (int b = 0; b < 16; ++b)
            for (std::ptrdiff_t i = 0; i < vrp.size; ++i)
                same = same && a.variables[b * n + vrp.offset + i] == a.vrp[b * vrp.size + i] &&
                       (i >= dcm.size || a.variables[b * n + dcm.offset + i] == a.dcm[b * dcm.size + i]);
        REQUIRE(same);
    }
    // a window that runs past the plan's last phase is refused
    TimeVaryingDCMPlanner shortPlanner;
    auto longH = std::make_shared<ParametersHandler::StdImplementation>();
    longH->setParameter("horizon", 500);
    REQUIRE(shortPlanner.initialize(longH));
    REQUIRE(shortPlanner.setContactPhaseLists(plans) && shortPlanner.setInitialDCM(xi0));
    REQUIRE_FALSE(shortPlanner.advance());
    REQUIRE_FALSE(shortPlanner.isValid());
}

// Three active contacts: the lists of ContactPhaseListTest.cpp:32-47 (left, right, additional;
// phases [4, 5) and [6, 7) with all three), feet turned out and a hand support ahead, so the
// three-contact polygons need 9 facets: refused at max_facets 8, planned at max_facets 16.
static ContactPhaseList threeContactPlan(double dx)
{
    ContactList left, right, additional;
    left.setDefaultName("left");
    right.setDefaultName("right");
    additional.setDefaultName("additional");
    const Transform pl = Transform::fromPlanar(dx, 0.14, 1.50);
    const Transform pr = Transform::fromPlanar(dx, -0.14, -0.03);
    const Transform pa = Transform::fromPlanar(dx + 0.19, 0.0, 0.85);
    left.addContact(pl, 0.0, 1.0);
    left.addContact(pl, 2.0, 5.0);
    left.addContact(pl, 6.0, 7.0);
    right.addContact(pr, 0.0, 3.0);
    right.addContact(pr, 4.0, 7.0);
    additional.addContact(pa, 4.0, 5.0);
    additional.addContact(pa, 6.0, 7.5);
    ContactPhaseList plan;
    plan.setLists({left, right, additional});
    return plan;
}

static void testPlannerThreeContacts()
{
    std::vector<ContactPhaseList> plans;
    std::vector<std::array<double, 2>> xi0;
    for (int b = 0; b < 8; ++b)
    {
        plans.push_back(threeContactPlan(0.002 * b));
        xi0.push_back({{0.002 * b + 0.01, 0.12}});   // near the first phase's centre (left+right)
    }
    auto narrow = std::make_shared<ParametersHandler::StdImplementation>();
    narrow->setParameter("horizon", 60);
    narrow->setParameter("sampling_time", 0.1);
    TimeVaryingDCMPlanner p8;
    REQUIRE(p8.initialize(narrow));
    REQUIRE(p8.setContactPhaseLists(plans) && p8.setInitialDCM(xi0));
    REQUIRE_FALSE(p8.advance());   // a 9-facet polygon does not fit 8 facet slots
    REQUIRE_FALSE(p8.isValid());

    auto wide = std::make_shared<ParametersHandler::StdImplementation>();
    wide->setParameter("horizon", 60);
    wide->setParameter("sampling_time", 0.1);
    wide->setParameter("max_facets", 16);
    TimeVaryingDCMPlanner p16;
    REQUIRE(p16.initialize(wide));
    REQUIRE(p16.setContactPhaseLists(plans) && p16.setInitialDCM(xi0));
    for (int step = 0; step < 10; ++step)
    {
        REQUIRE(p16.advance());
        REQUIRE(p16.isValid());
        const DCMPlanBatch& plan = p16.get();
        REQUIRE(plan.batch == 8 && plan.horizon == 60);
        bool ok = true;
        for (int b = 0; b < 8; ++b)
        {
            ok = ok && plan.status[b] == 0;
            const double* xi = &plan.dcm[static_cast<std::size_t>(b) * 61 * 2];
            const double* r = &plan.vrp[static_cast<std::size_t>(b) * 60 * 2];
            for (int k = 0; k < 60; ++k)
                for (int j = 0; j < 2; ++j)
                {
                    const double w = std::sqrt(9.81 / 0.53);
                    const double nxt = xi[2 * k + j] + (w * xi[2 * k + j] + (-w) * r[2 * k + j]) * 0.1;
                    ok = ok && std::fabs(nxt - xi[2 * (k + 1) + j]) < 1e-12;
                }
        }
        REQUIRE(ok);
    }
    auto bad = std::make_shared<ParametersHandler::StdImplementation>();
    bad->setParameter("max_facets", 17);
    TimeVaryingDCMPlanner pBad;
    REQUIRE_FALSE(pBad.initialize(bad));
}


// ---- ContinousContactModelTest.cpp:30-214 ------------------------------------------------------
static blf::Matrix3 rpy(double r, double p, double y)   // iDynTree Rotation::RPY = Rz(y) Ry(p) Rx(r)
{
    const double cr = std::cos(r), sr = std::sin(r), cp = std::cos(p), sp = std::sin(p);
    const double cy = std::cos(y), sy = std::sin(y);
    return {{cy * cp, cy * sp * sr - sy * cr, cy * sp * cr + sy * sr,
             sy * cp, sy * sp * sr + cy * cr, sy * sp * cr - cy * sr,
             -sp, cp * sr, cp * cr}};
}

static blf::Matrix3 expSkew(const blf::Vector3& v)   // Rodrigues
{
    const double th = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
    blf::Matrix3 K{{0, -v[2], v[1], v[2], 0, -v[0], -v[1], v[0], 0}}, K2{}, R{};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) K2[3 * i + j] += K[3 * i + k] * K[3 * k + j];
    const double a = th > 0 ? std::sin(th) / th : 1.0, b = th > 0 ? (1 - std::cos(th)) / (th * th) : 0.5;
    for (int i = 0; i < 9; ++i) R[i] = (i % 4 == 0 ? 1.0 : 0.0) + a * K[i] + b * K2[i];
    return R;
}

static blf::Matrix3 matmul(const blf::Matrix3& A, const blf::Matrix3& B)
{
    blf::Matrix3 C{};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) C[3 * i + j] += A[3 * i + k] * B[3 * k + j];
    return C;
}

static void testContinuousContact()
{
    using ContactModels::ContinuousContactModel;
    blf::Transform world_T_link;
    world_T_link.rotation = rpy(-0.15, 0.2, 0.1);
    world_T_link.position = {{-0.02, 0.01, 0.005}};
    const blf::Transform nullForceTransform = blf::Transform::Identity();
    std::mt19937 rng(7);
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    blf::Twist linkVelocity;
    for (auto& x : linkVelocity) x = u(rng);
    constexpr double springCoeff = 2000.0, damperCoeff = 100.0, length = 0.12, width = 0.09;
    auto handler = std::make_shared<ParametersHandler::StdImplementation>();
    handler->setParameter("spring_coeff", springCoeff);
    handler->setParameter("damper_coeff", damperCoeff);
    handler->setParameter("length", length);
    handler->setParameter("width", width);

    ContinuousContactModel model;
    REQUIRE(model.initialize(handler));
    model.setState(linkVelocity, world_T_link);
    model.setNullForceTransform(nullForceTransform);

    {   // "Test contact wrench": Monte Carlo integral of the point forces, tol 1e-2
        std::default_random_engine generator;
        generator.seed(42);
        std::uniform_real_distribution<double> xAxis(-length / 2, length / 2), yAxis(-width / 2, width / 2);
        const unsigned samples = 10000;
        std::vector<double> pts(2 * samples), f, t;
        for (unsigned i = 0; i < samples; ++i)
        {
            pts[2 * i] = xAxis(generator);
            pts[2 * i + 1] = yAxis(generator);
        }
        REQUIRE(model.getWrenchesAtPoints(pts, f, t));
        const double scale = length * width * std::abs(world_T_link.rotation[8]) / samples;
        const blf::Wrench& w = model.getContactWrench();
        for (int i = 0; i < 3; ++i)
        {
            double F = 0.0, T = 0.0;
            for (unsigned k = 0; k < samples; ++k) { F += f[3 * k + i]; T += t[3 * k + i]; }
            REQUIRE(std::abs(F * scale - w[i]) <= 1e-2);
            REQUIRE(std::abs(T * scale - w[3 + i]) <= 1e-2);
        }
        // single-point getters agree with the batched call
        const blf::Vector3 f0 = model.getForceAtPoint(pts[0], pts[1]);
        const blf::Vector3 t0 = model.getTorqueGeneratedAtPoint(pts[0], pts[1]);
        for (int i = 0; i < 3; ++i) REQUIRE(f0[i] == f[i] && t0[i] == t[i]);
        const blf::Vector3 out = model.getForceAtPoint(length, 0.0);
        REQUIRE(out[0] == 0.0 && out[1] == 0.0 && out[2] == 0.0);
    }
    {   // "Test regressor", tol 1e-7
        const blf::MatrixXd& reg = model.getRegressor();
        const blf::Wrench& w = model.getContactWrench();
        for (int i = 0; i < 6; ++i)
            REQUIRE(std::abs(reg(i, 0) * springCoeff + reg(i, 1) * damperCoeff - w[i]) <= 1e-7);
    }
    {   // cache protocol (ContactModel.cpp:12-92): cached until the state changes
        const blf::Wrench w1 = model.getContactWrench();
        const blf::Wrench* p1 = &model.getContactWrench();
        REQUIRE(p1 == &model.getContactWrench() && *p1 == w1);
        blf::Twist other = linkVelocity;
        other[0] += 0.5;
        model.setState(other, world_T_link);
        REQUIRE(model.getContactWrench()[0] != w1[0]);
        model.setState(linkVelocity, world_T_link);
        REQUIRE(model.getContactWrench() == w1);
        model.damperCoeff() = 0.0;           // the accessors do not invalidate (as the reference)
        REQUIRE(model.getContactWrench() == w1);
        model.setNullForceTransform(nullForceTransform);
        REQUIRE(model.getContactWrench()[0] != w1[0]);
        model.damperCoeff() = damperCoeff;
        model.setNullForceTransform(nullForceTransform);
    }
    {   // "Test contact dynamics": FD of the wrench vs autonomous + control * acc, tol 1e-4
        const double h = 1e-6;
        blf::Vector6 acc;
        acc.fill(1.0);
        blf::Vector6 rate = model.getAutonomousDynamics();
        const blf::Matrix6x6& C = model.getControlMatrix();
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) rate[i] += C[6 * i + j] * acc[j];
        blf::Wrench w[2];
        for (int s = 0; s < 2; ++s)
        {
            const double sg = s == 0 ? -1.0 : 1.0;
            blf::Transform T = world_T_link;
            for (int i = 0; i < 3; ++i) T.position[i] += sg * linkVelocity[i] * h;
            T.rotation = matmul(expSkew({{sg * linkVelocity[3] * h, sg * linkVelocity[4] * h,
                                          sg * linkVelocity[5] * h}}), world_T_link.rotation);
            blf::Twist v = linkVelocity;
            for (int i = 0; i < 6; ++i) v[i] += sg * acc[i] * h;
            model.setState(v, T);
            model.setNullForceTransform(nullForceTransform);
            w[s] = model.getContactWrench();
        }
        for (int i = 0; i < 6; ++i) REQUIRE(std::abs((w[1][i] - w[0][i]) / (2 * h) - rate[i]) <= 1e-4);
    }
    {   // missing parameter
        auto bad = std::make_shared<ParametersHandler::StdImplementation>();
        bad->setParameter("length", length);
        ContinuousContactModel m2;
        REQUIRE_FALSE(m2.initialize(bad));
    }
}

// ---- FloatingBaseSystemKinematics under ForwardEuler (FloatingBaseSystemKinematics.cpp:36-73) ---
static void testFloatingBaseKinematics()
{
    auto system = std::make_shared<FloatingBaseSystemKinematics>();
    auto handler = std::make_shared<ParametersHandler::StdImplementation>();
    handler->setParameter("rho", 0.01);
    REQUIRE(system->initalize(handler));
    const blf::Matrix3 R0 = rpy(0.1, -0.2, 0.3);
    blf::VectorXd s(24, 0.0), sd(24, 0.0);
    for (int i = 0; i < 24; ++i) sd[i] = 0.1 * i - 1.0;
    const blf::Vector6 twist{{0.1, -0.2, 0.05, 0.3, -0.1, 0.2}};
    REQUIRE(system->setState({blf::Vector3{{0.0, 0.0, 0.53}}, R0, s}));
    REQUIRE(system->setControlInput({twist, sd}));
    FloatingBaseSystemKinematics::StateDerivativeType dx;
    REQUIRE(system->dynamics(0.0, dx));
    const auto& [dp, dR, ds] = dx;
    const blf::Matrix3 W{{0, -twist[5], twist[4], twist[5], 0, -twist[3], -twist[4], twist[3], 0}};
    const blf::Matrix3 WR = matmul(W, R0);
    for (int i = 0; i < 3; ++i) REQUIRE(dp[i] == twist[i]);
    for (int i = 0; i < 9; ++i) REQUIRE(std::abs(dR[i] - WR[i]) < 1e-14);   // orthonormal R
    for (int i = 0; i < 24; ++i) REQUIRE(ds[i] == sd[i]);

    ForwardEuler<FloatingBaseSystemKinematics> integrator(1e-4);
    REQUIRE(integrator.setDynamicalSystem(system));
    const double T = 0.5;
    for (int k = 0; k < 5; ++k) REQUIRE(integrator.integrate(0.1 * k, 0.1 * (k + 1)));
    const auto& [p, R, q] = integrator.getSolution();
    // the stale-time last step adds one dT per call: t_eff = T + 5 dT
    const double te = T + 5 * 1e-4;
    REQUIRE(std::abs(p[2] - (0.53 + twist[2] * te)) < 1e-12);
    REQUIRE(std::abs(q[23] - sd[23] * te) < 1e-12);
    const blf::Matrix3 Rex = matmul(expSkew({{twist[3] * te, twist[4] * te, twist[5] * te}}), R0);
    for (int i = 0; i < 9; ++i) REQUIRE(std::abs(R[i] - Rex[i]) < 1e-4);
    // wrong sizes
    REQUIRE(system->setControlInput({twist, blf::VectorXd(3, 0.0)}));
    REQUIRE_FALSE(system->dynamics(0.0, dx));
}

// ---- IntegratorTest.cpp:77-126, "Floating base System Kinematics", restated literally ----------
// Random twist and 20 joint velocities (Eigen setRandom: uniform in [-1, 1]; here a seeded
// std::mt19937), identity rotation, zero position and joints, ForwardEuler at dT = 1e-4 called as
// integrate(0, dT) once per step for simulationTime = 2 s, every step's solution isApprox
// (Frobenius norms, Eigen's definition) the closed form at tolerance 1e-3: position p0 + t v,
// rotation AngleAxis(|w| t, w / |w|) R0, joints s0 + t sdot.
template <class A, class B>
static bool isApprox(const A& a, const B& b, double prec)
{
    double d = 0.0, na = 0.0, nb = 0.0;
    for (size_t i = 0; i < a.size(); ++i) {
        d += (a[i] - b[i]) * (a[i] - b[i]);
        na += a[i] * a[i];
        nb += b[i] * b[i];
    }
    return d <= prec * prec * std::min(na, nb);
}

static void testIntegratorKinematicsLiteral()
{
    constexpr double dT = 0.0001;
    constexpr double tolerance = 1e-3;
    constexpr double simulationTime = 2;
    auto system = std::make_shared<FloatingBaseSystemKinematics>();
    std::mt19937 gen(20201015);
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    blf::Vector6 twist;
    for (auto& v : twist) v = U(gen);
    blf::VectorXd jointVelocity(20);
    for (std::size_t i = 0; i < jointVelocity.size(); ++i) jointVelocity[i] = U(gen);
    const blf::Matrix3 rotation0{{1, 0, 0, 0, 1, 0, 0, 0, 1}};
    const blf::Vector3 position0{{0.0, 0.0, 0.0}};
    const blf::VectorXd jointPosition0(20, 0.0);
    const double wn = std::sqrt(twist[3] * twist[3] + twist[4] * twist[4] + twist[5] * twist[5]);
    auto closeFormSolution = [&](double t, blf::Vector3& pos, blf::Matrix3& rot, blf::VectorXd& q) {
        for (int i = 0; i < 3; ++i) pos[i] = position0[i] + t * twist[i];
        // AngleAxis(|w| t, w / |w|) = exp(skew(w t))
        rot = matmul(expSkew({{twist[3] / wn * (wn * t), twist[4] / wn * (wn * t), twist[5] / wn * (wn * t)}}),
                     rotation0);
        q.resize(20);
        for (int i = 0; i < 20; ++i) q[i] = jointPosition0[i] + t * jointVelocity[i];
    };
    REQUIRE(system->setControlInput({twist, jointVelocity}));
    REQUIRE(system->setState({position0, rotation0, jointPosition0}));
    ForwardEuler<FloatingBaseSystemKinematics> integrator(dT);
    REQUIRE(integrator.setDynamicalSystem(system));
    int bad = 0, steps = 0;
    for (int i = 0; i < simulationTime / dT; i++) {
        const auto& [basePosition, baseRotation, jointPosition] = integrator.getSolution();
        blf::Vector3 pe;
        blf::Matrix3 Re;
        blf::VectorXd qe;
        closeFormSolution(dT * i, pe, Re, qe);
        // one aggregate check per step, so a failure does not print 20 000 lines
        if (!isApprox(baseRotation, Re, tolerance) || !isApprox(basePosition, pe, tolerance)
            || !isApprox(jointPosition, qe, tolerance))
            ++bad;
        if (!integrator.integrate(0, dT)) ++bad;
        ++steps;
    }
    REQUIRE(steps == 20000);
    REQUIRE(bad == 0);
}

// ---- FloatingBaseDynamicalSystem (FloatingBaseSystemDynamics.cpp:102-251) on a 3-joint chain ---
static blf::RobotModel chainModel()
{
    blf::RobotModel m;
    m.ndof = 3;
    m.parent = {0, 1, 2};
    m.jointOrigin = {0.0, 0.0, -0.1, 0.0, 0.0, -0.3, 0.0, 0.0, -0.3};
    m.jointRotation.clear();
    for (int j = 0; j < 3; ++j) m.jointRotation.insert(m.jointRotation.end(), {1, 0, 0, 0, 1, 0, 0, 0, 1});
    m.jointAxis = {1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 1.0, 0.0};
    m.linkMass = {5.0, 2.0, 1.5, 1.0};
    m.linkCom = {0.0, 0.0, 0.0, 0.0, 0.0, -0.15, 0.0, 0.0, -0.15, 0.05, 0.0, -0.02};
    m.linkInertia.clear();
    for (double mass : m.linkMass)
        m.linkInertia.insert(m.linkInertia.end(), {0.01 * mass, 0, 0, 0, 0.012 * mass, 0, 0, 0, 0.008 * mass});
    m.frameLink = {3};
    m.framePose = {0.02, 0.0, -0.05, 1, 0, 0, 0, 1, 0, 0, 0, 1};
    return m;
}

static void testFloatingBaseDynamics()
{
    auto system = std::make_shared<FloatingBaseDynamicalSystem>();
    auto handler = std::make_shared<ParametersHandler::StdImplementation>();
    handler->setParameter("rho", 0.01);
    REQUIRE(system->initalize(handler));
    REQUIRE(system->setRobotModel(chainModel()));
    const blf::Matrix3 R0 = rpy(0.05, -0.1, 0.2);
    blf::VectorXd zero3(3, 0.0), q(3, 0.0);
    q[0] = 0.2; q[1] = -0.4; q[2] = 0.3;
    // free fall: nu = 0, tau = 0, no contacts -> base acceleration = g, joints at rest
    REQUIRE(system->setState({blf::Vector6{}, zero3, blf::Vector3{{0.0, 0.0, 1.0}}, R0, q}));
    REQUIRE(system->setControlInput({zero3, {}}));
    FloatingBaseDynamicalSystem::StateDerivativeType dx;
    REQUIRE(system->dynamics(0.0, dx));
    const auto& [ba, ja, dp, dR, dq] = dx;
    REQUIRE(std::abs(ba[2] + 9.81) < 1e-10);
    for (int i : {0, 1, 3, 4, 5}) REQUIRE(std::abs(ba[i]) < 1e-10);
    for (int i = 0; i < 3; ++i) REQUIRE(std::abs(ja[i]) < 1e-10);
    // ForwardEuler free fall: v_k = g k dT, z_k = z0 + g dT^2 k (k - 1) / 2 (k = number of steps)
    ForwardEuler<FloatingBaseDynamicalSystem> integrator(0.01);
    REQUIRE(integrator.setDynamicalSystem(system));
    REQUIRE(integrator.integrate(0.0, 0.1));
    const auto& [bv, jv, bp, bR, jp] = integrator.getSolution();
    // the FixedStepIntegrator schedule: ceil((T - t0) / dT) calls, the last one with the stale time
    const int iterations = static_cast<int>(std::ceil((0.1 - 0.0) / 0.01));
    const double last = 0.1 - (iterations >= 2 ? 0.01 * (iterations - 2) : 0.0);
    double v = 0.0, z = 1.0;
    for (int k = 0; k < iterations; ++k)
    {
        const double h = k + 1 < iterations ? 0.01 : last;
        z += v * h;
        v += -9.81 * h;
    }
    REQUIRE(std::abs(bv[2] - v) < 1e-10 && std::abs(bp[2] - z) < 1e-10);
    // the foot (z ~ 0.25) is below the null-force height 0.5: the contact pushes the robot up
    auto contact = std::make_shared<ContactModels::ContinuousContactModel>();
    auto cp = std::make_shared<ParametersHandler::StdImplementation>();
    cp->setParameter("length", 0.12);
    cp->setParameter("width", 0.09);
    cp->setParameter("spring_coeff", 3.0e4);
    cp->setParameter("damper_coeff", 300.0);
    REQUIRE(contact->initialize(cp));
    blf::Transform nullT;
    nullT.position = {{0.0, 0.0, 0.5}};
    contact->setNullForceTransform(nullT);
    REQUIRE(system->setState({blf::Vector6{}, zero3, blf::Vector3{{0.0, 0.0, 1.0}}, R0, q}));
    REQUIRE(system->setControlInput({zero3, {ContactWrench(0, contact)}}));
    REQUIRE(system->dynamics(0.0, dx));
    REQUIRE(std::isfinite(std::get<0>(dx)[2]) && std::get<0>(dx)[2] > -9.81 + 1e-3);   // pushed up
    // wrong sizes and a missing model are refused
    REQUIRE(system->setControlInput({blf::VectorXd(2, 0.0), {}}));
    REQUIRE_FALSE(system->dynamics(0.0, dx));
    FloatingBaseDynamicalSystem empty;
    REQUIRE_FALSE(empty.dynamics(0.0, dx));
    REQUIRE_FALSE(empty.setMassMatrixRegularization(blf::MatrixXd(9, 9)));
    REQUIRE_FALSE(system->setMassMatrixRegularization(blf::MatrixXd(8, 8)));
    REQUIRE(system->setMassMatrixRegularization(blf::MatrixXd(9, 9)));
}

// A ContactModel the kernel does not know (BLF_CONTACT_WRENCH): it forwards to a
// ContinuousContactModel, so the dynamics must equal the device law's, and it counts the
// setState calls (one per dynamics() and per Euler step, FloatingBaseSystemDynamics.cpp:225).
class ForwardingContact final : public ContactModels::ContactModel
{
    std::shared_ptr<ContactModels::ContinuousContactModel> m_inner;

    void computeContactWrench() final { m_contactWrench = m_inner->getContactWrench(); }
    void computeAutonomousDynamics() final { m_autonomousDynamics = m_inner->getAutonomousDynamics(); }
    void computeControlMatrix() final { m_controlMatrix = m_inner->getControlMatrix(); }
    void computeRegressor() final { m_regressor = m_inner->getRegressor(); }
    bool initializePrivate(std::weak_ptr<ParametersHandler::IParametersHandler> handler) final
    {
        return m_inner->initialize(handler);
    }
    void setStatePrivate(const blf::Twist& twist, const blf::Transform& transform) final
    {
        ++states;
        m_inner->setState(twist, transform);
    }
    void setNullForceTransformPrivate(const blf::Transform& transform) final
    {
        m_inner->setNullForceTransform(transform);
    }

public:
    int states{0};
    ForwardingContact() : m_inner(std::make_shared<ContactModels::ContinuousContactModel>()) {}
};

static void testFloatingBaseDynamicsAnyContactModel()
{
    auto params = std::make_shared<ParametersHandler::StdImplementation>();
    params->setParameter("length", 0.12);
    params->setParameter("width", 0.09);
    params->setParameter("spring_coeff", 3.0e4);
    params->setParameter("damper_coeff", 300.0);
    params->setParameter("rho", 0.01);
    blf::Transform nullT;
    nullT.position = {{0.01, -0.02, 0.5}};
    auto continuous = std::make_shared<ContactModels::ContinuousContactModel>();
    auto forwarding = std::make_shared<ForwardingContact>();
    auto second = std::make_shared<ContactModels::ContinuousContactModel>();
    for (ContactModels::ContactModel* c : {static_cast<ContactModels::ContactModel*>(continuous.get()),
                                           static_cast<ContactModels::ContactModel*>(forwarding.get()),
                                           static_cast<ContactModels::ContactModel*>(second.get())})
    {
        REQUIRE(c->initialize(params));
        c->setNullForceTransform(nullT);
    }
    const blf::Matrix3 R0 = rpy(0.05, -0.1, 0.2);
    blf::VectorXd tau(3, 0.0), q(3, 0.0), qd(3, 0.0);
    q[0] = 0.2; q[1] = -0.4; q[2] = 0.3;
    qd[0] = 0.3; qd[1] = -0.2; qd[2] = 0.5;
    tau[0] = 1.0; tau[2] = -0.5;
    const blf::Vector6 nu{{0.1, -0.05, -0.2, 0.3, 0.1, -0.2}};
    auto device = std::make_shared<FloatingBaseDynamicalSystem>();
    auto mixed = std::make_shared<FloatingBaseDynamicalSystem>();
    for (auto& s : {device, mixed})
    {
        REQUIRE(s->initalize(params));
        REQUIRE(s->setRobotModel(chainModel()));
        REQUIRE(s->setState({nu, qd, blf::Vector3{{0.0, 0.0, 0.85}}, R0, q}));
    }
    // the same two ContinuousContactModel wrenches on frame 0: both on the device, or one of them
    // through the forwarding model (its wrench evaluated on the host at the device's frame state)
    REQUIRE(device->setControlInput({tau, {ContactWrench(0, continuous), ContactWrench(0, second)}}));
    REQUIRE(mixed->setControlInput({tau, {ContactWrench(0, forwarding), ContactWrench(0, second)}}));
    FloatingBaseDynamicalSystem::StateDerivativeType d0, d1;
    REQUIRE(device->dynamics(0.0, d0));
    REQUIRE(mixed->dynamics(0.0, d1));
    REQUIRE(forwarding->states == 1);
    double scale = 0.0, diff = 0.0;
    for (int i = 0; i < 6; ++i)
    {
        scale = std::max(scale, std::abs(std::get<0>(d0)[i]));
        diff = std::max(diff, std::abs(std::get<0>(d0)[i] - std::get<0>(d1)[i]));
    }
    for (int j = 0; j < 3; ++j) diff = std::max(diff, std::abs(std::get<1>(d0)[j] - std::get<1>(d1)[j]));
    REQUIRE(scale > 1.0 && diff <= 1e-10 * scale);   // the contacts act (|base acc| >> 0) and agree
    // dynamics() leaves every contact model in its frame's state (the reference's side effect):
    // the device-evaluated model and the forwarded one now report the same wrench
    const blf::Wrench wc = continuous->getContactWrench(), wf = forwarding->getContactWrench();
    for (int i = 0; i < 6; ++i) REQUIRE(std::abs(wc[i] - wf[i]) <= 1e-9 * (1.0 + std::abs(wc[i])));
    // ForwardEuler: one host evaluation per step (5 steps), the same trajectory as the device law's
    ForwardEuler<FloatingBaseDynamicalSystem> e0(0.01), e1(0.01);
    REQUIRE(e0.setDynamicalSystem(device) && e1.setDynamicalSystem(mixed));
    REQUIRE(e0.integrate(0.0, 0.05) && e1.integrate(0.0, 0.05));
    REQUIRE(forwarding->states == 1 + 5);
    const auto& s0 = e0.getSolution();
    const auto& s1 = e1.getSolution();
    double sd = 0.0;
    for (int i = 0; i < 6; ++i) sd = std::max(sd, std::abs(std::get<0>(s0)[i] - std::get<0>(s1)[i]));
    for (int i = 0; i < 3; ++i)
    {
        sd = std::max(sd, std::abs(std::get<1>(s0)[i] - std::get<1>(s1)[i]));
        sd = std::max(sd, std::abs(std::get<4>(s0)[i] - std::get<4>(s1)[i]));
        sd = std::max(sd, std::abs(std::get<2>(s0)[i] - std::get<2>(s1)[i]));
    }
    REQUIRE(sd <= 1e-9);
    // a final time dT does not divide: the reference's schedule (ceil((T - t0) / dT) steps, the
    // last one with the stale time, FixedStepIntegrator.tpp:48-64) in the step-by-step path too
    ForwardEuler<FloatingBaseDynamicalSystem> f0(0.01), f1(0.01);
    REQUIRE(f0.setDynamicalSystem(device) && f1.setDynamicalSystem(mixed));
    const int before = forwarding->states;
    REQUIRE(f0.integrate(0.05, 0.095) && f1.integrate(0.05, 0.095));
    REQUIRE(forwarding->states == before + 5);   // ceil(0.045 / 0.01) steps, one evaluation each
    const auto& u0 = f0.getSolution();
    const auto& u1 = f1.getSolution();
    double ud = 0.0;
    for (int i = 0; i < 6; ++i) ud = std::max(ud, std::abs(std::get<0>(u0)[i] - std::get<0>(u1)[i]));
    for (int i = 0; i < 3; ++i) ud = std::max(ud, std::abs(std::get<2>(u0)[i] - std::get<2>(u1)[i]));
    REQUIRE(ud <= 1e-9);
    // a contact without a model is refused (ContactWrench owns its model, as the reference's)
    REQUIRE(mixed->setControlInput({tau, {ContactWrench(0, nullptr)}}));
    REQUIRE_FALSE(mixed->dynamics(0.0, d1));
}

// ---- fixed joints (blf::reduceFixedJoints): host-only checks of the merge -------------------------
// Whole-body mass and centre of mass at q = 0 (base at the origin) of a model, by a forward pass.
static std::array<double, 4> massAndCom(const blf::RobotModel& m)
{
    std::vector<std::array<double, 9>> R(m.ndof + 1);
    std::vector<std::array<double, 3>> p(m.ndof + 1);
    R[0] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    p[0] = {0, 0, 0};
    for (int j = 0; j < m.ndof; ++j)
    {
        const int P = m.parent[j], c = j + 1;
        for (int r = 0; r < 3; ++r)
        {
            p[c][r] = p[P][r];
            for (int k = 0; k < 3; ++k)
            {
                p[c][r] += R[P][3 * r + k] * m.jointOrigin[3 * j + k];
                R[c][3 * r + k] = 0.0;
                for (int l = 0; l < 3; ++l) R[c][3 * r + k] += R[P][3 * r + l] * m.jointRotation[9 * j + 3 * l + k];
            }
        }
    }
    std::array<double, 4> out{0, 0, 0, 0};
    for (int l = 0; l <= m.ndof; ++l)
    {
        out[0] += m.linkMass[l];
        for (int r = 0; r < 3; ++r)
        {
            double c = p[l][r];
            for (int k = 0; k < 3; ++k) c += R[l][3 * r + k] * m.linkCom[3 * l + k];
            out[1 + r] += m.linkMass[l] * c;
        }
    }
    for (int r = 0; r < 3; ++r) out[1 + r] /= out[0];
    return out;
}

static void testFixedJoints()
{
    {   // inconsistent models come back unchanged: non-topological, wrong sizes
        blf::RobotModel bad = chainModel();
        bad.fixedJoint = {0, 1, 0};
        bad.parent = {0, 2, 1};
        REQUIRE_FALSE(blf::fixedJointMergeable(bad));
        REQUIRE(blf::reduceFixedJoints(bad).fixedJoint.size() == 3);
        bad = chainModel();
        bad.fixedJoint = {0, 1, 0};
        bad.linkMass.pop_back();
        REQUIRE_FALSE(blf::fixedJointMergeable(bad));
        REQUIRE(blf::reduceFixedJoints(bad).ndof == 3);
    }
    blf::RobotModel full = chainModel();
    const blf::Matrix3 E1 = rpy(0.1, -0.2, 0.3);
    for (int k = 0; k < 9; ++k) full.jointRotation[9 + k] = E1[k];   // joint 1 mounted with a rotation
    full.fixedJoint = {0, 1, 1};                                     // joints 1 and 2 (a chain) fixed
    const blf::RobotModel red = blf::reduceFixedJoints(full);
    REQUIRE(red.ndof == 1 && red.parent.size() == 1 && red.linkMass.size() == 2 && red.fixedJoint.empty());
    REQUIRE(red.frameLink.size() == 1 && red.frameLink[0] == 1);   // the sole frame moved onto link 1
    const auto a = massAndCom(full), b = massAndCom(red);
    for (int i = 0; i < 4; ++i) REQUIRE(std::abs(a[i] - b[i]) < 1e-14);
    // the merged inertia stays symmetric positive definite
    const double* I = &red.linkInertia[9];
    REQUIRE(std::abs(I[1] - I[3]) < 1e-15 && std::abs(I[2] - I[6]) < 1e-15 && std::abs(I[5] - I[7]) < 1e-15);
    REQUIRE(I[0] > 0 && I[0] * I[4] - I[1] * I[3] > 0);
    // no fixed joint: unchanged; a malformed mask is refused by setRobotModel
    blf::RobotModel none = chainModel();
    none.fixedJoint = {0, 0, 0};
    REQUIRE(blf::reduceFixedJoints(none).ndof == 3);
    FloatingBaseDynamicalSystem sys;
    blf::RobotModel bad = chainModel();
    bad.fixedJoint = {1};
    REQUIRE_FALSE(sys.setRobotModel(bad));
}

static void testFixedJointsDevice()
{
    // the adapter merges on setRobotModel: one DoF left, free fall as for any model
    blf::RobotModel full = chainModel();
    full.fixedJoint = {0, 1, 1};
    auto system = std::make_shared<FloatingBaseDynamicalSystem>();
    auto handler = std::make_shared<ParametersHandler::StdImplementation>();
    handler->setParameter("rho", 0.01);
    REQUIRE(system->initalize(handler));
    REQUIRE(system->setRobotModel(full));
    blf::VectorXd one(1, 0.0), q(1, 0.2);
    REQUIRE(system->setState({blf::Vector6{}, one, blf::Vector3{{0.0, 0.0, 1.0}}, rpy(0.05, -0.1, 0.2), q}));
    REQUIRE(system->setControlInput({one, {}}));
    FloatingBaseDynamicalSystem::StateDerivativeType dx;
    REQUIRE(system->dynamics(0.0, dx));
    REQUIRE(std::get<1>(dx).size() == 1);
    REQUIRE(std::abs(std::get<0>(dx)[2] + 9.81) < 1e-10 && std::abs(std::get<1>(dx)[0]) < 1e-10);
    REQUIRE(system->setControlInput({blf::VectorXd(3, 0.0), {}}));   // the full model's size: refused
    REQUIRE_FALSE(system->dynamics(0.0, dx));
    // a prismatic middle joint (RobotModel::jointType): free fall as well; unknown types refused
    blf::RobotModel pri = chainModel();
    pri.jointType = {BLF_JOINT_REVOLUTE, BLF_JOINT_PRISMATIC, BLF_JOINT_REVOLUTE};
    REQUIRE(system->setRobotModel(pri));
    blf::VectorXd z3(3, 0.0), q3(3, 0.1);
    REQUIRE(system->setState({blf::Vector6{}, z3, blf::Vector3{{0.0, 0.0, 1.0}}, rpy(0.05, -0.1, 0.2), q3}));
    REQUIRE(system->setControlInput({z3, {}}));
    REQUIRE(system->dynamics(0.0, dx));
    REQUIRE(std::abs(std::get<0>(dx)[2] + 9.81) < 1e-10);
    for (int i = 0; i < 3; ++i) REQUIRE(std::abs(std::get<1>(dx)[i]) < 1e-10);
    pri.jointType = {0, 2, 0};
    REQUIRE_FALSE(system->setRobotModel(pri));
    pri.jointType = {0, 1};
    REQUIRE_FALSE(system->setRobotModel(pri));
}

// ---- ParametersHandlerYarpTest.cpp:30-140, on the reference's tests/config.ini -----------------
static std::string g_golden = "tests/golden";

static void testParametersHandler()
{
    using namespace ParametersHandler;
    auto handler = std::make_shared<StdImplementation>();
    REQUIRE(handler->setFromFile(g_golden + "/parameters_config.ini"));
    int answer = 0;
    REQUIRE(handler->getParameter("answer_to_the_ultimate_question_of_life", answer));
    REQUIRE(answer == 42);
    double pi = 0.0;
    REQUIRE(handler->getParameter("pi", pi));
    REQUIRE(pi == 3.14);
    std::string john;
    REQUIRE(handler->getParameter("John", john));
    REQUIRE(john == "Smith");
    REQUIRE_FALSE(handler->getParameter("pi", answer));   // 3.14 is not an integer
    handler->setParameter("John", "Doe");
    REQUIRE(handler->getParameter("John", john));
    REQUIRE(john == "Doe");
    const std::vector<int> fibonacci = {1, 1, 2, 3, 5, 8, 13, 21};
    std::vector<int> fib;
    REQUIRE(handler->getParameter("Fibonacci Numbers", fib));
    REQUIRE(fib == fibonacci);
    const std::vector<int> more = {21, 34, 55};
    handler->setParameter("Fibonacci Numbers", more);
    REQUIRE(handler->getParameter("Fibonacci Numbers", fib));
    REQUIRE(fib == more);

    // the [CARTOONS] section is a group
    auto cartoons = handler->getGroup("CARTOONS").lock();
    REQUIRE(cartoons);
    if (cartoons)
    {
        std::vector<std::string> nephews;
        REQUIRE(cartoons->getParameter("Donald's nephews", nephews));
        REQUIRE((nephews == std::vector<std::string>{"Huey", "Dewey", "Louie"}));
        REQUIRE(cartoons->getParameter("Fibonacci_Numbers", fib));
        REQUIRE(fib == fibonacci);
        REQUIRE(cartoons->getParameter("John", john));
        REQUIRE(john == "Doe");
    }
    REQUIRE(handler->toString().find("CARTOONS") != std::string::npos);

    // is Empty / set group / clear
    auto fresh = std::make_shared<StdImplementation>();
    REQUIRE_FALSE(fresh->getGroup("CARTOONS").lock());
    auto group = std::make_shared<StdImplementation>();
    REQUIRE(fresh->setGroup("CARTOONS", group));
    REQUIRE(fresh->getGroup("CARTOONS").lock());
    REQUIRE(group->isEmpty());
    group->setParameter("value", 10);
    REQUIRE_FALSE(group->isEmpty());
    REQUIRE_FALSE(handler->isEmpty());
    handler->clear();
    REQUIRE(handler->isEmpty());
    REQUIRE_FALSE(fresh->setGroup("null", nullptr));

    // the keys the DCM path reads, from a file
    auto cfg = std::make_shared<StdImplementation>();
    REQUIRE(cfg->setFromString("// contact model\nlength 0.12\nwidth 0.09 # m\nspring_coeff 2000\n"
                               "damper_coeff 100\nrho 0.01\nw_xi (100, 100)\nflag true\n"));
    double len = 0.0, k = 0.0, rho = 0.0;
    bool flag = false;
    std::vector<double> wxi;
    REQUIRE(cfg->getParameter("length", len) && len == 0.12);
    REQUIRE(cfg->getParameter("spring_coeff", k) && k == 2000.0);
    REQUIRE(cfg->getParameter("rho", rho) && rho == 0.01);
    REQUIRE(cfg->getParameter("w_xi", wxi) && wxi.size() == 2 && wxi[1] == 100.0);
    REQUIRE(cfg->getParameter("flag", flag) && flag);
    ContactModels::ContinuousContactModel model;
    REQUIRE(model.initialize(cfg));
    REQUIRE_FALSE(StdImplementation().setFromFile(g_golden + "/does_not_exist.ini"));
    REQUIRE_FALSE(cfg->setFromString("key (1, 2"));
    REQUIRE(cfg->isEmpty());
}

// `blf_host_tests urdf <file> [frames] [considered] [base]` (comma-separated lists; "-" for none,
// "*" for "every moving joint"): the C++ loader's model as JSON, for
// tests/test_host_cpp.py::test_cpp_urdf_loader_matches_python.
static std::vector<std::string> splitList(const std::string& s)
{
    std::vector<std::string> out;
    if (s == "-" || s.empty()) return out;
    std::size_t b = 0;
    for (;;)
    {
        const std::size_t e = s.find(',', b);
        out.push_back(s.substr(b, e == std::string::npos ? std::string::npos : e - b));
        if (e == std::string::npos) return out;
        b = e + 1;
    }
}

static int dumpUrdf(int argc, char** argv)
{
    if (argc < 3) return 2;
    blf::UrdfOptions opt;
    if (argc > 3) opt.frames = splitList(argv[3]);
    if (argc > 4 && std::string(argv[4]) != "*")
    {
        opt.hasConsideredJoints = true;
        opt.consideredJoints = splitList(argv[4]);
    }
    if (argc > 5 && std::string(argv[5]) != "-") opt.base = argv[5];
    blf::RobotModel m;
    std::vector<std::string> names;
    std::string err;
    if (!blf::loadUrdf(argv[2], opt, m, &names, &err))
    {
        std::printf("{\"error\": \"%s\"}\n", err.c_str());
        return 1;
    }
    auto arr = [](const char* key, const auto& v, bool last = false) {
        std::printf("\"%s\": [", key);
        for (std::size_t i = 0; i < v.size(); ++i)
            std::printf(i ? ", %.17g" : "%.17g", static_cast<double>(v[i]));
        std::printf(last ? "]" : "], ");
    };
    std::printf("{\"n\": %d, ", m.ndof);
    std::printf("\"names\": [");
    for (std::size_t i = 0; i < names.size(); ++i) std::printf(i ? ", \"%s\"" : "\"%s\"", names[i].c_str());
    std::printf("], ");
    arr("parent", m.parent);
    arr("joint_origin", m.jointOrigin);
    arr("joint_rot", m.jointRotation);
    arr("joint_axis", m.jointAxis);
    arr("joint_type", m.jointType);
    arr("link_mass", m.linkMass);
    arr("link_com", m.linkCom);
    arr("link_inertia", m.linkInertia);
    arr("frame_link", m.frameLink);
    arr("frame_pose", m.framePose, true);
    std::printf("}\n");
    return 0;
}

int main(int argc, char** argv)
{
    const std::string which = argc > 1 ? argv[1] : "all";
    if (which == "urdf") return dumpUrdf(argc, argv);
    if (const char* g = std::getenv("BLF_GOLDEN_DIR")) g_golden = g;
    const bool cpu = which == "cpu" || which == "all";
    const bool gpu = which == "gpu" || which == "all";
    struct T { const char* name; bool device; std::function<void()> fn; };
    const std::vector<T> tests = {
        {"ContactList", false, testContactList},
        {"ContactPhaseList", false, testContactPhaseList},
        {"VariablesHandler", false, testVariablesHandler},
        {"ParametersHandler (config.ini)", false, testParametersHandler},
        {"Integrator - Linear system", true, testIntegratorLTI},
        {"Integrator - host-side system", false, testIntegratorHostSystem},
        {"Integrator - host-side system == device LTI", true, testIntegratorHostSystemMatchesDevice},
        {"Integrator - LTI of any size", true, testIntegratorLTIAnySize},
        {"Convex Hull helper (2-D)", true, testConvexHull},
        {"Convex Hull helper (3-D, ConvexHullHelperTest.cpp)", true, testConvexHull3},
        {"Convex Hull helper (n-D)", true, testConvexHullN},
        {"QuinticSpline", true, testQuinticSpline},
        {"TimeVaryingDCMPlanner advance", true, testPlanner},
        {"TimeVaryingDCMPlanner three contacts", true, testPlannerThreeContacts},
        {"Continuous Contact", true, testContinuousContact},
        {"FloatingBaseSystemKinematics", true, testFloatingBaseKinematics},
        {"IntegratorTest: floating base kinematics (literal)", true, testIntegratorKinematicsLiteral},
        {"FloatingBaseDynamicalSystem", true, testFloatingBaseDynamics},
        {"FloatingBaseDynamicalSystem, any ContactModel", true, testFloatingBaseDynamicsAnyContactModel},
        {"Fixed joints (model merge)", false, testFixedJoints},
        {"Fixed / prismatic joints (device)", true, testFixedJointsDevice},
    };
    for (const auto& t : tests)
    {
        if ((t.device && !gpu) || (!t.device && !cpu)) continue;
        const int before = g_failed;
        t.fn();
        std::printf("%-32s %s\n", t.name, g_failed == before ? "ok" : "FAILED");
    }
    std::printf("%d checks, %d failed\n", g_checks, g_failed);
    return g_failed;
}
