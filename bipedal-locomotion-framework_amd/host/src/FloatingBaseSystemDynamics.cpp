/**
 * @file FloatingBaseSystemDynamics.cpp
 * Checks and messages follow src/System/src/FloatingBaseSystemDynamics.cpp:17-120; the dynamics
 * (:102-251) run on the device through blf_fbd_dynamics / blf_fbd_euler_integrate.
 */
#include <iostream>

#include <BipedalLocomotion/ContactModels/ContinuousContactModel.h>
#include <BipedalLocomotion/System/FloatingBaseSystemDynamics.h>

using namespace BipedalLocomotion::System;
using namespace BipedalLocomotion::ParametersHandler;

bool FloatingBaseDynamicalSystem::initalize(std::weak_ptr<IParametersHandler> handler)
{
    auto ptr = handler.lock();
    if (ptr == nullptr)
    {
        std::cerr << "[FloatingBaseDynamicalSystem::initalize] The parameter handler is expired. "
                     "Please call the function passing a pointer pointing an already allocated "
                     "memory."
                  << std::endl;
        return false;
    }
    if (!ptr->getParameter("rho", m_rho))
    {
        std::cerr << "[FloatingBaseDynamicalSystem::initalize] Unable to load the Baumgarte "
                     "stabilization parameter."
                  << std::endl;
        return false;
    }
    return true;
}

bool blf::fixedJointMergeable(const RobotModel& in)
{
    if (in.ndof < 0) return false;
    const std::size_t n0 = static_cast<std::size_t>(in.ndof);
    if (in.fixedJoint.size() != n0 || in.parent.size() != n0 || in.jointOrigin.size() != 3 * n0
        || in.jointRotation.size() != 9 * n0 || in.jointAxis.size() != 3 * n0
        || in.linkMass.size() != n0 + 1 || in.linkCom.size() != 3 * (n0 + 1)
        || in.linkInertia.size() != 9 * (n0 + 1) || in.framePose.size() != 12 * in.frameLink.size()
        || (!in.jointType.empty() && in.jointType.size() != n0))
        return false;
    // the merge re-indexes joints and links assuming topological order (a joint's parent link
    // precedes its child: parent[j] <= j), and moves frames by link index
    for (std::size_t j = 0; j < n0; ++j)
        if (in.parent[j] < 0 || in.parent[j] > static_cast<int32_t>(j)) return false;
    for (const int32_t l : in.frameLink)
        if (l < 0 || l > static_cast<int32_t>(n0)) return false;
    return true;
}

blf::RobotModel blf::reduceFixedJoints(const RobotModel& in)
{
    // an inconsistent model (sizes, order) comes back unchanged, its fixedJoint still set, so the
    // caller's own validation (setRobotModel) reports it instead of a merge reading out of bounds
    if (!fixedJointMergeable(in)) return in;
    RobotModel m = in;
    m.fixedJoint.clear();
    const int n0 = in.ndof;
    auto E = [&](int j, int r, int c) { return m.jointRotation[9 * j + 3 * r + c]; };
    // y = E_j x (3-vectors)
    auto rot = [&](int j, const double* x, double* y) {
        for (int r = 0; r < 3; ++r) y[r] = E(j, r, 0) * x[0] + E(j, r, 1) * x[1] + E(j, r, 2) * x[2];
    };
    // C = E_j A (3x3 row-major)
    auto rotm = [&](int j, const double* A, double* C) {
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c)
                C[3 * r + c] = E(j, r, 0) * A[c] + E(j, r, 1) * A[3 + c] + E(j, r, 2) * A[6 + c];
    };
    // I += m S(d), S(d) = |d|^2 1 - d d^T
    auto pax = [](double* I, double mass, const double* d) {
        const double dd = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) I[3 * r + c] += mass * ((r == c ? dd : 0.0) - d[r] * d[c]);
    };
    for (int j = n0 - 1; j >= 0; --j)
    {
        if (!in.fixedJoint[j]) continue;
        const int c = j + 1, P = m.parent[j];
        double cc[3], cn[3], Ic[9], T[9];
        rot(j, &m.linkCom[3 * c], cc);
        for (int a = 0; a < 3; ++a) cc[a] += m.jointOrigin[3 * j + a];   // child COM in P's frame
        const double mP = m.linkMass[P], mc = m.linkMass[c], mt = mP + mc;
        for (int a = 0; a < 3; ++a) cn[a] = mt > 0 ? (mP * m.linkCom[3 * P + a] + mc * cc[a]) / mt : m.linkCom[3 * P + a];
        // E_j I_c E_j^T
        rotm(j, &m.linkInertia[9 * c], T);
        for (int r = 0; r < 3; ++r)
            for (int k = 0; k < 3; ++k) Ic[3 * r + k] = T[3 * r] * E(j, k, 0) + T[3 * r + 1] * E(j, k, 1) + T[3 * r + 2] * E(j, k, 2);
        double dP[3], dc[3];
        for (int a = 0; a < 3; ++a) { dP[a] = m.linkCom[3 * P + a] - cn[a]; dc[a] = cc[a] - cn[a]; }
        double* IP = &m.linkInertia[9 * P];
        pax(IP, mP, dP);
        for (int k = 0; k < 9; ++k) IP[k] += Ic[k];
        pax(IP, mc, dc);
        m.linkMass[P] = mt;
        for (int a = 0; a < 3; ++a) m.linkCom[3 * P + a] = cn[a];
        for (int k = j + 1; k < m.ndof; ++k)   // joints on c move to P
            if (m.parent[k] == c)
            {
                double o[3], R[9];
                rot(j, &m.jointOrigin[3 * k], o);
                rotm(j, &m.jointRotation[9 * k], R);
                for (int a = 0; a < 3; ++a) m.jointOrigin[3 * k + a] = m.jointOrigin[3 * j + a] + o[a];
                for (int a = 0; a < 9; ++a) m.jointRotation[9 * k + a] = R[a];
                m.parent[k] = P;
            }
        for (std::size_t f = 0; f < m.frameLink.size(); ++f)   // frames on c move to P
            if (m.frameLink[f] == c)
            {
                double p[3], R[9];
                rot(j, &m.framePose[12 * f], p);
                rotm(j, &m.framePose[12 * f + 3], R);
                for (int a = 0; a < 3; ++a) m.framePose[12 * f + a] = m.jointOrigin[3 * j + a] + p[a];
                for (int a = 0; a < 9; ++a) m.framePose[12 * f + 3 + a] = R[a];
                m.frameLink[f] = P;
            }
        // drop joint j and link c; links above c shift down by one
        m.parent.erase(m.parent.begin() + j);
        m.jointOrigin.erase(m.jointOrigin.begin() + 3 * j, m.jointOrigin.begin() + 3 * j + 3);
        m.jointRotation.erase(m.jointRotation.begin() + 9 * j, m.jointRotation.begin() + 9 * j + 9);
        m.jointAxis.erase(m.jointAxis.begin() + 3 * j, m.jointAxis.begin() + 3 * j + 3);
        if (m.jointType.size() == static_cast<std::size_t>(m.ndof)) m.jointType.erase(m.jointType.begin() + j);
        m.linkMass.erase(m.linkMass.begin() + c);
        m.linkCom.erase(m.linkCom.begin() + 3 * c, m.linkCom.begin() + 3 * c + 3);
        m.linkInertia.erase(m.linkInertia.begin() + 9 * c, m.linkInertia.begin() + 9 * c + 9);
        for (auto& p : m.parent)
            if (p > c) --p;
        for (auto& l : m.frameLink)
            if (l > c) --l;
        --m.ndof;
    }
    return m;
}

bool FloatingBaseDynamicalSystem::setRobotModel(const blf::RobotModel& fullModel)
{
    if (!fullModel.fixedJoint.empty()
        && fullModel.fixedJoint.size() != static_cast<std::size_t>(fullModel.ndof))
    {
        std::cerr << "[FloatingBaseDynamicalSystem::setRobotModel] Corrupted robot model." << std::endl;
        return false;
    }
    // sizes are checked before the merge reads them (the merged model is checked again below)
    const std::size_t n0 = static_cast<std::size_t>(fullModel.ndof < 0 ? 0 : fullModel.ndof);
    if (!fullModel.fixedJoint.empty()
        && (fullModel.parent.size() != n0 || fullModel.jointOrigin.size() != 3 * n0
            || fullModel.jointRotation.size() != 9 * n0 || fullModel.jointAxis.size() != 3 * n0
            || fullModel.linkMass.size() != n0 + 1 || fullModel.linkCom.size() != 3 * (n0 + 1)
            || fullModel.linkInertia.size() != 9 * (n0 + 1)
            || fullModel.framePose.size() != 12 * fullModel.frameLink.size()))
    {
        std::cerr << "[FloatingBaseDynamicalSystem::setRobotModel] Corrupted robot model." << std::endl;
        return false;
    }
    for (std::size_t j = 0; j < fullModel.fixedJoint.size(); ++j)
        if (fullModel.parent[j] < 0 || fullModel.parent[j] > static_cast<int32_t>(j))
        {
            std::cerr << "[FloatingBaseDynamicalSystem::setRobotModel] The joints must be in "
                         "topological order (parent[j] <= j)."
                      << std::endl;
            return false;
        }
    const blf::RobotModel model = fullModel.fixedJoint.empty() ? fullModel : blf::reduceFixedJoints(fullModel);
    const std::size_t n = static_cast<std::size_t>(model.ndof);
    const std::size_t F = model.frameLink.size();
    if (model.ndof < 1 || model.ndof > BLF_FBD_MAX_DOFS || model.parent.size() != n
        || model.jointOrigin.size() != 3 * n || model.jointRotation.size() != 9 * n
        || model.jointAxis.size() != 3 * n || model.linkMass.size() != n + 1
        || model.linkCom.size() != 3 * (n + 1) || model.linkInertia.size() != 9 * (n + 1)
        || model.framePose.size() != 12 * F
        || (!model.jointType.empty() && model.jointType.size() != n))
    {
        std::cerr << "[FloatingBaseDynamicalSystem::setRobotModel] Corrupted robot model."
                  << std::endl;
        return false;
    }
    for (std::size_t j = 0; j < n; ++j)
        if (model.parent[j] < 0 || model.parent[j] > static_cast<int32_t>(j))
        {
            std::cerr << "[FloatingBaseDynamicalSystem::setRobotModel] The joints must be in "
                         "topological order (parent[j] <= j)."
                      << std::endl;
            return false;
        }
    for (const int32_t t : model.jointType)
        if (t != BLF_JOINT_REVOLUTE && t != BLF_JOINT_PRISMATIC)
        {
            std::cerr << "[FloatingBaseDynamicalSystem::setRobotModel] Unknown joint type " << t
                      << " (revolute or prismatic; fixed joints go in fixedJoint)." << std::endl;
            return false;
        }
    m_model = model;
    m_actuatedDoFs = n;
    m_hasModel = m_dParent.upload(model.parent) && m_dOrigin.upload(model.jointOrigin)
                 && m_dRot.upload(model.jointRotation) && m_dAxis.upload(model.jointAxis)
                 && m_dMass.upload(model.linkMass) && m_dCom.upload(model.linkCom)
                 && m_dInertia.upload(model.linkInertia) && m_dFrameLink.upload(model.frameLink)
                 && m_dFramePose.upload(model.framePose)
                 && (model.jointType.empty() || m_dJointType.upload(model.jointType));
    return m_hasModel;
}

bool FloatingBaseDynamicalSystem::setMassMatrixRegularization(const blf::MatrixXd& matrix)
{
    if (!m_hasModel)
    {
        std::cerr << "[FloatingBaseDynamicalSystem::setMassMatrixRegularization] Please call "
                     "'setRobotModel()' before."
                  << std::endl;
        return false;
    }
    const std::size_t rightSize = m_actuatedDoFs + m_baseDoFs;
    if (rightSize != matrix.rows() || matrix.cols() != matrix.rows())
    {
        std::cerr << "[FloatingBaseDynamicalSystem::setMassMatrixRegularization] The size of the "
                     "regularization matrix is not correct. The correct size is: "
                  << rightSize << " x " << rightSize << ". While the input of the function is a "
                  << matrix.rows() << " x " << matrix.cols() << " matrix." << std::endl;
        return false;
    }
    m_useMassMatrixRegularizationTerm = m_dReg.upload(matrix.data(), rightSize * rightSize);
    return m_useMassMatrixRegularizationTerm;
}

// device state layout: base vel 6 | joint vel n | base pos 3 | base rot 9 | joint pos n
bool FloatingBaseDynamicalSystem::prepare(const char* where, blf_fb_model& model,
                                          blf_fb_state& state, blf_fb_contacts& contacts)
{
    if (!m_hasModel)
    {
        std::cerr << "[" << where << "] Please call 'setRobotModel()' before." << std::endl;
        return false;
    }
    const auto& [baseVelocity, jointVelocity, basePosition, baseOrientation, jointPositions] = m_state;
    const auto& [jointTorques, contactWrenches] = m_controlInput;
    const std::size_t n = m_actuatedDoFs;
    if (jointVelocity.size() != n || jointPositions.size() != n || jointTorques.size() != n)
    {
        std::cerr << "[" << where << "] Wrong size of the vectors." << std::endl;
        return false;
    }
    if (contactWrenches.size() > BLF_FBD_MAX_CONTACTS)
    {
        std::cerr << "[" << where << "] At most " << BLF_FBD_MAX_CONTACTS << " contacts." << std::endl;
        return false;
    }
    std::vector<double> st(18 + 2 * n);
    for (int i = 0; i < 6; ++i) st[i] = baseVelocity[i];
    for (std::size_t i = 0; i < n; ++i) st[6 + i] = jointVelocity[i];
    for (int i = 0; i < 3; ++i) st[6 + n + i] = basePosition[i];
    for (int i = 0; i < 9; ++i) st[9 + n + i] = baseOrientation[i];
    for (std::size_t i = 0; i < n; ++i) st[18 + n + i] = jointPositions[i];
    std::vector<int32_t> frames, laws;
    std::vector<double> params, nulls;
    m_contactModels.clear();
    m_hostContacts = false;
    for (const auto& c : contactWrenches)
    {
        auto ptr = c.contactModel().lock();
        if (ptr == nullptr)
        {
            std::cerr << "[" << where << "] The contact model associated to the frame " << c.index()
                      << " has been expired." << std::endl;
            return false;
        }
        if (c.index() < 0 || c.index() >= static_cast<int>(m_model.frameLink.size()))
        {
            std::cerr << "[" << where << "] Unknown frame " << c.index() << "." << std::endl;
            return false;
        }
        frames.push_back(c.index());
        // a ContinuousContactModel is evaluated in the kernel; any other model by its own
        // getContactWrench() at the frame state the device computes (BLF_CONTACT_WRENCH)
        auto cm = std::dynamic_pointer_cast<ContactModels::ContinuousContactModel>(ptr);
        if (cm != nullptr)
        {
            laws.push_back(BLF_CONTACT_CONTINUOUS);
            params.insert(params.end(), {cm->length(), cm->width(), cm->springCoeff(), cm->damperCoeff()});
            const auto np = cm->nullForceTransform().packed();
            nulls.insert(nulls.end(), np.begin(), np.end());
        } else
        {
            laws.push_back(BLF_CONTACT_WRENCH);
            m_hostContacts = true;
            params.insert(params.end(), 4, 0.0);
            const auto np = blf::Transform::Identity().packed();
            nulls.insert(nulls.end(), np.begin(), np.end());
        }
        m_contactModels.push_back(ptr);
    }
    if (m_hostContacts
        && (!m_dContactLaw.upload(laws) || !m_dContactWrench.resize(6 * laws.size())))
        return false;
    if (!m_dState.upload(st) || !m_dTau.upload(jointTorques.data(), n)
        || !m_dContactFrame.upload(frames) || !m_dContactParams.upload(params)
        || !m_dNullPose.upload(nulls))
        return false;
    model.ndof = static_cast<int32_t>(n);
    model.nframes = static_cast<int32_t>(m_model.frameLink.size());
    model.parent = m_dParent.data();
    model.joint_origin = m_dOrigin.data();
    model.joint_rot = m_dRot.data();
    model.joint_axis = m_dAxis.data();
    model.link_mass = m_dMass.data();
    model.link_com = m_dCom.data();
    model.link_inertia = m_dInertia.data();
    model.frame_link = m_dFrameLink.data();
    model.frame_pose = m_dFramePose.data();
    model.joint_type = m_model.jointType.empty() ? nullptr : m_dJointType.data();
    for (int i = 0; i < 3; ++i) model.gravity[i] = m_gravity[i];
    model.rho = m_rho;
    double* s = m_dState.data();
    state.base_vel = s;
    state.joint_vel = s + 6;
    state.base_pos = s + 6 + n;
    state.base_rot = s + 9 + n;
    state.joint_pos = s + 18 + n;
    contacts.ncontacts = static_cast<int32_t>(frames.size());
    contacts.frame = m_dContactFrame.data();
    contacts.params = m_dContactParams.data();
    contacts.null_pose = m_dNullPose.data();
    contacts.law = m_hostContacts ? m_dContactLaw.data() : nullptr;
    contacts.wrench = m_hostContacts ? m_dContactWrench.data() : nullptr;
    return true;
}

// The reference's per-contact `contactPtr->setState(getFrameVel, getWorldTransform)` (FloatingBase
// SystemDynamics.cpp:225-226) at the device's frame state; then, when `wrenches` is set, the
// BLF_CONTACT_WRENCH contacts' getContactWrench() uploaded for the next launch.
bool FloatingBaseDynamicalSystem::updateContactModels(const char* where, const blf_fb_model& model,
                                                      const blf_fb_state& state, bool wrenches)
{
    const std::size_t C = m_contactModels.size();
    if (C == 0) return true;
    blf_handle* h = blf::threadHandle();
    if (!m_dFrameOut.resize(18 * C)) return false;
    double* pose = m_dFrameOut.data();
    if (!blf::report(blf_fb_frame_state(h, &model, &state, static_cast<int32_t>(C),
                                        m_dContactFrame.data(), 1, pose, pose + 12 * C, nullptr),
                     where))
        return false;
    std::vector<double> host(18 * C), wrench(6 * C, 0.0);
    if (!m_dFrameOut.download(host.data(), host.size())) return false;
    for (std::size_t c = 0; c < C; ++c)
    {
        blf::Transform T;
        blf::Twist tw;
        for (int i = 0; i < 3; ++i) T.position[i] = host[12 * c + i];
        for (int i = 0; i < 9; ++i) T.rotation[i] = host[12 * c + 3 + i];
        for (int i = 0; i < 6; ++i) tw[i] = host[12 * C + 6 * c + i];
        m_contactModels[c]->setState(tw, T);
        if (wrenches
            && std::dynamic_pointer_cast<ContactModels::ContinuousContactModel>(m_contactModels[c])
                   == nullptr)
        {
            const blf::Wrench& w = m_contactModels[c]->getContactWrench();
            for (int i = 0; i < 6; ++i) wrench[6 * c + i] = w[i];
        }
    }
    return !wrenches || m_dContactWrench.upload(wrench);
}

bool FloatingBaseDynamicalSystem::dynamics(const double& time, StateDerivativeType& stateDerivative)
{
    (void)time;
    const char* where = "FloatingBaseDynamicalSystem::dynamics";
    blf_fb_model model;
    blf_fb_state state;
    blf_fb_contacts contacts;
    blf_handle* h = blf::threadHandle();
    if (h == nullptr || !prepare(where, model, state, contacts)
        || !updateContactModels(where, model, state, m_hostContacts))
        return false;
    const std::size_t n = m_actuatedDoFs;
    if (!m_dOut.resize(18 + 2 * n)) return false;
    double* o = m_dOut.data();
    blf_fb_state out{o, o + 6, o + 6 + n, o + 9 + n, o + 18 + n};
    if (!blf::report(blf_fbd_dynamics(h, &model, &state, m_dTau.data(), &contacts,
                                      m_useMassMatrixRegularizationTerm ? m_dReg.data() : nullptr,
                                      1, &out, nullptr),
                     where))
        return false;
    std::vector<double> host(18 + 2 * n);
    if (!m_dOut.download(host.data(), host.size())) return false;
    auto& [baseAcceleration, jointAcceleration, baseLinearVelocity, baseRotationRate,
           jointVelocityOutput] = stateDerivative;
    for (int i = 0; i < 6; ++i) baseAcceleration[i] = host[i];
    jointAcceleration.resize(n);
    jointVelocityOutput.resize(n);
    for (std::size_t i = 0; i < n; ++i)
    {
        jointAcceleration[i] = host[6 + i];
        jointVelocityOutput[i] = host[18 + n + i];
    }
    for (int i = 0; i < 3; ++i) baseLinearVelocity[i] = host[6 + n + i];
    for (int i = 0; i < 9; ++i) baseRotationRate[i] = host[9 + n + i];
    return true;
}

bool FloatingBaseDynamicalSystem::forwardEulerIntegrate(double initialTime, double finalTime,
                                                        double dT)
{
    const char* where = "FixedStepIntegrator::integrate";
    blf_fb_model model;
    blf_fb_state state;
    blf_fb_contacts contacts;
    blf_handle* h = blf::threadHandle();
    if (h == nullptr || !prepare(where, model, state, contacts)) return false;
    const double* reg = m_useMassMatrixRegularizationTerm ? m_dReg.data() : nullptr;
    if (!m_hostContacts)
    {
        // every contact a ContinuousContactModel: the whole integration in one launch
        if (!blf::report(blf_fbd_euler_integrate(h, &model, &state, m_dTau.data(), &contacts, reg,
                                                 1, initialTime, finalTime, dT, nullptr),
                         where))
            return false;
    } else
    {
        // a model the device cannot evaluate: its wrench from the host before every step, as the
        // reference's dynamics() calls getContactWrench() at each step's start state; one launch
        // of one step each (the device's schedule, ForwardEuler.tpp:18-49)
        int32_t iterations = 0;
        double dT_last = 0.0, t_last = 0.0;
        if (!blf::report(blf_step_schedule(initialTime, finalTime, dT, &iterations, &dT_last, &t_last),
                         where))
            return false;
        for (int32_t it = 0; it < iterations; ++it)
        {
            const double step = it + 1 < iterations ? dT : dT_last;
            if (!updateContactModels(where, model, state, true)
                || !blf::report(blf_fbd_euler_integrate(h, &model, &state, m_dTau.data(), &contacts,
                                                        reg, 1, 0.0, step, step, nullptr),
                                where))
                return false;
        }
    }
    const std::size_t n = m_actuatedDoFs;
    std::vector<double> host(18 + 2 * n);
    if (!m_dState.download(host.data(), host.size())) return false;
    auto& [baseVelocity, jointVelocity, basePosition, baseOrientation, jointPositions] = m_state;
    for (int i = 0; i < 6; ++i) baseVelocity[i] = host[i];
    for (std::size_t i = 0; i < n; ++i)
    {
        jointVelocity[i] = host[6 + i];
        jointPositions[i] = host[18 + n + i];
    }
    for (int i = 0; i < 3; ++i) basePosition[i] = host[6 + n + i];
    for (int i = 0; i < 9; ++i) baseOrientation[i] = host[9 + n + i];
    return true;
}
