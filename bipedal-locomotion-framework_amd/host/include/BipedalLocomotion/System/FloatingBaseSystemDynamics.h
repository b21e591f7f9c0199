/**
 * @file FloatingBaseSystemDynamics.h
 * Drop-in for src/System/include/BipedalLocomotion/System/FloatingBaseSystemDynamics.h:30-157
 * (src/System/src/FloatingBaseSystemDynamics.cpp):
 *   state      (base velocity (mixed), joint velocities, base position, base orientation,
 *               joint positions)
 *   input      (joint torques, contact wrenches)
 *   derivative (base acceleration, joint accelerations, base linear velocity, base rotation rate,
 *               joint velocities)
 * The reference takes M, h and the frame Jacobians from iDynTree KinDynComputations, set with
 * setKinDyn(); this build has no iDynTree, so the robot is given as a kinematic tree with
 * setRobotModel() (blf::RobotModel, the layout of blf/robot.py) and the rigid-body terms are
 * computed on the device (blf_fbd_dynamics / blf_fbd_euler_integrate, include/blf/blf_c.h).
 * Contacts may hold any ContactModel.  A ContinuousContactModel is evaluated in the kernel
 * (BLF_CONTACT_CONTINUOUS); any other model is set to the frame state the device computes
 * (blf_fb_frame_state) and its getContactWrench() is passed to the kernel (BLF_CONTACT_WRENCH):
 * forwardEulerIntegrate() then launches one Euler step at a time, so that the wrench is taken at
 * every step's start state as in the reference.  dynamics() leaves every contact model in its
 * frame's state (the reference's setState side effect, FloatingBaseSystemDynamics.cpp:225-226);
 * the one-launch forwardEulerIntegrate() of ContinuousContactModel-only contacts does not.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_SYSTEM_FLOATING_BASE_SYSTEM_DYNAMICS_H
#define BLF_BIPEDAL_LOCOMOTION_SYSTEM_FLOATING_BASE_SYSTEM_DYNAMICS_H

#include <tuple>
#include <vector>

#include <BipedalLocomotion/System/ContactWrench.h>
#include <BipedalLocomotion/System/DynamicalSystem.h>
#include <blf/dense.h>
#include <blf/device.h>
#include <blf/spatial.h>

namespace blf
{
/** Kinematic tree of revolute, prismatic (jointType) and fixed (fixedJoint) joints on a floating
 *  base (see blf_fb_model in blf_c.h). */
struct RobotModel
{
    int ndof{0};
    std::vector<int32_t> parent;       /**< [n]        */
    std::vector<double> jointOrigin;   /**< [n][3]     */
    std::vector<double> jointRotation; /**< [n][9]     */
    std::vector<double> jointAxis;     /**< [n][3]     */
    std::vector<double> linkMass;      /**< [n+1]      */
    std::vector<double> linkCom;       /**< [n+1][3]   */
    std::vector<double> linkInertia;   /**< [n+1][9]   */
    std::vector<int32_t> frameLink;    /**< [F]        */
    std::vector<double> framePose;     /**< [F][12]    */
    /** [n] or empty: 1 marks a fixed joint (a URDF "fixed" joint, no DoF). setRobotModel merges
     *  each fixed joint's child link into its parent (reduceFixedJoints), as iDynTree's model has
     *  no DoF for it; the state and torque vectors then cover the remaining joints only. */
    std::vector<uint8_t> fixedJoint;
    /** [n] or empty (every joint revolute): BLF_JOINT_REVOLUTE / BLF_JOINT_PRISMATIC (the child
     *  link slides along the joint axis by q, URDF "prismatic"). */
    std::vector<int32_t> jointType;
};

/** The model with every joint marked in model.fixedJoint removed and its child link merged into
 *  the parent link (mass, COM, inertia by the parallel-axis theorem; child joints and frames
 *  re-expressed in the parent link's frame at q = 0), deepest first.  The result has an empty
 *  fixedJoint.  Its rigid-body terms equal the full model's with the fixed joints held at
 *  q = 0, q_dot = 0 (blf/robot.py reduce_fixed_joints, tests/test_fb_dynamics.py). */
RobotModel reduceFixedJoints(const RobotModel& model);
/** Whether reduceFixedJoints can merge `model`: consistent array sizes (fixedJoint of ndof
 *  entries), joints in topological order (parent[j] <= j), frames on existing links.  A model that
 *  fails this comes back from reduceFixedJoints unchanged. */
bool fixedJointMergeable(const RobotModel& model);
} // namespace blf

namespace BipedalLocomotion
{
namespace System
{

class FloatingBaseDynamicalSystem
    : public DynamicalSystem<
          std::tuple<blf::Vector6, blf::VectorXd, blf::Vector3, blf::Matrix3, blf::VectorXd>,
          std::tuple<blf::Vector6, blf::VectorXd, blf::Vector3, blf::Matrix3, blf::VectorXd>,
          std::tuple<blf::VectorXd, std::vector<ContactWrench>>>
{
    static constexpr std::size_t m_baseDoFs = 6;
    std::size_t m_actuatedDoFs{0};
    double m_rho{0.01};
    blf::Vector3 m_gravity{{0.0, 0.0, -9.81}};
    bool m_hasModel{false};
    bool m_useMassMatrixRegularizationTerm{false};
    blf::RobotModel m_model;
    blf::DeviceBuffer<int32_t> m_dParent, m_dFrameLink, m_dContactFrame, m_dJointType, m_dContactLaw;
    blf::DeviceBuffer<double> m_dOrigin, m_dRot, m_dAxis, m_dMass, m_dCom, m_dInertia, m_dFramePose;
    blf::DeviceBuffer<double> m_dReg, m_dState, m_dTau, m_dContactParams, m_dNullPose, m_dOut;
    blf::DeviceBuffer<double> m_dContactWrench, m_dFrameOut;
    std::vector<std::shared_ptr<ContactModels::ContactModel>> m_contactModels;
    bool m_hostContacts{false};   /**< a contact model the kernel cannot evaluate */

    bool prepare(const char* where, blf_fb_model& model, blf_fb_state& state,
                 blf_fb_contacts& contacts);
    bool updateContactModels(const char* where, const blf_fb_model& model,
                             const blf_fb_state& state, bool wrenches);

public:
    bool initalize(std::weak_ptr<ParametersHandler::IParametersHandler> handler) final;
    void setGravityVector(const blf::Vector3& gravity) { m_gravity = gravity; }
    /** Replaces setKinDyn(): the robot model whose rigid-body terms the device computes. */
    bool setRobotModel(const blf::RobotModel& model);
    bool setMassMatrixRegularization(const blf::MatrixXd& matrix);
    bool dynamics(const double& time, StateDerivativeType& stateDerivative) final;

    /** Device hook used by ForwardEuler<FloatingBaseDynamicalSystem>. */
    bool forwardEulerIntegrate(double initialTime, double finalTime, double dT);
};

} // namespace System
} // namespace BipedalLocomotion

#endif
