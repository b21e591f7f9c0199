/**
 * @file urdf.h
 * A robot description (URDF) -> blf::RobotModel, for FloatingBaseDynamicalSystem::setRobotModel.
 *
 * The reference's FloatingBaseDynamicalSystem takes its model from iDynTree
 * (src/System/src/FloatingBaseSystemDynamics.cpp:53-74, setKinDyn / setRobotModel), which a user
 * fills with iDynTree's ModelLoader from a URDF, optionally reduced to a list of "considered
 * joints" (the others locked).  iDynTree is not part of this build; loadUrdf is that path for the
 * C++ adapter, the same rules as the Python loader (blf/urdf.py, tests/test_urdf.py):
 *   * the tree rooted at the floating base (the one link that is no joint's child, or
 *     options.base); joints in depth-first preorder, children in document order, so
 *     parent[j] <= j;
 *   * joint origin xyz / rpy (R = Rz(y) Ry(p) Rx(r)) and axis (normalised, URDF default x);
 *     revolute / continuous -> revolute, prismatic -> prismatic, fixed and every joint outside
 *     options.consideredJoints -> merged into its parent link (blf::reduceFixedJoints);
 *     floating / planar joints inside the tree are refused;
 *   * link inertials: origin xyz -> COM, inertia about the COM rotated into the link frame
 *     (R I R^T); a link without <inertial> is massless;
 *   * options.frames: link names exposed as frames at their link's origin, following the merge.
 * With consideredJoints the degrees of freedom follow the list's order (as iDynTree orders them);
 * a joint listed before its parent's joint is refused.
 * The XML reader takes elements, attributes (with the five predefined entities), comments,
 * processing instructions, CDATA and a DOCTYPE; nothing in the file is executed.
 */
#ifndef BLF_HOST_URDF_H
#define BLF_HOST_URDF_H

#include <string>
#include <vector>

#include <BipedalLocomotion/System/FloatingBaseSystemDynamics.h>

namespace blf
{

struct UrdfOptions
{
    std::vector<std::string> frames;           /**< link names exposed as frames, in order */
    std::string base;                          /**< floating base link; empty: the root   */
    bool hasConsideredJoints{false};           /**< false: every moving joint is a DoF    */
    std::vector<std::string> consideredJoints; /**< the DoFs, in this order               */
};

/** Parse `source` (a URDF file path, or the XML itself when it starts with '<') into `model`
 *  (fixed joints already merged, fixedJoint empty).  jointNames (optional) receives the DoF names
 *  in model order.  Returns false with a message in *error (if given) on a malformed document or
 *  an unsupported model; `model` is then left unchanged. */
bool loadUrdf(const std::string& source, const UrdfOptions& options, RobotModel& model,
              std::vector<std::string>* jointNames = nullptr, std::string* error = nullptr);

} // namespace blf

#endif
