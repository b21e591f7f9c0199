/**
 * @file Contact.h
 * Drop-in for src/Planners/include/BipedalLocomotion/Planners/Contact.h:22-61.  The pose type
 * stands in for iDynTree::Transform (position + row-major rotation), which is not available.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_PLANNERS_CONTACT_H
#define BLF_BIPEDAL_LOCOMOTION_PLANNERS_CONTACT_H

#include <array>

#include <blf/spatial.h>
#include <cmath>
#include <string>

namespace BipedalLocomotion
{
namespace Planners
{

/** Homogeneous transform: p + R x. */
/** iDynTree::Transform stand-in (blf/spatial.h). */
using Transform = blf::Transform;

enum class ContactType
{
    FULL, /**< full (6D) contact */
    POINT /**< point contact */
};

struct Contact
{
    Transform pose{Transform::Identity()};
    double activationTime{0.0};
    double deactivationTime{0.0};
    std::string name{"Contact"};
    ContactType type{ContactType::FULL};
};

} // namespace Planners
} // namespace BipedalLocomotion

#endif
