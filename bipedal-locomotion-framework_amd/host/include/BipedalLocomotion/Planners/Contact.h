/**
 * @file Contact.h
 * Drop-in for src/Planners/include/BipedalLocomotion/Planners/Contact.h:22-61.  The pose type
 * stands in for iDynTree::Transform (position + row-major rotation), which is not available.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_PLANNERS_CONTACT_H
#define BLF_BIPEDAL_LOCOMOTION_PLANNERS_CONTACT_H

#include <array>
#include <cmath>
#include <string>

namespace BipedalLocomotion
{
namespace Planners
{

/** Homogeneous transform: p + R x. */
struct Transform
{
    std::array<double, 3> position{{0.0, 0.0, 0.0}};
    std::array<double, 9> rotation{{1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0}};

    static Transform Identity() { return Transform{}; }
    /** Planar pose: translation (x, y, z) and a yaw rotation about z. */
    static Transform fromPlanar(double x, double y, double yaw, double z = 0.0)
    {
        Transform t;
        t.position = {{x, y, z}};
        const double c = std::cos(yaw), s = std::sin(yaw);
        t.rotation = {{c, -s, 0.0, s, c, 0.0, 0.0, 0.0, 1.0}};
        return t;
    }
    /** Apply to a point. */
    std::array<double, 3> apply(const std::array<double, 3>& x) const
    {
        std::array<double, 3> out;
        for (int r = 0; r < 3; ++r)
            out[r] = position[r] + (rotation[3 * r] * x[0] + rotation[3 * r + 1] * x[1] + rotation[3 * r + 2] * x[2]);
        return out;
    }
};

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
