/**
 * @file spatial.h
 * Fixed-size spatial value types the C++ adapters use in place of iDynTree's (not available in
 * this build): Transform (position + row-major rotation, iDynTree::Transform), Twist / Wrench /
 * Vector6 (linear part first, iDynTree's order), Matrix3 / Matrix6x6 (row-major).
 */
#ifndef BLF_HOST_SPATIAL_H
#define BLF_HOST_SPATIAL_H

#include <array>
#include <cmath>

namespace blf
{

using Vector3 = std::array<double, 3>;
using Vector6 = std::array<double, 6>;
using Matrix3 = std::array<double, 9>;     /**< row-major */
using Matrix6x6 = std::array<double, 36>;  /**< row-major */
using Twist = Vector6;                     /**< (linear velocity, angular velocity), mixed */
using Wrench = Vector6;                    /**< (force, torque) */

struct Transform
{
    Vector3 position{{0.0, 0.0, 0.0}};
    Matrix3 rotation{{1.0, 0.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0}};

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
    Vector3 apply(const Vector3& x) const
    {
        Vector3 out;
        for (int r = 0; r < 3; ++r)
            out[r] = position[r] + (rotation[3 * r] * x[0] + rotation[3 * r + 1] * x[1] + rotation[3 * r + 2] * x[2]);
        return out;
    }
    /** (p, R) packed as the C ABI's 12-double pose. */
    std::array<double, 12> packed() const
    {
        std::array<double, 12> o;
        for (int i = 0; i < 3; ++i) o[i] = position[i];
        for (int i = 0; i < 9; ++i) o[3 + i] = rotation[i];
        return o;
    }
};

} // namespace blf

#endif // BLF_HOST_SPATIAL_H
