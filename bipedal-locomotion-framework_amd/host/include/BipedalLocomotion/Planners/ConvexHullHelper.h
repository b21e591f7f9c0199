/**
 * @file ConvexHullHelper.h
 * Drop-in for src/Planners/include/BipedalLocomotion/Planners/ConvexHullHelper.h:32-81
 * (src/Planners/src/ConvexHullHelper.cpp:35-117) for the planners' 2-D support polygons.
 * buildConvexHull runs blf_hull2d_hrep on the device (2 x p points, p <= 16); getA()/getB() return
 * the H-representation A x <= b (unit outward normals, merged collinear facets, counter-clockwise
 * order — Qhull's facet order is internal to Qhull, so only the facet SET is comparable);
 * doesPointBelongToConvexHull runs blf_hull2d_contains (strict `>` rejects, no tolerance).
 * Inputs with a row count other than 2 are rejected with false: 3-D hulls are not on the
 * accelerated path (scope).
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_PLANNERS_CONVEX_HULL_HELPER_H
#define BLF_BIPEDAL_LOCOMOTION_PLANNERS_CONVEX_HULL_HELPER_H

#include <cstddef>
#include <vector>

#include <blf/dense.h>
#include <blf/device.h>

namespace BipedalLocomotion
{
namespace Planners
{

class ConvexHullHelper
{
    blf::MatrixXd m_A;
    blf::VectorXd m_b;
    blf::DeviceBuffer<double> m_dPts, m_dA, m_dB, m_dQ;
    blf::DeviceBuffer<int32_t> m_dN, m_dInside;

public:
    /** points: 2 x p (one point per column).  Any matrix type with rows(), cols(), (i, j). */
    template <class Mat> bool buildConvexHull(const Mat& points)
    {
        return buildConvexHull(blf::MatrixXd::from(points));
    }
    bool buildConvexHull(const blf::MatrixXd& points);

    const blf::MatrixXd& getA() const { return m_A; }
    const blf::VectorXd& getB() const { return m_b; }

    template <class Vec> bool doesPointBelongToConvexHull(const Vec& point) const
    {
        blf::VectorXd p(static_cast<std::size_t>(point.size()));
        for (std::size_t i = 0; i < p.size(); ++i) p(i) = point(i);
        return doesPointBelongToConvexHull(p);
    }
    bool doesPointBelongToConvexHull(const blf::VectorXd& point) const;
};

} // namespace Planners
} // namespace BipedalLocomotion

#endif
