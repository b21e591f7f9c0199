/**
 * @file ConvexHullHelper.h
 * Drop-in for src/Planners/include/BipedalLocomotion/Planners/ConvexHullHelper.h:32-81
 * (src/Planners/src/ConvexHullHelper.cpp:35-117).
 * buildConvexHull runs blf_hull2d_hrep on the device for 2 x p points (the planners' support
 * polygons, p <= 16), blf_hull3d_hrep for 3 x p points (p <= 16; the reference's own test,
 * ConvexHullHelperTest.cpp:15-63, is 3-D) and blf_hullnd_hrep for any other n x p (1 <= n <= 8,
 * p <= 32; n = 1 is an extension -- the reference hands every matrix to Qhull, which refuses one
 * dimension, so its buildConvexHull fails there, while this one returns the rows +1 / -1 of the
 * interval); getA()/getB() return the H-representation A x <= b (unit outward normals; 2-D:
 * merged collinear facets, counter-clockwise; otherwise one row per distinct supporting
 * hyperplane, where Qhull "Qt" may give a split facet once per simplex — Qhull's facet order is
 * internal to Qhull, so only the SET of planes is comparable).  doesPointBelongToConvexHull runs
 * blf_hull2d_contains / blf_halfspace_contains (strict `>` rejects, no tolerance).  After a failed buildConvexHull (where Qhull would have thrown),
 * doesPointBelongToConvexHull returns false for every point instead of testing an empty H-rep.
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
    bool m_valid{false};   // the last buildConvexHull succeeded (a failed build rejects every point)
    bool buildConvexHullN(const blf::MatrixXd& points);

public:
    /** points: n x p (one point per column).  Any matrix type with rows(), cols(), (i, j). */
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
