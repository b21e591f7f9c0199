/**
 * @file ConvexHullHelper.cpp
 * Single-polygon calls into the batched device kernels (batch = 1).
 */
#include <algorithm>
#include <cmath>
#include <iostream>
#include <utility>
#include <vector>

#include <BipedalLocomotion/Planners/ConvexHullHelper.h>

using namespace BipedalLocomotion::Planners;

namespace
{
// The vertices of one face of a 3-D hull: the input points on the plane a.x = b (within tol),
// projected onto the plane, then the corners of their planar hull (Andrew's monotone chain,
// collinear points dropped: Qhull counts them as coplanar points, not vertices).
int faceVertexCount(const std::vector<double>& pts, std::size_t p, const double* a, double b, double tol)
{
    // an orthonormal basis (u, v) of the plane
    double u[3];
    if (std::abs(a[0]) < 0.9) { u[0] = 0.0; u[1] = a[2]; u[2] = -a[1]; }
    else { u[0] = -a[2]; u[1] = 0.0; u[2] = a[0]; }
    const double nu = std::sqrt(u[0] * u[0] + u[1] * u[1] + u[2] * u[2]);
    for (double& x : u) x /= nu;
    const double v[3] = {a[1] * u[2] - a[2] * u[1], a[2] * u[0] - a[0] * u[2], a[0] * u[1] - a[1] * u[0]};
    std::vector<std::pair<double, double>> q;
    for (std::size_t j = 0; j < p; ++j)
    {
        const double* x = &pts[3 * j];
        if (std::abs(a[0] * x[0] + a[1] * x[1] + a[2] * x[2] - b) > tol) continue;
        q.emplace_back(u[0] * x[0] + u[1] * x[1] + u[2] * x[2], v[0] * x[0] + v[1] * x[1] + v[2] * x[2]);
    }
    std::sort(q.begin(), q.end());
    q.erase(std::unique(q.begin(), q.end(),
                        [tol](const auto& l, const auto& r) {
                            return std::abs(l.first - r.first) <= tol && std::abs(l.second - r.second) <= tol;
                        }),
            q.end());
    if (q.size() < 3) return static_cast<int>(q.size());
    auto turn = [](const auto& o, const auto& a1, const auto& b1) {
        return (a1.first - o.first) * (b1.second - o.second) - (a1.second - o.second) * (b1.first - o.first);
    };
    const double eps = tol * tol;
    std::vector<std::pair<double, double>> h(2 * q.size());
    std::size_t k = 0;
    for (std::size_t i = 0; i < q.size(); ++i)   // lower chain
    {
        while (k >= 2 && turn(h[k - 2], h[k - 1], q[i]) <= eps) --k;
        h[k++] = q[i];
    }
    for (std::size_t i = q.size() - 1, t = k + 1; i-- > 0;)   // upper chain
    {
        while (k >= t && turn(h[k - 2], h[k - 1], q[i]) <= eps) --k;
        h[k++] = q[i];
    }
    return static_cast<int>(k - 1);
}
}  // namespace

// 3 x p points (p <= 16): blf_hull3d_hrep (the distinct supporting planes;
// ConvexHullHelperTest.cpp:15-63).  Any other n x p (n = 1 or n >= 4, or more points than the
// 2-D / 3-D kernels take): blf_hullnd_hrep, the same rule in any dimension.
bool ConvexHullHelper::buildConvexHullN(const blf::MatrixXd& points)
{
    const std::size_t p = points.cols(), dim = points.rows();
    const bool three = dim == 3 && p <= BLF_HULL_MAX_POINTS;
    if (dim < 1 || dim > BLF_HULLND_MAX_DIM)
    {
        std::cerr << "[ConvexHullHelper::buildConvexHull] Point sets of 1 to " << BLF_HULLND_MAX_DIM
                  << " dimensions are supported." << std::endl;
        return false;
    }
    if (p < dim + 1 || p > BLF_HULLND_MAX_POINTS)
    {
        std::cerr << "[ConvexHullHelper::buildConvexHull] Between " << dim + 1 << " and "
                  << BLF_HULLND_MAX_POINTS << " points are supported in " << dim << "-D." << std::endl;
        return false;
    }
    blf_handle* h = blf::threadHandle();
    if (h == nullptr) return false;
    std::vector<double> pts(dim * p);
    for (std::size_t j = 0; j < p; ++j)
        for (std::size_t c = 0; c < dim; ++c) pts[dim * j + c] = points(c, j);
    const int32_t n = static_cast<int32_t>(p);
    const int32_t M = three ? BLF_HULL3D_MAX_FACETS : BLF_HULLND_MAX_FACETS;
    if (!m_dPts.upload(pts) || !m_dN.upload(&n, 1) || !m_dA.resize(dim * M) || !m_dB.resize(M) ||
        !m_dInside.resize(1))
        return false;
    const blf_status st = three ? blf_hull3d_hrep(h, m_dPts.data(), m_dN.data(), n, M, 1, m_dA.data(),
                                                  m_dB.data(), m_dInside.data(), nullptr)
                                : blf_hullnd_hrep(h, static_cast<int32_t>(dim), m_dPts.data(), m_dN.data(),
                                                  n, M, 1, m_dA.data(), m_dB.data(), m_dInside.data(),
                                                  nullptr);
    if (!blf::report(st, "ConvexHullHelper::buildConvexHull")) return false;
    int32_t nf = -1;
    std::vector<double> A(dim * M), b(M);
    if (!m_dInside.download(&nf, 1) || !m_dA.download(A.data(), A.size()) ||
        !m_dB.download(b.data(), b.size()))
        return false;
    if (nf < 0)
    {
        std::cerr << "[ConvexHullHelper::buildConvexHull] Degenerate point set (fewer than "
                  << dim + 1 << " points spanning " << dim << " dimensions)." << std::endl;
        m_A.resize(0, dim);
        m_b.resize(0);
        return false;
    }
    // Rows as the reference's getA() has them in 3-D: Qhull's "Qt" output is one facet per
    // triangle, so a face with k vertices is k - 2 rows with the same plane
    // (ConvexHullHelper.cpp:60-86 of the reference: A is sized to facetList.count()).  The device
    // returns each distinct plane once.  In 4-D and above the count of a facet's simplices depends
    // on Qhull's triangulation, and each plane stays one row.
    std::vector<int> copies(static_cast<std::size_t>(nf), 1);
    if (dim == 3)
    {
        double scale = 1.0;
        for (const double x : pts) scale = std::max(scale, std::abs(x));
        for (int i = 0; i < nf; ++i)
            copies[i] = std::max(1, faceVertexCount(pts, p, &A[3 * i], b[i], 1e-9 * scale) - 2);
    }
    std::size_t rows = 0;
    for (const int c : copies) rows += static_cast<std::size_t>(c);
    m_A.resize(rows, dim);
    m_b.resize(rows);
    std::size_t r = 0;
    for (int i = 0; i < nf; ++i)
        for (int k = 0; k < copies[i]; ++k, ++r)
        {
            for (std::size_t c = 0; c < dim; ++c) m_A(r, c) = A[dim * i + c];
            m_b(r) = b[i];
        }
    return true;
}

bool ConvexHullHelper::buildConvexHull(const blf::MatrixXd& points)
{
    m_valid = false;
    if (points.rows() != 2 || points.cols() > BLF_HULL_MAX_POINTS)
        return m_valid = buildConvexHullN(points);
    const std::size_t p = points.cols();
    if (p < 3)
    {
        std::cerr << "[ConvexHullHelper::buildConvexHull] Between 3 and " << BLF_HULLND_MAX_POINTS
                  << " points are supported in 2-D." << std::endl;
        return false;
    }
    blf_handle* h = blf::threadHandle();
    if (h == nullptr) return false;
    std::vector<double> pts(2 * p);
    for (std::size_t j = 0; j < p; ++j)
    {
        pts[2 * j] = points(0, j);
        pts[2 * j + 1] = points(1, j);
    }
    const int32_t n = static_cast<int32_t>(p);
    const int32_t M = 2 * BLF_HULL_MAX_POINTS;
    if (!m_dPts.upload(pts) || !m_dN.upload(&n, 1) || !m_dA.resize(2 * M) || !m_dB.resize(M))
        return false;
    if (!m_dInside.resize(1)) return false;
    if (!blf::report(blf_hull2d_hrep(h, m_dPts.data(), m_dN.data(), n, M, 1, m_dA.data(),
                                     m_dB.data(), m_dInside.data(), nullptr),
                     "ConvexHullHelper::buildConvexHull"))
        return false;
    int32_t nf = -1;
    std::vector<double> A(2 * M), b(M);
    if (!m_dInside.download(&nf, 1) || !m_dA.download(A.data(), A.size()) ||
        !m_dB.download(b.data(), b.size()))
        return false;
    if (nf < 0)
    {
        std::cerr << "[ConvexHullHelper::buildConvexHull] Degenerate point set (fewer than three "
                     "non-collinear points)."
                  << std::endl;
        m_A.resize(0, 2);
        m_b.resize(0);
        return false;
    }
    m_A.resize(static_cast<std::size_t>(nf), 2);
    m_b.resize(static_cast<std::size_t>(nf));
    for (int i = 0; i < nf; ++i)
    {
        m_A(i, 0) = A[2 * i];
        m_A(i, 1) = A[2 * i + 1];
        m_b(i) = b[i];
    }
    m_valid = true;
    return true;
}

bool ConvexHullHelper::doesPointBelongToConvexHull(const blf::VectorXd& point) const
{
    if (point.size() != m_A.cols())
    {
        std::cerr << "[ConvexHullHelper::doesPointBelongToConvexHull] Unexpected size of the point."
                  << std::endl;
        return false;
    }
    if (!m_valid)
    {
        std::cerr << "[ConvexHullHelper::doesPointBelongToConvexHull] No convex hull: the last "
                     "buildConvexHull failed or was never called."
                  << std::endl;
        return false;
    }
    blf_handle* h = blf::threadHandle();
    if (h == nullptr) return false;
    auto* self = const_cast<ConvexHullHelper*>(this);
    const int32_t nf = static_cast<int32_t>(m_A.rows());
    if (m_A.cols() != 2)
    {
        const int32_t D = static_cast<int32_t>(m_A.cols());
        const int32_t M = nf > 0 ? nf : 1;
        std::vector<double> A(static_cast<std::size_t>(D) * M, 0.0), b(M, 0.0);
        for (int32_t i = 0; i < nf; ++i)
        {
            for (int32_t c = 0; c < D; ++c) A[static_cast<std::size_t>(D) * i + c] = m_A(i, c);
            b[i] = m_b(i);
        }
        if (!self->m_dA.upload(A) || !self->m_dB.upload(b) || !self->m_dN.upload(&nf, 1) ||
            !self->m_dQ.upload(point.data(), D) || !self->m_dInside.resize(1))
            return false;
        if (!blf::report(blf_halfspace_contains(h, self->m_dA.data(), self->m_dB.data(),
                                                self->m_dN.data(), D, M, self->m_dQ.data(), 1,
                                                self->m_dInside.data(), nullptr),
                         "ConvexHullHelper::doesPointBelongToConvexHull"))
            return false;
        int32_t inside = 0;
        return self->m_dInside.download(&inside, 1) && inside == 1;
    }
    const int32_t M = nf > 0 ? nf : 1;
    std::vector<double> A(2 * M, 0.0), b(M, 0.0);
    for (int32_t i = 0; i < nf; ++i)
    {
        A[2 * i] = m_A(i, 0);
        A[2 * i + 1] = m_A(i, 1);
        b[i] = m_b(i);
    }
    if (!self->m_dA.upload(A) || !self->m_dB.upload(b) || !self->m_dN.upload(&nf, 1) ||
        !self->m_dQ.upload(point.data(), 2) || !self->m_dInside.resize(1))
        return false;
    if (!blf::report(blf_hull2d_contains(h, self->m_dA.data(), self->m_dB.data(), self->m_dN.data(),
                                         M, self->m_dQ.data(), 1, self->m_dInside.data(), nullptr),
                     "ConvexHullHelper::doesPointBelongToConvexHull"))
        return false;
    int32_t inside = 0;
    return self->m_dInside.download(&inside, 1) && inside == 1;
}
