/**
 * @file ConvexHullHelper.cpp
 * Single-polygon calls into the batched device kernels (batch = 1).
 */
#include <iostream>

#include <BipedalLocomotion/Planners/ConvexHullHelper.h>

using namespace BipedalLocomotion::Planners;

// 3 x p points: blf_hull3d_hrep (the distinct supporting planes; ConvexHullHelperTest.cpp:15-63).
bool ConvexHullHelper::buildConvexHull3(const blf::MatrixXd& points)
{
    const std::size_t p = points.cols();
    if (p < 4 || p > BLF_HULL_MAX_POINTS)
    {
        std::cerr << "[ConvexHullHelper::buildConvexHull] Between 4 and " << BLF_HULL_MAX_POINTS
                  << " points are supported in 3-D." << std::endl;
        return false;
    }
    blf_handle* h = blf::threadHandle();
    if (h == nullptr) return false;
    std::vector<double> pts(3 * p);
    for (std::size_t j = 0; j < p; ++j)
        for (std::size_t c = 0; c < 3; ++c) pts[3 * j + c] = points(c, j);
    const int32_t n = static_cast<int32_t>(p);
    const int32_t M = BLF_HULL3D_MAX_FACETS;
    if (!m_dPts.upload(pts) || !m_dN.upload(&n, 1) || !m_dA.resize(3 * M) || !m_dB.resize(M) ||
        !m_dInside.resize(1))
        return false;
    if (!blf::report(blf_hull3d_hrep(h, m_dPts.data(), m_dN.data(), n, M, 1, m_dA.data(),
                                     m_dB.data(), m_dInside.data(), nullptr),
                     "ConvexHullHelper::buildConvexHull"))
        return false;
    int32_t nf = -1;
    std::vector<double> A(3 * M), b(M);
    if (!m_dInside.download(&nf, 1) || !m_dA.download(A.data(), A.size()) ||
        !m_dB.download(b.data(), b.size()))
        return false;
    if (nf < 0)
    {
        std::cerr << "[ConvexHullHelper::buildConvexHull] Degenerate point set (fewer than four "
                     "points not in one plane)."
                  << std::endl;
        m_A.resize(0, 3);
        m_b.resize(0);
        return false;
    }
    m_A.resize(static_cast<std::size_t>(nf), 3);
    m_b.resize(static_cast<std::size_t>(nf));
    for (int i = 0; i < nf; ++i)
    {
        for (int c = 0; c < 3; ++c) m_A(i, c) = A[3 * i + c];
        m_b(i) = b[i];
    }
    return true;
}

bool ConvexHullHelper::buildConvexHull(const blf::MatrixXd& points)
{
    m_valid = false;
    if (points.rows() == 3) return m_valid = buildConvexHull3(points);
    if (points.rows() != 2)
    {
        std::cerr << "[ConvexHullHelper::buildConvexHull] Only 2-D and 3-D point sets are "
                     "supported by the device hull."
                  << std::endl;
        return false;
    }
    const std::size_t p = points.cols();
    if (p < 3 || p > BLF_HULL_MAX_POINTS)
    {
        std::cerr << "[ConvexHullHelper::buildConvexHull] Between 3 and " << BLF_HULL_MAX_POINTS
                  << " points are supported." << std::endl;
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
