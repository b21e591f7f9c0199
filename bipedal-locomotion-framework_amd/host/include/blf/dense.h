/**
 * @file dense.h
 * Minimal dense vector / matrix value types used by the C++ adapters in place of Eigen (not
 * available in this build).  Any Eigen-like matrix (rows(), cols(), operator()(i, j)) is
 * accepted by the adapters' templated setters, so caller code written against the reference's
 * Eigen::Ref<const Eigen::MatrixXd> signatures keeps compiling when Eigen is present.
 */
#ifndef BLF_HOST_DENSE_H
#define BLF_HOST_DENSE_H

#include <cstddef>
#include <initializer_list>
#include <vector>

namespace blf
{

class VectorXd
{
    std::vector<double> m_v;

public:
    VectorXd() = default;
    explicit VectorXd(std::size_t n, double value = 0.0) : m_v(n, value) {}
    VectorXd(std::initializer_list<double> l) : m_v(l) {}
    std::size_t size() const { return m_v.size(); }
    void resize(std::size_t n) { m_v.resize(n); }
    void setZero() { for (double& x : m_v) x = 0.0; }
    double& operator()(std::size_t i) { return m_v[i]; }
    double operator()(std::size_t i) const { return m_v[i]; }
    double& operator[](std::size_t i) { return m_v[i]; }
    double operator[](std::size_t i) const { return m_v[i]; }
    double* data() { return m_v.data(); }
    const double* data() const { return m_v.data(); }
};

/** Row-major dense matrix. */
class MatrixXd
{
    std::size_t m_rows{0}, m_cols{0};
    std::vector<double> m_v;

public:
    MatrixXd() = default;
    MatrixXd(std::size_t r, std::size_t c, double value = 0.0) : m_rows(r), m_cols(c), m_v(r * c, value) {}
    MatrixXd(std::size_t r, std::size_t c, std::initializer_list<double> rowMajor)
        : m_rows(r), m_cols(c), m_v(rowMajor)
    {
        m_v.resize(r * c, 0.0);
    }
    std::size_t rows() const { return m_rows; }
    std::size_t cols() const { return m_cols; }
    void resize(std::size_t r, std::size_t c) { m_rows = r; m_cols = c; m_v.assign(r * c, 0.0); }
    double& operator()(std::size_t i, std::size_t j) { return m_v[i * m_cols + j]; }
    double operator()(std::size_t i, std::size_t j) const { return m_v[i * m_cols + j]; }
    double* data() { return m_v.data(); }
    const double* data() const { return m_v.data(); }

    /** Copy any matrix-like object exposing rows(), cols(), operator()(i, j). */
    template <class Mat> static MatrixXd from(const Mat& m)
    {
        MatrixXd out(static_cast<std::size_t>(m.rows()), static_cast<std::size_t>(m.cols()));
        for (std::size_t i = 0; i < out.rows(); ++i)
            for (std::size_t j = 0; j < out.cols(); ++j) out(i, j) = m(i, j);
        return out;
    }
};

} // namespace blf

#endif // BLF_HOST_DENSE_H
