/**
 * @file QuinticSpline.h
 * QuinticSpline (absent from the reference snapshot): piecewise quintic
 * through K+1 knots with position / velocity / acceleration prescribed at every knot, in D <= 3
 * axes.  Fitting and evaluation run on the device (blf_quintic_fit / blf_quintic_eval).  The
 * segment used for a query t is the last knot with t_j <= t clamped to [0, K-1] — the
 * getPresentContact rule of src/Planners/src/ContactList.cpp:190-202; the raw index (-1 before
 * the first knot) is reported as well.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_PLANNERS_QUINTIC_SPLINE_H
#define BLF_BIPEDAL_LOCOMOTION_PLANNERS_QUINTIC_SPLINE_H

#include <cstdint>
#include <vector>

#include <blf/device.h>

namespace BipedalLocomotion
{
namespace Planners
{

class QuinticSpline
{
    int m_knots{0};
    int m_dim{0};
    blf::DeviceBuffer<double> m_dT, m_dPva, m_dCoeffs, m_dQ, m_dOut;
    blf::DeviceBuffer<int32_t> m_dIdx;
    std::vector<double> m_times;

public:
    /**
     * times: K+1 increasing knot times; position/velocity/acceleration: (K+1) x D values each,
     * row-major (knot-major).
     */
    bool setKnots(const std::vector<double>& times, int dim, const std::vector<double>& position,
                  const std::vector<double>& velocity, const std::vector<double>& acceleration);

    /** Evaluate at each query time: pva [Q][3][D] (position, velocity, acceleration). */
    bool evaluate(const std::vector<double>& queries, std::vector<double>& pva,
                  std::vector<int32_t>& knotIndex);

    /** Coefficients [K][D][6] of p(tau) = sum c_i tau^i on each segment. */
    bool coefficients(std::vector<double>& coeffs) const;

    int numberOfKnots() const { return m_knots; }
    int dimension() const { return m_dim; }
};

} // namespace Planners
} // namespace BipedalLocomotion

#endif
