/**
 * @file ContinuousContactModel.h
 * Drop-in for src/ContactModels/include/BipedalLocomotion/ContactModels/ContinuousContactModel.h
 * (src/ContactModels/src/ContinuousContactModel.cpp): rectangular L x W contact patch of
 * springs k and dampers b.  Every quantity is computed on the device (blf_contact_model_eval /
 * blf_contact_point_wrench, include/blf/blf_c.h); on a device error the quantity is filled with
 * NaN and "[ContinuousContactModel::...]" is printed — there is no host fallback.
 * Parameters (initialize): "length", "width", "spring_coeff", "damper_coeff" (doubles).
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_CONTACT_MODELS_CONTINUOUS_CONTACT_MODEL_H
#define BLF_BIPEDAL_LOCOMOTION_CONTACT_MODELS_CONTINUOUS_CONTACT_MODEL_H

#include <vector>

#include <BipedalLocomotion/ContactModels/ContactModel.h>
#include <blf/device.h>

namespace BipedalLocomotion
{
namespace ContactModels
{

class ContinuousContactModel final : public ContactModel
{
    blf::Transform m_frameTransform;
    blf::Transform m_nullForceTransform;
    blf::Twist m_twist{};
    double m_springCoeff{0.0};
    double m_damperCoeff{0.0};
    double m_length{0.0};
    double m_width{0.0};
    blf::DeviceBuffer<double> m_dIn, m_dOut;

    /** Upload params / twist / pose / null pose; returns the packed device pointers. */
    bool upload();
    void evaluate(int which, double* host, int n, const char* where);

    void computeContactWrench() final;
    void computeAutonomousDynamics() final;
    void computeControlMatrix() final;
    void computeRegressor() final;
    bool initializePrivate(std::weak_ptr<ParametersHandler::IParametersHandler> handler) final;
    void setStatePrivate(const blf::Twist& twist, const blf::Transform& transform) final;
    void setNullForceTransformPrivate(const blf::Transform& transform) final;

public:
    ContinuousContactModel();

    /** Force on the surface element at (x, y) of the contact frame (zero outside the patch). */
    blf::Vector3 getForceAtPoint(const double& x, const double& y);
    /** Torque of that force about the contact frame origin. */
    blf::Vector3 getTorqueGeneratedAtPoint(const double& x, const double& y);
    /** Batched form of the two: points = {x0, y0, x1, y1, ...}; force / torque 3 per point. */
    bool getWrenchesAtPoints(const std::vector<double>& points, std::vector<double>& force,
                             std::vector<double>& torque);

    const double& length() const { return m_length; }
    const double& width() const { return m_width; }
    const blf::Transform& nullForceTransform() const { return m_nullForceTransform; }
    const double& springCoeff() const { return m_springCoeff; }
    double& springCoeff() { return m_springCoeff; }
    const double& damperCoeff() const { return m_damperCoeff; }
    double& damperCoeff() { return m_damperCoeff; }
};

} // namespace ContactModels
} // namespace BipedalLocomotion

#endif
