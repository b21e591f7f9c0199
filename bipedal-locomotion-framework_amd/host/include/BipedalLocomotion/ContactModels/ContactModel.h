/**
 * @file ContactModel.h
 * Drop-in for src/ContactModels/include/BipedalLocomotion/ContactModels/ContactModel.h:25-132
 * (src/ContactModels/src/ContactModel.cpp:12-92): the lazy-cache protocol.  initialize(),
 * setState() and setNullForceTransform() invalidate the four cached quantities; each get*()
 * computes its own quantity once (on the device, in the derived class) and returns the cache.
 * The get*() methods are non-const, as in the reference.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_CONTACT_MODELS_CONTACT_MODEL_H
#define BLF_BIPEDAL_LOCOMOTION_CONTACT_MODELS_CONTACT_MODEL_H

#include <memory>

#include <BipedalLocomotion/ParametersHandler/IParametersHandler.h>
#include <blf/dense.h>
#include <blf/spatial.h>

namespace BipedalLocomotion
{
namespace ContactModels
{

class ContactModel
{
    bool m_isContactWrenchComputed{false};
    bool m_isAutonomousDynamicsComputed{false};
    bool m_isControlMatrixComputed{false};
    bool m_isRegressorComputed{false};

    void invalidate()
    {
        m_isContactWrenchComputed = false;
        m_isControlMatrixComputed = false;
        m_isAutonomousDynamicsComputed = false;
        m_isRegressorComputed = false;
    }

protected:
    blf::Wrench m_contactWrench{};        /**< (force, torque), mixed representation */
    blf::Vector6 m_autonomousDynamics{};
    blf::Matrix6x6 m_controlMatrix{};
    blf::MatrixXd m_regressor{6, 2};

    virtual void computeContactWrench() = 0;
    virtual void computeAutonomousDynamics() = 0;
    virtual void computeControlMatrix() = 0;
    virtual void computeRegressor() = 0;
    virtual bool initializePrivate(std::weak_ptr<ParametersHandler::IParametersHandler> handler) = 0;
    virtual void setStatePrivate(const blf::Twist& twist, const blf::Transform& transform) = 0;
    virtual void setNullForceTransformPrivate(const blf::Transform& transform) = 0;

public:
    virtual ~ContactModel() = default;

    bool initialize(std::weak_ptr<ParametersHandler::IParametersHandler> handler)
    {
        invalidate();
        return initializePrivate(handler);
    }
    const blf::Wrench& getContactWrench()
    {
        if (!m_isContactWrenchComputed)
        {
            computeContactWrench();
            m_isContactWrenchComputed = true;
        }
        return m_contactWrench;
    }
    const blf::Vector6& getAutonomousDynamics()
    {
        if (!m_isAutonomousDynamicsComputed)
        {
            computeAutonomousDynamics();
            m_isAutonomousDynamicsComputed = true;
        }
        return m_autonomousDynamics;
    }
    const blf::Matrix6x6& getControlMatrix()
    {
        if (!m_isControlMatrixComputed)
        {
            computeControlMatrix();
            m_isControlMatrixComputed = true;
        }
        return m_controlMatrix;
    }
    const blf::MatrixXd& getRegressor()
    {
        if (!m_isRegressorComputed)
        {
            computeRegressor();
            m_isRegressorComputed = true;
        }
        return m_regressor;
    }
    void setState(const blf::Twist& twist, const blf::Transform& transform)
    {
        invalidate();
        setStatePrivate(twist, transform);
    }
    void setNullForceTransform(const blf::Transform& transform)
    {
        invalidate();
        setNullForceTransformPrivate(transform);
    }
};

} // namespace ContactModels
} // namespace BipedalLocomotion

#endif
