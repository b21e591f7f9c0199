/**
 * @file ContactWrench.h
 * Drop-in for src/System/include/BipedalLocomotion/System/ContactWrench.h:23-56: a contact model
 * acting on a frame of the robot model (the frame index replaces iDynTree::FrameIndex).
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_SYSTEM_CONTACT_WRENCH_H
#define BLF_BIPEDAL_LOCOMOTION_SYSTEM_CONTACT_WRENCH_H

#include <memory>

#include <BipedalLocomotion/ContactModels/ContactModel.h>

namespace BipedalLocomotion
{
namespace System
{

class ContactWrench
{
    int m_frame;
    std::shared_ptr<ContactModels::ContactModel> m_contactModel;

public:
    ContactWrench(const int& index, std::shared_ptr<ContactModels::ContactModel> model)
        : m_frame(index), m_contactModel(std::move(model))
    {
    }
    int& index() noexcept { return m_frame; }
    const int& index() const noexcept { return m_frame; }
    const std::weak_ptr<ContactModels::ContactModel> contactModel() const noexcept
    {
        return m_contactModel;
    }
};

} // namespace System
} // namespace BipedalLocomotion

#endif
