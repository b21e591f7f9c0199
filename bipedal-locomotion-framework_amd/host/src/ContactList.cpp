/**
 * @file ContactList.cpp
 * Semantics of src/Planners/src/ContactList.cpp (ordering, overlap rejection, editContact
 * neighbour checks, getPresentContact `<=` rule); messages keep the reference's prefixes.
 */
#include <cassert>
#include <iostream>
#include <iterator>

#include <BipedalLocomotion/Planners/ContactList.h>

using namespace BipedalLocomotion::Planners;

bool ContactList::addContact(const Contact& newContact)
{
    if (newContact.activationTime > newContact.deactivationTime)
    {
        std::cerr << "[ContactList::addContact] The activation time cannot be greater than the "
                     "deactivation time."
                  << std::endl;
        return false;
    }
    const auto res = m_contacts.insert(newContact);
    if (!res.second)
    {
        std::cerr << "[ContactList::addContact] Failed to insert new element. The new contact "
                     "(activationTime: "
                  << newContact.activationTime << " deactivationTime: "
                  << newContact.deactivationTime
                  << ") is not compatible with an element already present in the list "
                     "(activationTime: "
                  << res.first->activationTime << " deactivationTime: "
                  << res.first->deactivationTime << ")" << std::endl;
        return false;
    }
    return true;
}

bool ContactList::addContact(const Transform& newTransform, double activationTime,
                             double deactivationTime)
{
    Contact c;
    c.pose = newTransform;
    c.activationTime = activationTime;
    c.deactivationTime = deactivationTime;
    c.name = m_defaultName;
    c.type = m_defaultContactType;
    return addContact(c);
}

const Contact& ContactList::operator[](std::size_t index) const
{
    assert(index < size());
    // walk from the closer end
    if (index > size() / 2)
        return *std::next(rbegin(), static_cast<std::ptrdiff_t>(size() - index - 1));
    return *std::next(begin(), static_cast<std::ptrdiff_t>(index));
}

bool ContactList::editContact(const_iterator element, const Contact& newContact)
{
    if (element == end())
    {
        std::cerr << "[ContactList::addContact] The element is not valid." << std::endl;
        return false;
    }
    if (element != begin())
    {
        const auto previous = std::prev(element);
        if (newContact.activationTime < previous->deactivationTime)
        {
            std::cerr << "[ContactList::addContact] The new contact cannot have an activation "
                         "time smaller than the previous contact."
                      << std::endl;
            return false;
        }
    }
    const auto next = std::next(element);
    if (next != end() && newContact.deactivationTime > next->activationTime)
    {
        std::cerr << "[ContactList::addContact] The new contact cannot have a deactivation time "
                     "greater than the next contact."
                  << std::endl;
        return false;
    }
    m_contacts.erase(element);
    m_contacts.insert(next, newContact);
    return true;
}

ContactList::const_iterator ContactList::getPresentContact(double time) const
{
    for (auto it = rbegin(); it != rend(); ++it)
        if (it->activationTime <= time) return std::prev(it.base());
    return end();
}

bool ContactList::keepOnlyPresentContact(double time)
{
    const auto present = getPresentContact(time);
    if (present == end())
    {
        std::cerr << "[ContactList::addContact] No contact has activation time lower than the "
                     "specified time."
                  << std::endl;
        return false;
    }
    const Contact keep = *present;
    clear();
    addContact(keep);
    return true;
}
