/**
 * @file ContactList.h
 * Drop-in for src/Planners/include/BipedalLocomotion/Planners/ContactList.h:32-210
 * (src/Planners/src/ContactList.cpp).  An ordered set of non-overlapping contacts of one
 * end-effector: contact a precedes b iff a.deactivationTime < b.activationTime, so overlapping
 * or touching intervals are "equal" and the second insertion fails.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_PLANNERS_CONTACT_LIST_H
#define BLF_BIPEDAL_LOCOMOTION_PLANNERS_CONTACT_LIST_H

#include <cstddef>
#include <set>
#include <string>

#include <BipedalLocomotion/Planners/Contact.h>

namespace BipedalLocomotion
{
namespace Planners
{

class ContactList
{
    struct ContactCompare
    {
        bool operator()(const Contact& lhs, const Contact& rhs) const
        {
            return lhs.deactivationTime < rhs.activationTime;
        }
    };

    std::set<Contact, ContactCompare> m_contacts;
    std::string m_defaultName{"ContactList"};
    ContactType m_defaultContactType{ContactType::FULL};

public:
    using const_iterator = std::set<Contact, ContactCompare>::const_iterator;
    using const_reverse_iterator = std::set<Contact, ContactCompare>::const_reverse_iterator;

    void setDefaultName(const std::string& defaultName) { m_defaultName = defaultName; }
    const std::string& defaultName() const { return m_defaultName; }
    void setDefaultContactType(const ContactType& type) { m_defaultContactType = type; }
    const ContactType& defaultContactType() const { return m_defaultContactType; }

    /** false if activation > deactivation or the interval meets an existing contact. */
    bool addContact(const Contact& newContact);
    bool addContact(const Transform& newTransform, double activationTime, double deactivationTime);

    const_iterator erase(const_iterator iterator) { return m_contacts.erase(iterator); }
    const_iterator begin() const { return m_contacts.begin(); }
    const_iterator cbegin() const { return m_contacts.cbegin(); }
    const_reverse_iterator rbegin() const { return m_contacts.rbegin(); }
    const_reverse_iterator crbegin() const { return m_contacts.crbegin(); }
    const_iterator end() const { return m_contacts.end(); }
    const_iterator cend() const { return m_contacts.cend(); }
    const_reverse_iterator rend() const { return m_contacts.rend(); }
    const_reverse_iterator crend() const { return m_contacts.crend(); }

    const Contact& operator[](std::size_t index) const;
    std::size_t size() const { return m_contacts.size(); }
    const_iterator firstContact() const { return begin(); }
    const_iterator lastContact() const { return std::prev(end()); }

    /** Replace *element if the new interval still fits between its neighbours. */
    bool editContact(const_iterator element, const Contact& newContact);

    /** The last contact whose activation time is <= time, or end() if none. */
    const_iterator getPresentContact(double time) const;

    /** Keep only getPresentContact(time); false if there is none. */
    bool keepOnlyPresentContact(double time);

    void clear() { m_contacts.clear(); }
    void removeLastContact() { erase(lastContact()); }
};

} // namespace Planners
} // namespace BipedalLocomotion

#endif
