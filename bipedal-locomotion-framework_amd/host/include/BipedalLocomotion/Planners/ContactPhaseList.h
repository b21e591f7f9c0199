/**
 * @file ContactPhaseList.h
 * Drop-in for src/Planners/include/BipedalLocomotion/Planners/ContactPhase.h:25-48 and
 * ContactPhaseList.h:32-141 (src/Planners/src/ContactPhaseList.cpp:16-181).  Merges named
 * contact lists into phases [begin, end) with their active contacts.  The merge reproduces the
 * reference's sweep including its quirks: deactivations win ties with activations, and after a
 * deactivation event the NEXT deactivation time is compared with the next activation time
 * (ContactPhaseList.cpp:60), so coincident events can produce zero-length phases.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_PLANNERS_CONTACT_PHASE_LIST_H
#define BLF_BIPEDAL_LOCOMOTION_PLANNERS_CONTACT_PHASE_LIST_H

#include <cstddef>
#include <initializer_list>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include <BipedalLocomotion/Planners/ContactList.h>

namespace BipedalLocomotion
{
namespace Planners
{

struct ContactPhase
{
    double beginTime{0.0};
    double endTime{0.0};
    /** list name -> the active contact of that list (iterator into ContactPhaseList::lists()) */
    std::unordered_map<std::string, ContactList::const_iterator> activeContacts;
    bool isListIncluded(const std::string& key) const { return activeContacts.count(key) != 0; }
};

using ContactListMap = std::map<std::string, ContactList>;

class ContactPhaseList
{
    ContactListMap m_contactLists;
    std::vector<ContactPhase> m_phases;
    void createPhases();

public:
    using const_iterator = std::vector<ContactPhase>::const_iterator;
    using const_reverse_iterator = std::vector<ContactPhase>::const_reverse_iterator;

    void setLists(const ContactListMap& contactLists);
    /** Lists keyed by their defaultName(); false if two share a name. */
    bool setLists(const std::initializer_list<ContactList>& contactLists);
    const ContactListMap& lists() const { return m_contactLists; }

    const_iterator begin() const { return m_phases.begin(); }
    const_iterator cbegin() const { return m_phases.cbegin(); }
    const_reverse_iterator rbegin() const { return m_phases.rbegin(); }
    const_reverse_iterator crbegin() const { return m_phases.crbegin(); }
    const_iterator end() const { return m_phases.end(); }
    const_iterator cend() const { return m_phases.cend(); }
    const_reverse_iterator rend() const { return m_phases.rend(); }
    const_reverse_iterator crend() const { return m_phases.crend(); }
    const ContactPhase& operator[](std::size_t index) const { return m_phases[index]; }
    const_iterator firstPhase() const { return m_phases.begin(); }
    const_iterator lastPhase() const { return std::prev(m_phases.end()); }
    std::size_t size() const { return m_phases.size(); }
    void clear()
    {
        m_phases.clear();
        m_contactLists.clear();
    }

    /** Index of the phase with begin <= t < end, or -1 (the planners' knot -> phase rule). */
    int phaseIndexAt(double t) const;
};

} // namespace Planners
} // namespace BipedalLocomotion

#endif
