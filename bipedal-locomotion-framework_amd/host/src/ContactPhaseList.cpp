/**
 * @file ContactPhaseList.cpp
 * Event sweep over the activation / deactivation instants of all lists (semantics of
 * src/Planners/src/ContactPhaseList.cpp:16-84, restated in oracle/blf_oracle.c:
 * orc_contact_phases and pinned by tests/golden/contact_phases.json).
 */
#include <cassert>
#include <iostream>
#include <utility>

#include <BipedalLocomotion/Planners/ContactPhaseList.h>

using namespace BipedalLocomotion::Planners;

namespace
{
using Event = std::pair<std::string, ContactList::const_iterator>;
using Events = std::map<double, std::vector<Event>>;   // one entry per distinct instant
} // namespace

void ContactPhaseList::createPhases()
{
    m_phases.clear();
    Events act, deact;
    for (const auto& [name, list] : m_contactLists)
        for (auto it = list.begin(); it != list.end(); ++it)
        {
            act[it->activationTime].emplace_back(name, it);
            deact[it->deactivationTime].emplace_back(name, it);
        }
    if (act.empty()) return;

    auto a = act.begin();
    auto d = deact.begin();
    ContactPhase current;
    current.beginTime = a->first;
    for (const auto& e : a->second) current.activeContacts.insert(e);
    ++a;

    auto remaining = [&]() {
        return static_cast<std::size_t>(std::distance(a, act.end())) +
               static_cast<std::size_t>(std::distance(d, deact.end()));
    };
    auto close = [&](double t) {
        current.endTime = t;
        m_phases.push_back(current);
        current.beginTime = t;
    };
    while (remaining() > 1)
    {
        if (a == act.end() || d->first <= a->first)
        {
            close(d->first);
            for (const auto& e : d->second) current.activeContacts.erase(e.first);
            ++d;
            // the reference compares the NEXT deactivation with the next activation here
            if (a != act.end() && d != deact.end() && d->first == a->first)
            {
                for (const auto& e : a->second) current.activeContacts.insert(e);
                ++a;
            }
        } else
        {
            close(a->first);
            for (const auto& e : a->second) current.activeContacts.insert(e);
            ++a;
        }
    }
    assert(d != deact.end() && std::next(d) == deact.end());
    current.endTime = d->first;
    m_phases.push_back(current);
}

void ContactPhaseList::setLists(const ContactListMap& contactLists)
{
    m_contactLists = contactLists;
    createPhases();
}

bool ContactPhaseList::setLists(const std::initializer_list<ContactList>& contactLists)
{
    m_contactLists.clear();
    for (const ContactList& list : contactLists)
    {
        if (!m_contactLists.emplace(list.defaultName(), list).second)
        {
            std::cerr << "[ContactPhaseList::setLists] Multiple items have the same defaultName."
                      << std::endl;
            return false;
        }
    }
    createPhases();
    return true;
}

int ContactPhaseList::phaseIndexAt(double t) const
{
    for (std::size_t i = 0; i < m_phases.size(); ++i)
        if (m_phases[i].beginTime <= t && t < m_phases[i].endTime) return static_cast<int>(i);
    return -1;
}
