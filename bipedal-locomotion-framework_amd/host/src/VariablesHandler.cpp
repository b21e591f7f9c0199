/**
 * @file VariablesHandler.cpp
 */
#include <iostream>

#include <BipedalLocomotion/System/VariablesHandler.h>

using namespace BipedalLocomotion::System;

bool VariablesHandler::addVariable(const std::string& name, const std::size_t& size) noexcept
{
    if (m_variables.count(name) != 0)
    {
        std::cerr << "[VariableHandler::addVariable] The variable name " << name
                  << " already exists";
        return false;
    }
    IndexRange range;
    range.offset = static_cast<std::ptrdiff_t>(m_numberOfVariables);
    range.size = static_cast<std::ptrdiff_t>(size);
    m_variables.emplace(name, range);
    m_numberOfVariables += size;
    return true;
}

IndexRange VariablesHandler::getVariable(const std::string& name) const noexcept
{
    const auto it = m_variables.find(name);
    return it == m_variables.end() ? IndexRange::InvalidRange() : it->second;
}

const std::size_t& VariablesHandler::getNumberOfVariables() const noexcept
{
    return m_numberOfVariables;
}
