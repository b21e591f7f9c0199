/**
 * @file VariablesHandler.h
 * Drop-in for src/System/include/BipedalLocomotion/System/VariablesHandler.h:24-53
 * (src/System/src/VariablesHandler.cpp:13-48): named contiguous blocks of optimisation
 * variables.  The DCM QP's layout is ("dcm", 2(N+1)) then ("vrp", 2N).
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_SYSTEM_VARIABLES_HANDLER_H
#define BLF_BIPEDAL_LOCOMOTION_SYSTEM_VARIABLES_HANDLER_H

#include <cstddef>
#include <string>
#include <unordered_map>

namespace BipedalLocomotion
{
namespace System
{

/** Stand-in for iDynTree::IndexRange (offset, size; invalid = negative). */
struct IndexRange
{
    std::ptrdiff_t offset{-1};
    std::ptrdiff_t size{-1};
    bool isValid() const { return offset >= 0 && size >= 0; }
    static IndexRange InvalidRange() { return IndexRange{}; }
};

class VariablesHandler
{
    std::unordered_map<std::string, IndexRange> m_variables;
    std::size_t m_numberOfVariables{0};

public:
    /** Append a block; false if the name already exists. */
    bool addVariable(const std::string& name, const std::size_t& size) noexcept;
    /** The block's range, or IndexRange::InvalidRange() if unknown. */
    IndexRange getVariable(const std::string& name) const noexcept;
    const std::size_t& getNumberOfVariables() const noexcept;
};

} // namespace System
} // namespace BipedalLocomotion

#endif
