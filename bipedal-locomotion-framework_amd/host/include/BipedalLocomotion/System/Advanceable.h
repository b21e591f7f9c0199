/**
 * @file Advanceable.h
 * Drop-in for src/System/include/BipedalLocomotion/System/Advanceable.h:24-46: the receding-
 * horizon surface (get / isValid / advance).  blf's TimeVaryingDCMPlanner implements it.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_SYSTEM_ADVANCEABLE_H
#define BLF_BIPEDAL_LOCOMOTION_SYSTEM_ADVANCEABLE_H

namespace BipedalLocomotion
{
namespace System
{

template <typename T> class Advanceable
{
public:
    /** The current output (valid until the next advance()). */
    virtual const T& get() const = 0;

    /** True when get() holds a valid output. */
    virtual bool isValid() const = 0;

    /** Move the internal state one step forward; may change get(). */
    virtual bool advance() = 0;

    virtual ~Advanceable() = default;
};

} // namespace System
} // namespace BipedalLocomotion

#endif
