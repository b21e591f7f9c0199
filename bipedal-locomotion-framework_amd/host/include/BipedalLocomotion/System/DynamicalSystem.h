/**
 * @file DynamicalSystem.h
 * Drop-in for src/System/include/BipedalLocomotion/System/DynamicalSystem.h:33-104 (+ .tpp):
 * tuple-typed state / derivative / input, value-copy setters, pure dynamics(t, dx).  The
 * initialize entry point keeps the reference's spelling `initalize`.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_SYSTEM_DYNAMICAL_SYSTEM_H
#define BLF_BIPEDAL_LOCOMOTION_SYSTEM_DYNAMICAL_SYSTEM_H

#include <memory>
#include <tuple>
#include <type_traits>

#include <BipedalLocomotion/ParametersHandler/IParametersHandler.h>

namespace BipedalLocomotion
{

template <typename T, template <typename...> class Ref> struct is_specialization : std::false_type
{
};
template <template <typename...> class Ref, typename... Args>
struct is_specialization<Ref<Args...>, Ref> : std::true_type
{
};

namespace System
{

template <typename State, typename StateDerivative, typename Input> class DynamicalSystem
{
    static_assert(is_specialization<State, std::tuple>::value,
                  "The State type must be a specialization of std::tuple.");
    static_assert(is_specialization<StateDerivative, std::tuple>::value,
                  "The StateDerivative type must be a specialization of std::tuple.");
    static_assert(is_specialization<Input, std::tuple>::value,
                  "The Input type must be a specialization of std::tuple.");

public:
    using StateType = State;
    using StateDerivativeType = StateDerivative;
    using InputType = Input;

protected:
    InputType m_controlInput;
    StateType m_state;

public:
    virtual bool initalize(std::weak_ptr<ParametersHandler::IParametersHandler> handler)
    {
        (void)handler;
        return true;
    }
    virtual bool setState(const StateType& state)
    {
        m_state = state;
        return true;
    }
    const StateType& getState() const { return m_state; }
    virtual bool setControlInput(const InputType& controlInput)
    {
        m_controlInput = controlInput;
        return true;
    }
    virtual bool dynamics(const double& time, StateDerivativeType& stateDerivative) = 0;
    virtual ~DynamicalSystem() = default;
};

} // namespace System
} // namespace BipedalLocomotion

#endif
