/**
 * @file IParametersHandler.h
 * The subset of src/ParametersHandler/include/BipedalLocomotion/ParametersHandler/
 * IParametersHandler.h:26-249 that the DCM path's initialize() calls read (getParameter of
 * scalars/vectors by key), plus an in-memory StdImplementation.  The YARP-backed handler and
 * group nesting are out of scope.
 */
#ifndef BLF_BIPEDAL_LOCOMOTION_PARAMETERS_HANDLER_H
#define BLF_BIPEDAL_LOCOMOTION_PARAMETERS_HANDLER_H

#include <map>
#include <memory>
#include <string>
#include <vector>

namespace BipedalLocomotion
{
namespace ParametersHandler
{

class IParametersHandler
{
public:
    virtual bool getParameter(const std::string& name, double& value) const = 0;
    virtual bool getParameter(const std::string& name, int& value) const = 0;
    virtual bool getParameter(const std::string& name, std::vector<double>& value) const = 0;
    virtual void setParameter(const std::string& name, double value) = 0;
    virtual void setParameter(const std::string& name, int value) = 0;
    virtual void setParameter(const std::string& name, const std::vector<double>& value) = 0;
    virtual ~IParametersHandler() = default;
};

class StdImplementation : public IParametersHandler
{
    std::map<std::string, std::vector<double>> m_values;

public:
    bool getParameter(const std::string& name, double& value) const override
    {
        auto it = m_values.find(name);
        if (it == m_values.end() || it->second.size() != 1) return false;
        value = it->second[0];
        return true;
    }
    bool getParameter(const std::string& name, int& value) const override
    {
        double d;
        if (!getParameter(name, d)) return false;
        value = static_cast<int>(d);
        return static_cast<double>(value) == d;
    }
    bool getParameter(const std::string& name, std::vector<double>& value) const override
    {
        auto it = m_values.find(name);
        if (it == m_values.end()) return false;
        value = it->second;
        return true;
    }
    void setParameter(const std::string& name, double value) override { m_values[name] = {value}; }
    void setParameter(const std::string& name, int value) override
    {
        m_values[name] = {static_cast<double>(value)};
    }
    void setParameter(const std::string& name, const std::vector<double>& value) override
    {
        m_values[name] = value;
    }
};

} // namespace ParametersHandler
} // namespace BipedalLocomotion

#endif
