/**
 * @file IParametersHandler.h
 * The parameter-handler interface of src/ParametersHandler/include/BipedalLocomotion/
 * ParametersHandler/IParametersHandler.h:26-249 (scalars, strings, booleans and vectors of them
 * by key, nested groups, toString / isEmpty / clear), and StdImplementation, an in-memory handler
 * that also reads the reference's configuration files: the `.ini` format of
 * src/ParametersHandler/tests/config.ini that its YarpImplementation is filled from (keys, quoted
 * keys, values, parenthesised lists, `[GROUP]` sections, `//` and `#` comments).  YARP itself is
 * not a dependency.
 *
 * Differences from the reference a user can notice: vectors are std::vector (the reference's
 * GenericContainer::Vector views with a resize mode are not reproduced; a getParameter into a
 * std::vector always resizes it), and a group is reached only through getGroup / setGroup.
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
    using shared_ptr = std::shared_ptr<IParametersHandler>;
    using weak_ptr = std::weak_ptr<IParametersHandler>;

    virtual bool getParameter(const std::string& name, int& value) const = 0;
    virtual bool getParameter(const std::string& name, double& value) const = 0;
    virtual bool getParameter(const std::string& name, std::string& value) const = 0;
    virtual bool getParameter(const std::string& name, bool& value) const = 0;
    virtual bool getParameter(const std::string& name, std::vector<int>& value) const = 0;
    virtual bool getParameter(const std::string& name, std::vector<double>& value) const = 0;
    virtual bool getParameter(const std::string& name, std::vector<std::string>& value) const = 0;
    virtual bool getParameter(const std::string& name, std::vector<bool>& value) const = 0;

    virtual void setParameter(const std::string& name, const int& value) = 0;
    virtual void setParameter(const std::string& name, const double& value) = 0;
    virtual void setParameter(const std::string& name, const std::string& value) = 0;
    virtual void setParameter(const std::string& name, const char* value) = 0;
    virtual void setParameter(const std::string& name, const bool& value) = 0;
    virtual void setParameter(const std::string& name, const std::vector<int>& value) = 0;
    virtual void setParameter(const std::string& name, const std::vector<double>& value) = 0;
    virtual void setParameter(const std::string& name, const std::vector<std::string>& value) = 0;
    virtual void setParameter(const std::string& name, const std::vector<bool>& value) = 0;

    /** The group `name`; expired if there is none (IParametersHandler.h:203-209). */
    virtual weak_ptr getGroup(const std::string& name) const = 0;
    /** Add or replace a group; false for a null group (IParametersHandler.h:211-219). */
    virtual bool setGroup(const std::string& name, shared_ptr newGroup) = 0;
    virtual std::string toString() const = 0;
    virtual bool isEmpty() const = 0;
    virtual void clear() = 0;
    virtual ~IParametersHandler() = default;
};

/**
 * In-memory handler.  A value is a list of numbers or a list of strings (a scalar is a list of
 * one); booleans are stored as the numbers 0 / 1 and also read from "true" / "false".
 */
class StdImplementation : public IParametersHandler
{
public:
    struct Value
    {
        bool isString = false;
        std::vector<double> numbers;
        std::vector<std::string> strings;
    };

    StdImplementation() = default;

    /** Replace the content with a configuration file in the .ini format above; false (and the
     * handler left empty) if the file cannot be read or does not parse. */
    bool setFromFile(const std::string& path);
    /** The same from the text of such a file. */
    bool setFromString(const std::string& text);

    bool getParameter(const std::string& name, int& value) const override;
    bool getParameter(const std::string& name, double& value) const override;
    bool getParameter(const std::string& name, std::string& value) const override;
    bool getParameter(const std::string& name, bool& value) const override;
    bool getParameter(const std::string& name, std::vector<int>& value) const override;
    bool getParameter(const std::string& name, std::vector<double>& value) const override;
    bool getParameter(const std::string& name, std::vector<std::string>& value) const override;
    bool getParameter(const std::string& name, std::vector<bool>& value) const override;

    void setParameter(const std::string& name, const int& value) override;
    void setParameter(const std::string& name, const double& value) override;
    void setParameter(const std::string& name, const std::string& value) override;
    void setParameter(const std::string& name, const char* value) override;
    void setParameter(const std::string& name, const bool& value) override;
    void setParameter(const std::string& name, const std::vector<int>& value) override;
    void setParameter(const std::string& name, const std::vector<double>& value) override;
    void setParameter(const std::string& name, const std::vector<std::string>& value) override;
    void setParameter(const std::string& name, const std::vector<bool>& value) override;

    weak_ptr getGroup(const std::string& name) const override;
    bool setGroup(const std::string& name, shared_ptr newGroup) override;
    std::string toString() const override;
    bool isEmpty() const override;
    void clear() override;

private:
    const Value* find(const std::string& name) const;
    std::map<std::string, Value> m_values;
    std::map<std::string, shared_ptr> m_groups;
};

} // namespace ParametersHandler
} // namespace BipedalLocomotion

#endif
