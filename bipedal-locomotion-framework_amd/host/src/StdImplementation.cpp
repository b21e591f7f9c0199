/**
 * @file StdImplementation.cpp
 * In-memory IParametersHandler (src/ParametersHandler/include/BipedalLocomotion/
 * ParametersHandler/IParametersHandler.h:26-249) and a reader for the configuration-file format
 * the reference's YarpImplementation is filled from (src/ParametersHandler/tests/config.ini):
 *   key value                 a number or a word
 *   "quoted key" (1, 2, 3)    a parenthesised list, commas or blanks between the elements
 *   key "a string" "another"  several values: a list
 *   [GROUP]                   the keys below, up to the next [..], form the group GROUP
 *   // comment, # comment     to the end of the line (outside quotes)
 * An element that parses completely as a number (and is not quoted) is a number, anything else a
 * string; a list with a string element is a list of strings.
 */
#include <BipedalLocomotion/ParametersHandler/IParametersHandler.h>

#include <cmath>
#include <cstdlib>
#include <fstream>
#include <iostream>
#include <sstream>

namespace BipedalLocomotion
{
namespace ParametersHandler
{
namespace
{

struct Token
{
    std::string text;
    bool quoted = false;
};

// Splits one line (comments already removed) into tokens; a parenthesised list becomes the tokens
// between "(" and ")".  Returns false on an unterminated quote or parenthesis.
bool tokenize(const std::string& line, std::vector<Token>& out, std::vector<std::vector<Token>>& lists,
              std::vector<int>& listAt)
{
    size_t i = 0;
    int depth = 0;
    std::vector<Token> cur;
    while (i < line.size())
    {
        const char c = line[i];
        if (c == ' ' || c == '\t' || c == '\r' || (c == ',' && depth > 0))
        {
            ++i;
            continue;
        }
        if (c == '(')
        {
            if (depth > 0) return false;   // nested lists are not used by the DCM path
            depth = 1;
            cur.clear();
            ++i;
            continue;
        }
        if (c == ')')
        {
            if (depth == 0) return false;
            depth = 0;
            listAt.push_back(static_cast<int>(out.size()));
            out.push_back(Token{"", false});
            lists.push_back(cur);
            ++i;
            continue;
        }
        Token t;
        if (c == '"')
        {
            const size_t e = line.find('"', i + 1);
            if (e == std::string::npos) return false;
            t.text = line.substr(i + 1, e - i - 1);
            t.quoted = true;
            i = e + 1;
        } else
        {
            size_t e = i;
            while (e < line.size() && line[e] != ' ' && line[e] != '\t' && line[e] != '\r'
                   && line[e] != ',' && line[e] != '(' && line[e] != ')')
                ++e;
            t.text = line.substr(i, e - i);
            i = e;
        }
        (depth > 0 ? cur : out).push_back(t);
    }
    return depth == 0;
}

bool asNumber(const Token& t, double& v)
{
    if (t.quoted || t.text.empty()) return false;
    char* end = nullptr;
    v = std::strtod(t.text.c_str(), &end);
    return end && *end == '\0';
}

StdImplementation::Value makeValue(const std::vector<Token>& elems)
{
    StdImplementation::Value v;
    std::vector<double> nums;
    bool allNum = true;
    for (const auto& e : elems)
    {
        double d;
        if (asNumber(e, d)) nums.push_back(d);
        else allNum = false;
    }
    if (allNum)
    {
        v.numbers = nums;
    } else
    {
        v.isString = true;
        for (const auto& e : elems) v.strings.push_back(e.text);
    }
    return v;
}

std::string stripComment(const std::string& line)
{
    bool inQuote = false;
    for (size_t i = 0; i < line.size(); ++i)
    {
        if (line[i] == '"') inQuote = !inQuote;
        if (inQuote) continue;
        if (line[i] == '#') return line.substr(0, i);
        if (line[i] == '/' && i + 1 < line.size() && line[i + 1] == '/') return line.substr(0, i);
    }
    return line;
}

bool toBool(const StdImplementation::Value& v, size_t i, bool& b)
{
    if (v.isString)
    {
        if (v.strings[i] == "true") b = true;
        else if (v.strings[i] == "false") b = false;
        else return false;
        return true;
    }
    if (v.numbers[i] != 0.0 && v.numbers[i] != 1.0) return false;
    b = v.numbers[i] == 1.0;
    return true;
}

} // namespace

bool StdImplementation::setFromFile(const std::string& path)
{
    std::ifstream in(path);
    if (!in)
    {
        std::cerr << "[StdImplementation::setFromFile] Unable to open " << path << "." << std::endl;
        clear();
        return false;
    }
    std::stringstream ss;
    ss << in.rdbuf();
    return setFromString(ss.str());
}

bool StdImplementation::setFromString(const std::string& text)
{
    clear();
    std::istringstream in(text);
    std::string raw;
    StdImplementation* target = this;
    int lineNo = 0;
    while (std::getline(in, raw))
    {
        ++lineNo;
        std::string line = stripComment(raw);
        const size_t a = line.find_first_not_of(" \t\r");
        if (a == std::string::npos) continue;
        line = line.substr(a);
        if (line[0] == '[')
        {
            const size_t e = line.find(']');
            if (e == std::string::npos)
            {
                std::cerr << "[StdImplementation::setFromString] Line " << lineNo
                          << ": unterminated group name." << std::endl;
                clear();
                return false;
            }
            auto group = std::make_shared<StdImplementation>();
            m_groups[line.substr(1, e - 1)] = group;
            target = group.get();
            continue;
        }
        std::vector<Token> toks;
        std::vector<std::vector<Token>> lists;
        std::vector<int> listAt;
        if (!tokenize(line, toks, lists, listAt) || toks.empty()
            || (!listAt.empty() && listAt.front() == 0))
        {
            std::cerr << "[StdImplementation::setFromString] Line " << lineNo
                      << ": unable to parse." << std::endl;
            clear();
            return false;
        }
        const std::string key = toks[0].text;
        std::vector<Token> elems;
        if (listAt.size() == 1 && toks.size() == 2 && listAt[0] == 1)
        {
            elems = lists[0];                                   // key (a, b, c)
        } else if (listAt.empty())
        {
            elems.assign(toks.begin() + 1, toks.end());         // key v  or  key v1 v2 ...
        } else
        {
            std::cerr << "[StdImplementation::setFromString] Line " << lineNo
                      << ": a list must be the only value." << std::endl;
            clear();
            return false;
        }
        target->m_values[key] = makeValue(elems);
    }
    return true;
}

const StdImplementation::Value* StdImplementation::find(const std::string& name) const
{
    auto it = m_values.find(name);
    return it == m_values.end() ? nullptr : &it->second;
}

bool StdImplementation::getParameter(const std::string& name, double& value) const
{
    const Value* v = find(name);
    if (!v || v->isString || v->numbers.size() != 1) return false;
    value = v->numbers[0];
    return true;
}

bool StdImplementation::getParameter(const std::string& name, int& value) const
{
    double d;
    if (!getParameter(name, d) || d != std::floor(d)) return false;
    value = static_cast<int>(d);
    return true;
}

bool StdImplementation::getParameter(const std::string& name, std::string& value) const
{
    const Value* v = find(name);
    if (!v || !v->isString || v->strings.size() != 1) return false;
    value = v->strings[0];
    return true;
}

bool StdImplementation::getParameter(const std::string& name, bool& value) const
{
    const Value* v = find(name);
    if (!v || (v->isString ? v->strings.size() : v->numbers.size()) != 1) return false;
    return toBool(*v, 0, value);
}

bool StdImplementation::getParameter(const std::string& name, std::vector<double>& value) const
{
    const Value* v = find(name);
    if (!v || v->isString) return false;
    value = v->numbers;
    return true;
}

bool StdImplementation::getParameter(const std::string& name, std::vector<int>& value) const
{
    const Value* v = find(name);
    if (!v || v->isString) return false;
    std::vector<int> out;
    for (double d : v->numbers)
    {
        if (d != std::floor(d)) return false;
        out.push_back(static_cast<int>(d));
    }
    value = out;
    return true;
}

bool StdImplementation::getParameter(const std::string& name, std::vector<std::string>& value) const
{
    const Value* v = find(name);
    if (!v || !v->isString) return false;
    value = v->strings;
    return true;
}

bool StdImplementation::getParameter(const std::string& name, std::vector<bool>& value) const
{
    const Value* v = find(name);
    if (!v) return false;
    const size_t n = v->isString ? v->strings.size() : v->numbers.size();
    std::vector<bool> out(n);
    for (size_t i = 0; i < n; ++i)
    {
        bool b;
        if (!toBool(*v, i, b)) return false;
        out[i] = b;
    }
    value = out;
    return true;
}

void StdImplementation::setParameter(const std::string& name, const int& value)
{
    setParameter(name, static_cast<double>(value));
}

void StdImplementation::setParameter(const std::string& name, const double& value)
{
    Value v;
    v.numbers = {value};
    m_values[name] = v;
}

void StdImplementation::setParameter(const std::string& name, const std::string& value)
{
    Value v;
    v.isString = true;
    v.strings = {value};
    m_values[name] = v;
}

void StdImplementation::setParameter(const std::string& name, const char* value)
{
    setParameter(name, std::string(value));
}

void StdImplementation::setParameter(const std::string& name, const bool& value)
{
    setParameter(name, value ? 1.0 : 0.0);
}

void StdImplementation::setParameter(const std::string& name, const std::vector<int>& value)
{
    Value v;
    for (int i : value) v.numbers.push_back(static_cast<double>(i));
    m_values[name] = v;
}

void StdImplementation::setParameter(const std::string& name, const std::vector<double>& value)
{
    Value v;
    v.numbers = value;
    m_values[name] = v;
}

void StdImplementation::setParameter(const std::string& name, const std::vector<std::string>& value)
{
    Value v;
    v.isString = true;
    v.strings = value;
    m_values[name] = v;
}

void StdImplementation::setParameter(const std::string& name, const std::vector<bool>& value)
{
    Value v;
    for (bool b : value) v.numbers.push_back(b ? 1.0 : 0.0);
    m_values[name] = v;
}

IParametersHandler::weak_ptr StdImplementation::getGroup(const std::string& name) const
{
    auto it = m_groups.find(name);
    return it == m_groups.end() ? weak_ptr() : weak_ptr(it->second);
}

bool StdImplementation::setGroup(const std::string& name, shared_ptr newGroup)
{
    if (!newGroup) return false;
    m_groups[name] = newGroup;
    return true;
}

std::string StdImplementation::toString() const
{
    std::ostringstream o;
    o.precision(17);
    auto quote = [](const std::string& s) {
        return s.find_first_of(" \t,()") == std::string::npos ? s : "\"" + s + "\"";
    };
    for (const auto& [k, v] : m_values)
    {
        o << quote(k) << " ";
        const size_t n = v.isString ? v.strings.size() : v.numbers.size();
        if (n != 1) o << "(";
        for (size_t i = 0; i < n; ++i)
        {
            if (i) o << ", ";
            if (v.isString) o << "\"" << v.strings[i] << "\"";
            else o << v.numbers[i];
        }
        if (n != 1) o << ")";
        o << "\n";
    }
    for (const auto& [k, g] : m_groups) o << "[" << k << "]\n" << g->toString();
    return o.str();
}

bool StdImplementation::isEmpty() const
{
    return m_values.empty() && m_groups.empty();
}

void StdImplementation::clear()
{
    m_values.clear();
    m_groups.clear();
}

} // namespace ParametersHandler
} // namespace BipedalLocomotion
