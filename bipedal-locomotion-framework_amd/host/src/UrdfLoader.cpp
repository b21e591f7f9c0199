/**
 * @file UrdfLoader.cpp
 * blf::loadUrdf (host/include/blf/urdf.h): the C++ adapter's path from a robot description to a
 * blf::RobotModel, the rules of blf/urdf.py (tests/test_urdf.py pins both against each other,
 * tests/test_host_cpp.py::test_cpp_urdf_loader_matches_python).  Host bookkeeping only: the model
 * goes to the device through FloatingBaseDynamicalSystem::setRobotModel.
 */
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>

#include <blf/urdf.h>

namespace
{

// ---- a small XML reader: elements and attributes, everything else skipped ---------------------
struct XmlNode
{
    std::string tag;
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<std::unique_ptr<XmlNode>> kids;

    const std::string* attr(const std::string& name) const
    {
        for (const auto& a : attrs)
            if (a.first == name) return &a.second;
        return nullptr;
    }
    const XmlNode* child(const std::string& name) const
    {
        for (const auto& k : kids)
            if (k->tag == name) return k.get();
        return nullptr;
    }
};

class XmlReader
{
    const std::string& s;
    std::size_t i{0};

    bool fail(const std::string& what)
    {
        if (error.empty()) error = what + " (at byte " + std::to_string(i) + ")";
        return false;
    }
    bool starts(const char* p) const { return s.compare(i, std::char_traits<char>::length(p), p) == 0; }
    void skipSpace()
    {
        while (i < s.size() && std::isspace(static_cast<unsigned char>(s[i]))) ++i;
    }
    bool skipPast(const char* end)
    {
        const std::size_t e = s.find(end, i);
        if (e == std::string::npos) return fail(std::string("unterminated markup, expected ") + end);
        i = e + std::char_traits<char>::length(end);
        return true;
    }
    // comments, processing instructions, CDATA, DOCTYPE (with an internal subset)
    bool skipMisc(bool& skipped)
    {
        skipped = true;
        if (starts("<!--")) return skipPast("-->");
        if (starts("<?")) return skipPast("?>");
        if (starts("<![CDATA[")) return skipPast("]]>");
        if (starts("<!DOCTYPE"))
        {
            int depth = 0;
            for (; i < s.size(); ++i)
            {
                if (s[i] == '[') ++depth;
                else if (s[i] == ']') --depth;
                else if (s[i] == '>' && depth <= 0) { ++i; return true; }
            }
            return fail("unterminated DOCTYPE");
        }
        skipped = false;
        return true;
    }
    static bool nameChar(char c)
    {
        return !std::isspace(static_cast<unsigned char>(c)) && c != '/' && c != '>' && c != '='
               && c != '<' && c != '"' && c != '\'';
    }
    bool readName(std::string& out)
    {
        const std::size_t b = i;
        while (i < s.size() && nameChar(s[i])) ++i;
        if (i == b) return fail("expected a name");
        out.assign(s, b, i - b);
        return true;
    }
    bool decode(const std::string& raw, std::string& out)
    {
        out.clear();
        for (std::size_t k = 0; k < raw.size(); ++k)
        {
            if (raw[k] != '&') { out += raw[k]; continue; }
            const std::size_t e = raw.find(';', k);
            if (e == std::string::npos) return fail("unterminated entity");
            const std::string ent = raw.substr(k + 1, e - k - 1);
            if (ent == "lt") out += '<';
            else if (ent == "gt") out += '>';
            else if (ent == "amp") out += '&';
            else if (ent == "quot") out += '"';
            else if (ent == "apos") out += '\'';
            else if (ent.size() > 1 && ent[0] == '#')
            {
                const long v = ent[1] == 'x' ? std::strtol(ent.c_str() + 2, nullptr, 16)
                                             : std::strtol(ent.c_str() + 1, nullptr, 10);
                if (v <= 0 || v > 127) return fail("character reference outside ASCII");
                out += static_cast<char>(v);
            } else
                return fail("unknown entity &" + ent + ";");
            k = e;
        }
        return true;
    }
    bool element(XmlNode& n, int depth)
    {
        if (depth > 256) return fail("elements nested too deeply");
        if (i >= s.size() || s[i] != '<') return fail("expected an element");
        ++i;
        if (!readName(n.tag)) return false;
        for (;;)
        {
            skipSpace();
            if (i >= s.size()) return fail("unterminated start tag <" + n.tag);
            if (starts("/>")) { i += 2; return true; }
            if (s[i] == '>') { ++i; break; }
            std::string name, raw, value;
            if (!readName(name)) return false;
            skipSpace();
            if (i >= s.size() || s[i] != '=') return fail("expected '=' after attribute " + name);
            ++i;
            skipSpace();
            if (i >= s.size() || (s[i] != '"' && s[i] != '\'')) return fail("unquoted attribute " + name);
            const char q = s[i++];
            const std::size_t e = s.find(q, i);
            if (e == std::string::npos) return fail("unterminated attribute " + name);
            raw.assign(s, i, e - i);
            i = e + 1;
            if (!decode(raw, value)) return false;
            if (n.attr(name)) return fail("attribute " + name + " given twice");
            n.attrs.emplace_back(name, value);
        }
        for (;;)   // content
        {
            const std::size_t lt = s.find('<', i);
            if (lt == std::string::npos) return fail("unterminated element <" + n.tag + ">");
            i = lt;
            bool skipped = false;
            if (!skipMisc(skipped)) return false;
            if (skipped) continue;
            if (starts("</"))
            {
                i += 2;
                std::string name;
                if (!readName(name)) return false;
                skipSpace();
                if (name != n.tag || i >= s.size() || s[i] != '>')
                    return fail("mismatched end tag </" + name + "> for <" + n.tag + ">");
                ++i;
                return true;
            }
            n.kids.push_back(std::make_unique<XmlNode>());
            if (!element(*n.kids.back(), depth + 1)) return false;
        }
    }

public:
    std::string error;
    explicit XmlReader(const std::string& text) : s(text) {}
    bool document(XmlNode& root)
    {
        for (;;)
        {
            skipSpace();
            bool skipped = false;
            if (!skipMisc(skipped)) return false;
            if (!skipped) break;
        }
        if (!element(root, 0)) return false;
        for (;;)
        {
            skipSpace();
            if (i >= s.size()) return true;
            bool skipped = false;
            if (!skipMisc(skipped)) return false;
            if (!skipped) return fail("content after the root element");
        }
    }
};

// ---- URDF -> model ------------------------------------------------------------------------------
struct UrdfError
{
    std::string what;
};

void rpyMatrix(const double rpy[3], double R[9])   // Rz(y) Ry(p) Rx(r)
{
    const double cr = std::cos(rpy[0]), sr = std::sin(rpy[0]);
    const double cp = std::cos(rpy[1]), sp = std::sin(rpy[1]);
    const double cy = std::cos(rpy[2]), sy = std::sin(rpy[2]);
    const double Rx[9] = {1, 0, 0, 0, cr, -sr, 0, sr, cr};
    const double Ry[9] = {cp, 0, sp, 0, 1, 0, -sp, 0, cp};
    const double Rz[9] = {cy, -sy, 0, sy, cy, 0, 0, 0, 1};
    double T[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            T[3 * r + c] = Rz[3 * r] * Ry[c] + Rz[3 * r + 1] * Ry[3 + c] + Rz[3 * r + 2] * Ry[6 + c];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            R[3 * r + c] = T[3 * r] * Rx[c] + T[3 * r + 1] * Rx[3 + c] + T[3 * r + 2] * Rx[6 + c];
}

double number(const std::string& text, const std::string& what)
{
    const char* b = text.c_str();
    char* e = nullptr;
    const double v = std::strtod(b, &e);
    while (e && *e && std::isspace(static_cast<unsigned char>(*e))) ++e;
    if (e == b || (e && *e)) throw UrdfError{what + "=\"" + text + "\" is not a number"};
    return v;
}

void vec3(const XmlNode* el, const char* attr, const double dflt[3], double out[3])
{
    for (int a = 0; a < 3; ++a) out[a] = dflt[a];
    const std::string* v = el ? el->attr(attr) : nullptr;
    if (!v) return;
    std::istringstream in(*v);
    std::string tok;
    int k = 0;
    while (in >> tok)
    {
        if (k == 3) throw UrdfError{std::string(attr) + "=\"" + *v + "\" is not three numbers"};
        out[k++] = number(tok, attr);
    }
    if (k != 3) throw UrdfError{std::string(attr) + "=\"" + *v + "\" is not three numbers"};
}

void inertial(const XmlNode& link, double& mass, double com[3], double I[9])
{
    static const double zero[3] = {0, 0, 0};
    mass = 0.0;
    for (int a = 0; a < 3; ++a) com[a] = 0.0;
    for (int a = 0; a < 9; ++a) I[a] = 0.0;
    const XmlNode* ine = link.child("inertial");
    if (!ine) return;
    const XmlNode* org = ine->child("origin");
    double rpy[3], R[9], Ii[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    vec3(org, "xyz", zero, com);
    vec3(org, "rpy", zero, rpy);
    rpyMatrix(rpy, R);
    if (const XmlNode* m = ine->child("mass"))
        if (const std::string* v = m->attr("value")) mass = number(*v, "mass value");
    if (const XmlNode* in = ine->child("inertia"))
    {
        auto g = [&](const char* k) { const std::string* v = in->attr(k); return v ? number(*v, k) : 0.0; };
        const double xx = g("ixx"), xy = g("ixy"), xz = g("ixz"), yy = g("iyy"), yz = g("iyz"), zz = g("izz");
        const double J[9] = {xx, xy, xz, xy, yy, yz, xz, yz, zz};
        for (int a = 0; a < 9; ++a) Ii[a] = J[a];
    }
    const std::string* name = link.attr("name");
    if (mass < 0.0) throw UrdfError{"link " + (name ? *name : std::string("?")) + " has a negative mass"};
    double T[9];   // R I R^T
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            T[3 * r + c] = R[3 * r] * Ii[c] + R[3 * r + 1] * Ii[3 + c] + R[3 * r + 2] * Ii[6 + c];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            I[3 * r + c] = T[3 * r] * R[3 * c] + T[3 * r + 1] * R[3 * c + 1] + T[3 * r + 2] * R[3 * c + 2];
}

const std::string& requireAttr(const XmlNode* el, const char* name, const std::string& where)
{
    const std::string* v = el ? el->attr(name) : nullptr;
    if (!v) throw UrdfError{where + " has no " + name};
    return *v;
}

// blf/urdf.py reorder_joints: the joints in the order perm (perm[k] = the joint placed at k).
blf::RobotModel reorder(const blf::RobotModel& m, const std::vector<int>& perm,
                        std::vector<std::string>& names)
{
    const int n = m.ndof;
    std::vector<int32_t> newLink(n + 1, 0);
    for (int k = 0; k < n; ++k) newLink[perm[k] + 1] = k + 1;
    blf::RobotModel out = m;
    std::vector<std::string> late, nn(n);
    for (int k = 0; k < n; ++k)
    {
        const int o = perm[k];
        out.parent[k] = newLink[m.parent[o]];
        if (out.parent[k] > k) late.push_back(names[o]);
        for (int a = 0; a < 3; ++a) out.jointOrigin[3 * k + a] = m.jointOrigin[3 * o + a];
        for (int a = 0; a < 9; ++a) out.jointRotation[9 * k + a] = m.jointRotation[9 * o + a];
        for (int a = 0; a < 3; ++a) out.jointAxis[3 * k + a] = m.jointAxis[3 * o + a];
        if (!m.jointType.empty()) out.jointType[k] = m.jointType[o];
        out.linkMass[k + 1] = m.linkMass[o + 1];
        for (int a = 0; a < 3; ++a) out.linkCom[3 * (k + 1) + a] = m.linkCom[3 * (o + 1) + a];
        for (int a = 0; a < 9; ++a) out.linkInertia[9 * (k + 1) + a] = m.linkInertia[9 * (o + 1) + a];
        nn[k] = names[o];
    }
    if (!late.empty())
    {
        std::string list;
        for (const auto& l : late) list += (list.empty() ? "" : ", ") + l;
        throw UrdfError{"considered joints list " + list + " before their parent joints; list every "
                        "joint after its parent's (the kernels need parent[j] <= j)"};
    }
    for (auto& l : out.frameLink) l = newLink[l];
    names = nn;
    return out;
}

blf::RobotModel build(const XmlNode& robot, const blf::UrdfOptions& opt, std::vector<std::string>& dofNames)
{
    static const double zero[3] = {0, 0, 0}, xaxis[3] = {1, 0, 0};
    if (robot.tag != "robot") throw UrdfError{"the document's root element is not <robot>"};
    std::map<std::string, const XmlNode*> links;
    std::vector<std::string> linkOrder;
    for (const auto& k : robot.kids)
        if (k->tag == "link")
        {
            const std::string& name = requireAttr(k.get(), "name", "a <link>");
            if (links.count(name)) throw UrdfError{"link " + name + " is defined twice"};
            links[name] = k.get();
            linkOrder.push_back(name);
        }
    std::map<std::string, std::vector<const XmlNode*>> kids;
    std::map<std::string, const XmlNode*> parentJoint;
    for (const auto& k : robot.kids)
        if (k->tag == "joint")
        {
            const std::string& jn = requireAttr(k.get(), "name", "a <joint>");
            const std::string& pl = requireAttr(k->child("parent"), "link", "joint " + jn + "'s <parent>");
            const std::string& cl = requireAttr(k->child("child"), "link", "joint " + jn + "'s <child>");
            if (!links.count(pl) || !links.count(cl))
                throw UrdfError{"joint " + jn + " connects an undefined link"};
            if (parentJoint.count(cl)) throw UrdfError{"link " + cl + " is the child of two joints (not a tree)"};
            parentJoint[cl] = k.get();
            kids[pl].push_back(k.get());
        }
    std::string base = opt.base;
    if (base.empty())
    {
        std::vector<std::string> roots;
        for (const auto& l : linkOrder)
            if (!parentJoint.count(l)) roots.push_back(l);
        if (roots.size() != 1)
            throw UrdfError{"the links form " + std::to_string(roots.size()) + " trees; one expected"};
        base = roots[0];
    } else if (!links.count(base))
        throw UrdfError{"base link " + base + " is not in the model"};
    if (parentJoint.count(base)) throw UrdfError{"a base below the tree's root (re-rooting) is not supported"};

    // joints in depth-first preorder from the base, children in document order
    std::vector<const XmlNode*> order;
    std::map<std::string, int> linkIndex{{base, 0}};
    std::vector<std::string> stack{base};
    while (!stack.empty())
    {
        const std::string lk = stack.back();
        stack.pop_back();
        const auto it = kids.find(lk);
        if (it != kids.end())
            for (auto j = it->second.rbegin(); j != it->second.rend(); ++j)
                stack.push_back(*(*j)->child("child")->attr("link"));
        if (lk != base)
        {
            order.push_back(parentJoint[lk]);
            linkIndex[lk] = static_cast<int>(order.size());
        }
    }
    for (const auto& l : linkOrder)
        if (!linkIndex.count(l)) throw UrdfError{"link " + l + " is not connected to the base"};

    const int n = static_cast<int>(order.size());
    blf::RobotModel m;
    m.ndof = n;
    m.parent.assign(n, 0);
    m.jointOrigin.assign(3 * n, 0.0);
    m.jointRotation.assign(9 * n, 0.0);
    m.jointAxis.assign(3 * n, 0.0);
    m.jointType.assign(n, BLF_JOINT_REVOLUTE);
    m.fixedJoint.assign(n, 0);
    m.linkMass.assign(n + 1, 0.0);
    m.linkCom.assign(3 * (n + 1), 0.0);
    m.linkInertia.assign(9 * (n + 1), 0.0);
    std::vector<std::string> names(n);
    std::vector<std::string> all;
    for (int k = 0; k < n; ++k)
    {
        const XmlNode* j = order[k];
        names[k] = *j->attr("name");
        all.push_back(names[k]);
        const std::string* tp = j->attr("type");
        const std::string typ = tp ? *tp : "";
        const bool fixed = typ == "fixed";
        if (!fixed && typ != "revolute" && typ != "continuous" && typ != "prismatic")
            throw UrdfError{"joint " + names[k] + " of type " + typ + " is not supported (revolute, "
                            "continuous, prismatic, fixed)"};
        m.parent[k] = linkIndex[*j->child("parent")->attr("link")];
        const XmlNode* org = j->child("origin");
        double rpy[3], ax[3];
        vec3(org, "xyz", zero, &m.jointOrigin[3 * k]);
        vec3(org, "rpy", zero, rpy);
        rpyMatrix(rpy, &m.jointRotation[9 * k]);
        vec3(j->child("axis"), "xyz", xaxis, ax);
        const double na = std::sqrt(ax[0] * ax[0] + ax[1] * ax[1] + ax[2] * ax[2]);
        if (!fixed && !(na > 0.0)) throw UrdfError{"joint " + names[k] + " has a zero axis"};
        for (int a = 0; a < 3; ++a) m.jointAxis[3 * k + a] = na > 0.0 ? ax[a] / na : xaxis[a];
        if (typ == "prismatic") m.jointType[k] = BLF_JOINT_PRISMATIC;
        const bool locked = opt.hasConsideredJoints
                            && std::find(opt.consideredJoints.begin(), opt.consideredJoints.end(), names[k])
                                   == opt.consideredJoints.end();
        m.fixedJoint[k] = (fixed || locked) ? 1 : 0;
    }
    if (opt.hasConsideredJoints)
        for (const auto& c : opt.consideredJoints)
            if (std::find(all.begin(), all.end(), c) == all.end())
                throw UrdfError{"considered joint " + c + " is not in the model"};
    for (int l = 0; l <= n; ++l)
    {
        const std::string& ln = l == 0 ? base : *order[l - 1]->child("child")->attr("link");
        inertial(*links[ln], m.linkMass[l], &m.linkCom[3 * l], &m.linkInertia[9 * l]);
    }
    for (const auto& f : opt.frames)
    {
        const auto it = linkIndex.find(f);
        if (it == linkIndex.end()) throw UrdfError{"frame " + f + " is not a link of the model"};
        m.frameLink.push_back(it->second);
        const double pose[12] = {0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1};
        m.framePose.insert(m.framePose.end(), pose, pose + 12);
    }
    // merge the fixed / locked joints (their child links into the parents)
    std::vector<std::string> kept;
    for (int k = 0; k < n; ++k)
        if (!m.fixedJoint[k]) kept.push_back(names[k]);
    blf::RobotModel r = blf::reduceFixedJoints(m);
    r.fixedJoint.clear();
    if (opt.hasConsideredJoints)
    {
        std::vector<int> perm;
        for (std::size_t c = 0; c < opt.consideredJoints.size(); ++c)
        {
            const std::string& name = opt.consideredJoints[c];
            if (std::find(opt.consideredJoints.begin(), opt.consideredJoints.begin() + c, name)
                != opt.consideredJoints.begin() + c)
                continue;   // listed twice: the first place counts
            const auto it = std::find(kept.begin(), kept.end(), name);
            if (it != kept.end()) perm.push_back(static_cast<int>(it - kept.begin()));
        }
        bool identity = perm.size() == kept.size();
        for (std::size_t k = 0; identity && k < perm.size(); ++k) identity = perm[k] == static_cast<int>(k);
        if (!identity) r = reorder(r, perm, kept);
    }
    dofNames = kept;
    return r;
}

} // namespace

bool blf::loadUrdf(const std::string& source, const UrdfOptions& options, RobotModel& model,
                   std::vector<std::string>* jointNames, std::string* error)
{
    std::string text;
    std::size_t b = source.find_first_not_of(" \t\r\n");
    if (b != std::string::npos && source[b] == '<')
        text = source;
    else
    {
        std::ifstream in(source, std::ios::binary);
        if (!in)
        {
            if (error) *error = "loadUrdf: cannot open " + source;
            return false;
        }
        std::ostringstream ss;
        ss << in.rdbuf();
        text = ss.str();
    }
    XmlNode root;
    XmlReader reader(text);
    if (!reader.document(root))
    {
        if (error) *error = "loadUrdf: malformed XML: " + reader.error;
        return false;
    }
    try
    {
        std::vector<std::string> names;
        RobotModel m = build(root, options, names);
        model = std::move(m);
        if (jointNames) *jointNames = std::move(names);
        return true;
    } catch (const UrdfError& e)
    {
        if (error) *error = "loadUrdf: " + e.what;
        return false;
    }
}
