// mech_host.cpp -- host mechanism compiler of libbrhip.so (C++17, no GPU code).
//
// Reads the data formats the reference reads and flattens them into the SoA tables of
// br_mech_desc (include/brhip.h), so a Julia (or C) host can drive the engine without Python:
//   * CHEMKIN-II gas mechanisms       <- compile_gaschemistry(mech_file)      src/BatchReactor.jl:251-255
//   * NASA-7 therm.dat, molecular wt   <- IdealGas.create_thermo(gasphase, f)  :265
//   * surface-mechanism XML            <- SurfaceReactions.compile_mech(...)   :283-287
//   * batch.xml                        <- input_data(xmlroot, lib_dir, chem)   :238-306
// The arithmetic of every table entry (unit conversions, atomic-weight sums) is the one of the
// Python host compiler batchreactor.jl_amd/mechanism.py, operation for operation, so both give
// bit-identical tables (tests/test_host.py compares them).
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/brhip.h"

extern "C" void br_set_last_error(const char* msg);   // brhip.hip

namespace {

constexpr double R_GAS = 8.31446261815324;   // RxnHelperUtils.R (src/BatchReactor.jl:338)
constexpr double CAL = 4.184;

// Atomic weights [g/mol]; H/C/O/N fitted to the reference golden (mechanism.py ATOMIC_WEIGHTS)
const std::vector<std::pair<std::string, double>>& atomic_weights() {
    static const std::vector<std::pair<std::string, double>> aw = {
        {"H", 1.0078}, {"C", 12.0107}, {"O", 15.99977}, {"N", 14.00643}, {"AR", 39.948}, {"HE", 4.002602},
        {"NE", 20.1797}, {"S", 32.065}, {"CL", 35.453}, {"F", 18.9984}, {"E", 5.48579909e-4}};
    return aw;
}

struct MechError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// ---- string helpers (Python str semantics where the parser relies on them) -----------------
bool is_ws(unsigned char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\v' || c == '\f'; }
std::string strip(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && is_ws((unsigned char)s[a])) ++a;
    while (b > a && is_ws((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}
std::string upper(std::string s) {
    for (auto& c : s) c = (char)std::toupper((unsigned char)c);
    return s;
}
std::string lower(std::string s) {
    for (auto& c : s) c = (char)std::tolower((unsigned char)c);
    return s;
}
std::vector<std::string> split_ws(const std::string& s) {   // str.split()
    std::vector<std::string> out;
    size_t i = 0;
    while (i < s.size()) {
        while (i < s.size() && is_ws((unsigned char)s[i])) ++i;
        size_t j = i;
        while (j < s.size() && !is_ws((unsigned char)s[j])) ++j;
        if (j > i) out.push_back(s.substr(i, j - i));
        i = j;
    }
    return out;
}
std::vector<std::string> split(const std::string& s, const std::string& sep) {   // str.split(sep)
    std::vector<std::string> out;
    size_t i = 0;
    for (;;) {
        const size_t j = s.find(sep, i);
        if (j == std::string::npos) { out.push_back(s.substr(i)); return out; }
        out.push_back(s.substr(i, j - i));
        i = j + sep.size();
    }
}
std::string substr_py(const std::string& s, size_t a, size_t b) {   // s[a:b] with Python clipping
    if (a >= s.size()) return "";
    return s.substr(a, std::min(b, s.size()) - a);
}
bool starts_with(const std::string& s, const std::string& p) { return s.compare(0, p.size(), p) == 0; }
double to_double(const std::string& s0) {   // float(s): strips whitespace, whole string must parse
    const std::string s = strip(s0);
    if (s.empty()) throw MechError("empty number");
    char* end = nullptr;
    const double v = std::strtod(s.c_str(), &end);
    if (end != s.c_str() + s.size()) throw MechError("bad number '" + s + "'");
    return v;
}
double fortran_double(const std::string& s0) {   // mechanism.py _f: Fortran D exponents, blank = 0
    std::string s = strip(s0);
    for (auto& c : s) {
        if (c == 'D') c = 'E';
        else if (c == 'd') c = 'e';
    }
    return s.empty() ? 0.0 : to_double(s);
}
// leading decimal integer prefix: ("2", "H2O") for "2H2O"; ("", s) when there is none
std::pair<std::string, std::string> int_prefix(const std::string& s) {
    size_t i = 0;
    while (i < s.size() && std::isdigit((unsigned char)s[i])) ++i;
    return {s.substr(0, i), s.substr(i)};
}
std::vector<std::string> read_lines(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw MechError("cannot open " + path);
    std::vector<std::string> lines;
    std::string l;
    while (std::getline(f, l)) lines.push_back(l);   // '\n' removed; '\r' handled by the callers
    return lines;
}

// ---- NASA-7 therm.dat (fixed columns, CHEMKIN-II format) --------------------------------------
struct SpeciesThermo {
    std::vector<std::pair<std::string, int>> elements;   // in line order (molwt sums in this order)
    double tmid = 1000.0;
    double hi[7] = {}, lo[7] = {};
    double molwt() const {
        double w = 0.0;
        for (const auto& ec : elements) {
            double a = -1.0;
            for (const auto& p : atomic_weights()) if (p.first == ec.first) a = p.second;
            if (a < 0) throw MechError("unknown element " + ec.first);
            w += (double)ec.second * a;
        }
        return w * 1e-3;
    }
};
std::map<std::string, SpeciesThermo> read_therm(const std::string& path) {
    std::vector<std::string> lines = read_lines(path);
    for (auto& l : lines) while (!l.empty() && (l.back() == '\r' || l.back() == '\n')) l.pop_back();
    std::map<std::string, SpeciesThermo> out;
    size_t i = 0;
    while (i + 3 < lines.size()) {
        const std::string& l1 = lines[i];
        if (l1.size() >= 80 && l1[79] == '1' && !starts_with(l1, "!")) {
            const std::string &l2 = lines[i + 1], &l3 = lines[i + 2], &l4 = lines[i + 3];
            const auto nm = split_ws(substr_py(l1, 0, 18));
            if (nm.empty()) throw MechError("therm.dat: species line without a name");
            SpeciesThermo t;
            for (int k = 0; k < 4; ++k) {
                const std::string sym = upper(strip(substr_py(l1, 24 + 5 * k, 26 + 5 * k)));
                const std::string cnt = strip(substr_py(l1, 26 + 5 * k, 29 + 5 * k));
                if (!sym.empty() && sym != "0" && !cnt.empty() && to_double(cnt) != 0.0) {
                    const int c = (int)to_double(cnt);
                    bool found = false;
                    for (auto& e : t.elements) if (e.first == sym) { e.second += c; found = true; }
                    if (!found) t.elements.push_back({sym, c});
                }
            }
            const double tm = fortran_double(substr_py(l1, 65, 73));
            t.tmid = tm != 0.0 ? tm : 1000.0;
            double c[14];
            for (int k = 0; k < 5; ++k) c[k] = fortran_double(substr_py(l2, 15 * k, 15 * k + 15));
            for (int k = 0; k < 5; ++k) c[5 + k] = fortran_double(substr_py(l3, 15 * k, 15 * k + 15));
            for (int k = 0; k < 4; ++k) c[10 + k] = fortran_double(substr_py(l4, 15 * k, 15 * k + 15));
            for (int k = 0; k < 7; ++k) { t.hi[k] = c[k]; t.lo[k] = c[7 + k]; }
            out[upper(nm[0])] = t;
            i += 4;
            continue;
        }
        ++i;
    }
    return out;
}

// ---- CHEMKIN-II gas mechanism ------------------------------------------------------------------
struct GasReaction {
    std::string equation;
    std::vector<std::string> reactants, products;   // expanded species names
    bool reversible = true;
    int third_body = 0;                              // 0 none, 1 +M, 2 (+M) falloff
    double A = 0, beta = 0, EoR = 0;
    bool has_low = false;
    double low[3] = {0, 0, 0};
    std::vector<double> troe;
    std::vector<std::pair<std::string, double>> eff;   // insertion order
};

std::vector<std::string> gas_side(const std::string& text, const std::vector<std::string>& species, bool& has_m) {
    std::vector<std::string> out;
    has_m = false;
    for (const std::string& term0 : split(text, "+")) {
        const std::string term = strip(term0);
        if (term.empty()) continue;
        auto pr = int_prefix(term);
        const int coef = pr.first.empty() ? 1 : std::atoi(pr.first.c_str());
        const std::string name = pr.first.empty() ? term : pr.second;
        if (name == "M") { has_m = true; continue; }
        bool known = false;
        for (const auto& s : species) known |= (s == name);
        if (!known) throw MechError("unknown species '" + name + "'");
        for (int c = 0; c < coef; ++c) out.push_back(name);
    }
    return out;
}

void read_chemkin(const std::string& path, std::vector<std::string>& species, std::vector<GasReaction>& rxns) {
    static const std::vector<std::pair<std::string, double>> eunits = {
        {"CAL/MOLE", CAL / R_GAS}, {"KCAL/MOLE", 1000.0 * CAL / R_GAS}, {"JOULES/MOLE", 1.0 / R_GAS},
        {"KJOULES/MOLE", 1000.0 / R_GAS}, {"KELVINS", 1.0}};
    char section = 0;
    double efac = CAL / R_GAS;
    for (const std::string& raw : read_lines(path)) {
        std::string line = upper(strip(split(raw, "!")[0]));
        if (line.empty()) continue;
        const std::string word = split_ws(line)[0];
        if (starts_with(word, "ELEM")) { section = 'E'; continue; }
        if (starts_with(word, "SPEC")) {
            section = 'S';
            line = strip(line.substr(word.size()));
            if (line.empty()) continue;
        } else if (starts_with(word, "THERMO")) {
            section = 'T';
            continue;
        } else if (starts_with(word, "REAC")) {
            section = 'R';
            const auto toks = split_ws(line);
            for (const auto& u : eunits)
                for (const auto& t : toks) if (t == u.first) efac = u.second;
            continue;
        }
        if (word == "END") { section = 0; continue; }
        if (section == 'S') {
            for (const std::string& tok : split_ws(line)) {
                if (tok == "END") { section = 0; break; }
                bool have = false;
                for (const auto& s : species) have |= (s == tok);
                if (!have) species.push_back(tok);
            }
        } else if (section == 'R') {
            if (line.find('=') != std::string::npos) {
                const auto toks = split_ws(line);
                if (toks.size() < 4) throw MechError("reaction line '" + line + "'");
                const double A = to_double(toks[toks.size() - 3]), b = to_double(toks[toks.size() - 2]),
                             E = to_double(toks[toks.size() - 1]);
                std::string eq;
                for (size_t k = 0; k + 3 < toks.size(); ++k) eq += toks[k];
                const bool falloff = eq.find("(+M)") != std::string::npos;
                std::string eq2;
                for (const std::string& piece : split(eq, "(+M)")) eq2 += piece;
                std::vector<std::string> sides;
                bool rev = true;
                if (eq2.find("<=>") != std::string::npos) sides = split(eq2, "<=>");
                else if (eq2.find("=>") != std::string::npos) { sides = split(eq2, "=>"); rev = false; }
                else sides = split(eq2, "=");
                if (sides.size() != 2) throw MechError("reaction '" + eq + "'");
                GasReaction r;
                bool m1 = false, m2 = false;
                r.equation = eq;
                r.reactants = gas_side(sides[0], species, m1);
                r.products = gas_side(sides[1], species, m2);
                r.reversible = rev;
                r.third_body = falloff ? 2 : ((m1 || m2) ? 1 : 0);
                const int order = (int)r.reactants.size() + (r.third_body == 1 ? 1 : 0);
                r.A = A * std::pow(1e-6, (double)(order - 1));
                r.beta = b;
                r.EoR = E * efac;
                rxns.push_back(std::move(r));
            } else {
                if (rxns.empty()) continue;
                GasReaction& r = rxns.back();
                if (starts_with(line, "DUP")) continue;
                std::vector<std::string> parts;
                for (const auto& p : split(line, "/")) parts.push_back(strip(p));
                size_t i = 0;
                while (i + 1 < parts.size()) {
                    const std::string &key = parts[i], &val = parts[i + 1];
                    if (key.empty()) { ++i; continue; }
                    if (key == "LOW") {
                        const auto v = split_ws(val);
                        if (v.size() != 3) throw MechError("LOW needs 3 values");
                        r.has_low = true;
                        r.low[0] = to_double(v[0]) * std::pow(1e-6, (double)r.reactants.size());
                        r.low[1] = to_double(v[1]);
                        r.low[2] = to_double(v[2]) * efac;
                    } else if (key == "TROE") {
                        r.troe.clear();
                        for (const auto& t : split_ws(val)) r.troe.push_back(to_double(t));
                    } else if (key == "REV" || key == "SRI" || key == "PLOG" || key == "FORD" || key == "RORD" ||
                               key == "HIGH") {
                        throw MechError("unsupported auxiliary keyword " + key);
                    } else {
                        bool sp = false;
                        for (const auto& s : species) sp |= (s == key);
                        if (sp) {
                            const double e = to_double(val);
                            bool found = false;
                            for (auto& kv : r.eff) if (kv.first == key) { kv.second = e; found = true; }
                            if (!found) r.eff.push_back({key, e});
                        }
                    }
                    i += 2;
                }
            }
        }
    }
}

// ---- minimal XML reader (elements, attributes, text; comments, prolog and DOCTYPE skipped) --------
struct XNode {
    std::string tag;
    std::vector<std::pair<std::string, std::string>> attr;
    std::string text;   // character data before the first child (ElementTree .text)
    bool has_text = false;
    std::vector<std::unique_ptr<XNode>> kids;
    const XNode* find(const std::string& t) const {
        for (const auto& k : kids) if (k->tag == t) return k.get();
        return nullptr;
    }
    std::vector<const XNode*> findall(const std::string& t) const {
        std::vector<const XNode*> v;
        for (const auto& k : kids) if (k->tag == t) v.push_back(k.get());
        return v;
    }
    const std::string* get(const std::string& a) const {
        for (const auto& kv : attr) if (kv.first == a) return &kv.second;
        return nullptr;
    }
    // ElementTree findtext: None (nullptr) if no such child, "" if it has no text
    bool findtext(const std::string& t, std::string& out) const {
        const XNode* k = find(t);
        if (!k) return false;
        out = k->text;
        return true;
    }
};
std::string xml_unescape(const std::string& s) {
    std::string o;
    for (size_t i = 0; i < s.size(); ++i) {
        if (s[i] != '&') { o += s[i]; continue; }
        const size_t j = s.find(';', i);
        if (j == std::string::npos) throw MechError("xml: bad entity");
        const std::string e = s.substr(i + 1, j - i - 1);
        if (e == "amp") o += '&';
        else if (e == "lt") o += '<';
        else if (e == "gt") o += '>';
        else if (e == "quot") o += '"';
        else if (e == "apos") o += '\'';
        else if (!e.empty() && e[0] == '#') {
            const long c = (e.size() > 1 && (e[1] == 'x' || e[1] == 'X')) ? std::strtol(e.c_str() + 2, nullptr, 16)
                                                                          : std::strtol(e.c_str() + 1, nullptr, 10);
            if (c < 0 || c > 255) throw MechError("xml: character reference outside Latin-1");
            o += (char)c;
        } else throw MechError("xml: unknown entity &" + e + ";");
        i = j;
    }
    return o;
}
std::unique_ptr<XNode> parse_xml(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw MechError("cannot open " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string s = ss.str();
    size_t i = 0;
    std::unique_ptr<XNode> root;
    std::vector<XNode*> stack;
    auto add_text = [&](const std::string& t) {
        if (stack.empty()) return;
        XNode* top = stack.back();
        if (top->kids.empty()) { top->text += xml_unescape(t); top->has_text = true; }   // (tails are not kept)
    };
    while (i < s.size()) {
        if (s[i] != '<') {
            const size_t j = s.find('<', i);
            add_text(s.substr(i, (j == std::string::npos ? s.size() : j) - i));
            i = j == std::string::npos ? s.size() : j;
            continue;
        }
        if (s.compare(i, 4, "<!--") == 0) {
            const size_t j = s.find("-->", i + 4);
            if (j == std::string::npos) throw MechError("xml: unterminated comment");
            i = j + 3;
            continue;
        }
        if (s.compare(i, 2, "<?") == 0) {
            const size_t j = s.find("?>", i + 2);
            if (j == std::string::npos) throw MechError("xml: unterminated prolog");
            i = j + 2;
            continue;
        }
        if (s.compare(i, 9, "<![CDATA[") == 0) {
            const size_t j = s.find("]]>", i + 9);
            if (j == std::string::npos) throw MechError("xml: unterminated CDATA");
            if (!stack.empty() && stack.back()->kids.empty()) stack.back()->text += s.substr(i + 9, j - i - 9);
            i = j + 3;
            continue;
        }
        if (s.compare(i, 2, "<!") == 0) {   // DOCTYPE
            const size_t j = s.find('>', i + 2);
            if (j == std::string::npos) throw MechError("xml: unterminated declaration");
            i = j + 1;
            continue;
        }
        const size_t j = s.find('>', i + 1);
        if (j == std::string::npos) throw MechError("xml: unterminated tag");
        std::string body = s.substr(i + 1, j - i - 1);
        i = j + 1;
        if (!body.empty() && body[0] == '/') {   // end tag
            if (stack.empty() || stack.back()->tag != strip(body.substr(1))) throw MechError("xml: mismatched end tag");
            stack.pop_back();
            continue;
        }
        bool selfclose = false;
        if (!body.empty() && body.back() == '/') { selfclose = true; body.pop_back(); }
        auto node = std::make_unique<XNode>();
        size_t k = 0;
        while (k < body.size() && !is_ws((unsigned char)body[k])) ++k;
        node->tag = body.substr(0, k);
        while (k < body.size()) {   // attributes: name = "value" | 'value'
            while (k < body.size() && is_ws((unsigned char)body[k])) ++k;
            if (k >= body.size()) break;
            const size_t a0 = k;
            while (k < body.size() && body[k] != '=' && !is_ws((unsigned char)body[k])) ++k;
            const std::string an = body.substr(a0, k - a0);
            while (k < body.size() && is_ws((unsigned char)body[k])) ++k;
            if (k >= body.size() || body[k] != '=') throw MechError("xml: attribute without value");
            ++k;
            while (k < body.size() && is_ws((unsigned char)body[k])) ++k;
            if (k >= body.size() || (body[k] != '"' && body[k] != '\'')) throw MechError("xml: unquoted attribute");
            const char q = body[k++];
            const size_t v0 = k;
            while (k < body.size() && body[k] != q) ++k;
            if (k >= body.size()) throw MechError("xml: unterminated attribute");
            node->attr.push_back({an, xml_unescape(body.substr(v0, k - v0))});
            ++k;
        }
        XNode* raw = node.get();
        if (stack.empty()) {
            if (root) throw MechError("xml: more than one root element");
            root = std::move(node);
        } else {
            stack.back()->kids.push_back(std::move(node));
        }
        if (!selfclose) stack.push_back(raw);
    }
    if (!root || !stack.empty()) throw MechError("xml: incomplete document " + path);
    return root;
}

// "k1=v1, k2=v2" -> [(K1, v1), ...] (mechanism.py _kv_list: keys upper-cased, later keys win)
std::vector<std::pair<std::string, double>> kv_list(const std::string& text) {
    std::vector<std::pair<std::string, double>> out;
    for (const std::string& item : split(text, ",")) {
        const size_t e = item.find('=');
        if (e == std::string::npos) continue;
        const std::string k = upper(strip(item.substr(0, e)));
        const double v = to_double(item.substr(e + 1));
        bool found = false;
        for (auto& kv : out) if (kv.first == k) { kv.second = v; found = true; }
        if (!found) out.push_back({k, v});
    }
    return out;
}

// ---- surface-mechanism XML ---------------------------------------------------------------------
struct SurfReaction {
    std::vector<std::string> reactants, products;
    bool stick = false;
    double A = 0, beta = 0, Ea = 0;
    std::vector<std::pair<std::string, double>> coverage;   // insertion order
    int rid = -1;
};
struct SurfMech {
    std::vector<std::string> species;
    std::vector<double> sigma, theta0;
    double density = 0.0;
    std::vector<SurfReaction> rxns;
};
SurfMech read_surface_xml(const std::string& path, const std::vector<std::string>& gas_species) {
    auto root = parse_xml(path);
    const std::string* u = root->get("unit");
    const std::string unit = lower((u && !u->empty()) ? *u : std::string("kJ/mol"));
    const double efac = unit == "kj/mol" ? 1000.0 : unit == "j/mol" ? 1.0 : unit == "kcal/mol" ? 4184.0
                        : unit == "cal/mol" ? CAL : 1000.0;
    SurfMech sm;
    std::string sp;
    if (!root->findtext("species", sp)) throw MechError("surface mechanism without <species>");
    for (const auto& t : split_ws(sp)) sm.species.push_back(upper(t));
    const size_t ns = sm.species.size();
    sm.sigma.assign(ns, 1.0);
    sm.theta0.assign(ns, 0.0);
    auto sidx = [&](const std::string& k) -> int {
        for (size_t i = 0; i < ns; ++i) if (sm.species[i] == k) return (int)i;
        return -1;
    };
    if (const XNode* site = root->find("site")) {
        std::string t;
        if (site->findtext("coordination", t) && !t.empty())
            for (const auto& kv : kv_list(t)) if (sidx(kv.first) >= 0) sm.sigma[sidx(kv.first)] = kv.second;
        if (!site->findtext("density", t)) throw MechError("<site> without <density>");
        sm.density = to_double(t);
        if (site->findtext("initial", t) && !t.empty())
            for (const auto& kv : kv_list(t)) if (sidx(kv.first) >= 0) sm.theta0[sidx(kv.first)] = kv.second;
    }
    std::vector<std::string> known = sm.species;
    for (const auto& g : gas_species) known.push_back(upper(g));
    auto side = [&](const std::string& text) {
        std::vector<std::string> out;
        for (const std::string& t0 : split(text, "+")) {
            const std::string t = upper(strip(t0));
            if (t.empty()) continue;
            auto pr = int_prefix(t);
            const int c = pr.first.empty() ? 1 : std::atoi(pr.first.c_str());
            const std::string nm = pr.first.empty() ? t : strip(pr.second);
            bool ok = false;
            for (const auto& k : known) ok |= (k == nm);
            if (!ok) throw MechError("unknown surface-reaction species '" + nm + "'");
            for (int k = 0; k < c; ++k) out.push_back(nm);
        }
        return out;
    };
    for (const char* kind : {"stick", "arrhenius"}) {
        const XNode* blk = root->find(kind);
        if (!blk) continue;
        for (const XNode* rx : blk->findall("rxn")) {
            const auto eqp = split(rx->text, "@");
            if (eqp.size() != 2) throw MechError("surface reaction '" + rx->text + "'");
            const auto lr = split(eqp[0], "=>");
            if (lr.size() != 2) throw MechError("surface reaction '" + eqp[0] + "'");
            SurfReaction r;
            r.reactants = side(lr[0]);
            r.products = side(lr[1]);
            std::vector<double> vals;
            for (const auto& v : split_ws(eqp[1])) vals.push_back(to_double(v));
            if (std::strcmp(kind, "stick") == 0) {
                if (vals.empty()) throw MechError("sticking reaction without s0");
                r.stick = true;
                r.A = vals[0];
            } else {
                if (vals.size() < 3) throw MechError("Arrhenius reaction needs A, beta, Ea");
                int ms = 0;
                for (const auto& s : r.reactants) ms += sidx(s) >= 0 ? 1 : 0;
                const int mg = (int)r.reactants.size() - ms;
                r.A = vals[0] * std::pow(1e-4, (double)(ms - 1)) * std::pow(1e-6, (double)mg);
                r.beta = vals[1];
                r.Ea = vals[2] * efac;
            }
            const std::string* id = rx->get("id");
            r.rid = id ? std::atoi(id->c_str()) : -1;
            sm.rxns.push_back(std::move(r));
        }
    }
    for (const XNode* cov : root->findall("coverage")) {
        const std::string* ids = cov->get("id");
        if (!ids) throw MechError("<coverage> without id");
        for (const auto& kv : kv_list(cov->text)) {
            for (const auto& idt : split_ws(*ids)) {
                const int rid = std::atoi(idt.c_str());
                SurfReaction* tgt = nullptr;
                for (auto& r : sm.rxns) if (r.rid == rid) tgt = &r;   // last reaction with that id
                if (!tgt) throw MechError("<coverage> names unknown reaction id " + idt);
                bool found = false;
                for (auto& c : tgt->coverage) if (c.first == kv.first) { c.second = kv.second * efac; found = true; }
                if (!found) tgt->coverage.push_back({kv.first, kv.second * efac});
            }
        }
    }
    return sm;
}

}  // namespace

// ---- compiled host mechanism: owns the br_mech_desc arrays -------------------------------------
struct br_host_mech {
    int ng = 0, ns = 0, nrg = 0, nrs = 0, conv = BR_CONV_REFERENCE;
    double p_std = 1e5, site_density = 0.0;
    std::vector<std::string> names;   // gas then surface
    std::vector<double> molwt, nasa, sigma, theta0;
    std::vector<int> g_nf, g_nr, g_f, g_r, g_rev, g_tb, g_troe_n;
    std::vector<double> g_arr, g_low, g_troe, g_eff;
    std::vector<int> s_nf, s_np, s_f, s_p, s_stick, s_ncov, s_cov_sp;
    std::vector<double> s_arr, s_cov_eps;
};

namespace {
template <class T>
const T* ptr_or_null(const std::vector<T>& v) { return v.empty() ? nullptr : v.data(); }

br_host_mech* compile_host(const char* gas_mech, const char* therm, const char* surf_mech, const char* gasphase,
                           int conv) {
    auto h = std::make_unique<br_host_mech>();
    h->conv = conv;
    const auto thermo = read_therm(therm);
    std::vector<std::string> species;
    std::vector<GasReaction> rxns;
    if (gas_mech && *gas_mech) {
        read_chemkin(gas_mech, species, rxns);
    } else {
        if (!gasphase) throw MechError("no gas mechanism and no gas-phase species list");
        for (const auto& g : split_ws(gasphase)) species.push_back(upper(g));
    }
    for (auto& s : species) s = upper(s);
    const int ng = (int)species.size();
    if (ng == 0) throw MechError("no gas species");
    h->ng = ng;
    h->names = species;
    for (const auto& s : species) {
        auto it = thermo.find(s);
        if (it == thermo.end()) throw MechError("species not in therm.dat: " + s);
        h->molwt.push_back(it->second.molwt());
        h->nasa.push_back(it->second.tmid);
        for (int k = 0; k < 7; ++k) h->nasa.push_back(it->second.hi[k]);
        for (int k = 0; k < 7; ++k) h->nasa.push_back(it->second.lo[k]);
    }
    auto gi = [&](const std::string& s) {
        for (int k = 0; k < ng; ++k) if (species[k] == s) return k;
        throw MechError("species " + s);
    };
    // gas reactions
    const int nrg = (int)rxns.size();
    h->nrg = nrg;
    h->g_nf.assign(nrg, 0); h->g_nr.assign(nrg, 0);
    h->g_f.assign(4 * (size_t)nrg, -1); h->g_r.assign(4 * (size_t)nrg, -1);
    h->g_rev.assign(nrg, 0); h->g_tb.assign(nrg, 0); h->g_troe_n.assign(nrg, 0);
    h->g_arr.assign(3 * (size_t)nrg, 0.0); h->g_low.assign(3 * (size_t)nrg, 0.0); h->g_troe.assign(4 * (size_t)nrg, 0.0);
    h->g_eff.assign((size_t)nrg * ng, 1.0);
    for (int i = 0; i < nrg; ++i) {
        const GasReaction& r = rxns[i];
        if (r.reactants.size() > 4 || r.products.size() > 4)
            throw MechError("reaction " + r.equation + ": more than 4 entries per side");
        h->g_nf[i] = (int)r.reactants.size();
        h->g_nr[i] = (int)r.products.size();
        for (size_t e = 0; e < r.reactants.size(); ++e) h->g_f[4 * i + e] = gi(r.reactants[e]);
        for (size_t e = 0; e < r.products.size(); ++e) h->g_r[4 * i + e] = gi(r.products[e]);
        h->g_rev[i] = r.reversible ? 1 : 0;
        h->g_tb[i] = r.third_body;
        h->g_arr[3 * i] = r.A; h->g_arr[3 * i + 1] = r.beta; h->g_arr[3 * i + 2] = r.EoR;
        if (r.has_low) for (int c = 0; c < 3; ++c) h->g_low[3 * i + c] = r.low[c];
        if (!r.troe.empty()) {
            if (r.troe.size() > 4) throw MechError("TROE with more than 4 parameters");
            h->g_troe_n[i] = (int)r.troe.size();
            for (size_t c = 0; c < r.troe.size(); ++c) h->g_troe[4 * i + c] = r.troe[c];
        }
        for (const auto& kv : r.eff) h->g_eff[(size_t)i * ng + gi(kv.first)] = kv.second;
        if (r.third_body == 2 && !r.has_low) throw MechError("falloff reaction " + r.equation + " without LOW");
    }
    // surface reactions
    if (surf_mech && *surf_mech) {
        SurfMech sm = read_surface_xml(surf_mech, species);
        h->ns = (int)sm.species.size();
        h->site_density = sm.density;
        h->sigma = sm.sigma;
        h->theta0 = sm.theta0;
        for (const auto& s : sm.species) h->names.push_back(s);
        auto ci = [&](const std::string& s) {
            for (size_t k = 0; k < h->names.size(); ++k) if (h->names[k] == s) return (int)k;
            throw MechError("species " + s);
        };
        const int nrs = (int)sm.rxns.size();
        h->nrs = nrs;
        h->s_nf.assign(nrs, 0); h->s_np.assign(nrs, 0);
        h->s_f.assign(6 * (size_t)nrs, -1); h->s_p.assign(6 * (size_t)nrs, -1);
        h->s_stick.assign(nrs, 0); h->s_arr.assign(3 * (size_t)nrs, 0.0);
        h->s_ncov.assign(nrs, 0); h->s_cov_sp.assign(4 * (size_t)nrs, 0); h->s_cov_eps.assign(4 * (size_t)nrs, 0.0);
        for (int i = 0; i < nrs; ++i) {
            const SurfReaction& r = sm.rxns[i];
            if (r.reactants.size() > 6 || r.products.size() > 6 || r.coverage.size() > 4)
                throw MechError("surface reaction too large");
            h->s_nf[i] = (int)r.reactants.size();
            h->s_np[i] = (int)r.products.size();
            for (size_t e = 0; e < r.reactants.size(); ++e) h->s_f[6 * i + e] = ci(r.reactants[e]);
            for (size_t e = 0; e < r.products.size(); ++e) h->s_p[6 * i + e] = ci(r.products[e]);
            h->s_stick[i] = r.stick ? 1 : 0;
            h->s_arr[3 * i] = r.A; h->s_arr[3 * i + 1] = r.beta; h->s_arr[3 * i + 2] = r.Ea;
            h->s_ncov[i] = (int)r.coverage.size();
            for (size_t j = 0; j < r.coverage.size(); ++j) {
                h->s_cov_sp[4 * i + j] = ci(r.coverage[j].first);
                h->s_cov_eps[4 * i + j] = r.coverage[j].second;
            }
        }
    }
    return h.release();
}

int fail_msg(int code, const std::string& m) {
    br_set_last_error(m.c_str());
    return code;
}

void copy_str(char* dst, size_t cap, const std::string& s) {
    if (!dst || cap == 0) return;
    const size_t k = std::min(cap - 1, s.size());
    std::memcpy(dst, s.data(), k);
    dst[k] = 0;
}
// a name from batch.xml into a fixed field: an error instead of a silent truncation (a truncated
// species name would match nothing and drop its composition entry; a truncated path opens another
// file)
void copy_field(char* dst, size_t cap, const std::string& s, const char* what) {
    if (s.size() >= cap) throw MechError(std::string(what) + " too long (" + std::to_string(s.size()) + " characters, at most " +
                                         std::to_string(cap - 1) + ")");
    copy_str(dst, cap, s);
}

}  // namespace

extern "C" {

int br_mech_parse(const char* gas_mech_path, const char* therm_path, const char* surf_mech_path,
                  const char* gasphase, int conv, br_host_mech** out) {
    if (!out || !therm_path) return fail_msg(BR_ERR_INPUT, "br_mech_parse: null argument");
    *out = nullptr;
    try {
        *out = compile_host(gas_mech_path, therm_path, surf_mech_path, gasphase, conv);
    } catch (const std::exception& e) {
        return fail_msg(BR_ERR_INPUT, std::string("br_mech_parse: ") + e.what());
    }
    return 0;
}

int br_host_mech_free(br_host_mech* h) {
    delete h;
    return 0;
}

int br_host_mech_desc(const br_host_mech* h, br_mech_desc* d) {
    if (!h || !d) return fail_msg(BR_ERR_INPUT, "br_host_mech_desc: null argument");
    std::memset(d, 0, sizeof(*d));
    d->ng = h->ng; d->ns = h->ns; d->nrg = h->nrg; d->nrs = h->nrs;
    d->conv = h->conv;
    d->p_std = h->p_std;
    d->molwt = ptr_or_null(h->molwt); d->nasa = ptr_or_null(h->nasa);
    d->g_nf = ptr_or_null(h->g_nf); d->g_nr = ptr_or_null(h->g_nr); d->g_f = ptr_or_null(h->g_f);
    d->g_r = ptr_or_null(h->g_r); d->g_rev = ptr_or_null(h->g_rev); d->g_tb = ptr_or_null(h->g_tb);
    d->g_arr = ptr_or_null(h->g_arr); d->g_low = ptr_or_null(h->g_low); d->g_troe_n = ptr_or_null(h->g_troe_n);
    d->g_troe = ptr_or_null(h->g_troe); d->g_eff = ptr_or_null(h->g_eff);
    d->site_density = h->site_density;
    d->sigma = ptr_or_null(h->sigma);
    d->s_nf = ptr_or_null(h->s_nf); d->s_np = ptr_or_null(h->s_np); d->s_f = ptr_or_null(h->s_f);
    d->s_p = ptr_or_null(h->s_p); d->s_stick = ptr_or_null(h->s_stick); d->s_arr = ptr_or_null(h->s_arr);
    d->s_ncov = ptr_or_null(h->s_ncov); d->s_cov_sp = ptr_or_null(h->s_cov_sp); d->s_cov_eps = ptr_or_null(h->s_cov_eps);
    return 0;
}

int br_host_mech_sizes(const br_host_mech* h, int* ng, int* ns, int* nrg, int* nrs) {
    if (!h) return fail_msg(BR_ERR_INPUT, "br_host_mech_sizes: null handle");
    if (ng) *ng = h->ng;
    if (ns) *ns = h->ns;
    if (nrg) *nrg = h->nrg;
    if (nrs) *nrs = h->nrs;
    return 0;
}

int br_host_mech_species(const br_host_mech* h, int i, char* buf, size_t n) {
    if (!h || i < 0 || i >= (int)h->names.size()) return fail_msg(BR_ERR_INPUT, "br_host_mech_species: bad index");
    copy_str(buf, n, h->names[i]);
    return 0;
}

int br_host_mech_theta0(const br_host_mech* h, double* theta0) {
    if (!h || (!theta0 && h->ns)) return fail_msg(BR_ERR_INPUT, "br_host_mech_theta0: null argument");
    for (int i = 0; i < h->ns; ++i) theta0[i] = h->theta0[i];
    return 0;
}

int br_mech_compile(const char* gas_mech_path, const char* therm_path, const char* surf_mech_path,
                    const char* gasphase, int conv, int device, br_mech** out) {
    br_host_mech* h = nullptr;
    int rc = br_mech_parse(gas_mech_path, therm_path, surf_mech_path, gasphase, conv, &h);
    if (rc) return rc;
    br_mech_desc d;
    br_host_mech_desc(h, &d);
    rc = br_mech_create(&d, device, out);
    br_host_mech_free(h);
    return rc;
}

int br_read_batch_xml(const char* path, br_batch_input* b) {
    if (!path || !b) return fail_msg(BR_ERR_INPUT, "br_read_batch_xml: null argument");
    std::memset(b, 0, sizeof(*b));
    b->Asv = 1.0;   // a missing <Asv> acts as Asv = 1 (RxnHelperUtils.get_value_from_xml)
    try {
        auto root = parse_xml(path);
        std::string t;
        if (root->findtext("gas_mech", t) && !t.empty()) copy_field(b->gas_mech, sizeof(b->gas_mech), strip(t), "<gas_mech>");
        if (root->findtext("surface_mech", t) && !t.empty()) copy_field(b->surface_mech, sizeof(b->surface_mech), strip(t), "<surface_mech>");
        if (root->findtext("gasphase", t) && !t.empty()) {
            std::string g;
            for (const auto& s : split_ws(t)) g += (g.empty() ? "" : " ") + s;
            copy_field(b->gasphase, sizeof(b->gasphase), g, "<gasphase>");
        }
        struct { const char* tag; double* v; int* has; } num[] = {
            {"T", &b->T, &b->has_T}, {"p", &b->p, &b->has_p}, {"Asv", &b->Asv, &b->has_Asv}, {"time", &b->time, &b->has_time}};
        for (auto& e : num)
            if (root->findtext(e.tag, t)) { *e.v = to_double(t); *e.has = 1; }
        const char* ctag = nullptr;
        if (root->findtext("molefractions", t) && !t.empty()) { ctag = "molefractions"; b->comp_is_mass = 0; }
        else if (root->findtext("massfractions", t) && !t.empty()) { ctag = "massfractions"; b->comp_is_mass = 1; }
        if (ctag) {
            const auto kv = kv_list(t);
            if (kv.size() > BR_BATCH_MAXCOMP) throw MechError("too many composition entries");
            b->ncomp = (int)kv.size();
            for (size_t i = 0; i < kv.size(); ++i) {
                copy_field(b->comp_names[i], sizeof(b->comp_names[i]), kv[i].first, "composition species name");
                b->comp_values[i] = kv[i].second;
            }
        }
        if (!b->has_T || !b->has_p || !b->has_time || !ctag) throw MechError("batch.xml needs <T>, <p>, <time> and a composition");
    } catch (const std::exception& e) {
        return fail_msg(BR_ERR_INPUT, std::string("br_read_batch_xml: ") + e.what());
    }
    return 0;
}

}  // extern "C"
