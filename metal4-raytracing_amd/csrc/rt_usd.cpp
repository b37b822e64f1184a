// rt_usd.cpp — USD layer readers (.usda text, .usdc crate, .usdz package); see rt_usd.h.
#include "rt_usd.h"
#include <set>
#include <sys/stat.h>

#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>

namespace rt {
namespace usd {

Stage::Stage() {
    Prim root;
    root.name = "";
    root.path = "/";
    prims.push_back(root);
    by_path["/"] = 0;
}

int Stage::add_prim(int parent, const std::string& name) {
    const std::string& pp = prims[parent].path;
    std::string path = pp == "/" ? "/" + name : pp + "/" + name;
    auto it = by_path.find(path);
    if (it != by_path.end()) return it->second;
    Prim p;
    p.name = name;
    p.path = path;
    p.parent = parent;
    prims.push_back(p);
    const int id = (int)prims.size() - 1;
    prims[parent].children.push_back(id);
    by_path[path] = id;
    return id;
}

int Stage::add_detached(const std::string& path) {
    auto it = by_path.find(path);
    if (it != by_path.end()) return it->second;
    Prim p;
    const size_t k = path.find_last_of('/');
    p.name = k == std::string::npos ? path : path.substr(k + 1);
    p.path = path;
    prims.push_back(p);
    const int id = (int)prims.size() - 1;
    by_path[path] = id;
    return id;
}

// primvar elementSize from a file number (1 when absent, NaN or out of range)
static int element_size(double d) { return d >= 1.0 && d <= 65536.0 ? (int)d : 1; }

std::vector<int> Stage::preorder(int root, bool active_only) const {
    std::vector<int> out, todo{root};
    std::vector<char> seen(prims.size(), 0);
    while (!todo.empty()) {
        const int k = todo.back();
        todo.pop_back();
        if (k < 0 || (size_t)k >= prims.size() || seen[k]) continue;
        seen[k] = 1;
        if (active_only && !prims[k].active) continue;
        out.push_back(k);
        const std::vector<int>& ch = prims[k].children;
        for (size_t i = ch.size(); i-- > 0;) todo.push_back(ch[i]);
    }
    return out;
}

static float half_to_float(uint16_t h) {
    const uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
    uint32_t bits;
    if (e == 0) {
        if (m == 0) {
            bits = s;
        } else {   // subnormal: renormalise
            int k = 0;
            uint32_t mm = m;
            while (!(mm & 0x400u)) { mm <<= 1; ++k; }
            bits = s | ((uint32_t)(127 - 15 - k + 1) << 23) | ((mm & 0x3ffu) << 13);
        }
    } else if (e == 31) {
        bits = s | 0x7f800000u | (m << 13);
    } else {
        bits = s | ((e - 15 + 127) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &bits, 4);
    return f;
}

// ---- .usda ------------------------------------------------------------------------------------
namespace {

struct Tok {
    enum T { kEnd, kPunct, kIdent, kNum, kStr, kAsset, kPath, kErr } t = kEnd;
    std::string s;
    double v = 0.0;
};

class Lexer {
public:
    Lexer(const char* b, size_t n) : p_(b), e_(b + n) {}
    const Tok& peek(size_t k = 0) {
        while (buf_.size() <= k) buf_.push_back(lex());
        return buf_[k];
    }
    Tok next() {
        peek();
        Tok t = std::move(buf_.front());
        buf_.pop_front();
        return t;
    }
    int line() const { return line_; }

private:
    const char* p_;
    const char* e_;
    int line_ = 1;
    std::deque<Tok> buf_;

    static bool ident_start(char c) { return std::isalpha((unsigned char)c) || c == '_'; }
    static bool ident_char(char c) { return std::isalnum((unsigned char)c) || c == '_'; }

    Tok lex() {
        Tok t;
        while (p_ < e_) {
            if (*p_ == '\n') { ++line_; ++p_; }
            else if (std::isspace((unsigned char)*p_)) ++p_;
            else if (*p_ == '#') { while (p_ < e_ && *p_ != '\n') ++p_; }
            else break;
        }
        if (p_ >= e_) return t;
        const char c = *p_;
        if (std::strchr("()[]{}=,:;", c)) {
            t.t = Tok::kPunct;
            t.s = std::string(1, c);
            ++p_;
            return t;
        }
        if (c == '"' || c == '\'') {
            const bool triple = e_ - p_ >= 3 && p_[1] == c && p_[2] == c;
            p_ += triple ? 3 : 1;
            t.t = Tok::kStr;
            while (p_ < e_) {
                if (triple ? (e_ - p_ >= 3 && p_[0] == c && p_[1] == c && p_[2] == c) : *p_ == c) {
                    p_ += triple ? 3 : 1;
                    return t;
                }
                if (*p_ == '\\' && p_ + 1 < e_) {
                    const char x = p_[1];
                    t.s += x == 'n' ? '\n' : x == 't' ? '\t' : x;
                    p_ += 2;
                    continue;
                }
                if (*p_ == '\n') ++line_;
                t.s += *p_++;
            }
            t.t = Tok::kErr;
            return t;
        }
        if (c == '@') {
            const bool triple = e_ - p_ >= 3 && p_[1] == '@' && p_[2] == '@';
            p_ += triple ? 3 : 1;
            t.t = Tok::kAsset;
            while (p_ < e_) {
                if (triple ? (e_ - p_ >= 3 && p_[0] == '@' && p_[1] == '@' && p_[2] == '@') : *p_ == '@') {
                    p_ += triple ? 3 : 1;
                    return t;
                }
                t.s += *p_++;
            }
            t.t = Tok::kErr;
            return t;
        }
        if (c == '<') {
            ++p_;
            t.t = Tok::kPath;
            while (p_ < e_ && *p_ != '>') t.s += *p_++;
            if (p_ >= e_) { t.t = Tok::kErr; return t; }
            ++p_;
            return t;
        }
        const bool sign = (c == '-' || c == '+') && p_ + 1 < e_;
        const char c1 = sign ? p_[1] : c;
        if (std::isdigit((unsigned char)c1) || (c1 == '.' && p_ + (sign ? 2 : 1) < e_ && std::isdigit((unsigned char)p_[sign ? 2 : 1]))) {
            char* end = nullptr;
            t.v = std::strtod(p_, &end);
            if (!end || end == p_) { t.t = Tok::kErr; return t; }
            t.t = Tok::kNum;
            p_ = end;
            return t;
        }
        if (sign && e_ - p_ >= 4 && !std::strncmp(p_ + 1, "inf", 3)) {
            t.t = Tok::kNum;
            t.v = c == '-' ? -INFINITY : INFINITY;
            p_ += 4;
            return t;
        }
        if (ident_start(c)) {
            t.t = Tok::kIdent;
            // names: a:b:c, optionally followed by .timeSamples / .connect (property suffixes)
            while (p_ < e_ && (ident_char(*p_) || ((*p_ == ':' || *p_ == '.') && p_ + 1 < e_ && ident_start(p_[1]))))
                t.s += *p_++;
            return t;
        }
        t.t = Tok::kErr;
        t.s = std::string(1, c);
        return t;
    }
};

class UsdaParser {
public:
    UsdaParser(const char* b, size_t n, Stage& st) : lx_(b, n), st_(st) {}
    bool run(std::string& err) {
        if (lx_.peek().t == Tok::kPunct && lx_.peek().s == "(") {
            if (!layer_meta()) return fail(err);
        }
        while (lx_.peek().t != Tok::kEnd) {
            if (!is_ident({"def", "over", "class"})) { msg_ = "expected a prim"; return fail(err); }
            if (!prim(0)) return fail(err);
        }
        return true;
    }

private:
    Lexer lx_;
    Stage& st_;
    std::string msg_;

    bool fail(std::string& err) {
        err = "usda line " + std::to_string(lx_.line()) + ": " + (msg_.empty() ? "syntax error" : msg_);
        return false;
    }
    bool is_punct(const char* s, size_t k = 0) { const Tok& t = lx_.peek(k); return t.t == Tok::kPunct && t.s == s; }
    bool is_ident(std::initializer_list<const char*> names, size_t k = 0) {
        const Tok& t = lx_.peek(k);
        if (t.t != Tok::kIdent) return false;
        for (const char* n : names)
            if (t.s == n) return true;
        return false;
    }
    bool expect(const char* p) {
        if (!is_punct(p)) { msg_ = std::string("expected '") + p + "'"; return false; }
        lx_.next();
        return true;
    }
    // skips a balanced (...), [...] or {...} group starting at the current token
    bool skip_group() {
        int depth = 0;
        do {
            Tok t = lx_.next();
            if (t.t == Tok::kEnd || t.t == Tok::kErr) { msg_ = "unbalanced group"; return false; }
            if (t.t == Tok::kPunct && (t.s == "(" || t.s == "[" || t.s == "{")) ++depth;
            if (t.t == Tok::kPunct && (t.s == ")" || t.s == "]" || t.s == "}")) --depth;
        } while (depth > 0);
        return true;
    }

    // nesting of values and prims is bounded: hostile input must not exhaust the stack
    static constexpr int kMaxDepth = 64;
    int depth_ = 0;
    struct Nest {
        int& d;
        explicit Nest(int& d_) : d(d_) { ++d; }
        ~Nest() { --d; }
    };

    bool value(Value& v) {
        Nest nest(depth_);
        if (depth_ > kMaxDepth) { msg_ = "values nested too deeply"; return false; }
        const Tok& t = lx_.peek();
        if (t.t == Tok::kPunct && t.s == "[") {
            lx_.next();
            v.array = true;
            bool first = true;
            while (!is_punct("]")) {
                Value el;
                if (!value(el)) return false;
                if (el.kind == Value::kNum) {
                    if (first) v.comps = (int)el.num.size();
                    v.kind = Value::kNum;
                    v.num.insert(v.num.end(), el.num.begin(), el.num.end());
                } else if (el.kind == Value::kStr || el.kind == Value::kPath) {
                    v.kind = el.kind;
                    v.str.insert(v.str.end(), el.str.begin(), el.str.end());
                }
                first = false;
                if (is_punct(",")) lx_.next();
                else if (!is_punct("]")) { msg_ = "expected ',' or ']'"; return false; }
            }
            lx_.next();
            if (v.kind == Value::kNone) v.kind = Value::kNum;   // empty array
            return true;
        }
        if (t.t == Tok::kPunct && t.s == "(") {
            lx_.next();
            while (!is_punct(")")) {
                Value el;
                if (!value(el)) return false;
                if (el.kind == Value::kNum) {
                    v.kind = Value::kNum;
                    v.num.insert(v.num.end(), el.num.begin(), el.num.end());
                } else if (el.kind != Value::kNone) {
                    v.kind = el.kind;
                    v.str.insert(v.str.end(), el.str.begin(), el.str.end());
                }
                if (is_punct(",")) lx_.next();
                else if (!is_punct(")")) { msg_ = "expected ',' or ')'"; return false; }
            }
            lx_.next();
            v.comps = v.kind == Value::kNum ? (int)v.num.size() : 1;
            return true;
        }
        if (t.t == Tok::kPunct && t.s == "{") return skip_group();   // dictionaries
        Tok x = lx_.next();
        switch (x.t) {
        case Tok::kNum: v.kind = Value::kNum; v.num.push_back(x.v); return true;
        case Tok::kStr:
        case Tok::kAsset: v.kind = Value::kStr; v.str.push_back(x.s); return true;
        case Tok::kPath: v.kind = Value::kPath; v.str.push_back(x.s); return true;
        case Tok::kIdent:
            if (x.s == "true" || x.s == "false") { v.kind = Value::kNum; v.num.push_back(x.s == "true" ? 1.0 : 0.0); return true; }
            if (x.s == "None") { v.kind = Value::kNone; return true; }
            if (x.s == "inf" || x.s == "nan") { v.kind = Value::kNum; v.num.push_back(x.s == "inf" ? INFINITY : NAN); return true; }
            v.kind = Value::kStr;
            v.str.push_back(x.s);
            return true;
        default: msg_ = "bad value"; return false;
        }
    }

    // a reference / payload / sublayer list: None, one item or [items]; an item is @asset@, </path>
    // or @asset@</path>, optionally followed by a (layer offset / custom data) group
    bool arc_list(std::vector<Arc>& out) {
        if (is_ident({"None"})) { lx_.next(); return true; }
        const bool list = is_punct("[");
        if (list) lx_.next();
        while (!(list && is_punct("]"))) {
            Arc a;
            if (lx_.peek().t == Tok::kAsset) a.asset = lx_.next().s;
            if (lx_.peek().t == Tok::kPath) a.path = lx_.next().s;
            else if (a.asset.empty()) { msg_ = "expected a reference"; return false; }
            if (is_punct("(") && !skip_group()) return false;
            out.push_back(a);
            if (!list) return true;
            if (is_punct(",")) lx_.next();
            else if (!is_punct("]")) { msg_ = "expected ',' or ']'"; return false; }
        }
        lx_.next();
        return true;
    }
    // variants = { string set = "variant" ... }
    bool variant_selection(int id) {
        if (!expect("{")) return false;
        while (!is_punct("}")) {
            if (is_punct(";")) { lx_.next(); continue; }
            if (lx_.peek().t == Tok::kIdent && lx_.peek(1).t != Tok::kPunct) lx_.next();   // value type
            const Tok set = lx_.next();
            if (set.t != Tok::kIdent && set.t != Tok::kStr) { msg_ = "expected a variant set name"; return false; }
            if (!expect("=")) return false;
            const Tok var = lx_.next();
            if (var.t != Tok::kStr) { msg_ = "expected a variant name"; return false; }
            st_.prims[id].variant_sel[set.s] = var.s;
        }
        lx_.next();
        return true;
    }

    // arcs_for: -2 plain metadata, -1 the layer's (subLayers), >= 0 a prim's (references, payload,
    // variants)
    bool meta_entries(const std::function<void(const std::string&, const Value&)>& on, int arcs_for = -2) {
        if (!expect("(")) return false;
        while (!is_punct(")")) {
            const Tok& t = lx_.peek();
            if (t.t == Tok::kStr) { lx_.next(); continue; }   // doc string
            if (t.t == Tok::kPunct && t.s == ";") { lx_.next(); continue; }
            if (t.t != Tok::kIdent) { msg_ = "bad metadata"; return false; }
            std::string op;
            if (is_ident({"prepend", "append", "add", "delete", "reorder"}) && lx_.peek(1).t == Tok::kIdent) op = lx_.next().s;
            std::string key = lx_.next().s;
            if (lx_.peek().t == Tok::kIdent && !is_punct("=")) key = lx_.next().s;   // typed dictionary entry
            if (!expect("=")) return false;
            if (arcs_for >= -1 && (key == "references" || key == "payload" || key == "subLayers" || key == "inherits" ||
                                   key == "specializes")) {
                std::vector<Arc> arcs;
                if (!arc_list(arcs)) return false;
                if (op == "delete" || op == "reorder") continue;
                if (arcs_for == -1 && key == "subLayers")
                    for (const Arc& a : arcs) st_.sublayers.push_back(a.asset);
                if (arcs_for >= 0 && key == "references") {
                    auto& r = st_.prims[arcs_for].references;
                    r.insert(op == "prepend" ? r.begin() : r.end(), arcs.begin(), arcs.end());
                }
                if (arcs_for >= 0 && key == "payload") {
                    auto& r = st_.prims[arcs_for].payloads;
                    r.insert(op == "prepend" ? r.begin() : r.end(), arcs.begin(), arcs.end());
                }
                continue;   // inherits / specializes: class arcs, not followed
            }
            if (arcs_for >= 0 && key == "variants") {
                if (!variant_selection(arcs_for)) return false;
                continue;
            }
            Value v;
            if (!value(v)) return false;
            on(key, v);
        }
        lx_.next();
        return true;
    }

    bool layer_meta() {
        return meta_entries([this](const std::string& k, const Value& v) {
            if (k == "upAxis" && v.kind == Value::kStr && !v.str.empty()) st_.up_axis = v.str[0];
            if (k == "defaultPrim" && v.kind == Value::kStr && !v.str.empty()) st_.default_prim = v.str[0];
            if ((k == "timeCodesPerSecond" || k == "framesPerSecond") && v.kind == Value::kNum && !v.num.empty()) {
                if (k == "timeCodesPerSecond" || !tcps_set_) st_.time_codes_per_second = v.num[0];
                if (k == "timeCodesPerSecond") tcps_set_ = true;
            }
        }, -1);
    }
    bool tcps_set_ = false;

    bool prim(int parent) {
        Nest nest(depth_);
        if (depth_ > kMaxDepth) { msg_ = "prims nested too deeply"; return false; }
        lx_.next();   // specifier
        std::string type;
        if (lx_.peek().t == Tok::kIdent) type = lx_.next().s;
        if (lx_.peek().t != Tok::kStr) { msg_ = "expected a prim name"; return false; }
        const std::string name = lx_.next().s;
        const int id = st_.add_prim(parent, name);
        if (!type.empty()) st_.prims[id].type = type;
        if (is_punct("(") && !prim_meta(id)) return false;
        return prim_body(id);
    }
    bool prim_meta(int id) {
        return meta_entries([this, id](const std::string& k, const Value& v) {
            Prim& p = st_.prims[id];
            if (k == "apiSchemas")
                for (const auto& s : v.str) p.api_schemas.push_back(s);
            if (k == "active" && v.kind == Value::kNum && !v.num.empty()) p.active = v.num[0] != 0.0;
        }, id);
    }
    // { properties, child prims, variant sets } of prim id (or of a variant body)
    bool prim_body(int id) {
        if (!expect("{")) return false;
        while (!is_punct("}")) {
            if (lx_.peek().t == Tok::kEnd) { msg_ = "unterminated prim"; return false; }
            if (is_ident({"def", "over", "class"})) {
                if (!prim(id)) return false;
            } else if (is_ident({"variantSet"})) {
                // variantSet "set" = { "variant" (metadata) { body } ... }: each body is kept as a
                // detached prim "/Prim{set=variant}"; load_stage applies the selected one
                Nest nest(depth_);
                if (depth_ > kMaxDepth) { msg_ = "prims nested too deeply"; return false; }
                lx_.next();
                const Tok set = lx_.next();
                if (set.t != Tok::kStr) { msg_ = "expected a variant set name"; return false; }
                if (!expect("=") || !expect("{")) return false;
                while (!is_punct("}")) {
                    const Tok var = lx_.next();
                    if (var.t != Tok::kStr) { msg_ = "expected a variant name"; return false; }
                    const int body = st_.add_detached(st_.prims[id].path + "{" + set.s + "=" + var.s + "}");
                    st_.prims[id].variant_bodies[set.s][var.s] = body;
                    if (is_punct("(") && !prim_meta(body)) return false;
                    if (!prim_body(body)) return false;
                }
                lx_.next();
            } else if (is_ident({"reorder"})) {
                lx_.next();
                lx_.next();
                if (!expect("=")) return false;
                Value v;
                if (!value(v)) return false;
            } else if (is_punct(";")) {
                lx_.next();
            } else if (!property(id)) {
                return false;
            }
        }
        lx_.next();
        return true;
    }

    bool property(int id) {
        bool uniform = false;
        while (is_ident({"custom", "uniform", "varying", "config", "prepend", "append", "add", "delete"})) {
            if (lx_.peek().s == "uniform") uniform = true;
            lx_.next();
        }
        if (lx_.peek().t != Tok::kIdent) { msg_ = "expected a property"; return false; }
        if (lx_.peek().s == "rel") {
            lx_.next();
            if (lx_.peek().t != Tok::kIdent) { msg_ = "expected a relationship name"; return false; }
            std::string name = lx_.next().s;
            auto& targets = st_.prims[id].rels[name];
            if (is_punct("=")) {
                lx_.next();
                Value v;
                if (!value(v)) return false;
                if (v.kind == Value::kPath) targets = v.str;
            }
            if (is_punct("(") && !meta_entries([](const std::string&, const Value&) {})) return false;
            return true;
        }
        std::string type = lx_.next().s;
        if (is_punct("[") && is_punct("]", 1)) {
            lx_.next();
            lx_.next();
            type += "[]";
        }
        if (lx_.peek().t != Tok::kIdent) { msg_ = "expected an attribute name"; return false; }
        std::string name = lx_.next().s;
        bool ts = false, conn = false;
        auto strip = [&name](const char* suf) {
            const size_t n = std::strlen(suf);
            if (name.size() > n && name.compare(name.size() - n, n, suf) == 0) { name.resize(name.size() - n); return true; }
            return false;
        };
        if (strip(".timeSamples")) ts = true;
        else if (strip(".connect")) conn = true;
        else strip(".spline");
        Attr& a = st_.prims[id].attrs[name];
        a.type = type;
        a.uniform = a.uniform || uniform;
        if (is_punct("=")) {
            lx_.next();
            if (ts) {
                if (!expect("{")) return false;
                while (!is_punct("}")) {
                    Tok k = lx_.next();
                    if (k.t != Tok::kNum) { msg_ = "expected a time code"; return false; }
                    if (!expect(":")) return false;
                    Value v;
                    if (!value(v)) return false;
                    a.times.push_back(k.v);
                    a.samples.push_back(v);
                    if (is_punct(",")) lx_.next();
                }
                lx_.next();
            } else if (conn) {
                Value v;
                if (!value(v)) return false;
                if (v.kind == Value::kPath) a.connections = v.str;
            } else {
                Value v;
                if (!value(v)) return false;
                if (v.kind != Value::kNone) {
                    a.value = v;
                    a.has_default = true;
                }
            }
        }
        if (is_punct("(")) {
            if (!meta_entries([&a](const std::string& k, const Value& v) {
                    if (k == "interpolation" && v.kind == Value::kStr && !v.str.empty()) a.interpolation = v.str[0];
                    if (k == "elementSize" && v.kind == Value::kNum && !v.num.empty()) a.element_size = element_size(v.num[0]);
                }))
                return false;
        }
        return true;
    }
};

}  // namespace

bool parse_usda(const char* text, size_t n, Stage& st, std::string& err) {
    UsdaParser p(text, n, st);
    return p.run(err);
}

// ---- LZ4 block + TfFastCompression framing ---------------------------------------------------
bool lz4_block_decode(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_n) {
    const uint8_t* ip = src;
    const uint8_t* const iend = src + n;
    size_t op = 0;
    while (ip < iend) {
        const uint8_t token = *ip++;
        size_t lit = token >> 4;
        if (lit == 15) {
            uint8_t b;
            do {
                if (ip >= iend) return false;
                b = *ip++;
                lit += b;
            } while (b == 255);
        }
        if ((size_t)(iend - ip) < lit || cap - op < lit) return false;
        std::memcpy(dst + op, ip, lit);
        ip += lit;
        op += lit;
        if (ip >= iend) break;   // the last sequence holds literals only
        if (iend - ip < 2) return false;
        const size_t off = (size_t)ip[0] | ((size_t)ip[1] << 8);
        ip += 2;
        if (off == 0 || off > op) return false;
        size_t ml = token & 15u;
        if (ml == 15) {
            uint8_t b;
            do {
                if (ip >= iend) return false;
                b = *ip++;
                ml += b;
            } while (b == 255);
        }
        ml += 4;
        if (cap - op < ml) return false;
        for (size_t k = 0; k < ml; ++k, ++op) dst[op] = dst[op - off];   // overlapping copies
    }
    *out_n = op;
    return true;
}

// TfFastCompression::DecompressFromBuffer: first byte = chunk count (0 = one LZ4 block)
static bool fast_decompress(const uint8_t* src, size_t n, uint8_t* dst, size_t cap, size_t* out_n) {
    if (n < 1) return false;
    const int chunks = src[0];
    if (chunks == 0) return lz4_block_decode(src + 1, n - 1, dst, cap, out_n);
    size_t pos = 1, total = 0;
    for (int c = 0; c < chunks; ++c) {
        if (n - pos < 4) return false;
        int32_t sz;
        std::memcpy(&sz, src + pos, 4);
        pos += 4;
        if (sz < 0 || (size_t)sz > n - pos) return false;
        size_t got = 0;
        if (!lz4_block_decode(src + pos, (size_t)sz, dst + total, cap - total, &got)) return false;
        pos += (size_t)sz;
        total += got;
    }
    *out_n = total;
    return true;
}

// ---- .usdz (zip) ------------------------------------------------------------------------------
static uint32_t rd16(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
static uint32_t rd32(const uint8_t* p) { return rd16(p) | (rd16(p + 2) << 16); }

bool read_zip(const uint8_t* data, size_t n, std::vector<PackageFile>& files, std::string& err) {
    if (n < 22) { err = "zip: too short"; return false; }
    size_t eocd = (size_t)-1;
    for (size_t i = n - 22 + 1; i-- > 0 && n - i <= 22 + 65535;)
        if (rd32(data + i) == 0x06054b50u) { eocd = i; break; }
    if (eocd == (size_t)-1) { err = "zip: no end-of-central-directory record"; return false; }
    const uint32_t entries = rd16(data + eocd + 10), cd_off = rd32(data + eocd + 16);
    size_t p = cd_off;
    for (uint32_t e = 0; e < entries; ++e) {
        if (p + 46 > n || rd32(data + p) != 0x02014b50u) { err = "zip: bad central directory"; return false; }
        const uint32_t method = rd16(data + p + 10), csize = rd32(data + p + 20), usize = rd32(data + p + 24);
        const uint32_t nlen = rd16(data + p + 28), elen = rd16(data + p + 30), clen = rd16(data + p + 32);
        const uint32_t lho = rd32(data + p + 42);
        if (p + 46 + nlen > n) { err = "zip: bad entry name"; return false; }
        PackageFile f;
        f.name.assign((const char*)data + p + 46, nlen);
        p += 46 + nlen + elen + clen;
        if (csize == 0xffffffffu || usize == 0xffffffffu || lho == 0xffffffffu) { err = "zip: zip64 entries unsupported"; return false; }
        if (!f.name.empty() && f.name.back() == '/') continue;
        if ((size_t)lho + 30 > n || rd32(data + lho) != 0x04034b50u) { err = "zip: bad local header"; return false; }
        const size_t off = (size_t)lho + 30 + rd16(data + lho + 26) + rd16(data + lho + 28);
        if (off + csize > n) { err = "zip: truncated entry " + f.name; return false; }
        if (method == 0) {
            f.data.assign(data + off, data + off + csize);
        } else if (method == 8) {
            if ((uint64_t)usize > 1032ull * csize + 1024) { err = "zip: implausible size of " + f.name; return false; }
            f.data.resize(usize);
            z_stream zs;
            std::memset(&zs, 0, sizeof zs);
            if (inflateInit2(&zs, -MAX_WBITS) != Z_OK) { err = "zip: inflateInit2"; return false; }
            zs.next_in = const_cast<Bytef*>(data + off);
            zs.avail_in = csize;
            zs.next_out = f.data.data();
            zs.avail_out = usize;
            const int r = inflate(&zs, Z_FINISH);
            inflateEnd(&zs);
            if (r != Z_STREAM_END || zs.total_out != usize) { err = "zip: inflate failed for " + f.name; return false; }
        } else {
            err = "zip: compression method " + std::to_string(method) + " unsupported (" + f.name + ")";
            return false;
        }
        files.push_back(std::move(f));
    }
    return true;
}

// ---- .usdc (crate) ----------------------------------------------------------------------------
namespace {

enum CrateType {
    kBool = 1, kUChar, kInt, kUInt, kInt64, kUInt64, kHalf, kFloat, kDouble, kString, kToken, kAssetPath,
    kMatrix2d, kMatrix3d, kMatrix4d, kQuatd, kQuatf, kQuath, kVec2d, kVec2f, kVec2h, kVec2i, kVec3d, kVec3f,
    kVec3h, kVec3i, kVec4d, kVec4f, kVec4h, kVec4i, kDictionary, kTokenListOp, kStringListOp, kPathListOp,
    kReferenceListOp, kIntListOp, kInt64ListOp, kUIntListOp, kUInt64ListOp, kPathVector, kTokenVector,
    kSpecifier, kPermission, kVariability, kVariantSelectionMap, kTimeSamples, kPayload, kDoubleVector,
    kLayerOffsetVector, kStringVector, kValueBlock, kValue, kUnregisteredValue, kUnregisteredValueListOp,
    kPayloadListOp, kTimeCode
};

struct NumType {
    int comps = 0;   // 0 = not a numeric type
    int bytes = 0;   // per component
    char k = 0;      // b bool, B uchar, i int32, I uint32, l int64, L uint64, h half, f float, d double
    bool matrix = false, quat = false;
};

static NumType num_type(int t) {
    switch (t) {
    case kBool: return {1, 1, 'b'};
    case kUChar: return {1, 1, 'B'};
    case kInt: return {1, 4, 'i'};
    case kUInt: return {1, 4, 'I'};
    case kInt64: return {1, 8, 'l'};
    case kUInt64: return {1, 8, 'L'};
    case kHalf: return {1, 2, 'h'};
    case kFloat: return {1, 4, 'f'};
    case kDouble: case kTimeCode: return {1, 8, 'd'};
    case kMatrix2d: return {4, 8, 'd', true};
    case kMatrix3d: return {9, 8, 'd', true};
    case kMatrix4d: return {16, 8, 'd', true};
    case kQuatd: return {4, 8, 'd', false, true};
    case kQuatf: return {4, 4, 'f', false, true};
    case kQuath: return {4, 2, 'h', false, true};
    case kVec2d: return {2, 8, 'd'};
    case kVec2f: return {2, 4, 'f'};
    case kVec2h: return {2, 2, 'h'};
    case kVec2i: return {2, 4, 'i'};
    case kVec3d: return {3, 8, 'd'};
    case kVec3f: return {3, 4, 'f'};
    case kVec3h: return {3, 2, 'h'};
    case kVec3i: return {3, 4, 'i'};
    case kVec4d: return {4, 8, 'd'};
    case kVec4f: return {4, 4, 'f'};
    case kVec4h: return {4, 2, 'h'};
    case kVec4i: return {4, 4, 'i'};
    default: return {};
    }
}

static double read_num(const uint8_t* p, char k) {
    switch (k) {
    case 'b': case 'B': return (double)p[0];
    case 'i': { int32_t v; std::memcpy(&v, p, 4); return v; }
    case 'I': { uint32_t v; std::memcpy(&v, p, 4); return v; }
    case 'l': { int64_t v; std::memcpy(&v, p, 8); return (double)v; }
    case 'L': { uint64_t v; std::memcpy(&v, p, 8); return (double)v; }
    case 'h': { uint16_t v; std::memcpy(&v, p, 2); return half_to_float(v); }
    case 'f': { float v; std::memcpy(&v, p, 4); return v; }
    default: { double v; std::memcpy(&v, p, 8); return v; }
    }
}

class Crate {
public:
    Crate(const uint8_t* d, size_t n) : d_(d), n_(n) {}

    bool run(Stage& st, std::string& err) {
        if (!bootstrap() || !tokens() || !strings() || !fields() || !fieldsets() || !paths() || !specs() || !build(st)) {
            err = "usdc: " + msg_;
            return false;
        }
        return true;
    }

private:
    const uint8_t* d_;
    size_t n_;
    std::string msg_;
    int ver_[3] = {0, 0, 0};
    struct Section { std::string name; uint64_t start = 0, size = 0; };
    std::vector<Section> sections_;
    std::vector<std::string> tokens_;
    std::vector<uint32_t> strings_;
    std::vector<uint32_t> field_tok_;
    std::vector<uint64_t> field_rep_;
    std::vector<uint32_t> fieldsets_;
    std::vector<std::string> paths_;
    struct Spec { uint32_t path, fset, type; };
    std::vector<Spec> specs_;

    bool fail(const std::string& m) { if (msg_.empty()) msg_ = m; return false; }
    bool has(uint64_t off, uint64_t len) const { return off <= n_ && len <= n_ - off; }
    // `count` elements of `elem` bytes at `off` (overflow-safe: counts come from the file)
    bool has_n(uint64_t off, uint64_t count, uint64_t elem) const {
        return off <= n_ && (elem == 0 || count <= (n_ - off) / elem);
    }
    // a decoded element count a file of this size can carry (compressed integers take at least
    // two bits each before TfFastCompression, whose ratio is below 256:1)
    bool plausible(uint64_t count) const { return count <= (1ull << 28) && count <= 1024 * (uint64_t)n_ + 1024; }
    bool u64(uint64_t off, uint64_t& v) { if (!has(off, 8)) return fail("read past the end"); std::memcpy(&v, d_ + off, 8); return true; }
    bool u32(uint64_t off, uint32_t& v) { if (!has(off, 4)) return fail("read past the end"); std::memcpy(&v, d_ + off, 4); return true; }
    bool at_least(int a, int b, int c) const {
        return ver_[0] != a ? ver_[0] > a : ver_[1] != b ? ver_[1] > b : ver_[2] >= c;
    }
    const Section* section(const char* name) const {
        for (const Section& s : sections_)
            if (s.name == name) return &s;
        return nullptr;
    }

    bool bootstrap() {
        if (n_ < 88 || std::memcmp(d_, "PXR-USDC", 8) != 0) return fail("not a crate file");
        ver_[0] = d_[8]; ver_[1] = d_[9]; ver_[2] = d_[10];
        if (!at_least(0, 4, 0)) return fail("crate version < 0.4.0 unsupported");
        uint64_t toc;
        if (!u64(16, toc)) return false;
        uint64_t count;
        if (!u64(toc, count)) return false;
        if (count > 64) return fail("bad table of contents");
        for (uint64_t i = 0; i < count; ++i) {
            const uint64_t o = toc + 8 + i * 32;
            if (!has(o, 32)) return fail("truncated table of contents");
            Section s;
            s.name.assign((const char*)d_ + o, strnlen((const char*)d_ + o, 16));
            std::memcpy(&s.start, d_ + o + 16, 8);
            std::memcpy(&s.size, d_ + o + 24, 8);
            sections_.push_back(s);
        }
        return true;
    }

    // integer coding (Usd_IntegerCompression): common value, 2-bit codes, deltas
    template <class Int>
    bool decode_ints(const uint8_t* w, size_t wn, size_t count, std::vector<Int>& out) {
        typedef typename std::make_signed<Int>::type SInt;
        const size_t codes = (count * 2 + 7) / 8;
        if (wn < sizeof(SInt) + codes) return fail("integer block too short");
        SInt common;
        std::memcpy(&common, w, sizeof common);
        const uint8_t* cp = w + sizeof(SInt);
        const uint8_t* vp = cp + codes;
        const uint8_t* ve = w + wn;
        out.resize(count);
        SInt prev = 0;
        for (size_t i = 0; i < count; ++i) {
            const int code = (cp[i / 4] >> (2 * (i % 4))) & 3;
            SInt delta = common;
            if (code) {
                const size_t sz = sizeof(SInt) == 4 ? (code == 1 ? 1 : code == 2 ? 2 : 4) : (code == 1 ? 2 : code == 2 ? 4 : 8);
                if ((size_t)(ve - vp) < sz) return fail("integer data too short");
                if (sz == 1) { int8_t v; std::memcpy(&v, vp, 1); delta = v; }
                else if (sz == 2) { int16_t v; std::memcpy(&v, vp, 2); delta = v; }
                else if (sz == 4) { int32_t v; std::memcpy(&v, vp, 4); delta = v; }
                else { int64_t v; std::memcpy(&v, vp, 8); delta = (SInt)v; }
                vp += sz;
            }
            typedef typename std::make_unsigned<Int>::type UInt;
            prev = (SInt)((UInt)prev + (UInt)delta);   // wrapping (uint32 fieldset terminators)
            out[i] = (Int)prev;
        }
        return true;
    }
    // uint64 compressed size, then TfFastCompression of the integer coding; `pos` advances
    template <class Int>
    bool compressed_ints(uint64_t& pos, size_t count, std::vector<Int>& out) {
        uint64_t csize;
        if (!u64(pos, csize)) return false;
        pos += 8;
        if (!has(pos, csize)) return fail("compressed integers past the end");
        if (!plausible(count)) return fail("implausible integer count");
        if (count == 0) { out.clear(); pos += csize; return true; }
        std::vector<uint8_t> w(sizeof(Int) + (count * 2 + 7) / 8 + count * sizeof(Int) + 64);
        size_t got = 0;
        if (!fast_decompress(d_ + pos, (size_t)csize, w.data(), w.size(), &got)) return fail("LZ4 block");
        pos += csize;
        return decode_ints<Int>(w.data(), got, count, out);
    }

    bool tokens() {
        const Section* s = section("TOKENS");
        if (!s) return fail("no TOKENS section");
        uint64_t count, usize, csize;
        if (!u64(s->start, count) || !u64(s->start + 8, usize) || !u64(s->start + 16, csize)) return false;
        if (!has(s->start + 24, csize) || usize > (1ull << 31)) return fail("bad TOKENS section");
        std::vector<uint8_t> buf(usize + 16);
        size_t got = 0;
        if (!fast_decompress(d_ + s->start + 24, csize, buf.data(), buf.size(), &got)) return fail("TOKENS LZ4");
        size_t p = 0;
        for (uint64_t i = 0; i < count; ++i) {
            size_t e = p;
            while (e < got && buf[e]) ++e;
            if (e >= got && i + 1 < count) return fail("TOKENS truncated");
            tokens_.emplace_back((const char*)buf.data() + p, e - p);
            p = e + 1;
        }
        return true;
    }
    bool strings() {
        const Section* s = section("STRINGS");
        if (!s) return fail("no STRINGS section");
        uint64_t count;
        if (!u64(s->start, count)) return false;
        if (!has_n(s->start + 8, count, 4)) return fail("bad STRINGS section");
        strings_.resize(count);
        if (count) std::memcpy(strings_.data(), d_ + s->start + 8, count * 4);
        return true;
    }
    bool fields() {
        const Section* s = section("FIELDS");
        if (!s) return fail("no FIELDS section");
        uint64_t count, pos = s->start + 8;
        if (!u64(s->start, count)) return false;
        if (!compressed_ints<uint32_t>(pos, count, field_tok_)) return false;
        uint64_t rsize;
        if (!u64(pos, rsize)) return false;
        pos += 8;
        if (!has(pos, rsize) || !plausible(count)) return fail("bad FIELDS reps");
        field_rep_.resize(count);
        size_t got = 0;
        if (!fast_decompress(d_ + pos, rsize, (uint8_t*)field_rep_.data(), count * 8, &got) || got != count * 8)
            return fail("FIELDS reps LZ4");
        return true;
    }
    bool fieldsets() {
        const Section* s = section("FIELDSETS");
        if (!s) return fail("no FIELDSETS section");
        uint64_t count, pos = s->start + 8;
        if (!u64(s->start, count)) return false;
        return compressed_ints<uint32_t>(pos, count, fieldsets_);
    }
    bool paths() {
        const Section* s = section("PATHS");
        if (!s) return fail("no PATHS section");
        uint64_t total, count, pos = s->start + 16;
        if (!u64(s->start, total) || !u64(s->start + 8, count)) return false;
        std::vector<uint32_t> idx;
        std::vector<int32_t> elem, jump;
        if (!compressed_ints<uint32_t>(pos, count, idx) || !compressed_ints<int32_t>(pos, count, elem) ||
            !compressed_ints<int32_t>(pos, count, jump))
            return false;
        if (!plausible(total)) return fail("implausible path count");
        paths_.assign(total, std::string());
        // _BuildDecompressedPathsImpl: depth-first, children follow their parent, a positive
        // jump points at the sibling subtree.  Every entry is visited at most once (a crafted jump table that reaches an entry
        // twice would otherwise make the walk exponential): a second visit fails the file.
        std::vector<std::pair<size_t, std::string>> todo{{0, std::string()}};
        std::vector<uint8_t> visited(count, 0);
        while (!todo.empty()) {
            size_t cur = todo.back().first;
            std::string parent = todo.back().second;
            todo.pop_back();
            bool child = false, sibling = false;
            do {
                if (cur >= count) return fail("bad path tree");
                const size_t me = cur++;
                if (visited[me]) return fail("bad path tree (entry reached twice)");
                visited[me] = 1;
                if (idx[me] >= total) return fail("bad path index");
                std::string path;
                if (parent.empty()) {
                    path = "/";
                } else {
                    const int32_t ti = elem[me];
                    const uint32_t tok = (uint32_t)(ti < 0 ? -ti : ti);
                    if (tok >= tokens_.size()) return fail("bad path token");
                    // a variant selection element ("{set=variant}", SdfPath::AppendElementToken) follows
                    // its prim directly: "/Model{shape=a}", whose children are "/Model{shape=a}/Child"
                    // here (the .usda reader's detached variant bodies; SdfPath writes "...}Child")
                    const std::string& e = tokens_[tok];
                    path = ti < 0 ? parent + "." + e
                                  : (!e.empty() && e[0] == '{' && parent != "/") ? parent + e
                                  : (parent == "/" ? "/" : parent + "/") + e;
                }
                paths_[idx[me]] = path;
                child = jump[me] > 0 || jump[me] == -1;
                sibling = jump[me] >= 0;
                if (child) {
                    if (sibling) todo.push_back({me + (size_t)jump[me], parent});
                    parent = path;
                }
            } while (child || sibling);
        }
        return true;
    }
    bool specs() {
        const Section* s = section("SPECS");
        if (!s) return fail("no SPECS section");
        uint64_t count, pos = s->start + 8;
        if (!u64(s->start, count)) return false;
        std::vector<uint32_t> p, f, t;
        if (!compressed_ints<uint32_t>(pos, count, p) || !compressed_ints<uint32_t>(pos, count, f) ||
            !compressed_ints<uint32_t>(pos, count, t))
            return false;
        for (uint64_t i = 0; i < count; ++i) specs_.push_back({p[i], f[i], t[i]});
        return true;
    }

    std::string token(uint64_t i) { return i < tokens_.size() ? tokens_[i] : std::string(); }
    std::string str(uint64_t i) { return i < strings_.size() ? token(strings_[i]) : std::string(); }

    bool index_vector(uint64_t& pos, std::vector<uint32_t>& out) {
        uint64_t count;
        if (!u64(pos, count)) return false;
        if (!has_n(pos + 8, count, 4)) return fail("vector past the end");
        out.resize(count);
        if (count) std::memcpy(out.data(), d_ + pos + 8, count * 4);
        pos += 8 + count * 4;
        return true;
    }
    // SdfListOp: header bits, then explicit, added, prepended, appended, deleted, ordered items
    bool list_op(uint64_t pos, std::vector<uint32_t>& items) {
        if (!has(pos, 1)) return fail("list op past the end");
        const uint8_t h = d_[pos++];
        const uint8_t order[6] = {1u << 1, 1u << 2, 1u << 5, 1u << 6, 1u << 3, 1u << 4};
        for (int k = 0; k < 6; ++k) {
            if (!(h & order[k])) continue;
            std::vector<uint32_t> v;
            if (!index_vector(pos, v)) return false;
            if (k < 4) items.insert(items.end(), v.begin(), v.end());   // deleted / ordered items dropped
        }
        return true;
    }

    // numeric array payload: count, then raw or compressed elements
    bool num_array(uint64_t pos, const NumType& nt, bool compressed, int type, Value& v) {
        uint64_t count;
        if (at_least(0, 7, 0)) {
            if (!u64(pos, count)) return false;
            pos += 8;
        } else {
            uint32_t c32;
            if (!u32(pos, c32)) return false;
            count = c32;
            pos += 4;
        }
        if (count > (1ull << 31)) return fail("array too large");
        v.kind = Value::kNum;
        v.array = true;
        v.comps = nt.comps;
        const bool ints = nt.comps == 1 && (nt.k == 'i' || nt.k == 'I' || nt.k == 'l' || nt.k == 'L');
        const bool floats = nt.comps == 1 && (nt.k == 'h' || nt.k == 'f' || nt.k == 'd');
        if (compressed && ints) {
            if (nt.bytes == 4) {
                std::vector<int32_t> out;
                if (!compressed_ints<int32_t>(pos, count, out)) return false;
                for (int32_t x : out) v.num.push_back(nt.k == 'I' ? (double)(uint32_t)x : (double)x);
            } else {
                std::vector<int64_t> out;
                if (!compressed_ints<int64_t>(pos, count, out)) return false;
                for (int64_t x : out) v.num.push_back(nt.k == 'L' ? (double)(uint64_t)x : (double)x);
            }
            return true;
        }
        if (compressed && floats) {
            if (!has(pos, 1)) return fail("float array code past the end");
            const char code = (char)d_[pos++];
            if (code == 'i') {
                std::vector<int32_t> out;
                if (!compressed_ints<int32_t>(pos, count, out)) return false;
                for (int32_t x : out) v.num.push_back((double)x);
                return true;
            }
            if (code == 't') {
                uint32_t lut_n;
                if (!u32(pos, lut_n)) return false;
                pos += 4;
                if (!has(pos, (uint64_t)lut_n * nt.bytes)) return fail("float table past the end");
                std::vector<double> lut(lut_n);
                for (uint32_t i = 0; i < lut_n; ++i) lut[i] = read_num(d_ + pos + (uint64_t)i * nt.bytes, nt.k);
                pos += (uint64_t)lut_n * nt.bytes;
                std::vector<uint32_t> idx;
                if (!compressed_ints<uint32_t>(pos, count, idx)) return false;
                for (uint32_t i : idx) {
                    if (i >= lut_n) return fail("float table index");
                    v.num.push_back(lut[i]);
                }
                return true;
            }
            return fail("unknown float array code");
        }
        const uint64_t eb = (uint64_t)nt.comps * nt.bytes;
        if (!has_n(pos, count, eb)) return fail("array past the end");
        v.num.reserve(count * nt.comps);
        for (uint64_t i = 0; i < count * nt.comps; ++i) v.num.push_back(read_num(d_ + pos + i * nt.bytes, nt.k));
        if (nt.quat) reorder_quats(v);
        return true;
    }
    // GfQuat memory order (i, j, k, real) -> the text order (real, i, j, k) the stage uses
    static void reorder_quats(Value& v) {
        for (size_t q = 0; q + 3 < v.num.size(); q += 4) {
            const double r = v.num[q + 3];
            v.num[q + 3] = v.num[q + 2];
            v.num[q + 2] = v.num[q + 1];
            v.num[q + 1] = v.num[q];
            v.num[q] = r;
        }
    }

public:
    // ValueRep: bit 63 array, 62 inlined, 61 compressed, type in bits 48..55, payload in 0..47
    bool unpack(uint64_t rep, Value& v, int depth = 0) {
        const bool array = rep >> 63 & 1, inl = rep >> 62 & 1, comp = rep >> 61 & 1;
        const int type = (int)((rep >> 48) & 0xff);
        const uint64_t payload = rep & ((1ull << 48) - 1);
        const NumType nt = num_type(type);
        if (nt.comps) {
            if (array) {
                if (payload == 0 && !inl) { v.kind = Value::kNum; v.array = true; v.comps = nt.comps; return true; }
                return num_array(payload, nt, comp, type, v);
            }
            v.kind = Value::kNum;
            v.comps = nt.comps;
            if (inl) {
                if (nt.comps == 1) {
                    uint32_t bits = (uint32_t)payload;
                    if (nt.k == 'f' || nt.k == 'd') { float f; std::memcpy(&f, &bits, 4); v.num.push_back(f); }
                    else if (nt.k == 'h') v.num.push_back(half_to_float((uint16_t)bits));
                    else if (nt.k == 'i' || nt.k == 'l') v.num.push_back((double)(int32_t)bits);
                    else v.num.push_back((double)bits);
                } else if (nt.matrix) {   // diagonal, int8 entries
                    const int dim = nt.comps == 4 ? 2 : nt.comps == 9 ? 3 : 4;
                    v.num.assign(nt.comps, 0.0);
                    for (int i = 0; i < dim; ++i) v.num[i * dim + i] = (double)(int8_t)((payload >> (8 * i)) & 0xff);
                } else {                  // vectors, int8 components
                    for (int i = 0; i < nt.comps; ++i) v.num.push_back((double)(int8_t)((payload >> (8 * i)) & 0xff));
                    if (nt.quat) reorder_quats(v);
                }
                return true;
            }
            if (!has(payload, (uint64_t)nt.comps * nt.bytes)) return fail("value past the end");
            for (int i = 0; i < nt.comps; ++i) v.num.push_back(read_num(d_ + payload + (uint64_t)i * nt.bytes, nt.k));
            if (nt.quat) reorder_quats(v);
            return true;
        }
        switch (type) {
        case kToken:
        case kString:
        case kAssetPath: {
            v.kind = Value::kStr;
            auto one = [&](uint64_t i) { return type == kString ? str(i) : token(i); };
            if (!array) {
                if (inl) { v.str.push_back(one(payload)); return true; }
                uint32_t i;
                if (!u32(payload, i)) return false;
                v.str.push_back(one(i));
                return true;
            }
            v.array = true;
            if (payload == 0) return true;
            uint64_t count, pos = payload;
            if (at_least(0, 7, 0)) { if (!u64(pos, count)) return false; pos += 8; }
            else { uint32_t c; if (!u32(pos, c)) return false; count = c; pos += 4; }
            if (!has_n(pos, count, 4)) return fail("token array past the end");
            for (uint64_t k = 0; k < count; ++k) {
                uint32_t i;
                std::memcpy(&i, d_ + pos + 4 * k, 4);
                v.str.push_back(one(i));
            }
            return true;
        }
        case kTokenVector:
        case kPathVector:
        case kStringVector: {
            std::vector<uint32_t> idx;
            uint64_t pos = payload;
            if (!index_vector(pos, idx)) return false;
            v.kind = type == kPathVector ? Value::kPath : Value::kStr;
            v.array = true;
            for (uint32_t i : idx) v.str.push_back(type == kPathVector ? (i < paths_.size() ? paths_[i] : "") : type == kStringVector ? str(i) : token(i));
            return true;
        }
        case kTokenListOp:
        case kPathListOp:
        case kStringListOp: {
            std::vector<uint32_t> items;
            if (!list_op(payload, items)) return false;
            v.kind = type == kPathListOp ? Value::kPath : Value::kStr;
            v.array = true;
            for (uint32_t i : items) v.str.push_back(type == kPathListOp ? (i < paths_.size() ? paths_[i] : "") : type == kStringListOp ? str(i) : token(i));
            return true;
        }
        case kReferenceListOp:
        case kPayloadListOp: {
            // SdfListOp<SdfReference | SdfPayload>: each item is {asset path (string index), prim path
            // (path index), layer offset (two doubles; payloads from crate 0.8), custom data
            // (references: a dictionary, read only when empty)}; kept as (asset, path) string pairs
            uint64_t pos = payload;
            if (!has(pos, 1)) return fail("list op past the end");
            const uint8_t h = d_[pos++];
            const uint8_t order[6] = {1u << 1, 1u << 2, 1u << 5, 1u << 6, 1u << 3, 1u << 4};
            v.kind = Value::kStr;
            v.array = true;
            // kept items by list (file order: explicit, added, prepended, appended), composed below as
            // prepended + explicit + added + appended: a prepended arc is the strongest, as in the
            // text reader (`prepend references` goes to the front)
            std::vector<std::string> lists[4];
            for (int k = 0; k < 6; ++k) {
                if (!(h & order[k])) continue;
                uint64_t cnt;
                if (!u64(pos, cnt)) return false;
                pos += 8;
                if (cnt > (1u << 20)) return fail("list op too long");
                for (uint64_t i = 0; i < cnt; ++i) {
                    uint32_t a, pth;
                    if (!u32(pos, a) || !u32(pos + 4, pth)) return false;
                    pos += 8;
                    if (type == kReferenceListOp || at_least(0, 8, 0)) pos += 16;
                    if (type == kReferenceListOp) {
                        uint64_t nd;
                        if (!u64(pos, nd)) return false;
                        pos += 8;
                        if (nd != 0) {   // custom data is not read: the arcs of this field are dropped
                            v.kind = Value::kNone;
                            v.str.clear();
                            return true;
                        }
                    }
                    if (k < 4) {   // explicit / added / prepended / appended items (deleted / ordered dropped)
                        lists[k].push_back(str(a));
                        lists[k].push_back(pth < paths_.size() ? paths_[pth] : std::string());
                    }
                }
            }
            for (int k : {2, 0, 1, 3}) v.str.insert(v.str.end(), lists[k].begin(), lists[k].end());
            return true;
        }
        case kDoubleVector: {
            uint64_t count;
            if (!u64(payload, count)) return false;
            if (!has_n(payload + 8, count, 8)) return fail("double vector past the end");
            v.kind = Value::kNum;
            v.array = true;
            for (uint64_t i = 0; i < count; ++i) v.num.push_back(read_num(d_ + payload + 8 + 8 * i, 'd'));
            return true;
        }
        case kVariantSelectionMap: {
            // SdfVariantSelectionMap: uint64 count, then (set, variant) string indexes; kept as
            // [set, variant, set, variant, ...]
            uint64_t count;
            if (!u64(payload, count)) return false;
            if (!has_n(payload + 8, count, 8)) return fail("variant selection map past the end");
            v.kind = Value::kStr;
            v.array = true;
            for (uint64_t i = 0; i < count; ++i) {
                uint32_t a, b;
                if (!u32(payload + 8 + 8 * i, a) || !u32(payload + 12 + 8 * i, b)) return false;
                v.str.push_back(str(a));
                v.str.push_back(str(b));
            }
            return true;
        }
        case kSpecifier:
        case kVariability:
        case kPermission:
            v.kind = Value::kNum;
            v.num.push_back((double)(uint32_t)payload);
            return true;
        case kValueBlock:
            v.kind = Value::kNone;
            return true;
        default:
            v.kind = Value::kNone;   // dictionaries, references, payloads, ...: not needed by the path
            return true;
        }
    }

    // TimeSamples: [int64 jump][times rep] ... [int64 jump][uint64 n][n value reps]
    bool time_samples(uint64_t rep, Attr& a) {
        const uint64_t o = rep & ((1ull << 48) - 1);
        uint64_t ja, jb, n;
        if (!u64(o, ja)) return false;
        uint64_t times_rep;
        if (!u64(o + 8, times_rep)) return false;
        Value times;
        if (!unpack(times_rep, times)) return false;
        const uint64_t b = o + ja;
        if (!u64(b, jb) || !u64(b + 8, n)) return false;
        if (times.num.size() != n || !has_n(b + 16, n, 8)) return fail("bad time samples");
        for (uint64_t i = 0; i < n; ++i) {
            uint64_t r;
            std::memcpy(&r, d_ + b + 16 + 8 * i, 8);
            Value v;
            if (!unpack(r, v)) return false;
            a.times.push_back(times.num[i]);
            a.samples.push_back(v);
        }
        return true;
    }

private:
    // the prim at an absolute path, creating missing ancestors (iteratively: paths may be deep)
    static int ensure_prim(Stage& st, const std::string& path) {
        int id = 0;
        size_t b = 1;
        while (b < path.size()) {
            size_t e = path.find('/', b);
            if (e == std::string::npos) e = path.size();
            if (e > b) id = st.add_prim(id, path.substr(b, e - b));
            b = e + 1;
        }
        return id;
    }

    bool build(Stage& st) {
        enum { kSpecAttribute = 1, kSpecPrim = 6, kSpecPseudoRoot = 7, kSpecRelationship = 8, kSpecVariant = 10,
               kSpecVariantSet = 11 };
        std::map<int, std::vector<std::string>> child_order;
        // Variant specs first: every "{set=variant}" element of a spec path names a variant body,
        // kept as the detached prim "<owner>{set=variant}" in the owner's variant_bodies, as the
        // .usda reader keeps `variantSet` blocks (outer bodies before the bodies nested in them);
        // the prims, properties and arcs under it then land in the body, and load_stage applies
        // the selected one.  "{set=}" is the variant set spec itself (nothing to keep).
        for (const Spec& sp : specs_) {
            if (sp.path >= paths_.size()) return fail("spec path index");
            const std::string& path = paths_[sp.path];
            for (size_t j = path.find('}'); j != std::string::npos; j = path.find('}', j + 1)) {
                const size_t i = path.rfind('{', j);
                if (i == std::string::npos || i == 0) return fail("bad variant selection path");
                const size_t eq = path.find('=', i);
                if (eq == std::string::npos || eq > j || eq == i + 1) return fail("bad variant selection path");
                if (eq + 1 == j) continue;   // "{set=}"
                const std::string owner = path.substr(0, i);
                if (owner == "/" || owner.find('.') != std::string::npos) return fail("bad variant selection path");
                const int o = ensure_prim(st, owner);
                const int body = st.add_detached(path.substr(0, j + 1));
                st.prims[o].variant_bodies[path.substr(i + 1, eq - i - 1)].emplace(path.substr(eq + 1, j - eq - 1), body);
            }
        }
        for (const Spec& sp : specs_) {
            const std::string& path = paths_[sp.path];
            if (sp.type == kSpecVariantSet) continue;
            std::vector<std::pair<std::string, uint64_t>> f;
            for (uint32_t k = sp.fset; k < fieldsets_.size() && fieldsets_[k] != 0xffffffffu; ++k) {
                const uint32_t fi = fieldsets_[k];
                if (fi >= field_tok_.size()) return fail("field index");
                f.push_back({token(field_tok_[fi]), field_rep_[fi]});
            }
            if (sp.type == kSpecPseudoRoot) {
                for (auto& kv : f) {
                    Value v;
                    if (!unpack(kv.second, v)) return false;
                    if (kv.first == "upAxis" && !v.str.empty()) st.up_axis = v.str[0];
                    if (kv.first == "defaultPrim" && !v.str.empty()) st.default_prim = v.str[0];
                    if (kv.first == "timeCodesPerSecond" && !v.num.empty()) st.time_codes_per_second = v.num[0];
                    if (kv.first == "primChildren") child_order[0] = v.str;
                    if (kv.first == "subLayers" && v.kind == Value::kStr) st.sublayers = v.str;
                }
            } else if (sp.type == kSpecPrim || sp.type == kSpecVariant) {   // a variant spec: its body
                if (sp.type == kSpecPrim && !path.empty() && path.back() == '}') return fail("prim spec at a variant path");
                const int id = ensure_prim(st, path);
                for (auto& kv : f) {
                    Value v;
                    if (!unpack(kv.second, v)) return false;
                    Prim& p = st.prims[id];
                    if (kv.first == "typeName" && !v.str.empty()) p.type = v.str[0];
                    else if (kv.first == "apiSchemas") p.api_schemas = v.str;
                    else if (kv.first == "active" && !v.num.empty()) p.active = v.num[0] != 0.0;
                    else if (kv.first == "primChildren") child_order[id] = v.str;
                    else if (kv.first == "variantSelection" && v.kind == Value::kStr)
                        for (size_t i = 0; i + 1 < v.str.size(); i += 2) p.variant_sel[v.str[i]] = v.str[i + 1];
                    else if ((kv.first == "references" || kv.first == "payload") && v.kind == Value::kStr)
                        for (size_t i = 0; i + 1 < v.str.size(); i += 2)
                            (kv.first == "references" ? p.references : p.payloads).push_back(Arc{v.str[i], v.str[i + 1]});
                }
            } else if (sp.type == kSpecAttribute || sp.type == kSpecRelationship) {
                const size_t dot = path.find_last_of('.');
                if (dot == std::string::npos) continue;
                const int id = ensure_prim(st, path.substr(0, dot));
                const std::string name = path.substr(dot + 1);
                if (sp.type == kSpecRelationship) {
                    auto& targets = st.prims[id].rels[name];
                    for (auto& kv : f) {
                        if (kv.first != "targetPaths" && kv.first != "targetChildren") continue;
                        Value v;
                        if (!unpack(kv.second, v)) return false;
                        targets = v.str;
                    }
                    continue;
                }
                Attr& a = st.prims[id].attrs[name];
                for (auto& kv : f) {
                    if (kv.first == "timeSamples") {
                        if (!time_samples(kv.second, a)) return false;
                        continue;
                    }
                    Value v;
                    if (!unpack(kv.second, v)) return false;
                    if (kv.first == "typeName" && !v.str.empty()) a.type = v.str[0];
                    else if (kv.first == "default" && v.kind != Value::kNone) { a.value = v; a.has_default = true; }
                    else if (kv.first == "variability" && !v.num.empty()) a.uniform = v.num[0] == 1.0;
                    else if (kv.first == "interpolation" && !v.str.empty()) a.interpolation = v.str[0];
                    else if (kv.first == "elementSize" && !v.num.empty()) a.element_size = element_size(v.num[0]);
                    else if (kv.first == "connectionPaths") a.connections = v.str;
                }
            }
        }
        // children in primChildren order (the order ModelIO walks them in)
        for (auto& kv : child_order) {
            Prim& p = st.prims[kv.first];
            std::vector<int> ordered;
            for (const std::string& name : kv.second) {
                const int c = st.find(p.path == "/" ? "/" + name : p.path + "/" + name);
                // only real children, each once (a damaged primChildren list may name the prim
                // itself, an empty name, or one child twice)
                if (c > 0 && c != kv.first && st.prims[c].parent == kv.first &&
                    std::find(ordered.begin(), ordered.end(), c) == ordered.end())
                    ordered.push_back(c);
            }
            for (int c : p.children)
                if (std::find(ordered.begin(), ordered.end(), c) == ordered.end()) ordered.push_back(c);
            p.children = ordered;
        }
        return true;
    }
};

}  // namespace

bool parse_usdc(const uint8_t* data, size_t n, Stage& st, std::string& err) {
    Crate c(data, n);
    return c.run(st, err);
}

static bool parse_layer(const uint8_t* data, size_t n, Stage& st, std::string& err) {
    if (n >= 8 && !std::memcmp(data, "PXR-USDC", 8)) return parse_usdc(data, n, st, err);
    if (n >= 5 && !std::memcmp(data, "#usda", 5)) return parse_usda((const char*)data, n, st, err);
    err = "not a USD layer (neither PXR-USDC nor #usda)";
    return false;
}

// ---- composition ------------------------------------------------------------------------------
namespace {

constexpr int kMaxArcDepth = 16;              // nested layer loads (sublayer / reference chains)
constexpr size_t kMaxComposedPrims = 1u << 17;  // prims a composition may create (hostile fan-out)
constexpr uint64_t kMaxLayerBytes = 1ull << 31;   // a referenced layer file (regular files only)
constexpr uint64_t kMaxComposedBytes = 4ull << 30;   // attribute data merges may copy (hostile fan-out)

std::string dir_of(const std::string& id) {
    const size_t k = id.find_last_of('/');
    return k == std::string::npos ? std::string() : id.substr(0, k + 1);
}
// collapses "." and ".." segments (a leading "/" is kept)
std::string normalize(const std::string& p) {
    std::vector<std::string> seg;
    size_t b = 0;
    while (b <= p.size()) {
        size_t e = p.find('/', b);
        if (e == std::string::npos) e = p.size();
        const std::string x = p.substr(b, e - b);
        if (x == "..") { if (!seg.empty() && seg.back() != "..") seg.pop_back(); else seg.push_back(x); }
        else if (!x.empty() && x != ".") seg.push_back(x);
        b = e + 1;
    }
    std::string out = !p.empty() && p[0] == '/' ? "/" : "";
    for (size_t k = 0; k < seg.size(); ++k) out += (k ? "/" : "") + seg[k];
    return out;
}
// a path of the source subtree rooted at `from`, moved under `to`
std::string remap(const std::string& x, const std::string& from, const std::string& to) {
    if (from.empty() || from == to || x.compare(0, from.size(), from) != 0) return x;
    if (x.size() > from.size() && x[from.size()] != '/' && x[from.size()] != '.') return x;
    return to + x.substr(from.size());
}

class Composer {
public:
    explicit Composer(const std::vector<PackageFile>* pkg) : pkg_(pkg) {}
    std::string err;

    // layer `id` parsed and composed; shared by every arc that names it (no copy per arc)
    std::shared_ptr<const Stage> load(const std::string& id, int depth) {
        if (depth > kMaxArcDepth) {
            fail("composition nested deeper than " + std::to_string(kMaxArcDepth) + " layers");
            return nullptr;
        }
        auto c = cache_.find(id);
        if (c != cache_.end()) return c->second;
        if (loading_.count(id)) {
            fail("composition cycle through " + id);
            return nullptr;
        }
        std::vector<uint8_t> data;
        if (!read(id, data)) {
            fail("cannot open layer " + id);
            return nullptr;
        }
        auto L = std::make_shared<Stage>();
        L->layer_id = id;
        std::string e;
        if (!parse_layer(data.data(), data.size(), *L, e)) {
            fail(id + ": " + e);
            return nullptr;
        }
        loading_.insert(id);
        const bool ok = compose(id, *L, depth);
        loading_.erase(id);
        if (!ok) return nullptr;
        cache_[id] = L;
        return L;
    }

    // sublayers under the layer's own opinions, then every prim's arcs in namespace order.  Variant
    // selections are composed in the root layer (depth 0) only: a sublayer or referenced layer keeps
    // its selections and variant bodies unapplied, so the strongest selection of the whole stack
    // (the root's own, then its sublayers', then the referenced layers') picks the variant.
    bool compose(const std::string& id, Stage& L, int depth) {
        L.layer_id = id;
        const std::vector<std::string> subs = L.sublayers;
        L.sublayers.clear();
        for (const std::string& sub : subs) {
            const std::shared_ptr<const Stage> S = load(resolve(id, sub), depth + 1);
            if (!S) return false;
            if (!merge(L, 0, *S, 0, "", "")) return false;
            if (L.default_prim.empty()) L.default_prim = S->default_prim;
        }
        std::vector<int> todo{0};
        std::vector<uint8_t> seen;   // each prim once, whatever its children lists say
        while (!todo.empty()) {
            const int p = todo.back();
            todo.pop_back();
            if ((size_t)p >= seen.size()) seen.resize(L.prims.size() + 1, 0);
            if (seen[p]) continue;
            seen[p] = 1;
            if (!apply_arcs(id, L, p, depth, depth == 0)) return false;
            const std::vector<int>& ch = L.prims[p].children;
            for (auto it = ch.rbegin(); it != ch.rend(); ++it) todo.push_back(*it);
        }
        return true;
    }

private:
    const std::vector<PackageFile>* pkg_;
    std::set<std::string> loading_;
    std::map<std::string, std::shared_ptr<const Stage>> cache_;
    size_t budget_ = kMaxComposedPrims;
    uint64_t bytes_budget_ = kMaxComposedBytes;

    bool fail(const std::string& m) {
        err = m;
        return false;
    }
    // composition work (prims merged, arcs applied, internal snapshots copied) is bounded: a
    // hostile list of a million arcs must fail fast, not merge a subtree a million times
    bool spend(size_t n) {
        if (n > budget_) return fail("composed stage larger than " + std::to_string(kMaxComposedPrims) + " prims");
        budget_ -= n;
        return true;
    }
    // and so are the attribute bytes merges copy: a few references to one large mesh layer must
    // not multiply its arrays into terabytes
    bool spend_bytes(uint64_t n) {
        if (n > bytes_budget_) return fail("composed attribute data larger than " + std::to_string(kMaxComposedBytes >> 20) + " MiB");
        bytes_budget_ -= n;
        return true;
    }
    static uint64_t value_bytes(const Value& v) {
        uint64_t b = 8 * (uint64_t)v.num.size() + 32;
        for (const std::string& s : v.str) b += s.size() + 32;
        return b;
    }
    static uint64_t attr_bytes(const Attr& a) {
        uint64_t b = value_bytes(a.value) + 8 * (uint64_t)a.times.size();
        for (const Value& v : a.samples) b += value_bytes(v);
        for (const std::string& s : a.connections) b += s.size() + 32;
        return b;
    }
    // what a copy of a whole stage copies (an internal arc's snapshot of its layer)
    static uint64_t stage_bytes(const Stage& L) {
        uint64_t b = 0;
        for (const Prim& pr : L.prims) {
            b += 256;
            for (const auto& kv : pr.attrs) b += attr_bytes(kv.second);
        }
        return b;
    }
    // an asset path relative to the layer naming it (inside the package for a .usdz)
    std::string resolve(const std::string& from, const std::string& asset) const {
        if (!asset.empty() && asset[0] == '/') return normalize(pkg_ ? asset.substr(1) : asset);
        return normalize(dir_of(from) + asset);
    }
    bool read(const std::string& id, std::vector<uint8_t>& data) const {
        if (pkg_) {
            for (const PackageFile& f : *pkg_)
                if (normalize(f.name) == id) { data = f.data; return true; }
            return false;
        }
        // an asset path comes from the file: only a regular file of bounded size is read (a
        // reference to /dev/zero or a FIFO must not hang the loader)
        struct stat sb;
        if (stat(id.c_str(), &sb) != 0 || !S_ISREG(sb.st_mode) || (uint64_t)sb.st_size > kMaxLayerBytes) return false;
        FILE* f = std::fopen(id.c_str(), "rb");
        if (!f) return false;
        uint8_t buf[1 << 16];
        size_t k;
        while ((k = std::fread(buf, 1, sizeof buf, f)) > 0 && data.size() <= kMaxLayerBytes) data.insert(data.end(), buf, buf + k);
        std::fclose(f);
        return data.size() <= kMaxLayerBytes;
    }

    // Prim s of S (and its subtree) merged into prim d of D as the weaker opinion: only what D does
    // not author is taken; paths under `from` move under `to`.  S may be D (a variant body).
    bool merge(Stage& D, int d, const Stage& S, int s, const std::string from, const std::string to) {   // paths by value: D.prims may move
        std::vector<std::pair<int, int>> work{{d, s}};
        while (!work.empty()) {
            const auto [dd, ss] = work.back();
            work.pop_back();
            if (!spend(1)) return false;
            const Prim src = S.prims[ss];   // a copy: D's prims may move below when S is D
            Prim& dp = D.prims[dd];
            if (dp.type.empty()) dp.type = src.type;
            for (const std::string& a : src.api_schemas)
                if (std::find(dp.api_schemas.begin(), dp.api_schemas.end(), a) == dp.api_schemas.end()) dp.api_schemas.push_back(a);
            for (const auto& kv : src.attrs) {
                if (dp.attrs.count(kv.first)) continue;
                if (!spend_bytes(attr_bytes(kv.second))) return false;
                Attr a = kv.second;
                for (std::string& c : a.connections) c = remap(c, from, to);
                dp.attrs.emplace(kv.first, std::move(a));
            }
            for (const auto& kv : src.rels) {
                if (dp.rels.count(kv.first)) continue;
                std::vector<std::string> t = kv.second;
                for (std::string& x : t) x = remap(x, from, to);
                dp.rels.emplace(kv.first, std::move(t));
            }
            // arcs not yet applied: carried over, applied when the walk gets here; out of another layer
            // they keep resolving against that layer (its assets, its namespace for internal arcs)
            for (int k = 0; k < 2; ++k) {
                const std::vector<Arc>& from_arcs = k ? src.payloads : src.references;
                std::vector<Arc>& to_arcs = k ? dp.payloads : dp.references;
                for (Arc a : from_arcs) {
                    if (&S != &D && !a.resolved && !S.layer_id.empty()) {
                        a.asset = a.asset.empty() ? S.layer_id : resolve(S.layer_id, a.asset);
                        a.resolved = true;
                    }
                    to_arcs.push_back(std::move(a));
                }
            }
            for (const auto& kv : src.variant_sel) dp.variant_sel.emplace(kv.first, kv.second);
            // variant bodies: prim indices of S.  Within one stage they stay valid; from another stage
            // (a sublayer, a referenced layer) each body subtree is merged into a detached prim of D
            // at "<dest path>{set=variant}" first, and D's index is kept.  A body D already has for
            // that variant is the stronger opinion and stays.
            std::vector<std::pair<std::pair<std::string, std::string>, int>> foreign;
            for (const auto& kv : src.variant_bodies)
                for (const auto& v : kv.second) {
                    if (&S == &D) dp.variant_bodies[kv.first].emplace(v.first, v.second);
                    else if (!dp.variant_bodies.count(kv.first) || !dp.variant_bodies[kv.first].count(v.first))
                        foreign.push_back({{kv.first, v.first}, v.second});
                }
            const std::string dpath = dp.path;
            for (const auto& f : foreign) {   // (dp may move from here on)
                if (f.second <= 0 || (size_t)f.second >= S.prims.size()) continue;
                const int body = D.add_detached(dpath + "{" + f.first.first + "=" + f.first.second + "}");
                if (!merge(D, body, S, f.second, from, to)) return false;
                D.prims[dd].variant_bodies[f.first.first].emplace(f.first.second, body);
            }
            for (int c : src.children) {
                const std::string name = S.prims[c].name;
                const bool active = S.prims[c].active;
                const size_t before = D.prims.size();
                const int dc = D.add_prim(dd, name);
                if (D.prims.size() > before) D.prims[dc].active = active;
                work.push_back({dc, c});
            }
        }
        return true;
    }

    // the prim an arc targets: its path, else the layer's defaultPrim, else its first root prim
    static int target(const Stage& S, const Arc& a) {
        if (!a.path.empty()) return S.find(a.path);
        if (!S.default_prim.empty()) return S.find("/" + S.default_prim);
        return S.prims[0].children.empty() ? -1 : S.prims[0].children[0];
    }

    // LIVRPS below local opinions: the selected variants, then references, then payloads.  A
    // selection whose variant set has no body yet stays: a reference or payload merged later may
    // bring the set (the common pattern: the referencing prim selects a variant of the asset it
    // references); its own selection stays the stronger one (merge keeps existing selections).
    // Each set is composed once.
    bool apply_arcs(const std::string& id, Stage& L, int p, int depth, bool variants) {
        std::set<std::string> composed;
        for (int round = 0; round < kMaxArcDepth; ++round) {
            Prim& P = L.prims[p];
            std::vector<int> bodies;
            for (const auto& kv : P.variant_sel) {
                if (!variants) break;
                if (composed.count(kv.first)) continue;
                auto set = P.variant_bodies.find(kv.first);
                if (set == P.variant_bodies.end()) continue;
                auto var = set->second.find(kv.second);
                if (var == set->second.end()) continue;
                composed.insert(kv.first);
                bodies.push_back(var->second);
            }
            std::vector<Arc> arcs = P.references;
            arcs.insert(arcs.end(), P.payloads.begin(), P.payloads.end());
            P.references.clear();
            P.payloads.clear();
            if (bodies.empty() && arcs.empty()) {   // settled (a non-root layer keeps its variants for the stack)
                if (variants) {
                    P.variant_sel.clear();
                    P.variant_bodies.clear();
                }
                return true;
            }
            for (int b : bodies)
                if (!merge(L, p, L, b, L.prims[b].path, L.prims[p].path)) return false;
            // the internal arcs of one round all read this layer's namespace as it stood before the
            // round's merges (as in USD, where the arcs of one list target the authored namespace,
            // not each other's results): one snapshot per round, taken before the round's arcs merge
            // and charged once against the byte budget (thousands of rounds next to one large array
            // still fail fast instead of copying the layer thousands of times)
            auto is_internal = [&](const Arc& a) { return a.asset.empty() || (a.resolved && a.asset == id); };
            std::shared_ptr<const Stage> snapshot;
            if (std::any_of(arcs.begin(), arcs.end(), is_internal)) {
                if (!spend(L.prims.size()) || !spend_bytes(stage_bytes(L))) return false;
                snapshot = std::make_shared<const Stage>(L);
            }
            for (const Arc& a : arcs) {
                if (!spend(1)) return false;
                std::shared_ptr<const Stage> S;
                const bool internal = is_internal(a);
                if (internal) {
                    S = snapshot;
                } else if (!(S = load(a.resolved ? a.asset : resolve(id, a.asset), depth + 1))) return false;
                const int t = target(*S, a);
                if (t <= 0) return fail("reference target " + (a.path.empty() ? "(default prim)" : a.path) + " not found in " +
                                        (internal ? id : a.asset));
                if (internal && t == p) continue;
                if (!merge(L, p, *S, t, S->prims[t].path, L.prims[p].path)) return false;
            }
        }
        return fail("composition of " + L.prims[p].path + " does not settle");
    }
};

}  // namespace

static bool load_stage_impl(const std::string& path, Stage& st, std::vector<PackageFile>& files, std::string& err) {
    struct stat sb;
    if (stat(path.c_str(), &sb) != 0 || !S_ISREG(sb.st_mode) || (uint64_t)sb.st_size > kMaxLayerBytes) {
        err = "cannot open " + path + " (not a regular file of at most 2 GiB)";
        return false;
    }
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) { err = "cannot open " + path; return false; }
    std::vector<uint8_t> data;
    uint8_t buf[1 << 16];
    size_t k;
    while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) data.insert(data.end(), buf, buf + k);
    std::fclose(f);
    if (data.size() >= 4 && rd32(data.data()) == 0x04034b50u) {   // .usdz: the first layer is the root
        if (!read_zip(data.data(), data.size(), files, err)) return false;
        for (const PackageFile& pf : files) {
            const size_t dot = pf.name.find_last_of('.');
            const std::string ext = dot == std::string::npos ? "" : pf.name.substr(dot);
            if (ext == ".usd" || ext == ".usda" || ext == ".usdc") {
                if (!parse_layer(pf.data.data(), pf.data.size(), st, err)) return false;
                st.layer_id = normalize(pf.name);
                Composer comp(&files);
                if (!comp.compose(normalize(pf.name), st, 0)) { err = comp.err; return false; }
                return true;
            }
        }
        err = "usdz package without a USD layer";
        return false;
    }
    if (!parse_layer(data.data(), data.size(), st, err)) return false;
    st.layer_id = path;
    Composer comp(nullptr);
    if (!comp.compose(path, st, 0)) { err = comp.err; return false; }
    return true;
}

// Asset bytes are untrusted: a file that asks for more memory than the process has fails the load
// (RT_ERR_IO at rt_scene_add_usd) instead of letting std::bad_alloc cross the C-ABI.
bool load_stage(const std::string& path, Stage& st, std::vector<PackageFile>& files, std::string& err) {
    try {
        return load_stage_impl(path, st, files, err);
    } catch (const std::bad_alloc&) {
        err = "out of memory while reading " + path;
    } catch (const std::exception& e) {
        err = std::string("error while reading ") + path + ": " + e.what();
    }
    st = Stage();
    files.clear();
    return false;
}

}  // namespace usd
}  // namespace rt
