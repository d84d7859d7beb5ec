// gotemplate.cpp - see gotemplate.h.
//
// text/template subset (Go 1.19 semantics, text/template/exec.go): text and
// {{ pipeline }} actions with {{- / -}} trim markers and {{/* comments */}};
// if / with / range with else (and `else if`), end; `$v := pipeline`, $v, $;
// field chains on maps (a missing key is "<no value>"); literals (strings,
// integers, true / false / nil); function calls with operand arguments:
// the template funcs, YAML (controller.go:42-54) and the builtins not / and /
// or / eq / ne / len.  Printing follows fmt: strings verbatim, numbers as
// json.Number text, <no value> for nil.  Pipes ("|"), parentheses, printf
// and ranges over two variables are outside the subset.
//
// YAML (yaml.v2 over sigs.k8s.io/yaml v1.3.0): block mappings and sequences,
// flow [..] / {..}, plain / single- / double-quoted scalars, comments.  Plain
// scalars resolve as yaml.v2 does to null, bool (YAML 1.1 words), decimal
// int, or string (timestamps stay strings); other number forms (hex, octal,
// floats, ...) are outside the subset.  Output: encoding/json.Marshal of the
// tree (sorted keys, compact, HTML-safe).
#include "gotemplate.h"

#include <ctype.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>

namespace kwok {
namespace gotpl {

VPtr make_str(const std::string& s, const std::string& path) {
    auto v = std::make_shared<Value>();
    v->kind = Value::STR;
    v->s = s;
    v->path = path;
    return v;
}
VPtr make_null(const std::string& path) {
    auto v = std::make_shared<Value>();
    v->kind = Value::NUL;
    v->path = path;
    return v;
}
VPtr make_map(std::vector<std::pair<std::string, VPtr>> kv, const std::string& path) {
    auto v = std::make_shared<Value>();
    v->kind = Value::MAP;
    std::sort(kv.begin(), kv.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
    v->map = std::move(kv);
    v->path = path;
    return v;
}
VPtr make_list(std::vector<VPtr> items, const std::string& path) {
    auto v = std::make_shared<Value>();
    v->kind = Value::LIST;
    v->list = std::move(items);
    v->path = path;
    return v;
}
namespace {
VPtr make_noval(const std::string& path) {
    auto v = std::make_shared<Value>();
    v->path = path;
    return v;
}
VPtr make_bool(bool b) {
    auto v = std::make_shared<Value>();
    v->kind = Value::BOOL;
    v->b = b;
    return v;
}
VPtr make_num(const std::string& s) {
    auto v = std::make_shared<Value>();
    v->kind = Value::NUM;
    v->s = s;
    return v;
}
struct Fail {
    std::string msg;
};
[[noreturn]] void fail(const std::string& m) { throw Fail{m}; }
}  // namespace

VPtr with_paths(const VPtr& v, const std::string& path) {
    auto c = std::make_shared<Value>(*v);
    c->path = path;
    for (auto& kv : c->map) kv.second = with_paths(kv.second, path + "." + kv.first);
    for (auto& it : c->list) it = with_paths(it, path + "[]");
    return c;
}

// ---------------------------------------------------------------------------
// template parse
// ---------------------------------------------------------------------------
namespace {
enum TokKind { T_FIELD, T_VAR, T_STR, T_NUM, T_IDENT, T_DECL };
struct Tok {
    TokKind k;
    std::string v;
};
struct Pipe {
    std::string decl;  // "$x" for `$x := ...`
    std::vector<Tok> cmd;
};
struct Node {
    enum { TEXT, ACTION, IF, WITH, RANGE } kind;
    std::string text;
    Pipe pipe;
    std::vector<Node> body, else_body;
    bool has_else = false;
};

std::vector<Tok> tokenize(const std::string& src) {
    std::vector<Tok> out;
    size_t i = 0, n = src.size();
    auto ident_ch = [](char c) { return isalnum((unsigned char)c) || c == '_'; };
    while (i < n) {
        const char c = src[i];
        if (isspace((unsigned char)c)) {
            i++;
            continue;
        }
        if (c == ':' && i + 1 < n && src[i + 1] == '=') {
            out.push_back({T_DECL, ":="});
            i += 2;
        } else if (c == '"') {
            std::string s;
            size_t j = i + 1;
            for (; j < n && src[j] != '"'; j++) {
                if (src[j] == '\\' && j + 1 < n) {
                    const char e = src[++j];
                    s.push_back(e == 'n' ? '\n' : e == 't' ? '\t' : e == 'r' ? '\r' : e);
                } else {
                    s.push_back(src[j]);
                }
            }
            if (j >= n) fail("unterminated string in action");
            out.push_back({T_STR, s});
            i = j + 1;
        } else if (c == '`') {
            const size_t j = src.find('`', i + 1);
            if (j == std::string::npos) fail("unterminated raw string in action");
            out.push_back({T_STR, src.substr(i + 1, j - i - 1)});
            i = j + 1;
        } else if (isdigit((unsigned char)c) || (c == '-' && i + 1 < n && isdigit((unsigned char)src[i + 1]))) {
            size_t j = i + 1;
            while (j < n && (isdigit((unsigned char)src[j]))) j++;
            if (j < n && (src[j] == '.' || src[j] == 'e' || src[j] == 'x')) fail("non-integer number literals are outside the subset");
            out.push_back({T_NUM, src.substr(i, j - i)});
            i = j;
        } else if (c == '$' || c == '.') {
            size_t j = i + 1;
            if (c == '$')
                while (j < n && ident_ch(src[j])) j++;
            while (j < n && src[j] == '.' && j + 1 < n && ident_ch(src[j + 1])) {
                j++;
                while (j < n && ident_ch(src[j])) j++;
            }
            if (c == '.' && j == i + 1 && j < n && ident_ch(src[j])) {  // ".name"
                while (j < n && ident_ch(src[j])) j++;
                while (j < n && src[j] == '.' && j + 1 < n && ident_ch(src[j + 1])) {
                    j++;
                    while (j < n && ident_ch(src[j])) j++;
                }
            }
            out.push_back({c == '$' ? T_VAR : T_FIELD, src.substr(i, j - i)});
            i = j;
        } else if (ident_ch(c)) {
            size_t j = i;
            while (j < n && ident_ch(src[j])) j++;
            out.push_back({T_IDENT, src.substr(i, j - i)});
            i = j;
        } else {
            fail(std::string("'") + c + "' in an action is outside the covered template subset");
        }
    }
    return out;
}

Pipe make_pipe(std::vector<Tok> toks) {
    Pipe p;
    if (toks.size() >= 2 && toks[1].k == T_DECL) {
        if (toks[0].k != T_VAR) fail("bad declaration");
        p.decl = toks[0].v;
        toks.erase(toks.begin(), toks.begin() + 2);
    }
    if (toks.empty()) fail("empty pipeline");
    p.cmd = std::move(toks);
    return p;
}

std::vector<Node> parse_template(const std::string& text) {
    std::vector<Node> root;
    // stack of (node list being filled, owning block or null); chained `else if`
    // blocks end with their parent
    struct Frame {
        std::vector<Node>* list;
        Node* block;
        bool chained;
    };
    std::vector<Frame> st{{&root, nullptr, false}};
    size_t pos = 0;
    bool trim_next = false;
    while (true) {
        size_t i = text.find("{{", pos);
        std::string pre = text.substr(pos, i == std::string::npos ? std::string::npos : i - pos);
        if (trim_next) {
            size_t k = 0;
            while (k < pre.size() && isspace((unsigned char)pre[k])) k++;
            pre = pre.substr(k);
            trim_next = false;
        }
        if (i == std::string::npos) {
            if (!pre.empty()) st.back().list->push_back(Node{Node::TEXT, pre, {}, {}, {}, false});
            break;
        }
        const size_t j = text.find("}}", i + 2);
        if (j == std::string::npos) fail("unclosed action");
        std::string inner = text.substr(i + 2, j - i - 2);
        pos = j + 2;
        if (inner.size() >= 2 && inner[0] == '-' && isspace((unsigned char)inner[1])) {
            while (!pre.empty() && isspace((unsigned char)pre.back())) pre.pop_back();
            inner = inner.substr(2);
        }
        if (inner.size() >= 2 && inner.back() == '-' && isspace((unsigned char)inner[inner.size() - 2])) {
            inner = inner.substr(0, inner.size() - 2);
            trim_next = true;
        }
        if (!pre.empty()) st.back().list->push_back(Node{Node::TEXT, pre, {}, {}, {}, false});
        {
            size_t a = 0;
            while (a < inner.size() && isspace((unsigned char)inner[a])) a++;
            if (inner.compare(a, 2, "/*") == 0) {  // {{/* comment */}}
                const size_t e = inner.find("*/", a + 2);
                if (e == std::string::npos) fail("unclosed comment");
                continue;
            }
        }
        std::vector<Tok> toks = tokenize(inner);
        if (toks.empty()) fail("empty action");
        const Tok head = toks[0];
        if (head.k == T_IDENT && head.v == "end") {
            while (true) {
                if (st.size() < 2) fail("unexpected {{end}}");
                const bool chained = st.back().chained;
                st.pop_back();
                if (!chained) break;
            }
        } else if (head.k == T_IDENT && head.v == "else") {
            Frame& f = st.back();
            if (!f.block || f.block->has_else) fail("unexpected {{else}}");
            f.block->has_else = true;
            f.list = &f.block->else_body;
            if (toks.size() > 1) {  // else if / else with: a nested block that ends with this one
                if (st.size() > 64) fail("template blocks nested deeper than the covered subset");
                if (toks[1].k != T_IDENT || (toks[1].v != "if" && toks[1].v != "with")) fail("unsupported else clause");
                Node b{toks[1].v == "if" ? Node::IF : Node::WITH, "", make_pipe({toks.begin() + 2, toks.end()}), {}, {}, false};
                f.list->push_back(std::move(b));
                Node* nb = &f.list->back();
                st.push_back({&nb->body, nb, true});
            }
        } else if (head.k == T_IDENT && (head.v == "if" || head.v == "with" || head.v == "range")) {
            if (st.size() > 64) fail("template blocks nested deeper than the covered subset");
            Node b{head.v == "if" ? Node::IF : head.v == "with" ? Node::WITH : Node::RANGE, "",
                   make_pipe({toks.begin() + 1, toks.end()}), {}, {}, false};
            st.back().list->push_back(std::move(b));
            Node* nb = &st.back().list->back();
            st.push_back({&nb->body, nb, false});
        } else if (head.k == T_IDENT && (head.v == "define" || head.v == "template" || head.v == "block")) {
            fail("{{" + head.v + "}} is outside the covered template subset");
        } else {
            st.back().list->push_back(Node{Node::ACTION, "", make_pipe(toks), {}, {}, false});
        }
    }
    if (st.size() != 1) fail("unterminated block");
    return root;
}

// ---------------------------------------------------------------------------
// execution
// ---------------------------------------------------------------------------
bool truth(const VPtr& v) {
    switch (v->kind) {
        case Value::NOVAL:
        case Value::NUL: return false;
        case Value::BOOL: return v->b;
        case Value::NUM: return !(v->s == "0" || v->s == "-0");
        case Value::STR: return !v->s.empty();
        case Value::LIST: return !v->list.empty();
        case Value::MAP: return !v->map.empty();
    }
    return false;
}

std::string yaml_marshal(const VPtr& v, int indent);

struct Exec {
    const Env& env;
    std::vector<std::pair<std::string, VPtr>> vars;
    std::string out;

    bool allowed(const std::string& p) const {
        for (const std::string& a : *env.allowed_paths) {
            if (a == p) return true;
            if (a.size() >= 2 && a.compare(a.size() - 2, 2, ".*") == 0 && p.size() > a.size() - 2 &&
                p.compare(0, a.size() - 2, a, 0, a.size() - 2) == 0 && (p[a.size() - 2] == '.' || p[a.size() - 2] == '['))
                return true;
        }
        return false;
    }
    VPtr field(VPtr v, const std::string& chain) {  // ".a.b" (or "" for v)
        size_t i = 0;
        while (i < chain.size()) {
            if (chain[i] != '.') fail("bad field chain " + chain);
            size_t j = chain.find('.', i + 1);
            if (j == std::string::npos) j = chain.size();
            const std::string name = chain.substr(i + 1, j - i - 1);
            i = j;
            if (name.empty()) continue;
            if (v->kind != Value::MAP) fail("field ." + name + " of a non-map value is outside the subset");
            const std::string p = v->path + "." + name;
            if (env.allowed_paths && !allowed(p)) fail("the template reads " + p + ", which the engine does not hold");
            auto it = std::lower_bound(v->map.begin(), v->map.end(), name,
                                       [](const auto& kv, const std::string& k) { return kv.first < k; });
            v = (it != v->map.end() && it->first == name) ? it->second : make_noval(p);
        }
        return v;
    }
    VPtr var(const std::string& name) {
        for (auto it = vars.rbegin(); it != vars.rend(); ++it)
            if (it->first == name) return it->second;
        fail("undefined variable " + name);
    }
    VPtr operand(const Tok& t, const VPtr& dot) {
        switch (t.k) {
            case T_FIELD: return t.v == "." ? dot : field(dot, t.v);
            case T_VAR: {
                const size_t d = t.v.find('.');
                const VPtr base = var(t.v.substr(0, d));
                return d == std::string::npos ? base : field(base, t.v.substr(d));
            }
            case T_STR: return make_str(t.v);
            case T_NUM: return make_num(t.v[0] == '+' ? t.v.substr(1) : t.v);
            case T_IDENT:
                if (t.v == "true" || t.v == "false") return make_bool(t.v == "true");
                if (t.v == "nil") return make_null();
                return call(t.v, {});
            default: fail("bad operand");
        }
    }
    static bool basic_eq(const VPtr& a, const VPtr& b) {
        if (a->kind != b->kind) return false;
        if (a->kind == Value::BOOL) return a->b == b->b;
        if (a->kind == Value::STR || a->kind == Value::NUM) return a->s == b->s;
        if (a->kind == Value::NUL || a->kind == Value::NOVAL) return true;
        fail("eq / ne of composite values");
    }
    VPtr call(const std::string& fn, const std::vector<VPtr>& args) {
        auto it = env.funcs.find(fn);
        if (it != env.funcs.end()) {
            if (!args.empty()) fail(fn + " takes no arguments");
            return make_str(it->second());
        }
        if (fn == "YAML") {
            if (args.empty() || args.size() > 2) fail("YAML takes one or two arguments");
            int indent = 0;
            if (args.size() == 2) {
                if (args[1]->kind != Value::NUM) fail("YAML indent must be an integer");
                indent = atoi(args[1]->s.c_str());
            }
            return make_str(yaml_marshal(args[0], indent));
        }
        if (fn == "not" && args.size() == 1) return make_bool(!truth(args[0]));
        if ((fn == "and" || fn == "or") && !args.empty()) {
            for (size_t i = 0; i + 1 < args.size(); i++)
                if (truth(args[i]) != (fn == "and")) return args[i];
            return args.back();
        }
        if ((fn == "eq" || fn == "ne") && args.size() >= 2) {
            bool any = false;
            for (size_t i = 1; i < args.size(); i++) any |= basic_eq(args[0], args[i]);
            return make_bool(fn == "eq" ? any : !any);
        }
        if (fn == "len" && args.size() == 1) {
            const VPtr& a = args[0];
            if (a->kind == Value::STR) return make_num(std::to_string(a->s.size()));
            if (a->kind == Value::LIST) return make_num(std::to_string(a->list.size()));
            if (a->kind == Value::MAP) return make_num(std::to_string(a->map.size()));
            fail("len of a scalar");
        }
        fail("function " + fn + " is outside the covered template subset");
    }
    // returns the pipeline's value (nullptr for a declaration)
    VPtr pipe(const Pipe& p, const VPtr& dot) {
        VPtr v;
        const Tok& h = p.cmd[0];
        if (h.k == T_IDENT && p.cmd.size() > 1) {
            std::vector<VPtr> args;
            for (size_t i = 1; i < p.cmd.size(); i++) args.push_back(operand(p.cmd[i], dot));
            v = call(h.v, args);
        } else {
            if (p.cmd.size() != 1) fail("a pipeline of more than one operand is outside the subset");
            v = operand(h, dot);
        }
        if (!p.decl.empty()) {
            vars.push_back({p.decl, v});
            return nullptr;
        }
        return v;
    }
    void print(const VPtr& v) {
        switch (v->kind) {
            case Value::NOVAL:
            case Value::NUL: out += "<no value>"; break;
            case Value::BOOL: out += v->b ? "true" : "false"; break;
            case Value::NUM:
            case Value::STR: out += v->s; break;
            default: fail("printing a map or list is outside the covered subset (use YAML)");
        }
    }
    void run(const std::vector<Node>& nodes, const VPtr& dot) {
        for (const Node& n : nodes) {
            if (n.kind == Node::TEXT) {
                out += n.text;
            } else if (n.kind == Node::ACTION) {
                VPtr v = pipe(n.pipe, dot);
                if (v) print(v);
            } else {
                const size_t mark = vars.size();  // variables are scoped to the block
                VPtr v = pipe(n.pipe, dot);
                if (!v) fail("a declaration as a block condition is outside the subset");
                if (n.kind == Node::RANGE) {
                    std::vector<VPtr> items;
                    if (v->kind == Value::LIST) items = v->list;
                    else if (v->kind == Value::MAP)
                        for (auto& kv : v->map) items.push_back(kv.second);
                    else if (v->kind != Value::NOVAL && v->kind != Value::NUL) fail("range over a scalar");
                    if (!items.empty())
                        for (auto& it : items) run(n.body, it);
                    else if (n.has_else) run(n.else_body, dot);
                } else if (truth(v)) {
                    run(n.body, n.kind == Node::WITH ? v : dot);
                } else if (n.has_else) {
                    run(n.else_body, dot);
                }
                vars.resize(mark);
            }
        }
    }
};

// ---------------------------------------------------------------------------
// YAML func: sigs.k8s.io/yaml.Marshal (json -> yaml) + optional indentation.
// The exact text differs from yaml.v2's emitter, but it re-parses to the same
// tree, which is all that reaches the JSON output.
// ---------------------------------------------------------------------------
void json_quote(std::string& out, const std::string& s) {
    static const char hex[] = "0123456789abcdef";
    out.push_back('"');
    for (size_t i = 0; i < s.size(); i++) {
        const unsigned char c = (unsigned char)s[i];
        if (c == '"') out += "\\\"";
        else if (c == '\\') out += "\\\\";
        else if (c == '\n') out += "\\n";
        else if (c == '\r') out += "\\r";
        else if (c == '\t') out += "\\t";
        else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
            out += "\\u00";
            out.push_back(hex[c >> 4]);
            out.push_back(hex[c & 15]);
        } else if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
                   ((unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9)) {
            out += (unsigned char)s[i + 2] == 0xA8 ? "\\u2028" : "\\u2029";
            i += 2;
        } else out.push_back((char)c);
    }
    out.push_back('"');
}
void yaml_emit(std::string& o, const VPtr& v, int ind) {
    const std::string pad(ind, ' ');
    auto scalar = [](const VPtr& x) {
        std::string s;
        switch (x->kind) {
            case Value::NOVAL:
            case Value::NUL: return std::string("null");
            case Value::BOOL: return std::string(x->b ? "true" : "false");
            case Value::NUM: return x->s;
            case Value::STR: json_quote(s, x->s); return s;
            case Value::LIST: return std::string("[]");
            case Value::MAP: return std::string("{}");
        }
        return s;
    };
    auto composite = [](const VPtr& x) {
        return (x->kind == Value::LIST && !x->list.empty()) || (x->kind == Value::MAP && !x->map.empty());
    };
    if (v->kind == Value::MAP && !v->map.empty()) {
        for (auto& kv : v->map) {
            std::string k;
            json_quote(k, kv.first);
            o += pad + k + ":";
            if (composite(kv.second)) {
                o += "\n";
                yaml_emit(o, kv.second, ind + 2);
            } else {
                o += " " + scalar(kv.second) + "\n";
            }
        }
    } else if (v->kind == Value::LIST && !v->list.empty()) {
        for (auto& it : v->list) {
            o += pad + "-";
            if (composite(it)) {
                o += "\n";
                yaml_emit(o, it, ind + 2);
            } else {
                o += " " + scalar(it) + "\n";
            }
        }
    } else {
        o += pad + scalar(v) + "\n";
    }
}
std::string yaml_marshal(const VPtr& v, int indent) {
    std::string data;
    yaml_emit(data, v, 0);
    if (indent > 0) {  // strings.ReplaceAll("\n"+data, "\n", "\n"+pad)
        const std::string pad((size_t)indent * 2, ' ');
        std::string r;
        const std::string src = "\n" + data;
        for (char c : src) {
            r.push_back(c);
            if (c == '\n') r += pad;
        }
        data = r;
    }
    return data;
}

// ---------------------------------------------------------------------------
// YAML parse (block + flow subset) -> Value
// ---------------------------------------------------------------------------
struct Line {
    int indent;
    std::string s;  // content without indentation / comment / trailing space
};

// strip a comment (# after whitespace, outside quotes) and trailing space
std::string strip_comment(const std::string& s) {
    bool sq = false, dq = false;
    for (size_t i = 0; i < s.size(); i++) {
        const char c = s[i];
        if (dq) {
            if (c == '\\') i++;
            else if (c == '"') dq = false;
        } else if (sq) {
            if (c == '\'') sq = false;
        } else if (c == '"' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '[' || s[i - 1] == '{' || s[i - 1] == ',' ||
                                s[i - 1] == '-' || s[i - 1] == ':')) {
            dq = true;
        } else if (c == '\'' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '[' || s[i - 1] == '{' || s[i - 1] == ',')) {
            sq = true;
        } else if (c == '#' && (i == 0 || s[i - 1] == ' ' || s[i - 1] == '\t')) {
            std::string r = s.substr(0, i);
            while (!r.empty() && (r.back() == ' ' || r.back() == '\t')) r.pop_back();
            return r;
        }
    }
    std::string r = s;
    while (!r.empty() && (r.back() == ' ' || r.back() == '\t' || r.back() == '\r')) r.pop_back();
    return r;
}

VPtr plain_scalar(const std::string& s) {
    if (s.empty() || s == "~" || s == "null" || s == "Null" || s == "NULL") return make_null();
    static const char* t[] = {"y", "Y", "yes", "Yes", "YES", "true", "True", "TRUE", "on", "On", "ON"};
    static const char* f[] = {"n", "N", "no", "No", "NO", "false", "False", "FALSE", "off", "Off", "OFF"};
    for (const char* w : t)
        if (s == w) return make_bool(true);
    for (const char* w : f)
        if (s == w) return make_bool(false);
    // numbers (yaml.v2 resolve.go: strconv.ParseInt / ParseUint with base 0 on the
    // text without '_', then yamlStyleFloat): canonical decimal ints become
    // numbers; every other number form is refused rather than re-printed
    {
        const size_t i = (s[0] == '-' || s[0] == '+') ? 1 : 0;
        std::string p;
        for (size_t k = i; k < s.size(); k++)
            if (s[k] != '_') p.push_back(s[k]);
        auto all = [&](size_t from, const char* set) {
            if (from >= p.size()) return false;
            for (size_t k = from; k < p.size(); k++)
                if (!strchr(set, p[k])) return false;
            return true;
        };
        const bool prefixed = p.size() > 2 && p[0] == '0' &&
                              (((p[1] == 'x' || p[1] == 'X') && all(2, "0123456789abcdefABCDEF")) ||
                               ((p[1] == 'o' || p[1] == 'O') && all(2, "01234567")) ||
                               ((p[1] == 'b' || p[1] == 'B') && all(2, "01")));
        const bool decimal = all(0, "0123456789");
        bool fl = false;  // [0-9]+(\.[0-9]*)?([eE][-+]?[0-9]+)? or \.[0-9]+(...)
        {
            size_t k = 0, n = p.size(), d0;
            d0 = k;
            while (k < n && isdigit((unsigned char)p[k])) k++;
            bool mant = k > d0;
            if (k < n && p[k] == '.') {
                k++;
                const size_t d1 = k;
                while (k < n && isdigit((unsigned char)p[k])) k++;
                mant = mant || k > d1;
            }
            if (mant && k < n && (p[k] == 'e' || p[k] == 'E')) {
                k++;
                if (k < n && (p[k] == '+' || p[k] == '-')) k++;
                const size_t d2 = k;
                while (k < n && isdigit((unsigned char)p[k])) k++;
                if (k == d2) mant = false;
            }
            fl = mant && k == n;
        }
        if (decimal && s.find('_') == std::string::npos && s[0] != '+' && (p.size() == 1 || p[0] != '0')) {
            if (p.size() > 18) fail("integer " + s + " out of the covered range");
            return make_num(s);
        }
        if (decimal || prefixed || fl) fail("number form '" + s + "' is outside the covered YAML subset");
    }
    if (s == ".inf" || s == ".Inf" || s == ".INF" || s == "-.inf" || s == ".nan" || s == ".NaN" || s == ".NAN")
        fail("float " + s + " is outside the covered YAML subset");
    if (s[0] == '&' || s[0] == '*' || s[0] == '!' || s[0] == '|' || s[0] == '>' || s[0] == '%' || s[0] == '@' ||
        s[0] == '`')
        fail("YAML indicator '" + s.substr(0, 1) + "' is outside the covered subset");
    return make_str(s);
}

std::string dq_unescape(const std::string& s, size_t& i) {  // s[i] == '"'
    std::string o;
    for (i++; i < s.size() && s[i] != '"'; i++) {
        if (s[i] != '\\') {
            o.push_back(s[i]);
            continue;
        }
        if (++i >= s.size()) break;
        const char e = s[i];
        switch (e) {
            case 'n': o.push_back('\n'); break;
            case 't': o.push_back('\t'); break;
            case 'r': o.push_back('\r'); break;
            case '0': o.push_back('\0'); break;
            case '"': o.push_back('"'); break;
            case '/': o.push_back('/'); break;
            case '\\': o.push_back('\\'); break;
            case 'u': {
                if (i + 4 >= s.size()) fail("bad \\u escape");
                const unsigned cp = (unsigned)strtoul(s.substr(i + 1, 4).c_str(), nullptr, 16);
                i += 4;
                if (cp < 0x80) o.push_back((char)cp);
                else if (cp < 0x800) o.push_back((char)(0xC0 | (cp >> 6))), o.push_back((char)(0x80 | (cp & 63)));
                else {
                    if (cp >= 0xD800 && cp < 0xE000) fail("surrogate escapes are outside the subset");
                    o.push_back((char)(0xE0 | (cp >> 12)));
                    o.push_back((char)(0x80 | ((cp >> 6) & 63)));
                    o.push_back((char)(0x80 | (cp & 63)));
                }
                break;
            }
            default: fail(std::string("escape \\") + e + " is outside the covered subset");
        }
    }
    if (i >= s.size()) fail("unterminated double-quoted scalar");
    i++;
    return o;
}
std::string sq_unescape(const std::string& s, size_t& i) {  // s[i] == '\''
    std::string o;
    for (i++; i < s.size(); i++) {
        if (s[i] == '\'') {
            if (i + 1 < s.size() && s[i + 1] == '\'') {
                o.push_back('\'');
                i++;
            } else {
                i++;
                return o;
            }
        } else {
            o.push_back(s[i]);
        }
    }
    fail("unterminated single-quoted scalar");
}

// flow collection / scalar inside flow context, from s[i]
VPtr flow(const std::string& s, size_t& i, int depth = 0);
void skip_ws(const std::string& s, size_t& i) {
    while (i < s.size() && (s[i] == ' ' || s[i] == '\t')) i++;
}
VPtr flow_scalar(const std::string& s, size_t& i, bool key) {
    skip_ws(s, i);
    if (i < s.size() && s[i] == '"') return make_str(dq_unescape(s, i));
    if (i < s.size() && s[i] == '\'') return make_str(sq_unescape(s, i));
    size_t j = i;
    while (j < s.size() && s[j] != ',' && s[j] != ']' && s[j] != '}' && !(key && s[j] == ':')) j++;
    std::string t = s.substr(i, j - i);
    while (!t.empty() && t.back() == ' ') t.pop_back();
    i = j;
    return plain_scalar(t);
}
VPtr flow(const std::string& s, size_t& i, int depth) {
    if (depth > 64) fail("flow collection nested deeper than the covered subset");
    skip_ws(s, i);
    if (i >= s.size()) fail("truncated flow collection");
    if (s[i] == '[') {
        std::vector<VPtr> items;
        i++;
        skip_ws(s, i);
        if (i < s.size() && s[i] == ']') {
            i++;
            return make_list(items);
        }
        while (true) {
            items.push_back(flow(s, i, depth + 1));
            skip_ws(s, i);
            if (i < s.size() && s[i] == ',') {
                i++;
                continue;
            }
            if (i < s.size() && s[i] == ']') {
                i++;
                return make_list(items);
            }
            fail("bad flow sequence");
        }
    }
    if (s[i] == '{') {
        std::vector<std::pair<std::string, VPtr>> kv;
        i++;
        skip_ws(s, i);
        if (i < s.size() && s[i] == '}') {
            i++;
            return make_map(kv);
        }
        while (true) {
            VPtr k = flow_scalar(s, i, true);
            if (k->kind != Value::STR) fail("non-string mapping key");
            skip_ws(s, i);
            if (i >= s.size() || s[i] != ':') fail("bad flow mapping");
            i++;
            kv.push_back({k->s, flow(s, i, depth + 1)});
            skip_ws(s, i);
            if (i < s.size() && s[i] == ',') {
                i++;
                continue;
            }
            if (i < s.size() && s[i] == '}') {
                i++;
                break;
            }
            fail("bad flow mapping");
        }
        std::vector<std::string> keys;
        for (auto& p : kv) keys.push_back(p.first);
        std::sort(keys.begin(), keys.end());
        if (std::adjacent_find(keys.begin(), keys.end()) != keys.end()) fail("duplicate mapping key");
        return make_map(kv);
    }
    return flow_scalar(s, i, false);
}

// value text after "key:" or "- " on one line
VPtr inline_value(const std::string& t) {
    if (t.empty()) return make_null();
    size_t i = 0;
    VPtr v;
    if (t[0] == '[' || t[0] == '{') v = flow(t, i);
    else if (t[0] == '"') v = make_str(dq_unescape(t, i));
    else if (t[0] == '\'') v = make_str(sq_unescape(t, i));
    else return plain_scalar(t);
    skip_ws(t, i);
    if (i != t.size()) fail("trailing text after a YAML value: " + t);
    return v;
}

// position of the mapping indicator (": " or ':' at the end) outside quotes, or npos
size_t key_colon(const std::string& s) {
    size_t i = 0;
    if (s.empty()) return std::string::npos;
    if (s[0] == '"' || s[0] == '\'') {
        try {
            if (s[0] == '"') dq_unescape(s, i);
            else sq_unescape(s, i);
        } catch (const Fail&) {
            return std::string::npos;
        }
        skip_ws(s, i);
        return (i < s.size() && s[i] == ':' && (i + 1 == s.size() || s[i + 1] == ' ')) ? i : std::string::npos;
    }
    if (s[0] == '[' || s[0] == '{') return std::string::npos;
    for (; i < s.size(); i++)
        if (s[i] == ':' && (i + 1 == s.size() || s[i + 1] == ' ')) return i;
    return std::string::npos;
}

constexpr int MAX_DEPTH = 64;  // nesting of YAML / JSON collections and template blocks

struct YamlParser {
    std::vector<Line> lines;
    size_t at = 0;
    int depth = 0;

    VPtr node(int min_indent) {
        if (at >= lines.size() || lines[at].indent < min_indent) return make_null();
        if (++depth > MAX_DEPTH) fail("YAML nested deeper than the covered subset");
        struct Up {
            int& d;
            ~Up() { d--; }
        } up{depth};
        const Line& l = lines[at];
        if (l.s == "-" || l.s.compare(0, 2, "- ") == 0) return seq(l.indent);
        if (key_colon(l.s) != std::string::npos) return mapping(l.indent);
        at++;
        VPtr v = inline_value(l.s);
        if (at < lines.size() && lines[at].indent > l.indent) fail("multi-line scalars are outside the covered subset");
        return v;
    }
    VPtr seq(int ind) {
        std::vector<VPtr> items;
        while (at < lines.size() && lines[at].indent == ind && (lines[at].s == "-" || lines[at].s.compare(0, 2, "- ") == 0)) {
            Line& l = lines[at];
            if (l.s == "-") {
                at++;
                items.push_back(node(ind + 1));
                continue;
            }
            // "- x": the item's content as a line at the column of x
            size_t k = 1;
            while (k < l.s.size() && l.s[k] == ' ') k++;
            l.indent += (int)k;
            l.s = l.s.substr(k);
            items.push_back(node(l.indent));
        }
        if (at < lines.size() && lines[at].indent > ind) fail("bad YAML indentation");
        return make_list(items);
    }
    VPtr mapping(int ind) {
        std::vector<std::pair<std::string, VPtr>> kv;
        while (at < lines.size() && lines[at].indent == ind) {
            const Line l = lines[at];
            const size_t c = key_colon(l.s);
            if (c == std::string::npos) fail("expected a mapping key: " + l.s);
            std::string ks = l.s.substr(0, c);
            while (!ks.empty() && ks.back() == ' ') ks.pop_back();
            std::string key;
            if (!ks.empty() && (ks[0] == '"' || ks[0] == '\'')) {
                size_t i = 0;
                key = ks[0] == '"' ? dq_unescape(ks, i) : sq_unescape(ks, i);
            } else {
                VPtr kv2 = plain_scalar(ks);
                if (kv2->kind != Value::STR) fail("non-string mapping key '" + ks + "' is outside the covered subset");
                key = ks;
            }
            std::string rest = c + 1 < l.s.size() ? l.s.substr(c + 1) : "";
            size_t r = 0;
            while (r < rest.size() && rest[r] == ' ') r++;
            rest = rest.substr(r);
            at++;
            VPtr v;
            if (!rest.empty()) {
                v = inline_value(rest);
                if (at < lines.size() && lines[at].indent > ind) fail("multi-line scalars are outside the covered subset");
            } else if (at < lines.size() && lines[at].indent > ind) {
                v = node(ind + 1);
            } else if (at < lines.size() && lines[at].indent == ind &&
                       (lines[at].s == "-" || lines[at].s.compare(0, 2, "- ") == 0)) {
                v = seq(ind);  // a sequence may sit at its key's indentation
            } else {
                v = make_null();
            }
            for (auto& p : kv)
                if (p.first == key) fail("duplicate mapping key " + key);
            kv.push_back({key, v});
        }
        if (at < lines.size() && lines[at].indent > ind) fail("bad YAML indentation");
        return make_map(kv);
    }
};

void json_emit(std::string& o, const VPtr& v) {
    switch (v->kind) {
        case Value::NOVAL:
        case Value::NUL: o += "null"; break;
        case Value::BOOL: o += v->b ? "true" : "false"; break;
        case Value::NUM: o += v->s; break;
        case Value::STR: json_quote(o, v->s); break;
        case Value::LIST:
            o.push_back('[');
            for (size_t i = 0; i < v->list.size(); i++) {
                if (i) o.push_back(',');
                json_emit(o, v->list[i]);
            }
            o.push_back(']');
            break;
        case Value::MAP:
            o.push_back('{');
            for (size_t i = 0; i < v->map.size(); i++) {
                if (i) o.push_back(',');
                json_quote(o, v->map[i].first);
                o.push_back(':');
                json_emit(o, v->map[i].second);
            }
            o.push_back('}');
            break;
    }
}

// ---------------------------------------------------------------------------
// JSON parse (the documents of kwok_template_render)
// ---------------------------------------------------------------------------
struct JsonParser {
    const std::string& s;
    size_t i = 0;
    int depth = 0;
    void ws() {
        while (i < s.size() && isspace((unsigned char)s[i])) i++;
    }
    VPtr value() {
        ws();
        if (i >= s.size()) fail("truncated JSON");
        if (++depth > 64) fail("JSON nested deeper than the covered subset");
        struct Up {
            int& d;
            ~Up() { d--; }
        } up{depth};
        const char c = s[i];
        if (c == '{') {
            std::vector<std::pair<std::string, VPtr>> kv;
            i++;
            ws();
            if (i < s.size() && s[i] == '}') {
                i++;
                return make_map(kv);
            }
            while (true) {
                ws();
                if (i >= s.size() || s[i] != '"') fail("JSON key");
                std::string k = dq_unescape(s, i);
                ws();
                if (i >= s.size() || s[i] != ':') fail("JSON ':'");
                i++;
                kv.push_back({k, value()});
                ws();
                if (i < s.size() && s[i] == ',') {
                    i++;
                    continue;
                }
                if (i < s.size() && s[i] == '}') {
                    i++;
                    return make_map(kv);
                }
                fail("JSON object");
            }
        }
        if (c == '[') {
            std::vector<VPtr> items;
            i++;
            ws();
            if (i < s.size() && s[i] == ']') {
                i++;
                return make_list(items);
            }
            while (true) {
                items.push_back(value());
                ws();
                if (i < s.size() && s[i] == ',') {
                    i++;
                    continue;
                }
                if (i < s.size() && s[i] == ']') {
                    i++;
                    return make_list(items);
                }
                fail("JSON array");
            }
        }
        if (c == '"') return make_str(dq_unescape(s, i));
        if (s.compare(i, 4, "true") == 0) return i += 4, make_bool(true);
        if (s.compare(i, 5, "false") == 0) return i += 5, make_bool(false);
        if (s.compare(i, 4, "null") == 0) return i += 4, make_null();
        size_t j = i;
        while (j < s.size() && strchr("0123456789+-.eE", s[j])) j++;
        if (j == i) fail("JSON value");
        std::string num = s.substr(i, j - i);
        i = j;
        return make_num(num);  // decoder.UseNumber(): json.Number text
    }
};
}  // namespace

bool parse_json(const std::string& s, VPtr& out, std::string& err) {
    try {
        JsonParser p{s};
        out = p.value();
        p.ws();
        if (p.i != s.size()) fail("trailing JSON");
        return true;
    } catch (const Fail& f) {
        err = f.msg;
        return false;
    }
}

namespace {
VPtr yaml_tree(const std::string& yaml) {
    {
        YamlParser p;
        size_t pos = 0;
        bool started = false;
        while (pos <= yaml.size()) {
            size_t e = yaml.find('\n', pos);
            if (e == std::string::npos) e = yaml.size();
            std::string raw = yaml.substr(pos, e - pos);
            pos = e + 1;
            if (raw.find('\t') != std::string::npos && raw.find_first_not_of(" \t") != std::string::npos &&
                raw.find_first_not_of(' ') < raw.size() && raw[raw.find_first_not_of(' ')] == '\t')
                fail("tab indentation");
            int ind = 0;
            while (ind < (int)raw.size() && raw[(size_t)ind] == ' ') ind++;
            std::string s = strip_comment(raw.substr((size_t)ind));
            if (s.empty()) continue;
            if (!started && (s == "---" || s.compare(0, 4, "--- ") == 0)) {
                started = true;
                continue;
            }
            if (s == "---" || s == "...") break;  // only the first document
            started = true;
            p.lines.push_back({ind, s});
        }
        VPtr v = p.lines.empty() ? make_null() : p.node(p.lines[0].indent);
        if (p.at != p.lines.size()) fail("unparsed YAML from: " + p.lines[p.at].s);
        return v;
    }
}
}  // namespace

std::string to_json(const VPtr& v) {
    std::string o;
    json_emit(o, v);
    return o;
}

bool yaml_to_json(const std::string& yaml, std::string& out, std::string& err) {
    try {
        out = to_json(yaml_tree(yaml));
        return true;
    } catch (const Fail& f) {
        err = f.msg;
        return false;
    }
}

bool execute_template(const std::string& tpl, const VPtr& doc, const Env& env, std::string& text, std::string& err) {
    try {
        size_t a = 0, b = tpl.size();  // strings.TrimSpace
        while (a < b && isspace((unsigned char)tpl[a])) a++;
        while (b > a && isspace((unsigned char)tpl[b - 1])) b--;
        std::vector<Node> nodes = parse_template(tpl.substr(a, b - a));
        Exec x{env, {}, {}};
        x.vars.push_back({"$", doc});
        x.run(nodes, doc);
        text = std::move(x.out);
        return true;
    } catch (const Fail& f) {
        err = f.msg;
        return false;
    }
}

bool render_to_tree(const std::string& tpl, const VPtr& doc, const Env& env, VPtr& out, std::string& err) {
    try {
        size_t a = 0, b = tpl.size();  // strings.TrimSpace
        while (a < b && isspace((unsigned char)tpl[a])) a++;
        while (b > a && isspace((unsigned char)tpl[b - 1])) b--;
        std::vector<Node> nodes = parse_template(tpl.substr(a, b - a));
        Exec x{env, {}, {}};
        x.vars.push_back({"$", doc});
        x.run(nodes, doc);
        out = yaml_tree(x.out);
        return true;
    } catch (const Fail& f) {
        err = f.msg;
        return false;
    }
}

bool render_to_json(const std::string& tpl, const VPtr& doc, const Env& env, std::string& out, std::string& err) {
    VPtr t;
    if (!render_to_tree(tpl, doc, env, t, err)) return false;
    out = to_json(t);
    return true;
}

}  // namespace gotpl
}  // namespace kwok
