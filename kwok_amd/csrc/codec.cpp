// codec.cpp - watch-event ingest codec: Kubernetes Node / Pod JSON -> the
// kwok_node_event / kwok_pod_event records the tick engine ingests
// (the step before the hot path).
//
// It computes, on the host, the per-object facts the reference derives while
// routing watch events and rendering templates:
//   managed     nodeSelectorFunc        controller.go:81-98 (all / annotation selector /
//                                       label selector evaluated as the list/watch filter)
//   lockable    needLockNode            node_controller.go:210-223
//   DISREGARD   needLockPod selectors   pod_controller.go:252-269 (the nodeHas part is the
//                                       engine's node lookup)
//   DELETING    deletionTimestamp != nil pod_controller.go:306
//   HAS_FINALIZERS len(finalizers) != 0 pod_controller.go:161
//   STATUS_NONEMPTY `{{ with .status }}` pod.status.tpl:44 over json(corev1.PodStatus)
//   CONFORMS    computePatchData's SMP no-op test for conditions / containerStatuses /
//               initContainerStatuses / startTime (pod_controller.go:404-439)
//   addresses / allocatable / capacity: canonical compact JSON (sorted keys, Go escaping)
//               as `YAML . 1` + YAMLToJSON echo them into the init patch (node.status.tpl)
// Label selectors follow k8s.io/apimachinery labels.Parse's equality and set grammar
// (`k`, `!k`, `k=v`, `k==v`, `k!=v`, `k in (a,b)`, `k notin (a,b)`, comma = AND);
// `k>n` / `k<n` are rejected with KWOK_EINVAL.
//
// Strings referenced by the records point into the caller's arena (the document
// itself); a referenced string holding a JSON escape is outside the safe-string
// domain and the record is rejected (KWOK_EDOMAIN).  Canonical JSON for the
// three node blobs is written in place over the value's own span (it is never
// longer for the accepted domain), so the arena must be writable.
#include <algorithm>
#include <cstring>
#include <deque>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "../../include/kwok_engine.h"
#include "codec.h"
#include "templates.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

// ---------------------------------------------------------------- JSON DOM
struct JV {
    enum T { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
    bool b = false;
    bool escaped = false;   // STR: the source held an escape (span is not the value)
    std::string_view s;     // STR value / NUM text (a view of the source, or of the Doc's store)
    uint32_t off = 0, len = 0;  // source span of the value (STR: inside the quotes)
    std::vector<JV> a;
    std::vector<std::pair<std::string_view, JV>> o;

    const JV* get(std::string_view k) const {
        if (t != OBJ) return nullptr;
        for (auto& kv : o)
            if (kv.first == k) return &kv.second;
        return nullptr;
    }
    bool is_null() const { return t == NUL; }
};

struct Parser {
    const char* p;
    size_t n, i = 0;
    size_t base;
    std::deque<std::string>* store;  // decoded text of escaped strings (stable addresses)
    Parser(const char* arena, size_t off, size_t len, std::deque<std::string>* st)
        : p(arena + off), n(len), base(off), store(st) {}

    void ws() {
        while (i < n && (p[i] == ' ' || p[i] == '\t' || p[i] == '\n' || p[i] == '\r')) i++;
    }
    bool lit(const char* w) {
        size_t m = strlen(w);
        if (i + m > n || memcmp(p + i, w, m)) return false;
        i += m;
        return true;
    }
    static void put_utf8(std::string& s, uint32_t c) {
        if (c < 0x80) s += (char)c;
        else if (c < 0x800) { s += (char)(0xC0 | (c >> 6)); s += (char)(0x80 | (c & 63)); }
        else if (c < 0x10000) { s += (char)(0xE0 | (c >> 12)); s += (char)(0x80 | ((c >> 6) & 63)); s += (char)(0x80 | (c & 63)); }
        else { s += (char)(0xF0 | (c >> 18)); s += (char)(0x80 | ((c >> 12) & 63)); s += (char)(0x80 | ((c >> 6) & 63)); s += (char)(0x80 | (c & 63)); }
    }
    bool hex4(uint32_t* v) {
        if (i + 4 > n) return false;
        uint32_t x = 0;
        for (int k = 0; k < 4; k++) {
            char c = p[i++];
            x <<= 4;
            if (c >= '0' && c <= '9') x |= c - '0';
            else if (c >= 'a' && c <= 'f') x |= c - 'a' + 10;
            else if (c >= 'A' && c <= 'F') x |= c - 'A' + 10;
            else return false;
        }
        *v = x;
        return true;
    }
    bool str(JV& v) {
        if (i >= n || p[i] != '"') return false;
        i++;
        v.t = JV::STR;
        v.off = (uint32_t)(base + i);
        size_t start = i;
        std::string* buf = nullptr;
        while (i < n && p[i] != '"') {
            unsigned char c = (unsigned char)p[i];
            if (c < 0x20) return false;
            if (c != '\\') {
                if (buf) *buf += (char)c;
                i++;
                continue;
            }
            if (!buf) {
                store->emplace_back(p + start, i - start);
                buf = &store->back();
                v.escaped = true;
            }
            if (++i >= n) return false;
            char e = p[i++];
            switch (e) {
                case '"': *buf += '"'; break;
                case '\\': *buf += '\\'; break;
                case '/': *buf += '/'; break;
                case 'b': *buf += '\b'; break;
                case 'f': *buf += '\f'; break;
                case 'n': *buf += '\n'; break;
                case 'r': *buf += '\r'; break;
                case 't': *buf += '\t'; break;
                case 'u': {
                    uint32_t c1;
                    if (!hex4(&c1)) return false;
                    if (c1 >= 0xD800 && c1 < 0xDC00 && i + 6 <= n && p[i] == '\\' && p[i + 1] == 'u') {
                        i += 2;
                        uint32_t c2;
                        if (!hex4(&c2) || c2 < 0xDC00 || c2 >= 0xE000) return false;
                        c1 = 0x10000 + ((c1 - 0xD800) << 10) + (c2 - 0xDC00);
                    }
                    put_utf8(*buf, c1);
                    break;
                }
                default: return false;
            }
        }
        if (i >= n) return false;
        v.len = (uint32_t)(i - start);
        v.s = buf ? std::string_view(*buf) : std::string_view(p + start, i - start);
        i++;
        return true;
    }
    bool num(JV& v) {
        size_t s = i;
        if (i < n && p[i] == '-') i++;
        while (i < n && ((p[i] >= '0' && p[i] <= '9') || p[i] == '.' || p[i] == 'e' || p[i] == 'E' || p[i] == '+' ||
                         p[i] == '-'))
            i++;
        if (i == s) return false;
        v.t = JV::NUM;
        v.s = std::string_view(p + s, i - s);
        return true;
    }
    bool value(JV& v, int depth) {
        if (depth > 64) return false;
        ws();
        if (i >= n) return false;
        size_t s = i;
        bool ok;
        char c = p[i];
        if (c == '{') {
            v.t = JV::OBJ;
            i++;
            ws();
            v.o.reserve(8);
            if (i < n && p[i] == '}') { i++; ok = true; }
            else {
                ok = false;
                for (;;) {
                    ws();
                    JV k;
                    if (!str(k)) break;
                    ws();
                    if (i >= n || p[i] != ':') break;
                    i++;
                    v.o.emplace_back(k.s, JV());
                    if (!value(v.o.back().second, depth + 1)) break;
                    ws();
                    if (i < n && p[i] == ',') { i++; continue; }
                    if (i < n && p[i] == '}') { i++; ok = true; }
                    break;
                }
            }
        } else if (c == '[') {
            v.t = JV::ARR;
            i++;
            ws();
            if (i < n && p[i] == ']') { i++; ok = true; }
            else {
                ok = false;
                for (;;) {
                    v.a.emplace_back();
                    if (!value(v.a.back(), depth + 1)) break;
                    ws();
                    if (i < n && p[i] == ',') { i++; continue; }
                    if (i < n && p[i] == ']') { i++; ok = true; }
                    break;
                }
            }
        } else if (c == '"') {
            return str(v);
        } else if (c == 't') { v.t = JV::BOOL; v.b = true; ok = lit("true"); }
        else if (c == 'f') { v.t = JV::BOOL; ok = lit("false"); }
        else if (c == 'n') { v.t = JV::NUL; ok = lit("null"); }
        else ok = num(v);
        if (ok && v.t != JV::STR) { v.off = (uint32_t)(base + s); v.len = (uint32_t)(i - s); }
        return ok;
    }
    bool document(JV& v) {
        if (!value(v, 0)) return false;
        ws();
        return i == n;
    }
};

// Go encoding/json string escaping (HTML-safe, as json.Marshal does)
bool go_string(std::string& out, std::string_view s) {
    static const char* hx = "0123456789abcdef";
    out += '"';
    for (size_t k = 0; k < s.size(); k++) {
        unsigned char c = (unsigned char)s[k];
        if (c == '"' || c == '\\') { out += '\\'; out += (char)c; }
        else if (c == '\n') out += "\\n";
        else if (c == '\r') out += "\\r";
        else if (c == '\t') out += "\\t";
        else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
            out += "\\u00";
            out += hx[c >> 4];
            out += hx[c & 15];
        } else if (c == 0xE2 && k + 2 < s.size() && (unsigned char)s[k + 1] == 0x80 &&
                   ((unsigned char)s[k + 2] == 0xA8 || (unsigned char)s[k + 2] == 0xA9)) {
            out += (unsigned char)s[k + 2] == 0xA8 ? "\\u2028" : "\\u2029";
            k += 2;
        } else out += (char)c;
    }
    out += '"';
    return true;
}

bool plain_int(std::string_view t) {
    size_t k = t[0] == '-' ? 1 : 0;
    if (k >= t.size()) return false;
    if (t[k] == '0' && t.size() > k + 1) return false;
    for (; k < t.size(); k++)
        if (t[k] < '0' || t[k] > '9') return false;
    return true;
}

// canonical compact JSON (json.Marshal of the yaml round-tripped value:
// map keys sorted bytewise).  Non-integer numbers are outside the domain
// (yaml.v2 re-formats floats).
bool canon(std::string& out, const JV& v) {
    switch (v.t) {
        case JV::NUL: out += "null"; return true;
        case JV::BOOL: out += v.b ? "true" : "false"; return true;
        case JV::NUM:
            if (!plain_int(v.s)) return false;
            out += v.s;
            return true;
        case JV::STR: return go_string(out, v.s);
        case JV::ARR:
            out += '[';
            for (size_t k = 0; k < v.a.size(); k++) {
                if (k) out += ',';
                if (!canon(out, v.a[k])) return false;
            }
            out += ']';
            return true;
        case JV::OBJ: {
            std::vector<const std::pair<std::string_view, JV>*> kv;
            for (auto& e : v.o) kv.push_back(&e);
            std::stable_sort(kv.begin(), kv.end(), [](auto* x, auto* y) { return x->first < y->first; });
            for (size_t k = 1; k < kv.size(); k++)
                if (kv[k]->first == kv[k - 1]->first) return false;  // duplicate key
            out += '{';
            for (size_t k = 0; k < kv.size(); k++) {
                if (k) out += ',';
                go_string(out, kv[k]->first);
                out += ':';
                if (!canon(out, kv[k]->second)) return false;
            }
            out += '}';
            return true;
        }
    }
    return false;
}

// "zero value" in the omitempty sense: what a typed round trip drops
bool zeroish(const JV& v) {
    switch (v.t) {
        case JV::NUL: return true;
        case JV::BOOL: return !v.b;
        case JV::NUM: return v.s == "0";
        case JV::STR: return v.s.empty();
        case JV::ARR: return v.a.empty();
        case JV::OBJ:
            for (auto& kv : v.o)
                if (!zeroish(kv.second)) return false;
            return true;
    }
    return true;
}

// Deep equality after dropping zero-valued map entries on both sides (the
// corev1 struct round trip computePatchData does, pod_controller.go:420-433).
bool norm_equal(const JV& x, const JV& y) {
    if (zeroish(x) && zeroish(y)) return true;
    if (x.t != y.t) return false;
    switch (x.t) {
        case JV::NUL: return true;
        case JV::BOOL: return x.b == y.b;
        case JV::NUM: return x.s == y.s;
        case JV::STR: return x.s == y.s;
        case JV::ARR:
            if (x.a.size() != y.a.size()) return false;
            for (size_t k = 0; k < x.a.size(); k++)
                if (!norm_equal(x.a[k], y.a[k])) return false;
            return true;
        case JV::OBJ: {
            for (auto& kv : x.o) {
                const JV* o = y.get(kv.first);
                if (o ? !norm_equal(kv.second, *o) : !zeroish(kv.second)) return false;
            }
            for (auto& kv : y.o)
                if (!x.get(kv.first) && !zeroish(kv.second)) return false;
            return true;
        }
    }
    return false;
}

JV jstr(std::string_view s) { JV v; v.t = JV::STR; v.s = s; return v; }
JV jbool(bool b) { JV v; v.t = JV::BOOL; v.b = b; return v; }
JV jnum(const char* s) { JV v; v.t = JV::NUM; v.s = s; return v; }
JV jobj(std::vector<std::pair<std::string_view, JV>> o) { JV v; v.t = JV::OBJ; v.o = std::move(o); return v; }

// ---------------------------------------------------------------- selectors
// labels.Set as decoded from the object: (key, value) views into the document
using SMap = std::vector<std::pair<std::string_view, std::string_view>>;

struct Req {
    enum Op { IN, NOTIN, EXISTS, NOTEXISTS } op;
    std::string key;
    std::vector<std::string> vals;
};

struct Selector {
    bool set = false;  // false = nil selector (never matches / not configured)
    std::vector<Req> reqs;  // empty + set = labels.Everything()

    bool matches(const SMap& m) const {
        for (auto& r : reqs) {
            const std::string_view* val = nullptr;
            for (auto& kv : m)
                if (kv.first == r.key) val = &kv.second;  // last duplicate wins, as a Go map decode
            bool has = val != nullptr;
            bool in = has && std::find(r.vals.begin(), r.vals.end(), *val) != r.vals.end();
            switch (r.op) {
                case Req::IN: if (!in) return false; break;
                case Req::NOTIN: if (in) return false; break;
                case Req::EXISTS: if (!has) return false; break;
                case Req::NOTEXISTS: if (has) return false; break;
            }
        }
        return true;
    }
};

std::string trim(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && (s[a] == ' ' || s[a] == '\t')) a++;
    while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t')) b--;
    return s.substr(a, b - a);
}

bool name_ok(const std::string& s, bool allow_empty) {
    if (s.empty()) return allow_empty;
    for (char c : s)
        if (!((c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '-' || c == '_' ||
              c == '.' || c == '/'))
            return false;
    return true;
}

// labels.Parse (k8s.io/apimachinery v0.26 pkg/labels/selector.go), equality- and set-based terms
int parse_selector(const char* text, Selector* out) {
    out->set = false;
    out->reqs.clear();
    if (!text) return KWOK_OK;
    std::string s(text);
    if (trim(s).empty() && s.empty()) return KWOK_OK;  // "" -> nil (labelsParse, utils.go:205-210)
    out->set = true;
    std::vector<std::string> terms;
    int depth = 0;
    std::string cur;
    for (char c : s) {
        if (c == '(') depth++;
        if (c == ')') depth--;
        if (c == ',' && depth == 0) { terms.push_back(cur); cur.clear(); }
        else cur += c;
    }
    terms.push_back(cur);
    if (terms.size() == 1 && trim(terms[0]).empty()) return KWOK_OK;  // Everything
    for (auto& t0 : terms) {
        std::string t = trim(t0);
        Req r;
        if (t.empty()) return fail(KWOK_EINVAL, "selector: empty term in '" + s + "'");
        size_t sp = t.find(' ');
        size_t paren = t.find('(');
        if (t[0] == '!') {
            r.op = Req::NOTEXISTS;
            r.key = trim(t.substr(1));
        } else if (paren != std::string::npos && sp != std::string::npos && sp < paren) {
            r.key = t.substr(0, sp);
            std::string rest = trim(t.substr(sp));
            if (rest.compare(0, 2, "in") == 0 && (rest.size() > 2 && (rest[2] == ' ' || rest[2] == '('))) {
                r.op = Req::IN;
                rest = trim(rest.substr(2));
            } else if (rest.compare(0, 5, "notin") == 0 && rest.size() > 5 && (rest[5] == ' ' || rest[5] == '(')) {
                r.op = Req::NOTIN;
                rest = trim(rest.substr(5));
            } else return fail(KWOK_EINVAL, "selector: unknown set operator in '" + t + "'");
            if (rest.size() < 2 || rest.front() != '(' || rest.back() != ')')
                return fail(KWOK_EINVAL, "selector: bad value set in '" + t + "'");
            std::string body = rest.substr(1, rest.size() - 2), v;
            for (size_t k = 0; k <= body.size(); k++) {
                if (k == body.size() || body[k] == ',') {
                    std::string tv = trim(v);
                    if (!name_ok(tv, true)) return fail(KWOK_EINVAL, "selector: bad value in '" + t + "'");
                    r.vals.push_back(tv);
                    v.clear();
                } else v += body[k];
            }
        } else if (t.find('>') != std::string::npos || t.find('<') != std::string::npos) {
            return fail(KWOK_EINVAL, "selector: gt/lt terms are not supported: '" + t + "'");
        } else {
            size_t ne = t.find("!="), eq2 = t.find("=="), eq = t.find('=');
            if (ne != std::string::npos) {
                r.op = Req::NOTIN;
                r.key = trim(t.substr(0, ne));
                r.vals.push_back(trim(t.substr(ne + 2)));
            } else if (eq2 != std::string::npos) {
                r.op = Req::IN;
                r.key = trim(t.substr(0, eq2));
                r.vals.push_back(trim(t.substr(eq2 + 2)));
            } else if (eq != std::string::npos) {
                r.op = Req::IN;
                r.key = trim(t.substr(0, eq));
                r.vals.push_back(trim(t.substr(eq + 1)));
            } else {
                r.op = Req::EXISTS;
                r.key = t;
            }
            for (auto& v : r.vals)
                if (!name_ok(v, true)) return fail(KWOK_EINVAL, "selector: bad value in '" + t + "'");
        }
        if (!name_ok(r.key, false)) return fail(KWOK_EINVAL, "selector: bad key in '" + t + "'");
        out->reqs.push_back(std::move(r));
    }
    return KWOK_OK;
}

int string_map(const JV* v, SMap* m) {
    m->clear();
    if (!v || v->is_null()) return KWOK_OK;
    if (v->t != JV::OBJ) return fail(KWOK_EDOMAIN, "labels/annotations is not an object");
    for (auto& kv : v->o) {
        if (kv.second.t != JV::STR) return fail(KWOK_EDOMAIN, "label/annotation value is not a string");
        m->emplace_back(kv.first, kv.second.s);
    }
    return KWOK_OK;
}

// a string the record references by span: must be unescaped (the span is the value)
int ref(const JV* v, kwok_str* out, const char* what) {
    *out = kwok_str{0, 0};
    if (!v || v->is_null()) return KWOK_OK;
    if (v->t != JV::STR) return fail(KWOK_EDOMAIN, std::string(what) + " is not a string");
    if (v->escaped) return fail(KWOK_EDOMAIN, std::string(what) + " holds a JSON escape (not a safe string)");
    if (v->len) *out = kwok_str{v->off, v->len};
    return KWOK_OK;
}

// RFC3339 "YYYY-MM-DDTHH:MM:SSZ" (metav1.Time's wire form) -> unix seconds
bool parse_time(std::string_view s, int64_t* out) {
    if (s.size() != 20 || s[4] != '-' || s[7] != '-' || s[10] != 'T' || s[13] != ':' || s[16] != ':' || s[19] != 'Z')
        return false;
    auto d = [&](int a, int n, int* v) {
        *v = 0;
        for (int k = a; k < a + n; k++) {
            if (s[k] < '0' || s[k] > '9') return false;
            *v = *v * 10 + (s[k] - '0');
        }
        return true;
    };
    int Y, M, D, h, m, sec;
    if (!d(0, 4, &Y) || !d(5, 2, &M) || !d(8, 2, &D) || !d(11, 2, &h) || !d(14, 2, &m) || !d(17, 2, &sec)) return false;
    if (M < 1 || M > 12 || D < 1 || D > 31 || h > 23 || m > 59 || sec > 59) return false;
    // days from civil (proleptic Gregorian)
    int y = Y - (M <= 2);
    int era = (y >= 0 ? y : y - 399) / 400;
    int yoe = y - era * 400;
    int doy = (153 * (M + (M > 2 ? -3 : 9)) + 2) / 5 + D - 1;
    int doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    int64_t days = (int64_t)era * 146097 + doe - 719468;
    *out = days * 86400 + h * 3600 + m * 60 + sec;
    return true;
}

uint8_t pod_phase(std::string_view s) {
    if (s.empty()) return KWOK_PHASE_NONE;
    if (s == "Pending") return KWOK_PHASE_PENDING;
    if (s == "Running") return KWOK_PHASE_RUNNING;
    if (s == "Succeeded") return KWOK_PHASE_SUCCEEDED;
    if (s == "Failed") return KWOK_PHASE_FAILED;
    if (s == "Unknown") return KWOK_PHASE_UNKNOWN;
    return KWOK_PHASE_OTHER;
}

struct Doc {
    std::deque<std::string> store;
    JV root;
};

int parse_doc(const char* arena, size_t arena_len, size_t off, size_t len, Doc* d) {
    if (!arena || off > arena_len || len > arena_len - off || arena_len > 0xFFFFFFFFull)
        return fail(KWOK_EINVAL, "document span outside the arena (or arena > 4 GiB)");
    Parser ps(arena, off, len, &d->store);
    if (!ps.document(d->root) || d->root.t != JV::OBJ) return fail(KWOK_EDOMAIN, "malformed JSON object document");
    return KWOK_OK;
}

}  // namespace

struct kwok_codec {
    bool manage_all = false;
    Selector manage_ann, manage_label, disregard_ann, disregard_label;
};

extern "C" {

int kwok_codec_create(const kwok_codec_config* cfg, kwok_codec** out) {
    if (!cfg || !out) return fail(KWOK_EINVAL, "null argument");
    *out = nullptr;
    auto* c = new kwok_codec();
    int rc = KWOK_OK;
    c->manage_all = cfg->manage_all_nodes != 0;
    auto nonempty = [](const char* s) { return s && *s; };
    if (!c->manage_all) {  // controller.go:82-101: the first configured mode wins
        if (nonempty(cfg->manage_nodes_with_annotation_selector))
            rc = parse_selector(cfg->manage_nodes_with_annotation_selector, &c->manage_ann);
        else if (nonempty(cfg->manage_nodes_with_label_selector))
            rc = parse_selector(cfg->manage_nodes_with_label_selector, &c->manage_label);
        else rc = fail(KWOK_EINVAL, "no nodes are managed");
    }
    if (rc == KWOK_OK) rc = parse_selector(cfg->disregard_status_with_annotation_selector, &c->disregard_ann);
    if (rc == KWOK_OK) rc = parse_selector(cfg->disregard_status_with_label_selector, &c->disregard_label);
    if (rc != KWOK_OK) {
        delete c;
        return rc;
    }
    *out = c;
    return KWOK_OK;
}

void kwok_codec_destroy(kwok_codec* c) { delete c; }

const char* kwok_codec_last_error(void) { return g_err.c_str(); }

int kwok_selector_matches(const char* selector, const char* json_map, size_t len, int32_t* out) {
    Selector s;
    int rc = parse_selector(selector, &s);
    if (rc) return rc;
    JV v;
    std::deque<std::string> store;
    Parser ps(json_map, 0, len, &store);
    if (!ps.document(v) || (v.t != JV::OBJ && v.t != JV::NUL)) return fail(KWOK_EINVAL, "bad label map JSON");
    SMap m;
    if ((rc = string_map(&v, &m))) return rc;
    *out = s.set && s.matches(m) ? 1 : 0;
    return KWOK_OK;
}

}  // extern "C"

// the codec's selectors for the device scanner (json.hip): KWOK_EDOMAIN when they
// exceed its fixed tables (JSEL_REQ requirements, JSEL_VAL values, JSEL_BYTES bytes)
int kwok::codec_export(const kwok_codec* c, kwok::JsonCfg* out) {
    if (!c || !out) return KWOK_EINVAL;
    memset(out, 0, sizeof *out);
    out->manage_all = c->manage_all ? 1u : 0u;
    uint32_t nb = 0, nv = 0;
    auto put = [&](const std::string& t, uint16_t* off, uint16_t* len) {
        if (nb + t.size() > (size_t)JSEL_BYTES) return false;
        memcpy(out->bytes + nb, t.data(), t.size());
        *off = (uint16_t)nb;
        *len = (uint16_t)t.size();
        nb += (uint32_t)t.size();
        return true;
    };
    const Selector* src[4] = {&c->manage_ann, &c->manage_label, &c->disregard_ann, &c->disregard_label};
    JsonSel* dst[4] = {&out->man_ann, &out->man_lab, &out->dis_ann, &out->dis_lab};
    for (int q = 0; q < 4; q++) {
        const Selector& S = *src[q];
        JsonSel& D = *dst[q];
        D.set = S.set ? 1u : 0u;
        if (S.reqs.size() > (size_t)JSEL_REQ) return fail(KWOK_EDOMAIN, "selector: too many requirements for the device codec");
        D.nreq = (uint32_t)S.reqs.size();
        for (size_t r = 0; r < S.reqs.size(); r++) {
            const Req& R = S.reqs[r];
            D.op[r] = R.op == Req::IN ? JREQ_IN : R.op == Req::NOTIN ? JREQ_NOTIN : R.op == Req::EXISTS ? JREQ_EXISTS
                                                                                                         : JREQ_NOTEXISTS;
            if (!put(R.key, &D.key_off[r], &D.key_len[r])) return fail(KWOK_EDOMAIN, "selector: too long for the device codec");
            if (nv + R.vals.size() > (size_t)JSEL_VAL) return fail(KWOK_EDOMAIN, "selector: too many values for the device codec");
            D.val_first[r] = (uint8_t)nv;
            D.val_n[r] = (uint8_t)R.vals.size();
            for (auto& v : R.vals) {
                if (!put(v, &D.val_off[nv], &D.val_len[nv])) return fail(KWOK_EDOMAIN, "selector: too long for the device codec");
                nv++;
            }
        }
    }
    return KWOK_OK;
}

extern "C" {

int kwok_decode_node(const kwok_codec* c, char* arena, size_t arena_len, size_t doc_off, size_t doc_len,
                     kwok_node_event* ev) {
    if (!c || !ev) return fail(KWOK_EINVAL, "null argument");
    Doc d;
    int rc = parse_doc(arena, arena_len, doc_off, doc_len, &d);
    if (rc) return rc;
    memset(ev, 0, sizeof *ev);
    ev->op = KWOK_OP_UPSERT;
    const JV* md = d.root.get("metadata");
    if (!md || md->t != JV::OBJ) return fail(KWOK_EDOMAIN, "node without metadata");
    if ((rc = ref(md->get("name"), &ev->name, "metadata.name"))) return rc;
    if (!ev->name.len) return fail(KWOK_EDOMAIN, "node without a name");
    SMap ann, lab;
    if ((rc = string_map(md->get("annotations"), &ann)) || (rc = string_map(md->get("labels"), &lab))) return rc;
    // needHeartbeat = nodeSelectorFunc (controller.go:83-98); with a label selector the
    // apiserver filters the list/watch, so an object that reaches the codec is managed iff it matches
    if (c->manage_all) ev->managed = 1;
    else if (c->manage_ann.set) ev->managed = c->manage_ann.matches(ann);
    else ev->managed = c->manage_label.set && c->manage_label.matches(lab);
    // needLockNode (node_controller.go:210-223): empty maps never match
    bool disregard = (c->disregard_ann.set && !ann.empty() && c->disregard_ann.matches(ann)) ||
                     (c->disregard_label.set && !lab.empty() && c->disregard_label.matches(lab));
    ev->lockable = !disregard;
    const JV* st = d.root.get("status");
    if (st && st->t == JV::OBJ) {
        const JV* ph = st->get("phase");
        if (ph && ph->t == JV::STR) ev->phase = ph->s.empty() ? KWOK_PHASE_NONE : ph->s == "Running" ? KWOK_PHASE_RUNNING : KWOK_PHASE_OTHER;
        // addresses / allocatable / capacity: canonical JSON written over the value's own span
        const char* keys[3] = {"addresses", "allocatable", "capacity"};
        kwok_str* outs[3] = {&ev->addresses, &ev->allocatable, &ev->capacity};
        std::vector<std::pair<const JV*, kwok_str*>> blobs;
        for (int k = 0; k < 3; k++) {
            const JV* v = st->get(keys[k]);
            if (!v || v->t == JV::NUL) continue;
            if (v->t != (k == 0 ? JV::ARR : JV::OBJ)) return fail(KWOK_EDOMAIN, std::string("status.") + keys[k] + " has the wrong type");
            if ((k == 0 && v->a.empty()) || (k > 0 && v->o.empty())) continue;
            blobs.emplace_back(v, outs[k]);
        }
        const JV* ni = st->get("nodeInfo");
        if (ni && ni->t == JV::OBJ) {
            for (int k = 0; k < KWOK_NI_COUNT; k++) {
                static const char* nik[KWOK_NI_COUNT] = {"architecture", "bootID", "containerRuntimeVersion",
                                                         "kernelVersion", "kubeProxyVersion", "kubeletVersion",
                                                         "machineID", "operatingSystem", "osImage", "systemUUID"};
                if ((rc = ref(ni->get(nik[k]), &ev->node_info[k], nik[k]))) return rc;
            }
        }
        for (auto& b : blobs) {  // every string is parsed already: rewriting spans is safe now
            std::string js;
            if (!canon(js, *b.first)) return fail(KWOK_EDOMAIN, "node status blob outside the canonical JSON domain");
            if (js.size() > b.first->len) return fail(KWOK_EDOMAIN, "canonical node status blob longer than its source");
            memcpy(arena + b.first->off, js.data(), js.size());
            *b.second = kwok_str{b.first->off, (uint32_t)js.size()};
        }
    }
    return KWOK_OK;
}

int kwok_decode_pod(const kwok_codec* c, char* arena, size_t arena_len, size_t doc_off, size_t doc_len,
                    kwok_pod_doc* out) {
    if (!c || !out) return fail(KWOK_EINVAL, "null argument");
    Doc d;
    int rc = parse_doc(arena, arena_len, doc_off, doc_len, &d);
    if (rc) return rc;
    memset(out, 0, sizeof *out);
    kwok_pod_event& ev = out->ev;
    ev.op = KWOK_OP_UPSERT;
    ev.handle = -1;
    ev.spec_id = -1;
    ev.node_handle = -1;
    const JV* md = d.root.get("metadata");
    if (!md || md->t != JV::OBJ) return fail(KWOK_EDOMAIN, "pod without metadata");
    if ((rc = ref(md->get("name"), &out->name, "metadata.name")) ||
        (rc = ref(md->get("namespace"), &out->namespace_, "metadata.namespace")))
        return rc;
    // creationTimestamp: $startTime of pod.status.tpl, re-formatted by the engine from seconds
    const JV* ct = md->get("creationTimestamp");
    if (!ct || ct->t != JV::STR || !parse_time(ct->s, &ev.creation_unix))
        return fail(KWOK_EDOMAIN, "metadata.creationTimestamp missing or not YYYY-MM-DDTHH:MM:SSZ");
    std::string_view st_time = ct->s;
    SMap ann, lab;
    if ((rc = string_map(md->get("annotations"), &ann)) || (rc = string_map(md->get("labels"), &lab))) return rc;
    // needLockPod selectors (pod_controller.go:257-267): empty maps never match
    if ((c->disregard_ann.set && !ann.empty() && c->disregard_ann.matches(ann)) ||
        (c->disregard_label.set && !lab.empty() && c->disregard_label.matches(lab)))
        ev.flags |= KWOK_POD_DISREGARD;
    const JV* dt = md->get("deletionTimestamp");
    if (dt && !dt->is_null()) ev.flags |= KWOK_POD_DELETING;
    const JV* fin = md->get("finalizers");
    if (fin && fin->t == JV::ARR && !fin->a.empty()) ev.flags |= KWOK_POD_HAS_FINALIZERS;

    const JV* spec = d.root.get("spec");
    if (!spec || spec->t != JV::OBJ) return fail(KWOK_EDOMAIN, "pod without spec");
    if ((rc = ref(spec->get("nodeName"), &ev.node_name, "spec.nodeName"))) return rc;
    struct CS { const char* key; kwok_container* dst; uint32_t* n; };
    CS lists[2] = {{"containers", out->containers, &out->n_containers},
                   {"initContainers", out->init_containers, &out->n_init_containers}};
    for (auto& L : lists) {
        const JV* v = spec->get(L.key);
        if (!v || v->is_null()) continue;
        if (v->t != JV::ARR) return fail(KWOK_EDOMAIN, std::string("spec.") + L.key + " is not a list");
        if (v->a.size() > KWOK_DOC_MAX_CONTAINERS) return fail(KWOK_EDOMAIN, std::string("too many spec.") + L.key);
        for (auto& e : v->a) {
            if (e.t != JV::OBJ) return fail(KWOK_EDOMAIN, "container is not an object");
            kwok_container& k = L.dst[(*L.n)++];
            if ((rc = ref(e.get("name"), &k.name, "container name")) || (rc = ref(e.get("image"), &k.image, "container image")))
                return rc;
        }
    }
    const JV* gates = spec->get("readinessGates");
    if (gates && gates->t == JV::ARR) {
        if (gates->a.size() > KWOK_DOC_MAX_GATES) return fail(KWOK_EDOMAIN, "too many spec.readinessGates");
        for (auto& g : gates->a) {
            if (g.t != JV::OBJ) return fail(KWOK_EDOMAIN, "readiness gate is not an object");
            if ((rc = ref(g.get("conditionType"), &out->readiness_gates[out->n_readiness_gates++], "conditionType")))
                return rc;
        }
    }

    const JV* st = d.root.get("status");
    if (st && st->t != JV::OBJ && !st->is_null()) return fail(KWOK_EDOMAIN, "pod status is not an object");
    if (!st || st->is_null()) return KWOK_OK;
    if (!zeroish(*st)) ev.flags |= KWOK_POD_STATUS_NONEMPTY;
    const JV* ph = st->get("phase");
    if (ph && ph->t == JV::STR) ev.phase = pod_phase(ph->s);
    if ((rc = ref(st->get("hostIP"), &ev.host_ip, "status.hostIP")) || (rc = ref(st->get("podIP"), &ev.pod_ip, "status.podIP")))
        return rc;

    // CONFORMS: SMP(status, rendered) == status for the template's list/time fields (A.4)
    auto sv = [&](const kwok_str& s) { return std::string_view(arena + s.off, s.len); };
    bool conforms = true;
    // conditions: merge key `type`; each rendered condition must already be present with equal fields
    std::vector<std::string_view> types = {"Initialized", "Ready", "ContainersReady"};
    for (uint32_t k = 0; k < out->n_readiness_gates; k++) types.push_back(sv(out->readiness_gates[k]));
    const JV* conds = st->get("conditions");
    for (auto& t : types) {
        const JV* hit = nullptr;
        if (conds && conds->t == JV::ARR)
            for (auto& cnd : conds->a) {
                const JV* ty = cnd.get("type");
                if (ty && ty->t == JV::STR && ty->s == t) { hit = &cnd; break; }
            }
        const JV* s = hit ? hit->get("status") : nullptr;
        const JV* lt = hit ? hit->get("lastTransitionTime") : nullptr;
        if (!hit || !s || s->t != JV::STR || s->s != "True" || !lt || lt->t != JV::STR || lt->s != st_time) {
            conforms = false;
            break;
        }
    }
    // containerStatuses / initContainerStatuses: replaced wholesale by the rendered list
    for (int which = 0; which < 2 && conforms; which++) {
        const kwok_container* cs = which ? out->init_containers : out->containers;
        uint32_t n = which ? out->n_init_containers : out->n_containers;
        JV want;
        want.t = JV::ARR;
        for (uint32_t k = 0; k < n; k++) {
            JV state = which ? jobj({{"terminated", jobj({{"exitCode", jnum("0")}, {"finishedAt", jstr(st_time)},
                                                          {"reason", jstr("Completed")}, {"startedAt", jstr(st_time)}})}})
                             : jobj({{"running", jobj({{"startedAt", jstr(st_time)}})}});
            want.a.push_back(jobj({{"image", jstr(sv(cs[k].image))}, {"name", jstr(sv(cs[k].name))},
                                   {"ready", jbool(true)}, {"restartCount", jnum("0")}, {"state", state}}));
        }
        const JV* have = st->get(which ? "initContainerStatuses" : "containerStatuses");
        JV none;
        if (!norm_equal(have ? *have : none, want)) conforms = false;
    }
    const JV* stt = st->get("startTime");
    if (conforms && (!stt || stt->t != JV::STR || stt->s != st_time)) conforms = false;
    if (conforms) ev.flags |= KWOK_POD_CONFORMS;
    return KWOK_OK;
}

}  // extern "C"

namespace {
template <class F>
int batch(size_t n, int threads, int32_t* status, F&& one) {
    if (threads < 1) threads = 1;
    if ((size_t)threads > n) threads = (int)(n ? n : 1);
    std::vector<int> bad(threads, 0);
    auto run = [&](int t) {
        for (size_t i = t; i < n; i += threads) {  // strided: similar-size documents spread evenly
            int rc = one(i);
            if (status) status[i] = rc;
            if (rc) bad[t]++;
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < threads; t++) pool.emplace_back(run, t);
    run(0);
    for (auto& th : pool) th.join();
    int total = 0;
    for (int b : bad) total += b;
    return total;
}
}  // namespace

extern "C" {

int kwok_decode_nodes(const kwok_codec* c, char* arena, size_t arena_len, const uint64_t* doc_off,
                      const uint32_t* doc_len, size_t n, int threads, kwok_node_event* ev, int32_t* status) {
    if (!c || (n && (!doc_off || !doc_len || !ev))) return fail(KWOK_EINVAL, "null argument");
    return batch(n, threads, status, [&](size_t i) { return kwok_decode_node(c, arena, arena_len, doc_off[i], doc_len[i], &ev[i]); });
}

int kwok_decode_pods(const kwok_codec* c, char* arena, size_t arena_len, const uint64_t* doc_off,
                     const uint32_t* doc_len, size_t n, int threads, kwok_pod_doc* out, int32_t* status) {
    if (!c || (n && (!doc_off || !doc_len || !out))) return fail(KWOK_EINVAL, "null argument");
    return batch(n, threads, status, [&](size_t i) { return kwok_decode_pod(c, arena, arena_len, doc_off[i], doc_len[i], &out[i]); });
}

}  // extern "C"
