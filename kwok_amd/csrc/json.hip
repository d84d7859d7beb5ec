// json.hip - the watch-event codec's pod decode on the GPU (SURVEY.md §8(f)
// rank 2: "Watch-event -> SoA ingest codec ... later as a GPU JSON scanner").
//
// The host codec (codec.cpp, kwok_decode_pod) parses a Kubernetes Pod document
// into a DOM and derives the record kwok_ingest_pods takes: the routing flags of
// WatchPods / ListPods (pod_controller.go:252-269, 301-343: needLockPod's
// disregard selectors, deletionTimestamp, finalizers), the `{{ with .status }}`
// guard and computePatchData's strategic-merge no-op test (pod_controller.go:
// 404-439).  Here one thread scans one document in a single pass -
// no DOM: a streaming tokenizer (jparse) drives a handler (PodScan) that keeps
// only what the record needs, with the zero-value of every container tracked as
// the scan closes it (the omitempty semantics of the corev1 round trip).
//
// The scan decides exactly what the host codec decides, byte for byte, for the
// documents it accepts: the same kwok_pod_event (flags, phase, creation time,
// string spans into the arena), name, namespace and pod spec.  What it does not
// decide is listed for the host codec, never guessed (JSON_HOST):
//   * a JSON escape in a string that is compared or mapped (a key the scan
//     routes on, a label / annotation key, a selector-matched value, the status
//     phase, condition fields, container status fields): the host compares
//     decoded text.  Escapes in referenced strings are KWOK_EDOMAIN, as in the
//     host codec; escapes anywhere else change nothing.
// Documents outside the accepted JSON are KWOK_EDOMAIN, as malformed documents
// are for the host parser (same grammar: its lenient numbers, depth <= 64,
// surrogate pairs).
// A status that precedes the metadata or spec (its no-op test needs the creation
// time, the containers and readiness gates) is skipped by the first pass and
// scanned by a second one over its own bytes once the document has been read
// (Go's json.Marshal writes metadata, spec, status in that order; other writers
// need not).
#include <hip/hip_runtime.h>

#include "kernels.h"

namespace kwok {

namespace {

// ---------------------------------------------------------------------------
// a document's bytes, read 16 at a time (the arena is 16-aligned and padded).
// A 64-byte window (a quarter of the refills) measured slower: a C5 batch of 10k
// node documents 0.68 -> 1.01 ms in k_json_nodes - the scan is bound by its
// per-byte instructions and the lanes' divergent paths, not by the refills
// ---------------------------------------------------------------------------
// positions are 32-bit: the JSON entry points take arenas below 4 GiB (engine.cpp), and
// half the scan's position arithmetic was 64-bit pairs
typedef uint32_t jpos;
struct JRd {
    const uint8_t* a;
    jpos pos, end;
    jpos wb;
    uint4 w;
    __device__ __forceinline__ uint32_t at(jpos p) {
        const jpos b = p & ~15u;
        if (b != wb) {
            wb = b;
            w = *reinterpret_cast<const uint4*>(a + b);
        }
        // (the byte picked from values, not by a select of the window's field addresses,
        // which the compiler would form from `o < 4 ? w.x : ...`: an indexed load keeps
        // the reader - and the scan state beside it - in scratch memory)
        const uint32_t o = (uint32_t)(p - b);
        const uint64_t q = o < 8 ? ((uint64_t)w.y << 32 | w.x) : ((uint64_t)w.w << 32 | w.z);
        return (uint32_t)(q >> (8 * (o & 7))) & 0xFFu;
    }
    __device__ __forceinline__ int peek() { return pos < end ? (int)at(pos) : -1; }
    // bytes from p up to the first one that ends a string's plain run (a quote, a
    // backslash or a control character), within p's 16-byte window: that byte's
    // offset from p, or the bytes to the window's end when the window holds none
    __device__ __forceinline__ uint32_t plain_run(jpos p);
};

// bit k set for each byte k of x that ends a string's plain run: a quote, a
// backslash or a control character (SWAR: a byte is zero iff its high bit stays
// clear below; the four high bits gathered by one multiply)
__device__ __forceinline__ uint32_t str_special4(uint32_t x) {
    auto zero = [](uint32_t y) { return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y | 0x7F7F7F7Fu); };
    const uint32_t m = zero(x ^ 0x22222222u) | zero(x ^ 0x5C5C5C5Cu) | zero(x & 0xE0E0E0E0u);
    return (((m >> 7) & 0x01010101u) * 0x01020408u) >> 24;
}
__device__ __forceinline__ uint32_t JRd::plain_run(jpos p) {
    (void)at(p);
    const uint32_t o = (uint32_t)(p - wb);
    const uint32_t m = (str_special4(w.x) | str_special4(w.y) << 4 | str_special4(w.z) << 8 | str_special4(w.w) << 12) &
                       (0xFFFFu << o);
    return (m ? (uint32_t)__builtin_ctz(m) : 16u) - o;
}

__device__ __forceinline__ bool bytes_eq(JRd& r, jpos off, uint32_t len, const uint8_t* s, uint32_t n) {
    if (len != n) return false;
    for (uint32_t k = 0; k < n; k++)
        if (r.at(off + k) != s[k]) return false;
    return true;
}
__device__ __forceinline__ bool span_eq(JRd& r, jpos a, jpos b, uint32_t len) {
    for (uint32_t k = 0; k < len; k++)
        if (r.at(a + k) != r.at(b + k)) return false;
    return true;
}
template <int N>
__device__ __forceinline__ bool lit_eq(JRd& r, jpos off, uint32_t len, const char (&s)[N]) {
    if (len != N - 1) return false;
    for (int k = 0; k < N - 1; k++)
        if (r.at(off + k) != (uint8_t)s[k]) return false;
    return true;
}

// ---------------------------------------------------------------------------
// the tokenizer: codec.cpp Parser's grammar, events to a handler
// ---------------------------------------------------------------------------
enum : uint8_t { J_STR, J_NUM, J_TRUE, J_FALSE, J_NULL };
struct JTok {
    jpos off;  // STR: inside the quotes; else the token
    uint32_t len;
    uint8_t kind;
    bool esc;      // STR held an escape (the span is not the value)
    bool nz;       // not a zero value (omitempty sense: codec.cpp zeroish)
};

__device__ __forceinline__ bool hexv(uint32_t c, uint32_t& v) {
    if (c >= '0' && c <= '9') v = (v << 4) | (c - '0');
    else if (c >= 'a' && c <= 'f') v = (v << 4) | (c - 'a' + 10);
    else if (c >= 'A' && c <= 'F') v = (v << 4) | (c - 'A' + 10);
    else return false;
    return true;
}
__device__ __forceinline__ bool hex4(JRd& r, uint32_t& v) {
    if (r.pos + 4 > r.end) return false;
    v = 0;
    for (int k = 0; k < 4; k++)
        if (!hexv(r.at(r.pos++), v)) return false;
    return true;
}
// a string token at r.pos (the opening quote)
__device__ __forceinline__ bool jstring(JRd& r, JTok& t) {
    r.pos++;
    t.kind = J_STR;
    t.off = r.pos;
    t.esc = false;
    for (;;) {
        if (r.pos >= r.end) return false;
        {  // the plain bytes of the 16-byte window in one step
            const uint32_t k = r.plain_run(r.pos);
            if (k >= r.end - r.pos) {
                r.pos = r.end;  // (the document ends inside the string)
                return false;
            }
            r.pos += k;
            if (r.pos - r.wb == 16) continue;  // (no special byte in the window)
        }
        const uint32_t c = r.at(r.pos);
        if (c == '"') break;
        if (c < 0x20) return false;
        if (c != '\\') {
            r.pos++;
            continue;
        }
        t.esc = true;
        if (++r.pos >= r.end) return false;
        const uint32_t e = r.at(r.pos++);
        if (e == 'u') {
            uint32_t c1;
            if (!hex4(r, c1)) return false;
            if (c1 >= 0xD800 && c1 < 0xDC00 && r.pos + 6 <= r.end && r.at(r.pos) == '\\' && r.at(r.pos + 1) == 'u') {
                r.pos += 2;
                uint32_t c2;
                if (!hex4(r, c2) || c2 < 0xDC00 || c2 >= 0xE000) return false;
            }
        } else if (!(e == '"' || e == '\\' || e == '/' || e == 'b' || e == 'f' || e == 'n' || e == 'r' || e == 't')) {
            return false;
        }
    }
    t.len = (uint32_t)(r.pos - t.off);
    t.nz = t.len > 0;  // an escape decodes to at least one byte
    r.pos++;
    return true;
}

// Handler interface: key(d, tok) - a key of the object at depth d; begin(d, arr,
// parent_arr) / end(d, arr, nz) - a container at depth d; scalar(d, tok,
// parent_arr).  Returns false on malformed JSON.  d0 > 0: one value at depth d0
// starting at r.pos (a member the handler deferred), parsed up to its end.
template <class H>
__device__ bool jparse(JRd& r, H& h, int d0 = 0) {
    uint64_t arr = 0, nzm = 0;  // depth 0..63: the container is an array / holds a non-zero value
    bool arr64 = false, nz64 = false;
    auto is_arr = [&](int d) { return d < 64 ? ((arr >> d) & 1) != 0 : arr64; };
    auto set_nz = [&](int d) {
        if (d < 64) nzm |= 1ull << d;
        else nz64 = true;
    };
    auto ws = [&]() {
        for (;;) {
            const int c = r.peek();
            if (c != ' ' && c != '\t' && c != '\n' && c != '\r') return;
            r.pos++;
        }
    };
    int d = d0 - 1;  // the innermost open container
    int state = 0;  // 0: a value; 1: after a value; 2: a key
    for (;;) {
        ws();
        const int c = r.peek();
        if (state == 0) {
            const int vd = d + 1;
            if (vd > 64) return false;
            const bool pa = d >= 0 && is_arr(d);
            if (pa) set_nz(d);  // an array with an element is not zero
            if (c == '{' || c == '[') {
                r.pos++;
                const bool a = c == '[';
                if (vd < 64) {
                    arr = a ? arr | (1ull << vd) : arr & ~(1ull << vd);
                    nzm &= ~(1ull << vd);
                } else {
                    arr64 = a, nz64 = false;
                }
                d = vd;
                h.begin(d, a, pa);
                ws();
                if (r.peek() == (a ? ']' : '}')) {
                    r.pos++;
                    h.end(d, a, false);
                    d--;
                    state = 1;
                } else {
                    state = a ? 0 : 2;
                }
                continue;
            }
            JTok t;
            if (c == '"') {
                if (!jstring(r, t)) return false;
            } else if (c == 't' || c == 'f' || c == 'n') {
                const char* w = c == 't' ? "true" : c == 'f' ? "false" : "null";
                const uint32_t n = c == 'f' ? 5 : 4;
                if (r.pos + n > r.end) return false;
                for (uint32_t k = 0; k < n; k++)
                    if (r.at(r.pos + k) != (uint8_t)w[k]) return false;
                t.off = r.pos, t.len = n, t.esc = false;
                t.kind = c == 't' ? J_TRUE : c == 'f' ? J_FALSE : J_NULL;
                t.nz = c == 't';
                r.pos += n;
            } else {  // codec.cpp num(): '-'? then any run of [0-9.eE+-]
                const jpos s = r.pos;
                if (c == '-') r.pos++;
                for (;;) {
                    const int x = r.peek();
                    if ((x >= '0' && x <= '9') || x == '.' || x == 'e' || x == 'E' || x == '+' || x == '-') r.pos++;
                    else break;
                }
                if (r.pos == s) return false;
                t.off = s, t.len = (uint32_t)(r.pos - s), t.kind = J_NUM, t.esc = false;
                t.nz = !(t.len == 1 && r.at(s) == '0');
            }
            if (t.nz && d >= 0) set_nz(d);
            h.scalar(vd, t, pa);
            state = 1;
            continue;
        }
        if (state == 1) {
            if (d < d0) return d0 ? true : c == -1;  // only whitespace after the document's value
            const bool a = is_arr(d);
            if (c == ',') {
                r.pos++;
                state = a ? 0 : 2;
            } else if (c == (a ? ']' : '}')) {
                r.pos++;
                const bool nz = d < 64 ? ((nzm >> d) & 1) != 0 : nz64;
                h.end(d, a, nz);
                d--;
                if (nz && d >= 0) set_nz(d);
            } else {
                return false;
            }
            continue;
        }
        // state 2: a key, ':'
        if (c != '"') return false;
        JTok k;
        if (!jstring(r, k)) return false;
        ws();
        if (r.peek() != ':') return false;
        r.pos++;
        h.key(d, k);
        state = 0;
    }
}

// RFC3339 "YYYY-MM-DDTHH:MM:SSZ" -> unix seconds (codec.cpp parse_time)
__device__ bool jtime(JRd& r, jpos off, uint32_t len, int64_t* out) {
    if (len != 20) return false;
    uint32_t b[20];
    for (int k = 0; k < 20; k++) b[k] = r.at(off + k);
    if (b[4] != '-' || b[7] != '-' || b[10] != 'T' || b[13] != ':' || b[16] != ':' || b[19] != 'Z') return false;
    auto dg = [&](int a, int n, int* v) {
        *v = 0;
        for (int k = a; k < a + n; k++) {
            if (b[k] < '0' || b[k] > '9') return false;
            *v = *v * 10 + (int)(b[k] - '0');
        }
        return true;
    };
    int Y, M, D, hh, mm, ss;
    if (!dg(0, 4, &Y) || !dg(5, 2, &M) || !dg(8, 2, &D) || !dg(11, 2, &hh) || !dg(14, 2, &mm) || !dg(17, 2, &ss))
        return false;
    if (M < 1 || M > 12 || D < 1 || D > 31 || hh > 23 || mm > 59 || ss > 59) return false;
    const int y = Y - (M <= 2);
    const int era = (y >= 0 ? y : y - 399) / 400;
    const int yoe = y - era * 400;
    const int doy = (153 * (M + (M > 2 ? -3 : 9)) + 2) / 5 + D - 1;
    const int doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    const int64_t days = (int64_t)era * 146097 + doe - 719468;
    *out = days * 86400 + hh * 3600 + mm * 60 + ss;
    return true;
}

// ---------------------------------------------------------------------------
// the pod document (kwok_decode_pod)
// ---------------------------------------------------------------------------
// scan contexts: what a value at a position of the document means
enum : uint8_t {
    X_NONE = 0, X_ROOT, X_META, X_SPEC, X_STATUS,
    X_NAME, X_NS, X_CT, X_DT, X_FIN, X_ANN, X_LAB, X_ANNV, X_LABV,
    X_NODENAME, X_CONTS, X_INITS, X_GATES, X_CONT, X_INIT, X_GATE, X_CNAME, X_CIMAGE, X_INAME, X_IIMAGE, X_GTYPE,
    X_PHASE, X_HOSTIP, X_PODIP, X_STT, X_CONDS, X_COND, X_CTYPE, X_CSTAT, X_CLTT,
    X_CST, X_ICST, X_CSE, X_ICSE, X_SIMAGE, X_SNAME, X_READY, X_STATE, X_ISTATE, X_RUN, X_TERM,
    X_TS_ST, X_TS_REASON, X_ZV,
};
constexpr int XD = 8;  // contexts kept for depths 0..7 (deeper values are opaque: only their zero-ness counts)
constexpr uint32_t MAXC = KWOK_DOC_MAX_CONTAINERS, MAXG = KWOK_DOC_MAX_GATES;

struct Span {
    uint32_t off, len;
};

struct SelState {  // one selector over one label map: the last value per requirement key (labels.Set)
    uint32_t has, in;  // bit r: the key is present / its value is one of the requirement's values
};

struct PodScan {
    JRd* r;
    const JsonCfg* cfg;
    uint64_t cx = 0;      // context per depth (8 bits each)
    uint8_t next = X_NONE;  // the context of the value a key announced
    int err = 0;          // KWOK_EDOMAIN
    bool host = false;    // JSON_HOST
    bool root_obj = false;
    // first occurrences (codec.cpp JV::get returns the first key)
    uint32_t seen_root = 0, seen_meta = 0, seen_spec = 0, seen_status = 0;
    bool meta_done = false, spec_done = false, meta_obj = false, spec_obj = false;
    bool st_defer = false, pass2 = false;  // a status read before metadata / spec: scanned again at the end
    jpos st_pos = 0;                       // its '{'
    // metadata
    Span name{0, 0}, ns{0, 0};
    bool ct_ok = false;
    jpos ct_off = 0;
    int64_t creation = 0;
    uint8_t flags = 0, phase = 0;
    uint32_t n_ann = 0, n_lab = 0;
    SelState dis_ann{0, 0}, dis_lab{0, 0};
    uint32_t key_match = 0;  // the requirements whose key the current label entry has
    // spec
    Span node{0, 0};
    uint32_t n_cont = 0, n_init = 0, n_gates = 0;
    Span cname[MAXC], cimage[MAXC], iname[MAXC], iimage[MAXC], gate[MAXG];
    uint32_t elem_seen = 0;  // first name / image of the current container element
    // status
    bool has_status = false;
    Span hip{0, 0}, pip{0, 0};
    bool stt_ok = false;
    uint32_t cond_hit = 0, cond_ok = 0;  // per wanted condition type (3 + gates)
    uint32_t ce_seen = 0;                // the current condition element's type / status / ltt
    Span ctype{0, 0};
    bool ctype_set = false, cstat_ok = false, cltt_ok = false;
    bool cst_seen = false, icst_seen = false, cst_ok = true, icst_ok = true;
    int list = 0;                        // the open container-status list: 0 cst, 1 icst
    uint32_t lst_count = 0, k = 0;       // its elements; the current element
    uint32_t e_seen = 0, s_seen = 0, r_seen = 0;  // element / state / running (terminated) keys present

    __device__ uint8_t ctx(int d) const { return d < XD ? (uint8_t)(cx >> (8 * d)) : X_NONE; }
    __device__ void set_ctx(int d, uint8_t c) {
        if (d < XD) cx = (cx & ~(0xFFull << (8 * d))) | ((uint64_t)c << (8 * d));
    }
    __device__ void miss() { (list ? icst_ok : cst_ok) = false; }
    __device__ uint8_t first(uint32_t& seen, int bit, uint8_t c) {
        if (seen & (1u << bit)) return X_NONE;
        seen |= 1u << bit;
        return c;
    }
    // the value's context: the element context of an array parent, else what its key announced
    __device__ uint8_t value_ctx(int d, bool pa) {
        if (d == 0) return X_ROOT;
        if (!pa) return next;
        switch (ctx(d - 1)) {
            case X_CONTS: return X_CONT;
            case X_INITS: return X_INIT;
            case X_GATES: return X_GATE;
            case X_CONDS: return X_COND;
            case X_CST: return X_CSE;
            case X_ICST: return X_ICSE;
            case X_FIN: return X_NONE;
            default: return X_NONE;
        }
    }
    // a key the scan routes on must be compared as decoded text: escaped -> host
    __device__ bool k_is(const JTok& t, const char* s, uint32_t n) {
        if (t.len != n) return false;
        for (uint32_t q = 0; q < n; q++)
            if (r->at(t.off + q) != (uint8_t)s[q]) return false;
        return true;
    }
#define KIS(lit) k_is(t, lit, sizeof(lit) - 1)

    __device__ void key(int d, const JTok& t) {
        const uint8_t c = ctx(d);
        next = X_NONE;
        if (c == X_NONE || c == X_ZV) return;
        if (c == X_ANN || c == X_LAB) {  // a label / annotation entry
            (c == X_ANN ? n_ann : n_lab)++;
            next = c == X_ANN ? X_ANNV : X_LABV;
            key_match = 0;
            const JsonSel& S = c == X_ANN ? cfg->dis_ann : cfg->dis_lab;
            if (!S.set || !S.nreq) return;
            if (t.esc) {
                host = true;
                return;
            }
            for (uint32_t q = 0; q < S.nreq; q++)
                if (bytes_eq(*r, t.off, t.len, cfg->bytes + S.key_off[q], S.key_len[q])) key_match |= 1u << q;
            return;
        }
        if (t.esc) {  // a routed key whose decoded text the scan does not compare
            if (c == X_ROOT || c == X_META || c == X_SPEC || c == X_STATUS || c == X_CONT || c == X_INIT ||
                c == X_GATE || c == X_COND || c == X_CSE || c == X_ICSE || c == X_STATE || c == X_ISTATE ||
                c == X_RUN || c == X_TERM)
                host = true;
            return;
        }
        switch (c) {
            case X_ROOT:
                if (KIS("metadata")) next = first(seen_root, 0, X_META);
                else if (KIS("spec")) next = first(seen_root, 1, X_SPEC);
                else if (KIS("status")) next = first(seen_root, 2, X_STATUS);
                break;
            case X_META:
                if (KIS("name")) next = first(seen_meta, 0, X_NAME);
                else if (KIS("namespace")) next = first(seen_meta, 1, X_NS);
                else if (KIS("creationTimestamp")) next = first(seen_meta, 2, X_CT);
                else if (KIS("annotations")) next = first(seen_meta, 3, X_ANN);
                else if (KIS("labels")) next = first(seen_meta, 4, X_LAB);
                else if (KIS("deletionTimestamp")) next = first(seen_meta, 5, X_DT);
                else if (KIS("finalizers")) next = first(seen_meta, 6, X_FIN);
                break;
            case X_SPEC:
                if (KIS("nodeName")) next = first(seen_spec, 0, X_NODENAME);
                else if (KIS("containers")) next = first(seen_spec, 1, X_CONTS);
                else if (KIS("initContainers")) next = first(seen_spec, 2, X_INITS);
                else if (KIS("readinessGates")) next = first(seen_spec, 3, X_GATES);
                break;
            case X_CONT:
            case X_INIT:
                if (KIS("name")) next = first(elem_seen, 0, c == X_CONT ? X_CNAME : X_INAME);
                else if (KIS("image")) next = first(elem_seen, 1, c == X_CONT ? X_CIMAGE : X_IIMAGE);
                break;
            case X_GATE:
                if (KIS("conditionType")) next = first(elem_seen, 0, X_GTYPE);
                break;
            case X_STATUS:
                if (KIS("phase")) next = first(seen_status, 0, X_PHASE);
                else if (KIS("hostIP")) next = first(seen_status, 1, X_HOSTIP);
                else if (KIS("podIP")) next = first(seen_status, 2, X_PODIP);
                else if (KIS("conditions")) next = first(seen_status, 3, X_CONDS);
                else if (KIS("containerStatuses")) next = first(seen_status, 4, X_CST);
                else if (KIS("initContainerStatuses")) next = first(seen_status, 5, X_ICST);
                else if (KIS("startTime")) next = first(seen_status, 6, X_STT);
                break;
            case X_COND:
                if (KIS("type")) next = first(ce_seen, 0, X_CTYPE);
                else if (KIS("status")) next = first(ce_seen, 1, X_CSTAT);
                else if (KIS("lastTransitionTime")) next = first(ce_seen, 2, X_CLTT);
                break;
            // norm_equal(have, want): every occurrence of a key is compared; a key the
            // rendered status lacks must hold a zero value
            case X_CSE:
            case X_ICSE:
                if (KIS("image")) next = X_SIMAGE, e_seen |= 1;
                else if (KIS("name")) next = X_SNAME, e_seen |= 2;
                else if (KIS("ready")) next = X_READY, e_seen |= 4;
                else if (KIS("state")) next = c == X_CSE ? X_STATE : X_ISTATE, e_seen |= 8;
                else next = X_ZV;  // restartCount (rendered 0) and anything else
                break;
            case X_STATE:
                if (KIS("running")) next = X_RUN, s_seen |= 1;
                else next = X_ZV;
                break;
            case X_ISTATE:
                if (KIS("terminated")) next = X_TERM, s_seen |= 1;
                else next = X_ZV;
                break;
            case X_RUN:
                if (KIS("startedAt")) next = X_TS_ST, r_seen |= 1;
                else next = X_ZV;
                break;
            case X_TERM:
                if (KIS("finishedAt")) next = X_TS_ST, r_seen |= 2;
                else if (KIS("startedAt")) next = X_TS_ST, r_seen |= 1;
                else if (KIS("reason")) next = X_TS_REASON, r_seen |= 4;
                else next = X_ZV;  // exitCode (rendered 0) and anything else
                break;
            default:
                break;
        }
    }
#undef KIS

    // a referenced string (codec.cpp ref): null / absent -> empty; otherwise an unescaped string
    __device__ void ref(const JTok& t, Span& out) {
        if (t.kind == J_NULL) return;
        if (t.kind != J_STR || t.esc) {
            err = KWOK_EDOMAIN;
            return;
        }
        if (t.len) out = Span{(uint32_t)t.off, t.len};
    }
    // a compared string equal to the creation time (decoded text: escaped -> host)
    __device__ bool is_ct(const JTok& t) {
        if (t.kind != J_STR) return false;
        if (t.esc) {
            host = true;
            return false;
        }
        return ct_ok && t.len == 20 && span_eq(*r, t.off, ct_off, 20);
    }
    // a container-status field compared with the rendered string w (norm_equal)
    __device__ void cmp_str(const JTok& t, Span w) {
        if (!t.nz) {
            if (w.len) miss();
            return;
        }
        if (t.kind != J_STR) {
            miss();
            return;
        }
        if (t.esc) {
            host = true;
            return;
        }
        if (t.len != w.len || !span_eq(*r, t.off, w.off, w.len)) miss();
    }
    __device__ Span want_field(bool image) const {
        if (list == 0) return k < n_cont ? (image ? cimage[k] : cname[k]) : Span{0, 0};
        return k < n_init ? (image ? iimage[k] : iname[k]) : Span{0, 0};
    }

    __device__ void scalar(int d, const JTok& t, bool pa) {
        const uint8_t c = value_ctx(d, pa);
        if (d == 0) return;  // not an object: rejected at the end
        switch (c) {
            case X_META:
            case X_SPEC:
                err = KWOK_EDOMAIN;  // metadata / spec must be objects
                break;
            case X_STATUS:
                if (t.kind != J_NULL) err = KWOK_EDOMAIN;  // status: an object or null
                break;
            case X_NAME: ref(t, name); break;
            case X_NS: ref(t, ns); break;
            case X_NODENAME: ref(t, node); break;
            case X_HOSTIP: ref(t, hip); break;
            case X_PODIP: ref(t, pip); break;
            case X_CNAME: if (n_cont) ref(t, cname[n_cont - 1]); break;
            case X_CIMAGE: if (n_cont) ref(t, cimage[n_cont - 1]); break;
            case X_INAME: if (n_init) ref(t, iname[n_init - 1]); break;
            case X_IIMAGE: if (n_init) ref(t, iimage[n_init - 1]); break;
            case X_GTYPE: if (n_gates) ref(t, gate[n_gates - 1]); break;
            case X_CT:
                if (t.kind != J_STR) err = KWOK_EDOMAIN;
                else if (t.esc) host = true;
                else if (!jtime(*r, t.off, t.len, &creation)) err = KWOK_EDOMAIN;
                else ct_ok = true, ct_off = t.off;
                break;
            case X_DT:
                if (t.kind != J_NULL) flags |= KWOK_POD_DELETING;
                break;
            case X_ANN:
            case X_LAB:
                if (t.kind != J_NULL) err = KWOK_EDOMAIN;  // a label map: an object or null
                break;
            case X_ANNV:
            case X_LABV: {
                if (t.kind != J_STR) {
                    err = KWOK_EDOMAIN;  // label / annotation values are strings
                    break;
                }
                const bool ann = c == X_ANNV;
                const JsonSel& S = ann ? cfg->dis_ann : cfg->dis_lab;
                SelState& st = ann ? dis_ann : dis_lab;
                if (!key_match) break;
                if (t.esc) {
                    host = true;
                    break;
                }
                for (uint32_t q = 0; q < S.nreq; q++) {  // the last entry of a key wins (a Go map)
                    if (!((key_match >> q) & 1)) continue;
                    bool in = false;
                    for (uint32_t v = 0; v < S.val_n[q]; v++) {
                        const uint32_t vi = S.val_first[q] + v;
                        in |= bytes_eq(*r, t.off, t.len, cfg->bytes + S.val_off[vi], S.val_len[vi]);
                    }
                    st.has |= 1u << q;
                    st.in = in ? st.in | (1u << q) : st.in & ~(1u << q);
                }
                break;
            }
            case X_CONTS:
            case X_INITS:
                if (t.kind != J_NULL) err = KWOK_EDOMAIN;  // a list or null
                break;
            case X_CONT:
            case X_INIT:
            case X_GATE:
                err = KWOK_EDOMAIN;  // list elements are objects
                break;
            case X_PHASE:
                if (t.kind == J_STR) {
                    if (t.esc) {
                        host = true;
                        break;
                    }
                    if (!t.len) phase = KWOK_PHASE_NONE;
                    else if (lit_eq(*r, t.off, t.len, "Pending")) phase = KWOK_PHASE_PENDING;
                    else if (lit_eq(*r, t.off, t.len, "Running")) phase = KWOK_PHASE_RUNNING;
                    else if (lit_eq(*r, t.off, t.len, "Succeeded")) phase = KWOK_PHASE_SUCCEEDED;
                    else if (lit_eq(*r, t.off, t.len, "Failed")) phase = KWOK_PHASE_FAILED;
                    else if (lit_eq(*r, t.off, t.len, "Unknown")) phase = KWOK_PHASE_UNKNOWN;
                    else phase = KWOK_PHASE_OTHER;
                }
                break;
            case X_STT: stt_ok = is_ct(t); break;
            case X_CTYPE:
                if (t.kind == J_STR) {
                    if (t.esc) host = true;
                    else ctype = Span{(uint32_t)t.off, t.len}, ctype_set = true;
                }
                break;
            case X_CSTAT:
                if (t.kind == J_STR) {
                    if (t.esc) host = true;
                    else cstat_ok = lit_eq(*r, t.off, t.len, "True");
                }
                break;
            case X_CLTT: cltt_ok = is_ct(t); break;
            case X_CST:
            case X_ICST:  // not a list: equal to the rendered list only if both are zero
                list = c == X_ICST;
                (c == X_CST ? cst_seen : icst_seen) = true;
                if (t.nz || (c == X_CST ? n_cont : n_init)) miss();
                break;
            case X_CSE:
            case X_ICSE:  // a scalar element: the rendered element is an object
                list = c == X_ICSE;
                lst_count++;
                miss();
                break;
            case X_SIMAGE: cmp_str(t, want_field(true)); break;
            case X_SNAME: cmp_str(t, want_field(false)); break;
            case X_READY:
                if (t.kind != J_TRUE) miss();
                break;
            case X_STATE:
            case X_ISTATE:
            case X_RUN:
            case X_TERM:
                miss();  // the rendered value is an object
                break;
            case X_TS_ST:
                if (!is_ct(t)) miss();
                break;
            case X_TS_REASON:
                if (t.kind != J_STR) miss();
                else if (t.esc) host = true;
                else if (!lit_eq(*r, t.off, t.len, "Completed")) miss();
                break;
            case X_ZV:
                if (t.nz) miss();
                break;
            default:
                break;
        }
    }

    __device__ void begin(int d, bool a, bool pa) {
        const uint8_t c = value_ctx(d, pa);
        uint8_t mine = X_NONE;  // the context of this container's own members
        if (d == 0) {
            root_obj = !a;
            set_ctx(0, a ? X_NONE : X_ROOT);
            return;
        }
        switch (c) {
            case X_META: if (a) err = KWOK_EDOMAIN; else mine = X_META, meta_obj = true; break;
            case X_SPEC: if (a) err = KWOK_EDOMAIN; else mine = X_SPEC, spec_obj = true; break;
            case X_STATUS:
                if (a) {
                    err = KWOK_EDOMAIN;
                    break;
                }
                // its no-op test needs the creation time, containers and gates: before
                // them, skipped (X_NONE) and scanned by the second pass
                if (!pass2 && (!meta_done || !spec_done || !ct_ok)) {
                    st_defer = true;
                    st_pos = r->pos - 1;
                    break;
                }
                has_status = true;
                mine = X_STATUS;
                break;
            case X_NAME: case X_NS: case X_NODENAME: case X_HOSTIP: case X_PODIP:
            case X_CNAME: case X_CIMAGE: case X_INAME: case X_IIMAGE: case X_GTYPE:
            case X_CT: case X_ANNV: case X_LABV:
                err = KWOK_EDOMAIN;  // strings
                break;
            case X_DT: flags |= KWOK_POD_DELETING; break;
            case X_FIN: if (a) mine = X_FIN; break;
            case X_ANN: case X_LAB: if (a) err = KWOK_EDOMAIN; else mine = c; break;
            case X_CONTS: case X_INITS: if (!a) err = KWOK_EDOMAIN; else mine = c; break;
            case X_GATES: if (a) mine = X_GATES; break;  // not a list: ignored
            case X_CONT:
            case X_INIT: {
                if (a) {
                    err = KWOK_EDOMAIN;
                    break;
                }
                uint32_t& n = c == X_CONT ? n_cont : n_init;
                if (n >= MAXC) {
                    err = KWOK_EDOMAIN;  // too many containers
                    break;
                }
                (c == X_CONT ? cname : iname)[n] = Span{0, 0};
                (c == X_CONT ? cimage : iimage)[n] = Span{0, 0};
                n++;
                elem_seen = 0;
                mine = c;
                break;
            }
            case X_GATE:
                if (a) {
                    err = KWOK_EDOMAIN;
                    break;
                }
                if (n_gates >= MAXG) {
                    err = KWOK_EDOMAIN;
                    break;
                }
                gate[n_gates++] = Span{0, 0};
                elem_seen = 0;
                mine = X_GATE;
                break;
            case X_CONDS: if (a) mine = X_CONDS; break;
            case X_COND:
                if (!a) {
                    ce_seen = 0, ctype_set = cstat_ok = cltt_ok = false;
                    mine = X_COND;
                }
                break;
            case X_CST:
            case X_ICST:  // a list; any other container must be zero (and no container rendered)
                list = c == X_ICST;
                (c == X_CST ? cst_seen : icst_seen) = true;
                lst_count = 0;
                mine = c;
                break;
            case X_CSE:
            case X_ICSE:
                k = lst_count++;
                if (a) {
                    miss();  // the rendered element is an object
                } else {
                    e_seen = 0;
                    mine = c;
                }
                break;
            case X_STATE:
            case X_ISTATE:
                if (a) miss();
                else s_seen = 0, mine = c;
                break;
            case X_RUN:
            case X_TERM:
                if (a) miss();
                else r_seen = 0, mine = c;
                break;
            case X_SIMAGE:
            case X_SNAME:
            case X_READY:
            case X_TS_ST:
            case X_TS_REASON:
            case X_ZV:
                mine = c;  // a compared value that is a container: decided at its end, from its zero-ness
                break;
            default:
                break;
        }
        set_ctx(d, mine);
        if (d >= XD - 1 && mine != X_NONE && mine != X_ZV) host = true;  // (never at the depths a pod uses)
    }

    __device__ void end(int d, bool a, bool nz) {
        const uint8_t c = ctx(d);
        if (d == 1) {
            if (c == X_META) meta_done = true;
            if (c == X_SPEC) spec_done = true;
            if (c == X_STATUS && nz) flags |= KWOK_POD_STATUS_NONEMPTY;
        }
        switch (c) {
            case X_FIN:
                if (nz) flags |= KWOK_POD_HAS_FINALIZERS;  // a list with an element
                break;
            case X_COND:
                if (ctype_set) {
                    const uint32_t nw = 3 + n_gates;
                    for (uint32_t q = 0; q < nw; q++) {
                        if ((cond_hit >> q) & 1) continue;
                        bool m;
                        if (q == 0) m = lit_eq(*r, ctype.off, ctype.len, "Initialized");
                        else if (q == 1) m = lit_eq(*r, ctype.off, ctype.len, "Ready");
                        else if (q == 2) m = lit_eq(*r, ctype.off, ctype.len, "ContainersReady");
                        else m = gate[q - 3].len == ctype.len && span_eq(*r, gate[q - 3].off, ctype.off, ctype.len);
                        if (!m) continue;
                        cond_hit |= 1u << q;
                        if (cstat_ok && cltt_ok) cond_ok |= 1u << q;
                    }
                }
                break;
            case X_CST:
            case X_ICST:
                if (a ? lst_count != (c == X_CST ? n_cont : n_init) : (nz || (c == X_CST ? n_cont : n_init))) miss();
                break;
            case X_CSE:
            case X_ICSE: {
                const uint32_t n = c == X_CSE ? n_cont : n_init;
                if (k >= n) {
                    miss();
                    break;
                }
                uint32_t need = 4 | 8;  // ready, state
                if (want_field(true).len) need |= 1;
                if (want_field(false).len) need |= 2;
                if ((e_seen & need) != need) miss();
                break;
            }
            case X_STATE:
            case X_ISTATE:
                if (!(s_seen & 1)) miss();
                break;
            case X_RUN:
                if (!(r_seen & 1)) miss();
                break;
            case X_TERM:
                if ((r_seen & 7) != 7) miss();
                break;
            case X_SIMAGE:
            case X_SNAME:  // a container: equal to the rendered string only if both are zero
                if (nz || want_field(c == X_SIMAGE).len) miss();
                break;
            case X_READY:
            case X_TS_ST:
            case X_TS_REASON:
                miss();  // the rendered value is a non-zero scalar
                break;
            case X_ZV:
                if (nz) miss();
                break;
            default:
                break;
        }
    }

    __device__ bool matches(const JsonSel& S, const SelState& st) const {
        for (uint32_t q = 0; q < S.nreq; q++) {
            const bool has = (st.has >> q) & 1, in = (st.in >> q) & 1;
            switch (S.op[q]) {
                case JREQ_IN: if (!in) return false; break;
                case JREQ_NOTIN: if (in) return false; break;
                case JREQ_EXISTS: if (!has) return false; break;
                default: if (has) return false; break;
            }
        }
        return true;
    }
};

// FNV-1a 64 of the pod spec the engine interns (kwok_register_pod_spec): each
// container's name 0x1F image 0x1E, 0x1D, the init containers alike, 0x1D, each
// readiness gate 0x1E (engine.cpp json_spec_key is the same function)
// The walk over those bytes (engine.cpp json_spec_canon writes the same string)
template <class F>
__device__ __forceinline__ void spec_walk(JRd& r, const PodScan& p, F&& byte) {
    auto str = [&](Span s) {
        for (uint32_t q = 0; q < s.len; q++) byte(r.at(s.off + q));
    };
    for (uint32_t q = 0; q < p.n_cont; q++) str(p.cname[q]), byte(0x1F), str(p.cimage[q]), byte(0x1E);
    byte(0x1D);
    for (uint32_t q = 0; q < p.n_init; q++) str(p.iname[q]), byte(0x1F), str(p.iimage[q]), byte(0x1E);
    byte(0x1D);
    for (uint32_t q = 0; q < p.n_gates; q++) str(p.gate[q]), byte(0x1E);
}
// the key (FNV-1a 64) and a second, independent hash of the same bytes
__device__ void spec_keys(JRd& r, const PodScan& p, uint64_t& k1, uint64_t& k2) {
    uint64_t h = 0xCBF29CE484222325ull, g = 0x243F6A8885A308D3ull;
    spec_walk(r, p, [&](uint32_t b) {
        h = (h ^ b) * 0x100000001B3ull;
        g = (g + b + 1) * 0x9E3779B97F4A7C15ull;
        g ^= g >> 29;
    });
    k1 = h, k2 = g;
}
// the document's spec is exactly the registered one (a key hit is not proof)
__device__ bool spec_equal(JRd& r, const PodScan& p, const uint8_t* canon, uint2 ref) {
    uint32_t k = 0;
    bool eq = true;
    spec_walk(r, p, [&](uint32_t b) {
        eq = eq && k < ref.y && canon[ref.x + k] == (uint8_t)b;
        k++;
    });
    return eq && k == ref.y;
}

}  // namespace

// A batch of fewer documents than the chip has CUs x 4 waves goes one wave per block:
// each scanning wave reads 64 documents' 16-byte windows (64 lines per load), so
// waves spread over all CUs share no CU's SIMDs (a 10k-document node batch: 0.82 ms
// in 40 blocks of 4 waves, 0.68 ms in 157 blocks of one)
__host__ __device__ inline uint32_t json_block(uint32_t n) { return n < 256u * 64u * 4u ? 64u : 256u; }

// one thread per document
__global__ __launch_bounds__(256) void k_json_pods(JsonPodArgs A) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.n) return;
    const uint64_t off = A.doc_off[i];
    const uint32_t len = A.doc_len[i];
    kwok_pod_event ev;
    ev.op = KWOK_OP_UPSERT;
    ev.phase = 0;
    ev.flags = 0;
    ev.reserved0 = 0;
    ev.handle = -1;
    ev.spec_id = -1;
    ev.node_handle = -1;
    ev.creation_unix = 0;
    ev.node_name = ev.host_ip = ev.pod_ip = kwok_str{0, 0};
    JsonPodSide side{};
    int32_t status;
    PodScan p;
    if (off > A.arena_len || len > A.arena_len - off) {
        status = KWOK_EINVAL;  // (codec.cpp parse_doc: a span outside the arena)
    } else {
        JRd rd{A.arena, (jpos)off, (jpos)(off + len), ~0u, make_uint4(0, 0, 0, 0)};
        p.r = &rd;
        p.cfg = A.cfg;
        bool ok = !A.cfg->all_host && jparse(rd, p);
        if (ok && p.st_defer && !p.host && !p.err) {
            if (!p.meta_done || !p.spec_done || !p.ct_ok) {
                p.host = true;  // (the host decides a status it cannot test)
            } else {
                p.pass2 = true;
                p.next = X_STATUS;
                rd.pos = p.st_pos;
                ok = jparse(rd, p, 1);
            }
        }
        // (a document the scan routed past an escaped key may hold errors the host's
        // first-key lookup does not see: the host decides it, errors included)
        if (A.cfg->all_host) status = JSON_HOST;  // (selectors the device tables do not hold)
        else if (!ok || !p.root_obj) status = KWOK_EDOMAIN;
        else if (p.host) status = JSON_HOST;
        else if (p.err) status = p.err;
        else if (!p.meta_obj || !p.spec_obj || !p.ct_ok) status = KWOK_EDOMAIN;
        else status = KWOK_OK;
        if (status == KWOK_OK) {
            const JsonCfg& C = *A.cfg;
            uint8_t fl = p.flags;
            if ((C.dis_ann.set && p.n_ann && p.matches(C.dis_ann, p.dis_ann)) ||
                (C.dis_lab.set && p.n_lab && p.matches(C.dis_lab, p.dis_lab)))
                fl |= KWOK_POD_DISREGARD;
            if (p.has_status) {
                const uint32_t nw = 3 + p.n_gates, all = (nw >= 32 ? ~0u : (1u << nw) - 1u);
                const bool cst = p.cst_seen ? p.cst_ok : p.n_cont == 0;
                const bool icst = p.icst_seen ? p.icst_ok : p.n_init == 0;
                if (p.cond_hit == all && p.cond_ok == all && cst && icst && p.stt_ok) fl |= KWOK_POD_CONFORMS;
                ev.phase = p.phase;
                ev.host_ip = kwok_str{p.hip.off, p.hip.len};
                ev.pod_ip = kwok_str{p.pip.off, p.pip.len};
            }
            ev.flags = fl;
            ev.creation_unix = p.creation;
            ev.node_name = kwok_str{p.node.off, p.node.len};
            side.name_off = p.name.off, side.name_len = p.name.len;
            side.ns_off = p.ns.off, side.ns_len = p.ns.len;
            side.n_cont = (uint8_t)p.n_cont, side.n_init = (uint8_t)p.n_init, side.n_gates = (uint8_t)p.n_gates;
            spec_keys(rd, p, side.spec_key, side.spec_key2);
            side.spec_key &= A.key_mask;
        }
    }
    // the ingest form: the caller's op / handle, the registered spec (device table)
    if (A.op) {
        ev.op = A.op[i];
        ev.handle = A.handle[i];
        if (status == KWOK_OK && ev.op == KWOK_OP_UPSERT) {
            int32_t id = -1;
            uint32_t hs = 0;
            for (uint32_t q = 0, h = (uint32_t)side.spec_key & A.tab_mask; q <= A.tab_mask; q++, h = (h + 1) & A.tab_mask) {
                const uint64_t kk = A.tab_key[h];
                if (kk == side.spec_key) {
                    id = A.tab_id[h];
                    hs = h;
                    break;
                }
                if (!kk) break;
            }
            // a key hit whose strings differ from the registered spec's (FNV-1a is not
            // collision-resistant and specs come from users): the host decides it
            JRd rc{A.arena, (jpos)off, (jpos)(off + len), ~0u, make_uint4(0, 0, 0, 0)};
            if (id >= 0 && !spec_equal(rc, p, A.canon, A.tab_canon[hs])) status = JSON_SPEC_X;
            else if (id < 0) status = JSON_SPEC;
            else ev.spec_id = id;
        }
        const bool listed = status == JSON_HOST || status == JSON_SPEC || status == JSON_SPEC_X;
        if (status != KWOK_OK) ev.reserved0 = (uint8_t)(int8_t)(listed ? KWOK_EINVAL : status);
    }
    side.status = status;
    A.ev[i] = ev;
    A.side[i] = side;
    if (status == JSON_HOST || status == JSON_SPEC || status == JSON_SPEC_X) A.host_list[atomicAdd(A.n_host, 1u)] = A.base + i;
}

void launch_json_pods(const JsonPodArgs& A, hipStream_t st) {
    if (!A.n) return;
    const uint32_t bs = json_block(A.n);
    hipLaunchKernelGGL(k_json_pods, dim3((A.n + bs - 1) / bs), dim3(bs), 0, st, A);
}

// ---------------------------------------------------------------------------
// the node document (kwok_decode_node, codec.cpp): WatchNodes / ListNodes'
// routing facts (node_controller.go:206-223, 256-270) - needHeartbeat = the
// node selector (controller.go:81-98: all nodes, an annotation selector or a
// label selector), needLockNode = not disregarded (empty label maps never
// match) - and the A.5 inputs configureNode reads (node_controller.go:356-391):
// status.phase, the ten nodeInfo strings and the addresses / allocatable /
// capacity blobs.  Those blobs are re-serialised canonically by the host codec
// (`YAML . 1` echoes, node.status.tpl): a document holding a non-empty one is
// listed for the host (JSON_HOST), as is any string the scan would have to
// compare as decoded text (an escaped routed key, label key or compared value).
// kwok's own fleets create Nodes with an empty status: none of them is listed.
// ---------------------------------------------------------------------------
enum : uint8_t {
    N_NONE = 0, N_ROOT, N_META, N_STATUS, N_NAME, N_ANN, N_LAB, N_ANNV, N_LABV, N_PHASE, N_ADDR, N_ALLOC, N_CAP,
    N_INFO, N_INFOV,
};
struct NodeScan {
    JRd* r;
    const JsonCfg* cfg;
    uint64_t cx = 0;
    uint8_t next = N_NONE;
    uint8_t info_k = 0;   // the nodeInfo key the next value belongs to
    int err = 0;          // KWOK_EDOMAIN
    bool host = false;    // JSON_HOST
    bool root_obj = false, meta_obj = false;
    bool skip_status = false;  // a Deleted event: its status is not read (node_controller.go:265-269: the name only)
    uint32_t seen_root = 0, seen_meta = 0, seen_status = 0, seen_info = 0;
    Span name{0, 0};
    uint32_t n_ann = 0, n_lab = 0;
    uint32_t km_man = 0, km_dis = 0;  // the current entry's key: requirements of the manage / disregard selector
    SelState man{0, 0}, dis_a{0, 0}, dis_l{0, 0};
    uint8_t phase = KWOK_PHASE_NONE;
    Span info[KWOK_NI_COUNT];

    __device__ uint8_t ctx(int d) const { return d < XD ? (uint8_t)(cx >> (8 * d)) : N_NONE; }
    __device__ void set_ctx(int d, uint8_t c) {
        if (d < XD) cx = (cx & ~(0xFFull << (8 * d))) | ((uint64_t)c << (8 * d));
    }
    __device__ uint8_t first(uint32_t& seen, int bit, uint8_t c) {
        if (seen & (1u << bit)) return N_NONE;
        seen |= 1u << bit;
        return c;
    }
    __device__ bool k_is(const JTok& t, const char* s, uint32_t n) {
        if (t.len != n) return false;
        for (uint32_t q = 0; q < n; q++)
            if (r->at(t.off + q) != (uint8_t)s[q]) return false;
        return true;
    }
    // the selector that decides `managed` over this label map (null: none does)
    __device__ const JsonSel* man_sel(bool ann) const {
        if (cfg->manage_all) return nullptr;
        if (cfg->man_ann.set) return ann ? &cfg->man_ann : nullptr;
        return ann ? nullptr : &cfg->man_lab;
    }
    __device__ uint32_t key_reqs(const JsonSel* S, const JTok& t) {
        uint32_t m = 0;
        if (!S || !S->set) return 0;
        for (uint32_t q = 0; q < S->nreq; q++)
            if (bytes_eq(*r, t.off, t.len, cfg->bytes + S->key_off[q], S->key_len[q])) m |= 1u << q;
        return m;
    }
    __device__ void sel_value(const JsonSel* S, SelState& st, uint32_t km, const JTok& t) {
        for (uint32_t q = 0; q < S->nreq; q++) {  // the last entry of a key wins (a Go map)
            if (!((km >> q) & 1)) continue;
            bool in = false;
            for (uint32_t v = 0; v < S->val_n[q]; v++) {
                const uint32_t vi = S->val_first[q] + v;
                in |= bytes_eq(*r, t.off, t.len, cfg->bytes + S->val_off[vi], S->val_len[vi]);
            }
            st.has |= 1u << q;
            st.in = in ? st.in | (1u << q) : st.in & ~(1u << q);
        }
    }
#define KIS(lit) k_is(t, lit, sizeof(lit) - 1)
    __device__ void key(int d, const JTok& t) {
        const uint8_t c = ctx(d);
        next = N_NONE;
        if (c == N_NONE) return;
        if (c == N_ANN || c == N_LAB) {  // a label / annotation entry
            const bool ann = c == N_ANN;
            if (ann) n_ann++;  // (no reference picked by a condition: the scan's state stays in registers)
            else n_lab++;
            next = ann ? N_ANNV : N_LABV;
            const JsonSel* M = man_sel(ann);
            const JsonSel* D = ann ? &cfg->dis_ann : &cfg->dis_lab;
            const bool any = (M && M->set && M->nreq) || (D->set && D->nreq);
            km_man = km_dis = 0;
            if (!any) return;
            if (t.esc) {
                host = true;
                return;
            }
            km_man = key_reqs(M, t);
            km_dis = key_reqs(D, t);
            return;
        }
        if (t.esc) {  // a routed key whose decoded text the scan does not compare
            if (c == N_ROOT || c == N_META || c == N_STATUS || c == N_INFO) host = true;
            return;
        }
        switch (c) {
            case N_ROOT:
                if (KIS("metadata")) next = first(seen_root, 0, N_META);
                else if (KIS("status") && !skip_status) next = first(seen_root, 1, N_STATUS);
                break;
            case N_META:
                if (KIS("name")) next = first(seen_meta, 0, N_NAME);
                else if (KIS("annotations")) next = first(seen_meta, 1, N_ANN);
                else if (KIS("labels")) next = first(seen_meta, 2, N_LAB);
                break;
            case N_STATUS:
                if (KIS("phase")) next = first(seen_status, 0, N_PHASE);
                else if (KIS("addresses")) next = first(seen_status, 1, N_ADDR);
                else if (KIS("allocatable")) next = first(seen_status, 2, N_ALLOC);
                else if (KIS("capacity")) next = first(seen_status, 3, N_CAP);
                else if (KIS("nodeInfo")) next = first(seen_status, 4, N_INFO);
                break;
            case N_ALLOC:
            case N_CAP:
                host = true;  // a non-empty blob: its canonical form is the host codec's
                break;
            case N_INFO: {  // codec.cpp nik[], KWOK_NI_* order
#define NI(i, lit) else if (KIS(lit)) { next = first(seen_info, i, N_INFOV); info_k = i; }
                if (false) {}
                NI(0, "architecture") NI(1, "bootID") NI(2, "containerRuntimeVersion") NI(3, "kernelVersion")
                NI(4, "kubeProxyVersion") NI(5, "kubeletVersion") NI(6, "machineID") NI(7, "operatingSystem")
                NI(8, "osImage") NI(9, "systemUUID")
#undef NI
                break;
            }
            default:
                break;
        }
    }
#undef KIS
    __device__ uint8_t value_ctx(int d, bool pa) const { return d == 0 ? N_ROOT : pa ? N_NONE : next; }
    __device__ void ref(const JTok& t, Span& out) {  // codec.cpp ref
        if (t.kind == J_NULL) return;
        if (t.kind != J_STR || t.esc) {
            err = KWOK_EDOMAIN;
            return;
        }
        if (t.len) out = Span{(uint32_t)t.off, t.len};
    }
    __device__ void scalar(int d, const JTok& t, bool pa) {
        const uint8_t c = value_ctx(d, pa);
        if (d == 0) return;
        if (pa && ctx(d - 1) == N_ADDR) host = true;  // a non-empty addresses list (canonical: the host codec's)
        switch (c) {
            case N_META: err = KWOK_EDOMAIN; break;  // metadata must be an object (null included)
            case N_NAME: ref(t, name); break;
            case N_ANN:
            case N_LAB:
                if (t.kind != J_NULL) err = KWOK_EDOMAIN;  // a label map: an object or null
                break;
            case N_ANNV:
            case N_LABV: {
                if (t.kind != J_STR) {
                    err = KWOK_EDOMAIN;  // label / annotation values are strings
                    break;
                }
                if (!km_man && !km_dis) break;
                if (t.esc) {
                    host = true;
                    break;
                }
                const bool ann = c == N_ANNV;
                if (km_man) sel_value(man_sel(ann), man, km_man, t);
                if (km_dis) {
                    if (ann) sel_value(&cfg->dis_ann, dis_a, km_dis, t);
                    else sel_value(&cfg->dis_lab, dis_l, km_dis, t);
                }
                break;
            }
            case N_PHASE:
                if (t.kind == J_STR) {
                    if (t.esc) host = true;
                    else phase = !t.len ? KWOK_PHASE_NONE : lit_eq(*r, t.off, t.len, "Running") ? KWOK_PHASE_RUNNING
                                                                                                 : KWOK_PHASE_OTHER;
                }
                break;
            case N_ADDR:
            case N_ALLOC:
            case N_CAP:
                if (t.kind != J_NULL) err = KWOK_EDOMAIN;  // the wrong type
                break;
            case N_INFOV:  // (constant indices: an indexed span would keep the scan state in scratch)
                switch (info_k) {
                    case 0: ref(t, info[0]); break;
                    case 1: ref(t, info[1]); break;
                    case 2: ref(t, info[2]); break;
                    case 3: ref(t, info[3]); break;
                    case 4: ref(t, info[4]); break;
                    case 5: ref(t, info[5]); break;
                    case 6: ref(t, info[6]); break;
                    case 7: ref(t, info[7]); break;
                    case 8: ref(t, info[8]); break;
                    default: ref(t, info[9]); break;
                }
                break;
            default: break;
        }
    }
    __device__ void begin(int d, bool a, bool pa) {
        const uint8_t c = value_ctx(d, pa);
        uint8_t mine = N_NONE;
        if (d == 0) {
            root_obj = !a;
            set_ctx(0, a ? N_NONE : N_ROOT);
            return;
        }
        if (pa && ctx(d - 1) == N_ADDR) host = true;
        switch (c) {
            case N_META: if (a) err = KWOK_EDOMAIN; else mine = N_META, meta_obj = true; break;
            case N_STATUS: if (!a) mine = N_STATUS; break;  // (a status that is no object is ignored)
            case N_NAME: case N_ANNV: case N_LABV: case N_INFOV: err = KWOK_EDOMAIN; break;  // strings
            case N_ANN: case N_LAB: if (a) err = KWOK_EDOMAIN; else mine = c; break;
            case N_ADDR: if (!a) err = KWOK_EDOMAIN; else mine = c; break;
            case N_ALLOC: case N_CAP: if (a) err = KWOK_EDOMAIN; else mine = c; break;
            case N_INFO: if (!a) mine = N_INFO; break;  // (ignored unless an object)
            default: break;
        }
        set_ctx(d, mine);
    }
    __device__ void end(int, bool, bool) {}  // (a blob was listed at its first member; an empty one is absent)
    __device__ bool matches(const JsonSel& S, const SelState& st) const {
        for (uint32_t q = 0; q < S.nreq; q++) {
            const bool has = (st.has >> q) & 1, in = (st.in >> q) & 1;
            switch (S.op[q]) {
                case JREQ_IN: if (!in) return false; break;
                case JREQ_NOTIN: if (in) return false; break;
                case JREQ_EXISTS: if (!has) return false; break;
                default: if (has) return false; break;
            }
        }
        return true;
    }
};

// one thread per node document; op[i]: the caller's watch event (the record's op)
__global__ __launch_bounds__(256) void k_json_nodes(JsonNodeArgs A) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= A.n) return;
    const uint64_t off = A.doc_off[i];
    const uint32_t len = A.doc_len[i];
    kwok_node_event ev;
    ev.op = A.op[i];
    ev.managed = ev.lockable = 0;
    ev.phase = KWOK_PHASE_NONE;
    ev.name = ev.addresses = ev.allocatable = ev.capacity = kwok_str{0, 0};
    for (int k = 0; k < KWOK_NI_COUNT; k++) ev.node_info[k] = kwok_str{0, 0};
    int32_t status;
    NodeScan p;
    for (int k = 0; k < KWOK_NI_COUNT; k++) p.info[k] = Span{0, 0};
    if (off > A.arena_len || len > A.arena_len - off) {
        status = KWOK_EINVAL;  // (codec.cpp parse_doc: a span outside the arena)
    } else if (A.cfg->all_host) {
        status = JSON_HOST;
    } else {
        JRd rd{A.arena, (jpos)off, (jpos)(off + len), ~0u, make_uint4(0, 0, 0, 0)};
        p.r = &rd;
        p.cfg = A.cfg;
        p.skip_status = ev.op == KWOK_OP_DELETE;
        const bool ok = jparse(rd, p);
        // (a document the scan routed past an escaped key may hold errors the host's
        // first-key lookup does not see: the host decides it, errors included)
        if (!ok || !p.root_obj) status = KWOK_EDOMAIN;
        else if (p.host) status = JSON_HOST;
        else if (p.err) status = p.err;
        else if (!p.meta_obj || !p.name.len) status = KWOK_EDOMAIN;
        else status = KWOK_OK;
        if (status == KWOK_OK) {
            const JsonCfg& C = *A.cfg;
            ev.managed = C.manage_all ? 1 : C.man_ann.set ? (p.matches(C.man_ann, p.man) ? 1 : 0)
                                                           : (C.man_lab.set && p.matches(C.man_lab, p.man) ? 1 : 0);
            const bool disregard = (C.dis_ann.set && p.n_ann && p.matches(C.dis_ann, p.dis_a)) ||
                                   (C.dis_lab.set && p.n_lab && p.matches(C.dis_lab, p.dis_l));
            ev.lockable = disregard ? 0 : 1;
            ev.phase = p.phase;
            ev.name = kwok_str{p.name.off, p.name.len};
            for (int k = 0; k < KWOK_NI_COUNT; k++) ev.node_info[k] = kwok_str{p.info[k].off, p.info[k].len};
        }
    }
    if (status != KWOK_OK) ev.op = 0xFF;  // (not applied: the host completes it, or its status is the decode's)
    A.ev[i] = ev;
    A.status[i] = status;
    if (status == JSON_HOST) A.host_list[atomicAdd(A.n_host, 1u)] = A.base + i;
}

void launch_json_nodes(const JsonNodeArgs& A, hipStream_t st) {
    if (!A.n) return;
    const uint32_t bs = json_block(A.n);
    hipLaunchKernelGGL(k_json_nodes, dim3((A.n + bs - 1) / bs), dim3(bs), 0, st, A);
}

// node records of a batch gathered for the host (list[k] -> out[k]) / written back (in[k] -> list[k])
__global__ void k_node_gather(const kwok_node_event* ev, const uint32_t* list, uint32_t n, kwok_node_event* out) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) out[k] = ev[list[k]];
}
__global__ void k_node_scatter(kwok_node_event* ev, const kwok_node_event* in, const uint32_t* list, uint32_t n) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) ev[list[k]] = in[k];
}
void launch_node_gather(const kwok_node_event* ev, const uint32_t* list, uint32_t n, kwok_node_event* out, hipStream_t st) {
    if (n) hipLaunchKernelGGL(k_node_gather, dim3((n + 255) / 256), dim3(256), 0, st, ev, list, n, out);
}
void launch_node_scatter(kwok_node_event* ev, const kwok_node_event* in, const uint32_t* list, uint32_t n, hipStream_t st) {
    if (n) hipLaunchKernelGGL(k_node_scatter, dim3((n + 255) / 256), dim3(256), 0, st, ev, in, list, n);
}

}  // namespace kwok

namespace kwok {
// the listed documents' records and sides, compacted for the host (json_complete)
__global__ void k_json_gather(const kwok_pod_event* ev, const JsonPodSide* side, const uint32_t* list, uint32_t n,
                              kwok_pod_event* out_ev, JsonPodSide* out_side) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out_ev[i] = ev[list[i]];
    out_side[i] = side[list[i]];
}
// ... and the host's completed records back in place
__global__ void k_json_scatter(kwok_pod_event* ev, const kwok_pod_event* in, const uint32_t* list, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ev[list[i]] = in[i];
}
void launch_json_gather(const kwok_pod_event* ev, const JsonPodSide* side, const uint32_t* list, uint32_t n,
                        kwok_pod_event* out_ev, JsonPodSide* out_side, hipStream_t st) {
    if (n) hipLaunchKernelGGL(k_json_gather, dim3((n + 255) / 256), dim3(256), 0, st, ev, side, list, n, out_ev, out_side);
}
void launch_json_scatter(kwok_pod_event* ev, const kwok_pod_event* in, const uint32_t* list, uint32_t n, hipStream_t st) {
    if (n) hipLaunchKernelGGL(k_json_scatter, dim3((n + 255) / 256), dim3(256), 0, st, ev, in, list, n);
}
}  // namespace kwok
