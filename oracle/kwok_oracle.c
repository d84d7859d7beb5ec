/*
 * kwok_oracle.c - CPU ORACLE (test infrastructure only; never linked into or
 * called by the product).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg load it, as the checker / the CPU baseline.
 *
 * A plain, sequential C restatement of the reference's per-tick controller
 * work (hezhizhen/kwok, paths relative to the reference repo root):
 *   - ipPool Get/Put/Use/new            pkg/kwok/controllers/utils.go:52-117, addIP :37-50
 *   - heartbeat patch                   node_controller.go:145-204,393-401 + templates/node.heartbeat.tpl
 *   - node lock / init patch + A.5 test node_controller.go:301-391          + templates/node.status.tpl
 *   - pod lock / patch + A.4 test       pod_controller.go:205-250,377-439    + templates/pod.status.tpl
 *   - pod delete / finalizers / release pod_controller.go:155-202,306-343
 *   - event routing                     node_controller.go:256-270, pod_controller.go:301-343
 * rendered the way renderer.go:49-89 + sigs.k8s.io/yaml + encoding/json do
 * for the default templates (sorted keys, compact, HTML-escaped strings).
 * It uses its own data structures (string-keyed-equivalent hash sets for the
 * pool, linear scans, libc gmtime_r/snprintf for formatting) and shares only
 * the event record layout (include/kwok_engine.h) with the product.
 *
 * Parity pinning: this file is checked against the tests/golden JSON fixtures, which
 * tests/golden/make_golden.py derives by executing the reference's own .tpl
 * files through an independent text/template + YAML->JSON interpreter and the
 * reference's renderer_test.go known answers (see DESIGN.md "Oracle").
 *
 * Deterministic choices where the reference is nondeterministic (DESIGN.md
 * "Tick contract"): ipPool.Get reuses the LOWEST usable address (reference:
 * random map order, utils.go:87-91); events are coalesced per tick; pods are
 * evaluated and IPs assigned in canonical handle order.
 */
#include "kwok_oracle.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#define OMP_TID() omp_get_thread_num()
#else
#define OMP_TID() 0
#endif

/* ------------------------------------------------------------------------- */
/* small utilities                                                             */
/* ------------------------------------------------------------------------- */
typedef struct {
    char* p;
    size_t n, cap;
} buf_t;

static void buf_put(buf_t* b, const char* s, size_t n) {
    if (b->n + n + 1 > b->cap) {
        size_t c = b->cap ? b->cap : 4096;
        while (c < b->n + n + 1) c *= 2;
        b->p = (char*)realloc(b->p, c);
        b->cap = c;
    }
    memcpy(b->p + b->n, s, n);
    b->n += n;
    b->p[b->n] = 0;
}
static void buf_s(buf_t* b, const char* s) { buf_put(b, s, strlen(s)); }

/* encoding/json string encoding (HTML-safe, as json.Marshal) */
static void buf_jstr(buf_t* b, const char* s, size_t n) {
    static const char hex[] = "0123456789abcdef";
    buf_put(b, "\"", 1);
    for (size_t i = 0; i < n; i++) {
        unsigned char c = (unsigned char)s[i];
        if (c == '"') buf_s(b, "\\\"");
        else if (c == '\\') buf_s(b, "\\\\");
        else if (c == '\n') buf_s(b, "\\n");
        else if (c == '\r') buf_s(b, "\\r");
        else if (c == '\t') buf_s(b, "\\t");
        else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
            char u[6] = {'\\', 'u', '0', '0', hex[c >> 4], hex[c & 15]};
            buf_put(b, u, 6);
        } else buf_put(b, (const char*)&c, 1);
    }
    buf_put(b, "\"", 1);
}

static char* xstrndup(const char* s, size_t n) {
    char* r = (char*)malloc(n + 1);
    memcpy(r, s, n);
    r[n] = 0;
    return r;
}

/* time.Format(time.RFC3339) of a UTC time (metav1.Time marshals UTC). */
static void rfc3339(int64_t t, char out[32]) {
    time_t tt = (time_t)t;
    struct tm tm;
    gmtime_r(&tt, &tm);
    strftime(out, 32, "%Y-%m-%dT%H:%M:%SZ", &tm);
}

/* net.IP.String() of an IPv4 address */
static void ip_str(uint32_t ip, char out[16]) {
    snprintf(out, 16, "%u.%u.%u.%u", ip >> 24, (ip >> 16) & 255, (ip >> 8) & 255, ip & 255);
}

/* net.ParseIP (Go 1.19) of a dotted quad: four decimal fields 0..255 split by
 * single dots, no leading zeros (rejected since Go 1.17), nothing else.
 * Returns 0 on failure / empty.  IPv6 forms are outside the supported domain. */
static int ip_parse(const char* s, size_t n, uint32_t* out) {
    uint32_t v = 0;
    size_t i = 0;
    for (int field = 0; field < 4; field++) {
        if (field) {
            if (i >= n || s[i] != '.') return 0;
            i++;
        }
        size_t d = 0;
        uint32_t x = 0;
        while (i + d < n && s[i + d] >= '0' && s[i + d] <= '9' && d < 4) x = x * 10 + (uint32_t)(s[i + d++] - '0');
        if (d == 0 || d > 3 || x > 255 || (d > 1 && s[i] == '0')) return 0;
        v = v << 8 | x;
        i += d;
    }
    if (i != n) return 0;
    *out = v;
    return 1;
}

/* ------------------------------------------------------------------------- */
/* supported input domain: the engine rejects what it cannot   */
/* emit verbatim, and so does this oracle (KWOK_EDOMAIN)                     */
/* ------------------------------------------------------------------------- */
/* Does `v`, rendered as `key: {{ . }}` into the template's YAML, come back out
 * of sigs.k8s.io/yaml (over gopkg.in/yaml.v2 v2.4.0 resolve.go, [ext]) as the
 * same JSON string?  One plain scalar: alnum first, [A-Za-z0-9._/:@+-] and
 * spaces, no ": ", no trailing ':' / space.  Resolves to !!str: not a bool/null
 * spelling of resolveMap; a digit-led value, '_' removed, is neither an integer
 * literal (0x / 0o / 0b / decimal digits: ParseInt/ParseUint base 0) nor a
 * yamlStyleFloat (out-of-range literals are rejected as well). */
static int yaml_plain_string(const char* v, size_t n) {
    static const char* const resolve_map[] = {"y", "Y", "yes", "Yes", "YES", "true", "True", "TRUE", "on", "On", "ON",
                                              "n", "N", "no", "No", "NO", "false", "False", "FALSE", "off", "Off", "OFF",
                                              "null", "Null", "NULL"};
    if (n < 1 || n > 253) return 0;
    for (size_t i = 0; i < n; i++) {
        char c = v[i];
        int ok = (c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c && strchr("._/:@+- ", c));
        if (!ok) return 0;
        if (i == 0 && !((c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z'))) return 0;
        if (c == ':' && (i + 1 == n || v[i + 1] == ' ')) return 0;
    }
    if (v[n - 1] == ' ') return 0;
    for (size_t k = 0; k < sizeof(resolve_map) / sizeof(resolve_map[0]); k++)
        if (strlen(resolve_map[k]) == n && memcmp(resolve_map[k], v, n) == 0) return 0;
    if (v[0] < '0' || v[0] > '9') return 1;
    char p[256];
    size_t m = 0;
    for (size_t i = 0; i < n; i++)
        if (v[i] != '_') p[m++] = v[i];
    p[m] = 0;
    /* integer literals */
    const char* digits = "0123456789";
    size_t from = 0;
    if (m > 2 && p[0] == '0' && (p[1] == 'x' || p[1] == 'X')) digits = "0123456789abcdefABCDEF", from = 2;
    else if (m > 2 && p[0] == '0' && (p[1] == 'o' || p[1] == 'O')) digits = "01234567", from = 2;
    else if (m > 2 && p[0] == '0' && (p[1] == 'b' || p[1] == 'B')) digits = "01", from = 2;
    if (from < m && strspn(p + from, digits) == m - from) return 0;
    /* yamlStyleFloat, digit-led: [0-9]+(\.[0-9]*)?([eE][-+]?[0-9]+)? */
    size_t i = strspn(p, "0123456789");
    if (p[i] == '.') i += 1 + strspn(p + i + 1, "0123456789");
    if (p[i] == 'e' || p[i] == 'E') {
        size_t j = i + 1 + (p[i + 1] == '+' || p[i + 1] == '-');
        size_t d = strspn(p + j, "0123456789");
        if (d) i = j + d;
    }
    return p[i] != 0; /* the whole value matched: a float */
}

/* status.addresses / allocatable / capacity as compact JSON (json.Marshal of
 * the object): a list / an object without control characters */
static int json_blob_ok(const char* s, size_t n, char open) {
    if (n < 2 || s[0] != open || s[n - 1] != (open == '[' ? ']' : '}')) return 0;
    for (size_t i = 0; i < n; i++)
        if ((unsigned char)s[i] < 0x20) return 0;
    return 1;
}

static uint32_t fnv1a32(const char* s, size_t n) {
    uint32_t h = 0x811C9DC5u;
    for (size_t i = 0; i < n; i++) {
        h ^= (unsigned char)s[i];
        h *= 0x01000193u;
    }
    return h;
}

/* ------------------------------------------------------------------------- */
/* ipPool (utils.go:52-117).  used/usable are sets of addresses; the          */
/* reference keys them by the dotted string, which is 1:1 with the address.  */
/* ------------------------------------------------------------------------- */
typedef struct {
    uint64_t* keys; /* 0 = empty, 1 = tombstone, addr+2 otherwise */
    size_t cap, n, live;
} hset_t;

static size_t hs_slot(const hset_t* h, uint64_t k) { return (size_t)((k * 0x9E3779B97F4A7C15ull) >> 17) & (h->cap - 1); }
static int hs_has(const hset_t* h, uint64_t a) {
    if (!h->cap) return 0;
    uint64_t k = a + 2;
    for (size_t i = hs_slot(h, k);; i = (i + 1) & (h->cap - 1)) {
        if (h->keys[i] == 0) return 0;
        if (h->keys[i] == k) return 1;
    }
}
static void hs_add(hset_t* h, uint64_t a);
static void hs_grow(hset_t* h) {
    hset_t nh = {0};
    nh.cap = h->cap ? h->cap * 2 : 64;
    while (nh.cap < 4 * (h->live + 1)) nh.cap *= 2;
    nh.keys = (uint64_t*)calloc(nh.cap, sizeof(uint64_t));
    for (size_t i = 0; i < h->cap; i++)
        if (h->keys[i] > 1) hs_add(&nh, h->keys[i] - 2);
    free(h->keys);
    *h = nh;
}
static void hs_add(hset_t* h, uint64_t a) {
    if (hs_has(h, a)) return;
    if (2 * (h->n + 1) > h->cap) hs_grow(h);
    uint64_t k = a + 2;
    size_t i = hs_slot(h, k);
    while (h->keys[i] > 1) i = (i + 1) & (h->cap - 1);
    if (h->keys[i] == 0) h->n++;
    h->keys[i] = k;
    h->live++;
}
static void hs_del(hset_t* h, uint64_t a) {
    if (!h->cap) return;
    uint64_t k = a + 2;
    for (size_t i = hs_slot(h, k);; i = (i + 1) & (h->cap - 1)) {
        if (h->keys[i] == 0) return;
        if (h->keys[i] == k) {
            h->keys[i] = 1;
            h->live--;
            return;
        }
    }
}

typedef struct {
    uint32_t base;       /* parseCIDR keeps the host address of the CIDR string (utils.go:28-35) */
    uint32_t net, mask;  /* ipnet.Mask */
    uint64_t index;      /* ipPool.index */
    hset_t used, usable; /* ipPool.used / ipPool.usable */
    /* min-heap over usable (lazy deletion) for the lowest-address reuse rule */
    uint64_t* heap;
    size_t hn, hcap;
} pool_t;

static int cidr_contains(const pool_t* p, uint64_t a) { return a <= 0xFFFFFFFFull && ((uint32_t)a & p->mask) == p->net; }

static void heap_push(pool_t* p, uint64_t a) {
    if (p->hn == p->hcap) {
        p->hcap = p->hcap ? p->hcap * 2 : 64;
        p->heap = (uint64_t*)realloc(p->heap, p->hcap * sizeof(uint64_t));
    }
    size_t i = p->hn++;
    p->heap[i] = a;
    while (i && p->heap[(i - 1) / 2] > p->heap[i]) {
        uint64_t t = p->heap[i];
        p->heap[i] = p->heap[(i - 1) / 2];
        p->heap[(i - 1) / 2] = t;
        i = (i - 1) / 2;
    }
}
static uint64_t heap_pop(pool_t* p) {
    uint64_t top = p->heap[0];
    p->heap[0] = p->heap[--p->hn];
    size_t i = 0;
    for (;;) {
        size_t l = 2 * i + 1, r = l + 1, m = i;
        if (l < p->hn && p->heap[l] < p->heap[m]) m = l;
        if (r < p->hn && p->heap[r] < p->heap[m]) m = r;
        if (m == i) break;
        uint64_t t = p->heap[i];
        p->heap[i] = p->heap[m];
        p->heap[m] = t;
        i = m;
    }
    return top;
}
static void usable_add(pool_t* p, uint64_t a) {
    if (!hs_has(&p->usable, a)) {
        hs_add(&p->usable, a);
        heap_push(p, a);
    }
}

/* ipPool.new (utils.go:68-81): sequential from base, skip addresses in used */
static uint64_t pool_new(pool_t* p) {
    for (;;) {
        uint64_t ip = (uint64_t)p->base + p->index; /* addIP(cidr.IP, index) */
        p->index++;
        if (hs_has(&p->used, ip)) continue;
        hs_add(&p->used, ip);
        usable_add(p, ip);
        return ip;
    }
}
/* ipPool.Get (utils.go:83-98) with the lowest-usable-first reuse rule */
static uint64_t pool_get(pool_t* p) {
    uint64_t ip = 0;
    int have = 0;
    while (p->usable.live && p->hn) {
        uint64_t a = heap_pop(p);
        if (hs_has(&p->usable, a)) {
            ip = a;
            have = 1;
            break;
        }
    }
    if (!have) ip = pool_new(p);
    hs_del(&p->usable, ip);
    hs_add(&p->used, ip);
    return ip;
}
/* ipPool.Put (utils.go:100-108) */
static void pool_put(pool_t* p, uint64_t ip) {
    if (!cidr_contains(p, ip)) return;
    hs_del(&p->used, ip);
    usable_add(p, ip);
}
/* ipPool.Use (utils.go:110-117) */
static void pool_use(pool_t* p, uint64_t ip) {
    if (!cidr_contains(p, ip)) return;
    hs_add(&p->used, ip);
}

/* ------------------------------------------------------------------------- */
/* engine state                                                                */
/* ------------------------------------------------------------------------- */
typedef struct {
    int used, exists, managed, lockable, event_lock, conforms, refs, phase;
    char* name;
    size_t name_len;
    char* addresses;   /* compact JSON or NULL */
    char* allocatable;
    char* capacity;
    char* info[KWOK_NI_COUNT];
} onode_t;

typedef struct {
    int used, disregard, deleting, status_nonempty, conforms, has_fin, phase, event, delete_pending;
    int32_t node, spec;
    int64_t creation;
    uint32_t host_ip, pod_ip;
} opod_t;

typedef struct {
    char** cname;
    char** cimage;
    uint32_t nc;
    char** iname;
    char** iimage;
    uint32_t ni;
    char** gates;
    uint32_t ng;
} ospec_t;

struct kwok_oracle {
    kwok_config cfg;
    char cidr[64], node_ip_s[16];
    uint32_t node_ip;
    uint32_t B, cn, cp, b_lo, b_hi;
    onode_t* nodes;
    opod_t* pods;
    ospec_t* specs;
    uint32_t n_specs;
    pool_t pool;
    char start_s[32];
    char err[256];
    /* outputs of the last tick */
    buf_t arena;
    int32_t *hb, *ini, *pp, *del;
    uint64_t *ini_off, *pp_off;
    uint32_t *ini_len, *pp_len;
    uint8_t* del_fin;
    uint32_t n_hb, n_ini, n_pp, n_del, hb_len;
    uint32_t hb_epoch; /* bumped when the managed set changes */
    int threads;       /* host threads of the tick's sweeps (kwok_oracle_set_threads) */
    uint64_t hb_off;
    int cni;           /* Config.EnableCNI: IPs from cni.Setup (kwok_oracle_cni_assign), no ipPool */
};

static int owns(const kwok_oracle* o, uint32_t b) { return b >= o->b_lo && b < o->b_hi; }

int kwok_oracle_create(const kwok_config* cfg, kwok_oracle** out) {
    *out = NULL;
    if (!cfg || cfg->abi_version != KWOK_ABI_VERSION || cfg->custom_templates) return KWOK_EINVAL;
    if (!cfg->buckets || (cfg->buckets & (cfg->buckets - 1)) || !cfg->node_slots_per_bucket || !cfg->pod_slots_per_bucket)
        return KWOK_EINVAL;
    int W = cfg->world_size > 0 ? cfg->world_size : 1;
    if (W > 1 && !cfg->allgather) return KWOK_EINVAL;
    kwok_oracle* o = (kwok_oracle*)calloc(1, sizeof(*o));
    o->cfg = *cfg;
    o->cni = cfg->enable_cni != 0;
    o->cfg.world_size = W;
    o->B = cfg->buckets;
    o->cn = cfg->node_slots_per_bucket;
    /* handles are bucket * stride + slot: the oracle holds every bucket at its
     * largest capacity (the engine grows to it) */
    o->cp = cfg->pod_handle_stride ? cfg->pod_handle_stride : cfg->pod_slots_per_bucket;
    o->b_lo = (uint32_t)((uint64_t)cfg->rank * o->B / W);
    o->b_hi = (uint32_t)((uint64_t)(cfg->rank + 1) * o->B / W);
    /* parseCIDR (utils.go:28-35): net.ParseCIDR, then ipnet.IP = the parsed host IP */
    const char* slash = strchr(cfg->cidr, '/');
    uint32_t base;
    if (!slash || !ip_parse(cfg->cidr, (size_t)(slash - cfg->cidr), &base)) {
        free(o);
        return KWOK_EDOMAIN;
    }
    int plen = atoi(slash + 1);
    if (plen < 0 || plen > 32) {
        free(o);
        return KWOK_EDOMAIN;
    }
    o->pool.mask = plen == 0 ? 0 : (uint32_t)(0xFFFFFFFFull << (32 - plen));
    o->pool.net = base & o->pool.mask;
    o->pool.base = base;
    if (!ip_parse(cfg->node_ip, strlen(cfg->node_ip), &o->node_ip)) {
        free(o);
        return KWOK_EDOMAIN;
    }
    ip_str(o->node_ip, o->node_ip_s);
    rfc3339(cfg->start_time_unix, o->start_s);
    o->nodes = (onode_t*)calloc((size_t)o->B * o->cn, sizeof(onode_t));
    o->pods = (opod_t*)calloc((size_t)o->B * o->cp, sizeof(opod_t));
    o->specs = (ospec_t*)calloc(cfg->max_pod_specs ? cfg->max_pod_specs : 1024, sizeof(ospec_t));
    *out = o;
    return KWOK_OK;
}

static void free_node_status(onode_t* n) {
    free(n->addresses);
    free(n->allocatable);
    free(n->capacity);
    n->addresses = n->allocatable = n->capacity = NULL;
    for (int i = 0; i < KWOK_NI_COUNT; i++) {
        free(n->info[i]);
        n->info[i] = NULL;
    }
}

void kwok_oracle_destroy(kwok_oracle* o) {
    if (!o) return;
    for (size_t i = 0; i < (size_t)o->B * o->cn; i++) {
        free_node_status(&o->nodes[i]);
        free(o->nodes[i].name);
    }
    for (uint32_t s = 0; s < o->n_specs; s++) {
        ospec_t* sp = &o->specs[s];
        for (uint32_t i = 0; i < sp->nc; i++) free(sp->cname[i]), free(sp->cimage[i]);
        for (uint32_t i = 0; i < sp->ni; i++) free(sp->iname[i]), free(sp->iimage[i]);
        for (uint32_t i = 0; i < sp->ng; i++) free(sp->gates[i]);
        free(sp->cname), free(sp->cimage), free(sp->iname), free(sp->iimage), free(sp->gates);
    }
    free(o->specs);
    free(o->nodes);
    free(o->pods);
    free(o->pool.used.keys);
    free(o->pool.usable.keys);
    free(o->pool.heap);
    free(o->arena.p);
    free(o->hb), free(o->ini), free(o->pp), free(o->del);
    free(o->ini_off), free(o->pp_off), free(o->ini_len), free(o->pp_len), free(o->del_fin);
    free(o);
}

const char* kwok_oracle_last_error(const kwok_oracle* o) { return o ? o->err : "null oracle"; }

static char* dupstr(const char* arena, kwok_str s) { return s.len ? xstrndup(arena + s.off, s.len) : NULL; }
static int streq(const char* a, const char* b) { return strcmp(a ? a : "", b ? b : "") == 0; }

int kwok_oracle_register_pod_spec(kwok_oracle* o, const kwok_pod_spec* s, const char* arena, size_t arena_len,
                                  int32_t* out_id) {
    /* every value pod.status.tpl renders with {{ . }} must stay a string */
#define SAFE(ks) ((size_t)(ks).off + (ks).len <= arena_len && yaml_plain_string(arena + (ks).off, (ks).len))
    for (uint32_t i = 0; i < s->n_containers; i++)
        if (!SAFE(s->containers[i].name) || !SAFE(s->containers[i].image)) return KWOK_EDOMAIN;
    for (uint32_t i = 0; i < s->n_init_containers; i++)
        if (!SAFE(s->init_containers[i].name) || !SAFE(s->init_containers[i].image)) return KWOK_EDOMAIN;
    for (uint32_t i = 0; i < s->n_readiness_gates; i++)
        if (!SAFE(s->readiness_gates[i])) return KWOK_EDOMAIN;
#undef SAFE
    ospec_t sp = {0};
    sp.nc = s->n_containers;
    sp.ni = s->n_init_containers;
    sp.ng = s->n_readiness_gates;
    sp.cname = (char**)calloc(sp.nc + 1, sizeof(char*));
    sp.cimage = (char**)calloc(sp.nc + 1, sizeof(char*));
    sp.iname = (char**)calloc(sp.ni + 1, sizeof(char*));
    sp.iimage = (char**)calloc(sp.ni + 1, sizeof(char*));
    sp.gates = (char**)calloc(sp.ng + 1, sizeof(char*));
    for (uint32_t i = 0; i < sp.nc; i++) {
        sp.cname[i] = xstrndup(arena + s->containers[i].name.off, s->containers[i].name.len);
        sp.cimage[i] = xstrndup(arena + s->containers[i].image.off, s->containers[i].image.len);
    }
    for (uint32_t i = 0; i < sp.ni; i++) {
        sp.iname[i] = xstrndup(arena + s->init_containers[i].name.off, s->init_containers[i].name.len);
        sp.iimage[i] = xstrndup(arena + s->init_containers[i].image.off, s->init_containers[i].image.len);
    }
    for (uint32_t i = 0; i < sp.ng; i++) sp.gates[i] = xstrndup(arena + s->readiness_gates[i].off, s->readiness_gates[i].len);
    /* dedupe */
    for (uint32_t k = 0; k < o->n_specs; k++) {
        ospec_t* t = &o->specs[k];
        int same = t->nc == sp.nc && t->ni == sp.ni && t->ng == sp.ng;
        for (uint32_t i = 0; same && i < sp.nc; i++) same = streq(t->cname[i], sp.cname[i]) && streq(t->cimage[i], sp.cimage[i]);
        for (uint32_t i = 0; same && i < sp.ni; i++) same = streq(t->iname[i], sp.iname[i]) && streq(t->iimage[i], sp.iimage[i]);
        for (uint32_t i = 0; same && i < sp.ng; i++) same = streq(t->gates[i], sp.gates[i]);
        if (same) {
            for (uint32_t i = 0; i < sp.nc; i++) free(sp.cname[i]), free(sp.cimage[i]);
            for (uint32_t i = 0; i < sp.ni; i++) free(sp.iname[i]), free(sp.iimage[i]);
            for (uint32_t i = 0; i < sp.ng; i++) free(sp.gates[i]);
            free(sp.cname), free(sp.cimage), free(sp.iname), free(sp.iimage), free(sp.gates);
            *out_id = (int32_t)k;
            return KWOK_OK;
        }
    }
    uint32_t cap = o->cfg.max_pod_specs ? o->cfg.max_pod_specs : 1024;
    if (o->n_specs >= cap) return KWOK_EFULL;
    o->specs[o->n_specs] = sp;
    *out_id = (int32_t)o->n_specs++;
    return KWOK_OK;
}

/* node entry lookup: entries live in bucket fnv1a32(name) & (B-1) */
static int32_t node_find(kwok_oracle* o, const char* name, size_t n) {
    uint32_t b = fnv1a32(name, n) & (o->B - 1);
    for (uint32_t i = 0; i < o->cn; i++) {
        onode_t* e = &o->nodes[(size_t)b * o->cn + i];
        if (e->used && e->name_len == n && memcmp(e->name, name, n) == 0) return (int32_t)(b * o->cn + i);
    }
    return -1;
}
static int32_t node_entry(kwok_oracle* o, const char* name, size_t n, int* st) {
    int32_t h = node_find(o, name, n);
    if (h >= 0) return h;
    uint32_t b = fnv1a32(name, n) & (o->B - 1);
    if (!owns(o, b)) {
        *st = KWOK_ENOTMINE;
        return -1;
    }
    for (uint32_t i = 0; i < o->cn; i++) {
        onode_t* e = &o->nodes[(size_t)b * o->cn + i];
        if (!e->used) {
            memset(e, 0, sizeof(*e));
            e->used = 1;
            e->name = xstrndup(name, n);
            e->name_len = n;
            return (int32_t)(b * o->cn + i);
        }
    }
    *st = KWOK_EFULL;
    return -1;
}
static void node_maybe_free(kwok_oracle* o, int32_t h) {
    onode_t* e = &o->nodes[h];
    if (!e->exists && e->refs == 0) {
        free_node_status(e);
        free(e->name);
        memset(e, 0, sizeof(*e));
    }
}

/* A.5: configureNode's merge is a no-op iff all template defaults are in place */
static int node_conforms(const onode_t* n) {
    const char* ni_arch = n->info[KWOK_NI_ARCHITECTURE];
    return n->addresses && n->allocatable && n->capacity && n->phase == KWOK_PHASE_RUNNING && ni_arch &&
           n->info[KWOK_NI_KUBE_PROXY_VERSION] && n->info[KWOK_NI_KUBELET_VERSION] &&
           n->info[KWOK_NI_OPERATING_SYSTEM] && streq(n->info[KWOK_NI_SYSTEM_UUID], n->info[KWOK_NI_OS_IMAGE]);
}

int kwok_oracle_ingest_nodes(kwok_oracle* o, const kwok_node_event* ev, size_t n, const char* arena, size_t arena_len,
                             int32_t* out_handles, int32_t* out_status) {
    (void)arena_len;
    int rejected = 0;
    for (size_t i = 0; i < n; i++) {
        const kwok_node_event* e = &ev[i];
        const char* name = arena + e->name.off;
        int st = KWOK_OK;
        int32_t h = -1;
        if (e->name.len == 0 || e->name.len > 253) {
            st = KWOK_EDOMAIN;
        } else if (e->op == KWOK_OP_DELETE) {
            /* node_controller.go:265-269: Deleted -> nodesSets.Delete */
            h = node_find(o, name, e->name.len);
            if (h < 0) {
                uint32_t b = fnv1a32(name, e->name.len) & (o->B - 1);
                st = owns(o, b) ? KWOK_ENOTFOUND : KWOK_ENOTMINE;
            } else {
                onode_t* nd = &o->nodes[h];
                if (nd->managed) o->hb_epoch++;
                nd->exists = nd->managed = nd->event_lock = 0;
                free_node_status(nd);
                node_maybe_free(o, h);
            }
        } else {
            /* node.status.tpl renders nodeInfo values with {{ . }} and echoes the
             * JSON of addresses / allocatable / capacity */
            for (int k = 0; k < KWOK_NI_COUNT && st == KWOK_OK; k++)
                if (e->node_info[k].len && !yaml_plain_string(arena + e->node_info[k].off, e->node_info[k].len))
                    st = KWOK_EDOMAIN;
            const kwok_str* blobs[3] = {&e->addresses, &e->allocatable, &e->capacity};
            for (int k = 0; k < 3 && st == KWOK_OK; k++)
                if (blobs[k]->len && !json_blob_ok(arena + blobs[k]->off, blobs[k]->len, k == 0 ? '[' : '{'))
                    st = KWOK_EDOMAIN;
            if (st == KWOK_OK) h = node_entry(o, name, e->name.len, &st);
            if (h >= 0) {
                onode_t* nd = &o->nodes[h];
                free_node_status(nd);
                nd->addresses = dupstr(arena, e->addresses);
                nd->allocatable = dupstr(arena, e->allocatable);
                nd->capacity = dupstr(arena, e->capacity);
                for (int k = 0; k < KWOK_NI_COUNT; k++) nd->info[k] = dupstr(arena, e->node_info[k]);
                nd->phase = e->phase;
                nd->exists = 1;
                /* node_controller.go:257-264: needHeartbeat -> Put; needLockNode -> lock */
                if (e->managed) {
                    if (!nd->managed) o->hb_epoch++;
                    nd->managed = 1;
                    if (e->lockable) nd->event_lock = 1;
                }
                nd->lockable = e->lockable ? 1 : 0;
                nd->conforms = node_conforms(nd);
            }
        }
        if (out_handles) out_handles[i] = h;
        if (out_status) out_status[i] = st;
        if (st != KWOK_OK) rejected++;
    }
    return rejected;
}

int kwok_oracle_ingest_pods(kwok_oracle* o, const kwok_pod_event* ev, size_t n, const char* arena, size_t arena_len,
                            int32_t* out_handles, int32_t* out_status, uint32_t* out_released) {
    (void)arena_len;
    int rejected = 0;
    for (size_t i = 0; i < n; i++) {
        const kwok_pod_event* e = &ev[i];
        int st = KWOK_OK;
        int32_t h = e->handle;
        if (out_released) out_released[i] = 0;
        if (e->op == KWOK_OP_DELETE) {
            if (h < 0) {
                st = KWOK_EINVAL; /* a Deleted event names an object the caller ingested */
            } else if ((uint32_t)h >= o->B * o->cp || !o->pods[h].used) {
                st = KWOK_ENOTFOUND; /* a rejected record carries no handle (as an update's) */
                h = -1;
            } else {
                opod_t* p = &o->pods[h];
                int32_t nh = p->node;
                uint32_t ip = 0;
                /* pod_controller.go:329-336: release the event's podIP if the node is managed
                 * (EnableCNI: cni.Remove on the caller's side, :337-342) */
                if (!o->cni && o->nodes[nh].managed && ip_parse(arena + e->pod_ip.off, e->pod_ip.len, &ip) &&
                    cidr_contains(&o->pool, ip)) {
                    pool_put(&o->pool, ip);
                    if (out_released) out_released[i] = ip;
                }
                memset(p, 0, sizeof(*p));
                o->nodes[nh].refs--;
                node_maybe_free(o, nh);
            }
        } else {
            opod_t* p;
            uint32_t hip = 0, pip = 0;
            if (h >= 0 && ((uint32_t)h >= o->B * o->cp || !o->pods[h].used)) {
                st = KWOK_ENOTFOUND;
                h = -1;
            } else if ((e->host_ip.len && (!ip_parse(arena + e->host_ip.off, e->host_ip.len, &hip) || !hip)) ||
                       (e->pod_ip.len && (!ip_parse(arena + e->pod_ip.off, e->pod_ip.len, &pip) || !pip))) {
                st = KWOK_EDOMAIN; /* IPv4 dotted quads only */
                h = -1;
            } else if (e->spec_id < 0 || (uint32_t)e->spec_id >= o->n_specs || e->phase > KWOK_PHASE_UNKNOWN) {
                st = KWOK_EINVAL;
                h = -1;
            } else if (e->creation_unix < 0 || e->creation_unix > 0xFFFFFFFFll) {
                st = KWOK_EDOMAIN; /* creationTimestamp between 1970 and 2106 */
                h = -1;
            } else if (h < 0) {
                int32_t nh;
                if (e->node_handle >= 0) {
                    nh = e->node_handle;
                    if ((uint32_t)nh < o->b_lo * o->cn || (uint32_t)nh >= o->b_hi * o->cn) nh = -1, st = KWOK_ENOTMINE;
                    else if (!o->nodes[nh].used) nh = -1, st = KWOK_ENOTFOUND;
                } else if (e->node_name.len == 0 || e->node_name.len > 253) nh = -1, st = KWOK_EDOMAIN;
                else nh = node_entry(o, arena + e->node_name.off, e->node_name.len, &st);
                if (nh >= 0) {
                    uint32_t b = (uint32_t)nh / o->cn;
                    h = -1;
                    for (uint32_t k = 0; k < o->cp; k++)
                        if (!o->pods[(size_t)b * o->cp + k].used) {
                            h = (int32_t)(b * o->cp + k);
                            break;
                        }
                    if (h < 0) {
                        st = KWOK_EFULL;
                        node_maybe_free(o, nh);
                    } else {
                        memset(&o->pods[h], 0, sizeof(opod_t));
                        o->pods[h].used = 1;
                        o->pods[h].node = nh;
                        o->nodes[nh].refs++;
                    }
                }
            }
            if (h >= 0) {
                p = &o->pods[h];
                p->disregard = !!(e->flags & KWOK_POD_DISREGARD);
                p->deleting = !!(e->flags & KWOK_POD_DELETING);
                p->status_nonempty = !!(e->flags & KWOK_POD_STATUS_NONEMPTY) || hip || pip; /* an IP is status */
                p->conforms = !!(e->flags & KWOK_POD_CONFORMS);
                p->has_fin = !!(e->flags & KWOK_POD_HAS_FINALIZERS);
                p->phase = e->phase;
                p->spec = e->spec_id;
                p->creation = e->creation_unix;
                p->host_ip = hip;
                p->pod_ip = pip;
                int managed = o->nodes[p->node].managed;
                if (p->deleting) {
                    if (managed) p->delete_pending = 1; /* pod_controller.go:306-308 */
                } else if (managed && !p->disregard) {
                    p->event = 1; /* needLockPod (:252-269) -> lockChan (:318-319) */
                }
            }
        }
        if (out_handles) out_handles[i] = h;
        if (out_status) out_status[i] = st;
        if (st != KWOK_OK) rejected++;
    }
    return rejected;
}

/* kwok_ingest_pods_packed: the compact records as the kwok_pod_event they stand
 * for (dotted quads of the IPs, the node by handle), through the event switch
 * above; a create without a node handle is not expressible (KWOK_EINVAL) */
int kwok_oracle_ingest_pods_packed(kwok_oracle* o, const kwok_pod_rec* recs, size_t n, int32_t* out_handles,
                                   int8_t* out_status, uint32_t* out_released) {
    kwok_pod_event* ev = (kwok_pod_event*)calloc(n + 1, sizeof(kwok_pod_event));
    char* ar = (char*)calloc(32 * n + 1, 1);
    int32_t* st = (int32_t*)calloc(n + 1, sizeof(int32_t));
    int32_t* hs = (int32_t*)calloc(n + 1, sizeof(int32_t));
    size_t* pre = (size_t*)calloc(n + 1, sizeof(size_t)); /* records sent before record i */
    size_t m = 0, off = 0;
    int bad = 0;
    if (!ev || !ar || !st || !hs || !pre) {
        free(ev), free(ar), free(st), free(hs), free(pre);
        return KWOK_ENOMEM;
    }
    for (size_t i = 0; i < n; i++) {
        const kwok_pod_rec* r = &recs[i];
        const int create = (r->op & KWOK_REC_NEW) != 0;
        pre[i] = m;
        if (create && r->target < 0) {
            st[i] = KWOK_EINVAL; /* not sent */
            continue;
        }
        st[i] = 1; /* sent: the status comes from the event switch */
        kwok_pod_event* e = &ev[m++];
        e->op = r->op & ~KWOK_REC_NEW;
        e->flags = r->flags & 31;
        e->phase = r->flags >> KWOK_REC_PHASE_SHIFT;
        e->spec_id = r->spec_id;
        e->handle = create ? -1 : r->target;
        e->node_handle = create ? r->target : -1;
        e->creation_unix = r->creation;
        uint32_t ips[2] = {r->host_ip, r->pod_ip};
        kwok_str* dst[2] = {&e->host_ip, &e->pod_ip};
        for (int k = 0; k < 2; k++) {
            if (!ips[k]) continue;
            const int len = sprintf(ar + off, "%u.%u.%u.%u", ips[k] >> 24, (ips[k] >> 16) & 255, (ips[k] >> 8) & 255,
                                    ips[k] & 255);
            dst[k]->off = (uint32_t)off;
            dst[k]->len = (uint32_t)len;
            off += (size_t)len;
        }
    }
    int32_t* st2 = (int32_t*)calloc(m + 1, sizeof(int32_t));
    uint32_t* rel = (uint32_t*)calloc(m + 1, sizeof(uint32_t));
    const int rc = st2 && rel ? kwok_oracle_ingest_pods(o, ev, m, ar, off, hs, st2, rel) : KWOK_ENOMEM;
    if (rc >= 0) {
        for (size_t i = 0; i < n; i++) {
            const int sent = st[i] == 1;
            const int code = sent ? st2[pre[i]] : st[i];
            if (out_status) out_status[i] = (int8_t)code;
            if (out_handles) out_handles[i] = sent ? hs[pre[i]] : -1;
            if (out_released) out_released[i] = sent ? rel[pre[i]] : 0;
            bad += code != KWOK_OK;
        }
    }
    free(ev), free(ar), free(st), free(hs), free(pre), free(st2), free(rel);
    return rc < 0 ? rc : bad;
}

/* kwok_ingest_pods_packed12: each record as the kwok_pod_rec it stands for
 * (KWOK_REC_HOST_NODE_IP: hostIP = the configured NodeIP; value: a create's
 * creationTimestamp, any other record's podIP, an update keeping the held pod's
 * creation time), through the packed path; the handles of the KWOK_REC_NEW
 * records only, in create order.  The creation time an update keeps is the
 * pod's when the update applies: the batch runs in pieces, cut before an update
 * of a handle the state does not hold yet (one created earlier in the batch). */
int kwok_oracle_ingest_pods_packed12(kwok_oracle* o, const kwok_pod_rec12* recs, size_t n, int32_t* out_new_handles,
                                     size_t new_cap, int8_t* out_status, uint32_t* out_released) {
    kwok_pod_rec* r = (kwok_pod_rec*)calloc(n + 1, sizeof(kwok_pod_rec));
    int32_t* hs = (int32_t*)calloc(n + 1, sizeof(int32_t));
    int8_t* st = (int8_t*)calloc(n + 1, 1);
    uint32_t* rel = (uint32_t*)calloc(n + 1, sizeof(uint32_t));
    if (!r || !hs || !st || !rel) {
        free(r), free(hs), free(st), free(rel);
        return KWOK_ENOMEM;
    }
    const size_t npods = (size_t)o->B * o->cp;
    int rc = 0, bad = 0;
    size_t run = 0;  /* the first record not yet applied */
    for (size_t i = 0; i <= n && rc >= 0; i++) {
        const int held_later = i < n && !(recs[i].op & KWOK_REC_NEW) &&
                               (recs[i].op & (uint8_t)~KWOK_REC_HOST_NODE_IP) == KWOK_OP_UPSERT &&
                               recs[i].target >= 0 && (size_t)recs[i].target < npods && !o->pods[recs[i].target].used;
        if ((i == n || held_later) && i > run) {  /* apply [run, i) */
            rc = kwok_oracle_ingest_pods_packed(o, r + run, i - run, hs + run, st + run, rel + run);
            if (rc >= 0) bad += rc;
            run = i;
        }
        if (i == n || rc < 0) break;
        const int nw = (recs[i].op & KWOK_REC_NEW) != 0;
        const int32_t h = recs[i].target;
        r[i].op = recs[i].op & (uint8_t)~KWOK_REC_HOST_NODE_IP;
        r[i].flags = recs[i].flags;
        r[i].spec_id = recs[i].spec_id;
        r[i].target = h;
        r[i].host_ip = (recs[i].op & KWOK_REC_HOST_NODE_IP) ? o->node_ip : 0;
        r[i].pod_ip = nw ? 0u : recs[i].value;
        r[i].creation = nw ? recs[i].value
                           : (h >= 0 && (size_t)h < npods && o->pods[h].used ? (uint32_t)o->pods[h].creation : 0u);
    }
    if (rc >= 0) {
        size_t k = 0;
        for (size_t i = 0; i < n; i++) {
            if (out_status) out_status[i] = st[i];
            if (out_released) out_released[i] = rel[i];
            if (recs[i].op & KWOK_REC_NEW) {
                if (k < new_cap) out_new_handles[k] = hs[i];
                k++;
            }
        }
        rc = k > new_cap ? KWOK_EINVAL : bad;
    }
    free(r), free(hs), free(st), free(rel);
    return rc;
}

static inline int keep_eval(const kwok_oracle* o, size_t h);
/* EnableCNI: the pods the next tick evaluates without a podIP (configurePod's
 * cni.Setup set, pod_controller.go:383-389), canonical order */
int kwok_oracle_cni_pending(kwok_oracle* o, int32_t* out, size_t cap, size_t* n_out) {
    if (!o->cni || !n_out) return KWOK_EINVAL;
    size_t n = 0;
    for (size_t h = 0; h < (size_t)o->B * o->cp; h++)
        if (!o->pods[h].delete_pending && keep_eval(o, h) && !o->pods[h].pod_ip) {
            if (n < cap) out[n] = (int32_t)h;
            n++;
        }
    *n_out = n;
    return n <= cap ? KWOK_OK : KWOK_EINVAL;
}
/* ... and the IPs cni.Setup returned: pod.Status.PodIP = ips[0] (:388) */
int kwok_oracle_cni_assign(kwok_oracle* o, const int32_t* handles, const uint32_t* ips, size_t n, int32_t* out_status) {
    if (!o->cni) return KWOK_EINVAL;
    int rejected = 0;
    for (size_t i = 0; i < n; i++) {
        int st = KWOK_OK;
        if (handles[i] < 0 || (uint32_t)handles[i] >= o->B * o->cp || !o->pods[handles[i]].used) st = KWOK_ENOTFOUND;
        else if (!ips[i]) st = KWOK_EDOMAIN;
        else {
            o->pods[handles[i]].pod_ip = ips[i];
            o->pods[handles[i]].status_nonempty = 1;
        }
        if (out_status) out_status[i] = st;
        rejected += st != KWOK_OK;
    }
    return rejected;
}

int kwok_oracle_pool_put(kwok_oracle* o, const uint32_t* ips, size_t n) {
    for (size_t i = 0; i < n; i++) pool_put(&o->pool, ips[i]);
    return KWOK_OK;
}

/* ------------------------------------------------------------------------- */
/* renderers: the default .tpl files -> YAML -> JSON, for the default templates       */
/* ------------------------------------------------------------------------- */
/* node.heartbeat.tpl:1-31: five conditions, keys in sorted JSON order */
static void render_conditions(buf_t* b, const char* now, const char* start) {
    static const char* c[5][4] = {
        {"kubelet is posting ready status", "KubeletReady", "True", "Ready"},
        {"kubelet has sufficient disk space available", "KubeletHasSufficientDisk", "False", "OutOfDisk"},
        {"kubelet has sufficient memory available", "KubeletHasSufficientMemory", "False", "MemoryPressure"},
        {"kubelet has no disk pressure", "KubeletHasNoDiskPressure", "False", "DiskPressure"},
        {"RouteController created a route", "RouteCreated", "False", "NetworkUnavailable"},
    };
    buf_s(b, "[");
    for (int i = 0; i < 5; i++) {
        if (i) buf_s(b, ",");
        buf_s(b, "{\"lastHeartbeatTime\":");
        buf_jstr(b, now, strlen(now));
        buf_s(b, ",\"lastTransitionTime\":");
        buf_jstr(b, start, strlen(start));
        buf_s(b, ",\"message\":");
        buf_jstr(b, c[i][0], strlen(c[i][0]));
        buf_s(b, ",\"reason\":");
        buf_jstr(b, c[i][1], strlen(c[i][1]));
        buf_s(b, ",\"status\":");
        buf_jstr(b, c[i][2], strlen(c[i][2]));
        buf_s(b, ",\"type\":");
        buf_jstr(b, c[i][3], strlen(c[i][3]));
        buf_s(b, "}");
    }
    buf_s(b, "]");
}

/* configureHeartbeatNode (node_controller.go:393-401) */
static void render_heartbeat(buf_t* b, const char* now, const char* start) {
    buf_s(b, "{\"status\":{\"conditions\":");
    render_conditions(b, now, start);
    buf_s(b, "}}");
}

/* configureNode patch (node_controller.go:356-391), node.status.tpl + "\n" + node.heartbeat.tpl */
static void render_node_init(kwok_oracle* o, buf_t* b, const onode_t* n, const char* now) {
    static const char* dflt[KWOK_NI_COUNT] = {"amd64", "", "", "", "fake", "fake", "", "linux", "", ""};
    static const char* key[KWOK_NI_COUNT] = {"architecture", "bootID", "containerRuntimeVersion", "kernelVersion",
                                             "kubeProxyVersion", "kubeletVersion", "machineID", "operatingSystem",
                                             "osImage", "systemUUID"};
    static const char* dres = "{\"cpu\":\"1k\",\"memory\":\"1Ti\",\"pods\":\"1M\"}";
    buf_s(b, "{\"status\":{\"addresses\":");
    if (n->addresses) buf_s(b, n->addresses); /* {{ YAML . 1 }} echo: JSON -> YAML -> JSON identity */
    else {
        buf_s(b, "[{\"address\":");
        buf_jstr(b, o->node_ip_s, strlen(o->node_ip_s));
        buf_s(b, ",\"type\":\"InternalIP\"}]");
    }
    buf_s(b, ",\"allocatable\":");
    buf_s(b, n->allocatable ? n->allocatable : dres);
    buf_s(b, ",\"capacity\":");
    buf_s(b, n->capacity ? n->capacity : dres);
    buf_s(b, ",\"conditions\":");
    render_conditions(b, now, o->start_s);
    /* `with .nodeInfo` is always true: NodeSystemInfo is a struct, never omitted */
    buf_s(b, ",\"nodeInfo\":{");
    for (int k = 0; k < KWOK_NI_COUNT; k++) {
        /* node.status.tpl:40: systemUUID is rendered from `with .osImage` */
        const char* v = n->info[k == KWOK_NI_SYSTEM_UUID ? KWOK_NI_OS_IMAGE : k];
        if (!v) v = dflt[k];
        if (k) buf_s(b, ",");
        buf_jstr(b, key[k], strlen(key[k]));
        buf_s(b, ":");
        buf_jstr(b, v, strlen(v));
    }
    buf_s(b, "},\"phase\":\"Running\"}}");
}

/* computePatchData render of pod.status.tpl (pod_controller.go:404-408) */
static void render_pod(kwok_oracle* o, buf_t* b, const opod_t* p, uint32_t pod_ip) {
    char st[32], ip[16];
    rfc3339(p->creation, st); /* $startTime := .metadata.creationTimestamp */
    const ospec_t* s = &o->specs[p->spec];
    buf_s(b, "{\"status\":{\"conditions\":[");
    static const char* ctypes[3] = {"Initialized", "Ready", "ContainersReady"};
    for (uint32_t i = 0; i < 3 + s->ng; i++) {
        const char* t = i < 3 ? ctypes[i] : s->gates[i - 3];
        if (i) buf_s(b, ",");
        buf_s(b, "{\"lastTransitionTime\":");
        buf_jstr(b, st, strlen(st));
        buf_s(b, ",\"status\":\"True\",\"type\":");
        buf_jstr(b, t, strlen(t));
        buf_s(b, "}");
    }
    buf_s(b, "],\"containerStatuses\":");
    if (!s->nc) buf_s(b, "null"); /* empty `range` leaves `containerStatuses:` -> null */
    else {
        buf_s(b, "[");
        for (uint32_t i = 0; i < s->nc; i++) {
            if (i) buf_s(b, ",");
            buf_s(b, "{\"image\":");
            buf_jstr(b, s->cimage[i], strlen(s->cimage[i]));
            buf_s(b, ",\"name\":");
            buf_jstr(b, s->cname[i], strlen(s->cname[i]));
            buf_s(b, ",\"ready\":true,\"restartCount\":0,\"state\":{\"running\":{\"startedAt\":");
            buf_jstr(b, st, strlen(st));
            buf_s(b, "}}}");
        }
        buf_s(b, "]");
    }
    if (p->status_nonempty) { /* {{ with .status }} hostIP / podIP */
        ip_str(p->host_ip ? p->host_ip : o->node_ip, ip);
        buf_s(b, ",\"hostIP\":");
        buf_jstr(b, ip, strlen(ip));
    }
    buf_s(b, ",\"initContainerStatuses\":");
    if (!s->ni) buf_s(b, "null");
    else {
        buf_s(b, "[");
        for (uint32_t i = 0; i < s->ni; i++) {
            if (i) buf_s(b, ",");
            buf_s(b, "{\"image\":");
            buf_jstr(b, s->iimage[i], strlen(s->iimage[i]));
            buf_s(b, ",\"name\":");
            buf_jstr(b, s->iname[i], strlen(s->iname[i]));
            buf_s(b, ",\"ready\":true,\"restartCount\":0,\"state\":{\"terminated\":{\"exitCode\":0,\"finishedAt\":");
            buf_jstr(b, st, strlen(st));
            buf_s(b, ",\"reason\":\"Completed\",\"startedAt\":");
            buf_jstr(b, st, strlen(st));
            buf_s(b, "}}}");
        }
        buf_s(b, "]");
    }
    buf_s(b, ",\"phase\":\"Running\"");
    if (p->status_nonempty) {
        ip_str(pod_ip, ip);
        buf_s(b, ",\"podIP\":");
        buf_jstr(b, ip, strlen(ip));
    }
    buf_s(b, ",\"startTime\":");
    buf_jstr(b, st, strlen(st));
    buf_s(b, "}}");
}

/* ------------------------------------------------------------------------- */
/* tick                                                                        */
/*                                                                             */
/* The per-object sweeps run on o->threads host threads (OpenMP, when built  */
/* with it; kwok_oracle_set_threads).  Every sweep splits its index range     */
/* into contiguous per-thread pieces whose results are concatenated in thread */
/* order, and everything order-dependent on shared state (DeletePod          */
/* bookkeeping, ipPool Use / Put / Get) stays sequential, so the outputs are  */
/* the same for any thread count (tests/test_oracle_golden.py).              */
/* ------------------------------------------------------------------------- */
typedef struct {
    uint32_t* v;
    size_t n, cap;
} u32vec;
static void vreserve(u32vec* a, size_t n) {
    if (a->n + n > a->cap) {
        size_t c = a->cap ? a->cap : 64;
        while (c < a->n + n) c *= 2;
        a->v = (uint32_t*)realloc(a->v, c * sizeof(uint32_t));
        a->cap = c;
    }
}
static void vpush(u32vec* a, uint32_t x) {
    vreserve(a, 1);
    a->v[a->n++] = x;
}

static int nthr(const kwok_oracle* o) { return o->threads > 0 ? o->threads : 1; }
int kwok_oracle_set_threads(kwok_oracle* o, int n) {
#ifdef _OPENMP
    o->threads = n > 0 ? n : omp_get_max_threads();
#else
    o->threads = 1;
    (void)n;
#endif
    return o->threads;
}

/* the indices i in [0, n) with KEEP(o, i), ascending (a macro: the predicate
 * is inlined into the sweep) */
#define PFILTER(o, n, KEEP, out)                                                  \
    do {                                                                          \
        const int T_ = nthr(o);                                                   \
        const size_t n_ = (n);                                                    \
        u32vec* part_ = (u32vec*)calloc((size_t)T_, sizeof(u32vec));              \
        _Pragma("omp parallel num_threads(T_)") {                                 \
            const int t_ = OMP_TID();                                             \
            for (size_t i_ = n_ * t_ / T_, hi_ = n_ * (t_ + 1) / T_; i_ < hi_; i_++) \
                if (KEEP(o, i_)) vpush(&part_[t_], (uint32_t)i_);                  \
        }                                                                         \
        pconcat(part_, T_, out);                                                  \
    } while (0)
static void pconcat(u32vec* part, int T, u32vec* out) {
    size_t tot = 0;
    for (int t = 0; t < T; t++) tot += part[t].n;
    vreserve(out, tot);
    for (int t = 0; t < T; t++) {
        memcpy(out->v + out->n, part[t].v, part[t].n * sizeof(uint32_t));
        out->n += part[t].n;
        free(part[t].v);
    }
    free(part);
}

/* LockNode set: heartbeat feedback (every managed lockable node) + event locks */
static int node_locked(const onode_t* n) { return n->used && n->exists && ((n->managed && n->lockable) || n->event_lock); }
static inline int keep_del(const kwok_oracle* o, size_t h) { return o->pods[h].used && o->pods[h].delete_pending; }
static inline int keep_lock(const kwok_oracle* o, size_t h) { return node_locked(&o->nodes[h]); }
static inline int keep_managed(const kwok_oracle* o, size_t h) { return o->nodes[h].used && o->nodes[h].managed; }
/* LockPods: lock events + LockPodsOnNode of every locked managed node */
static inline int keep_eval(const kwok_oracle* o, size_t h) {
    const opod_t* p = &o->pods[h];
    if (!p->used) return 0;
    const onode_t* n = &o->nodes[p->node];
    return p->event || (node_locked(n) && n->managed && !p->disregard);
}
/* computePatchData (pod_controller.go:404-439); EnableCNI: configurePod fails
 * (no patch) while cni.Setup has not given the pod an IP (:383-389) */
static int pod_needs_patch(const kwok_oracle* o, const opod_t* p) {
    if (o->cni) return p->pod_ip && (p->phase != KWOK_PHASE_RUNNING || !p->conforms || !p->host_ip);
    return p->phase != KWOK_PHASE_RUNNING || !p->conforms || !p->host_ip || !p->pod_ip;
}

static void arena_reserve(buf_t* b, size_t n) {
    if (b->n + n + 1 > b->cap) {
        size_t c = b->cap ? b->cap : 4096;
        while (c < b->n + n + 1) c *= 2;
        b->p = (char*)realloc(b->p, c);
        b->cap = c;
    }
}

/* render items [0, n) of a list in parallel (render(o, buf, i) appends item i's
 * patch, or nothing) and append them to the arena in list order; off / len get
 * each rendered item's arena offset and length (compacted: k-th rendered) */
typedef int (*render_fn)(kwok_oracle* o, buf_t* b, size_t i, const char* now);
static size_t prender(kwok_oracle* o, size_t n, render_fn render, const char* now, uint64_t* off, uint32_t* len,
                      size_t* which) {
    const int T = nthr(o);
    buf_t* bufs = (buf_t*)calloc((size_t)T, sizeof(buf_t));
    size_t* cnt = (size_t*)calloc((size_t)T + 1, sizeof(size_t));
    size_t* first = (size_t*)calloc((size_t)T + 1, sizeof(size_t));
    size_t* loc = (size_t*)calloc(n + 1, sizeof(size_t)); /* per rendered item: offset in its thread buffer */
    uint32_t* lens = (uint32_t*)calloc(n + 1, sizeof(uint32_t));
    size_t* idx = (size_t*)calloc(n + 1, sizeof(size_t));
    /* pass 1: count per thread (rendered items are those that produce bytes) */
#pragma omp parallel num_threads(T)
    {
        const int t = OMP_TID();
        size_t k = 0;
        for (size_t i = n * t / T, hi = n * (t + 1) / T; i < hi; i++) {
            const size_t before = bufs[t].n;
            if (render(o, &bufs[t], i, now)) {
                loc[n * t / T + k] = before;
                lens[n * t / T + k] = (uint32_t)(bufs[t].n - before);
                idx[n * t / T + k] = i;
                k++;
            }
        }
        cnt[t] = k;
    }
    size_t tot = 0, bytes = 0;
    for (int t = 0; t < T; t++) {
        first[t] = bytes;
        bytes += bufs[t].n;
        tot += cnt[t];
    }
    const size_t base = o->arena.n;
    arena_reserve(&o->arena, bytes);
    size_t k = 0;
    for (int t = 0; t < T; t++) {
        for (size_t j = 0; j < cnt[t]; j++, k++) {
            const size_t s = n * t / T + j;
            off[k] = base + first[t] + loc[s];
            len[k] = lens[s];
            if (which) which[k] = idx[s];
        }
    }
#pragma omp parallel for num_threads(T) schedule(static, 1)
    for (int t = 0; t < T; t++) {
        if (bufs[t].n) memcpy(o->arena.p + base + first[t], bufs[t].p, bufs[t].n);
        free(bufs[t].p);
    }
    o->arena.n = base + bytes;
    o->arena.p[o->arena.n] = 0;
    free(bufs), free(cnt), free(first), free(loc), free(lens), free(idx);
    return tot;
}

/* per-tick scratch of the renderers */
typedef struct {
    const uint32_t* list; /* locks / evals */
    const uint32_t* ip;   /* evals: the podIP each pod renders */
} rctx_t;
static rctx_t g_rctx; /* set around each prender call (the oracle is not re-entrant) */

static int render_init_item(kwok_oracle* o, buf_t* b, size_t i, const char* now) {
    const onode_t* n = &o->nodes[g_rctx.list[i]];
    if (n->conforms) return 0;
    render_node_init(o, b, n, now);
    return 1;
}
static int render_pod_item(kwok_oracle* o, buf_t* b, size_t i, const char* now) {
    (void)now;
    const opod_t* p = &o->pods[g_rctx.list[i]];
    if (!pod_needs_patch(o, p)) return 0;
    render_pod(o, b, p, g_rctx.ip[i]);
    return 1;
}

/* the apiserver applies a node init patch: defaults now in place */
static void node_apply_init(kwok_oracle* o, onode_t* n) {
    static const char* dflt[KWOK_NI_COUNT] = {"amd64", "", "", "", "fake", "fake", "", "linux", "", ""};
    for (int k = 0; k < KWOK_NI_COUNT; k++)
        if (!n->info[k] && dflt[k][0]) n->info[k] = xstrndup(dflt[k], strlen(dflt[k]));
    free(n->info[KWOK_NI_SYSTEM_UUID]);
    n->info[KWOK_NI_SYSTEM_UUID] =
        n->info[KWOK_NI_OS_IMAGE] ? xstrndup(n->info[KWOK_NI_OS_IMAGE], strlen(n->info[KWOK_NI_OS_IMAGE])) : NULL;
    if (!n->addresses) {
        buf_t a = {0};
        buf_s(&a, "[{\"address\":");
        buf_jstr(&a, o->node_ip_s, strlen(o->node_ip_s));
        buf_s(&a, ",\"type\":\"InternalIP\"}]");
        n->addresses = a.p;
    }
    if (!n->allocatable) n->allocatable = xstrndup("{\"cpu\":\"1k\",\"memory\":\"1Ti\",\"pods\":\"1M\"}", 39);
    if (!n->capacity) n->capacity = xstrndup("{\"cpu\":\"1k\",\"memory\":\"1Ti\",\"pods\":\"1M\"}", 39);
    n->phase = KWOK_PHASE_RUNNING;
    n->conforms = 1;
}

#define GROW(ptr, n) ptr = realloc(ptr, ((n) + 1) * sizeof(*(ptr)))

/* exchange header (sharded mode); lists follow */
typedef struct {
    uint64_t alloc, n_use, n_rel;
    uint64_t counters[KWOK_COUNTER_COUNT];
} xhdr_t;

int kwok_oracle_tick(kwok_oracle* o, int64_t now_unix, kwok_tick_result* res) {
    const size_t NN = (size_t)o->B * o->cn, NP = (size_t)o->B * o->cp;
    const int T = nthr(o);
    char now[32];
    rfc3339(now_unix, now);
    uint64_t cnt[KWOK_COUNTER_COUNT] = {0};
    o->arena.n = 0;
    o->n_hb = o->n_ini = o->n_pp = o->n_del = 0;
    u32vec rel = {0}, use = {0}, evals = {0}, locks = {0}, dels = {0}, hbl = {0};

    /* 1. deletions (DeletePods/DeletePod :155-202); the Deleted event releases the IP */
    PFILTER(o, NP, keep_del, &dels);
    GROW(o->del, dels.n);
    GROW(o->del_fin, dels.n);
    for (size_t i = 0; i < dels.n; i++) {
        const size_t h = dels.v[i];
        opod_t* p = &o->pods[h];
        o->del[o->n_del] = (int32_t)h;
        o->del_fin[o->n_del++] = (uint8_t)p->has_fin;
        cnt[KWOK_CNT_DELETE]++;
        int32_t nh = p->node;
        if (!o->cni && o->nodes[nh].managed && p->pod_ip && cidr_contains(&o->pool, p->pod_ip)) vpush(&rel, p->pod_ip);
        memset(p, 0, sizeof(*p));
        o->nodes[nh].refs--;
        node_maybe_free(o, nh);
    }
    cnt[KWOK_CNT_RELEASE] = rel.n;
    PFILTER(o, NN, keep_lock, &locks);
    PFILTER(o, NP, keep_eval, &evals);
    /* configurePod (:378-382): Use of every evaluated in-CIDR podIP.  Use of an
     * address already in `used` changes nothing, so only the others are listed. */
    {
        uint8_t* fresh = (uint8_t*)calloc(evals.n + 1, 1);
        uint64_t alloc_local = 0;
#pragma omp parallel for num_threads(T) reduction(+ : alloc_local)
        for (size_t i = 0; i < evals.n; i++) {
            const opod_t* p = &o->pods[evals.v[i]];
            if (o->cni) continue; /* EnableCNI: no ipPool.Use / Get (pod_controller.go:378-389) */
            if (p->pod_ip && cidr_contains(&o->pool, p->pod_ip) && !hs_has(&o->pool.used, p->pod_ip)) fresh[i] = 1;
            if (p->status_nonempty && !p->pod_ip) alloc_local++;
        }
        for (size_t i = 0; i < evals.n; i++)
            if (fresh[i]) vpush(&use, o->pods[evals.v[i]].pod_ip);
        free(fresh);
        cnt[KWOK_CNT_ALLOC] = alloc_local;
    }
    /* counters known before emission (the exchange needs them) */
    {
        uint64_t hb = 0, ready = 0, init = 0, pp = 0, total = 0, pend = 0, run = 0;
#pragma omp parallel for num_threads(T) reduction(+ : hb, ready)
        for (size_t h = 0; h < NN; h++) {
            const onode_t* n = &o->nodes[h];
            if (n->used && n->managed) {
                hb++;
                if (n->conforms || node_locked(n)) ready++;
            }
        }
#pragma omp parallel for num_threads(T) reduction(+ : init)
        for (size_t i = 0; i < locks.n; i++) init += !o->nodes[locks.v[i]].conforms;
        uint8_t* patched = (uint8_t*)calloc(NP + 1, 1);
#pragma omp parallel for num_threads(T) reduction(+ : pp)
        for (size_t i = 0; i < evals.n; i++)
            if (pod_needs_patch(o, &o->pods[evals.v[i]])) {
                pp++;
                patched[evals.v[i]] = 1;
            }
#pragma omp parallel for num_threads(T) reduction(+ : total, pend, run)
        for (size_t h = 0; h < NP; h++) {
            const opod_t* p = &o->pods[h];
            if (!p->used) continue;
            total++;
            const int ph = patched[h] ? KWOK_PHASE_RUNNING : p->phase;
            pend += ph == KWOK_PHASE_PENDING;
            run += ph == KWOK_PHASE_RUNNING;
        }
        free(patched);
        cnt[KWOK_CNT_HEARTBEAT] = cnt[KWOK_CNT_NODES_MANAGED] = hb;
        cnt[KWOK_CNT_NODES_READY] = ready;
        cnt[KWOK_CNT_LOCK_CHECKED] = locks.n;
        cnt[KWOK_CNT_NODE_INIT] = init;
        cnt[KWOK_CNT_EVALUATED] = evals.n;
        cnt[KWOK_CNT_POD_PATCH] = pp;
        cnt[KWOK_CNT_PODS_TOTAL] = total;
        cnt[KWOK_CNT_PODS_PENDING] = pend;
        cnt[KWOK_CNT_PODS_RUNNING] = run;
    }

    /* 2. exchange (sharded mode) and the pool phases: Uses, then Puts */
    uint64_t alloc_before = 0, alloc_after = 0;
    uint64_t fleet[KWOK_COUNTER_COUNT];
    memcpy(fleet, cnt, sizeof(fleet));
    int W = o->cfg.world_size;
    if (W > 1) {
        /* step 1: headers (sizes); step 2: padded lists */
        xhdr_t hdr = {cnt[KWOK_CNT_ALLOC], use.n, rel.n, {0}};
        memcpy(hdr.counters, cnt, sizeof(cnt));
        xhdr_t* all = (xhdr_t*)calloc((size_t)W, sizeof(xhdr_t));
        if (o->cfg.allgather(o->cfg.allgather_user, &hdr, sizeof(hdr), all)) return KWOK_ECOMM;
        size_t maxl = 0;
        for (int r = 0; r < W; r++) {
            size_t l = all[r].n_use + all[r].n_rel;
            if (l > maxl) maxl = l;
        }
        uint32_t* mine = (uint32_t*)calloc(maxl + 1, 4);
        if (use.n) memcpy(mine, use.v, 4 * use.n);
        if (rel.n) memcpy(mine + use.n, rel.v, 4 * rel.n);
        uint32_t* lists = (uint32_t*)calloc((size_t)W * (maxl + 1), 4);
        if (o->cfg.allgather(o->cfg.allgather_user, mine, 4 * (maxl + 1), lists)) return KWOK_ECOMM;
        memset(fleet, 0, sizeof(fleet));
        for (int r = 0; r < W; r++) {
            for (int k = 0; k < KWOK_COUNTER_COUNT; k++) fleet[k] += all[r].counters[k];
            if (r < o->cfg.rank) alloc_before += all[r].alloc;
            if (r > o->cfg.rank) alloc_after += all[r].alloc;
        }
        for (int r = 0; r < W; r++)
            for (uint64_t k = 0; k < all[r].n_use; k++) pool_use(&o->pool, lists[(size_t)r * (maxl + 1) + k]);
        for (int r = 0; r < W; r++)
            for (uint64_t k = 0; k < all[r].n_rel; k++)
                pool_put(&o->pool, lists[(size_t)r * (maxl + 1) + all[r].n_use + k]);
        free(all), free(mine), free(lists);
    } else {
        for (size_t i = 0; i < use.n; i++) pool_use(&o->pool, use.v[i]);
        for (size_t i = 0; i < rel.n; i++) pool_put(&o->pool, rel.v[i]);
    }

    /* 3. heartbeat: every managed node (canonical order), identical bodies */
    {
        buf_t hbb = {0};
        render_heartbeat(&hbb, now, o->start_s);
        o->hb_len = (uint32_t)hbb.n;
        o->hb_off = o->arena.n;
        PFILTER(o, NN, keep_managed, &hbl);
        GROW(o->hb, hbl.n);
        memcpy(o->hb, hbl.v, hbl.n * sizeof(int32_t));
        o->n_hb = (uint32_t)hbl.n;
        arena_reserve(&o->arena, (size_t)o->n_hb * hbb.n);
        char* dst = o->arena.p + o->arena.n;
#pragma omp parallel for num_threads(T)
        for (size_t i = 0; i < o->n_hb; i++) memcpy(dst + i * hbb.n, hbb.p, hbb.n);
        o->arena.n += (size_t)o->n_hb * hbb.n;
        o->arena.p[o->arena.n] = 0;
        free(hbb.p);
    }

    /* 4. node lock (LockNode / configureNode): init patches, then the apiserver applies them */
    {
        GROW(o->ini, locks.n);
        GROW(o->ini_off, locks.n);
        GROW(o->ini_len, locks.n);
        size_t* which = (size_t*)calloc(locks.n + 1, sizeof(size_t));
        g_rctx.list = locks.v;
        o->n_ini = cnt[KWOK_CNT_NODE_INIT] ? (uint32_t)prender(o, locks.n, render_init_item, now, o->ini_off, o->ini_len, which) : 0;
        for (uint32_t k = 0; k < o->n_ini; k++) o->ini[k] = (int32_t)locks.v[which[k]];
#pragma omp parallel for num_threads(T)
        for (uint32_t k = 0; k < o->n_ini; k++) node_apply_init(o, &o->nodes[o->ini[k]]);
        free(which);
    }
#pragma omp parallel for num_threads(T)
    for (size_t h = 0; h < NN; h++) o->nodes[h].event_lock = 0;

    /* 5. pod lock in canonical order; Gets of lower ranks come first */
    {
        uint32_t* ip = (uint32_t*)calloc(evals.n + 1, sizeof(uint32_t));
        for (uint64_t k = 0; k < alloc_before; k++) (void)pool_get(&o->pool);
        for (size_t i = 0; i < evals.n; i++) {
            const opod_t* p = &o->pods[evals.v[i]];
            /* `{{ with .podIP }} . {{ else }} PodIP {{ end }}` inside `{{ with .status }}` */
            ip[i] = (!o->cni && p->status_nonempty && !p->pod_ip) ? (uint32_t)pool_get(&o->pool) : p->pod_ip;
        }
        for (uint64_t k = 0; k < alloc_after; k++) (void)pool_get(&o->pool);
        GROW(o->pp, evals.n);
        GROW(o->pp_off, evals.n);
        GROW(o->pp_len, evals.n);
        size_t* which = (size_t*)calloc(evals.n + 1, sizeof(size_t));
        g_rctx.list = evals.v;
        g_rctx.ip = ip;
        o->n_pp = cnt[KWOK_CNT_POD_PATCH] ? (uint32_t)prender(o, evals.n, render_pod_item, now, o->pp_off, o->pp_len, which) : 0;
        for (uint32_t k = 0; k < o->n_pp; k++) o->pp[k] = (int32_t)evals.v[which[k]];
        /* the apiserver applies each patch */
#pragma omp parallel for num_threads(T)
        for (uint32_t k = 0; k < o->n_pp; k++) {
            opod_t* p = &o->pods[o->pp[k]];
            if (p->status_nonempty) {
                if (!p->host_ip) p->host_ip = o->node_ip;
                p->pod_ip = ip[which[k]];
            }
            p->phase = KWOK_PHASE_RUNNING;
            p->conforms = 1;
            p->status_nonempty = 1;
        }
        free(which);
        free(ip);
    }
#pragma omp parallel for num_threads(T)
    for (size_t h = 0; h < NP; h++) o->pods[h].event = 0, o->pods[h].delete_pending &= o->pods[h].used;

    free(rel.v), free(use.v), free(evals.v), free(locks.v), free(dels.v), free(hbl.v);
    if (res) {
        memset(res, 0, sizeof(*res));
        res->n_heartbeat = o->n_hb;
        res->heartbeat_len = o->hb_len;
        res->heartbeat_stride = o->hb_len;
        res->n_node_init = o->n_ini;
        res->n_pod_patch = o->n_pp;
        res->n_delete = o->n_del;
        res->heartbeat_epoch = o->hb_epoch;
        res->arena_bytes = o->arena.n;
        memcpy(res->counters, fleet, sizeof(fleet));
        memcpy(res->local_counters, cnt, sizeof(cnt));
    }
    return KWOK_OK;
}

int kwok_oracle_read_outputs(kwok_oracle* o, kwok_outputs* out) {
    if (out->heartbeat_nodes) memcpy(out->heartbeat_nodes, o->hb, 4 * o->n_hb);
    out->heartbeat_off = o->hb_off;
    if (out->node_init_nodes) memcpy(out->node_init_nodes, o->ini, 4 * o->n_ini);
    if (out->node_init_off) memcpy(out->node_init_off, o->ini_off, 8 * o->n_ini);
    if (out->node_init_len) memcpy(out->node_init_len, o->ini_len, 4 * o->n_ini);
    if (out->pod_patch_pods) memcpy(out->pod_patch_pods, o->pp, 4 * o->n_pp);
    if (out->pod_patch_off) memcpy(out->pod_patch_off, o->pp_off, 8 * o->n_pp);
    if (out->pod_patch_len) memcpy(out->pod_patch_len, o->pp_len, 4 * o->n_pp);
    if (out->delete_pods) memcpy(out->delete_pods, o->del, 4 * o->n_del);
    if (out->delete_has_finalizers) memcpy(out->delete_has_finalizers, o->del_fin, o->n_del);
    out->arena_shift = 0;
    out->arena_copied = 0;
    if (out->arena) {
        if (out->flags & KWOK_READ_HEARTBEAT_ONCE) { /* one body, then the patches */
            size_t hb = o->n_hb ? o->hb_len : 0, first = (size_t)o->n_hb * o->hb_len, rest = o->arena.n - first;
            if (out->arena_cap < hb + rest) return KWOK_EINVAL;
            memcpy(out->arena, o->arena.p, hb);
            memcpy(out->arena + hb, o->arena.p + first, rest);
            out->arena_shift = first - hb;
            out->arena_copied = hb + rest;
        } else {
            if (out->arena_cap < o->arena.n) return KWOK_EINVAL;
            memcpy(out->arena, o->arena.p, o->arena.n);
            out->arena_copied = o->arena.n;
        }
    }
    return KWOK_OK;
}

int kwok_oracle_read_arena(kwok_oracle* o, uint64_t off, uint64_t len, void* dst) {
    if (off > o->arena.n || len > o->arena.n - off || (len && !dst)) return KWOK_EINVAL;
    if (len) memcpy(dst, o->arena.p + off, len);
    return KWOK_OK;
}

int kwok_oracle_node_has(kwok_oracle* o, const char* name, size_t len) {
    int32_t h = node_find(o, name, len);
    return h >= 0 && o->nodes[h].managed;
}

uint64_t kwok_oracle_node_size(kwok_oracle* o) {
    uint64_t n = 0;
    for (size_t h = 0; h < (size_t)o->B * o->cn; h++) n += o->nodes[h].used && o->nodes[h].managed;
    return n;
}

int kwok_oracle_dump_pods(kwok_oracle* o, int32_t first, uint32_t count, uint8_t* used, uint8_t* phase,
                          uint32_t* host_ip, uint32_t* pod_ip) {
    for (uint32_t i = 0; i < count; i++) {
        size_t h = (size_t)first + i;
        const opod_t* p = h < (size_t)o->B * o->cp ? &o->pods[h] : NULL;
        if (used) used[i] = p ? (uint8_t)p->used : 0;
        if (phase) phase[i] = p && p->used ? (uint8_t)p->phase : 0;
        if (host_ip) host_ip[i] = p && p->used ? p->host_ip : 0;
        if (pod_ip) pod_ip[i] = p && p->used ? p->pod_ip : 0;
    }
    return KWOK_OK;
}
