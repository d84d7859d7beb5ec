// CPU check of k_emit's table-driven pod path: for pod specs
// under the default template and the custom templates given on the command
// line, every status shape and a spread of creation times / IPs, the bytes the
// kernel forms as table[unit] | window(value row, overlay) equal the patch
// assembled from the spec program (the host assembly kwok_pod_template_patch
// uses).  The value-row layout and the window arithmetic restate
// kernels.hip emit_row_tab / ext16 / flat_store.  Used by tests/test_unit_tables.py.
#include <cstdio>
#include <cstring>
#include <ctime>
#include <fstream>
#include <sstream>

#include "device.h"
#include "templates.h"

using namespace kwok;

static std::string rfc3339(int64_t u) {
    time_t t = (time_t)u;
    struct tm tm;
    gmtime_r(&t, &tm);
    char b[32];
    strftime(b, sizeof b, "%Y-%m-%dT%H:%M:%SZ", &tm);
    return b;
}

// the patch from the program: A | "hostIP":"H", | B | "podIP":"P", | C (timestamp slots filled)
static std::string assemble(const SpecProgram& p, const std::string& ts, const std::string& h, const std::string& q,
                            bool status) {
    auto fill = [&](const std::string& seg, const std::string& kind) {
        std::string o = seg;
        for (size_t i = 0; i < o.size(); i++)
            if ((uint8_t)kind[i] != KIND_LIT) o[i] = ts[(uint8_t)kind[i]];
        return o;
    };
    std::string o = fill(p.a, p.ka);
    if (status) o += "\"hostIP\":\"" + h + "\",";
    o += fill(p.b, p.kb);
    if (status) o += "\"podIP\":\"" + q + "\",";
    return o + fill(p.c, p.kc);
}

// the kernel's bytes for one job: value row (biased by VROW_BIAS, the 16 bytes
// before it zero) and 16-byte units table | window(row, desc & 0xFF) | window(row, desc >> 8)
static std::string emulate(const std::string& tab, const std::vector<uint16_t>& desc, uint32_t U, uint32_t shape,
                           const std::string& ts, const std::string& h, const std::string& q, size_t len) {
    uint8_t row[VROW_BIAS + VROW_STRIDE + 8] = {};
    memcpy(row + VROW_BIAS + VROW_TS, ts.data(), ts.size());
    if (shape) {
        memcpy(row + VROW_BIAS + VROW_H, h.data(), h.size());
        memcpy(row + VROW_BIAS + VROW_P, q.data(), q.size());
    }
    std::string out;
    for (uint32_t u = 0; u * 16 < len; u++) {
        const size_t e = (size_t)shape * U + u;
        uint8_t v[16];
        memcpy(v, tab.data() + e * 16, 16);
        for (int k = 0; k < 2; k++) {
            const uint32_t off = k ? desc[e] >> 8 : desc[e] & 0xFF;
            for (int i = 0; i < 16; i++) v[i] |= row[off + i];  // off 0: the zero lead
        }
        out.append((const char*)v, 16);
    }
    return out.substr(0, len);
}

static std::string ip(uint32_t a) {
    char b[20];
    snprintf(b, sizeof b, "%u.%u.%u.%u", a >> 24, (a >> 16) & 255, (a >> 8) & 255, a & 255);
    return b;
}

int main(int argc, char** argv) {
    std::vector<std::vector<Container>> C = {{{"fake-pod", "fake"}}, {{"a", "img-a"}, {"b", "img/b:v2"}}, {},
                                             {{"c0", "quay.io/org/image-00:tag"}, {"c1", "x"}, {"c2", "busybox:1.36"}}};
    std::vector<std::vector<Container>> I = {{}, {{"init", "busybox"}}, {{"i0", "registry.k8s.io/pause:3.9"}}, {}};
    std::vector<std::vector<std::string>> G = {{}, {"g.io/x"}, {"g.io/a", "g.io/b"}, {}};
    std::vector<std::string> tpls = {""};  // "": the default program (build_spec_program)
    for (int i = 1; i < argc; i++) {
        std::ifstream f(argv[i]);
        std::stringstream ss;
        ss << f.rdbuf();
        tpls.push_back(ss.str());
    }
    // IPs of every string length 7..15 (the shape's h / p)
    const uint32_t ips[9] = {0x01020304, 0x0A020304, 0x0A140304, 0x0A141E04, 0x0A141E28,
                             0x640A0A32, 0x64640A32, 0xC0A86414, 0xFFFFFFFF};
    long checked = 0, bad = 0, two = 0;
    for (size_t t = 0; t < tpls.size(); t++) {
        for (size_t s = 0; s < C.size(); s++) {
            SpecProgram p;
            std::string why;
            if (tpls[t].empty()) p = build_spec_program(C[s], I[s], G[s]);
            else if (!compile_pod_template(tpls[t], C[s], I[s], G[s], "2024-01-01T00:00:00Z", p, why)) {
                printf("template %zu spec %zu: rejected (%s)\n", t, s, why.c_str());
                continue;
            }
            std::string tab;
            std::vector<uint16_t> desc;
            if (!build_unit_tables(p, tab, desc)) {
                printf("template %zu spec %zu: no tables\n", t, s);
                continue;
            }
            for (uint16_t d : desc) two += (d >> 8) != 0;
            const uint32_t U = p.max_len / 16;
            for (uint32_t shape = 0; shape < (uint32_t)EMIT_SHAPES; shape++) {
                for (int r = 0; r < 3; r++) {
                    const std::string ts = rfc3339(86400LL * 365 * (1 + 30 * r) + 3599 * shape + 7 * r);
                    const uint32_t hi = shape ? (shape - 1) / 9 : 0, pi = shape ? (shape - 1) % 9 : 0;
                    const std::string h = ip(ips[hi]), q = ip(ips[pi]);
                    if (shape && (h.size() != 7 + hi || q.size() != 7 + pi)) {
                        printf("bad IP table\n");
                        return 2;
                    }
                    const std::string want = assemble(p, ts, h, q, shape != 0);
                    const std::string got = emulate(tab, desc, U, shape, ts, h, q, want.size());
                    checked++;
                    if (got != want) {
                        if (bad++ < 5)
                            printf("MISMATCH template %zu spec %zu shape %u\n  want %s\n  got  %s\n", t, s, shape,
                                   want.c_str(), got.c_str());
                    }
                }
            }
        }
    }
    printf("checked %ld patches, %ld mismatches, %ld two-overlay units\n", checked, bad, two);
    return bad ? 1 : 0;
}
