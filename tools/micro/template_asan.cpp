// Host sanitizer harness for the template renderer / compiler (gotemplate.cpp,
// templates.cpp): every length-prefixed template of the input file (written by
// tools/template_asan.sh: the test templates and random mutations of them) is
// rendered over a pod and a node document and compiled as a pod status and a
// node initialization template; any outcome but a crash / sanitizer report is fine.
#include <cstdio>
#include <string>
#include <vector>

#include "gotemplate.h"
#include "templates.h"

using namespace kwok;
int main(int argc, char** argv) {
    FILE* f = fopen(argc > 1 ? argv[1] : "/tmp/template_asan/tpl.bin", "rb");
    if (!f) return 3;
    std::vector<std::string> tpls;
    uint32_t n;
    while (fread(&n, 4, 1, f) == 1) {
        std::string s(n, '\0');
        if (fread(&s[0], 1, n, f) != n) return 4;
        tpls.push_back(s);
    }
    gotpl::VPtr doc;
    std::string err;
    gotpl::parse_json(
        "{\"metadata\":{\"name\":\"p\",\"creationTimestamp\":\"2024-01-01T00:00:00Z\"},\"spec\":{\"containers\":"
        "[{\"name\":\"c\",\"image\":\"i\"}],\"readinessGates\":[{\"conditionType\":\"g\"}]},\"status\":{\"phase\":"
        "\"Pending\",\"allocatable\":{\"cpu\":\"1\"},\"nodeInfo\":{\"osImage\":\"x\"}}}",
        doc, err);
    gotpl::Env env;
    env.funcs["Now"] = [] { return std::string("2024-01-01T00:00:30Z"); };
    env.funcs["NodeIP"] = [] { return std::string("10.0.0.1"); };
    env.funcs["PodIP"] = [] { return std::string("10.0.0.2"); };
    size_t ok = 0, compiled = 0;
    for (const auto& t : tpls) {
        std::string out;
        ok += gotpl::render_to_json(t, doc, env, out, err);
        SpecProgram p;
        compiled += compile_pod_template(t, {{"c", "img"}, {"d", "x/y:1"}}, {{"i", "busybox"}}, {"g.io/x"},
                                         "2024-01-01T00:00:00Z", p, err);
        NodeBlob b;
        std::string info[10];
        info[8] = "ubuntu";
        compiled += compile_node_template(t, "", "{\"cpu\":\"4\"}", "", info, 2, "10.9.9.9", "2024-01-01T00:00:00Z", b, err);
    }
    printf("templates %zu rendered %zu compiled %zu\n", tpls.size(), ok, compiled);
    return 0;
}
