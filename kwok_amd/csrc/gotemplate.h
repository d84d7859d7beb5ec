// gotemplate.h - the host-side renderer behind custom pod status templates
// (Config.PodStatusTemplate, controller.go:74-76): the subset of Go's
// text/template that renderer.renderToJSON executes (renderer.go:49-89), the
// template funcs (controller.go:35-54, pod_controller.go:115-122), and
// sigs.k8s.io/yaml.YAMLToJSON (yaml.v2 / YAML 1.1 typing -> encoding/json:
// sorted keys, compact, HTML-safe escapes).
//
// It runs at spec registration only: templates.cpp renders a custom template
// over symbolic pod documents and compiles the result into the same A | B | C
// byte program the default template uses (the kernels are unchanged).  Inputs
// outside the covered subset fail with a message; callers map that to
// KWOK_EDOMAIN.
#pragma once
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>

namespace kwok {
namespace gotpl {

struct Value;
using VPtr = std::shared_ptr<const Value>;
struct Value {
    enum Kind { NOVAL, NUL, BOOL, NUM, STR, LIST, MAP } kind = NOVAL;
    bool b = false;
    std::string s;                                 // STR text, NUM literal (json.Number)
    std::vector<VPtr> list;                        // LIST
    std::vector<std::pair<std::string, VPtr>> map;  // MAP, sorted by key
    std::string path;                              // where it sits in the document ("$.spec.containers[]")
};
VPtr make_str(const std::string& s, const std::string& path = "");
VPtr make_map(std::vector<std::pair<std::string, VPtr>> kv, const std::string& path = "");
VPtr make_list(std::vector<VPtr> items, const std::string& path = "");
VPtr make_null(const std::string& path = "");
// child paths follow the parent's: map field "$.a" -> "$.a.b", list item "$.a[]"
VPtr with_paths(const VPtr& v, const std::string& path);

struct Env {
    // template funcs by name (zero-argument funcs return a string)
    std::map<std::string, std::function<std::string()>> funcs;
    // nullptr: any field may be read; else only paths in the set ("$.a.*": $.a's subtree)
    const std::vector<std::string>* allowed_paths = nullptr;
};

// renderToJSON: TrimSpace, parse, execute over doc, YAMLToJSON.  false + err on
// anything outside the covered subset (or a Go template / YAML error).
bool render_to_json(const std::string& tpl, const VPtr& doc, const Env& env, std::string& out, std::string& err);
// the same, stopping at the YAML tree (a null value for an empty output)
bool render_to_tree(const std::string& tpl, const VPtr& doc, const Env& env, VPtr& out, std::string& err);
std::string to_json(const VPtr& v);  // encoding/json.Marshal
// template execution alone (the text YAMLToJSON would read)
bool execute_template(const std::string& tpl, const VPtr& doc, const Env& env, std::string& text, std::string& err);

// helpers exposed for tests (kwok_template_render) and the compiler
bool parse_json(const std::string& s, VPtr& out, std::string& err);
bool yaml_to_json(const std::string& yaml, std::string& out, std::string& err);

}  // namespace gotpl
}  // namespace kwok
