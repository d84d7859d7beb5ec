// templates.h - fixed-layout byte programs for the reference's three default
// templates (pkg/kwok/controllers/templates/{node.heartbeat,node.status,
// pod.status}.tpl) as they come out of renderer.go:49-89 (text/template ->
// sigs.k8s.io/yaml.YAMLToJSON -> json.Marshal: sorted keys, compact) and the
// {"status": ...} wrapper (node_controller.go:388,398; pod_controller.go:399).
// The kernels only fill timestamp/IP slots and splice per-object blobs.
#pragma once
#include <stdint.h>

#include <string>
#include <vector>

namespace kwok {

constexpr uint8_t KIND_LIT = 0xFF;  // literal byte; otherwise an index into a 20-byte timestamp

struct HeartbeatTemplate {
    std::string bytes;              // the patch (HB_LEN bytes by default), timestamp slots zero-filled
    std::vector<uint16_t> now_slots;   // offsets of Now values (lastHeartbeatTime)
    std::vector<uint16_t> start_slots; // offsets of StartTime values (lastTransitionTime)
    uint32_t conds_off = 0, conds_len = 0;  // the conditions list (spliced into node init patches)
};
HeartbeatTemplate build_heartbeat_template();
// A custom heartbeat template (Config.NodeHeartbeatTemplate, controller.go:77):
// rendered with sentinel Now values (StartTime and NodeIP are fixed), it must
// be {"status":{"conditions":[...]}} of at most HB_MAX_STRIDE bytes, the same
// for every node (it may read no node field); every Now becomes a slot.
bool compile_heartbeat_template(const std::string& tpl, const std::string& start_time, const std::string& node_ip,
                                HeartbeatTemplate& out, std::string& err);

struct SpecProgram {
    std::string a, b, c;           // segments (timestamp slots zero-filled)
    std::string ka, kb, kc;        // per-byte kind (KIND_LIT or 0..19)
    uint32_t max_len;              // a+b+c + 53 (hostIP/podIP pieces at 15-char IPs)
};
struct Container {
    std::string name, image;
};
SpecProgram build_spec_program(const std::vector<Container>& containers, const std::vector<Container>& init,
                               const std::vector<std::string>& gates);

// node init blob, framed so the init patch is pre + conditions + post:
//   pre  = {"status":{"addresses":..,"allocatable":..,"capacity":..,"conditions":
//   post = ,"nodeInfo":{..},"phase":"Running"}}
struct NodeBlob {
    std::string pre, post;
};
NodeBlob build_node_blob(const std::string& addresses_json, const std::string& allocatable_json,
                         const std::string& capacity_json, const std::string info[10], const std::string& node_ip);

// A custom pod status template (Config.PodStatusTemplate, controller.go:76)
// compiled into the same program: rendered (gotemplate.h) over symbolic pod
// documents of this spec - every status shape the engine emits, two sets of
// sentinel timestamps / IPs - and accepted only if the outputs prove the
// A | "hostIP":"H", | B | "podIP":"P", | C layout with creationTimestamp slots.
// false + err: outside what the kernels emit (the caller's KWOK_EDOMAIN).
bool compile_pod_template(const std::string& tpl, const std::vector<Container>& containers,
                          const std::vector<Container>& init, const std::vector<std::string>& gates,
                          const std::string& start_time, SpecProgram& out, std::string& err);

// A custom node initialization template (Config.NodeInitializationTemplate,
// controller.go:75) for one node's status fields, compiled into the framed
// blob: NewNodeController renders it followed by the heartbeat template
// (node_controller.go:101), so the init patch is pre | the heartbeat's
// conditions list (the kernels' CONDS, with Now / StartTime) | post.
// phase: KWOK_PHASE_NONE / RUNNING / OTHER of the node event.
bool compile_node_template(const std::string& tpl, const std::string& addresses_json,
                           const std::string& allocatable_json, const std::string& capacity_json,
                           const std::string info[10], int phase, const std::string& node_ip,
                           const std::string& start_time, const HeartbeatTemplate& hb, NodeBlob& out,
                           std::string& err);
// the heartbeat patch / its conditions list (CONDS) at now / start (RFC3339)
std::string heartbeat_patch(const HeartbeatTemplate& hb, const std::string& now, const std::string& start);
std::string heartbeat_conditions(const HeartbeatTemplate& hb, const std::string& now, const std::string& start);

// k_emit's timestamp-slot lookup of a spec (false: layout outside what it handles)
bool build_ts_lookup(const SpecProgram& p, std::vector<uint16_t>& out);
// k_emit's unit tables of a spec (device.h, "table-driven pod path"):
// EMIT_SHAPES x (max_len / 16) units, 16 static bytes each (tab) and an overlay
// word (desc: offset | offset << 8).  false: a unit needs more than two overlays.
bool build_unit_tables(const SpecProgram& p, std::string& tab, std::vector<uint16_t>& desc);

// domain checks (DESIGN.md "Supported domain")
bool safe_string(const char* s, size_t n);
bool valid_json_blob(const char* s, size_t n, char open);
bool parse_ipv4(const char* s, size_t n, uint32_t* out);  // canonical dotted quad only
std::string format_ipv4(uint32_t ip);
void json_string(std::string& out, const std::string& s);

}  // namespace kwok
