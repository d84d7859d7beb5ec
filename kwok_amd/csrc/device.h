// device.h - layouts shared by the host runtime (engine.cpp) and the gfx950
// kernels (kernels.hip).  Everything the kernels touch lives in HBM as
// struct-of-arrays indexed by LOCAL slot (slot - first owned slot).
#pragma once
#include <stdint.h>

namespace kwok {

// ---- node state byte (d_node_state) ----------------------------------------
enum : uint8_t {
    NS_EXISTS = 1,      // the Node object exists (not Deleted)
    NS_MANAGED = 2,     // in nodesSets (node_controller.go:259-260, :267-268)
    NS_LOCKABLE = 4,    // needLockNode on its latest event (:210-223)
    NS_CONFORMS = 8,    // configureNode would return nil (A.5)
    NS_EVENT_LOCK = 16, // a watch/list event queued it for LockNode (:261-263)
};

// ---- pod state word (d_pod_state): flags in bits 0..7, phase in 8..10 -------
enum : uint16_t {
    PS_USED = 1,
    PS_DISREGARD = 2,
    PS_DELETE_PENDING = 4, // deletionTimestamp && nodeHas at event time (pod_controller.go:306-308)
    PS_HAS_FIN = 8,
    PS_STATUS_NONEMPTY = 16,
    PS_CONFORMS = 32,
    PS_EVENT = 64,         // needLockPod at event time -> lockPodChan (:318-319)
    PS_HAS_HOST_IP = 128,
};
constexpr int PS_PHASE_SHIFT = 8;
constexpr uint16_t PS_PHASE_MASK = 7u << PS_PHASE_SHIFT;
constexpr uint32_t PHASE_PENDING = 1, PHASE_RUNNING = 2;

// ---- tile geometry -----------------------------------------------------------
constexpr int BLOCK = 256;          // 4 waves of 64
constexpr int NODE_PER_THREAD = 4;  // node tile = 1024 slots
constexpr int POD_PER_THREAD = 8;   // pod tile  = 2048 slots
constexpr int NODE_TILE = BLOCK * NODE_PER_THREAD;
constexpr int POD_TILE = BLOCK * POD_PER_THREAD;

// ---- fixed template geometry (default templates) -----------------------------
constexpr int HB_LEN = 1059;     // {"status":{"conditions":[5 conditions]}} with 20-byte T/S
constexpr int HB_STRIDE = 1072;  // 16-byte aligned arena stride
constexpr int HB_PREFIX = 24;    // {"status":{"conditions":
constexpr int CONDS_LEN = HB_LEN - HB_PREFIX - 2;  // the conditions list "[...]"
constexpr int TS_LEN = 20;       // RFC3339 UTC "YYYY-MM-DDTHH:MM:SSZ"
constexpr int HB_NSLOTS = 10;    // 5 x (lastHeartbeatTime, lastTransitionTime)

// per-tile and per-block aggregates of the classify phase.  The first
// AG_NSCAN fields are exclusive-scanned into output ordinals / offsets (BYTES:
// node-init bytes for node tiles, pod-patch bytes for pod tiles; node tiles
// precede pod tiles, so one scan lays out [inits | pod patches]); the rest are
// only summed.
enum AggField {
    AG_HB = 0, AG_INIT, AG_DEL, AG_PP, AG_BYTES, AG_ALLOC,                  // scanned
    AG_INIT_BYTES, AG_LOCK, AG_MANAGED, AG_READY, AG_EVAL, AG_TOTAL, AG_PENDING, AG_RUNNING, AG_REL,
    AG_COUNT
};
constexpr int AG_NSCAN = 6;
constexpr int AG_STRIDE = 16;

// per-tick header: written on device, copied back to the host
struct TickHdr {
    // local counts / layout (scan kernel)
    uint32_t n_hb, n_init, n_pp, n_del;
    uint32_t n_use, n_rel, n_alloc_local, n_eval;
    uint32_t n_lock, overflow, pad0, pad1;
    uint64_t init_bytes, pp_bytes;
    uint64_t hb_base, init_base, pod_base, arena_bytes;
    uint64_t local_counters[16];
    uint64_t counters[16];       // fleet (summed over ranks)
    // pool (post exchange)
    uint64_t alloc_total, alloc_base, usable_total, take_usable, fresh_in, fresh_out_start;
    uint64_t cursor_index;       // ipPool.index after the tick
    uint64_t rel_total;          // releases this tick, all ranks (pending in rel_bm)
    // s_memrealtime (100 MHz) stamps, CLK_* (block 0; the last two only in profiled ticks)
    uint64_t clk[8];
    // host-visible only (not published): TICK_ERR_* set by a timed-out grid barrier
    uint32_t err, pad2;
};

constexpr uint32_t TICK_ERR_BARRIER = 1;  // a grid barrier timed out
constexpr uint32_t TICK_ERR_LAYOUT = 2;   // device heartbeat count != the host's managed-node count
enum : int {
    CLK_ENTRY = 0,   // block 0 starts the FRONT phases
    CLK_P1,          // block 0 done classifying
    CLK_BAR,         // block 0 leaves the first grid barrier
    CLK_BASES,       // block 0 done with bases / header
    CLK_BACK,        // block 0 starts the BACK phases
    CLK_POOL,        // block 0 done with the pool phase (emission starts)
    CLK_ENTRY_MIN,   // earliest block start          (profiled ticks)
    CLK_P1_MAX,      // latest block done classifying (profiled ticks)
};

// grid-barrier state of the persistent tick kernel (device memory, zeroed once):
// generation, top counter and 8 group counters, each on its own 128-byte line
constexpr int BAR_LINE = 32, BAR_GEN = 0, BAR_TOP = BAR_LINE, BAR_GRP = 2 * BAR_LINE;
struct GridBar {
    uint32_t w[(2 + 8) * BAR_LINE];
    unsigned long long neg_entry_max, p1_max;  // profiled ticks: max(~entry), max(phase-1 end)
};

// exchange message, one per rank (allgather)
constexpr int XINLINE = 2048;
struct XMsg {
    uint64_t alloc, n_use, n_rel, pad;
    uint64_t counters[16];
    uint32_t ips[XINLINE];  // uses then releases (when they fit)
};

// pool geometry
struct PoolGeom {
    uint32_t net;        // network address
    uint32_t base;       // host address of the CIDR string (ipPool base)
    uint64_t size;       // 2^(32-prefix) addresses
    uint64_t words;      // size/64 (bitmap words), >= 1
};

// ingest ops
struct NodeOp {
    uint32_t slot;
    uint8_t and_mask, or_bits, set_blob, pad;
    uint64_t blob;  // off | pre_len<<32 | post_len<<48
};
struct PodOp {
    uint32_t slot;
    uint16_t keep_mask, bits;  // state = (state & keep_mask) | bits
    uint16_t node, spec;
    uint32_t ctime, host_ip, pod_ip;
    uint32_t set_fields;       // overwrite node/spec/ctime/IPs
};

// spec descriptor: A | B | C segments of the pod patch (see templates.cpp)
struct SpecDesc {
    uint32_t off;             // into spec byte/kind arrays
    uint16_t len_a, len_b, len_c;
    uint16_t max_len;         // 16-aligned arena reservation
};

}  // namespace kwok
