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
    NS_SLOT = 32,       // the slot holds a node entry (an existing node, or one that pods still
                        // reference: deleted, or a placeholder named by a pod's spec.nodeName)
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
    // bits 8..10: phase.  Bits 11-12 mirror pod_ip (written with it): the tick's
    // classification reads these instead of the 4-byte address, which it needs only
    // for a Use or a release (loaded then)
    PS_IP_SET = 1u << 11,   // pod_ip != 0
    PS_IP_POOL = 1u << 12,  // pod_ip != 0 and inside the CIDR (ipPool Put / Use apply)
};
constexpr uint16_t PS_IP_BITS = PS_IP_SET | PS_IP_POOL;
constexpr int PS_PHASE_SHIFT = 8;
constexpr uint16_t PS_PHASE_MASK = 7u << PS_PHASE_SHIFT;
constexpr uint32_t PHASE_PENDING = 1, PHASE_RUNNING = 2;

// ---- k_tick geometry ----------------------------------------------------------
// Chain block b owns the contiguous bucket range [nb*b/Gc, nb*(b+1)/Gc) of the
// rank: its node slots and its live pod slots (each bucket's pods below the
// host-maintained fill mark, in 8-slot groups).  Node chunk = 1024 node slots,
// pod chunk = 256 live groups (2048 pod slots); emission works chunk by chunk.
constexpr int BLOCK = 256;          // 4 waves of 64
constexpr int NODE_PER_THREAD = 4;
constexpr int POD_PER_THREAD = 8;   // one 8-slot group per thread per chunk
constexpr int NODE_CHUNK = BLOCK * NODE_PER_THREAD;
constexpr int POD_CHUNK = BLOCK * POD_PER_THREAD;
constexpr int MAX_BPB = 64;               // buckets per chain block
constexpr int NODE_LDS = 16384;           // node slots per chain block (LDS node flags)
constexpr int MAX_NODE_CHUNKS = NODE_LDS / NODE_CHUNK;  // 16
constexpr int MAX_POD_CHUNKS = 64;        // pod chunks per chain block (u64 dirty mask)
constexpr int SPEC_GROUPS = 2;            // pod groups per thread loaded before the fill marks land
#ifndef KWOK_ROW_BATCH
#define KWOK_ROW_BATCH 2
#endif
constexpr int ROW_BATCH = KWOK_ROW_BATCH; // heartbeat-once ticks: pod rows per thread loaded together, one batch ahead
#ifndef KWOK_NODE_PRE
#define KWOK_NODE_PRE 4
#endif
constexpr int NODE_PRE = KWOK_NODE_PRE;   // node chunks of a chain block loaded in its first round trip
#ifndef KWOK_RT1_NODES_FIRST
#define KWOK_RT1_NODES_FIRST 1              // ... issued before the speculative pod groups
#endif
// split ticks (k_pod_jobs): a chain block's live groups in runs of 64, one wave each
constexpr int WC_GROUPS = 64;
constexpr int MAX_WC = MAX_POD_CHUNKS * BLOCK / WC_GROUPS;  // 256 wave chunks per chain block
constexpr int WC_DIRTY_WORDS = MAX_WC / 32;
constexpr int TRACE_SLOTS = 24;         // KWOK_TICK_TRACE=1: per-block phase stamps
constexpr int SPEC_LDS = 256;           // k_tick caches the reservations of up to this many specs

// ---- fixed template geometry (default templates) -----------------------------
constexpr int HB_LEN = 1059;     // {"status":{"conditions":[5 conditions]}} with 20-byte T/S
constexpr int HB_STRIDE = 1072;  // 16-byte aligned arena stride
constexpr int HB_PREFIX = 24;    // {"status":{"conditions":
constexpr int CONDS_LEN = HB_LEN - HB_PREFIX - 2;  // the conditions list "[...]"
constexpr int TS_LEN = 20;       // RFC3339 UTC "YYYY-MM-DDTHH:MM:SSZ"
constexpr int HB_NSLOTS = 10;    // 5 x (lastHeartbeatTime, lastTransitionTime)
// a custom heartbeat template (KWOK_TPL_HEARTBEAT) may render up to this many bytes;
// the geometry of the default one above is the streamer's fast path
constexpr int HB_MAX_STRIDE = 1280;
constexpr int HB_MAX_UNITS = HB_MAX_STRIDE / 16;

// per-chain-block record of the classify phase (16 x u32, one 64-byte line).
// The first AG_NSCAN fields are exclusive-scanned over blocks into output
// ordinals / byte offsets; the rest are only summed.  DIRTY = 1 when the block
// has anything to emit or a state word to rewrite (else it skips emission).
enum AggField {
    AG_INIT = 0, AG_INIT_BYTES, AG_DEL, AG_PP, AG_PP_BYTES, AG_ALLOC,  // scanned
    AG_HB, AG_LOCK, AG_MANAGED, AG_READY, AG_EVAL, AG_TOTAL, AG_PENDING, AG_RUNNING, AG_REL, AG_DIRTY,
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
    // s_memrealtime (100 MHz) stamps, CLK_*
    uint64_t clk[8];
    // host-visible only (not published): TICK_ERR_* set by a timed-out wait
    uint32_t err, pad2;
    // single rank: the tick's field totals (AG_*), written by the chain block whose
    // accumulator add completed each field; the host derives the header from them
    uint64_t tot[16];
    // multi rank: a BACK launch found exchange lists too long to be inline
    uint32_t xovf;
    // multi rank: some rank's message carried its foreign-IP flag (BACK, every rank alike)
    uint32_t xforeign;
    // k_once found work to emit (a delete, patch, Get, Put, Use, event or node init): the
    // host runs the tick again with k_tick (kernels queued behind it skipped)
    uint32_t redo, pad3;
};

constexpr uint32_t TICK_ERR_BARRIER = 1;  // a cross-block wait timed out
constexpr uint32_t TICK_ERR_LAYOUT = 2;   // device heartbeat count != the host's managed-node count
constexpr uint32_t TICK_ERR_SEQ = 4;      // multi rank: the gathered messages are of different ticks
constexpr uint32_t TICK_ERR_EMIT = 8;     // a fused pod emission met a spec without unit tables (host flag stale)
enum : int {
    CLK_ENTRY = 0,   // block 0 starts the tick (FRONT launch)
    CLK_P1_MAX,      // the last chain block arrives (classification complete)
    CLK_HDR,         // the last arriver has published the header / exchange message
    CLK_BACK,        // BACK phases start (multi-rank: BACK launch, block 0)
    CLK_POOL,        // pool phase done (pool leader)
    CLK_ENTRY_MIN,   // earliest chain block start       (profiled ticks)
    CLK_STREAM_END,  // latest heartbeat streamer exit   (profiled ticks, read by the host)
    CLK_RSVD,
};

// k_once (heartbeat-once ticks with nothing to emit): one wave per bucket,
// ONCE_WAVES buckets per block; its counts in ONCE_ACC_WORDS packed words
constexpr int ONCE_WAVES = 8;
constexpr int ONCE_ACC_WORDS = 5;       // (hb, lock) (managed, ready) (eval, total) (pending, running) (rare, -)
constexpr int ONCE_FIELD_BITS = 27;     // each packed partial sum < 2^27 (node / pod slots of the rank)
constexpr int ONCE_NODE_LDS = 1024;     // node slots per bucket it handles (S.cn)
constexpr uint32_t ONCE_SUM_OFF = 0, ONCE_SUM_BUILD = 1, ONCE_SUM_USE = 2;  // k_once's per-bucket summaries

// cross-block state of the tick kernel (device memory, zeroed at create and
// after a failed tick), every word on its own 128-byte line
struct GridBar {
    unsigned long long arrive;  // monotonic: one add per chain block per FRONT launch
    unsigned long long pad0[15];
    uint32_t pcnt, pad1[31];    // pool-phase barrier: arrivals of the current instance
    uint32_t pgen, pad2[31];    //                     generation
    unsigned long long neg_entry_max, p1_max, stream_end_max, pad3[13];  // profiled ticks
    uint32_t skip, pad4[31];    // a tick the host must finish (multi rank: a BACK stopped for long lists; k_once:
                                // work to emit): launches queued behind it skip
    unsigned long long acc[16][16];  // single rank: field accumulators (arrivals << ACC_SHIFT | sum), one line each
    // k_once: packed accumulators (arrivals << ACC_SHIFT | hi << 27 | lo), per XCD shard [0, 8) and the
    // fleet [8], word w of a shard on a line of its own
    unsigned long long once_acc[9][ONCE_ACC_WORDS][16];
};
constexpr int ACC_SHIFT = 54;  // arrivals in the top 10 bits (<= 1023 chain blocks), sums below
constexpr unsigned long long ACC_MASK = (1ull << ACC_SHIFT) - 1;
constexpr int MAX_CHAIN = 512;  // k_tick chain blocks (reduce_records' LDS; engine_create clamps to it)
static_assert(MAX_CHAIN < (1 << (64 - ACC_SHIFT)), "the accumulators count arrivals of every chain block");

// split ticks: what k_pod_jobs needs of a chain block that has pod jobs (written
// by that block in k_tick's BACK phases, after the pool phase): its first output
// ordinals / byte offset, the tick's layout and pool plan, and the tick's tag
struct JobBase {
    uint64_t del, pp, pp_bytes, alloc;     // the block's exclusive prefix (AG_DEL, AG_PP, AG_PP_BYTES, AG_ALLOC)
    uint64_t pod_base, alloc_base;         // Layout
    uint64_t take, fin, fout0;             // PoolPlan
    uint32_t tag, pad;
};

// exchange message, one per rank (allgather)
constexpr int XINLINE = 2048;
struct XMsg {
    uint64_t alloc, n_use, n_rel;
    uint64_t seq;  // the FRONT launch's tick tag: equal on every rank that ticks in step
    uint64_t foreign;  // the rank's sticky foreign-IP flag (engine.cpp quiet ticks: Use checks skipped
                       // only while no rank ever had one)
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

// the PS_IP_* bits of a podIP
#if defined(__HIPCC__)
__host__ __device__
#endif
inline uint16_t ip_state_bits(const PoolGeom& g, uint32_t ip) {
    if (!ip) return 0;
    const bool pool = ip >= g.net && (uint64_t)(ip - g.net) < g.size;
    return (uint16_t)(PS_IP_SET | (pool ? PS_IP_POOL : 0));
}

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
    uint32_t set_fields;       // 1: overwrite node/spec/ctime/IPs; 2: podIP only (kwok_cni_assign)
};

// ---- GPU pod ingest (ingest.hip) ---------------------------------------------
// A pod record after the checks that depend only on the record itself (arena
// bounds, IPv4 strings, spec id, phase, creation time, handle -> bucket),
// written by k_ing_prep at the record's batch index.  The per-bucket apply
// pass reads these in bucket order (a stable sort of the batch by bucket).
struct PodRec {             // 32 bytes
    uint32_t bucket;        // owned local bucket whose slots the record may change (REC_NONE: none)
    uint32_t pos;           // existing: the handle's index in its bucket; create by handle: the node's index
    uint32_t hip, pip;      // UPSERT: status.hostIP / status.podIP (0: empty); DELETE: the parsed podIP
    uint32_t ctime;
    uint16_t spec;          // UPSERT with fst == KWOK_OK: the spec id
    uint8_t op, phase, flags, chk;  // chk: REC_*
    int8_t fst;             // UPSERT: the first failing field check (KWOK_OK: none)
    int8_t pst;             // existing: the handle lookup's status
    uint8_t is_new;         // kwok_pod_rec12: a KWOK_REC_NEW record (its handle goes to out_new_handles)
    uint8_t pad[3];
};
static_assert(sizeof(PodRec) == 32, "prepared pod records are 32 bytes");
constexpr uint32_t REC_NONE = 0xFFFFFFFFu;
enum : uint8_t {
    REC_EXISTING = 1,  // handle >= 0
    REC_DEL_IP = 2,    // DELETE: the event's podIP parsed
    REC_BY_NAME = 4,   // create naming its node by spec.nodeName: the apply pass resolves the name in
                       // the bucket's node directory when it reaches the record (a placeholder entry
                       // if none, pod_controller.go routing of spec.nodeName)
    REC_KEEP_CTIME = 8,  // kwok_pod_rec12 update of a held pod: its creationTimestamp stays (immutable)
};
// per-batch counters of the GPU ingest (device memory, read back by the host)
struct IngSummary {
    uint32_t n_byname;      // owned by-name creates (diagnostics)
    uint32_t rejected;      // records with a status other than KWOK_OK
    uint32_t n_freed;       // node entries the apply pass freed (diagnostics)
    uint32_t n_placeholders;  // placeholder node entries by-name creates made (diagnostics)
    uint32_t need;          // growth check: max over the buckets that would overflow (live pods +
                            // creates > cp), else 0
    uint32_t foreign;       // an in-CIDR podIP the engine did not assign to that pod entered (or left) the
                            // pool: a create with a podIP, an update to another podIP, a Deleted event
                            // releasing an address its pod does not hold (quiet ticks, engine.cpp)
    uint32_t n_new;         // kwok_pod_rec12: the batch's KWOK_REC_NEW records up to this chunk
    uint32_t pad;
};

// ---- the watch-event codec on the GPU (json.hip) -------------------------------
// A compiled labels.Parse selector (codec.cpp parse_selector), flattened for the
// device: requirement r is op[r] on key bytes[key_off[r], +key_len[r]) with values
// val_*[val_first[r], +val_n[r]).  set = 0: the nil selector.
constexpr int JSEL_REQ = 8, JSEL_VAL = 32, JSEL_BYTES = 2048;
enum : uint8_t { JREQ_IN = 0, JREQ_NOTIN, JREQ_EXISTS, JREQ_NOTEXISTS };
struct JsonSel {
    uint32_t set, nreq;
    uint8_t op[JSEL_REQ], val_first[JSEL_REQ], val_n[JSEL_REQ], pad[JSEL_REQ];
    uint16_t key_off[JSEL_REQ], key_len[JSEL_REQ];
    uint16_t val_off[JSEL_VAL], val_len[JSEL_VAL];
};
// the codec's configuration (kwok_codec_config as compiled by kwok_codec_create)
struct JsonCfg {
    uint32_t manage_all;
    uint32_t all_host;  // the selectors exceed these tables: every document goes to the host codec
    JsonSel man_ann, man_lab, dis_ann, dis_lab;
    uint8_t bytes[JSEL_BYTES];  // every selector's keys and values
};
// per decoded pod document, beside its kwok_pod_event
struct JsonPodSide {
    uint32_t name_off, name_len, ns_off, ns_len;  // metadata.name / namespace (kwok_pod_doc)
    uint64_t spec_key;    // json_spec_key of its containers / init containers / readiness gates
    uint64_t spec_key2;   // a second, independent hash of the same bytes (json_complete's batch-local specs)
    uint8_t n_cont, n_init, n_gates, pad;
    int32_t status;       // KWOK_OK / KWOK_EDOMAIN / KWOK_EINVAL, or JSON_HOST / JSON_SPEC / JSON_SPEC_X
};
constexpr int32_t JSON_HOST = 1;  // outside what the device scanner decides: the host codec decodes it
constexpr int32_t JSON_SPEC = 2;  // decoded; its pod spec is not registered yet (the host registers it)
constexpr int32_t JSON_SPEC_X = 3;  // decoded; its spec key is a registered spec's, its strings are not (the host decodes it)

// ---- node directory (device-authoritative, ingest.hip) -------------------------
// A node slot's name lives on the device: node_key[slot] = fnv1a32(name) | len << 32
// (0: no entry), node_name[slot * NAME_STRIDE ...] its bytes.  A name's bucket is
// fnv1a32(name) & (B - 1) (the reference's nodes are routed by name, node_controller.go:
// 256-270); lookups compare the keys of the bucket's Cn slots, then the bytes.
constexpr uint32_t NAME_STRIDE = 256;  // names are 1..253 bytes
constexpr uint32_t NODE_NAME_MAX = 253;
// A node watch record after the checks that depend on the record alone (k_nd_prep),
// at its batch index; its name bytes at names[i * NAME_STRIDE].
struct NodeRec {            // 16 bytes
    uint32_t hash;          // fnv1a32(name)
    uint8_t len, op, fl, pad;  // fl: NR_*
    uint64_t blob;          // UPSERT: the node's init blob word (node_blob)
};
enum : uint8_t { NR_MANAGED = 1, NR_LOCKABLE = 2, NR_CONFORMS = 4, NR_HOST = 8 };
// per-batch counters of a node batch (device memory, read back by the host)
struct NodeSummary {
    uint32_t n_host;        // UPSERT records whose status strings need the host (blob, conforms)
    uint32_t rejected;
    int32_t d_managed;      // managed-set size change
    uint32_t changed;       // the managed set changed (heartbeat handle list epoch)
    uint32_t freed, created, pad[2];
};

// spec descriptor: A | B | C segments of the pod patch (see templates.cpp)
struct SpecDesc {
    uint32_t off;             // into the spec byte array (timestamp slots zero)
    uint16_t len_a, len_b, len_c;
    uint16_t max_len;         // 16-aligned arena reservation
    uint32_t nxt_off;         // its timestamp lookup: spec_nxt[nxt_off + d] (build_ts_lookup)
    uint16_t n_ts, pad;
    uint32_t tab_off;         // its unit tables (build_unit_tables), NO_TAB: the general emitter only
};
constexpr uint32_t NO_TAB = 0xFFFFFFFFu;

// ---- k_emit's table-driven pod path ------------------------------------------
// A pod patch's byte layout depends only on its spec and status shape: empty
// status (shape 0), or the lengths h, p (7..15) of its hostIP / podIP strings
// (shape 1 + (h-7)*9 + (p-7)).  Per spec and shape the host tabulates every
// 16-byte unit of the patch: its static bytes (zero at the creationTimestamp
// slots and the IP digits) and up to two overlays, each a byte offset into the
// job's value row (a 16-byte window of it lands on the unit).  Value row, per
// job, VROW_STRIDE bytes in LDS: the timestamp at VROW_TS, the hostIP string at
// VROW_H, the podIP string at VROW_P, zeros elsewhere; the 16 bytes before a
// row are the previous row's zero tail (or a zero lead pad).  An overlay
// offset is stored biased by VROW_BIAS (0: no overlay, a zero window).
constexpr int EMIT_SHAPES = 82;
constexpr int VROW_STRIDE = 100, VROW_TS = 0, VROW_H = 36, VROW_P = 68, VROW_BIAS = 16;
constexpr uint32_t MAX_TAB_UNITS = 1u << 22;  // all specs' tables (64 MiB of static bytes)
constexpr inline uint32_t emit_shape(uint32_t h, uint32_t p) { return 1u + (h - 7u) * 9u + (p - 7u); }
// byte padding around the spec / blob arrays the emitter reads 4-byte words of
// (a 16-byte window reads up to 15 bytes before a segment and 20 past it)
constexpr int SRC_PAD_FRONT = 16, SRC_PAD_BACK = 64;

}  // namespace kwok
