// kernels.h - device state handle + launchers (host side of kernels.hip)
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/kwok_engine.h"
#include "device.h"

namespace kwok {

struct ListDesc {
    const uint32_t* use;
    const uint32_t* rel;
    uint32_t n_use, n_rel;
    uint32_t count_from_hdr;  // single rank: counts live in TickHdr
    uint32_t pad;
};

// Everything a kernel needs, passed by value (pointers into HBM).
struct DevState {
    // nodes (local slots)
    uint8_t* node_state;
    uint64_t* node_blob;
    uint8_t* node_tick;
    uint32_t n_node_slots;
    // node directory (ingest.hip): names of the node entries, managed / zombie entries per bucket
    uint64_t* node_key;        // [NL] fnv1a32(name) | len << 32, 0: free
    uint8_t* node_name;        // [NL * NAME_STRIDE]
    uint32_t* mb_count;        // [nb] managed nodes per owned bucket (heartbeat handle bases: k_hb_pre)
    uint32_t* zb_count;        // [nb] zombie entries per owned bucket (NS_SLOT without NS_EXISTS)
    // pods (local slots)
    uint16_t* pod_state;
    uint16_t* pod_node;
    uint16_t* pod_spec;
    uint32_t* pod_ctime;
    uint32_t* pod_ip;
    uint32_t* host_ip;
    uint32_t n_pod_slots;
    uint32_t cn, cp;
    uint32_t nb;               // owned buckets
    uint32_t n_chain;          // k_tick chain blocks (own bucket ranges); streamer blocks follow them
    uint32_t n_pool_extra;     // multi rank: BACK launch blocks past the chain blocks that only take part
                               // in the pool phase (the CUs' spare k_tick slots; 0 on heartbeat-once engines)
    int32_t node_handle_base, pod_handle_base;
    // pool replica
    uint64_t* used_bm;
    uint64_t* usable_bm;
    uint64_t* rel_bm;        // Puts of this tick, folded into used/usable by k_pool_prep
    uint64_t* pool_index;    // ipPool.index (persistent)
    uint32_t* pool_blk;      // per word-block counts (usable, free)
    uint32_t* alloc_addr;    // this rank's allocated addresses, by local ordinal
    PoolGeom pool;
    // pod spec programs / node blobs
    const SpecDesc* specs;
    const uint8_t* spec_bytes;     // SRC_PAD_FRONT bytes into a padded device array
    const uint8_t* blob;           // (likewise) framed node init blobs: pre | post
    const uint16_t* spec_nxt;      // timestamp lookups of every spec (SpecDesc::nxt_off)
    const uint4* unit_tab;         // unit tables of every spec (SpecDesc::tab_off, build_unit_tables)
    const uint16_t* unit_desc;     //   and their overlay words
    uint32_t n_specs, spec_total;  // spec descriptors; bytes of the concatenated spec programs
    uint32_t nxt_total;            // entries of spec_nxt
    uint32_t blob_total;           // bytes of the interned node blobs
    // heartbeat template
    const uint8_t* hb_static;
    const uint8_t* hb_kind;
    // per tick
    TickHdr* hdr;
    XMsg* xmsg;
    uint32_t* use_list;      // multi-rank exchange lists
    uint32_t* rel_list;
    uint32_t* list_counts;   // [2]: n_use, n_rel (reset by k_emit)
    int world;
    int multi;               // FRONT / exchange / BACK ticks (world > 1, or forced for tests)
    int rank;
    const XMsg* xall;        // [world] gathered exchange messages (multi rank)
    uint8_t* arena;
    uint64_t arena_cap;
    int32_t* hb_nodes;
    int32_t* init_nodes;
    uint64_t* init_off;
    uint32_t* init_len;
    int32_t* pp_pods;
    uint64_t* pp_off;
    uint32_t* pp_len;
    uint4* pp_job;             // per pod patch: podIP (0: no status section), hostIP, creationTimestamp, spec (k_emit)
    uint64_t* init_job;        // per node init: its blob (k_emit)
    uint32_t* emit_n;          // [2]: pod patches, node inits whose bytes k_emit writes
    int32_t* del_pods;
    uint8_t* del_fin;
    uint32_t node_ip;
    TickHdr* hdr_host;         // pinned host copy of the tick header (written by k_emit_pods)
    uint16_t* pod_fill;        // per owned bucket: upper bound of used pod slots (only grows; the ingest pass)
    const uint32_t* hb_pre;    // [n_chain + 1] managed nodes before each chain block (k_hb_pre)
    const uint32_t* hb_bpre;   // [nb + 1] managed nodes before each owned bucket (k_hb_pre; k_once)
    GridBar* bar;              // cross-block state
    uint32_t* blockagg;        // [n_chain][AG_STRIDE] per-chain-block records of the classify phase
    uint64_t* dmask;           // [n_chain][2] dirty pod-chunk / node-chunk masks (FRONT -> BACK)
    uint32_t* list_blk;        // multi rank: [n_chain][2] the block's Use / release list lengths; its entries sit in
                               // use_list / rel_list from its first pod slot (bk0 * cp) on
    uint4* wc_pre;             // split ticks: [n_chain][MAX_WC] in-block exclusive prefix of (del, pp, pp bytes, alloc)
    uint32_t* wc_dirty;        //   per 64-group wave chunk, and [n_chain][WC_DIRTY_WORDS] its dirty bits (FRONT)
    JobBase* jbase;            //   [n_chain] (BACK) -> k_pod_jobs
    uint64_t* trace;           // [grid][TRACE_SLOTS] per-block phase stamps (KWOK_TICK_TRACE=1), else null
    uint4* once_sum;           // [nb] k_once per-bucket summaries (ONCE_SUM_BUILD / _USE)
    uint64_t* jtrace;          // [n_chain * MAX_WC][4] k_pod_jobs per-wave stamps (KWOK_JOBS_TRACE=file), else null
    const DevState* self;      // this struct's copy in device memory (out-of-line kernel phases)
    uint32_t stream_delay;     // streamers start this many 10 ns ticks late (KWOK_TICK_STREAM_DELAY_NS, diagnostics)
    uint32_t stream_share;     // /1024 of the heartbeat stream written by the streamer blocks (the rest: chain blocks)
    uint32_t hb_nt;            // heartbeat stores non-temporal (streams larger than the Infinity Cache)
    uint32_t hb_once;          // KWOK_CFG_HEARTBEAT_ONCE: one heartbeat body per tick, not one per node
    uint32_t cni;              // Config.EnableCNI: pod IPs come from the caller's CNI (kwok_cni_assign), not the ipPool
    uint32_t custom_pod;       // Config.PodStatusTemplate is custom: the caller's CONFORMS digest is ignored
    uint32_t use_events_only;  // this tick Use-checks only pods with an event (a quiet tick: kwok_tick_submit)
    uint32_t foreign;          // multi rank: this rank's sticky foreign-IP flag, sent in the exchange message
    uint32_t xcap_u, xcap_r;   // multi rank, TICK_XSPEC: the list allgather's Use / release capacity per rank
    uint32_t fuse_pods;        // split ticks: k_pod_jobs writes the pod patch bytes itself (every spec has unit tables)
    uint32_t sparse_jobs;      // unfused split ticks: FRONT publishes its dirty groups (gjob), k_sparse_jobs builds the jobs
    uint4* gjob;               //   [n_chain][MAX_WC * WC_GROUPS]: slot, masks (del | need << 8 | alloc << 16 | j << 24 |
                               //   any held hostIP << 30 | any held podIP << 31), patch bytes, tick tag
    uint32_t buckets;          // B (all ranks)
    uint32_t b_lo;             // first owned bucket
    uint32_t pod_stride;       // pod handle = (b_lo + slot / cp) * pod_stride + slot % cp
    // heartbeat geometry (default: HB_STRIDE / 16, HB_PREFIX, CONDS_LEN; a custom template's otherwise)
    uint32_t hb_units;         // 16-byte units per heartbeat slot (arena stride = 16 x hb_units)
    uint32_t conds_off, conds_len;  // the conditions list inside the heartbeat (spliced into node inits)
};

__device__ __host__ inline int32_t pod_handle_of(const DevState& S, uint32_t slot) {
    return (int32_t)((S.b_lo + slot / S.cp) * S.pod_stride + slot % S.cp);
}

void launch_apply_ops(const DevState& S, const NodeOp* nops, uint32_t nn, const PodOp* pops, uint32_t np,
                      hipStream_t st);
void launch_pool_puts_now(const DevState& S, const uint32_t* ips, uint32_t n, hipStream_t st);
void launch_pool_apply(const DevState& S, const ListDesc* ld, int nranks, uint32_t max_n, hipStream_t st);
// multi rank, long lists: the chain blocks' Use / release segments -> dst (uses, then releases, canonical order);
// rel_at: where the releases start (~0u: right after the uses); cap_u / cap_r: entries kept (the rest dropped)
void launch_gather_lists(const DevState& S, uint32_t* dst, hipStream_t st, uint32_t rel_at = ~0u,
                         uint32_t cap_u = ~0u, uint32_t cap_r = ~0u);
// TICK_XSPEC: every rank's gathered lists (rank r at recv + r * (cap_u + cap_r), releases from cap_u) into
// `used` / rel_bm when every rank's lists fit the capacities (the messages say); otherwise nothing
void launch_pool_apply_spec(const DevState& S, const uint32_t* recv, hipStream_t st);
// KWOK_EMULATE_RANKS diagnostics: xw - 1 synthetic ranks' messages / long lists from this rank's
void launch_emulate_msgs(const DevState& S, XMsg* X, uint32_t xw, hipStream_t st);
void launch_emulate_lists(const DevState& S, uint32_t* recv, uint64_t maxl, uint32_t xw, uint32_t n, hipStream_t st);
// EnableCNI: handles of the pods the next tick evaluates that hold no podIP
// (configurePod's cni.Setup set), appended in any order at out[*count]
void launch_cni_pending(const DevState& S, int32_t* out, uint32_t* count, hipStream_t st);

// the tick kernel: n_chain chain blocks (+ n_stream heartbeat streamers in
// launches with TICK_FRONT).  Chain blocks wait on each other only in ticks
// with work to emit, so they must be co-resident (tick_occupancy).
// pool phase: bitmap words per thread of a word-block (BLOCK * POOL_WPT words; a
// multi-rank engine takes 8, kernels.hip POOL_WPT_MULTI).  The per-word-block
// counts (pool_blk) are allocated for POOL_WPT_MIN, the smallest a build uses.
#ifndef KWOK_POOL_WPT
#define KWOK_POOL_WPT 2
#endif
constexpr int POOL_WPT = KWOK_POOL_WPT;
constexpr int POOL_WPT_MIN = 1;
constexpr int TICK_FRONT = 1, TICK_BACK = 2, TICK_PROF = 4, TICK_PRIO = 8, TICK_NOSTREAM = 16,  // NOSTREAM: diagnostics only
              TICK_XLISTS = 32,  // BACK: the exchange lists were applied by k_pool_apply
              TICK_SPLIT = 64,   // the pod jobs are built by k_pod_jobs after the tick's launch(es)
              TICK_XSPEC = 128;  // BACK: the lists went out in a second allgather of capacity xcap_u + xcap_r
                                 // and k_pool_apply_spec applied them if every rank's fit
// tag: this tick's nonzero id (single-rank dirty records); arrive_target: the
// arrival count at which every chain block of this FRONT launch has arrived
void launch_tick(const DevState& S, uint32_t n_stream, uint64_t now, uint64_t start, uint32_t n_hb, int phases,
                 uint32_t tag, uint64_t arrive_target, hipStream_t st, hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
// a heartbeat-once tick expected to have nothing to emit (single rank): one
// wave per bucket counts it; a tick that has work after all sets TickHdr::redo
// and GridBar::skip (the host runs it again with launch_tick)
// sum_mode: ONCE_SUM_OFF / _BUILD (also write the per-bucket summaries of generation gen) /
// _USE (read those summaries instead of the pod rows where they apply)
void launch_tick_once(const DevState& S, uint64_t now, uint64_t start, uint32_t n_hb, int phases, uint32_t sum_mode,
                      uint32_t gen, hipStream_t st, hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
uint32_t once_blocks(const DevState& S);
// split ticks: the pod jobs (deletes, patch job records, state transitions) of
// every dirty 64-group run of every chain block, one wave each
// k_pod_jobs; a fused launch (DevState::fuse_pods) also writes the node inits with init_blocks blocks
// (DevState::sparse_jobs: k_sparse_jobs from the groups FRONT published instead of k_pod_jobs<false>)
void launch_pod_jobs(const DevState& S, uint32_t tag, hipStream_t st, uint32_t init_blocks, uint64_t now, uint64_t start,
                     hipEvent_t t0 = nullptr, hipEvent_t t1 = nullptr);
int tick_occupancy();  // resident k_tick blocks per CU
// the patch bytes of the tick's jobs (after its k_tick launch(es), on the same stream)
void launch_emit(const DevState& S, uint32_t grid, uint64_t now, uint64_t start, hipStream_t st);
int emit_occupancy();  // resident k_emit blocks per CU

// ---- GPU pod ingest (ingest.hip): kwok_ingest_pods / kwok_cni_assign --------
struct IngestBatch {
    const void* ev;            // [n] kwok_pod_event (packed: kwok_pod_rec), on the device or read in place
    uint32_t n;
    uint32_t n_specs;
    uint32_t packed;           // 1: kwok_pod_rec records (no arena); 2: kwok_pod_rec12
    uint32_t spec;             // the apply pass was queued without the host's growth check: it returns at once
                               // when the chunk needs more pod slots than a bucket has (sum->need > cp) or an
                               // earlier chunk of the batch did (*abort), setting *abort (the host redoes them)
    const uint8_t* arena;      // the batch's string arena (device copy)
    uint64_t arena_len;
    PodRec* rec;               // [n] prepared records
    uint32_t* keys;            // [n] sort key: owned local bucket, or nb (nothing to apply)
    uint32_t* keys_sorted;     // [n]
    uint32_t* idx_sorted;      // [n] batch indices in (bucket, batch order)
    int32_t* out_handle;       // [n]
    int32_t* out_status;       // [n]
    uint32_t* out_released;    // [n]
    uint32_t* beg;             // [nb] first sorted position of each bucket
    uint32_t* end;             // [nb]
    IngSummary* sum;
    uint32_t* abort;           // [1] per batch (spec)
    // kwok_pod_rec12: handles of the creates only.  The chunk starts at a multiple of
    // 256 records; k_ing_prep counts the KWOK_REC_NEW records of each 256-record tile
    // of the batch (tile_new[tile0 + block]), k_ing_new_handles writes their handles
    // at their ordinals among the batch's creates (tile_pre: the tiles' prefixes)
    uint32_t* tile_new;
    uint32_t* tile_pre;
    uint32_t tile0;
};
size_t ingest_sort_bytes(uint32_t n, uint32_t key_bits);  // the bucket sort's (or rocprim's) temporary storage
// prep (+ growth counts) for every record
void launch_ingest_prep(const DevState& S, const IngestBatch& I, hipStream_t st);
// the batch's per-record statuses as bytes (kwok_ingest_pods_packed's out_status)
void launch_ingest_status8(const IngestBatch& I, int8_t* dst, hipStream_t st);
// the per-record results written into mapped host arrays (device addresses of kwok_host_alloc memory; null: skip)
void launch_ingest_results(const IngestBatch& I, int32_t* handles, int32_t* status, int8_t* status8, uint32_t* released,
                           hipStream_t st);
// kwok_pod_rec12: the chunk's creates' handles at their ordinals in new_handles (< cap),
// after scanning the NEW counts of the batch's tiles up to the chunk's last (sum->n_new)
void launch_ingest_new_handles(const IngestBatch& I, int32_t* new_handles, uint32_t cap, hipStream_t st);
// after the sort: live pods + creates of every bucket with creates -> sum->need
void launch_ingest_need(const DevState& S, const IngestBatch& I, hipStream_t st);
// stable sort by bucket, bucket ranges
int launch_ingest_sort(const DevState& S, const IngestBatch& I, void* tmp, size_t tmp_bytes, uint32_t key_bits,
                       hipStream_t st);
// the WatchPods / ListPods event switch, per bucket in event order (one wave per bucket)
void launch_ingest_apply(const DevState& S, const IngestBatch& I, hipStream_t st);

// ---- the watch-event codec on the GPU (json.hip): one thread per pod document ----
struct JsonPodArgs {
    const uint8_t* arena;        // the documents (16-aligned, 16 bytes of padding past arena_len)
    uint64_t arena_len;
    const uint64_t* doc_off;
    const uint32_t* doc_len;
    uint32_t n;
    uint32_t tab_mask;           // the spec table (kwok_register_pod_spec): open addressing, mask + 1 slots
    const JsonCfg* cfg;
    const uint8_t* op;           // ingest form (null: decode only): the caller's op and handle per document,
    const int32_t* handle;       //   the spec id from the table, a failed decode's status in reserved0
    const uint64_t* tab_key;     // json_spec_key (0: empty slot)
    const int32_t* tab_id;
    const uint2* tab_canon;      // per slot: its spec's canonical string (offset, length) in canon, checked
    const uint8_t* canon;        //   byte for byte against the document's spec after a key hit
    uint64_t key_mask;           // ~0 (KWOK_DEBUG_SPEC_KEY_BITS: fewer bits, for collision tests)
    kwok_pod_event* ev;          // [n] out
    JsonPodSide* side;           // [n] out
    uint32_t* host_list;         // [n] out: documents the host completes (JSON_HOST / JSON_SPEC), as base + index
    uint32_t base;               // the batch index of document 0 of this launch (a piece of the batch)
    uint32_t* n_host;            // [1] (zeroed by the caller)
};
void launch_json_pods(const JsonPodArgs& A, hipStream_t st);
// one thread per node document (kwok_ingest_nodes_json)
struct JsonNodeArgs {
    const uint8_t* arena;        // the documents (16 bytes of padding past arena_len)
    uint64_t arena_len;
    const uint64_t* doc_off;
    const uint32_t* doc_len;
    const uint8_t* op;           // the caller's watch event per document (the record's op)
    uint32_t n;
    const JsonCfg* cfg;
    kwok_node_event* ev;         // [n] out (op 0xFF: not applied - listed for the host, or a failed decode)
    int32_t* status;             // [n] out: KWOK_OK / KWOK_EDOMAIN / KWOK_EINVAL / JSON_HOST
    uint32_t* host_list;         // [n] out: documents the host codec decodes (JSON_HOST), as base + index
    uint32_t* n_host;            // [1] (zeroed by the caller)
    uint32_t base;               // the batch index of document 0 of this launch (a piece of the batch)
};
void launch_json_nodes(const JsonNodeArgs& A, hipStream_t st);
void launch_node_gather(const kwok_node_event* ev, const uint32_t* list, uint32_t n, kwok_node_event* out, hipStream_t st);
void launch_node_scatter(kwok_node_event* ev, const kwok_node_event* in, const uint32_t* list, uint32_t n, hipStream_t st);
void launch_json_gather(const kwok_pod_event* ev, const JsonPodSide* side, const uint32_t* list, uint32_t n,
                        kwok_pod_event* out_ev, JsonPodSide* out_side, hipStream_t st);
void launch_json_scatter(kwok_pod_event* ev, const kwok_pod_event* in, const uint32_t* list, uint32_t n, hipStream_t st);

// ---- node batches on the GPU (kwok_ingest_nodes, node_controller.go:256-270) ----
struct NodeBatch {
    const kwok_node_event* ev;  // [n] on the device or read in place
    uint32_t n;
    uint32_t host_all;          // custom node template: every UPSERT's blob comes from the host
    uint32_t force;             // k_nd_apply runs although records await the host (0: it returns then,
                                // having been queued behind the prep speculatively)
    uint32_t pad0;
    const uint8_t* arena;
    uint64_t arena_len;
    uint64_t empty_blob;        // the blob word of an empty status (default template)
    NodeRec* rec;               // [n]
    uint8_t* names;             // [n * NAME_STRIDE] the records' names
    uint32_t* keys;             // [n] owned local bucket, or nb (decided by prep / the host)
    uint32_t* keys_sorted;
    uint32_t* idx_sorted;
    uint32_t* beg;              // [nb]
    uint32_t* end;              // [nb]
    int32_t* out_handle;        // [n]
    int32_t* out_status;        // [n]
    uint32_t* host_idx;         // [n] UPSERT records the host completes (status strings)
    NodeSummary* sum;
};
// one host-completed record: its status, or its blob and flags
struct NodeFix {
    uint32_t idx;
    int32_t status;  // KWOK_OK: apply with blob / conforms
    uint64_t blob;
    uint32_t conforms, pad;
};
// record-local checks, names copied, hashes, statuses that need no state
void launch_node_prep(const DevState& S, const NodeBatch& N, hipStream_t st);
void launch_node_fix(const DevState& S, const NodeBatch& N, const NodeFix* fix, uint32_t n_fix, hipStream_t st);
// stable sort by bucket + bucket ranges (tmp: rocprim temporary storage, ingest_sort_bytes)
int launch_node_sort(const DevState& S, const NodeBatch& N, void* tmp, size_t tmp_bytes, uint32_t key_bits,
                     hipStream_t st);
// the WatchNodes / ListNodes event switch, one wave per bucket in event order
void launch_node_apply(const DevState& S, const NodeBatch& N, hipStream_t st);
// zombie node entries (deleted / placeholder) no pod references any more are freed
void launch_free_zombies(const DevState& S, hipStream_t st);
// the managed nodes before each chain block and each bucket (heartbeat handle bases) from mb_count
void launch_hb_pre(const DevState& S, uint32_t* hb_pre, uint32_t* hb_bpre, hipStream_t st);
// kwok_node_has: names[i * NAME_STRIDE] (lens[i] bytes) -> out[i] = the entry's node_state (0: none)
void launch_node_lookup(const DevState& S, const uint8_t* names, const uint32_t* lens, uint32_t n, uint32_t* out,
                        hipStream_t st);
// kwok_cni_assign: statuses of every record; wr[i]: record i is the handle's last
// valid assignment (it writes the podIP)
void launch_cni_assign(const DevState& S, const int32_t* handles, const uint32_t* ips, const uint8_t* wr, uint32_t n,
                       int32_t* status, uint32_t* rejected, hipStream_t st);

}  // namespace kwok
