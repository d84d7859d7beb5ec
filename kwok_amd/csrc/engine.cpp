// engine.cpp - host runtime behind include/kwok_engine.h.
//
// Owns one GPU: device SoA state, the output arena, the replicated ipPool
// bitmaps and (multi-rank) an RCCL communicator.  Host-side it keeps only what
// the slot policy needs (names -> node slots, slot occupancy, refcounts); all
// per-object status lives in HBM and is advanced by the kernels of one tick.
//
// Reference interfaces replaced (hezhizhen/kwok, pkg/kwok/controllers):
//   NewController / NewNodeController / NewPodController  controller.go:80-152,
//                                                          node_controller.go:79-117, pod_controller.go:84-128
//   WatchNodes/ListNodes, WatchPods/ListPods event switch node_controller.go:256-295, pod_controller.go:301-367
//   KeepNodeHeartbeat, LockNodes, LockPods, DeletePods    node_controller.go:175-204,301-354, pod_controller.go:155-250
//   ipPool                                                utils.go:52-117
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <string.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/kwok_engine.h"
#include "codec.h"
#include "device.h"
#include "gotemplate.h"
#include "kernels.h"
#include "templates.h"

using namespace kwok;

namespace {

// FNV-1a 64 of a pod spec's strings (json.hip spec_key is the same function):
// each container's name 0x1F image 0x1E, 0x1D, the init containers alike, 0x1D,
// each readiness gate 0x1E
// The canonical byte string the key hashes; the GPU codec compares a document's
// spec with it after a table hit (the key alone is not collision-resistant)
std::string json_spec_canon(const std::vector<Container>& cs, const std::vector<Container>& ics,
                            const std::vector<std::string>& gates) {
    std::string o;
    for (auto& c : cs) o += c.name, o += '\x1F', o += c.image, o += '\x1E';
    o += '\x1D';
    for (auto& c : ics) o += c.name, o += '\x1F', o += c.image, o += '\x1E';
    o += '\x1D';
    for (auto& g : gates) o += g, o += '\x1E';
    return o;
}
// KWOK_DEBUG_SPEC_KEY_BITS=b (tests): keys cut to their low b bits, so that
// distinct specs collide and the device's byte check decides
uint64_t spec_key_mask() {  // (read per call: registrations and decode launches are rare)
    const char* v = getenv("KWOK_DEBUG_SPEC_KEY_BITS");
    const unsigned b = v ? (unsigned)atoi(v) : 64u;
    return b >= 64 || b == 0 ? ~0ull : (1ull << b) - 1ull;
}
uint64_t json_spec_key(const std::string& canon) {
    uint64_t h = 0xCBF29CE484222325ull;
    for (unsigned char c : canon) h = (h ^ c) * 0x100000001B3ull;
    return h & spec_key_mask();
}
uint64_t json_spec_key(const std::vector<Container>& cs, const std::vector<Container>& ics,
                       const std::vector<std::string>& gates) {
    return json_spec_key(json_spec_canon(cs, ics, gates));
}

thread_local std::string g_create_err;  // kwok_last_error(NULL) after a failed create
using clk = std::chrono::steady_clock;
double ms_between(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); }

uint32_t fnv1a32(const char* s, size_t n) {
    uint32_t h = 0x811C9DC5u;
    for (size_t i = 0; i < n; i++) {
        h ^= (unsigned char)s[i];
        h *= 0x01000193u;
    }
    return h;
}

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
};

// Persistent host worker threads for the ingest partitions (started on first
// use): run(n, f) calls f(0) on the caller and f(1..n-1) on the workers, and
// returns when all are done.
class WorkPool {
  public:
    ~WorkPool() {
        {
            std::lock_guard<std::mutex> l(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void run(int n, const std::function<void(int)>& f) {
        while ((int)th_.size() < n - 1) {
            const int id = (int)th_.size() + 1;
            th_.emplace_back([this, id] { loop(id); });
        }
        {
            std::lock_guard<std::mutex> l(m_);
            job_ = &f;
            width_ = n;
            left_ = n - 1;
            gen_++;
        }
        cv_.notify_all();
        f(0);
        std::unique_lock<std::mutex> l(m_);
        done_.wait(l, [&] { return left_ == 0; });
        job_ = nullptr;
    }

  private:
    void loop(int id) {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> l(m_);
        for (;;) {
            cv_.wait(l, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            if (id >= width_) continue;  // this run uses fewer workers
            const std::function<void(int)>* f = job_;
            l.unlock();
            (*f)(id);
            l.lock();
            if (--left_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* job_ = nullptr;
    uint64_t gen_ = 0;
    int width_ = 0, left_ = 0;
    bool stop_ = false;
};

}  // namespace

struct kwok_engine {
    kwok_config cfg{};
    std::string err;
    int W = 1, rank = 0, dev = 0;
    int XW = 1;  // exchange messages per tick: W, or KWOK_EMULATE_RANKS on a one-rank multi engine (diagnostics)
    bool multi = false;  // the FRONT / exchange / BACK tick (W > 1, or KWOK_FORCE_MULTI with one rank)
    uint32_t B = 0, Cn = 0, Cp = 0, b_lo = 0, b_hi = 0, nb = 0, NL = 0, PL = 0;
    uint32_t Hs = 0;  // pod handle stride: handle = bucket * Hs + slot in the bucket; Cp grows up to it
    PoolGeom pool{};
    uint32_t node_ip = 0;
    std::string node_ip_s;
    int64_t start = 0;
    hipStream_t st = nullptr;   // tick pipeline
    hipEvent_t fence = nullptr; // recorded (system-scope release) before device -> host copies of kernel output
    hipStream_t rst = nullptr;  // kwok_read_outputs: copies of a collected tick, beside the next tick's kernels
    // large arena reads split over more copy streams (KWOK_READ_STREAMS, default 1: two or
    // four streams measured no faster than one, ~44 GB/s device-to-host either way)
    int read_streams = 1;
    hipStream_t rsx[3] = {};
    hipEvent_t rd_go = nullptr, rd_part[3] = {};
    DevState S{};

    // ---- nodes: the directory (names -> slots), occupancy, managed / zombie counts
    // live on the device (ingest.hip); the host keeps the managed-set size ----
    uint64_t n_managed = 0;
    bool hb_pre_dirty = true;                        // the per-chain-block heartbeat bases need k_hb_pre
    uint32_t hb_epoch = 0;                           // kwok_tick_result.heartbeat_epoch: bumped when the managed set changes
    uint32_t* d_hb_pre = nullptr;
    uint32_t* d_hb_bpre = nullptr;                   // [nb + 1] per-bucket bases (k_once)
    // pods: no host mirror.  The device's pod_state (USED = slot occupancy),
    // pod_node and node_state (NS_SLOT) are the state the GPU ingest pass
    // (ingest.hip) applies batches to; pod_fill is its per-bucket fill mark.
    uint16_t* d_pod_fill = nullptr;

    // ---- host work of node batches: the status strings of UPSERT records with a
    // non-empty status (string checks, blob interning, custom node templates), on up
    // to n_part host threads ----
    int n_part = 1;
    std::vector<uint32_t> puts;  // kwok_pool_put (other ranks' ingest-time releases), staged for flush_ops
    void* pinned = nullptr;
    size_t pinned_cap = 0;
    void* d_ops = nullptr;
    size_t d_ops_cap = 0;

    // ---- GPU pod ingest (ingest.hip) ----
    struct Ingest {
        size_t cap = 0;          // records the per-record buffers hold
        size_t arena_cap = 0;
        size_t sort_bytes = 0;
        void* d_ev = nullptr;
        uint8_t* d_arena = nullptr;
        PodRec* rec = nullptr;
        uint32_t *keys = nullptr, *keys_sorted = nullptr, *idx_sorted = nullptr;
        int32_t *out_handle = nullptr, *out_status = nullptr;
        int8_t* out_status8 = nullptr;  // kwok_ingest_pods_packed: the statuses as bytes
        uint32_t* out_released = nullptr;
        void* sort_tmp = nullptr;
        // kwok_ingest_pods_packed12: NEW records per 256-record tile, the tiles' prefixes,
        // the creates' handles in create order
        uint32_t *tile_new = nullptr, *tile_pre = nullptr;
        int32_t* new_handle = nullptr;
        // per bucket (allocated once)
        uint32_t *beg = nullptr, *end = nullptr;
        uint32_t* abort = nullptr;          // [1] a chunk of the batch needs growth (speculative apply passes)
        IngSummary* sums = nullptr;         // [nsums] one per chunk of a batch
        IngSummary* sums_h = nullptr;       // pinned
        size_t nsums = 0;
        IngSummary* sum = nullptr;
        // node batches (kwok_ingest_nodes): records, names, prepared records, host list
        size_t ncap = 0;
        kwok_node_event* d_nev = nullptr;
        uint8_t* d_nnames = nullptr;  // [ncap * NAME_STRIDE]
        NodeRec* nrec = nullptr;
        uint32_t* host_idx = nullptr;
        NodeFix* d_nfix = nullptr;
        NodeSummary* nsum = nullptr;
        NodeSummary* nsum_h = nullptr;  // pinned
        int32_t* res_h = nullptr;       // pinned [2 * ncap]: handles, statuses
        IngSummary* sum_h = nullptr;  // pinned
        // a batch runs in chunks (KWOK_INGEST_CHUNK records): chunk k+1's prep reads its
        // records over the link on `pst` while chunk k is applied and its results copied
        // back on the engine stream
        IngSummary* sum1 = nullptr;
        hipStream_t pst = nullptr, dst = nullptr;  // prep (H2D + k_ing_prep) / results (D2H)
        hipEvent_t tev[8] = {};  // KWOK_INGEST_PROF: device-side phase stamps of a two-chunk batch
        hipEvent_t go = nullptr, prepped[2] = {nullptr, nullptr}, used[2] = {nullptr, nullptr};
        hipEvent_t idone = nullptr;  // a pod batch's last operation (the host spins on it: KWOK_SYNC)
        hipEvent_t rdone = nullptr;  // the results stream's work of a batch (kwok_pod_rec12: before the summaries)
        size_t chunk = 1048576;
    } ing;

    // ---- the pod codec on the GPU (json.hip): per-document buffers, the codec's
    // selectors, the spec table (kwok_spec_key -> spec id) ----
    struct Json {
        size_t cap = 0;
        uint64_t* off = nullptr;
        uint32_t* len = nullptr;
        uint8_t* op = nullptr;
        int32_t* handle = nullptr;
        JsonPodSide* side = nullptr;
        uint32_t* host_list = nullptr;
        kwok_pod_event* fix_ev = nullptr;  // the listed documents' records (gathered, completed, scattered)
        JsonPodSide* fix_side = nullptr;
        uint32_t* n_host = nullptr;        // device [1]
        uint32_t* n_host_h = nullptr;      // pinned [1]
        JsonCfg* cfg = nullptr;
        JsonCfg* cfg_h = nullptr;          // pinned staging
        uint64_t* tab_key = nullptr;
        int32_t* tab_id = nullptr;
        int32_t* nstat = nullptr;          // node documents: the device decode's status per document
        kwok_node_event* nev_fix = nullptr;  // node records gathered for / scattered from the host
        size_t ncap = 0;
        uint2* tab_canon = nullptr;        // per slot: offset / length of its spec's canonical string in canon
        uint8_t* canon = nullptr;          // the registered specs' canonical strings (json_spec_canon)
        size_t canon_cap = 0;
        uint32_t tab_mask = 0;
        bool tab_dirty = true;
    } json;
    std::unordered_map<uint64_t, int32_t> spec_keys;  // kwok_spec_key -> spec id (-2: two specs share the key)
    std::unordered_map<uint64_t, std::string> spec_canon;  // kwok_spec_key -> the canonical string of its spec

    // ---- specs / blobs ----
    std::unordered_map<std::string, int32_t> spec_ids;
    uint32_t hb_len = HB_LEN, hb_stride = HB_STRIDE;  // heartbeat patch bytes / arena stride (16-aligned)
    HeartbeatTemplate hb_tpl;     // the heartbeat template (default or compiled from Config.NodeHeartbeatTemplate)
    bool custom_hb = false;
    std::string hb_tpl_text;
    bool custom_pod = false;      // Config.PodStatusTemplate in use (compiled per spec)
    bool custom_node = false;     // Config.NodeInitializationTemplate in use (compiled per node status)
    std::string pod_tpl, node_tpl, start_s;  // their texts; StartTime() (RFC3339 of start_time_unix)
    std::unordered_map<std::string, uint64_t> node_tpl_blobs;  // node status fields -> compiled blob
    std::vector<SpecDesc> specs_h;
    std::string spec_bytes_h;
    DevBuf<SpecDesc> d_specs;
    DevBuf<uint8_t> d_spec_bytes;
    std::vector<uint16_t> spec_nxt_h;  // timestamp lookups of every spec (build_ts_lookup)
    DevBuf<uint16_t> d_spec_nxt;
    DevBuf<uint8_t> d_unit_tab;      // k_emit's unit tables (16 bytes per unit), appended per spec
    DevBuf<uint16_t> d_unit_desc;
    uint32_t tab_units = 0;
    uint32_t max_pod_len = 0;
    std::unordered_map<std::string, uint64_t> blob_ids;
    uint64_t empty_blob = 0;      // the blob of a node with an empty status (every status field absent)
    std::atomic<bool> has_empty_blob{false};
    std::string blob_h;
    size_t blob_up_lo = SIZE_MAX;  // blob_h bytes from here on are not on the device yet (upload_blobs)
    DevBuf<uint8_t> d_blob;
    uint32_t max_init_len = 0;

    // ---- tick ----
    // A tick's outputs (header, lists, arena) live in one of two slots, so tick N+1
    // can be queued while tick N is collected (kwok_tick_submit / _collect).  Slot 1
    // is allocated on the first submit that finds slot 0 busy.
    struct TickSlot {
        TickHdr* hdr_h = nullptr;  // pinned: k_tick publishes the field totals here
        uint8_t* arena = nullptr;
        uint64_t arena_cap = 0;
        int32_t *hb_nodes = nullptr, *init_nodes = nullptr, *pp_pods = nullptr, *del_pods = nullptr;
        uint64_t *init_off = nullptr, *pp_off = nullptr;
        uint32_t *init_len = nullptr, *pp_len = nullptr;
        uint8_t* del_fin = nullptr;
        DevState* d_S = nullptr;    // S with this slot's outputs, in device memory (out-of-line kernel phases)
        DevState* S_pin = nullptr;  // pinned staging for its upload
        DevState S_up{};            // the copy last uploaded
        hipEvent_t done = nullptr;  // recorded after the tick's launches
        hipEvent_t pev[8] = {};     // profiling: FRONT(+BACK) launch start/stop, BACK launch start/stop, k_emit,
                                    // k_pod_jobs
        uint4* pp_job = nullptr;    // k_tick -> k_emit job records
        uint64_t* init_job = nullptr;
        uint32_t* emit_n = nullptr;
        bool emit_queued = false;   // k_emit was enqueued behind the tick's launches
        bool split = false;         // TICK_SPLIT: k_pod_jobs builds the pod jobs after the tick's launches
        bool fuse = false;          // ... and writes their patch bytes itself (DevState::fuse_pods)
        bool inits_folded = false;  // ... and the node inits' too (no k_emit launch: KWOK_FOLD_INITS)
        bool quiet = false;         // only pods with an event are Use-checked (kwok_engine::quiet)
        bool once = false;          // launched as k_once (a heartbeat-once tick expected to have nothing to emit)
        bool once_use = false;      // ... reading the per-bucket summaries (counted when it retires as a once tick)
        hipEvent_t rd = nullptr;    // kwok_read_arena_async: the last read queued from this slot's arena
        bool rd_pending = false;    //   (a submit or an arena growth that takes the slot waits for it)
        bool no_once = false;       // k_once found work: the tick runs again with k_tick
        bool alloc = false;
        // the tick in the slot
        int state = 0;  // SLOT_FREE, SLOT_QUEUED (enqueued), SLOT_DONE (finished on the host, not collected)
        uint64_t now = 0, target = 0;
        uint32_t tag = 0;
        uint32_t epoch = 0;         // heartbeat_epoch of the tick
        int rc = 0;
        std::string err;
        kwok_tick_result res{};
    };
    TickSlot slots[2];
    int queue[2] = {-1, -1};  // queued / done slots in submission order
    int nq = 0;
    int cur = -1;             // slot of the last collected tick (kwok_read_outputs)
    size_t NLa = 0, PLa = 0;  // output list capacities
    uint64_t arena_need = 0;  // worst-case output bytes of one tick
    ListDesc* d_ld = nullptr;  // [W] or scratch
    ncclComm_t comm = nullptr;
    XMsg* d_xall = nullptr;
    XMsg* h_xall = nullptr;  // pinned
    uint32_t* d_xsend = nullptr;
    uint32_t* d_xrecv = nullptr;
    size_t xlist_cap = 0;
    // TICK_XSPEC: after a tick whose lists were too long to be inline, the next
    // ticks send their lists in a second allgather right behind the messages (no
    // host round trip) with capacities from that tick's longest lists; every rank
    // takes the same decisions (from the same gathered messages, in lockstep)
    uint32_t xspec_u = 0, xspec_r = 0;  // capacities per rank (0: off)
    uint32_t xspec_ttl = 0;             // ticks left
    uint32_t xspec_alloc = 0;           // entries allocated per rank in d_ssend / d_srecv
    uint32_t* d_ssend = nullptr;
    uint32_t* d_srecv = nullptr;
    int xspec_env = -1;                 // KWOK_XSPEC: 0 off, N: ticks kept on after a long-list tick (default 256)
    uint64_t xspec_miss = 0;  // diagnostics: speculative ticks whose lists did not fit
    uint32_t n_stream = 0;      // k_tick heartbeat streamer blocks (the chain blocks: S.n_chain)
    uint32_t emit_grid = 0;     // k_emit blocks
    bool emit_hint = true;      // events were ingested since the last submit: the tick likely emits patches
    bool sync_spin = true;      // spin on a tick's completion event (KWOK_SYNC=spin, the default)
    bool chain_prio = false;    // KWOK_TICK_PRIO=1: s_setprio 3 on the chain blocks
    bool no_stream = false;     // KWOK_TICK_NO_STREAM=1: diagnostics - heartbeat bodies not written
    bool split_jobs = true;     // KWOK_SPLIT=0: pod jobs of event ticks in the chain blocks (A/B)
    int fuse_emit = -1;         // KWOK_FUSE_EMIT: 1 always / 0 never fuse the pod bytes into k_pod_jobs; -1 dense ticks
    bool sparse_jobs = true;    // unfused split ticks: k_sparse_jobs over FRONT's group records (KWOK_SPARSE_JOBS=0: off)
    bool fold_inits = true;     // KWOK_FOLD_INITS=0: a fused tick's node inits by k_emit (A/B)
    uint64_t pod_records_since_tick = 0;  // pod records ingested since the last tick was enqueued (fused emission)
    uint32_t n_untabled = 0;    // registered specs without unit tables (no fused emission while any)
    // Quiet ticks.  A tick's Use(podIP) of an evaluated pod (pod_controller.go:
    // 378-382) is a no-op when the address is already in `used`.  Only a Put clears
    // a bit, and Puts come from ingest (Deleted events), kwok_pool_put, and the
    // deletions a tick makes of the pods marked at the ingest before it.  So after
    // two submits with nothing in between, the previous tick Use-checked every
    // evaluated pod and released nothing: this tick need only Use-check pods with
    // an event (single rank; KWOK_QUIET=0 checks every pod).
    // Also, while every in-CIDR podIP a live pod holds was assigned to it by this
    // engine (no pod was created or updated with a podIP of its own, and no Deleted
    // event released an address its pod did not hold: the GPU apply pass flags
    // those, IngSummary::foreign), every such address has exactly one holder and
    // stays in `used` until that holder is deleted: then no Use changes anything
    // and the Use checks of pods without an event are skipped in every tick.
    uint32_t quiet = 0;         // submits since the last ingest / pool_put / cni_assign
    bool foreign_ips = false;   // sticky: a podIP not assigned by this engine entered the pool
    bool global_foreign = false;  // multi rank, sticky: some rank's exchange message carried its foreign_ips
    bool quiet_ok = true;
    bool once_ok = true;        // KWOK_ONCE=0: heartbeat-once ticks always run k_tick (A/B)
    // k_once's per-bucket summaries (DevState::once_sum): valid while nothing has changed a
    // pod state since the BUILD tick of generation sum_gen was enqueued (every ingest, CNI
    // assignment, pool Put, zombie sweep and k_tick launch clears sum_valid)
    bool once_sum_ok = true;    // KWOK_ONCE_SUM=0: every k_once tick reads the pod rows (A/B)
    bool sum_valid = false;
    uint32_t sum_gen = 0;
    uint64_t stats[KWOK_STAT_COUNT] = {};  // kwok_engine_stats
    uint8_t* dump_h = nullptr;  // kwok_dump_pods' page-locked staging
    size_t dump_cap = 0;
    bool ingest_zc = true;      // KWOK_INGEST_ZC=0: pod batches in kwok_host_alloc memory copied to HBM first
    bool results_stream = true;   // KWOK_INGEST_RS=0: a chunked batch's results copied on the engine stream
    bool results_kernel = false;  // KWOK_INGEST_RESULTS_KERNEL=1: pod batch results written into mapped host arrays by a kernel
    double last_chunk_cut = 0.4;  // KWOK_INGEST_LAST_CUT: a chunked batch's last chunk is (1 - this) of the others
    bool new_mapped = true;       // KWOK_INGEST_NEW_MAPPED=0: kwok_pod_rec12 create handles copied back, not written in place
    int nt_env = -1;            // KWOK_HB_NT (0 / 1: heartbeat stores plain / non-temporal), else automatic
    int share_env = -1;         // KWOK_TICK_STREAM_SHARE (/1024 of the stream to the streamer blocks), else automatic
    uint32_t tick_tag = 0;      // nonzero id of the last FRONT launch
    uint64_t front_launches = 0;  // FRONT launches since the cross-block state was last zeroed
    // diagnostics
    bool prof = false;
    double prof_ms[KWOK_T_COUNT] = {};
    uint64_t prof_ticks = 0;
    double host_ms[KWOK_H_COUNT] = {};
    // KWOK_TICK_TRACE=1: per-block phase stamps, summarised on stderr at destroy
    std::vector<uint64_t> trace_h;
    double trace_sum[TRACE_SLOTS + 2][3] = {};  // chain stamps, streamer entry / exit
    uint64_t trace_ticks = 0, trace_seen = 0;
    uint64_t host_ticks = 0;
    // a failed tick leaves device and host state out of step: every later call
    // fails with KWOK_EDEVICE (destroy and recreate the engine, re-ingest by List)
    bool poisoned = false;
    bool iprof = false;
    WorkPool workers;  // host threads of the ingest partitions  // KWOK_INGEST_PROF=1: host ingest / retire phase times on stderr
    uint32_t debug_fail_chunk = 0;  // KWOK_DEBUG_INGEST_FAIL_CHUNK=N: chunk N of a pod batch fails before its apply (tests)
    uint32_t debug_fail_apply = 0;  // KWOK_DEBUG_INGEST_FAIL_APPLY=N: chunk N fails after its first apply pass (tests)
    // the pod batch in progress changed the state (placeholder nodes, capacity, the
    // apply pass): a failure from then on leaves the batch partly applied (poison)
    bool ing_mutated = false;
    uint32_t ing_chunk = 0;     // the chunk ingest_chunk works on (debug injection)
    uint64_t debug_fault_tick = 0;  // KWOK_DEBUG_LAYOUT_FAULT_TICK=N: tick N gets a wrong heartbeat layout (tests)

    int fail(int code, const char* fmt, ...) {
        char b[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(b, sizeof b, fmt, ap);
        va_end(ap);
        err = b;
        return code;
    }
    bool owns(uint32_t bucket) const { return bucket >= b_lo && bucket < b_hi; }
    // pod handle <-> local slot (bucket_local * Cp + index)
    int32_t pod_handle(uint32_t slot) const { return (int32_t)((b_lo + slot / Cp) * Hs + slot % Cp); }
    // KWOK_OK (slot set), KWOK_ENOTMINE (another rank's bucket) or KWOK_ENOTFOUND
    int pod_slot(int64_t h, uint32_t* slot) const {
        if (h < 0 || h / Hs >= B) return KWOK_ENOTFOUND;
        const uint32_t b = (uint32_t)(h / Hs), i = (uint32_t)(h % Hs);
        if (!owns(b)) return KWOK_ENOTMINE;
        if (i >= Cp) return KWOK_ENOTFOUND;
        *slot = (b - b_lo) * Cp + i;
        return KWOK_OK;
    }
};

#define HIPCHK(e, x)                                                                              \
    do {                                                                                          \
        hipError_t _r = (x);                                                                      \
        if (_r != hipSuccess) return (e)->fail(KWOK_EDEVICE, "%s: %s", #x, hipGetErrorString(_r)); \
    } while (0)

namespace {

// kwok_host_alloc buffers (base -> length, device address, mmap'd + registered)
struct HostReg {
    size_t len;
    uint8_t* dev;
    bool mmapped;
};
std::mutex g_host_mu;
std::map<uintptr_t, HostReg> g_host_reg;
// the device address of [p, p + n) when it lies inside one kwok_host_alloc
// buffer (kernels read it in place over the link), else null
const void* host_mapped(const void* p, size_t n) {
    const uintptr_t a = (uintptr_t)p;
    std::lock_guard<std::mutex> l(g_host_mu);
    auto it = g_host_reg.upper_bound(a);
    if (it == g_host_reg.begin()) return nullptr;
    --it;
    const HostReg& r = it->second;
    if (!r.dev || a + n > it->first + r.len) return nullptr;
    return r.dev + (a - it->first);
}

template <class T>
int dalloc(kwok_engine* e, T** p, size_t n) {
    size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
    hipError_t r = hipMalloc((void**)p, bytes);
    if (r != hipSuccess) return e->fail(KWOK_ENOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(r));
    r = hipMemsetAsync(*p, 0, bytes, e->st);
    if (r != hipSuccess) return e->fail(KWOK_EDEVICE, "hipMemset: %s", hipGetErrorString(r));
    return KWOK_OK;
}

// grow a device buffer to hold `bytes` (keeps contents)
template <class T>
int dgrow(kwok_engine* e, DevBuf<T>& b, size_t n) {
    if (n <= b.n) return KWOK_OK;
    size_t cap = std::max<size_t>(n, b.n * 2 + 64);
    T* p = nullptr;
    if (hipMalloc((void**)&p, cap * sizeof(T)) != hipSuccess) return e->fail(KWOK_ENOMEM, "grow %zu", cap * sizeof(T));
    if (b.p) {
        HIPCHK(e, hipMemcpyAsync(p, b.p, b.n * sizeof(T), hipMemcpyDeviceToDevice, e->st));
        HIPCHK(e, hipStreamSynchronize(e->st));
        (void)hipFree(b.p);
    }
    b.p = p;
    b.n = cap;
    return KWOK_OK;
}

int ensure_pinned(kwok_engine* e, size_t bytes) {
    if (bytes <= e->pinned_cap) return KWOK_OK;
    if (e->pinned) (void)hipHostFree(e->pinned);
    e->pinned_cap = std::max(bytes, e->pinned_cap * 2);
    if (hipHostMalloc(&e->pinned, e->pinned_cap, hipHostMallocDefault) != hipSuccess)
        return e->fail(KWOK_ENOMEM, "pinned %zu", e->pinned_cap);
    if (e->d_ops_cap < e->pinned_cap) {
        if (e->d_ops) (void)hipFree(e->d_ops);
        e->d_ops_cap = e->pinned_cap;
        if (hipMalloc(&e->d_ops, e->d_ops_cap) != hipSuccess) return e->fail(KWOK_ENOMEM, "ops %zu", e->d_ops_cap);
    }
    return KWOK_OK;
}


// Run f(p) for every ingest partition p: on n_part host threads when the batch
// is large enough to pay for them, else in order on the caller's thread.
template <class F>
void run_parts(kwok_engine* e, bool parallel, F&& f) {
    if (!parallel || e->n_part == 1) {
        for (int p = 0; p < e->n_part; p++) f(p);
        return;
    }
    const std::function<void(int)> fn = [&f](int p) { f(p); };
    e->workers.run(e->n_part, fn);
}
constexpr size_t NODE_PAR_MIN = 2048;  // node records (the per-record work is heavier)

// kwok_pool_put's staged releases -> one host-to-device copy -> the pool
int flush_ops(kwok_engine* e) {
    const size_t nu = e->puts.size();
    if (!nu) return KWOK_OK;
    if (int rc = ensure_pinned(e, nu * 4 + 256)) return rc;
    memcpy(e->pinned, e->puts.data(), nu * 4);
    HIPCHK(e, hipMemcpyAsync(e->d_ops, e->pinned, nu * 4, hipMemcpyHostToDevice, e->st));
    // ingest-time releases of other ranks (pod_controller.go:329-336)
    launch_pool_puts_now(e->S, (const uint32_t*)e->d_ops, (uint32_t)nu, e->st);
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipStreamSynchronize(e->st));
    e->puts.clear();
    return KWOK_OK;
}

int upload_specs(kwok_engine* e) {
    int rc;
    if ((rc = dgrow(e, e->d_specs, e->specs_h.size()))) return rc;
    // the kernels read the spec bytes as 32-bit words, up to SRC_PAD_FRONT bytes
    // before a segment and SRC_PAD_BACK past the end
    std::string bytes(SRC_PAD_FRONT, '\0');
    bytes += e->spec_bytes_h;
    bytes.resize(((bytes.size() + 3) & ~(size_t)3) + SRC_PAD_BACK, '\0');
    if ((rc = dgrow(e, e->d_spec_bytes, bytes.size()))) return rc;
    if ((rc = dgrow(e, e->d_spec_nxt, std::max<size_t>(e->spec_nxt_h.size(), 1)))) return rc;
    HIPCHK(e, hipMemcpyAsync(e->d_specs.p, e->specs_h.data(), e->specs_h.size() * sizeof(SpecDesc),
                             hipMemcpyHostToDevice, e->st));
    HIPCHK(e, hipMemcpyAsync(e->d_spec_bytes.p, bytes.data(), bytes.size(), hipMemcpyHostToDevice, e->st));
    if (!e->spec_nxt_h.empty())
        HIPCHK(e, hipMemcpyAsync(e->d_spec_nxt.p, e->spec_nxt_h.data(), e->spec_nxt_h.size() * 2, hipMemcpyHostToDevice, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    e->S.specs = e->d_specs.p;
    e->S.spec_bytes = e->d_spec_bytes.p + SRC_PAD_FRONT;
    e->S.spec_nxt = e->d_spec_nxt.p;
    e->S.nxt_total = (uint32_t)e->spec_nxt_h.size();
    e->S.n_specs = (uint32_t)e->specs_h.size();
    e->S.spec_total = (uint32_t)e->spec_bytes_h.size();
    return KWOK_OK;
}

int drain(kwok_engine* e);  // finish every queued tick on the host (below)
int tick_submit_check(kwok_engine* e, int64_t now_unix);  // kwok_tick_submit's checks / the rest (below)
int tick_submit_impl(kwok_engine* e, int64_t now_unix);
int enqueue_tick(kwok_engine* e, int k, bool requeue);
int poisoned(kwok_engine* e) {
    return e->fail(KWOK_EDEVICE, "a failed tick left the engine out of step with the device: destroy it and "
                                 "recreate it (re-ingest by List)");
}

// the output arena must hold the worst case of one tick.  It changes when the
// capacity, the specs or the node blobs do (ingest, registration), and is
// reserved then for the slots the next submit may take (a free slot whose outputs
// the caller is not reading), not inside that tick: the 1M x 10M fleet's first
// tick would otherwise reallocate ~8 GB (~0.7 ms of its enqueue).  A slot still
// queued grows at its next submit.
enum { SLOT_FREE = 0, SLOT_QUEUED = 1, SLOT_DONE = 2 };
int grow_arena(kwok_engine* e, kwok_engine::TickSlot& T);
int size_arena(kwok_engine* e) {
    e->arena_need = (uint64_t)e->NL * e->hb_stride + (uint64_t)e->NL * ((e->max_init_len + 15u) & ~15u) +
                    (uint64_t)e->PL * e->max_pod_len + 256;
    for (int i = 0; i < 2; i++) {
        kwok_engine::TickSlot& T = e->slots[i];
        if (T.alloc && T.state == SLOT_FREE && i != e->cur)
            if (int rc = grow_arena(e, T)) return rc;
    }
    return KWOK_OK;
}
int grow_arena(kwok_engine* e, kwok_engine::TickSlot& T) {  // T holds no queued tick
    if (e->arena_need <= T.arena_cap) return KWOK_OK;
    if (T.rd_pending) {  // (an asynchronous read of the old arena still in flight)
        if (hipEventSynchronize(T.rd) != hipSuccess) return e->fail(KWOK_EDEVICE, "kwok_read_arena_async");
        T.rd_pending = false;
    }
    const uint64_t need = std::max<uint64_t>(e->arena_need, T.arena_cap + T.arena_cap / 2);
    if (T.arena) (void)hipFree(T.arena);
    T.arena = nullptr;
    T.arena_cap = 0;
    if (hipMalloc((void**)&T.arena, need) != hipSuccess) return e->fail(KWOK_ENOMEM, "arena %llu", (unsigned long long)need);
    T.arena_cap = need;
    if (getenv("KWOK_DEBUG_POISON"))  // diagnostics: bytes no kernel writes read as 0xEE, not as stale data
        HIPCHK(e, hipMemsetAsync(T.arena, 0xEE, need, e->st));
    return KWOK_OK;
}
int alloc_slot(kwok_engine* e, int k) {
    kwok_engine::TickSlot& T = e->slots[k];
    int rc = 0;
    if ((rc = dalloc(e, &T.hb_nodes, e->NLa)) || (rc = dalloc(e, &T.init_nodes, e->NLa)) ||
        (rc = dalloc(e, &T.init_off, e->NLa)) || (rc = dalloc(e, &T.init_len, e->NLa)) ||
        (rc = dalloc(e, &T.pp_pods, e->PLa)) || (rc = dalloc(e, &T.pp_off, e->PLa)) || (rc = dalloc(e, &T.pp_len, e->PLa)) ||
        (rc = dalloc(e, &T.del_pods, e->PLa)) || (rc = dalloc(e, &T.del_fin, e->PLa)) || (rc = dalloc(e, &T.d_S, 1)) ||
        (rc = dalloc(e, &T.pp_job, e->PLa)) || (rc = dalloc(e, &T.init_job, e->NLa)) || (rc = dalloc(e, &T.emit_n, 2)))
        return rc;
    // the header is coherent host memory written with system-scope stores, so the
    // completion event needs no system-scope release (measured ~1.7 us per tick)
    if (hipHostMalloc((void**)&T.hdr_h, sizeof(TickHdr), hipHostMallocCoherent) != hipSuccess ||
        hipHostMalloc((void**)&T.S_pin, sizeof(DevState), hipHostMallocDefault) != hipSuccess)
        return e->fail(KWOK_ENOMEM, "pinned tick header");
    memset(T.hdr_h, 0, sizeof(TickHdr));
    if (hipEventCreateWithFlags(&T.done, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess)
        return e->fail(KWOK_EDEVICE, "event create");
    for (auto& ev : T.pev)
        if (e->prof && !ev) HIPCHK(e, hipEventCreate(&ev));
    T.alloc = true;
    return KWOK_OK;
}
void free_slot(kwok_engine::TickSlot& T) {
    void* ptrs[] = {T.arena, T.hb_nodes, T.init_nodes, T.init_off, T.init_len, T.pp_pods,
                    T.pp_off, T.pp_len, T.del_pods, T.del_fin, T.d_S, T.pp_job, T.init_job, T.emit_n};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (T.hdr_h) (void)hipHostFree(T.hdr_h);
    if (T.S_pin) (void)hipHostFree(T.S_pin);
    if (T.done) (void)hipEventDestroy(T.done);
    if (T.rd) (void)hipEventDestroy(T.rd);
    for (auto& ev : T.pev)
        if (ev) (void)hipEventDestroy(ev);
}
// this slot's outputs into S (what launches read), uploaded to the slot's device copy if changed
int bind_slot(kwok_engine* e, int k) {
    kwok_engine::TickSlot& T = e->slots[k];
    DevState& S = e->S;
    S.arena = T.arena;
    S.arena_cap = T.arena_cap;
    S.hb_nodes = T.hb_nodes;
    S.init_nodes = T.init_nodes;
    S.init_off = T.init_off;
    S.init_len = T.init_len;
    S.pp_pods = T.pp_pods;
    S.pp_off = T.pp_off;
    S.pp_len = T.pp_len;
    S.del_pods = T.del_pods;
    S.del_fin = T.del_fin;
    S.hdr_host = T.hdr_h;
    S.self = T.d_S;
    S.pp_job = T.pp_job;
    S.init_job = T.init_job;
    S.emit_n = T.emit_n;
    if (memcmp(&T.S_up, &S, sizeof(DevState)) != 0) {  // pointers / sizes changed since the last upload
        *T.S_pin = S;  // the slot's previous upload has completed (its tick was collected)
        HIPCHK(e, hipMemcpyAsync(T.d_S, T.S_pin, sizeof(DevState), hipMemcpyHostToDevice, e->st));
        T.S_up = S;
    }
    return KWOK_OK;
}

uint64_t intern_blob(kwok_engine* e, const NodeBlob& b, int* rc) {
    std::string key = b.pre + '\x01' + b.post;
    auto it = e->blob_ids.find(key);
    if (it != e->blob_ids.end()) return it->second;
    // k_emit keeps patch positions in 16 bits
    if (b.pre.size() + e->hb_tpl.conds_len + b.post.size() > 0xFFF0 || e->blob_h.size() > 0xFFFFFFFFull - 0x20000) {
        *rc = KWOK_EDOMAIN;
        return 0;
    }
    uint64_t off = e->blob_h.size();
    e->blob_h += b.pre;
    e->blob_h += b.post;
    uint64_t word = off | ((uint64_t)b.pre.size() << 32) | ((uint64_t)b.post.size() << 48);
    e->blob_ids.emplace(key, word);
    uint32_t ilen = (uint32_t)b.pre.size() + e->hb_tpl.conds_len + (uint32_t)b.post.size();
    e->max_init_len = std::max(e->max_init_len, ilen);
    e->blob_up_lo = std::min<size_t>(e->blob_up_lo, off);  // uploaded once per batch (upload_blobs)
    return word;
}

// Tick completion events skip the system-scope release (the tick header is
// written with system-scope stores), so before a copy engine reads what the
// kernels wrote, record an event that performs it: the kernels' dirty L2 lines
// (per XCD, not coherent with the copy engine) are written back first.
int release_for_host(kwok_engine* e) {
    HIPCHK(e, hipEventRecord(e->fence, e->st));
    return KWOK_OK;
}

// The blobs interned since the last upload -> the device copy (SRC_PAD_FRONT
// zero bytes, the blobs, SRC_PAD_BACK zero bytes: k_emit reads around them).
// Once per node batch, after every ingest thread is done appending to blob_h,
// and synchronised before return: blob_h (pageable) may grow at the next batch.
int upload_blobs(kwok_engine* e) {
    if (e->blob_up_lo >= e->blob_h.size()) return KWOK_OK;
    const size_t lo = e->blob_up_lo;
    const size_t padded = ((SRC_PAD_FRONT + e->blob_h.size() + 3) & ~(size_t)3) + SRC_PAD_BACK;
    if (padded > e->d_blob.n) {
        uint8_t* p = nullptr;
        const size_t cap = std::max<size_t>(padded, 2 * e->d_blob.n);
        if (hipMalloc((void**)&p, cap) != hipSuccess) return e->fail(KWOK_ENOMEM, "blob %zu", cap);
        HIPCHK(e, hipMemsetAsync(p, 0, cap, e->st));
        if (e->d_blob.p) HIPCHK(e, hipMemcpyAsync(p, e->d_blob.p, SRC_PAD_FRONT + lo, hipMemcpyDeviceToDevice, e->st));
        HIPCHK(e, hipStreamSynchronize(e->st));
        if (e->d_blob.p) (void)hipFree(e->d_blob.p);
        e->d_blob.p = p;
        e->d_blob.n = cap;
    }
    HIPCHK(e, hipMemcpyAsync(e->d_blob.p + SRC_PAD_FRONT + lo, e->blob_h.data() + lo, e->blob_h.size() - lo,
                             hipMemcpyHostToDevice, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    e->blob_up_lo = SIZE_MAX;
    e->S.blob = e->d_blob.p + SRC_PAD_FRONT;
    e->S.blob_total = (uint32_t)e->blob_h.size();
    return KWOK_OK;
}

bool node_conforms(const kwok_node_event& ev, const std::string info[10]) {
    // A.5: configureNode's merged status equals the original iff no default applies
    return ev.addresses.len && ev.allocatable.len && ev.capacity.len && ev.phase == KWOK_PHASE_RUNNING &&
           !info[KWOK_NI_ARCHITECTURE].empty() && !info[KWOK_NI_KUBE_PROXY_VERSION].empty() &&
           !info[KWOK_NI_KUBELET_VERSION].empty() && !info[KWOK_NI_OPERATING_SYSTEM].empty() &&
           info[KWOK_NI_SYSTEM_UUID] == info[KWOK_NI_OS_IMAGE];
}

int parse_opt_ip(const char* arena, kwok_str s, uint32_t* ip) {
    *ip = 0;
    if (!s.len) return KWOK_OK;
    if (!parse_ipv4(arena + s.off, s.len, ip) || *ip == 0) return KWOK_EDOMAIN;
    return KWOK_OK;
}

int exchange(kwok_engine* e, void* send, size_t bytes, void* recv) {
    if (e->comm) {
        ncclResult_t r = ncclAllGather(send, recv, bytes, ncclUint8, e->comm, e->st);
        if (r != ncclSuccess) return e->fail(KWOK_ECOMM, "ncclAllGather: %s", ncclGetErrorString(r));
        return KWOK_OK;
    }
    // host-memory exchange through the caller's allgather
    std::vector<char> hs(bytes), hr(bytes * e->W);
    if (int rc = release_for_host(e)) return rc;
    HIPCHK(e, hipMemcpyAsync(hs.data(), send, bytes, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    if (e->cfg.allgather(e->cfg.allgather_user, hs.data(), bytes, hr.data()))
        return e->fail(KWOK_ECOMM, "allgather callback failed");
    HIPCHK(e, hipMemcpyAsync(recv, hr.data(), bytes * e->W, hipMemcpyHostToDevice, e->st));
    return KWOK_OK;
}

// Grow every bucket's pod capacity to new_cp (<= the handle stride): the device
// pod arrays are re-laid out bucket by bucket (a bucket's pods keep their index,
// so handles, canonical order and IP order are unchanged); per-slot lists are
// reallocated.  Runs between ticks (drained), before a batch's apply pass.
int grow_pods(kwok_engine* e, uint32_t new_cp) {
    const uint32_t old = e->Cp, nb = e->nb;
    if (new_cp <= old) return KWOK_OK;
    hipStream_t st = e->st;
    DevState& S = e->S;
    const size_t PL2 = (size_t)nb * new_cp, PLa2 = PL2 + 16;
    auto relayout = [&](auto*& p) -> int {
        using T = std::remove_reference_t<decltype(*p)>;
        T* q = nullptr;
        if (hipMalloc((void**)&q, PLa2 * sizeof(T)) != hipSuccess) return e->fail(KWOK_ENOMEM, "grow pods");
        HIPCHK(e, hipMemsetAsync(q, 0, PLa2 * sizeof(T), st));
        HIPCHK(e, hipMemcpy2DAsync(q, (size_t)new_cp * sizeof(T), p, (size_t)old * sizeof(T), (size_t)old * sizeof(T), nb,
                                   hipMemcpyDeviceToDevice, st));
        HIPCHK(e, hipStreamSynchronize(st));
        (void)hipFree(p);
        p = q;
        return KWOK_OK;
    };
    auto resize = [&](auto*& p, bool keep) -> int {  // per-ordinal lists: contents kept (the last tick's outputs)
        using T = std::remove_reference_t<decltype(*p)>;
        T* q = nullptr;
        if (hipMalloc((void**)&q, PLa2 * sizeof(T)) != hipSuccess) return e->fail(KWOK_ENOMEM, "grow pod lists");
        HIPCHK(e, hipMemsetAsync(q, 0, PLa2 * sizeof(T), st));
        if (keep && p) HIPCHK(e, hipMemcpyAsync(q, p, e->PLa * sizeof(T), hipMemcpyDeviceToDevice, st));
        HIPCHK(e, hipStreamSynchronize(st));
        if (p) (void)hipFree(p);
        p = q;
        return KWOK_OK;
    };
    int rc = 0;
    if ((rc = relayout(S.pod_state)) || (rc = relayout(S.pod_node)) || (rc = relayout(S.pod_spec)) ||
        (rc = relayout(S.pod_ctime)) || (rc = relayout(S.pod_ip)) || (rc = relayout(S.host_ip)) ||
        (rc = resize(S.alloc_addr, false)) || (rc = resize(S.use_list, false)) || (rc = resize(S.rel_list, false)))
        return rc;
    for (auto& T : e->slots) {
        if (!T.alloc) continue;
        if ((rc = resize(T.pp_pods, true)) || (rc = resize(T.pp_off, true)) || (rc = resize(T.pp_len, true)) ||
            (rc = resize(T.del_pods, true)) || (rc = resize(T.del_fin, true)) || (rc = resize(T.pp_job, true)))
            return rc;
    }
    e->Cp = new_cp;
    e->PL = (uint32_t)PL2;
    e->PLa = PLa2;
    S.cp = new_cp;
    S.n_pod_slots = e->PL;
    return size_arena(e);
}

// ---- GPU pod ingest: host side -------------------------------------------------
uint32_t sort_bits(const kwok_engine* e) {  // sort keys are local buckets 0..nb (nb: nothing to apply)
    uint32_t b = 1;
    while ((1ull << b) <= e->nb) b++;
    return b;
}
// per-record device buffers for batches of n records (grown with headroom)
int ingest_reserve(kwok_engine* e, size_t n, size_t arena_len) {
    auto& G = e->ing;
    if (n > G.cap) {
        const size_t cap = std::max<size_t>(n + n / 4, 4096);
        void* ptrs[] = {G.d_ev, G.rec, G.keys, G.keys_sorted, G.idx_sorted, G.out_handle, G.out_status,
                        G.out_released, G.sort_tmp, G.out_status8, G.tile_new, G.tile_pre, G.new_handle};
        for (void* p : ptrs)
            if (p) (void)hipFree(p);
        G.d_ev = G.sort_tmp = nullptr;
        G.tile_new = G.tile_pre = nullptr;
        G.new_handle = nullptr;
        G.out_status8 = nullptr;
        G.rec = nullptr;
        G.keys = G.keys_sorted = G.idx_sorted = G.out_released = nullptr;
        G.out_handle = G.out_status = nullptr;
        G.cap = G.sort_bytes = 0;
        int rc = 0;
        if ((rc = dalloc(e, (uint8_t**)&G.d_ev, cap * sizeof(kwok_pod_event))) || (rc = dalloc(e, &G.rec, cap)) ||
            (rc = dalloc(e, &G.keys, cap)) || (rc = dalloc(e, &G.keys_sorted, cap)) || (rc = dalloc(e, &G.idx_sorted, cap)) ||
            (rc = dalloc(e, &G.out_handle, cap)) || (rc = dalloc(e, &G.out_status, cap)) ||
            (rc = dalloc(e, &G.out_released, cap)) || (rc = dalloc(e, &G.out_status8, cap)) ||
            (rc = dalloc(e, &G.tile_new, cap / 256 + 2)) || (rc = dalloc(e, &G.tile_pre, cap / 256 + 2)) ||
            (rc = dalloc(e, &G.new_handle, cap)))
            return rc;
        G.sort_bytes = ingest_sort_bytes((uint32_t)cap, 32);
        if ((rc = dalloc(e, (uint8_t**)&G.sort_tmp, G.sort_bytes))) return rc;
        G.cap = cap;
    }
    if (arena_len > G.arena_cap) {
        if (G.d_arena) (void)hipFree(G.d_arena);
        G.d_arena = nullptr;
        G.arena_cap = 0;
        const size_t cap = std::max<size_t>(arena_len + arena_len / 4, 1 << 16);
        if (int rc = dalloc(e, &G.d_arena, cap)) return rc;
        G.arena_cap = cap;
    }
    return KWOK_OK;
}
IngestBatch ingest_batch(kwok_engine* e, uint32_t n, size_t arena_len) {
    auto& G = e->ing;
    IngestBatch I{};
    I.ev = G.d_ev;
    I.n = n;
    I.n_specs = (uint32_t)e->specs_h.size();
    I.arena = G.d_arena;
    I.arena_len = arena_len;
    I.rec = G.rec;
    I.keys = G.keys;
    I.keys_sorted = G.keys_sorted;
    I.idx_sorted = G.idx_sorted;
    I.out_handle = G.out_handle;
    I.out_status = G.out_status;
    I.out_released = G.out_released;
    I.beg = G.beg;
    I.end = G.end;
    I.sum = G.sum;
    return I;
}
// the batch summary -> pinned host memory (waits for the stream)
int read_summary(kwok_engine* e, const IngSummary* sum = nullptr) {
    if (int rc = release_for_host(e)) return rc;
    HIPCHK(e, hipMemcpyAsync(e->ing.sum_h, sum ? sum : e->ing.sum, sizeof(IngSummary), hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    return KWOK_OK;
}
// The largest pod capacity a chain block's pod chunks cover (engine_create's limit)
uint32_t max_pod_capacity(const kwok_engine* e) {
    const uint64_t bpb = (e->nb + e->S.n_chain - 1) / e->S.n_chain;
    const uint64_t lim = (uint64_t)MAX_POD_CHUNKS * BLOCK * POD_PER_THREAD / bpb;
    return (uint32_t)std::min<uint64_t>(e->Hs, lim & ~7ull);
}

}  // namespace

// ===========================================================================
// C-ABI
// ===========================================================================
extern "C" {

uint32_t kwok_abi_version(void) { return KWOK_ABI_VERSION; }

int kwok_comm_id(uint8_t out[KWOK_COMM_ID_BYTES]) {
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return KWOK_ECOMM;
    static_assert(sizeof(id) <= KWOK_COMM_ID_BYTES, "comm id size");
    memset(out, 0, KWOK_COMM_ID_BYTES);
    memcpy(out, &id, sizeof(id));
    return KWOK_OK;
}

const char* kwok_finalizer_patch(size_t* len) {
    static const char p[] = "{\"metadata\":{\"finalizers\":null}}";  // pod_controller.go:45
    if (len) *len = sizeof(p) - 1;
    return p;
}

uint32_t kwok_bucket_of(const char* name, size_t len, uint32_t buckets) { return fnv1a32(name, len) & (buckets - 1); }

namespace {
thread_local std::string g_tpl_err;
}
const char* kwok_template_last_error(void) { return g_tpl_err.c_str(); }

int kwok_heartbeat_template_patch(const char* tpl, int64_t start_unix, const char* node_ip, int64_t now_unix, char* out,
                                  size_t cap, size_t* out_len) {
    if (!node_ip || !out_len || (cap && !out)) return KWOK_EINVAL;
    g_tpl_err.clear();
    auto rfc3339 = [](int64_t u) {
        time_t t = (time_t)u;
        struct tm tm;
        gmtime_r(&t, &tm);
        char b[32];
        strftime(b, sizeof b, "%Y-%m-%dT%H:%M:%SZ", &tm);
        return std::string(b);
    };
    HeartbeatTemplate hb = build_heartbeat_template();
    if (tpl && !compile_heartbeat_template(tpl, rfc3339(start_unix), node_ip, hb, g_tpl_err)) return KWOK_EDOMAIN;
    const std::string o = heartbeat_patch(hb, rfc3339(now_unix), rfc3339(start_unix));
    *out_len = o.size();
    if (o.size() > cap) return KWOK_EINVAL;
    memcpy(out, o.data(), o.size());
    return KWOK_OK;
}

int kwok_node_template_patch(const char* tpl, const char* heartbeat_tpl, const kwok_node_event* ev, const char* arena,
                             size_t arena_len, int64_t start_unix, const char* node_ip, int64_t now_unix, char* out,
                             size_t cap, size_t* out_len) {
    if (!tpl || !ev || !node_ip || !out_len || (cap && !out)) return KWOK_EINVAL;
    g_tpl_err.clear();
    auto get = [&](kwok_str s) { return (size_t)s.off + s.len <= arena_len ? std::string(arena + s.off, s.len) : std::string(); };
    std::string info[KWOK_NI_COUNT];
    for (int k = 0; k < KWOK_NI_COUNT; k++) info[k] = get(ev->node_info[k]);
    auto rfc3339 = [](int64_t u) {
        time_t t = (time_t)u;
        struct tm tm;
        gmtime_r(&t, &tm);
        char b[32];
        strftime(b, sizeof b, "%Y-%m-%dT%H:%M:%SZ", &tm);
        return std::string(b);
    };
    HeartbeatTemplate hb = build_heartbeat_template();
    if (heartbeat_tpl && !compile_heartbeat_template(heartbeat_tpl, rfc3339(start_unix), node_ip, hb, g_tpl_err))
        return KWOK_EDOMAIN;
    NodeBlob nb;
    if (!compile_node_template(tpl, get(ev->addresses), get(ev->allocatable), get(ev->capacity), info, ev->phase, node_ip,
                               rfc3339(start_unix), hb, nb, g_tpl_err))
        return KWOK_EDOMAIN;
    const std::string o = nb.pre + heartbeat_conditions(hb, rfc3339(now_unix), rfc3339(start_unix)) + nb.post;
    *out_len = o.size();
    if (o.size() > cap) return KWOK_EINVAL;
    memcpy(out, o.data(), o.size());
    return KWOK_OK;
}

int kwok_pod_template_patch(const char* tpl, const kwok_pod_spec* spec, const char* arena, size_t arena_len,
                            int64_t start_unix, const char* node_ip, int64_t creation_unix, uint32_t host_ip,
                            uint32_t pod_ip, int32_t status_nonempty, char* out, size_t cap, size_t* out_len) {
    if (!tpl || !spec || !node_ip || !out_len || (cap && !out)) return KWOK_EINVAL;
    g_tpl_err.clear();
    auto get = [&](kwok_str s) { return (size_t)s.off + s.len <= arena_len ? std::string(arena + s.off, s.len) : std::string(); };
    std::vector<Container> cs, ics;
    std::vector<std::string> gates;
    for (uint32_t i = 0; i < spec->n_containers; i++) cs.push_back({get(spec->containers[i].name), get(spec->containers[i].image)});
    for (uint32_t i = 0; i < spec->n_init_containers; i++)
        ics.push_back({get(spec->init_containers[i].name), get(spec->init_containers[i].image)});
    for (uint32_t i = 0; i < spec->n_readiness_gates; i++) gates.push_back(get(spec->readiness_gates[i]));
    auto rfc3339 = [](int64_t u) {
        time_t t = (time_t)u;
        struct tm tm;
        gmtime_r(&t, &tm);
        char b[32];
        strftime(b, sizeof b, "%Y-%m-%dT%H:%M:%SZ", &tm);
        return std::string(b);
    };
    SpecProgram p;
    if (!compile_pod_template(tpl, cs, ics, gates, rfc3339(start_unix), p, g_tpl_err)) return KWOK_EDOMAIN;
    const std::string ts = rfc3339(creation_unix);
    auto fill = [&](const std::string& seg, const std::string& kind) {
        std::string o = seg;
        for (size_t i = 0; i < o.size(); i++)
            if ((uint8_t)kind[i] != KIND_LIT) o[i] = ts[(uint8_t)kind[i]];
        return o;
    };
    std::string o = fill(p.a, p.ka);
    if (status_nonempty) {  // the kernels' `{{ with .status }}` pieces (k_emit)
        uint32_t nip = 0;
        parse_ipv4(node_ip, strlen(node_ip), &nip);
        o += "\"hostIP\":\"" + format_ipv4(host_ip ? host_ip : nip) + "\",";
        o += fill(p.b, p.kb);
        o += "\"podIP\":\"" + format_ipv4(pod_ip) + "\",";
    } else {
        o += fill(p.b, p.kb);
    }
    o += fill(p.c, p.kc);
    *out_len = o.size();
    if (o.size() > cap) return KWOK_EINVAL;
    memcpy(out, o.data(), o.size());
    return KWOK_OK;
}

int kwok_template_render(const char* tpl, size_t tpl_len, const char* doc, size_t doc_len, const char* funcs,
                         size_t funcs_len, char* out, size_t cap, size_t* out_len) {
    using namespace kwok::gotpl;
    if (!tpl || !doc || !out_len || (cap && !out)) return KWOK_EINVAL;
    g_tpl_err.clear();
    VPtr d, f;
    if (!parse_json(std::string(doc, doc_len), d, g_tpl_err)) return KWOK_EDOMAIN;
    Env env;
    if (funcs && funcs_len) {
        if (!parse_json(std::string(funcs, funcs_len), f, g_tpl_err)) return KWOK_EDOMAIN;
        if (f->kind != Value::MAP) {
            g_tpl_err = "funcs must be a JSON object of strings";
            return KWOK_EINVAL;
        }
        for (auto& kv : f->map) {
            const std::string v = kv.second->s;
            env.funcs[kv.first] = [v] { return v; };
        }
    }
    std::string o;
    if (!render_to_json(std::string(tpl, tpl_len), d, env, o, g_tpl_err)) return KWOK_EDOMAIN;
    *out_len = o.size();
    if (o.size() > cap) return KWOK_EINVAL;
    memcpy(out, o.data(), o.size());
    return KWOK_OK;
}
int32_t kwok_rank_of_bucket(uint32_t bucket, uint32_t buckets, int32_t world) {
    return (int32_t)(((uint64_t)bucket * (uint64_t)world) / buckets);
}

const char* kwok_last_error(const kwok_engine* e) { return e ? e->err.c_str() : g_create_err.c_str(); }

void kwok_engine_destroy(kwok_engine* e) {
    if (!e) return;
    if (e->trace_ticks) {
        static const char* names[TRACE_SLOTS] = {"entry", "nodes-done", "pods-done", "arrived", "reduced", "pool-done",
                                                 "exit", "header-done", "node-flags", "pool-folded", "block-sum",
                                                 "drained", "hb-handles", "share-done", "nodes-emitted", "back-start",
                                                 // tick_back's pool phase (multi rank: the BACK launch)
                                                 "B-entry", "B-records", "B-prepped", "B-scanned", "B-selected",
                                                 "-", "-", "-"};
        fprintf(stderr, "[kwok trace] %u chain + %u streamer blocks, %llu ticks, us after the first chain block "
                        "start (min / median / max block)\n",
                e->S.n_chain, e->n_stream, (unsigned long long)e->trace_ticks);
        for (int k = 0; k < TRACE_SLOTS; k++)
            if (names[k][0] != '-' && e->trace_sum[k][2] > 0)
                fprintf(stderr, "[kwok trace] chain    %-11s %8.2f %8.2f %8.2f\n", names[k],
                        e->trace_sum[k][0] / e->trace_ticks, e->trace_sum[k][1] / e->trace_ticks,
                        e->trace_sum[k][2] / e->trace_ticks);
        for (int k = 0; k < 2; k++)
            fprintf(stderr, "[kwok trace] streamer %-11s %8.2f %8.2f %8.2f\n", k ? "exit" : "entry",
                    e->trace_sum[TRACE_SLOTS + k][0] / e->trace_ticks, e->trace_sum[TRACE_SLOTS + k][1] / e->trace_ticks,
                    e->trace_sum[TRACE_SLOTS + k][2] / e->trace_ticks);
    }
    if (e->st) (void)hipStreamSynchronize(e->st);
    if (e->rst) (void)hipStreamSynchronize(e->rst);  // (asynchronous arena reads)
    for (int i = 0; i < 3; i++) {
        if (e->rsx[i]) (void)hipStreamSynchronize(e->rsx[i]), (void)hipStreamDestroy(e->rsx[i]);
        if (e->rd_part[i]) (void)hipEventDestroy(e->rd_part[i]);
    }
    if (e->rd_go) (void)hipEventDestroy(e->rd_go);
    void* ptrs[] = {e->S.trace, e->S.jtrace, e->S.once_sum, e->S.node_state, e->S.node_blob, e->S.node_tick, e->S.pod_state, e->S.pod_node, e->S.pod_spec,
                    e->S.pod_ctime, e->S.pod_ip, e->S.host_ip, e->S.used_bm, e->S.usable_bm, e->S.pool_index,
                    e->S.pool_blk, e->S.alloc_addr, e->S.rel_bm, e->S.list_counts, (void*)e->S.hb_static,
                    (void*)e->S.hb_kind, e->S.bar, e->S.blockagg, e->S.dmask, e->S.list_blk, e->S.wc_pre, e->S.wc_dirty, e->S.jbase, e->S.gjob, e->d_hb_pre, e->d_hb_bpre, e->S.hdr, e->S.xmsg, e->S.node_key, e->S.node_name, e->S.mb_count, e->S.zb_count,
                    e->S.use_list, e->S.rel_list, e->d_specs.p, e->d_spec_bytes.p, e->d_spec_nxt.p, e->d_unit_tab.p, e->d_unit_desc.p, e->d_blob.p, e->d_ops,
                    e->d_ld, e->d_xall, e->d_xsend, e->d_xrecv, e->d_ssend, e->d_srecv};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (auto& T : e->slots) free_slot(T);
    {
        auto& g = e->ing;
        void* ip[] = {g.d_ev, g.d_arena, g.rec, g.keys, g.keys_sorted, g.idx_sorted, g.out_handle, g.out_status,
                      g.out_released, g.sort_tmp, g.abort, g.sums, g.beg, g.end, g.sum, g.sum1, g.tile_new, g.tile_pre,
                      g.new_handle,
                      g.out_status8, g.d_nev, g.d_nnames, g.nrec, g.host_idx, g.d_nfix, g.nsum};
        for (void* p : ip)
            if (p) (void)hipFree(p);
        if (g.sum_h) (void)hipHostFree(g.sum_h);
        if (g.nsum_h) (void)hipHostFree(g.nsum_h);
        if (g.sums_h) (void)hipHostFree(g.sums_h);
        if (g.res_h) (void)hipHostFree(g.res_h);
        hipEvent_t evs[] = {g.go, g.prepped[0], g.prepped[1], g.used[0], g.used[1], g.rdone, g.idone};
        for (hipEvent_t x : evs)
            if (x) (void)hipEventDestroy(x);
        if (g.pst) (void)hipStreamDestroy(g.pst);
        if (g.dst) (void)hipStreamDestroy(g.dst);
    }
    {
        auto& J = e->json;
        void* jp[] = {J.off, J.len, J.op, J.handle, J.side, J.host_list, J.fix_ev, J.fix_side, J.n_host, J.cfg,
                      J.tab_key, J.tab_id, J.tab_canon, J.canon, J.nstat, J.nev_fix};
        for (void* p : jp)
            if (p) (void)hipFree(p);
        if (J.cfg_h) (void)hipHostFree(J.cfg_h);
        if (J.n_host_h) (void)hipHostFree(J.n_host_h);
    }
    if (e->h_xall) (void)hipHostFree(e->h_xall);
    if (e->pinned) (void)hipHostFree(e->pinned);
    if (e->dump_h) (void)hipHostFree(e->dump_h);
    if (e->comm) ncclCommDestroy(e->comm);
    if (e->d_pod_fill) (void)hipFree(e->d_pod_fill);
    if (e->fence) (void)hipEventDestroy(e->fence);
    if (e->rst) (void)hipStreamDestroy(e->rst);
    if (e->st) (void)hipStreamDestroy(e->st);
    delete e;
}

int kwok_engine_create(const kwok_config* cfg, kwok_engine** out) {
    if (!out) return KWOK_EINVAL;
    *out = nullptr;
    if (!cfg || cfg->abi_version != KWOK_ABI_VERSION) return KWOK_EINVAL;
    if ((cfg->custom_templates & ~(KWOK_TPL_POD | KWOK_TPL_NODE_INIT | KWOK_TPL_HEARTBEAT)) || (cfg->flags & ~1u) ||
        ((cfg->custom_templates & KWOK_TPL_POD) && !cfg->pod_status_template) ||
        ((cfg->custom_templates & KWOK_TPL_NODE_INIT) && !cfg->node_init_template) ||
        ((cfg->custom_templates & KWOK_TPL_HEARTBEAT) && !cfg->node_heartbeat_template))
        return KWOK_EINVAL;
    const uint32_t hs = cfg->pod_handle_stride ? cfg->pod_handle_stride : cfg->pod_slots_per_bucket;
    if (!cfg->buckets || (cfg->buckets & (cfg->buckets - 1)) || cfg->node_slots_per_bucket % 4 ||
        !cfg->node_slots_per_bucket || cfg->node_slots_per_bucket > 65536 || cfg->pod_slots_per_bucket % 8 ||
        !cfg->pod_slots_per_bucket || hs % 8 || hs < cfg->pod_slots_per_bucket ||
        hs > 65528 /* fill marks are u16 */ || (uint64_t)cfg->buckets * hs > 0x7FFFFFFFull /* int32 handles */)
        return KWOK_EINVAL;
    int W = cfg->world_size > 0 ? cfg->world_size : 1;
    if (cfg->rank < 0 || cfg->rank >= W || (W > 1 && !cfg->comm_id && !cfg->allgather) || (uint32_t)W > cfg->buckets)
        return KWOK_EINVAL;
    kwok_engine* e = new kwok_engine();
    e->cfg = *cfg;
    e->W = W;
    // KWOK_FORCE_MULTI=1 (tests): one rank through the multi-rank tick, so the exchange
    // (RCCL with comm_id, else the allgather callback) runs on a single GPU
    e->multi = W > 1 || (getenv("KWOK_FORCE_MULTI") && (cfg->comm_id || cfg->allgather));
    e->rank = cfg->rank;
    e->dev = cfg->device;
    e->B = cfg->buckets;
    e->Cn = cfg->node_slots_per_bucket;
    e->Cp = cfg->pod_slots_per_bucket;
    e->Hs = hs;
    e->b_lo = (uint32_t)((uint64_t)cfg->rank * e->B / W);
    e->b_hi = (uint32_t)((uint64_t)(cfg->rank + 1) * e->B / W);
    // kwok_rank_of_bucket must agree with [b_lo, b_hi)
    e->nb = e->b_hi - e->b_lo;
    e->NL = e->nb * e->Cn;
    e->PL = e->nb * e->Cp;
    e->start = cfg->start_time_unix;
    auto bail = [&](int rc) {
        g_create_err = e->err.empty() ? std::string("create failed (") + std::to_string(rc) + ")" : e->err;
        kwok_engine_destroy(e);
        return rc;
    };
    // parseCIDR (utils.go:28-35): keep the host IP of the CIDR string as the pool base
    if (!cfg->cidr || !cfg->node_ip) return bail(KWOK_EINVAL);
    const char* slash = strchr(cfg->cidr, '/');
    uint32_t base = 0;
    if (!slash || !parse_ipv4(cfg->cidr, (size_t)(slash - cfg->cidr), &base)) return bail(KWOK_EDOMAIN);
    int plen = atoi(slash + 1);
    if (plen < 4 || plen > 32) return bail(KWOK_EDOMAIN);  // pool bitmaps: <= 2^28 addresses (32 MiB each)
    uint32_t mask = plen == 32 ? 0xFFFFFFFFu : (uint32_t)(0xFFFFFFFFull << (32 - plen));
    e->pool.net = base & mask;
    e->pool.base = base;
    e->pool.size = 1ull << (32 - plen);
    e->pool.words = (e->pool.size + 63) / 64;
    if (!parse_ipv4(cfg->node_ip, strlen(cfg->node_ip), &e->node_ip) || !e->node_ip) return bail(KWOK_EDOMAIN);
    e->node_ip_s = format_ipv4(e->node_ip);
    if (cfg->start_time_unix < 0 || cfg->start_time_unix > 0xFFFFFFFFll) return bail(KWOK_EDOMAIN);
    {
        time_t t = (time_t)cfg->start_time_unix;
        struct tm tm;
        gmtime_r(&t, &tm);
        char b[32];
        strftime(b, sizeof b, "%Y-%m-%dT%H:%M:%SZ", &tm);  // time.RFC3339 in UTC
        e->start_s = b;
    }
    // the heartbeat template first: its conditions list is part of every node init patch
    e->hb_tpl = build_heartbeat_template();
    if (cfg->custom_templates & KWOK_TPL_HEARTBEAT) {
        e->custom_hb = true;
        e->hb_tpl_text = cfg->node_heartbeat_template;
        std::string why;
        if (!compile_heartbeat_template(e->hb_tpl_text, e->start_s, e->node_ip_s, e->hb_tpl, why))
            return bail(e->fail(KWOK_EDOMAIN, "node heartbeat template: %s", why.c_str()));
    }
    e->hb_len = (uint32_t)e->hb_tpl.bytes.size();
    e->hb_stride = (e->hb_len + 15u) & ~15u;
    if (cfg->custom_templates & KWOK_TPL_NODE_INIT) {
        // compiled per node status at ingest; a trial node rejects a template outside the subset here
        e->custom_node = true;
        e->node_tpl = cfg->node_init_template;
        NodeBlob b;
        std::string why, info[KWOK_NI_COUNT];
        if (!compile_node_template(e->node_tpl, "", "", "", info, KWOK_PHASE_NONE, e->node_ip_s, e->start_s, e->hb_tpl, b,
                                   why))
            return bail(e->fail(KWOK_EDOMAIN, "node initialization template: %s", why.c_str()));
    }
    if (cfg->custom_templates & KWOK_TPL_POD) {
        // compiled per spec at kwok_register_pod_spec; a trial spec rejects a template
        // outside the covered subset here already
        e->custom_pod = true;
        e->pod_tpl = cfg->pod_status_template;
        SpecProgram p;
        std::string why;
        if (!compile_pod_template(e->pod_tpl, {Container{"c", "img"}}, {}, {}, e->start_s, p, why))
            return bail(e->fail(KWOK_EDOMAIN, "pod status template: %s", why.c_str()));
    }

    {
        hipError_t r = hipSetDevice(e->dev);
        if (r != hipSuccess) return bail(e->fail(KWOK_EDEVICE, "hipSetDevice(%d): %s", e->dev, hipGetErrorString(r)));
    }
    {
        hipError_t r = hipStreamCreateWithFlags(&e->st, hipStreamNonBlocking);
        if (r == hipSuccess) r = hipEventCreateWithFlags(&e->fence, hipEventDisableTiming);
        if (r == hipSuccess) r = hipStreamCreateWithFlags(&e->rst, hipStreamNonBlocking);
        if (r != hipSuccess) return bail(e->fail(KWOK_EDEVICE, "stream/event create: %s", hipGetErrorString(r)));
    }
    DevState& S = e->S;
    {
        // k_tick's grid: chain blocks (KWOK_TICK_BLOCKS_PER_CU per CU, default 1)
        // must be co-resident (dirty ticks wait on each other); streamer blocks
        // (KWOK_TICK_STREAMERS_PER_CU, default 1) only stream and exit.  Lower
        // both when several engines share one GPU (their grids must fit together).
        int cus = 0, occ = tick_occupancy(), want = 1, wants = 1;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, e->dev);
        // heartbeat-once ticks stream one body: the CU's second k_tick slot goes to a
        // second chain block (twice the classification loads in flight), and a few
        // streamer blocks write the body after the chain blocks
        const bool once = (cfg->flags & KWOK_CFG_HEARTBEAT_ONCE) != 0;
        if (once) want = 2;
        if (const char* v = getenv("KWOK_TICK_BLOCKS_PER_CU")) want = std::max(1, atoi(v));
        if (const char* v = getenv("KWOK_TICK_STREAMERS_PER_CU")) wants = std::max(1, atoi(v));
        if (cus <= 0 || occ <= 0) return bail(e->fail(KWOK_EDEVICE, "k_tick occupancy query failed"));
        S.n_chain = std::min<uint32_t>((uint32_t)(cus * std::min(occ, want)), (uint32_t)MAX_CHAIN);
        // KWOK_TICK_CHAIN_BLOCKS: fewer chain blocks, so that the grids of many engines
        // sharing one GPU (the 8-rank C3 test) are co-resident together
        if (const char* v = getenv("KWOK_TICK_CHAIN_BLOCKS")) S.n_chain = std::min<uint32_t>(S.n_chain, (uint32_t)std::max(1, atoi(v)));
        // (heartbeat-once: no streamer blocks - the one body is a chain block's slice,
        // written after its arrival, not by blocks that wait for the chain's CUs)
        e->n_stream = once ? 0u : (uint32_t)(cus * wants);
        // multi rank: the BACK launch fills the CUs' spare k_tick slots with pool-only
        // blocks (the pool phase's word-blocks over more blocks; all co-resident).  Not
        // when several engines share the GPU (KWOK_TICK_BLOCKS_PER_CU / _CHAIN_BLOCKS:
        // their grids must fit together, and a BACK launch waits for all its blocks)
        const bool shared = getenv("KWOK_TICK_BLOCKS_PER_CU") || getenv("KWOK_TICK_CHAIN_BLOCKS");
        S.n_pool_extra = shared ? 0u : (uint32_t)std::min<int64_t>(std::max<int64_t>(0, (int64_t)cus * occ - S.n_chain), e->n_stream);
        if (const char* v = getenv("KWOK_POOL_EXTRA"))
            S.n_pool_extra = (uint32_t)std::min<int64_t>(std::max(0, atoi(v)), std::min<int64_t>((int64_t)cus * occ - S.n_chain, e->n_stream));
        e->emit_grid = (uint32_t)(cus * std::max(1, std::min(emit_occupancy(), 8)));
        if (const char* v = getenv("KWOK_EMIT_BLOCKS_PER_CU")) e->emit_grid = (uint32_t)(cus * std::max(1, std::min(atoi(v), 8)));
        if (const char* v = getenv("KWOK_TICK_STREAMERS")) e->n_stream = (uint32_t)std::max(1, atoi(v));
        const char* pr = getenv("KWOK_TICK_PRIO");
        e->chain_prio = pr && pr[0] == '1';
        if (const char* v = getenv("KWOK_TICK_STREAM_DELAY_NS")) S.stream_delay = (uint32_t)std::max(0, atoi(v) / 10);
        if (const char* v = getenv("KWOK_TICK_STREAM_SHARE")) e->share_env = std::min(1024, std::max(0, atoi(v)));
        if (const char* v = getenv("KWOK_HB_NT")) e->nt_env = atoi(v) != 0;
        if (const char* v = getenv("KWOK_DEBUG_LAYOUT_FAULT_TICK")) e->debug_fault_tick = strtoull(v, nullptr, 10);
        if (const char* v = getenv("KWOK_DEBUG_INGEST_FAIL_CHUNK")) e->debug_fail_chunk = (uint32_t)strtoul(v, nullptr, 10);
        if (const char* v = getenv("KWOK_DEBUG_INGEST_FAIL_APPLY")) e->debug_fail_apply = (uint32_t)strtoul(v, nullptr, 10);
        e->iprof = getenv("KWOK_INGEST_PROF") != nullptr;
        if (const char* v = getenv("KWOK_INGEST_RESULTS_KERNEL")) e->results_kernel = v[0] == '1';
        if (const char* v = getenv("KWOK_INGEST_RS")) e->results_stream = v[0] != '0';
        if (const char* v = getenv("KWOK_INGEST_NEW_MAPPED")) e->new_mapped = v[0] != '0';
        if (const char* v = getenv("KWOK_INGEST_LAST_CUT")) e->last_chunk_cut = std::min(0.9, std::max(0.0, atof(v)));
        if (e->iprof)
            for (hipEvent_t& x : e->ing.tev) (void)hipEventCreate(&x);
        const char* ns = getenv("KWOK_TICK_NO_STREAM");
        e->no_stream = ns && ns[0] == '1';
        const char* qt = getenv("KWOK_QUIET");
        e->quiet_ok = !(qt && qt[0] == '0');
        const char* sj = getenv("KWOK_SPLIT");
        e->split_jobs = !(sj && sj[0] == '0');
        if (const char* v = getenv("KWOK_READ_STREAMS")) e->read_streams = std::max(1, std::min(4, atoi(v)));
        const char* sj2 = getenv("KWOK_SPARSE_JOBS");  // 0: k_pod_jobs<false> re-classifies the runs (A/B)
        e->sparse_jobs = !(sj2 && sj2[0] == '0');
        const char* fe = getenv("KWOK_FUSE_EMIT");
        e->fuse_emit = fe && fe[0] ? (fe[0] == '0' ? 0 : 1) : -1;
        const char* fi = getenv("KWOK_FOLD_INITS");
        e->fold_inits = !(fi && fi[0] == '0');
        const char* on = getenv("KWOK_ONCE");
        e->once_ok = !(on && on[0] == '0');
        const char* os = getenv("KWOK_ONCE_SUM");
        e->once_sum_ok = !(os && os[0] == '0');
        const char* zc = getenv("KWOK_INGEST_ZC");
        e->ingest_zc = !(zc && zc[0] == '0');
    }
    S.n_node_slots = e->NL;
    S.n_pod_slots = e->PL;
    S.nb = e->nb;
    S.cn = e->Cn;
    S.cp = e->Cp;
    S.node_handle_base = (int32_t)(e->b_lo * e->Cn);
    S.pod_handle_base = 0;  // pod handles: pod_handle_of (stride)
    S.hb_units = e->hb_stride / 16;
    S.conds_off = e->hb_tpl.conds_off;
    S.conds_len = e->hb_tpl.conds_len;
    S.b_lo = e->b_lo;
    S.pod_stride = e->Hs;
    S.pool = e->pool;
    S.node_ip = e->node_ip;
    e->XW = W;
    if (const char* v = getenv("KWOK_XSPEC")) e->xspec_env = atoi(v);
    if (const char* v = getenv("KWOK_EMULATE_RANKS"))
        if (e->multi && W == 1) e->XW = std::max(1, std::min(atoi(v), 64));
    S.world = e->XW;  // the messages BACK folds
    S.multi = e->multi ? 1 : 0;
    S.cni = cfg->enable_cni ? 1u : 0u;
    S.custom_pod = (cfg->custom_templates & KWOK_TPL_POD) ? 1u : 0u;
    S.hb_once = (cfg->flags & KWOK_CFG_HEARTBEAT_ONCE) ? 1u : 0u;
    S.buckets = e->B;
    {
        // a chain block's bucket range must fit its LDS node flags and 64 pod chunks
        const uint32_t bpb = (e->nb + S.n_chain - 1) / S.n_chain;
        if (bpb > (uint32_t)MAX_BPB || (uint64_t)bpb * e->Cn > (uint64_t)NODE_LDS ||
            (uint64_t)bpb * (e->Cp / POD_PER_THREAD) > (uint64_t)MAX_POD_CHUNKS * BLOCK)
            return bail(e->fail(KWOK_EDOMAIN,
                                "%u buckets x (%u node, %u pod slots) per k_tick chain block exceed its limits "
                                "(%d buckets, %d node slots, %d pod groups): shard over more GPUs",
                                bpb, e->Cn, e->Cp, MAX_BPB, NODE_LDS, MAX_POD_CHUNKS * BLOCK));
    }
    const uint32_t nblk = (uint32_t)((e->pool.words + BLOCK * POOL_WPT_MIN - 1) / (BLOCK * POOL_WPT_MIN));
    // node / pod arrays: whole 16-byte vectors at the end (Cn % 4 == 0, Cp % 8 == 0)
    const size_t NLa = (size_t)e->NL + 16, PLa = (size_t)e->PL + 16;
    e->NLa = NLa;
    e->PLa = PLa;
    int rc = 0;
    if ((rc = dalloc(e, &S.node_state, NLa)) || (rc = dalloc(e, &S.node_blob, NLa)) ||
        (rc = dalloc(e, &S.node_tick, NLa)) || (rc = dalloc(e, &S.pod_state, PLa)) ||
        (rc = dalloc(e, &S.pod_node, PLa)) || (rc = dalloc(e, &S.pod_spec, PLa)) ||
        (rc = dalloc(e, &S.pod_ctime, PLa)) || (rc = dalloc(e, &S.pod_ip, PLa)) ||
        (rc = dalloc(e, &S.host_ip, PLa)) || (rc = dalloc(e, &S.used_bm, e->pool.words)) ||
        (rc = dalloc(e, &S.usable_bm, e->pool.words)) || (rc = dalloc(e, &S.rel_bm, e->pool.words)) ||
        (rc = dalloc(e, &S.list_counts, 2)) || (rc = dalloc(e, &e->d_pod_fill, e->nb)) || (rc = dalloc(e, &S.pool_index, 1)) ||
        (rc = dalloc(e, &S.pool_blk, 2 * (size_t)nblk)) || (rc = dalloc(e, &S.bar, 1)) ||
        (rc = dalloc(e, &S.blockagg, (size_t)S.n_chain * AG_STRIDE)) ||
        (rc = dalloc(e, &S.dmask, (size_t)S.n_chain * 2)) || (rc = dalloc(e, &S.list_blk, (size_t)S.n_chain * 2)) || (rc = dalloc(e, &e->d_hb_pre, (size_t)S.n_chain + 1)) ||
        (rc = dalloc(e, &e->d_hb_bpre, (size_t)e->nb + 1)) ||
        (rc = dalloc(e, &S.wc_pre, (size_t)S.n_chain * MAX_WC)) ||
        (rc = dalloc(e, &S.wc_dirty, (size_t)S.n_chain * WC_DIRTY_WORDS)) || (rc = dalloc(e, &S.jbase, (size_t)S.n_chain)) ||
        (e->sparse_jobs && (rc = dalloc(e, &S.gjob, (size_t)S.n_chain * MAX_WC * WC_GROUPS))) ||
        (getenv("KWOK_TICK_TRACE") && (rc = dalloc(e, &S.trace, (size_t)(S.n_chain + e->n_stream) * TRACE_SLOTS))) ||
        (getenv("KWOK_JOBS_TRACE") && (rc = dalloc(e, &S.jtrace, (size_t)S.n_chain * (MAX_WC + 4) * 4))) ||
        (rc = dalloc(e, &S.alloc_addr, PLa)) || (rc = dalloc(e, (uint8_t**)&S.hb_static, HB_MAX_STRIDE)) ||
        (rc = dalloc(e, (uint8_t**)&S.hb_kind, HB_MAX_STRIDE)) ||
        (rc = dalloc(e, &S.hdr, 1)) || (rc = dalloc(e, &S.xmsg, 1)) || (rc = dalloc(e, &S.use_list, PLa)) ||
        (rc = dalloc(e, &S.rel_list, PLa)) || (rc = dalloc(e, &e->d_ld, (size_t)std::max(e->XW, 1))) ||
        (rc = dalloc(e, &S.node_key, NLa)) || (rc = dalloc(e, &S.node_name, NLa * NAME_STRIDE)) ||
        (rc = dalloc(e, &S.mb_count, e->nb)) || (rc = dalloc(e, &S.zb_count, e->nb)) ||
        (rc = dalloc(e, &S.once_sum, e->nb)) ||
        (rc = alloc_slot(e, 0)))
        return bail(rc);
    // heartbeat template: static bytes + kinds (0..19 Now, 20..39 StartTime)
    {
        const HeartbeatTemplate& hb = e->hb_tpl;
        std::vector<uint8_t> bytes(HB_MAX_STRIDE, 0), kind(HB_MAX_STRIDE, 0xFF);
        memcpy(bytes.data(), hb.bytes.data(), hb.bytes.size());
        for (uint16_t o : hb.now_slots)
            for (int i = 0; i < TS_LEN; i++) kind[o + i] = (uint8_t)i;
        for (uint16_t o : hb.start_slots)
            for (int i = 0; i < TS_LEN; i++) kind[o + i] = (uint8_t)(TS_LEN + i);
        // on the engine's stream, after dalloc's zero fills (a null-stream copy is
        // not ordered with a non-blocking stream: the fill could land after it)
        hipError_t r = hipMemcpyAsync((void*)S.hb_static, bytes.data(), HB_MAX_STRIDE, hipMemcpyHostToDevice, e->st);
        if (r == hipSuccess) r = hipMemcpyAsync((void*)S.hb_kind, kind.data(), HB_MAX_STRIDE, hipMemcpyHostToDevice, e->st);
        if (r == hipSuccess) r = hipStreamSynchronize(e->st);
        if (r != hipSuccess) return bail(e->fail(KWOK_EDEVICE, "template upload: %s", hipGetErrorString(r)));
    }
    {
        const char* sy = getenv("KWOK_SYNC");
        e->sync_spin = !(sy && strcmp(sy, "block") == 0);
    }
    S.hb_pre = e->d_hb_pre;
    S.hb_bpre = e->d_hb_bpre;
    S.pod_fill = e->d_pod_fill;
    S.rank = e->rank;
    if (e->multi) {
        if ((rc = dalloc(e, &e->d_xall, (size_t)e->XW))) return bail(rc);
        S.xall = e->d_xall;
        if (hipHostMalloc((void**)&e->h_xall, sizeof(XMsg) * e->XW, hipHostMallocDefault) != hipSuccess)
            return bail(KWOK_ENOMEM);
        if (cfg->comm_id) {
            ncclUniqueId id;
            memcpy(&id, cfg->comm_id, sizeof(id));
            ncclResult_t r = ncclCommInitRank(&e->comm, W, id, e->rank);
            if (r != ncclSuccess) return bail(e->fail(KWOK_ECOMM, "ncclCommInitRank: %s", ncclGetErrorString(r)));
        }
    }
    {
        // host threads of node batches' string work: KWOK_INGEST_THREADS, else up to 16
        unsigned hw = std::thread::hardware_concurrency();
        int np = (int)std::min(16u, hw ? hw : 1u);
        if (const char* v = getenv("KWOK_INGEST_THREADS")) np = atoi(v);
        e->n_part = std::max(1, std::min(np, 64));
    }
    {  // GPU pod ingest: per-bucket / per-node-slot scratch and the batch summary
        auto& g = e->ing;
        if ((rc = dalloc(e, &g.abort, 1)) || (rc = dalloc(e, &g.beg, e->nb)) || (rc = dalloc(e, &g.end, e->nb)) ||
            (rc = dalloc(e, &g.sum, 1)) || (rc = dalloc(e, &g.nsum, 1)) || (rc = dalloc(e, &g.sum1, 1)))
            return bail(rc);
        if (hipHostMalloc((void**)&g.sum_h, sizeof(IngSummary), hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void**)&g.nsum_h, sizeof(NodeSummary), hipHostMallocDefault) != hipSuccess)
            return bail(KWOK_ENOMEM);
        hipError_t r = hipStreamCreateWithFlags(&g.pst, hipStreamNonBlocking);
        if (r == hipSuccess) r = hipStreamCreateWithFlags(&g.dst, hipStreamNonBlocking);
        hipEvent_t* evs[] = {&g.go, &g.prepped[0], &g.prepped[1], &g.used[0], &g.used[1], &g.rdone, &g.idone};
        for (hipEvent_t* x : evs)
            if (r == hipSuccess) r = hipEventCreateWithFlags(x, hipEventDisableTiming);
        if (r != hipSuccess) return bail(e->fail(KWOK_EDEVICE, "ingest stream/events: %s", hipGetErrorString(r)));
        if (const char* v = getenv("KWOK_INGEST_CHUNK")) g.chunk = std::max<size_t>(1, strtoull(v, nullptr, 10));
        // The runtime creates a copy engine's queue the first time it hands that engine a
        // copy, holding the submitting host thread ~6 ms (C4: one or two batches of a
        // process's first ~10 paid it inside the timed ingest, whatever the host memory;
        // tools/gpu_r4v.sh, profiles/r4v_sdma_ab.txt).  Copies in both directions on every
        // stream the engine uses, several in flight at once, spread over the engines here
        // at create time instead (KWOK_COPY_WARM=0: off).
        const char* cw = getenv("KWOK_COPY_WARM");
        if (!(cw && cw[0] == '0')) {
            const size_t wb = (size_t)8 << 20;
            void *hbuf = nullptr, *dbuf = nullptr;
            if (hipHostMalloc(&hbuf, wb * 4, hipHostMallocDefault) == hipSuccess && hipMalloc(&dbuf, wb * 4) == hipSuccess) {
                hipStream_t ss[4] = {e->st, g.pst, g.dst, e->rst};
                for (int round = 0; round < 4; round++)
                    for (int q = 0; q < 4; q++) {
                        char* h = (char*)hbuf + (size_t)q * wb;
                        char* d = (char*)dbuf + (size_t)q * wb;
                        (void)hipMemcpyAsync(round & 1 ? h : d, round & 1 ? d : h, wb,
                                             round & 1 ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice, ss[q]);
                    }
                for (hipStream_t x : ss) (void)hipStreamSynchronize(x);
            }
            if (dbuf) (void)hipFree(dbuf);
            if (hbuf) (void)hipHostFree(hbuf);
        }
    }
    e->max_init_len = 0;
    if ((rc = size_arena(e)) || (rc = grow_arena(e, e->slots[0]))) return bail(rc);
    // a warm-up launch of k_tick (phases 0: every block returns at once): the runtime
    // sets up the queue's scratch for the kernel here, not inside the first tick
    // (measured ~0.3-0.6 ms on the initial tick when k_tick's frame is not empty)
    launch_tick(S, e->n_stream, 0, 0, 0, 0, 0, 0, e->st);
    {
        hipError_t r = hipStreamSynchronize(e->st);
        if (r != hipSuccess) return bail(e->fail(KWOK_EDEVICE, "create sync: %s", hipGetErrorString(r)));
    }
    *out = e;
    return KWOK_OK;
}

int kwok_register_pod_spec(kwok_engine* e, const kwok_pod_spec* spec, const char* arena, size_t arena_len,
                           int32_t* out_id) {
    if (!e || !spec || !out_id) return KWOK_EINVAL;
    if (e->poisoned) return poisoned(e);
    drain(e);  // the host mirrors reflect every submitted tick
    if (e->poisoned) return poisoned(e);
    auto get = [&](kwok_str s, std::string& o) {
        if ((size_t)s.off + s.len > arena_len) return false;
        o.assign(arena + s.off, s.len);
        return safe_string(o.data(), o.size());
    };
    std::vector<Container> cs(spec->n_containers), ics(spec->n_init_containers);
    std::vector<std::string> gates(spec->n_readiness_gates);
    for (uint32_t i = 0; i < spec->n_containers; i++)
        if (!get(spec->containers[i].name, cs[i].name) || !get(spec->containers[i].image, cs[i].image))
            return e->fail(KWOK_EDOMAIN, "container %u: not a safe string", i);
    for (uint32_t i = 0; i < spec->n_init_containers; i++)
        if (!get(spec->init_containers[i].name, ics[i].name) || !get(spec->init_containers[i].image, ics[i].image))
            return e->fail(KWOK_EDOMAIN, "init container %u: not a safe string", i);
    for (uint32_t i = 0; i < spec->n_readiness_gates; i++)
        if (!get(spec->readiness_gates[i], gates[i])) return e->fail(KWOK_EDOMAIN, "readiness gate %u: not a safe string", i);
    SpecProgram p;
    if (e->custom_pod) {
        std::string why;
        if (!compile_pod_template(e->pod_tpl, cs, ics, gates, e->start_s, p, why))
            return e->fail(KWOK_EDOMAIN, "pod status template: %s", why.c_str());
    } else {
        p = build_spec_program(cs, ics, gates);
    }
    if (p.max_len > 0xFFF0) return e->fail(KWOK_EDOMAIN, "pod patch longer than 64 KiB");
    std::vector<uint16_t> nxt;
    if (!build_ts_lookup(p, nxt)) return e->fail(KWOK_EDOMAIN, "pod patch layout outside the emitter's domain");
    std::string tab;
    std::vector<uint16_t> tdesc;
    const bool tabled = build_unit_tables(p, tab, tdesc);  // else: the general emitter path only
    std::string key = p.a + '\x01' + p.ka + '\x01' + p.b + '\x01' + p.kb + '\x01' + p.c + '\x01' + p.kc;
    std::string canon = json_spec_canon(cs, ics, gates);
    const uint64_t skey = json_spec_key(canon);  // the GPU codec finds the spec by this key (and checks canon)
    auto note = [&](int32_t id) {
        auto k = e->spec_keys.emplace(skey, id);
        if (k.second) e->spec_canon[skey] = std::move(canon);
        if (!k.second && k.first->second != id) k.first->second = -2;  // (a 64-bit collision: the host decides)
        if (k.second || k.first->second == -2) e->json.tab_dirty = true;
    };
    auto it = e->spec_ids.find(key);
    if (it != e->spec_ids.end()) {
        *out_id = it->second;
        note(it->second);
        return KWOK_OK;
    }
    uint32_t cap = e->cfg.max_pod_specs ? std::min<uint32_t>(e->cfg.max_pod_specs, 65535) : 1024;
    if (e->specs_h.size() >= cap) return e->fail(KWOK_EFULL, "max_pod_specs reached");
    SpecDesc d{};
    d.off = (uint32_t)e->spec_bytes_h.size();
    d.len_a = (uint16_t)p.a.size();
    d.len_b = (uint16_t)p.b.size();
    d.len_c = (uint16_t)p.c.size();
    d.max_len = (uint16_t)p.max_len;
    d.nxt_off = (uint32_t)e->spec_nxt_h.size();
    d.tab_off = NO_TAB;
    // KWOK_EMIT_TAB_UNITS caps the table units (tests: 0 = the general emitter only, small = mixed chunks)
    const char* cap_env = getenv("KWOK_EMIT_TAB_UNITS");
    const size_t tab_cap = cap_env ? (size_t)strtoull(cap_env, nullptr, 10) : (size_t)MAX_TAB_UNITS;
    if (tabled && e->tab_units + tdesc.size() <= std::min(tab_cap, (size_t)MAX_TAB_UNITS)) {
        const size_t n = e->tab_units + tdesc.size();
        int rc;
        if ((rc = dgrow(e, e->d_unit_tab, n * 16)) || (rc = dgrow(e, e->d_unit_desc, n))) return rc;
        HIPCHK(e, hipMemcpyAsync(e->d_unit_tab.p + (size_t)e->tab_units * 16, tab.data(), tab.size(),
                                 hipMemcpyHostToDevice, e->st));
        HIPCHK(e, hipMemcpyAsync(e->d_unit_desc.p + e->tab_units, tdesc.data(), tdesc.size() * 2,
                                 hipMemcpyHostToDevice, e->st));
        d.tab_off = e->tab_units;
        e->tab_units = (uint32_t)n;
        e->S.unit_tab = reinterpret_cast<const uint4*>(e->d_unit_tab.p);
        e->S.unit_desc = e->d_unit_desc.p;
    }
    if (d.tab_off == NO_TAB) e->n_untabled++;
    const std::string kinds = p.ka + p.kb + p.kc;
    for (size_t i = 0; i < kinds.size(); i++)  // slot starts (kinds 0..19 in a row)
        if (kinds[i] == 0) d.n_ts++;
    e->spec_nxt_h.insert(e->spec_nxt_h.end(), nxt.begin(), nxt.end());
    e->spec_bytes_h += p.a + p.b + p.c;
    e->specs_h.push_back(d);
    int rc = upload_specs(e);
    if (rc) return rc;
    e->max_pod_len = std::max(e->max_pod_len, p.max_len);
    if ((rc = size_arena(e))) return rc;
    *out_id = (int32_t)(e->specs_h.size() - 1);
    e->spec_ids.emplace(key, *out_id);
    note(*out_id);
    return KWOK_OK;
}

// node batch buffers for n records (the pod batch's sort buffers are shared)
int node_reserve(kwok_engine* e, size_t n, size_t arena_len) {
    auto& G = e->ing;
    if (int rc = ingest_reserve(e, n, arena_len)) return rc;
    if (n <= G.ncap) return KWOK_OK;
    void* ptrs[] = {G.d_nev, G.d_nnames, G.nrec, G.host_idx, G.d_nfix};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (G.res_h) (void)hipHostFree(G.res_h);
    G.d_nev = nullptr, G.d_nnames = nullptr, G.nrec = nullptr, G.host_idx = nullptr, G.d_nfix = nullptr, G.res_h = nullptr;
    G.ncap = 0;
    const size_t cap = std::max<size_t>(n + n / 4, 4096);
    int rc = 0;
    if ((rc = dalloc(e, &G.d_nev, cap)) || (rc = dalloc(e, &G.d_nnames, cap * NAME_STRIDE)) || (rc = dalloc(e, &G.nrec, cap)) ||
        (rc = dalloc(e, &G.host_idx, cap)) || (rc = dalloc(e, &G.d_nfix, cap)))
        return rc;
    if (hipHostMalloc((void**)&G.res_h, cap * 8, hipHostMallocDefault) != hipSuccess) return e->fail(KWOK_ENOMEM, "node results");
    G.ncap = cap;
    return KWOK_OK;
}

// The status of a node the device could not settle alone (a non-empty status, or
// a custom node template): the string checks and the init blob (node.init.tpl /
// Config.NodeInitializationTemplate), CONFORMS (A.5).  Host string work, on the
// partition threads; blob interning under blob_mu.
NodeFix complete_node(kwok_engine* e, const kwok_node_event& x, uint32_t idx, const char* arena, std::mutex& blob_mu) {
    NodeFix f{};
    f.idx = idx;
    int st = KWOK_OK;
    std::string info[KWOK_NI_COUNT];
    for (int k = 0; k < KWOK_NI_COUNT && st == KWOK_OK; k++)
        if (x.node_info[k].len) {
            info[k].assign(arena + x.node_info[k].off, x.node_info[k].len);
            if (!safe_string(info[k].data(), info[k].size())) st = KWOK_EDOMAIN;
        }
    std::string js[3];
    const kwok_str* jr[3] = {&x.addresses, &x.allocatable, &x.capacity};
    for (int k = 0; k < 3 && st == KWOK_OK; k++)
        if (jr[k]->len) {
            js[k].assign(arena + jr[k]->off, jr[k]->len);
            if (!valid_json_blob(js[k].data(), js[k].size(), k == 0 ? '[' : '{')) st = KWOK_EDOMAIN;
        }
    if (st == KWOK_OK) {
        std::lock_guard<std::mutex> lock(blob_mu);
        if (e->custom_node) {
            // one compile per distinct status (the fields the template may read)
            std::string key = std::to_string(x.phase);
            for (int k = 0; k < 3; k++) key += '\x01' + js[k];
            for (int k = 0; k < KWOK_NI_COUNT; k++) key += '\x01' + info[k];
            auto it = e->node_tpl_blobs.find(key);
            if (it != e->node_tpl_blobs.end()) {
                f.blob = it->second;
            } else {
                NodeBlob nb;
                std::string why;
                if (!compile_node_template(e->node_tpl, js[0], js[1], js[2], info, x.phase, e->node_ip_s, e->start_s,
                                           e->hb_tpl, nb, why)) {
                    st = KWOK_EDOMAIN;
                } else {
                    f.blob = intern_blob(e, nb, &st);
                    if (st == KWOK_OK) e->node_tpl_blobs.emplace(std::move(key), f.blob);
                }
            }
        } else {
            f.blob = intern_blob(e, build_node_blob(js[0], js[1], js[2], info, e->node_ip_s), &st);
        }
    }
    f.status = st;
    f.conforms = st == KWOK_OK && !e->custom_node && node_conforms(x, info) ? 1u : 0u;
    return f;
}

// kwok_ingest_nodes: the WatchNodes / ListNodes event switch (node_controller.go:
// 256-270) on the GPU over the device node directory (ingest.hip): prep, the host's
// completions of non-empty statuses, a stable sort by bucket, one wave per bucket
// in event order.  Two host round trips per batch (the prep summary, the results).
// kwok_ingest_nodes_json: the records were decoded on the device (G.d_nev, the
// documents in G.d_arena); the records the host completes come from here
struct NodeJsonCtx {
    const char* arena;                            // the caller's documents (device-decoded records' spans)
    const std::unordered_map<uint32_t, uint32_t>* hdoc;  // document -> its host decode (hrec / hbuf)
    const std::vector<kwok_node_event>* hrec;     // host-decoded records, spans into their hbuf
    const std::vector<std::string>* hbuf;
};
int ingest_nodes_impl(kwok_engine* e, const kwok_node_event* ev, size_t n, const char* arena, size_t arena_len,
                      int32_t* out_handles, int32_t* out_status, const NodeJsonCtx* nj);
int kwok_ingest_nodes(kwok_engine* e, const kwok_node_event* ev, size_t n, const char* arena, size_t arena_len,
                      int32_t* out_handles, int32_t* out_status) {
    if (!e || (n && !ev) || n > 0x7FFFFFF0ull || (arena_len && !arena)) return KWOK_EINVAL;
    if (e->poisoned) return poisoned(e);
    drain(e);  // the device state reflects every submitted tick
    if (e->poisoned) return poisoned(e);
    e->emit_hint = true;
    e->quiet = 0;
    e->sum_valid = false;
    if (!n) return 0;
    int rc = node_reserve(e, n, arena_len);
    if (rc) return rc;
    return ingest_nodes_impl(e, ev, n, arena, arena_len, out_handles, out_status, nullptr);
}
int ingest_nodes_impl(kwok_engine* e, const kwok_node_event* ev, size_t n, const char* arena, size_t arena_len,
                      int32_t* out_handles, int32_t* out_status, const NodeJsonCtx* nj) {
    const auto t0 = clk::now();
    int rc = 0;
    auto& G = e->ing;
    hipStream_t st = e->st;
    // the empty-status blob (kwok's own fleets create Nodes with an empty status)
    if (!e->custom_node && !e->has_empty_blob.load()) {
        std::string empty[KWOK_NI_COUNT];
        int brc = KWOK_OK;
        const uint64_t b = intern_blob(e, build_node_blob("", "", "", empty, e->node_ip_s), &brc);
        if (brc) return e->fail(brc, "empty node status blob");
        e->empty_blob = b;
        e->has_empty_blob.store(true);
    }
    // the batch in kwok_host_alloc memory is read in place by k_nd_prep; any other is copied
    // (kwok_ingest_nodes_json: both on the device already)
    const void* zev = !nj && e->ingest_zc ? host_mapped(ev, n * sizeof(kwok_node_event)) : nullptr;
    const void* zar = !nj && e->ingest_zc && arena_len ? host_mapped(arena, arena_len) : nullptr;
    if (!zev && !nj) HIPCHK(e, hipMemcpyAsync(G.d_nev, ev, n * sizeof(kwok_node_event), hipMemcpyHostToDevice, st));
    if (arena_len && !zar && !nj) HIPCHK(e, hipMemcpyAsync(G.d_arena, arena, arena_len, hipMemcpyHostToDevice, st));
    NodeBatch N{};
    N.ev = static_cast<const kwok_node_event*>(zev ? zev : (const void*)G.d_nev);
    N.n = (uint32_t)n;
    N.host_all = e->custom_node ? 1u : 0u;
    N.arena = zar ? static_cast<const uint8_t*>(zar) : G.d_arena;
    N.arena_len = arena_len;
    N.empty_blob = e->empty_blob;
    N.rec = G.nrec;
    N.names = G.d_nnames;
    N.keys = G.keys;
    N.keys_sorted = G.keys_sorted;
    N.idx_sorted = G.idx_sorted;
    N.beg = G.beg;
    N.end = G.end;
    N.out_handle = G.out_handle;
    N.out_status = G.out_status;
    N.host_idx = G.host_idx;
    N.sum = G.nsum;
    HIPCHK(e, hipMemsetAsync(G.nsum, 0, sizeof(NodeSummary), st));
    launch_node_prep(e->S, N, st);
    HIPCHK(e, hipGetLastError());
    // sort + apply + results queued right behind the prep: the apply pass returns at
    // once on the device when the prep listed records for the host (then the host
    // completes them and runs the sort and the pass again); one round trip otherwise
    auto sort_apply_results = [&]() -> int {
        if (launch_node_sort(e->S, N, G.sort_tmp, G.sort_bytes, sort_bits(e), st))
            return e->fail(KWOK_EDEVICE, "node sort");
        launch_node_apply(e->S, N, st);
        HIPCHK(e, hipGetLastError());
        if (int r = release_for_host(e)) return r;
        if (out_handles) HIPCHK(e, hipMemcpyAsync(G.res_h, G.out_handle, n * 4, hipMemcpyDeviceToHost, st));
        if (out_status) HIPCHK(e, hipMemcpyAsync(G.res_h + n, G.out_status, n * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(e, hipMemcpyAsync(G.nsum_h, G.nsum, sizeof(NodeSummary), hipMemcpyDeviceToHost, st));
        HIPCHK(e, hipStreamSynchronize(st));
        return KWOK_OK;
    };
    // from the apply pass on the batch is in the device state: a failure poisons the engine
    auto failed = [&](int r) {
        e->poisoned = true;
        return r;
    };
    if ((rc = upload_blobs(e))) return rc;  // (the empty-status blob, first batch)
    if ((rc = sort_apply_results())) return failed(rc);
    const auto t1 = clk::now();
    const uint32_t n_host = G.nsum_h->n_host;
    if (n_host) {
        // the records whose status strings need the host, in batch order (blob offsets do not
        // depend on it, but a deterministic interning order keeps the blob store reproducible)
        std::vector<uint32_t> idx(n_host);
        HIPCHK(e, hipMemcpyAsync(idx.data(), G.host_idx, (size_t)n_host * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(e, hipStreamSynchronize(st));
        std::sort(idx.begin(), idx.end());
        std::vector<NodeFix> fix(n_host);
        std::mutex blob_mu;
        const bool par = n_host >= NODE_PAR_MIN && e->n_part > 1;
        // kwok_ingest_nodes_json: the listed records the device decoded come back from
        // the device (their spans index the caller's documents); the host-decoded ones
        // are at hand with their canonical blobs
        std::vector<kwok_node_event> dev_rec;
        if (nj) {
            dev_rec.resize(n_host);
            HIPCHK(e, hipMemcpyAsync(G.host_idx, idx.data(), (size_t)n_host * 4, hipMemcpyHostToDevice, st));
            launch_node_gather(G.d_nev, G.host_idx, n_host, e->json.nev_fix, st);
            HIPCHK(e, hipGetLastError());
            HIPCHK(e, hipMemcpyAsync(dev_rec.data(), e->json.nev_fix, (size_t)n_host * sizeof(kwok_node_event),
                                     hipMemcpyDeviceToHost, st));
            HIPCHK(e, hipStreamSynchronize(st));
        }
        run_parts(e, par, [&](int p) {
            const size_t lo = par ? (size_t)n_host * p / e->n_part : (p ? n_host : 0);
            const size_t hi = par ? (size_t)n_host * (p + 1) / e->n_part : n_host;
            for (size_t k = lo; k < hi; k++) {
                if (!nj) {
                    fix[k] = complete_node(e, ev[idx[k]], idx[k], arena, blob_mu);
                    continue;
                }
                auto h = nj->hdoc->find(idx[k]);
                fix[k] = h == nj->hdoc->end()
                             ? complete_node(e, dev_rec[k], idx[k], nj->arena, blob_mu)
                             : complete_node(e, (*nj->hrec)[h->second], idx[k], (*nj->hbuf)[h->second].data(), blob_mu);
            }
        });
        if ((rc = upload_blobs(e))) return rc;
        HIPCHK(e, hipMemcpyAsync(G.d_nfix, fix.data(), fix.size() * sizeof(NodeFix), hipMemcpyHostToDevice, st));
        launch_node_fix(e->S, N, G.d_nfix, n_host, st);
        HIPCHK(e, hipGetLastError());
        N.force = 1;
        if ((rc = sort_apply_results())) return failed(rc);
    }
    const auto t2 = clk::now();
    if (out_handles) memcpy(out_handles, G.res_h, n * 4);
    if (out_status) memcpy(out_status, G.res_h + n, n * 4);
    const NodeSummary sum = *G.nsum_h;
    e->n_managed = (uint64_t)((int64_t)e->n_managed + sum.d_managed);
    if (sum.changed) {
        e->hb_pre_dirty = true;
        e->hb_epoch++;  // the managed set changed in this batch
    }
    if ((rc = size_arena(e))) return failed(rc);
    if (e->iprof)
        fprintf(stderr, "[kwok ingest] %zu node records (GPU%s): prep + sort + apply + results %.3f ms, host %u "
                        "records + again %.3f ms (%u created, %u freed)\n", n, zev ? ", read in place" : "",
                ms_between(t0, t1), n_host, ms_between(t1, t2), sum.created, sum.freed);
    return (int)sum.rejected;
}

// The stable sort by bucket of one chunk and its growth check (k_ing_need counts
// the creates in each bucket's sorted range), queued on the engine stream
int enqueue_sort_need(kwok_engine* e, const IngestBatch& I) {
    auto& G = e->ing;
    hipStream_t st = e->st;
    if (launch_ingest_sort(e->S, I, G.sort_tmp, G.sort_bytes, sort_bits(e), st))
        return e->fail(KWOK_EDEVICE, "ingest sort");
    launch_ingest_need(e->S, I, st);
    HIPCHK(e, hipGetLastError());
    return KWOK_OK;
}
// ... and its apply pass (spec: queued without the host's growth check; the pass
// then returns on the device if the chunk needs growth)
int enqueue_apply(kwok_engine* e, IngestBatch I, bool spec) {
    I.spec = spec ? 1u : 0u;
    if (I.n) e->ing_mutated = true;  // pod slots, node entries and references and the pool change from here on
    launch_ingest_apply(e->S, I, e->st);
    HIPCHK(e, hipGetLastError());
    return KWOK_OK;
}

// One chunk of a pod batch after its prep (I: the chunk's records, indices
// chunk-local), with the host in the loop: the growth check, the stable sort by
// bucket and the apply pass (by-name creates resolve their node in it).  Returns
// the chunk's rejected count (>= 0) or an error.  (The batch path queues the
// chunks without it and comes here only for a chunk that needs growth.)
int ingest_chunk(kwok_engine* e, const IngestBatch& I) {
    auto& G = e->ing;
    int rc = 0;
    if ((rc = enqueue_sort_need(e, I))) return rc;
    if ((rc = read_summary(e, I.sum))) return rc;
    const IngSummary sum = *G.sum_h;
    // growth: every bucket to a larger capacity (up to the handle stride) when the
    // chunk's creates could fill one
    if (sum.need > e->Cp) {
        const uint32_t cap = max_pod_capacity(e);
        if (cap > e->Cp) {
            e->ing_mutated = true;  // (a failed growth leaves the layout half changed)
            const uint32_t want = (uint32_t)std::min<uint64_t>(cap, std::max<uint64_t>(((uint64_t)sum.need + 7) & ~7ull, 2ull * e->Cp));
            if (e->iprof) fprintf(stderr, "[kwok grow] pod capacity per bucket %u -> %u\n", e->Cp, want);
            if ((rc = grow_pods(e, want))) return rc;
        }
    }
    if ((rc = enqueue_apply(e, I, false))) return rc;
    if ((rc = read_summary(e, I.sum))) return rc;
    if (G.sum_h->foreign) e->foreign_ips = true;
    return (int)G.sum_h->rejected;
}

// kwok_ingest_pods / kwok_ingest_pods_packed: recs are kwok_pod_event (with their
// string arena) or, packed, kwok_pod_rec (no arena); statuses to out_status
// (int32) or out_status8 (int8)
// resident: the records (kwok_pod_event) and their arena are on the device already,
// in the ingest buffers (kwok_ingest_pods_json decoded them there)
// packed: 0 kwok_pod_event, 1 kwok_pod_rec, 2 kwok_pod_rec12 (the creates' handles to
// out_new[k < new_cap], in create order; out_handles unused)
int ingest_pods_impl(kwok_engine* e, const void* recs, int packed, size_t n, const char* arena, size_t arena_len,
                     int32_t* out_handles, int32_t* out_status, int8_t* out_status8, uint32_t* out_released,
                     bool resident = false, int32_t* out_new = nullptr, size_t new_cap = 0, int64_t tick_now = -1) {
    const size_t RB = packed == 2 ? sizeof(kwok_pod_rec12) : packed ? sizeof(kwok_pod_rec) : sizeof(kwok_pod_event);
    static_assert(sizeof(kwok_pod_rec12) == 12, "kwok_pod_rec12 is 12 bytes");
    auto rec_at = [&](const void* base, size_t i) { return static_cast<const uint8_t*>(base) + i * RB; };
    if (e->poisoned) return poisoned(e);
    drain(e);  // the device state reflects every submitted tick
    if (e->poisoned) return poisoned(e);
    if (tick_now >= 0) {  // (checked before anything is queued)
        if (e->multi) return e->fail(KWOK_EINVAL, "ingest + tick in one call: single-rank engines only");
        if (int rc = tick_submit_check(e, tick_now)) return rc;
    }
    e->emit_hint = true;
    e->quiet = 0;
    e->sum_valid = false;
    if (!n) return tick_now >= 0 ? tick_submit_impl(e, tick_now) : 0;
    e->pod_records_since_tick += n;
    const auto t0 = clk::now();
    int rc = ingest_reserve(e, n, arena_len);
    if (rc) return rc;
    auto& G = e->ing;
    hipStream_t st = e->st, ps = G.pst;
    // Chunks of the batch in event order: applying them one after the other is
    // applying the batch (every record is applied in event order; a chunk is what
    // a separate call with those records would do).  The copy engine moves chunk
    // k+1's records to HBM (and k_ing_prep prepares them) on the prep stream while
    // the engine stream applies chunk k, and chunk k's results go back on the
    // results stream: the link carries the batch once in each direction, with the
    // apply passes under it.  The last chunk is shorter (its apply and results are
    // the part nothing hides).  The prep of chunk k + 2 waits until chunk k has
    // released its accumulator set.
    // kwok_pod_rec12's chunks start at multiples of 256 records (its create counts are
    // per 256-record tile, tile_new[lo / 256 + block]); its chunks hold at least 512
    // records, so that every chunk start rounds to a new tile and no chunk is empty.
    // The other wire forms split anywhere.
    const size_t chunk = packed == 2 ? std::max<size_t>(G.chunk, 512) : G.chunk;
    const uint32_t K = n > chunk ? (uint32_t)((n + chunk - 1) / chunk) : 1u;
    const double W = K > 1 ? K - e->last_chunk_cut : 1.0;
    const size_t lo_mask = packed == 2 ? ~(size_t)255 : ~(size_t)0;
    auto lo_of = [&](uint32_t k) { return k >= K ? n : (size_t)((double)n * k / W) & lo_mask; };
    // a one-chunk batch in kwok_host_alloc memory is read in place by k_ing_prep
    // (the only kernel that reads the records and their strings): one pass over
    // the link, no copy engine (KWOK_INGEST_ZC=0: copy it to HBM first).  Chunked
    // batches are copied: kernels reading host memory in place hold their CUs for
    // the link's latency, and the apply passes beside them stall (1M deletes + 1M
    // creates in 4 chunks: 4.9 ms read in place against 2.8 ms copied).
    if (K > G.nsums) {  // one summary per chunk: the batch reads them back once, at its end
        if (G.sums) (void)hipFree(G.sums);
        if (G.sums_h) (void)hipHostFree(G.sums_h);
        G.sums = nullptr, G.sums_h = nullptr, G.nsums = 0;
        const size_t m = std::max<size_t>(K, 16);
        if ((rc = dalloc(e, &G.sums, m))) return rc;
        if (hipHostMalloc((void**)&G.sums_h, m * sizeof(IngSummary), hipHostMallocDefault) != hipSuccess)
            return e->fail(KWOK_ENOMEM, "ingest summaries");
        G.nsums = m;
    }
    // (kwok_pod_rec12 records are read as three dwords: in place only when 4-byte aligned)
    const bool zc_ok = e->ingest_zc && K == 1 && !resident && (packed != 2 || ((uintptr_t)recs & 3) == 0);
    // kwok_pod_rec12's create handles: written by the kernel straight into a
    // kwok_host_alloc out_new_handles (each chunk's as it completes; no copy at the
    // batch's end), else into HBM and copied back after the last chunk.  With the
    // tick behind the batch they always take the copy: the kernel's writes over the
    // link hold CUs beside the tick's persistent blocks (C4 step 1.08-1.10 -> 1.04-1.05
    // ms, profiles/r13_new_handles_ab.txt; as two calls the in-place form is as fast)
    int32_t* new_map = packed == 2 && new_cap && e->new_mapped && tick_now < 0
                           ? (int32_t*)host_mapped(out_new, new_cap * 4)
                           : nullptr;
    int32_t* new_dst = new_map ? new_map : G.new_handle;
    const void* zev = zc_ok ? host_mapped(recs, n * RB) : nullptr;
    const void* zar = zc_ok && arena_len ? host_mapped(arena, arena_len) : nullptr;
    auto chunk_batch = [&](uint32_t k) {
        const size_t lo = lo_of(k);
        IngestBatch b = ingest_batch(e, (uint32_t)(lo_of(k + 1) - lo), arena_len);
        b.packed = (uint32_t)packed;
        if (packed == 2) b.tile_new = G.tile_new, b.tile_pre = G.tile_pre, b.tile0 = (uint32_t)(lo / 256);
        b.ev = rec_at(zev ? zev : (const void*)G.d_ev, lo);
        if (zar) b.arena = (const uint8_t*)zar;
        b.rec += lo, b.keys += lo, b.keys_sorted += lo, b.idx_sorted += lo;
        b.out_handle += lo, b.out_status += lo, b.out_released += lo;
        b.sum = G.sums + k;
        b.abort = G.abort;
        return b;
    };
    // prep of chunk k on stream s (the batch: the prep stream; a redo: the engine stream)
    auto prep_on = [&](uint32_t k, hipStream_t s) -> int {
        const IngestBatch b = chunk_batch(k);
        HIPCHK(e, hipMemsetAsync(b.sum, 0, sizeof(IngSummary), s));
        if (!zev && !resident)
            HIPCHK(e, hipMemcpyAsync(const_cast<uint8_t*>(rec_at(G.d_ev, lo_of(k))), rec_at(recs, lo_of(k)), (size_t)b.n * RB,
                                     hipMemcpyHostToDevice, s));
        launch_ingest_prep(e->S, b, s);
        HIPCHK(e, hipGetLastError());
        return KWOK_OK;
    };
    const bool tstamp = e->iprof && G.tev[0] && K == 2;
    clk::time_point t_copy0 = t0, t_synced = t0;
    // (the copy goes ahead of the summary reset: the link starts as early as possible.
    // Chunk 0 waits for the engine stream's earlier work first - the buffers' zeroing
    // when ingest_reserve just allocated them, above all)
    auto prep = [&](uint32_t k) -> int {
        const IngestBatch b = chunk_batch(k);
        if (k == 0) {
            t_copy0 = clk::now();
            HIPCHK(e, hipStreamWaitEvent(ps, G.go, 0));
        }
        if (tstamp) HIPCHK(e, hipEventRecord(G.tev[2 * k], ps));  // 0 / 2: chunk k's copy starts
        if (!zev && !resident)
            HIPCHK(e, hipMemcpyAsync(const_cast<uint8_t*>(rec_at(G.d_ev, lo_of(k))), rec_at(recs, lo_of(k)), (size_t)b.n * RB,
                                     hipMemcpyHostToDevice, ps));
        if (k >= 2) HIPCHK(e, hipStreamWaitEvent(ps, G.used[k & 1], 0));
        HIPCHK(e, hipMemsetAsync(b.sum, 0, sizeof(IngSummary), ps));
        launch_ingest_prep(e->S, b, ps);
        HIPCHK(e, hipGetLastError());
        if (tstamp) HIPCHK(e, hipEventRecord(G.tev[2 * k + 1], ps));  // 1 / 3: its prep done
        HIPCHK(e, hipEventRecord(G.prepped[k & 1], ps));
        return KWOK_OK;
    };
    e->ing_mutated = false;  // set by ingest_chunk once the batch changes any state
    // the prep stream starts after the work already queued on the engine stream
    // results of chunk k (after its apply pass, on the results stream) -> the caller's arrays
    auto results = [&](uint32_t k, hipStream_t rs) -> int {
        const size_t lo = lo_of(k);
        const IngestBatch I = chunk_batch(k);
        // KWOK_INGEST_RESULTS_KERNEL=1: results into kwok_host_alloc arrays written by a
        // kernel through their mapped addresses instead of the copy engine (slower:
        // 1.9 vs 1.45 ms per C4 batch; kept for A/B of the host-side stalls, §11)
        int32_t* mh = out_handles ? (int32_t*)host_mapped(out_handles + lo, (size_t)I.n * 4) : nullptr;
        int32_t* ms = out_status ? (int32_t*)host_mapped(out_status + lo, (size_t)I.n * 4) : nullptr;
        int8_t* m8 = out_status8 ? (int8_t*)host_mapped(out_status8 + lo, I.n) : nullptr;
        uint32_t* mr = out_released ? (uint32_t*)host_mapped(out_released + lo, (size_t)I.n * 4) : nullptr;
        if (packed == 2) {  // the chunk's creates' handles at their ordinals (copied back at the batch's end)
            launch_ingest_new_handles(I, new_dst, (uint32_t)std::min<size_t>(new_cap, new_map ? new_cap : G.cap), rs);
            HIPCHK(e, hipGetLastError());
        }
        const bool mapped = e->results_kernel && (!out_handles || mh) && (!out_status || ms) && (!out_status8 || m8) &&
                            (!out_released || mr);
        if (mapped) {
            launch_ingest_results(I, mh, ms, m8, mr, rs);
            HIPCHK(e, hipGetLastError());
            HIPCHK(e, hipEventRecord(e->fence, rs));  // (system-scope release: the host reads them)
            return KWOK_OK;
        }
        if (out_handles) HIPCHK(e, hipMemcpyAsync(out_handles + lo, I.out_handle, (size_t)I.n * 4, hipMemcpyDeviceToHost, rs));
        if (out_status) HIPCHK(e, hipMemcpyAsync(out_status + lo, I.out_status, (size_t)I.n * 4, hipMemcpyDeviceToHost, rs));
        if (out_status8) {  // one byte per record over the link
            launch_ingest_status8(I, G.out_status8 + lo, rs);
            HIPCHK(e, hipGetLastError());
            HIPCHK(e, hipMemcpyAsync(out_status8 + lo, G.out_status8 + lo, I.n, hipMemcpyDeviceToHost, rs));
        }
        if (out_released)
            HIPCHK(e, hipMemcpyAsync(out_released + lo, I.out_released, (size_t)I.n * 4, hipMemcpyDeviceToHost, rs));
        return KWOK_OK;
    };
    // The whole batch is queued without a host round trip per chunk: each chunk's
    // growth check (k_ing_need), sort and apply pass go behind its prep, and the
    // apply pass itself returns when the chunk needs more pod slots than a bucket
    // has (or an earlier chunk did).  One read-back of the chunks' summaries at the
    // end: the rare chunk that needs growth and the chunks after it are then applied
    // again with the host in the loop (ingest_chunk), in order.
    int tick_k = -1;  // tick mode: the slot of the tick queued behind the batch
    auto run = [&]() -> int {
        HIPCHK(e, hipEventRecord(G.go, st));
        if (arena_len && !zar && !resident) {  // (the arena ahead of the records: prep reads both)
            HIPCHK(e, hipStreamWaitEvent(ps, G.go, 0));  // (its buffer's zeroing, if just allocated)
            HIPCHK(e, hipMemcpyAsync(G.d_arena, arena, arena_len, hipMemcpyHostToDevice, ps));
        }
        for (uint32_t k = 0; k < std::min<uint32_t>(K, 2); k++)
            if (int r = prep(k)) return r;
        HIPCHK(e, hipMemsetAsync(G.abort, 0, 4, st));
        // (tick mode: the results always on their own stream, the tick's launches on the engine's)
        hipStream_t rs = (K > 1 && e->results_stream) || tick_now >= 0 ? G.dst : st;
        for (uint32_t k = 0; k < K; k++) {
            const IngestBatch I = chunk_batch(k);
            HIPCHK(e, hipStreamWaitEvent(st, G.prepped[k & 1], 0));
            if (e->debug_fail_chunk == k + 1) return e->fail(KWOK_EDEVICE, "injected failure of ingest chunk %u", k);
            if (int r = enqueue_sort_need(e, I)) return r;
            if (int r = enqueue_apply(e, I, true)) return r;
            if (tstamp) HIPCHK(e, hipEventRecord(G.tev[4 + k], st));  // 4 / 5: chunk k applied
            // chunk k's results on the results stream; its accumulator set free for chunk k + 2
            HIPCHK(e, hipEventRecord(G.used[k & 1], st));
            if (rs != st) HIPCHK(e, hipStreamWaitEvent(rs, G.used[k & 1], 0));
            if (int r = results(k, rs)) return r;
            if (k + 2 < K)
                if (int r2 = prep(k + 2)) return r2;
        }
        if (int r = release_for_host(e)) return r;
        if (tick_now >= 0) {
            // the tick, right behind the last apply pass (its kernels run while the results
            // travel); every launch of it skips while G.abort says a chunk needs growth
            HIPCHK(e, hipMemcpyAsync(&e->S.bar->skip, G.abort, 4, hipMemcpyDeviceToDevice, st));
            if (int r = tick_submit_impl(e, tick_now)) return r;
            tick_k = e->queue[e->nq - 1];
        }
        // the host waits for the results stream alone when the tick is behind the batch
        hipStream_t ws = tick_now >= 0 ? rs : st;
        if (packed == 2) {  // the creates' handles (every chunk's), and the summaries after them (n_new)
            if (new_map) HIPCHK(e, hipEventRecord(e->fence, rs));  // (system-scope release: the host reads them)
            else HIPCHK(e, hipMemcpyAsync(out_new, G.new_handle, std::min(new_cap, n) * 4, hipMemcpyDeviceToHost, rs));
            if (rs != st && ws == st) {
                HIPCHK(e, hipEventRecord(G.rdone, rs));
                HIPCHK(e, hipStreamWaitEvent(st, G.rdone, 0));
            }
        }
        if (packed != 2 && rs != st && ws == st) {  // (the results stream joins the engine stream: one wait below)
            HIPCHK(e, hipEventRecord(G.rdone, rs));
            HIPCHK(e, hipStreamWaitEvent(st, G.rdone, 0));
        }
        // (tick mode: rs waited for the last apply pass, whose summary is then final)
        HIPCHK(e, hipMemcpyAsync(G.sums_h, G.sums, (size_t)K * sizeof(IngSummary), hipMemcpyDeviceToHost, ws));
        if (tstamp) HIPCHK(e, hipEventRecord(G.tev[6], rs));  // 6: results copied
        const auto tq = clk::now();
        if (e->sync_spin) {  // spin on the batch's last operation (as a tick's completion: no wake-up latency)
            HIPCHK(e, hipEventRecord(G.idone, ws));
            hipError_t q;
            while ((q = hipEventQuery(G.idone)) == hipErrorNotReady) {
            }
            if (q != hipSuccess) return e->fail(KWOK_EDEVICE, "ingest: %s", hipGetErrorString(q));
        } else {
            HIPCHK(e, hipStreamSynchronize(ws));
        }
        t_synced = clk::now();
        if (tstamp) {
            float ms[6] = {};
            for (int q = 1; q < 7; q++) (void)hipEventElapsedTime(&ms[q - 1], G.tev[0], G.tev[q]);
            fprintf(stderr, "[kwok ingest]   queued in %.3f ms; device from chunk 0's copy: prep0 %.3f, copy1 start %.3f, "
                            "prep1 %.3f, apply0 %.3f, apply1 %.3f, results %.3f ms\n", ms_between(t0, tq), ms[0], ms[1],
                    ms[2], ms[3], ms[4], ms[5]);
        }
        if (e->iprof) fprintf(stderr, "[kwok ingest]   %u chunk%s queued and applied +%.3f ms\n", K, K == 1 ? "" : "s",
                              ms_between(t0, clk::now()));
        int rejected = 0;
        uint32_t k = 0;
        for (; k < K; k++) {
            const IngSummary& q = G.sums_h[k];
            if (q.need > e->Cp) break;  // its pass (and every later chunk's) returned: growth first
            rejected += (int)q.rejected;
            if (q.foreign) e->foreign_ips = true;
            if (e->debug_fail_apply == k + 1)
                return e->fail(KWOK_EDEVICE, "injected failure after the apply pass of ingest chunk %u", k);
        }
        const bool regrow = k < K;
        for (; k < K; k++) {  // chunks from the first that needs growth: the host in the loop
            if (e->iprof) fprintf(stderr, "[kwok ingest]   chunk %u again with the growth check\n", k);
            if (int r = prep_on(k, st)) return r;
            e->ing_chunk = k;
            const int r = ingest_chunk(e, chunk_batch(k));
            if (r < 0) return r;
            if (e->debug_fail_apply == k + 1)
                return e->fail(KWOK_EDEVICE, "injected failure after the apply pass of ingest chunk %u", k);
            rejected += r;
            if (int r2 = results(k, st)) return r2;
            if (packed == 2 && k + 1 == K) {
                if (new_map) HIPCHK(e, hipEventRecord(e->fence, st));
                else HIPCHK(e, hipMemcpyAsync(out_new, G.new_handle, std::min(new_cap, n) * 4, hipMemcpyDeviceToHost, st));
                HIPCHK(e, hipMemcpyAsync(G.sums_h + k, G.sums + k, sizeof(IngSummary), hipMemcpyDeviceToHost, st));
            }
            HIPCHK(e, hipStreamSynchronize(st));
        }
        if (regrow && tick_k >= 0) {  // the tick's launches skipped: queued again behind the chunks
            kwok_engine::TickSlot& T = e->slots[tick_k];
            if (int r = grow_arena(e, T)) return r;  // (the growth may have raised the tick's worst case)
            memset(T.hdr_h, 0, sizeof(TickHdr));
            HIPCHK(e, hipMemsetAsync(&e->S.bar->skip, 0, sizeof(uint32_t), st));
            if (int r = enqueue_tick(e, tick_k, true)) return r;
        }
        return rejected;
    };
    rc = run();
    // kwok_pod_rec12 with more creates than out_new_handles holds: the batch is applied
    // (not a failure of the engine), the call reports the lost handles.  A batch that
    // fails once it changed the state (a chunk applied, or the failing chunk's own
    // apply pass, placeholders or growth) is partly in the state: every later call fails
    if (rc >= 0 && packed == 2 && G.sums_h[K - 1].n_new > new_cap)
        rc = e->fail(KWOK_EINVAL, "kwok_ingest_pods_packed12: %u creates, out_new_handles holds %zu",
                     G.sums_h[K - 1].n_new, new_cap);
    else if (rc < 0 && e->ing_mutated)
        e->poisoned = true;
    if (rc < 0 && tick_k >= 0 && e->poisoned) {  // the tick behind a batch that failed half applied fails with it
        kwok_engine::TickSlot& T = e->slots[tick_k];
        if (T.state == SLOT_QUEUED) {
            (void)hipStreamSynchronize(st);
            T.state = SLOT_DONE;
            T.rc = rc;
            T.err = e->err;
        }
    }
    // nothing of this batch stays queued on the engine / prep / results streams (a failed
    // chunk included; a batch that ran to its end synchronised them in run(): the engine
    // stream's applies waited for every prep, the results stream was synchronised)
    if (rc < 0) {
        if (hipStreamSynchronize(st) != hipSuccess && rc >= 0) rc = e->fail(KWOK_EDEVICE, "ingest engine stream");
        if (hipStreamSynchronize(ps) != hipSuccess && rc >= 0) rc = e->fail(KWOK_EDEVICE, "ingest prep stream");
        if (hipStreamSynchronize(G.dst) != hipSuccess && rc >= 0) rc = e->fail(KWOK_EDEVICE, "ingest results stream");
    }
    if (e->iprof)
        fprintf(stderr, "[kwok ingest] %zu pod records (GPU%s, %u chunk%s%s): %.3f ms (first copy queued at %.3f, synced at %.3f)\n",
                n, zev ? ", read in place" : "", K, K == 1 ? "" : "s",
                packed == 2 ? (new_map ? ", create handles mapped" : ", create handles copied") : "", ms_between(t0, clk::now()),
                ms_between(t0, t_copy0), ms_between(t0, t_synced));
    return rc;
}

int kwok_ingest_pods(kwok_engine* e, const kwok_pod_event* ev, size_t n, const char* arena, size_t arena_len,
                     int32_t* out_handles, int32_t* out_status, uint32_t* out_released) {
    if (!e || (n && !ev) || n > 0x7FFFFFF0ull || (arena_len && !arena)) return KWOK_EINVAL;
    return ingest_pods_impl(e, ev, 0, n, arena, arena_len, out_handles, out_status, nullptr, out_released);
}

int kwok_ingest_pods_packed(kwok_engine* e, const kwok_pod_rec* recs, size_t n, int32_t* out_handles, int8_t* out_status,
                            uint32_t* out_released) {
    if (!e || (n && !recs) || n > 0x7FFFFFF0ull) return KWOK_EINVAL;
    return ingest_pods_impl(e, recs, 1, n, nullptr, 0, out_handles, nullptr, out_status, out_released);
}

int kwok_ingest_pods_packed12(kwok_engine* e, const kwok_pod_rec12* recs, size_t n, int32_t* out_new_handles,
                              size_t new_cap, int8_t* out_status, uint32_t* out_released) {
    if (!e || (n && !recs) || n > 0x7FFFFFF0ull || (new_cap && !out_new_handles)) return KWOK_EINVAL;
    return ingest_pods_impl(e, recs, 2, n, nullptr, 0, nullptr, nullptr, out_status, out_released, false,
                            out_new_handles, new_cap);
}

int kwok_ingest_pods_packed12_tick(kwok_engine* e, const kwok_pod_rec12* recs, size_t n, int32_t* out_new_handles,
                                   size_t new_cap, int8_t* out_status, uint32_t* out_released, int64_t now_unix) {
    if (!e || (n && !recs) || n > 0x7FFFFFF0ull || (new_cap && !out_new_handles) || now_unix < 0) return KWOK_EINVAL;
    return ingest_pods_impl(e, recs, 2, n, nullptr, 0, nullptr, nullptr, out_status, out_released, false,
                            out_new_handles, new_cap, now_unix);
}

// ---- the pod codec on the GPU (json.hip) ------------------------------------
namespace {
int json_reserve(kwok_engine* e, size_t n) {
    auto& J = e->json;
    if (!J.cfg) {
        int rc = 0;
        if ((rc = dalloc(e, &J.cfg, 1)) || (rc = dalloc(e, &J.n_host, 1))) return rc;
        if (hipHostMalloc((void**)&J.cfg_h, sizeof(JsonCfg), hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void**)&J.n_host_h, sizeof(uint32_t), hipHostMallocDefault) != hipSuccess)
            return e->fail(KWOK_ENOMEM, "GPU codec staging");
    }
    if (n > J.cap) {
        void* ptrs[] = {J.off, J.len, J.op, J.handle, J.side, J.host_list, J.fix_ev, J.fix_side};
        for (void* p : ptrs)
            if (p) (void)hipFree(p);
        J.off = nullptr, J.len = nullptr, J.op = nullptr, J.handle = nullptr, J.side = nullptr;
        J.host_list = nullptr, J.fix_ev = nullptr, J.fix_side = nullptr;
        J.cap = 0;
        const size_t cap = std::max<size_t>(n + n / 4, 4096);
        int rc = 0;
        if ((rc = dalloc(e, &J.off, cap)) || (rc = dalloc(e, &J.len, cap)) || (rc = dalloc(e, &J.op, cap)) ||
            (rc = dalloc(e, &J.handle, cap)) || (rc = dalloc(e, &J.side, cap)) || (rc = dalloc(e, &J.host_list, cap)) ||
            (rc = dalloc(e, &J.fix_ev, cap)) || (rc = dalloc(e, &J.fix_side, cap)))
            return rc;
        J.cap = cap;
    }
    if (J.tab_dirty) {  // the spec table: open addressing at <= 50% load, rebuilt from spec_keys
        uint32_t slots = 1024;
        while (slots < 2 * e->spec_keys.size() + 2) slots <<= 1;
        if (slots - 1 != J.tab_mask || !J.tab_key) {
            if (J.tab_key) (void)hipFree(J.tab_key);
            if (J.tab_id) (void)hipFree(J.tab_id);
            if (J.tab_canon) (void)hipFree(J.tab_canon);
            J.tab_key = nullptr, J.tab_id = nullptr, J.tab_canon = nullptr;
            int rc = 0;
            if ((rc = dalloc(e, &J.tab_key, slots)) || (rc = dalloc(e, &J.tab_id, slots)) ||
                (rc = dalloc(e, &J.tab_canon, slots)))
                return rc;
            J.tab_mask = slots - 1;
        }
        std::vector<uint64_t> key(slots, 0);
        std::vector<int32_t> id(slots, -1);
        std::vector<uint2> cref(slots, uint2{0, 0});
        std::string canon;
        for (auto& kv : e->spec_keys) {
            uint64_t k = kv.first ? kv.first : 1;  // (0 marks an empty slot: key 0 is never found)
            if (!kv.first) continue;
            uint32_t h = (uint32_t)k & J.tab_mask;
            while (key[h]) h = (h + 1) & J.tab_mask;
            key[h] = k;
            id[h] = kv.second;
            const std::string& c = e->spec_canon[kv.first];
            cref[h] = uint2{(uint32_t)canon.size(), (uint32_t)c.size()};
            canon += c;
        }
        if (canon.size() + 16 > J.canon_cap) {
            if (J.canon) (void)hipFree(J.canon);
            J.canon = nullptr, J.canon_cap = 0;
            const size_t cap = std::max<size_t>(2 * canon.size() + 16, 4096);
            if (int rc = dalloc(e, &J.canon, cap)) return rc;
            J.canon_cap = cap;
        }
        HIPCHK(e, hipMemcpyAsync(J.tab_key, key.data(), slots * 8, hipMemcpyHostToDevice, e->st));
        HIPCHK(e, hipMemcpyAsync(J.tab_id, id.data(), slots * 4, hipMemcpyHostToDevice, e->st));
        HIPCHK(e, hipMemcpyAsync(J.tab_canon, cref.data(), slots * sizeof(uint2), hipMemcpyHostToDevice, e->st));
        if (!canon.empty()) HIPCHK(e, hipMemcpyAsync(J.canon, canon.data(), canon.size(), hipMemcpyHostToDevice, e->st));
        HIPCHK(e, hipStreamSynchronize(e->st));
        J.tab_dirty = false;
    }
    return KWOK_OK;
}

// decode documents [0, n) on the device: the arena and the spans go to the ingest
// buffers, k_json_pods writes the records there (ingest form when op != null);
// returns the number of documents listed for the host (JSON_HOST / JSON_SPEC)
int json_decode(kwok_engine* e, const kwok_codec* c, const char* arena, size_t arena_len, const uint64_t* doc_off,
                const uint32_t* doc_len, size_t n, const uint8_t* op, const int32_t* handle, uint32_t* n_host) {
    auto& G = e->ing;
    auto& J = e->json;
    hipStream_t st = e->st;
    int rc = ingest_reserve(e, n, arena_len + 16);  // (the scanner reads whole 16-byte windows)
    if (rc) return rc;
    if ((rc = json_reserve(e, n))) return rc;
    // selectors beyond the device's tables (JSEL_*): every document is decoded by the
    // host codec (JSON_HOST), as any other document the scanner does not decide
    if ((rc = codec_export(c, J.cfg_h))) {
        if (rc != KWOK_EDOMAIN) return e->fail(rc, "%s", kwok_codec_last_error());
        memset(J.cfg_h, 0, sizeof(JsonCfg));
        J.cfg_h->all_host = 1;
    }
    HIPCHK(e, hipMemcpyAsync(J.cfg, J.cfg_h, sizeof(JsonCfg), hipMemcpyHostToDevice, st));
    HIPCHK(e, hipMemcpyAsync(J.off, doc_off, n * 8, hipMemcpyHostToDevice, st));
    HIPCHK(e, hipMemcpyAsync(J.len, doc_len, n * 4, hipMemcpyHostToDevice, st));
    if (op) {
        HIPCHK(e, hipMemcpyAsync(J.op, op, n, hipMemcpyHostToDevice, st));
        HIPCHK(e, hipMemcpyAsync(J.handle, handle, n * 4, hipMemcpyHostToDevice, st));
    }
    HIPCHK(e, hipMemsetAsync(J.n_host, 0, 4, st));
    // Documents in arena order (offsets non-decreasing, the usual batch): the arena
    // crosses the link in K pieces on the prep stream, and each piece's documents
    // are decoded on the engine stream as soon as it has landed - the decode runs
    // under the copy, which bounds the call (the link: ~2.7 GB per C4 tick).
    // Otherwise one copy, then one decode.
    bool sorted = true;
    for (size_t i = 1; i < n && sorted; i++) sorted = doc_off[i] >= doc_off[i - 1] + doc_len[i - 1];
    const uint32_t K = sorted && arena_len > (64u << 20) ? (uint32_t)std::min<size_t>(8, n / 4096 + 1) : 1u;
    hipStream_t ps = G.pst;
    HIPCHK(e, hipEventRecord(G.go, st));  // the copies start after the engine stream's earlier work
    HIPCHK(e, hipStreamWaitEvent(ps, G.go, 0));
    const bool tprof = e->iprof && G.tev[0];
    if (tprof) HIPCHK(e, hipEventRecord(G.tev[0], ps));
    uint64_t copied = 0;
    for (uint32_t k = 0; k < K; k++) {
        const size_t d0 = n * k / K, d1 = n * (k + 1) / K;
        const uint64_t hi = k + 1 == K ? arena_len : std::min<uint64_t>(arena_len, doc_off[d1 - 1] + doc_len[d1 - 1]);
        if (hi > copied) {
            HIPCHK(e, hipMemcpyAsync(G.d_arena + copied, arena + copied, hi - copied, hipMemcpyHostToDevice, ps));
            copied = hi;
        }
        HIPCHK(e, hipEventRecord(G.prepped[k & 1], ps));
        HIPCHK(e, hipStreamWaitEvent(st, G.prepped[k & 1], 0));
        JsonPodArgs A{};
        A.arena = G.d_arena;
        A.arena_len = arena_len;
        A.doc_off = J.off + d0;
        A.doc_len = J.len + d0;
        A.n = (uint32_t)(d1 - d0);
        A.base = (uint32_t)d0;
        A.tab_mask = J.tab_mask;
        A.cfg = J.cfg;
        A.op = op ? J.op + d0 : nullptr;
        A.handle = op ? J.handle + d0 : nullptr;
        A.tab_key = J.tab_key;
        A.tab_id = J.tab_id;
        A.tab_canon = J.tab_canon;
        A.key_mask = spec_key_mask();
        A.canon = J.canon;
        A.ev = static_cast<kwok_pod_event*>(G.d_ev) + d0;
        A.side = J.side + d0;
        A.host_list = J.host_list;
        A.n_host = J.n_host;
        launch_json_pods(A, st);
        HIPCHK(e, hipGetLastError());
    }
    if (tprof) HIPCHK(e, hipEventRecord(G.tev[1], ps));
    if (tprof) HIPCHK(e, hipEventRecord(G.tev[2], st));
    HIPCHK(e, hipMemcpyAsync(J.n_host_h, J.n_host, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(e, hipStreamSynchronize(st));
    *n_host = *J.n_host_h;
    if (tprof) {
        float c = 0, d = 0;
        (void)hipEventElapsedTime(&c, G.tev[0], G.tev[1]);
        (void)hipEventElapsedTime(&d, G.tev[0], G.tev[2]);
        fprintf(stderr, "[kwok json]   %u piece%s: copies %.3f ms (%.1f GB/s), decoded %.3f ms after the first copy\n", K,
                K == 1 ? "" : "s", c, arena_len / (c * 1e6), d);
    }
    return KWOK_OK;
}

// the documents the scanner listed: decoded by the host codec (JSON_HOST), or their
// spec registered (JSON_SPEC: one host decode per new spec key); their records
// completed and written back.  ingest: the records take the caller's op / handle
// and a spec id (kwok_ingest_pods_json); else they stay as the codec writes them
// (names / spec keys back in names_ns / spec_key of the caller, indexed by document).
int json_complete(kwok_engine* e, const kwok_codec* c, const char* arena, size_t arena_len, const uint64_t* doc_off,
                  const uint32_t* doc_len, uint32_t nh, const uint8_t* op, const int32_t* handle,
                  std::vector<JsonPodSide>* sides_out, std::vector<uint32_t>* list_out) {
    auto& G = e->ing;
    auto& J = e->json;
    hipStream_t st = e->st;
    if (!nh) return KWOK_OK;
    std::vector<uint32_t> list(nh);
    std::vector<kwok_pod_event> ev(nh);
    std::vector<JsonPodSide> side(nh);
    launch_json_gather(static_cast<const kwok_pod_event*>(G.d_ev), J.side, J.host_list, nh, J.fix_ev, J.fix_side, st);
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipMemcpyAsync(list.data(), J.host_list, (size_t)nh * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(e, hipMemcpyAsync(ev.data(), J.fix_ev, (size_t)nh * sizeof(kwok_pod_event), hipMemcpyDeviceToHost, st));
    HIPCHK(e, hipMemcpyAsync(side.data(), J.fix_side, (size_t)nh * sizeof(JsonPodSide), hipMemcpyDeviceToHost, st));
    HIPCHK(e, hipStreamSynchronize(st));
    // specs registered here (JSON_SPEC), by both of the device's keys of their
    // canonical string (kwok_spec_key and a second, independent 64-bit hash): a later
    // document of the batch with both keys takes that spec without a host decode
    struct K2Hash {
        size_t operator()(const std::pair<uint64_t, uint64_t>& k) const { return (size_t)(k.first ^ (k.second * 31)); }
    };
    std::unordered_map<std::pair<uint64_t, uint64_t>, int32_t, K2Hash> fresh;
    char* ar = const_cast<char*>(arena);  // (kwok_decode_pod writes only node blobs)
    kwok_pod_doc d;
    for (uint32_t q = 0; q < nh; q++) {
        const uint32_t i = list[q];
        JsonPodSide& s = side[q];
        const bool ups = !op || op[i] == KWOK_OP_UPSERT;
        const std::pair<uint64_t, uint64_t> dkey{s.spec_key, s.spec_key2};  // (the device's, before the host decode)
        const bool miss = s.status == JSON_SPEC;  // (JSON_SPEC_X, a key that collides with a registered spec: decoded)
        if (miss) {
            auto f = fresh.find(dkey);
            if (f != fresh.end()) {
                ev[q].spec_id = f->second;
                ev[q].reserved0 = 0;
                s.status = KWOK_OK;
                continue;
            }
        }
        // the host codec decides this document (a new spec: one decode registers it)
        int rc = kwok_decode_pod(c, ar, arena_len, doc_off[i], doc_len[i], &d);
        kwok_pod_event x = rc == KWOK_OK ? d.ev : kwok_pod_event{};
        int32_t id = -1;
        if (rc == KWOK_OK) {
            kwok_pod_spec sp{d.containers, d.n_containers, d.init_containers, d.n_init_containers,
                             d.readiness_gates, d.n_readiness_gates};
            s.name_off = d.name.off, s.name_len = d.name.len, s.ns_off = d.namespace_.off, s.ns_len = d.namespace_.len;
            s.n_cont = (uint8_t)d.n_containers, s.n_init = (uint8_t)d.n_init_containers;
            s.n_gates = (uint8_t)d.n_readiness_gates;
            s.spec_key = kwok_spec_key(&sp, arena, arena_len);
            if (op && ups) {
                const int r2 = kwok_register_pod_spec(e, &sp, arena, arena_len, &id);
                if (r2 == KWOK_OK && miss) fresh[dkey] = id;
                else if (r2 == KWOK_EDOMAIN || r2 == KWOK_EFULL) rc = r2;  // the spec is outside the domain
                else return r2;
            }
        }
        if (op) {
            x.op = op[i];
            x.handle = handle[i];
            x.spec_id = ups ? id : -1;
            x.node_handle = -1;
            x.reserved0 = rc == KWOK_OK ? 0 : (uint8_t)(int8_t)rc;
        } else if (rc != KWOK_OK) {
            x = kwok_pod_event{};
        }
        ev[q] = x;
        s.status = rc;
    }
    HIPCHK(e, hipMemcpyAsync(J.fix_ev, ev.data(), (size_t)nh * sizeof(kwok_pod_event), hipMemcpyHostToDevice, st));
    launch_json_scatter(static_cast<kwok_pod_event*>(G.d_ev), J.fix_ev, J.host_list, nh, st);
    HIPCHK(e, hipGetLastError());
    HIPCHK(e, hipStreamSynchronize(st));
    if (sides_out) *sides_out = std::move(side);
    if (list_out) *list_out = std::move(list);
    return KWOK_OK;
}
}  // namespace

uint64_t kwok_spec_key(const kwok_pod_spec* spec, const char* arena, size_t arena_len) {
    if (!spec) return 0;
    auto str = [&](kwok_str s) {
        return (size_t)s.off + s.len <= arena_len ? std::string(arena + s.off, s.len) : std::string();
    };
    std::vector<Container> cs(spec->n_containers), ics(spec->n_init_containers);
    std::vector<std::string> gates(spec->n_readiness_gates);
    for (uint32_t i = 0; i < spec->n_containers; i++) cs[i] = {str(spec->containers[i].name), str(spec->containers[i].image)};
    for (uint32_t i = 0; i < spec->n_init_containers; i++)
        ics[i] = {str(spec->init_containers[i].name), str(spec->init_containers[i].image)};
    for (uint32_t i = 0; i < spec->n_readiness_gates; i++) gates[i] = str(spec->readiness_gates[i]);
    return json_spec_key(cs, ics, gates);
}

// ---- node documents on the GPU (json.hip k_json_nodes) -----------------------
// kwok_ingest_nodes_json: WatchNodes / ListNodes from the documents themselves
// (node_controller.go:206-279): decoded on the device, the host codec only for
// the documents the scanner lists (a non-empty addresses / allocatable /
// capacity blob, whose canonical form is the host's, or an escaped routed
// string), then kwok_ingest_nodes' GPU event switch over the records, which
// stay on the device.
namespace {
// documents [0, n) decoded on the device: records in ing.d_nev (op: the caller's, or
// KWOK_OP_UPSERT when op is null; 0xFF for a document not decided there), the
// decode statuses into dstat, the number listed for the host (json.host_list) in *nh
int json_nodes_decode(kwok_engine* e, const kwok_codec* c, const char* arena, size_t arena_len, const uint64_t* doc_off,
                      const uint32_t* doc_len, const uint8_t* op, size_t n, std::vector<int32_t>& dstat, uint32_t* nh) {
    const auto t0 = clk::now();
    int rc = node_reserve(e, n, arena_len + 16);  // (the scanner reads whole 16-byte windows)
    if (rc) return rc;
    if ((rc = json_reserve(e, n))) return rc;
    auto& G = e->ing;
    auto& J = e->json;
    if (n > J.ncap) {
        if (J.nstat) (void)hipFree(J.nstat);
        if (J.nev_fix) (void)hipFree(J.nev_fix);
        J.nstat = nullptr, J.nev_fix = nullptr, J.ncap = 0;
        const size_t cap = std::max<size_t>(n + n / 4, 4096);
        if ((rc = dalloc(e, &J.nstat, cap)) || (rc = dalloc(e, &J.nev_fix, cap))) return rc;
        J.ncap = cap;
    }
    hipStream_t st = e->st, ps = G.pst;
    if ((rc = codec_export(c, J.cfg_h))) {  // (selectors beyond the device tables: every document to the host)
        if (rc != KWOK_EDOMAIN) return e->fail(rc, "%s", kwok_codec_last_error());
        memset(J.cfg_h, 0, sizeof(JsonCfg));
        J.cfg_h->all_host = 1;
    }
    HIPCHK(e, hipMemcpyAsync(J.cfg, J.cfg_h, sizeof(JsonCfg), hipMemcpyHostToDevice, st));
    HIPCHK(e, hipMemcpyAsync(J.off, doc_off, n * 8, hipMemcpyHostToDevice, st));
    HIPCHK(e, hipMemcpyAsync(J.len, doc_len, n * 4, hipMemcpyHostToDevice, st));
    if (op) HIPCHK(e, hipMemcpyAsync(J.op, op, n, hipMemcpyHostToDevice, st));
    else HIPCHK(e, hipMemsetAsync(J.op, KWOK_OP_UPSERT, n, st));
    HIPCHK(e, hipMemsetAsync(J.n_host, 0, 4, st));
    // the arena in pieces on the prep stream, each piece's documents decoded as it lands
    bool sorted = true;
    for (size_t i = 1; i < n && sorted; i++) sorted = doc_off[i] >= doc_off[i - 1] + doc_len[i - 1];
    const uint32_t K = sorted && arena_len > (64u << 20) ? (uint32_t)std::min<size_t>(8, n / 4096 + 1) : 1u;
    HIPCHK(e, hipEventRecord(G.go, st));
    HIPCHK(e, hipStreamWaitEvent(ps, G.go, 0));
    uint64_t copied = 0;
    for (uint32_t k = 0; k < K; k++) {
        const size_t d0 = n * k / K, d1 = n * (k + 1) / K;
        const uint64_t hi = k + 1 == K ? arena_len : std::min<uint64_t>(arena_len, doc_off[d1 - 1] + doc_len[d1 - 1]);
        if (hi > copied) {
            HIPCHK(e, hipMemcpyAsync(G.d_arena + copied, arena + copied, hi - copied, hipMemcpyHostToDevice, ps));
            copied = hi;
        }
        HIPCHK(e, hipEventRecord(G.prepped[k & 1], ps));
        HIPCHK(e, hipStreamWaitEvent(st, G.prepped[k & 1], 0));
        JsonNodeArgs A{};
        A.arena = G.d_arena;
        A.arena_len = arena_len;
        A.doc_off = J.off + d0;
        A.doc_len = J.len + d0;
        A.op = J.op + d0;
        A.n = (uint32_t)(d1 - d0);
        A.cfg = J.cfg;
        A.ev = G.d_nev + d0;
        A.status = J.nstat + d0;
        A.host_list = J.host_list;
        A.n_host = J.n_host;
        A.base = (uint32_t)d0;
        launch_json_nodes(A, st);
        HIPCHK(e, hipGetLastError());
    }
    const auto tq = clk::now();
    dstat.resize(n);
    HIPCHK(e, hipMemcpyAsync(dstat.data(), J.nstat, n * 4, hipMemcpyDeviceToHost, st));
    HIPCHK(e, hipMemcpyAsync(J.n_host_h, J.n_host, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(e, hipStreamSynchronize(st));
    *nh = *J.n_host_h;
    if (e->iprof)
        fprintf(stderr, "[kwok json]   %zu node documents: queued %.3f ms, decoded + statuses back %.3f ms\n", n,
                ms_between(t0, tq), ms_between(tq, clk::now()));
    return KWOK_OK;
}
// the documents json_nodes_decode listed, sorted
int json_nodes_listed(kwok_engine* e, uint32_t nh, std::vector<uint32_t>& list) {
    list.resize(nh);
    if (!nh) return KWOK_OK;
    HIPCHK(e, hipMemcpyAsync(list.data(), e->json.host_list, (size_t)nh * 4, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    std::sort(list.begin(), list.end());
    return KWOK_OK;
}
}  // namespace

// ---- node documents on the GPU (json.hip k_json_nodes) -----------------------
// kwok_ingest_nodes_json: WatchNodes / ListNodes from the documents themselves
// (node_controller.go:206-279): decoded on the device, the host codec only for
// the documents the scanner lists (a non-empty addresses / allocatable /
// capacity blob, whose canonical form is the host's, or an escaped routed
// string), then kwok_ingest_nodes' GPU event switch over the records, which
// stay on the device.
int kwok_ingest_nodes_json(kwok_engine* e, const kwok_codec* c, const char* arena, size_t arena_len,
                           const uint64_t* doc_off, const uint32_t* doc_len, const uint8_t* op, size_t n,
                           int32_t* out_handles, int32_t* out_status, size_t* n_host) {
    if (!e || !c || (n && (!doc_off || !doc_len || !op)) || (arena_len && !arena) || n > 0x7FFFFFF0ull ||
        arena_len > 0xFFFFFFF0ull)
        return KWOK_EINVAL;
    if (e->poisoned) return poisoned(e);
    drain(e);
    if (e->poisoned) return poisoned(e);
    e->emit_hint = true;
    e->quiet = 0;
    e->sum_valid = false;
    if (n_host) *n_host = 0;
    if (!n) return 0;
    const auto t0 = clk::now();
    std::vector<int32_t> dstat;
    uint32_t nh = 0;
    int rc = json_nodes_decode(e, c, arena, arena_len, doc_off, doc_len, op, n, dstat, &nh);
    if (rc) return rc;
    auto& G = e->ing;
    auto& J = e->json;
    hipStream_t st = e->st;
    // the listed documents: the host codec on a private copy of each (it writes the
    // canonical blobs over their spans); their records to the device, spans moved to
    // the batch's arena (the device only bounds-checks the blob spans: the host
    // completion below interns the canonical bytes from the private copy)
    std::unordered_map<uint32_t, uint32_t> hdoc;
    std::vector<kwok_node_event> hrec(nh), hdev(nh);
    std::vector<std::string> hbuf(nh);
    if (nh) {
        std::vector<uint32_t> list;
        if ((rc = json_nodes_listed(e, nh, list))) return rc;
        const bool par = nh >= NODE_PAR_MIN && e->n_part > 1;
        run_parts(e, par, [&](int p) {
            const size_t lo = par ? (size_t)nh * p / e->n_part : (p ? nh : 0);
            const size_t hi = par ? (size_t)nh * (p + 1) / e->n_part : nh;
            for (size_t q = lo; q < hi; q++) {
                const uint32_t i = list[q];
                hbuf[q].assign(arena + doc_off[i], doc_len[i]);
                kwok_node_event x{};
                const int r = kwok_decode_node(c, hbuf[q].data(), hbuf[q].size(), 0, hbuf[q].size(), &x);
                hrec[q] = x;
                kwok_node_event d = x;
                auto mv = [&](kwok_str& s) {
                    if (s.len) s.off += (uint32_t)doc_off[i];
                };
                mv(d.name), mv(d.addresses), mv(d.allocatable), mv(d.capacity);
                for (int k = 0; k < KWOK_NI_COUNT; k++) mv(d.node_info[k]);
                d.op = r == KWOK_OK ? op[i] : (uint8_t)0xFF;
                if (r != KWOK_OK) d.name = kwok_str{0, 0};
                hdev[q] = d;
                dstat[i] = r;
            }
        });
        for (uint32_t q = 0; q < nh; q++) hdoc.emplace(list[q], q);
        HIPCHK(e, hipMemcpyAsync(J.host_list, list.data(), (size_t)nh * 4, hipMemcpyHostToDevice, st));
        HIPCHK(e, hipMemcpyAsync(J.nev_fix, hdev.data(), (size_t)nh * sizeof(kwok_node_event), hipMemcpyHostToDevice, st));
        launch_node_scatter(G.d_nev, J.nev_fix, J.host_list, nh, st);
        HIPCHK(e, hipGetLastError());
    }
    if (n_host) *n_host = nh;
    if (e->iprof)
        fprintf(stderr, "[kwok json] %zu node documents decoded on the GPU (%u by the host): %.2f ms\n", n, nh,
                ms_between(t0, clk::now()));
    NodeJsonCtx ctx{arena, &hdoc, &hrec, &hbuf};
    std::vector<int32_t> stat(out_status ? 0 : n);
    int32_t* so = out_status ? out_status : stat.data();
    rc = ingest_nodes_impl(e, nullptr, n, arena, arena_len, out_handles, so, &ctx);
    if (rc < 0) return rc;
    for (size_t i = 0; i < n; i++)  // a document that failed to decode: its decode status
        if (dstat[i] != KWOK_OK) {
            so[i] = dstat[i];
            if (out_handles) out_handles[i] = -1;
        }
    return rc;
}

// kwok_decode_nodes_gpu: the decode alone (tests): the records kwok_decode_nodes
// would write, the listed documents decoded by the host codec in place (it
// re-serialises their blobs over their spans, as kwok_decode_nodes does)
int kwok_decode_nodes_gpu(kwok_engine* e, const kwok_codec* c, char* arena, size_t arena_len, const uint64_t* doc_off,
                          const uint32_t* doc_len, size_t n, kwok_node_event* ev, int32_t* status, size_t* n_host) {
    if (!e || !c || (n && (!doc_off || !doc_len || !ev || !status)) || (arena_len && !arena) || n > 0x7FFFFFF0ull ||
        arena_len > 0xFFFFFFF0ull)
        return KWOK_EINVAL;
    if (e->poisoned) return poisoned(e);
    drain(e);
    if (e->poisoned) return poisoned(e);
    if (n_host) *n_host = 0;
    if (!n) return 0;
    std::vector<int32_t> dstat;
    uint32_t nh = 0;
    int rc = json_nodes_decode(e, c, arena, arena_len, doc_off, doc_len, nullptr, n, dstat, &nh);
    if (rc) return rc;
    HIPCHK(e, hipMemcpyAsync(ev, e->ing.d_nev, n * sizeof(kwok_node_event), hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    std::vector<uint32_t> list;
    if ((rc = json_nodes_listed(e, nh, list))) return rc;
    for (uint32_t i : list) {
        kwok_node_event x{};
        dstat[i] = kwok_decode_node(c, arena, arena_len, doc_off[i], doc_len[i], &x);
        ev[i] = x;
    }
    int bad = 0;
    for (size_t i = 0; i < n; i++) {
        status[i] = dstat[i];
        if (dstat[i] != KWOK_OK) ev[i] = kwok_node_event{};
        else ev[i].op = KWOK_OP_UPSERT;
        bad += dstat[i] != KWOK_OK;
    }
    if (n_host) *n_host = nh;
    return bad;
}

int kwok_decode_pods_gpu(kwok_engine* e, const kwok_codec* c, const char* arena, size_t arena_len,
                         const uint64_t* doc_off, const uint32_t* doc_len, size_t n, kwok_pod_event* ev,
                         kwok_str* name_ns, uint64_t* spec_key, int32_t* status, size_t* n_host) {
    if (!e || !c || (n && (!doc_off || !doc_len || !ev || !status)) || (arena_len && !arena) || n > 0x7FFFFFF0ull)
        return KWOK_EINVAL;
    if (e->poisoned) return poisoned(e);
    drain(e);
    if (e->poisoned) return poisoned(e);
    if (n_host) *n_host = 0;
    if (!n) return 0;
    uint32_t nh = 0;
    int rc = json_decode(e, c, arena, arena_len, doc_off, doc_len, n, nullptr, nullptr, &nh);
    if (rc) return rc;
    std::vector<JsonPodSide> hs;
    std::vector<uint32_t> hl;
    if ((rc = json_complete(e, c, arena, arena_len, doc_off, doc_len, nh, nullptr, nullptr, &hs, &hl))) return rc;
    std::vector<JsonPodSide> side(n);
    HIPCHK(e, hipMemcpyAsync(ev, e->ing.d_ev, n * sizeof(kwok_pod_event), hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipMemcpyAsync(side.data(), e->json.side, n * sizeof(JsonPodSide), hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    for (size_t q = 0; q < hl.size(); q++) side[hl[q]] = hs[q];  // the host-decided documents
    int bad = 0;
    for (size_t i = 0; i < n; i++) {
        status[i] = side[i].status;
        bad += side[i].status != KWOK_OK;
        if (name_ns) {
            name_ns[2 * i] = kwok_str{side[i].name_off, side[i].name_len};
            name_ns[2 * i + 1] = kwok_str{side[i].ns_off, side[i].ns_len};
        }
        if (spec_key) spec_key[i] = side[i].spec_key;
    }
    if (n_host) *n_host = nh;
    return bad;
}

int kwok_ingest_pods_json(kwok_engine* e, const kwok_codec* c, const char* arena, size_t arena_len,
                          const uint64_t* doc_off, const uint32_t* doc_len, const uint8_t* op, const int32_t* handle,
                          size_t n, int32_t* out_handles, int32_t* out_status, uint32_t* out_released, size_t* n_host) {
    if (!e || !c || (n && (!doc_off || !doc_len || !op || !handle)) || (arena_len && !arena) || n > 0x7FFFFFF0ull)
        return KWOK_EINVAL;
    if (e->poisoned) return poisoned(e);
    drain(e);
    if (e->poisoned) return poisoned(e);
    if (n_host) *n_host = 0;
    if (!n) return 0;
    const auto t0 = clk::now();
    uint32_t nh = 0;
    int rc = json_decode(e, c, arena, arena_len, doc_off, doc_len, n, op, handle, &nh);
    if (rc) return rc;
    if ((rc = json_complete(e, c, arena, arena_len, doc_off, doc_len, nh, op, handle, nullptr, nullptr))) return rc;
    if (n_host) *n_host = nh;
    if (e->iprof)
        fprintf(stderr, "[kwok json] %zu pod documents decoded on the GPU (%u by the host): %.2f ms\n", n, nh,
                ms_between(t0, clk::now()));
    // the event switch over the decoded records, which stayed on the device
    return ingest_pods_impl(e, e->ing.d_ev, 0, n, nullptr, arena_len, out_handles, out_status, nullptr, out_released,
                            true);
}

int kwok_pack_pod_events(const kwok_pod_event* ev, size_t n, const char* arena, size_t arena_len, kwok_pod_rec* out,
                         int32_t* status) {
    if ((n && (!ev || !out)) || (arena_len && !arena)) return KWOK_EINVAL;
    int bad = 0;
    auto ip_of = [&](kwok_str s, uint32_t* ip) {  // "" -> 0; otherwise a canonical, non-zero dotted quad
        *ip = 0;
        if (!s.len) return true;
        if ((uint64_t)s.off + s.len > arena_len) return false;
        return parse_ipv4(arena + s.off, s.len, ip) && *ip != 0;
    };
    for (size_t i = 0; i < n; i++) {
        const kwok_pod_event& x = ev[i];
        kwok_pod_rec r{};
        int st = KWOK_OK;
        const bool create = x.op == KWOK_OP_UPSERT && x.handle < 0;
        r.op = (uint8_t)(x.op | (create ? KWOK_REC_NEW : 0u));
        r.flags = (uint8_t)((x.flags & 31u) | ((x.phase & 7u) << KWOK_REC_PHASE_SHIFT));
        r.spec_id = x.op == KWOK_OP_UPSERT ? (uint16_t)x.spec_id : (uint16_t)0;
        r.target = create ? x.node_handle : x.handle;
        if (x.op != KWOK_OP_UPSERT && x.op != KWOK_OP_DELETE) st = KWOK_EINVAL;
        else if (create && x.node_handle < 0) st = KWOK_EINVAL;  // by spec.nodeName: the full form only
        else if (x.phase > KWOK_PHASE_UNKNOWN) st = KWOK_EINVAL;  // (a pod phase: the device prep's bound)
        else if (x.op == KWOK_OP_UPSERT && (x.spec_id < 0 || x.spec_id > 0xFFFF)) st = KWOK_EINVAL;
        else if (x.op == KWOK_OP_UPSERT && (x.creation_unix < 0 || x.creation_unix > 0xFFFFFFFFll)) st = KWOK_EDOMAIN;
        else if (x.op == KWOK_OP_UPSERT && (!ip_of(x.host_ip, &r.host_ip) || !ip_of(x.pod_ip, &r.pod_ip)))
            st = KWOK_EDOMAIN;
        else if (x.op == KWOK_OP_DELETE && !ip_of(x.pod_ip, &r.pod_ip)) r.pod_ip = 0;  // not released (as unparsed)
        r.creation = x.op == KWOK_OP_UPSERT && st == KWOK_OK ? (uint32_t)x.creation_unix : 0u;
        if (status) status[i] = st;
        if (st == KWOK_OK) out[i] = r;
        bad += st != KWOK_OK;
    }
    return bad;
}

int kwok_cni_pending(kwok_engine* e, int32_t* out, size_t cap, size_t* n_out) {
    if (!e || !n_out || (cap && !out)) return KWOK_EINVAL;
    if (e->poisoned) return poisoned(e);
    if (!e->S.cni) return e->fail(KWOK_EINVAL, "kwok_cni_pending: the engine was created without enable_cni");
    drain(e);
    if (e->poisoned) return poisoned(e);
    // scratch: the exchange list buffer (multi-rank ticks only, none in flight) and its counter
    HIPCHK(e, hipMemsetAsync(e->S.list_counts, 0, 4, e->st));
    launch_cni_pending(e->S, (int32_t*)e->S.use_list, e->S.list_counts, e->st);
    HIPCHK(e, hipGetLastError());
    uint32_t cnt = 0;
    if (int rc = release_for_host(e)) return rc;
    HIPCHK(e, hipMemcpyAsync(&cnt, e->S.list_counts, 4, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    std::vector<int32_t> h(cnt);
    if (cnt) {
        HIPCHK(e, hipMemcpyAsync(h.data(), e->S.use_list, (size_t)cnt * 4, hipMemcpyDeviceToHost, e->st));
        HIPCHK(e, hipStreamSynchronize(e->st));
    }
    (void)hipMemsetAsync(e->S.list_counts, 0, 8, e->st);
    std::sort(h.begin(), h.end());  // canonical order
    *n_out = cnt;
    if (cap < cnt) return e->fail(KWOK_EINVAL, "kwok_cni_pending: %u pods pending, buffer holds %zu", cnt, cap);
    if (cnt) memcpy(out, h.data(), (size_t)cnt * 4);
    return KWOK_OK;
}

int kwok_cni_assign(kwok_engine* e, const int32_t* handles, const uint32_t* ips, size_t n, int32_t* out_status) {
    if (!e || (n && (!handles || !ips)) || n > 0x7FFFFFF0ull) return KWOK_EINVAL;
    if (e->poisoned) return poisoned(e);
    if (!e->S.cni) return e->fail(KWOK_EINVAL, "kwok_cni_assign: the engine was created without enable_cni");
    drain(e);
    if (e->poisoned) return poisoned(e);
    if (!n) return 0;
    e->quiet = 0;
    e->sum_valid = false;
    // a handle assigned twice keeps its last valid IP (configurePod runs once per tick)
    std::vector<uint8_t> wr(n, 0);
    {
        std::unordered_map<int32_t, size_t> last;
        for (size_t i = 0; i < n; i++)
            if (ips[i]) last[handles[i]] = i;
        for (const auto& kv : last) wr[kv.second] = 1;
    }
    int rc = ingest_reserve(e, n, 0);
    if (rc) return rc;
    auto& G = e->ing;
    hipStream_t st = e->st;
    // scratch: the ingest buffers (handles, IPs, write flags, statuses)
    HIPCHK(e, hipMemsetAsync(G.sum, 0, sizeof(IngSummary), st));
    HIPCHK(e, hipMemcpyAsync(G.keys, handles, n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(e, hipMemcpyAsync(G.keys_sorted, ips, n * 4, hipMemcpyHostToDevice, st));
    HIPCHK(e, hipMemcpyAsync(G.idx_sorted, wr.data(), n, hipMemcpyHostToDevice, st));
    launch_cni_assign(e->S, (const int32_t*)G.keys, G.keys_sorted, (const uint8_t*)G.idx_sorted, (uint32_t)n,
                      G.out_status, &G.sum->rejected, st);
    HIPCHK(e, hipGetLastError());
    if ((rc = read_summary(e))) return rc;
    if (out_status) {
        HIPCHK(e, hipMemcpyAsync(out_status, G.out_status, n * 4, hipMemcpyDeviceToHost, st));
        HIPCHK(e, hipStreamSynchronize(st));
    }
    return (int)G.sum_h->rejected;
}

int kwok_pool_put(kwok_engine* e, const uint32_t* ips, size_t n) {
    if (!e || (n && !ips)) return KWOK_EINVAL;
    if (e->poisoned) return poisoned(e);
    drain(e);  // the host mirrors reflect every submitted tick
    if (e->poisoned) return poisoned(e);
    e->puts.insert(e->puts.end(), ips, ips + n);
    e->quiet = 0;
    e->sum_valid = false;
    e->foreign_ips = true;  // releases of another rank's pods (multi rank)
    return flush_ops(e);
}

namespace {

// k_emit for slot k's tick (S bound to slot k), behind its k_tick launch(es)
int enqueue_emit(kwok_engine* e, int k) {
    kwok_engine::TickSlot& T = e->slots[k];
    if (e->prof) HIPCHK(e, hipEventRecord(T.pev[4], e->st));
    launch_emit(e->S, e->emit_grid, T.now, (uint64_t)e->start, e->st);
    HIPCHK(e, hipGetLastError());
    if (e->prof) HIPCHK(e, hipEventRecord(T.pev[5], e->st));
    T.emit_queued = true;
    return KWOK_OK;
}

// Enqueue one tick on e->st into slot k.  Single rank: ONE persistent k_tick
// launch (no host synchronisation, no graph needed).  Multi-rank: k_tick FRONT
// (classify, bases, exchange message) -> allgather -> k_tick BACK (fold
// messages, lists, pool, emission).  requeue: the slot's tick was skipped on
// the device (queued behind a tick that needed finish_long_lists) and runs
// again with its own tag and arrival target.
int enqueue_tick(kwok_engine* e, int k, bool requeue) {
    DevState& S = e->S;
    kwok_engine::TickSlot& T = e->slots[k];
    hipStream_t st = e->st;
    // KWOK_INGEST_PROF: the host time to each launch of the tick (us after entry)
    const auto q0 = clk::now();
    double qs[4] = {-1, -1, -1, -1};  // hb_pre queued, slot bound, k_tick / k_once queued, k_pod_jobs queued
    auto qstamp = [&](int i) { if (e->iprof) qs[i] = ms_between(q0, clk::now()) * 1e3; };
    hipEvent_t* ev = e->prof ? T.pev : nullptr;
    uint32_t nhb = (uint32_t)e->n_managed;  // = the device's count of managed local node slots
    if (e->debug_fault_tick && e->front_launches + 1 == e->debug_fault_tick && !requeue) nhb++;  // tests: TICK_ERR_LAYOUT
    if (e->hb_pre_dirty) {
        // heartbeat handles are written in node order at per-chain-block bases:
        // managed nodes of the buckets before each block's range (k_hb_pre, from
        // the node batches' per-bucket counts)
        launch_hb_pre(S, e->d_hb_pre, e->d_hb_bpre, st);
        HIPCHK(e, hipGetLastError());
        e->hb_pre_dirty = false;
        qstamp(0);
    }
    // a long heartbeat stream is shared with the chain blocks once they are done
    // (measured at C2: 921/1024 to the streamers; short streams: streamers only)
    // a stream that fits the 256 MB Infinity Cache is rewritten from it every tick
    // (plain stores); a larger one (1M nodes: 1.07 GB) is written non-temporally:
    // 239 -> 216 us per 1M x 10M tick (no L2 pollution under the chain's reads,
    // no dirty L2 left for the kernel-end write-back)
    const uint64_t hb_bytes = (S.hb_once ? std::min<uint32_t>(nhb, 1u) : nhb) * (uint64_t)e->hb_stride;
    S.hb_nt = e->nt_env >= 0 ? (uint32_t)e->nt_env : (hb_bytes >= (256ull << 20) ? 1u : 0u);
    // the streamers' share: with the non-temporal stream the chain blocks finish
    // sooner (1M x 10M: classification 172 -> 122 us) and take more of the tail
    // (tools/share_sweep2.sh: 921 -> 860 /1024, 217 -> 208 us per tick)
    // ticks that likely emit pod jobs (events since the last tick) build them in
    // k_pod_jobs, one wave per two dirty 64-group runs, instead of the chain blocks'
    // serial chunk walk (KWOK_SPLIT=0: the chain blocks, for A/B)
    T.split = T.emit_queued && e->split_jobs;
    // ... writing the pod patch bytes there too when every spec has unit tables
    // (no 16-byte job record per patch written by k_pod_jobs and read back by k_emit)
    // and the tick is dense: pod records ingested since the last tick (creates,
    // updates, deletes: a bound on the patches their pods can need) >= 1/4 of the pod slots,
    // so most dirty runs hold hundreds of jobs (1M x 10M initial tick: emission
    // 1.79 -> 1.72 ms).  A sparse tick's runs hold a few jobs each; their serial
    // emission per wave loses to k_emit's packed 64-job chunks (C4 churn tick
    // 0.51 -> 0.57 ms fused; tools/gpu_r6b.sh)
    if (!requeue) {  // (a requeued tick keeps its decision)
        const bool dense = e->pod_records_since_tick * 4 >= (uint64_t)S.nb * e->Cp;
        e->pod_records_since_tick = 0;
        T.fuse = T.split && e->n_untabled == 0 && (e->fuse_emit > 0 || (e->fuse_emit < 0 && dense));
    }
    S.fuse_pods = T.fuse ? 1u : 0u;
    S.sparse_jobs = T.split && !T.fuse && e->sparse_jobs ? 1u : 0u;
    T.inits_folded = false;  // (set where k_pod_jobs is launched)
    // ... and leave the whole stream to the streamers: a dirty chain block's share
    // of it would hold up the pool phase, which waits for every dirty block
    S.stream_share = e->n_stream == 0 ? 0u
                     : e->share_env >= 0 ? (uint32_t)e->share_env
                                         : (hb_bytes < (32ull << 20) || T.split ? 1024u : (S.hb_nt ? 860u : 921u));
    S.use_events_only = T.quiet ? 1u : 0u;
    S.foreign = e->foreign_ips ? 1u : 0u;
    int rc = bind_slot(e, k);
    if (rc) return rc;
    qstamp(1);
    const int prof = (ev ? TICK_PROF : 0) | (e->chain_prio ? TICK_PRIO : 0) | (e->no_stream ? TICK_NOSTREAM : 0) |
                     (T.split ? TICK_SPLIT : 0);
    if (!requeue) {
        T.no_once = false;
        memset(T.hdr_h, 0, sizeof(TickHdr));  // the slot's previous tick was collected
        if (++e->tick_tag == 0) e->tick_tag = 1;
        T.tag = e->tick_tag;
        T.target = ++e->front_launches * S.n_chain;
    }
    const uint64_t now = T.now;
    // a heartbeat-once tick expected to have nothing to emit (no events since the
    // previous tick, quiet Use checks) runs k_once: one wave per bucket, every load
    // of the bucket in flight at once.  One that has work after all is run again
    // with k_tick by retire (TickHdr::redo; a launch queued behind it skips)
    T.once = !e->multi && S.hb_once && e->once_ok && !T.emit_queued && !T.split && T.quiet && !T.no_once &&
             S.cn <= (uint32_t)ONCE_NODE_LDS && e->PL < (1u << ONCE_FIELD_BITS) && e->NL < (1u << ONCE_FIELD_BITS);
    if (T.once) {
        // per-bucket summaries: BUILD them on the first once tick after a change, USE them after
        uint32_t mode = ONCE_SUM_OFF;
        if (e->once_sum_ok && e->Cp <= 0xFFFFu) {
            if (!e->sum_valid) {
                if (++e->sum_gen == 0) e->sum_gen = 1;
                e->sum_valid = true;
                mode = ONCE_SUM_BUILD;
            } else {
                mode = ONCE_SUM_USE;
            }
        }
        T.once_use = mode == ONCE_SUM_USE;
        launch_tick_once(S, now, (uint64_t)e->start, nhb, prof & TICK_PROF, mode, e->sum_gen, st, ev ? ev[0] : nullptr,
                         ev ? ev[1] : nullptr);
        HIPCHK(e, hipGetLastError());
        qstamp(2);
    } else if (!e->multi) {
        e->sum_valid = false;  // (a k_tick may change pod states)
        launch_tick(S, e->n_stream, now, (uint64_t)e->start, nhb, TICK_FRONT | TICK_BACK | prof, T.tag, T.target, st,
                    ev ? ev[0] : nullptr, ev ? ev[1] : nullptr);
        HIPCHK(e, hipGetLastError());
        qstamp(2);
    } else {
        e->sum_valid = false;
        launch_tick(S, e->n_stream, now, (uint64_t)e->start, nhb, TICK_FRONT | prof, T.tag, T.target, st,
                    ev ? ev[0] : nullptr, ev ? ev[1] : nullptr);
        // one allgather of the fixed-size exchange message, then BACK: it folds the
        // gathered messages and applies the inline lists itself (no host round trip).
        // Lists too long to be inline: BACK flags it and the host finishes the tick
        // with a second allgather (finish_long_lists).
        // After a long-list tick (TICK_XSPEC): the lists follow in a second allgather
        // of fixed capacity and k_pool_apply_spec applies them if every rank's fit.
        if (!requeue && e->xspec_ttl && --e->xspec_ttl == 0) e->xspec_u = e->xspec_r = 0;
        const bool spec = e->xspec_u + e->xspec_r != 0;
        if (spec) {
            S.xcap_u = e->xspec_u, S.xcap_r = e->xspec_r;
            launch_gather_lists(S, e->d_ssend, st, S.xcap_u, S.xcap_u, S.xcap_r);
            HIPCHK(e, hipGetLastError());
        }
        rc = exchange(e, S.xmsg, sizeof(XMsg), e->d_xall);
        if (rc) return rc;
        if (e->XW > e->W) launch_emulate_msgs(S, e->d_xall, (uint32_t)e->XW, st);  // (diagnostics: one rank, XW > 1)
        if (spec) {
            const uint32_t per = S.xcap_u + S.xcap_r;
            if ((rc = exchange(e, e->d_ssend, (size_t)per * 4, e->d_srecv))) return rc;
            if (e->XW > e->W) launch_emulate_lists(S, e->d_srecv, per, (uint32_t)e->XW, per, st);  // (diagnostics)
            launch_pool_apply_spec(S, e->d_srecv, st);
            HIPCHK(e, hipGetLastError());
        }
        launch_tick(S, e->n_stream, now, (uint64_t)e->start, nhb, TICK_BACK | prof | (spec ? TICK_XSPEC : 0), T.tag,
                    T.target, st, ev ? ev[2] : nullptr, ev ? ev[3] : nullptr);
        HIPCHK(e, hipGetLastError());
    }
    // a fused launch writes the node inits too (its last blocks): no k_emit
    T.inits_folded = T.fuse && e->fold_inits;
    if (T.split) {
        launch_pod_jobs(S, T.tag, st, T.inits_folded ? e->emit_grid : 0u, now, (uint64_t)e->start, ev ? ev[6] : nullptr,
                        ev ? ev[7] : nullptr);
        HIPCHK(e, hipGetLastError());
        qstamp(3);
    }
    // the patch bytes, when events since the last tick make jobs likely (otherwise
    // retire launches k_emit if the tick turns out to have jobs)
    if (T.emit_queued && !T.inits_folded && (rc = enqueue_emit(e, k))) return rc;
    HIPCHK(e, hipEventRecord(T.done, st));
    if (e->iprof)
        fprintf(stderr, "[kwok enqueue] us: hb_pre %.1f, bound %.1f, tick %.1f, pod_jobs %.1f, all %.1f\n", qs[0], qs[1], qs[2],
                qs[3], ms_between(q0, clk::now()) * 1e3);
    return KWOK_OK;
}
// multi rank, after the BACK launch of slot k's tick found lists too long to be
// inline (the same on every rank: the flag comes from the gathered messages):
// gather the lists, apply every rank's Uses and Puts, and run BACK again.  A tick
// queued behind it skipped on the device (GridBar::skip) and is enqueued again.
int finish_long_lists(kwok_engine* e, int k, int next) {
    DevState& S = e->S;
    kwok_engine::TickSlot& T = e->slots[k];
    hipStream_t st = e->st;
    T.hdr_h->xovf = 0;
    // the skipped tick's allgather re-gathered the same messages (its FRONT did not run)
    if (int rc = release_for_host(e)) return rc;
    HIPCHK(e, hipStreamSynchronize(st));
    HIPCHK(e, hipMemcpyAsync(e->h_xall, e->d_xall, sizeof(XMsg) * e->XW, hipMemcpyDeviceToHost, st));
    HIPCHK(e, hipStreamSynchronize(st));
    uint64_t maxl = 0, mu = 0, mr = 0;
    for (int r = 0; r < e->XW; r++) {
        maxl = std::max<uint64_t>(maxl, e->h_xall[r].n_use + e->h_xall[r].n_rel);
        mu = std::max<uint64_t>(mu, e->h_xall[r].n_use);
        mr = std::max<uint64_t>(mr, e->h_xall[r].n_rel);
    }
    if (e->xspec_env != 0) {
        // the next ticks' speculative list exchange: room for 1.25x this tick's
        // longest lists (the same on every rank: the gathered messages)
        if (e->xspec_u + e->xspec_r) e->xspec_miss++;
        auto cap = [](uint64_t m) { return (uint32_t)std::min<uint64_t>(((m + m / 4) | 1023) + 1, 1u << 30); };
        const bool miss = e->xspec_u + e->xspec_r != 0;  // a speculative tick whose lists did not fit: grow
        const uint32_t cu = miss ? std::max(e->xspec_u, cap(mu)) : cap(mu), cr = miss ? std::max(e->xspec_r, cap(mr)) : cap(mr);
        if (cu + cr > e->xspec_alloc) {
            if (e->d_ssend) (void)hipFree(e->d_ssend);
            if (e->d_srecv) (void)hipFree(e->d_srecv);
            e->d_ssend = e->d_srecv = nullptr;
            e->xspec_alloc = 0;
            if (hipMalloc((void**)&e->d_ssend, (size_t)(cu + cr) * 4) != hipSuccess ||
                hipMalloc((void**)&e->d_srecv, (size_t)(cu + cr) * 4 * e->XW) != hipSuccess)
                return e->fail(KWOK_ENOMEM, "speculative exchange lists");
            e->xspec_alloc = cu + cr;
        }
        e->xspec_u = cu, e->xspec_r = cr;
        e->xspec_ttl = e->xspec_env > 0 ? (uint32_t)e->xspec_env : 256u;
    }
    if (maxl > e->xlist_cap) {
        if (e->d_xsend) (void)hipFree(e->d_xsend);
        if (e->d_xrecv) (void)hipFree(e->d_xrecv);
        e->xlist_cap = maxl;
        if (hipMalloc((void**)&e->d_xsend, maxl * 4) != hipSuccess ||
            hipMalloc((void**)&e->d_xrecv, maxl * 4 * e->XW) != hipSuccess)
            return e->fail(KWOK_ENOMEM, "exchange lists");
    }
    int rc = bind_slot(e, k);
    if (rc) return rc;
    S.fuse_pods = T.fuse ? 1u : 0u;
    S.sparse_jobs = T.split && !T.fuse && e->sparse_jobs ? 1u : 0u;
    HIPCHK(e, hipMemsetAsync(&S.bar->skip, 0, sizeof(uint32_t), st));
    const XMsg& me = e->h_xall[e->rank];
    if (me.n_use + me.n_rel) {  // the chain blocks' list segments, gathered in block order
        launch_gather_lists(S, e->d_xsend, st);
        HIPCHK(e, hipGetLastError());
    }
    rc = exchange(e, e->d_xsend, maxl * 4, e->d_xrecv);
    if (rc) return rc;
    if (e->XW > e->W)  // (diagnostics)
        launch_emulate_lists(S, e->d_xrecv, maxl, (uint32_t)e->XW, (uint32_t)(me.n_use + me.n_rel), st);
    std::vector<ListDesc> ld(e->XW);
    for (int r = 0; r < e->XW; r++) {
        ld[r].use = e->d_xrecv + (size_t)r * maxl;
        ld[r].rel = e->d_xrecv + (size_t)r * maxl + e->h_xall[r].n_use;
        ld[r].n_use = (uint32_t)e->h_xall[r].n_use;
        ld[r].n_rel = (uint32_t)e->h_xall[r].n_rel;
    }
    HIPCHK(e, hipMemcpyAsync(e->d_ld, ld.data(), sizeof(ListDesc) * e->XW, hipMemcpyHostToDevice, st));
    launch_pool_apply(S, e->d_ld, e->XW, (uint32_t)maxl, st);  // every rank's Uses, then Puts pending
    launch_tick(S, e->n_stream, T.now, (uint64_t)e->start, (uint32_t)e->n_managed,
                TICK_BACK | TICK_XLISTS | (T.split ? TICK_SPLIT : 0), T.tag, T.target, st);
    HIPCHK(e, hipGetLastError());
    T.inits_folded = T.fuse && e->fold_inits;
    if (T.split) {
        launch_pod_jobs(S, T.tag, st, T.inits_folded ? e->emit_grid : 0u, T.now, (uint64_t)e->start);
        HIPCHK(e, hipGetLastError());
    }
    if (T.inits_folded) T.emit_queued = true;  // (the fused launch wrote every patch)
    else if ((rc = enqueue_emit(e, k))) return rc;  // this launch built the jobs
    HIPCHK(e, hipStreamSynchronize(st));
    if (next >= 0) return enqueue_tick(e, next, true);
    return KWOK_OK;
}

// single rank: the kernel publishes the tick's field totals (TickHdr::tot); the
// counts, output layout and counters follow from them
void derive_header(TickHdr& H, uint64_t arena_cap, uint32_t hb_stride, bool hb_once) {
    const uint64_t* t = H.tot;
    H.n_hb = (uint32_t)t[AG_HB];
    H.n_init = (uint32_t)t[AG_INIT];
    H.n_pp = (uint32_t)t[AG_PP];
    H.n_del = (uint32_t)t[AG_DEL];
    H.n_use = 0;
    H.n_rel = (uint32_t)t[AG_REL];
    H.n_alloc_local = (uint32_t)t[AG_ALLOC];
    H.n_eval = (uint32_t)t[AG_EVAL];
    H.n_lock = (uint32_t)t[AG_LOCK];
    H.init_bytes = t[AG_INIT_BYTES];
    H.pp_bytes = t[AG_PP_BYTES];
    H.hb_base = 0;
    H.init_base = (uint64_t)(hb_once ? std::min<uint32_t>(H.n_hb, 1u) : H.n_hb) * hb_stride;
    H.pod_base = H.init_base + H.init_bytes;
    H.arena_bytes = H.pod_base + H.pp_bytes;
    H.overflow = H.arena_bytes > arena_cap;
    const int map[13] = {AG_HB, AG_INIT, AG_PP, AG_DEL, AG_ALLOC, AG_REL, AG_EVAL,
                         AG_LOCK, AG_MANAGED, AG_READY, AG_TOTAL, AG_PENDING, AG_RUNNING};
    for (int k = 0; k < 16; k++) H.local_counters[k] = H.counters[k] = k < 13 ? t[map[k]] : 0;
    H.alloc_total = t[AG_ALLOC];
    H.alloc_base = 0;
    H.rel_total = t[AG_REL];
}

bool trace_enabled(const kwok_engine* e) { return e->S.trace != nullptr; }

// KWOK_JOBS_TRACE=file: the k_pod_jobs wave stamps of the last tick with pod jobs
// (tools/jobs_trace.py reads them), zeroed for the next
void jobs_trace_dump(kwok_engine* e) {
    const size_t n = (size_t)e->S.n_chain * (MAX_WC + 4) * 4;
    std::vector<uint64_t> h(n);
    if (hipMemcpy(h.data(), e->S.jtrace, n * 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemset(e->S.jtrace, 0, n * 8) != hipSuccess)
        return;
    if (FILE* f = fopen(getenv("KWOK_JOBS_TRACE"), "wb")) {
        fwrite(h.data(), 8, n, f);
        fclose(f);
    }
}

// per stamp k: earliest / median / latest block, microseconds after the earliest block start
void trace_tick(kwok_engine* e) {
    const size_t G = e->S.n_chain, N = G + e->n_stream;
    static const int skip = getenv("KWOK_TICK_TRACE_SKIP") ? atoi(getenv("KWOK_TICK_TRACE_SKIP")) : 5;
    static const uint64_t only = getenv("KWOK_TICK_TRACE_COUNT") ? strtoull(getenv("KWOK_TICK_TRACE_COUNT"), nullptr, 10) : 0;
    if ((int)++e->trace_seen <= skip) return;  // skip the initial (bulk) ticks
    if (only && e->trace_ticks >= only) return;  // KWOK_TICK_TRACE_COUNT: summarise only the first traced ticks
    const size_t TS = TRACE_SLOTS;
    e->trace_h.assign(N * TS, 0);
    if (release_for_host(e) || hipMemcpyAsync(e->trace_h.data(), e->S.trace, N * TS * 8, hipMemcpyDeviceToHost, e->st) != hipSuccess ||
        hipMemsetAsync(e->S.trace, 0, N * TS * 8, e->st) != hipSuccess || hipStreamSynchronize(e->st) != hipSuccess)
        return;
    uint64_t t0 = ~0ull;
    for (size_t b = 0; b < G; b++) t0 = std::min(t0, e->trace_h[b * TS]);
    // stamps a block did not reach this tick (a clean block skips the pool phase) are 0
    auto summarise = [&](size_t lo, size_t hi, int k, double* out) {
        std::vector<double> v;
        for (size_t b = lo; b < hi; b++)
            if (e->trace_h[b * TS + k] >= t0) v.push_back((double)(e->trace_h[b * TS + k] - t0) * 0.01);
        if (v.empty()) return;
        std::sort(v.begin(), v.end());
        out[0] += v[0];
        out[1] += v[v.size() / 2];
        out[2] += v[v.size() - 1];
    };
    for (int k = 0; k < TRACE_SLOTS; k++) summarise(0, G, k, e->trace_sum[k]);
    summarise(G, N, 0, e->trace_sum[TRACE_SLOTS]);
    summarise(G, N, 6, e->trace_sum[TRACE_SLOTS + 1]);
    if (getenv("KWOK_TICK_TRACE_SLOW")) {  // per XCC: median / max pods-done and arrival; the slowest blocks
        std::vector<double> pd[16], ar[16];
        std::vector<std::pair<double, size_t>> slow;
        for (size_t b = 0; b < G; b++) {
            const uint64_t* T = &e->trace_h[b * TS];
            if (T[2] < t0 || T[3] < t0) continue;
            const uint32_t x = (uint32_t)(T[21] >> 28) & 15u;
            pd[x].push_back((double)(T[2] - t0) * 0.01);
            ar[x].push_back((double)(T[3] - t0) * 0.01);
            slow.emplace_back((double)(T[3] - t0) * 0.01, b);
        }
        for (int x = 0; x < 16; x++) {
            if (pd[x].empty()) continue;
            std::sort(pd[x].begin(), pd[x].end());
            std::sort(ar[x].begin(), ar[x].end());
            fprintf(stderr, "[kwok trace xcc %d] blocks %zu pods-done %.1f / %.1f arrived %.1f / %.1f\n", x, pd[x].size(),
                    pd[x][pd[x].size() / 2], pd[x].back(), ar[x][ar[x].size() / 2], ar[x].back());
        }
        std::sort(slow.rbegin(), slow.rend());
        for (size_t q = 0; q < std::min<size_t>(8, slow.size()); q++) {
            const uint64_t* T = &e->trace_h[slow[q].second * TS];
            fprintf(stderr, "[kwok trace slow] block %zu hw %08llx nodes %.1f pods %.1f sum %.1f drained %.1f arrived %.1f\n",
                    slow[q].second, (unsigned long long)T[21], (double)(T[1] - t0) * 0.01, (double)(T[2] - t0) * 0.01,
                    (double)(T[10] - t0) * 0.01, (double)(T[11] - t0) * 0.01, (double)(T[3] - t0) * 0.01);
        }
    }
    if (getenv("KWOK_TICK_TRACE_RAW")) {  // the last block's 16 stamps (ad-hoc kernel probes), us after t0
        fprintf(stderr, "[kwok trace raw]");
        for (size_t k = 0; k < TS; k++) {
            const uint64_t v = e->trace_h[(N - 1) * TS + k];
            fprintf(stderr, " %.3f", k == 8 ? (double)v : v >= t0 ? (double)(v - t0) * 0.01 : -1.0);
        }
        fprintf(stderr, "\n");
    }
    e->trace_ticks++;
}



// k_once met work to emit in slot k's tick (a delete, patch, Get, Put, Use, pod
// event or node init): run the tick again with k_tick (same tag and arrival
// target: k_once made no arrivals).  The launch queued behind it skipped on the
// device (GridBar::skip); retire enqueues it again afterwards.
int redo_tick(kwok_engine* e, int k) {
    kwok_engine::TickSlot& T = e->slots[k];
    e->stats[KWOK_STAT_ONCE_REDO]++;
    e->sum_valid = false;
    memset(T.hdr_h, 0, sizeof(TickHdr));
    HIPCHK(e, hipMemsetAsync(&e->S.bar->skip, 0, sizeof(uint32_t), e->st));
    T.no_once = true;
    if (int rc = enqueue_tick(e, k, true)) return rc;
    HIPCHK(e, hipEventSynchronize(T.done));
    return KWOK_OK;
}

// Finish the oldest queued tick on the host: wait for it, complete a multi-rank
// tick with long lists, derive the header, check errors, mirror DeletePods into
// the host slot state.  The result stays in the slot until kwok_tick_collect.
int retire(kwok_engine* e) {
    int qi = -1;
    for (int i = 0; i < e->nq; i++)
        if (e->slots[e->queue[i]].state == SLOT_QUEUED) {
            qi = i;
            break;
        }
    if (qi < 0) return KWOK_OK;
    const int k = e->queue[qi];
    const int next = qi + 1 < e->nq ? e->queue[qi + 1] : -1;  // a tick queued behind this one
    kwok_engine::TickSlot& T = e->slots[k];
    T.state = SLOT_DONE;
    T.rc = KWOK_OK;
    // every failure here leaves the device state (advanced by the kernels) and the
    // host mirrors / the caller's view out of step: the engine is poisoned, and a
    // tick queued behind this one (it ran on that state) fails with it
    auto failed = [&](int rc) {
        T.rc = rc;
        T.err = e->err;
        e->poisoned = true;
        if (next >= 0 && e->slots[next].state == SLOT_QUEUED) {
            kwok_engine::TickSlot& U = e->slots[next];
            (void)hipStreamSynchronize(e->st);
            U.state = SLOT_DONE;
            U.rc = rc;
            U.err = e->err;
        }
        return rc;
    };
    const auto t1 = clk::now();
    if (e->sync_spin) {
        // spin on the tick's completion event: a blocking wait sleeps and pays the
        // wake-up latency on every tick
        hipError_t q;
        while ((q = hipEventQuery(T.done)) == hipErrorNotReady) {
        }
        if (q != hipSuccess) return failed(e->fail(KWOK_EDEVICE, "tick: %s", hipGetErrorString(q)));
    } else if (hipEventSynchronize(T.done) != hipSuccess) {
        return failed(e->fail(KWOK_EDEVICE, "tick event sync"));
    }
    if (e->multi && T.hdr_h->xovf) {
        int rc = finish_long_lists(e, k, next);
        if (rc) return failed(rc);
    }
    if (e->multi && T.hdr_h->xforeign) e->global_foreign = true;  // (the BACK launch that ran to the end)
    bool requeue_next = false;
    if (T.once && T.hdr_h->redo) {
        if (int rc = redo_tick(e, k)) return failed(rc);
        requeue_next = next >= 0 && e->slots[next].state == SLOT_QUEUED;
    }
    const auto t2 = clk::now();
    if (!e->multi) derive_header(*T.hdr_h, T.arena_cap, e->hb_stride, e->S.hb_once != 0);
    const TickHdr& H = *T.hdr_h;
    if (!H.err && (H.n_pp || H.n_init) && !T.emit_queued) {
        // jobs nobody expected (no events since the previous tick): their bytes now
        int rc = bind_slot(e, k);
        if (!rc) rc = enqueue_emit(e, k);
        if (rc) return failed(rc);
        if (hipEventRecord(T.done, e->st) != hipSuccess || hipEventSynchronize(T.done) != hipSuccess)
            return failed(e->fail(KWOK_EDEVICE, "k_emit"));
    }
    if (trace_enabled(e)) trace_tick(e);
    if (e->S.jtrace && H.n_pp) jobs_trace_dump(e);
    if (H.err) {
        const uint32_t err = H.err;
        // a tick queued behind a failed one ran on its state: fail it as well
        (void)hipStreamSynchronize(e->st);
        (void)hipMemsetAsync(e->S.bar, 0, sizeof(GridBar), e->st);  // the next tick starts from a clean count
        (void)hipStreamSynchronize(e->st);
        e->front_launches = 0;
        int rc = (err & TICK_ERR_BARRIER)
                     ? e->fail(KWOK_EDEVICE, "k_tick cross-block wait timed out (%u chain blocks not co-resident?)",
                               e->S.n_chain)
                 : (err & TICK_ERR_SEQ)
                     ? e->fail(KWOK_ECOMM, "ranks out of step: the gathered exchange messages are of different ticks")
                 : (err & TICK_ERR_EMIT)
                     ? e->fail(KWOK_EDEVICE, "k_pod_jobs: a pod spec without unit tables in a fused emission")
                     : e->fail(KWOK_EDEVICE, "k_tick: device heartbeat count differs from the host's (%llu)",
                               (unsigned long long)e->n_managed);
        e->poisoned = true;
        if (next >= 0) {
            kwok_engine::TickSlot& U = e->slots[next];
            U.state = SLOT_DONE;
            U.rc = rc;
            U.err = e->err;
        }
        return failed(rc);
    }
    if (e->prof) {
        // kernel time from the launch events; the phase split from the kernel's
        // s_memrealtime stamps (100 MHz)
        float k0 = 0, k1 = 0;
        (void)hipEventElapsedTime(&k0, T.pev[0], T.pev[1]);
        if (e->multi) (void)hipEventElapsedTime(&k1, T.pev[2], T.pev[3]);
        float k2 = 0;
        if (T.emit_queued && !T.inits_folded) (void)hipEventElapsedTime(&k2, T.pev[4], T.pev[5]);
        float k3 = 0;
        if (T.split) (void)hipEventElapsedTime(&k3, T.pev[6], T.pev[7]);
        const double kern = (double)k0 + k1 + k2 + k3;
        // the streamers' latest exit, kept on the device (they never touch the header)
        unsigned long long send = 0;
        (void)release_for_host(e);
        (void)hipMemcpyAsync(&send, &e->S.bar->stream_end_max, 8, hipMemcpyDeviceToHost, e->st);
        (void)hipMemsetAsync(&e->S.bar->stream_end_max, 0, 8, e->st);
        (void)hipStreamSynchronize(e->st);
        T.hdr_h->clk[CLK_STREAM_END] = send;
        auto span = [&](int a, int b) { return H.clk[b] > H.clk[a] ? (double)(H.clk[b] - H.clk[a]) * 1e-5 : 0.0; };
        const double classify = span(CLK_ENTRY_MIN, CLK_P1_MAX), stream = span(CLK_ENTRY_MIN, CLK_STREAM_END);
        const double header = span(CLK_P1_MAX, CLK_HDR), pool = span(CLK_BACK, CLK_POOL);
        e->prof_ms[KWOK_T_CLASSIFY] += classify;
        e->prof_ms[KWOK_T_STREAM] += stream;
        e->prof_ms[KWOK_T_HEADER] += header;
        e->prof_ms[KWOK_T_EXCHANGE] += e->multi ? span(CLK_HDR, CLK_BACK) : 0.0;
        e->prof_ms[KWOK_T_POOL] += pool;
        // what follows the header in the chain (pool, job lists) beyond the stream, and k_emit
        e->prof_ms[KWOK_T_EMIT] += std::max(0.0, k0 + k1 - std::max(classify + header + pool, stream)) + k2 + k3;
        e->prof_ms[KWOK_T_KERNEL] += kern;
        e->prof_ms[KWOK_T_EMIT_KERNEL] += k2 + k3;  // k_emit and k_pod_jobs (split ticks)
        e->prof_ticks++;
    }
    if (H.overflow) return failed(e->fail(KWOK_ENOMEM, "output arena overflow (%llu bytes)", (unsigned long long)H.arena_bytes));
    // deleted nodes (and placeholders) whose last pod this tick deleted: their
    // entries go (k_free_zombies, queued on the engine stream: a tick already
    // queued behind this one reads no such node; every ingest follows it)
    if (H.n_del) {
        e->sum_valid = false;
        launch_free_zombies(e->S, e->st);
        if (hipGetLastError() != hipSuccess) return failed(e->fail(KWOK_EDEVICE, "k_free_zombies"));
    }
    kwok_tick_result& r = T.res;
    memset(&r, 0, sizeof(r));
    r.n_heartbeat = H.n_hb;
    r.heartbeat_len = e->hb_len;
    r.heartbeat_stride = e->S.hb_once ? 0 : e->hb_stride;
    r.n_node_init = H.n_init;
    r.n_pod_patch = H.n_pp;
    r.n_delete = H.n_del;
    r.heartbeat_epoch = T.epoch;
    r.arena_bytes = H.arena_bytes;
    for (int c = 0; c < KWOK_COUNTER_COUNT; c++) {
        r.counters[c] = H.counters[c];
        r.local_counters[c] = H.local_counters[c];
    }
    const auto t3 = clk::now();
    if (e->iprof && (H.n_pp || H.n_del || H.n_init))
        fprintf(stderr, "[kwok retire] wait %.3f ms, post %.3f ms\n", ms_between(t1, t2), ms_between(t2, t3));
    e->host_ms[KWOK_H_WAIT] += ms_between(t1, t2);
    e->host_ms[KWOK_H_POST] += ms_between(t2, t3);
    e->host_ms[KWOK_H_TOTAL] += ms_between(t1, t3);
    e->host_ticks++;
    e->stats[T.once ? KWOK_STAT_TICKS_ONCE : KWOK_STAT_TICKS_FULL]++;
    if (T.once && T.once_use) e->stats[KWOK_STAT_ONCE_SUMMARY]++;  // (a launch that skipped or was redone read none)
    if (requeue_next) {  // the tick queued behind a redone one skipped on the device
        if (int rc = enqueue_tick(e, next, true)) {
            kwok_engine::TickSlot& U = e->slots[next];
            U.state = SLOT_DONE;
            U.rc = rc;
            U.err = e->err;
            e->poisoned = true;
        }
    }
    return KWOK_OK;
}


// every queued tick finished on the host (before anything that reads or changes
// the host mirrors or device state outside the tick stream)
int drain(kwok_engine* e) {
    for (int i = 0; i < e->nq; i++)
        if (e->slots[e->queue[i]].state == SLOT_QUEUED) retire(e);  // per-tick failures stay in the slots
    return KWOK_OK;
}
}  // namespace

namespace {
// what kwok_tick_submit checks before it queues anything
int tick_submit_check(kwok_engine* e, int64_t now_unix) {
    if (now_unix < 0 || now_unix > 0xFFFFFFFFll) return e->fail(KWOK_EDOMAIN, "now out of range");
    if (e->nq >= 2) return e->fail(KWOK_EBUSY, "two ticks outstanding: collect one first");
    if (e->nq >= 1 && (e->prof || trace_enabled(e)))
        return e->fail(KWOK_EBUSY, "profiled / traced ticks are not queued behind each other");
    return KWOK_OK;
}
}  // namespace

extern "C" int kwok_tick_submit(kwok_engine* e, int64_t now_unix) {
    if (!e) return KWOK_EINVAL;
    if (e->poisoned) return poisoned(e);
    if (int rc = tick_submit_check(e, now_unix)) return rc;
    return tick_submit_impl(e, now_unix);
}

namespace {
// kwok_tick_submit after its checks (kwok_ingest_pods_packed12_tick queues it
// behind the batch's apply passes)
int tick_submit_impl(kwok_engine* e, int64_t now_unix) {
    const auto t0 = clk::now();
    // multi rank: the previous tick is finished (its long-list allgather, if any,
    // included) before this one's collectives are enqueued, so every rank issues
    // its collectives in the same order whatever its submit / collect pattern
    if (e->multi) drain(e);
    if (e->poisoned) return poisoned(e);  // the drained tick failed (its error stays collectable)
    const auto t_drained = clk::now();
    int k = -1;
    for (int pass = 0; pass < 2 && k < 0; pass++)  // prefer keeping the last collected tick's outputs
        for (int i = 0; i < 2 && k < 0; i++)
            if (e->slots[i].alloc && e->slots[i].state == SLOT_FREE && (pass == 1 || i != e->cur)) k = i;
    if (k < 0) {
        int rc = alloc_slot(e, 1);
        if (rc) return rc;
        k = 1;
    }
    kwok_engine::TickSlot& T = e->slots[k];
    int rc = grow_arena(e, T);
    if (rc) return rc;
    if (T.rd_pending) {  // the tick's kernels write the arena after the reads queued from it
        HIPCHK(e, hipStreamWaitEvent(e->st, T.rd, 0));
        T.rd_pending = false;
    }
    if (k == e->cur) e->cur = -1;  // its outputs are overwritten
    T.now = (uint64_t)now_unix;
    T.epoch = e->hb_epoch;
    T.emit_queued = e->emit_hint;
    e->emit_hint = false;
    // multi rank: every rank's pods hold the addresses the global pool gave them
    // unless some rank ever took a foreign one - its flag travels in the exchange
    // message; a rank that became foreign since the last exchange cannot make a
    // Use of this tick a change (its Puts come after the Uses, its ingest-time
    // releases reach the others through kwok_pool_put, which marks them foreign)
    T.quiet = e->quiet_ok && (e->multi ? !e->foreign_ips && !e->global_foreign : (e->quiet >= 2 || !e->foreign_ips));
    if (e->quiet < 0xFFFFFFFFu) e->quiet++;
    rc = enqueue_tick(e, k, false);
    if (rc) return rc;
    T.state = SLOT_QUEUED;
    e->queue[e->nq++] = k;
    if (e->iprof)
        fprintf(stderr, "[kwok submit] enqueue %.3f ms (drain %.3f)\n", ms_between(t0, clk::now()), ms_between(t0, t_drained));
    e->host_ms[KWOK_H_ENQUEUE] += ms_between(t0, clk::now());
    e->host_ms[KWOK_H_TOTAL] += ms_between(t0, clk::now());
    return KWOK_OK;
}
}  // namespace

extern "C" int kwok_engine_stats(const kwok_engine* e, uint64_t out[KWOK_STAT_COUNT]) {
    if (!e || !out) return KWOK_EINVAL;
    for (int i = 0; i < KWOK_STAT_COUNT; i++) out[i] = e->stats[i];
    return KWOK_OK;
}

extern "C" int kwok_tick_collect(kwok_engine* e, kwok_tick_result* res) {
    if (!e) return KWOK_EINVAL;
    if (e->nq == 0) return e->fail(KWOK_EINVAL, "no tick submitted");
    const int k = e->queue[0];
    kwok_engine::TickSlot& T = e->slots[k];
    if (T.state == SLOT_QUEUED) retire(e);
    e->queue[0] = e->queue[1];
    e->queue[1] = -1;
    e->nq--;
    T.state = SLOT_FREE;
    if (T.rc) {
        e->err = T.err;
        return T.rc;
    }
    e->cur = k;
    if (res) *res = T.res;
    return KWOK_OK;
}

extern "C" int kwok_tick(kwok_engine* e, int64_t now_unix, kwok_tick_result* res) {
    if (!e) return KWOK_EINVAL;
    if (e->nq) return e->fail(KWOK_EBUSY, "ticks outstanding: kwok_tick_collect them first");
    int rc = kwok_tick_submit(e, now_unix);
    return rc ? rc : kwok_tick_collect(e, res);
}

int kwok_read_outputs(kwok_engine* e, kwok_outputs* o) {
    if (!e || !o) return KWOK_EINVAL;
    if (e->poisoned) return poisoned(e);
    if (e->cur < 0) return e->fail(KWOK_EINVAL, "no collected tick (or its slot was reused by a submit)");
    const kwok_engine::TickSlot& S = e->slots[e->cur];  // outputs of the last collected tick
    const TickHdr& H = *S.hdr_h;
    // the copies run on their own stream once the tick is done, so they overlap a
    // tick already queued behind it (kwok_tick_submit before kwok_read_outputs);
    // the fence event there writes the kernels' L2 lines back for the copy engine
    hipStream_t st = e->rst;
    HIPCHK(e, hipStreamWaitEvent(st, S.done, 0));
    HIPCHK(e, hipEventRecord(e->fence, st));
    auto cp = [&](void* dst, const void* src, size_t bytes) -> hipError_t {
        if (!dst || !bytes) return hipSuccess;
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st);
    };
    o->heartbeat_off = H.hb_base;
    HIPCHK(e, cp(o->heartbeat_nodes, S.hb_nodes, (size_t)H.n_hb * 4));
    HIPCHK(e, cp(o->node_init_nodes, S.init_nodes, (size_t)H.n_init * 4));
    HIPCHK(e, cp(o->node_init_off, S.init_off, (size_t)H.n_init * 8));
    HIPCHK(e, cp(o->node_init_len, S.init_len, (size_t)H.n_init * 4));
    HIPCHK(e, cp(o->pod_patch_pods, S.pp_pods, (size_t)H.n_pp * 4));
    HIPCHK(e, cp(o->pod_patch_off, S.pp_off, (size_t)H.n_pp * 8));
    HIPCHK(e, cp(o->pod_patch_len, S.pp_len, (size_t)H.n_pp * 4));
    HIPCHK(e, cp(o->delete_pods, S.del_pods, (size_t)H.n_del * 4));
    HIPCHK(e, cp(o->delete_has_finalizers, S.del_fin, (size_t)H.n_del));
    o->arena_shift = 0;
    o->arena_copied = 0;
    if (o->arena) {
        if (o->flags & KWOK_READ_HEARTBEAT_ONCE) {
            // one heartbeat body, then the node-init / pod patch region (init_base..)
            const uint64_t hb = H.n_hb ? (uint64_t)e->hb_stride : 0, patches = H.arena_bytes - H.init_base;
            if (o->arena_cap < hb + patches)
                return e->fail(KWOK_EINVAL, "arena_cap < %llu", (unsigned long long)(hb + patches));
            HIPCHK(e, cp(o->arena, S.arena, hb));
            HIPCHK(e, cp(o->arena + hb, S.arena + H.init_base, patches));
            o->arena_shift = H.init_base - hb;
            o->arena_copied = hb + patches;
        } else {
            if (o->arena_cap < H.arena_bytes)
                return e->fail(KWOK_EINVAL, "arena_cap < %llu", (unsigned long long)H.arena_bytes);
            HIPCHK(e, cp(o->arena, S.arena, H.arena_bytes));
            o->arena_copied = H.arena_bytes;
        }
    }
    HIPCHK(e, hipStreamSynchronize(st));
    return KWOK_OK;
}

// Page-locked batch buffers: 2 MiB-aligned anonymous memory on transparent huge
// pages where the kernel grants them, registered (and mapped) with the runtime
// (the GPU walks 512x fewer page translations than over 4 KiB pages);
// KWOK_HOST_ALLOC=hip: hipHostMalloc instead.  Both are in the registry, with
// their device addresses: kwok_ingest_pods reads a batch in such a buffer in
// place (host_mapped).
void* kwok_host_alloc(size_t bytes) {
    bytes = bytes ? bytes : 1;
    const char* how = getenv("KWOK_HOST_ALLOC");
    if (!(how && strcmp(how, "hip") == 0)) {
        const size_t huge = (size_t)2 << 20, len = (bytes + huge - 1) & ~(huge - 1);
        void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p != MAP_FAILED) {
            const char* thp = getenv("KWOK_HOST_THP");
            if (!(thp && thp[0] == '0')) (void)madvise(p, len, MADV_HUGEPAGE);
            memset(p, 0, len);  // first touch: the pages exist (huge where granted) before pinning
            if (hipHostRegister(p, len, hipHostRegisterMapped) == hipSuccess) {
                void* dev = nullptr;
                if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess) dev = nullptr;
                std::lock_guard<std::mutex> l(g_host_mu);
                g_host_reg[(uintptr_t)p] = HostReg{len, (uint8_t*)dev, true};
                return p;
            }
            munmap(p, len);
        }
    }
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) return nullptr;
    void* dev = nullptr;
    if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess) dev = nullptr;
    std::lock_guard<std::mutex> l(g_host_mu);
    g_host_reg[(uintptr_t)p] = HostReg{bytes, (uint8_t*)dev, false};
    return p;
}

void kwok_host_free(void* p) {
    if (!p) return;
    HostReg r{0, nullptr, false};
    bool found = false;
    {
        std::lock_guard<std::mutex> l(g_host_mu);
        auto it = g_host_reg.find((uintptr_t)p);
        if (it != g_host_reg.end()) r = it->second, found = true, g_host_reg.erase(it);
    }
    if (found && r.mmapped) {
        (void)hipHostUnregister(p);
        munmap(p, r.len);
    } else {
        (void)hipHostFree(p);
    }
}

// dst <- src (len bytes) on the read stream (after its fence), a large read in
// parts over the extra read streams, joined back on the read stream
int read_copy(kwok_engine* e, void* dst, const uint8_t* src, uint64_t len) {
    const int ns = len >= (16ull << 20) ? std::max(1, std::min(e->read_streams, 4)) : 1;
    if (ns > 1) {
        if (!e->rd_go) HIPCHK(e, hipEventCreateWithFlags(&e->rd_go, hipEventDisableTiming));
        for (int i = 0; i < ns - 1; i++) {
            if (!e->rsx[i]) HIPCHK(e, hipStreamCreateWithFlags(&e->rsx[i], hipStreamNonBlocking));
            if (!e->rd_part[i]) HIPCHK(e, hipEventCreateWithFlags(&e->rd_part[i], hipEventDisableTiming));
        }
        HIPCHK(e, hipEventRecord(e->rd_go, e->rst));
    }
    const uint64_t step = ((len + ns - 1) / ns + 4095) & ~4095ull;
    for (int i = ns - 1; i >= 0; i--) {
        const uint64_t lo = std::min<uint64_t>(len, step * i), hi = std::min<uint64_t>(len, step * (i + 1));
        if (hi <= lo) continue;
        hipStream_t s = i ? e->rsx[i - 1] : e->rst;
        if (i) HIPCHK(e, hipStreamWaitEvent(s, e->rd_go, 0));
        HIPCHK(e, hipMemcpyAsync(static_cast<uint8_t*>(dst) + lo, src + lo, hi - lo, hipMemcpyDeviceToHost, s));
        if (i) {
            HIPCHK(e, hipEventRecord(e->rd_part[i - 1], s));
            HIPCHK(e, hipStreamWaitEvent(e->rst, e->rd_part[i - 1], 0));
        }
    }
    return KWOK_OK;
}

int kwok_read_arena(kwok_engine* e, uint64_t off, uint64_t len, void* dst) {
    if (!e || (len && !dst)) return KWOK_EINVAL;
    if (e->poisoned) return poisoned(e);
    if (e->cur < 0) return e->fail(KWOK_EINVAL, "no collected tick (or its slot was reused by a submit)");
    const kwok_engine::TickSlot& S = e->slots[e->cur];
    const uint64_t total = S.hdr_h->arena_bytes;
    if (off > total || len > total - off)
        return e->fail(KWOK_EINVAL, "arena range [%llu, +%llu) outside the tick's %llu bytes", (unsigned long long)off,
                       (unsigned long long)len, (unsigned long long)total);
    if (!len) return KWOK_OK;
    hipStream_t st = e->rst;  // beside a tick queued behind the collected one (as kwok_read_outputs)
    HIPCHK(e, hipStreamWaitEvent(st, S.done, 0));
    HIPCHK(e, hipEventRecord(e->fence, st));
    if (int rc = read_copy(e, dst, S.arena + off, len)) return rc;
    HIPCHK(e, hipStreamSynchronize(st));
    return KWOK_OK;
}

// kwok_read_arena queued without waiting: dst should be kwok_host_alloc memory (the
// copy engine writes it while the caller goes on: the next batch's ingest, the
// next tick); kwok_read_wait waits for every read queued so far.  The slot stays
// the caller's until the next submit that takes it, which waits for the reads on
// the device (or, when the arena must grow, on the host)
int kwok_read_arena_async(kwok_engine* e, uint64_t off, uint64_t len, void* dst) {
    if (!e || (len && !dst)) return KWOK_EINVAL;
    if (e->poisoned) return poisoned(e);
    if (e->cur < 0) return e->fail(KWOK_EINVAL, "no collected tick (or its slot was reused by a submit)");
    kwok_engine::TickSlot& S = e->slots[e->cur];
    const uint64_t total = S.hdr_h->arena_bytes;
    if (off > total || len > total - off)
        return e->fail(KWOK_EINVAL, "arena range [%llu, +%llu) outside the tick's %llu bytes", (unsigned long long)off,
                       (unsigned long long)len, (unsigned long long)total);
    if (!len) return KWOK_OK;
    hipStream_t st = e->rst;
    if (!S.rd && hipEventCreateWithFlags(&S.rd, hipEventDisableTiming) != hipSuccess)
        return e->fail(KWOK_EDEVICE, "event create");
    HIPCHK(e, hipStreamWaitEvent(st, S.done, 0));
    HIPCHK(e, hipEventRecord(e->fence, st));
    if (int rc = read_copy(e, dst, S.arena + off, len)) return rc;
    HIPCHK(e, hipEventRecord(S.rd, st));
    S.rd_pending = true;
    return KWOK_OK;
}

int kwok_read_wait(kwok_engine* e) {
    if (!e) return KWOK_EINVAL;
    HIPCHK(e, hipStreamSynchronize(e->rst));
    for (auto& T : e->slots) T.rd_pending = false;
    return KWOK_OK;
}

int kwok_device_outputs(kwok_engine* e, kwok_device_view* v) {
    if (!e || !v) return KWOK_EINVAL;
    if (e->cur < 0) return e->fail(KWOK_EINVAL, "no collected tick (or its slot was reused by a submit)");
    const kwok_engine::TickSlot& T = e->slots[e->cur];
    v->arena = T.arena;
    v->heartbeat_nodes = T.hb_nodes;
    v->pod_patch_pods = T.pp_pods;
    v->pod_patch_off = T.pp_off;
    v->pod_patch_len = T.pp_len;
    v->stream = e->st;
    return KWOK_OK;
}

int kwok_profile_enable(kwok_engine* e, int on) {
    if (!e) return KWOK_EINVAL;
    drain(e);
    for (auto& T : e->slots)
        for (auto& ev : T.pev)
            if (T.alloc && !ev) HIPCHK(e, hipEventCreate(&ev));
    e->prof = on != 0;
    memset(e->prof_ms, 0, sizeof e->prof_ms);
    e->prof_ticks = 0;
    return KWOK_OK;
}

int kwok_profile_read(kwok_engine* e, double ms_sum[KWOK_T_COUNT], uint64_t* ticks) {
    if (!e) return KWOK_EINVAL;
    if (ms_sum) memcpy(ms_sum, e->prof_ms, sizeof e->prof_ms);
    if (ticks) *ticks = e->prof_ticks;
    return KWOK_OK;
}

int kwok_profile_host(kwok_engine* e, int reset, double ms_sum[KWOK_H_COUNT], uint64_t* ticks) {
    if (!e) return KWOK_EINVAL;
    if (ms_sum) memcpy(ms_sum, e->host_ms, sizeof e->host_ms);
    if (ticks) *ticks = e->host_ticks;
    if (reset) {
        memset(e->host_ms, 0, sizeof e->host_ms);
        e->host_ticks = 0;
    }
    return KWOK_OK;
}

int kwok_node_has(kwok_engine* e, const char* name, size_t len) {
    // nodesSets.Has (node_controller.go:140-143): the device directory's entry is managed
    if (!e || !name || !len || len > NODE_NAME_MAX || e->poisoned) return 0;
    if (ensure_pinned(e, NAME_STRIDE + 64)) return 0;
    uint8_t* h = static_cast<uint8_t*>(e->pinned);
    uint8_t* d = static_cast<uint8_t*>(e->d_ops);
    memcpy(h, name, len);
    const uint32_t n32 = (uint32_t)len;
    memcpy(h + NAME_STRIDE, &n32, 4);
    uint32_t res = 0;
    if (hipMemcpyAsync(d, h, NAME_STRIDE + 4, hipMemcpyHostToDevice, e->st) != hipSuccess) return 0;
    launch_node_lookup(e->S, d, reinterpret_cast<const uint32_t*>(d + NAME_STRIDE), 1,
                       reinterpret_cast<uint32_t*>(d + NAME_STRIDE + 16), e->st);
    if (hipGetLastError() != hipSuccess || release_for_host(e) ||
        hipMemcpyAsync(h + NAME_STRIDE + 16, d + NAME_STRIDE + 16, 4, hipMemcpyDeviceToHost, e->st) != hipSuccess ||
        hipStreamSynchronize(e->st) != hipSuccess)
        return 0;
    memcpy(&res, h + NAME_STRIDE + 16, 4);
    return (res & NS_MANAGED) != 0;
}

uint64_t kwok_node_size(kwok_engine* e) { return e ? e->n_managed : 0; }

int kwok_dump_pods(kwok_engine* e, int32_t first, uint32_t count, uint8_t* used, uint8_t* phase, uint32_t* host_ip,
                   uint32_t* pod_ip) {
    if (!e) return KWOK_EINVAL;
    if (e->poisoned) return poisoned(e);
    drain(e);
    // through the engine's page-locked dump buffer: a device-to-host copy into
    // pageable memory made later copies of the ingest path stall (measured: every
    // other 2M-record churn batch paid 6-20 ms before its first device operation)
    const size_t PL = e->PL, need = PL * 10;
    if (need > e->dump_cap) {
        if (e->dump_h) (void)hipHostFree(e->dump_h);
        e->dump_h = nullptr;
        e->dump_cap = 0;
        if (hipHostMalloc((void**)&e->dump_h, need, hipHostMallocDefault) != hipSuccess)
            return e->fail(KWOK_ENOMEM, "dump buffer %zu", need);
        e->dump_cap = need;
    }
    uint32_t* hh = reinterpret_cast<uint32_t*>(e->dump_h);
    uint32_t* ph = hh + PL;
    const uint16_t* sth = reinterpret_cast<const uint16_t*>(ph + PL);
    if (int rc = release_for_host(e)) return rc;
    HIPCHK(e, hipMemcpyAsync((void*)sth, e->S.pod_state, PL * 2, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipMemcpyAsync(hh, e->S.host_ip, PL * 4, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipMemcpyAsync(ph, e->S.pod_ip, PL * 4, hipMemcpyDeviceToHost, e->st));
    HIPCHK(e, hipStreamSynchronize(e->st));
    for (uint32_t i = 0; i < count; i++) {
        uint32_t l = 0;
        bool ok = e->pod_slot((int64_t)first + i, &l) == KWOK_OK && (sth[l] & PS_USED);
        if (used) used[i] = ok;
        if (phase) phase[i] = ok ? (uint8_t)((sth[(size_t)l] & PS_PHASE_MASK) >> PS_PHASE_SHIFT) : 0;
        if (host_ip) host_ip[i] = ok && (sth[(size_t)l] & PS_HAS_HOST_IP) ? hh[(size_t)l] : 0;
        if (pod_ip) pod_ip[i] = ok ? ph[(size_t)l] : 0;
    }
    return KWOK_OK;
}

}  // extern "C"
