/*
 * kwok_engine.h - C-ABI of the MI355X-native kwok fake-kubelet tick engine.
 *
 * This is the drop-in boundary for the per-tick work of the reference's
 * pkg/kwok/controllers package (hezhizhen/kwok).  The Go side keeps the
 * reference's API (Config, NewController, NodeController, PodController,
 * watch/list/patch plumbing via client-go) and, instead of rendering templates
 * and evaluating strategic-merge predicates per object, pushes decoded watch
 * events into this library in batches and applies the patches/deletes it
 * returns.  No torch or C++ types appear here: plain integers, pointers and
 * sizes only (cgo / ctypes / JNI friendly).  See INTEGRATION.md for the cgo
 * binding and DESIGN.md for the tick contract.
 *
 * Entry point -> reference interface it replaces (paths relative to the
 * reference repo root):
 *   kwok_engine_create       controllers.NewController       pkg/kwok/controllers/controller.go:80-152
 *                            (NewNodeController node_controller.go:79-117,
 *                             NewPodController pod_controller.go:84-128,
 *                             parseCIDR/newIPPool utils.go:28-35,68)
 *   kwok_ingest_nodes        NodeController.WatchNodes/ListNodes event switch
 *                                                            node_controller.go:256-270,286-295
 *   kwok_ingest_pods         PodController.WatchPods/ListPods event switch
 *                                                            pod_controller.go:301-343,361-367
 *   kwok_register_pod_spec   (spec part of the pod JSON document renderToJSON
 *                             feeds to pod.status.tpl)      renderer.go:65-75
 *   kwok_tick                one heartbeat interval: KeepNodeHeartbeat +
 *                            LockNodes/LockNode/configureNode + LockPodsOnNode +
 *                            LockPods/LockPod/configurePod/computePatchData +
 *                            DeletePods/DeletePod + ipPool Get/Put/Use
 *                                                            node_controller.go:145-204,301-401
 *                                                            pod_controller.go:155-250,371-439
 *                                                            utils.go:83-117
 *   kwok_read_outputs        the PatchStatus / Patch / Delete request bodies
 *                                                            node_controller.go:152,345;
 *                                                            pod_controller.go:162,172,221
 *   kwok_node_has / _size    NodeController.Has / Size        node_controller.go:403-409
 *   kwok_pool_put            ipPool.Put (replicating an ingest-time release
 *                            to the other ranks' pool replicas) utils.go:100-108
 *   kwok_cni_pending /       EnableCNI: the pods configurePod would call cni.Setup
 *   kwok_cni_assign          for, and the IPs it returned    pod_controller.go:383-389
 */
#ifndef KWOK_ENGINE_H
#define KWOK_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KWOK_ABI_VERSION 5u
#define KWOK_COMM_ID_BYTES 128u

/* ---- status codes (int return values; per-record codes in out_status) ---- */
enum {
    KWOK_OK = 0,
    KWOK_EINVAL = -1,     /* bad argument / config */
    KWOK_ENOMEM = -2,     /* host or device allocation failed */
    KWOK_EDOMAIN = -3,    /* input outside the supported domain (e.g. not a "safe string",
                             IPv6, custom templates) - rejected, never emulated */
    KWOK_EFULL = -4,      /* bucket slot capacity exhausted */
    KWOK_EDEVICE = -5,    /* HIP runtime error */
    KWOK_ECOMM = -6,      /* RCCL / exchange error */
    KWOK_ENOTFOUND = -7,  /* unknown handle */
    KWOK_ENOTMINE = -8,   /* object hashes to a bucket owned by another rank (not an error
                             for a sharded caller: route it to the owning rank) */
    KWOK_EBUSY = -9       /* ticks outstanding (kwok_tick_submit / kwok_tick_collect order) */
};

enum { KWOK_OP_UPSERT = 1 /* watch.Added / watch.Modified / list item */, KWOK_OP_DELETE = 2 /* watch.Deleted */ };

/* corev1 PodPhase / NodePhase as far as the templates and predicates care */
enum {
    KWOK_PHASE_NONE = 0, KWOK_PHASE_PENDING = 1, KWOK_PHASE_RUNNING = 2,
    KWOK_PHASE_SUCCEEDED = 3, KWOK_PHASE_FAILED = 4, KWOK_PHASE_UNKNOWN = 5,
    KWOK_PHASE_OTHER = 6 /* any other node phase, e.g. "Terminated" */
};

/* pod event flags */
enum {
    KWOK_POD_DISREGARD = 1u << 0,       /* disregardStatusWith{Annotation,Label}Selector matched
                                           (pod_controller.go:257-267) */
    KWOK_POD_DELETING = 1u << 1,        /* metadata.deletionTimestamp != nil (:306) */
    KWOK_POD_STATUS_NONEMPTY = 1u << 2, /* json(pod.status) is a non-empty map: the
                                           `{{ with .status }}` guard of pod.status.tpl:44 */
    KWOK_POD_CONFORMS = 1u << 3,        /* status.conditions / containerStatuses /
                                           initContainerStatuses / startTime already equal what
                                           pod.status.tpl renders (strategic-merge no-op for
                                           those fields, pod_controller.go:411-435) */
    KWOK_POD_HAS_FINALIZERS = 1u << 4   /* len(metadata.finalizers) != 0 (:161) */
};

/* byte range inside the caller's string arena passed with each batch */
typedef struct kwok_str {
    uint32_t off;
    uint32_t len;
} kwok_str;

/* status.nodeInfo fields in JSON key order (node.status.tpl:31-42) */
enum {
    KWOK_NI_ARCHITECTURE = 0, KWOK_NI_BOOT_ID, KWOK_NI_CONTAINER_RUNTIME_VERSION,
    KWOK_NI_KERNEL_VERSION, KWOK_NI_KUBE_PROXY_VERSION, KWOK_NI_KUBELET_VERSION,
    KWOK_NI_MACHINE_ID, KWOK_NI_OPERATING_SYSTEM, KWOK_NI_OS_IMAGE, KWOK_NI_SYSTEM_UUID,
    KWOK_NI_COUNT
};

typedef struct kwok_node_event {
    uint8_t op;        /* KWOK_OP_* */
    uint8_t managed;   /* needHeartbeat(node) = nodeSelectorFunc(node)  (node_controller.go:206) */
    uint8_t lockable;  /* needLockNode(node)                            (node_controller.go:210) */
    uint8_t phase;     /* status.phase: NONE, RUNNING or OTHER */
    kwok_str name;
    kwok_str addresses;   /* compact JSON of status.addresses   (len 0 = absent/empty) */
    kwok_str allocatable; /* compact JSON of status.allocatable (len 0 = absent/empty) */
    kwok_str capacity;    /* compact JSON of status.capacity    (len 0 = absent/empty) */
    kwok_str node_info[KWOK_NI_COUNT]; /* status.nodeInfo.* (len 0 = "") */
} kwok_node_event;

typedef struct kwok_pod_event {
    uint8_t op;        /* KWOK_OP_* */
    uint8_t phase;     /* status.phase */
    uint8_t flags;     /* KWOK_POD_* */
    uint8_t reserved0; /* 0; nonzero: the record's status (an int8 KWOK_E*), not applied (a failed GPU decode) */
    int32_t handle;    /* UPSERT of a new pod: -1; otherwise the handle returned at add */
    int32_t spec_id;   /* from kwok_register_pod_spec */
    int32_t node_handle; /* -1: resolve node_name */
    int64_t creation_unix; /* metadata.creationTimestamp (seconds, UTC) */
    kwok_str node_name;  /* spec.nodeName */
    kwok_str host_ip;    /* status.hostIP (dotted IPv4 or empty) */
    kwok_str pod_ip;     /* status.podIP  (dotted IPv4 or empty) */
} kwok_pod_event;

/* The compact wire form of a pod event (20 bytes, kwok_ingest_pods_packed):
 * the same event as kwok_pod_event with its strings already parsed - IPs as
 * IPv4 integers, the node as its handle - so a churn batch moves ~20 B per
 * record over the link instead of ~54 (a 48-byte record plus dotted quads).
 * A create names its node by handle only (a pod naming a node the engine does
 * not hold by handle goes through kwok_ingest_pods, by spec.nodeName). */
typedef struct kwok_pod_rec {
    uint8_t op;          /* KWOK_OP_UPSERT / KWOK_OP_DELETE, | KWOK_REC_NEW for a create */
    uint8_t flags;       /* KWOK_POD_* in bits 0-4, status.phase (KWOK_PHASE_*) in bits 5-7 */
    uint16_t spec_id;    /* UPSERT: from kwok_register_pod_spec */
    int32_t target;      /* the pod's handle; with KWOK_REC_NEW: the handle of its node */
    uint32_t creation;   /* metadata.creationTimestamp, unix seconds (UTC) */
    uint32_t host_ip;    /* status.hostIP as an IPv4 integer (0: empty) */
    uint32_t pod_ip;     /* status.podIP  as an IPv4 integer (0: empty) */
} kwok_pod_rec;
#define KWOK_REC_NEW 0x80u
#define KWOK_REC_PHASE_SHIFT 5

/* The 12-byte wire form (kwok_ingest_pods_packed12): kwok_pod_rec with one value
 * word instead of three.
 *   hostIP: configurePod renders status.hostIP as the pod's own or NodeIP
 *     (pod.status.tpl `hostIP: {{ with .hostIP }} {{ . }} {{ else }} {{ NodeIP }}`),
 *     so a pod kwok has run holds NodeIP and a new one none: KWOK_REC_HOST_NODE_IP
 *     in op says hostIP = the engine's node_ip, its absence an empty hostIP.
 *   creationTimestamp: immutable (metadata), so only a create carries it; an
 *     update or delete of a pod the engine holds keeps the one it was created with.
 * value = a create's creationTimestamp (unix seconds; the new pod holds no podIP),
 * any other record's status.podIP (0: empty).  A pod with another hostIP, or
 * created with a podIP, goes through kwok_ingest_pods_packed. */
typedef struct kwok_pod_rec12 {
    uint8_t op;          /* KWOK_OP_UPSERT / KWOK_OP_DELETE, | KWOK_REC_NEW, | KWOK_REC_HOST_NODE_IP */
    uint8_t flags;       /* as kwok_pod_rec */
    uint16_t spec_id;    /* as kwok_pod_rec */
    int32_t target;      /* as kwok_pod_rec */
    uint32_t value;      /* KWOK_REC_NEW: metadata.creationTimestamp; otherwise status.podIP */
} kwok_pod_rec12;
#define KWOK_REC_HOST_NODE_IP 0x40u

typedef struct kwok_container {
    kwok_str name;
    kwok_str image;
} kwok_container;

typedef struct kwok_pod_spec {
    const kwok_container* containers;      uint32_t n_containers;      /* spec.containers */
    const kwok_container* init_containers; uint32_t n_init_containers; /* spec.initContainers */
    const kwok_str* readiness_gates;       uint32_t n_readiness_gates; /* spec.readinessGates[].conditionType */
} kwok_pod_spec;

/* Allgather over host memory: every rank contributes `bytes` from `send`;
 * `recv` receives world_size * bytes, rank-major.  Return 0 on success. */
typedef int (*kwok_allgather_fn)(void* user, const void* send, size_t bytes, void* recv);

typedef struct kwok_config {
    uint32_t abi_version;          /* KWOK_ABI_VERSION */
    const char* cidr;              /* Config.CIDR,   e.g. "10.0.0.1/24" (controller.go:72) */
    const char* node_ip;           /* Config.NodeIP, e.g. "196.168.0.1" (controller.go:73) */
    int64_t start_time_unix;       /* the StartTime() template func (controller.go:39-41) */
    int32_t enable_cni;            /* Config.EnableCNI: pod IPs come from the caller's CNI plugin
                                      (kwok_cni_pending / kwok_cni_assign); the ipPool is unused */
    int32_t custom_templates;      /* bit mask: 0 = templates.Default*; KWOK_TPL_POD: pod_status_template
                                      below, KWOK_TPL_NODE_INIT: node_init_template, KWOK_TPL_HEARTBEAT:
                                      node_heartbeat_template */
    uint32_t buckets;              /* power of two; node -> bucket = fnv1a32(name) & (buckets-1) */
    uint32_t node_slots_per_bucket;
    uint32_t pod_slots_per_bucket; /* initial pod capacity of a bucket (multiple of 8); grows up to
                                      pod_handle_stride when a bucket fills */
    uint32_t max_pod_specs;
    int32_t rank;                  /* this engine owns buckets [rank*B/W, (rank+1)*B/W) */
    int32_t world_size;
    int32_t device;                /* HIP device ordinal (ignored by the CPU oracle) */
    const uint8_t* comm_id;        /* KWOK_COMM_ID_BYTES from kwok_comm_id(): RCCL exchange */
    kwok_allgather_fn allgather;   /* alternative host-memory exchange (used when comm_id == NULL) */
    void* allgather_user;
    uint32_t pod_handle_stride;    /* pod handle = bucket * pod_handle_stride + slot in the bucket:
                                      the most pods one bucket can hold (multiple of 8, <= 65528;
                                      0 = pod_slots_per_bucket, i.e. no growth).  Handles stay valid
                                      when a bucket's capacity grows (KWOK_EFULL only past it). */
    uint32_t flags;                /* KWOK_CFG_* */
    const char* pod_status_template; /* KWOK_TPL_POD: Config.PodStatusTemplate (controller.go:76),
                                        compiled per registered pod spec into the kernels' byte
                                        program; KWOK_EDOMAIN when its output does not fit that
                                        program (see kwok_pod_template_patch) */
    const char* node_init_template;  /* KWOK_TPL_NODE_INIT: Config.NodeInitializationTemplate
                                        (controller.go:75), compiled per distinct node status into
                                        the node's init blob (see kwok_node_template_patch) */
    const char* node_heartbeat_template; /* KWOK_TPL_HEARTBEAT: Config.NodeHeartbeatTemplate
                                        (controller.go:77): must render the same conditions list for
                                        every node, <= 1280 bytes (see kwok_heartbeat_template_patch) */
} kwok_config;
enum { KWOK_TPL_POD = 1, KWOK_TPL_NODE_INIT = 2, KWOK_TPL_HEARTBEAT = 4 };
/* kwok_config.flags */
enum {
    /* every heartbeat patch of a tick is the same body (node_controller.go:393-401):
       materialise ONE (at heartbeat_off; kwok_tick_result.heartbeat_stride = 0) with
       the full handle list, for callers that send one body to every node (the
       cgo drop-in does) - the tick then moves the SoA state, not n copies */
    KWOK_CFG_HEARTBEAT_ONCE = 1
};

/* fleet counters (kwok_tick_result.counters, summed over ranks) */
enum {
    KWOK_CNT_HEARTBEAT = 0,   /* heartbeat patches emitted this tick */
    KWOK_CNT_NODE_INIT,       /* node lock (initialisation) patches emitted */
    KWOK_CNT_POD_PATCH,       /* pod status patches emitted */
    KWOK_CNT_DELETE,          /* pods deleted (DeletePod) */
    KWOK_CNT_ALLOC,           /* ipPool.Get calls */
    KWOK_CNT_RELEASE,         /* ipPool.Put calls from this tick's deletions */
    KWOK_CNT_EVALUATED,       /* pods evaluated (LockPod) incl. no-ops */
    KWOK_CNT_LOCK_CHECKED,    /* nodes lock-checked (LockNode) incl. no-ops */
    KWOK_CNT_NODES_MANAGED,   /* NodeController.Size() after the tick */
    KWOK_CNT_NODES_READY,     /* managed nodes whose status is initialised */
    KWOK_CNT_PODS_TOTAL,
    KWOK_CNT_PODS_PENDING,
    KWOK_CNT_PODS_RUNNING,
    KWOK_COUNTER_COUNT
};

typedef struct kwok_tick_result {
    uint32_t n_heartbeat;       /* number of heartbeat patches (one per managed node) */
    uint32_t heartbeat_len;     /* bytes of every heartbeat patch (identical bodies) */
    uint64_t heartbeat_stride;  /* arena distance between consecutive heartbeat patches (0 with
                                   KWOK_CFG_HEARTBEAT_ONCE: one body for every handle) */
    uint32_t n_node_init;
    uint32_t n_pod_patch;
    uint32_t n_delete;
    uint32_t heartbeat_epoch;   /* changes whenever the heartbeat handle list changes (the
                                   managed set, node_controller.go:259-269); a caller that
                                   kept the list of an earlier tick with the same epoch
                                   need not read it again */
    uint64_t arena_bytes;       /* bytes of the output arena in use */
    uint64_t counters[KWOK_COUNTER_COUNT];       /* fleet-wide (all ranks) */
    uint64_t local_counters[KWOK_COUNTER_COUNT]; /* this rank */
} kwok_tick_result;

/* kwok_outputs.flags */
enum {
    /* the host arena receives ONE heartbeat body (all heartbeat patches of a tick
       are identical, node_controller.go:393-401) followed by the node-init / pod
       patch region: host offset = arena offset - arena_shift */
    KWOK_READ_HEARTBEAT_ONCE = 1u
};

/* Host buffers the caller provides to kwok_read_outputs (NULL = skip). */
typedef struct kwok_outputs {
    int32_t* heartbeat_nodes;       /* [n_heartbeat] node handles, canonical order */
    uint64_t heartbeat_off;         /* out: arena offset of heartbeat patch 0 */
    int32_t* node_init_nodes;       /* [n_node_init] */
    uint64_t* node_init_off;        /* [n_node_init] arena offsets */
    uint32_t* node_init_len;        /* [n_node_init] */
    int32_t* pod_patch_pods;        /* [n_pod_patch] pod handles, canonical order */
    uint64_t* pod_patch_off;
    uint32_t* pod_patch_len;
    int32_t* delete_pods;           /* [n_delete] pod handles to Patch(finalizers)+Delete */
    uint8_t* delete_has_finalizers; /* [n_delete] 1 = send kwok_finalizer_patch() first */
    uint8_t* arena;                 /* [arena_cap] copy of the output arena */
    uint64_t arena_cap;
    uint32_t flags;                 /* KWOK_READ_* */
    uint32_t reserved0;
    uint64_t arena_shift;           /* out: node_init_off / pod_patch_off - arena_shift = the
                                       offset in the host arena (0 without HEARTBEAT_ONCE) */
    uint64_t arena_copied;          /* out: bytes written to the host arena */
} kwok_outputs;

typedef struct kwok_engine kwok_engine;

uint32_t kwok_abi_version(void);
int kwok_comm_id(uint8_t out[KWOK_COMM_ID_BYTES]);

int kwok_engine_create(const kwok_config* cfg, kwok_engine** out);
void kwok_engine_destroy(kwok_engine* e);
const char* kwok_last_error(const kwok_engine* e);

/* Register a pod spec (containers, init containers, readiness gates); identical
 * specs share one id.  Strings must be "safe"  or KWOK_EDOMAIN. */
int kwok_register_pod_spec(kwok_engine* e, const kwok_pod_spec* spec, const char* arena,
                           size_t arena_len, int32_t* out_id);

/* Ingest a batch of watch events in order.  out_handles[i] receives the node/pod
 * handle (canonical slot id), out_status[i] a per-record code (KWOK_OK,
 * KWOK_EDOMAIN, KWOK_EFULL, KWOK_ENOTFOUND, KWOK_ENOTMINE).  Returns the number of
 * rejected records (>= 0) or a negative error for the whole batch.  Both event
 * switches run on the GPU, in event order per bucket, over device-resident state
 * (the node directory of names and the pod slots); records and arena in
 * kwok_host_alloc memory are read in place, other buffers are copied first.
 * Nodes: only a non-empty status (its JSON blobs and nodeInfo strings) or a
 * custom node template takes host string work. */
int kwok_ingest_nodes(kwok_engine* e, const kwok_node_event* ev, size_t n, const char* arena,
                      size_t arena_len, int32_t* out_handles, int32_t* out_status);
/* out_released (optional) receives, per DELETE record, the IPv4 address released
 * into the pool (0 if none); sharded callers replicate these to the other ranks
 * with kwok_pool_put before the next tick.  A pod batch of more than
 * KWOK_INGEST_CHUNK records (environment, default 1048576) is applied in chunks
 * of consecutive records; a negative return after a chunk was applied poisons
 * the engine (the batch is partly in the state: every later call fails). */
int kwok_ingest_pods(kwok_engine* e, const kwok_pod_event* ev, size_t n, const char* arena,
                     size_t arena_len, int32_t* out_handles, int32_t* out_status,
                     uint32_t* out_released);
/* kwok_ingest_pods over the compact wire form: the same event switch, the same
 * per-record results (out_status as int8_t codes; out_released optional).  A
 * batch in kwok_host_alloc memory of up to KWOK_INGEST_CHUNK records is read in
 * place by the GPU. */
int kwok_ingest_pods_packed(kwok_engine* e, const kwok_pod_rec* recs, size_t n, int32_t* out_handles,
                            int8_t* out_status, uint32_t* out_released);
/* kwok_ingest_pods_packed over kwok_pod_rec12 records, returning the handles of
 * the creates only (every other record's handle is its target, which the caller
 * holds): out_new_handles[k] = the handle of the batch's k-th KWOK_REC_NEW record
 * (-1 when rejected; out_status says why), for k < new_cap.  new_cap must be at
 * least the number of KWOK_REC_NEW records: handles past it are not returned and
 * the call returns KWOK_EINVAL once the batch is applied (the engine stays
 * usable); entries past that number are undefined.  out_status (int8, per
 * record) and out_released as kwok_ingest_pods_packed.  Over the link: 12 bytes
 * per record in, 1 byte per record and 4 per create back (C4: 24 + 6 MB per 2M
 * records, against 40 + 10 MB for kwok_pod_rec). */
int kwok_ingest_pods_packed12(kwok_engine* e, const kwok_pod_rec12* recs, size_t n, int32_t* out_new_handles,
                              size_t new_cap, int8_t* out_status, uint32_t* out_released);
/* kwok_ingest_pods_packed12, then kwok_tick_submit(e, now_unix) queued right behind
 * the batch's apply passes (single-rank engines): the tick's kernels run while
 * the per-record results travel back, so a churn step (a batch, then a tick) does
 * not wait for the results and the call's return before its tick starts.
 * Returns as kwok_ingest_pods_packed12 once the results are in the caller's
 * arrays; the tick is then collected with kwok_tick_collect (it may still be
 * running).  The tick submit's own checks (now, two ticks outstanding, profiled
 * queues) are made before the batch is touched.  A chunk that needs more pod
 * slots than a bucket has makes the tick's launches skip on the device; the
 * call grows the buckets, applies the chunk and queues the tick again.
 * Equivalent to the two calls, record for record and tick for tick
 * (tests/test_c4_churn_gpu.py, tests/test_growth_gpu.py). */
int kwok_ingest_pods_packed12_tick(kwok_engine* e, const kwok_pod_rec12* recs, size_t n, int32_t* out_new_handles,
                                   size_t new_cap, int8_t* out_status, uint32_t* out_released, int64_t now_unix);
/* Host only: kwok_pod_event records (strings in `arena`) -> the compact form,
 * with the checks that need the strings (canonical dotted quads, creation time
 * range, spec id and phase bounds).  status[i] = KWOK_OK, KWOK_EDOMAIN (an IP,
 * a time outside the domain) or KWOK_EINVAL (a create naming its node by
 * spec.nodeName: not expressible, use kwok_ingest_pods); out[i] is valid only
 * for KWOK_OK.  Returns the number of records not packed. */
int kwok_pack_pod_events(const kwok_pod_event* ev, size_t n, const char* arena, size_t arena_len, kwok_pod_rec* out,
                         int32_t* status);
/* Page-locked host memory for ingest batches.  kwok_ingest_pods copies its
 * records, string arena and per-record results between host and GPU (the pod
 * event switch runs on the device); buffers from kwok_host_alloc move by DMA at
 * the link's rate, pageable ones through the runtime's staging copies (2-8x
 * slower for a 2M-record batch, and noisier).  A caller that decodes watch
 * events straight into such buffers (the codec's output, a cgo slice over C
 * memory) pays no extra host copy.  NULL on failure; kwok_host_free releases. */
void* kwok_host_alloc(size_t bytes);
void kwok_host_free(void* p);
int kwok_pool_put(kwok_engine* e, const uint32_t* ips, size_t n);

/* EnableCNI (kwok_config.enable_cni = 1).  The reference calls cni.Setup inside
 * configurePod for an evaluated pod without a podIP and renders the patch with
 * the IP it returns (pod_controller.go:383-389); a Deleted event calls
 * cni.Remove instead of ipPool.Put (:337-342).  With the engine:
 *   before a tick, kwok_cni_pending lists (canonical order) the pods that tick
 *   will evaluate that hold no podIP; the caller runs cni.Setup for each and
 *   hands the first IPs back with kwok_cni_assign; the tick then patches them
 *   with those IPs.  A pod still without an IP is not patched (as a failed
 *   cni.Setup).  The ipPool is never used: no Get, Use or Put; the caller runs
 *   cni.Remove on Deleted events (the engine's own deletions included).
 * kwok_cni_pending: *n_out = the number of pending pods; KWOK_EINVAL (n_out set)
 * when cap is smaller.  kwok_cni_assign: out_status[i] per record (KWOK_OK,
 * KWOK_ENOTFOUND, KWOK_ENOTMINE, KWOK_EDOMAIN for IP 0); returns the number of
 * rejected records or a negative error. */
int kwok_cni_pending(kwok_engine* e, int32_t* out, size_t cap, size_t* n_out);
int kwok_cni_assign(kwok_engine* e, const int32_t* handles, const uint32_t* ips, size_t n, int32_t* out_status);

/* Advance one heartbeat interval at fixed clock now_unix (the Now() template
 * func).  Blocks until the tick's outputs are ready.  = kwok_tick_submit +
 * kwok_tick_collect; KWOK_EBUSY while submitted ticks are not collected. */
int kwok_tick(kwok_engine* e, int64_t now_unix, kwok_tick_result* res);
/* The same tick in two halves, so that tick N+1 runs on the device while the
 * caller collects and consumes tick N (at most two ticks outstanding):
 *   kwok_tick_submit   enqueue the tick (returns without waiting).
 *   kwok_tick_collect  wait for the oldest submitted tick and return its result;
 *                      kwok_read_outputs / kwok_device_outputs then refer to it,
 *                      until the next kwok_tick_submit.
 * Results equal kwok_tick's for the same call sequence.  Ingest, spec
 * registration, kwok_pool_put and kwok_dump_pods first finish every submitted
 * tick on the host (their results stay collectable), so events apply after the
 * ticks submitted before them.
 * Multi rank (world_size > 1): every rank must tick the same sequence of ticks
 * (the exchange messages carry the tick's sequence number; ranks out of step
 * fail the tick with KWOK_ECOMM), and kwok_tick_submit first finishes the
 * previous tick on the host, so each rank issues its collectives in the same
 * order whatever its submit / collect pattern.
 * A failed tick (KWOK_EDEVICE / KWOK_ECOMM from collect) leaves the device
 * and host state out of step: every later call fails with KWOK_EDEVICE until the
 * engine is destroyed and recreated (state rebuilt from a List, as on restart). */
int kwok_tick_submit(kwok_engine* e, int64_t now_unix);
int kwok_tick_collect(kwok_engine* e, kwok_tick_result* res);
int kwok_read_outputs(kwok_engine* e, kwok_outputs* out);
/* Bytes [off, off + len) of the last collected tick's output arena (the arena
 * offsets kwok_read_outputs reports without KWOK_READ_HEARTBEAT_ONCE:
 * heartbeat_off, node_init_off[i], pod_patch_off[i]) copied into dst.  For
 * callers that read the patches in bounded pieces: the initial tick of a
 * 1M-node / 10M-pod fleet is ~7 GB of patches (a cgo caller must not size one
 * copy with a C int).  The patches lie in increasing offset order (node inits,
 * then pod patches, each in canonical order).  KWOK_EINVAL outside the arena. */
int kwok_read_arena(kwok_engine* e, uint64_t off, uint64_t len, void* dst);
/* kwok_read_arena queued on the engine's read stream without waiting (dst:
 * kwok_host_alloc memory, which the copy engine fills while the caller goes on -
 * the next batch's ingest and tick overlap the link's device-to-host direction);
 * kwok_read_wait waits for every read queued so far.  A later submit that takes
 * the read slot waits for its reads on the device.  (Stands in for the same
 * read sequence as kwok_read_arena: engine_cgo.go applyPatches, INTEGRATION.md.) */
int kwok_read_arena_async(kwok_engine* e, uint64_t off, uint64_t len, void* dst);
int kwok_read_wait(kwok_engine* e);

/* The constant merge patch sent before Delete when a pod has finalizers
 * (removeFinalizers, pod_controller.go:45). */
const char* kwok_finalizer_patch(size_t* len);

/* nodesSets.Has: the node of that name is in the managed set (a device lookup in
 * the node directory; waits for the engine stream). */
int kwok_node_has(kwok_engine* e, const char* name, size_t len);
uint64_t kwok_node_size(kwok_engine* e);

/* State dump for tests / checkpoint: pods with handles in [first, first+count). */
int kwok_dump_pods(kwok_engine* e, int32_t first, uint32_t count, uint8_t* used, uint8_t* phase,
                   uint32_t* host_ip, uint32_t* pod_ip);

/* Device-resident outputs of the last collected tick, for zero-copy consumers
 * (valid until the next kwok_tick_submit / kwok_tick). */
typedef struct kwok_device_view {
    const void* arena;
    const int32_t* heartbeat_nodes;
    const int32_t* pod_patch_pods;
    const uint64_t* pod_patch_off;
    const uint32_t* pod_patch_len;
    void* stream;                   /* hipStream_t the engine runs on */
} kwok_device_view;
int kwok_device_outputs(kwok_engine* e, kwok_device_view* view);

/* Diagnostics: device time per tick (enable resets the accumulators).
 * KERNEL is the tick kernel's launch duration(s) from HIP events; the phase
 * split comes from the kernel's own clock stamps: CLASSIFY = first chain block
 * start to the last chain block's arrival, STREAM = first chain block start to
 * the last heartbeat streamer's exit, HEADER = the last arriver's reduction and
 * header publication, EXCHANGE = between the two launches of a multi-rank tick
 * (allgather + pool apply), POOL = ipPool phase (ticks with Gets / Puts),
 * EMIT = the rest of the launch beyond the longer of chain and stream, plus the patch-byte
 * kernel; EMIT_KERNEL = the emission kernels alone (ticks with patches: k_emit, plus
 * k_pod_jobs on split ticks, which writes the pod patch bytes when fused). */
enum { KWOK_T_CLASSIFY = 0, KWOK_T_STREAM, KWOK_T_HEADER, KWOK_T_EXCHANGE, KWOK_T_POOL, KWOK_T_EMIT,
       KWOK_T_KERNEL, KWOK_T_EMIT_KERNEL /* the emission kernels (k_pod_jobs + k_emit) */, KWOK_T_COUNT };
int kwok_profile_enable(kwok_engine* e, int on);
int kwok_profile_read(kwok_engine* e, double ms_sum[KWOK_T_COUNT], uint64_t* ticks);
/* Host-side wall time of kwok_tick (always measured): enqueue,
 * waiting for the device, host bookkeeping after the wait, whole call. */
enum { KWOK_H_ENQUEUE = 0, KWOK_H_WAIT, KWOK_H_POST, KWOK_H_TOTAL, KWOK_H_COUNT };
int kwok_profile_host(kwok_engine* e, int reset, double ms_sum[KWOK_H_COUNT], uint64_t* ticks);
/* Which tick kernel ran (diagnostics, tests): heartbeat-once ticks expected to
 * have nothing to emit run a counting kernel (k_once); one that had work after
 * all runs again with the full tick kernel.  Counts since create. */
enum { KWOK_STAT_TICKS_FULL = 0 /* ticks run by the full tick kernel (redone ticks included) */,
       KWOK_STAT_TICKS_ONCE /* heartbeat-once ticks completed by the counting kernel */,
       KWOK_STAT_ONCE_REDO /* counting-kernel ticks that had work and ran again with the full kernel */,
       KWOK_STAT_ONCE_SUMMARY /* counting-kernel launches that read the per-bucket summaries, not the pod rows */,
       KWOK_STAT_COUNT };
int kwok_engine_stats(const kwok_engine* e, uint64_t out[KWOK_STAT_COUNT]);

/* Host only (no device): renderer.renderToJSON (renderer.go:49-89) - the
 * covered subset of Go text/template, then sigs.k8s.io/yaml.YAMLToJSON - of
 * template `tpl` over the JSON document `doc` (the object as json.Marshal gives
 * it), with template funcs given as a JSON object of strings ({"Now": "...",
 * "NodeIP": "...", ...}; YAML is built in).  This is the renderer custom pod
 * status templates are compiled with.  *out_len = the output length
 * (KWOK_EINVAL when cap is smaller); KWOK_EDOMAIN for a template, document or
 * YAML outside the covered subset, with the reason in kwok_template_last_error(). */
int kwok_template_render(const char* tpl, size_t tpl_len, const char* doc, size_t doc_len, const char* funcs,
                         size_t funcs_len, char* out, size_t cap, size_t* out_len);
const char* kwok_template_last_error(void);
/* Host only: a custom pod status template compiled for one pod spec (as
 * kwok_register_pod_spec does with custom_templates = 1), then assembled on the
 * host exactly as the kernels assemble it: the patch bytes of a pod with that
 * spec, creationTimestamp, hostIP (0: NodeIP), podIP and status emptiness.
 * KWOK_EDOMAIN (reason in kwok_template_last_error) when the template does not
 * compile to the kernels' program. */
int kwok_pod_template_patch(const char* tpl, const kwok_pod_spec* spec, const char* arena, size_t arena_len,
                            int64_t start_unix, const char* node_ip, int64_t creation_unix, uint32_t host_ip,
                            uint32_t pod_ip, int32_t status_nonempty, char* out, size_t cap, size_t* out_len);
/* Host only: the init patch (LockNode / configureNode) of the node in `ev` under
 * a custom node initialization template, at heartbeat time now_unix, as the
 * engine compiles and the kernels assemble it. */
int kwok_node_template_patch(const char* tpl, const char* heartbeat_tpl, const kwok_node_event* ev, const char* arena,
                             size_t arena_len, int64_t start_unix, const char* node_ip, int64_t now_unix, char* out,
                             size_t cap, size_t* out_len);
/* Host only: the heartbeat patch (configureHeartbeatNode) under a custom
 * heartbeat template (NULL: the default) at now_unix. */
int kwok_heartbeat_template_patch(const char* tpl, int64_t start_unix, const char* node_ip, int64_t now_unix, char* out,
                                  size_t cap, size_t* out_len);

/* Bucket of a node name (fnv1a32 & (buckets-1)) and its owning rank. */
uint32_t kwok_bucket_of(const char* name, size_t len, uint32_t buckets);
int32_t kwok_rank_of_bucket(uint32_t bucket, uint32_t buckets, int32_t world_size);

/* ---- watch-event ingest codec (host only, no device calls) ----
 * Decodes one Kubernetes Node / Pod JSON document (as a watch event or list
 * item carries it) into the record kwok_ingest_nodes / kwok_ingest_pods take,
 * evaluating the controller's selectors and the pod template's no-op test on
 * the host:
 *   kwok_codec_create   the selector half of controllers.NewController
 *                       controller.go:80-101, labelsParse utils.go:205-210
 *   kwok_decode_node    WatchNodes / ListNodes per-object work before Put/lock
 *                       (needHeartbeat, needLockNode) node_controller.go:206-223,256-270
 *   kwok_decode_pod     WatchPods / ListPods per-object work (needLockPod's selectors,
 *                       deletionTimestamp, finalizers) pod_controller.go:252-269,301-343,
 *                       plus computePatchData's SMP no-op test   pod_controller.go:404-439
 * kwok_str refs point into the caller's arena (the document); node status
 * blobs are canonicalised in place, so the arena is written.  The record's
 * op is UPSERT and handle / spec_id / node_handle are -1: the caller sets op
 * for watch.Deleted, and registers the pod spec (kwok_register_pod_spec) from
 * the decoded containers / init containers / readiness gates. */
typedef struct kwok_codec_config {
    int32_t manage_all_nodes;                          /* Config.ManageAllNodes */
    const char* manage_nodes_with_annotation_selector; /* Config.ManageNodesWithAnnotationSelector */
    const char* manage_nodes_with_label_selector;      /* ...WithLabelSelector: applied as the list/watch filter */
    const char* disregard_status_with_annotation_selector;
    const char* disregard_status_with_label_selector;
} kwok_codec_config;

#define KWOK_DOC_MAX_CONTAINERS 32u
#define KWOK_DOC_MAX_GATES 16u

typedef struct kwok_pod_doc {
    kwok_pod_event ev;
    kwok_str name;        /* metadata.name */
    kwok_str namespace_;  /* metadata.namespace */
    uint32_t n_containers, n_init_containers, n_readiness_gates, reserved0;
    kwok_container containers[KWOK_DOC_MAX_CONTAINERS];
    kwok_container init_containers[KWOK_DOC_MAX_CONTAINERS];
    kwok_str readiness_gates[KWOK_DOC_MAX_GATES];
} kwok_pod_doc;

typedef struct kwok_codec kwok_codec;
int kwok_codec_create(const kwok_codec_config* cfg, kwok_codec** out);
void kwok_codec_destroy(kwok_codec* c);
const char* kwok_codec_last_error(void); /* this thread's last codec error */
/* labels.Parse(selector).Matches(json_map) (json_map: a JSON object of strings or null) */
int kwok_selector_matches(const char* selector, const char* json_map, size_t len, int32_t* out);
int kwok_decode_node(const kwok_codec* c, char* arena, size_t arena_len, size_t doc_off, size_t doc_len,
                     kwok_node_event* ev);
int kwok_decode_pod(const kwok_codec* c, char* arena, size_t arena_len, size_t doc_off, size_t doc_len,
                    kwok_pod_doc* out);
/* Batches over documents at doc_off[i] / doc_len[i] of one arena, decoded by
 * `threads` host threads (documents must not overlap).  status[i] (optional)
 * gets each document's code; returns the number of rejected documents. */
int kwok_decode_nodes(const kwok_codec* c, char* arena, size_t arena_len, const uint64_t* doc_off,
                      const uint32_t* doc_len, size_t n, int threads, kwok_node_event* ev, int32_t* status);
int kwok_decode_pods(const kwok_codec* c, char* arena, size_t arena_len, const uint64_t* doc_off,
                     const uint32_t* doc_len, size_t n, int threads, kwok_pod_doc* out, int32_t* status);

/* ---- the pod codec on the GPU ("later as a GPU JSON
 * scanner"): the same per-document decision as kwok_decode_pod, made on the
 * engine's device by a one-pass scanner (one thread per document; a status
 * ahead of metadata / spec is scanned again once they are read).  Documents
 * the scanner leaves undecided (a JSON escape in a compared string, a status
 * with no metadata, spec or creation time to test against, a spec whose key
 * matches a registered spec's while its strings differ) are decoded by the
 * host codec, and counted in
 * *n_host; nothing is guessed.  Selectors larger than the device's tables (8
 * requirements, 32 values, 2 KiB of keys and values per codec) send every
 * document to the host codec.  Node documents: kwok_ingest_nodes_json below.
 *
 * kwok_decode_pods_gpu: the decode alone (tests, diagnostics): per document its
 *   kwok_pod_event (op UPSERT, handle / spec_id / node_handle -1, as
 *   kwok_decode_pod), name_ns[2i] / name_ns[2i+1] = metadata.name / namespace,
 *   spec_key[i] = kwok_spec_key of its containers / init containers / readiness
 *   gates (optional), status[i].  Returns the number of rejected documents.
 * kwok_ingest_pods_json: WatchPods / ListPods from the documents themselves
 *   (pod_controller.go:252-269, 301-343): decode on the device, then the GPU
 *   event switch of kwok_ingest_pods over the decoded records, which never leave
 *   the device.  op[i] / handle[i]: the caller's event (KWOK_OP_UPSERT with the
 *   handle of a known pod or -1, KWOK_OP_DELETE with its handle); a new pod's
 *   node by its spec.nodeName; pod specs are registered as they first appear
 *   (kwok_register_pod_spec).  A document that fails to decode gets its decode
 *   status in out_status and changes nothing.  Outputs as kwok_ingest_pods. */
uint64_t kwok_spec_key(const kwok_pod_spec* spec, const char* arena, size_t arena_len);
int kwok_decode_pods_gpu(kwok_engine* e, const kwok_codec* c, const char* arena, size_t arena_len,
                         const uint64_t* doc_off, const uint32_t* doc_len, size_t n, kwok_pod_event* ev,
                         kwok_str* name_ns, uint64_t* spec_key, int32_t* status, size_t* n_host);
int kwok_ingest_pods_json(kwok_engine* e, const kwok_codec* c, const char* arena, size_t arena_len,
                          const uint64_t* doc_off, const uint32_t* doc_len, const uint8_t* op, const int32_t* handle,
                          size_t n, int32_t* out_handles, int32_t* out_status, uint32_t* out_released, size_t* n_host);
/* kwok_ingest_nodes_json: WatchNodes / ListNodes from the node documents
 * themselves (node_controller.go:206-279): decoded on the device - name,
 * needHeartbeat (the codec's node selector, controller.go:81-98),
 * needLockNode's disregard selectors, status.phase and the ten nodeInfo
 * strings - then the GPU event switch of kwok_ingest_nodes over the decoded
 * records, which never leave the device.  A document with a non-empty
 * addresses / allocatable / capacity blob (re-serialised canonically by the
 * host codec, `YAML . 1` in node.status.tpl) or an escaped routed string is
 * decoded by the host codec and counted in *n_host.  op[i]: the watch event
 * (KWOK_OP_UPSERT / KWOK_OP_DELETE; a Deleted event's status is not read:
 * WatchNodes uses its name only, node_controller.go:265-269, so the last state
 * of a node kwok patched needs no host codec).  A document that fails to decode gets its
 * decode status (handle -1) and changes nothing.  Outputs and return as
 * kwok_ingest_nodes.  The arena must be below 4 GiB (kwok_str offsets). */
int kwok_ingest_nodes_json(kwok_engine* e, const kwok_codec* c, const char* arena, size_t arena_len,
                           const uint64_t* doc_off, const uint32_t* doc_len, const uint8_t* op, size_t n,
                           int32_t* out_handles, int32_t* out_status, size_t* n_host);
/* kwok_decode_nodes_gpu: the decode alone (tests, diagnostics): per document
 * the kwok_node_event kwok_decode_node writes (op UPSERT) and its status; the
 * documents the device leaves undecided are decoded by the host codec in place
 * (which re-serialises their blobs over their own spans, as kwok_decode_nodes
 * does: the arena is written).  Returns the number of rejected documents. */
int kwok_decode_nodes_gpu(kwok_engine* e, const kwok_codec* c, char* arena, size_t arena_len, const uint64_t* doc_off,
                          const uint32_t* doc_len, size_t n, kwok_node_event* ev, int32_t* status, size_t* n_host);

#ifdef __cplusplus
}
#endif
#endif /* KWOK_ENGINE_H */
