// ingest.hip - kwok_ingest_pods on the GPU: the WatchPods / ListPods event
// switch (pod_controller.go:301-343; routing of ListPods items, :357-368) over
// a batch of watch records, in event order per bucket.
//
// The device holds the pod slot state (pod_state's USED bit is the occupancy
// of a slot; pod_node the node a pod is bound to; node_state's NS_SLOT the
// occupancy of a node slot), so a batch never round-trips per record through
// host mirrors.  A batch is:
//
//   k_ing_prep    one thread per record: every check that depends on the
//                 record alone (arena bounds, IPv4 strings, spec id, phase,
//                 creation time, handle -> owned bucket), the statuses that
//                 need no state, per-bucket create counts (growth check), the
//                 owned by-name creates (spec.nodeName: the host resolves the
//                 name to its node slot).
//   k_ing_need    live pods + creates of every bucket with creates.
//   radix sort    a stable sort of the batch by bucket (rocprim), bucket ranges.
//   k_ing_apply   one wave per bucket, its records in event order: the slot
//                 policy (lowest free slot, canonical), coalescing by applying
//                 each record to the state in order, node references (a
//                 deleted node's entry lives while pods reference it,
//                 node_controller.go:265-269), ingest-time IP release
//                 (ipPool.Put, pod_controller.go:329-336), statuses and handles.
//
// Records are 48-byte kwok_pod_event; the per-record work is a handful of
// loads and stores, so the batch is bound by its H2D copy and by the serial
// chain of one bucket's records (~500 per bucket at 2M records over 4096
// buckets), not by HBM bandwidth.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "../../include/kwok_engine.h"
#include "device.h"
#include "kernels.h"

namespace kwok {
namespace {

__device__ __forceinline__ uint32_t lane() { return threadIdx.x & 63u; }
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t k) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)k); }
__device__ __forceinline__ uint64_t rdl64(uint64_t v, uint32_t k) {
    return (uint64_t)rdl((uint32_t)v, k) | ((uint64_t)rdl((uint32_t)(v >> 32), k) << 32);
}
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void mem_sync() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// loads of state this wave may have stored earlier in the batch: agent-scope
// (coherent) loads, so a stale line in the CU's vector L1 is never returned
template <class T>
__device__ __forceinline__ T ld_coh(const T* p) {
    return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld16_coh(const uint16_t* p) {
    // 32-bit coherent load of the aligned word holding *p
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t w = ld_coh(reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3));
    return (a & 2) ? (w >> 16) : (w & 0xFFFFu);
}
__device__ __forceinline__ uint32_t ld8_coh(const uint8_t* p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t w = ld_coh(reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3));
    return (w >> (8 * (a & 3))) & 0xFFu;
}

// parse_ipv4 (templates.cpp): canonical dotted quads only
__device__ bool d_parse_ipv4(const uint8_t* s, uint32_t n, uint32_t* out) {
    if (n < 7 || n > 15) return false;
    uint32_t v = 0, i = 0;
    int parts = 0;
    while (i < n) {
        uint32_t j = i, x = 0;
        while (j < n && j - i < 4) {
            const uint32_t c = s[j];
            if (c < '0' || c > '9') break;
            x = x * 10u + (c - '0');
            j++;
        }
        if (j == i || j - i > 3 || x > 255 || (j - i > 1 && s[i] == '0')) return false;
        v = (v << 8) | x;
        parts++;
        if (j < n) {
            if (s[j] != '.' || j + 1 == n) return false;
            j++;
        }
        i = j;
    }
    if (parts != 4) return false;
    *out = v;
    return true;
}
__device__ __forceinline__ int d_parse_opt_ip(const uint8_t* arena, kwok_str s, uint32_t* ip) {
    *ip = 0;
    if (!s.len) return KWOK_OK;
    if (!d_parse_ipv4(arena + s.off, s.len, ip) || *ip == 0) return KWOK_EDOMAIN;
    return KWOK_OK;
}
__device__ __forceinline__ uint32_t d_fnv1a32(const uint8_t* s, uint32_t n) {
    uint32_t h = 0x811C9DC5u;
    for (uint32_t i = 0; i < n; i++) h = (h ^ s[i]) * 0x01000193u;
    return h;
}
__device__ __forceinline__ bool d_in_cidr(const PoolGeom& g, uint32_t ip) {
    return (uint64_t)(ip - g.net) < g.size && ip >= g.net;
}

// ---------------------------------------------------------------------------
// k_ing_prep: record-local checks (the host prep of round 2, engine.cpp) and
// every status that does not depend on state.  keys[i] = the owned local bucket
// whose records the apply pass takes in order, or nb (decided here).
// ---------------------------------------------------------------------------
// The compact record (kwok_pod_rec): its strings were parsed by the caller, so
// only the checks on values remain; a create names its node by handle.
__device__ void prep_packed(const DevState& S, const IngestBatch& I, uint32_t i) {
    const uint8_t* p = static_cast<const uint8_t*>(I.ev) + (size_t)i * sizeof(kwok_pod_rec);
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p);  // 20 bytes: five dwords
    const uint32_t w0 = w[0], ctime = w[2], hip = w[3], pip = w[4];
    const int32_t target = (int32_t)w[1];
    const uint32_t op = w0 & 0x7Fu, create = w0 & KWOK_REC_NEW, fl = (w0 >> 8) & 0xFFu, spec = w0 >> 16;
    PodRec r;
    r.bucket = REC_NONE;
    r.pos = 0;
    r.hip = r.pip = 0;
    r.ctime = 0;
    r.spec = 0;
    r.op = (uint8_t)op;
    r.phase = (uint8_t)(fl >> KWOK_REC_PHASE_SHIFT);
    r.flags = (uint8_t)(fl & 31u);
    r.chk = 0;
    r.fst = KWOK_OK;
    r.pst = KWOK_OK;
    r.pad[0] = r.pad[1] = r.pad[2] = r.pad[3] = 0;
    int st = 1;  // 1: the apply pass decides
    if (op == KWOK_OP_DELETE) {
        if (pip) r.pip = pip, r.chk |= REC_DEL_IP;
    } else if (op == KWOK_OP_UPSERT) {
        r.hip = hip, r.pip = pip;
        if (spec >= I.n_specs) r.fst = KWOK_EINVAL;
        else if (r.phase > KWOK_PHASE_UNKNOWN) r.fst = KWOK_EINVAL;
        else r.ctime = ctime, r.spec = (uint16_t)spec;
    }
    if (!create && target >= 0) {
        r.chk |= REC_EXISTING;
        const uint32_t h = (uint32_t)target, b = h / S.pod_stride;
        if (b >= S.buckets) r.pst = KWOK_ENOTFOUND;
        else if (b < S.b_lo || b >= S.b_lo + S.nb) r.pst = KWOK_ENOTMINE;
        else r.bucket = b - S.b_lo, r.pos = h - b * S.pod_stride;
        if (r.pst != KWOK_OK) st = r.pst;
    } else if (!create || op != KWOK_OP_UPSERT || target < 0) {
        st = KWOK_EINVAL;  // a DELETE / update needs its handle, a create its node's handle
    } else if (r.fst != KWOK_OK) {
        st = r.fst;
    } else {
        const int64_t l = (int64_t)target - (int64_t)S.b_lo * S.cn;
        if (l >= 0 && l < (int64_t)S.n_node_slots) r.bucket = (uint32_t)(l / S.cn), r.pos = (uint32_t)(l % S.cn);
        else st = KWOK_ENOTMINE;
    }
    if (st == 1 && op == KWOK_OP_UPSERT && create) atomicAdd(&I.creates[r.bucket], 1u);
    if (st == 1 && op == KWOK_OP_DELETE && !I.dels[r.bucket]) I.dels[r.bucket] = 1u;
    I.rec[i] = r;
    I.keys[i] = st == 1 ? r.bucket : S.nb;
    if (st != 1) {
        I.out_handle[i] = -1;
        I.out_status[i] = st;
        I.out_released[i] = 0;
        if (st != KWOK_OK) atomicAdd(&I.sum->rejected, 1u);
    }
}

__global__ void k_ing_prep(DevState S, IngestBatch I) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= I.n) return;
    if (I.packed) {
        prep_packed(S, I, i);
        return;
    }
    const kwok_pod_event x = static_cast<const kwok_pod_event*>(I.ev)[i];
    PodRec r;
    r.bucket = REC_NONE;
    r.pos = 0;
    r.hip = r.pip = 0;
    r.ctime = 0;
    r.spec = 0;
    r.op = x.op;
    r.phase = x.phase;
    r.flags = x.flags;
    r.chk = 0;
    r.fst = KWOK_OK;
    r.pst = KWOK_OK;
    r.pad[0] = r.pad[1] = r.pad[2] = r.pad[3] = 0;
    int st = 1;  // 1: the apply pass decides
    auto in_arena = [&](kwok_str s) { return (uint64_t)s.off + s.len <= I.arena_len; };
    if (!in_arena(x.node_name) || !in_arena(x.host_ip) || !in_arena(x.pod_ip)) {
        st = KWOK_EDOMAIN;
    } else {
        if (x.op == KWOK_OP_DELETE) {
            uint32_t ip = 0;
            if (x.pod_ip.len && d_parse_ipv4(I.arena + x.pod_ip.off, x.pod_ip.len, &ip)) r.pip = ip, r.chk |= REC_DEL_IP;
        } else if (x.op == KWOK_OP_UPSERT) {
            if (d_parse_opt_ip(I.arena, x.host_ip, &r.hip) || d_parse_opt_ip(I.arena, x.pod_ip, &r.pip)) r.fst = KWOK_EDOMAIN;
            else if (x.spec_id < 0 || (uint32_t)x.spec_id >= I.n_specs) r.fst = KWOK_EINVAL;
            else if (x.phase > KWOK_PHASE_UNKNOWN) r.fst = KWOK_EINVAL;
            else if (x.creation_unix < 0 || x.creation_unix > 0xFFFFFFFFll) r.fst = KWOK_EDOMAIN;
            else r.ctime = (uint32_t)x.creation_unix, r.spec = (uint16_t)x.spec_id;  // max_pod_specs <= 65535
        }
        if (x.handle >= 0) {
            // pod_slot: handle = bucket * stride + index; the index < Cp check is the apply
            // pass's (a growth between the two changes Cp)
            r.chk |= REC_EXISTING;
            const uint32_t h = (uint32_t)x.handle, b = h / S.pod_stride;
            if (b >= S.buckets) r.pst = KWOK_ENOTFOUND;
            else if (b < S.b_lo || b >= S.b_lo + S.nb) r.pst = KWOK_ENOTMINE;
            else r.bucket = b - S.b_lo, r.pos = h - b * S.pod_stride;
            if (r.pst != KWOK_OK) st = r.pst;
        } else if (x.op != KWOK_OP_UPSERT) {
            st = KWOK_EINVAL;  // a DELETE needs a handle; any other op is invalid
        } else if (r.fst != KWOK_OK) {
            st = r.fst;        // a create with a bad field changes nothing
        } else if (x.node_handle >= 0) {
            const int64_t l = (int64_t)x.node_handle - (int64_t)S.b_lo * S.cn;
            if (l >= 0 && l < (int64_t)S.n_node_slots) r.bucket = (uint32_t)(l / S.cn), r.pos = (uint32_t)(l % S.cn);
            else st = KWOK_ENOTMINE;
        } else {
            r.chk |= REC_BY_NAME;
            if (!x.node_name.len || x.node_name.len > 253) {
                st = KWOK_EDOMAIN;
            } else {
                const uint32_t b = d_fnv1a32(I.arena + x.node_name.off, x.node_name.len) & (S.buckets - 1);
                if (b < S.b_lo || b >= S.b_lo + S.nb) st = KWOK_ENOTMINE;
                else r.bucket = b - S.b_lo, I.byname[atomicAdd(&I.sum->n_byname, 1u)] = i;
            }
        }
        // growth check: creates per bucket (an upper bound: the batch's deletes are not netted out)
        if (st == 1 && x.op == KWOK_OP_UPSERT && x.handle < 0) atomicAdd(&I.creates[r.bucket], 1u);
        // buckets where a pod leaves at ingest (a node entry may be freed mid-batch: by-name resolution)
        if (st == 1 && x.op == KWOK_OP_DELETE && !I.dels[r.bucket]) I.dels[r.bucket] = 1u;
    }
    I.rec[i] = r;
    I.keys[i] = st == 1 ? r.bucket : S.nb;
    if (st != 1) {
        I.out_handle[i] = -1;
        I.out_status[i] = st;
        I.out_released[i] = 0;
        if (st != KWOK_OK) atomicAdd(&I.sum->rejected, 1u);
    }
}

// ---------------------------------------------------------------------------
// k_ing_need: one wave per bucket with creates: live pods (USED below the fill
// mark) + creates -> the batch's growth need (max over buckets)
// ---------------------------------------------------------------------------
__global__ void k_ing_need(DevState S, IngestBatch I) {
    const uint32_t b = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (b >= S.nb) return;
    const uint32_t c = I.creates[b];
    if (!c) return;
    const uint32_t fill = S.pod_fill[b];
    const uint16_t* ps = S.pod_state + (size_t)b * S.cp;
    uint32_t live = 0;
    for (uint32_t s = lane(); s < fill; s += 64) live += ps[s] & PS_USED;
    for (int o = 32; o; o >>= 1) live += (uint32_t)__shfl_xor((int)live, o);
    if (lane() == 0) {
        atomicMax(&I.sum->need, live + c);
        I.creates[b] = 0;  // zero for the next batch
    }
}

// host resolutions of by-name creates: code = node index in the bucket, or
// 0x8000'0000 | (uint8)status (final), or 0x4000'0000 (REC_HARD: resolved later)
__global__ void k_ing_fix(DevState S, IngestBatch I, const uint32_t* fix, uint32_t n_fix) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_fix) return;
    const uint32_t i = fix[2 * k], code = fix[2 * k + 1];
    if (code & 0x80000000u) {
        const int st = (int)(int8_t)(code & 0xFFu);
        I.out_handle[i] = -1;
        I.out_status[i] = st;
        I.out_released[i] = 0;
        I.keys[i] = S.nb;
        I.rec[i].chk = (uint8_t)(I.rec[i].chk | REC_FINAL);  // (a stopped bucket's record: skipped on relaunch)
        if (st != KWOK_OK) atomicAdd(&I.sum->rejected, 1u);
    } else if (code & 0x40000000u) {
        I.rec[i].chk = (uint8_t)((I.rec[i].chk | REC_HARD) & ~REC_RESOLVED);
    } else {
        I.rec[i].pos = code;
        I.rec[i].chk = (uint8_t)((I.rec[i].chk | REC_RESOLVED) & ~REC_HARD);
    }
}

// bucket ranges of the sorted batch: beg / end (zeroed before: empty buckets are [0, 0))
__global__ void k_ing_ranges(DevState S, IngestBatch I) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= I.n) return;
    const uint32_t k = I.keys_sorted[p];
    if (k >= S.nb) return;
    if (p == 0 || I.keys_sorted[p - 1] != k) I.beg[k] = p;
    if (p + 1 == I.n || I.keys_sorted[p + 1] != k) I.end[k] = p + 1;
}

// ---------------------------------------------------------------------------
// k_ing_apply: one wave per bucket, its records in event order.
// ---------------------------------------------------------------------------
constexpr int APPLY_WAVES = 4;
constexpr uint32_t MAX_BM_WORDS = 65536 / 64;  // Cp <= 65528 (pod_handle_stride)

struct Bucket {
    uint32_t b, cp, cn, fill;
    size_t sbase, nbase;  // first pod / node slot of the bucket
    uint64_t* bm;         // LDS occupancy bitmap, Cp bits
    uint32_t nw, hint;    // words; no free slot below word `hint`
};

// is node index nd of the bucket still referenced by a live pod?  (the
// wave's own stores drained first; coherent loads)
__device__ bool node_referenced(const DevState& S, const Bucket& B, uint32_t nd) {
    mem_sync();
    bool hit = false;
    for (uint32_t s0 = 0; s0 < B.fill; s0 += 64) {
        const uint32_t s = s0 + lane();
        bool h = false;
        if (s < B.fill && ((B.bm[s >> 6] >> (s & 63)) & 1)) h = ld16_coh(S.pod_node + B.sbase + s) == nd;
        if (__ballot(h)) {
            hit = true;
            break;
        }
    }
    return hit;
}
// the lowest free pod slot of the bucket (-1: none below Cp)
__device__ int32_t first_free(Bucket& B) {
    for (uint32_t w0 = B.hint; w0 < B.nw; w0 += 64) {
        const uint32_t q = w0 + lane();
        uint64_t word = ~0ull;
        if (q < B.nw) {
            word = B.bm[q];
            if (q == B.nw - 1 && (B.cp & 63)) word |= ~0ull << (B.cp & 63);  // bits past Cp are not slots
        }
        const uint64_t m = __ballot(word != ~0ull);
        if (m) {
            const uint32_t j = (uint32_t)__builtin_ctzll(m);
            const uint64_t wj = rdl64(word, j);
            B.hint = w0 + j;
            return (int32_t)((w0 + j) * 64 + (uint32_t)__builtin_ctzll(~wj));
        }
        B.hint = w0 + 64 < B.nw ? w0 + 64 : B.nw;
    }
    return -1;
}

__device__ __forceinline__ uint32_t wave_incl(uint32_t x) {
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, (unsigned)o);
        if ((int)lane() >= o) x += y;
    }
    return x;
}

// the state word a pod record sets (WatchPods routing, pod_controller.go:301-319)
__device__ __forceinline__ uint32_t pod_bits(const DevState& S, uint32_t flags, uint32_t phase, uint32_t hip,
                                             uint32_t pip, uint32_t ns) {
    uint32_t bits = PS_USED | (phase << PS_PHASE_SHIFT);
    if (flags & KWOK_POD_DISREGARD) bits |= PS_DISREGARD;
    if (flags & KWOK_POD_HAS_FINALIZERS) bits |= PS_HAS_FIN;
    // a status that holds an IP is not empty (`{{ with .status }}`)
    if ((flags & KWOK_POD_STATUS_NONEMPTY) || hip || pip) bits |= PS_STATUS_NONEMPTY;
    // the caller's digest is of the default template; with a custom one a pod
    // conforms once the engine has patched it (an extra, idempotent patch at most)
    if ((flags & KWOK_POD_CONFORMS) && !S.custom_pod) bits |= PS_CONFORMS;
    if (hip) bits |= PS_HAS_HOST_IP;
    bits |= ip_state_bits(S.pool, pip);
    if (flags & KWOK_POD_DELETING) {
        if (ns & NS_MANAGED) bits |= PS_DELETE_PENDING;  // pod_controller.go:306-308 -> deletePodChan
    } else if ((ns & NS_MANAGED) && !(flags & KWOK_POD_DISREGARD)) {
        bits |= PS_EVENT;  // needLockPod (:252-269) -> lockPodChan
    }
    return bits;
}

__global__ __launch_bounds__(64 * APPLY_WAVES) void k_ing_apply(DevState S, IngestBatch I) {
    __shared__ uint64_t bm_all[APPLY_WAVES][MAX_BM_WORDS];
    __shared__ uint32_t flist_all[APPLY_WAVES][64];  // a chunk's creates' slots (parallel path)
    const uint32_t w = threadIdx.x >> 6, l = lane();
    const uint32_t b = blockIdx.x * APPLY_WAVES + w;
    if (b >= S.nb) return;
    const uint32_t pbeg = I.beg[b], pend = I.end[b];
    if (pbeg >= pend) return;
    Bucket B;
    B.b = b;
    B.cp = S.cp;
    B.cn = S.cn;
    B.fill = S.pod_fill[b];
    B.sbase = (size_t)b * S.cp;
    B.nbase = (size_t)b * S.cn;
    B.bm = bm_all[w];
    B.nw = (S.cp + 63) / 64;
    B.hint = 0;
    const uint32_t fill0 = B.fill;
    // occupancy bitmap of [0, fill): pod_state's USED bits (8 slots per 16-byte load)
    for (uint32_t q = l; q < B.nw; q += 64) {
        uint64_t word = 0;
        for (uint32_t g = 0; g < 8; g++) {
            const uint32_t s = q * 64 + g * 8;
            if (s >= B.fill) break;
            const uint4 v = *reinterpret_cast<const uint4*>(S.pod_state + B.sbase + s);
            const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                word |= (uint64_t)(u[k] & PS_USED) << (g * 8 + 2 * k);
                word |= (uint64_t)((u[k] >> 16) & PS_USED) << (g * 8 + 2 * k + 1);
            }
        }
        B.bm[q] = word;
    }
    lds_sync();
    const uint32_t keep_ex = PS_EVENT | PS_DELETE_PENDING;
    uint32_t rejected = 0;
    bool stopped = false, foreign = false;
    uint32_t p0 = pbeg;
    for (; p0 < pend && !stopped; p0 += 64) {
        mem_sync();  // the previous chunk's stores, before this chunk's (coherent) loads
        const uint32_t p = p0 + l;
        const bool v = p < pend;
        const uint32_t idx = v ? I.idx_sorted[p] : 0u;
        uint4 ra = make_uint4(0, 0, 0, 0), rb = ra;
        if (v) {
            const uint4* rp = reinterpret_cast<const uint4*>(I.rec + idx);
            ra = rp[0];
            rb = rp[1];
        }
        // PodRec: bucket, pos, hip, pip | ctime, spec|op<<16|phase<<24, flags|chk<<8|fst<<16|pst<<24, pad
        const uint32_t pos = ra.y;
        const uint32_t hop = rb.y, hfl = rb.z;
        const uint32_t chk = (hfl >> 8) & 0xFFu;
        // prefetch: an existing pod's state and node; the node's state
        const bool ex = v && (chk & REC_EXISTING) && pos < B.cp;
        uint32_t st0 = 0, nd0 = pos, ip0 = 0;
        if (ex) {
            st0 = ld16_coh(S.pod_state + B.sbase + pos);
            nd0 = ld16_coh(S.pod_node + B.sbase + pos);
            ip0 = ld_coh(S.pod_ip + B.sbase + pos);
        }
        uint32_t ns0 = 0;
        if (v && nd0 < B.cn) ns0 = ld8_coh(S.node_state + B.nbase + nd0);
        // ---- parallel path: a chunk in which no record can see another's effect
        // except through the creates' slot order (no DELETE, no record waiting for
        // the host, no slot named twice, no existing record on a free slot beside
        // creates, enough free slots for every create: no node entry can go) ----
        {
            const uint32_t op = (hop >> 16) & 0xFFu, fl = hfl & 0xFFu;
            const int fst = (int)(int8_t)((hfl >> 16) & 0xFFu);
            const bool act = v && !(chk & REC_FINAL);
            const bool exl = act && (chk & REC_EXISTING);
            const bool used = exl && pos < B.cp && ((B.bm[pos >> 6] >> (pos & 63)) & 1);
            const bool crt = act && !exl;  // (prep decided creates with a bad field, or foreign / unknown)
            const bool take = crt && (ns0 & NS_SLOT);
            const uint32_t key = exl ? pos : (0x80000000u | l);
            bool dup = false;
            for (uint32_t j = 0; j < 63; j++) dup |= (l > j) && key == rdl(key, j);
            bool par = !__ballot((act && ((chk & REC_HARD) && !(chk & REC_RESOLVED))) || (act && op == KWOK_OP_DELETE) || dup) &&
                       !(__ballot(exl && !used) && __ballot(crt));
            uint32_t* flist = flist_all[w];
            const uint64_t tm = __ballot(take);
            const uint32_t c = (uint32_t)__popcll(tm);
            if (par && c) {  // the lowest c free slots, in order
                uint32_t got = 0;
                for (uint32_t wq = B.hint; got < c && wq < B.nw; wq += 64) {
                    const uint32_t q = wq + l;
                    uint64_t word = ~0ull;
                    if (q < B.nw) {
                        word = B.bm[q];
                        if (q == B.nw - 1 && (B.cp & 63)) word |= ~0ull << (B.cp & 63);
                    }
                    uint64_t fr = ~word;
                    const uint32_t cntf = (uint32_t)__popcll(fr);
                    const uint32_t incl = wave_incl(cntf);
                    uint32_t r = got + incl - cntf;
                    while (fr && r < c) {
                        flist[r++] = q * 64 + (uint32_t)__builtin_ctzll(fr);
                        fr &= fr - 1;
                    }
                    got += rdl(incl, 63);
                }
                lds_sync();
                par = got >= c;  // too few: EFULL (and its node check) in event order
            }
            if (par) {
                const uint32_t r = (uint32_t)__popcll(tm & ((1ull << l) - 1ull));
                if (c) {
                    const uint32_t last = flist[c - 1];  // the highest slot taken
                    if (take) atomicOr((unsigned long long*)&B.bm[flist[r] >> 6], 1ull << (flist[r] & 63));
                    B.hint = last >> 6;
                    if (last + 1 > B.fill) B.fill = min(B.cp, (last + 8u) & ~7u);
                }
                int stt = KWOK_OK;
                uint32_t slot = pos, cur = st0, nd = nd0;
                int32_t handle = -1;
                if (exl) {
                    stt = !used ? KWOK_ENOTFOUND : op == KWOK_OP_UPSERT ? fst : KWOK_EINVAL;
                } else if (crt) {
                    nd = pos;
                    if (!take) stt = KWOK_ENOTFOUND;
                    else slot = flist[r], cur = 0;
                }
                if (act && stt == KWOK_OK) {
                    // an in-CIDR podIP this pod did not hold (a create with one, an update to another)
                    foreign |= ra.w && d_in_cidr(S.pool, ra.w) && (!exl || ra.w != ip0);
                    const uint32_t nst = (cur & (exl ? keep_ex : 0u)) | pod_bits(S, fl, hop >> 24, ra.z, ra.w, ns0);
                    const size_t g = B.sbase + slot;
                    S.pod_state[g] = (uint16_t)nst;
                    S.pod_node[g] = (uint16_t)nd;
                    S.pod_spec[g] = (uint16_t)(hop & 0xFFFFu);
                    S.pod_ctime[g] = rb.x;
                    S.host_ip[g] = ra.z;
                    S.pod_ip[g] = ra.w;
                    handle = (int32_t)((S.b_lo + b) * S.pod_stride + slot);
                }
                if (act) {
                    I.out_handle[idx] = handle;
                    I.out_status[idx] = stt;
                    I.out_released[idx] = 0;
                }
                rejected += (uint32_t)__popcll(__ballot(act && stt != KWOK_OK));
                lds_sync();
                continue;
            }
        }
        // ---- serial path: the records one at a time, in event order ----
        // in-chunk hazards: lane j keeps what record j wrote (slot, its state / node;
        // a freed node index)
        uint32_t wslot = ~0u, wst = 0, wnd = 0, wip = 0, wfreed = ~0u;
        const uint32_t cnt = pend - p0 < 64u ? pend - p0 : 64u;
        for (uint32_t k = 0; k < cnt; k++) {
            const uint32_t kchk = rdl(chk, k);
            const uint32_t kop = (rdl(hop, k) >> 16) & 0xFFu;
            if (kchk & REC_FINAL) continue;  // its status came from the host's resolution
            if ((kchk & REC_HARD) && !(kchk & REC_RESOLVED)) {
                // by name, and the node entry may have been freed by the records before:
                // the host resolves it and launches the bucket again from here
                if (l == 0) {
                    I.beg[b] = p0 + k;
                    I.stopped[atomicAdd(&I.sum->n_stopped, 1u)] = b;
                }
                stopped = true;
                break;
            }
            const uint32_t kidx = rdl(idx, k), kpos = rdl(pos, k);
            const uint32_t kfl = rdl(hfl, k);
            const uint32_t flags = kfl & 0xFFu;
            const int fst = (int)(int8_t)((kfl >> 16) & 0xFFu);
            const bool existing = kchk & REC_EXISTING;
            int stt = KWOK_OK;
            int32_t handle = -1;
            uint32_t released = 0;
            uint32_t cur = rdl(st0, k), nd = rdl(nd0, k), curip = rdl(ip0, k);
            if (existing) {
                if (kpos >= B.cp || !((B.bm[kpos >> 6] >> (kpos & 63)) & 1)) {
                    stt = KWOK_ENOTFOUND;
                } else {
                    const uint64_t m = __ballot(wslot == kpos);
                    if (m) {  // an earlier record of this chunk wrote the slot
                        const uint32_t j = 63u - (uint32_t)__builtin_clzll(m);
                        cur = rdl(wst, j);
                        nd = rdl(wnd, j);
                        curip = rdl(wip, j);
                    }
                }
            }
            uint32_t ns = rdl(ns0, k);
            if (nd != rdl(nd0, k) && nd < B.cn) {  // the slot's node changed in this chunk: its state now
                mem_sync();
                ns = ld8_coh(S.node_state + B.nbase + nd);
            }
            if (nd < B.cn) {
                const uint64_t m = __ballot(wfreed == nd);
                if (m) ns = 0;  // freed by an earlier record of this chunk
            }
            auto free_node = [&](uint32_t n) {  // the node entry goes (free_node_if_unused)
                if (l == 0) {
                    S.node_state[B.nbase + n] = 0;
                    S.node_blob[B.nbase + n] = 0;
                    I.freed[atomicAdd(&I.sum->n_freed, 1u)] = (uint32_t)(B.nbase + n);
                }
                if (l == k) wfreed = n;
            };
            if (stt == KWOK_OK && kop == KWOK_OP_DELETE) {
                // pod_controller.go:329-336: release the event object's podIP if the node is managed
                // (EnableCNI: the caller's cni.Remove instead, :337-342)
                const uint32_t ip = rdl(ra.w, k);
                if (!S.cni && (ns & NS_MANAGED) && (kchk & REC_DEL_IP) && d_in_cidr(S.pool, ip)) {
                    released = ip;
                    foreign |= ip != curip;  // a release of an address its pod does not hold
                    if (l == 0) {
                        const uint64_t bit = ip - S.pool.net;
                        atomicAnd((unsigned long long*)&S.used_bm[bit >> 6], ~(1ull << (bit & 63)));
                        atomicOr((unsigned long long*)&S.usable_bm[bit >> 6], 1ull << (bit & 63));
                    }
                }
                if (l == 0) {
                    S.pod_state[B.sbase + kpos] = 0;
                    B.bm[kpos >> 6] &= ~(1ull << (kpos & 63));
                }
                lds_sync();
                if ((kpos >> 6) < B.hint) B.hint = kpos >> 6;
                if (l == k) wslot = kpos, wst = 0, wnd = nd, wip = 0;
                // the node entry of a deleted (or placeholder) node lives while pods reference it
                if ((ns & NS_SLOT) && !(ns & NS_EXISTS) && !node_referenced(S, B, nd)) free_node(nd);
                handle = (int32_t)((S.b_lo + b) * S.pod_stride + kpos);
            } else if (stt == KWOK_OK && kop == KWOK_OP_UPSERT) {
                stt = fst;
                uint32_t slot = kpos;
                if (stt == KWOK_OK && !existing) {
                    nd = kpos;  // the node's index (by handle, or resolved by the host)
                    if (!(ns & NS_SLOT)) stt = KWOK_ENOTFOUND;
                    if (stt == KWOK_OK) {
                        const int32_t s = first_free(B);
                        if (s < 0) {
                            stt = KWOK_EFULL;
                            if (!(ns & NS_EXISTS) && !node_referenced(S, B, nd)) free_node(nd);
                        } else {
                            slot = (uint32_t)s;
                            if (l == 0) B.bm[slot >> 6] |= 1ull << (slot & 63);
                            lds_sync();
                            if (slot + 1 > B.fill) B.fill = min(B.cp, (slot + 8u) & ~7u);
                            cur = 0;
                        }
                    }
                }
                if (stt == KWOK_OK) {
                    const uint32_t hip = rdl(ra.z, k), pip = rdl(ra.w, k);
                    foreign |= pip && d_in_cidr(S.pool, pip) && (!existing || pip != curip);
                    const uint32_t bits = pod_bits(S, flags, rdl(hop, k) >> 24, hip, pip, ns);
                    const uint32_t nst = (cur & (existing ? keep_ex : 0u)) | bits;
                    if (l == 0) {
                        const size_t g = B.sbase + slot;
                        S.pod_state[g] = (uint16_t)nst;
                        S.pod_node[g] = (uint16_t)nd;
                        S.pod_spec[g] = (uint16_t)(rdl(hop, k) & 0xFFFFu);
                        S.pod_ctime[g] = rdl(rb.x, k);
                        S.host_ip[g] = hip;
                        S.pod_ip[g] = pip;
                    }
                    if (l == k) wslot = slot, wst = nst, wnd = nd, wip = pip;
                    handle = (int32_t)((S.b_lo + b) * S.pod_stride + slot);
                }
            } else if (stt == KWOK_OK) {
                stt = KWOK_EINVAL;
            }
            if (stt != KWOK_OK) rejected++;
            if (l == 0) {
                I.out_handle[kidx] = stt == KWOK_OK ? handle : -1;
                I.out_status[kidx] = stt;
                I.out_released[kidx] = released;
            }
        }
    }
    if (l == 0) {
        if (B.fill != fill0) S.pod_fill[b] = (uint16_t)B.fill;
        if (!stopped) I.beg[b] = pend;  // done: a relaunch after a stop skips the bucket
        if (rejected) atomicAdd(&I.sum->rejected, rejected);
    }
    if (__ballot(foreign) && l == 0) {
        atomicOr(&I.sum->foreign, 1u);
    }
}

// live pods referencing node slot slots[i] (one wave each)
__global__ void k_node_refs(DevState S, const uint32_t* slots, uint32_t n, uint32_t* refs) {
    const uint32_t i = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (i >= n) return;
    const uint32_t slot = slots[i], b = slot / S.cn, nd = slot % S.cn;
    const uint32_t fill = S.pod_fill[b];
    const size_t sb = (size_t)b * S.cp;
    uint32_t c = 0;
    // 8 slots per lane per step (16-byte loads of state and node index): few round trips
    for (uint32_t s = lane() * 8; s < fill; s += 512) {
        const uint4 st = *reinterpret_cast<const uint4*>(S.pod_state + sb + s);
        const uint4 ndw = *reinterpret_cast<const uint4*>(S.pod_node + sb + s);
        const uint32_t a[4] = {st.x, st.y, st.z, st.w}, q[4] = {ndw.x, ndw.y, ndw.z, ndw.w};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            c += (a[k] & PS_USED) && (q[k] & 0xFFFFu) == nd;
            c += ((a[k] >> 16) & PS_USED) && (q[k] >> 16) == nd;
        }
    }
    for (int o = 32; o; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o);
    if (lane() == 0) refs[i] = c;
}

// kwok_cni_assign (handles deduplicated by the host, last assignment kept):
// configurePod's pod.Status.PodIP = ips[0] (pod_controller.go:388)
__global__ void k_cni_assign(DevState S, const int32_t* handles, const uint32_t* ips, const uint8_t* wr, uint32_t n,
                             int32_t* status, uint32_t* rejected) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t h = handles[i];
    int st = KWOK_OK;
    size_t slot = 0;
    if (h < 0 || (uint32_t)h / S.pod_stride >= S.buckets) {
        st = KWOK_ENOTFOUND;
    } else {
        const uint32_t b = (uint32_t)h / S.pod_stride, idx = (uint32_t)h - b * S.pod_stride;
        if (b < S.b_lo || b >= S.b_lo + S.nb) st = KWOK_ENOTMINE;
        else if (idx >= S.cp) st = KWOK_ENOTFOUND;
        else {
            slot = (size_t)(b - S.b_lo) * S.cp + idx;
            if (!(S.pod_state[slot] & PS_USED)) st = KWOK_ENOTFOUND;
            else if (!ips[i]) st = KWOK_EDOMAIN;
        }
    }
    if (st == KWOK_OK && wr[i]) {  // the last valid assignment of the handle
        S.pod_ip[slot] = ips[i];
        S.pod_state[slot] = (uint16_t)((S.pod_state[slot] & ~PS_IP_BITS) | PS_STATUS_NONEMPTY | ip_state_bits(S.pool, ips[i]));
    }
    if (st != KWOK_OK) atomicAdd(rejected, 1u);
    status[i] = st;
}

inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

}  // namespace

size_t ingest_sort_bytes(uint32_t n, uint32_t key_bits) {
    size_t bytes = 0;
    rocprim::counting_iterator<uint32_t> it(0u);
    (void)rocprim::radix_sort_pairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, it,
                                    (uint32_t*)nullptr, n, 0u, key_bits);
    return bytes;
}

__global__ void k_ing_status8(IngestBatch I, int8_t* dst) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < I.n) dst[i] = (int8_t)I.out_status[i];
}
void launch_ingest_status8(const IngestBatch& I, int8_t* dst, hipStream_t st) {
    if (I.n) hipLaunchKernelGGL(k_ing_status8, dim3(cdiv(I.n, 256)), dim3(256), 0, st, I, dst);
}
void launch_ingest_prep(const DevState& S, const IngestBatch& I, hipStream_t st) {
    if (I.n) hipLaunchKernelGGL(k_ing_prep, dim3(cdiv(I.n, 256)), dim3(256), 0, st, S, I);
}
void launch_ingest_need(const DevState& S, const IngestBatch& I, hipStream_t st) {
    hipLaunchKernelGGL(k_ing_need, dim3(cdiv(S.nb, 4)), dim3(256), 0, st, S, I);
}
void launch_ingest_fix(const DevState& S, const IngestBatch& I, const uint32_t* fix, uint32_t n_fix, hipStream_t st) {
    if (n_fix) hipLaunchKernelGGL(k_ing_fix, dim3(cdiv(n_fix, 256)), dim3(256), 0, st, S, I, fix, n_fix);
}
int launch_ingest_sort(const DevState& S, const IngestBatch& I, void* tmp, size_t tmp_bytes, uint32_t key_bits,
                       hipStream_t st) {
    if (!I.n) return 0;
    rocprim::counting_iterator<uint32_t> it(0u);
    if (rocprim::radix_sort_pairs(tmp, tmp_bytes, I.keys, I.keys_sorted, it, I.idx_sorted, I.n, 0u, key_bits, st) !=
        hipSuccess)
        return -1;
    hipLaunchKernelGGL(k_ing_ranges, dim3(cdiv(I.n, 256)), dim3(256), 0, st, S, I);
    return 0;
}
void launch_ingest_apply(const DevState& S, const IngestBatch& I, hipStream_t st) {
    hipLaunchKernelGGL(k_ing_apply, dim3(cdiv(S.nb, APPLY_WAVES)), dim3(64 * APPLY_WAVES), 0, st, S, I);
}
void launch_node_refs(const DevState& S, const uint32_t* slots, uint32_t n, uint32_t* refs, hipStream_t st) {
    if (n) hipLaunchKernelGGL(k_node_refs, dim3(cdiv(n, 4)), dim3(256), 0, st, S, slots, n, refs);
}
void launch_cni_assign(const DevState& S, const int32_t* handles, const uint32_t* ips, const uint8_t* wr, uint32_t n,
                       int32_t* status, uint32_t* rejected, hipStream_t st) {
    if (n) hipLaunchKernelGGL(k_cni_assign, dim3(cdiv(n, 256)), dim3(256), 0, st, S, handles, ips, wr, n, status, rejected);
}

}  // namespace kwok
