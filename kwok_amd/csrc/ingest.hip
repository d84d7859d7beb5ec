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
//                 creation time, handle -> owned bucket, spec.nodeName -> its
//                 bucket), the statuses that need no state.
//   bucket sort   a stable counting sort of the batch by bucket, every bucket's
//                 range (k_bs_*; rocprim's radix sort past 8447 local buckets).
//   k_ing_need    live pods + creates of every bucket with creates (growth check).
//   k_ing_apply   one wave per bucket, its records in event order: the slot
//                 policy (lowest free slot, canonical), coalescing by applying
//                 each record to the state in order, a by-name create's node
//                 resolved in the bucket's node directory (a placeholder entry
//                 if it has none), node references (a deleted node's entry
//                 lives while pods reference it, node_controller.go:265-269),
//                 ingest-time IP release (ipPool.Put, pod_controller.go:329-336),
//                 statuses and handles.
//
// Node batches (kwok_ingest_nodes, node_controller.go:256-270) take the same
// shape over the device-side node directory (node_key / node_name): k_nd_prep
// (record checks, names copied and hashed; statuses that need the host's string
// work are completed by k_nd_fix), the same stable sort, and k_nd_apply, one wave
// per bucket in event order (lookup, lowest free entry, managed-set counts,
// references of a deleted node).
//
// Records are 48-byte kwok_pod_event; the per-record work is a handful of
// loads and stores, so the batch is bound by its H2D copy and by the serial
// chain of one bucket's records (~500 per bucket at 2M records over 4096
// buckets), not by HBM bandwidth.
#include <hip/hip_runtime.h>

#include <cstddef>
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
// The compact records (kwok_pod_rec, kwok_pod_rec12): their strings were parsed
// by the caller, so only the checks on values remain; a create names its node by
// handle.  kwok_pod_rec12 carries one value word: KWOK_REC_HOST_NODE_IP stands
// for the engine's node_ip, a create's value is its creationTimestamp (no
// podIP), any other record's its podIP (an update keeps the pod's creation
// time: REC_KEEP_CTIME).  Returns whether the record is a KWOK_REC_NEW one.
__device__ bool prep_packed(const DevState& S, const IngestBatch& I, uint32_t i) {
    uint32_t w0, ctime, hip, pip;
    int32_t target;
    bool keep = false;
    if (I.packed == 2) {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(I.ev) + (size_t)i * sizeof(kwok_pod_rec12));
        w0 = w[0], target = (int32_t)w[1];  // 12 bytes: three dwords
        const uint32_t val = w[2];
        hip = (w0 & KWOK_REC_HOST_NODE_IP) ? S.node_ip : 0u;
        w0 &= ~KWOK_REC_HOST_NODE_IP;
        const bool nw = (w0 & KWOK_REC_NEW) != 0;
        ctime = nw ? val : 0u;
        pip = nw ? 0u : val;
        keep = !nw;
    } else {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(I.ev) + (size_t)i * sizeof(kwok_pod_rec));
        w0 = w[0], target = (int32_t)w[1], ctime = w[2], hip = w[3], pip = w[4];  // 20 bytes: five dwords
    }
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
    r.is_new = create ? 1 : 0;
    r.pad[0] = r.pad[1] = r.pad[2] = 0;
    int st = 1;  // 1: the apply pass decides
    if (op == KWOK_OP_DELETE) {
        if (pip) r.pip = pip, r.chk |= REC_DEL_IP;
    } else if (op == KWOK_OP_UPSERT) {
        r.hip = hip, r.pip = pip;
        if (spec >= I.n_specs) r.fst = KWOK_EINVAL;
        else if (r.phase > KWOK_PHASE_UNKNOWN) r.fst = KWOK_EINVAL;
        else r.ctime = ctime, r.spec = (uint16_t)spec;
        if (keep) r.chk |= REC_KEEP_CTIME;
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
    I.rec[i] = r;
    I.keys[i] = st == 1 ? r.bucket : S.nb;
    if (st != 1) {
        I.out_handle[i] = -1;
        I.out_status[i] = st;
        I.out_released[i] = 0;
        if (st != KWOK_OK) atomicAdd(&I.sum->rejected, 1u);
    }
    return create != 0;
}

__global__ void k_ing_prep(DevState S, IngestBatch I) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (I.packed) {
        const bool nw = i < I.n && prep_packed(S, I, i);
        if (I.tile_new) {  // kwok_pod_rec12: the block's creates (blocks are the batch's 256-record tiles)
            const int c = __syncthreads_count(nw);
            if (threadIdx.x == 0) I.tile_new[I.tile0 + blockIdx.x] = (uint32_t)c;
        }
        return;
    }
    if (i >= I.n) return;
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
    r.is_new = 0;
    r.pad[0] = r.pad[1] = r.pad[2] = 0;
    int st = 1;  // 1: the apply pass decides
    auto in_arena = [&](kwok_str s) { return (uint64_t)s.off + s.len <= I.arena_len; };
    if (x.reserved0) {
        st = (int8_t)x.reserved0;  // a record the GPU codec could not decode (kwok_ingest_pods_json)
    } else if (!in_arena(x.node_name) || !in_arena(x.host_ip) || !in_arena(x.pod_ip)) {
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
                else r.bucket = b - S.b_lo, atomicAdd(&I.sum->n_byname, 1u);
            }
        }
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
// k_ing_need: one wave per bucket, after the sort: the creates among the
// bucket's records (an UPSERT without a handle) + its live pods (USED below the
// fill mark) -> the batch's growth need (max over buckets with creates; an upper
// bound: the batch's deletes are not netted out).  (Counting the creates here
// instead of with a global atomic per create in k_ing_prep: 0.5M creates over
// 4096 counters held the prep ~40 us.)
static_assert(offsetof(PodRec, spec) == 20 && offsetof(PodRec, op) == 22 && offsetof(PodRec, chk) == 25,
              "k_ing_need reads op and chk as the words at bytes 20 and 24 of a PodRec");
__global__ void k_ing_need(DevState S, IngestBatch I) {
    const uint32_t b = blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6);
    if (b >= S.nb) return;
    const uint32_t pbeg = I.beg[b], pend = I.end[b], fill0 = S.pod_fill[b];
    if (!(pbeg < pend && pend <= I.n && I.keys_sorted[pbeg] == b)) return;  // (a stale range: not this batch's)
    // the fill mark bounds the live pods and the bucket's records its creates: when
    // that bound fits, the bucket cannot overflow
    if (fill0 + (pend - pbeg) <= S.cp) return;
    uint32_t c = 0;
    for (uint32_t p0 = pbeg; p0 < pend; p0 += 64 * 8) {  // (eight records per lane in flight)
        uint32_t ix[8], w0[8], w1[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t p = p0 + 64 * q + lane();
            ix[q] = p < pend ? I.idx_sorted[p] : ~0u;
        }
#pragma unroll
        for (int q = 0; q < 8; q++) {  // PodRec bytes 20..27: spec, op, phase | flags, chk, fst, pst
            const uint32_t* rw = reinterpret_cast<const uint32_t*>(I.rec + (ix[q] != ~0u ? ix[q] : 0u)) + 5;
            w0[q] = ix[q] != ~0u ? rw[0] : 0u;
            w1[q] = ix[q] != ~0u ? rw[1] : 0u;
        }
#pragma unroll
        for (int q = 0; q < 8; q++)
            c += ix[q] != ~0u && ((w0[q] >> 16) & 0xFFu) == KWOK_OP_UPSERT && !((w1[q] >> 8) & REC_EXISTING);
    }
    for (int o = 32; o; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o);
    if (!c) return;
    // live pods: the bucket's state words below the fill mark, 8 per lane-load
    const uint32_t fill = fill0;
    const uint16_t* ps = S.pod_state + (size_t)b * S.cp;  // (cp and fill are multiples of 8: 16-byte aligned rows)
    uint32_t live = 0;
    for (uint32_t s0 = lane() * 8; s0 < fill; s0 += 64 * 8 * 4) {
        uint4 v[4];
#pragma unroll
        for (int q = 0; q < 4; q++)
            v[q] = s0 + q * 512 < fill ? *reinterpret_cast<const uint4*>(ps + s0 + q * 512) : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t w[4] = {v[q].x, v[q].y, v[q].z, v[q].w};
#pragma unroll
            for (int j = 0; j < 4; j++) live += (w[j] & PS_USED) + ((w[j] >> 16) & PS_USED);
        }
    }
    for (int o = 32; o; o >>= 1) live += (uint32_t)__shfl_xor((int)live, o);
    // only a bucket that would overflow raises the need (one device-scope atomic on one
    // word from each of 4096 waves cost ~50 us)
    if (lane() == 0 && live + c > S.cp) atomicMax(&I.sum->need, live + c);
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

// ---- node directory (device.h): one wave owns a bucket's entries at a time ----
__device__ __forceinline__ uint64_t name_key(uint32_t h, uint32_t len) { return (uint64_t)h | ((uint64_t)len << 32); }
// lane l's 4 name bytes (zero past len) from any alignment
__device__ __forceinline__ uint32_t name_word(const uint8_t* nm, uint32_t len, uint32_t o) {
    uint32_t w = 0;
    for (uint32_t j = 0; j < 4; j++)
        if (o + j < len) w |= (uint32_t)nm[o + j] << (8 * j);
    return w;
}
// do node entry g's name bytes equal nm's (len bytes)?  (coherent loads: this wave may have written them)
__device__ bool name_eq(const DevState& S, size_t g, const uint8_t* nm, uint32_t len) {
    const uint32_t o = lane() * 4;
    bool bad = false;
    if (o < len) bad = ld_coh(reinterpret_cast<const uint32_t*>(S.node_name + g * NAME_STRIDE + o)) != name_word(nm, len, o);
    return !__ballot(bad);
}
// the index of bucket b's entry named nm, or -1.  The bucket's keys are loaded
// DIR_UNROLL x 64 at a time (one round trip for buckets of up to 512 entries)
constexpr uint32_t DIR_UNROLL = 8;
__device__ int32_t dir_find(const DevState& S, uint32_t b, uint64_t key, const uint8_t* nm, uint32_t len) {
    const size_t nbase = (size_t)b * S.cn;
    for (uint32_t j0 = 0; j0 < S.cn; j0 += 64 * DIR_UNROLL) {
        uint64_t k[DIR_UNROLL];
#pragma unroll
        for (uint32_t u = 0; u < DIR_UNROLL; u++) {
            const uint32_t j = j0 + u * 64 + lane();
            k[u] = j < S.cn ? ld_coh(S.node_key + nbase + j) : 0ull;
        }
#pragma unroll
        for (uint32_t u = 0; u < DIR_UNROLL; u++) {
            uint64_t m = __ballot(k[u] == key);
            while (m) {
                const uint32_t c = j0 + u * 64 + (uint32_t)__builtin_ctzll(m);
                if (name_eq(S, nbase + c, nm, len)) return (int32_t)c;
                m &= m - 1;
            }
        }
    }
    return -1;
}
// the lowest free entry of bucket b (no NS_SLOT; the host's first_free of round 3), or -1
__device__ int32_t dir_free(const DevState& S, uint32_t b) {
    const size_t nbase = (size_t)b * S.cn;
    for (uint32_t j0 = 0; j0 < S.cn; j0 += 64) {
        const uint32_t j = j0 + lane();
        const uint64_t m = __ballot(j < S.cn && !(ld8_coh(S.node_state + nbase + j) & NS_SLOT));
        if (m) return (int32_t)(j0 + (uint32_t)__builtin_ctzll(m));
    }
    return -1;
}
// entry g takes the name (its state is the caller's)
__device__ void dir_write(const DevState& S, size_t g, uint64_t key, const uint8_t* nm, uint32_t len) {
    const uint32_t o = lane() * 4;
    if (o < len) *reinterpret_cast<uint32_t*>(S.node_name + g * NAME_STRIDE + o) = name_word(nm, len, o);
    if (lane() == 0) S.node_key[g] = key;
}
// entry g goes (no name, no state, no blob)
__device__ __forceinline__ void dir_clear(const DevState& S, size_t g) {
    if (lane() == 0) {
        S.node_key[g] = 0;
        S.node_state[g] = 0;
        S.node_blob[g] = 0;
    }
}
// does a live pod of bucket b (pods below its fill mark) reference node index nd?
// (node batches: no pod changes during one, plain loads)
__device__ bool pods_reference(const DevState& S, uint32_t b, uint32_t nd) {
    constexpr uint32_t U = 4;  // 512-slot steps whose loads are in flight together
    const uint32_t fill = S.pod_fill[b];
    const size_t sb = (size_t)b * S.cp;
    for (uint32_t s0 = 0; s0 < fill; s0 += 512 * U) {
        uint4 st[U], ndw[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t s = s0 + u * 512 + lane() * 8;
            st[u] = ndw[u] = make_uint4(0, 0, 0, 0);
            if (s < fill) {
                st[u] = *reinterpret_cast<const uint4*>(S.pod_state + sb + s);
                ndw[u] = *reinterpret_cast<const uint4*>(S.pod_node + sb + s);
            }
        }
        bool h = false;
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint32_t a[4] = {st[u].x, st[u].y, st[u].z, st[u].w}, q[4] = {ndw[u].x, ndw[u].y, ndw[u].z, ndw[u].w};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                h |= (a[k] & PS_USED) && (q[k] & 0xFFFFu) == nd;
                h |= ((a[k] >> 16) & PS_USED) && (q[k] >> 16) == nd;
            }
        }
        if (__ballot(h)) return true;
    }
    return false;
}
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
    __shared__ uint8_t dtag_all[APPLY_WAVES][1024];  // a chunk's slots named twice? (lane ids by slot hash)
    const uint32_t w = threadIdx.x >> 6, l = lane();
    const uint32_t b = blockIdx.x * APPLY_WAVES + w;
    if (I.spec) {
        // queued ahead of the host's growth check: a chunk that could fill a bucket (or
        // follows one that could) changes nothing; the host grows and applies it again
        const bool over = I.sum->need > S.cp;
        if (over && blockIdx.x == 0 && threadIdx.x == 0) *I.abort = 1u;
        if (over || __hip_atomic_load(I.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    }
    if (b >= S.nb) return;
    const uint32_t pbeg = I.beg[b], pend = I.end[b];
    if (pbeg >= pend || pend > I.n || I.keys_sorted[pbeg] != b) return;  // (stale ranges: k_nd_apply)
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
    // the next chunk's records (idx_sorted / rec are this pass's inputs: no hazard),
    // loaded one chunk ahead so that a chunk waits on its state loads only
    uint32_t nidx = 0;
    uint4 na = make_uint4(0, 0, 0, 0), nb = na;
    auto fetch = [&](uint32_t q0) {
        const uint32_t p = q0 + l;
        nidx = 0;
        na = nb = make_uint4(0, 0, 0, 0);
        if (p < pend) {
            nidx = I.idx_sorted[p];
            const uint4* rp = reinterpret_cast<const uint4*>(I.rec + nidx);
            na = rp[0];
            nb = rp[1];
        }
    };
    fetch(pbeg);
    // occupancy bitmap of [0, fill): pod_state's USED bits (8 slots per 16-byte
    // load, a lane's 8 loads in flight together)
    for (uint32_t q = l; q < B.nw; q += 64) {
        uint4 vs[8];
#pragma unroll
        for (uint32_t g = 0; g < 8; g++) {
            const uint32_t s = q * 64 + g * 8;
            vs[g] = s < B.fill ? *reinterpret_cast<const uint4*>(S.pod_state + B.sbase + s) : make_uint4(0, 0, 0, 0);
        }
        uint64_t word = 0;
#pragma unroll
        for (uint32_t g = 0; g < 8; g++) {
            const uint32_t u[4] = {vs[g].x, vs[g].y, vs[g].z, vs[g].w};
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
    uint32_t rejected = 0, n_freed = 0, n_ph = 0;
    int32_t dzb = 0;  // zombie entries made (placeholders) and freed
    bool foreign = false;
    uint32_t p0 = pbeg;
    for (; p0 < pend; p0 += 64) {
        mem_sync();  // the previous chunk's stores, before this chunk's (coherent) loads
        const uint32_t p = p0 + l;
        const bool v = p < pend;
        const uint32_t idx = nidx;
        const uint4 ra = na, rb = nb;
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
        if (p0 + 64 < pend) fetch(p0 + 64);
        // ---- parallel path: a chunk in which no record can see another's effect
        // except through the creates' slot order (no DELETE, no by-name create, no
        // slot named twice, no existing record on a free slot beside creates, enough
        // free slots for every create: no node entry can go) ----
        {
            const uint32_t op = (hop >> 16) & 0xFFu, fl = hfl & 0xFFu;
            const int fst = (int)(int8_t)((hfl >> 16) & 0xFFu);
            const bool act = v;
            const bool exl = act && (chk & REC_EXISTING);
            const bool used = exl && pos < B.cp && ((B.bm[pos >> 6] >> (pos & 63)) & 1);
            const bool crt = act && !exl;  // (prep decided creates with a bad field, or foreign / unknown)
            const bool take = crt && (ns0 & NS_SLOT);
            // a slot named by two records of the chunk: each lane writes its id at its slot's
            // hash; a lane that reads another's id shares the hash, and one ballot per
            // such slot value finds whether two lanes name it (a few rounds, not 63)
            bool dup = false;
            {
                uint8_t* tg = dtag_all[w];
                if (exl) tg[pos & 1023u] = (uint8_t)l;
                lds_sync();
                uint64_t todo = __ballot(exl && tg[pos & 1023u] != (uint8_t)l);
                while (todo && !dup) {
                    const uint32_t kl = rdl(pos, (uint32_t)__builtin_ctzll(todo));
                    const uint64_t m = __ballot(exl && pos == kl);
                    dup = __popcll(m) > 1;
                    todo &= ~m;
                }
            }
            bool par = !__ballot((act && !exl && (chk & REC_BY_NAME)) || (act && op == KWOK_OP_DELETE)) && !dup &&
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
                    if (!(exl && (chk & REC_KEEP_CTIME))) S.pod_ctime[g] = rb.x;
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
            // a create naming its node by spec.nodeName: the bucket's entry of that name
            // now (after the records before it), or a placeholder entry the pod references
            // (the oracle's node_entry); EFULL when the bucket has no free entry
            const bool byname = !existing && (kchk & REC_BY_NAME) && kop == KWOK_OP_UPSERT && fst == KWOK_OK;
            int bst = KWOK_OK;
            uint32_t bnd = kpos;
            if (byname) {
                const kwok_str nr = static_cast<const kwok_pod_event*>(I.ev)[kidx].node_name;
                const uint8_t* nm = I.arena + nr.off;
                const uint64_t key = name_key(d_fnv1a32(nm, nr.len), nr.len);
                mem_sync();
                int32_t r = dir_find(S, b, key, nm, nr.len);
                if (r < 0) {
                    r = dir_free(S, b);
                    if (r < 0) {
                        bst = KWOK_EFULL;
                    } else {
                        dir_write(S, B.nbase + r, key, nm, nr.len);
                        if (l == 0) {
                            S.node_state[B.nbase + r] = NS_SLOT;
                            S.node_blob[B.nbase + r] = 0;
                        }
                        dzb++, n_ph++;
                        if (wfreed == (uint32_t)r) wfreed = ~0u;  // the index holds an entry again
                    }
                }
                if (r >= 0) {
                    bnd = (uint32_t)r;
                    mem_sync();
                    ns = ld8_coh(S.node_state + B.nbase + bnd);
                }
            } else {
                if (nd != rdl(nd0, k) && nd < B.cn) {  // the slot's node changed in this chunk: its state now
                    mem_sync();
                    ns = ld8_coh(S.node_state + B.nbase + nd);
                }
                if (nd < B.cn) {
                    const uint64_t m = __ballot(wfreed == nd);
                    if (m) ns = 0;  // freed by an earlier record of this chunk
                }
            }
            auto free_node = [&](uint32_t n) {  // the node entry goes (free_node_if_unused)
                dir_clear(S, B.nbase + n);
                dzb--, n_freed++;  // (a zombie: NS_SLOT without NS_EXISTS)
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
                stt = fst != KWOK_OK ? fst : bst;
                uint32_t slot = kpos;
                if (stt == KWOK_OK && !existing) {
                    nd = bnd;  // the node's index (by handle, or resolved by name above)
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
                        if (!(existing && (kchk & REC_KEEP_CTIME))) S.pod_ctime[g] = rdl(rb.x, k);
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
        if (dzb) S.zb_count[b] += (uint32_t)dzb;
        if (rejected) atomicAdd(&I.sum->rejected, rejected);
        if (n_freed) atomicAdd(&I.sum->n_freed, n_freed);
        if (n_ph) atomicAdd(&I.sum->n_placeholders, n_ph);
    }
    if (__ballot(foreign) && l == 0) {
        atomicOr(&I.sum->foreign, 1u);
    }
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


// ===========================================================================
// Node batches: the WatchNodes / ListNodes event switch (node_controller.go:
// 256-270) over the device node directory.
// ===========================================================================
// k_nd_prep: one thread per record.  Name bounds (1..253 bytes inside the
// arena), op, the status strings inside the arena; the name copied to
// names[i * NAME_STRIDE] and hashed (its bucket; another rank's: ENOTMINE).  An
// UPSERT with an empty status renders the empty-status blob (kwok's own fleets);
// any other status (or a custom node template) is completed by the host
// (string checks, blob, CONFORMS: k_nd_fix) before the sort.
__global__ void k_nd_prep(DevState S, NodeBatch N) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N.n) return;
    const kwok_node_event x = N.ev[i];
    NodeRec r;
    r.hash = 0;
    r.len = 0;
    r.op = x.op;
    r.fl = (uint8_t)((x.managed ? NR_MANAGED : 0) | (x.lockable ? NR_LOCKABLE : 0));
    r.pad = 0;
    r.blob = 0;
    auto in_arena = [&](kwok_str q) { return (uint64_t)q.off + q.len <= N.arena_len; };
    int st = 1;  // 1: the apply pass decides
    bool host = false, mine = false;
    uint32_t bucket = S.nb;
    if (!x.name.len || x.name.len > NODE_NAME_MAX || !in_arena(x.name)) {
        st = KWOK_EDOMAIN;
    } else if (x.op != KWOK_OP_DELETE && x.op != KWOK_OP_UPSERT) {
        st = KWOK_EINVAL;
    } else {
        bool inside = true, empty = true;
        if (x.op == KWOK_OP_UPSERT) {
            const kwok_str* q = &x.addresses;  // addresses, allocatable, capacity, node_info[]
            for (int k = 0; k < 3 + KWOK_NI_COUNT; k++) inside &= in_arena(q[k]), empty &= q[k].len == 0;
        }
        if (!inside) {
            st = KWOK_EDOMAIN;
        } else {
            // the name by aligned dwords (a batch read in place crosses the link: one
            // round trip for a name of up to 61 bytes instead of one per byte), copied
            // and hashed; longer names byte by byte
            const uint8_t* nm = N.arena + x.name.off;
            uint8_t* dst = N.names + (size_t)i * NAME_STRIDE;
            uint32_t h = 0x811C9DC5u;
            const uintptr_t p0 = reinterpret_cast<uintptr_t>(nm);
            const uint32_t lead = (uint32_t)(p0 & 3u), nw = (lead + x.name.len + 3u) / 4u;
            constexpr uint32_t NW = 16;
            if (nw <= NW) {
                const uint32_t* src = reinterpret_cast<const uint32_t*>(p0 & ~(uintptr_t)3);
                uint32_t wv[NW + 1];
#pragma unroll
                for (uint32_t q = 0; q < NW; q++) wv[q] = q < nw ? src[q] : 0u;
                wv[NW] = 0u;
#pragma unroll
                for (uint32_t q = 0; q < NW; q++) {
                    if (4 * q >= x.name.len) break;
                    const uint32_t w = lead ? __builtin_amdgcn_alignbit(wv[q + 1], wv[q], 8 * lead) : wv[q];
                    *reinterpret_cast<uint32_t*>(dst + 4 * q) = w;
#pragma unroll
                    for (uint32_t c = 0; c < 4; c++)
                        if (4 * q + c < x.name.len) h = (h ^ ((w >> (8 * c)) & 0xFFu)) * 0x01000193u;
                }
            } else {
                for (uint32_t j = 0; j < x.name.len; j++) {
                    const uint8_t c = nm[j];
                    dst[j] = c;
                    h = (h ^ c) * 0x01000193u;
                }
            }
            r.hash = h;
            r.len = (uint8_t)x.name.len;
            const uint32_t b = h & (S.buckets - 1);
            mine = b >= S.b_lo && b < S.b_lo + S.nb;
            if (mine) bucket = b - S.b_lo;
            host = x.op == KWOK_OP_UPSERT && (!empty || N.host_all);
            if (host) {
                r.pad = mine ? 0 : 1;  // the host's string checks come first; then ENOTMINE (k_nd_fix)
                N.host_idx[atomicAdd(&N.sum->n_host, 1u)] = i;
            } else if (!mine) {
                st = KWOK_ENOTMINE;
            } else if (x.op == KWOK_OP_UPSERT) {
                r.blob = N.empty_blob;  // an empty status: no CONFORMS (addresses etc. are absent, A.5)
            }
        }
    }
    if (host) r.fl |= NR_HOST;
    N.rec[i] = r;
    N.keys[i] = st == 1 && mine ? bucket : S.nb;
    if (st != 1) {
        N.out_handle[i] = -1;
        N.out_status[i] = st;
        if (st != KWOK_OK) atomicAdd(&N.sum->rejected, 1u);
    }
}

// the host's completions: a status (the record changes nothing) or blob + CONFORMS
__global__ void k_nd_fix(DevState S, NodeBatch N, const NodeFix* fix, uint32_t n_fix) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_fix) return;
    const NodeFix f = fix[k];
    const uint32_t i = f.idx;
    const bool foreign = N.rec[i].pad != 0;
    if (f.status != KWOK_OK || foreign) {
        N.out_handle[i] = -1;
        N.out_status[i] = f.status != KWOK_OK ? f.status : KWOK_ENOTMINE;
        N.keys[i] = S.nb;
        atomicAdd(&N.sum->rejected, 1u);
    } else {
        N.rec[i].blob = f.blob;
        if (f.conforms) N.rec[i].fl = (uint8_t)(N.rec[i].fl | NR_CONFORMS);
    }
}

__global__ void k_nd_ranges(DevState S, NodeBatch N) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N.n) return;
    const uint32_t k = N.keys_sorted[p];
    if (k >= S.nb) return;
    if (p == 0 || N.keys_sorted[p - 1] != k) N.beg[k] = p;
    if (p + 1 == N.n || N.keys_sorted[p + 1] != k) N.end[k] = p + 1;
}

// k_nd_apply: one wave per bucket, its records in event order (the round-3 host
// pass, engine.cpp, restated per bucket: slots, names and states are per bucket)
__global__ __launch_bounds__(64 * APPLY_WAVES) void k_nd_apply(DevState S, NodeBatch N) {
    const uint32_t l = lane();
    const uint32_t b = blockIdx.x * APPLY_WAVES + (threadIdx.x >> 6);
    if (b >= S.nb) return;
    // the bucket's records: k_nd_ranges wrote beg / end of the buckets present; a
    // bucket absent from this batch may hold an older batch's range, which no
    // sorted key of this batch matches (no memset of the ranges per batch)
    const uint32_t pbeg = N.beg[b], pend = N.end[b];
    if (pbeg >= pend || pend > N.n || N.keys_sorted[pbeg] != b) return;
    if (!N.force && N.sum->n_host) return;  // the host completes records first, then launches this again
    const size_t nbase = (size_t)b * S.cn;
    int32_t dman = 0, dzb = 0;
    uint32_t rejected = 0, freed = 0, created = 0;
    bool changed = false;
    for (uint32_t p = pbeg; p < pend; p++) {
        const uint32_t idx = N.idx_sorted[p];
        const NodeRec r = N.rec[idx];
        const uint8_t* nm = N.names + (size_t)idx * NAME_STRIDE;
        const uint64_t key = name_key(r.hash, r.len);
        mem_sync();  // this wave's stores of the records before, ahead of its coherent loads
        int32_t nd = dir_find(S, b, key, nm, r.len);
        int st = KWOK_OK;
        int32_t handle = -1;
        if (r.op == KWOK_OP_DELETE) {
            // node_controller.go:265-269: Deleted -> nodesSets.Delete; the entry lives
            // while pods reference it (a zombie), else it goes
            if (nd < 0) {
                st = KWOK_ENOTFOUND;
            } else {
                const size_t g = nbase + (uint32_t)nd;
                const uint32_t ns = ld8_coh(S.node_state + g);
                if (ns & NS_MANAGED) dman--, changed = true;
                const bool zombie = (ns & NS_SLOT) && !(ns & NS_EXISTS);
                if (!pods_reference(S, b, (uint32_t)nd)) {
                    dir_clear(S, g);
                    dzb -= zombie ? 1 : 0;
                    freed++;
                } else {
                    if (l == 0)
                        S.node_state[g] = (uint8_t)(ns & ~(NS_EXISTS | NS_MANAGED | NS_EVENT_LOCK | NS_CONFORMS | NS_LOCKABLE));
                    dzb += zombie ? 0 : 1;
                }
                handle = (int32_t)((S.b_lo + b) * S.cn + (uint32_t)nd);
            }
        } else {
            // Added / Modified: the entry (a new one at the lowest free index), then
            // needHeartbeat -> nodesSets.Put (never undone but by Delete), needLockNode
            // -> the lock queue (:256-264)
            uint32_t ns = 0;
            if (nd < 0) {
                nd = dir_free(S, b);
                if (nd < 0) st = KWOK_EFULL;
                else dir_write(S, nbase + (uint32_t)nd, key, nm, r.len), created++;
            } else {
                ns = ld8_coh(S.node_state + nbase + (uint32_t)nd);
            }
            if (st == KWOK_OK) {
                const size_t g = nbase + (uint32_t)nd;
                if ((ns & NS_SLOT) && !(ns & NS_EXISTS)) dzb--;  // a zombie exists again
                const bool put = (r.fl & NR_MANAGED) && !(ns & NS_MANAGED);
                if (put) dman++, changed = true;
                const bool managed = (ns & NS_MANAGED) || (r.fl & NR_MANAGED);
                const bool lock = (r.fl & NR_MANAGED) && (r.fl & NR_LOCKABLE);
                const uint32_t bits = NS_SLOT | NS_EXISTS | (managed ? NS_MANAGED : 0) | ((r.fl & NR_LOCKABLE) ? NS_LOCKABLE : 0) |
                                      ((r.fl & NR_CONFORMS) ? NS_CONFORMS : 0) | (lock ? NS_EVENT_LOCK : 0);
                if (l == 0) {
                    S.node_state[g] = (uint8_t)((ns & (lock ? 0u : (uint32_t)NS_EVENT_LOCK)) | bits);
                    S.node_blob[g] = r.blob;
                }
                handle = (int32_t)((S.b_lo + b) * S.cn + (uint32_t)nd);
            }
        }
        if (st != KWOK_OK) rejected++;
        if (l == 0) {
            N.out_handle[idx] = handle;
            N.out_status[idx] = st;
        }
    }
    if (l == 0) {
        if (dman) S.mb_count[b] += (uint32_t)dman;
        if (dzb) S.zb_count[b] += (uint32_t)dzb;
        if (dman) atomicAdd(&N.sum->d_managed, dman);
        if (changed) atomicOr(&N.sum->changed, 1u);
        if (rejected) atomicAdd(&N.sum->rejected, rejected);
        if (freed) atomicAdd(&N.sum->freed, freed);
        if (created) atomicAdd(&N.sum->created, created);
    }
}

// after a tick that deleted pods: zombie entries (deleted nodes, placeholders) no
// live pod references any more go, as the last pod's removal at ingest frees them
// (one wave per bucket holding zombies)
__global__ __launch_bounds__(256) void k_free_zombies(DevState S) {
    const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (b >= S.nb || S.zb_count[b] == 0) return;
    const size_t nbase = (size_t)b * S.cn;
    uint32_t gone = 0;
    for (uint32_t j0 = 0; j0 < S.cn; j0 += 64) {
        const uint32_t j = j0 + lane();
        uint32_t ns = j < S.cn ? S.node_state[nbase + j] : 0u;
        uint64_t m = __ballot((ns & NS_SLOT) && !(ns & NS_EXISTS));
        while (m) {
            const uint32_t c = j0 + (uint32_t)__builtin_ctzll(m);
            m &= m - 1;
            if (!pods_reference(S, b, c)) dir_clear(S, nbase + c), gone++;
        }
    }
    if (gone && lane() == 0) S.zb_count[b] -= gone;
}

// heartbeat handle bases: hb_pre[c] = managed nodes of the buckets before chain
// block c's range [nb*c/Gc, ...); hb_pre[Gc] = all; bpre[bk] = managed nodes of
// the buckets before bucket bk, bpre[nb] = all (one block)
__global__ __launch_bounds__(1024) void k_hb_pre(DevState S, uint32_t* pre, uint32_t* bpre) {
    __shared__ uint32_t part[1024];
    const uint32_t t = threadIdx.x, T = blockDim.x, nc = S.n_chain;
    auto lo = [&](uint32_t c) { return (uint32_t)((uint64_t)S.nb * c / nc); };
    const uint32_t c0 = (uint32_t)((uint64_t)nc * t / T), c1 = (uint32_t)((uint64_t)nc * (t + 1) / T);
    uint32_t sum = 0;
    for (uint32_t bk = lo(c0); bk < lo(c1); bk++) sum += S.mb_count[bk];
    part[t] = sum;
    __syncthreads();
    for (uint32_t o = 1; o < T; o <<= 1) {  // inclusive scan
        const uint32_t v = t >= o ? part[t - o] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint32_t acc = part[t] - sum;
    for (uint32_t c = c0; c < c1; c++) {
        pre[c] = acc;
        for (uint32_t bk = lo(c); bk < lo(c + 1); bk++) {
            bpre[bk] = acc;
            acc += S.mb_count[bk];
        }
    }
    if (t == T - 1) pre[nc] = bpre[S.nb] = acc;
}

// kwok_node_has: one wave per name
__global__ void k_node_lookup(DevState S, const uint8_t* names, const uint32_t* lens, uint32_t n, uint32_t* out) {
    const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;
    const uint8_t* nm = names + (size_t)i * NAME_STRIDE;
    const uint32_t len = lens[i];
    uint32_t res = 0;
    if (len && len <= NODE_NAME_MAX) {
        const uint32_t h = d_fnv1a32(nm, len), b = h & (S.buckets - 1);
        if (b >= S.b_lo && b < S.b_lo + S.nb) {
            const int32_t nd = dir_find(S, b - S.b_lo, name_key(h, len), nm, len);
            if (nd >= 0) res = S.node_state[(size_t)(b - S.b_lo) * S.cn + (uint32_t)nd];
        }
    }
    if (lane() == 0) out[i] = res;
}

inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

}  // namespace

// ---------------------------------------------------------------------------
// The stable sort by bucket: a counting sort over the batch's keys (local
// buckets 0..nb, nb = nothing to apply), in tiles of BS_TILE records.
//   k_bs_hist     per tile: its key counts (LDS histogram) -> hist[tile][key]
//   k_bs_cols     per key: the exclusive prefix over the tiles, in place; the total
//   k_bs_scatter  per tile: the exclusive scan of the totals (each key's first
//                 sorted position; block 0 writes every bucket's range [beg, end)),
//                 then the tile's W waves take a sub-tile each (the key's records in the
//                 earlier sub-tiles counted first), its records in order, 64 at a time:
//                 the lanes of a key (LDS tags, a ballot per shared key) take consecutive positions after
//                 the key's running count in LDS -> idx_sorted (keys_sorted only at
//                 each bucket's first position: what the range checks read; the
//                 records land ~1 per bucket per tile, so every store is a line of
//                 its own and the fewer the better)
// Every global input of a block is loaded in unrolled batches (a strided loop
// with one load per trip waits out one round trip per trip).
// Three small launches instead of rocPRIM's radix sort, which on these batches
// (12-bit keys, 0.7-1.3M records) ran the onesweep path at ~75 us or its block
// merge sort path at ~120 us (17 launches).  Every bucket's range is written, so
// no range of an earlier batch survives (k_ing_ranges / k_nd_ranges are not run).
// ---------------------------------------------------------------------------
constexpr uint32_t BS_TILE = 4096;
constexpr uint32_t BS_MAX_KEYS = 8448;  // 8192 local buckets + 1 (k_bs_scatter's LDS: 4 waves past BS_KEYS8 keys, ~135 KB)
struct BucketSort {
    const uint32_t* keys;
    uint32_t n, nk;         // records, keys (nb + 1)
    uint32_t* hist;         // [tiles][nk]
    uint32_t* tot;          // [nk] totals, then each key's base
    uint32_t* keys_sorted;
    uint32_t* idx_sorted;
    uint32_t* beg;          // [nk - 1] bucket ranges
    uint32_t* end;
};
__global__ void k_bs_hist(BucketSort B) {
    extern __shared__ uint32_t h[];
    const uint32_t t = blockIdx.x;
    for (uint32_t k = threadIdx.x; k < B.nk; k += blockDim.x) h[k] = 0;
    const uint32_t i0 = t * BS_TILE, i1 = min(i0 + BS_TILE, B.n);
    constexpr uint32_t R = BS_TILE / 256;  // keys per thread (blockDim 256)
    uint32_t key[R];
#pragma unroll
    for (uint32_t q = 0; q < R; q++) {
        const uint32_t i = i0 + q * 256 + threadIdx.x;
        key[q] = i < i1 ? B.keys[i] : ~0u;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < R; q++)
        if (key[q] != ~0u) atomicAdd(&h[key[q]], 1u);
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < B.nk; k += blockDim.x) B.hist[(size_t)t * B.nk + k] = h[k];
}
// 64 keys per block, their tiles in 16 groups (one wave each): every thread sums
// its group's counts (loads in flight together), the groups' sums are scanned in
// LDS, and the thread writes its group's exclusive prefixes
constexpr uint32_t BS_GROUPS = 16;
__global__ void k_bs_cols(BucketSort B, uint32_t tiles) {
    __shared__ uint32_t gs[BS_GROUPS][64];
    const uint32_t k = blockIdx.x * 64 + lane(), g = threadIdx.x >> 6;
    const uint32_t tpg = (tiles + BS_GROUPS - 1) / BS_GROUPS;
    const uint32_t t0 = min(g * tpg, tiles), t1 = min(t0 + tpg, tiles);
    const bool ok = k < B.nk;
    constexpr uint32_t R = 16;  // a group's counts held in registers (tiles <= 256: 1M records)
    uint32_t v[R], sum = 0;
#pragma unroll
    for (uint32_t q = 0; q < R; q++) v[q] = ok && t0 + q < t1 ? B.hist[(size_t)(t0 + q) * B.nk + k] : 0u;
#pragma unroll
    for (uint32_t q = 0; q < R; q++) sum += v[q];
    if (ok)
        for (uint32_t t = t0 + R; t < t1; t++) sum += B.hist[(size_t)t * B.nk + k];
    gs[g][lane()] = sum;
    __syncthreads();
    uint32_t run = 0, all = 0;
    for (uint32_t q = 0; q < BS_GROUPS; q++) {
        const uint32_t x = gs[q][lane()];
        run += q < g ? x : 0u;
        all += x;
    }
    if (!ok) return;
#pragma unroll
    for (uint32_t q = 0; q < R; q++)
        if (t0 + q < t1) {
            B.hist[(size_t)(t0 + q) * B.nk + k] = run;
            run += v[q];
        }
    for (uint32_t t = t0 + R; t < t1; t++) {
        const uint32_t x = B.hist[(size_t)t * B.nk + k];
        B.hist[(size_t)t * B.nk + k] = run;
        run += x;
    }
    if (g == 0) B.tot[k] = all;
}
// W waves per tile, a sub-tile of BS_TILE / W records each: every wave counts its
// sub-tile's keys (u16 pairs in LDS), the counts become per-wave offsets (the key's
// records in the tile's earlier sub-tiles), and the waves place their records at
// the same time, each in order, 64 at a time (W = 8: 8 rounds per tile, not 64)
template <uint32_t W, uint32_t NKMAX>
__global__ __launch_bounds__(64 * W) void k_bs_scatter(BucketSort B) {
    constexpr uint32_t NT = 64 * W, SUB = BS_TILE / W, IT = SUB / 64, PER = NKMAX / NT;
    __shared__ uint32_t cnt[NKMAX];          // each key's first position in the tile
    __shared__ uint32_t offp[W][NKMAX / 2];  // per wave, per key (u16 pairs): its offset past cnt
    __shared__ uint8_t tag[W][NKMAX];        // per wave: the lane that wrote a key last
    __shared__ uint32_t wsum[W];
    const uint32_t t = blockIdx.x, w = threadIdx.x >> 6, l = lane(), nk = B.nk, nkp = (nk + 1) / 2;
    const uint32_t i0 = t * BS_TILE, i1 = min(i0 + BS_TILE, B.n), s0 = i0 + w * SUB;
    // the key totals and the tile's prefixes (thread th: keys [th * PER, +PER)) and
    // the wave's keys, all loads in flight together
    const uint32_t k0 = threadIdx.x * PER;
    uint32_t tot[PER], hst[PER], key[IT], sum = 0;
#pragma unroll
    for (uint32_t q = 0; q < PER; q++) {
        const bool ok = k0 + q < nk;
        tot[q] = ok ? B.tot[k0 + q] : 0u;
        hst[q] = ok ? B.hist[(size_t)t * nk + k0 + q] : 0u;
    }
#pragma unroll
    for (uint32_t q = 0; q < IT; q++) {
        const uint32_t i = s0 + q * 64 + l;
        key[q] = i < i1 ? B.keys[i] : ~0u;
    }
    uint32_t* ow32 = offp[w];
    for (uint32_t j = l; j < nkp; j += 64) ow32[j] = 0;
#pragma unroll
    for (uint32_t q = 0; q < PER; q++) sum += tot[q];
    uint32_t x = sum;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (l >= (uint32_t)o) x += y;
    }
    if (l == 63) wsum[w] = x;
    lds_sync();  // (the wave's zeroes before its counts)
#pragma unroll
    for (uint32_t q = 0; q < IT; q++)
        if (key[q] != ~0u) atomicAdd(&ow32[key[q] >> 1], 1u << (16 * (key[q] & 1)));
    __syncthreads();
    uint32_t pre = x - sum;
    for (uint32_t q = 0; q < w; q++) pre += wsum[q];
#pragma unroll
    for (uint32_t q = 0; q < PER; q++) {
        const uint32_t k = k0 + q;
        if (k < nk) {
            cnt[k] = pre + hst[q];
            if (t == 0 && k + 1 < nk) {
                B.beg[k] = pre, B.end[k] = pre + tot[q];
                if (tot[q]) B.keys_sorted[pre] = k;  // (the consumers check a range's first key only)
            }
        }
        pre += tot[q];
    }
    // the waves' counts -> exclusive offsets over the waves (both halves at once: < 2^16)
    for (uint32_t j = threadIdx.x; j < nkp; j += NT) {
        uint32_t run = 0;
#pragma unroll
        for (uint32_t q = 0; q < W; q++) {
            const uint32_t c = offp[q][j];
            offp[q][j] = run;
            run += c;
        }
    }
    __syncthreads();
    uint16_t* ow = reinterpret_cast<uint16_t*>(ow32);
    uint8_t* tg = tag[w];
    const uint64_t lt = (1ull << l) - 1ull;
#pragma unroll
    for (uint32_t q = 0; q < IT; q++) {
        if (s0 + q * 64 >= i1) break;
        const uint32_t i = s0 + q * 64 + l;
        const bool valid = i < i1;
        const uint32_t k = valid ? key[q] : 0u;
        // lanes that share a key (rare: ~0.5 pairs per 64 records over 4096 buckets)
        // rank among themselves in lane order; every other lane is alone.  Each lane
        // writes its lane id to its key's tag: a lane that reads another's id shares
        // its key, and one ballot per shared key finds the key's lanes
        if (valid) tg[k] = (uint8_t)l;
        lds_sync();
        uint64_t todo = __ballot(valid && tg[k] != (uint8_t)l);
        uint32_t rank = 0, grp = 1;
        bool last = true;
        while (todo) {
            const uint32_t kl = (uint32_t)__builtin_amdgcn_readlane((int)k, (int)__builtin_ctzll(todo));
            const uint64_t m = __ballot(valid && k == kl);
            if (valid && k == kl) {
                rank = (uint32_t)__popcll(m & lt);
                grp = (uint32_t)__popcll(m);
                last = (m >> l) == 1ull;
            }
            todo &= ~m;
        }
        if (valid) {
            const uint32_t c = ow[k];
            B.idx_sorted[cnt[k] + c + rank] = i;
            if (last) ow[k] = (uint16_t)(c + grp);  // the key's last lane
        }
        lds_sync();
    }
}
constexpr uint32_t BS_KEYS8 = 4608;  // the 8-wave scatter's key limit (its LDS: ~129 KB)
size_t bucket_sort_bytes(uint32_t n, uint32_t nk) { return ((size_t)((n + BS_TILE - 1) / BS_TILE) * nk + nk + 64) * 4; }
bool bucket_sort(const uint32_t* keys, uint32_t n, uint32_t nk, uint32_t* keys_sorted, uint32_t* idx_sorted, uint32_t* beg,
                 uint32_t* end, void* tmp, size_t tmp_bytes, hipStream_t st) {
    if (nk > BS_MAX_KEYS || bucket_sort_bytes(n, nk) > tmp_bytes) return false;
    const uint32_t tiles = (n + BS_TILE - 1) / BS_TILE;
    BucketSort B{keys, n, nk, static_cast<uint32_t*>(tmp), static_cast<uint32_t*>(tmp) + (size_t)tiles * nk, keys_sorted,
                 idx_sorted, beg, end};
    hipLaunchKernelGGL(k_bs_hist, dim3(tiles), dim3(256), nk * 4, st, B);
    hipLaunchKernelGGL(k_bs_cols, dim3((nk + 63) / 64), dim3(64 * BS_GROUPS), 0, st, B, tiles);
    if (nk <= BS_KEYS8) hipLaunchKernelGGL((k_bs_scatter<8, BS_KEYS8>), dim3(tiles), dim3(512), 0, st, B);
    else hipLaunchKernelGGL((k_bs_scatter<4, BS_MAX_KEYS>), dim3(tiles), dim3(256), 0, st, B);
    return true;
}

size_t ingest_sort_bytes(uint32_t n, uint32_t key_bits) {
    size_t bytes = 0;
    rocprim::counting_iterator<uint32_t> it(0u);
    (void)rocprim::radix_sort_pairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr, it,
                                    (uint32_t*)nullptr, n, 0u, key_bits);
    return std::max(bytes, bucket_sort_bytes(n, BS_MAX_KEYS));
}

// kwok_pod_rec12's create handles.  k_ing_tile_scan (one block): the exclusive
// prefixes of the NEW counts of the batch's tiles [0, ntiles) and their total;
// k_ing_new_handles (a block per tile of the chunk): each create's ordinal = its
// tile's prefix + the creates before it in the tile.
__global__ void k_ing_tile_scan(IngestBatch I, uint32_t ntiles) {
    __shared__ uint32_t wsum[16];
    const uint32_t per = (ntiles + blockDim.x - 1) / blockDim.x;
    const uint32_t t0 = min(threadIdx.x * per, ntiles), t1 = min(t0 + per, ntiles);
    uint32_t s = 0;
    for (uint32_t t = t0; t < t1; t++) s += I.tile_new[t];
    uint32_t x = s;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (lane() >= (uint32_t)o) x += y;
    }
    const uint32_t w = threadIdx.x >> 6;
    if (lane() == 63) wsum[w] = x;
    __syncthreads();
    uint32_t pre = x - s, all = 0;
    for (uint32_t q = 0; q < blockDim.x / 64; q++) {
        pre += q < w ? wsum[q] : 0u;
        all += wsum[q];
    }
    for (uint32_t t = t0; t < t1; t++) {
        I.tile_pre[t] = pre;
        pre += I.tile_new[t];
    }
    if (threadIdx.x == 0) I.sum->n_new = all;
}
__global__ void k_ing_new_handles(IngestBatch I, int32_t* dst, uint32_t cap) {
    __shared__ uint32_t wc[4];
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool nw = i < I.n && I.rec[i].is_new;
    const uint64_t m = __ballot(nw);
    const uint32_t w = threadIdx.x >> 6;
    if (lane() == 0) wc[w] = (uint32_t)__popcll(m);
    __syncthreads();
    if (!nw) return;
    uint32_t ord = I.tile_pre[I.tile0 + blockIdx.x] + (uint32_t)__popcll(m & ((1ull << lane()) - 1ull));
    for (uint32_t q = 0; q < w; q++) ord += wc[q];
    if (ord < cap) dst[ord] = I.out_handle[i];
}
void launch_ingest_new_handles(const IngestBatch& I, int32_t* new_handles, uint32_t cap, hipStream_t st) {
    const uint32_t tiles = cdiv(I.n, 256);
    hipLaunchKernelGGL(k_ing_tile_scan, dim3(1), dim3(1024), 0, st, I, I.tile0 + tiles);
    if (I.n) hipLaunchKernelGGL(k_ing_new_handles, dim3(tiles), dim3(256), 0, st, I, new_handles, cap);
}

__global__ void k_ing_status8(IngestBatch I, int8_t* dst) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < I.n) dst[i] = (int8_t)I.out_status[i];
}
void launch_ingest_status8(const IngestBatch& I, int8_t* dst, hipStream_t st) {
    if (I.n) hipLaunchKernelGGL(k_ing_status8, dim3(cdiv(I.n, 256)), dim3(256), 0, st, I, dst);
}
// the batch's results straight into the caller's kwok_host_alloc arrays (their
// device addresses; null: not wanted), four records per thread, no copy engine
__global__ void k_ing_results(IngestBatch I, int32_t* handles, int32_t* status, int8_t* status8, uint32_t* released) {
    const uint32_t i0 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;
#pragma unroll
    for (uint32_t q = 0; q < 4; q++) {
        const uint32_t i = i0 + q;
        if (i >= I.n) break;
        if (handles) handles[i] = I.out_handle[i];
        if (status) status[i] = I.out_status[i];
        if (status8) status8[i] = (int8_t)I.out_status[i];
        if (released) released[i] = I.out_released[i];
    }
}
void launch_ingest_results(const IngestBatch& I, int32_t* handles, int32_t* status, int8_t* status8, uint32_t* released,
                           hipStream_t st) {
    if (I.n) hipLaunchKernelGGL(k_ing_results, dim3(cdiv(I.n, 1024)), dim3(256), 0, st, I, handles, status, status8, released);
}
void launch_ingest_prep(const DevState& S, const IngestBatch& I, hipStream_t st) {
    // (256-record blocks: kwok_pod_rec12's create counts are per 256-record tile)
    if (I.n) hipLaunchKernelGGL(k_ing_prep, dim3(cdiv(I.n, 256)), dim3(256), 0, st, S, I);
}
void launch_ingest_need(const DevState& S, const IngestBatch& I, hipStream_t st) {
    hipLaunchKernelGGL(k_ing_need, dim3(cdiv(S.nb, 4)), dim3(256), 0, st, S, I);
}
int launch_ingest_sort(const DevState& S, const IngestBatch& I, void* tmp, size_t tmp_bytes, uint32_t key_bits,
                       hipStream_t st) {
    if (!I.n) return 0;
    if (bucket_sort(I.keys, I.n, S.nb + 1, I.keys_sorted, I.idx_sorted, I.beg, I.end, tmp, tmp_bytes, st)) return 0;
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
void launch_node_prep(const DevState& S, const NodeBatch& N, hipStream_t st) {
    if (N.n) hipLaunchKernelGGL(k_nd_prep, dim3(cdiv(N.n, 256)), dim3(256), 0, st, S, N);
}
void launch_node_fix(const DevState& S, const NodeBatch& N, const NodeFix* fix, uint32_t n_fix, hipStream_t st) {
    if (n_fix) hipLaunchKernelGGL(k_nd_fix, dim3(cdiv(n_fix, 256)), dim3(256), 0, st, S, N, fix, n_fix);
}
int launch_node_sort(const DevState& S, const NodeBatch& N, void* tmp, size_t tmp_bytes, uint32_t key_bits,
                     hipStream_t st) {
    if (!N.n) return 0;
    if (bucket_sort(N.keys, N.n, S.nb + 1, N.keys_sorted, N.idx_sorted, N.beg, N.end, tmp, tmp_bytes, st)) return 0;
    rocprim::counting_iterator<uint32_t> it(0u);
    if (rocprim::radix_sort_pairs(tmp, tmp_bytes, N.keys, N.keys_sorted, it, N.idx_sorted, N.n, 0u, key_bits, st) !=
        hipSuccess)
        return -1;
    hipLaunchKernelGGL(k_nd_ranges, dim3(cdiv(N.n, 256)), dim3(256), 0, st, S, N);
    return 0;
}
void launch_node_apply(const DevState& S, const NodeBatch& N, hipStream_t st) {
    hipLaunchKernelGGL(k_nd_apply, dim3(cdiv(S.nb, APPLY_WAVES)), dim3(64 * APPLY_WAVES), 0, st, S, N);
}
void launch_free_zombies(const DevState& S, hipStream_t st) {
    hipLaunchKernelGGL(k_free_zombies, dim3(cdiv(S.nb, 4)), dim3(256), 0, st, S);
}
void launch_hb_pre(const DevState& S, uint32_t* hb_pre, uint32_t* hb_bpre, hipStream_t st) {
    hipLaunchKernelGGL(k_hb_pre, dim3(1), dim3(1024), 0, st, S, hb_pre, hb_bpre);
}
void launch_node_lookup(const DevState& S, const uint8_t* names, const uint32_t* lens, uint32_t n, uint32_t* out,
                        hipStream_t st) {
    if (n) hipLaunchKernelGGL(k_node_lookup, dim3(cdiv(n, 4)), dim3(256), 0, st, S, names, lens, n, out);
}
void launch_cni_assign(const DevState& S, const int32_t* handles, const uint32_t* ips, const uint8_t* wr, uint32_t n,
                       int32_t* status, uint32_t* rejected, hipStream_t st) {
    if (n) hipLaunchKernelGGL(k_cni_assign, dim3(cdiv(n, 256)), dim3(256), 0, st, S, handles, ips, wr, n, status, rejected);
}

}  // namespace kwok
