// kernels.hip - gfx950 kernels of one kwok controller tick.
//
// A tick is a fixed pipeline of memory-bound sweeps over struct-of-arrays
// state in HBM; nothing here is a dense contraction, so there is no MFMA:
//
//   k_classify   one pass over node + pod slots: per-tile counts, pool
//                use/release candidate lists            (node_controller.go:206-223,
//                                                        pod_controller.go:252-269,306-343,377-439)
//   k_scan       one block: exclusive scan of tile counts -> output layout,
//                fleet counters, per-tick heartbeat template (Now/StartTime)
//   k_pool_*     ipPool Use / Put / Get-plan / select+commit on replicated
//                used/usable bitmaps                      (utils.go:52-117)
//   k_emit       second pass: compaction (wave ballots + block scans) of
//                heartbeat / node-init / pod-patch / delete lists, byte
//                emission of node-init and pod patches (wave per patch),
//                state transitions
//   k_hb_fill    the dominant kernel: n_managed identical 1059-byte heartbeat
//                patches streamed from an LDS-staged template with 16-byte
//                stores                                   (node_controller.go:145-204,393-401)
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "device.h"
#include "kernels.h"

namespace kwok {

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }

// wave-wide inclusive scan (64 lanes)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    const int l = lane_id();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        uint32_t y = __shfl_up(x, off, 64);
        if (l >= off) x += y;
    }
    return x;
}

// block-wide exclusive scan of NF u32 fields; returns totals.  BLOCK=256.
template <int NF>
__device__ __forceinline__ void block_excl_scan(uint32_t (&v)[NF], uint32_t (&tot)[NF]) {
    __shared__ uint32_t wsum[BLOCK / 64][NF];
    const int l = lane_id(), w = wave_id();
    uint32_t incl[NF];
#pragma unroll
    for (int f = 0; f < NF; f++) {
        incl[f] = wave_incl_scan(v[f]);
        if (l == 63) wsum[w][f] = incl[f];
    }
    __syncthreads();
#pragma unroll
    for (int f = 0; f < NF; f++) {
        uint32_t pre = 0, t = 0;
#pragma unroll
        for (int k = 0; k < BLOCK / 64; k++) {
            uint32_t s = wsum[k][f];
            pre += (k < w) ? s : 0u;
            t += s;
        }
        v[f] = pre + incl[f] - v[f];
        tot[f] = t;
    }
    __syncthreads();
}

template <int NF>
__device__ __forceinline__ void block_sum(uint32_t (&v)[NF]) {
    uint32_t tot[NF];
    block_excl_scan<NF>(v, tot);
#pragma unroll
    for (int f = 0; f < NF; f++) v[f] = tot[f];
}

// append x to a device list with one atomic per wave
__device__ __forceinline__ void wave_append(bool pred, uint32_t x, uint32_t* list, uint32_t* counter) {
    uint64_t m = __ballot(pred);
    if (!m) return;
    uint32_t base = 0;
    const int l = lane_id();
    int leader = __ffsll((unsigned long long)m) - 1;
    if (l == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    if (pred) list[base + __popcll(m & ((1ull << l) - 1))] = x;
}

__device__ __forceinline__ bool in_cidr(const PoolGeom& g, uint32_t ip) {
    return (uint64_t)(ip - g.net) < g.size && ip >= g.net;
}
__device__ __forceinline__ bool bm_test(const uint64_t* bm, uint64_t bit) { return (bm[bit >> 6] >> (bit & 63)) & 1; }

// RFC3339 UTC of unix seconds, packed into 3 x u64 (20 bytes, little endian)
struct Ts {
    uint64_t w0, w1, w2;
};
__device__ __forceinline__ Ts format_ts(uint64_t t) {
    uint32_t days = (uint32_t)(t / 86400u), rem = (uint32_t)(t % 86400u);
    uint32_t hh = rem / 3600u, mi = (rem % 3600u) / 60u, ss = rem % 60u;
    // civil_from_days (proleptic Gregorian), days since 1970-01-01
    uint32_t z = days + 719468u;
    uint32_t era = z / 146097u;
    uint32_t doe = z - era * 146097u;
    uint32_t yoe = (doe - doe / 1460u + doe / 36524u - doe / 146096u) / 365u;
    uint32_t y = yoe + era * 400u;
    uint32_t doy = doe - (365u * yoe + yoe / 4u - yoe / 100u);
    uint32_t mp = (5u * doy + 2u) / 153u;
    uint32_t d = doy - (153u * mp + 2u) / 5u + 1u;
    uint32_t m = mp < 10u ? mp + 3u : mp - 9u;
    y += (m <= 2u);
    auto c = [](uint32_t v) -> uint64_t { return (uint64_t)('0' + v); };
    Ts r;
    r.w0 = c(y / 1000u) | c((y / 100u) % 10u) << 8 | c((y / 10u) % 10u) << 16 | c(y % 10u) << 24 |
           (uint64_t)'-' << 32 | c(m / 10u) << 40 | c(m % 10u) << 48 | (uint64_t)'-' << 56;
    r.w1 = c(d / 10u) | c(d % 10u) << 8 | (uint64_t)'T' << 16 | c(hh / 10u) << 24 | c(hh % 10u) << 32 |
           (uint64_t)':' << 40 | c(mi / 10u) << 48 | c(mi % 10u) << 56;
    r.w2 = (uint64_t)':' | c(ss / 10u) << 8 | c(ss % 10u) << 16 | (uint64_t)'Z' << 24;
    return r;
}
__device__ __forceinline__ uint32_t ts_byte(const Ts& t, uint32_t i) {
    uint64_t w = i < 8 ? t.w0 : (i < 16 ? t.w1 : t.w2);
    return (uint32_t)(w >> (8 * (i & 7))) & 0xFF;
}

// net.IP.String() of an IPv4 address packed into 2 x u64 (<= 15 bytes)
struct IpStr {
    uint64_t lo, hi;
    uint32_t len;
};
__device__ __forceinline__ IpStr format_ip(uint32_t ip) {
    IpStr r{0, 0, 0};
    auto put = [&](uint32_t ch) {
        if (r.len < 8) r.lo |= (uint64_t)ch << (8 * r.len);
        else r.hi |= (uint64_t)ch << (8 * (r.len - 8));
        r.len++;
    };
#pragma unroll
    for (int k = 3; k >= 0; k--) {
        uint32_t o = (ip >> (8 * k)) & 255u;
        if (o >= 100u) put('0' + o / 100u);
        if (o >= 10u) put('0' + (o / 10u) % 10u);
        put('0' + o % 10u);
        if (k) put('.');
    }
    return r;
}
__device__ __forceinline__ uint32_t ip_byte(const IpStr& s, uint32_t i) {
    return (uint32_t)((i < 8 ? s.lo >> (8 * i) : s.hi >> (8 * (i - 8))) & 0xFF);
}

__device__ __forceinline__ uint32_t ip_len(uint32_t ip) {
    uint32_t n = 3;
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t o = (ip >> (8 * k)) & 255u;
        n += 1u + (o >= 10u) + (o >= 100u);
    }
    return n;
}

__device__ __forceinline__ uint32_t lit_byte(const char* s, uint32_t i) { return (uint32_t)(uint8_t)s[i]; }

// ---------------------------------------------------------------------------
// per-object predicates (shared by k_classify and k_emit)
// ---------------------------------------------------------------------------
struct NodeCls {
    bool hb, lock, init, ready, managed;
};
__device__ __forceinline__ NodeCls classify_node(uint8_t s) {
    NodeCls c;
    c.managed = s & NS_MANAGED;
    c.hb = c.managed;  // KeepNodeHeartbeat: every node in nodesSets
    // LockNode: heartbeat feedback re-locks every managed lockable node; plus queued events
    c.lock = (s & NS_EXISTS) && ((c.managed && (s & NS_LOCKABLE)) || (s & NS_EVENT_LOCK));
    c.init = c.lock && !(s & NS_CONFORMS);
    c.ready = c.managed && ((s & NS_CONFORMS) || c.lock);
    return c;
}
// node tick flags for the pod side (written by classify, read by emit)
enum : uint8_t { NT_RELOCK = 1, NT_MANAGED = 2 };
__device__ __forceinline__ uint8_t node_tick_flags(uint8_t s) {
    NodeCls c = classify_node(s);
    return (uint8_t)((c.lock && c.managed ? NT_RELOCK : 0) | (c.managed ? NT_MANAGED : 0));
}

struct PodCls {
    bool used, del, eval, alloc, need;
    uint32_t phase;
};
__device__ __forceinline__ PodCls classify_pod(uint16_t st, uint8_t ntf, uint32_t pod_ip) {
    PodCls c;
    c.used = st & PS_USED;
    c.del = c.used && (st & PS_DELETE_PENDING);
    c.eval = c.used && !c.del && ((st & PS_EVENT) || ((ntf & NT_RELOCK) && !(st & PS_DISREGARD)));
    c.phase = (st & PS_PHASE_MASK) >> PS_PHASE_SHIFT;
    // `{{ with .status }} ... {{ with .podIP }} . {{ else }} {{ PodIP }}` (pod.status.tpl:44-47)
    c.alloc = c.eval && (st & PS_STATUS_NONEMPTY) && pod_ip == 0;
    // computePatchData: Pending always patches; otherwise the strategic merge must change something
    c.need = c.eval && (c.phase != PHASE_RUNNING || !(st & PS_CONFORMS) || !(st & PS_HAS_HOST_IP) || pod_ip == 0);
    return c;
}

__device__ __forceinline__ uint32_t init_patch_len(uint64_t blob) {
    uint32_t pre = (uint32_t)(blob >> 32) & 0xFFFF, post = (uint32_t)(blob >> 48);
    return 11u + pre + 14u + (uint32_t)CONDS_LEN + 1u + post + 2u;
}

// ---------------------------------------------------------------------------
// k_classify
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(BLOCK) void k_classify(DevState S) {
    const uint32_t tile = blockIdx.x;
    const int t = threadIdx.x;
    if (tile < S.node_tiles) {
        const uint32_t first = tile * NODE_TILE + t * NODE_PER_THREAD;
        uint32_t f[6] = {0, 0, 0, 0, 0, 0};  // hb, init, init_bytes, lock, managed, ready
        uint32_t packed = 0;
        if (first < S.n_node_slots) packed = *reinterpret_cast<const uint32_t*>(S.node_state + first);
        uint32_t tick = 0;
#pragma unroll
        for (int k = 0; k < NODE_PER_THREAD; k++) {
            uint8_t s = (uint8_t)(packed >> (8 * k));
            NodeCls c = classify_node(s);
            f[0] += c.hb;
            f[3] += c.lock;
            f[4] += c.managed;
            f[5] += c.ready;
            if (c.init) {
                f[1]++;
                f[2] += (init_patch_len(S.node_blob[first + k]) + 15u) & ~15u;
            }
            tick |= (uint32_t)node_tick_flags(s) << (8 * k);
        }
        if (first < S.n_node_slots) *reinterpret_cast<uint32_t*>(S.node_tick + first) = tick;
        block_sum<6>(f);
        if (t == 0) {
            uint32_t* o = S.tiles + (size_t)tile * TF_STRIDE;
            o[TF_HB] = f[0];
            o[TF_INIT] = f[1];
            o[TF_INIT_BYTES] = f[2];
            o[TF_LOCK] = f[3];
            o[TF_MANAGED] = f[4];
            o[TF_READY] = f[5];
        }
        return;
    }
    const uint32_t ptile = tile - S.node_tiles;
    const uint32_t first = ptile * POD_TILE + t * POD_PER_THREAD;
    uint32_t f[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // del, eval, alloc, pp, pp_bytes, total, pending, running, rel
    // slots at or above the bucket's fill mark are known empty: no loads
    const bool live = first < S.n_pod_slots && (first % S.cp) < S.pod_fill[first / S.cp];
    uint4 st4 = make_uint4(0, 0, 0, 0), nd4 = make_uint4(0, 0, 0, 0), ipa = make_uint4(0, 0, 0, 0),
          ipb = make_uint4(0, 0, 0, 0);
    if (live) {
        st4 = *reinterpret_cast<const uint4*>(S.pod_state + first);
        nd4 = *reinterpret_cast<const uint4*>(S.pod_node + first);
        ipa = *reinterpret_cast<const uint4*>(S.pod_ip + first);
        ipb = *reinterpret_cast<const uint4*>(S.pod_ip + first + 4);
    }
    const uint32_t stw[4] = {st4.x, st4.y, st4.z, st4.w};
    const uint32_t ndw[4] = {nd4.x, nd4.y, nd4.z, nd4.w};
    const uint32_t ips[8] = {ipa.x, ipa.y, ipa.z, ipa.w, ipb.x, ipb.y, ipb.z, ipb.w};
    const uint32_t bucket_local = first / S.cp;  // 8 slots never straddle a bucket (cp % 8 == 0)
#pragma unroll
    for (int k = 0; k < POD_PER_THREAD; k++) {
        uint16_t st = (uint16_t)(stw[k >> 1] >> (16 * (k & 1)));
        uint16_t nl = (uint16_t)(ndw[k >> 1] >> (16 * (k & 1)));
        uint32_t ip = ips[k];
        uint8_t ns = 0;
        if (st & PS_USED) ns = S.node_state[bucket_local * S.cn + nl];
        uint8_t ntf = node_tick_flags(ns);
        PodCls c = classify_pod(st, ntf, ip);
        f[0] += c.del;
        f[1] += c.eval;
        f[2] += c.alloc;
        // the Deleted event of a pod we delete: release if the node is managed and the IP in CIDR
        bool rel = c.del && (ntf & NT_MANAGED) && ip && in_cidr(S.pool, ip);
        // configurePod (pod_controller.go:378-382): Use() an existing in-CIDR IP; only
        // addresses not already in `used` change the pool
        bool use = c.eval && ip && in_cidr(S.pool, ip) && !bm_test(S.used_bm, ip - S.pool.net);
        if (S.world == 1) {
            // single rank: Use() in place; the Put of a released address waits in rel_bm
            // and is folded by k_pool_prep, after every Use of this tick (Use -> Put order)
            const uint64_t bit = ip - S.pool.net;
            if (use) atomicOr((unsigned long long*)&S.used_bm[bit >> 6], 1ull << (bit & 63));
            if (rel) atomicOr((unsigned long long*)&S.rel_bm[bit >> 6], 1ull << (bit & 63));
        } else {
            wave_append(rel, ip, S.rel_list, &S.list_counts[1]);
            wave_append(use, ip, S.use_list, &S.list_counts[0]);
        }
        f[8] += rel;
        if (c.need) {
            f[3]++;
            f[4] += S.specs[S.pod_spec[first + k]].max_len;
        }
        bool total = c.used && !c.del;
        f[5] += total;
        f[6] += total && !c.need && c.phase == PHASE_PENDING;
        f[7] += total && (c.need || c.phase == PHASE_RUNNING);
    }
    block_sum<9>(f);
    if (t == 0) {
        uint32_t* o = S.tiles + (size_t)tile * TF_STRIDE;
        o[TF_DEL] = f[0];
        o[TF_EVAL] = f[1];
        o[TF_ALLOC] = f[2];
        o[TF_PP] = f[3];
        o[TF_PP_BYTES] = f[4];
        o[TF_TOTAL] = f[5];
        o[TF_PENDING] = f[6];
        o[TF_RUNNING] = f[7];
        o[TF_REL] = f[8];
    }
}

// ---------------------------------------------------------------------------
// k_scan: one block of 256 threads.  Exclusive scan of the tile counts ->
// tile bases; arena layout; counters; per-tick heartbeat template.  Wave
// shuffles inside each wave, one LDS exchange across the 16 waves.
// ---------------------------------------------------------------------------
constexpr int SCAN_THREADS = 512;  // 256-VGPR budget: partials stay in registers
constexpr int SCAN_WAVES = SCAN_THREADS / 64;

__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t x) {
    const int l = lane_id();
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        unsigned long long y = __shfl_up((unsigned long long)x, off, 64);
        if (l >= off) x += y;
    }
    return x;
}
__device__ __forceinline__ uint64_t wave_sum64(uint64_t x) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor((unsigned long long)x, off, 64);
    return x;
}

// tile record -> the 7 scanned fields and 8 reduced fields
struct TileVals {
    uint32_t sc[7], cn[8];
};
__device__ __forceinline__ void load_tile(const DevState& S, uint32_t i, TileVals& v) {
    const uint4* o = reinterpret_cast<const uint4*>(S.tiles + (size_t)i * TF_STRIDE);
    const uint4 a = o[0], b = o[1], c = o[2], d = o[3];
    const uint32_t f[16] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
    if (i < S.node_tiles) {
        v.sc[0] = f[TF_HB], v.sc[1] = f[TF_INIT], v.sc[2] = f[TF_INIT_BYTES];
        v.sc[3] = v.sc[4] = v.sc[5] = v.sc[6] = 0;
        v.cn[0] = f[TF_LOCK], v.cn[1] = f[TF_MANAGED], v.cn[2] = f[TF_READY];
        v.cn[3] = v.cn[4] = v.cn[5] = v.cn[6] = v.cn[7] = 0;
    } else {
        v.sc[0] = v.sc[1] = v.sc[2] = 0;
        v.sc[3] = f[TF_DEL], v.sc[4] = f[TF_PP], v.sc[5] = f[TF_PP_BYTES], v.sc[6] = f[TF_ALLOC];
        v.cn[0] = v.cn[1] = v.cn[2] = 0;
        v.cn[3] = f[TF_EVAL], v.cn[4] = f[TF_TOTAL], v.cn[5] = f[TF_PENDING], v.cn[6] = f[TF_RUNNING];
        v.cn[7] = f[TF_REL];
    }
}

__global__ __launch_bounds__(SCAN_THREADS) void k_scan(DevState S, uint64_t start_unix, int world_size) {
    const uint64_t now_unix = *(volatile const uint64_t*)S.tick_now;  // pinned host scalar
    const int t = threadIdx.x, l = lane_id(), w = wave_id();
    const uint32_t T = S.node_tiles + S.pod_tiles;
    const uint32_t per = (T + SCAN_THREADS - 1) / SCAN_THREADS;
    const uint32_t lo = min(T, t * per), hi = min(T, lo + per);
    // scanned: hb, init, init_bytes (node tiles); del, pp, pp_bytes, alloc (pod tiles)
    // reduced: lock, managed, ready (nodes); eval, total, pending, running, rel (pods)
    constexpr int NS = 7, NC = 8;
    uint32_t sc[NS] = {0, 0, 0, 0, 0, 0, 0}, cn[NC] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t i = lo; i < hi; i++) {
        TileVals v;
        load_tile(S, i, v);
#pragma unroll
        for (int f = 0; f < NS; f++) sc[f] += v.sc[f];
#pragma unroll
        for (int f = 0; f < NC; f++) cn[f] += v.cn[f];
    }
    __shared__ uint64_t wtot[SCAN_WAVES][NS];
    __shared__ uint64_t wcnt[SCAN_WAVES][NC];
    uint64_t ex[NS];
#pragma unroll
    for (int f = 0; f < NS; f++) {
        uint64_t inc = wave_incl_scan64(sc[f]);
        ex[f] = inc - sc[f];
        if (l == 63) wtot[w][f] = inc;
    }
#pragma unroll
    for (int f = 0; f < NC; f++) {
        uint64_t r = wave_sum64(cn[f]);
        if (l == 0) wcnt[w][f] = r;
    }
    __syncthreads();
    uint64_t total[NS];
#pragma unroll
    for (int f = 0; f < NS; f++) {
        uint64_t pre = 0, tot = 0;
#pragma unroll
        for (int k = 0; k < SCAN_WAVES; k++) {
            uint64_t v = wtot[k][f];
            pre += k < w ? v : 0;
            tot += v;
        }
        ex[f] += pre;
        total[f] = tot;
    }
    for (uint32_t i = lo; i < hi; i++) {
        TileVals v;
        load_tile(S, i, v);
        uint64_t* b = S.tile_base + (size_t)i * 4;
        if (i < S.node_tiles) {
            b[0] = ex[0], b[1] = ex[1], b[2] = ex[2];
        } else {
            b[0] = ex[3], b[1] = ex[4], b[2] = ex[5], b[3] = ex[6];
        }
#pragma unroll
        for (int f = 0; f < NS; f++) ex[f] += v.sc[f];
    }
    TickHdr* H = S.hdr;
    if (t == 0) {
        uint64_t red[NC];
        for (int f = 0; f < NC; f++) {
            red[f] = 0;
            for (int k = 0; k < SCAN_WAVES; k++) red[f] += wcnt[k][f];
        }
        H->n_hb = (uint32_t)total[0];
        H->n_init = (uint32_t)total[1];
        H->init_bytes = total[2];
        H->n_del = (uint32_t)total[3];
        H->n_pp = (uint32_t)total[4];
        H->pp_bytes = total[5];
        H->n_alloc_local = (uint32_t)total[6];
        H->n_lock = (uint32_t)red[0];
        H->n_eval = (uint32_t)red[3];
        H->n_rel = (uint32_t)red[7];
        H->n_use = world_size > 1 ? S.list_counts[0] : 0;
        H->hb_base = 0;
        H->init_base = total[0] * (uint64_t)HB_STRIDE;
        H->pod_base = H->init_base + total[2];
        H->arena_bytes = H->pod_base + total[5];
        H->overflow = H->arena_bytes > S.arena_cap;
        uint64_t* L = H->local_counters;
        L[0] = total[0];  // heartbeat
        L[1] = total[1];  // node_init
        L[2] = total[4];  // pod_patch
        L[3] = total[3];  // delete
        L[4] = total[6];  // alloc
        L[5] = red[7];    // release
        L[6] = red[3];    // evaluated
        L[7] = red[0];    // lock_checked
        L[8] = red[1];    // nodes_managed
        L[9] = red[2];    // nodes_ready
        L[10] = red[4];   // pods_total
        L[11] = red[5];   // pods_pending
        L[12] = red[6];   // pods_running
        for (int k = 13; k < 16; k++) L[k] = 0;
        if (world_size == 1) {
            for (int k = 0; k < 16; k++) H->counters[k] = L[k];
            H->alloc_total = total[6];
            H->alloc_base = 0;
            H->rel_total = red[7];
        } else {
            XMsg* X = S.xmsg;
            X->alloc = total[6];
            X->n_use = S.list_counts[0];
            X->n_rel = S.list_counts[1];
            for (int k = 0; k < 16; k++) X->counters[k] = L[k];
        }
    }
    // exchange message lists (multi-rank), inline when they fit
    if (world_size > 1) {
        const uint32_t nu = S.list_counts[0], nr = S.list_counts[1];
        if (nu + nr <= (uint32_t)XINLINE) {
            for (uint32_t i = t; i < nu; i += SCAN_THREADS) S.xmsg->ips[i] = S.use_list[i];
            for (uint32_t i = t; i < nr; i += SCAN_THREADS) S.xmsg->ips[nu + i] = S.rel_list[i];
        }
    }
    // per-tick heartbeat template: static bytes + Now / StartTime in the 10 slots
    Ts now = format_ts(now_unix), st = format_ts(start_unix);
    for (int i = t; i < HB_STRIDE; i += SCAN_THREADS) {
        uint8_t k = S.hb_kind[i];
        uint32_t b;
        if (k == 0xFF) b = S.hb_static[i];
        else if (k < TS_LEN) b = ts_byte(now, k);
        else b = ts_byte(st, k - TS_LEN);
        S.hb_tmpl[i] = (uint8_t)b;
    }
}

// ---------------------------------------------------------------------------
// k_xreduce (multi-rank): fold the gathered exchange headers
// ---------------------------------------------------------------------------
__global__ void k_xreduce(DevState S, const XMsg* all, int world_size, int rank) {
    if (threadIdx.x != 0) return;
    TickHdr* H = S.hdr;
    uint64_t tot = 0, base = 0;
    for (int k = 0; k < 16; k++) H->counters[k] = 0;
    for (int r = 0; r < world_size; r++) {
        if (r < rank) base += all[r].alloc;
        tot += all[r].alloc;
        for (int k = 0; k < 16; k++) H->counters[k] += all[r].counters[k];
    }
    H->alloc_total = tot;
    H->alloc_base = base;
    uint64_t rel = 0;
    for (int r = 0; r < world_size; r++) rel += all[r].n_rel;
    H->rel_total = rel;
}

// ---------------------------------------------------------------------------
// ipPool kernels on the replicated bitmaps
//
// Order inside a tick (DESIGN.md "Tick contract"): every Use (configurePod,
// pod_controller.go:378-382) -> every Put of this tick's deletions
// (pod_controller.go:329-336 / utils.go:100-108) -> the Gets (utils.go:83-98)
// in canonical order.  Uses set `used` directly; Puts accumulate in rel_bm
// (atomic ORs commute with the Uses) and k_pool_prep folds them:
//   used &= ~rel, usable |= rel.
// ---------------------------------------------------------------------------
// ingest-time Put (a Deleted watch event), applied immediately
__global__ void k_pool_puts_now(DevState S, const uint32_t* ips, uint32_t n) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        uint32_t ip = ips[i];
        if (!in_cidr(S.pool, ip)) continue;
        uint64_t b = ip - S.pool.net;
        atomicAnd((unsigned long long*)&S.used_bm[b >> 6], ~(1ull << (b & 63)));
        atomicOr((unsigned long long*)&S.usable_bm[b >> 6], 1ull << (b & 63));
    }
}
// multi-rank: every rank's Uses into used_bm, every rank's Puts into rel_bm
__global__ void k_pool_apply(DevState S, const ListDesc* ld, int nranks) {
    for (int r = 0; r < nranks; r++) {
        const ListDesc d = ld[r];
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < d.n_use + d.n_rel; i += gridDim.x * blockDim.x) {
            bool use = i < d.n_use;
            uint32_t ip = use ? d.use[i] : d.rel[i - d.n_use];
            if (!in_cidr(S.pool, ip)) continue;
            uint64_t b = ip - S.pool.net;
            atomicOr((unsigned long long*)&(use ? S.used_bm : S.rel_bm)[b >> 6], 1ull << (b & 63));
        }
    }
}

// free bits for ipPool.new at or after the fresh cursor.  Addresses still
// usable this tick are excluded: fresh allocation only happens once Get's
// reuse branch has taken every usable address (take = U whenever F > 0).
__device__ __forceinline__ uint64_t free_mask(const DevState& S, uint64_t w, uint64_t used, uint64_t usable,
                                              uint64_t cursor_bit) {
    uint64_t lo = w * 64;
    if (lo + 64 <= cursor_bit) return 0;
    uint64_t m = ~used & ~usable;
    if (cursor_bit > lo) m &= ~0ull << (cursor_bit - lo);
    if (lo + 64 > S.pool.size) m &= (S.pool.size - lo >= 64) ? ~0ull : ((1ull << (S.pool.size - lo)) - 1);
    return m;
}
__device__ __forceinline__ uint64_t cursor_bit(const DevState& S) {
    uint64_t a = (uint64_t)S.pool.base + *S.pool_index;  // ipPool.new: addIP(cidr.IP, index)
    return a >= S.pool.net ? a - S.pool.net : 0;
}

constexpr int POOL_WPT = 4;                  // bitmap words per thread
constexpr int POOL_WPB = BLOCK * POOL_WPT;   // bitmap words per block

// fold this tick's Puts, then count usable / free bits per block for the plan
__global__ __launch_bounds__(BLOCK) void k_pool_prep(DevState S) {
    const TickHdr* H = S.hdr;
    const bool fold = H->rel_total != 0, count = H->alloc_total != 0;
    if (!fold && !count) return;
    const uint64_t cb = cursor_bit(S);
    uint32_t f[2] = {0, 0};
    for (int k = 0; k < POOL_WPT; k++) {
        uint64_t w = (uint64_t)blockIdx.x * POOL_WPB + threadIdx.x * POOL_WPT + k;
        if (w >= S.pool.words) break;
        uint64_t used = S.used_bm[w], usable = S.usable_bm[w];
        if (fold) {
            uint64_t r = S.rel_bm[w];
            if (r) {
                used &= ~r;
                usable |= r;
                S.used_bm[w] = used;
                S.usable_bm[w] = usable;
                S.rel_bm[w] = 0;
            }
        }
        f[0] += __popcll(usable);
        f[1] += __popcll(free_mask(S, w, used, usable, cb));
    }
    if (!count) return;
    block_sum<2>(f);
    if (threadIdx.x == 0) {
        S.pool_blk[2 * blockIdx.x] = f[0];
        S.pool_blk[2 * blockIdx.x + 1] = f[1];
    }
}

// select + commit.  Allocation ordinal g (global, canonical order):
//   g < take                -> g-th lowest usable address (the build's reuse rule)
//   g < take + fresh_in     -> (g-take)-th free in-CIDR address from the cursor
//   otherwise               -> fresh_out_start + (g - take - fresh_in)  (beyond the CIDR)
// Every rank commits ALL allocations to its replica; it records the addresses
// of its own ordinals [alloc_base, alloc_base + n_alloc_local).  Each block
// derives the plan from the per-block counts itself (no separate launch).
__global__ __launch_bounds__(BLOCK) void k_pool_select(DevState S, uint32_t nblk) {
    TickHdr* H = S.hdr;
    const uint64_t A = H->alloc_total;
    if (A == 0) return;
    __shared__ uint64_t sh[4];  // U, Fin, block base usable, block base free
    if (threadIdx.x < 64) {
        uint64_t u = 0, fr = 0, bu = 0, bf = 0;
        for (uint32_t i = threadIdx.x; i < nblk; i += 64) {
            uint64_t a = S.pool_blk[2 * i], c = S.pool_blk[2 * i + 1];
            u += a;
            fr += c;
            if (i < blockIdx.x) bu += a, bf += c;
        }
        u = wave_sum64(u);
        fr = wave_sum64(fr);
        bu = wave_sum64(bu);
        bf = wave_sum64(bf);
        if (threadIdx.x == 0) sh[0] = u, sh[1] = fr, sh[2] = bu, sh[3] = bf;
    }
    __syncthreads();
    const uint64_t U = sh[0], Fin = sh[1];
    const uint64_t take = A < U ? A : U, F = A - take, fin = F < Fin ? F : Fin, fout = F - fin;
    const uint64_t cur = (uint64_t)S.pool.base + *S.pool_index;
    const uint64_t end = (uint64_t)S.pool.net + S.pool.size;
    const uint64_t fout0 = cur > end ? cur : end;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        H->usable_total = U;
        H->take_usable = take;
        H->fresh_in = fin;
        H->fresh_out_start = fout0;
        // ipPool.index after the last fresh address (k_emit commits it);
        // fin > 0 && fout == 0: the thread that selects the last one sets it below
        if (fout) H->cursor_index = fout0 + fout - S.pool.base;
        else if (fin == 0) H->cursor_index = *S.pool_index;
    }
    const uint64_t lo_g = H->alloc_base, hi_g = lo_g + H->n_alloc_local;
    const uint64_t cb = cursor_bit(S);
    const bool advance = fin > 0 && fout == 0;
    uint32_t c[2][POOL_WPT];
    uint64_t wu[POOL_WPT], wf[POOL_WPT];
    uint32_t v[2] = {0, 0};
    for (int k = 0; k < POOL_WPT; k++) {
        uint64_t w = (uint64_t)blockIdx.x * POOL_WPB + threadIdx.x * POOL_WPT + k;
        uint64_t used = w < S.pool.words ? S.used_bm[w] : ~0ull;
        wu[k] = w < S.pool.words ? S.usable_bm[w] : 0;
        wf[k] = w < S.pool.words ? free_mask(S, w, used, wu[k], cb) : 0;
        c[0][k] = __popcll(wu[k]);
        c[1][k] = __popcll(wf[k]);
        v[0] += c[0][k];
        v[1] += c[1][k];
    }
    uint32_t tot[2];
    block_excl_scan<2>(v, tot);
    uint64_t ru = sh[2] + v[0];
    uint64_t rf = sh[3] + v[1];
    for (int k = 0; k < POOL_WPT; k++) {
        uint64_t w = (uint64_t)blockIdx.x * POOL_WPB + threadIdx.x * POOL_WPT + k;
        if (w >= S.pool.words) break;
        if (ru < take && wu[k]) {
            uint64_t n = take - ru < c[0][k] ? take - ru : c[0][k];
            uint64_t m = wu[k], sel = 0;
            for (uint64_t j = 0; j < n; j++) {
                uint32_t b = (uint32_t)(__ffsll((unsigned long long)m) - 1);
                m &= m - 1;
                sel |= 1ull << b;
                uint64_t g = ru + j;
                if (g >= lo_g && g < hi_g) S.alloc_addr[g - lo_g] = S.pool.net + (uint32_t)(w * 64 + b);
            }
            S.usable_bm[w] &= ~sel;  // ipPool.Get: delete(usable, ip) ...
            S.used_bm[w] |= sel;     // ... used[ip]   (one thread owns word w)
        }
        ru += c[0][k];
        if (rf < fin && wf[k]) {
            uint64_t n = fin - rf < c[1][k] ? fin - rf : c[1][k];
            uint64_t m = wf[k], sel = 0;
            uint32_t b = 0;
            for (uint64_t j = 0; j < n; j++) {
                b = (uint32_t)(__ffsll((unsigned long long)m) - 1);
                m &= m - 1;
                sel |= 1ull << b;
                uint64_t g = take + rf + j;
                if (g >= lo_g && g < hi_g) S.alloc_addr[g - lo_g] = S.pool.net + (uint32_t)(w * 64 + b);
            }
            S.used_bm[w] |= sel;  // ipPool.new: used[ip]  (usable add + Get delete net to nothing)
            if (advance && rf + n == fin) H->cursor_index = (uint64_t)S.pool.net + w * 64 + b + 1 - S.pool.base;
        }
        rf += c[1][k];
    }
}

// ---------------------------------------------------------------------------
// k_emit: compaction + byte emission + state transitions
// ---------------------------------------------------------------------------
struct PodJob {
    uint32_t slot;   // local slot
    uint32_t off;    // byte offset within the tile's pod region
    uint32_t pod_ip; // rendered podIP (0 = no status section)
    uint32_t host_ip;
};
struct InitJob {
    uint32_t slot;
    uint32_t off;
};

// one wave writes one pod patch: A [+ "hostIP":"H",] B [+ "podIP":"P",] C
__device__ void write_pod_patch(const DevState& S, const PodJob& j, uint8_t* out) {
    const SpecDesc sd = S.specs[S.pod_spec[j.slot]];
    const Ts ts = format_ts(S.pod_ctime[j.slot]);
    const bool st = j.host_ip != 0;
    const IpStr H = format_ip(j.host_ip), P = format_ip(j.pod_ip);
    const uint32_t la = sd.len_a, lb = sd.len_b, lc = sd.len_c;
    const uint32_t lh = st ? 10u + H.len + 2u : 0u, lp = st ? 9u + P.len + 2u : 0u;
    const uint32_t len = la + lh + lb + lp + lc;
    const uint8_t* bytes = S.spec_bytes + sd.off;
    const uint8_t* kinds = S.spec_kinds + sd.off;
    const char* kh = "\"hostIP\":\"";
    const char* kp = "\"podIP\":\"";
    for (uint32_t q0 = lane_id() * 4u; q0 < len; q0 += 256u) {
        uint32_t w = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            uint32_t q = q0 + k, b = 0;
            if (q < len) {
                uint32_t p = q;
                uint32_t seg_off;  // offset into the concatenated spec bytes (A|B|C)
                bool tmpl = false;
                if (p < la) {
                    tmpl = true;
                    seg_off = p;
                } else if ((p -= la) < lh) {
                    if (p < 10u) b = lit_byte(kh, p);
                    else if (p < 10u + H.len) b = ip_byte(H, p - 10u);
                    else b = (p == 10u + H.len) ? '"' : ',';
                } else if ((p -= lh) < lb) {
                    tmpl = true;
                    seg_off = la + p;
                } else if ((p -= lb) < lp) {
                    if (p < 9u) b = lit_byte(kp, p);
                    else if (p < 9u + P.len) b = ip_byte(P, p - 9u);
                    else b = (p == 9u + P.len) ? '"' : ',';
                } else {
                    p -= lp;
                    tmpl = true;
                    seg_off = la + lb + p;
                }
                if (tmpl) {
                    uint8_t kd = kinds[seg_off];
                    b = kd == 0xFF ? bytes[seg_off] : ts_byte(ts, kd);
                }
            }
            w |= b << (8 * k);
        }
        *reinterpret_cast<uint32_t*>(out + q0) = w;
    }
}

// one wave writes one node init patch: {"status":{ pre ,"conditions": CONDS , post }}
__device__ void write_init_patch(const DevState& S, uint64_t blob, uint8_t* out) {
    const uint32_t boff = (uint32_t)blob, pre = (uint32_t)(blob >> 32) & 0xFFFF, post = (uint32_t)(blob >> 48);
    const uint32_t len = init_patch_len(blob);
    const uint8_t* bb = S.blob + boff;
    const uint8_t* conds = S.hb_tmpl + HB_PREFIX;
    const char* p0 = "{\"status\":{";
    const char* p1 = ",\"conditions\":";
    for (uint32_t q0 = lane_id() * 4u; q0 < len; q0 += 256u) {
        uint32_t w = 0;
#pragma unroll
        for (uint32_t k = 0; k < 4; k++) {
            uint32_t q = q0 + k, b = 0;
            if (q < len) {
                uint32_t p = q;
                if (p < 11u) b = lit_byte(p0, p);
                else if ((p -= 11u) < pre) b = bb[p];
                else if ((p -= pre) < 14u) b = lit_byte(p1, p);
                else if ((p -= 14u) < (uint32_t)CONDS_LEN) b = conds[p];
                else if ((p -= CONDS_LEN) < 1u) b = ',';
                else if ((p -= 1u) < post) b = bb[pre + p];
                else b = '}';
            }
            w |= b << (8 * k);
        }
        *reinterpret_cast<uint32_t*>(out + q0) = w;
    }
}

// node tiles: heartbeat list, node-init patches, node state (runs on the heartbeat stream)
__global__ __launch_bounds__(BLOCK) void k_emit_nodes(DevState S) {
    const uint32_t tile = blockIdx.x;
    const int t = threadIdx.x;
    const TickHdr* H = S.hdr;
    __shared__ InitJob ijobs[NODE_TILE];
    {
        const uint32_t first = tile * NODE_TILE + t * NODE_PER_THREAD;
        const uint64_t* base = S.tile_base + (size_t)tile * 4;
        uint32_t packed = 0;
        if (first < S.n_node_slots) packed = *reinterpret_cast<const uint32_t*>(S.node_state + first);
        NodeCls c[NODE_PER_THREAD];
        uint32_t v[3] = {0, 0, 0};  // hb, init, init bytes
        uint32_t ilen[NODE_PER_THREAD];
        uint64_t blob[NODE_PER_THREAD];
#pragma unroll
        for (int k = 0; k < NODE_PER_THREAD; k++) {
            c[k] = classify_node((uint8_t)(packed >> (8 * k)));
            v[0] += c[k].hb;
            ilen[k] = 0;
            blob[k] = 0;
            if (c[k].init) {
                blob[k] = S.node_blob[first + k];
                ilen[k] = init_patch_len(blob[k]);
                v[1]++;
                v[2] += (ilen[k] + 15u) & ~15u;
            }
        }
        uint32_t tot[3];
        block_excl_scan<3>(v, tot);
        InitJob* ij = ijobs;
        uint32_t newpacked = 0;
        uint32_t ji = v[1];
#pragma unroll
        for (int k = 0; k < NODE_PER_THREAD; k++) {
            const int32_t handle = S.node_handle_base + (int32_t)(first + k);
            if (c[k].hb) S.hb_nodes[base[0] + v[0]++] = handle;
            uint8_t s = (uint8_t)(packed >> (8 * k));
            if (c[k].init) {
                uint64_t ord = base[1] + ji;
                uint64_t off = H->init_base + base[2] + v[2];
                S.init_nodes[ord] = handle;
                S.init_off[ord] = off;
                S.init_len[ord] = ilen[k];
                ij[ji].slot = first + k;
                ij[ji].off = v[2];
                ji++;
                v[2] += (ilen[k] + 15u) & ~15u;
                s |= NS_CONFORMS;  // the apiserver applied the init patch
            }
            s &= (uint8_t)~NS_EVENT_LOCK;
            newpacked |= (uint32_t)s << (8 * k);
        }
        if (first < S.n_node_slots) *reinterpret_cast<uint32_t*>(S.node_state + first) = newpacked;
        __syncthreads();
        const uint64_t tile_bytes = H->init_base + base[2];
        for (uint32_t j = wave_id(); j < tot[1]; j += BLOCK / 64) {
            InitJob jb = ij[j];
            write_init_patch(S, S.node_blob[jb.slot], S.arena + tile_bytes + jb.off);
        }
    }
}

// pod tiles: delete list, IP assignment, pod patches, pod state; publishes the
// tick header to pinned host memory
__global__ __launch_bounds__(BLOCK) void k_emit_pods(DevState S) {
    const uint32_t ptile = blockIdx.x;
    const uint32_t tile = S.node_tiles + ptile;
    const int t = threadIdx.x;
    const TickHdr* H = S.hdr;
    if (ptile == 0 && t < 64) {
        // the header is final here (scan, pool plan): publish it zero-copy
        const uint64_t* src = reinterpret_cast<const uint64_t*>(H);
        uint64_t* dst = reinterpret_cast<uint64_t*>(S.hdr_host);
        for (int i = t; i < (int)(sizeof(TickHdr) / 8); i += 64) dst[i] = src[i];
        if (t == 0) {
            if (H->alloc_total) *S.pool_index = H->cursor_index;
            S.list_counts[0] = 0;  // multi-rank exchange lists for the next tick
            S.list_counts[1] = 0;
        }
        __threadfence_system();
    }
    __shared__ PodJob jobs[POD_TILE];  // 32 KiB
    const uint64_t* base = S.tile_base + (size_t)tile * 4;  // del, pp, pp_bytes, alloc
    const uint32_t first = ptile * POD_TILE + t * POD_PER_THREAD;
    const bool live = first < S.n_pod_slots && (first % S.cp) < S.pod_fill[first / S.cp];
    uint16_t st[POD_PER_THREAD];
    uint32_t ip[POD_PER_THREAD];
    PodCls c[POD_PER_THREAD];
    uint32_t v[4] = {0, 0, 0, 0};  // del, pp, pp bytes, alloc
    const uint32_t bucket_local = first / S.cp;
    {
        uint4 st4 = make_uint4(0, 0, 0, 0), nd4 = make_uint4(0, 0, 0, 0), ipa = make_uint4(0, 0, 0, 0),
              ipb = make_uint4(0, 0, 0, 0);
        if (live) {
            st4 = *reinterpret_cast<const uint4*>(S.pod_state + first);
            nd4 = *reinterpret_cast<const uint4*>(S.pod_node + first);
            ipa = *reinterpret_cast<const uint4*>(S.pod_ip + first);
            ipb = *reinterpret_cast<const uint4*>(S.pod_ip + first + 4);
        }
        const uint32_t stw[4] = {st4.x, st4.y, st4.z, st4.w};
        const uint32_t ndw[4] = {nd4.x, nd4.y, nd4.z, nd4.w};
        const uint32_t ips[8] = {ipa.x, ipa.y, ipa.z, ipa.w, ipb.x, ipb.y, ipb.z, ipb.w};
#pragma unroll
        for (int k = 0; k < POD_PER_THREAD; k++) {
            st[k] = (uint16_t)(stw[k >> 1] >> (16 * (k & 1)));
            uint16_t nl = (uint16_t)(ndw[k >> 1] >> (16 * (k & 1)));
            ip[k] = ips[k];
            uint8_t ntf = (st[k] & PS_USED) ? S.node_tick[bucket_local * S.cn + nl] : 0;
            c[k] = classify_pod(st[k], ntf, ip[k]);
            v[0] += c[k].del;
            if (c[k].need) {
                v[1]++;
                v[2] += S.specs[S.pod_spec[first + k]].max_len;
            }
            v[3] += c[k].alloc;
        }
    }
    uint32_t tot[4];
    block_excl_scan<4>(v, tot);
    const uint64_t take = H->take_usable, fin = H->fresh_in, fout0 = H->fresh_out_start, abase = H->alloc_base;
    uint32_t jl = v[1];
    bool dirty = false;
#pragma unroll
    for (int k = 0; k < POD_PER_THREAD; k++) {
        const uint32_t slot = first + k;
        const int32_t handle = S.pod_handle_base + (int32_t)slot;
        uint16_t s = st[k];
        if (c[k].del) {
            uint64_t ord = base[0] + v[0]++;
            S.del_pods[ord] = handle;
            S.del_fin[ord] = (s & PS_HAS_FIN) ? 1 : 0;
            s = 0;  // DeletePod -> Delete(grace 0): the object is gone
            dirty = true;
        }
        if (c[k].eval) {
            uint32_t pip = ip[k];
            if (c[k].alloc) {
                uint64_t o = base[3] + v[3]++;
                uint64_t g = abase + o;
                pip = g < take + fin ? S.alloc_addr[o] : (uint32_t)(fout0 + (g - take - fin));
            }
            if (c[k].need) {
                const bool stat = s & PS_STATUS_NONEMPTY;
                uint32_t hip = 0;
                if (stat) {
                    hip = (s & PS_HAS_HOST_IP) ? S.host_ip[slot] : S.node_ip;
                    if (!(s & PS_HAS_HOST_IP)) S.host_ip[slot] = hip;
                    if (pip != ip[k]) S.pod_ip[slot] = pip;
                }
                uint64_t ord = base[1] + jl;
                const SpecDesc& sd = S.specs[S.pod_spec[slot]];
                uint32_t len = sd.len_a + sd.len_b + sd.len_c + (stat ? 23u + ip_len(hip) + ip_len(pip) : 0u);
                S.pp_pods[ord] = handle;
                S.pp_off[ord] = H->pod_base + base[2] + v[2];
                S.pp_len[ord] = len;
                jobs[jl] = PodJob{slot, v[2], stat ? pip : 0u, hip};
                jl++;
                v[2] += S.specs[S.pod_spec[slot]].max_len;
                // the apiserver applied the patch
                s = (uint16_t)((s & ~PS_PHASE_MASK) | (PHASE_RUNNING << PS_PHASE_SHIFT) | PS_CONFORMS |
                               PS_STATUS_NONEMPTY | (stat ? PS_HAS_HOST_IP : 0));
            }
            s &= (uint16_t)~PS_EVENT;
            dirty = true;
        }
        st[k] = s;
    }
    if (live && dirty) {
        uint4 o;
        o.x = st[0] | (uint32_t)st[1] << 16;
        o.y = st[2] | (uint32_t)st[3] << 16;
        o.z = st[4] | (uint32_t)st[5] << 16;
        o.w = st[6] | (uint32_t)st[7] << 16;
        *reinterpret_cast<uint4*>(S.pod_state + first) = o;
    }
    __syncthreads();
    uint8_t* tile_out = S.arena + H->pod_base + base[2];
    for (uint32_t j = wave_id(); j < tot[1]; j += BLOCK / 64) write_pod_patch(S, jobs[j], tile_out + jobs[j].off);
}

// ---------------------------------------------------------------------------
// k_hb_fill: the n_hb heartbeat patches, 67 x 16 B each, from LDS
// ---------------------------------------------------------------------------
constexpr int HB_CHUNKS = HB_STRIDE / 16;  // 67
__global__ __launch_bounds__(BLOCK) void k_hb_fill(DevState S) {
    __shared__ uint4 tmpl[HB_CHUNKS];
    if (threadIdx.x < HB_CHUNKS) tmpl[threadIdx.x] = reinterpret_cast<const uint4*>(S.hb_tmpl)[threadIdx.x];
    __syncthreads();
    const uint64_t nchunks = (uint64_t)S.hdr->n_hb * HB_CHUNKS;
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    u32x4* dst = reinterpret_cast<u32x4*>(S.arena + S.hdr->hb_base);
    const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
    uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    uint32_t m = (uint32_t)(i % HB_CHUNKS);
    const uint32_t dm = (uint32_t)(stride % HB_CHUNKS);
    for (; i < nchunks; i += stride) {
        const uint4 v = tmpl[m];
        u32x4 w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, &dst[i]);  // write-once stream: do not keep in L2
        m += dm;
        if (m >= HB_CHUNKS) m -= HB_CHUNKS;
    }
}

// ---------------------------------------------------------------------------
// ingest + utility kernels
// ---------------------------------------------------------------------------
__global__ void k_apply_node_ops(DevState S, const NodeOp* ops, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    NodeOp o = ops[i];
    S.node_state[o.slot] = (uint8_t)((S.node_state[o.slot] & o.and_mask) | o.or_bits);
    if (o.set_blob) S.node_blob[o.slot] = o.blob;
}
__global__ void k_apply_pod_ops(DevState S, const PodOp* ops, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    PodOp o = ops[i];
    S.pod_state[o.slot] = (uint16_t)((S.pod_state[o.slot] & o.keep_mask) | o.bits);
    if (o.set_fields) {  // add / modify carry the whole decoded object
        S.pod_node[o.slot] = o.node;
        S.pod_spec[o.slot] = o.spec;
        S.pod_ctime[o.slot] = o.ctime;
        S.host_ip[o.slot] = o.host_ip;
        S.pod_ip[o.slot] = o.pod_ip;
    }
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
static inline uint32_t cdiv(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

void launch_apply_ops(const DevState& S, const NodeOp* nops, uint32_t nn, const PodOp* pops, uint32_t np,
                      hipStream_t st) {
    if (nn) hipLaunchKernelGGL(k_apply_node_ops, dim3(cdiv(nn, 256)), dim3(256), 0, st, S, nops, nn);
    if (np) hipLaunchKernelGGL(k_apply_pod_ops, dim3(cdiv(np, 256)), dim3(256), 0, st, S, pops, np);
}

void launch_pool_puts_now(const DevState& S, const uint32_t* ips, uint32_t n, hipStream_t st) {
    uint32_t g = n ? cdiv(n, 256) : 1;
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_pool_puts_now, dim3(g), dim3(256), 0, st, S, ips, n);
}

void launch_pool_apply(const DevState& S, const ListDesc* ld, int nranks, uint32_t max_n, hipStream_t st) {
    uint32_t g = max_n ? cdiv(max_n, 256) : 1;
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_pool_apply, dim3(g), dim3(256), 0, st, S, ld, nranks);
}

void launch_tick_front(const DevState& S, uint64_t start, int world, hipStream_t st) {
    hipLaunchKernelGGL(k_classify, dim3(S.node_tiles + S.pod_tiles), dim3(BLOCK), 0, st, S);
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(SCAN_THREADS), 0, st, S, start, world);
}

void launch_xreduce(const DevState& S, const XMsg* all, int world, int rank, hipStream_t st) {
    hipLaunchKernelGGL(k_xreduce, dim3(1), dim3(64), 0, st, S, all, world, rank);
}

void launch_pool_alloc(const DevState& S, hipStream_t st) {
    uint32_t nblk = cdiv(S.pool.words, POOL_WPB);
    hipLaunchKernelGGL(k_pool_prep, dim3(nblk), dim3(BLOCK), 0, st, S);
    hipLaunchKernelGGL(k_pool_select, dim3(nblk), dim3(BLOCK), 0, st, S, nblk);
}

void launch_emit_nodes(const DevState& S, hipStream_t st) {
    hipLaunchKernelGGL(k_emit_nodes, dim3(S.node_tiles), dim3(BLOCK), 0, st, S);
}

void launch_emit_pods(const DevState& S, hipStream_t st) {
    hipLaunchKernelGGL(k_emit_pods, dim3(S.pod_tiles), dim3(BLOCK), 0, st, S);
}

void launch_hb_fill(const DevState& S, uint32_t grid, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
    if (t0) hipExtLaunchKernelGGL(k_hb_fill, dim3(grid), dim3(BLOCK), 0, st, t0, t1, 0, S);  // kernel-exact timing
    else hipLaunchKernelGGL(k_hb_fill, dim3(grid), dim3(BLOCK), 0, st, S);
}

}  // namespace kwok
