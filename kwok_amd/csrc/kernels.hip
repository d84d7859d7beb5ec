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
    uint32_t f[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // del, eval, alloc, pp, pp_bytes, total, pending, running
    const bool live = first < S.n_pod_slots;
    uint4 st4 = make_uint4(0, 0, 0, 0), nd4 = make_uint4(0, 0, 0, 0), ipa = make_uint4(0, 0, 0, 0),
          ipb = make_uint4(0, 0, 0, 0);
    if (live) {
        st4 = *reinterpret_cast<const uint4*>(S.pod_state + first);
        if (st4.x | st4.y | st4.z | st4.w) {
            nd4 = *reinterpret_cast<const uint4*>(S.pod_node + first);
            ipa = *reinterpret_cast<const uint4*>(S.pod_ip + first);
            ipb = *reinterpret_cast<const uint4*>(S.pod_ip + first + 4);
        }
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
        wave_append(rel, ip, S.rel_list, &S.hdr->n_rel);
        wave_append(use, ip, S.use_list, &S.hdr->n_use);
        if (c.need) {
            f[3]++;
            f[4] += S.specs[S.pod_spec[first + k]].max_len;
        }
        bool total = c.used && !c.del;
        f[5] += total;
        f[6] += total && !c.need && c.phase == PHASE_PENDING;
        f[7] += total && (c.need || c.phase == PHASE_RUNNING);
    }
    block_sum<8>(f);
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
    }
}

// ---------------------------------------------------------------------------
// k_scan: one block of 1024 threads.  Exclusive scan of the tile counts ->
// tile bases; arena layout; counters; per-tick heartbeat template.
// ---------------------------------------------------------------------------
constexpr int SCAN_THREADS = 1024;
__global__ __launch_bounds__(SCAN_THREADS) void k_scan(DevState S, uint64_t now_unix, uint64_t start_unix,
                                                        int world_size) {
    const int t = threadIdx.x;
    const uint32_t T = S.node_tiles + S.pod_tiles;
    const uint32_t per = (T + SCAN_THREADS - 1) / SCAN_THREADS;
    const uint32_t lo = min(T, t * per), hi = min(T, lo + per);
    // fields scanned: hb, init, init_bytes (nodes); del, pp, pp_bytes, alloc (pods)
    constexpr int NS = 7;
    const int fld[NS] = {TF_HB, TF_INIT, TF_INIT_BYTES, TF_DEL, TF_PP, TF_PP_BYTES, TF_ALLOC};
    uint64_t sum[NS] = {0, 0, 0, 0, 0, 0, 0};
    uint64_t cnt[6] = {0, 0, 0, 0, 0, 0};  // lock, managed, ready, eval, total, pending+running packed below
    uint64_t pend = 0, run = 0;
    for (uint32_t i = lo; i < hi; i++) {
        const uint32_t* o = S.tiles + (size_t)i * TF_STRIDE;
        bool node = i < S.node_tiles;
#pragma unroll
        for (int f = 0; f < NS; f++) sum[f] += (node == (f < 3)) ? o[fld[f]] : 0u;
        if (node) {
            cnt[0] += o[TF_LOCK];
            cnt[1] += o[TF_MANAGED];
            cnt[2] += o[TF_READY];
        } else {
            cnt[3] += o[TF_EVAL];
            cnt[4] += o[TF_TOTAL];
            pend += o[TF_PENDING];
            run += o[TF_RUNNING];
        }
    }
    // block scan (u64) through LDS, Hillis-Steele over 1024 entries
    __shared__ uint64_t sh[SCAN_THREADS];
    uint64_t excl[NS];
    uint64_t total[NS];
    for (int f = 0; f < NS; f++) {
        sh[t] = sum[f];
        __syncthreads();
        for (int off = 1; off < SCAN_THREADS; off <<= 1) {
            uint64_t y = t >= off ? sh[t - off] : 0;
            __syncthreads();
            sh[t] += y;
            __syncthreads();
        }
        excl[f] = sh[t] - sum[f];
        total[f] = sh[SCAN_THREADS - 1];
        __syncthreads();
    }
    // reductions of the plain counters
    uint64_t red[8] = {cnt[0], cnt[1], cnt[2], cnt[3], cnt[4], pend, run, 0};
    for (int f = 0; f < 7; f++) {
        sh[t] = red[f];
        __syncthreads();
        for (int s = SCAN_THREADS / 2; s > 0; s >>= 1) {
            if (t < s) sh[t] += sh[t + s];
            __syncthreads();
        }
        red[f] = sh[0];
        __syncthreads();
    }
    // second pass: per-tile bases
    uint64_t run_b[NS];
    for (int f = 0; f < NS; f++) run_b[f] = excl[f];
    for (uint32_t i = lo; i < hi; i++) {
        const uint32_t* o = S.tiles + (size_t)i * TF_STRIDE;
        uint64_t* b = S.tile_base + (size_t)i * 4;
        if (i < S.node_tiles) {
            b[0] = run_b[0];
            b[1] = run_b[1];
            b[2] = run_b[2];
            run_b[0] += o[TF_HB];
            run_b[1] += o[TF_INIT];
            run_b[2] += o[TF_INIT_BYTES];
        } else {
            b[0] = run_b[3];
            b[1] = run_b[4];
            b[2] = run_b[5];
            b[3] = run_b[6];
            run_b[3] += o[TF_DEL];
            run_b[4] += o[TF_PP];
            run_b[5] += o[TF_PP_BYTES];
            run_b[6] += o[TF_ALLOC];
        }
    }
    TickHdr* H = S.hdr;
    if (t == 0) {
        H->n_hb = (uint32_t)total[0];
        H->n_init = (uint32_t)total[1];
        H->init_bytes = total[2];
        H->n_del = (uint32_t)total[3];
        H->n_pp = (uint32_t)total[4];
        H->pp_bytes = total[5];
        H->n_alloc_local = (uint32_t)total[6];
        H->n_lock = (uint32_t)red[0];
        H->n_eval = (uint32_t)red[3];
        H->hb_base = 0;
        H->init_base = total[0] * (uint64_t)HB_STRIDE;
        H->pod_base = H->init_base + total[2];
        H->arena_bytes = H->pod_base + total[5];
        H->overflow = H->arena_bytes > S.arena_cap;
        uint64_t* L = H->local_counters;
        L[0] = total[0];         // heartbeat
        L[1] = total[1];         // node_init
        L[2] = total[4];         // pod_patch
        L[3] = total[3];         // delete
        L[4] = total[6];         // alloc
        L[5] = H->n_rel;         // release
        L[6] = red[3];           // evaluated
        L[7] = red[0];           // lock_checked
        L[8] = red[1];           // nodes_managed
        L[9] = red[2];           // nodes_ready
        L[10] = red[4];          // pods_total
        L[11] = red[5];          // pods_pending
        L[12] = red[6];          // pods_running
        if (world_size == 1) {
            for (int k = 0; k < 16; k++) H->counters[k] = L[k];
            H->alloc_total = total[6];
            H->alloc_base = 0;
        }
    }
    // exchange message (multi-rank): header + inline lists
    if (world_size > 1) {
        __syncthreads();
        XMsg* X = S.xmsg;
        uint32_t nu = H->n_use, nr = H->n_rel;
        if (t == 0) {
            X->alloc = total[6];
            X->n_use = nu;
            X->n_rel = nr;
            for (int k = 0; k < 16; k++) X->counters[k] = H->local_counters[k];
        }
        if (nu + nr <= (uint32_t)XINLINE) {
            for (uint32_t i = t; i < nu; i += SCAN_THREADS) X->ips[i] = S.use_list[i];
            for (uint32_t i = t; i < nr; i += SCAN_THREADS) X->ips[nu + i] = S.rel_list[i];
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
}

// ---------------------------------------------------------------------------
// ipPool kernels on the replicated bitmaps
// ---------------------------------------------------------------------------
// Use (utils.go:110-117): set `used` for every listed in-CIDR address
__global__ void k_pool_uses(DevState S, const ListDesc* ld, int nranks) {
    for (int r = 0; r < nranks; r++) {
        uint32_t n = nranks == 1 && ld[0].count_from_hdr ? S.hdr->n_use : ld[r].n_use;
        const uint32_t* ips = ld[r].use;
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
            uint32_t ip = ips[i];
            if (!in_cidr(S.pool, ip)) continue;
            uint64_t b = ip - S.pool.net;
            atomicOr((unsigned long long*)&S.used_bm[b >> 6], 1ull << (b & 63));
        }
    }
}
// Put (utils.go:100-108): delete from used, add to usable
__global__ void k_pool_puts(DevState S, const ListDesc* ld, int nranks) {
    for (int r = 0; r < nranks; r++) {
        uint32_t n = nranks == 1 && ld[0].count_from_hdr ? S.hdr->n_rel : ld[r].n_rel;
        const uint32_t* ips = ld[r].rel;
        for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
            uint32_t ip = ips[i];
            if (!in_cidr(S.pool, ip)) continue;
            uint64_t b = ip - S.pool.net;
            atomicAnd((unsigned long long*)&S.used_bm[b >> 6], ~(1ull << (b & 63)));
            atomicOr((unsigned long long*)&S.usable_bm[b >> 6], 1ull << (b & 63));
        }
    }
}

// free bits of `used` at or after the fresh cursor (ipPool.new skips used)
__device__ __forceinline__ uint64_t free_mask(const DevState& S, uint64_t w, uint64_t cursor_bit) {
    uint64_t lo = w * 64;
    if (lo + 64 <= cursor_bit) return 0;
    // ipPool.new skips `used`; addresses still usable this tick are all taken
    // by Get's reuse branch before any fresh allocation happens (take = U when F > 0)
    uint64_t m = ~S.used_bm[w] & ~S.usable_bm[w];
    if (cursor_bit > lo) m &= ~0ull << (cursor_bit - lo);
    if (lo + 64 > S.pool.size) m &= (S.pool.size - lo >= 64) ? ~0ull : ((1ull << (S.pool.size - lo)) - 1);
    return m;
}
__device__ __forceinline__ uint64_t cursor_bit(const DevState& S) {
    uint64_t a = (uint64_t)S.pool.base + *S.pool_index;  // ipPool.new: addIP(cidr.IP, index)
    return a >= S.pool.net ? a - S.pool.net : 0;
}

constexpr int POOL_WPB = BLOCK * 4;  // bitmap words per block

// K1: per-block counts of usable bits and free bits (from cursor)
__global__ __launch_bounds__(BLOCK) void k_pool_count(DevState S) {
    if (S.hdr->alloc_total == 0) return;
    const uint64_t cb = cursor_bit(S);
    uint32_t f[2] = {0, 0};
    for (int k = 0; k < 4; k++) {
        uint64_t w = (uint64_t)blockIdx.x * POOL_WPB + threadIdx.x * 4 + k;
        if (w < S.pool.words) {
            f[0] += __popcll(S.usable_bm[w]);
            f[1] += __popcll(free_mask(S, w, cb));
        }
    }
    block_sum<2>(f);
    if (threadIdx.x == 0) {
        S.pool_blk[2 * blockIdx.x] = f[0];
        S.pool_blk[2 * blockIdx.x + 1] = f[1];
    }
}

// K2: one thread-block: scan block sums; plan = take `take_usable` lowest
// usable addresses (the build's deterministic reuse rule), then fresh ones.
__global__ __launch_bounds__(SCAN_THREADS) void k_pool_plan(DevState S, uint32_t nblk) {
    TickHdr* H = S.hdr;
    if (H->alloc_total == 0) return;
    __shared__ uint64_t su[SCAN_THREADS], sf[SCAN_THREADS];
    const int t = threadIdx.x;
    const uint32_t per = (nblk + SCAN_THREADS - 1) / SCAN_THREADS;
    const uint32_t lo = min(nblk, t * per), hi = min(nblk, lo + per);
    uint64_t u = 0, fr = 0;
    for (uint32_t i = lo; i < hi; i++) u += S.pool_blk[2 * i], fr += S.pool_blk[2 * i + 1];
    su[t] = u;
    sf[t] = fr;
    __syncthreads();
    for (int off = 1; off < SCAN_THREADS; off <<= 1) {
        uint64_t a = t >= off ? su[t - off] : 0, b = t >= off ? sf[t - off] : 0;
        __syncthreads();
        su[t] += a;
        sf[t] += b;
        __syncthreads();
    }
    uint64_t eu = su[t] - u, ef = sf[t] - fr;
    for (uint32_t i = lo; i < hi; i++) {
        S.pool_blk_base[2 * i] = eu;
        S.pool_blk_base[2 * i + 1] = ef;
        eu += S.pool_blk[2 * i];
        ef += S.pool_blk[2 * i + 1];
    }
    if (t == 0) {
        uint64_t U = su[SCAN_THREADS - 1], Fin = sf[SCAN_THREADS - 1];
        uint64_t A = H->alloc_total;
        uint64_t take = A < U ? A : U;
        uint64_t F = A - take;
        uint64_t fin = F < Fin ? F : Fin;
        uint64_t fout = F - fin;
        uint64_t cur = (uint64_t)S.pool.base + *S.pool_index;
        uint64_t end = (uint64_t)S.pool.net + S.pool.size;
        H->usable_total = U;
        H->take_usable = take;
        H->fresh_in = fin;
        H->fresh_out_start = cur > end ? cur : end;
        // index after the last fresh address; committed to pool_index by k_emit
        H->cursor_index = fout ? H->fresh_out_start + fout - S.pool.base : *S.pool_index;
        // (fin > 0 && fout == 0: k_pool_select sets it)
    }
}

__device__ __forceinline__ uint32_t select_bit(uint64_t m, uint32_t k) {
    // position of the k-th (0-based) set bit of m
    for (uint32_t i = 0; i < k; i++) m &= m - 1;
    return (uint32_t)(__ffsll((unsigned long long)m) - 1);
}

// K3: select + commit.  Allocation ordinal g (global, canonical order):
//   g < take_usable           -> g-th lowest usable address
//   g < take_usable+fresh_in  -> (g-take)-th free in-CIDR address from the cursor
//   otherwise                 -> fresh_out_start + (g - take - fresh_in)   (beyond the CIDR)
// Every rank commits ALL A allocations to its pool replica; it records the
// addresses of its own range [alloc_base, alloc_base + n_alloc_local).
__global__ __launch_bounds__(BLOCK) void k_pool_select(DevState S) {
    TickHdr* H = S.hdr;
    if (H->alloc_total == 0) return;
    const uint64_t take = H->take_usable, fin = H->fresh_in;
    const uint64_t lo_g = H->alloc_base, hi_g = lo_g + H->n_alloc_local;
    const uint64_t cb = cursor_bit(S);
    const bool advance = fin > 0 && H->alloc_total == take + fin;
    uint32_t c[2][4];
    uint64_t wu[4], wf[4];
    uint32_t v[2] = {0, 0};
    for (int k = 0; k < 4; k++) {
        uint64_t w = (uint64_t)blockIdx.x * POOL_WPB + threadIdx.x * 4 + k;
        wu[k] = w < S.pool.words ? S.usable_bm[w] : 0;
        wf[k] = w < S.pool.words ? free_mask(S, w, cb) : 0;
        c[0][k] = __popcll(wu[k]);
        c[1][k] = __popcll(wf[k]);
        v[0] += c[0][k];
        v[1] += c[1][k];
    }
    uint32_t tot[2];
    block_excl_scan<2>(v, tot);
    uint64_t ru = S.pool_blk_base[2 * blockIdx.x] + v[0];
    uint64_t rf = S.pool_blk_base[2 * blockIdx.x + 1] + v[1];
    for (int k = 0; k < 4; k++) {
        uint64_t w = (uint64_t)blockIdx.x * POOL_WPB + threadIdx.x * 4 + k;
        if (w >= S.pool.words) break;
        // usable bits with rank < take
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
            S.usable_bm[w] &= ~sel;  // ipPool.Get: delete(usable) ...
            S.used_bm[w] |= sel;     // ... used[ip] = struct{}{}  (one thread owns word w)
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
            S.used_bm[w] |= sel;  // ipPool.new: used[ip] (usable set/unset nets to unchanged)
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

__global__ __launch_bounds__(BLOCK) void k_emit(DevState S) {
    const uint32_t tile = blockIdx.x;
    const int t = threadIdx.x;
    const TickHdr* H = S.hdr;
    if (tile == 0 && t == 0 && H->alloc_total) *S.pool_index = H->cursor_index;
    __shared__ PodJob jobs[POD_TILE];  // 32 KiB (node tiles reuse it for InitJob)
    if (tile < S.node_tiles) {
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
        InitJob* ij = reinterpret_cast<InitJob*>(jobs);
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
        return;
    }
    // ---- pods ----
    const uint32_t ptile = tile - S.node_tiles;
    const uint64_t* base = S.tile_base + (size_t)tile * 4;  // del, pp, pp_bytes, alloc
    const uint32_t first = ptile * POD_TILE + t * POD_PER_THREAD;
    const bool live = first < S.n_pod_slots;
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
            if (st4.x | st4.y | st4.z | st4.w) {
                nd4 = *reinterpret_cast<const uint4*>(S.pod_node + first);
                ipa = *reinterpret_cast<const uint4*>(S.pod_ip + first);
                ipb = *reinterpret_cast<const uint4*>(S.pod_ip + first + 4);
            }
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
    uint4* dst = reinterpret_cast<uint4*>(S.arena + S.hdr->hb_base);
    const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
    uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    uint32_t m = (uint32_t)(i % HB_CHUNKS);
    const uint32_t dm = (uint32_t)(stride % HB_CHUNKS);
    for (; i < nchunks; i += stride) {
        dst[i] = tmpl[m];
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
__global__ void k_reset_lists(DevState S) {
    if (threadIdx.x == 0) {
        S.hdr->n_use = 0;
        S.hdr->n_rel = 0;
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

void launch_pool_lists(const DevState& S, const ListDesc* ld, int nranks, bool uses, uint32_t max_n,
                       hipStream_t st) {
    uint32_t g = max_n ? cdiv(max_n, 256) : 1024;
    if (g > 2048) g = 2048;
    if (uses) hipLaunchKernelGGL(k_pool_uses, dim3(g), dim3(256), 0, st, S, ld, nranks);
    else hipLaunchKernelGGL(k_pool_puts, dim3(g), dim3(256), 0, st, S, ld, nranks);
}

void launch_tick_front(const DevState& S, uint64_t now, uint64_t start, int world, hipStream_t st) {
    hipLaunchKernelGGL(k_reset_lists, dim3(1), dim3(64), 0, st, S);
    hipLaunchKernelGGL(k_classify, dim3(S.node_tiles + S.pod_tiles), dim3(BLOCK), 0, st, S);
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(SCAN_THREADS), 0, st, S, now, start, world);
}

void launch_xreduce(const DevState& S, const XMsg* all, int world, int rank, hipStream_t st) {
    hipLaunchKernelGGL(k_xreduce, dim3(1), dim3(64), 0, st, S, all, world, rank);
}

void launch_pool_alloc(const DevState& S, hipStream_t st) {
    uint32_t nblk = cdiv(S.pool.words, POOL_WPB);
    hipLaunchKernelGGL(k_pool_count, dim3(nblk), dim3(BLOCK), 0, st, S);
    hipLaunchKernelGGL(k_pool_plan, dim3(1), dim3(SCAN_THREADS), 0, st, S, nblk);
    hipLaunchKernelGGL(k_pool_select, dim3(nblk), dim3(BLOCK), 0, st, S);
}

void launch_emit(const DevState& S, hipStream_t st) {
    hipLaunchKernelGGL(k_emit, dim3(S.node_tiles + S.pod_tiles), dim3(BLOCK), 0, st, S);
}

void launch_hb_fill(const DevState& S, uint32_t grid, hipStream_t st) {
    hipLaunchKernelGGL(k_hb_fill, dim3(grid), dim3(BLOCK), 0, st, S);
}

}  // namespace kwok
