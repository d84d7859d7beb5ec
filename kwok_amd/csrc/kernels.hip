// kernels.hip - gfx950 kernels of one kwok controller tick.
//
// A tick is a set of memory-bound sweeps over struct-of-arrays state in HBM;
// nothing here is a dense contraction, so there is no MFMA.  The single-rank
// tick is ONE launch (k_tick) of two kinds of blocks:
//
//   chain blocks     one per bucket range: classify nodes and live pod groups
//                    (node_controller.go:206-223,356-391; pod_controller.go:
//                    252-269,306-343,377-439), heartbeat handle list, Use/Put
//                    bits; publish a record and arrive.  Only blocks with
//                    something to emit go on: prefix over the records, the
//                    ipPool phase (utils.go:52-117) in ticks with Gets or Puts,
//                    compaction + byte emission of their dirty chunks.
//   streamer blocks  the n_managed identical 1059-byte heartbeat patches
//                    (node_controller.go:145-204,393-401) from an LDS template
//                    with 16-byte non-temporal stores, overlapping the
//                    latency-bound classification.
//
// In the steady state no block waits on another: the last chain block to
// arrive reduces the records into the tick header.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stddef.h>

#include <type_traits>

#include "device.h"
#include "kernels.h"

namespace kwok {

// ---------------------------------------------------------------------------
// small device helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }  // uniform

// wave-wide inclusive scan (64 lanes) with DPP row shifts and row broadcasts:
// six VALU adds with a cross-lane source operand, no LDS round trip (a
// __shfl_up is a ds_bpermute, ~100+ cycles each, six of them dependent).
// Every lane of the wave must be active.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_src(uint32_t x) {
    // lanes whose source lies outside the row / rows outside ROW_MASK read 0
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROW_MASK, 0xF, false);
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += dpp_src<0x111, 0xF>(x);  // row_shr:1
    x += dpp_src<0x112, 0xF>(x);  // row_shr:2
    x += dpp_src<0x114, 0xF>(x);  // row_shr:4
    x += dpp_src<0x118, 0xF>(x);  // row_shr:8   -> inclusive within each row of 16
    x += dpp_src<0x142, 0xA>(x);  // row_bcast:15 (lane 15 of row r into row r+1, rows 1 and 3)
    x += dpp_src<0x143, 0xC>(x);  // row_bcast:31 (lane 31 into rows 2 and 3)
    return x;
}
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint64_t dpp_src64(uint64_t x) {
    const uint32_t lo = dpp_src<CTRL, ROW_MASK>((uint32_t)x), hi = dpp_src<CTRL, ROW_MASK>((uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t x) {
    x += dpp_src64<0x111, 0xF>(x);
    x += dpp_src64<0x112, 0xF>(x);
    x += dpp_src64<0x114, 0xF>(x);
    x += dpp_src64<0x118, 0xF>(x);
    x += dpp_src64<0x142, 0xA>(x);
    x += dpp_src64<0x143, 0xC>(x);
    return x;
}
// wave total, uniform (scalar) result
__device__ __forceinline__ uint64_t wave_sum64(uint64_t x) {
    x = wave_incl_scan64(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, 63);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), 63);
    return ((uint64_t)hi << 32) | lo;
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

// the same over one wave (no barrier): v <- exclusive prefix, tot <- wave totals
template <int NF>
__device__ __forceinline__ void wave_excl_scan(uint32_t (&v)[NF], uint32_t (&tot)[NF]) {
#pragma unroll
    for (int f = 0; f < NF; f++) {
        const uint32_t incl = wave_incl_scan(v[f]);
        tot[f] = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        v[f] = incl - v[f];
    }
}

template <int NF>
__device__ __forceinline__ void block_sum(uint32_t (&v)[NF]) {
    uint32_t tot[NF];
    block_excl_scan<NF>(v, tot);
#pragma unroll
    for (int f = 0; f < NF; f++) v[f] = tot[f];
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
    // branch-free: each octet's digits packed (1-3 bytes) and its '.', appended
    // to a 128-bit little-endian accumulator at the running length
    uint64_t lo = 0, hi = 0;
    uint32_t n = 0;
#pragma unroll
    for (int k = 3; k >= 0; k--) {
        const uint32_t o = (ip >> (8 * k)) & 255u;
        const uint32_t d2 = o / 100u, d1 = (o / 10u) % 10u, d0 = o % 10u;
        const uint32_t w = o >= 100u ? 3u : (o >= 10u ? 2u : 1u);
        uint32_t v = o >= 100u ? ('0' + d2) | ('0' + d1) << 8 | ('0' + d0) << 16
                                : (o >= 10u ? ('0' + d1) | ('0' + d0) << 8 : ('0' + d0));
        uint32_t m = w;
        if (k) {
            v |= (uint32_t)'.' << (8 * w);
            m++;
        }
        // append the m (<= 4) bytes of v at byte n (< 16)
        const uint64_t x = v;
        const uint32_t sh = 8u * (n & 7u);
        const uint64_t part_lo = x << sh, spill = sh ? x >> (64u - sh) : 0ull;
        lo |= n < 8u ? part_lo : 0ull;
        hi |= n < 8u ? spill : part_lo;
        n += m;
    }
    IpStr r;
    r.lo = lo;
    r.hi = hi;
    r.len = n;
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

// byte i (< 16) of a short literal, from two compile-time words (no memory access)
struct Lit16 {
    uint64_t lo, hi;
};
constexpr Lit16 lit16(const char* s) {
    Lit16 r{0, 0};
    for (int i = 0; i < 16 && s[i]; i++) {
        if (i < 8) r.lo |= (uint64_t)(uint8_t)s[i] << (8 * i);
        else r.hi |= (uint64_t)(uint8_t)s[i] << (8 * (i - 8));
    }
    return r;
}

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
__device__ __forceinline__ PodCls classify_pod(uint16_t st, uint8_t ntf, uint32_t pod_ip, bool cni) {
    PodCls c;
    c.used = st & PS_USED;
    c.del = c.used && (st & PS_DELETE_PENDING);
    c.eval = c.used && !c.del && ((st & PS_EVENT) || ((ntf & NT_RELOCK) && !(st & PS_DISREGARD)));
    c.phase = (st & PS_PHASE_MASK) >> PS_PHASE_SHIFT;
    // `{{ with .status }} ... {{ with .podIP }} . {{ else }} {{ PodIP }}` (pod.status.tpl:44-47);
    // EnableCNI: the podIP comes from cni.Setup instead (pod_controller.go:383-389)
    c.alloc = !cni && c.eval && (st & PS_STATUS_NONEMPTY) && pod_ip == 0;
    // computePatchData: Pending always patches; otherwise the strategic merge must change something.
    // EnableCNI: a pod without an IP is waiting for cni.Setup (configurePod fails: no patch)
    c.need = c.eval && (cni ? pod_ip != 0 && (c.phase != PHASE_RUNNING || !(st & PS_CONFORMS) || !(st & PS_HAS_HOST_IP))
                            : (c.phase != PHASE_RUNNING || !(st & PS_CONFORMS) || !(st & PS_HAS_HOST_IP) || pod_ip == 0));
    return c;
}

// framed blob (templates.cpp build_node_blob): pre | heartbeat conditions | post
__device__ __forceinline__ uint32_t init_patch_len(const DevState& S, uint64_t blob) {
    const uint32_t pre = (uint32_t)(blob >> 32) & 0xFFFF, post = (uint32_t)(blob >> 48);
    return pre + S.conds_len + post;
}

// ---------------------------------------------------------------------------
// ipPool phase (only in ticks with Gets or Puts)
//
// Order inside a tick (DESIGN.md "Tick contract"): every Use (configurePod,
// pod_controller.go:378-382) -> every Put of this tick's deletions
// (pod_controller.go:329-336 / utils.go:100-108) -> the Gets (utils.go:83-98)
// in canonical order.  Uses set `used` directly; Puts accumulate in rel_bm
// (atomic ORs commute with the Uses) and the prep step folds them:
//   used &= ~rel, usable |= rel.
// ---------------------------------------------------------------------------
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

// bitmap words per word-block: BLOCK * W, W = POOL_WPT_MULTI on a multi-rank
// engine (the N-rank pool is N times larger: half the passes, twice the loads in
// flight), POOL_WPT otherwise (a single rank's pool phase runs among its dirty
// blocks: more, smaller word-blocks keep them all busy)
constexpr int POOL_WPT_MULTI = 8;
static_assert(POOL_WPT >= POOL_WPT_MIN, "pool_blk is allocated for POOL_WPT_MIN");

// a thread's words of one word-block (pass k: word wb * POOL_WPB + k * BLOCK +
// thread), as the prep pass left them: the select pass of the same block takes
// them from registers instead of reading them again
template <int W>
struct PoolWords {
    uint64_t used[W], usable[W];
};
template <int W>
__device__ __forceinline__ void pool_prep_wblock(const DevState& S, uint32_t wb, bool fold, bool count, PoolWords<W>& pw) {
    const uint64_t cb = cursor_bit(S);
    uint32_t f[2] = {0, 0};
#pragma unroll
    for (int k = 0; k < W; k++) {
        const uint64_t w = (uint64_t)wb * (BLOCK * W) + (uint64_t)k * BLOCK + threadIdx.x;
        pw.used[k] = ~0ull, pw.usable[k] = 0ull;
        if (w >= S.pool.words) continue;
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
        pw.used[k] = used, pw.usable[k] = usable;
    }
    block_sum<2>(f);
    if (threadIdx.x == 0 && count) {
        S.pool_blk[2 * wb] = f[0];
        S.pool_blk[2 * wb + 1] = f[1];
    }
}

struct PoolPlan {
    uint64_t U, Fin, take, fin, fout, fout0;
};
// The word-block counts' prefixes, read once per block: thread t sums its chunk
// [t * per, +per) of the counts, the chunk sums are scanned over the block into
// LDS and the totals returned; a word-block's prefix is then its chunk's plus
// the counts before it inside the chunk (pool_prefix).  (Reading every count
// per selected word-block cost the /4 pool of an 8-rank fleet - 4096 word-blocks,
// 8 per chain block - a serial 64-step loop per word-block.)
struct PoolPre {
    uint64_t U, Fin;
    uint32_t per;
};
__device__ __forceinline__ PoolPre pool_scan(const DevState& S, uint32_t nwb, uint64_t (&cp)[2][BLOCK]) {
    __shared__ uint64_t ws[BLOCK / 64][2];
    const uint32_t per = (nwb + BLOCK - 1) / BLOCK;
    const uint32_t i0 = min(threadIdx.x * per, nwb), i1 = min(i0 + per, nwb);
    uint64_t v[2] = {0, 0};
#pragma unroll 8
    for (uint32_t i = i0; i < i1; i++) v[0] += S.pool_blk[2 * i], v[1] += S.pool_blk[2 * i + 1];
    const int l = lane_id(), w = wave_id();
    uint64_t incl[2];
#pragma unroll
    for (int f = 0; f < 2; f++) {
        incl[f] = wave_incl_scan64(v[f]);
        if (l == 63) ws[w][f] = incl[f];
    }
    __syncthreads();
    uint64_t tot[2];
#pragma unroll
    for (int f = 0; f < 2; f++) {
        uint64_t pre = 0, t = 0;
#pragma unroll
        for (int k = 0; k < BLOCK / 64; k++) {
            const uint64_t s = ws[k][f];
            pre += k < w ? s : 0ull;
            t += s;
        }
        cp[f][threadIdx.x] = pre + incl[f] - v[f];
        tot[f] = t;
    }
    __syncthreads();
    return PoolPre{tot[0], tot[1], per};
}
// usable / free bits of the word-blocks before wb (uniform)
__device__ __forceinline__ void pool_prefix(const DevState& S, const PoolPre& q, const uint64_t (&cp)[2][BLOCK], uint32_t wb,
                                            uint64_t* bu, uint64_t* bf) {
    const uint32_t o = wb / q.per;
    uint64_t u = 0, f = 0;
    for (uint32_t i = o * q.per + lane_id(); i < wb; i += 64) u += S.pool_blk[2 * i], f += S.pool_blk[2 * i + 1];
    *bu = cp[0][o] + wave_sum64(u);
    *bf = cp[1][o] + wave_sum64(f);
}
// every block derives the same plan from the totals
__device__ __forceinline__ PoolPlan pool_plan(const DevState& S, uint64_t A, const PoolPre& q) {
    PoolPlan p;
    p.U = q.U;
    p.Fin = q.Fin;
    p.take = A < p.U ? A : p.U;
    const uint64_t F = A - p.take;
    p.fin = F < p.Fin ? F : p.Fin;
    p.fout = F - p.fin;
    const uint64_t cur = (uint64_t)S.pool.base + *S.pool_index;
    const uint64_t end = (uint64_t)S.pool.net + S.pool.size;
    p.fout0 = cur > end ? cur : end;
    return p;
}

// the n-th (0-indexed) set bit of m (m has more than n set bits): a popcount
// binary search, branch-free
__device__ __forceinline__ uint32_t nth_set_bit(uint64_t m, uint32_t n) {
    uint32_t pos = 0;
#pragma unroll
    for (int wd = 32; wd >= 1; wd >>= 1) {
        const uint32_t c = (uint32_t)__popcll(m & ((1ull << wd) - 1ull));
        const bool up = n >= c;
        n = up ? n - c : n;
        m = up ? m >> wd : m;
        pos += up ? (uint32_t)wd : 0u;
    }
    return pos;
}
// the lowest n of the cnt set bits of m
__device__ __forceinline__ uint64_t lowest_bits(uint64_t m, uint32_t n, uint32_t cnt) {
    if (n >= cnt) return m;
    if (n == 0) return 0;
    return m & ((1ull << nth_set_bit(m, n)) - 1ull);
}
// The wave's selections as alloc_addr entries, written coalesced.  Lane l took
// the lowest n of the set bits of m (word w0 + l); the wave's selections are the
// ordinals [g0, g0 + total) in lane order.  Every word taken whole (a fresh
// fleet's run of free words): the addresses are the words' bits in order, one
// entry per lane per store.  At most 8 per word (a churned pool's scattered
// usable addresses): each lane its own, one per step.  Otherwise lane by lane (a
// uniform walk over the lanes that took bits): the wave writes lane j's
// selections together, lane l its (l)-th set bit.  Only this rank's ordinals
// [lo_g, hi_g) are recorded.
__device__ __forceinline__ void wave_write_addrs(const DevState& S, uint64_t g0, uint32_t n, uint64_t m, uint64_t w0,
                                                 uint64_t lo_g, uint64_t hi_g) {
    const uint32_t l = lane_id();
    const uint32_t incl = wave_incl_scan(n);
    const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    if (total == 0) return;
    if (g0 >= hi_g || g0 + total <= lo_g) return;
    if (__ballot(n != 64u) == 0) {
        for (uint32_t p = l; p < total; p += 64) {
            const uint64_t g = g0 + p;
            if (g >= lo_g && g < hi_g) S.alloc_addr[g - lo_g] = S.pool.net + (uint32_t)(w0 * 64 + p);
        }
        return;
    }
    const uint32_t ex = incl - n;
    // sparse words (a churned fleet's reused addresses: a few per word): each lane
    // writes its own selections, one per step, neighbouring lanes' ordinals adjacent
    uint32_t mx = n;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    if (mx <= 8u) {
        uint64_t mm = m;
        for (uint32_t i = 0; i < mx; i++) {
            if (i < n) {
                const uint64_t g = g0 + ex + i;
                if (g >= lo_g && g < hi_g) S.alloc_addr[g - lo_g] = S.pool.net + (uint32_t)((w0 + l) * 64 + __builtin_ctzll(mm));
                mm &= mm - 1;
            }
        }
        return;
    }
    for (uint64_t act = __ballot(n != 0); act; act &= act - 1) {
        const int j = (int)__builtin_ctzll(act);
        const uint32_t nj = (uint32_t)__builtin_amdgcn_readlane((int)n, j);
        const uint32_t exj = (uint32_t)__builtin_amdgcn_readlane((int)ex, j);
        const uint64_t mj = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)m, j) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(m >> 32), j) << 32);
        if (l < nj) {
            const uint64_t g = g0 + exj + l;
            if (g >= lo_g && g < hi_g) S.alloc_addr[g - lo_g] = S.pool.net + (uint32_t)((w0 + (uint32_t)j) * 64 + nth_set_bit(mj, l));
        }
    }
}

// select + commit for word-block wb.  Allocation ordinal g (global, canonical order):
//   g < take            -> g-th lowest usable address (the build's reuse rule)
//   g < take + fin      -> (g-take)-th free in-CIDR address from the cursor
//   otherwise           -> fout0 + (g - take - fin)          (beyond the CIDR)
// Every rank commits ALL allocations to its replica; it records the addresses
// of its own ordinals [alloc_base, alloc_base + n_alloc_local).
// Words are taken k-major (pass k: words wb * POOL_WPB + k * BLOCK + thread), so
// a pass's words are consecutive across the block and its selections are one
// contiguous ordinal range per wave: each lane commits its word's selections
// as two masks, and the wave writes their addresses coalesced (one alloc_addr
// entry per lane per store, instead of a serial bit walk per lane with one
// scattered store per address: the 1M x 10M initial tick's 10M fresh Gets).
// pw: the block's words of wb from its prep pass (null: read them)
template <int W>
__device__ __forceinline__ void pool_select_wblock(const DevState& S, uint32_t wb, const PoolPlan& p, uint64_t base_u, uint64_t base_f,
                                   uint64_t lo_g, uint64_t hi_g, uint64_t* cursor_out, const PoolWords<W>* pw) {
    const uint64_t take = p.take, fin = p.fin;
    const uint64_t cb = cursor_bit(S);
    const bool advance = fin > 0 && p.fout == 0;
    // every word of the word-block loaded up front (the passes below synchronise the
    // block: a load inside them would be a round trip per pass)
    uint64_t xu[W], xs[W];
#pragma unroll
    for (int k = 0; k < W; k++) {
        const uint64_t w = (uint64_t)wb * (BLOCK * W) + (uint64_t)k * BLOCK + threadIdx.x;
        const bool valid = w < S.pool.words;
        xu[k] = pw ? pw->used[k] : (valid ? S.used_bm[w] : ~0ull);
        xs[k] = pw ? pw->usable[k] : (valid ? S.usable_bm[w] : 0ull);
    }
#pragma unroll
    for (int k = 0; k < W; k++) {
        const uint64_t w = (uint64_t)wb * (BLOCK * W) + (uint64_t)k * BLOCK + threadIdx.x;
        const bool valid = w < S.pool.words;
        const uint64_t used = xu[k];
        const uint64_t wu = xs[k];
        const uint64_t wf = valid ? free_mask(S, w, used, wu, cb) : 0ull;
        const uint32_t cu = (uint32_t)__popcll(wu), cf = (uint32_t)__popcll(wf);
        uint32_t v[2] = {cu, cf}, tot[2];
        block_excl_scan<2>(v, tot);
        const uint64_t ru = base_u + v[0], rf = base_f + v[1];
        const uint32_t nu = ru < take ? (uint32_t)min((uint64_t)cu, take - ru) : 0u;
        const uint32_t nf = rf < fin ? (uint32_t)min((uint64_t)cf, fin - rf) : 0u;
        const uint64_t selu = lowest_bits(wu, nu, cu), self = lowest_bits(wf, nf, cf);
        if (selu) S.usable_bm[w] = wu & ~selu;  // ipPool.Get: delete(usable, ip) ...
        if (selu | self) S.used_bm[w] = used | selu | self;  // ... used[ip]; ipPool.new: used[ip]  (one thread owns word w)
        if (advance && nf && rf + nf == fin)
            *cursor_out = (uint64_t)S.pool.net + w * 64 + nth_set_bit(wf, nf - 1) + 1 - S.pool.base;
        const uint64_t w0 = (uint64_t)wb * (BLOCK * W) + (uint64_t)k * BLOCK + (threadIdx.x & ~63u);
        const uint64_t gu0 = (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)ru) |
                             ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(ru >> 32)) << 32);
        const uint64_t gf0 = (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)rf) |
                             ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(rf >> 32)) << 32);
        wave_write_addrs(S, gu0, nu, wu, w0, lo_g, hi_g);
        wave_write_addrs(S, take + gf0, nf, wf, w0, lo_g, hi_g);
        base_u += tot[0];
        base_f += tot[1];
    }
}

// ---------------------------------------------------------------------------
// cross-block hand-offs (MI355X_MICROARCH.md "Workgroup dispatch, XCD placement
// & inter-workgroup visibility", valid forms; cdna_hip_programming.md §6 G16)
//
//   * per-block records: stored write-through (sc1) by wave 0, drained with
//     vmcnt(0), then ONE returning agent-scope add on ONE arrival counter.  The
//     block whose add completes the tick's count (the "last arriver") and the
//     blocks that poll the counter (sc1 loads) read the records with sc1 loads.
//   * the pool phase (ticks with Gets or Puts) uses a sense-reversal barrier
//     among its participants: release fence -> arrive -> poll -> acquire fence.
// Every spin is bounded (2 s of s_memrealtime) and flags the tick as failed.
// ---------------------------------------------------------------------------
template <class T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ T ld_sc1(const T* p) {
    return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st32_sc1(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld32_sc1(const uint32_t* p) {
    return __hip_atomic_load(const_cast<uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr uint64_t SPIN_LIMIT = 200000000ull;  // 2 s at 100 MHz

// append x to a device list with one atomic per wave; entries are stored
// write-through: the FRONT launch's last arriver reads them (multi-rank)
// multi rank: the chain block's exchange lists.  Each block appends to its own
// segment of use_list / rel_list (from its first pod slot: a block never holds
// more entries than pod slots) through LDS counters, so an append costs no
// global round trip; the lengths go out with the block's record
// (publish_and_arrive) and the segments are gathered in block order.
__device__ __forceinline__ uint32_t* list_lds() {
    __shared__ uint32_t c[3];  // Use count, release count, the segment base (the block's first pod slot)
    return c;
}
__device__ __forceinline__ void wave_append(bool pred, uint32_t x, uint32_t* list, int which) {
    uint64_t m = __ballot(pred);
    if (!m) return;
    uint32_t base = 0;
    const int l = lane_id();
    int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t* c = list_lds();
    if (l == leader) base = atomicAdd(&c[which], (uint32_t)__popcll(m));
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
    if (pred) st32_sc1(&list[c[2] + base + __popcll(m & ((1ull << l) - 1))], x);
}

// publish this block's record and arrive; returns the arrival counter before
// this block's add (uniform).  A wave that issued pool atomics or exchange-list
// stores drained them in the classify slow path, before the barrier here; the
// block's other stores (output lists) are issued after the arrival.
__device__ __forceinline__ uint64_t publish_and_arrive(const DevState& S, uint32_t b, const uint32_t (&rec)[AG_STRIDE]) {
    __shared__ unsigned long long sh_old;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's list entries (wave_append)
    __syncthreads();
    if (threadIdx.x < 64) {
        const int l = lane_id();
        if (l < AG_STRIDE / 2) {
            uint64_t v = 0;
#pragma unroll
            for (int i = 0; i < AG_STRIDE / 2; i++)
                if (l == i) v = (uint64_t)rec[2 * i] | (uint64_t)rec[2 * i + 1] << 32;
            st_sc1(reinterpret_cast<uint64_t*>(S.blockagg + (size_t)b * AG_STRIDE) + l, v);
        }
        if (l < 2) st32_sc1(&S.list_blk[2 * b + l], list_lds()[l]);  // the block's list lengths
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (l == 0)
            sh_old = __hip_atomic_fetch_add(&S.bar->arrive, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    return sh_old;
}

// poll the arrival counter (sc1) until every chain block of this tick arrived,
// then acquire (the pool phase reads bitmaps other blocks changed)
// stores to the pinned host header: system scope (write-through to host memory),
// so the host sees them once the tick's completion event fires (that event has no
// system-scope release of its own)
template <class T, class V>
__device__ __forceinline__ void st_host(T* p, V v) {
    __hip_atomic_store(p, (T)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void wait_arrivals(const DevState& S, uint64_t target) {
    if (threadIdx.x == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (ld_sc1(&S.bar->arrive) < target) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_LIMIT) {
                __hip_atomic_store(&S.hdr_host->err, TICK_ERR_BARRIER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}

// sense-reversal barrier among the n blocks of the pool phase
// TICK_XSPEC: every rank's lists fit the speculative exchange's capacities
__device__ __forceinline__ bool spec_fits(const DevState& S) {
    bool ok = true;
    for (int r = 0; r < S.world; r++) ok &= S.xall[r].n_use <= S.xcap_u && S.xall[r].n_rel <= S.xcap_r;
    return ok;
}
__device__ __forceinline__ void pool_barrier(const DevState& S, uint32_t n) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        GridBar* bar = S.bar;
        const uint32_t gen = __hip_atomic_load(&bar->pgen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const uint32_t a = __hip_atomic_fetch_add(&bar->pcnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
        if (a == n) {
            __hip_atomic_store(&bar->pcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&bar->pgen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(&bar->pgen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_LIMIT) {
                    __hip_atomic_store(&S.hdr_host->err, TICK_ERR_BARRIER, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    break;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
}

// block-wide sums of N u64 partials (every thread gets the totals)
template <int N>
__device__ __forceinline__ void block_sum64(uint64_t (&v)[N]) {
    __shared__ uint64_t part[BLOCK / 64][N];
#pragma unroll
    for (int f = 0; f < N; f++) {
        const uint64_t s = wave_sum64(v[f]);
        if (lane_id() == 0) part[wave_id()][f] = s;
    }
    __syncthreads();
#pragma unroll
    for (int f = 0; f < N; f++) {
        uint64_t s = 0;
#pragma unroll
        for (int w = 0; w < BLOCK / 64; w++) s += part[w][f];
        v[f] = s;
    }
    __syncthreads();
}

// prefix over chain blocks < b and totals over all chain blocks of the records
// (sc1 loads: the records may have been published in this launch).  The
// records are transposed through LDS: thread (f, p) = (t / 16, t % 16) sums
// field f of records p, p + 16, ... and a 16-lane DPP row reduction finishes.
constexpr int REC_PITCH = AG_STRIDE + 1;  // conflict-free column reads
struct Sums {
    uint64_t pre[AG_STRIDE], tot[AG_STRIDE];
};
__device__ __forceinline__ uint64_t row_sum16(uint64_t x) {  // lane 15 of each 16-lane row: the row total
    x += dpp_src64<0x111, 0xF>(x);
    x += dpp_src64<0x112, 0xF>(x);
    x += dpp_src64<0x114, 0xF>(x);
    x += dpp_src64<0x118, 0xF>(x);
    return x;
}
// tag != 0 (single rank): only dirty blocks publish records, marked with the
// tick's tag in AG_DIRTY; any other record is stale and counts as zero (a clean
// block has nothing in any scanned field).
__device__ __forceinline__ void reduce_records(const DevState& S, uint32_t b, uint32_t tag, uint32_t* recs, Sums* out) {
    for (uint32_t j = threadIdx.x; j < S.n_chain; j += BLOCK) {
        const uint64_t* p = reinterpret_cast<const uint64_t*>(S.blockagg + (size_t)j * AG_STRIDE);
        uint64_t q[AG_STRIDE / 2];
#pragma unroll
        for (int i = 0; i < AG_STRIDE / 2; i++) q[i] = ld_sc1(p + i);
        const bool keep = !tag || (uint32_t)(q[AG_DIRTY / 2] >> (32 * (AG_DIRTY & 1))) == tag;
#pragma unroll
        for (int i = 0; i < AG_STRIDE / 2; i++) {
            uint32_t lo = keep ? (uint32_t)q[i] : 0u, hi = keep ? (uint32_t)(q[i] >> 32) : 0u;
            if (tag && 2 * i + 1 == AG_DIRTY) hi = keep ? 1u : 0u;
            recs[j * REC_PITCH + 2 * i] = lo;
            recs[j * REC_PITCH + 2 * i + 1] = hi;
        }
    }
    __syncthreads();
    const uint32_t f = threadIdx.x >> 4, p = threadIdx.x & 15;
    uint64_t tot = 0, pre = 0;
    for (uint32_t j = p; j < S.n_chain; j += 16) {
        const uint32_t v = recs[j * REC_PITCH + f];
        tot += v;
        pre += j < b ? v : 0u;
    }
    tot = row_sum16(tot);
    pre = row_sum16(pre);
    if (p == 15) {
        out->tot[f] = tot;
        out->pre[f] = pre;
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// chain-block geometry: the block's bucket range, its live pod groups
// ---------------------------------------------------------------------------
__device__ __forceinline__ void block_range(const DevState& S, uint32_t b, uint32_t& bk0, uint32_t& nbk) {
    bk0 = (uint32_t)((uint64_t)S.nb * b / S.n_chain);
    nbk = (uint32_t)((uint64_t)S.nb * (b + 1) / S.n_chain) - bk0;
}
// gpre[j] = live 8-slot pod groups of the block's buckets before j (fill marks
// are multiples of 8).  Wave 0 only; the caller synchronises.
__device__ __forceinline__ void load_gpre(const DevState& S, uint32_t bk0, uint32_t nbk, uint32_t* gpre) {
    if (threadIdx.x < 64) {
        const int l = lane_id();
        const uint32_t g = l < (int)nbk ? (uint32_t)S.pod_fill[bk0 + l] >> 3 : 0u;
        gpre[l + 1] = wave_incl_scan(g);
        if (l == 0) gpre[0] = 0;
    }
}
// largest j with gpre[j] <= gi (a bucket that has groups)
__device__ __forceinline__ uint32_t find_bucket(const uint32_t* gpre, uint32_t nbk, uint32_t gi) {
    uint32_t lo = 0, hi = nbk;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (gpre[mid] <= gi) lo = mid;
        else hi = mid;
    }
    return lo;
}

// one 8-slot pod group: state, node index and podIP words (one HBM round trip)
struct PodGrp {
    uint32_t slot;  // first local slot; ~0u when the group holds no pods
    uint32_t j;     // bucket within the block
    uint32_t stw[4], ndw[4];  // state / node-index words, two pods each (kept packed: registers)
    uint32_t ip[POD_PER_THREAD];
    __device__ __forceinline__ uint32_t st(int k) const { return (stw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu; }
    __device__ __forceinline__ uint32_t nl(int k) const { return (ndw[k >> 1] >> (16 * (k & 1))) & 0xFFFFu; }
};
// (with_ip = false: the podIPs stay 0, for load_group_ips_set after the state lands)
__device__ __forceinline__ void load_group(const DevState& S, const uint32_t* gpre, uint32_t bk0, uint32_t nbk,
                                           uint32_t ng, uint32_t gi, PodGrp& g, bool with_ip = true) {
    uint4 st4 = make_uint4(0, 0, 0, 0), nd4 = st4, ipa = st4, ipb = st4;
    g.slot = ~0u;
    g.j = 0;
    if (gi < ng) {
        const uint32_t j = find_bucket(gpre, nbk, gi);
        g.j = j;
        g.slot = (bk0 + j) * S.cp + (gi - gpre[j]) * (uint32_t)POD_PER_THREAD;
        st4 = *reinterpret_cast<const uint4*>(S.pod_state + g.slot);
        nd4 = *reinterpret_cast<const uint4*>(S.pod_node + g.slot);
        if (with_ip) {
            ipa = *reinterpret_cast<const uint4*>(S.pod_ip + g.slot);
            ipb = *reinterpret_cast<const uint4*>(S.pod_ip + g.slot + 4);
        }
    }
    g.stw[0] = st4.x, g.stw[1] = st4.y, g.stw[2] = st4.z, g.stw[3] = st4.w;
    g.ndw[0] = nd4.x, g.ndw[1] = nd4.y, g.ndw[2] = nd4.z, g.ndw[3] = nd4.w;
    g.ip[0] = ipa.x, g.ip[1] = ipa.y, g.ip[2] = ipa.z, g.ip[3] = ipa.w;
    g.ip[4] = ipb.x, g.ip[5] = ipb.y, g.ip[6] = ipb.z, g.ip[7] = ipb.w;
}
// could this pod need a patch (computePatchData), given it is evaluated?  (podIP == 0:
// the state's PS_IP_SET, so the podIPs need not have landed)
__device__ __forceinline__ bool maybe_need(uint16_t st) {
    const uint32_t phase = (st & PS_PHASE_MASK) >> PS_PHASE_SHIFT;
    return (st & PS_USED) &&
           (phase != PHASE_RUNNING || !(st & PS_CONFORMS) || !(st & PS_HAS_HOST_IP) || !(st & PS_IP_SET));
}
// the podIPs of a group loaded without them, when one of its pods holds one
// (PS_IP_SET; a pod without it has pod_ip 0): the dense initial tick's new pods
// hold none, so their 4 bytes each are not read
__device__ __forceinline__ void load_group_ips_set(const DevState& S, PodGrp& g) {
    bool any = false;
#pragma unroll
    for (int k = 0; k < POD_PER_THREAD; k++) any |= (g.st(k) & PS_IP_SET) != 0;
    if (any && g.slot != ~0u) {
        const uint4 ipa = *reinterpret_cast<const uint4*>(S.pod_ip + g.slot);
        const uint4 ipb = *reinterpret_cast<const uint4*>(S.pod_ip + g.slot + 4);
        g.ip[0] = ipa.x, g.ip[1] = ipa.y, g.ip[2] = ipa.z, g.ip[3] = ipa.w;
        g.ip[4] = ipb.x, g.ip[5] = ipb.y, g.ip[6] = ipb.z, g.ip[7] = ipb.w;
    }
}
// spec ids of a group, loaded only when one of its pods may need a patch
__device__ __forceinline__ void load_spec_ids(const DevState& S, const PodGrp& g, uint16_t (&sp)[POD_PER_THREAD]) {
    bool any = false;
#pragma unroll
    for (int k = 0; k < POD_PER_THREAD; k++) any |= maybe_need(g.st(k));
    uint4 v = make_uint4(0, 0, 0, 0);
    if (any && g.slot != ~0u) v = *reinterpret_cast<const uint4*>(S.pod_spec + g.slot);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < POD_PER_THREAD; k++) sp[k] = (uint16_t)(w[k >> 1] >> (16 * (k & 1)));
}
// the spec words of a group with a pod that needs a patch (its byte count)
__device__ __forceinline__ uint4 load_spec_words(const DevState& S, const PodGrp& g, uint32_t need) {
    uint4 v = make_uint4(0, 0, 0, 0);
#ifdef DIAG_NO_SPECW  // timing builds only
    return v;
#endif
    if (need && g.slot != ~0u) v = *reinterpret_cast<const uint4*>(S.pod_spec + g.slot);
    return v;
}
// nflags holds the flags of the block's buckets from bucket j0 on
__device__ __forceinline__ uint8_t group_node_flags(const DevState& S, const uint8_t* nflags, const PodGrp& g, int k,
                                                    uint32_t j0 = 0) {
    return (g.st(k) & PS_USED) ? nflags[(g.j - j0) * S.cn + g.nl(k)] : (uint8_t)0;
}

// ---------------------------------------------------------------------------
// classify phase (FRONT): predicates A.4 / A.5 over the block's nodes and live
// pod groups; Use / Put bits (single rank: in place; multi rank: exchange
// lists); heartbeat handles at the host-maintained base; per-thread counts
// ---------------------------------------------------------------------------
// Per-group predicate masks (bit k = pod k of the 8-slot group), computed
// branch-free from the packed state words: the steady state is a sweep of
// ~20 VALU ops per pod.  Everything rare (a Use that changes the pool, a
// release, a patch - whose byte count needs the spec) runs in a slow path
// entered only when some lane of the wave needs it.
struct GroupMasks {
    uint32_t del, eval, alloc, need, rel, usec, total, pend, run, dirty;
};
__device__ __forceinline__ GroupMasks group_masks(const DevState& S, const PodGrp& g, const uint8_t (&ntf)[POD_PER_THREAD]) {
    // SWAR over the packed state words: each 32-bit op evaluates two pods (bit 0 and
    // bit 16 of every plane); integer arithmetic keeps it all in VGPRs
    static_assert(PS_USED == 1 && PS_DISREGARD == 2 && PS_DELETE_PENDING == 4 && PS_STATUS_NONEMPTY == 16 &&
                      PS_CONFORMS == 32 && PS_EVENT == 64 && PS_HAS_HOST_IP == 128 && PS_PHASE_SHIFT == 8 &&
                      NT_RELOCK == 1 && NT_MANAGED == 2 && PHASE_PENDING == 1 && PHASE_RUNNING == 2 &&
                      PS_IP_SET == (1u << 11) && PS_IP_POOL == (1u << 12),
                  "state bit layout");
    constexpr uint32_t M = 0x00010001u;
    GroupMasks m{0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const uint32_t s = g.stw[w];
        const uint32_t nf = (uint32_t)ntf[2 * w] | (uint32_t)ntf[2 * w + 1] << 16;
        // podIP == 0 / in the CIDR: the state's PS_IP_SET / PS_IP_POOL (pod_ip itself is
        // loaded only for a Use or a release)
        const uint32_t ipz = ~(s >> 11) & M;
        const uint32_t inc_pool = (s >> 12) & M;
        const uint32_t used = s & M, disr = (s >> 1) & M, del = used & (s >> 2);
        const uint32_t nonempty = (s >> 4) & M, conf = (s >> 5) & M, event = (s >> 6) & M, hhost = (s >> 7) & M;
        const uint32_t ph = (s >> 8) & (7u * M);
        const uint32_t xr = ph ^ (PHASE_RUNNING * M), xp = ph ^ (PHASE_PENDING * M);
        const uint32_t running = ~(xr | (xr >> 1) | (xr >> 2)) & M, pending = ~(xp | (xp >> 1) | (xp >> 2)) & M;
        const uint32_t relock = nf & M, managed = (nf >> 1) & M;
        const uint32_t live = used & ~del & M;
        // needLockPod / heartbeat re-lock (pod_controller.go:252-269, node_controller.go:152)
        const uint32_t eval = live & (event | (relock & ~disr));
        // computePatchData: Pending always patches; otherwise the strategic merge must change something
        // (EnableCNI: not before cni.Setup gave the pod an IP)
        const uint32_t stale = (running & conf & hhost) ^ M;
        const uint32_t need = S.cni ? eval & stale & ~ipz : eval & (stale | ipz);
        // `{{ with .status }} ... {{ with .podIP }} . {{ else }} {{ PodIP }}` (pod.status.tpl:44-47);
        // EnableCNI: no ipPool (no Get, Use or Put)
        const uint32_t alloc = S.cni ? 0u : eval & nonempty & ipz;
        const uint32_t inc = S.cni ? 0u : inc_pool;
        auto put = [w](uint32_t& mask, uint32_t plane) { mask |= ((plane & 1u) | ((plane >> 15) & 2u)) << (2 * w); };
        put(m.del, del & M);
        put(m.eval, eval);
        put(m.alloc, alloc);
        put(m.need, need);
        put(m.rel, del & managed & inc);
        // quiet ticks (use_events_only): every live pod's address is already in `used`
        // unless an event changed the pod since (engine.cpp, kwok_tick_submit)
#ifdef DIAG_NO_USE  // timing builds only
        put(m.usec, 0u);
#else
        put(m.usec, eval & inc & (S.use_events_only ? event : M));
#endif
        put(m.total, live);
        put(m.pend, live & ~need & pending);
        put(m.run, live & (need | running));
        put(m.dirty, (del & M) | need | (eval & event));
    }
    return m;
}

// The heartbeat-once rows' fast path: the same planes as group_masks, reduced
// straight to the four counts a clean group contributes (eval, total, pending,
// running: popcounts of the two-pod planes) and one `rare` flag (any delete,
// patch, Get, Put, Use or event: the group then takes the full path), without
// packing ten per-pod masks (~40% of group_masks' VALU work)
__device__ __forceinline__ bool group_counts_fast(const DevState& S, const PodGrp& g, const uint8_t (&ntf)[POD_PER_THREAD],
                                                  uint32_t& n_eval, uint32_t& n_total, uint32_t& n_pend,
                                                  uint32_t& n_run) {
    // the planes are used at bit 0 (even pod) and bit 16 (odd pod) only: the shifted
    // copies of the word are combined unmasked and masked once at the end
    constexpr uint32_t M = 0x00010001u;
    uint32_t rare = 0, pe = 0, pt = 0, pp = 0, pr = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const uint32_t s = g.stw[w];
        const uint32_t nf = (uint32_t)ntf[2 * w] | (uint32_t)ntf[2 * w + 1] << 16;
        const uint32_t s1 = s >> 1, s2 = s >> 2, s4 = s >> 4, s5 = s >> 5, s6 = s >> 6, s7 = s >> 7;
        const uint32_t s8 = s >> 8, s9 = s >> 9, s10 = s >> 10, s11 = s >> 11, s12 = s >> 12;
        const uint32_t del = s & s2;                     // USED & DELETE_PENDING
        const uint32_t live = s & ~s2;                   // USED, not DELETE_PENDING
        const uint32_t eval = live & (s6 | (nf & ~s1));  // EVENT, or RELOCK & !DISREGARD
        const uint32_t running = s9 & ~(s8 | s10), pending = s8 & ~(s9 | s10);
        const uint32_t ok = running & s5 & s7;           // Running, CONFORMS, HAS_HOST_IP
        // computePatchData: a no-op unless the podIP is empty (IP_SET = s11); EnableCNI: not before it has one
        const uint32_t need = S.cni ? eval & ~ok & s11 : eval & ~(ok & s11);
        const uint32_t alloc = S.cni ? 0u : eval & s4 & ~s11;                             // STATUS_NONEMPTY, no podIP
        const uint32_t usec = S.cni ? 0u : eval & s12 & (S.use_events_only ? s6 : ~0u);  // IP_POOL
        rare |= del | need | alloc | usec | (eval & s6);
        pe += eval & M, pt += live & M, pp += live & pending & ~need & M, pr += live & (need | running) & M;
    }
    n_eval += (pe & 0xFFFFu) + (pe >> 16);  // at most 4 per half
    n_total += (pt & 0xFFFFu) + (pt >> 16);
    n_pend += (pp & 0xFFFFu) + (pp >> 16);
    n_run += (pr & 0xFFFFu) + (pr >> 16);
    return (rare & M) != 0;
}

// `used` bits of a group's Use candidates (bit k set = already in `used`).
// Pods of one bucket hold consecutive addresses (canonical allocation order),
// so a group's addresses usually fall in two adjacent words: load those two
// (UsedWords); a group that straddles more is resolved word by word.
struct UsedWords {
    uint64_t w0, a, b;
    bool near;
};
__device__ __forceinline__ UsedWords used_words(const DevState& S, const PodGrp& g, uint32_t usec) {
    UsedWords u{0, 0, 0, true};
    if (!usec) return u;
    const uint32_t k0 = (uint32_t)__builtin_ctz(usec);
    uint32_t ip0 = g.ip[0];
#pragma unroll
    for (int k = 1; k < POD_PER_THREAD; k++) ip0 = (uint32_t)k == k0 ? g.ip[k] : ip0;
    u.w0 = (uint64_t)(ip0 - S.pool.net) >> 6;
#pragma unroll
    for (int k = 0; k < POD_PER_THREAD; k++) {
        const uint64_t w = (uint64_t)(g.ip[k] - S.pool.net) >> 6;
        u.near &= !((usec >> k) & 1) || w == u.w0 || w == u.w0 + 1;
    }
    if (u.near) {
        u.a = S.used_bm[u.w0];
        u.b = u.w0 + 1 < S.pool.words ? S.used_bm[u.w0 + 1] : 0ull;
    }
    return u;
}
__device__ __forceinline__ uint32_t used_bits(const DevState& S, const PodGrp& g, uint32_t usec, const UsedWords& u) {
    uint32_t bits = 0;
    if (u.near) {
#pragma unroll
        for (int k = 0; k < POD_PER_THREAD; k++) {
            const uint64_t bit = g.ip[k] - S.pool.net;
            const uint64_t w = (bit >> 6) == u.w0 ? u.a : u.b;
            bits |= (uint32_t)((w >> (bit & 63)) & 1) << k;
        }
    } else {
#pragma unroll
        for (int k = 0; k < POD_PER_THREAD; k++)
            if ((usec >> k) & 1) {
                const uint64_t bit = g.ip[k] - S.pool.net;
                bits |= (uint32_t)((S.used_bm[bit >> 6] >> (bit & 63)) & 1) << k;
            }
    }
    return bits & usec;
}

// counts of one group into f, and its rare pre-count work (wave-uniform entry):
// the byte counts of patches (spec lengths) and the releases of deleted pods.
// Returns the group's patch bytes.
// spw: the group's spec words (load_spec_words, issued with the row's other
// loads); smax: the specs' reservations in LDS (null: read the descriptors)
__device__ __forceinline__ uint32_t count_group(const DevState& S, const PodGrp& g, const GroupMasks& m,
                                                uint32_t (&f)[AG_STRIDE], const uint4& spw, const uint16_t* smax) {
    uint32_t bytes = 0;
    f[AG_DEL] += __popc(m.del);
    f[AG_EVAL] += __popc(m.eval);
    f[AG_ALLOC] += __popc(m.alloc);
    f[AG_REL] += __popc(m.rel);
    f[AG_PP] += __popc(m.need);
    f[AG_TOTAL] += __popc(m.total);
    f[AG_PENDING] += __popc(m.pend);
    f[AG_RUNNING] += __popc(m.run);
    if (__builtin_expect(__ballot((m.rel | m.need) != 0) != 0, 0)) {
        const uint32_t w[4] = {spw.x, spw.y, spw.z, spw.w};
        // single rank: a group's released addresses usually share one bitmap word
        // (consecutive allocations): one atomic for all of them, else one per pod
        uint64_t rm = 0;
        uint32_t rw = 0;
        bool one = !S.multi && m.rel != 0;
        if (one) {
            uint32_t ip0 = g.ip[0];
#pragma unroll
            for (int k = 1; k < POD_PER_THREAD; k++) ip0 = (uint32_t)__builtin_ctz(m.rel) == (uint32_t)k ? g.ip[k] : ip0;
            rw = (ip0 - S.pool.net) >> 6;
#pragma unroll
            for (int k = 0; k < POD_PER_THREAD; k++) {
                const uint32_t bit = g.ip[k] - S.pool.net;
                const bool r = (m.rel >> k) & 1;
                one &= !r || (bit >> 6) == rw;
                rm |= r ? 1ull << (bit & 63) : 0ull;
            }
#ifndef DIAG_NO_REL  // timing builds only (tools/build_variant.sh): the releases skipped
            if (one) atomicOr((unsigned long long*)&S.rel_bm[rw], rm);
#endif
        }
#pragma unroll
        for (int k = 0; k < POD_PER_THREAD; k++) {
            const uint32_t ip = g.ip[k];
            const uint64_t bit = ip - S.pool.net;
            const bool r = (m.rel >> k) & 1;
            // the Deleted event of a pod we delete: Put if the node is managed and the IP in CIDR
            // (pod_controller.go:329-336).  Single rank: the Put waits in rel_bm, folded in
            // the pool phase after every Use of this tick (Use -> Put)
            if (!S.multi) {
#ifndef DIAG_NO_REL
                if (r && !one) atomicOr((unsigned long long*)&S.rel_bm[bit >> 6], 1ull << (bit & 63));
#endif
            } else {
                wave_append(r, ip, S.rel_list, 1);  // ballots over every lane
            }
            if ((m.need >> k) & 1) {
                const uint32_t sp = (w[k >> 1] >> (16 * (k & 1))) & 0xFFFFu;
                bytes += smax ? (uint32_t)smax[sp] : (uint32_t)S.specs[sp].max_len;
            }
        }
        f[AG_PP_BYTES] += bytes;
        // (multi rank: the release list entries are drained before the block's
        // arrival, publish_and_arrive)
    }
    return bytes;
}

// split ticks: a dirty group's counts into its 64-group run (LDS, [MAX_WC][4]
// then the dirty bits); gi = the group's index among the block's live groups
__device__ __forceinline__ void wc_add(uint32_t* wcnt, uint32_t gi, const GroupMasks& m, uint32_t bytes) {
#ifdef DIAG_NO_WC  // timing builds only
    return;
#endif
    if (!m.dirty) return;
    const uint32_t w = gi / WC_GROUPS;
    if (m.del) atomicAdd(&wcnt[4 * w], (uint32_t)__popc(m.del));
    if (m.need) {
        atomicAdd(&wcnt[4 * w + 1], (uint32_t)__popc(m.need));
        atomicAdd(&wcnt[4 * w + 2], bytes);
    }
    if (m.alloc) atomicAdd(&wcnt[4 * w + 3], (uint32_t)__popc(m.alloc));
    atomicOr(&wcnt[4 * MAX_WC + (w >> 5)], 1u << (w & 31));
}
// ... and (DevState::sparse_jobs) the dirty group itself for k_sparse_jobs: its slot,
// masks and patch bytes at its index among the block's live groups, tagged with the
// tick (a group clean this tick keeps an older tag: k_sparse_jobs reads it as clean)
__device__ __forceinline__ void gjob_put(const DevState& S, uint32_t b, uint32_t gi, const PodGrp& g, const GroupMasks& m,
                                         uint32_t bytes, uint32_t tag) {
    if (!m.dirty) return;
    // a pod of the group holds a hostIP / a podIP: k_sparse_jobs reads those words (a
    // patch rewrites the group's words whole, its other pods' addresses included)
    uint32_t hipf = 0, ipf = 0;
#pragma unroll
    for (int k = 0; k < POD_PER_THREAD; k++) {
        hipf |= g.st(k) >> 7;   // PS_HAS_HOST_IP
        ipf |= g.st(k) >> 11;   // PS_IP_SET
    }
    const uint32_t mk = m.del | m.need << 8 | m.alloc << 16 | g.j << 24 | (hipf & 1u) << 30 | (ipf & 1u) << 31;
    S.gjob[(size_t)b * (MAX_WC * WC_GROUPS) + gi] = make_uint4(g.slot, mk, m.need ? bytes : 0u, tag);
}
// ... and, once the block's counts are complete, the runs' exclusive prefixes and
// dirty bits to global memory for k_pod_jobs (wave 0; ng = the block's live groups)
__device__ __forceinline__ void wc_publish(const DevState& S, uint32_t b, uint32_t ng, const uint32_t* wcnt) {
    if (threadIdx.x >= 64) return;
    const int l = lane_id();
    constexpr int PER = MAX_WC / 64;
    const uint32_t nwc = (ng + WC_GROUPS - 1) / WC_GROUPS;
    uint32_t v[PER][4], s[4] = {0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < PER; e++)
#pragma unroll
        for (int f = 0; f < 4; f++) {
            v[e][f] = wcnt[4 * (PER * l + e) + f];
            s[f] += v[e][f];
        }
    uint32_t run[4];
#pragma unroll
    for (int f = 0; f < 4; f++) run[f] = wave_incl_scan(s[f]) - s[f];
    uint4* dst = S.wc_pre + (size_t)b * MAX_WC;
#pragma unroll
    for (int e = 0; e < PER; e++) {
        const uint32_t w = PER * l + e;
        if (w < nwc) dst[w] = make_uint4(run[0], run[1], run[2], run[3]);
#pragma unroll
        for (int f = 0; f < 4; f++) run[f] += v[e][f];
    }
    if (l < WC_DIRTY_WORDS) S.wc_dirty[(size_t)b * WC_DIRTY_WORDS + l] = wcnt[4 * MAX_WC + l];
}

// configurePod (pod_controller.go:378-382): Use() of the group's evaluated in-CIDR
// podIPs that are not in `used` (wave-uniform entry; rare outside restarts)
__device__ __forceinline__ void apply_uses(const DevState& S, const PodGrp& g, uint32_t use) {
    if (__builtin_expect(__ballot(use != 0) != 0, 0)) {
#pragma unroll
        for (int k = 0; k < POD_PER_THREAD; k++) {
            const uint32_t ip = g.ip[k];
            const uint64_t bit = ip - S.pool.net;
            const bool u = (use >> k) & 1;
            if (!S.multi) {
                if (u) atomicOr((unsigned long long*)&S.used_bm[bit >> 6], 1ull << (bit & 63));
            } else {
                wave_append(u, ip, S.use_list, 0);
            }
        }
    }
}

// one 8-slot group at a known slot (~0u: none), pods at or past `fill` read as
// empty.  with_ip = false: state and node words only (the classification's
// predicates read the podIP bits of the state; load_group_ips adds the
// addresses when a Use or a release needs them)
__device__ __forceinline__ void load_group_at(const DevState& S, uint32_t slot, uint32_t j, PodGrp& g,
                                              bool with_ip = true) {
    uint4 st4 = make_uint4(0, 0, 0, 0), nd4 = st4, ipa = st4, ipb = st4;
    g.slot = slot;
    g.j = j;
    if (slot != ~0u) {
        st4 = *reinterpret_cast<const uint4*>(S.pod_state + slot);
        nd4 = *reinterpret_cast<const uint4*>(S.pod_node + slot);
        if (with_ip) {
            ipa = *reinterpret_cast<const uint4*>(S.pod_ip + slot);
            ipb = *reinterpret_cast<const uint4*>(S.pod_ip + slot + 4);
        }
    }
    g.stw[0] = st4.x, g.stw[1] = st4.y, g.stw[2] = st4.z, g.stw[3] = st4.w;
    g.ndw[0] = nd4.x, g.ndw[1] = nd4.y, g.ndw[2] = nd4.z, g.ndw[3] = nd4.w;
    g.ip[0] = ipa.x, g.ip[1] = ipa.y, g.ip[2] = ipa.z, g.ip[3] = ipa.w;
    g.ip[4] = ipb.x, g.ip[5] = ipb.y, g.ip[6] = ipb.z, g.ip[7] = ipb.w;
}
// the podIPs of a group loaded without them, for the lanes that need them (a Use
// check or a release: GroupMasks usec / rel); wave-uniform entry
__device__ __forceinline__ void load_group_ips(const DevState& S, PodGrp& g, bool need) {
    if (__builtin_expect(__ballot(need) == 0, 1)) return;
    if (need && g.slot != ~0u) {
        const uint4 ipa = *reinterpret_cast<const uint4*>(S.pod_ip + g.slot);
        const uint4 ipb = *reinterpret_cast<const uint4*>(S.pod_ip + g.slot + 4);
        g.ip[0] = ipa.x, g.ip[1] = ipa.y, g.ip[2] = ipa.z, g.ip[3] = ipa.w;
        g.ip[4] = ipb.x, g.ip[5] = ipb.y, g.ip[6] = ipb.z, g.ip[7] = ipb.w;
    }
}
// a speculatively loaded group past its bucket's fill mark holds no pods
__device__ __forceinline__ void clip_group(PodGrp& g, bool live) {
    if (!live) {
        g.slot = ~0u;
#pragma unroll
        for (int w = 0; w < 4; w++) g.stw[w] = 0;
    }
}
__device__ __forceinline__ GroupMasks masks_of(const DevState& S, const uint8_t* nflags, const PodGrp& g) {
    uint8_t n[POD_PER_THREAD];
#pragma unroll
    for (int k = 0; k < POD_PER_THREAD; k++) n[k] = group_node_flags(S, nflags, g, k);
    return group_masks(S, g, n);
}

// block-wide totals of N u32 fields (every thread gets them; one barrier pair)
template <int N>
__device__ __forceinline__ void block_total(uint32_t (&v)[N]) {
    __shared__ uint32_t part[BLOCK / 64][N];
#pragma unroll
    for (int f = 0; f < N; f++) {
        const uint32_t s = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(v[f]), 63);
        if (lane_id() == 0) part[wave_id()][f] = s;
    }
    __syncthreads();
#pragma unroll
    for (int f = 0; f < N; f++) {
        uint32_t s = 0;
#pragma unroll
        for (int w = 0; w < BLOCK / 64; w++) s += part[w][f];
        v[f] = s;
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// emission: compaction of the output lists, byte emission, state transitions.
// Only chunks marked dirty by the classify phase are visited: a clean chunk
// contributes nothing to any scanned field.
// ---------------------------------------------------------------------------
struct Layout {
    uint64_t init_base;   // arena offset of the node-init patches (= n_hb x HB_STRIDE)
    uint64_t pod_base;    // arena offset of the pod patches (after every init patch)
    uint64_t alloc_base;  // this rank's first global allocation ordinal
    PoolPlan plan;
};
struct Bases {
    uint64_t v[AG_NSCAN];  // running prefix of the scanned fields
};

// node chunk at block-local node offset i0 (node slots nbase + [i0, i0 + 1024))
__device__ __forceinline__ void emit_node_chunk(const DevState& S, uint32_t nbase, uint32_t i0, uint32_t nn, Bases& run,
                                const Layout& L) {
    const uint32_t i = i0 + threadIdx.x * NODE_PER_THREAD;
    const uint32_t first = nbase + i;
    uint32_t packed = 0;
    if (i < nn) packed = *reinterpret_cast<const uint32_t*>(S.node_state + first);
    NodeCls c[NODE_PER_THREAD];
    uint32_t v[2] = {0, 0};  // init, init bytes
    uint32_t ilen[NODE_PER_THREAD];
    uint64_t blob[NODE_PER_THREAD];
#pragma unroll
    for (int k = 0; k < NODE_PER_THREAD; k++) {
        c[k] = classify_node((uint8_t)(packed >> (8 * k)));
        ilen[k] = 0;
        blob[k] = 0;
        if (c[k].init) {
            blob[k] = S.node_blob[first + k];
            ilen[k] = init_patch_len(S, blob[k]);
            v[0]++;
            v[1] += (ilen[k] + 15u) & ~15u;
        }
    }
    uint32_t tot[2];
    block_excl_scan<2>(v, tot);
    const uint64_t chunk_bytes = L.init_base + run.v[AG_INIT_BYTES];
    uint32_t newpacked = 0, ji = v[0];
#pragma unroll
    for (int k = 0; k < NODE_PER_THREAD; k++) {
        uint8_t s = (uint8_t)(packed >> (8 * k));
        if (c[k].init) {
            const uint64_t ord = run.v[AG_INIT] + ji;
            S.init_nodes[ord] = S.node_handle_base + (int32_t)(first + k);
            S.init_off[ord] = chunk_bytes + v[1];
            S.init_len[ord] = ilen[k];
            S.init_job[ord] = blob[k];  // the patch bytes: k_emit
            ji++;
            v[1] += (ilen[k] + 15u) & ~15u;
            s |= NS_CONFORMS;  // the apiserver applied the init patch
        }
        s &= (uint8_t)~NS_EVENT_LOCK;
        newpacked |= (uint32_t)s << (8 * k);
    }
    if (i < nn && newpacked != packed) *reinterpret_cast<uint32_t*>(S.node_state + first) = newpacked;
    __syncthreads();
    run.v[AG_INIT] += tot[0];
    run.v[AG_INIT_BYTES] += tot[1];
}

// pod chunk c: the block's live groups [c*256, c*256 + 256)
constexpr uint32_t POD_STAGE_WORDS = 512 * (16 + 8) / 4;  // per wave: 512 jobs x (record + offset)
constexpr uint32_t POD_STAGE_WORDS_F = 512 * 16 / 4;      // fused (k_pod_jobs<true>): the records only
// fused emission (k_pod_jobs<true>): the patch bytes of a wave's staged jobs,
// written by the wave itself (defined with k_emit's table path below)
struct TabWave {  // k_emit's EmitWave, table path only: job records, value rows
    uint4 rec[64];
    uint8_t seg[(VROW_BIAS + 64 * VROW_STRIDE + 4 + 15) & ~15];
};
__device__ __forceinline__ void fused_pod_emit(const DevState& S, TabWave* W, const uint4* stg, uint32_t n, uint64_t ord0, uint64_t off0);
// A thread's jobs take consecutive ordinals (thread-major canonical order), so a
// wave's jobs are one contiguous ordinal range: their 16-byte k_emit records and
// 8-byte arena offsets are staged in LDS (`stage`, 12 KiB per wave: up to 512
// jobs) and written out as whole rows instead of one cache line per lane per
// pod (the initial 1M x 10M tick's job stores: ~270 of its ~510 us of pod
// emission).
// NC dirty chunks at a time (cs[0] < cs[1] in canonical order): their loads,
// classification and scans overlap, and the block synchronises once per NC
// chunks.  A chunk costs ~9 us of mostly fixed latency (group loads ~2, scan ~1,
// emission with its reused-address loads ~3.6, the closing barrier ~2.3: trace
// of the 1M x 10M churn tick, which visits all 19 chunks of every block).
// WAVE: the same for one wave's 64-group run on its own (k_pod_jobs): wave
// scans, no block barrier; gidx = the thread's group index in each chunk.
// FUSE (k_pod_jobs<true>): the staged records carry the patch length (record.w
// = spec | len << 16) and the wave emits their bytes itself (fused_pod_emit, over
// its own stage); no k_emit job records, offsets written by the emission.
template <int NC, bool WAVE = false, bool FUSE = false>
__device__ __forceinline__ void emit_pod_chunks(const DevState& S, const uint32_t* gpre, const uint8_t* nflags, uint32_t bk0,
                                                uint32_t nbk, uint32_t ng, const uint32_t (&gidx)[NC], Bases& run,
                                                const Layout& L, uint32_t* stage, uint32_t nj0 = 0, uint32_t jt = 0) {
    PodGrp g[NC];
    uint16_t sp[NC][POD_PER_THREAD];
#pragma unroll
    for (int i = 0; i < NC; i++) load_group(S, gpre, bk0, nbk, ng, gidx[i], g[i], !FUSE);
    if constexpr (FUSE) {  // (issued with the spec ids: the same round trip)
#pragma unroll
        for (int i = 0; i < NC; i++) load_group_ips_set(S, g[i]);
    }
#pragma unroll
    for (int i = 0; i < NC; i++) load_spec_ids(S, g[i], sp[i]);
    PodCls cl[NC][POD_PER_THREAD];
    // every global input of the emission loop below is loaded here, before the
    // scan, as one batch of independent loads (inside the loop, each pod's spec
    // descriptor / reused address was a dependent round trip of its own):
    // the spec lengths (one descriptor when the group's pods share a spec, the
    // usual case), the pods' creation times and held host IPs
    uint32_t sd_len[NC][POD_PER_THREAD], sd_max[NC][POD_PER_THREAD], ctm[NC][POD_PER_THREAD], hipk[NC][POD_PER_THREAD];
    uint32_t v[4 * NC];  // per chunk: del, pp, pp bytes, alloc
#pragma unroll
    for (int i = 0; i < NC; i++) {
        bool any_need = false, one_spec = true;
#pragma unroll
        for (int k = 0; k < POD_PER_THREAD; k++) {
            cl[i][k] = classify_pod(g[i].st(k), group_node_flags(S, nflags, g[i], k, nj0), g[i].ip[k], S.cni != 0);
            any_need |= cl[i][k].need;
            one_spec &= sp[i][k] == sp[i][0];
        }
        if (any_need) {
            if (one_spec) {
                const SpecDesc& sd = S.specs[sp[i][0]];
                const uint32_t ln = (uint32_t)sd.len_a + sd.len_b + sd.len_c, mx = sd.max_len;
#pragma unroll
                for (int k = 0; k < POD_PER_THREAD; k++) sd_len[i][k] = ln, sd_max[i][k] = mx;
            } else {
#pragma unroll
                for (int k = 0; k < POD_PER_THREAD; k++) {
                    const SpecDesc& sd = S.specs[sp[i][k]];
                    sd_len[i][k] = (uint32_t)sd.len_a + sd.len_b + sd.len_c;
                    sd_max[i][k] = sd.max_len;
                }
            }
            const uint4 ta = *reinterpret_cast<const uint4*>(S.pod_ctime + g[i].slot);
            const uint4 tb = *reinterpret_cast<const uint4*>(S.pod_ctime + g[i].slot + 4);
            // held host IPs only when a pod holds one (a pod without PS_HAS_HOST_IP gets the
            // node's; its host_ip word is not read, and is written as 0 with the group's)
            bool any_hip = false;
#pragma unroll
            for (int k = 0; k < POD_PER_THREAD; k++) any_hip |= (g[i].st(k) & PS_HAS_HOST_IP) != 0;
            uint4 ha = make_uint4(0, 0, 0, 0), hb = ha;
            if (any_hip) {
                ha = *reinterpret_cast<const uint4*>(S.host_ip + g[i].slot);
                hb = *reinterpret_cast<const uint4*>(S.host_ip + g[i].slot + 4);
            }
            ctm[i][0] = ta.x, ctm[i][1] = ta.y, ctm[i][2] = ta.z, ctm[i][3] = ta.w;
            ctm[i][4] = tb.x, ctm[i][5] = tb.y, ctm[i][6] = tb.z, ctm[i][7] = tb.w;
            hipk[i][0] = ha.x, hipk[i][1] = ha.y, hipk[i][2] = ha.z, hipk[i][3] = ha.w;
            hipk[i][4] = hb.x, hipk[i][5] = hb.y, hipk[i][6] = hb.z, hipk[i][7] = hb.w;
        } else {
#pragma unroll
            for (int k = 0; k < POD_PER_THREAD; k++) sd_len[i][k] = sd_max[i][k] = ctm[i][k] = hipk[i][k] = 0;
        }
        v[4 * i] = v[4 * i + 1] = v[4 * i + 2] = v[4 * i + 3] = 0;
#pragma unroll
        for (int k = 0; k < POD_PER_THREAD; k++) {
            v[4 * i] += cl[i][k].del;
            if (cl[i][k].need) {
                v[4 * i + 1]++;
                v[4 * i + 2] += sd_max[i][k];
            }
            v[4 * i + 3] += cl[i][k].alloc;
        }
    }
    uint32_t my_alloc[NC];
#pragma unroll
    for (int i = 0; i < NC; i++) my_alloc[i] = v[4 * i + 3];
    uint32_t tot[4 * NC];
    if constexpr (WAVE) wave_excl_scan<4 * NC>(v, tot);
    else block_excl_scan<4 * NC>(v, tot);
    // chunk i's bases: the running prefix plus the totals of the chunks before it
    Bases rb[NC];
#pragma unroll
    for (int i = 0; i < NC; i++) {
        rb[i] = run;
#pragma unroll
        for (int j = 0; j < i; j++) {
            rb[i].v[AG_DEL] += tot[4 * j];
            rb[i].v[AG_PP] += tot[4 * j + 1];
            rb[i].v[AG_PP_BYTES] += tot[4 * j + 2];
            rb[i].v[AG_ALLOC] += tot[4 * j + 3];
        }
    }
    const uint64_t take = L.plan.take, fin = L.plan.fin, fout0 = L.plan.fout0;
    // the thread's reused / in-bitmap addresses: ordinals [base + v[3], + my_alloc), one batch
    uint32_t areuse[NC][POD_PER_THREAD];
#pragma unroll
    for (int i = 0; i < NC; i++)
#pragma unroll
        for (int k = 0; k < POD_PER_THREAD; k++) {
            const uint64_t o = rb[i].v[AG_ALLOC] + v[4 * i + 3] + (uint32_t)k;
            areuse[i][k] = ((uint32_t)k < my_alloc[i] && L.alloc_base + o < take + fin) ? S.alloc_addr[o] : 0u;
        }
    uint4* stg = reinterpret_cast<uint4*>(stage + (threadIdx.x >> 6) * (FUSE ? POD_STAGE_WORDS_F : POD_STAGE_WORDS));
    uint64_t* stg_off = reinterpret_cast<uint64_t*>(stg + 512);
#pragma unroll
    for (int i = 0; i < NC; i++) {
        const Bases& r = rb[i];
        const PodGrp& gi = g[i];
        const uint64_t chunk_bytes = L.pod_base + r.v[AG_PP_BYTES];
        uint32_t vdel = v[4 * i], jl = v[4 * i + 1], vbytes = v[4 * i + 2];
        const uint32_t va = v[4 * i + 3];
        const uint32_t wpre = (uint32_t)__shfl((int)jl, 0);  // the wave's first job (block-chunk relative)
        bool dirty = false;
        uint16_t nst[POD_PER_THREAD];
        uint32_t ai = 0;
        // the group's hostIP / podIP words after the patches (the loaded values
        // where unchanged): written as two 16-byte stores each, not one per pod
        uint32_t nh[POD_PER_THREAD], np[POD_PER_THREAD];
        bool wh = false, wp = false;
#pragma unroll
        for (int k = 0; k < POD_PER_THREAD; k++) nh[k] = hipk[i][k], np[k] = gi.ip[k];
        // the group's 8 slots share a bucket (bk0 + j): handles without a division
        const uint32_t gb = bk0 + gi.j;
        const int32_t h0 = (int32_t)((S.b_lo + gb) * S.pod_stride + (gi.slot - gb * S.cp));
#pragma unroll
        for (int k = 0; k < POD_PER_THREAD; k++) {
            const int32_t handle = h0 + k;
            uint16_t s = gi.st(k);
            if (cl[i][k].del) {
                const uint64_t ord = r.v[AG_DEL] + vdel++;
                S.del_pods[ord] = handle;
                S.del_fin[ord] = (s & PS_HAS_FIN) ? 1 : 0;
                s = 0;  // DeletePod -> Delete(grace 0): the object is gone
            }
            if (cl[i][k].eval) {
                uint32_t pip = gi.ip[k];
                if (cl[i][k].alloc) {
                    const uint32_t a = ai++;  // the thread's a-th allocation
                    const uint64_t o = r.v[AG_ALLOC] + va + a;
                    const uint64_t gidx = L.alloc_base + o;
                    uint32_t ra = areuse[i][0];
#pragma unroll
                    for (int q = 1; q < POD_PER_THREAD; q++) ra = a == (uint32_t)q ? areuse[i][q] : ra;
                    pip = gidx < take + fin ? ra : (uint32_t)(fout0 + (gidx - take - fin));
                }
                if (cl[i][k].need) {
                    const bool stat = s & PS_STATUS_NONEMPTY;
                    uint32_t hip = 0;
                    if (stat) {
                        hip = (s & PS_HAS_HOST_IP) ? hipk[i][k] : S.node_ip;
                        if (!(s & PS_HAS_HOST_IP)) nh[k] = hip, wh = true;
                        if (pip != gi.ip[k]) np[k] = pip, wp = true;
                    }
                    const uint64_t ord = r.v[AG_PP] + jl;
                    const uint32_t len = sd_len[i][k] + (stat ? 23u + ip_len(hip) + ip_len(pip) : 0u);
                    S.pp_pods[ord] = handle;
                    if constexpr (!FUSE) stg_off[jl - wpre] = chunk_bytes + vbytes;
                    S.pp_len[ord] = len;
                    // the bytes: k_emit (FUSE: this wave, below; len <= max_len < 2^16)
                    stg[jl - wpre] = make_uint4(stat ? pip : 0u, hip, ctm[i][k], FUSE ? (uint32_t)sp[i][k] | len << 16 : sp[i][k]);
                    jl++;
                    vbytes += sd_max[i][k];
                    // the apiserver applied the patch
                    s = (uint16_t)((s & ~PS_PHASE_MASK) | (PHASE_RUNNING << PS_PHASE_SHIFT) | PS_CONFORMS |
                                   PS_STATUS_NONEMPTY | (stat ? PS_HAS_HOST_IP : 0));
                    if (stat) s = (uint16_t)((s & ~PS_IP_BITS) | ip_state_bits(S.pool, pip));
                }
                s &= (uint16_t)~PS_EVENT;
            }
            dirty |= s != gi.st(k);
            nst[k] = s;
        }
        uint32_t fuse_n = 0;  // FUSE: the wave's job count (emitted below, after the state stores)
        uint64_t fuse_off0 = 0;
        if constexpr (FUSE) {
            fuse_n = (uint32_t)__shfl((int)jl, 63) - wpre;
            fuse_off0 = chunk_bytes + (uint32_t)__shfl((int)v[4 * i + 2], 0);  // the wave's first job's offset
        } else {  // the wave's staged records -> pp_job[base + wpre, base + wend); the wave's
           // LDS operations run in order, so the next chunk's staging follows these reads
            const uint32_t wend = (uint32_t)__shfl((int)jl, 63);
            uint4* dst = S.pp_job + r.v[AG_PP] + wpre;
            uint64_t* dst_off = S.pp_off + r.v[AG_PP] + wpre;
            for (uint32_t q = lane_id(); q < wend - wpre; q += 64) dst[q] = stg[q], dst_off[q] = stg_off[q];
        }
        if (wh) {
            *reinterpret_cast<uint4*>(S.host_ip + gi.slot) = make_uint4(nh[0], nh[1], nh[2], nh[3]);
            *reinterpret_cast<uint4*>(S.host_ip + gi.slot + 4) = make_uint4(nh[4], nh[5], nh[6], nh[7]);
        }
        if (wp) {
            *reinterpret_cast<uint4*>(S.pod_ip + gi.slot) = make_uint4(np[0], np[1], np[2], np[3]);
            *reinterpret_cast<uint4*>(S.pod_ip + gi.slot + 4) = make_uint4(np[4], np[5], np[6], np[7]);
        }
        if (gi.slot != ~0u && dirty) {
            uint4 o;
            o.x = nst[0] | (uint32_t)nst[1] << 16;
            o.y = nst[2] | (uint32_t)nst[3] << 16;
            o.z = nst[4] | (uint32_t)nst[5] << 16;
            o.w = nst[6] | (uint32_t)nst[7] << 16;
            *reinterpret_cast<uint4*>(S.pod_state + gi.slot) = o;
        }
        if constexpr (FUSE) {  // the staged jobs' bytes: the wave's stage becomes the emission's rows
            __builtin_amdgcn_wave_barrier();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (S.jtrace && lane_id() == 0) {
                const size_t q = (size_t)jt * 4;
                S.jtrace[q + 1] = __builtin_amdgcn_s_memrealtime();
                S.jtrace[q + 3] = (uint64_t)fuse_n << 32 | __builtin_amdgcn_s_getreg((4) | (15 << 11)) |
                                  (uint64_t)(__builtin_amdgcn_s_getreg((20) | (15 << 11)) & 15u) << 28;
            }
            fused_pod_emit(S, reinterpret_cast<TabWave*>(stg), stg, fuse_n, r.v[AG_PP] + wpre, fuse_off0);
        }
    }
    if constexpr (!WAVE) __syncthreads();
#pragma unroll
    for (int i = 0; i < NC; i++) {
        run.v[AG_DEL] += tot[4 * i];
        run.v[AG_PP] += tot[4 * i + 1];
        run.v[AG_PP_BYTES] += tot[4 * i + 2];
        run.v[AG_ALLOC] += tot[4 * i + 3];
    }
}

// ---------------------------------------------------------------------------
// heartbeat stream: n_hb identical 1059-byte patches, 67 x 16 B each, from an
// LDS template with 16-byte stores (node_controller.go:145-157)
// ---------------------------------------------------------------------------
constexpr int HB_CHUNKS = HB_STRIDE / 16;  // 67
// The stream is written in groups of 4 slots (4 x 67 = 268 units of 16 B): lane l
// of a wave writes units 64k + l (k = 0..4) of a group, which are always the same
// template units, so a wave keeps its 5 template units in registers and the loop
// is 5 plain 16-byte stores per group (no LDS read per store).
constexpr uint32_t HB_GROUP_SLOTS = 4, HB_GROUP_UNITS = HB_GROUP_SLOTS * HB_CHUNKS;  // 268
static_assert(HB_GROUP_UNITS > 256 && HB_GROUP_UNITS <= 320, "5 stores of a wave per group");
static_assert(HB_GROUP_SLOTS * HB_MAX_UNITS <= 320, "custom heartbeats: still 5 stores of a wave per group");
// A custom heartbeat (any 16-byte unit count up to HB_MAX_UNITS): the same
// group walk with the unit count a launch argument, every store predicated.
__device__ __noinline__ void hb_fill_groups_any(const DevState& S, const uint4* tmpl, uint64_t n_hb, uint64_t g0,
                                                uint64_t g1) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint32_t l = lane_id(), w = wave_id(), U = S.hb_units, GU = HB_GROUP_SLOTS * U;
    u32x4 r[5];
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const uint4 v = tmpl[(64u * k + l) % U];
        r[k] = u32x4{v.x, v.y, v.z, v.w};
    }
    const uint64_t units = n_hb * U;
    u32x4* dst = reinterpret_cast<u32x4*>(S.arena);
    for (uint64_t g = g0 + w; g < g1; g += BLOCK / 64) {
        const uint64_t u0 = g * GU + l;
        u32x4* p = dst + u0;
        if (S.hb_nt) {
#pragma unroll
            for (int k = 0; k < 5; k++)
                if (64u * k + l < GU && u0 + 64u * k < units) __builtin_nontemporal_store(r[k], p + 64 * k);
        } else {
#pragma unroll
            for (int k = 0; k < 5; k++)
                if (64u * k + l < GU && u0 + 64u * k < units) p[64 * k] = r[k];
        }
    }
}
// groups [g0, g1) of the heartbeat region (units past n_hb slots are not written).
// GEN: a custom heartbeat geometry (k_tick<true>); the default one compiles
// without the general walk so its register allocation is untouched.
template <bool GEN>
__device__ __forceinline__ void hb_fill_groups(const DevState& S, const uint4* tmpl, uint64_t n_hb, uint64_t g0,
                                               uint64_t g1) {
    if (GEN) {
        hb_fill_groups_any(S, tmpl, n_hb, g0, g1);
        return;
    }
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const uint32_t l = lane_id(), w = wave_id();
    u32x4 r[5];
#pragma unroll
    for (int k = 0; k < 5; k++) {
        const uint4 v = tmpl[(64u * k + l) % HB_CHUNKS];
        r[k] = u32x4{v.x, v.y, v.z, v.w};
    }
    const uint64_t units = n_hb * HB_CHUNKS;
    u32x4* dst = reinterpret_cast<u32x4*>(S.arena);  // heartbeat region starts at arena offset 0
    for (uint64_t g = g0 + w; g < g1; g += BLOCK / 64) {
        const uint64_t u0 = g * HB_GROUP_UNITS + l;
        u32x4* p = dst + u0;
        if (S.hb_nt && u0 + 256u < units) {  // a whole group, non-temporal (S.hb_nt: uniform)
#pragma unroll
            for (int k = 0; k < 4; k++) __builtin_nontemporal_store(r[k], p + 64 * k);
            if (l < HB_GROUP_UNITS - 256u) __builtin_nontemporal_store(r[4], p + 256);
        } else if (u0 + 256u < units) {  // a whole group (every group but possibly the last)
#pragma unroll
            for (int k = 0; k < 4; k++) p[64 * k] = r[k];  // plain stores: 7.5 TB/s (tools/micro/fill.hip)
            if (l < HB_GROUP_UNITS - 256u) p[256] = r[4];
        } else {
#pragma unroll
            for (int k = 0; k < 5; k++)
                if (64u * k + l < HB_GROUP_UNITS && u0 + 64u * k < units) p[64 * k] = r[k];
        }
    }
}

// static shares of the heartbeat stream: the streamer blocks split the first
// stream_share/1024 of it, and every chain block writes an equal slice of the
// rest once its own work is done (so the stream's tail overlaps nothing idle)
// a chain block's slice of the stream is not empty (block-uniform; heartbeat-once
// engines have no streamers: one chain block writes the one body)
__device__ __forceinline__ bool hb_share_any(const DevState& S, uint64_t n_hb, uint32_t idx, uint32_t cnt) {
    const uint64_t groups = (n_hb + HB_GROUP_SLOTS - 1) / HB_GROUP_SLOTS;
    const uint64_t cut = groups * S.stream_share / 1024, n = groups - cut;
    return n * idx / cnt < n * (idx + 1) / cnt;
}
template <bool GEN>
__device__ __forceinline__ void hb_fill_share(const DevState& S, const uint4* tmpl, uint64_t n_hb, bool streamer,
                                              uint32_t idx, uint32_t cnt) {
    const uint64_t groups = (n_hb + HB_GROUP_SLOTS - 1) / HB_GROUP_SLOTS;
    const uint64_t cut = groups * S.stream_share / 1024;
    const uint64_t lo = streamer ? 0 : cut, n = streamer ? cut : groups - cut;
    hb_fill_groups<GEN>(S, tmpl, n_hb, lo + n * idx / cnt, lo + n * (idx + 1) / cnt);
}

// per-tick heartbeat template in LDS: static bytes + Now / StartTime slots
__device__ __forceinline__ void build_hb_template(const DevState& S, uint8_t* tmpl, uint64_t now_unix, uint64_t start_unix) {
    const Ts now = format_ts(now_unix), st = format_ts(start_unix);
    for (int i = threadIdx.x; i < (int)(16u * S.hb_units); i += BLOCK) {
        const uint8_t k = S.hb_kind[i];
        uint32_t b;
        if (k == 0xFF) b = S.hb_static[i];
        else if (k < TS_LEN) b = ts_byte(now, k);
        else b = ts_byte(st, k - TS_LEN);
        tmpl[i] = (uint8_t)b;
    }
    __syncthreads();
}

// ---------------------------------------------------------------------------
// header / exchange message (FRONT launch, written by the last arriver).  The
// header is assembled in LDS and stored with one coalesced pass to the device
// copy and (single rank) the pinned host copy; the host reads it after the
// launch completes.  Single rank: when a pool phase follows, its leader
// publishes the Get plan / cursor (skip_alloc) and its stamps (skip_pool).
// ---------------------------------------------------------------------------
// heartbeat bodies the tick materialises: one per managed node, or one in all
// (KWOK_CFG_HEARTBEAT_ONCE: every node's patch is that body)
__device__ __forceinline__ uint32_t hb_bodies(const DevState& S, uint32_t n_hb) { return S.hb_once ? min(n_hb, 1u) : n_hb; }

// word i of the tick header (TickHdr as 61 x u64), computed by thread i
__device__ __forceinline__ uint64_t header_word(int i, const uint64_t* tot, uint32_t n_hb, uint32_t hb_stride, uint32_t nu,
                                                uint64_t pool_index, uint64_t arena_cap, bool single, const uint64_t* clk) {
    constexpr int W_LC = offsetof(TickHdr, local_counters) / 8, W_C = offsetof(TickHdr, counters) / 8;
    constexpr int W_CLK = offsetof(TickHdr, clk) / 8;
    static_assert(offsetof(TickHdr, init_bytes) == 48 && offsetof(TickHdr, local_counters) == 96 &&
                      offsetof(TickHdr, alloc_total) == 352 && offsetof(TickHdr, clk) == 416 &&
                      offsetof(TickHdr, err) == 480,
                  "TickHdr layout");
    const uint64_t patch_base = (uint64_t)n_hb * hb_stride;  // n_hb: the heartbeat bodies materialised
    const uint64_t arena_bytes = patch_base + tot[AG_INIT_BYTES] + tot[AG_PP_BYTES];
    auto pair = [](uint64_t lo, uint64_t hi) { return (uint64_t)(uint32_t)lo | (uint64_t)(uint32_t)hi << 32; };
    if (i >= W_LC && i < W_C + 16) {
        // local_counters / counters: heartbeat, node_init, pod_patch, delete, alloc, release,
        // evaluated, lock_checked, nodes_managed, nodes_ready, pods_total, pods_pending, pods_running
        const int k = (i - W_LC) & 15;
        constexpr uint64_t MAP = (uint64_t)AG_HB | (uint64_t)AG_INIT << 4 | (uint64_t)AG_PP << 8 | (uint64_t)AG_DEL << 12 |
                                 (uint64_t)AG_ALLOC << 16 | (uint64_t)AG_REL << 20 | (uint64_t)AG_EVAL << 24 |
                                 (uint64_t)AG_LOCK << 28 | (uint64_t)AG_MANAGED << 32 | (uint64_t)AG_READY << 36 |
                                 (uint64_t)AG_TOTAL << 40 | (uint64_t)AG_PENDING << 44 | (uint64_t)AG_RUNNING << 48;
        if (k >= 13 || (i >= W_C && !single)) return 0;  // fleet counters: the BACK launch (multi rank)
        return tot[(MAP >> (4 * k)) & 15];
    }
    if (i >= W_CLK && i < W_CLK + 8) return clk[i - W_CLK];
    switch (i) {
        case 0: return pair(tot[AG_HB], tot[AG_INIT]);
        case 1: return pair(tot[AG_PP], tot[AG_DEL]);
        case 2: return pair(nu, tot[AG_REL]);
        case 3: return pair(tot[AG_ALLOC], tot[AG_EVAL]);
        case 4: return pair(tot[AG_LOCK], arena_bytes > arena_cap);
        case 6: return tot[AG_INIT_BYTES];
        case 7: return tot[AG_PP_BYTES];
        case 9: return patch_base;                        // init_base (hb_base, word 8, is 0)
        case 10: return patch_base + tot[AG_INIT_BYTES];  // pod_base
        case 11: return arena_bytes;
        case 44: return single ? tot[AG_ALLOC] : 0;       // alloc_total (alloc_base, word 45, is 0)
        case 50: return pool_index;                       // cursor_index: the pool phase overwrites it
        case 51: return single ? tot[AG_REL] : 0;         // rel_total
        default: return 0;                                // pads, hb_base, alloc_base, the Get plan
    }
}

// ---------------------------------------------------------------------------
// header / exchange message (FRONT launch, written by the last arriver): one
// header word per thread, stored to the device copy and (single rank) the
// pinned host copy; the host reads it after the launch completes.  Single
// rank: when a pool phase follows, its leader publishes the Get plan / cursor
// (skip_alloc) and its stamps (skip_pool) itself, concurrently.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void write_front_header(const DevState& S, const Sums& r, uint32_t n_hb, uint64_t pool_index,
                                                   uint64_t c_p1, bool prof, uint32_t tag) {
    const uint64_t* tot = r.tot;
    const bool single = !S.multi;
    // multi rank: the blocks' list lengths (every block arrived: their records and lengths are out)
    __shared__ uint32_t lsum[2];
    if (threadIdx.x < 2) lsum[threadIdx.x] = 0;
    __syncthreads();
    if (!single) {
        uint32_t u = 0, r = 0;
        for (uint32_t b = threadIdx.x; b < S.n_chain; b += BLOCK) u += ld32_sc1(&S.list_blk[2 * b]), r += ld32_sc1(&S.list_blk[2 * b + 1]);
        if (u) atomicAdd(&lsum[0], u);
        if (r) atomicAdd(&lsum[1], r);
    }
    __syncthreads();
    const uint32_t nu = lsum[0], nr = lsum[1];
    uint64_t clk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    clk[CLK_P1_MAX] = c_p1;
    if (prof) clk[CLK_ENTRY_MIN] = ~ld_sc1(&S.bar->neg_entry_max);
    clk[CLK_HDR] = __builtin_amdgcn_s_memrealtime();
    constexpr int NW = offsetof(TickHdr, err) / 8;
    constexpr int A0 = offsetof(TickHdr, usable_total) / 8, A1 = offsetof(TickHdr, rel_total) / 8;
    constexpr int C0 = offsetof(TickHdr, clk) / 8;
    const bool skip_alloc = single && tot[AG_ALLOC] != 0, skip_pool = single && (tot[AG_ALLOC] | tot[AG_REL]) != 0;
    const int i = threadIdx.x;
    if (i < NW) {
        const uint64_t w = header_word(i, tot, hb_bodies(S, n_hb), 16u * S.hb_units, nu, pool_index, S.arena_cap, single, clk);
        const bool pool_clk = i == C0 + CLK_BACK || i == C0 + CLK_POOL;
        // the pool leader may already have written its fields (it runs concurrently)
        if (!(skip_pool && (pool_clk || (i >= A0 && i < A1)))) reinterpret_cast<uint64_t*>(S.hdr)[i] = w;
        if (single && !(skip_alloc && i >= A0 && i < A1) && !(skip_pool && pool_clk))
            st_host(reinterpret_cast<uint64_t*>(S.hdr_host) + i, w);
    }
    if (i == 0) {
        if (tot[AG_HB] != n_hb)  // the heartbeat stream was laid out for the host's count
            __hip_atomic_store(&S.hdr_host->err, TICK_ERR_LAYOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (prof) __hip_atomic_store(&S.bar->neg_entry_max, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!single) {
            XMsg* X = S.xmsg;
            X->alloc = tot[AG_ALLOC];
            X->seq = tag;
            X->foreign = S.foreign;
            X->n_use = nu;
            X->n_rel = nr;
            constexpr int LC = offsetof(TickHdr, local_counters) / 8;
            for (int k = 0; k < 16; k++)
                X->counters[k] = header_word(LC + k, tot, hb_bodies(S, n_hb), 16u * S.hb_units, nu, pool_index,
                                             S.arena_cap, single, clk);
        }
    }
    if (!single && nu + nr <= (uint32_t)XINLINE && nu + nr) {  // exchange lists inline when they fit
        uint32_t pu = 0, pr = nu;  // the blocks' segments in block order
        for (uint32_t b = 0; b < S.n_chain; b++) {
            const uint32_t cu = ld32_sc1(&S.list_blk[2 * b]), cr = ld32_sc1(&S.list_blk[2 * b + 1]);
            if (!(cu | cr)) continue;
            uint32_t bk0, nbk;
            block_range(S, b, bk0, nbk);
            const uint32_t seg = bk0 * S.cp;
            for (uint32_t j = threadIdx.x; j < cu; j += BLOCK) S.xmsg->ips[pu + j] = ld32_sc1(&S.use_list[seg + j]);
            for (uint32_t j = threadIdx.x; j < cr; j += BLOCK) S.xmsg->ips[pr + j] = ld32_sc1(&S.rel_list[seg + j]);
            pu += cu, pr += cr;
        }
    }
}

// multi rank (BACK launch, block 0): copy the device header to the pinned host copy
__device__ __forceinline__ void publish_header(const DevState& S) {
    __syncthreads();
    const uint64_t* src = reinterpret_cast<const uint64_t*>(S.hdr);
    uint64_t* dst = reinterpret_cast<uint64_t*>(S.hdr_host);
    for (int i = threadIdx.x; i < (int)(offsetof(TickHdr, err) / 8); i += BLOCK) st_host(dst + i, src[i]);
    __syncthreads();
}

// KeepNodeHeartbeat handles (node_controller.go:175-204): the block's managed
// nodes in node order from the host-maintained base, after the block arrived
// (nothing waits on them)
// the block's managed nodes' handles, in node order, from position hb_run: each
// thread takes a contiguous run of the block's nodes (node order = thread order),
// so one block scan of the per-thread counts places them all
__device__ __forceinline__ void write_hb_handles(const DevState& S, const uint32_t* nflags32, uint32_t nbase, uint32_t nn,
                                                 uint32_t hb_run) {
    const uint8_t* nf = reinterpret_cast<const uint8_t*>(nflags32);
    const uint32_t q = (nn + BLOCK - 1) / BLOCK;
    const uint32_t a = min(nn, threadIdx.x * q), e = min(nn, a + q);
    uint32_t c[1] = {0}, tot[1];
    for (uint32_t i = a; i < e; i++) c[0] += (nf[i] >> 1) & 1u;  // NT_MANAGED
    block_excl_scan<1>(c, tot);
    uint32_t pos = hb_run + c[0];
    for (uint32_t i = a; i < e; i++)
        if ((nf[i] >> 1) & 1u) {
            if (pos < S.n_node_slots) S.hb_nodes[pos] = S.node_handle_base + (int32_t)(nbase + i);
            pos++;
        }
}

// pointers into k_tick's LDS for the out-of-line BACK phases
struct TickLds {
    uint32_t* recs;
    uint32_t* nflags32;
    uint32_t* gpre;
    Sums* sums;
    Layout* L;
};

// The pool phase's passes among np blocks (this one: pidx): fold the tick's Puts
// and count every word-block, the barrier, the plan from the counts, then the
// Gets' selection (A > 0).  W: bitmap words per thread of a word-block.
template <int W>
__device__ __forceinline__ void pool_passes(const DevState& S, uint32_t pidx, uint32_t np, uint64_t A, uint64_t rel_total,
                                            uint64_t alloc_base, uint64_t n_alloc_local, uint64_t (&cp)[2][BLOCK],
                                            PoolPlan& plan, uint64_t& cursor, uint64_t* stamps) {
    const uint32_t nwb = (uint32_t)((S.pool.words + BLOCK * W - 1) / (BLOCK * W));
    PoolWords<W> pw;  // the block's first word-block, kept for its select pass
    for (uint32_t wb = pidx; wb < nwb; wb += np) {
        PoolWords<W> x;
        pool_prep_wblock<W>(S, wb, rel_total != 0, A != 0, x);
        if (wb == pidx) pw = x;
    }
    if (stamps) stamps[18] = __builtin_amdgcn_s_memrealtime();
    pool_barrier(S, np);
    if (stamps) stamps[9] = __builtin_amdgcn_s_memrealtime();
    if (!A) return;
    const PoolPre q = pool_scan(S, nwb, cp);
    plan = pool_plan(S, A, q);
    if (stamps) stamps[19] = __builtin_amdgcn_s_memrealtime();
    for (uint32_t wb = pidx; wb < nwb; wb += np) {
        uint64_t bu, bf;
        pool_prefix(S, q, cp, wb, &bu, &bf);
        // every Get is taken before this word-block (and so before the block's later
        // ones): nothing to select from here on (a pool much larger than the fleet)
        if (bu >= plan.take && bf >= plan.fin) break;
        pool_select_wblock<W>(S, wb, plan, bu, bf, alloc_base, alloc_base + n_alloc_local, &cursor,
                              wb == pidx ? &pw : nullptr);
    }
}

// BACK phases of a chain block that has something to emit (and, multi rank,
// every block when the pool phase runs): prefix over the records, ipPool phase,
// emission.  Out of line so the steady-state path keeps its registers; the
// device state is read through its copy in device memory (S.self).
__device__ __forceinline__ void tick_back(const DevState* __restrict__ G, TickLds l, uint32_t b, uint32_t bk0, uint32_t nbk,
                                       uint64_t pod_mask, uint32_t node_mask, uint32_t my_init, bool have_sums,
                                       int phases, uint32_t n_hb, uint64_t now_unix, uint64_t start_unix, uint64_t xA,
                                       uint64_t xrel, uint64_t xbase, uint32_t tag) {
    const DevState& S = *G;
    const int t = threadIdx.x;
    TickHdr* H = S.hdr;
    const uint32_t nn = nbk * S.cn, nbase = bk0 * S.cn;
#define TSTAMP(k)                                                                                         \
    do {                                                                                                  \
        if (S.trace && t == 0) S.trace[(size_t)b * TRACE_SLOTS + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
    TSTAMP(16);
    if (!have_sums) reduce_records(S, b, 0, l.recs, l.sums);
    TSTAMP(17);

    // ---- pool phase (ticks with Gets or Puts) -------------------------------------
    const bool single = !S.multi;
    const uint64_t A = single ? l.sums->tot[AG_ALLOC] : xA;
    const uint64_t rel_total = single ? l.sums->tot[AG_REL] : xrel;
    const uint64_t alloc_base = single ? 0 : xbase;
    const uint64_t n_alloc_local = l.sums->tot[AG_ALLOC];
    // participants: single rank - the dirty blocks (every Get / Put belongs to one);
    // multi rank - every block (each rank commits every rank's Gets to its replica)
    // (+ the BACK launch's pool-only blocks, S.n_pool_extra: the whole grid)
    const uint32_t np = single ? (uint32_t)l.sums->tot[AG_DIRTY] : gridDim.x;
    const uint32_t pidx = single ? (uint32_t)l.sums->pre[AG_DIRTY] : b;
    const bool dirty = (pod_mask | node_mask) != 0;
    PoolPlan plan{};
    uint64_t cursor = ~0ull;
    if (A || rel_total) {
        if (single && pidx == 0 && t == 0) H->clk[CLK_BACK] = __builtin_amdgcn_s_memrealtime();
        uint64_t* stamps = S.trace && t == 0 ? S.trace + (size_t)b * TRACE_SLOTS : nullptr;
        __shared__ uint64_t cp[2][BLOCK];
        if (single)
            pool_passes<POOL_WPT>(S, pidx, np, A, rel_total, alloc_base, n_alloc_local, cp, plan, cursor, stamps);
        else
            pool_passes<POOL_WPT_MULTI>(S, pidx, np, A, rel_total, alloc_base, n_alloc_local, cp, plan, cursor, stamps);
        if (A) {
            TSTAMP(20);
            // ipPool.index after the last fresh address (committed after the barrier)
            if (cursor != ~0ull) H->cursor_index = cursor;
            if (pidx == 0 && t == 0) {
                H->usable_total = plan.U;
                H->take_usable = plan.take;
                H->fresh_in = plan.fin;
                H->fresh_out_start = plan.fout0;
                if (plan.fout) H->cursor_index = plan.fout0 + plan.fout - S.pool.base;
                else if (plan.fin == 0) H->cursor_index = *S.pool_index;
            }
            pool_barrier(S, np);
            if (pidx == 0 && t == 0) *S.pool_index = H->cursor_index;
        }
        if (pidx == 0 && t == 0) {
            H->clk[CLK_POOL] = __builtin_amdgcn_s_memrealtime();
            if (single) {  // the last arriver published everything else (publish_header)
                TickHdr* P = S.hdr_host;
                if (A) {
                    st_host(&P->usable_total, H->usable_total);
                    st_host(&P->take_usable, H->take_usable);
                    st_host(&P->fresh_in, H->fresh_in);
                    st_host(&P->fresh_out_start, H->fresh_out_start);
                    st_host(&P->cursor_index, H->cursor_index);
                }
                st_host(&P->clk[CLK_BACK], H->clk[CLK_BACK]);
                st_host(&P->clk[CLK_POOL], H->clk[CLK_POOL]);
                __threadfence_system();
            }
        }
        TSTAMP(5);
    }
    if (!single && b == 0) publish_header(S);  // multi rank: counts, exchange totals and pool fields
    if (!dirty) {
        TSTAMP(6);
        return;
    }

    // ---- emission of the dirty chunks ----------------------------------------------
    if (!(phases & TICK_FRONT)) {  // BACK launch: the block's pod groups and node flags again
        load_gpre(S, bk0, nbk, l.gpre);
        if (pod_mask)
            for (uint32_t i = t * 4; i < nn; i += NODE_CHUNK)
                l.nflags32[i / 4] = *reinterpret_cast<const uint32_t*>(S.node_tick + nbase + i);
        __syncthreads();
    }
    if (t == 0) {
        const uint64_t patch_base = (uint64_t)hb_bodies(S, n_hb) * (16u * S.hb_units);
        l.L->init_base = patch_base;
        l.L->pod_base = patch_base + l.sums->tot[AG_INIT_BYTES];
        l.L->alloc_base = alloc_base;
        l.L->plan = plan;
    }
    __syncthreads();
    const Layout L = *l.L;
    Bases run;
    for (int f = 0; f < AG_NSCAN; f++) run.v[f] = l.sums->pre[f];
    TSTAMP(15);
    for (uint32_t m = node_mask; m; m &= m - 1) {
        const uint32_t k = (uint32_t)__builtin_ctz(m);
        emit_node_chunk(S, nbase, k * NODE_CHUNK, nn, run, L);
    }
    TSTAMP(14);
    if (phases & TICK_SPLIT) {
        // split tick: k_pod_jobs emits the pod chunks, one wave per dirty 64-group
        // run of this block (FRONT published the runs' prefixes); it starts here
        if (pod_mask && t == 0) {
            JobBase jb;
            jb.del = run.v[AG_DEL];
            jb.pp = run.v[AG_PP];
            jb.pp_bytes = run.v[AG_PP_BYTES];
            jb.alloc = run.v[AG_ALLOC];
            jb.pod_base = L.pod_base;
            jb.alloc_base = L.alloc_base;
            jb.take = L.plan.take;
            jb.fin = L.plan.fin;
            jb.fout0 = L.plan.fout0;
            jb.tag = tag;
            jb.pad = 0;
            S.jbase[b] = jb;
        }
        TSTAMP(6);
        return;
    }
    const uint32_t ng = l.gpre[nbk];
    for (uint64_t m = pod_mask; m;) {  // dirty chunks two at a time, in canonical order
        const uint32_t c0 = (uint32_t)__builtin_ctzll(m);
        m &= m - 1;
        if (m) {
            const uint32_t gx[2] = {c0 * BLOCK + t, (uint32_t)__builtin_ctzll(m) * BLOCK + t};
            m &= m - 1;
            emit_pod_chunks<2>(S, l.gpre, reinterpret_cast<const uint8_t*>(l.nflags32), bk0, nbk, ng, gx, run, L, l.recs);
        } else {
            const uint32_t gx[1] = {c0 * BLOCK + t};
            emit_pod_chunks<1>(S, l.gpre, reinterpret_cast<const uint8_t*>(l.nflags32), bk0, nbk, ng, gx, run, L, l.recs);
        }
    }
    TSTAMP(6);
#undef TSTAMP
}

// ---------------------------------------------------------------------------
// k_tick: one controller tick.  Single rank: ONE launch (FRONT | BACK).
// Multi rank: FRONT launch -> exchange -> BACK launch.
//
// Blocks [0, n_chain) are chain blocks, each owning a contiguous bucket range;
// blocks [n_chain, grid) (FRONT only) stream the heartbeat bodies and touch
// nothing else, so the bandwidth-bound stream overlaps the latency-bound
// classification.
//
//   FRONT  per chain block: node states -> heartbeat handles (host-maintained
//          base), node flags into LDS; live pod groups -> predicates, Use /
//          Put; one block record; arrive.  The LAST arriver reduces the records
//          into the tick header (single rank) / exchange message (multi rank).
//          A block with nothing to emit is done here (the steady state).
//   BACK   per dirty chain block (single rank: after every block arrived):
//          prefix over the records; the pool phase among the dirty blocks when
//          the tick has Gets or Puts (multi rank: among all blocks); emission
//          of the dirty chunks.
// ---------------------------------------------------------------------------
template <bool GEN_HB>
__global__ __launch_bounds__(BLOCK, 2) void k_tick(DevState S, uint64_t now_unix, uint64_t start_unix,
                                                   uint32_t n_hb, int phases, uint32_t tag, uint64_t arrive_target) {
    const int t = threadIdx.x;
    const uint32_t b = blockIdx.x;
    // reduce_records; then emit_pod_chunk's staging (two k_tick blocks per CU still fit)
    __shared__ uint32_t recs[MAX_CHAIN * REC_PITCH > (BLOCK / 64) * POD_STAGE_WORDS ? MAX_CHAIN * REC_PITCH
                                                                                   : (BLOCK / 64) * POD_STAGE_WORDS];
    __shared__ uint4 hb_tmpl4[HB_MAX_UNITS];
    __shared__ uint32_t nflags32[NODE_LDS / 4];
    __shared__ uint32_t gpre[MAX_BPB + 1];
    __shared__ uint16_t spec_max[SPEC_LDS];  // the specs' reservations (n_specs <= SPEC_LDS)
    __shared__ uint32_t sh_mask[4];  // pod chunk mask lo / hi, node chunk mask, most groups in a bucket
    __shared__ Sums sums;
    __shared__ Layout sh_L;
    uint8_t* hb_tmpl = reinterpret_cast<uint8_t*>(hb_tmpl4);
    const uint8_t* nflags = reinterpret_cast<const uint8_t*>(nflags32);
    if (phases == 0) return;  // the engine's warm-up launch (its scratch is set up before the first tick)
    if (!(phases & TICK_XLISTS) && __hip_atomic_load(&S.bar->skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
        return;  // queued behind a tick the host has not finished (long lists; k_once redo): re-launched later
#define TSTAMP(k)                                                                                         \
    do {                                                                                                  \
        if (S.trace && t == 0) S.trace[(size_t)b * TRACE_SLOTS + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
    // trace runs only: drain this wave's memory operations, then stamp (perturbs the overlap)
#define TWAIT(k)                                                     \
    do {                                                             \
        if (S.trace) {                                               \
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
            TSTAMP(k);                                               \
        }                                                            \
    } while (0)
    TSTAMP(0);
    if (S.trace && t == 0)  // (diagnostics: where the block runs - HW_ID, XCC_ID << 28)
        S.trace[(size_t)b * TRACE_SLOTS + 21] = (uint64_t)__builtin_amdgcn_s_getreg((4) | (15 << 11)) |
                                                (uint64_t)(__builtin_amdgcn_s_getreg((20) | (15 << 11)) & 15u) << 28;

    // ---- heartbeat streamers ------------------------------------------------------
    // (a multi-rank BACK launch's blocks past the chain blocks are pool-only blocks)
    if (b >= S.n_chain && (phases & TICK_FRONT)) {
        build_hb_template(S, hb_tmpl, now_unix, start_unix);
        if (S.stream_delay) {  // diagnostics: hold the stream back while the chain's first round trips run
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while (__builtin_amdgcn_s_memrealtime() - t0 < S.stream_delay) __builtin_amdgcn_s_sleep(4);
        }
        if (!(phases & TICK_NOSTREAM))
            hb_fill_share<GEN_HB>(S, hb_tmpl4, hb_bodies(S, n_hb), true, b - S.n_chain, gridDim.x - S.n_chain);
        if ((phases & TICK_PROF) && t == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            atomicMax(&S.bar->stream_end_max, (unsigned long long)__builtin_amdgcn_s_memrealtime());
        }
        TSTAMP(6);
        return;
    }

    if (phases & TICK_PRIO) __builtin_amdgcn_s_setprio(3);  // chain waves issue ahead of the streamers
    uint32_t bk0, nbk;
    block_range(S, b, bk0, nbk);
    const uint32_t nn = nbk * S.cn, nbase = bk0 * S.cn;
    TickHdr* H = S.hdr;
    uint64_t pod_mask = 0;
    uint32_t node_mask = 0;
    uint32_t my_init = 0;
    bool have_sums = false;
    uint64_t xA = 0, xrel = 0, xbase = 0;  // multi rank: fleet Gets / Puts, this rank's first Get ordinal

    if (phases & TICK_FRONT) {
        if (t == 0 && (phases & TICK_PROF))
            atomicMax(&S.bar->neg_entry_max, ~(unsigned long long)__builtin_amdgcn_s_memrealtime());
        if (t < 3) sh_mask[t] = 0;
        const bool single = !S.multi;
        if (t < 3) list_lds()[t] = t == 2 ? bk0 * S.cp : 0u;  // (multi rank: the block's list segment)
        const bool split = (phases & TICK_SPLIT) != 0;
        uint32_t* wcnt = recs;  // split: the 64-group runs' counts (recs is free until reduce_records)
        if (split)
            for (uint32_t i = t; i < 4 * MAX_WC + WC_DIRTY_WORDS; i += BLOCK) wcnt[i] = 0;
        const uint32_t hb_base = S.hb_pre[b];
        // round trip 1, all loads independent: the fill marks, the node states and,
        // speculatively, SPEC_GROUPS pod groups per thread at a static thread ->
        // (bucket, group) map; groups past a bucket's fill mark are discarded when it
        // lands (a bucket with more groups takes one more round trip per extra row)
        const uint32_t tpb = BLOCK / (nbk ? nbk : 1u);  // threads per bucket
        const uint32_t j = t / tpb, l = t - j * tpb;
        const bool jv = j < nbk;
        const uint32_t gcap = S.cp / POD_PER_THREAD;
        // the node states of the block's first NODE_PRE chunks first: loads complete in
        // issue order, so the node classification below waits for these and the fill
        // marks only, not for the pod groups behind them
        uint32_t packed_pre[NODE_PRE];
        auto load_nodes = [&]() {
#pragma unroll
            for (int c = 0; c < NODE_PRE; c++) {
                const uint32_t i = (uint32_t)c * NODE_CHUNK + t * NODE_PER_THREAD;
                packed_pre[c] = i < nn ? *reinterpret_cast<const uint32_t*>(S.node_state + nbase + i) : 0u;
            }
        };
#if KWOK_RT1_NODES_FIRST
        load_nodes();
#endif
        const uint32_t fill = jv ? S.pod_fill[bk0 + j] : 0u;
        PodGrp G[SPEC_GROUPS];
#pragma unroll
        for (int q = 0; q < SPEC_GROUPS; q++) {
            const uint32_t a = l + q * tpb;
            load_group_at(S, jv && a < gcap ? (bk0 + j) * S.cp + a * POD_PER_THREAD : ~0u, j, G[q], false);
        }
#if !KWOK_RT1_NODES_FIRST
        load_nodes();
#endif
        const uint64_t pool_index = single ? 0 : *S.pool_index;  // multi rank: the header's default cursor
        if (jv && l == 0) gpre[j + 1] = fill / POD_PER_THREAD;
        const uint16_t* smax = S.n_specs <= (uint32_t)SPEC_LDS ? spec_max : nullptr;
        for (uint32_t i = t; i < S.n_specs && i < (uint32_t)SPEC_LDS; i += BLOCK) spec_max[i] = S.specs[i].max_len;
        uint32_t f[AG_STRIDE];
#pragma unroll
        for (int i = 0; i < AG_STRIDE; i++) f[i] = 0;
        // ---- nodes: needLockNode / configureNode (A.5), node flags for the pods -----
        uint32_t nmask = 0;
        for (uint32_t i0 = 0; i0 < nn; i0 += NODE_CHUNK) {
            const uint32_t i = i0 + t * NODE_PER_THREAD;
            uint32_t packed = 0;
#pragma unroll
            for (int c = 0; c < NODE_PRE; c++) packed = i0 == (uint32_t)c * NODE_CHUNK ? packed_pre[c] : packed;
            if (i0 >= (uint32_t)NODE_PRE * NODE_CHUNK && i < nn)
                packed = *reinterpret_cast<const uint32_t*>(S.node_state + nbase + i);
            uint32_t tick = 0;
            bool dirty = false;
#pragma unroll
            for (int k = 0; k < NODE_PER_THREAD; k++) {
                const uint8_t s = (uint8_t)(packed >> (8 * k));
                const NodeCls c = classify_node(s);
                f[AG_HB] += c.hb;
                f[AG_LOCK] += c.lock;
                f[AG_MANAGED] += c.managed;
                f[AG_READY] += c.ready;
                if (c.init) {
                    f[AG_INIT]++;
                    f[AG_INIT_BYTES] += (init_patch_len(S, S.node_blob[nbase + i + k]) + 15u) & ~15u;
                }
                dirty |= c.init || (s & NS_EVENT_LOCK);
                tick |= (uint32_t)node_tick_flags(s) << (8 * k);
            }
            if (i < nn) {
                nflags32[i / 4] = tick;
                if (!single || split) *reinterpret_cast<uint32_t*>(S.node_tick + nbase + i) = tick;
            }
            if (dirty) nmask |= 1u << (i0 / NODE_CHUNK);
        }
        __syncthreads();  // node flags, fill marks
        TSTAMP(8);
        if (t < 64) {     // gpre: live groups of the buckets before j; the block's largest bucket
            const uint32_t g = t < (int)nbk ? gpre[t + 1] : 0u;
            const uint32_t inc = wave_incl_scan(g);
            uint32_t mx = g;
            for (int o = 32; o; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
            gpre[t + 1] = inc;
            if (t == 0) gpre[0] = 0, sh_mask[3] = mx;
        }
        __syncthreads();
        TSTAMP(1);
        // ---- pods: the speculative groups, then any further rows (rare) ------------
        uint64_t pmask = 0;
        // heartbeat-once ticks: a wave whose speculative groups are all clean only counts them
        bool spec_clean = false;
        if (S.hb_once && !split) {
            bool rare = false;
            uint32_t ne = 0, nt = 0, npd = 0, nr = 0;
#pragma unroll
            for (int q = 0; q < SPEC_GROUPS; q++) {
                clip_group(G[q], jv && (l + q * tpb) * POD_PER_THREAD < fill);
                uint8_t nf[POD_PER_THREAD];
#pragma unroll
                for (int k = 0; k < POD_PER_THREAD; k++) nf[k] = group_node_flags(S, nflags, G[q], k);
                rare |= group_counts_fast(S, G[q], nf, ne, nt, npd, nr);
            }
            if (__builtin_expect(__ballot(rare) == 0, 1)) {
                f[AG_EVAL] += ne;
                f[AG_TOTAL] += nt;
                f[AG_PENDING] += npd;
                f[AG_RUNNING] += nr;
                spec_clean = true;
            }
        }
        if (!spec_clean) {
            // the groups' spec words and the `used` words of their Use candidates
            // (configurePod, pod_controller.go:378-382): one round trip for all of them
            uint4 spw[SPEC_GROUPS];
            UsedWords uw[SPEC_GROUPS];
#pragma unroll
            for (int q = 0; q < SPEC_GROUPS; q++) {
                const uint32_t a = l + q * tpb;
                clip_group(G[q], jv && a * POD_PER_THREAD < fill);
                const GroupMasks m = masks_of(S, nflags, G[q]);
                spw[q] = load_spec_words(S, G[q], m.need);
                load_group_ips(S, G[q], (m.usec | m.rel) != 0);
                uw[q] = used_words(S, G[q], m.usec);
            }
#pragma unroll
            for (int q = 0; q < SPEC_GROUPS; q++) {
                const uint32_t a = l + q * tpb;
                const GroupMasks m = masks_of(S, nflags, G[q]);
                const uint32_t gbytes = count_group(S, G[q], m, f, spw[q], smax);
                // emission chunks are runs of 256 live groups in slot order (gpre)
                if (m.dirty) pmask |= 1ull << ((gpre[j] + a) / BLOCK);
                if (split) wc_add(wcnt, gpre[j] + a, m, gbytes);
                if (split && S.sparse_jobs) gjob_put(S, b, gpre[j] + a, G[q], m, gbytes, tag);
                // single rank: into `used` now; multi rank: the Use list (the exchange message)
                apply_uses(S, G[q], m.usec & ~used_bits(S, G[q], m.usec, uw[q]));
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        const uint32_t maxg = sh_mask[3];
        auto row_slot = [&](uint32_t a) {
            return jv && a * POD_PER_THREAD < fill ? (bk0 + j) * S.cp + a * POD_PER_THREAD : ~0u;
        };
        const uint32_t once_iters = SPEC_GROUPS * tpb < maxg ? (maxg - SPEC_GROUPS * tpb + ROW_BATCH * tpb - 1) / (ROW_BATCH * tpb) : 0u;
        // (not on split ticks: rows with work to emit are most rows there, and a rare
        // row costs the lean loop's load plus two round trips of its own)
        if (once_iters && S.hb_once && !split && once_iters <= 64) {
            // heartbeat-once ticks (nothing to hide the chain under): ROW_BATCH rows per
            // iteration, their state and node words only, loaded one iteration ahead; a
            // batch with nothing but counts (every row of a quiet steady tick) is counted
            // from the state planes.  A batch with a delete, patch, Get, Put, Use or event
            // is noted and taken by the full path after the loop (the loop body stays
            // small: its registers hold the loads in flight, not the rare path's)
            auto lean = [&](uint32_t a, uint4& st, uint4& nd) {
                const uint32_t slot = row_slot(a);
                st = nd = make_uint4(0, 0, 0, 0);
                if (slot != ~0u) {
                    st = *reinterpret_cast<const uint4*>(S.pod_state + slot);
                    nd = *reinterpret_cast<const uint4*>(S.pod_node + slot);
                }
            };
            uint64_t rare_iters = 0;  // wave-uniform
            uint4 Ns[ROW_BATCH], Nn[ROW_BATCH];
#pragma unroll
            for (int r = 0; r < ROW_BATCH; r++) lean(l + SPEC_GROUPS * tpb + r * tpb, Ns[r], Nn[r]);
            uint32_t n_eval = 0, n_total = 0, n_pend = 0, n_run = 0;
            for (uint32_t it = 0; it < once_iters; it++) {
                uint4 Hs[ROW_BATCH], Hn[ROW_BATCH];
#pragma unroll
                for (int r = 0; r < ROW_BATCH; r++) Hs[r] = Ns[r], Hn[r] = Nn[r];
                const uint32_t an = SPEC_GROUPS * tpb + (it + 1) * ROW_BATCH * tpb;
#pragma unroll
                for (int r = 0; r < ROW_BATCH; r++) {
                    if (an < maxg) lean(l + an + r * tpb, Ns[r], Nn[r]);
                    else Ns[r] = Nn[r] = make_uint4(0, 0, 0, 0);
                }
                bool rare = false;
                uint32_t ce = 0, ct = 0, cpn = 0, cr = 0;
#pragma unroll
                for (int r = 0; r < ROW_BATCH; r++) {
                    PodGrp g;
                    g.slot = 0, g.j = j;
                    g.stw[0] = Hs[r].x, g.stw[1] = Hs[r].y, g.stw[2] = Hs[r].z, g.stw[3] = Hs[r].w;
                    g.ndw[0] = Hn[r].x, g.ndw[1] = Hn[r].y, g.ndw[2] = Hn[r].z, g.ndw[3] = Hn[r].w;
                    uint8_t nf[POD_PER_THREAD];
#pragma unroll
                    for (int k = 0; k < POD_PER_THREAD; k++) nf[k] = group_node_flags(S, nflags, g, k);
                    rare |= group_counts_fast(S, g, nf, ce, ct, cpn, cr);
                }
                if (__builtin_expect(__ballot(rare) == 0, 1)) n_eval += ce, n_total += ct, n_pend += cpn, n_run += cr;
                else rare_iters |= 1ull << it;
            }
            f[AG_EVAL] += n_eval;
            f[AG_TOTAL] += n_total;
            f[AG_PENDING] += n_pend;
            f[AG_RUNNING] += n_run;
            while (rare_iters) {
                const uint32_t it = (uint32_t)__builtin_ctzll(rare_iters);
                rare_iters &= rare_iters - 1;
                for (int r = 0; r < ROW_BATCH; r++) {
                    const uint32_t a = l + SPEC_GROUPS * tpb + it * ROW_BATCH * tpb + r * tpb;
                    PodGrp g;
                    load_group_at(S, a < maxg ? row_slot(a) : ~0u, j, g);
                    const GroupMasks m = masks_of(S, nflags, g);
                    const uint4 sw = load_spec_words(S, g, m.need);
                    const UsedWords u = used_words(S, g, m.usec);
                    const uint32_t gbytes = count_group(S, g, m, f, sw, smax);
                    if (m.dirty) pmask |= 1ull << ((gpre[j] + a) / BLOCK);
                    if (split) wc_add(wcnt, gpre[j] + a, m, gbytes);
                    if (split && S.sparse_jobs) gjob_put(S, b, gpre[j] + a, g, m, gbytes, tag);
                    apply_uses(S, g, m.usec & ~used_bits(S, g, m.usec, u));
                }
            }
        } else if (SPEC_GROUPS * tpb < maxg) {
            // one row per iteration, the next row's group loads in flight under this
            // row's spec / Use loads (one round trip per row, not two); the podIPs
            // only for a row with a Use or a release
            PodGrp H;
            load_group_at(S, row_slot(l + SPEC_GROUPS * tpb), j, H, false);
            for (uint32_t a0 = SPEC_GROUPS * tpb; a0 < maxg; a0 += tpb) {
                const uint32_t a = l + a0;
                const GroupMasks m = masks_of(S, nflags, H);
                PodGrp N;
                load_group_at(S, a0 + tpb < maxg ? row_slot(a + tpb) : ~0u, j, N, false);
                const uint4 sw = load_spec_words(S, H, m.need);
                load_group_ips(S, H, (m.usec | m.rel) != 0);
                const UsedWords u = used_words(S, H, m.usec);
                const uint32_t gbytes = count_group(S, H, m, f, sw, smax);
                if (m.dirty) pmask |= 1ull << ((gpre[j] + a) / BLOCK);
                if (split) wc_add(wcnt, gpre[j] + a, m, gbytes);
                if (split && S.sparse_jobs) gjob_put(S, b, gpre[j] + a, H, m, gbytes, tag);
                apply_uses(S, H, m.usec & ~used_bits(S, H, m.usec, u));
                H = N;
            }
        }
        TSTAMP(2);
        if (nmask) atomicOr(&sh_mask[2], nmask);
        if (pmask) {
            if ((uint32_t)pmask) atomicOr(&sh_mask[0], (uint32_t)pmask);
            if ((uint32_t)(pmask >> 32)) atomicOr(&sh_mask[1], (uint32_t)(pmask >> 32));
        }
        block_total<AG_STRIDE>(f);  // synchronises: the masks are complete
        TSTAMP(10);
        pod_mask = (uint64_t)sh_mask[0] | (uint64_t)sh_mask[1] << 32;
        node_mask = sh_mask[2];
        const bool dirty = (pod_mask | node_mask) != 0;
        my_init = f[AG_INIT];
        if (single) {
            // ---- single rank: field accumulators; no block waits for another --------
            // A dirty block first publishes its record (tagged with this tick) for the
            // emission prefix of the dirty blocks after it.
            f[AG_DIRTY] = dirty ? tag : 0u;
            if (dirty && t < AG_STRIDE / 2) {
                uint64_t w = 0;  // (selects, not f[2 * t]: a lane-indexed array would live in scratch)
#pragma unroll
                for (int i = 0; i < AG_STRIDE / 2; i++)
                    w = t == i ? ((uint64_t)f[2 * i] | (uint64_t)f[2 * i + 1] << 32) : w;
                st_sc1(reinterpret_cast<uint64_t*>(S.blockagg + (size_t)b * AG_STRIDE) + t, w);
            }
            uint32_t acc_v = 0;  // lane t < AG_DIRTY: this block's value of field t
#pragma unroll
            for (int i = 0; i < AG_DIRTY; i++) acc_v = t == i ? f[i] : acc_v;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            TSTAMP(11);
            // arrive (after this block's Uses and record): the dirty blocks count arrivals
            if (t == 0) __hip_atomic_fetch_add(&S.bar->arrive, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // lane t owns field t: one returning add of (one arrival | this block's
            // value); the block whose add completes the count holds the tick's total.
            // The adds queue behind each other (~2 us for 256 blocks): their results are
            // looked at only after this block's slice of the stream.
            unsigned long long acc_old = 0;
            const uint64_t c_arrive = __builtin_amdgcn_s_memrealtime();
            if (t < AG_DIRTY) acc_old = atomicAdd(&S.bar->acc[t][0], (1ull << ACC_SHIFT) | acc_v);
            TSTAMP(3);
            write_hb_handles(S, nflags32, nbase, nn, hb_base);
            TSTAMP(12);
            if (S.stream_share < 1024 && !(phases & TICK_NOSTREAM) && hb_share_any(S, hb_bodies(S, n_hb), b, S.n_chain)) {
                build_hb_template(S, hb_tmpl, now_unix, start_unix);  // (this block's slice of the stream)
                hb_fill_share<GEN_HB>(S, hb_tmpl4, hb_bodies(S, n_hb), false, b, S.n_chain);
            }
            TSTAMP(13);
            if (t < AG_DIRTY && (acc_old >> ACC_SHIFT) == S.n_chain - 1u) {
                const uint64_t total = (acc_old & ACC_MASK) + acc_v;
                st_sc1(&S.bar->acc[t][0], 0ull);  // the next tick starts from zero
                st_host(&S.hdr_host->tot[t], total);
                // for k_emit, which runs after this launch (a fused split tick: k_pod_jobs writes the bytes)
                if (t == AG_PP) S.emit_n[0] = ((phases & TICK_SPLIT) && S.fuse_pods) ? 0u : (uint32_t)total;
                if (t == AG_INIT) S.emit_n[1] = (uint32_t)total;
                if (t == AG_HB) {
                    if (total != n_hb)  // the heartbeat stream was laid out for the host's count
                        st_host(&S.hdr_host->err, TICK_ERR_LAYOUT);
                    st_host(&S.hdr_host->clk[CLK_P1_MAX], c_arrive);  // the last arrival
                    if (phases & TICK_PROF) {
                        st_host(&S.hdr_host->clk[CLK_ENTRY_MIN], ~ld_sc1(&S.bar->neg_entry_max));
                        st_sc1(&S.bar->neg_entry_max, 0ull);
                    }
                    TSTAMP(7);
                }
            }
            if (!dirty) {
                TSTAMP(6);
                return;
            }
            if (split && pod_mask) wc_publish(S, b, gpre[nbk], wcnt);  // (wait_arrivals synchronises)
            wait_arrivals(S, arrive_target);
            reduce_records(S, b, tag, recs, &sums);
            TSTAMP(4);
            have_sums = true;
        } else {
            // ---- multi rank: records; the last arriver writes the exchange message -----
            if (t == 0) {
                S.dmask[2 * b] = pod_mask;
                S.dmask[2 * b + 1] = node_mask;
            }
            f[AG_DIRTY] = dirty ? 1u : 0u;
            if (split && pod_mask) wc_publish(S, b, gpre[nbk], wcnt);  // for the BACK launch's k_pod_jobs
            const uint64_t old = publish_and_arrive(S, b, f);
            TSTAMP(3);
            if ((old + 1) % S.n_chain == 0) {
                const uint64_t c = __builtin_amdgcn_s_memrealtime();
                reduce_records(S, b, 0, recs, &sums);
                write_front_header(S, sums, n_hb, pool_index, c, (phases & TICK_PROF) != 0, tag);
                if (t < 2) S.emit_n[t] = 0u;  // set by BACK once it builds the jobs
                TSTAMP(7);
            }
            write_hb_handles(S, nflags32, nbase, nn, hb_base);
            if (S.stream_share < 1024 && !(phases & TICK_NOSTREAM) && hb_share_any(S, hb_bodies(S, n_hb), b, S.n_chain)) {
                build_hb_template(S, hb_tmpl, now_unix, start_unix);
                hb_fill_share<GEN_HB>(S, hb_tmpl4, hb_bodies(S, n_hb), false, b, S.n_chain);
            }
            return;  // the BACK launch follows the exchange
        }
    } else {
        // BACK launch (multi rank).  Every block folds the gathered exchange
        // messages (W of them): the fleet's Gets, this rank's first ordinal, Puts
        const XMsg* X = S.xall;
        uint64_t base = 0;
        uint32_t maxl = 0;
        bool step = true;
        for (int r = 0; r < S.world; r++) {
            const uint64_t al = X[r].alloc;
            xA += al;
            if (r < S.rank) base += al;
            xrel += X[r].n_rel;
            maxl = max(maxl, (uint32_t)(X[r].n_use + X[r].n_rel));
            step &= X[r].seq == tag;
        }
        if (!step && b == 0 && t == 0) st_host(&S.hdr_host->err, TICK_ERR_SEQ);  // ranks out of step: results void
        xbase = base;
        // TICK_XSPEC: the second allgather ran speculatively (the previous tick had long
        // lists) and k_pool_apply_spec applied every rank's lists if they fit
        const bool spec = (phases & TICK_XSPEC) && spec_fits(S);
        if (!(phases & TICK_XLISTS) && !spec) {
            if (maxl > (uint32_t)XINLINE) {
                // lists that did not fit inline: the host runs the second allgather,
                // applies them and launches BACK again (TICK_XLISTS)
                if (b == 0 && t == 0) {
                    st_host(&S.hdr_host->xovf, 1u);
                    // a tick already queued behind this one must not run before the
                    // host finishes this one (kwok_tick_submit): its launches skip
                    __hip_atomic_store(&S.bar->skip, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                return;
            }
            // every rank's Uses into `used`, every rank's Puts into rel_bm (folded in
            // the pool phase after all of them: Use -> Put), from the inline lists
            for (int r = 0; r < S.world; r++) {
                const uint32_t nu = (uint32_t)X[r].n_use, nl = nu + (uint32_t)X[r].n_rel;
                for (uint32_t i = b * BLOCK + t; i < nl; i += gridDim.x * BLOCK) {
                    const uint32_t ip = X[r].ips[i];
                    if (!in_cidr(S.pool, ip)) continue;
                    const uint64_t bit = ip - S.pool.net;
                    atomicOr((unsigned long long*)&(i < nu ? S.used_bm : S.rel_bm)[bit >> 6], 1ull << (bit & 63));
                }
            }
            if (xA || xrel) pool_barrier(S, gridDim.x);  // the pool phase reads every rank's bits
        }
        if (b == 0 && t < 2)  // this launch builds k_emit's jobs (a fused split tick: k_pod_jobs writes the pod bytes)
            S.emit_n[t] = t ? H->n_init : (((phases & TICK_SPLIT) && S.fuse_pods) ? 0u : H->n_pp);
        if (b == 0 && t < 16) {  // fleet counters
            uint64_t c = 0;
            for (int r = 0; r < S.world; r++) c += X[r].counters[t];
            H->counters[t] = c;
            if (t == 0) {
                H->alloc_total = xA;
                H->alloc_base = xbase;
                H->rel_total = xrel;
                uint32_t fx = 0;
                for (int r = 0; r < S.world; r++) fx |= X[r].foreign ? 1u : 0u;
                H->xforeign = fx;
                st_host(&S.hdr_host->xforeign, fx);
            }
        }
        // this block's masks from the FRONT launch (a pool-only block has none)
        if (t == 0) {
            const bool chain = b < S.n_chain;
            sh_mask[0] = chain ? (uint32_t)S.dmask[2 * b] : 0u;
            sh_mask[1] = chain ? (uint32_t)(S.dmask[2 * b] >> 32) : 0u;
            sh_mask[2] = chain ? (uint32_t)S.dmask[2 * b + 1] : 0u;
            if (b == 0) {
                H->clk[CLK_BACK] = __builtin_amdgcn_s_memrealtime();
                S.list_counts[0] = 0;  // exchange lists for the next tick
                S.list_counts[1] = 0;
            }
        }
        __syncthreads();
        pod_mask = (uint64_t)sh_mask[0] | (uint64_t)sh_mask[1] << 32;
        node_mask = sh_mask[2];
        my_init = b < S.n_chain ? S.blockagg[(size_t)b * AG_STRIDE + AG_INIT] : 0u;  // the FRONT launch's record
    }
    tick_back(S.self, TickLds{recs, nflags32, gpre, &sums, &sh_L}, b, bk0, nbk,
              pod_mask, node_mask, my_init, have_sums, phases, n_hb, now_unix, start_unix, xA, xrel, xbase, tag);
#undef TSTAMP
#undef TWAIT
}

// ---------------------------------------------------------------------------
// k_once: a heartbeat-once tick expected to have nothing to emit
// (KWOK_CFG_HEARTBEAT_ONCE, single rank, no events ingested since the previous
// tick, quiet Use checks) - the steady tick of the cgo drop-in.  Its work is
// k_tick's FRONT classification, counted: KeepNodeHeartbeat's handle list
// (node_controller.go:159-172), needLockNode / configureNode's predicate per node
// (:210-223, 356-391), needLockPod / configurePod / computePatchData's per pod
// (pod_controller.go:252-269, 371-439), and ONE heartbeat body (:393-401).
//
// One wave per bucket with every load of the bucket in flight at once: the node
// bytes, then the pod state rows (no chain of round trips).  The pods' node
// indices are read only when the bucket's node entries disagree on the re-lock
// flag: with every node of a bucket re-locked (or none), a pod's node cannot
// change its counts.  A wave that meets work to emit (a delete, patch, Get, Put,
// Use, pod event, node init or queued node lock) marks the tick: its last
// arriver then sets TickHdr::redo and GridBar::skip instead of completing it,
// and the host runs the tick again with k_tick (launches queued behind it skip
// and are enqueued again).  Counts go to per-XCD shards of packed accumulators
// (blocks are dealt to the 8 XCDs round robin); a shard's last arriver adds its
// totals to the fleet words, whose last arriver publishes them.  A completed
// tick adds n_chain to GridBar::arrive, as k_tick's chain blocks would have.
// ---------------------------------------------------------------------------
constexpr int ONCE_ROWS = 8;          // 64-group rows (512 pod slots) of a bucket a wave holds in registers
constexpr int ONCE_SPEC_ROWS = 4;     // rows loaded before the bucket's fill mark lands
constexpr int ONCE_NODE_WORDS = ONCE_NODE_LDS / 256;  // node-state words per lane
constexpr uint32_t ONCE_M27 = (1u << ONCE_FIELD_BITS) - 1u;

// the fleet total of packed word k (the last arriver of word k)
__device__ __forceinline__ void once_publish(const DevState& S, uint32_t k, uint64_t total, uint32_t n_hb, int phases,
                                             uint64_t c_arrive) {
    TickHdr* P = S.hdr_host;
    const uint64_t lo = total & ONCE_M27, hi = total >> ONCE_FIELD_BITS;
    switch (k) {
        case 0:
            st_host(&P->tot[AG_HB], lo);
            st_host(&P->tot[AG_LOCK], hi);
            if (lo != n_hb) st_host(&P->err, TICK_ERR_LAYOUT);  // the host's managed-node count
            st32_sc1(&S.emit_n[0], 0u);
            st32_sc1(&S.emit_n[1], 0u);
            st_host(&P->clk[CLK_P1_MAX], c_arrive);
            if (phases & TICK_PROF) {
                st_host(&P->clk[CLK_ENTRY_MIN], ~ld_sc1(&S.bar->neg_entry_max));
                st_sc1(&S.bar->neg_entry_max, 0ull);
            }
            break;
        case 1:
            st_host(&P->tot[AG_MANAGED], lo);
            st_host(&P->tot[AG_READY], hi);
            break;
        case 2:
            st_host(&P->tot[AG_EVAL], lo);
            st_host(&P->tot[AG_TOTAL], hi);
            break;
        case 3:
            st_host(&P->tot[AG_PENDING], lo);
            st_host(&P->tot[AG_RUNNING], hi);
            break;
        default:
            if (lo) {  // work to emit: the host finishes the tick with k_tick
                st32_sc1(&S.bar->skip, 1u);
                st_host(&P->redo, 1u);
            } else {   // the arrivals k_tick's chain blocks would have made (GridBar::arrive is cumulative)
                __hip_atomic_fetch_add(&S.bar->arrive, (unsigned long long)S.n_chain, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
    }
}

// one 8-slot group of a k_once bucket: group_counts_fast's planes for a quiet
// tick (Use checks of pods with an event only: such a pod is evaluated, which
// is work to emit anyway), counted as if nothing were rare - a rare group voids
// the tick (it runs again with k_tick).  rl: the pods' RELOCK flags as two-pod
// planes (bit 0 / bit 16 of each word).  Returns whether anything is rare.
template <bool CNI>
__device__ __forceinline__ uint32_t once_group(const uint32_t (&stw)[4], const uint32_t (&rl)[4], uint32_t& n_eval,
                                               uint32_t& n_total, uint32_t& n_pend, uint32_t& n_run) {
    constexpr uint32_t M = 0x00010001u;
    uint32_t rare = 0, pe = 0, pt = 0, pp = 0, pr = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const uint32_t s = stw[w];
        const uint32_t s1 = s >> 1, s2 = s >> 2, s5 = s >> 5, s6 = s >> 6, s7 = s >> 7;
        const uint32_t s8 = s >> 8, s9 = s >> 9, s10 = s >> 10, s11 = s >> 11;
        const uint32_t live = s & ~s2;                       // USED, not DELETE_PENDING
        const uint32_t eval = live & (s6 | (rl[w] & ~s1));  // EVENT, or RELOCK & !DISREGARD
        const uint32_t running = s9 & ~(s8 | s10), pending = s8 & ~(s9 | s10);
        const uint32_t ok = running & s5 & s7;               // Running, CONFORMS, HAS_HOST_IP
        // computePatchData's patch (a Get with it when the podIP is empty); EnableCNI: only once it has one
        const uint32_t need = CNI ? eval & ~ok & s11 : eval & ~(ok & s11);
        rare |= (s & s2) | need | (eval & s6);               // a delete, a patch, an event
        pe += eval & M, pt += live & M, pp += live & pending & M, pr += live & running & M;
    }
    n_eval += (pe & 0xFFFFu) + (pe >> 16);
    n_total += (pt & 0xFFFFu) + (pt >> 16);
    n_pend += (pp & 0xFFFFu) + (pp >> 16);
    n_run += (pr & 0xFFFFu) + (pr >> 16);
    return rare & M;
}

// once_group for a summary (ONCE_SUM_BUILD): the group under both uniform RELOCK
// flags (every pod's node re-locked, none), for a bucket whose node entries agree
template <bool CNI>
__device__ __forceinline__ void once_group_both(const uint32_t (&stw)[4], uint32_t& ev0, uint32_t& ev1, uint32_t& rare0,
                                                uint32_t& rare1) {
    constexpr uint32_t M = 0x00010001u;
    uint32_t r0 = 0, r1 = 0, e0 = 0, e1 = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const uint32_t s = stw[w];
        const uint32_t s1 = s >> 1, s2 = s >> 2, s5 = s >> 5, s6 = s >> 6, s7 = s >> 7;
        const uint32_t s8 = s >> 8, s9 = s >> 9, s10 = s >> 10, s11 = s >> 11;
        const uint32_t live = s & ~s2;
        const uint32_t a = live & s6, b = live & (s6 | ~s1);  // eval without / with RELOCK
        const uint32_t running = s9 & ~(s8 | s10);
        const uint32_t ok = running & s5 & s7;
        const uint32_t na = CNI ? a & ~ok & s11 : a & ~(ok & s11), nb = CNI ? b & ~ok & s11 : b & ~(ok & s11);
        const uint32_t base = (s & s2) | (a & s6);  // (eval & EVENT is the same under both flags)
        r0 |= base | na, r1 |= base | nb;
        e0 += a & M, e1 += b & M;
    }
    ev0 += (e0 & 0xFFFFu) + (e0 >> 16);
    ev1 += (e1 & 0xFFFFu) + (e1 >> 16);
    rare0 |= r0 & M, rare1 |= r1 & M;
}

// Per-bucket summaries (ONCE_SUM_*): a steady fleet's pod states do not change
// between heartbeat-once ticks that emit nothing, and a pod's counts depend on
// its node only through the RELOCK flag - uniform over a bucket whose node
// entries agree.  A BUILD tick reads every pod state row as usual and also writes
// each bucket's counts under both uniform flags (uint4: eval | eval-with-RELOCK,
// total | pending, running | rare bits, generation).  A USE tick, enqueued only
// while no ingest, CNI assignment, pool Put or k_tick has run since the BUILD
// (the host's DevState::once_sum validity), reads the node words and the 16-byte
// summary instead of the pod rows; a bucket whose nodes disagree on RELOCK, or
// whose summary is of another generation, is read in full.
template <bool CNI, uint32_t SUM>  // SUM: ONCE_SUM_OFF / _BUILD / _USE (each its own registers)
__global__ __launch_bounds__(64 * ONCE_WAVES, 2) void k_once(DevState S, uint64_t now_unix, uint64_t start_unix,
                                                            uint32_t n_hb, int phases, uint32_t gen) {
    __shared__ uint32_t nfl32[ONCE_WAVES][ONCE_NODE_LDS / 4];  // the bucket's node tick flags, per wave
    __shared__ uint64_t part[ONCE_WAVES][ONCE_ACC_WORDS];
    __shared__ uint8_t tmpl[16 * HB_MAX_UNITS];
    const uint32_t t = threadIdx.x, l = t & 63u, w = (uint32_t)wave_id(), b = blockIdx.x;
    if (ld32_sc1(&S.bar->skip)) return;  // queued behind a tick the host must finish (re-enqueued then)
    const bool stamp = S.trace && t == 0 && b < S.n_chain;
#define OSTAMP(k) \
    if (stamp) S.trace[(size_t)b * TRACE_SLOTS + (k)] = __builtin_amdgcn_s_memrealtime()
    OSTAMP(0);
    // profiled ticks: the earliest start, from the first block of each XCD (512 adds to one
    // word would serialise ~6 us into the kernel)
    if ((phases & TICK_PROF) && t == 0 && b < 8u)
        atomicMax(&S.bar->neg_entry_max, ~(unsigned long long)__builtin_amdgcn_s_memrealtime());
    const uint32_t bk = b * ONCE_WAVES + w;
    uint32_t hb = 0, lock = 0, mng = 0, rdy = 0, ev = 0, tot = 0, pnd = 0, run = 0, rare = 0;
    uint32_t be0 = 0, be1 = 0, br0 = 0, br1 = 0;  // SUM == ONCE_SUM_BUILD: eval / rare under both uniform flags
    if (bk < S.nb) {  // (wave-uniform)
        const uint32_t cn = S.cn, cp = S.cp;
        const uint32_t fill = min((uint32_t)S.pod_fill[bk], cp);
        // ---- every load of the bucket: node bytes first (classified first), pod state rows
        const uint8_t* nst = S.node_state + (size_t)bk * cn;
        uint32_t nw[ONCE_NODE_WORDS];
#pragma unroll
        for (int c = 0; c < ONCE_NODE_WORDS; c++) {
            const uint32_t i = 4u * (l + 64u * c);
            nw[c] = 0;
            if (256u * c < cn && i < cn) nw[c] = *reinterpret_cast<const uint32_t*>(nst + i);
        }
        const uint16_t* pst = S.pod_state + (size_t)bk * cp;
        constexpr bool use = SUM == ONCE_SUM_USE;
        uint4 sm = make_uint4(0, 0, 0, 0), st[ONCE_ROWS];
        if (use) sm = S.once_sum[bk];  // (one address: one request)
#pragma unroll
        for (int r = 0; r < ONCE_ROWS; r++) {
            const uint32_t g8 = 8u * (l + 64u * r);
            st[r] = make_uint4(0, 0, 0, 0);
            if (!use && g8 < (r < ONCE_SPEC_ROWS ? cp : fill)) st[r] = *reinterpret_cast<const uint4*>(pst + g8);
        }
        // ---- nodes: LockNode / configureNode (A.5), heartbeat handles, re-lock flags
        uint32_t or0 = 0, and0 = 1, has = 0, base = S.hb_bpre[bk];
#pragma unroll
        for (int c = 0; c < ONCE_NODE_WORDS; c++) {
            if (256u * c < cn) {  // (uniform)
                const uint32_t word = nw[c], i0 = 4u * (l + 64u * c);
                uint32_t tickw = 0, m = 0;
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint8_t s = (uint8_t)(word >> (8 * k));
                    const NodeCls nc = classify_node(s);
                    hb += nc.hb;
                    lock += nc.lock;
                    mng += nc.managed;
                    rdy += nc.ready;
                    rare |= (nc.init || (s & NS_EVENT_LOCK)) ? 1u : 0u;
                    const uint32_t f = node_tick_flags(s);
                    tickw |= f << (8 * k);
                    if (s) or0 |= f & 1u, and0 &= f & 1u, has = 1;
                    m += (uint32_t)nc.managed << k;
                }
                if (i0 < cn) nfl32[w][l + 64u * c] = tickw;
                // KeepNodeHeartbeat's handles, node order: the wave's managed nodes of this word
                const uint32_t cnt = (uint32_t)__popc(m), inc = wave_incl_scan(cnt);
                uint32_t pos = base + inc - cnt;
                for (uint32_t mm = m; mm; mm &= mm - 1) {
                    if (pos < S.n_node_slots)
                        S.hb_nodes[pos] = S.node_handle_base + (int32_t)((size_t)bk * cn + i0 + (uint32_t)__builtin_ctz(mm));
                    pos++;
                }
                base += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
            }
        }
        // a pod's node matters only if the bucket's node entries disagree on RELOCK
        const bool any_set = __ballot(has && or0) != 0, any_clr = __ballot(has && !and0) != 0;
        const bool uni = !(any_set && any_clr);
        const uint8_t u = any_set ? (uint8_t)NT_RELOCK : (uint8_t)0;
        OSTAMP(8);
        const uint16_t* pnd_ = S.pod_node + (size_t)bk * cp;
        // ---- pods: needLockPod / computePatchData, counted (once_group)
        auto count_row = [&](uint32_t g8, const uint4& s4, const uint32_t (&rl)[4]) {
            const bool in = g8 < fill;
            const uint32_t stw[4] = {in ? s4.x : 0u, in ? s4.y : 0u, in ? s4.z : 0u, in ? s4.w : 0u};
            rare |= once_group<CNI>(stw, rl, ev, tot, pnd, run);
            if constexpr (SUM == ONCE_SUM_BUILD) once_group_both<CNI>(stw, be0, be1, br0, br1);
        };
        auto lds_flags = [&](const uint4& n4, uint32_t (&rl)[4]) {
            const uint8_t* nfw = reinterpret_cast<const uint8_t*>(nfl32[w]);
            const uint32_t q[4] = {n4.x, n4.y, n4.z, n4.w};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t a = nfw[min(q[k] & 0xFFFFu, (uint32_t)ONCE_NODE_LDS - 1u)];
                const uint32_t c = nfw[min(q[k] >> 16, (uint32_t)ONCE_NODE_LDS - 1u)];
                rl[k] = a | c << 16;  // (NT_RELOCK is bit 0)
            }
        };
        if (use && uni && sm.w == gen) {  // the bucket's summary (lane 0's counts; rare from any lane)
            if (l == 0) {
                ev += u ? sm.x >> 16 : sm.x & 0xFFFFu;
                tot += sm.y & 0xFFFFu, pnd += sm.y >> 16, run += sm.z & 0xFFFFu;
            }
            rare |= (sm.z >> (u ? 17 : 16)) & 1u;
        } else if (uni) {
            if (use) {  // (another generation: the rows now)
#pragma unroll
                for (int r = 0; r < ONCE_ROWS; r++) {
                    const uint32_t g8 = 8u * (l + 64u * r);
                    if (g8 < fill) st[r] = *reinterpret_cast<const uint4*>(pst + g8);
                }
            }
            const uint32_t p = u ? 0x00010001u : 0u;
            const uint32_t rl[4] = {p, p, p, p};
#pragma unroll
            for (int r = 0; r < ONCE_ROWS; r++) count_row(8u * (l + 64u * r), st[r], rl);
            for (uint32_t r = ONCE_ROWS; 512u * r < fill; r++) {  // buckets of more than 4096 pod slots
                const uint32_t g8 = 8u * (l + 64u * r);
                const uint4 s4 = g8 < fill ? *reinterpret_cast<const uint4*>(pst + g8) : make_uint4(0, 0, 0, 0);
                count_row(g8, s4, rl);
            }
        } else {
            uint4 nd[ONCE_ROWS];
#pragma unroll
            for (int r = 0; r < ONCE_ROWS; r++) {
                const uint32_t g8 = 8u * (l + 64u * r);
                nd[r] = g8 < fill ? *reinterpret_cast<const uint4*>(pnd_ + g8) : make_uint4(0, 0, 0, 0);
                if (use && g8 < fill) st[r] = *reinterpret_cast<const uint4*>(pst + g8);
            }
            __builtin_amdgcn_wave_barrier();  // (the wave's node flags are in LDS)
#pragma unroll
            for (int r = 0; r < ONCE_ROWS; r++) {
                uint32_t rl[4];
                lds_flags(nd[r], rl);
                count_row(8u * (l + 64u * r), st[r], rl);
            }
            for (uint32_t r = ONCE_ROWS; 512u * r < fill; r++) {
                const uint32_t g8 = 8u * (l + 64u * r);
                uint4 s4 = make_uint4(0, 0, 0, 0), n4 = s4;
                if (g8 < fill) {
                    s4 = *reinterpret_cast<const uint4*>(pst + g8);
                    n4 = *reinterpret_cast<const uint4*>(pnd_ + g8);
                }
                uint32_t rl[4];
                lds_flags(n4, rl);
                count_row(g8, s4, rl);
            }
        }
        OSTAMP(2);
    }
    // ---- counts: wave -> block -> XCD shard -> fleet
    auto wsum = [](uint32_t x) { return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan(x), 63); };
    {
        const uint64_t v0 = wsum(hb) | wsum(lock) << ONCE_FIELD_BITS, v1 = wsum(mng) | wsum(rdy) << ONCE_FIELD_BITS;
        const uint64_t v2 = wsum(ev) | wsum(tot) << ONCE_FIELD_BITS, v3 = wsum(pnd) | wsum(run) << ONCE_FIELD_BITS;
        const uint64_t v4 = __ballot(rare != 0) ? 1u : 0u;
        if (l == 0) part[w][0] = v0, part[w][1] = v1, part[w][2] = v2, part[w][3] = v3, part[w][4] = v4;
        if constexpr (SUM == ONCE_SUM_BUILD) {  // the bucket's summary (one wave = one bucket)
            const uint32_t E0 = (uint32_t)wsum(be0), E1 = (uint32_t)wsum(be1);
            const uint32_t k0 = __ballot(br0 != 0) ? 1u : 0u, k1 = __ballot(br1 != 0) ? 1u : 0u;
            if (l == 0 && bk < S.nb)
                S.once_sum[bk] = make_uint4(E0 | E1 << 16, (uint32_t)(v2 >> ONCE_FIELD_BITS) | (uint32_t)(v3 & ONCE_M27) << 16,
                                            (uint32_t)(v3 >> ONCE_FIELD_BITS) | k0 << 16 | k1 << 17, gen);
        }
    }
    __syncthreads();
    if (t < (uint32_t)ONCE_ACC_WORDS) {
        uint64_t v = 0;
#pragma unroll
        for (int i = 0; i < ONCE_WAVES; i++) v += part[i][t];
        const uint32_t G = gridDim.x, x = b & 7u, nsh = min(G, 8u), nx = (G - x + 7u) / 8u;
        const unsigned long long old = atomicAdd(&S.bar->once_acc[x][t][0], (1ull << ACC_SHIFT) | v);
        if ((old >> ACC_SHIFT) == nx - 1u) {  // the shard is complete
            const uint64_t sx = (old & ACC_MASK) + v;
            st_sc1(&S.bar->once_acc[x][t][0], 0ull);  // the next tick starts from zero
            const unsigned long long o2 = atomicAdd(&S.bar->once_acc[8][t][0], (1ull << ACC_SHIFT) | sx);
            if ((o2 >> ACC_SHIFT) == nsh - 1u) {
                st_sc1(&S.bar->once_acc[8][t][0], 0ull);
                once_publish(S, t, (o2 & ACC_MASK) + sx, n_hb, phases, __builtin_amdgcn_s_memrealtime());
            }
        }
    }
    OSTAMP(3);
    // ---- the one heartbeat body (hb_bodies), arena offset 0
    if (b == 0 && n_hb) {
        const Ts nw = format_ts(now_unix), sw = format_ts(start_unix);
        const uint32_t nb16 = 16u * S.hb_units;
        for (uint32_t i = t; i < nb16; i += 64u * ONCE_WAVES) {
            const uint8_t k = S.hb_kind[i];
            tmpl[i] = (uint8_t)(k == 0xFF ? S.hb_static[i] : k < TS_LEN ? ts_byte(nw, k) : ts_byte(sw, k - TS_LEN));
        }
        __syncthreads();
        for (uint32_t i = t; i < S.hb_units; i += 64u * ONCE_WAVES)
            reinterpret_cast<uint4*>(S.arena)[i] = reinterpret_cast<const uint4*>(tmpl)[i];
    }
    OSTAMP(6);
#undef OSTAMP
}

uint32_t once_blocks(const DevState& S) { return (S.nb + ONCE_WAVES - 1) / ONCE_WAVES; }

void launch_tick_once(const DevState& S, uint64_t now, uint64_t start, uint32_t n_hb, int phases, uint32_t sum_mode,
                      uint32_t gen, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
    const uint32_t grid = once_blocks(S);
    decltype(&k_once<false, ONCE_SUM_OFF>) kern;
    if (sum_mode == ONCE_SUM_BUILD) kern = S.cni ? k_once<true, ONCE_SUM_BUILD> : k_once<false, ONCE_SUM_BUILD>;
    else if (sum_mode == ONCE_SUM_USE) kern = S.cni ? k_once<true, ONCE_SUM_USE> : k_once<false, ONCE_SUM_USE>;
    else kern = S.cni ? k_once<true, ONCE_SUM_OFF> : k_once<false, ONCE_SUM_OFF>;
    if (t0)
        hipExtLaunchKernelGGL(kern, dim3(grid), dim3(64 * ONCE_WAVES), 0, st, t0, t1, 0, S, now, start, n_hb, phases, gen);
    else hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * ONCE_WAVES), 0, st, S, now, start, n_hb, phases, gen);
}

// ---------------------------------------------------------------------------
// k_pod_jobs: the pod emission of a split tick (TICK_SPLIT), launched after its
// k_tick launch(es).  In a chain block the pod chunks are a serial walk (one
// wave per SIMD, ~9 us of mostly fixed latency per 2048-pod chunk); here every
// dirty 64-group run of every chain block is one independent wave: its first
// ordinals / byte offset are the block's JobBase plus the run's in-block prefix
// (both from k_tick), its node flags the FRONT's node_tick bytes, and the run's
// deletes, job records and state transitions are exactly what the chain block
// would have written (emit_pod_chunks<1, true>, canonical order).
// pod_controller.go:155-183 (DeletePods), 404-439 (configurePod / patch jobs).
// ---------------------------------------------------------------------------
constexpr int JOB_WAVES = 4;
// KWOK_JOBS_TRACE diagnostics: per item (entry, emission start, exit, hw ids | jobs << 32)
__device__ __forceinline__ void jstamp(const DevState& S, uint32_t item, int k, uint64_t v) {
    if (S.jtrace && lane_id() == 0) S.jtrace[(size_t)item * 4 + k] = v;
}
constexpr int JOB_NC = 2;  // consecutive runs per wave, their loads and scans interleaved
constexpr int JOB_NF_BYTES = 768;  // node flags staged per wave (two buckets of ~350 node slots)
// One wave's runs c0 .. c0 + NC - 1 of chain block b (item: the trace slot)
template <bool FUSE>
__device__ __forceinline__ void pod_jobs_item(const DevState& S, uint32_t tag, uint32_t b, uint32_t c0, uint32_t item,
                                              uint32_t* stage, uint32_t* gpre, uint32_t* nf) {
    constexpr int NC = FUSE ? 1 : JOB_NC;  // fused: one run per wave (its emission holds the registers)
    jstamp(S, item, 0, __builtin_amdgcn_s_memrealtime());
    if (b >= S.n_chain || c0 >= (uint32_t)MAX_WC) return;
    // every input of the wave's setup in one round trip: the block's JobBase, the
    // runs' dirty bits and prefix, the fill marks of the block's buckets
    const JobBase* JB = S.jbase + b;
    const uint32_t jtag = JB->tag;
    const uint32_t dirty = (S.wc_dirty[(size_t)b * WC_DIRTY_WORDS + (c0 >> 5)] >> (c0 & 31)) & (NC == 2 ? 3u : 1u);
    const uint4 wp = S.wc_pre[(size_t)b * MAX_WC + c0];
    uint32_t bk0, nbk;
    block_range(S, b, bk0, nbk);
    const int l = lane_id();
    const uint32_t fill = l < (int)nbk ? (uint32_t)S.pod_fill[bk0 + l] : 0u;
    Bases run;
    run.v[AG_INIT] = run.v[AG_INIT_BYTES] = 0;
    run.v[AG_DEL] = JB->del;
    run.v[AG_PP] = JB->pp;
    run.v[AG_PP_BYTES] = JB->pp_bytes;
    run.v[AG_ALLOC] = JB->alloc;
    Layout L;
    L.init_base = 0;
    L.pod_base = JB->pod_base;
    L.alloc_base = JB->alloc_base;
    L.plan = PoolPlan{0, 0, JB->take, JB->fin, 0, JB->fout0};
    if (jtag != tag || !dirty) return;  // the block has no pod jobs this tick / the runs are clean
    run.v[AG_DEL] += wp.x;
    run.v[AG_PP] += wp.y;
    run.v[AG_PP_BYTES] += wp.z;
    run.v[AG_ALLOC] += wp.w;
    const uint32_t inc = wave_incl_scan(fill >> 3);
    gpre[l + 1] = inc;
    if (l == 0) gpre[0] = 0;
    const uint32_t ng = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    __builtin_amdgcn_wave_barrier();  // (one wave's LDS operations complete in order)
    // the node tick flags of the buckets the two runs span, into LDS with coalesced
    // loads (the groups then read them there, not with eight byte loads each)
    const uint8_t* nflags = S.node_tick + (size_t)bk0 * S.cn;
    uint32_t nj0 = 0;
    if (c0 * WC_GROUPS < ng) {
        const uint32_t ja = find_bucket(gpre, nbk, c0 * WC_GROUPS);
        const uint32_t jb = find_bucket(gpre, nbk, min((c0 + NC) * WC_GROUPS, ng) - 1u);
        const uint32_t nwords = (jb - ja + 1u) * S.cn / 4u;  // (cn % 4 == 0)
        if (nwords * 4u <= (uint32_t)JOB_NF_BYTES) {
            const uint32_t* src = reinterpret_cast<const uint32_t*>(nflags + (size_t)ja * S.cn);
            for (uint32_t v = (uint32_t)l; v < nwords; v += 64) nf[v] = src[v];
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            nflags = reinterpret_cast<const uint8_t*>(nf);
            nj0 = ja;
        }
    }
    // both runs (a clean one has nothing to count or emit, so the second run's
    // bases follow from the first's totals either way)
    uint32_t gx[NC];
#pragma unroll
    for (int i = 0; i < NC; i++) gx[i] = (c0 + i) * WC_GROUPS + (uint32_t)l;
    emit_pod_chunks<NC, true, FUSE>(S, gpre, nflags, bk0, nbk, ng, gx, run, L, stage, nj0, item);
    jstamp(S, item, 2, __builtin_amdgcn_s_memrealtime());
}
// One rank's Use or release list ORed into a bitmap, OR_RUN consecutive entries
// per thread: entries that fall in one bitmap word one after the other (a
// rank's lists follow canonical order, and addresses were handed out lowest
// first in that order, so neighbours usually share a word) take ONE atomic
// together.  A list in no order costs what one atomic per entry costs.
// (chunk c covers entries [c * OR_RUN, +OR_RUN) of a; out-of-CIDR entries skipped)
constexpr uint32_t OR_RUN = 16;
__device__ __forceinline__ void or_run(const PoolGeom& g, uint64_t* bm, const uint32_t* a, uint32_t n, uint32_t c) {
    const uint32_t s0 = c * OR_RUN, e = min(s0 + OR_RUN, n);
    uint32_t ip[OR_RUN];
#pragma unroll
    for (uint32_t k = 0; k < OR_RUN; k++) ip[k] = s0 + k < e ? a[s0 + k] : 0u;  // (loads in flight together)
    uint64_t m = 0, w = ~0ull;
#pragma unroll
    for (uint32_t k = 0; k < OR_RUN; k++) {
        if (s0 + k >= e || !in_cidr(g, ip[k])) continue;
        const uint64_t bit = ip[k] - g.net;
        if ((bit >> 6) != w) {
            if (m) atomicOr((unsigned long long*)&bm[w], m);
            w = bit >> 6, m = 0;
        }
        m |= 1ull << (bit & 63);
    }
    if (m) atomicOr((unsigned long long*)&bm[w], m);
}
// every rank's Uses into used_bm and releases into rel_bm: chunks of OR_RUN
// entries over all ranks' lists (rank-major; each rank's Use chunks, then its
// release chunks), the grid striding over the chunks
template <class ListOf>
__device__ __forceinline__ void or_lists(const DevState& S, int nranks, ListOf list) {
    const uint32_t stride = gridDim.x * blockDim.x;
    uint32_t c0 = 0;  // the chunks of the ranks before r
    for (int r = 0; r < nranks; r++) {
        const uint32_t* u, * rl;
        uint32_t nu, nr;
        list(r, u, nu, rl, nr);
        const uint32_t cu = (nu + OR_RUN - 1) / OR_RUN, cr = (nr + OR_RUN - 1) / OR_RUN;
        // this thread's first chunk at or after c0
        const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
        const uint32_t first = c0 + (t + stride - c0 % stride) % stride;
        for (uint32_t c = first; c < c0 + cu + cr; c += stride) {
            if (c - c0 < cu) or_run(S.pool, S.used_bm, u, nu, c - c0);
            else or_run(S.pool, S.rel_bm, rl, nr, c - c0 - cu);
        }
        c0 += cu + cr;
    }
}

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
// EnableCNI: the pods the next tick evaluates (the eval predicate of
// classify_pod over the current node states) that hold no podIP
__global__ void k_cni_pending(DevState S, int32_t* out, uint32_t* count) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < S.n_pod_slots; i += gridDim.x * blockDim.x) {
        const uint16_t st = S.pod_state[i];
        if (!(st & PS_USED)) continue;
        const uint32_t b = i / S.cp;
        const uint8_t ntf = node_tick_flags(S.node_state[(size_t)b * S.cn + S.pod_node[i]]);
        const PodCls c = classify_pod(st, ntf, S.pod_ip[i], true);
        if (c.eval && S.pod_ip[i] == 0) out[atomicAdd(count, 1u)] = pod_handle_of(S, i);
    }
}
// multi-rank: every rank's Uses into used_bm, every rank's Puts into rel_bm
__global__ void k_pool_apply(DevState S, const ListDesc* ld, int nranks) {
    or_lists(S, nranks, [&](int r, const uint32_t*& u, uint32_t& nu, const uint32_t*& rl, uint32_t& nr) {
        const ListDesc d = ld[r];
        u = d.use, nu = d.n_use, rl = d.rel, nr = d.n_rel;
    });
}

// KWOK_EMULATE_RANKS (diagnostics, one rank): messages 1..xw-1 are copies of
// this rank's message 0, their inline addresses moved by r * size / xw inside the
// CIDR, so BACK folds and applies xw ranks' worth of Gets, Uses and Puts
__device__ __forceinline__ uint32_t emul_shift(const PoolGeom& g, uint32_t ip, uint32_t r, uint32_t xw) {
    if (!in_cidr(g, ip)) return ip;
    uint64_t v = (uint64_t)(ip - g.net) + (g.size / xw) * r;  // < 2 * size (r < xw)
    if (v >= g.size) v -= g.size;
    return g.net + (uint32_t)v;
}
__global__ void k_emulate_msgs(DevState S, XMsg* X, uint32_t xw) {
    const uint32_t r = blockIdx.x + 1;
    if (r >= xw) return;
    const XMsg& m = X[0];
    XMsg& o = X[r];
    const uint32_t nl = (uint32_t)min<uint64_t>(m.n_use + m.n_rel, (uint64_t)XINLINE);
    for (uint32_t i = threadIdx.x; i < nl; i += blockDim.x) o.ips[i] = emul_shift(S.pool, m.ips[i], r, xw);
    if (threadIdx.x == 0) {
        o.alloc = m.alloc, o.n_use = m.n_use, o.n_rel = m.n_rel, o.seq = m.seq, o.foreign = m.foreign;
        for (int k = 0; k < 16; k++) o.counters[k] = m.counters[k];
    }
}
// ... and their long lists: slot 0 of each rank-major list block copied, moved
// (grid.y = the synthetic rank, r - 1)
__global__ void k_emulate_lists(DevState S, uint32_t* recv, uint64_t maxl, uint32_t xw, uint32_t n) {
    const uint32_t r = blockIdx.y + 1;
    uint32_t* dst = recv + r * maxl;
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
        dst[k] = emul_shift(S.pool, recv[k], r, xw);
}

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
    uint16_t st = (uint16_t)((S.pod_state[o.slot] & o.keep_mask) | o.bits);
    if (o.set_fields) st = (uint16_t)((st & ~PS_IP_BITS) | ip_state_bits(S.pool, o.pod_ip));
    S.pod_state[o.slot] = st;
    if (o.set_fields == 1) {  // add / modify carry the whole decoded object
        S.pod_node[o.slot] = o.node;
        S.pod_spec[o.slot] = o.spec;
        S.pod_ctime[o.slot] = o.ctime;
        S.host_ip[o.slot] = o.host_ip;
        S.pod_ip[o.slot] = o.pod_ip;
    } else if (o.set_fields == 2) {  // kwok_cni_assign: the podIP cni.Setup returned
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

void launch_cni_pending(const DevState& S, int32_t* out, uint32_t* count, hipStream_t st) {
    uint32_t g = cdiv(S.n_pod_slots, 256);
    if (g > 4096) g = 4096;
    hipLaunchKernelGGL(k_cni_pending, dim3(g ? g : 1), dim3(256), 0, st, S, out, count);
}

void launch_emulate_msgs(const DevState& S, XMsg* X, uint32_t xw, hipStream_t st) {
    if (xw > 1) hipLaunchKernelGGL(k_emulate_msgs, dim3(xw - 1), dim3(256), 0, st, S, X, xw);
}
void launch_emulate_lists(const DevState& S, uint32_t* recv, uint64_t maxl, uint32_t xw, uint32_t n, hipStream_t st) {
    if (xw > 1 && n) hipLaunchKernelGGL(k_emulate_lists, dim3(std::min<uint32_t>(cdiv(n, 256), 512), xw - 1), dim3(256), 0, st, S,
                                        recv, maxl, xw, n);
}
// one block per chain block: its Use and release segments to their place in dst
// (every block's Uses, then every block's releases, in block order)
__global__ void k_gather_lists(DevState S, uint32_t* dst, uint32_t rel_at, uint32_t cap_u, uint32_t cap_r) {
    const uint32_t b = blockIdx.x;
    __shared__ uint32_t pre[4];  // Uses / releases of the blocks before b, all Uses
    if (threadIdx.x < 4) pre[threadIdx.x] = 0;
    __syncthreads();
    uint32_t pu = 0, pr = 0, tu = 0;
    for (uint32_t q = threadIdx.x; q < S.n_chain; q += blockDim.x) {
        const uint32_t cu = S.list_blk[2 * q], cr = S.list_blk[2 * q + 1];
        tu += cu;
        if (q < b) pu += cu, pr += cr;
    }
    if (pu) atomicAdd(&pre[0], pu);
    if (pr) atomicAdd(&pre[1], pr);
    if (tu) atomicAdd(&pre[2], tu);
    __syncthreads();
    const uint32_t cu = S.list_blk[2 * b], cr = S.list_blk[2 * b + 1];
    uint32_t bk0, nbk;
    block_range(S, b, bk0, nbk);
    const uint32_t seg = bk0 * S.cp;
    const uint32_t r0 = rel_at == ~0u ? pre[2] : rel_at;
    for (uint32_t j = threadIdx.x; j < cu && pre[0] + j < cap_u; j += blockDim.x) dst[pre[0] + j] = S.use_list[seg + j];
    for (uint32_t j = threadIdx.x; j < cr && pre[1] + j < cap_r; j += blockDim.x) dst[r0 + pre[1] + j] = S.rel_list[seg + j];
}
void launch_gather_lists(const DevState& S, uint32_t* dst, hipStream_t st, uint32_t rel_at, uint32_t cap_u,
                         uint32_t cap_r) {
    hipLaunchKernelGGL(k_gather_lists, dim3(S.n_chain), dim3(256), 0, st, S, dst, rel_at, cap_u, cap_r);
}
__global__ void k_pool_apply_spec(DevState S, const uint32_t* recv) {
    // a tick skipped behind one the host finishes (GridBar::skip): its FRONT did not run
    if (__hip_atomic_load(&S.bar->skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
    if (!spec_fits(S)) return;  // BACK takes the long-list way (the host's second exchange)
    const uint64_t per = (uint64_t)S.xcap_u + S.xcap_r;
    or_lists(S, S.world, [&](int r, const uint32_t*& u, uint32_t& nu, const uint32_t*& rl, uint32_t& nr) {
        u = recv + r * per, nu = (uint32_t)S.xall[r].n_use;
        rl = u + S.xcap_u, nr = (uint32_t)S.xall[r].n_rel;
    });
}
void launch_pool_apply_spec(const DevState& S, const uint32_t* recv, hipStream_t st) {
    hipLaunchKernelGGL(k_pool_apply_spec, dim3(1024), dim3(256), 0, st, S, recv);
}
void launch_pool_apply(const DevState& S, const ListDesc* ld, int nranks, uint32_t max_n, hipStream_t st) {
    uint32_t g = max_n ? cdiv((uint64_t)cdiv(max_n, OR_RUN) * (uint32_t)nranks, 256) : 1;
    if (g > 1024) g = 1024;
    hipLaunchKernelGGL(k_pool_apply, dim3(g), dim3(256), 0, st, S, ld, nranks);
}


void launch_tick(const DevState& S, uint32_t n_stream, uint64_t now, uint64_t start, uint32_t n_hb, int phases,
                 uint32_t tag, uint64_t arrive_target, hipStream_t st, hipEvent_t t0, hipEvent_t t1) {
    const uint32_t grid = S.n_chain + ((phases & TICK_FRONT) ? n_stream : (S.multi ? S.n_pool_extra : 0u));
    auto kern = S.hb_units == (uint32_t)HB_CHUNKS ? k_tick<false> : k_tick<true>;
    if (t0)
        hipExtLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), 0, st, t0, t1, 0, S, now, start, n_hb, phases, tag,
                              arrive_target);
    else hipLaunchKernelGGL(kern, dim3(grid), dim3(BLOCK), 0, st, S, now, start, n_hb, phases, tag, arrive_target);
}

// ---------------------------------------------------------------------------
// k_emit: the patch bytes of a tick's node inits and pod patches, from the job
// records k_tick wrote (S.init_job / S.pp_job at the ordinals of init_off /
// pp_off; pod_controller.go:404-439 over pod.status.tpl, node_controller.go:
// 356-391 over node.status.tpl + node.heartbeat.tpl).  Launched after the
// tick's k_tick on the same stream (only for ticks with jobs).
//
// The work unit is 16 output bytes, assembled in registers and written with
// one 16-byte store.  A patch is a sequence of regions, each >= 16 bytes:
//   pod, status non-empty:  A | "hostIP":"H", | B | "podIP":"P", | C
//   pod, status empty:      A B C                  (one region)
//   node init:              pre | CONDS | post     (framed blob; the tick's
//                                                   heartbeat conditions)
// so a unit spans at most two regions, and (pods) overlaps at most one
// 20-byte creationTimestamp slot of the template (build_ts_lookup).  A wave
// takes 64 consecutive jobs at a time:
//   phase 1  lane j <- job j: the job's timestamp and hostIP / podIP pieces
//            into the wave's LDS record, its region bounds, its unit count;
//            a DPP scan gives the units' job-relative numbering;
//   phase 2  the chunk's units, 64 per pass (one per lane): the lane's job
//            (a uniform walk over the few jobs a pass touches), two 16-byte
//            source windows (5 dword reads + alignbyte each), a byte-mask
//            merge at the region boundary, the timestamp overlay, the store.
// Sources (spec programs, blobs, the heartbeat conditions, the job records)
// are read from LDS; a spec set or blob set too large for the block's cache
// is read from global memory instead (same code, generic pointers).
// ---------------------------------------------------------------------------
constexpr int EMIT_BLOCK = 256;
#ifndef EMIT_TAB_G
#define EMIT_TAB_G 8  // table path: lanes per job
#endif
#ifndef EMIT_FLAT_UNR
#define EMIT_FLAT_UNR 4  // one-spec chunks: 1 KiB stores per lane step
#endif
#ifndef EMIT_TAB_UNR
#define EMIT_TAB_UNR 5  // table path: units per lane per step (G * UNR = 40: a default pod patch)
#endif
static_assert(EMIT_BLOCK == BLOCK, "build_hb_template strides by BLOCK");
#ifndef EMIT_EC_PROG
#define EMIT_EC_PROG 4096  // spec programs cached in LDS (bytes)
#endif
#ifndef EMIT_EC_NXT
#define EMIT_EC_NXT 1152   // their timestamp lookups (entries)
#endif
#ifndef EMIT_EC_BLOB
#define EMIT_EC_BLOB 2048  // node blobs (bytes)
#endif
constexpr int EC_PROG = EMIT_EC_PROG, EC_NXT = EMIT_EC_NXT, EC_BLOB = EMIT_EC_BLOB;
constexpr uint32_t SEG_STRIDE = 56;  // per job: "hostIP":"H", (28 bytes) | "podIP":"P", (28 bytes)
constexpr uint32_t TS_STRIDE = 36;   // per job: its 20-byte timestamp, then 16 zero bytes
constexpr uint32_t TS_FIRST = 16;    // 16 zero bytes before job 0's timestamp
constexpr uint32_t TS_ZERO = TS_FIRST + 64 * TS_STRIDE;  // 20+ zero bytes (a unit with no slot)
constexpr uint32_t TS_AREA = TS_ZERO + 32;
constexpr uint32_t HB_LDS = HB_MAX_STRIDE + 32;  // the heartbeat template: CONDS at conds_off, read up to 32 bytes around it
static_assert(HB_LDS >= HB_STRIDE && HB_LDS >= ((HB_PREFIX + CONDS_LEN + 15) & ~15) + 32, "heartbeat template in LDS");
// the table path's value rows (device.h) alias seg / ts (a chunk takes one path)
constexpr uint32_t VROW_AREA = VROW_BIAS + 64 * VROW_STRIDE + 4;  // lead pad, rows, the last window's 5th dword
constexpr uint32_t EMIT_GEN_AREA = SRC_PAD_FRONT + 64 * SEG_STRIDE + SRC_PAD_BACK + TS_AREA;
struct EmitWave {
    uint4 rec[64];   // per job: arena offset / 16, region starts 1|2 and 3|4 (u16; 0xFFFF: none), template offset
                     // (table path: arena offset / 16, table unit base, unit count)
    uint32_t nxt[64];  // pods: the spec's timestamp lookup offset
    uint8_t seg[SRC_PAD_FRONT + 64 * SEG_STRIDE + SRC_PAD_BACK];
    uint8_t ts[TS_AREA];
    uint8_t vx[VROW_AREA > EMIT_GEN_AREA ? ((VROW_AREA - EMIT_GEN_AREA + 3) & ~3u) : 4];
};
static_assert(offsetof(EmitWave, ts) == offsetof(EmitWave, seg) + sizeof(EmitWave::seg) &&
                  offsetof(EmitWave, vx) == offsetof(EmitWave, ts) + sizeof(EmitWave::ts) &&
                  sizeof(EmitWave::seg) + sizeof(EmitWave::ts) + sizeof(EmitWave::vx) >= VROW_AREA,
              "value rows fit over seg | ts | vx");
static_assert(VROW_STRIDE % 4 == 0 && (VROW_STRIDE / 4) % 2 == 1, "rows: whole dwords, an odd count (banks)");
static_assert(VROW_TS == 0 && VROW_H == 36 && VROW_P == 68 && VROW_STRIDE == 100,
              "emit_phase1_tab writes the row as 25 dwords: TS 0-4, H 9-12, P 17-20");
struct EmitLds {
    uint16_t nxt[EC_NXT];
    uint8_t prog[SRC_PAD_FRONT + EC_PROG + SRC_PAD_BACK];
    uint8_t blob[SRC_PAD_FRONT + EC_BLOB + SRC_PAD_BACK];
    uint8_t hb[HB_LDS];  // the tick's heartbeat template
    uint32_t spec_ok, blob_ok;
    EmitWave w[EMIT_BLOCK / 64];
};
static_assert(sizeof(EmitLds) <= 40960, "four k_emit blocks per CU");

// a 16-byte unit of patch output, non-temporal (written once, read by the host's
// copy engine): 1M x 10M initial k_emit 1.70 -> 1.62 ms against plain stores
__device__ __forceinline__ void emit_st(uint8_t* arena, uint64_t off, uint4 v) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#ifdef EMIT_NT  // A/B builds (plain stores: initial-tick emission -2-4%, round 5)
    __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(arena + off));
#else
    *reinterpret_cast<u32x4*>(arena + off) = u32x4{v.x, v.y, v.z, v.w};
#endif
}
__device__ __forceinline__ uint32_t rdlane(uint32_t v, uint32_t k) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)k); }

// 16 bytes at byte offset `off` of a 4-byte aligned source (LDS or global)
__device__ __forceinline__ uint4 ext16(const uint8_t* base, uint32_t off) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(base) + (off >> 2);
    const uint32_t sh = off & 3u;
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
    return make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                      __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
}

// `"<key>":"<ip>",` as 7 dwords (key: KLEN bytes, 10 for hostIP, 9 for podIP)
template <int KLEN>
__device__ __forceinline__ void write_seg(uint8_t* dst, Lit16 key, const IpStr& ip) {
    uint32_t d[6] = {(uint32_t)ip.lo, (uint32_t)(ip.lo >> 32), (uint32_t)ip.hi, (uint32_t)(ip.hi >> 32), 0u, 0u};
    const uint64_t tail = 0x2C22ull << (8u * (ip.len & 3u));  // '"' ',' after the address
    const uint32_t m = ip.len >> 2;
#pragma unroll
    for (uint32_t k = 0; k < 5; k++) d[k] |= (m == k ? (uint32_t)tail : 0u) | (m + 1u == k ? (uint32_t)(tail >> 32) : 0u);
    const uint32_t kw[4] = {(uint32_t)key.lo, (uint32_t)(key.lo >> 32), (uint32_t)key.hi, (uint32_t)(key.hi >> 32)};
    uint32_t* o = reinterpret_cast<uint32_t*>(dst);
#pragma unroll
    for (int i = 0; i < 7; i++) {
        const int b = 4 * i - KLEN;  // offset into `<ip>",` of this dword's first byte
        uint32_t v = i < 4 ? kw[i] : 0u;
        if (b >= 0) v |= __builtin_amdgcn_alignbyte(d[(b >> 2) + 1], d[b >> 2], (uint32_t)(b & 3));
        else if (b > -4) v |= d[0] << (8 * -b);
        o[i] = v;
    }
}

// the block's sources in LDS (when they fit), the tick's heartbeat template,
// zeroed job records
__device__ __forceinline__ void stage_emit(const DevState& S, EmitLds* L, bool pods, bool nodes, uint64_t now_unix,
                                           uint64_t start_unix) {
    const uint32_t t = threadIdx.x;
    const bool sp = pods && S.spec_total <= (uint32_t)EC_PROG && S.nxt_total <= (uint32_t)EC_NXT;
    const bool bl = nodes && S.blob_total <= (uint32_t)EC_BLOB;
    if (sp) {
        for (uint32_t i = t; i < S.nxt_total; i += BLOCK) L->nxt[i] = S.spec_nxt[i];
        const uint32_t* src = reinterpret_cast<const uint32_t*>(S.spec_bytes - SRC_PAD_FRONT);  // the padded array
        uint32_t* dst = reinterpret_cast<uint32_t*>(L->prog);
        for (uint32_t i = t; i < (SRC_PAD_FRONT + S.spec_total + 3) / 4 + SRC_PAD_BACK / 4; i += BLOCK) dst[i] = src[i];
    }
    if (bl) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(S.blob - SRC_PAD_FRONT);
        uint32_t* dst = reinterpret_cast<uint32_t*>(L->blob);
        for (uint32_t i = t; i < (SRC_PAD_FRONT + S.blob_total + 3) / 4 + SRC_PAD_BACK / 4; i += BLOCK) dst[i] = src[i];
    }
    uint32_t* z = reinterpret_cast<uint32_t*>(L->w);
    for (uint32_t i = t; i < sizeof(L->w) / 4; i += BLOCK) z[i] = 0u;
    for (uint32_t i = 16u * S.hb_units + t; i < HB_LDS; i += BLOCK) L->hb[i] = 0;
    if (t == 0) {
        L->spec_ok = sp ? 1u : 0u;
        L->blob_ok = bl ? 1u : 0u;
    }
    if (nodes) build_hb_template(S, L->hb, now_unix, start_unix);  // synchronises
    __syncthreads();
}

// phase 1: lane l <- job q; returns its number of 16-byte units
template <bool POD>
__device__ __forceinline__ uint32_t emit_phase1(const DevState& S, EmitWave* W, uint32_t q, uint32_t n) {
    const uint32_t l = lane_id();
    uint32_t nu = 0, o16 = 0, e12 = 0xFFFFFFFFu, e34 = 0xFFFFFFFFu, toff = 0, nxo = 0;
    if (q < n) {
        uint64_t off;
        uint32_t len;
        if (POD) {
            const uint4 j = S.pp_job[q];  // podIP (0: no status section), hostIP, creationTimestamp, spec
            off = S.pp_off[q];
            len = S.pp_len[q];
            const SpecDesc sd = S.specs[j.w];
            toff = sd.off;
            nxo = sd.nxt_off;
            const Ts ts = format_ts(j.z);
            uint32_t* tw = reinterpret_cast<uint32_t*>(W->ts + TS_FIRST + l * TS_STRIDE);
            tw[0] = (uint32_t)ts.w0;
            tw[1] = (uint32_t)(ts.w0 >> 32);
            tw[2] = (uint32_t)ts.w1;
            tw[3] = (uint32_t)(ts.w1 >> 32);
            tw[4] = (uint32_t)ts.w2;
            if (j.y != 0) {  // `{{ with .status }}`: hostIP / podIP (pod.status.tpl:44-47)
                const IpStr H = format_ip(j.y), P = format_ip(j.x);
                uint8_t* sg = W->seg + SRC_PAD_FRONT + l * SEG_STRIDE;
                write_seg<10>(sg, lit16("\"hostIP\":\""), H);
                write_seg<9>(sg + 28, lit16("\"podIP\":\""), P);
                const uint32_t e1 = sd.len_a, e2 = e1 + 12u + H.len, e3 = e2 + sd.len_b, e4 = e3 + 11u + P.len;
                e12 = e1 | e2 << 16;
                e34 = e3 | e4 << 16;
            }
        } else {
            const uint64_t b = S.init_job[q];
            off = S.init_off[q];
            len = S.init_len[q];
            toff = (uint32_t)b;
            const uint32_t pre = (uint32_t)(b >> 32) & 0xFFFFu;
            e12 = pre | (pre + S.conds_len) << 16;
        }
        o16 = (uint32_t)(off >> 4);
        nu = (len + 15u) >> 4;
    }
    W->rec[l] = make_uint4(o16, e12, e34, toff);
    W->nxt[l] = nxo;
    return nu;
}

// phase 2: the units of the chunk's cnt jobs (ustart: lane j = job j's first unit).
// Every region's bytes sit at (output position + delta(region)) of its source:
//   pods:  A: tmpl          H: seg(k) - e1      B: tmpl - (e2 - e1)
//          P: seg(k)+28 - e3                    C: tmpl - (e2 - e1) - (e4 - e3)
//   inits: pre: blob        CONDS: hb + 24 - e1  post: blob + e1 - e2
// (tmpl / blob: the job's template offset in the spec / blob array).
struct EmitSrc {
    const uint8_t* lds;
    const uint8_t* tbase;  // template source: the LDS cache, else the global array (flat reads)
    uint32_t o_seg, o_ts, o_tmpl;
};
// unit x (byte offset, a multiple of 16) of job k: its 16 bytes and arena offset
template <bool POD, bool CACHED>
__device__ __forceinline__ uint4 emit_unit(const DevState& S, const EmitLds* L, const EmitWave* W, const EmitSrc& E,
                                           uint32_t k, uint32_t x, uint64_t& dst) {
    const uint4 R = W->rec[k];
    const uint32_t e1 = R.y & 0xFFFFu, e2 = R.y >> 16, e3 = R.z & 0xFFFFu, e4 = R.z >> 16, toff = R.w;
    const uint32_t y = x + 15u;
    // region deltas (see above) and starts, selected by the region bits of x and y
    const uint32_t seg_k = E.o_seg + k * SEG_STRIDE;
    const uint32_t d0 = E.o_tmpl + toff;
    const uint32_t d1 = POD ? seg_k - e1 : (uint32_t)offsetof(EmitLds, hb) + S.conds_off - e1;
    const uint32_t d2 = POD ? d0 - (e2 - e1) : d0 + e1 - e2;
    const uint32_t d3 = seg_k + 28u - e3;
    const uint32_t d4 = d2 - (e4 - e3);
    const bool x1 = x >= e1, x2 = x >= e2, x3 = x >= e3, x4 = x >= e4;
    const bool y1 = y >= e1, y2 = y >= e2, y3 = y >= e3, y4 = y >= e4;
    uint32_t dx = d0, dy = d0, sy = 0;
    dx = x1 ? d1 : dx, dx = x2 ? d2 : dx, dx = x3 ? d3 : dx, dx = x4 ? d4 : dx;
    dy = y1 ? d1 : dy, dy = y2 ? d2 : dy, dy = y3 ? d3 : dy, dy = y4 ? d4 : dy;
    sy = y1 ? e1 : sy, sy = y2 ? e2 : sy, sy = y3 ? e3 : sy, sy = y4 ? e4 : sy;
    const uint32_t rx = (uint32_t)x1 + x2 + x3 + x4, ry = (uint32_t)y1 + y2 + y3 + y4;
    const uint32_t n = rx == ry ? 16u : sy - x;  // bytes of the unit in x's region
    // template regions: pods 0, 2, 4; inits 0, 2
    const bool tx = POD ? !(rx & 1u) : rx != 1u, ty = POD ? !(ry & 1u) : ry != 1u;
    const uint8_t* bx = (CACHED || !tx) ? E.lds : E.tbase;
    const uint8_t* by = (CACHED || !ty) ? E.lds : E.tbase;
    const uint4 v1 = ext16(bx, x + dx), v2 = ext16(by, x + dy);
    uint32_t o[4];
    const uint32_t vv1[4] = {v1.x, v1.y, v1.z, v1.w}, vv2[4] = {v2.x, v2.y, v2.z, v2.w};
#pragma unroll
    for (int d = 0; d < 4; d++) {
        const int c = min(max((int)n - 4 * d, 0), 4);  // bytes of dword d from x's region
        const uint32_t m = c == 4 ? 0xFFFFFFFFu : (1u << (8 * c)) - 1u;
        o[d] = (vv1[d] & m) | (vv2[d] & ~m);
    }
    if (POD) {
        // the timestamp slot (at most one) in the unit's template region; template
        // coordinate of output position p in a template region: p + delta - d0
        const bool tt = tx || ty;
        const uint32_t dT = tx ? dx : dy;
        const uint32_t w0 = tx ? x : sy, w1 = (tx && rx != ry) ? sy : x + 16u;
        const uint32_t tw0 = w0 + dT - d0, tw1 = w1 + dT - d0;
        const uint32_t ni = tt ? W->nxt[k] + (tw0 >> 2) : 0u;
        const uint32_t s = CACHED ? (uint32_t)L->nxt[ni] : (uint32_t)S.spec_nxt[ni];
        const bool ov = tt && s < tw1 && s + (uint32_t)TS_LEN > tw0;
        const uint32_t so = s + d0 - dT;  // output position of the slot
        const uint4 t4 = ext16(E.lds, E.o_ts + (ov ? TS_FIRST + k * TS_STRIDE + x - so : TS_ZERO));
        o[0] |= t4.x;
        o[1] |= t4.y;
        o[2] |= t4.z;
        o[3] |= t4.w;
    }
    dst = ((uint64_t)R.x << 4) + x;
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// two units per lane per pass (u and u + 64): two independent LDS chains in flight
template <bool POD, bool CACHED>
__device__ __forceinline__ void emit_phase2(const DevState& S, const EmitLds* L, const EmitWave* W, uint32_t cnt,
                                            uint32_t ustart, uint32_t utot) {
    const uint32_t l = lane_id();
    EmitSrc E;
    E.lds = reinterpret_cast<const uint8_t*>(L);
    E.o_seg = (uint32_t)((const uint8_t*)W->seg - E.lds) + SRC_PAD_FRONT;
    E.o_ts = (uint32_t)((const uint8_t*)W->ts - E.lds);
    E.tbase = CACHED ? E.lds : (POD ? S.spec_bytes : S.blob);
    E.o_tmpl = CACHED ? (uint32_t)(POD ? offsetof(EmitLds, prog) : offsetof(EmitLds, blob)) + SRC_PAD_FRONT : 0u;
    uint32_t kcur = 0;
    for (uint32_t u0 = 0; u0 < utot; u0 += 128u) {
        // past the chunk's units a lane redoes its last unit and does not store it
        const uint32_t ua = min(u0 + l, utot - 1u), ub = min(u0 + 64u + l, utot - 1u);
        // each unit's job: the last job of the pass whose first unit is <= it
        uint32_t ka = kcur, kb = kcur, sa = rdlane(ustart, kcur), sb = sa;
        for (uint32_t j = kcur + 1; j < cnt; j++) {
            const uint32_t s = rdlane(ustart, j);
            if (s > u0 + 127u) break;
            const bool ga = ua >= s, gb = ub >= s;
            ka = ga ? j : ka;
            sa = ga ? s : sa;
            kb = gb ? j : kb;
            sb = gb ? s : sb;
        }
        kcur = rdlane(kb, 63);
        uint64_t da, db;
        const uint4 va = emit_unit<POD, CACHED>(S, L, W, E, ka, (ua - sa) << 4, da);
        const uint4 vb = emit_unit<POD, CACHED>(S, L, W, E, kb, (ub - sb) << 4, db);
        if (u0 + l < utot) emit_st(S.arena, da, va);
        if (u0 + 64u + l < utot) emit_st(S.arena, db, vb);
    }
}

// ---- table-driven pod path (device.h): lane l <- job q of the chunk --------
struct TabJob {
    uint32_t o16, tb, nu, mu;  // mu: the spec's reservation in units (max_len / 16)
    bool ok;  // the job's spec has unit tables (or q >= n)
    Ts ts;
    IpStr h, p;
};
// a job's records (loaded one chunk ahead) and the lane's last spec descriptor
struct JobRaw {
    uint4 j;  // podIP (0: no status section), hostIP, creationTimestamp, spec
    uint64_t off;
    uint32_t len;
};
__device__ __forceinline__ JobRaw job_raw(const DevState& S, uint64_t q, uint32_t n) {
    JobRaw R;
    R.j = make_uint4(0u, 0u, 0u, 0u), R.off = 0, R.len = 0;
    if (q < n) R.j = S.pp_job[q], R.off = S.pp_off[q], R.len = S.pp_len[q];
    return R;
}
struct SpecCache {
    uint32_t id, tab_off, max_len;
};
__device__ __forceinline__ TabJob emit_job_tab(const DevState& S, const JobRaw& R, bool live, SpecCache& sc) {
    TabJob J;
    J.o16 = J.tb = J.nu = J.mu = 0;
    J.ok = true;
    J.h.lo = J.h.hi = J.p.lo = J.p.hi = 0;
    J.ts.w0 = J.ts.w1 = J.ts.w2 = 0;
    if (live) {
        const uint4 j = R.j;
        if (j.w != sc.id) {  // usually every job of a wave shares one spec: one load per lane
            const SpecDesc& sd = S.specs[j.w];
            sc.id = j.w, sc.tab_off = sd.tab_off, sc.max_len = sd.max_len;
        }
        J.ok = sc.tab_off != NO_TAB;
        J.ts = format_ts(j.z);
        uint32_t shape = 0;
        if (j.y != 0) {  // `{{ with .status }}`: hostIP / podIP (pod.status.tpl:44-47)
            J.h = format_ip(j.y);
            J.p = format_ip(j.x);
            shape = emit_shape(J.h.len, J.p.len);
        }
        J.mu = sc.max_len >> 4;
        J.tb = sc.tab_off + shape * J.mu;
        J.o16 = (uint32_t)(R.off >> 4);
        J.nu = (R.len + 15u) >> 4;
    }
    return J;
}
// the job's value row (25 dwords: TS, zeros, H, zeros, P, zeros) and record
template <class WV>
__device__ __forceinline__ void emit_row_tab(WV* W, const TabJob& J) {
    const uint32_t l = lane_id();
    uint32_t* r = reinterpret_cast<uint32_t*>(W->seg + VROW_BIAS + l * VROW_STRIDE);
    const uint32_t v[25] = {(uint32_t)J.ts.w0, (uint32_t)(J.ts.w0 >> 32), (uint32_t)J.ts.w1, (uint32_t)(J.ts.w1 >> 32),
                            (uint32_t)J.ts.w2, 0u, 0u, 0u, 0u,
                            (uint32_t)J.h.lo, (uint32_t)(J.h.lo >> 32), (uint32_t)J.h.hi, (uint32_t)(J.h.hi >> 32),
                            0u, 0u, 0u, 0u,
                            (uint32_t)J.p.lo, (uint32_t)(J.p.lo >> 32), (uint32_t)J.p.hi, (uint32_t)(J.p.hi >> 32),
                            0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < 25; i++) r[i] = v[i];
    if (l < 4) reinterpret_cast<uint32_t*>(W->seg)[l] = 0u;  // the lead pad (row 0's zero window)
    W->rec[l] = make_uint4(J.o16, J.tb, J.nu, 0u);
}
// G lanes per job, G * UNR units of it per step (unit li + G * i for lane li).
// Steps are (job pass, unit step) pairs, software-pipelined: the next step's
// record and table loads are issued before this step's value-row reads and
// stores, so the table round trip hides behind a step of stores.
template <int UNR>
struct TabStep {
    uint4 t[UNR];
    uint32_t d[UNR];
    uint32_t o16, nu, k, u0;
};
template <int G, int UNR, class WV>
__device__ __forceinline__ TabStep<UNR> tab_load(const DevState& S, const WV* W, uint32_t cnt, uint32_t item,
                                                 uint32_t nsteps) {
    const uint32_t l = lane_id(), li = l % G;
    const uint32_t pass = item / nsteps, step = item - pass * nsteps;  // wave-uniform
    TabStep<UNR> T;
    T.k = pass * (64 / G) + l / G;
    T.u0 = step * (G * UNR) + li;
    uint32_t tb = 0;
    T.nu = 0, T.o16 = 0;
    if (T.k < cnt) {
        const uint4 R = W->rec[T.k];
        T.o16 = R.x, tb = R.y, T.nu = R.z;
    }
#pragma unroll
    for (int i = 0; i < UNR; i++) {  // past the job's units: reload its last unit (no store)
        const uint32_t u = T.nu ? min(T.u0 + G * i, T.nu - 1u) : 0u;
        T.t[i] = S.unit_tab[tb + u];
        T.d[i] = S.unit_desc[tb + u];
    }
    return T;
}
template <int G, int UNR, class WV>
__device__ __forceinline__ void tab_store(const DevState& S, const WV* W, const TabStep<UNR>& T) {
    const uint8_t* row = W->seg + T.k * VROW_STRIDE;  // biased: row k starts VROW_BIAS bytes in
    uint32_t dor = 0;
#pragma unroll
    for (int i = 0; i < UNR; i++) dor |= T.d[i];
    uint4 v[UNR];
#pragma unroll
    for (int i = 0; i < UNR; i++) v[i] = ext16(row, T.d[i] & 0xFFu);
    if (__builtin_expect(dor >> 8, 0)) {  // a second field in a unit
#pragma unroll
        for (int i = 0; i < UNR; i++) {
            const uint4 w = ext16(row, T.d[i] >> 8);
            v[i].x |= w.x, v[i].y |= w.y, v[i].z |= w.z, v[i].w |= w.w;
        }
    }
#pragma unroll
    for (int i = 0; i < UNR; i++) {
        const uint32_t u = T.u0 + G * i;
        if (u < T.nu)
            emit_st(S.arena, (uint64_t)(T.o16 + u) << 4,
                    make_uint4(T.t[i].x | v[i].x, T.t[i].y | v[i].y, T.t[i].z | v[i].z, T.t[i].w | v[i].w));
    }
}
// maxnu: the chunk's largest unit count (wave-uniform)
template <int G, int UNR, class WV>
__device__ __forceinline__ void emit_phase2_tab(const DevState& S, const WV* W, uint32_t cnt, uint32_t maxnu) {
    const uint32_t nsteps = (maxnu + G * UNR - 1) / (G * UNR);
    const uint32_t items = ((cnt + 64 / G - 1) / (64 / G)) * nsteps;
    if (items == 0) return;
    TabStep<UNR> cur = tab_load<G, UNR>(S, W, cnt, 0, nsteps);
    for (uint32_t it = 0; it < items; it++) {
        TabStep<UNR> nxt;
        if (it + 1 < items) nxt = tab_load<G, UNR>(S, W, cnt, it + 1, nsteps);
        tab_store<G, UNR>(S, W, cur);
        cur = nxt;
    }
}

// Chunks of one spec (every job reserves the same max_len = MU units, so the
// chunk's patches are one contiguous run of cnt * MU units): lane l takes units
// l + 64 i of the run, so every store is a whole 1 KiB of the arena.  A unit's
// job / unit index advance incrementally; units of a job's reservation past its
// patch are not stored.  Software-pipelined like the G-lane path.
template <int UNR>
struct FlatStep {
    uint4 t[UNR];
    uint32_t d[UNR], k[UNR], ok[UNR];
};
template <int UNR, class WV>
__device__ __forceinline__ FlatStep<UNR> flat_load(const DevState& S, const WV* W, uint32_t& k, uint32_t& u,
                                                   uint32_t dk, uint32_t du, uint32_t mu, uint32_t cnt) {
    FlatStep<UNR> F;
#pragma unroll
    for (int i = 0; i < UNR; i++) {
        const bool live = k < cnt;
        const uint4 R = W->rec[live ? k : 0u];  // arena offset / 16, table unit base, unit count
        F.k[i] = k;
#ifdef EMIT_PATCH_ONLY  // A/B builds: only the patch's units
        F.ok[i] = live && u < R.z;
#else  // the whole reservation (zeros past the patch): the run is one unbroken stream of
       // whole 128-byte lines, none written in part (initial-tick emission -2-4%, round 5)
        F.ok[i] = live;
#endif
        const uint32_t uu = F.ok[i] ? u : 0u;
#ifdef EMIT_DIAG_NO_TAB  // timing builds only: no table loads
        F.t[i] = make_uint4(uu, R.y, 0u, 0u);
        F.d[i] = uu & 63u;
#else
        F.t[i] = S.unit_tab[R.y + uu];
        F.d[i] = S.unit_desc[R.y + uu];
#endif
        k += dk, u += du;
        if (u >= mu) u -= mu, k++;
    }
    return F;
}
template <int UNR, class WV>
__device__ __forceinline__ void flat_store(const DevState& S, const WV* W, const FlatStep<UNR>& F, uint64_t o16,
                                           uint32_t g) {
    uint32_t dor = 0;
#pragma unroll
    for (int i = 0; i < UNR; i++) dor |= F.d[i];
    uint4 v[UNR];
#pragma unroll
    for (int i = 0; i < UNR; i++) v[i] = ext16(W->seg + F.k[i] * VROW_STRIDE, F.d[i] & 0xFFu);
    if (__builtin_expect(dor >> 8, 0)) {  // a second field in a unit
#pragma unroll
        for (int i = 0; i < UNR; i++) {
            const uint4 w = ext16(W->seg + F.k[i] * VROW_STRIDE, F.d[i] >> 8);
            v[i].x |= w.x, v[i].y |= w.y, v[i].z |= w.z, v[i].w |= w.w;
        }
    }
#pragma unroll
    for (int i = 0; i < UNR; i++)
        if (F.ok[i])
            emit_st(S.arena, (o16 + g + 64u * i) << 4,
                    make_uint4(F.t[i].x | v[i].x, F.t[i].y | v[i].y, F.t[i].z | v[i].z, F.t[i].w | v[i].w));
}
template <int UNR, class WV>
__device__ __forceinline__ void emit_phase2_flat(const DevState& S, const WV* W, uint32_t cnt, uint32_t mu) {
    const uint32_t l = lane_id();
    const uint64_t o16 = W->rec[0].x;
    const uint32_t total = cnt * mu;
    uint32_t k = l / mu, u = l - (l / mu) * mu;
    const uint32_t dk = 64u / mu, du = 64u - dk * mu;
    FlatStep<UNR> cur = flat_load<UNR>(S, W, k, u, dk, du, mu, cnt);
    for (uint32_t g0 = 0; g0 < total; g0 += 64u * UNR) {
        FlatStep<UNR> nxt;
        if (g0 + 64u * UNR < total) nxt = flat_load<UNR>(S, W, k, u, dk, du, mu, cnt);
        flat_store<UNR>(S, W, cur, o16, g0 + l);
        cur = nxt;
    }
}

// ---- fused pod emission (k_pod_jobs<true>) ---------------------------------
// A wave's jobs (staged records, record.w = spec | len << 16, consecutive
// ordinals from ord0, reservations back to back from off0) in chunks of 64:
// their arena offsets (a wave scan of the specs' max_len), pp_off, and the
// bytes by the table path as k_emit writes them.  The host fuses only while
// every spec has unit tables; a job without them fails the tick (TICK_ERR_EMIT).
static_assert(sizeof(TabWave::seg) >= VROW_AREA, "value rows fit TabWave");
static_assert(sizeof(TabWave) <= POD_STAGE_WORDS_F * 4, "TabWave aliases a wave's fused stage");
__device__ __forceinline__ void fused_pod_emit(const DevState& S, TabWave* W, const uint4* stg, uint32_t n, uint64_t ord0, uint64_t off0) {
    const uint32_t l = lane_id();
    // the wave's <= 512 records into registers (lane l: jobs l, l + 64, ...): the
    // stage they leave is W (TabWave aliases it)
    uint4 rr[8];
#pragma unroll
    for (int q = 0; q < 8; q++) rr[q] = 64u * q + l < n ? stg[64u * q + l] : make_uint4(0u, 0u, 0u, 0u);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    SpecCache sc{0xFFFFFFFFu, NO_TAB, 0u};
    uint64_t base = off0;
    bool bad = false;
    for (uint32_t c = 0; c < n; c += 64u) {
        const uint32_t cnt = min(64u, n - c);
        const bool live = l < cnt;
        JobRaw R;
        R.j = rr[0];
#pragma unroll
        for (int k = 0; k < 7; k++) rr[k] = rr[k + 1];  // (a select on the chunk index would put rr in scratch)
        R.len = R.j.w >> 16;
        R.j.w &= 0xFFFFu;
        if (live && R.j.w != sc.id) {
            const SpecDesc& sd = S.specs[R.j.w];
            sc.id = R.j.w, sc.tab_off = sd.tab_off, sc.max_len = sd.max_len;
        }
        const uint32_t mb = live ? sc.max_len : 0u;
        const uint32_t incl = wave_incl_scan(mb);
        R.off = base + (incl - mb);
        base += rdlane(incl, 63);
        if (live) S.pp_off[ord0 + c + l] = R.off;
        const TabJob J = emit_job_tab(S, R, live, sc);
        if (__ballot(!J.ok) != 0) {
            bad = true;
            continue;
        }
        emit_row_tab(W, J);
        uint32_t mx = J.nu;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
        const uint32_t mu = __builtin_amdgcn_readfirstlane(J.mu);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the rows before phase 2 reads them
        if (__ballot(live && J.mu != mu) == 0) emit_phase2_flat<EMIT_FLAT_UNR>(S, W, cnt, mu);
        else emit_phase2_tab<EMIT_TAB_G, EMIT_TAB_UNR>(S, W, cnt, __builtin_amdgcn_readfirstlane(mx));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // phase 2's reads before the next rows
    }
    if (bad && l == 0) st_host(&S.hdr_host->err, TICK_ERR_EMIT);
}

// ---- node inits of one blob (the common case: nodes created alike) --------
// When every job of a chunk frames the same blob, its init patches are all the
// same bytes: the wave renders the patch once into LDS (seg | ts | vx) with the
// general unit emitter, then streams cnt copies of it with aligned 16-byte LDS
// reads (the jobs sit back to back in the arena, init_patch_len rounded to 16).
constexpr uint32_t INIT_RENDER_MAX = (SRC_PAD_FRONT + 64 * SEG_STRIDE + SRC_PAD_BACK + TS_AREA) & ~15u;

// the chunk's cnt init jobs, all of one blob, nu units each (records in W->rec)
template <bool CACHED>
__device__ __forceinline__ void emit_init_copies(const DevState& S, const EmitLds* L, EmitWave* W, uint32_t cnt,
                                                 uint32_t nu) {
    const uint32_t l = lane_id();
    EmitSrc E;
    E.lds = reinterpret_cast<const uint8_t*>(L);
    E.o_seg = 0, E.o_ts = 0;
    E.tbase = CACHED ? E.lds : S.blob;
    E.o_tmpl = CACHED ? (uint32_t)offsetof(EmitLds, blob) + SRC_PAD_FRONT : 0u;
    uint4* img = reinterpret_cast<uint4*>(W->seg);  // 16-byte aligned
    for (uint32_t u = l; u < nu; u += 64) {  // render job 0's patch
        uint64_t dst;
        img[u] = emit_unit<false, CACHED>(S, L, W, E, 0, u << 4, dst);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t o16 = W->rec[0].x;  // the chunk's jobs are contiguous from job 0's offset
    const uint32_t total = cnt * nu;
    uint32_t u = l % nu;
    const uint32_t step = 64u % nu;
    for (uint32_t g = l; g < total; g += 64) {
        emit_st(S.arena, (o16 + g) << 4, img[u]);
        u += step;
        u = u >= nu ? u - nu : u;
    }
}

template <bool POD, bool CACHED>
__device__ __forceinline__ void emit_jobs(const DevState& S, EmitLds* L, uint32_t w0, uint32_t nw, uint32_t n) {
    EmitWave* W = &L->w[wave_id()];
    SpecCache sc{0xFFFFFFFFu, NO_TAB, 0u};
    JobRaw nxt;
    if (POD) nxt = job_raw(S, (uint64_t)w0 * 64u + lane_id(), n);
    for (uint32_t ch = w0; ch * 64u < n; ch += nw) {
        const uint32_t cnt = min(64u, n - ch * 64u);
        if (POD) {
            const JobRaw cur = nxt;
            nxt = job_raw(S, (uint64_t)(ch + nw) * 64u + lane_id(), n);  // the wave's next chunk, in flight
            const TabJob J = emit_job_tab(S, cur, ch * 64u + lane_id() < n, sc);
            if (__ballot(!J.ok) == 0) {  // every job of the chunk has tables
                emit_row_tab(W, J);
                uint32_t mx = J.nu;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
                const uint32_t mu = __builtin_amdgcn_readfirstlane(J.mu);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the rows before phase 2 reads them
                if (__ballot(ch * 64u + lane_id() < n && J.mu != mu) == 0)
                    emit_phase2_flat<EMIT_FLAT_UNR>(S, W, cnt, mu);
                else
                    emit_phase2_tab<EMIT_TAB_G, EMIT_TAB_UNR>(S, W, cnt, __builtin_amdgcn_readfirstlane(mx));
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // phase 2's reads before the next rows
                continue;
            }
        }
        const uint32_t nu = emit_phase1<POD>(S, W, ch * 64u + lane_id(), n);
        const uint32_t incl = wave_incl_scan(nu);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the records before phase 2 reads them
        if (!POD) {
            const uint64_t q = (uint64_t)ch * 64u + lane_id();
            const uint64_t blob = q < n ? S.init_job[q] : 0ull;
            const uint64_t b0 = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(blob >> 32)) << 32) |
                                __builtin_amdgcn_readfirstlane((uint32_t)blob);
            const uint32_t nu0 = __builtin_amdgcn_readfirstlane(nu);
            if (__ballot(q < n && blob != b0) == 0 && nu0 * 16u <= INIT_RENDER_MAX) {
                emit_init_copies<CACHED>(S, L, W, cnt, nu0);
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                continue;
            }
        }
        emit_phase2<POD, CACHED>(S, L, W, cnt, incl - nu, rdlane(incl, 63));
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // phase 2's reads before the next records
    }
}

__global__ __launch_bounds__(EMIT_BLOCK, 4) void k_emit(DevState S, uint64_t now_unix, uint64_t start_unix) {
    __shared__ EmitLds L;
    // the tick's launches were skipped: queued behind one the host has not finished, or
    // (kwok_ingest_pods_packed12_tick) behind a batch whose chunk needs more pod slots
    if (__hip_atomic_load(&S.bar->skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
    const uint32_t n_pp = S.emit_n[0], n_init = S.emit_n[1];
    if (n_pp == 0 && n_init == 0) return;
    stage_emit(S, &L, n_pp != 0, n_init != 0, now_unix, start_unix);
    const uint32_t w0 = blockIdx.x * (EMIT_BLOCK / 64) + wave_id(), nw = gridDim.x * (EMIT_BLOCK / 64);
#ifdef EMIT_DIAG_NO_INITS  // timing builds only (tools/build_variant.sh): one job kind skipped
    if (false) {
#else
    if (n_init) {
#endif
        if (L.blob_ok) emit_jobs<false, true>(S, &L, w0, nw, n_init);
        else emit_jobs<false, false>(S, &L, w0, nw, n_init);
    }
#ifdef EMIT_DIAG_NO_PODS
    if (false) {
#else
    if (n_pp) {
#endif
        if (L.spec_ok) emit_jobs<true, true>(S, &L, w0, nw, n_pp);
        else emit_jobs<true, false>(S, &L, w0, nw, n_pp);
    }
}

void launch_emit(const DevState& S, uint32_t grid, uint64_t now, uint64_t start, hipStream_t st) {
    hipLaunchKernelGGL(k_emit, dim3(grid), dim3(EMIT_BLOCK), 0, st, S, now, start);
}

// FUSE: the runs' pod patch bytes too (fused_pod_emit over each run's staged jobs,
// when every spec has unit tables): no job records written and read back by k_emit.
// Its waves take the runs run-major (run c0 of every chain block, then c0 + 1, ...):
// the empty runs past the blocks' pods are the grid's last waves, and the dispatch
// order mixes the blocks' regions of the arena.  The fused grid's last blocks (from
// pod_blocks on) write the tick's node inits as k_emit would (one launch for the
// whole emission: they start as the pod waves drain and fill the CUs those leave).
struct JobsLdsF {
    uint32_t stage[JOB_WAVES * POD_STAGE_WORDS_F];
    uint32_t gpre_w[JOB_WAVES][MAX_BPB + 1];
    uint32_t nf_w[JOB_WAVES][JOB_NF_BYTES / 4];  // the node flags of the runs' buckets
};
struct JobsLds {
    uint32_t stage[JOB_WAVES * POD_STAGE_WORDS];
    uint32_t gpre_w[JOB_WAVES][MAX_BPB + 1];
    uint32_t nf_w[JOB_WAVES][JOB_NF_BYTES / 4];
};
union FusedLds {
    JobsLdsF j;
    EmitLds e;
};
static_assert(64 * JOB_WAVES == EMIT_BLOCK, "node-init blocks of k_pod_jobs<true> are k_emit blocks");
#ifndef JOBS_MIN_WAVES_UNFUSED
#define JOBS_MIN_WAVES_UNFUSED 1
#endif
#define JOBS_MIN_WAVES (FUSE ? 3 : JOBS_MIN_WAVES_UNFUSED)  // waves per SIMD
template <bool FUSE>
__global__ __launch_bounds__(64 * JOB_WAVES, JOBS_MIN_WAVES) void k_pod_jobs(DevState S, uint32_t tag, uint32_t wg_per_block,
                                                                          uint32_t pod_blocks, uint64_t now_unix,
                                                                          uint64_t start_unix) {
    constexpr int NC = FUSE ? 1 : JOB_NC;
    __shared__ typename std::conditional<FUSE, FusedLds, JobsLds>::type sh;
    auto& J = reinterpret_cast<typename std::conditional<FUSE, JobsLdsF, JobsLds>::type&>(sh);
    static_assert(JOB_NC == 2 && MAX_WC % 32 == 0, "a wave's runs share one dirty word");
    const uint32_t w = (uint32_t)wave_id(), it = blockIdx.x * JOB_WAVES + w;
    if constexpr (FUSE) {
        if (blockIdx.x >= pod_blocks) {  // node inits (block-uniform)
            if (__hip_atomic_load(&S.bar->skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
            const uint32_t n_init = S.emit_n[1];
            if (n_init == 0) return;
            EmitLds* L = reinterpret_cast<EmitLds*>(&sh);
            stage_emit(S, L, false, true, now_unix, start_unix);
            const uint32_t w0 = (blockIdx.x - pod_blocks) * JOB_WAVES + w, nw = (gridDim.x - pod_blocks) * JOB_WAVES;
            if (L->blob_ok) emit_jobs<false, true>(S, L, w0, nw, n_init);
            else emit_jobs<false, false>(S, L, w0, nw, n_init);
            return;
        }
    }
    uint32_t b, c0;
#ifndef JOBS_BLOCK_MAJOR  // (A/B builds)
    if constexpr (FUSE) {
        c0 = it / S.n_chain, b = it - c0 * S.n_chain;
    } else
#endif
    {
        b = blockIdx.x / wg_per_block;
        c0 = ((blockIdx.x - b * wg_per_block) * JOB_WAVES + w) * NC;  // the wave's first run
    }
    pod_jobs_item<FUSE>(S, tag, b, c0, it, J.stage, J.gpre_w[w], J.nf_w[w]);
}

// ---------------------------------------------------------------------------
// k_sparse_jobs: the pod jobs of an unfused split tick (a churn tick: a fifth of
// the pods deleted or created, the initial tick's dense shape takes the fused
// k_pod_jobs<true>) from the dirty groups FRONT published (gjob_put): one wave per
// 64-group run of a chain block, lane l the run's group l.  FRONT already
// classified every group against the same state and node flags (its masks are
// what k_pod_jobs<false> derived again), so the run costs two dependent round
// trips: {bases, the run's prefix, its 64 group records}, then {the dirty groups'
// state / spec / creation-time / IP words, the reused addresses of its Gets} (the
// ordinals come from a wave scan of the records' counts), and the stores.  No fill
// marks, node flags or group prefix are read.  The outputs are k_pod_jobs<false>'s,
// byte for byte: DeletePods' list (pod_controller.go:155-183), the patch jobs for
// k_emit in canonical order (configurePod / computePatchData :377-439, the pool's
// Gets, utils.go:83-108), the state transitions.
// ---------------------------------------------------------------------------
constexpr int SJ_WAVES = 4;
__global__ __launch_bounds__(64 * SJ_WAVES, 4) void k_sparse_jobs(DevState S, uint32_t tag, uint32_t blocks_per_chain) {
    // the specs' patch lengths / reservations (len << 16 | max_len), loaded with the
    // first round trip into the wave's LDS: a patch's spec is then no dependent load
    __shared__ uint32_t spec_lm_w[SJ_WAVES][SPEC_LDS];
    const bool spec_lds = S.n_specs <= (uint32_t)SPEC_LDS;
    const uint32_t b = blockIdx.x / blocks_per_chain;
    const uint32_t c = (blockIdx.x - b * blocks_per_chain) * SJ_WAVES + (uint32_t)wave_id();  // the wave's run
    if (b >= S.n_chain || c >= (uint32_t)MAX_WC) return;
    const int l = lane_id();
    uint32_t* spec_lm = spec_lm_w[wave_id()];
    uint32_t spw_l[SPEC_LDS / 64];
#pragma unroll
    for (int q = 0; q < SPEC_LDS / 64; q++) {
        const uint32_t i = (uint32_t)(l + 64 * q);
        spw_l[q] = 0;
        if (spec_lds && i < S.n_specs) {
            const SpecDesc& sd = S.specs[i];
            spw_l[q] = ((uint32_t)sd.len_a + sd.len_b + sd.len_c) << 16 | sd.max_len;
        }
    }
    // round trip 1 (all independent): the block's bases, the run's dirty bit and prefix, its groups
    const JobBase* JB = S.jbase + b;
    const uint32_t jtag = JB->tag;
    const uint32_t dbit = (S.wc_dirty[(size_t)b * WC_DIRTY_WORDS + (c >> 5)] >> (c & 31)) & 1u;
    const uint4 wp = S.wc_pre[(size_t)b * MAX_WC + c];
    const uint4 gj = S.gjob[((size_t)b * MAX_WC + c) * WC_GROUPS + l];
    const uint64_t b_del = JB->del, b_pp = JB->pp, b_bytes = JB->pp_bytes, b_alloc = JB->alloc;
    const uint64_t pod_base = JB->pod_base, alloc_base = JB->alloc_base, take = JB->take, fin = JB->fin, fout0 = JB->fout0;
    if (jtag != tag || !dbit) return;  // the block has no pod jobs this tick / the run is clean
    const bool valid = gj.w == tag;     // (a group clean this tick holds an older record)
    const uint32_t mk = valid ? gj.y : 0u;
    const uint32_t dm = mk & 0xFFu, nm = (mk >> 8) & 0xFFu, am = (mk >> 16) & 0xFFu, j = (mk >> 24) & 63u;
    const uint32_t slot = gj.x;
    uint32_t v[4] = {(uint32_t)__popc(dm), (uint32_t)__popc(nm), valid ? gj.z : 0u, (uint32_t)__popc(am)}, tot[4];
    const uint32_t n_alloc = v[3];
    wave_excl_scan<4>(v, tot);
    const uint64_t o_del = b_del + wp.x + v[0], o_pp = b_pp + wp.y + v[1], o_alloc = b_alloc + wp.w + v[3];
    uint64_t off = pod_base + b_bytes + wp.z + v[2];
    // round trip 2: the group's words; the reused addresses of its Gets (ordinals known)
    uint4 st4 = make_uint4(0, 0, 0, 0), sp4 = st4, ta = st4, tb = st4, ha = st4, hb = st4, pa = st4, pb = st4;
    if (valid) {
        st4 = *reinterpret_cast<const uint4*>(S.pod_state + slot);
        if (nm) {
            sp4 = *reinterpret_cast<const uint4*>(S.pod_spec + slot);
            ta = *reinterpret_cast<const uint4*>(S.pod_ctime + slot);
            tb = *reinterpret_cast<const uint4*>(S.pod_ctime + slot + 4);
            if (mk >> 30 & 1u) {
                ha = *reinterpret_cast<const uint4*>(S.host_ip + slot);
                hb = *reinterpret_cast<const uint4*>(S.host_ip + slot + 4);
            }
            if (mk >> 31) {
                pa = *reinterpret_cast<const uint4*>(S.pod_ip + slot);
                pb = *reinterpret_cast<const uint4*>(S.pod_ip + slot + 4);
            }
        }
    }
    uint32_t areuse[POD_PER_THREAD];
#pragma unroll
    for (int k = 0; k < POD_PER_THREAD; k++) {
        const uint64_t o = o_alloc + (uint32_t)k;
        areuse[k] = ((uint32_t)k < n_alloc && alloc_base + o < take + fin) ? S.alloc_addr[o] : 0u;
    }
#pragma unroll
    for (int q = 0; q < SPEC_LDS / 64; q++) spec_lm[l + 64 * q] = spw_l[q];
    __builtin_amdgcn_wave_barrier();  // (one wave's LDS operations complete in order)
    if (!valid) return;
    const uint32_t stw[4] = {st4.x, st4.y, st4.z, st4.w}, spw[4] = {sp4.x, sp4.y, sp4.z, sp4.w};
    const uint32_t ctm[POD_PER_THREAD] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
    const uint32_t hipk[POD_PER_THREAD] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
    const uint32_t ip0[POD_PER_THREAD] = {pa.x, pa.y, pa.z, pa.w, pb.x, pb.y, pb.z, pb.w};
    auto st_of = [&](int k) { return (uint16_t)(stw[k >> 1] >> (16 * (k & 1))); };
    auto sp_of = [&](int k) { return (uint16_t)(spw[k >> 1] >> (16 * (k & 1))); };
    // the spec lengths (LDS; else one descriptor when the group's patched pods share a spec)
    uint32_t sd_len[POD_PER_THREAD], sd_max[POD_PER_THREAD];
    if (spec_lds) {
#pragma unroll
        for (int k = 0; k < POD_PER_THREAD; k++) {
            const uint32_t lm = (nm >> k) & 1u ? spec_lm[sp_of(k)] : 0u;
            sd_len[k] = lm >> 16, sd_max[k] = lm & 0xFFFFu;
        }
    } else {
        bool one = true;
#pragma unroll
        for (int k = 0; k < POD_PER_THREAD; k++) one &= !((nm >> k) & 1u) || sp_of(k) == sp_of(__builtin_ctz(nm | 256u) & 7);
        if (nm && one) {
            const SpecDesc& sd = S.specs[sp_of(__builtin_ctz(nm) & 7)];
            const uint32_t ln = (uint32_t)sd.len_a + sd.len_b + sd.len_c, mx = sd.max_len;
#pragma unroll
            for (int k = 0; k < POD_PER_THREAD; k++) sd_len[k] = ln, sd_max[k] = mx;
        } else {
#pragma unroll
            for (int k = 0; k < POD_PER_THREAD; k++) {
                sd_len[k] = sd_max[k] = 0;
                if ((nm >> k) & 1u) {
                    const SpecDesc& sd = S.specs[sp_of(k)];
                    sd_len[k] = (uint32_t)sd.len_a + sd.len_b + sd.len_c;
                    sd_max[k] = sd.max_len;
                }
            }
        }
    }
    uint32_t bk0, nbk;
    block_range(S, b, bk0, nbk);
    const uint32_t gb = bk0 + j;
    const int32_t h0 = (int32_t)((S.b_lo + gb) * S.pod_stride + (slot - gb * S.cp));
    uint64_t od = o_del, op = o_pp;
    uint32_t ai = 0;
    uint32_t nst[POD_PER_THREAD], nh[POD_PER_THREAD], np[POD_PER_THREAD];
    bool dirty = false, wh = false, wpi = false;
#pragma unroll
    for (int k = 0; k < POD_PER_THREAD; k++) {
        const int32_t handle = h0 + k;
        const uint16_t s0 = st_of(k);
        uint16_t s = s0;
        nh[k] = hipk[k], np[k] = ip0[k];
        if ((dm >> k) & 1u) {
            S.del_pods[od] = handle;
            S.del_fin[od] = (s & PS_HAS_FIN) ? 1 : 0;
            od++;
            s = 0;  // DeletePod -> Delete(grace 0): the object is gone
        } else if (s & PS_USED) {
            if ((nm >> k) & 1u) {
                uint32_t pip = ip0[k];
                if ((am >> k) & 1u) {  // the lane's a-th Get (ordinal o_alloc + a)
                    const uint32_t a = ai++;
                    const uint64_t gidx = alloc_base + o_alloc + a;
                    uint32_t ra = areuse[0];
#pragma unroll
                    for (int q = 1; q < POD_PER_THREAD; q++) ra = a == (uint32_t)q ? areuse[q] : ra;
                    pip = gidx < take + fin ? ra : (uint32_t)(fout0 + (gidx - take - fin));
                }
                const bool stat = s & PS_STATUS_NONEMPTY;
                uint32_t hip = 0;
                if (stat) {
                    hip = (s & PS_HAS_HOST_IP) ? hipk[k] : S.node_ip;
                    if (!(s & PS_HAS_HOST_IP)) nh[k] = hip, wh = true;
                    if (pip != ip0[k]) np[k] = pip, wpi = true;
                }
                const uint32_t len = sd_len[k] + (stat ? 23u + ip_len(hip) + ip_len(pip) : 0u);
                S.pp_pods[op] = handle;
                S.pp_len[op] = len;
                S.pp_off[op] = off;
                S.pp_job[op] = make_uint4(stat ? pip : 0u, hip, ctm[k], sp_of(k));
                op++;
                off += sd_max[k];
                // the apiserver applied the patch
                s = (uint16_t)((s & ~PS_PHASE_MASK) | (PHASE_RUNNING << PS_PHASE_SHIFT) | PS_CONFORMS | PS_STATUS_NONEMPTY |
                               (stat ? PS_HAS_HOST_IP : 0));
                if (stat) s = (uint16_t)((s & ~PS_IP_BITS) | ip_state_bits(S.pool, pip));
            }
            s &= (uint16_t)~PS_EVENT;  // (a live pod with an event is evaluated)
        }
        dirty |= s != s0;
        nst[k] = s;
    }
    if (wh) {
        *reinterpret_cast<uint4*>(S.host_ip + slot) = make_uint4(nh[0], nh[1], nh[2], nh[3]);
        *reinterpret_cast<uint4*>(S.host_ip + slot + 4) = make_uint4(nh[4], nh[5], nh[6], nh[7]);
    }
    if (wpi) {
        *reinterpret_cast<uint4*>(S.pod_ip + slot) = make_uint4(np[0], np[1], np[2], np[3]);
        *reinterpret_cast<uint4*>(S.pod_ip + slot + 4) = make_uint4(np[4], np[5], np[6], np[7]);
    }
    if (dirty)
        *reinterpret_cast<uint4*>(S.pod_state + slot) =
            make_uint4(nst[0] | nst[1] << 16, nst[2] | nst[3] << 16, nst[4] | nst[5] << 16, nst[6] | nst[7] << 16);
}

// init_blocks: the fused launch's node-init blocks (0: k_emit writes the node inits)
void launch_pod_jobs(const DevState& S, uint32_t tag, hipStream_t st, uint32_t init_blocks, uint64_t now, uint64_t start,
                     hipEvent_t t0, hipEvent_t t1) {
    // the largest chain block's runs: its buckets x their capacity in 8-slot groups
    const uint32_t bpb = (S.nb + S.n_chain - 1) / S.n_chain;
    const uint32_t runs = cdiv((uint64_t)bpb * (S.cp / POD_PER_THREAD), WC_GROUPS);
    if (S.sparse_jobs && !S.fuse_pods) {
        const uint32_t bpc = cdiv(runs < (uint32_t)MAX_WC ? runs : (uint32_t)MAX_WC, SJ_WAVES);
        if (t0)
            hipExtLaunchKernelGGL(k_sparse_jobs, dim3(S.n_chain * bpc), dim3(64 * SJ_WAVES), 0, st, t0, t1, 0, S, tag, bpc);
        else hipLaunchKernelGGL(k_sparse_jobs, dim3(S.n_chain * bpc), dim3(64 * SJ_WAVES), 0, st, S, tag, bpc);
        return;
    }
    uint32_t wpb = cdiv(cdiv(runs < (uint32_t)MAX_WC ? runs : (uint32_t)MAX_WC, S.fuse_pods ? 1 : JOB_NC), JOB_WAVES);
    wpb = wpb ? wpb : 1u;
    const uint32_t pod_blocks = S.n_chain * wpb, grid = pod_blocks + (S.fuse_pods ? init_blocks : 0u);
    auto kern = S.fuse_pods ? k_pod_jobs<true> : k_pod_jobs<false>;
    if (t0)
        hipExtLaunchKernelGGL(kern, dim3(grid), dim3(64 * JOB_WAVES), 0, st, t0, t1, 0, S, tag, wpb, pod_blocks, now, start);
    else hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * JOB_WAVES), 0, st, S, tag, wpb, pod_blocks, now, start);
}

int emit_occupancy() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_emit, EMIT_BLOCK, 0) != hipSuccess) return 0;
    return n;
}

int tick_occupancy() {
    int n = 0, m = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k_tick<false>, BLOCK, 0) != hipSuccess) return 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&m, k_tick<true>, BLOCK, 0) != hipSuccess) return 0;
    return std::min(n, m);
}

}  // namespace kwok
