// param.hip -- k_pq: the cooperative owner of a hot-parameter resource's segment.
//
// A resource whose rules are all QPS-grade ParamFlowRules (passDefaultLocalCheck / passThrottleLocalCheck with a
// fixed paramIdx; no flow or degrade rules, engine.cpp PF_PQ) is decided by one workgroup per segment instead of
// one lane.  The reference runs, per ENTRY (param/slots/HotParamSlotChainBuilder.java:38-51):
//   ParamFlowSlot.checkFlow  -- every rule in order, each a CacheMap access of the rule's (time, token) map for
//                               the argument value, first block wins (ParamFlowSlot.java:77-101,
//                               ParamFlowChecker.java:121-248);
//   StatisticSlot            -- pass / block counters, curThreadNum (StatisticSlot.java:54-133);
//   ParamFlowStatisticEntryCallback.onPass -- the thread-count map's access for the value (ParameterMetric.java:126-149)
// and per EXIT StatisticSlot.exit.  Nothing reads the node's windows (no flow / degrade rule), so the statistics
// are a reduction per 500 ms bucket, and a value's param state depends only on the earlier checks of the same
// (rule, value) -- SURVEY.md §8(a) P3 -- except through LRU residency: whether a value is still in its
// capacity-bounded map depends on every value accessed since.
//
// Residency without a sequential walk: a map holds the `cap` most recently used keys, so an access to key v hits
// iff v was live at the tile start with recency rank r (r live keys more recent) and fewer than cap distinct keys
// were accessed in between:
//     D = r + #{ first accesses j of the tile before this one : key_j was not live, or had rank > r } < cap,
// and any repeat of a key inside the tile hits (a tile holds < cap accesses).  Ranks are popcounts over the map's
// live-stamp ring (pmap.h), held in LDS for the whole segment.  So a tile of accesses is decided at once:
//   sort the tile's accesses by (key, position) in LDS; group leaders probe the map (cuckoo buckets in HBM / L2);
//   D from the leaders' ranks (an upper bound r + #earlier leaders settles nearly all); one lane per key group walks
//   its accesses in order through the token bucket / throttle (only same-key state is involved); then the group's
//   new stamp, values and ring bits are committed, the oldest untouched keys beyond cap evicted (their ring bits
//   cleared) and new keys placed in free or dead slots.
// The thread-count map of paramIdx 0 is updated the same way from the tile's passed ENTRYs (count + 1, or 1 for a
// key that was not live).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "chain.h"
#include "pmap.h"

using namespace sg;

#define PQ_MAXP 4          // param rules of a k_pq resource (engine.cpp PF_PQ)
#define PQ_RBW 512         // ring words a map may have (2^15 bits: capacity <= 8176, durationInSec <= 2)
#define PQ_EPL 2           // events per lane per tile
#define PQ_NPEND 64        // keys waiting for a displacement walk per tile (more: BF_PTAB_FULL)
#define PQ_CLW 256         // claim bitmap words (>= buckets * 8 / 64 for capacity <= 8176)
#define RANK_REP (-1)      // not a first access of its key in the tile
#define RANK_NEW 0x7FFFFFFF

template <int NW>
struct PqSh {
    static constexpr uint32_t HW = NW * 64;
    static constexpr uint32_t TE = HW * PQ_EPL;
    Node node;
    DRule rules[PQ_MAXP];
    PMap hdr[PQ_MAXP + 1];          // rule maps, then the thread-count map of paramIdx 0
    uint32_t mid[PQ_MAXP + 1];
    uint64_t bm[PQ_MAXP + 1][PQ_RBW];
    uint32_t wpre[PQ_RBW];          // live stamps before each ring word (stamp order from thr)
    uint64_t claim[PQ_CLW];
    uint64_t tkey[TE];              // tile event -> argument key
    int32_t tdt[TE];                // tile event -> time - t0
    uint32_t tcz[TE];               // tile event -> count | rt << 16
    uint32_t tkx[TE];               // tile event -> kind | flags << 8 | code << 16 (kind 0xFF: past the segment)
    uint32_t tx[TE];                // tile event -> SEv.x (EXIT / TRACE reference)
    int32_t lrank[TE];              // tile event -> RANK_* or the leader's rank at the tile start
    uint32_t tA[TE];                // tile event -> accesses of the map before it in the tile
    uint32_t tver[TE];              // tile event -> walk verdict (by sorted position first)
    uint32_t tdec[TE];              // tile event -> decision word (EXIT references inside the tile)
    uint64_t skey[TE];
    uint32_t sidx[TE];
    uint32_t olist[TE];             // residency: live first accesses at the LRU end (tile position << 12 | rank)
    uint32_t sorted_n;              // skey / sidx hold the last map phase's accesses sorted by (key, position): how many
    uint32_t red[NW][8];
    int64_t red64[NW][2];
    uint32_t flags_or, npend;
    uint32_t freach;                // segment position + 1 of the tile's first ENTRY reaching rule k0
    uint64_t pend_key[PQ_NPEND];
    int64_t pend_stamp[PQ_NPEND];
    PData pend_dat[PQ_NPEND];
#ifdef SG_KPROF
    unsigned long long pt[16];      // phase cycles (thread 0's view; tools/pqprobe.py)
    unsigned long long pt_t;
#endif
};

__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// SG_KPROF builds: thread 0 charges the cycles since the last mark to phase k (call after a barrier)
#ifdef SG_KPROF
#define PQ_MARK(k)                                                  \
    if (threadIdx.x == 0) {                                         \
        const unsigned long long _n = __builtin_amdgcn_s_memtime(); \
        sh.pt[k] += _n - sh.pt_t;                                   \
        sh.pt_t = _n;                                               \
    }
#else
#define PQ_MARK(k)
#endif
__device__ __forceinline__ uint64_t ld64(const void* p) {
    return __hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int64_t uni64_pq(int64_t v) {  // LDS-broadcast value as a provably uniform scalar
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(uint64_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t ld32(const void* p) {
    return __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A key's slot in its two buckets (-1: absent).  All eight keys of a bucket are loaded before any is compared:
// a compare-and-exit loop would make each load wait for the previous one (eight HBM / L2 round trips).
__device__ __forceinline__ int32_t pq_find(const PBucket* B, uint32_t b1, uint32_t b2, uint64_t key) {
    uint64_t k1[PM_BKT], k2[PM_BKT];  // both buckets in one round of loads (most probes of a churning map miss)
#pragma unroll
    for (int j = 0; j < PM_BKT; ++j) {
        k1[j] = ld64(&B[b1].key[j]);
        k2[j] = ld64(&B[b2].key[j]);
    }
    int32_t r = -1;
#pragma unroll
    for (int j = PM_BKT - 1; j >= 0; --j)
        if (k2[j] == key) r = (int32_t)(b2 * PM_BKT + j);
#pragma unroll
    for (int j = PM_BKT - 1; j >= 0; --j)
        if (k1[j] == key) r = (int32_t)(b1 * PM_BKT + j);
    return r;
}
__device__ __forceinline__ bool ring_live(const PMap& m, const uint64_t* bm, int64_t s);
// bit j: slot j of bucket b is free (never used, or its key's stamp is dead by the ring), keys and stamps loaded at once
__device__ __forceinline__ uint32_t pq_free_mask(const PBucket* B, uint32_t b, const PMap& m, const uint64_t* bm) {
    uint64_t k[PM_BKT];
    int64_t st[PM_BKT];
#pragma unroll
    for (int j = 0; j < PM_BKT; ++j) {
        k[j] = ld64(&B[b].key[j]);
        st[j] = (int64_t)ld64(&B[b].stamp[j]);
    }
    uint32_t f = 0;
#pragma unroll
    for (int j = 0; j < PM_BKT; ++j)
        if (k[j] == PK_EMPTY || !ring_live(m, bm, st[j])) f |= 1u << j;
    return f;
}

// exclusive block scan of one u32 per lane; *tot = block total (uniform)
template <int NW>
__device__ __forceinline__ uint32_t pq_scan(PqSh<NW>& sh, uint32_t v, uint32_t* tot) {
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
        if (l >= (uint32_t)o) x += y;
    }
    if (l == 63) sh.red[w][7] = x;
    __syncthreads();
    uint32_t pre = 0, t = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const uint32_t c = sh.red[k][7];
        if ((uint32_t)k < w) pre += c;
        t += c;
    }
    __syncthreads();
    *tot = t;
    return pre + x - v;
}

// ring helpers on the LDS copy of map k
__device__ __forceinline__ uint32_t ring_word(const PMap& m, int64_t s) {
    return (uint32_t)(((uint64_t)s & (uint64_t)((1ull << m.rb_log2) - 1)) >> 6);
}
__device__ __forceinline__ bool ring_live(const PMap& m, const uint64_t* bm, int64_t s) {
    if (s < m.thr || s >= m.clock) return false;
    const uint64_t p = (uint64_t)s & (uint64_t)((1ull << m.rb_log2) - 1);
    return ((bm[p >> 6] >> (p & 63)) & 1ull) != 0;
}

// Tighten thr to the lowest live stamp; renumber the live stamps densely (pm_compact, in parallel) when the ring
// would otherwise wrap onto a live stamp within the next `k` stamps.
// wpre[w] = live stamps in the W ring words before word w, in stamp order from word w0 (a thread takes
// ceil(W / lanes) consecutive words: W can exceed the 256-lane owner's lanes)
template <int NW>
__device__ __forceinline__ void pq_word_ranks(PqSh<NW>& sh, int mk, uint32_t w0, uint32_t W) {
    constexpr uint32_t HW = PqSh<NW>::HW;
    const uint32_t per = (W + HW - 1) / HW, l0 = threadIdx.x * per;
    uint32_t c = 0;
    for (uint32_t u = 0; u < per; ++u)
        if (l0 + u < W) c += (uint32_t)__popcll(sh.bm[mk][(w0 + l0 + u) & (W - 1)]);
    uint32_t tot;
    uint32_t run = pq_scan<NW>(sh, c, &tot);
    for (uint32_t u = 0; u < per; ++u)
        if (l0 + u < W) {
            const uint32_t w = (w0 + l0 + u) & (W - 1);
            sh.wpre[w] = run;
            run += (uint32_t)__popcll(sh.bm[mk][w]);
        }
}
template <int NW>
__device__ void pq_reserve(PqSh<NW>& sh, int mk, const DevState& S, uint32_t k) {
    PMap& m = sh.hdr[mk];
    const int64_t RB = (int64_t)1 << m.rb_log2;
    const uint32_t W = (uint32_t)(RB >> 6);
    if (m.clock + (int64_t)k - m.thr <= RB - 64) return;  // uniform (LDS header)
    __syncthreads();
    if (threadIdx.x == 0) m.thr = pm_first_live(m, sh.bm[mk], m.thr);
    __syncthreads();
    if (m.clock + (int64_t)k - m.thr <= RB - 64) return;
    // ranks of the live stamps in stamp order
    pq_word_ranks<NW>(sh, mk, ring_word(m, m.thr), W);
    __syncthreads();
    const int64_t base = m.clock - (int64_t)m.live;
    PBucket* B = S.pbkt + m.base;
    const uint32_t nslot = m.nb * PM_BKT;
    for (uint32_t i = threadIdx.x; i < nslot; i += PqSh<NW>::HW) {
        const uint32_t b = i / PM_BKT, j = i % PM_BKT;
        const uint64_t key = ld64(&B[b].key[j]);
        const int64_t s = (int64_t)ld64(&B[b].stamp[j]);
        if (key == PK_EMPTY) continue;
        if (!ring_live(m, sh.bm[mk], s)) {  // a dead slot's stamp may fall in the renumbered range: retire it
            B[b].stamp[j] = PM_DEAD;
            continue;
        }
        const uint64_t p = (uint64_t)s & (uint64_t)(RB - 1);
        const uint32_t rk = sh.wpre[p >> 6] + (uint32_t)__popcll(sh.bm[mk][p >> 6] & ((1ull << (p & 63)) - 1ull));
        B[b].stamp[j] = base + (int64_t)rk;
    }
    __syncthreads();
    for (uint32_t w = threadIdx.x; w < W; w += PqSh<NW>::HW) sh.bm[mk][w] = 0;
    __syncthreads();
    for (int64_t s = base + threadIdx.x; s < m.clock; s += PqSh<NW>::HW) {
        const uint64_t p = (uint64_t)s & (uint64_t)(RB - 1);
        atomicOr(reinterpret_cast<unsigned long long*>(&sh.bm[mk][p >> 6]), 1ull << (p & 63));
    }
    __syncthreads();
    if (threadIdx.x == 0) m.thr = base;
    __syncthreads();
}

// one bitonic compare-exchange stage (k, j) over LDS pairs [0, P)
template <int NW>
__device__ __forceinline__ void pq_sort_stage(PqSh<NW>& sh, uint32_t P, uint32_t k, uint32_t j) {
    for (uint32_t i = threadIdx.x; i < P / 2; i += PqSh<NW>::HW) {
        const uint32_t lo = 2 * j * (i / j) + (i % j), hi = lo + j;
        const bool up = (lo & k) == 0;
        const uint64_t ka = sh.skey[lo], kb = sh.skey[hi];
        const uint32_t ia = sh.sidx[lo], ib = sh.sidx[hi];
        const bool gt = ka > kb || (ka == kb && ia > ib);
        if (gt == up) {
            sh.skey[lo] = kb; sh.skey[hi] = ka;
            sh.sidx[lo] = ib; sh.sidx[hi] = ia;
        }
    }
    lds_sync();
}
// (key, idx) of the lane l ^ m of this wave
__device__ __forceinline__ void pq_xchg(uint64_t k, uint32_t i, uint32_t m, uint64_t& tk, uint32_t& ti) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)k, (int)m, 64);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(k >> 32), (int)m, 64);
    ti = (uint32_t)__shfl_xor((int)i, (int)m, 64);
    tk = ((uint64_t)hi << 32) | lo;
}
// element e keeps the smaller of (mine, theirs) iff it is the lower position of its pair in an ascending block
__device__ __forceinline__ void pq_keep(uint64_t& mk, uint32_t& mi, uint64_t tk, uint32_t ti, bool keep_min) {
    const bool mine_lt = mk < tk || (mk == tk && mi < ti);
    if (mine_lt != keep_min) { mk = tk; mi = ti; }
}
// Bitonic sort of (skey, sidx) pairs [0, P) in LDS, P a power of two.  From P >= 128 a wave holds 128 consecutive
// elements in registers (two a lane): the stages whose partners are less than 128 apart run as register / lane
// exchanges without a block barrier; only the stages across waves (j >= 128: 10 of the 66 for P = 2048) go
// through LDS.
template <int NW>
__device__ void pq_sort(PqSh<NW>& sh, uint32_t P) {
    if (P < 128) {
        for (uint32_t k = 2; k <= P; k <<= 1)
            for (uint32_t j = k >> 1; j > 0; j >>= 1) pq_sort_stage<NW>(sh, P, k, j);
        return;
    }
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t e0 = w * 128 + 2 * lane;
    const bool act = e0 < P;
    uint64_t ka = 0, kb = 0;
    uint32_t ia = 0, ib = 0;
    if (act) { ka = sh.skey[e0]; ia = sh.sidx[e0]; kb = sh.skey[e0 + 1]; ib = sh.sidx[e0 + 1]; }
    for (uint32_t k = 2; k <= P; k <<= 1) {
        uint32_t j = k >> 1;
        if (j >= 128) {
            lds_sync();  // every wave is done reading the lists it loaded
            if (act) { sh.skey[e0] = ka; sh.sidx[e0] = ia; sh.skey[e0 + 1] = kb; sh.sidx[e0 + 1] = ib; }
            lds_sync();
            for (; j >= 128; j >>= 1) pq_sort_stage<NW>(sh, P, k, j);
            if (act) { ka = sh.skey[e0]; ia = sh.sidx[e0]; kb = sh.skey[e0 + 1]; ib = sh.sidx[e0 + 1]; }
        }
        for (; j >= 2; j >>= 1) {  // partner lane l ^ (j / 2), same parity
            uint64_t tk;
            uint32_t ti;
            pq_xchg(ka, ia, j >> 1, tk, ti);
            pq_keep(ka, ia, tk, ti, ((e0 & k) == 0) == ((e0 & j) == 0));
            pq_xchg(kb, ib, j >> 1, tk, ti);
            pq_keep(kb, ib, tk, ti, (((e0 + 1) & k) == 0) == (((e0 + 1) & j) == 0));
        }
        {   // j = 1: the lane's own pair
            const bool up = (e0 & k) == 0;
            const bool gt = ka > kb || (ka == kb && ia > ib);
            if (gt == up) {
                const uint64_t x = ka; ka = kb; kb = x;
                const uint32_t y = ia; ia = ib; ib = y;
            }
        }
    }
    lds_sync();
    if (act) { sh.skey[e0] = ka; sh.sidx[e0] = ia; sh.skey[e0 + 1] = kb; sh.sidx[e0 + 1] = ib; }
    lds_sync();
}

enum { PW_TOKEN = 0, PW_THROTTLE = 1, PW_COUNT = 2 };
// thread-count map operations of a tile event (PW_COUNT; tkx bits 24-26), ParameterMetric.java:117-241:
//   OP_ADD   addThreadCount of a passed ENTRY: putIfAbsent(v, 0) then increment, or put(v, 1) when absent;
//   OP_CHK   a THREAD-grade rule's check (ParamFlowChecker.java:101-119): get(v) (a touch if present), pass iff
//            count + 1 <= threshold, then OP_ADD for the entry that passed (the rule is the resource's last);
//   OP_SUB   decreaseThreadCount of an EXIT: putIfAbsent(v, 0) -- an absent value stays at 0 -- else decrement,
//            removed at <= 0;
//   OP_SUBC  OP_SUB iff the referenced ENTRY (same tile, same key) passed its OP_CHK.
enum { OP_NONE = 0, OP_ADD = 1, OP_CHK = 2, OP_SUB = 3, OP_SUBC = 4 };
#define TV_BLOCK 1u      // walk verdict: blocked
#define TV_HIT 4u        // leader event: its key was resident at its first access
#define TV_INS 0x100u    // the access inserted its key
#define TV_REM 0x200u    // the access removed its key
#define GS_PRES 0x80000000u
#define GS_TOUCH 0x40000000u
#define GS_CNT 0x3FFFFFFFu

__device__ __forceinline__ uint32_t pq_op(uint32_t kx) { return (kx >> 24) & 7u; }

// the threshold of a THREAD-grade rule for value v: its hot item, else (long) count
__device__ __forceinline__ int64_t pq_thread_thr(const DevState& S, const DRule* r, uint64_t v) {
    for (uint32_t i = 0; i < r->hot_n; ++i) {
        const DHot h = S.hot[r->hot_off + i];
        if (h.key == v) return (int64_t)h.count;
    }
    return j_d2l(r->count);
}

// one access of a thread-count map by the state machine of its op; returns TV_* bits
__device__ __forceinline__ uint32_t pq_count_op(uint32_t op, bool& pres, int64_t& c, int64_t thr) {
    if (op == OP_ADD || op == OP_CHK) {
        if (op == OP_CHK && (pres ? c : 0) + 1 > thr) return TV_BLOCK;  // the get only
        if (pres) { ++c; return 0; }
        pres = true; c = 1;
        return TV_INS;
    }
    if (op == OP_SUB) {
        if (!pres) { pres = true; c = 0; return TV_INS; }
        if (--c <= 0) { pres = false; c = 0; return TV_REM; }
    }
    return 0;
}

// Exact sequential residency of one thread-count map's tile (one lane, in LDS): ops in tile order, each
// insertion beyond cap evicting the oldest untouched key (the lowest live ring bit).  An access touches its key
// (moves it to the MRU end) unless it does nothing: an EXIT whose ENTRY was blocked, a blocked check of an absent
// value.  Taken only when the no-eviction hypothesis fails.  Leaves on every group leader whether the key was
// resident at the group's first touching access (TV_HIT), the touched / evicted keys' ring bits cleared, and
// returns the map's size at the tile end.
template <int NW>
__device__ __noinline__ uint32_t pq_count_seq(PqSh<NW>& sh, int mk, const DRule* r, const DevState& S, uint32_t tbase) {
    PMap& m = sh.hdr[mk];
    const int64_t RB = (int64_t)1 << m.rb_log2;
    const uint32_t W = (uint32_t)(RB >> 6);
    const uint32_t w0 = ring_word(m, m.thr);
    uint64_t* bm = sh.bm[mk];
    int64_t size = m.live;
    uint32_t kw = 0;
    for (uint32_t e = 0; e < PqSh<NW>::TE; ++e) {
        uint32_t op = pq_op(sh.tkx[e]);
        if (op == OP_NONE) continue;
        const uint32_t g = (uint32_t)sh.lrank[e];
        const uint32_t gs = sh.tdec[g];
        const bool touched = (gs & GS_TOUCH) != 0;
        bool pres, live_bit = false;
        int64_t c;
        const int64_t st = (int64_t)sh.tkey[g];
        if (!touched) {  // resident iff its ring bit survived the evictions so far
            live_bit = st >= 0 && ring_live(m, bm, st);
            pres = live_bit;
            c = pres ? (int64_t)(gs & GS_CNT) : 0;
        } else {
            pres = (gs & GS_PRES) != 0;
            c = (int64_t)(gs & GS_CNT);
        }
        if (op == OP_SUBC) op = (sh.tver[sh.tx[e] - tbase] & TV_BLOCK) ? OP_NONE : OP_SUB;
        const bool pb = pres;
        const uint32_t v = pq_count_op(op, pres, c, op == OP_CHK ? pq_thread_thr(S, r, sh.skey[g]) : 0);
        sh.tver[e] = (sh.tver[e] & TV_HIT) | v;
        const bool t_now = op != OP_NONE && (pb || (v & TV_INS));
        if (t_now && !touched) {
            if (live_bit) {
                const uint64_t p = (uint64_t)st & (uint64_t)(RB - 1);
                bm[p >> 6] &= ~(1ull << (p & 63));
            }
            if (pb) sh.tver[sh.sidx[g]] |= TV_HIT;  // read by the leader's walk
        }
        if (v & TV_INS) ++size;
        if (v & TV_REM) --size;
        if (size > (int64_t)m.cap) {  // evict the oldest untouched key
            while (kw < W) {
                const uint32_t w = (w0 + kw) & (W - 1);
                const uint64_t x = bm[w];
                if (x) { bm[w] = x & (x - 1); break; }
                ++kw;
            }
            --size;
        }
        if (touched || t_now) sh.tdec[g] = (pres ? GS_PRES : 0u) | GS_TOUCH | ((uint32_t)c & GS_CNT);
    }
    return (uint32_t)size;
}

// One map's accesses of the tile (acc[e] for the lane's events e = tid * PQ_EPL + q): residency, the walk of
// every key group (WALK), commit.  Verdicts of the walks land in sh.tver[e]: TV_BLOCK | wait << 16.
// tbase: segment position of the tile's first event (OP_SUBC references).
// presorted (a thread-count map of increments only): the accesses are the passed subset of the last rule map
// phase's accesses, with the same keys, so its sorted list is kept as it is instead of sorting again.
template <int NW>
__device__ __noinline__ void pq_map_phase(PqSh<NW>& sh, int mk, int walk, const DRule* r, const DevState& S, int64_t t0,
                                          uint32_t tbase, const bool (&acc)[PQ_EPL], uint32_t* bflags,
                                          bool force_seq = false, bool presorted = false) {
    constexpr uint32_t HW = PqSh<NW>::HW;
    constexpr uint32_t SP = PqSh<NW>::TE / HW;  // sorted positions per lane
    const uint32_t tid = threadIdx.x;
    // (a) accesses before each event, in tile order
    uint32_t la = 0;
    bool rm_l = false, nacq1 = false;
#pragma unroll
    for (int q = 0; q < PQ_EPL; ++q) {
        la += acc[q] ? 1u : 0u;
        if (acc[q] && walk == PW_COUNT && pq_op(sh.tkx[tid * PQ_EPL + q]) != OP_ADD) rm_l = true;
        if (acc[q] && (sh.tcz[tid * PQ_EPL + q] & 0xFFFFu) != 1u) nacq1 = true;
    }
    uint32_t na;
    uint32_t a0 = pq_scan<NW>(sh, la, &na);
    const uint32_t prev_n = sh.sorted_n;  // read before any lane rewrites it (pq_scan ends with a barrier)
    __syncthreads();
    if (tid == 0) sh.sorted_n = na;
    if (na == 0) return;  // uniform
    // a thread-count tile with gets or decrements: residency by the no-eviction hypothesis, verified after the
    // walks (the rank rule below counts every first access as an insertion and knows no removals)
    const bool rmode = __syncthreads_or(rm_l) != 0;
    const bool all_acq1 = __syncthreads_or(nacq1) == 0;  // every access acquires 1 (the walks' closed forms)
    const bool keep_sorted = presorted && !rmode;
#pragma unroll
    for (int q = 0; q < PQ_EPL; ++q) {
        const uint32_t e = tid * PQ_EPL + q;
        sh.tA[e] = a0;
        sh.lrank[e] = RANK_REP;
        if (keep_sorted) sh.olist[e] = acc[q] ? 1u : 0u;
        else if (acc[q]) { sh.skey[a0] = sh.tkey[e]; sh.sidx[a0] = e; }
        if (acc[q]) ++a0;
    }
    uint32_t P = 64;
    while (P < na) P <<= 1;
    if (keep_sorted) {
        // stable compaction of the previous sorted list to this phase's accesses (lanes own consecutive positions)
        __syncthreads();
        uint64_t kk[PQ_EPL];
        uint32_t ki[PQ_EPL], nk = 0;
#pragma unroll
        for (int q = 0; q < PQ_EPL; ++q) {
            const uint32_t s0 = tid * PQ_EPL + q;
            ki[q] = s0 < prev_n ? sh.sidx[s0] : 0xFFFFFFFFu;
            kk[q] = s0 < prev_n ? sh.skey[s0] : PK_EMPTY;
            if (ki[q] != 0xFFFFFFFFu && sh.olist[ki[q]]) ++nk;
            else ki[q] = 0xFFFFFFFFu;
        }
        uint32_t tot;
        uint32_t o = pq_scan<NW>(sh, nk, &tot);  // (its barriers: every lane has read the old list)
#pragma unroll
        for (int q = 0; q < PQ_EPL; ++q)
            if (ki[q] != 0xFFFFFFFFu) { sh.skey[o] = kk[q]; sh.sidx[o] = ki[q]; ++o; }
        if (tot != na) atomicOr(bflags, BF_PQ_INVARIANT);  // not the subset it must be: fails the engine loudly
    }
    for (uint32_t i = na + tid; i < P; i += HW) { sh.skey[i] = PK_EMPTY; sh.sidx[i] = 0xFFFFFFFFu; }
    pq_reserve<NW>(sh, mk, S, na);
    __syncthreads();
    PQ_MARK(1)
    if (!keep_sorted) pq_sort<NW>(sh, P);
    PQ_MARK(2)
    PMap& m = sh.hdr[mk];
    const int64_t RB = (int64_t)1 << m.rb_log2;
    const uint32_t W = (uint32_t)(RB >> 6);
    const int64_t clock0 = m.clock;
    const uint32_t live0 = m.live, cap = m.cap;
    pq_word_ranks<NW>(sh, mk, ring_word(m, m.thr), W);  // ranks: live stamps before each ring word, from thr
    __syncthreads();
    // (b) group leaders probe the map; their ranks by tile event
    PBucket* B = S.pbkt + m.base;
    PData* D = S.pdat + m.base * PM_BKT;
    int32_t gslot[SP];
    bool glive[SP], glead[SP];
    int64_t gst[SP];
    PData gd[SP];
#pragma unroll
    for (uint32_t q = 0; q < SP; ++q) {
        const uint32_t s = tid + q * HW;
        glead[q] = false; glive[q] = false; gslot[q] = -1; gst[q] = 0;
        gd[q].v0 = 0; gd[q].v1 = 0; gd[q].pad = 0;
        if (s >= na) continue;
        const uint64_t key = sh.skey[s];
        if (s > 0 && sh.skey[s - 1] == key) continue;
        glead[q] = true;
        uint32_t b1, b2;
        pm_buckets(m.nb, key, b1, b2);
        gslot[q] = pq_find(B, b1, b2, key);
        int32_t rank = RANK_NEW;
        if (gslot[q] >= 0) {
            // the stamp and the slot's values in one round of loads (the values are used only if the stamp is live)
            const uint64_t* dp = reinterpret_cast<const uint64_t*>(&D[gslot[q]]);
            gst[q] = (int64_t)ld64(&B[gslot[q] / PM_BKT].stamp[gslot[q] % PM_BKT]);
            const int64_t dv0 = (int64_t)ld64(dp);
            const uint64_t dv1 = ld64(dp + 1);
            glive[q] = ring_live(m, sh.bm[mk], gst[q]);
            if (glive[q]) {
                const uint64_t p = (uint64_t)gst[q] & (uint64_t)(RB - 1);
                const uint32_t below = sh.wpre[p >> 6] + (uint32_t)__popcll(sh.bm[mk][p >> 6] & ((1ull << (p & 63)) - 1ull));
                rank = (int32_t)(live0 - below - 1);
                gd[q].v0 = dv0;
                gd[q].v1 = (int32_t)(uint32_t)dv1;
            }
        }
        sh.lrank[sh.sidx[s]] = rank;
    }
    __syncthreads();
    PQ_MARK(3)
    // (c) residency of every first access: the upper bound r + (first accesses before it) settles it unless the key
    // is near the LRU end; then the exact count of the earlier first accesses of keys older than it
    if (!rmode) {
        // D = rk + N + G: N the tile's earlier first accesses of keys that were not live, G those of live keys older
        // than this one (rank > rk).  G only matters when rk + F >= cap, i.e. rk >= cap - nf, so only live first
        // accesses ranked >= cap - nf (the LRU end: few, old keys are rarely accessed again) are listed, in tile
        // order, and G is counted over that list instead of over the whole tile.
        uint32_t lf = 0, ln = 0;
#pragma unroll
        for (int q = 0; q < PQ_EPL; ++q) {
            const int32_t rk = sh.lrank[tid * PQ_EPL + q];
            lf += rk != RANK_REP ? 1u : 0u;
            ln += rk == RANK_NEW ? 1u : 0u;
        }
        uint32_t nf, nn;
        uint32_t F = pq_scan<NW>(sh, lf, &nf);
        uint32_t N = pq_scan<NW>(sh, ln, &nn);
        const uint32_t rlo = nf < cap ? cap - nf : 0u;
        uint32_t lo = 0;
#pragma unroll
        for (int q = 0; q < PQ_EPL; ++q) {
            const int32_t rk = sh.lrank[tid * PQ_EPL + q];
            lo += (rk != RANK_REP && rk != RANK_NEW && (uint32_t)rk >= rlo) ? 1u : 0u;
        }
        uint32_t no;
        uint32_t O = pq_scan<NW>(sh, lo, &no);
#pragma unroll
        for (int q = 0; q < PQ_EPL; ++q) {
            const uint32_t e = tid * PQ_EPL + q;
            const int32_t rk = sh.lrank[e];
            if (rk != RANK_REP && rk != RANK_NEW && (uint32_t)rk >= rlo) sh.olist[O++] = (e << 12) | (uint32_t)rk;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < PQ_EPL; ++q) {
            const uint32_t e = tid * PQ_EPL + q;
            const int32_t rk = sh.lrank[e];
            if (rk == RANK_REP) continue;
            uint32_t hit = 0;
            if (rk != RANK_NEW) {
                if ((uint32_t)rk + F < cap) hit = TV_HIT;
                else if ((uint32_t)rk + N < cap) {
                    uint32_t d = (uint32_t)rk + N;
                    for (uint32_t k = 0; k < no && d < cap; ++k) {
                        const uint32_t x = sh.olist[k];
                        if ((x >> 12) >= e) break;
                        if ((x & 0xFFFu) > (uint32_t)rk) ++d;
                    }
                    hit = d < cap ? TV_HIT : 0u;
                }
            }
            sh.tver[e] = hit;  // leader residency, read by the group's walker
            ++F;
            if (rk == RANK_NEW) ++N;
        }
    } else {
#pragma unroll
        for (int q = 0; q < PQ_EPL; ++q) {
            const uint32_t e = tid * PQ_EPL + q;
            const int32_t rk = sh.lrank[e];
            if (rk != RANK_REP) sh.tver[e] = rk != RANK_NEW ? TV_HIT : 0u;
        }
    }
    __syncthreads();
    PQ_MARK(4)
    // (d) walks: one lane per key group, its accesses in tile order; a thread-count tile that fails the
    // no-eviction check is replayed by pq_count_seq and walked again with its residencies
    uint32_t gend[SP], glast[SP];
    PData gfin[SP];
    bool gpres[SP], gtouch[SP];
    int mode = rmode ? 1 : 0;  // 0: rank rule, 1: no-eviction hypothesis (verified), 2: sequential replay
    uint32_t seq_size = 0;
    // group ends without a sequential scan of the sorted keys: the leaders' sorted positions by group index
    uint32_t gidx[SP], ngrp = 0;
#pragma unroll
    for (uint32_t q = 0; q < SP; ++q) {
        uint32_t tq;
        gidx[q] = ngrp + pq_scan<NW>(sh, glead[q] ? 1u : 0u, &tq);
        if (glead[q]) sh.olist[gidx[q]] = tid + q * HW;
        ngrp += tq;
    }
    __syncthreads();
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (uint32_t q = 0; q < SP; ++q) {
            const uint32_t s = tid + q * HW;
            gend[q] = s;
            gfin[q] = gd[q];
            gpres[q] = false;
            gtouch[q] = false;
            glast[q] = 0;
            if (!glead[q]) continue;
            const uint32_t e0 = sh.sidx[s];
            const bool ghit = (sh.tver[e0] & TV_HIT) != 0;
            const uint64_t key = sh.skey[s];
            const uint32_t send = gidx[q] + 1 < ngrp ? sh.olist[gidx[q] + 1] : na;
            gend[q] = send;
            PData st = gd[q];
            if (walk == PW_COUNT) {
                bool pres = ghit;
                int64_t c = ghit ? gd[q].v0 : 0;
                if (!rmode) {  // increments only (OP_ADD): the first access inserts an absent key, each adds one
                    for (uint32_t p = s; p < send; ++p) sh.tver[sh.sidx[p]] = (p == s && !ghit) ? TV_INS : 0u;
                    st.v0 = c + (int64_t)(send - s);
                    gpres[q] = true;
                    gtouch[q] = true;
                    glast[q] = sh.sidx[send - 1];
                    gfin[q] = st;
                    continue;
                }
                const int64_t thr = r ? pq_thread_thr(S, r, key) : 0;
                for (uint32_t p = s; p < send; ++p) {
                    const uint32_t e = sh.sidx[p];
                    uint32_t op = pq_op(sh.tkx[e]);
                    if (op == OP_SUBC) op = (sh.tver[sh.tx[e] - tbase] & TV_BLOCK) ? OP_NONE : OP_SUB;
                    const bool pb = pres;
                    const uint32_t v = pq_count_op(op, pres, c, thr);
                    sh.tver[e] = v;
                    if (op != OP_NONE && (pb || (v & TV_INS))) { gtouch[q] = true; glast[q] = e; }
                    if (rmode) sh.lrank[e] = (int32_t)s;  // the event's group (pq_count_seq)
                }
                st.v0 = c;
                gpres[q] = pres;
                gfin[q] = st;
                continue;
            }
            gpres[q] = true;
            gtouch[q] = true;
            glast[q] = sh.sidx[send - 1];
            int64_t tcl = 0;
            int32_t maxc = 0;
            {   // the value's token count: its hot item, else (int) / (long) count
                bool hf = false;
                int32_t hc = 0;
                for (uint32_t i = 0; i < r->hot_n; ++i) {
                    const DHot h = S.hot[r->hot_off + i];
                    if (h.key == key) { hf = true; hc = h.count; break; }
                }
                tcl = hf ? (int64_t)hc : (walk == PW_THROTTLE ? r->token_count_l : (int64_t)r->token_count);
                maxc = j_iadd((int32_t)tcl, r->burst);
            }
            const int64_t dur_ms = r->duration_sec * 1000;
            bool first_miss = !ghit;
            if (ghit && all_acq1) {
                // A resident value whose group's LAST access is blocked with the state it had at the group start is
                // blocked throughout, and a blocked check changes nothing (times only grow along the group): no token
                // refill before it (passTime <= duration) with no token left; a throttle's expected pass time still
                // at least maxQueue ahead.  The group is then one check instead of a walk.
                const int64_t tl = t0 + sh.tdt[glast[q]];
                bool blocked;
                if (walk == PW_THROTTLE) {
                    const int64_t expected = st.v0 + j_round(1.0 * 1000 * 1 * (double)r->duration_sec / (double)tcl);
                    blocked = !(expected <= tl || expected - tl < r->max_queue);
                } else {
                    blocked = tl - st.v0 <= dur_ms && j_iadd(st.v1, -1) < 0;
                }
                if (blocked) {
                    for (uint32_t p = s; p < send; ++p) sh.tver[sh.sidx[p]] = TV_BLOCK;
                    gfin[q] = st;
                    continue;
                }
            }
            for (uint32_t p = s; p < send; ++p) {
                const uint32_t e = sh.sidx[p];
                const int64_t t = t0 + sh.tdt[e];
                const int acq = (int)(sh.tcz[e] & 0xFFFFu);
                uint32_t v = 0;
                if (walk == PW_THROTTLE) {  // passThrottleLocalCheck (ParamFlowChecker.java:198-248)
                    if (first_miss) {
                        st.v0 = t;
                    } else {
                        const int64_t cost = j_round(1.0 * 1000 * acq * (double)r->duration_sec / (double)tcl);
                        const int64_t expected = st.v0 + cost;
                        if (expected <= t || expected - t < r->max_queue) {
                            const int64_t w = expected - t;
                            st.v0 = w > 0 ? expected : t;
                            if (w > 0) v = (uint32_t)(w > 0xFFFF ? 0xFFFF : w) << 16;
                        } else {
                            v = TV_BLOCK;
                        }
                    }
                } else {  // passDefaultLocalCheck (ParamFlowChecker.java:121-196)
                    if (first_miss) {
                        st.v0 = t;
                        st.v1 = j_iadd(maxc, -acq);
                    } else {
                        const int64_t pass_time = t - st.v0;
                        if (pass_time > dur_ms) {
                            const int32_t to_add = (int32_t)((pass_time * tcl) / dur_ms);
                            const int32_t sum = j_iadd(st.v1, to_add);
                            const int32_t nq = sum > maxc ? j_iadd(maxc, -acq) : j_iadd(sum, -acq);
                            if (nq < 0) v = TV_BLOCK;
                            else { st.v1 = nq; st.v0 = t; }
                        } else if (j_iadd(st.v1, -acq) >= 0) {
                            st.v1 = j_iadd(st.v1, -acq);
                        } else {
                            v = TV_BLOCK;
                        }
                    }
                }
                first_miss = false;
                sh.tver[e] = v;
            }
            gfin[q] = st;
        }
        __syncthreads();
        if (mode != 1) break;
        // the hypothesis holds iff the map's size, live0 + insertions - removals so far, never exceeds cap
        int32_t run = 0, lmax = 0;
#pragma unroll
        for (int q = 0; q < PQ_EPL; ++q) {
            const uint32_t v = sh.tver[tid * PQ_EPL + q];
            if (acc[q]) run += ((v & TV_INS) ? 1 : 0) - ((v & TV_REM) ? 1 : 0);
            lmax = run > lmax ? run : lmax;
        }
        uint32_t tot;
        const int32_t pre = (int32_t)pq_scan<NW>(sh, (uint32_t)run, &tot);
        const int32_t peak = (int32_t)live0 + pre + lmax;
        if (!force_seq && __syncthreads_or(peak > (int32_t)cap) == 0) break;  // (force_seq: SG_DEBUG_FLAGS 32)
        // replay: per group its stamp (or -1) and count in LDS, then one lane in tile order
#pragma unroll
        for (uint32_t q = 0; q < SP; ++q) {
            if (!glead[q]) continue;
            const uint32_t s = tid + q * HW;
            sh.tkey[s] = glive[q] ? (uint64_t)gst[q] : ~0ull;
            sh.tdec[s] = glive[q] ? (uint32_t)(gd[q].v0 < 0 ? 0 : gd[q].v0 > (int64_t)GS_CNT ? GS_CNT : gd[q].v0) : 0u;
        }
#pragma unroll
        for (int q = 0; q < PQ_EPL; ++q) sh.tver[tid * PQ_EPL + q] = 0;
        __syncthreads();
        if (tid == 0) sh.red64[0][0] = (int64_t)pq_count_seq<NW>(sh, mk, r, S, tbase);
        __syncthreads();
        seq_size = (uint32_t)sh.red64[0][0];
        __syncthreads();
        mode = 2;
    }
    PQ_MARK(5)
    // (e) commit: touched keys leave their old stamp; the oldest untouched keys beyond cap are evicted
    uint32_t nnew = 0;
#pragma unroll
    for (uint32_t q = 0; q < SP; ++q) {
        if (!glead[q]) continue;
        if (glive[q] && gtouch[q]) {  // an untouched key keeps its place
            const uint64_t p = (uint64_t)gst[q] & (uint64_t)(RB - 1);
            atomicAnd(reinterpret_cast<unsigned long long*>(&sh.bm[mk][p >> 6]), ~(1ull << (p & 63)));
        }
        if (mode == 0) nnew += glive[q] ? 0u : 1u;
        else nnew += (glive[q] && gtouch[q] ? 1u : 0u) | (gtouch[q] && gpres[q] ? 0x10000u : 0u);
    }
    uint32_t ntot;
    (void)pq_scan<NW>(sh, nnew, &ntot);  // (barrier: the cleared bits are in place)
    const uint32_t E = mode == 0 && live0 + ntot > cap ? live0 + ntot - cap : 0u;
    const uint32_t live1 = mode == 0 ? live0 + ntot - E
                         : mode == 1 ? live0 - (ntot & 0xFFFFu) + (ntot >> 16) : seq_size;
    if (E) {
        const uint32_t w0 = ring_word(m, m.thr);
        const uint32_t w = (w0 + tid) & (W - 1);
        const uint64_t word = tid < W ? sh.bm[mk][w] : 0ull;
        uint32_t tot;
        const uint32_t before = pq_scan<NW>(sh, (uint32_t)__popcll(word), &tot);
        if (tid < W && before < E && word) {
            uint64_t x = word;
            uint32_t k = E - before;
            while (x && k) { x &= x - 1; --k; }  // clear the lowest E - before set bits
            sh.bm[mk][w] = x;
        }
    }
    for (uint32_t i = tid; i < PQ_CLW; i += HW) sh.claim[i] = 0;
    __syncthreads();
    // new stamps: the group's last access; keys with a slot (live or dead) keep it; a key removed by the tile
    // keeps its slot with a dead stamp
    bool need[SP];
    int64_t gns[SP];
#pragma unroll
    for (uint32_t q = 0; q < SP; ++q) {
        need[q] = false;
        gns[q] = 0;
        if (!glead[q] || !gpres[q] || !gtouch[q]) continue;
        gns[q] = clock0 + (int64_t)sh.tA[glast[q]];  // the group's last touching access
        const uint64_t p = (uint64_t)gns[q] & (uint64_t)(RB - 1);
        atomicOr(reinterpret_cast<unsigned long long*>(&sh.bm[mk][p >> 6]), 1ull << (p & 63));
        if (gslot[q] >= 0) {
            B[gslot[q] / PM_BKT].stamp[gslot[q] % PM_BKT] = gns[q];
            D[gslot[q]] = gfin[q];
            const uint32_t i = (uint32_t)gslot[q];
            atomicOr(reinterpret_cast<unsigned long long*>(&sh.claim[i >> 6]), 1ull << (i & 63));
        } else {
            need[q] = true;
        }
    }
    if (tid == 0) {
        m.clock = clock0 + (int64_t)na;
        m.live = live1;
        sh.npend = 0;
    }
    __syncthreads();
    PQ_MARK(6)
    // keys without a slot: a free slot (never used, or dead by the ring) of the less loaded bucket, claimed in LDS
#pragma unroll
    for (uint32_t q = 0; q < SP; ++q) {
        if (!need[q]) continue;
        const uint64_t key = sh.skey[tid + q * HW];
        uint32_t b1, b2;
        pm_buckets(m.nb, key, b1, b2);
        bool placed = false;
        // the slots of both buckets that are free in HBM (never used, or dead by the ring): one round of loads
        const uint32_t hf1 = pq_free_mask(B, b1, m, sh.bm[mk]), hf2 = pq_free_mask(B, b2, m, sh.bm[mk]);
        for (int attempt = 0; attempt < 4 && !placed; ++attempt) {
            int f1 = -1, f2 = -1, n1 = 0, n2 = 0;
            for (int j = 0; j < PM_BKT; ++j) {
                const uint32_t i1 = b1 * PM_BKT + j, i2 = b2 * PM_BKT + j;
                const bool c1 = (sh.claim[i1 >> 6] >> (i1 & 63)) & 1ull, c2 = (sh.claim[i2 >> 6] >> (i2 & 63)) & 1ull;
                const bool fr1 = !c1 && ((hf1 >> j) & 1u);
                const bool fr2 = !c2 && ((hf2 >> j) & 1u);
                if (fr1) { if (f1 < 0) f1 = j; } else ++n1;
                if (fr2) { if (f2 < 0) f2 = j; } else ++n2;
            }
            const bool u1 = f1 >= 0 && (f2 < 0 || n1 <= n2);
            if (!u1 && f2 < 0) break;
            const uint32_t i = u1 ? b1 * PM_BKT + (uint32_t)f1 : b2 * PM_BKT + (uint32_t)f2;
            const unsigned long long old =
                atomicOr(reinterpret_cast<unsigned long long*>(&sh.claim[i >> 6]), 1ull << (i & 63));
            if ((old >> (i & 63)) & 1ull) continue;  // another lane took it first
            B[i / PM_BKT].key[i % PM_BKT] = key;
            B[i / PM_BKT].stamp[i % PM_BKT] = gns[q];
            D[i] = gfin[q];
            placed = true;
        }
        if (!placed) {
            const uint32_t k = atomicAdd(&sh.npend, 1u);
            if (k < PQ_NPEND) { sh.pend_key[k] = key; sh.pend_stamp[k] = gns[q]; sh.pend_dat[k] = gfin[q]; }
            else atomicOr(bflags, BF_PTAB_FULL);
        }
    }
    __syncthreads();
    PQ_MARK(7)
    if (tid == 0 && sh.npend) {  // displacement walks (pmap.h pm_insert_new), one lane
        const uint32_t np = sh.npend < PQ_NPEND ? sh.npend : PQ_NPEND;
        for (uint32_t k = 0; k < np; ++k) {
            uint64_t ck = sh.pend_key[k];
            int64_t cs = sh.pend_stamp[k];
            PData cd = sh.pend_dat[k];
            uint32_t b1, b2;
            pm_buckets(m.nb, ck, b1, b2);
            uint32_t b = b1;
            bool done = false;
            for (int step = 0; step < 256 && !done; ++step) {
                for (int j = 0; j < PM_BKT; ++j) {
                    const uint64_t kk = ld64(&B[b].key[j]);
                    if (kk == PK_EMPTY || !ring_live(m, sh.bm[mk], (int64_t)ld64(&B[b].stamp[j]))) {
                        B[b].key[j] = ck; B[b].stamp[j] = cs; D[b * PM_BKT + j] = cd;
                        done = true;
                        break;
                    }
                }
                if (done) break;
                const int j = (int)((cs + step * 5) & 7);
                const uint64_t nk = ld64(&B[b].key[j]);
                const int64_t ns = (int64_t)ld64(&B[b].stamp[j]);
                const PData nd = D[b * PM_BKT + j];
                B[b].key[j] = ck; B[b].stamp[j] = cs; D[b * PM_BKT + j] = cd;
                ck = nk; cs = ns; cd = nd;
                b = pm_alt(m.nb, ck, b);
            }
            if (!done) atomicOr(bflags, BF_PTAB_FULL);
        }
        __threadfence_block();
    }
    __syncthreads();
    PQ_MARK(8)
}

// StatisticSlot on the ClusterNode for one tile (StatisticSlot.java:54-173, ClusterNode.trace): the events of
// one 500 ms bucket are one bucket update (nothing reads the windows in between); an EXIT / TRACE counts iff its
// ENTRY passed (CtSph exits a blocked entry internally: no statistics)
template <int NW>
__device__ __noinline__ void pq_fold(PqSh<NW>& sh, const Ctx& C, int64_t t0, uint32_t tb, uint32_t start, uint32_t len,
                                     const uint32_t* dec, uint32_t* bflags) {
    constexpr uint32_t TE = PqSh<NW>::TE;
    const uint32_t tid = threadIdx.x;
    const uint32_t ne = len - tb < TE ? len - tb : TE;
    int64_t bcur = (t0 + sh.tdt[0]) / 500;
    const int64_t blast = (t0 + sh.tdt[ne - 1]) / 500;
    // effectiveness of this lane's EXIT / TRACEs (bit q)
    uint32_t effm = 0;
#pragma unroll
    for (int q = 0; q < PQ_EPL; ++q) {
        const uint32_t e = tid * PQ_EPL + q, p = tb + e;
        if (p >= len) continue;
        const uint32_t kx = sh.tkx[e], kind = kx & 0xFFu, code = (kx >> 16) & 0xFFu;
        if (kind == SG_EV_ENTRY) continue;
        bool eff;
        if (code == RC_NONE || code == RC_PASSED) eff = true;  // the chain exists (k_pq runs only then)
        else if (code == RC_NOT) eff = false;
        else {
            const uint32_t rel = sh.tx[e] - start;
            if (rel >= p) { atomicOr(bflags, BF_BAD_REF); eff = false; }
            else if (rel >= tb) eff = st_passed(sh.tdec[rel - tb] & 0xFF);
            else eff = st_passed(ld32(&dec[sh.tx[e]]) & 0xFF);
        }
        if (eff) effm |= 1u << q;
    }
    for (;;) {
        uint32_t a[8] = {0, 0, 0, 0, 0, 0xFFFFFFFFu, 0, 0};  // pass block succ rt exc minrt thread touched
        int64_t nxt = INT64_MAX;
#pragma unroll
        for (int q = 0; q < PQ_EPL; ++q) {
            const uint32_t e = tid * PQ_EPL + q;
            if (tb + e >= len) continue;
            const int64_t bk = (t0 + sh.tdt[e]) / 500;
            if (bk != bcur) {
                if (bk > bcur && bk < nxt) nxt = bk;
                continue;
            }
            const uint32_t kx = sh.tkx[e], kind = kx & 0xFFu, cz = sh.tcz[e], cnt = cz & 0xFFFFu, rt = cz >> 16;
            if (kind == SG_EV_ENTRY) {
                a[7] += 1;
                if (st_passed(sh.tdec[e] & 0xFF)) { a[0] += cnt; a[6] += 1; }
                else a[1] += cnt;
            } else if ((effm >> q) & 1) {
                if (kind == SG_EV_EXIT) {
                    a[7] += 1;
                    a[2] += cnt; a[3] += rt; a[5] = rt < a[5] ? rt : a[5]; a[6] -= 1;
                } else if (cnt > 0) {
                    a[7] += 1;
                    a[4] += cnt;
                }
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const uint32_t y = (uint32_t)__shfl_xor((int)a[k], o, 64);
                a[k] = k == 5 ? (y < a[k] ? y : a[k]) : a[k] + y;
            }
            const int64_t yn = __shfl_xor(nxt, o, 64);
            nxt = yn < nxt ? yn : nxt;
        }
        const uint32_t w = tid >> 6;
        if ((tid & 63) == 0) {
#pragma unroll
            for (int k = 0; k < 8; ++k) sh.red[w][k] = a[k];
            sh.red64[w][0] = nxt;
        }
        __syncthreads();
        if (tid == 0) {
            uint32_t s[8] = {0, 0, 0, 0, 0, 0xFFFFFFFFu, 0, 0};
            int64_t nx = INT64_MAX;
            for (int ww = 0; ww < NW; ++ww) {
                for (int k = 0; k < 8; ++k) s[k] = k == 5 ? (sh.red[ww][k] < s[k] ? sh.red[ww][k] : s[k]) : s[k] + sh.red[ww][k];
                nx = sh.red64[ww][0] < nx ? sh.red64[ww][0] : nx;
            }
            if (s[7]) {  // the bucket's first touching event resets a stale bucket (LeapArray.currentWindow)
                Node& N = sh.node;
                const int64_t tc = bcur * 500;
                const int64_t mrt = s[5] == 0xFFFFFFFFu ? INT64_MAX : (int64_t)s[5];
                const int sl = sec_current(N, tc, C.max_rt);
                sec_add(N, sl, s[0], s[1], s[2], s[3], s[4], mrt);
                min_current(N, C.minb, tc, C.max_rt, C.pflags);
                min_add(N, s[0], s[1], s[2], s[3], s[4], mrt);
                N.thread += (int32_t)s[6];
            }
            sh.red64[0][1] = nx;
        }
        __syncthreads();
        const int64_t nn = uni64_pq(sh.red64[0][1]);
        if (nn == INT64_MAX || nn > blast) break;
        bcur = nn;
        __syncthreads();
    }
}

// XF_PVPQ segments pvalue.hip decided (SEG_PV): StatisticSlot over the final verdicts (StatisticSlot.java:54-173),
// a workgroup per segment, 4 events a lane a round, one node update per 500 ms bucket (as pq_fold); the passed
// ENTRYs without an argument get their word here (the ones with one got theirs, with a throttle's wait, from the
// walk).  An EXIT naming an ENTRY of the batch reads that ENTRY's record flags, not its word (written concurrently).
// the workgroup's sums of one 500 ms bucket onto the node (tid 0): LeapArray.currentWindow (the bucket's first
// touching event resets a stale bucket), then the additions; uniform call (barriers)
template <int NW>
__device__ __forceinline__ void pvf_apply(uint32_t (&a)[8], int64_t b, Node& node, const Ctx& C, uint32_t (*red)[8]) {
    const uint32_t tid = threadIdx.x, l = tid & 63, w = tid >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t y = (uint32_t)__shfl_xor((int)a[k], o, 64);
            a[k] = k == 5 ? (y < a[k] ? y : a[k]) : a[k] + y;
        }
    }
    if (l == 0) {
#pragma unroll
        for (int k = 0; k < 8; ++k) red[w][k] = a[k];
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t t[8] = {0, 0, 0, 0, 0, 0xFFFFFFFFu, 0, 0};
        for (int ww = 0; ww < NW; ++ww)
            for (int k = 0; k < 8; ++k) t[k] = k == 5 ? (red[ww][k] < t[k] ? red[ww][k] : t[k]) : t[k] + red[ww][k];
        if (t[7]) {
            const int64_t tc = b * 500;
            const int64_t mrt = t[5] == 0xFFFFFFFFu ? INT64_MAX : (int64_t)t[5];
            const int sl = sec_current(node, tc, C.max_rt);
            sec_add(node, sl, t[0], t[1], t[2], t[3], t[4], mrt);
            min_current(node, C.minb, tc, C.max_rt, C.pflags);
            min_add(node, t[0], t[1], t[2], t[3], t[4], mrt);
            node.thread += (int32_t)t[6];
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = k == 5 ? 0xFFFFFFFFu : 0u;
}

// XF_PVPQ segments pvalue.hip decided (SEG_PV): StatisticSlot over the final verdicts (StatisticSlot.java:54-173),
// a workgroup per segment, 8 events a lane a round, one node update per 500 ms bucket (as pq_fold): a round within
// the pending bucket (its first and last events' times tell, the events being in time order) only adds to the
// lanes' sums.  The passed ENTRYs without an argument get their word here (the ones with one got theirs, with a
// throttle's wait, from the walk).  An EXIT naming an ENTRY of the batch reads that ENTRY's record flags, not its
// word (written concurrently).
template <int NW>
__global__ __launch_bounds__(NW * 64) void k_pvf(const SEv* __restrict__ recs, const Seg* __restrict__ segs,
                                                 const uint32_t* __restrict__ order, uint32_t m, DevState S, DevCfg cfg,
                                                 int64_t t0, uint32_t* __restrict__ dec, uint32_t* __restrict__ bflags) {
    constexpr uint32_t HW = NW * 64, EPL = 8;
    __shared__ Node node;
    __shared__ uint32_t red[NW][8];
    __shared__ int64_t rnx[NW];
    __shared__ int64_t bnext;
    if (blockIdx.x >= m) return;
    const Seg sg = segs[order[blockIdx.x]];
    if (!(sg.bin & SEG_PV)) return;  // (k_pq's full pass decides the others)
    const uint32_t tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const Prog pg = S.prog[sg.res];
    const Ctx C{S.minb + (uint64_t)sg.res * 60, cfg.max_rt, pg.pflags};
    if (tid == 0) {
        node_load(node, S, sg.res);
        if (sg.len && (t0 + recs[sg.start].dt) < (node.sb[0].ws > node.sb[1].ws ? node.sb[0].ws : node.sb[1].ws))
            atomicOr(bflags, BF_BACKWARD);  // Q3
    }
    __syncthreads();
    uint32_t a[8] = {0, 0, 0, 0, 0, 0xFFFFFFFFu, 0, 0};  // pass block succ rt exc minrt thread touched (pending bucket)
    int64_t pend = INT64_MIN;                            // the pending bucket (uniform)
    for (uint32_t base = 0; base < sg.len; base += HW * EPL) {
        SEv ev[EPL];
        bool in[EPL], eff[EPL], pass[EPL];
        int64_t bk[EPL];
#pragma unroll
        for (uint32_t q = 0; q < EPL; ++q) {
            const uint32_t p = base + q * HW + tid;
            in[q] = p < sg.len;
            eff[q] = pass[q] = false;
            bk[q] = INT64_MAX;
            if (!in[q]) continue;
            ev[q] = recs[sg.start + p];
            bk[q] = (t0 + ev[q].dt) / 500;
            if (ev[q].kind == SG_EV_ENTRY) {
                pass[q] = !(ev[q].flags & RF_PBLK);
                if (!(ev[q].flags & SG_F_HAS_ARG)) dec[sg.start + p] = mk_dec(ST_PASS, 0, 0);
            } else if (ev[q].code == RC_NONE || ev[q].code == RC_PASSED) {
                eff[q] = true;
            } else if (ev[q].code == RC_BATCH) {
                const uint32_t rel = ev[q].x - sg.start;
                if (rel >= p) atomicOr(bflags, BF_BAD_REF);
                else eff[q] = !(recs[ev[q].x].flags & RF_PBLK);
            }
        }
        const uint32_t rend = sg.len - base < HW * EPL ? sg.len : base + HW * EPL;
        const int64_t bfirst = (t0 + recs[sg.start + base].dt) / 500, blast = (t0 + recs[sg.start + rend - 1].dt) / 500;
        if (bfirst == blast && (pend == bfirst || pend == INT64_MIN)) {  // (uniform) one bucket, the pending one
            pend = bfirst;
#pragma unroll
            for (uint32_t q = 0; q < EPL; ++q) {
                if (!in[q]) continue;
                const uint32_t cnt = ev[q].cnt, rt = ev[q].rt;
                if (ev[q].kind == SG_EV_ENTRY) {
                    a[7] += 1;
                    if (pass[q]) { a[0] += cnt; a[6] += 1; }
                    else a[1] += cnt;
                } else if (eff[q]) {
                    if (ev[q].kind == SG_EV_EXIT) { a[7] += 1; a[2] += cnt; a[3] += rt; a[5] = rt < a[5] ? rt : a[5]; a[6] -= 1; }
                    else if (cnt > 0) { a[7] += 1; a[4] += cnt; }
                }
            }
            continue;
        }
        if (pend != INT64_MIN) { pvf_apply<NW>(a, pend, node, C, red); pend = INT64_MIN; }
        int64_t bcur = bfirst;
        while (bcur != INT64_MAX) {
            int64_t nxt = INT64_MAX;
#pragma unroll
            for (uint32_t q = 0; q < EPL; ++q) {
                if (!in[q]) continue;
                if (bk[q] != bcur) {
                    if (bk[q] > bcur && bk[q] < nxt) nxt = bk[q];
                    continue;
                }
                const uint32_t cnt = ev[q].cnt, rt = ev[q].rt;
                if (ev[q].kind == SG_EV_ENTRY) {
                    a[7] += 1;
                    if (pass[q]) { a[0] += cnt; a[6] += 1; }
                    else a[1] += cnt;
                } else if (eff[q]) {
                    if (ev[q].kind == SG_EV_EXIT) { a[7] += 1; a[2] += cnt; a[3] += rt; a[5] = rt < a[5] ? rt : a[5]; a[6] -= 1; }
                    else if (cnt > 0) { a[7] += 1; a[4] += cnt; }
                }
            }
            for (int o = 32; o > 0; o >>= 1) { const int64_t y = __shfl_xor(nxt, o, 64); nxt = y < nxt ? y : nxt; }
            if (l == 0) rnx[w] = nxt;
            __syncthreads();
            if (tid == 0) {
                int64_t nx = INT64_MAX;
                for (int ww = 0; ww < NW; ++ww) nx = rnx[ww] < nx ? rnx[ww] : nx;
                bnext = nx;
            }
            // the round's last bucket stays pending (the next round may continue it)
            __syncthreads();
            const int64_t nb = uni64_pq(bnext);
            if (nb == INT64_MAX) { pend = bcur; break; }
            pvf_apply<NW>(a, bcur, node, C, red);
            bcur = nb;
        }
    }
    if (pend != INT64_MIN) pvf_apply<NW>(a, pend, node, C, red);
    if (tid == 0) {
        min_flush(node, C.minb);
        node_store(node, S, sg.res, pg.pflags);
    }
}

// MODE (XF_MIX segments, whose flow / degrade chain a k_jac owner decides between the two passes):
//   PQ_FULL  the resource's whole decision (PF_PQ);
//   PQ_PRE   ParamFlowSlot's QPS checks only.  Nothing before ParamFlowSlot blocks, so they see every ENTRY whatever
//            the later slots decide; a blocked ENTRY gets its final dec[] word and RF_PBLK, the
//            passed ones are left to the owner.  No statistics, no thread-count map;
//   PQ_POST  ParamFlowStatisticEntryCallback / ExitCallback from the final verdicts: the thread-count map of
//            paramIdx 0 (passed ENTRYs add, EXITs of passed ENTRYs release) and the node's ParameterMetric bits.
enum { PQ_FULL = 0, PQ_PRE = 1, PQ_POST = 2 };
// one segment by one workgroup (every return below is uniform over the workgroup)
template <int NW, int MODE>
__device__ __forceinline__ void pq_seg(PqSh<NW>& sh, const Seg sg, SEv* __restrict__ recs,
                                       const sg_event* __restrict__ ev, const uint32_t* __restrict__ vals,
                                       const DevState& S, const DevCfg& cfg, int64_t t0, uint32_t* __restrict__ dec,
                                       uint32_t* __restrict__ bflags) {
    constexpr uint32_t HW = PqSh<NW>::HW, TE = PqSh<NW>::TE;
    const uint32_t tid = threadIdx.x;
    if (MODE == PQ_PRE && (sg.bin & SEG_PV)) return;    // pvalue.hip decided its param checks
    if (MODE == PQ_FULL && (sg.bin & SEG_PV)) return;   // (XF_PVPQ: k_pvf folds its statistics)
    if (MODE == PQ_POST && (sg.bin & SEG_PVT)) return;  // pvalue.hip's post pass took its thread-count map
    const uint32_t res = sg.res;
    const Prog pg = S.prog[res];
    const int np = pg.n_param;
    const Ctx C{S.minb + (uint64_t)res * 60, cfg.max_rt, pg.pflags};
    // an XF_PVPQ segment pvalue.hip's passes took: its param verdicts are in (RF_PBLK, the passed words with their
    // throttle wait), its thread-count map and ParameterMetric bits are the post pass's -- only the statistics here
    const bool pvd = MODE == PQ_FULL && (sg.bin & SEG_PV) != 0;
    if (tid == 0) {
        node_load(sh.node, S, res);
        sh.flags_or = 0;
        sh.sorted_n = 0;
#ifdef SG_KPROF
        for (int k = 0; k < 16; ++k) sh.pt[k] = 0;
        sh.pt_t = __builtin_amdgcn_s_memtime();
#endif
    }
    if ((int)tid < np) sh.rules[tid] = S.rules[pg.rule_off + tid];
    __syncthreads();
    // the maps: rule maps (QPS rules), then the thread-count map of paramIdx 0
    const uint32_t tm = (pg.tm_base == NO_ID) ? NO_ID : S.tmid[pg.tm_base];
    if (tid <= PQ_MAXP) {
        uint32_t id = NO_ID;
        if (MODE != PQ_POST && (int)tid < np && sh.rules[tid].behavior != PB_INIT_ONLY &&
            sh.rules[tid].grade == SG_FLOW_GRADE_QPS)
            id = sh.rules[tid].pmap;
        if (tid == PQ_MAXP) id = MODE == PQ_PRE ? NO_ID : tm;
        if (pvd) id = NO_ID;  // (no map is this kernel's)
        sh.mid[tid] = id;
        if (id != NO_ID) sh.hdr[tid] = S.pmap[id];
    }
    __syncthreads();
    const bool chain = (sh.node.flags & NI_CHAIN) != 0;  // the host routes switch_on == 0 to k_lane
    if (!chain) {  // no slot chain: every ENTRY is NO_CHECK, nothing is counted, no map is touched
        if (MODE == PQ_FULL)
            for (uint32_t p = tid; p < sg.len; p += HW)
                if (recs[sg.start + p].kind == SG_EV_ENTRY) dec[sg.start + p] = mk_dec(ST_NO_CHECK, 0, 0);
        return;  // (XF_MIX: the owner writes them)
    }
    for (int k = 0; k <= PQ_MAXP; ++k) {
        if (sh.mid[k] == NO_ID) continue;
        const uint32_t W = 1u << (sh.hdr[k].rb_log2 - 6);
        for (uint32_t w = tid; w < W; w += HW) sh.bm[k][w] = S.pbm[sh.hdr[k].bm + w];
    }
    if (MODE != PQ_POST && tid == 0 && sg.len && (t0 + recs[sg.start].dt) < (sh.node.sb[0].ws > sh.node.sb[1].ws ? sh.node.sb[0].ws : sh.node.sb[1].ws))
        atomicOr(bflags, BF_BACKWARD);  // Q3: the clock went back across batches
    // tm bit of paramIdx 0 for a passed ENTRY: it has visited every rule (ParamFlowSlot sets the bits of the
    // rules it checks: ni_tm(paramIdx), or an initialise-only run's map set)
    uint32_t all_bits = NI_PM;
    for (int k = 0; k < np; ++k) {
        const DRule& r = sh.rules[k];
        if (r.behavior == PB_INIT_ONLY) all_bits |= (uint32_t)r.burst << NI_TM_SHIFT;
        else if (r.param_idx < SG_MAX_ARGS) all_bits |= ni_tm((uint32_t)r.param_idx);
    }
    const bool tm_on = tm != NO_ID && ((sh.node.flags | all_bits) & ni_tm(0)) != 0 && !pvd;
    // the THREAD-grade rule (at most one, the last checked, paramIdx 0: engine.cpp PF_PQ) and the first rule whose
    // visit sets the paramIdx-0 thread-map bit; an EXIT decrements only once NI_PM and that bit are set
    int tk = -1, k0 = -1;
    for (int k = 0; k < np; ++k) {
        const DRule& r = sh.rules[k];
        if (r.behavior != PB_INIT_ONLY && r.grade == SG_FLOW_GRADE_THREAD) tk = k;
        const uint32_t b = r.behavior == PB_INIT_ONLY ? (uint32_t)r.burst << NI_TM_SHIFT
                           : (r.param_idx < SG_MAX_ARGS ? ni_tm((uint32_t)r.param_idx) : 0u);
        if (k0 < 0 && (b & ni_tm(0))) k0 = k;
    }
    // EXITs at segment positions >= tm_from release thread counts (uniform)
    uint32_t tm_from = ((sh.node.flags & (NI_PM | ni_tm(0))) == (NI_PM | ni_tm(0))) ? 0u : 0xFFFFFFFFu;

    // The passes around an owner (XF_MIX) walk only the events that touch a map, listed in order into the segment's
    // pend[] scratch (free outside the owner's run): the pre pass the ENTRYs with args[0], the post pass the passed
    // ones and the EXITs releasing args.  A C6 head segment of 4M events is then 2M / ~0.2M accesses.  The post pass
    // takes every ENTRY's visits of the rules (the node's ParameterMetric bits, the first visit of rule k0) from the
    // final verdicts on the way.
    uint32_t nev = sg.len;
    if (MODE != PQ_FULL) {
        uint32_t kbits[PQ_MAXP];
        for (int k = 0; k < PQ_MAXP; ++k) {
            kbits[k] = 0;
            if (k < np) {
                const DRule& r = sh.rules[k];
                kbits[k] = r.behavior == PB_INIT_ONLY ? (uint32_t)r.burst << NI_TM_SHIFT
                           : NI_PM | (r.param_idx < SG_MAX_ARGS ? ni_tm((uint32_t)r.param_idx) : 0u);
            }
        }
        if (tid == 0) sh.freach = 0xFFFFFFFFu;
        __syncthreads();
        uint32_t fbits = 0, base = 0;
        for (uint32_t c = 0; c < sg.len; c += HW) {  // (uniform trip count)
            const uint32_t p = c + tid;
            bool take = false;
            if (p < sg.len) {
                const uint32_t w = reinterpret_cast<const uint4*>(recs)[sg.start + p].w;
                const uint32_t kind = w & 0xFFu, fl = (w >> 8) & 0xFFu;
                if (MODE == PQ_PRE) {
                    take = kind == SG_EV_ENTRY && (fl & SG_F_HAS_ARG);
                } else if (kind == SG_EV_ENTRY) {  // the final verdict as the rule it stopped at
                    const uint32_t d = dec[sg.start + p];
                    uint32_t stq = 0;
                    if (!st_passed(d & 0xFFu)) {
                        stq = (uint32_t)np + 1;  // a flow / degrade stage blocked it: every param rule was visited
                        if ((d & 0xFFu) == ST_BLOCK_PARAM)
                            for (int k = 0; k < np; ++k)
                                if (sh.rules[k].behavior != PB_INIT_ONLY && sh.rules[k].slot == ((d >> 8) & 0xFFu))
                                    stq = (uint32_t)k + 1;
                    }
                    for (int k = 0; k < np; ++k)
                        if (stq == 0 || stq > (uint32_t)k) {
                            fbits |= kbits[k] | NI_PM;
                            if (k == k0) atomicMin(&sh.freach, p + 1);
                        }
                    take = stq == 0 && (fl & SG_F_HAS_ARG);
                } else if (kind == SG_EV_EXIT) {
                    take = (fl & SG_F_EXIT_ARGS) != 0;
                }
            }
            uint32_t tot;
            const uint32_t o = pq_scan<NW>(sh, take ? 1u : 0u, &tot);
            if (take) S.pend[sg.start + base + o] = p;
            base += tot;
        }
        if (fbits) atomicOr(&sh.flags_or, fbits);
        nev = base;
        __syncthreads();
        if (MODE == PQ_POST && tm_from == 0xFFFFFFFFu) tm_from = sh.freach;
    }

    for (uint32_t tb = 0; tb < nev; tb += TE) {
        // ---- 1. the tile's events
        uint32_t st[PQ_EPL], wt[PQ_EPL];  // st: 0 pending / passed, else the blocking rule + 1
        uint32_t pp[PQ_EPL];              // segment positions (the listed ones around an owner)
#pragma unroll
        for (int q = 0; q < PQ_EPL; ++q) {
            const uint32_t e = tid * PQ_EPL + q, ci = tb + e;
            const bool ok = ci < nev;
            const uint32_t p = MODE == PQ_FULL ? ci : (ok ? S.pend[sg.start + ci] : 0xFFFFFFFFu);
            pp[q] = ok ? p : 0xFFFFFFFFu;
            SEv r;
            r.kind = 0xFF; r.flags = 0; r.code = 0; r.dt = 0; r.cnt = 0; r.rt = 0; r.x = 0;
            if (ok) r = recs[sg.start + p];
            st[q] = 0;
            wt[q] = 0;
            sh.tdt[e] = r.dt;
            sh.tcz[e] = (uint32_t)r.cnt | ((uint32_t)r.rt << 16);
            sh.tkx[e] = (uint32_t)r.kind | ((uint32_t)r.flags << 8) | ((uint32_t)r.code << 16);
            sh.tx[e] = r.x;
            // args[0]'s key: k_rs_first put it in the key ring (sg_submit's aux, or sg_submit_ex's table entry)
            if (r.kind == SG_EV_ENTRY && (r.flags & SG_F_HAS_ARG))
                sh.tkey[e] = S.key_ring[(S.gbase + (vals[sg.start + p] & 0x7FFFFFFFu)) & cfg.ring_mask];
        }
        __syncthreads();
        // ---- 2. ParamFlowSlot: the rules in order
        bool ran_qps = false;  // a rule map phase of this tile left its sorted accesses in skey / sidx
        if (tid == 0 && MODE == PQ_FULL) sh.freach = 0xFFFFFFFFu;
        __syncthreads();
        PQ_MARK(0)
        if (pvd) {  // the value-parallel pre pass's verdicts (one checked rule: rules[0])
#pragma unroll
            for (int q = 0; q < PQ_EPL; ++q) {
                const uint32_t e = tid * PQ_EPL + q, kx = sh.tkx[e];
                if ((kx & 0xFFu) != SG_EV_ENTRY || tb + e >= sg.len) continue;
                if ((kx >> 8) & RF_PBLK) st[q] = 1;
                else if ((kx >> 8) & SG_F_HAS_ARG) wt[q] = ld32(&dec[sg.start + tb + e]) >> 16;
            }
        }
        for (int k = 0; k < np; ++k) {
            const DRule& r = sh.rules[k];
            if (MODE == PQ_POST || pvd) break;  // (its visits were taken with the list / by pvalue.hip)
            bool reach = false;
#pragma unroll
            for (int q = 0; q < PQ_EPL; ++q) {
                const bool rq = (sh.tkx[tid * PQ_EPL + q] & 0xFFu) == SG_EV_ENTRY && st[q] == 0;
                reach |= rq;
                if (rq && k == k0 && tb + tid * PQ_EPL + q < sg.len) atomicMin(&sh.freach, tb + tid * PQ_EPL + q + 1);
            }
            if (reach) {
                const uint32_t bits = r.behavior == PB_INIT_ONLY ? (uint32_t)r.burst << NI_TM_SHIFT
                                      : NI_PM | (r.param_idx < SG_MAX_ARGS ? ni_tm((uint32_t)r.param_idx) : 0u);
                atomicOr(&sh.flags_or, bits | NI_PM);
            }
            if (r.behavior == PB_INIT_ONLY || r.param_idx != 0) continue;  // no check (idx >= args.length)
            if (r.grade != SG_FLOW_GRADE_QPS) continue;                     // the THREAD rule: phase 3
            const int walk = r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER ? PW_THROTTLE : PW_TOKEN;
            bool acc[PQ_EPL];
#pragma unroll
            for (int q = 0; q < PQ_EPL; ++q) {
                const uint32_t e = tid * PQ_EPL + q, kx = sh.tkx[e];
                acc[q] = false;
                if (!((kx & 0xFFu) == SG_EV_ENTRY && ((kx >> 8) & SG_F_HAS_ARG) && st[q] == 0)) continue;
                const uint64_t key = sh.tkey[e];
                const int acq = (int)(sh.tcz[e] & 0xFFFFu);
                bool hf = false;
                int32_t hc = 0;
                for (uint32_t i = 0; i < r.hot_n; ++i) {
                    const DHot h = S.hot[r.hot_off + i];
                    if (h.key == key) { hf = true; hc = h.count; break; }
                }
                // checks before any map access: a zero token count, an acquire above maxCount
                if (walk == PW_THROTTLE) {
                    if ((hf ? (int64_t)hc : r.token_count_l) == 0) { st[q] = (uint32_t)k + 1; continue; }
                } else {
                    const int32_t tc = hf ? hc : r.token_count;
                    if (tc == 0 || acq > j_iadd(tc, r.burst)) { st[q] = (uint32_t)k + 1; continue; }
                }
                acc[q] = true;
            }
            pq_map_phase<NW>(sh, k, walk, &r, S, t0, sg.start + tb, acc, bflags);
            ran_qps = true;
#pragma unroll
            for (int q = 0; q < PQ_EPL; ++q) {
                if (!acc[q]) continue;
                const uint32_t v = sh.tver[tid * PQ_EPL + q];
                if (v & 1) st[q] = (uint32_t)k + 1;
                else wt[q] += v >> 16;
            }
            __syncthreads();  // tver is rewritten by the next phase
        }
        // ---- 3. the thread-count map of paramIdx 0: the THREAD rule's checks (OP_CHK), else
        // ParamFlowStatisticEntryCallback.onPass of the passed ENTRYs (OP_ADD), and the EXITs' releases
        // (ParamFlowStatisticExitCallback.onExit -> decreaseThreadCount of the ENTRY's argument, OP_SUB)
        __syncthreads();  // every lane's atomicMin on freach is in
        if (MODE == PQ_FULL && tm_from == 0xFFFFFFFFu) tm_from = sh.freach;  // uniform (LDS)
        if (MODE != PQ_PRE && tm_on) {
#pragma unroll
            for (int q = 0; q < PQ_EPL; ++q) sh.tdec[tid * PQ_EPL + q] = st[q];
            __syncthreads();
            bool acc[PQ_EPL];
#pragma unroll
            for (int q = 0; q < PQ_EPL; ++q) {
                const uint32_t e = tid * PQ_EPL + q, p = pp[q], kx = sh.tkx[e], kind = kx & 0xFFu;
                const bool ok = p != 0xFFFFFFFFu;
                uint32_t op = OP_NONE;
                if (ok && kind == SG_EV_ENTRY) {
                    if (((kx >> 8) & SG_F_HAS_ARG) && st[q] == 0) op = tk >= 0 ? OP_CHK : OP_ADD;
                } else if (ok && kind == SG_EV_EXIT && ((kx >> 8) & SG_F_EXIT_ARGS) && p >= tm_from
                           && S.key_ring) {
                    const uint32_t code = (kx >> 16) & 0xFFu;
                    // Entry.exit(count, args) with args of its own (sg_submit_ex) releases those, even naming no
                    // ENTRY; else args[0] of its ENTRY (lane_exit, ParamFlowStatisticExitCallback)
                    const bool own = ((kx >> 8) & RF_OWN_ARGS) != 0;
                    uint64_t ref = SG_REF_NONE;
                    if (code == RC_PASSED) {
                        if (!own) ref = ev[vals[sg.start + p] & 0x7FFFFFFFu].aux & SG_REF_NONE;
                        op = OP_SUB;
                    } else if (code == RC_NONE && own) {
                        op = OP_SUB;
                    } else if (code == RC_BATCH) {
                        const uint32_t rel = sh.tx[e] - sg.start;
                        if (rel < p) {
                            ref = S.gbase + (vals[sh.tx[e]] & 0x7FFFFFFFu);
                            if (MODE == PQ_FULL && rel >= tb) op = sh.tdec[rel - tb] != 0 ? OP_NONE : (tk >= 0 ? OP_SUBC : OP_SUB);
                            else op = st_passed(ld32(&dec[sh.tx[e]]) & 0xFF) ? OP_SUB : OP_NONE;  // (post: final)
                        }
                    }
                    if (op != OP_NONE) {
                        if (own) ref = S.gbase + (vals[sg.start + p] & 0x7FFFFFFFu);
                        const uint64_t key = S.key_ring[ref & cfg.ring_mask];
                        if (key == NO_KEY) op = OP_NONE;
                        else sh.tkey[e] = key;
                    }
                }
                sh.tkx[e] = (kx & 0x00FFFFFFu) | (op << 24);
                acc[q] = op != OP_NONE;
            }
            __syncthreads();
            PQ_MARK(9)
            pq_map_phase<NW>(sh, PQ_MAXP, PW_COUNT, tk >= 0 ? &sh.rules[tk] : nullptr, S, t0, sg.start + tb, acc, bflags,
                             (cfg.dbg_flags & 32) != 0, ran_qps && !(cfg.dbg_flags & 256));
            PQ_MARK(10)
            if (tk >= 0) {
#pragma unroll
                for (int q = 0; q < PQ_EPL; ++q)
                    if (pq_op(sh.tkx[tid * PQ_EPL + q]) == OP_CHK && (sh.tver[tid * PQ_EPL + q] & TV_BLOCK)) st[q] = (uint32_t)tk + 1;
            }
            __syncthreads();
        } else if (MODE == PQ_FULL && tk >= 0) {  // no thread-count map: every count reads 0
#pragma unroll
            for (int q = 0; q < PQ_EPL; ++q) {
                const uint32_t e = tid * PQ_EPL + q, kx = sh.tkx[e];
                if ((kx & 0xFFu) == SG_EV_ENTRY && ((kx >> 8) & SG_F_HAS_ARG) && st[q] == 0 &&
                    1 > pq_thread_thr(S, &sh.rules[tk], sh.tkey[e]))
                    st[q] = (uint32_t)tk + 1;
            }
        }
        // ---- 4. decisions
        if (MODE == PQ_PRE) {  // the param-blocked ENTRYs: final words, marked for the owner
#pragma unroll
            for (int q = 0; q < PQ_EPL; ++q) {
                const uint32_t p = pp[q];
                if (p != 0xFFFFFFFFu && st[q] != 0 && (sh.tkx[tid * PQ_EPL + q] & 0xFFu) == SG_EV_ENTRY) {
                    dec[sg.start + p] = mk_dec(ST_BLOCK_PARAM, sh.rules[st[q] - 1].slot, 0);
                    recs[sg.start + p].flags = (uint8_t)(((sh.tkx[tid * PQ_EPL + q] >> 8) & 0xFFu) | RF_PBLK);
                }
            }
        } else if (MODE == PQ_FULL) {
#pragma unroll
            for (int q = 0; q < PQ_EPL; ++q) {
                const uint32_t e = tid * PQ_EPL + q, p = tb + e;
                uint32_t d = mk_dec(ST_NOT_ENTRY, 0, 0);
                if ((sh.tkx[e] & 0xFFu) == SG_EV_ENTRY) {
                    d = st[q] == 0 ? mk_dec(ST_PASS, 0, wt[q]) : mk_dec(ST_BLOCK_PARAM, sh.rules[st[q] - 1].slot, 0);
                    if (p < sg.len) dec[sg.start + p] = d;
                }
                sh.tdec[e] = d;
            }
            __syncthreads();
            // ---- 5. StatisticSlot: one bucket update per 500 ms bucket of the tile
            PQ_MARK(11)
            pq_fold<NW>(sh, C, t0, tb, sg.start, sg.len, dec, bflags);
        }
        __syncthreads();  // full fence: this tile's dec[] words are visible to the next tiles' EXIT lookups
        PQ_MARK(12)
    }
#ifdef SG_KPROF
    if (S.dbg && tid == 0) {  // every block's phase cycles summed; [24] segments, [25] events, [26] longest segment
        for (int k = 0; k < 13; ++k) atomicAdd(&S.dbg[8 + k], sh.pt[k]);
        atomicAdd(&S.dbg[24], 1ull);
        atomicAdd(&S.dbg[25], (unsigned long long)sg.len);
        atomicMax(&S.dbg[26], (unsigned long long)sg.len);
    }
#endif
    // ---- segment end: node, map headers and rings back to HBM
    if (MODE == PQ_FULL && tid == 0) {
        Node& N = sh.node;
        N.flags |= sh.flags_or;
        min_flush(N, C.minb);
        node_store(N, S, res, pg.pflags);
    }
    if (MODE == PQ_POST && tid == 0 && sh.flags_or) atomicOr(&S.info[res].flags, sh.flags_or);  // (the owner wrote the node)
    for (int k = 0; k <= PQ_MAXP; ++k) {
        if (sh.mid[k] == NO_ID) continue;
        const uint32_t W = 1u << (sh.hdr[k].rb_log2 - 6);
        for (uint32_t w = tid; w < W; w += HW) S.pbm[sh.hdr[k].bm + w] = sh.bm[k][w];
        if (tid == 0) pm_store(S, sh.mid[k], sh.hdr[k]);
    }
}

template <int NW, int MODE>
__global__ __launch_bounds__(NW * 64) void k_pq(SEv* __restrict__ recs, const sg_event* __restrict__ ev,
                                                const uint32_t* __restrict__ vals, const Seg* __restrict__ segs,
                                                const uint32_t* __restrict__ order, uint32_t m, DevState S, DevCfg cfg,
                                                int64_t t0, uint32_t* __restrict__ dec, uint32_t* __restrict__ bflags) {
    __shared__ PqSh<NW> sh;
    if (blockIdx.x >= m) return;
    pq_seg<NW, MODE>(sh, segs[order[blockIdx.x]], recs, ev, vals, S, cfg, t0, dec, bflags);
}
// the segments of a list whose length is on the device (the ones pvalue.hip left), workgroups looping over it
template <int NW, int MODE>
__global__ __launch_bounds__(NW * 64) void k_pq_list(SEv* __restrict__ recs, const sg_event* __restrict__ ev,
                                                     const uint32_t* __restrict__ vals, const Seg* __restrict__ segs,
                                                     const uint32_t* __restrict__ order, const uint32_t* __restrict__ cnt,
                                                     DevState S, DevCfg cfg, int64_t t0, uint32_t* __restrict__ dec,
                                                     uint32_t* __restrict__ bflags) {
    __shared__ PqSh<NW> sh;
    const uint32_t n = *cnt;
    for (uint32_t k = blockIdx.x; k < n; k += gridDim.x) {
        pq_seg<NW, MODE>(sh, segs[order[k]], recs, ev, vals, S, cfg, t0, dec, bflags);
        __syncthreads();
    }
}

// ---- elastic map regions (dev_types.h PM_MIN_NB): pm_move / pm_grow live in pmap.h (k_tiny grows maps too)
// the listed moves, a wavefront per map: every live key of the old region into the new one (PK_EMPTY-filled pool),
// claimed by compare-and-swap in either of its buckets; the rare key finding both full is placed afterwards by one
// lane with pm_move's displacement walk.  The map's order lives in its stamps and ring, not in the slots, so the
// placement is free.  (Most moves are of small maps: 16 to 128 slots.)
__global__ __launch_bounds__(256) void k_pm_move_list(const uint4* __restrict__ mv, const uint32_t* __restrict__ nmv,
                                                      uint32_t mcap, DevState S, uint32_t* __restrict__ bflags) {
    __shared__ uint32_t npend[4];
    __shared__ uint32_t pend[4][64];
    const uint32_t wv = threadIdx.x >> 6, l = threadIdx.x & 63;
    const uint32_t n = *nmv < mcap ? *nmv : mcap;
    for (uint32_t k = blockIdx.x * 4 + wv; k < n; k += gridDim.x * 4) {
        const uint4 v = mv[k];
        const uint32_t id = v.x, nn = v.w;
        const uint64_t nbase = (uint64_t)v.y | ((uint64_t)v.z << 32);
        const PMap m = S.pmap[id];
        if (l == 0) npend[wv] = 0;
        __builtin_amdgcn_wave_barrier();
        const PBucket* OB = S.pbkt + m.base;
        const PData* OD = S.pdat + m.base * PM_BKT;
        PBucket* NB = S.pbkt + nbase;
        PData* ND = S.pdat + nbase * PM_BKT;
        const uint64_t* bm = S.pbm + m.bm;
        for (uint32_t sl = l; sl < m.nb * PM_BKT; sl += 64) {
            const uint64_t ck = OB[sl / PM_BKT].key[sl % PM_BKT];
            const int64_t cs = OB[sl / PM_BKT].stamp[sl % PM_BKT];
            if (ck == PK_EMPTY || !pm_live(m, bm, cs)) continue;
            uint32_t b1, b2;
            pm_buckets(nn, ck, b1, b2);
            bool placed = false;
            for (int h = 0; h < 2 && !placed; ++h) {
                const uint32_t bb = h ? b2 : b1;
                for (int q = 0; q < PM_BKT; ++q) {
                    if (NB[bb].key[q] != PK_EMPTY) continue;
                    const unsigned long long o = atomicCAS(reinterpret_cast<unsigned long long*>(&NB[bb].key[q]),
                                                           (unsigned long long)PK_EMPTY, (unsigned long long)ck);
                    if (o == PK_EMPTY) {
                        NB[bb].stamp[q] = cs;
                        ND[bb * PM_BKT + q] = OD[sl];
                        placed = true;
                        break;
                    }
                }
            }
            if (!placed) {
                const uint32_t p = atomicAdd(&npend[wv], 1u);
                if (p < 64) pend[wv][p] = sl;
                else atomicOr(bflags, BF_PTAB_FULL);
            }
        }
        __threadfence_block();
        __builtin_amdgcn_wave_barrier();
        if (l == 0) {
            const uint32_t np = npend[wv] < 64 ? npend[wv] : 64u;
            for (uint32_t f = 0; f < np; ++f) {
                const uint32_t sl = pend[wv][f];
                uint64_t ck = OB[sl / PM_BKT].key[sl % PM_BKT];
                int64_t cs = OB[sl / PM_BKT].stamp[sl % PM_BKT];
                PData cd = OD[sl];
                uint32_t b1, b2;
                pm_buckets(nn, ck, b1, b2);
                uint32_t c = b1;
                bool placed = false;
                for (int step = 0; step < 512 && !placed; ++step) {
                    for (int q = 0; q < PM_BKT; ++q)
                        if (NB[c].key[q] == PK_EMPTY) { NB[c].key[q] = ck; NB[c].stamp[q] = cs; ND[c * PM_BKT + q] = cd; placed = true; break; }
                    if (placed) break;
                    const int q = (int)((cs + step * 5) & 7);
                    const uint64_t nk = NB[c].key[q];
                    const int64_t ns = NB[c].stamp[q];
                    const PData nd = ND[c * PM_BKT + q];
                    NB[c].key[q] = ck; NB[c].stamp[q] = cs; ND[c * PM_BKT + q] = cd;
                    ck = nk; cs = ns; cd = nd;
                    c = pm_alt(nn, ck, c);
                }
                if (!placed) atomicOr(bflags, BF_PTAB_FULL);
            }
            PMap* hd = &S.pmap[id];
            hd->base = nbase;
            hd->nb = nn;
        }
        __builtin_amdgcn_wave_barrier();
    }
}
// Decide stage, before every kernel that touches the maps: the maps a segment may add keys to -- its QPS rules'
// maps and its thread-count maps -- grown for the segment's events (an upper bound of its accesses); one lane each.
// (Maps of STRATEGY_RELATE members, whose events sort under another resource, are grown to capacity at rule load.)
// Two passes a batch: the first asks for the on-device compaction when the pool runs short (rescue = the batch's
// epoch), the second runs only after one (PC_RESCUE = epoch) and finds the pool used up for real.
__global__ __launch_bounds__(256) void k_pm_grow(const Seg* __restrict__ segs, const uint32_t* __restrict__ mp, DevState S,
                                                 unsigned long long* pool_next, uint64_t pool_nb, uint32_t* bflags,
                                                 uint4* mv, uint32_t* nmv, uint32_t mcap, uint32_t epoch, uint32_t second) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (second && pool_next[PC_RESCUE] != epoch) return;
    if (s >= *mp) return;
    const Seg sg = segs[s];
    const Prog pg = S.prog[sg.res];
    if (pg.tm_base == NO_ID && pg.n_param == 0) return;
    // an argument that is a Collection / array is one access per element (PM_ARGL): no bound, full size
    const uint64_t adds = (S.prio && (S.prio[sg.res] & PM_ARGL)) ? 0xFFFFFFFFull : (uint64_t)sg.len;
    for (int k = 0; k < pg.n_param; ++k) {
        const DRule& r = S.rules[pg.rule_off + k];
        if (r.behavior != PB_INIT_ONLY && r.grade == SG_FLOW_GRADE_QPS)
            pm_grow(S, r.pmap, adds, pool_next, pool_nb, bflags, mv, nmv, mcap, second ? 0u : epoch);
    }
    if (pg.tm_base != NO_ID)
        for (int i = 0; i < SG_MAX_ARGS; ++i) {
            const uint32_t id = S.tmid[pg.tm_base + i];
            if (id != NO_ID) pm_grow(S, id, adds, pool_next, pool_nb, bflags, mv, nmv, mcap, second ? 0u : epoch);
        }
}
// listed maps to full size (rule load: STRATEGY_RELATE members)
__global__ void k_pm_grow_ids(const uint32_t* __restrict__ ids, uint32_t n, DevState S, unsigned long long* pool_next,
                              uint64_t pool_nb, uint32_t* bflags) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) pm_grow(S, ids[i], 0xFFFFFFFFull, pool_next, pool_nb, bflags);
}

// ---- pool compaction on the device: every map's region, back to back in map order, into the other pool (the
// regions maps grew out of are dropped); the rings stay where they are.  Between batches (engine.cpp compact_pmaps,
// ctl = null) the pools then swap; inside a batch whose growth found the pool short (ctl[PC_RESCUE] = epoch: every
// kernel of the chain returns at once otherwise) the compacted prefix is copied back (k_pc_back), so the kernels
// already queued with this pool's address see the maps in place.
// (grid-stride over the maps: inside a batch the chain is launched every time and must cost a few microseconds when
// no rescue is due; cnt (optional): the scan's device count, n on a rescue and 0 otherwise)
__global__ void k_pc_nb(const PMap* __restrict__ pm, uint32_t n, uint32_t* __restrict__ sz,
                        const unsigned long long* __restrict__ ctl, uint32_t epoch, uint32_t* __restrict__ cnt) {
    const bool go = !ctl || ctl[PC_RESCUE] == epoch;
    if (cnt && blockIdx.x == 0 && threadIdx.x == 0) *cnt = go ? n : 0u;
    if (!go) return;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) sz[i] = pm[i].nb;
}
// a wavefront per map: buckets (128 B) and values (8 x 16 B a bucket) as 16-byte words; the header's base last
__global__ __launch_bounds__(256) void k_pc_copy(PMap* __restrict__ pm, uint32_t n, const uint32_t* __restrict__ off,
                                                 const PBucket* __restrict__ ob, const PData* __restrict__ od,
                                                 PBucket* __restrict__ nbk, PData* __restrict__ nd,
                                                 unsigned long long* __restrict__ pool_next, uint32_t cond,
                                                 uint32_t epoch) {
    if (cond && pool_next[PC_RESCUE] != epoch) return;
    const uint32_t l = threadIdx.x & 63;
    for (uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += gridDim.x * 4) {  // (a wavefront per map)
    const PMap m = pm[i];
    const uint64_t nb = off[i];
    const uint4* sb = reinterpret_cast<const uint4*>(ob + m.base);
    uint4* db = reinterpret_cast<uint4*>(nbk + nb);
    for (uint32_t w = l; w < m.nb * 8u; w += 64) db[w] = sb[w];  // (PBucket: 8 x 16 B)
    const uint4* sd = reinterpret_cast<const uint4*>(od + m.base * PM_BKT);
    uint4* dd = reinterpret_cast<uint4*>(nd + nb * PM_BKT);
    for (uint32_t w = l; w < m.nb * PM_BKT; w += 64) dd[w] = sd[w];  // (PData: 16 B)
    if (l == 0) {
        pm[i].base = nb;
        if (i == n - 1) {
            pool_next[PC_NEXT] = nb + m.nb;
            pool_next[PC_FLOOR] = nb + m.nb;
        }
    }
    }
}
// the rescue's copy back: the compacted prefix [0, ctl[PC_NEXT]) of the other pool over this one
__global__ __launch_bounds__(256) void k_pc_back(PBucket* __restrict__ b1, PData* __restrict__ d1,
                                                 const PBucket* __restrict__ b2, const PData* __restrict__ d2,
                                                 unsigned long long* __restrict__ ctl, uint32_t epoch) {
    if (ctl[PC_RESCUE] != epoch) return;
    const uint64_t nb = ctl[PC_NEXT];
    const uint64_t nw = nb * 8, stride = (uint64_t)gridDim.x * blockDim.x;  // (PBucket: 8 x 16 B; PData: 16 B a slot)
    const uint4* sb = reinterpret_cast<const uint4*>(b2);
    uint4* db = reinterpret_cast<uint4*>(b1);
    const uint4* sd = reinterpret_cast<const uint4*>(d2);
    uint4* dd = reinterpret_cast<uint4*>(d1);
    for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += stride) {
        db[w] = sb[w];
        dd[w] = sd[w];
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) ctl[PC_RESCUES] += 1;
}

namespace sg {
hipError_t launch_scan_n(const uint32_t* in, uint32_t* out, uint64_t n, const uint32_t* ndev, uint32_t* part,
                         uint32_t* total, hipStream_t st);  // kernels.hip
// mv / nmv / mcap: the move list (null: each lane moves its maps itself)
// The batch's map growth (pool_next = the pool's control words): a first pass; then, only if that pass found the pool
// short, the compaction into the other pool (b2 / d2), its copy back and a second pass (every kernel of the rescue
// returns at once otherwise: no host round trip in the decide stage).  nm maps; sz / off / part: compaction scratch.
hipError_t launch_pm_grow(const Seg* segs, const uint32_t* mp, uint32_t mb, const DevState& S, unsigned long long* pool_next,
                          uint64_t pool_nb, uint32_t* bflags, uint4* mv, uint32_t* nmv, uint32_t mcap, uint32_t epoch,
                          uint32_t nm, PBucket* b2, PData* d2, uint32_t* sz, uint32_t* off, uint32_t* part,
                          hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                          hipStream_t st) {
    if (!mb) return hipSuccess;
    if (!mcap) mv = nullptr;
    for (uint32_t second = 0; second < 2; ++second) {
        if (mv) {
            const hipError_t e = hipMemsetAsync(nmv, 0, 4, st);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(k_pm_grow, dim3((mb + 255) / 256), dim3(256), 0, st, segs, mp, S, pool_next, pool_nb, bflags,
                           mv, nmv, mcap, epoch, second);
        if (mv) hipLaunchKernelGGL(k_pm_move_list, dim3(mcap < 16384 ? (mcap + 3) / 4 : 4096), dim3(256), 0, st, mv, nmv, mcap, S, bflags);
        if (second || !nm || !b2) break;
        // (a fixed small grid each: a batch without a rescue pays a few microseconds for the chain, not a grid over
        // every map; the scan runs over the device count, 0 then)
        uint32_t* cnt = part + mcap + 4095;  // (part: mcap + 4096 words, the scan uses nm / 4096 + 2 of them)
        const uint32_t gnb = std::min<uint32_t>((nm + 255) / 256, 1024u), gcp = std::min<uint32_t>((nm + 3) / 4, 2048u);
        hipLaunchKernelGGL(k_pc_nb, dim3(gnb), dim3(256), 0, st, S.pmap, nm, sz, (const unsigned long long*)pool_next,
                           epoch, cnt);
        const hipError_t e = launch_scan_n(sz, off, nm, cnt, part, nullptr, st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_pc_copy, dim3(gcp), dim3(256), 0, st, S.pmap, nm, off, S.pbkt, S.pdat, b2, d2,
                           pool_next, 1u, epoch);
        hipLaunchKernelGGL(k_pc_back, dim3(2048), dim3(256), 0, st, S.pbkt, S.pdat, b2, d2, pool_next, epoch);
    }
    return hipGetLastError();
}
// sz / off: n words each; part: scan partials
hipError_t launch_pm_compact(PMap* pm, uint32_t n, const PBucket* ob, const PData* od, PBucket* nbk, PData* nd,
                             uint32_t* sz, uint32_t* off, uint32_t* part, unsigned long long* pool_next,
                             hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                             hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_pc_nb, dim3(std::min<uint32_t>((n + 255) / 256, 1024u)), dim3(256), 0, st, pm, n, sz,
                       (const unsigned long long*)nullptr, 0u, (uint32_t*)nullptr);
    const hipError_t e = scan(sz, off, n, part, nullptr, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pc_copy, dim3(std::min<uint32_t>((n + 3) / 4, 2048u)), dim3(256), 0, st, pm, n, off, ob, od, nbk,
                       nd, pool_next, 0u, 0u);
    return hipGetLastError();
}
hipError_t launch_pm_grow_ids(const uint32_t* ids, uint32_t n, const DevState& S, unsigned long long* pool_next,
                              uint64_t pool_nb, uint32_t* bflags, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_pm_grow_ids, dim3((n + 255) / 256), dim3(256), 0, st, ids, n, S, pool_next, pool_nb, bflags);
    return hipGetLastError();
}
hipError_t launch_pq(int wide, const SEv* recs, const sg_event* ev, const uint32_t* vals, const Seg* segs,
                     const uint32_t* order, uint32_t m, const DevState& S, const DevCfg& cfg, int64_t t0, uint32_t* dec,
                     uint32_t* bflags, hipStream_t st) {
    if (!m) return hipSuccess;
    // the wide owner: 1024 lanes (128 VGPRs a lane: ~120 spilled) measured 15 % faster on C5 than 512 lanes with
    // 256 VGPRs and no spill (SG_DEBUG_FLAGS 128 selects that form, for A/B runs)
    SEv* r = const_cast<SEv*>(recs);  // (PQ_FULL reads the records only)
    if (S.key_ring) {  // the XF_PVPQ segments pvalue.hip decided: their statistics (the others' WGs return at once)
        if (wide) hipLaunchKernelGGL(k_pvf<16>, dim3(m), dim3(1024), 0, st, recs, segs, order, m, S, cfg, t0, dec, bflags);
        else hipLaunchKernelGGL(k_pvf<4>, dim3(m), dim3(256), 0, st, recs, segs, order, m, S, cfg, t0, dec, bflags);
    }
    if (wide && (cfg.dbg_flags & 128))
        hipLaunchKernelGGL((k_pq<8, PQ_FULL>), dim3(m), dim3(512), 0, st, r, ev, vals, segs, order, m, S, cfg, t0, dec, bflags);
    else if (wide)
        hipLaunchKernelGGL((k_pq<16, PQ_FULL>), dim3(m), dim3(1024), 0, st, r, ev, vals, segs, order, m, S, cfg, t0, dec, bflags);
    else hipLaunchKernelGGL((k_pq<4, PQ_FULL>), dim3(m), dim3(256), 0, st, r, ev, vals, segs, order, m, S, cfg, t0, dec, bflags);
    return hipGetLastError();
}
// XF_MIX segments: the pre pass (post = 0) before the cooperative owners, the post pass (post = 1) after them and
// k_fill; list = the narrow segments (k_pq<4>), list + wide_off the wide ones (k_pq<16>)
// rest / rest_n (optional): the wide segments pvalue.hip left, listed on the device: a few workgroups loop over
// them instead of one launched (and mostly idle: a k_pq<16> workgroup holds a CU's LDS) per wide segment
hipError_t launch_pq_mix(int post, SEv* recs, const sg_event* ev, const uint32_t* vals, const Seg* segs,
                         const uint32_t* list, uint32_t n_narrow, uint64_t wide_off, uint32_t n_wide, const DevState& S,
                         const DevCfg& cfg, int64_t t0, uint32_t* dec, uint32_t* bflags, hipStream_t st,
                         const uint32_t* rest, const uint32_t* rest_n) {
    if (n_wide && rest) {
        const uint32_t g = n_wide < 256 ? n_wide : 256;
        if (post) hipLaunchKernelGGL((k_pq_list<16, PQ_POST>), dim3(g), dim3(1024), 0, st, recs, ev, vals, segs, rest,
                                     rest_n, S, cfg, t0, dec, bflags);
        else hipLaunchKernelGGL((k_pq_list<16, PQ_PRE>), dim3(g), dim3(1024), 0, st, recs, ev, vals, segs, rest, rest_n,
                                S, cfg, t0, dec, bflags);
    } else if (n_wide) {
        if (post) hipLaunchKernelGGL((k_pq<16, PQ_POST>), dim3(n_wide), dim3(1024), 0, st, recs, ev, vals, segs,
                                     list + wide_off, n_wide, S, cfg, t0, dec, bflags);
        else hipLaunchKernelGGL((k_pq<16, PQ_PRE>), dim3(n_wide), dim3(1024), 0, st, recs, ev, vals, segs, list + wide_off,
                                n_wide, S, cfg, t0, dec, bflags);
    }
    if (n_narrow) {
        if (post) hipLaunchKernelGGL((k_pq<4, PQ_POST>), dim3(n_narrow), dim3(256), 0, st, recs, ev, vals, segs, list,
                                     n_narrow, S, cfg, t0, dec, bflags);
        else hipLaunchKernelGGL((k_pq<4, PQ_PRE>), dim3(n_narrow), dim3(256), 0, st, recs, ev, vals, segs, list, n_narrow,
                                S, cfg, t0, dec, bflags);
    }
    return hipGetLastError();
}
} // namespace sg
