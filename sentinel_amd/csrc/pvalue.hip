// pvalue.hip -- ParamFlowSlot's pre pass for the long segments of mixed resources (XF_MIX), value-parallel.
//
// k_pq decides a segment a tile at a time in one workgroup, so one hot resource's argument accesses run in series
// (C6: 2M accesses of one resource per batch).  For a resource with one QPS token-bucket rule
// (ParamFlowChecker.passDefaultLocalCheck, ParamFlowChecker.java:121-196) the verdict of an access depends only on
// the earlier accesses of the same value -- and on LRU residency in the rule's CacheMap (ParameterMetric.java:37-39,
// SURVEY Q13), whose closed form is the LRU stack distance: with prev(j) the previous access of access j's value,
//     j hits  <=>  D(j) = #{k in (prev(j), j) : prev(k) < prev(j)} < cap
// (the distinct values accessed since; DESIGN.md §9.1 has the derivation and the check against an exact LRU), and a
// first access of a value that was live at the segment start with recency rank r hits iff
//     r + #{first accesses k < j of values ranked below r or absent} < cap.
// So the pass runs over all long mixed segments of the batch at once:
//   prep     one workgroup per segment: eligibility, the accesses counted (the checks before any map access --
//            token count 0, acquire above maxCount -- decided here), the map's ring prefix counts;
//   fill     accesses in order into dense arrays, each value's group id from a per-segment hash table;
//   sort     the (group id, access) pairs, stable radix (kernels.hip): each value's accesses contiguous, in order;
//   prev     previous access of the same value; the first access probes the map (slot, recency rank, state);
//   blocks   prev / rank values sorted per 256-access block, for counts with an early exit at cap;
//   resid    hit / miss of every access;
//   walk     one lane per value through passDefaultLocalCheck (a miss re-inserts the value with a full bucket);
//            blocked ENTRYs get their word and RF_PBLK, exactly as k_pq's pre pass;
//   commit   one workgroup per segment: the map after the segment -- the cap most recent values (accessed ones by
//            last access, then untouched live ones in their old order) with fresh stamps, reused or new slots.
// Segments that are not eligible (more than one checked rule, a throttle, lists) keep the k_pq pre pass.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "chain.h"
#include "pmap.h"

using namespace sg;

#define PV_B 256u          // block of accesses with sorted prev / rank copies
#define PV_INF 0x7FFFFFFF  // rank of a value absent at the segment start
#define PV_NONE (-1)

__device__ __forceinline__ uint32_t pv_word(const PMap& m, int64_t s) {
    return (uint32_t)(((uint64_t)s & (uint64_t)((1ull << m.rb_log2) - 1)) >> 6);
}
// recency rank at the start (live keys more recent) of a live stamp, from the ring and its per-word prefix counts
__device__ __forceinline__ int32_t pv_rank(const PMap& m, const uint64_t* bm, const uint32_t* pre, int64_t s) {
    const uint64_t p = (uint64_t)s & (uint64_t)((1ull << m.rb_log2) - 1);
    const uint32_t below = pre[p >> 6] + (uint32_t)__popcll(bm[p >> 6] & ((1ull << (p & 63)) - 1ull));
    return (int32_t)m.live - 1 - (int32_t)below;
}

// the program's one checked param rule (QPS, DefaultController or throttle) and no other checked rule; -1: not eligible
__device__ __forceinline__ int pv_rule(const DevState& S, const Prog& pg) {
    int k1 = -1;
    for (int k = 0; k < pg.n_param; ++k) {
        const DRule& r = S.rules[pg.rule_off + k];
        if (r.behavior == PB_INIT_ONLY) continue;
        if (k1 >= 0 || r.param_idx != 0 || r.grade != SG_FLOW_GRADE_QPS ||
            (r.behavior != SG_CONTROL_BEHAVIOR_DEFAULT && r.behavior != SG_CONTROL_BEHAVIOR_RATE_LIMITER))
            return -1;  // (a throttle only in XF_PVPQ programs: XF_MIX has none)
        k1 = k;
    }
    return k1;
}

// the value's token count (a hot item's, else the rule's: int for passDefaultLocalCheck, long -- held clamped to int
// here -- for passThrottleLocalCheck)
__device__ __forceinline__ int32_t pv_tc(const DevState& S, const DRule& r, uint64_t key) {
    for (uint32_t i = 0; i < r.hot_n; ++i) {
        const DHot h = S.hot[r.hot_off + i];
        if (h.key == key) return h.count;
    }
    if (r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER)
        return r.token_count_l > 0x7FFFFFFF ? 0x7FFFFFFF : (int32_t)r.token_count_l;
    return r.token_count;
}

template <int NW>
__device__ __forceinline__ uint32_t pv_scan(uint32_t v, uint32_t* red, uint32_t* tot) {  // block exclusive scan
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
        if (l >= (uint32_t)o) x += y;
    }
    if (l == 63) red[w] = x;
    __syncthreads();
    uint32_t pre = 0, t = 0;
#pragma unroll
    for (int k = 0; k < NW; ++k) {
        const uint32_t c = red[k];
        if ((uint32_t)k < w) pre += c;
        t += c;
    }
    __syncthreads();
    *tot = t;
    return pre + x - v;
}

// the map's per-word live-stamp prefix counts in stamp order from thr (ppre: free scratch of this map here), by
// a 256-lane workgroup
__device__ void pv_ring_prefix(const DevState& S, const PMap& mp, uint32_t* red) {
    const uint32_t W = 1u << (mp.rb_log2 - 6), w0 = pv_word(mp, mp.thr);
    const uint32_t per = (W + 255) / 256, l0 = threadIdx.x * per;
    uint32_t c = 0;
    for (uint32_t u = 0; u < per; ++u)
        if (l0 + u < W) c += (uint32_t)__popcll(S.pbm[mp.bm + ((w0 + l0 + u) & (W - 1))]);
    uint32_t t2;
    uint32_t run = pv_scan<4>(c, red, &t2);
    for (uint32_t u = 0; u < per; ++u)
        if (l0 + u < W) {
            const uint32_t w = (w0 + l0 + u) & (W - 1);
            S.ppre[mp.bm + w] = run;
            run += (uint32_t)__popcll(S.pbm[mp.bm + w]);
        }
}

// ---- prep: one workgroup per listed segment: eligibility, extraction chunks (the map's ring prefix counts: k_pv_rpre)
// The chain test is the state after this batch's grants (CtSph.lookProcessChain): with every chain granted
// (grant_all, no STRATEGY_RELATE component in the list) a resource without NI_CHAIN gets one in this batch iff the
// segment holds an ENTRY that looks its chain up (k_chain), so prep may run beside the grants (launch_pv_a early,
// beside the previous batch's decide stage) and still routes every segment the same way.
#define PV_CH 4096u  // positions per extraction chunk
__global__ __launch_bounds__(256) void k_pv_prep(const SEv* __restrict__ recs, const uint32_t* __restrict__ vals,
                                                 Seg* __restrict__ segs, const uint32_t* __restrict__ list, uint32_t m,
                                                 DevState S, PvSeg* __restrict__ pv, uint32_t* __restrict__ rest,
                                                 uint32_t grant_all) {
    __shared__ uint32_t okf, look, scan_f;
    const uint32_t i = blockIdx.x, tid = threadIdx.x;
    if (i >= m) return;
    const Seg sg = segs[list[i]];
    const Prog pg = S.prog[sg.res];
    const int k1 = pv_rule(S, pg);
    // The node's flags are read ONCE (thread 0) and broadcast: with the early pre pass k_chain may set NI_CHAIN
    // beside this kernel, and every wave must take the same branch around the barriers below.
    if (tid == 0) {
        const uint32_t f = S.info[sg.res].flags;
        // eligible: one checked rule, its map within the commit's LDS (<= PQ_MAX_CAP), no argument lists, a chain
        uint32_t ok = k1 >= 0 && !(S.prio && (S.prio[sg.res] & PM_ARGL));
        if (ok && S.pmap[S.rules[pg.rule_off + k1].pmap].cap > PQ_MAX_CAP) ok = 0;
        const bool chain = (f & NI_CHAIN) != 0;
        const bool scan = ok && !chain && grant_all && !(f & NI_REJECTED) && !(pg.multi & PX_MULTI);
        okf = ok && chain;  // final unless the ENTRY scan below runs
        scan_f = scan ? 1u : 0u;
        look = 0;
    }
    __syncthreads();
    if (__builtin_amdgcn_readfirstlane((int)scan_f)) {
        for (uint32_t p0 = 0; p0 < sg.len; p0 += 256) {  // (uniform trip count; the first ENTRY is near the start)
            const uint32_t p = p0 + tid;
            if (p < sg.len && recs[sg.start + p].kind == SG_EV_ENTRY &&
                (!S.ext || S.ext[vals[sg.start + p] & 0x7FFFFFFFu].context_id <= S.max_ctx))
                look = 1;
            if (__syncthreads_or(look)) break;
        }
        if (tid == 0) okf = look != 0;  // (ok held: the scan runs only for an eligible segment)
        __syncthreads();
    }
    if (!__builtin_amdgcn_readfirstlane((int)okf)) {  // k_pq's pre pass: rest[1 + k], count rest[0] (an XF_PVPQ segment: k_pq's full pass decides it)
        if (tid == 0) {
            PvSeg z{};
            z.ok = 0;
            pv[i] = z;
            if (!(pg.xf & XF_PVPQ)) rest[1 + atomicAdd(&rest[0], 1u)] = list[i];
        }
        return;
    }
    const DRule& r = S.rules[pg.rule_off + k1];
    if (tid == 0) {
        PvSeg o{};
        o.ok = 1; o.mid = r.pmap; o.rk = (uint32_t)k1; o.nch = (sg.len + PV_CH - 1) / PV_CH;
        pv[i] = o;
        segs[list[i]].bin = sg.bin | SEG_PV;  // (k_pq's pre pass leaves it)
    }
}

// the maps' ring prefix counts of the eligible segments (after the maps' growth: a map region moves)
__global__ __launch_bounds__(256) void k_pv_rpre(const PvSeg* __restrict__ pv, uint32_t m, DevState S) {
    __shared__ uint32_t red[4];
    const uint32_t i = blockIdx.x;
    if (i >= m || !pv[i].ok) return;
    pv_ring_prefix(S, S.pmap[pv[i].mid], red);
}

// the chunk table: (listed segment, first position) of every chunk, segment by segment; tot[1] = chunks
__global__ __launch_bounds__(256) void k_pv_chunks(PvSeg* __restrict__ pv, uint32_t m, PvBuf B, uint32_t* __restrict__ tot) {
    __shared__ uint32_t red[4];
    uint32_t base = 0;
    for (uint32_t c = 0; c < m; c += 256) {
        const uint32_t i = c + threadIdx.x;
        const uint32_t v = i < m ? pv[i].nch : 0u;
        uint32_t t;
        const uint32_t o = base + pv_scan<4>(v, red, &t);
        if (i < m) {
            pv[i].ch0 = o;
            for (uint32_t k = 0; k < v; ++k) B.chunk[o + k] = make_uint2(i, k * PV_CH);
        }
        base += t;
    }
    if (threadIdx.x == 0) tot[1] = base;
}

// ---- count: one workgroup per chunk: its accesses; the checks before any map access decided here
__global__ __launch_bounds__(256) void k_pv_count(SEv* __restrict__ recs, const uint32_t* __restrict__ vals,
                                                  const Seg* __restrict__ segs, const uint32_t* __restrict__ list,
                                                  DevState S, DevCfg cfg, const PvSeg* __restrict__ pv, PvBuf B,
                                                  const uint32_t* __restrict__ tot, uint32_t* __restrict__ dec) {
    __shared__ uint32_t red[4];
    const uint32_t c = blockIdx.x, tid = threadIdx.x;
    if (c >= tot[1]) return;
    const uint2 ch = B.chunk[c];
    const PvSeg ps = pv[ch.x];
    const Seg sg = segs[list[ch.x]];
    const DRule& r = S.rules[S.prog[sg.res].rule_off + ps.rk];
    const uint32_t end = sg.len - ch.y < PV_CH ? sg.len : ch.y + PV_CH;
    uint32_t cnt = 0;
    for (uint32_t p = ch.y + tid; p < end; p += 256) {
        const SEv e = recs[sg.start + p];
        if (e.kind != SG_EV_ENTRY || !(e.flags & SG_F_HAS_ARG)) continue;
        const uint64_t key = S.key_ring[(S.gbase + (vals[sg.start + p] & 0x7FFFFFFFu)) & cfg.ring_mask];
        const int32_t tc = pv_tc(S, r, key);
        const bool thr = r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER;
        if (tc == 0 || (!thr && (int32_t)e.cnt > j_iadd(tc, r.burst))) {  // blocked before any map access
            dec[sg.start + p] = mk_dec(ST_BLOCK_PARAM, r.slot, 0);
            recs[sg.start + p].flags = (uint8_t)(e.flags | RF_PBLK);
            continue;
        }
        ++cnt;
    }
    uint32_t t;
    (void)pv_scan<4>(cnt, red, &t);
    if (tid == 0) B.ccnt[c] = t;
}

// dense offsets: chunks' (exclusive scan), segments' first access and count; tot[0] = all accesses (one block)
__global__ __launch_bounds__(256) void k_pv_offsets(PvSeg* __restrict__ pv, uint32_t m, PvBuf B, uint32_t* __restrict__ tot) {
    __shared__ uint32_t red[4];
    const uint32_t nc = tot[1];
    uint32_t base = 0;
    for (uint32_t c = 0; c < nc; c += 256) {
        const uint32_t k = c + threadIdx.x;
        const uint32_t v = k < nc ? B.ccnt[k] : 0u;
        uint32_t t;
        const uint32_t o = pv_scan<4>(v, red, &t);
        if (k < nc) B.cof[k] = base + o;
        base += t;
    }
    if (threadIdx.x == 0) { B.cof[nc] = base; tot[0] = base; }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < m; i += 256) {
        if (!pv[i].ok) continue;
        const uint32_t a = B.cof[pv[i].ch0], e = B.cof[pv[i].ch0 + pv[i].nch];
        pv[i].off = a;
        pv[i].n = e - a;
    }
}

// ---- fill: one workgroup per chunk: accesses in order into the dense arrays, group ids from the segment's table
__global__ __launch_bounds__(256) void k_pv_fill(const SEv* __restrict__ recs, const uint32_t* __restrict__ vals,
                                                 const Seg* __restrict__ segs, const uint32_t* __restrict__ list,
                                                 DevState S, DevCfg cfg, const PvSeg* __restrict__ pv, PvBuf B,
                                                 const uint32_t* __restrict__ tot) {
    __shared__ uint32_t red[4];
    const uint32_t c = blockIdx.x, tid = threadIdx.x;
    if (c >= tot[1]) return;
    const uint2 ch = B.chunk[c];
    const PvSeg ps = pv[ch.x];
    const Seg sg = segs[list[ch.x]];
    const DRule& r = S.rules[S.prog[sg.res].rule_off + ps.rk];
    const uint32_t end = sg.len - ch.y < PV_CH ? sg.len : ch.y + PV_CH;
    const uint64_t H = 2ull * ps.n;  // the segment's table slots
    unsigned long long* tab = B.htab + 2ull * ps.off;
    uint32_t base = B.cof[c];
    for (uint32_t c0 = ch.y; c0 < end; c0 += 256) {  // (uniform trip count)
        const uint32_t p = c0 + tid;
        bool take = false;
        uint64_t key = 0;
        int32_t tc = 0;
        SEv e;
        if (p < end) {
            e = recs[sg.start + p];
            if (e.kind == SG_EV_ENTRY && (e.flags & SG_F_HAS_ARG) && !(e.flags & RF_PBLK)) {
                key = S.key_ring[(S.gbase + (vals[sg.start + p] & 0x7FFFFFFFu)) & cfg.ring_mask];
                tc = pv_tc(S, r, key);
                take = true;
            }
        }
        uint32_t t;
        const uint32_t o = pv_scan<4>(take ? 1u : 0u, red, &t);
        if (take) {
            const uint32_t g = base + o;
            B.key[g] = key;
            B.pos[g] = p;
            B.dt[g] = e.dt;
            B.acq[g] = e.cnt;
            B.tc[g] = tc;
            B.seg[g] = ch.x;
            B.prev[g] = PV_NONE;
            B.w[g] = -1;
            B.fslot[g] = -1;
            B.keep[g] = 0;
            uint64_t h = mix64(key ^ 0x5BD1E9955BD1E995ull) % H;  // the value's slot: its group id
            for (;;) {
                const unsigned long long cur = tab[h];
                if (cur == key) break;
                if (cur == PK_EMPTY) {
                    const unsigned long long prv = atomicCAS(&tab[h], (unsigned long long)PK_EMPTY, (unsigned long long)key);
                    if (prv == PK_EMPTY || prv == key) break;
                }
                h = h + 1 == H ? 0 : h + 1;
            }
            B.gid[g] = (uint32_t)(2ull * ps.off + h);
            B.idx[g] = g;
        }
        base += t;
    }
}

// padding of the sort arrays beyond the accesses: [tot, cap) sorts last
__global__ void k_pv_pad(PvBuf B, const uint32_t* __restrict__ tot, uint32_t cap) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < cap && g >= *tot) { B.gid[g] = 0xFFFFFFFFu; B.idx[g] = g; B.tc[g] = 0; }
}

// ---- prev / first accesses (sorted order: after the sort B.gid / B.idx hold the sorted keys / accesses)
__global__ void k_pv_prev(PvBuf B, const uint32_t* __restrict__ tot, const PvSeg* __restrict__ pv, DevState S) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= *tot) return;
    const uint32_t g = B.idx[q], gd = B.gid[q];
    const bool first = q == 0 || B.gid[q - 1] != gd;
    if (!first) { B.prev[g] = (int32_t)B.idx[q - 1]; return; }
    // the value's first access of the segment: its slot in the map, its rank (if live), its state
    const PvSeg ps = pv[B.seg[g]];
    const PMap mp = S.pmap[ps.mid];
    const uint64_t key = B.key[g];
    uint32_t b1, b2;
    pm_buckets(mp.nb, key, b1, b2);
    const PBucket* BK = S.pbkt + mp.base;
    int32_t slot = -1;
    for (int j = PM_BKT - 1; j >= 0; --j) if (BK[b2].key[j] == key) slot = (int32_t)(b2 * PM_BKT + j);
    for (int j = PM_BKT - 1; j >= 0; --j) if (BK[b1].key[j] == key) slot = (int32_t)(b1 * PM_BKT + j);
    B.fslot[g] = slot;
    int32_t w = PV_INF;
    if (slot >= 0) {
        const int64_t s = BK[slot / PM_BKT].stamp[slot % PM_BKT];
        if (pm_live(mp, S.pbm + mp.bm, s)) {
            w = pv_rank(mp, S.pbm + mp.bm, S.ppre + mp.bm, s);
            const PData d = S.pdat[mp.base * PM_BKT + slot];
            B.flast[g] = d.v0;
            B.ftok[g] = d.v1;
        }
    }
    B.w[g] = w;
}

// ---- blocks: prev and rank values sorted within each 256-access block (bitonic in LDS)
__global__ __launch_bounds__(256) void k_pv_blocks(PvBuf B, const uint32_t* __restrict__ tot) {
    __shared__ int32_t a[PV_B], b[PV_B];
    const uint32_t n = *tot, base = blockIdx.x * PV_B, t = threadIdx.x;
    if (base >= n) return;
    a[t] = base + t < n ? B.prev[base + t] : 0x7FFFFFFF;
    b[t] = base + t < n ? B.w[base + t] : 0x7FFFFFFF;
    __syncthreads();
    for (uint32_t k = 2; k <= PV_B; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            const uint32_t x = t ^ j;
            if (x > t) {
                const bool up = (t & k) == 0;
                if ((a[t] > a[x]) == up) { const int32_t v = a[t]; a[t] = a[x]; a[x] = v; }
                if ((b[t] > b[x]) == up) { const int32_t v = b[t]; b[t] = b[x]; b[x] = v; }
            }
            __syncthreads();
        }
    if (base + t < n) { B.sprev[base + t] = a[t]; B.sw[base + t] = b[t]; }
}

// #{k in (lo, hi) : prev[k] < v}, stopping once it reaches lim
__device__ int32_t pv_count_lt(const PvBuf& B, int64_t lo, int64_t hi, int32_t v, int32_t lim) {
    int32_t c = 0;
    int64_t k = lo + 1;
    while (k < hi && (k % PV_B) != 0) { c += B.prev[k] < v; ++k; }
    if (c >= lim) return c;
    while (k + PV_B <= hi) {
        const int32_t* s = B.sprev + k;
        uint32_t l = 0, h = PV_B;  // first element >= v
        while (l < h) { const uint32_t md = (l + h) >> 1; if (s[md] < v) l = md + 1; else h = md; }
        c += (int32_t)l;
        k += PV_B;
        if (c >= lim) return c;
    }
    while (k < hi) { c += B.prev[k] < v; ++k; }
    return c;
}
// #{k in [lo, hi) : w[k] > r}, stopping once it reaches lim
__device__ int32_t pv_count_gt(const PvBuf& B, int64_t lo, int64_t hi, int32_t r, int32_t lim) {
    int32_t c = 0;
    int64_t k = lo;
    while (k < hi && (k % PV_B) != 0) { c += B.w[k] > r; ++k; }
    if (c >= lim) return c;
    while (k + PV_B <= hi) {
        const int32_t* s = B.sw + k;
        uint32_t l = 0, h = PV_B;  // first element > r
        while (l < h) { const uint32_t md = (l + h) >> 1; if (s[md] <= r) l = md + 1; else h = md; }
        c += (int32_t)(PV_B - l);
        k += PV_B;
        if (c >= lim) return c;
    }
    while (k < hi) { c += B.w[k] > r; ++k; }
    return c;
}

// ---- residency of every access.  Exact counts (pv_count_lt / gt) only in a narrow band; around it bounds settle
// an access in O(1):
//   a repeat (prev p, at g): its window (p, g) holds fewer than cap values when g - p - 1 < cap; else by the
//     horizons Z[b] of the block starts P_b = 256 b (the end y of the shortest window (P_b, y) holding cap distinct
//     values, cap of P_b's segment): windows (P_b1, g) and (P_b2, g), b1 = p / 256 < b2, enclose / lie inside
//     (p, g), so g < Z[b1] is a hit (P_b1 in the segment) and g >= Z[b2] a miss;
//   a first access of a value of rank r: hit iff r + #(earlier first accesses of values absent or ranked below r)
//     < cap; that count lies between the segment's earlier new values (NN) and earlier first accesses (NF).
__global__ void k_pv_fflags(PvBuf B, const uint32_t* __restrict__ tot, uint32_t cap) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= cap || g >= *tot) return;  // (the scans run over the accesses only)
    const int32_t w = B.w[g];
    reinterpret_cast<uint32_t*>(B.gdt)[g] = w >= 0 ? 1u : 0u;  // -> NF (scan)
    B.gaw[g] = w == PV_INF ? 1u : 0u;                          // -> NN (scan)
}
// one wavefront per block start: Z[b] (0xFFFFFFFF: the accesses end first), 64 blocks a round
__global__ __launch_bounds__(256) void k_pv_horizon(PvBuf B, const uint32_t* __restrict__ tot,
                                                    const PvSeg* __restrict__ pv, DevState S,
                                                    uint32_t* __restrict__ Z) {
    const uint32_t b = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
    const uint32_t n = *tot;
    if ((uint64_t)b * PV_B >= n) return;
    const int32_t P = (int32_t)(b * PV_B);
    const int32_t cap = (int32_t)S.pmap[pv[B.seg[P]].mid].cap;
    const uint32_t nblk = (n + PV_B - 1) / PV_B;
    int32_t need = cap;
    uint32_t z = 0xFFFFFFFFu;
    for (uint32_t c0 = b; c0 < nblk; c0 += 64) {
        const uint32_t c = c0 + l;
        int32_t cnt = 0;
        if (c < nblk) {  // #{k in block c, k > P : prev(k) <= P}
            const int32_t* sp = B.sprev + (uint64_t)c * PV_B;
            uint32_t lo = 0, hi = PV_B;
            while (lo < hi) { const uint32_t md = (lo + hi) >> 1; if (sp[md] <= P) lo = md + 1; else hi = md; }
            cnt = (int32_t)lo - (c == b ? 1 : 0);  // (k = P itself: prev(P) < P)
        }
        int32_t inc = cnt;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int32_t y = __shfl_up(inc, o, 64);
            if (l >= (uint32_t)o) inc += y;
        }
        const uint64_t reach = __ballot(inc >= need);
        if (reach) {
            const uint32_t lf = (uint32_t)__ffsll((unsigned long long)reach) - 1;
            int32_t left = need - __shfl(inc - cnt, lf, 64);  // values still to find inside block c0 + lf
            const uint32_t k0 = (c0 + lf) * PV_B;
            for (uint32_t r = 0; r < PV_B; r += 64) {  // positions in order, a wavefront at a time
                const uint32_t k = k0 + r + l;
                const bool f = k < n && (int32_t)k > P && B.prev[k] <= P;
                const uint64_t bm = __ballot(f);
                const int32_t nf = __popcll(bm);
                if (nf >= left) {  // the left-th flagged position
                    uint64_t x = bm;
                    for (int q = 1; q < left; ++q) x &= x - 1;
                    z = k0 + r + (uint32_t)(__ffsll((unsigned long long)x) - 1) + 1;
                    break;
                }
                left -= nf;
            }
            break;
        }
        need -= __shfl(inc, 63, 64);
    }
    if (l == 0) Z[b] = z;
}
__global__ void k_pv_resid(PvBuf B, const uint32_t* __restrict__ tot, const PvSeg* __restrict__ pv, DevState S,
                           const uint32_t* __restrict__ NF, const uint32_t* __restrict__ NN,
                           const uint32_t* __restrict__ Z) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= *tot) return;
    const PvSeg ps = pv[B.seg[g]];
    const int32_t cap = (int32_t)S.pmap[ps.mid].cap;
    const int32_t p = B.prev[g];
    bool hit;
    if (p >= 0) {
        if ((int64_t)g - p - 1 < cap) hit = true;
        else {
            const uint32_t b1 = (uint32_t)p / PV_B;  // (Z[b1] only from inside the segment: its cap)
            if (b1 * PV_B >= ps.off && g < Z[b1]) hit = true;
            else if (g >= Z[b1 + 1]) hit = false;
            else hit = pv_count_lt(B, p, g, p, cap) < cap;
        }
    } else {
        const int32_t r = B.w[g];
        if (r == PV_INF) hit = false;
        else {
            const int32_t nf = (int32_t)(NF[g] - NF[ps.off]), nn = (int32_t)(NN[g] - NN[ps.off]);
            if (r + nf < cap) hit = true;
            else if (r + nn >= cap) hit = false;
            else hit = pv_count_gt(B, ps.off, g, r, cap - r) < cap - r;
        }
    }
    B.hit[g] = hit ? 1 : 0;
}

// ---- gather: the walk's inputs in sorted order (each value's accesses contiguous), misses per 256 positions
__global__ void k_pv_gather(const Seg* __restrict__ segs, const uint32_t* __restrict__ list, PvBuf B,
                            const uint32_t* __restrict__ tot) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= *tot) return;
    const uint32_t g = B.idx[q];
    B.gdt[q] = B.dt[g];
    const bool hit = B.hit[g] != 0;
    B.gaw[q] = (B.acq[g] & 0xFFFFu) | (hit ? 0x10000u : 0u);
    B.gpos[q] = segs[list[B.seg[g]]].start + B.pos[g];
    reinterpret_cast<uint32_t*>(B.sw)[q] = hit ? 0u : 1u;  // -> MC: misses before each sorted position (scan)
}

// the value groups of the sorted accesses, densely: F[q] = q starts a group (scan -> its index), list G[index] = q
__global__ void k_pv_gflags(PvBuf B, const uint32_t* __restrict__ tot, uint32_t cap, uint32_t* __restrict__ F) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= cap || q >= *tot) return;  // (the scans run over the accesses only)
    F[q] = q == 0 || B.gid[q] != B.gid[q - 1] ? 1u : 0u;
}
__global__ void k_pv_glist(PvBuf B, const uint32_t* __restrict__ tot, const uint32_t* __restrict__ X,
                           uint32_t* __restrict__ G) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= *tot) return;
    if (q == 0 || B.gid[q] != B.gid[q - 1]) G[X[q]] = q;
}

// first miss in sorted positions [lo, hi) (hi if none); MC = exclusive scan of the miss flags (binary search)
__device__ uint32_t pv_first_miss(const PvBuf& B, const uint32_t* __restrict__ MC, uint32_t lo, uint32_t hi) {
    if (lo >= hi) return hi;
    const uint32_t m0 = MC[lo];
    const uint32_t mend = MC[hi - 1] + ((B.gaw[hi - 1] & 0x10000u) ? 0u : 1u);  // misses before hi
    if (mend == m0) return hi;
    uint32_t a = lo + 1, b = hi;  // the first y in (lo, hi] with misses-before(y) > m0 is the miss + 1
    while (a < b) {
        const uint32_t md = (a + b) >> 1;
        if (MC[md] > m0) b = md; else a = md + 1;
    }
    return a - 1;
}

// ---- walk: one lane per value through passDefaultLocalCheck.  Once the bucket is empty, every access up to the
// next refill (pass time > durationInSec) blocks without a state change -- unless an acquire is 0 (jumps off for a
// batch with such ENTRYs: BF_ZERO_CNT) or a miss re-inserts the value -- so the lane jumps there by binary search
// over the value's times and leaves the stretch's verdicts to k_pv_ranges: a hot value is ~ (batch seconds /
// durationInSec) x maxCount steps, not one step an access.
__global__ void k_pv_walk(SEv* __restrict__ recs, const Seg* __restrict__ segs, const uint32_t* __restrict__ list,
                          PvBuf B, uint32_t* __restrict__ tot, const PvSeg* __restrict__ pv, DevState S, int64_t t0,
                          uint32_t* __restrict__ dec, uint32_t jumps, uint32_t range_cap, uint32_t* __restrict__ bflags,
                          const uint32_t* __restrict__ GL) {
    const uint32_t gi = blockIdx.x * blockDim.x + threadIdx.x;  // the value group (GL: their starts, tot[8] of them)
    const uint32_t n = tot[0], ng = tot[8];
    if (gi >= ng) return;
    const uint32_t q0 = GL[gi], qb = gi + 1 < ng ? GL[gi + 1] : n;
    const uint32_t g0 = B.idx[q0];
    const uint32_t si = B.seg[g0];
    const PvSeg ps = pv[si];
    const Seg sg = segs[list[si]];
    const DRule& r = S.rules[S.prog[sg.res].rule_off + ps.rk];
    const int64_t D = r.duration_sec * 1000;
    const int32_t tc = B.tc[g0], maxc = j_iadd(tc, r.burst);
    const uint32_t blk = mk_dec(ST_BLOCK_PARAM, r.slot, 0);
    const bool thr = r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER;  // passThrottleLocalCheck (XF_PVPQ only)
    const bool pvpq = (S.prog[sg.res].xf & XF_PVPQ) != 0;             // passed words are final: written here
    int64_t last = B.flast[g0];  // (valid when the first access hits: the value was live)
    int32_t tok = thr ? 0 : B.ftok[g0];  // (a throttle map's second value stays 0)
    uint32_t q = q0, steps = 0;
    while (q < qb) {
        ++steps;
        const int64_t t = t0 + B.gdt[q];
        const uint32_t aw = B.gaw[q];
        const int32_t a = (int32_t)(aw & 0xFFFFu);
        if (thr) {  // ParamFlowChecker.java:198-248: timeRecorderMap, the expected pass time within maxQueueingTime
            bool pass = true;
            int64_t wt = 0;
            if (!(aw & 0x10000u)) {
                last = t;
            } else {
                const int64_t cost = j_round(1.0 * 1000 * a * (double)r.duration_sec / (double)tc);
                const int64_t expected = last + cost;
                if (expected <= t || expected - t < r.max_queue) {
                    wt = expected - t;
                    last = wt > 0 ? expected : t;
                } else {
                    pass = false;
                }
            }
            const uint32_t rp = B.gpos[q];
            if (!pass) {
                dec[rp] = blk;
                recs[rp].flags = (uint8_t)(recs[rp].flags | RF_PBLK);
            } else if (pvpq) {
                dec[rp] = mk_dec(ST_PASS, 0, wt);
            }
            ++q;
            if (!pass && jumps && q < qb) {
                // every access before last + cost(1) - (maxQueue - 1) blocks (cost grows with the acquire)
                const int64_t c1 = j_round(1.0 * 1000 * 1 * (double)r.duration_sec / (double)tc);
                const int64_t lim64 = last + c1 - (r.max_queue > 0 ? r.max_queue - 1 : 0) - 1 - t0;  // blocked: dt <= lim
                const int32_t lim = lim64 > 0x7FFFFFFF ? 0x7FFFFFFF : lim64 < -0x7FFFFFFF ? -0x7FFFFFFF : (int32_t)lim64;
                uint32_t lo = q, hi = qb;
                while (lo < hi) { const uint32_t md = (lo + hi) >> 1; if (B.gdt[md] <= lim) lo = md + 1; else hi = md; }
                const uint32_t tgt = pv_first_miss(B, reinterpret_cast<const uint32_t*>(B.sw), q, lo);
                if (tgt > q + 8) {
                    const uint32_t k = atomicAdd(&tot[2], 1u);
                    if (k < range_cap) { B.range[k] = make_uint4(q, tgt, blk, 0u); q = tgt; }
                    else atomicSub(&tot[2], 1u);
                }
            }
            continue;
        }
        bool pass;
        if (!(aw & 0x10000u)) {  // a miss: inserted (timeCounters / tokenCounters.putIfAbsent)
            last = t;
            tok = j_iadd(maxc, -a);
            pass = true;
        } else {
            const int64_t pt = t - last;
            if (pt > D) {
                const int32_t add = (int32_t)((pt * (int64_t)tc) / D);
                const int32_t sum = j_iadd(tok, add);
                const int32_t nq = sum > maxc ? j_iadd(maxc, -a) : j_iadd(sum, -a);
                pass = nq >= 0;
                if (pass) { tok = nq; last = t; }
            } else {
                pass = j_iadd(tok, -a) >= 0;
                if (pass) tok = j_iadd(tok, -a);
            }
        }
        if (!pass) {
            const uint32_t rp = B.gpos[q];
            dec[rp] = blk;
            recs[rp].flags = (uint8_t)(recs[rp].flags | RF_PBLK);
        } else if (pvpq) {
            dec[B.gpos[q]] = mk_dec(ST_PASS, 0, 0);
        }
        ++q;
        if (jumps && tok == 0 && q < qb) {
            // the first access that may refill: time > last + D (times are non-decreasing within the value)
            const int64_t lim64 = last + D - t0;
            const int32_t lim = lim64 > 0x7FFFFFFF ? 0x7FFFFFFF : (int32_t)lim64;
            uint32_t lo = q, hi = qb;
            while (lo < hi) { const uint32_t md = (lo + hi) >> 1; if (B.gdt[md] <= lim) lo = md + 1; else hi = md; }
            const uint32_t tgt = pv_first_miss(B, reinterpret_cast<const uint32_t*>(B.sw), q, lo);
            if (tgt > q + 8) {  // a stretch of blocks: to k_pv_ranges
                const uint32_t k = atomicAdd(&tot[2], 1u);
                if (k < range_cap) { B.range[k] = make_uint4(q, tgt, blk, 0u); q = tgt; }
                else atomicSub(&tot[2], 1u);  // (full: walk it)
            }
        }
    }
    if (steps > 256) atomicMax(&tot[3], steps);  // (diagnostics: the longest walk)
    // the value's last access g: it stays iff fewer than cap distinct values are accessed after it, i.e. it is among
    // the segment's cap latest last accesses (the commit counts them with a scan)
    const uint32_t g = B.idx[qb - 1];
    B.keep[g] = 1;  // (the commit keeps the cap latest of these)
    B.flast[g] = last;
    B.ftok[g] = tok;
    B.fslot[g] = B.fslot[g0];  // (the value's slot, carried to its last access for the commit)
}

// blocked stretches of the walk: a workgroup per stretch
__global__ __launch_bounds__(256) void k_pv_ranges(SEv* __restrict__ recs, PvBuf B, const uint32_t* __restrict__ tot,
                                                   uint32_t range_cap, uint32_t* __restrict__ dec) {
    const uint32_t nr = tot[2] < range_cap ? tot[2] : range_cap;
    for (uint32_t k = blockIdx.x; k < nr; k += gridDim.x) {
        const uint4 rg = B.range[k];
        for (uint32_t q = rg.x + threadIdx.x; q < rg.y; q += 256) {
            const uint32_t rp = B.gpos[q];
            dec[rp] = rg.z;
            recs[rp].flags = (uint8_t)(recs[rp].flags | RF_PBLK);
        }
    }
}

// ==== the post pass (ParamFlowStatisticEntryCallback / ExitCallback from the final verdicts, k_pq PQ_POST):
// thread-count map of paramIdx 0, ParameterMetric.java:117-241 -- a passed ENTRY adds (putIfAbsent then increment),
// an EXIT of a passed ENTRY releases (an absent value is put at 0; at <= 0 removed).  Two cases per segment:
//   increments only (no release: C6's EXITs carry no args) -- every op touches and inserts, so residency is the
//     pre pass's LRU stack distance (k_pv_prev / blocks / resid over the thread-count map) and a value's count
//     restarts at 1 after each miss; the commit keeps the cap most recent, as the pre pass's;
//   with releases -- removals break the stack distance; under the hypothesis that the map never grows beyond cap
//     within the segment (no eviction) each value's ops are independent: one lane per value walks them, the map's
//     size over the segment is a scan of the walks' +1 / -1, and the commit keeps every value present at its last
//     op.  A segment whose peak passes cap is left to k_pq's sequential replay.
#define PVT_ADD 1u
#define PVT_SUB 3u

// rule k visited by an ENTRY of final word d (PQ_POST's prologue): passed -> every rule; blocked by param rule k ->
// rules 0..k; blocked by a later slot -> every rule
__device__ __forceinline__ uint32_t pvt_stq(const DevState& S, const Prog& pg, uint32_t d) {
    if (st_passed(d & 0xFFu)) return 0;
    uint32_t stq = (uint32_t)pg.n_param + 1;
    if ((d & 0xFFu) == ST_BLOCK_PARAM)
        for (int k = 0; k < pg.n_param; ++k) {
            const DRule& r = S.rules[pg.rule_off + k];
            if (r.behavior != PB_INIT_ONLY && r.slot == ((d >> 8) & 0xFFu)) stq = (uint32_t)k + 1;
        }
    return stq;
}
__device__ __forceinline__ uint32_t pvt_kbits(const DRule& r) {
    return r.behavior == PB_INIT_ONLY ? (uint32_t)r.burst << NI_TM_SHIFT
                                      : NI_PM | (r.param_idx < SG_MAX_ARGS ? ni_tm((uint32_t)r.param_idx) : 0u);
}

// the op of segment position p (k_pq phase 3 of the post pass) and its value's key
__device__ __forceinline__ uint32_t pvt_op(const SEv& e, uint32_t p, const Seg& sg, uint32_t tm_from,
                                           const sg_event* __restrict__ ev, const uint32_t* __restrict__ vals,
                                           const DevState& S, const DevCfg& cfg, const uint32_t* __restrict__ dec,
                                           uint64_t& key) {
    const uint32_t gp = sg.start + p;
    if (e.kind == SG_EV_ENTRY) {
        if (!(e.flags & SG_F_HAS_ARG) || !st_passed(dec[gp] & 0xFFu)) return 0;
        key = S.key_ring[(S.gbase + (vals[gp] & 0x7FFFFFFFu)) & cfg.ring_mask];
        return PVT_ADD;
    }
    if (e.kind != SG_EV_EXIT || !(e.flags & SG_F_EXIT_ARGS) || p < tm_from) return 0;
    const bool own = (e.flags & RF_OWN_ARGS) != 0;
    uint64_t ref = SG_REF_NONE;
    uint32_t op = 0;
    if (e.code == RC_PASSED) {
        if (!own) ref = ev[vals[gp] & 0x7FFFFFFFu].aux & SG_REF_NONE;
        op = PVT_SUB;
    } else if (e.code == RC_NONE && own) {
        op = PVT_SUB;
    } else if (e.code == RC_BATCH) {
        const uint32_t rel = e.x - sg.start;
        if (rel < p) {
            ref = S.gbase + (vals[e.x] & 0x7FFFFFFFu);
            op = st_passed(dec[e.x] & 0xFFu) ? PVT_SUB : 0u;
        }
    }
    if (op) {
        if (own) ref = S.gbase + (vals[gp] & 0x7FFFFFFFu);
        key = S.key_ring[ref & cfg.ring_mask];
        if (key == NO_KEY) op = 0;
    }
    return op;
}

// per listed segment (a workgroup each): eligibility -- a chain, a thread-count map of paramIdx 0 that is on, within
// the commit's LDS, no THREAD-grade rule (XF_MIX) -- the first rule whose visit sets the map's bit (k0), the map's
// ring prefix counts (ranks of the increments-only case)
__global__ __launch_bounds__(256) void k_pvt_prep(const Seg* __restrict__ segs, const uint32_t* __restrict__ list,
                                                  uint32_t m, DevState S, PvSeg* __restrict__ pv) {
    __shared__ uint32_t red[4];
    __shared__ uint32_t okf;
    const uint32_t i = blockIdx.x;
    if (i >= m) return;
    const Seg sg = segs[list[i]];
    const Prog pg = S.prog[sg.res];
    const uint32_t flags = S.info[sg.res].flags;
    const uint32_t tm = pg.tm_base == NO_ID ? NO_ID : S.tmid[pg.tm_base];
    if (threadIdx.x == 0) {
        PvSeg o{};
        uint32_t all_bits = NI_PM, k0 = 0xFFFFFFFFu;
        bool thr = false;
        for (int k = 0; k < pg.n_param; ++k) {
            const DRule& r = S.rules[pg.rule_off + k];
            const uint32_t b = pvt_kbits(r);
            all_bits |= b;
            if (k0 == 0xFFFFFFFFu && (b & ni_tm(0))) k0 = (uint32_t)k;
            if (r.behavior != PB_INIT_ONLY && r.grade == SG_FLOW_GRADE_THREAD) thr = true;
        }
        bool ok = (flags & NI_CHAIN) && tm != NO_ID && S.key_ring && !thr && ((flags | all_bits) & ni_tm(0));
        if ((pg.xf & XF_PVPQ) && !(sg.bin & SEG_PV)) ok = false;  // (k_pq's full pass took its thread-count map)
        if (ok) {
            const PMap mp = S.pmap[tm];
            ok = mp.cap <= PQ_MAX_CAP && (mp.rb_log2 - 6) <= 9;
        }
        if (ok) {
            o.ok = 1; o.mid = tm; o.rk = k0; o.nch = (sg.len + PV_CH - 1) / PV_CH;
            o.freach = 0xFFFFFFFFu;
            o.tm0 = (flags & (NI_PM | ni_tm(0))) == (NI_PM | ni_tm(0)) ? 1u : 0u;
        }
        pv[i] = o;
        okf = o.ok;
    }
    __syncthreads();
    if (okf) pv_ring_prefix(S, S.pmap[tm], red);
}

// per chunk: the rules its ENTRYs visited (the node's bits) and the first ENTRY visiting rule k0
__global__ __launch_bounds__(256) void k_pvt_reach(const SEv* __restrict__ recs, const Seg* __restrict__ segs,
                                                   const uint32_t* __restrict__ list, DevState S, PvSeg* __restrict__ pv,
                                                   PvBuf B, const uint32_t* __restrict__ tot,
                                                   const uint32_t* __restrict__ dec) {
    __shared__ uint32_t sb, sr;
    const uint32_t c = blockIdx.x, tid = threadIdx.x;
    if (c >= tot[1]) return;
    if (tid == 0) { sb = 0; sr = 0xFFFFFFFFu; }
    __syncthreads();
    const uint2 ch = B.chunk[c];
    const PvSeg ps = pv[ch.x];
    const Seg sg = segs[list[ch.x]];
    const Prog pg = S.prog[sg.res];
    const uint32_t end = sg.len - ch.y < PV_CH ? sg.len : ch.y + PV_CH;
    uint32_t fb = 0, fr = 0xFFFFFFFFu;
    for (uint32_t p = ch.y + tid; p < end; p += 256) {
        if (recs[sg.start + p].kind != SG_EV_ENTRY) continue;
        const uint32_t stq = pvt_stq(S, pg, dec[sg.start + p]);
        for (int k = 0; k < pg.n_param; ++k)
            if (stq == 0 || stq > (uint32_t)k) {
                fb |= pvt_kbits(S.rules[pg.rule_off + k]) | NI_PM;
                if ((uint32_t)k == ps.rk && p + 1 < fr) fr = p + 1;
            }
    }
    if (fb) atomicOr(&sb, fb);
    if (fr != 0xFFFFFFFFu) atomicMin(&sr, fr);
    __syncthreads();
    if (tid == 0) {
        if (sb) atomicOr(&pv[ch.x].fbits, sb);
        if (sr != 0xFFFFFFFFu) atomicMin(&pv[ch.x].freach, sr);
    }
}

// per chunk: its ops
__global__ __launch_bounds__(256) void k_pvt_count(const SEv* __restrict__ recs, const sg_event* __restrict__ ev,
                                                   const uint32_t* __restrict__ vals, const Seg* __restrict__ segs,
                                                   const uint32_t* __restrict__ list, DevState S, DevCfg cfg,
                                                   PvSeg* __restrict__ pv, PvBuf B, const uint32_t* __restrict__ tot,
                                                   const uint32_t* __restrict__ dec) {
    __shared__ uint32_t red[4];
    const uint32_t c = blockIdx.x, tid = threadIdx.x;
    if (c >= tot[1]) return;
    const uint2 ch = B.chunk[c];
    const PvSeg ps = pv[ch.x];
    const Seg sg = segs[list[ch.x]];
    const uint32_t tm_from = ps.tm0 ? 0u : ps.freach;
    const uint32_t end = sg.len - ch.y < PV_CH ? sg.len : ch.y + PV_CH;
    uint32_t cnt = 0, sub = 0;
    for (uint32_t p = ch.y + tid; p < end; p += 256) {
        uint64_t key;
        const uint32_t op = pvt_op(recs[sg.start + p], p, sg, tm_from, ev, vals, S, cfg, dec, key);
        cnt += op ? 1u : 0u;
        sub |= op == PVT_SUB ? 1u : 0u;
    }
    uint32_t t;
    (void)pv_scan<4>(cnt, red, &t);
    if (tid == 0) B.ccnt[c] = t;
    if (sub) pv[ch.x].sub = 1;  // (any lane: one value)
}

// per chunk: the ops in order into the dense arrays (acq: the op), group ids from the segment's table
__global__ __launch_bounds__(256) void k_pvt_fill(const SEv* __restrict__ recs, const sg_event* __restrict__ ev,
                                                  const uint32_t* __restrict__ vals, const Seg* __restrict__ segs,
                                                  const uint32_t* __restrict__ list, DevState S, DevCfg cfg,
                                                  const PvSeg* __restrict__ pv, PvBuf B, const uint32_t* __restrict__ tot,
                                                  const uint32_t* __restrict__ dec) {
    __shared__ uint32_t red[4];
    const uint32_t c = blockIdx.x, tid = threadIdx.x;
    if (c >= tot[1]) return;
    const uint2 ch = B.chunk[c];
    const PvSeg ps = pv[ch.x];
    const Seg sg = segs[list[ch.x]];
    const uint32_t tm_from = ps.tm0 ? 0u : ps.freach;
    const uint32_t end = sg.len - ch.y < PV_CH ? sg.len : ch.y + PV_CH;
    const uint64_t H = 2ull * ps.n;
    unsigned long long* tab = B.htab + 2ull * ps.off;
    uint32_t base = B.cof[c];
    for (uint32_t c0 = ch.y; c0 < end; c0 += 256) {  // (uniform trip count)
        const uint32_t p = c0 + tid;
        uint64_t key = 0;
        const uint32_t op = p < end ? pvt_op(recs[sg.start + p], p, sg, tm_from, ev, vals, S, cfg, dec, key) : 0u;
        uint32_t t;
        const uint32_t o = pv_scan<4>(op ? 1u : 0u, red, &t);
        if (op) {
            const uint32_t g = base + o;
            B.key[g] = key;
            B.pos[g] = p;
            B.acq[g] = op;
            B.seg[g] = ch.x;
            B.tc[g] = 0;
            B.prev[g] = PV_NONE;
            B.w[g] = -1;
            B.fslot[g] = -1;
            B.keep[g] = 0;
            uint64_t h = mix64(key ^ 0x5BD1E9955BD1E995ull) % H;
            for (;;) {
                const unsigned long long cur = tab[h];
                if (cur == key) break;
                if (cur == PK_EMPTY) {
                    const unsigned long long prv = atomicCAS(&tab[h], (unsigned long long)PK_EMPTY, (unsigned long long)key);
                    if (prv == PK_EMPTY || prv == key) break;
                }
                h = h + 1 == H ? 0 : h + 1;
            }
            B.gid[g] = (uint32_t)(2ull * ps.off + h);
            B.idx[g] = g;
        }
        base += t;
    }
}

// one lane per value (sorted order; k_pv_prev probed the map at its first op: w = rank or PV_INF, flast = count).
// Increments only: c + 1 on a hit, 1 on a miss (put(v, 1) after an eviction); the value stays iff fewer than cap
// distinct values follow its last op.  With releases: the ops' state machine, tc[g] = the op's change of the
// map's size.
__global__ void k_pvt_walk(PvBuf B, const uint32_t* __restrict__ tot, const PvSeg* __restrict__ pv, DevState S) {
    const uint32_t q0 = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = tot[0];
    if (q0 >= n) return;
    const uint32_t gd = B.gid[q0];
    if (q0 > 0 && B.gid[q0 - 1] == gd) return;
    uint32_t qb = q0 + 1;
    while (qb < n && B.gid[qb] == gd) ++qb;  // (a value's ops: its passed ENTRYs and their EXITs)
    const uint32_t g0 = B.idx[q0];
    const PvSeg ps = pv[B.seg[g0]];
    bool pres = B.w[g0] != PV_INF;
    int64_t c = pres ? B.flast[g0] : 0;
    const uint32_t g = B.idx[qb - 1];
    if (!ps.sub) {
        for (uint32_t q = q0; q < qb; ++q) c = B.hit[B.idx[q]] ? c + 1 : 1;
        B.keep[g] = 1;  // (its last op: the commit keeps the cap latest)
    } else {
        for (uint32_t q = q0; q < qb; ++q) {
            const uint32_t gq = B.idx[q];
            int32_t d = 0;
            if (B.acq[gq] == PVT_ADD) {
                if (pres) ++c;
                else { pres = true; c = 1; d = 1; }
            } else {
                if (!pres) { pres = true; c = 0; d = 1; }
                else if (--c <= 0) { pres = false; c = 0; d = -1; }
            }
            B.tc[gq] = d;
        }
        B.keep[g] = pres ? 1 : 0;
    }
    B.flast[g] = c;
    B.ftok[g] = 0;
    B.fslot[g] = B.fslot[g0];
}

// the map's size over the segment: peak growth over its start size (X: exclusive scan of tc as uint32)
__global__ void k_pvt_peak(PvBuf B, const uint32_t* __restrict__ X, const uint32_t* __restrict__ tot,
                           PvSeg* __restrict__ pv) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    const bool in = g < tot[0];
    const uint32_t s = in ? B.seg[g] : 0xFFFFFFFFu;
    int32_t v = 0;
    if (in) v = (int32_t)(X[g] + (uint32_t)B.tc[g] - X[pv[s].off]);
    const uint32_t s0 = (uint32_t)__shfl((int)s, 0, 64);
    if (__all(s == s0)) {  // one segment in the wave: one atomic
        for (int o = 32; o > 0; o >>= 1) { const int32_t y = __shfl_xor(v, o, 64); v = y > v ? y : v; }
        if ((threadIdx.x & 63) == 0 && in && v > 0) atomicMax(&pv[s].peak, v);
    } else if (in && v > 0) {
        atomicMax(&pv[s].peak, v);
    }
}

// ---- commit: the map after the segment.  Per access first (grids over the accesses): the kept values listed in
// last-access order (keep flags -> exclusive scan -> list), the touched values' old stamps cleared from the map's
// ring; then one workgroup per segment over at most cap kept values and the map's slots.
// A segment commits unless its post pass (tmode, releases) found the map outgrowing cap: k_pq's replay then.
__device__ __forceinline__ bool pv_commits(const PvSeg& ps, const PMap& mp, uint32_t tmode) {
    return ps.ok && !(tmode && ps.sub && (int64_t)mp.live + ps.peak > (int64_t)mp.cap);
}
__global__ void k_pv_keepw(PvBuf B, const uint32_t* __restrict__ tot, uint32_t cap) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < cap && g < *tot) B.tc[g] = (uint32_t)B.keep[g];  // (the scans run over the accesses only)
}
// X = exclusive scan of keep (the flagged last accesses): the list L[X[g]] = g (segment-major, last-access order
// within a segment); and the old stamps of the values live at the start and accessed (first accesses: w a rank)
// leave the ring
__global__ void k_pv_klist(PvBuf B, const uint32_t* __restrict__ X, uint32_t* __restrict__ L,
                           const uint32_t* __restrict__ tot, const PvSeg* __restrict__ pv, DevState S, uint32_t tmode) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= *tot) return;
    if (B.keep[g]) L[X[g]] = g;
    const int32_t w = B.w[g], sl = B.fslot[g];
    if (w < 0 || w == PV_INF || sl < 0) return;
    const PvSeg ps = pv[B.seg[g]];
    const PMap mp = S.pmap[ps.mid];
    if (!pv_commits(ps, mp, tmode)) return;
    const int64_t st = S.pbkt[mp.base + sl / PM_BKT].stamp[sl % PM_BKT];
    const uint64_t p = (uint64_t)st & (uint64_t)((1ull << mp.rb_log2) - 1);
    atomicAnd(reinterpret_cast<unsigned long long*>(&S.pbm[mp.bm + (p >> 6)]), ~(1ull << (p & 63)));
}

#define PV_RW 512u   // ring words (cap <= PQ_MAX_CAP)
#define PV_CW 256u   // claim words (slots <= map_buckets(PQ_MAX_CAP) * 8)
// tmode (the post pass): the thread-count map; the segment gets SEG_PVT and its ParameterMetric bits
__global__ __launch_bounds__(1024) void k_pv_commit(PvBuf B, const PvSeg* __restrict__ pv, uint32_t m, DevState S,
                                                    uint32_t* __restrict__ bflags, uint32_t tmode,
                                                    Seg* __restrict__ segs, const uint32_t* __restrict__ list,
                                                    const uint32_t* __restrict__ X, const uint32_t* __restrict__ L,
                                                    uint32_t* __restrict__ ndone, uint32_t* __restrict__ rest) {
    __shared__ uint64_t ring[PV_RW];
    __shared__ uint32_t pre[PV_RW];
    __shared__ unsigned long long claim[PV_CW];
    __shared__ uint32_t red[16];
    __shared__ uint32_t nfail;
    __shared__ uint32_t fail[64];
    const uint32_t i = blockIdx.x, tid = threadIdx.x;
    if (i >= m) return;
    const PvSeg ps = pv[i];
    PMap mp = S.pmap[ps.ok ? ps.mid : 0];
    if (!pv_commits(ps, mp, tmode)) {  // (post pass) k_pq's post pass: rest[1 + k], count rest[0]
        if (tmode && tid == 0) {  // (an XF_PVPQ segment the pre pass did not take: k_pq's full pass did it all)
            const Seg sgc = segs[list[i]];
            if (!(S.prog[sgc.res].xf & XF_PVPQ) || (sgc.bin & SEG_PV)) rest[1 + atomicAdd(&rest[0], 1u)] = list[i];
        }
        return;
    }
    const uint32_t W = 1u << (mp.rb_log2 - 6);
    const int32_t cap = (int32_t)mp.cap;
    PBucket* BK = S.pbkt + mp.base;
    PData* DT = S.pdat + mp.base * PM_BKT;
    const uint32_t nslot = mp.nb * PM_BKT;
    for (uint32_t w = tid; w < W; w += 1024) ring[w] = S.pbm[mp.bm + w];  // (untouched live stamps: k_pv_klist)
    for (uint32_t w = tid; w < PV_CW; w += 1024) claim[w] = 0;
    if (tid == 0) nfail = 0;
    // (1) the accessed values that stay: the flagged last accesses L[X[off], X[off] + G) in order; the latest
    // KA = min(G, cap) of them (an LRU map holds the cap most recently used), or (releases) every value present
    const uint32_t G = ps.n ? X[ps.off + ps.n - 1] + (uint32_t)B.keep[ps.off + ps.n - 1] - X[ps.off] : 0u;
    const uint32_t KA = (tmode && ps.sub) || G < (uint32_t)cap ? G : (uint32_t)cap;
    const uint32_t ks = ps.n ? X[ps.off] + (G - KA) : 0u;
    __syncthreads();
    // (2) untouched live values: the (cap - KA) most recent stay; prefix counts of their stamps from thr
    const uint32_t w0 = pv_word(mp, mp.thr);
    {
        const uint32_t per = (W + 1023) / 1024, l0 = tid * per;
        uint32_t c = 0;
        for (uint32_t u = 0; u < per; ++u)
            if (l0 + u < W) c += (uint32_t)__popcll(ring[(w0 + l0 + u) & (W - 1)]);
        uint32_t tU;
        uint32_t run = pv_scan<16>(c, red, &tU);
        for (uint32_t u = 0; u < per; ++u)
            if (l0 + u < W) {
                const uint32_t w = (w0 + l0 + u) & (W - 1);
                pre[w] = run;
                run += (uint32_t)__popcll(ring[w]);
            }
        if (tid == 0) red[15] = tU;
    }
    __syncthreads();
    const uint32_t U = red[15];
    const uint32_t KU = U < (uint32_t)cap - KA ? U : (uint32_t)cap - KA;  // untouched values that stay
    const int64_t base = mp.clock;                                          // new stamps [base, base + KU + KA)
    // (3) untouched values: new stamps in their old order, claimed slots; the others die with the old stamps
    for (uint32_t sl = tid; sl < nslot; sl += 1024) {
        const uint64_t key = BK[sl / PM_BKT].key[sl % PM_BKT];
        if (key == PK_EMPTY) continue;
        const int64_t s = BK[sl / PM_BKT].stamp[sl % PM_BKT];
        if (!(s >= mp.thr && s < mp.clock)) continue;
        const uint64_t p = (uint64_t)s & (uint64_t)((1ull << mp.rb_log2) - 1);
        const uint64_t bit = 1ull << (p & 63);
        if (!(ring[p >> 6] & bit)) continue;
        const uint32_t below = pre[p >> 6] + (uint32_t)__popcll(ring[p >> 6] & (bit - 1ull));
        if (below + KU < U) continue;  // not among the KU most recent untouched
        BK[sl / PM_BKT].stamp[sl % PM_BKT] = base + (int64_t)(below - (U - KU));
        atomicOr(&claim[sl >> 6], 1ull << (sl & 63));
    }
    __syncthreads();
    // (4) accessed values that stay, in last-access order: new stamps above; their slot reused or claimed
    for (uint32_t rank = tid; rank < KA; rank += 1024) {
        const uint32_t g = L[ks + rank];
        const int64_t s = base + (int64_t)KU + (int64_t)rank;
        PData d;
        d.v0 = B.flast[g]; d.v1 = B.ftok[g]; d.pad = 0;
        const int32_t sl = B.fslot[g];
        if (sl >= 0) {
            BK[sl / PM_BKT].stamp[sl % PM_BKT] = s;
            DT[sl] = d;
            atomicOr(&claim[sl >> 6], 1ull << (sl & 63));
        } else {
            B.fslot[g] = -2 - (int32_t)rank;  // placed below
        }
    }
    __syncthreads();
    // (5) new values: a free slot (empty, or an old value's that did not stay) in either bucket
    for (uint32_t kr = tid; kr < KA; kr += 1024) {
        const uint32_t g = L[ks + kr];
        if (B.fslot[g] >= 0) continue;
        const uint32_t rank = (uint32_t)(-2 - B.fslot[g]);
        const uint64_t key = B.key[g];
        const int64_t s = base + (int64_t)KU + (int64_t)rank;
        uint32_t b1, b2;
        pm_buckets(mp.nb, key, b1, b2);
        int32_t got = -1;
        for (int h = 0; h < 2 && got < 0; ++h) {
            const uint32_t bb = h ? b2 : b1;
            for (int j = 0; j < PM_BKT && got < 0; ++j) {
                const uint32_t sl = bb * PM_BKT + j;
                const unsigned long long o = atomicOr(&claim[sl >> 6], 1ull << (sl & 63));
                if (!(o & (1ull << (sl & 63)))) got = (int32_t)sl;
            }
        }
        PData d;
        d.v0 = B.flast[g]; d.v1 = B.ftok[g]; d.pad = 0;
        if (got >= 0) {
            BK[got / PM_BKT].key[got % PM_BKT] = key;
            BK[got / PM_BKT].stamp[got % PM_BKT] = s;
            DT[got] = d;
        } else {
            const uint32_t f = atomicAdd(&nfail, 1u);
            if (f < 64) fail[f] = g;
            else atomicOr(bflags, BF_PTAB_FULL);
        }
    }
    __syncthreads();
    // (6) the rare value whose two buckets are taken: a displacement walk (one lane), moving claimed values to their
    // other bucket; slots claimed by nobody are free
    if (tid == 0) {
        const uint32_t nf = nfail < 64 ? nfail : 64;
        for (uint32_t f = 0; f < nf; ++f) {
            const uint32_t g = fail[f];
            uint64_t ck = B.key[g];
            int64_t cs = base + (int64_t)KU + (int64_t)(uint32_t)(-2 - B.fslot[g]);
            PData cd;
            cd.v0 = B.flast[g]; cd.v1 = B.ftok[g]; cd.pad = 0;
            uint32_t b1, b2;
            pm_buckets(mp.nb, ck, b1, b2);
            uint32_t bb = b1;
            bool done = false;
            for (int step = 0; step < 512 && !done; ++step) {
                for (int j = 0; j < PM_BKT; ++j) {
                    const uint32_t sl = bb * PM_BKT + j;
                    if (!((claim[sl >> 6] >> (sl & 63)) & 1ull)) {
                        claim[sl >> 6] |= 1ull << (sl & 63);
                        BK[bb].key[j] = ck; BK[bb].stamp[j] = cs; DT[sl] = cd;
                        done = true;
                        break;
                    }
                }
                if (done) break;
                const int j = (int)((cs + step * 5) & 7);  // swap with a claimed value, carry it to its other bucket
                const uint32_t sl = bb * PM_BKT + j;
                const uint64_t nk = BK[bb].key[j];
                const int64_t ns = BK[bb].stamp[j];
                const PData nd = DT[sl];
                BK[bb].key[j] = ck; BK[bb].stamp[j] = cs; DT[sl] = cd;
                ck = nk; cs = ns; cd = nd;
                bb = pm_alt(mp.nb, ck, bb);
            }
            if (!done) atomicOr(bflags, BF_PTAB_FULL);
        }
    }
    __syncthreads();
    // (7) the ring holds exactly the new stamps; header
    const uint32_t K = KU + KA;
    for (uint32_t w = tid; w < W; w += 1024) ring[w] = 0;
    __syncthreads();
    for (uint32_t k = tid; k < K; k += 1024) {
        const uint64_t p = (uint64_t)(base + (int64_t)k) & (uint64_t)((1ull << mp.rb_log2) - 1);
        atomicOr(reinterpret_cast<unsigned long long*>(&ring[p >> 6]), 1ull << (p & 63));
    }
    __syncthreads();
    for (uint32_t w = tid; w < W; w += 1024) S.pbm[mp.bm + w] = ring[w];
    if (tid == 0) {
        PMap* h = &S.pmap[ps.mid];
        h->clock = base + (int64_t)K;
        h->thr = base;
        h->live = K;
        if (tmode) {
            const Seg sg = segs[list[i]];
            segs[list[i]].bin = sg.bin | SEG_PVT;
            if (ps.fbits) atomicOr(&S.info[sg.res].flags, ps.fbits);
            atomicAdd(ndone, 1u);
        }
    }
}

namespace sg {
// the accesses [0, tot) by group id, stable (tot on the device: the tiles past it idle; pads [tot, cap))
static hipError_t pv_sort(PvBuf B, uint32_t cap, uint32_t* tot, uint32_t* hist, uint32_t* part, hipStream_t st,
                          hipError_t (*radix_hist)(const uint32_t*, uint64_t, const uint32_t*, int, uint32_t*, uint32_t, hipStream_t),
                          hipError_t (*radix_scatter)(const uint32_t*, const uint32_t*, uint64_t, const uint32_t*, int,
                                                      const uint32_t*, uint32_t, uint32_t*, uint32_t*, hipStream_t),
                          hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                          uint32_t tile) {
    hipError_t e = hipSuccess;
    const uint32_t nb = (cap + 255) / 256;
    hipLaunchKernelGGL(k_pv_pad, dim3(nb), dim3(256), 0, st, B, tot, cap);
    // group ids < 2 x cap: stable LSD radix on 8-bit digits (each value's accesses stay in access order)
    int bits = 1;
    while (bits < 32 && (1ull << bits) < 2ull * cap) ++bits;
    const int passes = (bits + 7) / 8;
    const uint32_t nblocks = (cap + tile - 1) / tile;
    uint32_t *kin = B.gid, *vin = B.idx, *kout = B.gid2, *vout = B.idx2;
    for (int p = 0; p < passes; ++p) {
        e = radix_hist(kin, cap, tot, p * 8, hist, nblocks, st);
        if (e == hipSuccess) e = scan(hist, hist, (uint64_t)nblocks << 8, part, nullptr, st);
        if (e == hipSuccess) e = radix_scatter(kin, vin, cap, tot, p * 8, hist, nblocks, kout, vout, st);
        if (e != hipSuccess) return e;
        uint32_t* tk = kin; kin = kout; kout = tk;
        uint32_t* tv = vin; vin = vout; vout = tv;
    }
    if (kin != B.gid) {  // sorted arrays back into gid / idx (an odd number of passes)
        e = hipMemcpyAsync(B.gid, kin, (uint64_t)cap * 4, hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess) e = hipMemcpyAsync(B.idx, vin, (uint64_t)cap * 4, hipMemcpyDeviceToDevice, st);
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// the scans below run over the accesses only (tot[0] on the device), not the scratch capacity (kernels.hip)
hipError_t launch_scan_n(const uint32_t* in, uint32_t* out, uint64_t n, const uint32_t* ndev, uint32_t* part,
                         uint32_t* total, hipStream_t st);

// residency (after k_pv_prev / k_pv_blocks): NF / NN prefix counts in gdt / gaw, horizons in gpos
static hipError_t pv_resid(PvBuf B, uint32_t cap, uint32_t* tot, const PvSeg* pv, const DevState& S, uint32_t* part,
                           hipStream_t st,
                           hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t)) {
    const uint32_t nb = (cap + 255) / 256, nblk = (cap + PV_B - 1) / PV_B;
    uint32_t* nf = reinterpret_cast<uint32_t*>(B.gdt);
    hipLaunchKernelGGL(k_pv_fflags, dim3(nb), dim3(256), 0, st, B, tot, cap);
    hipError_t e = launch_scan_n(nf, nf, cap, tot, part, nullptr, st);
    if (e == hipSuccess) e = launch_scan_n(B.gaw, B.gaw, cap, tot, part, nullptr, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pv_horizon, dim3((nblk + 3) / 4), dim3(256), 0, st, B, tot, pv, S, B.gpos);
    hipLaunchKernelGGL(k_pv_resid, dim3(nb), dim3(256), 0, st, B, tot, pv, S, nf, B.gaw, B.gpos);
    return hipGetLastError();
}

// the commit's kept list (gdt: exclusive scan of the keep flags, idx2: the list) and the touched stamps' removal
static hipError_t pv_klist(PvBuf B, uint32_t cap, uint32_t* tot, const PvSeg* pv, const DevState& S, uint32_t tmode,
                           uint32_t* part, hipStream_t st,
                           hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t)) {
    const uint32_t nb = (cap + 255) / 256;
    hipLaunchKernelGGL(k_pv_keepw, dim3(nb), dim3(256), 0, st, B, tot, cap);
    const hipError_t e = launch_scan_n(reinterpret_cast<const uint32_t*>(B.tc), reinterpret_cast<uint32_t*>(B.gdt), cap,
                                       tot, part, nullptr, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pv_klist, dim3(nb), dim3(256), 0, st, B, reinterpret_cast<const uint32_t*>(B.gdt), B.idx2, tot,
                       pv, S, tmode);
    return hipGetLastError();
}

// the value-parallel pre pass over the wide XF_MIX list (cap accesses at most); pv[] tells k_pq which segments
// are done.  Scratch: PvBuf arrays of cap entries (chunks: cap / PV_CH + m), htab 2 x cap, radix scratch (hist,
// part), tot (device words: [0] accesses, [1] chunks, [2] ranges, [3] longest walk, [8] groups).  In two parts:
// (a) extraction and sort touch no map (they overlap the maps' growth on the main stream), (b) the rest after it.
// jumps: the batch has no zero-acquire ENTRY.
hipError_t launch_pv_a(SEv* recs, const uint32_t* vals, Seg* segs, const uint32_t* list, uint32_t m,
                       const DevState& S, const DevCfg& cfg, uint32_t* dec, PvSeg* pv, PvBuf B, uint32_t cap,
                       uint32_t* tot, uint32_t* hist, uint32_t* part, hipStream_t st,
                       hipError_t (*radix_hist)(const uint32_t*, uint64_t, const uint32_t*, int, uint32_t*, uint32_t, hipStream_t),
                       hipError_t (*radix_scatter)(const uint32_t*, const uint32_t*, uint64_t, const uint32_t*, int,
                                                   const uint32_t*, uint32_t, uint32_t*, uint32_t*, hipStream_t),
                       hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                       uint32_t tile, uint32_t* rest, uint32_t grant_all) {
    if (!m || !cap) return hipSuccess;
    const uint32_t nchunk = cap / PV_CH + m + 1;
    hipError_t e = hipMemsetAsync(tot, 0, 16, st);
    if (e == hipSuccess) e = hipMemsetAsync(B.htab, 0xFF, 2ull * cap * 8, st);  // the segments' tables: PK_EMPTY
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(rest, 0, 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pv_prep, dim3(m), dim3(256), 0, st, recs, vals, segs, list, m, S, pv, rest, grant_all);
    hipLaunchKernelGGL(k_pv_chunks, dim3(1), dim3(256), 0, st, pv, m, B, tot);
    hipLaunchKernelGGL(k_pv_count, dim3(nchunk), dim3(256), 0, st, recs, vals, segs, list, S, cfg, pv, B, tot, dec);
    hipLaunchKernelGGL(k_pv_offsets, dim3(1), dim3(256), 0, st, pv, m, B, tot);
    hipLaunchKernelGGL(k_pv_fill, dim3(nchunk), dim3(256), 0, st, recs, vals, segs, list, S, cfg, pv, B, tot);
    return pv_sort(B, cap, tot, hist, part, st, radix_hist, radix_scatter, scan, tile);
}
hipError_t launch_pv_b(SEv* recs, Seg* segs, const uint32_t* list, uint32_t m, const DevState& S, int64_t t0,
                       uint32_t* dec, uint32_t* bflags, PvSeg* pv, PvBuf B, uint32_t cap, uint32_t* tot, uint32_t* part,
                       uint32_t jumps, hipStream_t st,
                       hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                       uint32_t* rest) {
    if (!m || !cap) return hipSuccess;
    hipError_t e = hipSuccess;
    const uint32_t nb = (cap + 255) / 256;
    hipLaunchKernelGGL(k_pv_rpre, dim3(m), dim3(256), 0, st, pv, m, S);
    hipLaunchKernelGGL(k_pv_prev, dim3(nb), dim3(256), 0, st, B, tot, pv, S);
    hipLaunchKernelGGL(k_pv_blocks, dim3((cap + PV_B - 1) / PV_B), dim3(PV_B), 0, st, B, tot);
    e = pv_resid(B, cap, tot, pv, S, part, st, scan);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pv_gather, dim3(nb), dim3(256), 0, st, segs, list, B, tot);
    {   // MC in place (its values up to tot read only the flags before them)
        uint32_t* mc = reinterpret_cast<uint32_t*>(B.sw);
        e = launch_scan_n(mc, mc, cap, tot, part, nullptr, st);
        if (e != hipSuccess) return e;
    }
    // the groups' starts, densely (flags in gid2, scanned in place, count in tot[8]; list in idx2)
    hipLaunchKernelGGL(k_pv_gflags, dim3(nb), dim3(256), 0, st, B, tot, cap, B.gid2);
    e = launch_scan_n(B.gid2, B.gid2, cap, tot, part, tot + 8, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pv_glist, dim3(nb), dim3(256), 0, st, B, tot, B.gid2, B.idx2);
    hipLaunchKernelGGL(k_pv_walk, dim3(nb), dim3(256), 0, st, recs, segs, list, B, tot, pv, S, t0, dec, jumps, cap, bflags,
                       B.idx2);
    hipLaunchKernelGGL(k_pv_ranges, dim3(2048), dim3(256), 0, st, recs, B, tot, cap, dec);
    e = pv_klist(B, cap, tot, pv, S, 0u, part, st, scan);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pv_commit, dim3(m), dim3(1024), 0, st, B, pv, m, S, bflags, 0u, segs, list,
                       reinterpret_cast<const uint32_t*>(B.gdt), B.idx2, nullptr, rest);
    return hipGetLastError();
}

// the post pass over the wide XF_MIX list (after the final verdicts; before k_pq's post pass, which leaves the
// segments with SEG_PVT); tot: 4 device words of its own
hipError_t launch_pvt(SEv* recs, const sg_event* ev, const uint32_t* vals, Seg* segs, const uint32_t* list, uint32_t m,
                      const DevState& S, const DevCfg& cfg, uint32_t* dec, uint32_t* bflags, PvSeg* pv, PvBuf B,
                      uint32_t cap, uint32_t* tot, uint32_t* hist, uint32_t* part, hipStream_t st,
                      hipError_t (*radix_hist)(const uint32_t*, uint64_t, const uint32_t*, int, uint32_t*, uint32_t, hipStream_t),
                      hipError_t (*radix_scatter)(const uint32_t*, const uint32_t*, uint64_t, const uint32_t*, int,
                                                      const uint32_t*, uint32_t, uint32_t*, uint32_t*, hipStream_t),
                      hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                      uint32_t tile, uint32_t* rest) {
    if (!m || !cap) return hipSuccess;
    const uint32_t nchunk = cap / PV_CH + m + 1;
    hipError_t e = hipMemsetAsync(tot, 0, 16, st);
    if (e == hipSuccess) e = hipMemsetAsync(B.htab, 0xFF, 2ull * cap * 8, st);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(rest, 0, 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pvt_prep, dim3(m), dim3(256), 0, st, segs, list, m, S, pv);
    hipLaunchKernelGGL(k_pv_chunks, dim3(1), dim3(256), 0, st, pv, m, B, tot);
    hipLaunchKernelGGL(k_pvt_reach, dim3(nchunk), dim3(256), 0, st, recs, segs, list, S, pv, B, tot, dec);
    hipLaunchKernelGGL(k_pvt_count, dim3(nchunk), dim3(256), 0, st, recs, ev, vals, segs, list, S, cfg, pv, B, tot, dec);
    hipLaunchKernelGGL(k_pv_offsets, dim3(1), dim3(256), 0, st, pv, m, B, tot);
    hipLaunchKernelGGL(k_pvt_fill, dim3(nchunk), dim3(256), 0, st, recs, ev, vals, segs, list, S, cfg, pv, B, tot, dec);
    e = pv_sort(B, cap, tot, hist, part, st, radix_hist, radix_scatter, scan, tile);
    if (e != hipSuccess) return e;
    const uint32_t nb = (cap + 255) / 256;
    hipLaunchKernelGGL(k_pv_prev, dim3(nb), dim3(256), 0, st, B, tot, pv, S);
    hipLaunchKernelGGL(k_pv_blocks, dim3((cap + PV_B - 1) / PV_B), dim3(PV_B), 0, st, B, tot);
    e = pv_resid(B, cap, tot, pv, S, part, st, scan);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pvt_walk, dim3(nb), dim3(256), 0, st, B, tot, pv, S);
    // (the peak of the segments with releases; the scan's output in gdt: free in the post pass)
    e = launch_scan_n(reinterpret_cast<const uint32_t*>(B.tc), reinterpret_cast<uint32_t*>(B.gdt), cap, tot, part,
                      nullptr, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pvt_peak, dim3(nb), dim3(256), 0, st, B, reinterpret_cast<const uint32_t*>(B.gdt), tot, pv);
    e = pv_klist(B, cap, tot, pv, S, 1u, part, st, scan);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pv_commit, dim3(m), dim3(1024), 0, st, B, pv, m, S, bflags, 1u, segs, list,
                       reinterpret_cast<const uint32_t*>(B.gdt), B.idx2, tot + 3, rest);
    return hipGetLastError();
}

} // namespace sg
