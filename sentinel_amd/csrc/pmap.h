// pmap.h -- ParameterMetric's bounded LRU CacheMaps on the device (dev_types.h PMap / PBucket / PData).
//
// ConcurrentLinkedHashMap access order (param/slots/statistic/cache/ConcurrentLinkedHashMapWrapper.java:35-44,
// ParameterMetric.java:37-241), restated as exact LRU for one caller: get / putIfAbsent of a
// present key make it the most recently used; an insert into a full map evicts the least recently used key.
//
// Recency is a stamp per key (the map's access counter at its last access).  The live keys' stamps are the
// set bits of a ring bitmap; the least recently used key is the lowest set bit, its recency rank (how many
// live keys are more recent) a popcount.  Evicting or erasing a key clears its bit only: a slot whose stamp's
// bit is clear is dead and is reused by inserts (a dead slot still holding the key being inserted is reused by
// that key, so a key has at most one slot).  The ring holds 2^rb_log2 stamps; all live stamps lie in
// [thr, clock) with clock - thr <= 2^rb_log2 - 64 (pm_reserve; when hot keys keep the oldest key alive for a
// whole ring, the live stamps are renumbered densely, pm_compact).
//
// The functions below are the sequential (one lane) operations k_lane uses; k_pq (param.hip) decides a tile
// of accesses of one map at once with the same representation and the helpers at the top.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "chain.h"
#include "dev_types.h"

// The map operations are __host__ __device__ so that tests/pmap_host.cpp can check them against a reference LRU
// on the CPU (PM_FLAG raises a batch flag: an atomic on the device, a plain or on the host).
#define PM_FN __host__ __device__
#if defined(__HIP_DEVICE_COMPILE__)
#define PM_FLAG(p, f) atomicOr((p), (f))
#else
#define PM_FLAG(p, f) (*(p) |= (f))
#endif

namespace sg {

#define PM_DEAD INT64_MIN  // stamp of a slot retired by pm_compact: below every thr

PM_FN inline int64_t pm_rbits(const PMap& m) { return (int64_t)1 << m.rb_log2; }
// the two candidate buckets of a key (multiply-shift range reduction of two halves of one hash)
PM_FN inline void pm_buckets(uint32_t nb, uint64_t v, uint32_t& b1, uint32_t& b2) {
    const uint64_t h = mix64(v ^ 0x9E3779B97F4A7C15ull);
    b1 = (uint32_t)(((h >> 32) * (uint64_t)nb) >> 32);
    b2 = (uint32_t)(((h & 0xFFFFFFFFull) * (uint64_t)nb) >> 32);
    if (b2 == b1) b2 = b1 + 1 == nb ? 0u : b1 + 1;
}
PM_FN inline uint32_t pm_alt(uint32_t nb, uint64_t v, uint32_t b) {
    uint32_t b1, b2;
    pm_buckets(nb, v, b1, b2);
    return b == b1 ? b2 : b1;
}
PM_FN inline bool pm_bit(const uint64_t* bm, const PMap& m, int64_t s) {
    const uint64_t p = (uint64_t)s & (uint64_t)(pm_rbits(m) - 1);
    return ((bm[p >> 6] >> (p & 63)) & 1ull) != 0;
}
PM_FN inline void pm_setbit(uint64_t* bm, const PMap& m, int64_t s) {
    const uint64_t p = (uint64_t)s & (uint64_t)(pm_rbits(m) - 1);
    bm[p >> 6] |= 1ull << (p & 63);
}
PM_FN inline void pm_clrbit(uint64_t* bm, const PMap& m, int64_t s) {
    const uint64_t p = (uint64_t)s & (uint64_t)(pm_rbits(m) - 1);
    bm[p >> 6] &= ~(1ull << (p & 63));
}
// a slot with this stamp holds a live key (its key is not PK_EMPTY)
PM_FN inline bool pm_live(const PMap& m, const uint64_t* bm, int64_t s) {
    return s >= m.thr && s < m.clock && pm_bit(bm, m, s);
}
// the lowest live stamp >= from (clock if none)
PM_FN inline int64_t pm_first_live(const PMap& m, const uint64_t* bm, int64_t from) {
    const int64_t RB = pm_rbits(m);
    int64_t s = from;
    while (s < m.clock) {
        const uint64_t p = (uint64_t)s & (uint64_t)(RB - 1);
        const uint32_t o = (uint32_t)(p & 63);
        const uint64_t w = bm[p >> 6] >> o;
        if (w) {
            const int64_t r = s + (int64_t)__builtin_ffsll((long long)w) - 1;
            return r < m.clock ? r : m.clock;
        }
        s += 64 - o;
    }
    return m.clock;
}

struct PRef {       // one map's storage
    PBucket* B;
    PData* D;
    uint64_t* bm;
    uint32_t* pre;
};
PM_FN inline PRef pm_ref(const DevState& S, const PMap& m) {
    PRef r;
    r.B = S.pbkt + m.base;
    r.D = S.pdat + m.base * PM_BKT;
    r.bm = S.pbm + m.bm;
    r.pre = S.ppre + m.bm;
    return r;
}
PM_FN inline void pm_store(const DevState& S, uint32_t id, const PMap& m) {
    PMap* h = &S.pmap[id];
    h->clock = m.clock;
    h->thr = m.thr;
    h->live = m.live;
}

// Renumber the live stamps densely to [clock - live, clock), keeping their order (the ring is about to wrap
// onto a live stamp because hot keys kept the oldest live key alive for a whole ring).  Dead slots get PM_DEAD:
// their old stamps may lie in the renumbered range, whose bits are set again.
PM_FN inline void pm_compact(PMap& m, const PRef& R) {
    const int64_t RB = pm_rbits(m);
    const uint32_t W = (uint32_t)(RB >> 6);
    m.thr = pm_first_live(m, R.bm, m.thr);
    const uint32_t w0 = (uint32_t)(((uint64_t)m.thr & (uint64_t)(RB - 1)) >> 6);
    uint32_t acc = 0;
    for (uint32_t l = 0; l < W; ++l) {  // live stamps before each word, in stamp order from thr
        const uint32_t w = (w0 + l) & (W - 1);
        R.pre[w] = acc;
        acc += (uint32_t)__builtin_popcountll(R.bm[w]);
    }
    const int64_t base = m.clock - (int64_t)m.live;
    for (uint32_t b = 0; b < m.nb; ++b)
        for (int j = 0; j < PM_BKT; ++j) {
            const int64_t s = R.B[b].stamp[j];
            if (R.B[b].key[j] == PK_EMPTY) continue;
            if (!pm_live(m, R.bm, s)) {  // a dead slot's stamp may fall in the renumbered range: retire it
                R.B[b].stamp[j] = PM_DEAD;
                continue;
            }
            const uint64_t p = (uint64_t)s & (uint64_t)(RB - 1);
            const uint32_t rk = R.pre[p >> 6] + (uint32_t)__builtin_popcountll(R.bm[p >> 6] & ((1ull << (p & 63)) - 1ull));
            R.B[b].stamp[j] = base + (int64_t)rk;
        }
    for (uint32_t w = 0; w < W; ++w) R.bm[w] = 0;
    for (int64_t s = base; s < m.clock; ++s) pm_setbit(R.bm, m, s);
    m.thr = base;
}
// room for k new stamps: clock + k - thr <= ring - 64 (the live range never wraps into its first word)
PM_FN inline void pm_reserve(PMap& m, const PRef& R, uint32_t k) {
    const int64_t lim = pm_rbits(m) - 64;
    if (m.clock + (int64_t)k - m.thr <= lim) return;
    m.thr = pm_first_live(m, R.bm, m.thr);
    if (m.clock + (int64_t)k - m.thr <= lim) return;
    pm_compact(m, R);
}
PM_FN inline int32_t pm_lookup(const PMap& m, const PBucket* B, uint64_t v) {
    uint32_t b1, b2;
    pm_buckets(m.nb, v, b1, b2);
#pragma unroll
    for (int j = 0; j < PM_BKT; ++j)
        if (B[b1].key[j] == v) return (int32_t)(b1 * PM_BKT + j);
#pragma unroll
    for (int j = 0; j < PM_BKT; ++j)
        if (B[b2].key[j] == v) return (int32_t)(b2 * PM_BKT + j);
    return -1;
}
PM_FN inline bool pm_slot_free(const PMap& m, const PRef& R, uint32_t b, int j) {
    return R.B[b].key[j] == PK_EMPTY || !pm_live(m, R.bm, R.B[b].stamp[j]);
}
// evict the least recently used key (the map is full)
PM_FN inline void pm_evict_oldest(PMap& m, const PRef& R) {
    const int64_t s = pm_first_live(m, R.bm, m.thr);
    if (s < m.clock) {
        pm_clrbit(R.bm, m, s);
        m.live--;
    }
    m.thr = s + 1 < m.clock ? s + 1 : m.clock;
}
// Place a key that has no slot as live with the next stamp and zeroed values: a free slot of the bucket with
// fewer live keys, else live keys are moved to their other bucket (cuckoo displacement) to open one.  Returns
// its slot.  The walk's failure (BF_PTAB_FULL: the batch fails with SG_ECAPACITY) cannot happen below ~90 %
// load; the tables run at <= 50 %.
PM_FN inline int32_t pm_insert_new(PMap& m, const PRef& R, uint64_t v, uint32_t* bflags) {
    uint32_t b1, b2;
    pm_buckets(m.nb, v, b1, b2);
    const int64_t s = m.clock++;
    pm_setbit(R.bm, m, s);  // first: the slot the key lands in is live for the displacement walk below
    PData z;
    z.v0 = 0; z.v1 = 0; z.pad = 0;
    int f1 = -1, f2 = -1, n1 = 0, n2 = 0;
    for (int j = 0; j < PM_BKT; ++j) {
        if (pm_slot_free(m, R, b1, j)) { if (f1 < 0) f1 = j; } else ++n1;
        if (pm_slot_free(m, R, b2, j)) { if (f2 < 0) f2 = j; } else ++n2;
    }
    const bool u1 = f1 >= 0 && (f2 < 0 || n1 <= n2);
    if (u1 || f2 >= 0) {
        const uint32_t b = u1 ? b1 : b2;
        const int j = u1 ? f1 : f2;
        R.B[b].key[j] = v;
        R.B[b].stamp[j] = s;
        R.D[b * PM_BKT + j] = z;
        return (int32_t)(b * PM_BKT + j);
    }
    // displacement walk: carry (key, stamp, values) into bucket b, swapping out a live key when b is full
    uint64_t ck = v;
    int64_t cs = s;
    PData cd = z;
    uint32_t b = b1;
    for (int step = 0; step < 256; ++step) {
        int fb = -1;
        for (int q = 0; q < PM_BKT; ++q)
            if (pm_slot_free(m, R, b, q)) { fb = q; break; }
        if (fb >= 0) {
            R.B[b].key[fb] = ck;
            R.B[b].stamp[fb] = cs;
            R.D[b * PM_BKT + fb] = cd;
            return pm_lookup(m, R.B, v);
        }
        const int q = (int)((m.clock + (uint64_t)step * 5) & 7);
        const uint64_t nk = R.B[b].key[q];
        const int64_t ns = R.B[b].stamp[q];
        const PData nd = R.D[b * PM_BKT + q];
        R.B[b].key[q] = ck;
        R.B[b].stamp[q] = cs;
        R.D[b * PM_BKT + q] = cd;
        ck = nk; cs = ns; cd = nd;
        b = pm_alt(m.nb, ck, b);
    }
    PM_FLAG(bflags, (uint32_t)BF_PTAB_FULL);  // the carried key is lost: the batch is failed (SG_ECAPACITY)
    const int32_t i = pm_lookup(m, R.B, v);
    return i >= 0 ? i : 0;
}
// new stamp for the key in slot i (it was live with stamp `old` if was_live)
PM_FN inline void pm_restamp(PMap& m, const PRef& R, int32_t i, bool was_live) {
    const uint32_t b = (uint32_t)i / PM_BKT;
    const int j = i % PM_BKT;
    if (was_live) pm_clrbit(R.bm, m, R.B[b].stamp[j]);
    const int64_t s = m.clock++;
    R.B[b].stamp[j] = s;
    pm_setbit(R.bm, m, s);
}
// CacheMap.putIfAbsent / the access of a put: the key becomes the most recently used.  Returns its slot;
// *present = it was in the map (else it was inserted with zeroed values, evicting the LRU key of a full map).
PM_FN inline int32_t pm_put(PMap& m, const PRef& R, uint64_t v, bool* present, uint32_t* bflags) {
    pm_reserve(m, R, 1);
    int32_t i = pm_lookup(m, R.B, v);
    if (i >= 0 && pm_live(m, R.bm, R.B[i / PM_BKT].stamp[i % PM_BKT])) {
        pm_restamp(m, R, i, true);
        *present = true;
        return i;
    }
    *present = false;
    if (m.live >= m.cap) pm_evict_oldest(m, R);
    m.live++;
    if (i < 0) return pm_insert_new(m, R, v, bflags);
    pm_restamp(m, R, i, false);  // the key's own dead slot
    PData z;
    z.v0 = 0; z.v1 = 0; z.pad = 0;
    R.D[i] = z;
    return i;
}
// CacheMap.get: the slot of a present key (made the most recently used), else -1
PM_FN inline int32_t pm_get(PMap& m, const PRef& R, uint64_t v) {
    const int32_t i = pm_lookup(m, R.B, v);
    if (i < 0 || !pm_live(m, R.bm, R.B[i / PM_BKT].stamp[i % PM_BKT])) return -1;
    pm_reserve(m, R, 1);  // may renumber the stamps: the slot's liveness was read before, its stamp after
    pm_restamp(m, R, i, true);
    return i;
}
// CacheMap.remove of a present key
PM_FN inline void pm_erase(PMap& m, const PRef& R, int32_t i) {
    pm_clrbit(R.bm, m, R.B[i / PM_BKT].stamp[i % PM_BKT]);
    m.live--;
}

#ifdef __HIPCC__
// ---- elastic map regions (dev_types.h PM_MIN_NB)
// Move map id to a region of nn buckets at nbase (fresh pool buckets: every key PK_EMPTY): its live keys, with their
// stamps and values, by two-choice cuckoo placement (every key of the new table is live: a slot is free iff empty).
__device__ inline void pm_move(const DevState& S, uint32_t id, PMap m, uint64_t nbase, uint32_t nn, uint32_t* bflags) {
    const PBucket* OB = S.pbkt + m.base;
    const PData* OD = S.pdat + m.base * PM_BKT;
    PBucket* NB = S.pbkt + nbase;
    PData* ND = S.pdat + nbase * PM_BKT;
    const uint64_t* bm = S.pbm + m.bm;
    for (uint32_t b = 0; b < m.nb; ++b) {
        for (int j = 0; j < PM_BKT; ++j) {
            uint64_t ck = OB[b].key[j];
            int64_t cs = OB[b].stamp[j];
            if (ck == PK_EMPTY || !pm_live(m, bm, cs)) continue;
            PData cd = OD[b * PM_BKT + j];
            uint32_t b1, b2;
            pm_buckets(nn, ck, b1, b2);
            uint32_t c = b1;
            bool placed = false;
            for (int step = 0; step < 512 && !placed; ++step) {
                for (int q = 0; q < PM_BKT; ++q) {  // a free slot in either candidate (the first step) or in c
                    if (NB[c].key[q] == PK_EMPTY) { NB[c].key[q] = ck; NB[c].stamp[q] = cs; ND[c * PM_BKT + q] = cd; placed = true; break; }
                }
                if (placed) break;
                if (step == 0) {
                    for (int q = 0; q < PM_BKT; ++q) {
                        if (NB[b2].key[q] == PK_EMPTY) { NB[b2].key[q] = ck; NB[b2].stamp[q] = cs; ND[b2 * PM_BKT + q] = cd; placed = true; break; }
                    }
                    if (placed) break;
                }
                const int q = (int)((cs + step * 5) & 7);  // displace one key of c to its other bucket
                const uint64_t nk = NB[c].key[q];
                const int64_t ns = NB[c].stamp[q];
                const PData nd = ND[c * PM_BKT + q];
                NB[c].key[q] = ck; NB[c].stamp[q] = cs; ND[c * PM_BKT + q] = cd;
                ck = nk; cs = ns; cd = nd;
                c = pm_alt(nn, ck, c);
            }
            if (!placed) atomicOr(bflags, BF_PTAB_FULL);  // (cannot happen at <= 50 % load)
        }
    }
    PMap* h = &S.pmap[id];
    h->base = nbase;
    h->nb = nn;
}
// the map before up to `adds` more keys arrive: at most half its slots used, else a region twice as large (or
// large enough), up to map_buckets(cap)
// mv (k_pm_grow): the move is listed for k_pm_move_list (a workgroup per map) instead of done by this lane
// pool_next = the pool's control words (PC_*).  rescue != 0: a region the pool cannot hold yet is a request for the
// batch's on-device compaction (PC_RESCUE = rescue, the map keeps its region for now); 0: the pool is used up
__device__ inline void pm_grow(const DevState& S, uint32_t id, uint64_t adds, unsigned long long* pool_next, uint64_t pool_nb,
                        uint32_t* bflags, uint4* mv = nullptr, uint32_t* nmv = nullptr, uint32_t mcap = 0,
                        uint32_t rescue = 0) {
    const PMap m = S.pmap[id];
    uint64_t need = (uint64_t)m.live + adds;
    if (need > m.cap) need = m.cap;
    const uint32_t want = map_buckets((uint32_t)need), full = map_buckets(m.cap);
    if (want <= m.nb) return;
    uint32_t nn = want > 2 * m.nb ? want : 2 * m.nb;
    if (nn > full) nn = full;
    const uint64_t nbase = atomicAdd(pool_next, (unsigned long long)nn);
    if (nbase + nn > pool_nb) {
        if (rescue) pool_next[PC_RESCUE] = rescue;
        else atomicOr(bflags, BF_POOL_FULL);
        return;
    }
    if (mv) {
        const uint32_t k = atomicAdd(nmv, 1u);
        if (k < mcap) { mv[k] = make_uint4(id, (uint32_t)nbase, (uint32_t)(nbase >> 32), nn); return; }
    }
    pm_move(S, id, m, nbase, nn, bflags);
}
#endif  // __HIPCC__

} // namespace sg
