// kernels.hip -- grouping, scans, snapshots and state initialisation of the MI355X
// Sentinel engine (the decide kernels live in decide.hip).
//
// Per sg_submit batch (n events already in HBM):
//   1. group   : stable LSD radix sort of (res_id, event index) -- keys read straight
//                out of the 24-byte event records on the first pass (k_radix_*); ties keep
//                submission order, so every resource's events stay in event order
//   2. scan    : reduce-then-scan exclusive prefix sums (segment starts, snapshot offsets)
// plus the per-second MetricNode snapshot (StatisticNode.metrics) and engine initialisation.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/sentinel_gpu.h"
#include "dev_types.h"

using namespace sg;

#define WAVE 64

// =================================================================================
// 1. grouping: stable LSD radix sort on res_id
// =================================================================================
#define RS_THREADS 256
#ifndef RS_ITEMS
#define RS_ITEMS 16
#endif
#define RS_TILE (RS_THREADS * RS_ITEMS)
#define RS_BINS 256

// Per-block digit histogram in LDS with one atomic per group of equal digits in a wave (DB
// ballots find the peers): Zipf-hot resources put most of a wave on one digit, which would
// otherwise serialise 64 LDS atomics on one address.
template <int DB>
__device__ __forceinline__ void hist_add(uint32_t* h, uint32_t d, bool valid) {
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < DB; ++b) {
        const uint64_t bb = __ballot((d >> b) & 1);
        peers &= ((d >> b) & 1) ? bb : ~bb;
    }
    const int l = threadIdx.x & 63;
    const uint64_t lt = (l == 0) ? 0ull : (~0ull >> (64 - l));
    if (valid && (peers & lt) == 0) atomicAdd(&h[d], (uint32_t)__popcll(peers));
}

// First pass over the caller's events, in submission order (coalesced): validates the batch,
// builds the 16-byte decide record of every event (references to ENTRYs of earlier batches are
// resolved against the status ring here; same-batch references keep the ENTRY's batch index and
// are mapped to its sorted position after the sort), writes the sort keys/values (value bit 31 =
// "is an ENTRY", so the inverse permutation also says whether a reference hits an ENTRY) and the
// histogram of the first radix digit.
template <int DB>
__global__ __launch_bounds__(RS_THREADS) void k_rs_first(const sg_event* __restrict__ ev, uint64_t n, uint32_t max_res,
                                                      uint64_t gbase, const uint8_t* __restrict__ ring,
                                                      uint64_t ring_mask, int32_t max_rt, SEv* __restrict__ rec_o,
                                                      uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                      uint32_t* __restrict__ ghist, uint32_t nblocks,
                                                      uint32_t* __restrict__ bflags, int64_t* __restrict__ t0_out,
                                                      uint32_t* __restrict__ prio, uint64_t* __restrict__ key_ring,
                                                      const uint32_t* __restrict__ comp,
                                                      const sg_event_ext* __restrict__ ext,
                                                      const sg_arg* __restrict__ args, uint64_t n_args,
                                                      uint32_t max_ctx) {
    constexpr int NB = 1 << DB;
    __shared__ uint32_t h[NB];
    for (int i = threadIdx.x; i < NB; i += RS_THREADS) h[i] = 0;
    __syncthreads();
    const int64_t t0 = ev[0].ts;
    if (blockIdx.x == 0 && threadIdx.x == 0) *t0_out = t0;
    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
    uint32_t fl = 0;
    uint32_t hkey[RS_ITEMS];
#pragma unroll
    for (int it = 0; it < RS_ITEMS; ++it) {
        const uint64_t i = base + (uint64_t)it * RS_THREADS + threadIdx.x;
        hkey[it] = 0;
        if (i >= n) continue;
        const sg_event e = ev[i];
        if (e.res_id >= max_res) fl |= BF_BAD_RES;
        const int64_t dt = e.ts - t0;
        if (dt < 0 || dt > 0x7FFFFFFFLL) fl |= (dt < 0 ? BF_BACKWARD : BF_TSPAN);
        if (i > 0 && ev[i - 1].ts > e.ts) fl |= BF_BACKWARD;  // ABI: non-decreasing ts
        SEv r;
        r.dt = (int32_t)dt;
        r.x = 0;
        r.cnt = e.count;
        r.rt = 0;
        r.kind = e.kind;
        r.flags = (uint8_t)(e.flags & 0x3Fu);  // the ABI's SG_F_* bits only (RF_* are internal)
        r.code = RC_NONE;
        r.pad = 0;
        uint32_t mark = 0;  // PM_* marks for the resource
        uint64_t key0 = (e.flags & SG_F_HAS_ARG) ? e.aux : NO_KEY;
        uint32_t tag = 0;        // origin / context node tag (dev_types.h TAG_*)
        bool own_args = false;   // the event's args come from the table
        if (ext) {  // sg_submit_ex: validate the event's args; a NullContext event is k_lane's
            const sg_event_ext x = ext[i];
            if (x.n_args > SG_MAX_ARGS || (uint64_t)x.arg_off + x.n_args > n_args) fl |= BF_BAD_ARGS;
            else if (x.n_args) {
                for (uint32_t k = 0; k < x.n_args; ++k) {
                    const sg_arg a = args[x.arg_off + k];
                    if (a.kind > SG_ARG_LIST || (a.kind == SG_ARG_LIST && (a.key > n_args || a.len > n_args - a.key)))
                        fl |= BF_BAD_ARGS;
                    else if (a.kind == SG_ARG_LIST) {
                        mark |= PM_ARGL;  // (at any index: one map access per element, param.hip k_pm_grow)
                        for (uint32_t q = 0; q < a.len; ++q)
                            if (args[a.key + q].kind > SG_ARG_SCALAR) fl |= BF_BAD_ARGS;
                    }
                }
                const sg_arg a0 = args[x.arg_off];
                key0 = a0.kind == SG_ARG_SCALAR ? a0.key : NO_KEY;
                own_args = true;
            }
            if (x.context_id > max_ctx) mark |= PM_LANE;
            // ClusterBuilderSlot / NodeSelectorSlot keep an origin node and a DefaultNode per context for every
            // entry, whatever the rules (ClusterBuilderSlot.java:74-99, NodeSelectorSlot.java:134-176)
            else if (x.origin_id != 0 || x.context_id != 0) {
                mark |= PM_AUX;
                if (x.origin_id >> TAG_ORIGIN_BITS) mark |= PM_LANE;  // not packable: k_lane reads the ext itself
                else tag = x.origin_id | (x.context_id << TAG_ORIGIN_BITS);
            }
        }
        if (own_args) {  // the record's HAS_ARG: args[0] is a scalar (a k_pq check / thread-count key)
            r.flags = (uint8_t)((r.flags & ~SG_F_HAS_ARG) | (key0 != NO_KEY ? SG_F_HAS_ARG : 0));
            if (e.kind == SG_EV_EXIT) {
                r.flags |= RF_OWN_ARGS;
                if (e.flags & SG_F_EXIT_ARGS) mark |= PM_XARGS;
            }
        }
        r.x = tag;  // ENTRY (and an EXIT / TRACE naming no ENTRY of this batch): its node tag
        if (e.kind == SG_EV_ENTRY) {
            // the arg an exit(count, args) of this ENTRY will decrement (ParamFlowStatisticExitCallback)
            if (key_ring) key_ring[(gbase + i) & ring_mask] = key0;
            // a prioritized ENTRY makes the resource's borrow ring live; an upstream block is k_lane's (a
            // separate mark array: this stage may run while the previous batch's decide stores NodeInfo)
            if (e.flags & SG_F_PRIORITIZED) mark |= PM_PRIO;
            if (e.flags & SG_F_BLOCKED_UPSTREAM) mark |= PM_LANE;
        } else {
            if (e.kind == SG_EV_EXIT) {
                const int64_t raw = (int64_t)(e.aux >> 48);
                r.rt = (uint16_t)(raw > max_rt ? max_rt : raw);
                // Entry.exit(count, args) with its own args: the key its release decrements (k_pq reads it here)
                if (own_args && key_ring) key_ring[(gbase + i) & ring_mask] = key0;
            }
            const uint64_t ref = e.aux & SG_REF_NONE;
            if (ref != SG_REF_NONE) {
                if (ref >= gbase) {
                    // an EXIT/TRACE must follow its ENTRY (that the ENTRY is of its own resource is checked
                    // after the sort, where the two sit a few positions apart: k_block_sums)
                    if (ref - gbase >= i) fl |= BF_BAD_REF;
                    else { r.code = RC_BATCH; r.x = (uint32_t)(ref - gbase); }
                } else {  // an ENTRY of an earlier batch: its status is read from the ring by k_resolve,
                          // after the earlier batches are decided (this stage overlaps the previous decide)
                    r.code = RC_PREV;
                    r.x = (uint32_t)(ref & ring_mask);
                }
            }
        }
        if (mark && e.res_id < max_res && (prio[e.res_id] & mark) != mark) atomicOr(&prio[e.res_id], mark);
        rec_o[i] = r;
        // sort key: the resource, or its STRATEGY_RELATE component's representative (one segment)
        const uint32_t key = (comp && e.res_id < max_res) ? comp[e.res_id] : e.res_id;
        keys[i] = key;
        vals[i] = (uint32_t)i | (e.kind == SG_EV_ENTRY ? 0x80000000u : 0u);
        hkey[it] = key;
    }
#pragma unroll
    for (int it = 0; it < RS_ITEMS; ++it) {
        const uint64_t i = base + (uint64_t)it * RS_THREADS + threadIdx.x;
        hist_add<DB>(h, hkey[it] & (NB - 1), i < n);
    }
    if (fl) atomicOr(bflags, fl);
    __syncthreads();
    for (int b = threadIdx.x; b < NB; b += RS_THREADS) ghist[(uint64_t)b * nblocks + blockIdx.x] = h[b];
}

// =================================================================================
// 1b. grouping by a hot / cold split (the default group stage)
// =================================================================================
// Zipf traffic puts most of a batch on a few hundred resources (C4: the ~540 resources of >= 4096 events hold ~65 %
// of a 2^25-event batch), and LSD radix passes over them move every event three times to end where one counting
// split would put it.  The resources that were hot in the previous batch (k_hot_build, from its segments) get
// dense ids h < nhot: their events go to their final sorted positions in ONE pass (per-tile counts per hot id, a
// scan, a scatter), hot id by hot id, each in event order.  Only the cold rest takes the radix passes.  Every
// resource's events end contiguous and in event order -- all the decide stage needs (segments are not in resource
// order: hot ids first, then the cold keys sorted).
//
//   k_grp_first  : events read once in submission order: the batch's validation, marks and key ring (as
//                  k_rs_first), the tile's stable rank of every hot event within its hot id (word[i] = W_HOT |
//                  h << 12 | rank), the tile's hot-id counts, and the cold events' (key, index) compacted per
//                  tile with the first radix digit's histogram
//   radix passes : the cold (key, index) only (k_radix_scatter with per-tile counts on the first pass); the last
//                  pass writes the sorted values and pos_of at hot_total + its position
//   k_grp_records: events read again: every event's sorted position (hot: scanned tile offset + rank; cold:
//                  pos_of), same-batch references mapped to sorted positions, the 16-byte record written there
#define HOT_MAX 1024u
#define HOT_NONE 0xFFFFu
#define W_HOT 0x80000000u   // word: a hot event (W_HOT | W_ENT? | hot id << 12 | rank in its tile's run)
#define W_ENT 0x40000000u   // word: an ENTRY (hot or cold); a cold event's word is W_ENT? | its sorted position
#define W_POS 0x3FFFFFFFu   // (the last cold radix pass writes it: batches of < 2^30 events)

template <int DB>
__global__ __launch_bounds__(RS_THREADS) void k_grp_first(const sg_event* __restrict__ ev, uint64_t n, uint32_t max_res,
                                                       uint64_t gbase, uint64_t ring_mask, uint32_t* __restrict__ bflags,
                                                       int64_t* __restrict__ t0_out, uint32_t* __restrict__ prio,
                                                       uint64_t* __restrict__ key_ring, const uint32_t* __restrict__ comp,
                                                       const sg_event_ext* __restrict__ ext, const sg_arg* __restrict__ args,
                                                       uint64_t n_args, uint32_t max_ctx,
                                                       const uint16_t* __restrict__ hot_tab, uint32_t nhot,
                                                       uint32_t nblocks, uint32_t* __restrict__ words,
                                                       uint32_t* __restrict__ hot_hist, uint32_t* __restrict__ ckeys,
                                                       uint32_t* __restrict__ cvals, uint32_t* __restrict__ ccnt,
                                                       uint32_t* __restrict__ chist) {
    constexpr int NB = 1 << DB;
    __shared__ uint32_t wcnt[4][HOT_MAX];  // per-wave hot-id counts, then per-wave rank offsets
    __shared__ uint32_t h[NB];
    __shared__ uint32_t cw[4];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    for (int i = threadIdx.x; i < NB; i += RS_THREADS) h[i] = 0;
    for (uint32_t i = threadIdx.x; i < 4 * HOT_MAX; i += RS_THREADS) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const int64_t t0 = ev[0].ts;
    if (blockIdx.x == 0 && threadIdx.x == 0) *t0_out = t0;
    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
    const uint64_t wbase = base + (uint64_t)w * (RS_TILE / 4);
    const uint64_t lt = (l == 0) ? 0ull : (~0ull >> (64 - l));
    uint32_t fl = 0;
    uint32_t kk[RS_ITEMS], rk[RS_ITEMS];  // key; hot: id << 16 | wave rank, cold: wave rank
    uint32_t hotm = 0, entm = 0;          // per item: hot, ENTRY
    uint32_t ccount = 0;                  // the wave's cold items so far
#pragma unroll
    for (int it = 0; it < RS_ITEMS; ++it) {  // per-wave rounds of 64 consecutive events: coalesced, in event order
        const uint64_t i = wbase + (uint64_t)it * WAVE + l;
        const bool valid = i < n;
        uint32_t key = 0, hid = HOT_NONE;
        if (valid) {
            const sg_event e = ev[i];
            if (e.res_id >= max_res) fl |= BF_BAD_RES;
            const int64_t dt = e.ts - t0;
            if (dt < 0 || dt > 0x7FFFFFFFLL) fl |= (dt < 0 ? BF_BACKWARD : BF_TSPAN);
            if (i > 0 && ev[i - 1].ts > e.ts) fl |= BF_BACKWARD;  // ABI: non-decreasing ts
            uint32_t mark = 0;  // PM_* marks for the resource
            uint64_t key0 = (e.flags & SG_F_HAS_ARG) ? e.aux : NO_KEY;
            bool own_args = false;
            if (ext) {  // sg_submit_ex: validate the event's args; a NullContext event is k_lane's
                const sg_event_ext x = ext[i];
                if (x.n_args > SG_MAX_ARGS || (uint64_t)x.arg_off + x.n_args > n_args) fl |= BF_BAD_ARGS;
                else if (x.n_args) {
                    for (uint32_t k = 0; k < x.n_args; ++k) {
                        const sg_arg a = args[x.arg_off + k];
                        if (a.kind > SG_ARG_LIST || (a.kind == SG_ARG_LIST && (a.key > n_args || a.len > n_args - a.key)))
                            fl |= BF_BAD_ARGS;
                        else if (a.kind == SG_ARG_LIST) {
                            mark |= PM_ARGL;
                            for (uint32_t q = 0; q < a.len; ++q)
                                if (args[a.key + q].kind > SG_ARG_SCALAR) fl |= BF_BAD_ARGS;
                        }
                    }
                    const sg_arg a0 = args[x.arg_off];
                    key0 = a0.kind == SG_ARG_SCALAR ? a0.key : NO_KEY;
                    own_args = true;
                }
                if (x.context_id > max_ctx) mark |= PM_LANE;
                else if (x.origin_id != 0 || x.context_id != 0) {
                    mark |= PM_AUX;
                    if (x.origin_id >> TAG_ORIGIN_BITS) mark |= PM_LANE;
                }
            }
            if (own_args && e.kind == SG_EV_EXIT && (e.flags & SG_F_EXIT_ARGS)) mark |= PM_XARGS;
            if (e.kind == SG_EV_ENTRY) {
                if (key_ring) key_ring[(gbase + i) & ring_mask] = key0;
                if (e.flags & SG_F_PRIORITIZED) mark |= PM_PRIO;
                if (e.flags & SG_F_BLOCKED_UPSTREAM) mark |= PM_LANE;
            } else if (e.kind == SG_EV_EXIT && own_args && key_ring) {
                key_ring[(gbase + i) & ring_mask] = key0;
            }
            if (e.kind != SG_EV_ENTRY) {
                const uint64_t ref = e.aux & SG_REF_NONE;
                if (ref != SG_REF_NONE && ref >= gbase && ref - gbase >= i) fl |= BF_BAD_REF;  // must follow its ENTRY
            }
            if (mark && e.res_id < max_res && (prio[e.res_id] & mark) != mark) atomicOr(&prio[e.res_id], mark);
            key = (comp && e.res_id < max_res) ? comp[e.res_id] : e.res_id;
            if (key < max_res) hid = hot_tab[key];
            if (e.kind == SG_EV_ENTRY) entm |= 1u << it;
        }
        kk[it] = key;
        const bool hot = valid && hid < nhot;
        // hot: the rank among the wave's earlier items of the same id (peers by ballots over the id's bits)
        uint64_t peers = __ballot(hot);
#pragma unroll
        for (int b = 0; b < 10; ++b) {
            const uint64_t bb = __ballot((hid >> b) & 1);
            peers &= ((hid >> b) & 1) ? bb : ~bb;
        }
        const uint32_t hrank = __popcll(peers & lt);
        uint32_t* myc = wcnt[w];
        const uint32_t old = hot ? myc[hid] : 0u;  // (read by every peer before its first one bumps it)
        if (hot && hrank == 0) myc[hid] = old + (uint32_t)__popcll(peers);
        const uint64_t cb = __ballot(valid && !hot);
        if (hot) {
            hotm |= 1u << it;
            rk[it] = (hid << 16) | (old + hrank);
        } else {
            rk[it] = ccount + (uint32_t)__popcll(cb & lt);
        }
        ccount += (uint32_t)__popcll(cb);
        hist_add<DB>(h, key & (NB - 1), valid && !hot);
    }
    if (l == 0) cw[w] = ccount;
    if (fl) atomicOr(bflags, fl);
    __syncthreads();
    // per hot id: the waves' offsets (exclusive over waves) in place, the tile's count to its row of the hot
    // counts (tile-major: one contiguous row a tile; k_hot_scan_* turn them into the runs' positions)
    for (uint32_t d = threadIdx.x; d < nhot; d += RS_THREADS) {
        uint32_t acc = 0;
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) { const uint32_t c = wcnt[ww][d]; wcnt[ww][d] = acc; acc += c; }
        hot_hist[(uint64_t)blockIdx.x * nhot + d] = acc;
    }
    uint32_t coff = 0;
    for (int ww = 0; ww < w; ++ww) coff += cw[ww];
    if (threadIdx.x == 0) ccnt[blockIdx.x] = cw[0] + cw[1] + cw[2] + cw[3];
    for (int b = threadIdx.x; b < NB; b += RS_THREADS) chist[(uint64_t)b * nblocks + blockIdx.x] = h[b];
    __syncthreads();
#pragma unroll
    for (int it = 0; it < RS_ITEMS; ++it) {
        const uint64_t i = wbase + (uint64_t)it * WAVE + l;
        if (i >= n) continue;
        const uint32_t ent = ((entm >> it) & 1) ? W_ENT : 0u;
        if ((hotm >> it) & 1) {
            const uint32_t hid = rk[it] >> 16;
            words[i] = W_HOT | ent | (hid << 12) | (wcnt[w][hid] + (rk[it] & 0xFFFFu));
        } else {
            words[i] = ent;
            const uint64_t o = base + coff + rk[it];  // the tile's cold items, compacted in event order
            ckeys[o] = kk[it];
            cvals[o] = (uint32_t)i | (((entm >> it) & 1) ? 0x80000000u : 0u);
        }
    }
}

// ---- the hot runs' sorted positions: the tile-major counts C[tile][h] become P[tile][h] = the first position of
// tile's run of hot id h = sum over h' < h of h''s total + sum over tiles < tile of C[.][h] (hot ids in order,
// each in tile order).  Reduce-then-scan along the tiles, TC tiles a chunk, rows read and written contiguous.
#define HS_TC 16u  // (16 tiles a chunk: 512 chunks of a 2^25-event batch; 64 measured ~1 % slower in the pipeline)
// partial sums of every chunk: part[chunk][h]
__global__ __launch_bounds__(256) void k_hot_scan_a(const uint32_t* __restrict__ C, uint32_t nblocks, uint32_t nhot,
                                                    uint32_t* __restrict__ part) {
    const uint32_t c = blockIdx.x, t0 = c * HS_TC, t1 = min(nblocks, t0 + HS_TC);
    for (uint32_t h = threadIdx.x; h < nhot; h += 256) {
        uint32_t a = 0;
        for (uint32_t t = t0; t < t1; ++t) a += C[(uint64_t)t * nhot + h];
        part[(uint64_t)c * nhot + h] = a;
    }
}
// one workgroup: every chunk's exclusive prefix per h (in place), the ids' totals and bases: hb[h] = first position of
// id h, hb[HOT_MAX + h] = its total; out[0] = hot_total
__global__ __launch_bounds__(HOT_MAX) void k_hot_scan_b(uint32_t* __restrict__ part, uint32_t nch, uint32_t nhot,
                                                        uint32_t* __restrict__ hb, uint32_t* __restrict__ out) {
    __shared__ uint32_t ws[HOT_MAX / 64];
    const uint32_t h = threadIdx.x, l = h & 63, wv = h >> 6;
    uint32_t tot = 0;
    if (h < nhot) {
        // the column's loads 16 chunks at a time (one dependent L2 round trip per chunk made this single workgroup
        // ~0.22 ms of a C4 batch's serial group stage: 512 chunks)
        constexpr uint32_t U = 16;
        uint32_t c = 0;
        for (; c + U <= nch; c += U) {
            uint32_t v[U];
#pragma unroll
            for (uint32_t k = 0; k < U; ++k) v[k] = part[(uint64_t)(c + k) * nhot + h];
#pragma unroll
            for (uint32_t k = 0; k < U; ++k) {
                part[(uint64_t)(c + k) * nhot + h] = tot;
                tot += v[k];
            }
        }
        for (; c < nch; ++c) {
            const uint32_t v = part[(uint64_t)c * nhot + h];
            part[(uint64_t)c * nhot + h] = tot;
            tot += v;
        }
    }
    uint32_t x = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if ((int)l >= o) x += y;
    }
    if (l == 63) ws[wv] = x;
    __syncthreads();
    uint32_t pre = 0, all = 0;
    for (uint32_t k = 0; k < HOT_MAX / 64; ++k) { if (k < wv) pre += ws[k]; all += ws[k]; }
    if (h < nhot) { hb[h] = pre + x - tot; hb[HOT_MAX + h] = tot; }
    if (h == 0) *out = all;
}
// P in place of C: chunk base (hb + part) and a running sum down the chunk's tiles
__global__ __launch_bounds__(256) void k_hot_scan_c(uint32_t* __restrict__ C, uint32_t nblocks, uint32_t nhot,
                                                    const uint32_t* __restrict__ part, const uint32_t* __restrict__ hb) {
    const uint32_t c = blockIdx.x, t0 = c * HS_TC, t1 = min(nblocks, t0 + HS_TC);
    for (uint32_t h = threadIdx.x; h < nhot; h += 256) {
        uint32_t run = hb[h] + part[(uint64_t)c * nhot + h];
        for (uint32_t t = t0; t < t1; ++t) {
            const uint32_t v = C[(uint64_t)t * nhot + h];
            C[(uint64_t)t * nhot + h] = run;
            run += v;
        }
    }
}

// The sorted position of event j from its word (hot: the tile's run start + rank; cold: the word itself)
__device__ __forceinline__ uint32_t grp_pos(uint64_t j, uint32_t wd, const uint32_t* __restrict__ P, uint32_t nhot) {
    if (wd & W_HOT) return P[(j / RS_TILE) * nhot + ((wd >> 12) & (HOT_MAX - 1))] + (wd & 0xFFFu);
    return wd & W_POS;
}

// Every event's 16-byte record at its sorted position: a workgroup of 256 lanes per quarter of a 4096-event tile
// (4 events a lane, in submission order; four workgroups a CU).  The quarter's hot events are staged in LDS in
// (hot id, rank) order -- a quarter's events of one id hold consecutive ranks of the tile's run, r0 .. r0 + c -- and
// leave as runs of consecutive positions (records and sorted values); a cold event's record goes straight to its
// position (the cold sort placed it).  References to ENTRYs of this batch become the ENTRY's sorted position: an
// EXIT sits ~RT of traffic after its ENTRY, so the ENTRY's word and position are recent lines.  A reference must
// name an earlier ENTRY of the same resource: two hot events by their ids here, two cold ones by their sort keys in
// k_block_sums (sorted order); one naming a non-ENTRY resolves like an unknown entry.  References into earlier
// batches are listed (prev) for k_resolve.
#define GR_THREADS 256
#define GR_EVENTS (RS_TILE / 4)
#define GR_ITEMS (GR_EVENTS / GR_THREADS)
__global__ __launch_bounds__(GR_THREADS) void k_grp_records(const sg_event* __restrict__ ev, uint64_t n,
                                                            uint64_t gbase, uint64_t ring_mask, int32_t max_rt,
                                                            const uint32_t* __restrict__ words,
                                                            const uint32_t* __restrict__ P, uint32_t nhot,
                                                            uint32_t nblocks, const uint32_t* __restrict__ hb,
                                                            SEv* __restrict__ recs,
                                                            uint32_t* __restrict__ svals, uint32_t* __restrict__ prev,
                                                            uint32_t* __restrict__ nprev, uint32_t* __restrict__ bst,
                                                            uint32_t* __restrict__ bflags,
                                                            const sg_event_ext* __restrict__ ext,
                                                            const sg_arg* __restrict__ args, uint32_t max_ctx,
                                                            Link* __restrict__ link, uint32_t epoch) {
    __shared__ uint4 srec[GR_EVENTS];        // the quarter's hot records in (hot id, rank) order
    __shared__ uint32_t spos[GR_EVENTS], sval[GR_EVENTS];
    __shared__ uint32_t lo[HOT_MAX];         // per hot id: the quarter's count, then its first local slot
    __shared__ uint32_t r0[HOT_MAX];         // ... its first rank in the tile's run
    __shared__ uint32_t prow[HOT_MAX];       // ... the tile's run's first sorted position
    __shared__ uint32_t ws[GR_THREADS / 64];
    __shared__ uint32_t nh_q;
    const uint32_t t = threadIdx.x, l = t & 63, wv = t >> 6;
    const uint32_t tile = blockIdx.x >> 2;
    const uint64_t base = (uint64_t)tile * RS_TILE + (uint64_t)(blockIdx.x & 3) * GR_EVENTS;
    // the quarter's events and words first (their loads in flight across the setup below)
    sg_event e[GR_ITEMS];
    uint32_t wd[GR_ITEMS];
#pragma unroll
    for (int it = 0; it < GR_ITEMS; ++it) {  // (clamped, unconditional loads: no wait between them)
        const uint64_t i = base + (uint64_t)it * GR_THREADS + t;
        const uint64_t ic = i < n ? i : n - 1;
        e[it] = ev[ic];
        wd[it] = words[ic];
    }
#pragma unroll
    for (int it = 0; it < GR_ITEMS; ++it)
        if (base + (uint64_t)it * GR_THREADS + t >= n) { e[it].kind = 0xFF; wd[it] = 0; }
    for (uint32_t h = t; h < nhot; h += GR_THREADS) {
        lo[h] = 0;
        r0[h] = 0xFFFFFFFFu;
        prow[h] = P[(uint64_t)tile * nhot + h];
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < GR_ITEMS; ++it)
        if (wd[it] & W_HOT) {
            const uint32_t h = (wd[it] >> 12) & (HOT_MAX - 1);
            atomicAdd(&lo[h], 1u);
            atomicMin(&r0[h], wd[it] & 0xFFFu);
        }
    __syncthreads();
    {   // local slots: exclusive scan of the counts over the ids (4 ids a lane)
        constexpr uint32_t PER = HOT_MAX / GR_THREADS;
        uint32_t c[PER], sum = 0;
#pragma unroll
        for (uint32_t k = 0; k < PER; ++k) {
            const uint32_t h = t * PER + k;
            c[k] = h < nhot ? lo[h] : 0u;
            sum += c[k];
        }
        uint32_t x = sum;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if ((int)l >= o) x += y;
        }
        if (l == 63) ws[wv] = x;
        __syncthreads();
        uint32_t pre = 0, all = 0;
        for (uint32_t k = 0; k < GR_THREADS / 64; ++k) { if (k < wv) pre += ws[k]; all += ws[k]; }
        uint32_t run = pre + x - sum;
#pragma unroll
        for (uint32_t k = 0; k < PER; ++k) {
            const uint32_t h = t * PER + k;
            if (h < nhot) lo[h] = run;
            run += c[k];
        }
        if (t == 0) nh_q = all;
    }
    __syncthreads();
    const int64_t t0 = ev[0].ts;
    // every item's own position (hot: its run's start in LDS; cold: pos_of) and its reference's word, all loads
    // issued before any is used (each item's chain is a few dependent cache lines: overlap them)
    uint32_t p[GR_ITEMS], wj[GR_ITEMS];
    uint64_t jj[GR_ITEMS];
#pragma unroll
    for (int it = 0; it < GR_ITEMS; ++it) {
        const uint64_t i = base + (uint64_t)it * GR_THREADS + t;
        jj[it] = ~0ull;
        wj[it] = 0;
        p[it] = 0;
        if (i >= n) continue;
        if (!(wd[it] & W_HOT)) p[it] = wd[it] & W_POS;
        if (e[it].kind != SG_EV_ENTRY) {
            const uint64_t ref = e[it].aux & SG_REF_NONE;
            if (ref != SG_REF_NONE && ref >= gbase && ref - gbase < i) jj[it] = ref - gbase;  // (k_grp_first flagged the others)
        }
    }
    // the referenced ENTRYs' words, then the hot ones' run starts: clamped, unconditional loads, each kind issued
    // together (a load under a per-lane condition gets its own wait)
#pragma unroll
    for (int it = 0; it < GR_ITEMS; ++it) {
        const uint32_t x = words[jj[it] == ~0ull ? 0ull : jj[it]];
        wj[it] = jj[it] == ~0ull ? 0u : x;
    }
    uint32_t pj[GR_ITEMS];
#pragma unroll
    for (int it = 0; it < GR_ITEMS; ++it) {
        const uint64_t j = jj[it] == ~0ull ? 0ull : jj[it];
        pj[it] = P[(wj[it] & W_HOT) ? (j / RS_TILE) * nhot + ((wj[it] >> 12) & (HOT_MAX - 1)) : 0];
    }
#pragma unroll
    for (int it = 0; it < GR_ITEMS; ++it)  // (= grp_pos)
        pj[it] = jj[it] == ~0ull ? 0u : (wj[it] & W_HOT) ? pj[it] + (wj[it] & 0xFFFu) : (wj[it] & W_POS);
    // the records
    bool bad = false, zero = false;
#pragma unroll
    for (int it = 0; it < GR_ITEMS; ++it) {
        const uint64_t i = base + (uint64_t)it * GR_THREADS + t;
        bool is_prev = false;
        uint32_t q = 0;
        if (i < n) {
            const sg_event& ee = e[it];
            const uint32_t w = wd[it];
            const bool hot = (w & W_HOT) != 0;
            const bool entry = ee.kind == SG_EV_ENTRY;
            const uint32_t hid = (w >> 12) & (HOT_MAX - 1);
            q = hot ? prow[hid] + (w & 0xFFFu) : p[it];
            SEv r;
            r.dt = (int32_t)(ee.ts - t0);
            r.x = 0;
            r.cnt = ee.count;
            r.rt = 0;
            r.kind = ee.kind;
            r.flags = (uint8_t)(ee.flags & 0x3Fu);  // the ABI's SG_F_* bits only (RF_* are internal)
            r.code = RC_NONE;
            r.pad = 0;
            uint32_t tag = 0;
            bool own_args = false;
            uint64_t key0 = (ee.flags & SG_F_HAS_ARG) ? ee.aux : NO_KEY;
            if (ext) {
                const sg_event_ext x = ext[i];
                if (x.n_args && x.n_args <= SG_MAX_ARGS) {
                    const sg_arg a0 = args[x.arg_off];
                    key0 = a0.kind == SG_ARG_SCALAR ? a0.key : NO_KEY;
                    own_args = true;
                }
                if (x.context_id <= max_ctx && (x.origin_id != 0 || x.context_id != 0) && !(x.origin_id >> TAG_ORIGIN_BITS))
                    tag = x.origin_id | (x.context_id << TAG_ORIGIN_BITS);
            }
            if (own_args) {
                r.flags = (uint8_t)((r.flags & ~SG_F_HAS_ARG) | (key0 != NO_KEY ? SG_F_HAS_ARG : 0));
                if (ee.kind == SG_EV_EXIT) r.flags |= RF_OWN_ARGS;
            }
            r.x = tag;
            if (entry) {
                zero |= ee.count == 0;
            } else {
                if (ee.kind == SG_EV_EXIT) {
                    const int64_t raw = (int64_t)(ee.aux >> 48);
                    r.rt = (uint16_t)(raw > max_rt ? max_rt : raw);
                }
                const uint64_t ref = ee.aux & SG_REF_NONE;
                if (jj[it] != ~0ull) {
                    if (wj[it] & W_ENT) {
                        // one hot and one cold, or two hot ids: not the same resource (two cold: k_block_sums)
                        if (((wj[it] ^ w) & W_HOT) || (hot && ((wj[it] >> 12) & (HOT_MAX - 1)) != hid)) bad = true;
                        r.code = RC_BATCH;
                        r.x = pj[it];
                    } else {
                        r.code = ee.kind == SG_EV_EXIT ? RC_NONE : RC_NOT;
                    }
                } else if (ref != SG_REF_NONE && ref < gbase) {
                    // an ENTRY of an earlier batch: its status is read from the ring by k_resolve
                    r.code = RC_PREV;
                    r.x = (uint32_t)(ref & ring_mask);
                    is_prev = true;
                }
                if (r.code == RC_NONE || r.code == RC_PREV) atomicOr(&bst[q >> 10], BST_STATIC);
            }
            uint4 rv;
            __builtin_memcpy(&rv, &r, sizeof(rv));
            if (hot) {
                const uint32_t slot = lo[hid] + (w & 0xFFFu) - r0[hid];
                srec[slot] = rv;
                spos[slot] = q;
                sval[slot] = (uint32_t)i | (entry ? 0x80000000u : 0u);
            } else {
                reinterpret_cast<uint4*>(recs)[q] = rv;
            }
        }
        // wave-aggregated prev-list slots
        const uint64_t pb = __ballot(is_prev);
        if (pb) {
            const int lead = __ffsll((long long)pb) - 1;
            uint32_t b0 = 0;
            if ((int)l == lead) b0 = atomicAdd(nprev, (uint32_t)__popcll(pb));
            b0 = __shfl(b0, lead, 64);
            if (is_prev) prev[b0 + __popcll(pb & ((1ull << l) - 1))] = q;
        }
    }
    if (__ballot(bad) && l == 0) atomicOr(bflags, BF_BAD_REF);
    if (__ballot(zero) && l == 0) atomicOr(bflags, BF_ZERO_CNT);
    __syncthreads();
    // the hot runs leave in slot order: consecutive slots of one id are consecutive positions.  On the way, the
    // sorted-order side tables of the hot region (k_block_sums does the cold one): each 1024-position block's ENTRY
    // count sum (a segmented wave sum over equal blocks: a run's positions are consecutive) and the forward link of
    // every referenced ENTRY (an EXIT run names an earlier tile's run of ENTRYs: nearby link slots).
    const uint32_t nh = nh_q;
    bool multi = false;
    for (uint32_t k0 = 0; k0 < nh; k0 += GR_THREADS) {  // (wave-uniform trip count)
        const uint32_t k = k0 + t;
        uint32_t key = 0xFFFFFFFFu, v = 0;
        if (k < nh) {
            const uint32_t q = spos[k];
            const uint4 rv = srec[k];
            reinterpret_cast<uint4*>(recs)[q] = rv;
            svals[q] = sval[k];
            key = q >> 10;
            const uint32_t kind = rv.w & 0xFFu, code = (rv.w >> 16) & 0xFFu;
            if (kind == SG_EV_ENTRY) v = rv.z & 0xFFFFu;
        }
        // segmented inclusive sum over runs of equal blocks; the last lane of each run adds it
        const uint32_t kp = __shfl_up(key, 1, 64), kn = __shfl_down(key, 1, 64);
        bool f = l == 0 || kp != key;
        uint32_t x = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            const bool g = __shfl_up(f ? 1 : 0, o, 64) != 0;
            if ((int)l >= o) {
                if (!f) x += y;
                f = f || g;
            }
        }
        if ((l == 63 || kn != key) && key != 0xFFFFFFFFu && x) atomicAdd(&bst[key], x);
    }
    // the links: every exchange of the quarter issued before any old value is looked at
    unsigned long long* xd[GR_ITEMS];
    unsigned long long xv[GR_ITEMS];
#pragma unroll
    for (int it = 0; it < GR_ITEMS; ++it) {
        const uint32_t k = (uint32_t)it * GR_THREADS + t;
        xd[it] = nullptr;
        xv[it] = 0;
        if (k < nh) {
            const uint4 rv = srec[k];
            const uint32_t kind = rv.w & 0xFFu, code = (rv.w >> 16) & 0xFFu;
            if (kind != SG_EV_ENTRY && code == RC_BATCH) {
                xd[it] = reinterpret_cast<unsigned long long*>(kind == SG_EV_EXIT ? &link[rv.y].exit_l
                                                                                  : &link[rv.y].trace_l);
                xv[it] = ((unsigned long long)epoch << 32) | spos[k];
            }
        }
    }
    static_assert(GR_ITEMS == 4, "four exchanges a lane");
    auto xch = [&](int it) -> uint32_t { return xd[it] ? (uint32_t)(atomicExch(xd[it], xv[it]) >> 32) : 0u; };
    const uint32_t o0 = xch(0), o1 = xch(1), o2 = xch(2), o3 = xch(3);
    if (o0 == epoch || o1 == epoch || o2 == epoch || o3 == epoch) multi = true;  // (epochs start at 1)
    if (__ballot(multi) && l == 0) atomicOr(bflags, BF_MULTI_LINK);
}

// Decisions back to submission order from the words (the hot / cold stage's inverse permutation): only ENTRYs are
// gathered (every other event's word is mk_dec(ST_NOT_ENTRY, 0, 0)); the status ring keeps every event's status
// for references from later batches.  The hot positions read their tile's row of P (a few lines a tile).
#define POSTW_ITEMS 4
__global__ __launch_bounds__(256) void k_post_w(const uint32_t* __restrict__ words, const uint32_t* __restrict__ P,
                                                uint32_t nhot, const uint32_t* __restrict__ dec, uint64_t n,
                                                uint64_t gbase, uint8_t* __restrict__ ring, uint64_t ring_mask,
                                                uint32_t* __restrict__ out) {
    const uint64_t base = (uint64_t)blockIdx.x * (256 * POSTW_ITEMS) + threadIdx.x;
    uint32_t w[POSTW_ITEMS], d[POSTW_ITEMS];
#pragma unroll
    for (int k = 0; k < POSTW_ITEMS; ++k) {
        const uint64_t i = base + (uint64_t)k * 256;
        w[k] = i < n ? words[i] : 0u;
    }
    // (the hot rows' positions, then the decisions: clamped, unconditional loads, each kind issued together -- a
    // load under a per-lane condition gets its own wait)
    uint32_t pr[POSTW_ITEMS];
#pragma unroll
    for (int k = 0; k < POSTW_ITEMS; ++k) {
        const uint64_t i = base + (uint64_t)k * 256;
        pr[k] = P[(w[k] & W_HOT) ? (i / RS_TILE) * nhot + ((w[k] >> 12) & (HOT_MAX - 1)) : 0];
    }
#pragma unroll
    for (int k = 0; k < POSTW_ITEMS; ++k) {
        const uint32_t q = (w[k] & W_HOT) ? pr[k] + (w[k] & 0xFFFu) : (w[k] & W_POS);
        const uint32_t x = dec[(w[k] & W_ENT) ? q : 0u];
        d[k] = (w[k] & W_ENT) ? x : (uint32_t)ST_NOT_ENTRY;  // (= mk_dec(ST_NOT_ENTRY, 0, 0))
    }
#pragma unroll
    for (int k = 0; k < POSTW_ITEMS; ++k) {
        const uint64_t i = base + (uint64_t)k * 256;
        if (i < n) {
            out[i] = d[k];
            ring[(gbase + i) & ring_mask] = (uint8_t)(d[k] & 0xFF);
        }
    }
}

// The hot ids' segments (hot id order, the non-empty ones) from their bases and totals (hb): segs[0 .. k),
// out[0] = k.  One workgroup of HOT_MAX lanes.
__global__ __launch_bounds__(HOT_MAX) void k_hot_segs(const uint32_t* __restrict__ hb, uint32_t nhot,
                                                      const uint32_t* __restrict__ hot_list, Seg* __restrict__ segs,
                                                      uint32_t* __restrict__ out) {
    __shared__ uint32_t ws[HOT_MAX / 64];
    const uint32_t t = threadIdx.x, l = t & 63, wv = t >> 6;
    const uint32_t len = t < nhot ? hb[HOT_MAX + t] : 0u;
    const uint32_t f = len ? 1u : 0u;
    uint32_t x = f;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if ((int)l >= o) x += y;
    }
    if (l == 63) ws[wv] = x;
    __syncthreads();
    uint32_t pre = 0, all = 0;
    for (uint32_t k = 0; k < HOT_MAX / 64; ++k) { if (k < wv) pre += ws[k]; all += ws[k]; }
    if (f) {
        Seg sg;
        sg.res = hot_list[t];
        sg.start = hb[t];
        sg.len = 0;
        sg.bin = 0;
        segs[pre + x - f] = sg;
    }
    if (t == 0) out[0] = all;
}

// The next batch's hot ids: the segments of this one with >= min_len events (at most HOT_MAX, first come); the
// previous ids are cleared first (k_hot_clear).  hot_n = the new count (for the host with the batch's head).
__global__ void k_hot_clear(uint16_t* __restrict__ hot_tab, const uint32_t* __restrict__ hot_list, uint32_t nhot) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < nhot) hot_tab[hot_list[t]] = (uint16_t)HOT_NONE;
}
// (after k_seg_bin: Seg.len is set)
__global__ __launch_bounds__(256) void k_hot_build(const Seg* __restrict__ segs, const uint32_t* __restrict__ mp,
                                                   uint32_t min_len, uint32_t max_res, uint16_t* __restrict__ hot_tab,
                                                   uint32_t* __restrict__ hot_list, uint32_t* __restrict__ hot_n) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= *mp || segs[s].len < min_len || segs[s].res >= max_res) return;  // (a batch the host will refuse)
    const uint32_t k = atomicAdd(hot_n, 1u);
    if (k >= HOT_MAX) return;
    const uint32_t r = segs[s].res;
    hot_tab[r] = (uint16_t)k;
    hot_list[k] = r;
}

template <int DB>
// ndev (optional): the key count on the device, at most n (the grid is sized for n)
__global__ __launch_bounds__(RS_THREADS) void k_radix_hist(const uint32_t* __restrict__ keys, uint64_t n, int shift,
                                                        uint32_t* __restrict__ ghist, uint32_t nblocks,
                                                        const uint32_t* __restrict__ ndev) {
    constexpr int NB = 1 << DB;
    if (ndev && *ndev < n) n = *ndev;
    __shared__ uint32_t h[NB];
    for (int i = threadIdx.x; i < NB; i += RS_THREADS) h[i] = 0;
    __syncthreads();
    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
#pragma unroll
    for (int it = 0; it < RS_ITEMS; ++it) {
        const uint64_t i = base + (uint64_t)it * RS_THREADS + threadIdx.x;
        hist_add<DB>(h, i < n ? (keys[i] >> shift) & (NB - 1) : 0u, i < n);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < NB; b += RS_THREADS) ghist[(uint64_t)b * nblocks + blockIdx.x] = h[b];
}

// Stable scatter of one DB-bit digit (8 or 10).  Wave w of a tile owns the contiguous quarter
// [base + w*1024, base + (w+1)*1024) and walks it in 16 coalesced rounds of 64, so input order is
// (wave, round, lane): every wave ranks its own items against a wave-private digit counter
// (peers by DB ballots, no block barrier per round), one block-wide scan turns the four waves'
// counts into digit-run offsets, and the tile is placed digit-sorted in LDS.  It then leaves in
// digit runs, so the writes of a run are consecutive addresses.  The last pass also writes the
// inverse permutation pos_of[idx] = sorted position | ENTRY bit.  (The per-block digit histograms
// of k_rs_first / k_radix_hist count the same 4096-item tile, in any order.)  8-bit digits: two 10-bit
// passes for 1M resources measured slower (1024 digit runs per 4096-item tile are too short to write
// coalesced).
template <int DB>
__global__ __launch_bounds__(RS_THREADS) void k_radix_scatter(const uint32_t* __restrict__ keys_in,
                                                           const uint32_t* __restrict__ vals_in, uint64_t n, int shift,
                                                           const uint32_t* __restrict__ goff, uint32_t nblocks,
                                                           uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
                                                           uint32_t* __restrict__ pos_of, const uint32_t* __restrict__ ndev,
                                                           const uint32_t* __restrict__ tcnt,
                                                           const uint32_t* __restrict__ dbase, uint32_t wfmt) {
    constexpr int NB = 1 << DB;
    if (ndev && *ndev < n) n = *ndev;
    if ((uint64_t)blockIdx.x * RS_TILE >= n) return;  // (a tile past the device count: nothing to move)
    // tcnt (optional): tile t holds tcnt[t] items at its start (k_grp_first's compacted cold items), the rest of
    // its span is not input; dbase (optional): every destination is offset by *dbase
    if (tcnt) n = (uint64_t)blockIdx.x * RS_TILE + tcnt[blockIdx.x];
    const uint32_t ob = dbase ? *dbase : 0u;
    constexpr int DPT = NB / RS_THREADS;  // digits per thread in the offset scan
    static_assert(NB % RS_THREADS == 0, "whole digits per thread");
    __shared__ uint32_t sk[RS_TILE], sv[RS_TILE];
    __shared__ uint32_t wcnt[4][NB];   // per-wave digit counts, then per-wave digit offsets
    __shared__ int64_t gdst[NB];       // global position of local position 0 of each digit's run
    __shared__ uint32_t wtot[4];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
    const uint64_t wbase = base + (uint64_t)w * (RS_TILE / 4);
    const uint32_t cnt_tile = (uint32_t)((n - base) < RS_TILE ? (n - base) : RS_TILE);
    uint32_t kk[RS_ITEMS], vv[RS_ITEMS], rk[RS_ITEMS];
#pragma unroll
    for (int it = 0; it < RS_ITEMS; ++it) {  // per-wave rounds of 64 consecutive items: coalesced
        const uint64_t i = wbase + (uint64_t)it * WAVE + l;
        kk[it] = i < n ? keys_in[i] : 0u;
        vv[it] = i < n ? vals_in[i] : 0u;
    }
    for (int i = threadIdx.x; i < 4 * NB; i += RS_THREADS) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint64_t lt_mask = (l == 0) ? 0ull : (~0ull >> (64 - l));
    uint32_t* myc = wcnt[w];
#pragma unroll
    for (int it = 0; it < RS_ITEMS; ++it) {
        const uint64_t i = wbase + (uint64_t)it * WAVE + l;
        const bool valid = i < n;
        const uint32_t d = (kk[it] >> shift) & (NB - 1);
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (int b = 0; b < DB; ++b) {
            const uint64_t bb = __ballot((d >> b) & 1);
            peers &= ((d >> b) & 1) ? bb : ~bb;
        }
        const uint32_t rank = __popcll(peers & lt_mask);
        // every lane of the wave reads the digit's count before its first peer (rank 0) bumps it;
        // LDS instructions of one wave execute in order
        const uint32_t old = valid ? myc[d] : 0u;
        rk[it] = old + rank;
        if (valid && rank == 0) myc[d] = old + (uint32_t)__popcll(peers);
    }
    __syncthreads();
    {   // thread t owns digits [t*DPT, (t+1)*DPT): run offsets (exclusive scan over digits), then the waves
        uint32_t c[DPT][4], t = 0;
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const int d = threadIdx.x * DPT + j;
#pragma unroll
            for (int ww = 0; ww < 4; ++ww) { c[j][ww] = wcnt[ww][d]; t += c[j][ww]; }
        }
        uint32_t x = t;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(x, o, 64);
            if (l >= o) x += y;
        }
        if (l == 63) wtot[w] = x;
        __syncthreads();
        uint32_t acc = x - t;
        for (int ww = 0; ww < w; ++ww) acc += wtot[ww];
#pragma unroll
        for (int j = 0; j < DPT; ++j) {
            const int d = threadIdx.x * DPT + j;
            gdst[d] = (int64_t)goff[(uint64_t)d * nblocks + blockIdx.x] - (int64_t)acc;
#pragma unroll
            for (int ww = 0; ww < 4; ++ww) { wcnt[ww][d] = acc; acc += c[j][ww]; }
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < RS_ITEMS; ++it) {
        const uint64_t i = wbase + (uint64_t)it * WAVE + l;
        if (i < n) {
            const uint32_t lp = myc[(kk[it] >> shift) & (NB - 1)] + rk[it];
            sk[lp] = kk[it];
            sv[lp] = vv[it];
        }
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < cnt_tile; p += RS_THREADS) {  // digit runs: consecutive addresses
        const uint32_t k = sk[p], v = sv[p];
        const uint64_t dst = (uint64_t)(gdst[(k >> shift) & (NB - 1)] + (int64_t)p) + ob;
        keys_out[dst] = k;
        vals_out[dst] = v;
        // the inverse permutation: pos_of[index] = position | ENTRY << 31, or (wfmt: the hot / cold stage's word of
        // a cold event) position | ENTRY << 30 (W_ENT)
        if (pos_of) pos_of[v & 0x7FFFFFFFu] = (uint32_t)dst | (wfmt ? (v >> 1) & 0x40000000u : (v & 0x80000000u));
    }
}

// =================================================================================
// exclusive scan of uint32 (reduce-then-scan)
// =================================================================================
#define SC_THREADS 256
#define SC_ITEMS 16
#define SC_TILE (SC_THREADS * SC_ITEMS)

__device__ uint32_t block_excl_scan(uint32_t v, uint32_t* total) {
    __shared__ uint32_t ws[SC_THREADS / WAVE];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    uint32_t x = v;
    #pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(x, o, 64);
        if (l >= o) x += y;
    }
    if (l == 63) ws[w] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    #pragma unroll
    for (int i = 0; i < SC_THREADS / WAVE; ++i) { if (i < w) pre += ws[i]; tot += ws[i]; }
    __syncthreads();
    if (total) *total = tot;
    return pre + x - v;
}

// ndev (optional): the element count on the device, at most n (the grid covers n): tiles past it add nothing
__global__ __launch_bounds__(SC_THREADS) void k_scan_reduce(const uint32_t* __restrict__ in, uint64_t n, uint32_t* __restrict__ part,
                                                         const uint32_t* __restrict__ ndev) {
    if (ndev && *ndev < n) n = *ndev;
    uint64_t base = (uint64_t)blockIdx.x * SC_TILE;
    if (base >= n) {
        if (threadIdx.x == 0) part[blockIdx.x] = 0;
        return;
    }
    uint32_t s = 0;
    for (int it = 0; it < SC_ITEMS; ++it) {
        uint64_t i = base + (uint64_t)it * SC_THREADS + threadIdx.x;
        if (i < n) s += in[i];
    }
    uint32_t tot;
    block_excl_scan(s, &tot);
    if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// single workgroup scans the partials (nparts <= SC_TILE * ...) sequentially in tiles
__global__ __launch_bounds__(SC_THREADS) void k_scan_top(uint32_t* __restrict__ part, uint32_t nparts, uint32_t* __restrict__ total_out) {
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nparts; base += SC_THREADS) {
        uint32_t i = base + threadIdx.x;
        uint32_t v = i < nparts ? part[i] : 0;
        uint32_t tot;
        uint32_t ex = block_excl_scan(v, &tot);
        if (i < nparts) part[i] = carry + ex;
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0 && total_out) *total_out = carry;
}

__global__ __launch_bounds__(SC_THREADS) void k_scan_down(const uint32_t* __restrict__ in, uint64_t n, const uint32_t* __restrict__ part,
                                                       uint32_t* __restrict__ out, const uint32_t* __restrict__ ndev) {
    if (ndev && *ndev < n) n = *ndev;
    if ((uint64_t)blockIdx.x * SC_TILE >= n) return;
    // each thread owns SC_ITEMS consecutive items (blocked) for a sequential local scan
    uint64_t base = (uint64_t)blockIdx.x * SC_TILE + (uint64_t)threadIdx.x * SC_ITEMS;
    uint32_t loc[SC_ITEMS];
    uint32_t s = 0;
    #pragma unroll
    for (int k = 0; k < SC_ITEMS; ++k) {
        uint64_t i = base + k;
        loc[k] = i < n ? in[i] : 0;
        s += loc[k];
    }
    uint32_t ex = block_excl_scan(s, nullptr) + part[blockIdx.x];
    #pragma unroll
    for (int k = 0; k < SC_ITEMS; ++k) {
        uint64_t i = base + k;
        if (i < n) out[i] = ex;
        ex += loc[k];
    }
}

// =================================================================================
// 4. per-second MetricNode snapshot (StatisticNode.metrics, StatisticNode.java:124-151)
// =================================================================================
__device__ __forceinline__ bool snap_valid(const Bkt& b, int64_t now, int64_t cur, int64_t last) {
    if (b.ws < 0 || now - b.ws > 60000) return false;
    int64_t rt = b.succ != 0 ? b.rt / b.succ : b.rt;
    bool in_time = b.ws > last && b.ws < cur;
    bool nz = b.pass > 0 || b.block > 0 || b.succ > 0 || b.exc > 0 || rt > 0 || b.occ > 0;
    return in_time && nz;
}

// pass 1: details() side effect (reset the current bucket) + count per resource
__global__ void k_snap_count(Bkt* __restrict__ minb, const NodeInfo* __restrict__ info, uint32_t nres, int64_t now,
                             int32_t max_rt, uint32_t* __restrict__ cnt) {
    uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nres) return;
    if (!(info[r].flags & NI_CHAIN)) { cnt[r] = 0; return; }
    int64_t cur = now - now % 1000;
    int slot = (int)((now / 1000) % 60);
    Bkt& c = minb[(uint64_t)r * 60 + slot];
    if (c.ws < cur) { // LeapArray.currentWindow(now): create / reset
        c.ws = cur; c.pass = 0; c.block = 0; c.exc = 0; c.succ = 0; c.rt = 0; c.occ = 0; c.minrt = max_rt;
    }
    int64_t last = info[r].last_fetch;
    uint32_t k = 0;
    for (int s = 0; s < 60; ++s) if (snap_valid(minb[(uint64_t)r * 60 + s], now, cur, last)) ++k;
    cnt[r] = k;
}

__global__ void k_snap_emit(const Bkt* __restrict__ minb, NodeInfo* __restrict__ info, uint32_t nres, int64_t now,
                            const uint32_t* __restrict__ off, sg_metric_node* __restrict__ outp, uint64_t cap) {
    uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= nres) return;
    if (!(info[r].flags & NI_CHAIN)) return;
    int64_t cur = now - now % 1000;
    int64_t last = info[r].last_fetch, nl = last;
    uint64_t o = off[r];
    for (int s = 0; s < 60; ++s) {
        Bkt b = minb[(uint64_t)r * 60 + s];
        if (!snap_valid(b, now, cur, last)) continue;
        if (o < cap) {
            sg_metric_node m;
            m.timestamp = b.ws;
            m.pass_qps = b.pass;
            m.block_qps = b.block;
            m.success_qps = b.succ;
            m.exception_qps = b.exc;
            m.rt = b.succ != 0 ? b.rt / b.succ : b.rt;
            m.occupied_pass_qps = b.occ;
            m.res_id = r;
            m.reserved = 0;
            outp[o] = m;
        }
        ++o;
        if (b.ws > nl) nl = b.ws;
    }
    info[r].last_fetch = nl;
}

// =================================================================================
// state initialisation / flag updates
// =================================================================================
__global__ void k_init_state(Bkt* __restrict__ sec, Bkt* __restrict__ minb, NodeInfo* __restrict__ info,
                             int64_t* __restrict__ borrow, uint32_t nres) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    Bkt z;
    z.ws = -1; z.pass = 0; z.block = 0; z.exc = 0; z.succ = 0; z.rt = 0; z.occ = 0; z.minrt = 0;
    if (i < (uint64_t)nres * 60) minb[i] = z;
    if (i < (uint64_t)nres * 2) {
        sec[i] = z;
        borrow[2 * i] = -1;  // borrow slot never created
        borrow[2 * i + 1] = 0;
    }
    if (i < nres) {
        NodeInfo n;
        n.thread = 0; n.flags = 0; n.exc_sum_sec = -1; n.exc_sum = 0; n.last_fetch = -1;
        info[i] = n;
    }
}
// upd[i] = (set ? 1<<63 : 0) | flags << 32 | res
__global__ void k_set_flags(NodeInfo* __restrict__ info, const uint64_t* __restrict__ upd, uint32_t n) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t u = upd[i];
    uint32_t res = (uint32_t)u;
    uint32_t f = (uint32_t)((u >> 32) & 0x7FFFFFFFu);
    if (u >> 63) info[res].flags |= f;
    else info[res].flags &= ~f;
}
// the ParameterMetric map regions that survive a rule reload, moved into the new pools: one workgroup per
// region, tri[3 * i] = {source word, destination word, words}
__global__ void k_region_copy(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst, const uint64_t* __restrict__ tri) {
    const uint64_t s = tri[3 * blockIdx.x], d = tri[3 * blockIdx.x + 1], n = tri[3 * blockIdx.x + 2];
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) dst[d + i] = src[s + i];
}

// =================================================================================
// host-callable launch wrappers (engine.cpp)
// =================================================================================
namespace sg {

hipError_t launch_rs_first(const sg_event* ev, uint64_t n, uint32_t max_res, uint64_t gbase, const uint8_t* ring,
                           uint64_t ring_mask, int32_t max_rt, SEv* rec_o, uint32_t* keys, uint32_t* vals,
                           uint32_t* ghist, uint32_t nblocks, uint32_t* bflags, int64_t* t0_out, uint32_t* prio,
                           uint64_t* key_ring, const uint32_t* comp, const sg_event_ext* ext, const sg_arg* args,
                           uint64_t n_args, uint32_t max_ctx, hipStream_t st) {
    hipLaunchKernelGGL(k_rs_first<8>, dim3(nblocks), dim3(RS_THREADS), 0, st, ev, n, max_res, gbase, ring, ring_mask,
                       max_rt, rec_o, keys, vals, ghist, nblocks, bflags, t0_out, prio, key_ring, comp, ext, args,
                       n_args, max_ctx);
    return hipGetLastError();
}
hipError_t launch_radix_hist(const uint32_t* keys, uint64_t n, int shift, uint32_t* ghist, uint32_t nblocks,
                             hipStream_t st) {
    hipLaunchKernelGGL(k_radix_hist<8>, dim3(nblocks), dim3(RS_THREADS), 0, st, keys, n, shift, ghist, nblocks,
                       (const uint32_t*)nullptr);
    return hipGetLastError();
}
// the same over min(n, *ndev) keys (a count known on the device only; the grid is sized for n)
hipError_t launch_radix_hist_n(const uint32_t* keys, uint64_t n, const uint32_t* ndev, int shift, uint32_t* ghist,
                               uint32_t nblocks, hipStream_t st) {
    hipLaunchKernelGGL(k_radix_hist<8>, dim3(nblocks), dim3(RS_THREADS), 0, st, keys, n, shift, ghist, nblocks, ndev);
    return hipGetLastError();
}
hipError_t launch_radix_scatter_n(const uint32_t* kin, const uint32_t* vin, uint64_t n, const uint32_t* ndev, int shift,
                                  const uint32_t* goff, uint32_t nblocks, uint32_t* kout, uint32_t* vout, hipStream_t st) {
    hipLaunchKernelGGL(k_radix_scatter<8>, dim3(nblocks), dim3(RS_THREADS), 0, st, kin, vin, n, shift, goff, nblocks,
                       kout, vout, (uint32_t*)nullptr, ndev, (const uint32_t*)nullptr, (const uint32_t*)nullptr, 0u);
    return hipGetLastError();
}
hipError_t launch_radix_scatter(const uint32_t* kin, const uint32_t* vin, uint64_t n, int shift, const uint32_t* goff,
                                uint32_t nblocks, uint32_t* kout, uint32_t* vout, uint32_t* pos_of, hipStream_t st) {
    hipLaunchKernelGGL(k_radix_scatter<8>, dim3(nblocks), dim3(RS_THREADS), 0, st, kin, vin, n, shift, goff, nblocks,
                       kout, vout, pos_of, (const uint32_t*)nullptr, (const uint32_t*)nullptr, (const uint32_t*)nullptr, 0u);
    return hipGetLastError();
}
// the cold passes of the hot / cold group stage: tcnt = per-tile counts (first pass), ndev = the cold count (later
// passes), dbase = hot_total (last pass: sorted values at their final positions, and the cold events' words =
// position | W_ENT into pos_of = the words array)
hipError_t launch_radix_scatter_x(const uint32_t* kin, const uint32_t* vin, uint64_t n, const uint32_t* ndev,
                                  const uint32_t* tcnt, const uint32_t* dbase, int shift, const uint32_t* goff,
                                  uint32_t nblocks, uint32_t* kout, uint32_t* vout, uint32_t* pos_of, hipStream_t st) {
    hipLaunchKernelGGL(k_radix_scatter<8>, dim3(nblocks), dim3(RS_THREADS), 0, st, kin, vin, n, shift, goff, nblocks,
                       kout, vout, pos_of, ndev, tcnt, dbase, 1u);
    return hipGetLastError();
}
hipError_t launch_grp_first(const sg_event* ev, uint64_t n, uint32_t max_res, uint64_t gbase, uint64_t ring_mask,
                            uint32_t* bflags, int64_t* t0_out, uint32_t* prio, uint64_t* key_ring, const uint32_t* comp,
                            const sg_event_ext* ext, const sg_arg* args, uint64_t n_args, uint32_t max_ctx,
                            const uint16_t* hot_tab, uint32_t nhot, uint32_t nblocks, uint32_t* words,
                            uint32_t* hot_hist, uint32_t* ckeys, uint32_t* cvals, uint32_t* ccnt, uint32_t* chist,
                            hipStream_t st) {
    hipLaunchKernelGGL(k_grp_first<8>, dim3(nblocks), dim3(RS_THREADS), 0, st, ev, n, max_res, gbase, ring_mask, bflags,
                       t0_out, prio, key_ring, comp, ext, args, n_args, max_ctx, hot_tab, nhot, nblocks, words, hot_hist,
                       ckeys, cvals, ccnt, chist);
    return hipGetLastError();
}
hipError_t launch_hot_scan(uint32_t* C, uint32_t nblocks, uint32_t nhot, uint32_t* part, uint32_t* hb, uint32_t* total,
                           hipStream_t st) {
    if (!nhot) return hipMemsetAsync(total, 0, 4, st);
    const uint32_t nch = (nblocks + HS_TC - 1) / HS_TC;
    hipLaunchKernelGGL(k_hot_scan_a, dim3(nch), dim3(256), 0, st, C, nblocks, nhot, part);
    hipLaunchKernelGGL(k_hot_scan_b, dim3(1), dim3(HOT_MAX), 0, st, part, nch, nhot, hb, total);
    hipLaunchKernelGGL(k_hot_scan_c, dim3(nch), dim3(256), 0, st, C, nblocks, nhot, part, hb);
    return hipGetLastError();
}
hipError_t launch_grp_records(const sg_event* ev, uint64_t n, uint64_t gbase, uint64_t ring_mask, int32_t max_rt,
                              const uint32_t* words, const uint32_t* P, uint32_t nhot, uint32_t nblocks,
                              const uint32_t* hb, SEv* recs, uint32_t* svals, uint32_t* prev,
                              uint32_t* nprev, uint32_t* bst, uint32_t* bflags, const sg_event_ext* ext,
                              const sg_arg* args, uint32_t max_ctx, Link* link, uint32_t epoch, hipStream_t st) {
    hipLaunchKernelGGL(k_grp_records, dim3(nblocks * 4), dim3(GR_THREADS), 0, st, ev, n, gbase, ring_mask, max_rt, words, P,
                       nhot, nblocks, hb, recs, svals, prev, nprev, bst, bflags, ext, args, max_ctx, link, epoch);
    return hipGetLastError();
}
hipError_t launch_hot_segs(const uint32_t* hb, uint32_t nhot, const uint32_t* hot_list, Seg* segs, uint32_t* out,
                           hipStream_t st) {
    hipLaunchKernelGGL(k_hot_segs, dim3(1), dim3(HOT_MAX), 0, st, hb, nhot, hot_list, segs, out);
    return hipGetLastError();
}
hipError_t launch_hot_build(const Seg* segs, const uint32_t* mp, uint32_t mb, uint32_t min_len, uint32_t max_res, uint16_t* hot_tab,
                            uint32_t* hot_list, uint32_t nhot_old, uint32_t* hot_n, hipStream_t st) {
    if (nhot_old) hipLaunchKernelGGL(k_hot_clear, dim3((nhot_old + 255) / 256), dim3(256), 0, st, hot_tab, hot_list, nhot_old);
    if (mb) hipLaunchKernelGGL(k_hot_build, dim3((mb + 255) / 256), dim3(256), 0, st, segs, mp, min_len, max_res, hot_tab,
                               hot_list, hot_n);
    return hipGetLastError();
}
__global__ void k_cold_n(uint64_t n, const uint32_t* __restrict__ hot_total, uint32_t* __restrict__ out) {
    if (threadIdx.x == 0) *out = (uint32_t)(n - *hot_total);
}
hipError_t launch_cold_n(uint64_t n, const uint32_t* hot_total, uint32_t* out, hipStream_t st) {
    hipLaunchKernelGGL(k_cold_n, dim3(1), dim3(64), 0, st, n, hot_total, out);
    return hipGetLastError();
}
uint32_t hot_max() { return HOT_MAX; }

// A batch of one tile (n <= RS_TILE, the drop-in's synchronous calls): its cold (key, index) pairs -- compacted at
// the tile's start by k_grp_first, *cnt of them -- sorted in one workgroup instead of the radix passes' ~14 launches.
// A bitonic sort of (key << 32 | input position) is the stable sort by key the passes make; the outputs are the last
// pass's: sorted keys and values at *dbase + rank, and each cold event's word = its position | W_ENT.
__global__ __launch_bounds__(1024) void k_cold_small(const uint32_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                     const uint32_t* __restrict__ cnt_p, const uint32_t* __restrict__ dbase,
                                                     uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                     uint32_t* __restrict__ words) {
    __shared__ unsigned long long s[RS_TILE];
    const uint32_t cnt = *cnt_p, ob = *dbase, t = threadIdx.x;
    uint32_t n2 = 1;
    while (n2 < cnt) n2 <<= 1;
    for (uint32_t i = t; i < n2; i += blockDim.x)
        s[i] = i < cnt ? (((unsigned long long)kin[i] << 32) | i) : ~0ull;
    __syncthreads();
    for (uint32_t k = 2; k <= n2; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t i = t; i < n2; i += blockDim.x) {
                const uint32_t l = i ^ j;
                if (l > i) {
                    const unsigned long long a = s[i], b = s[l];
                    if (((i & k) == 0) == (a > b)) { s[i] = b; s[l] = a; }
                }
            }
            __syncthreads();
        }
    for (uint32_t i = t; i < cnt; i += blockDim.x) {
        const uint32_t idx = (uint32_t)s[i], key = (uint32_t)(s[i] >> 32), v = vin[idx], dst = ob + i;
        kout[dst] = key;
        vout[dst] = v;
        words[v & 0x7FFFFFFFu] = dst | ((v >> 1) & W_ENT);
    }
}
hipError_t launch_cold_small(const uint32_t* kin, const uint32_t* vin, const uint32_t* cnt, const uint32_t* dbase,
                             uint32_t* kout, uint32_t* vout, uint32_t* words, hipStream_t st) {
    hipLaunchKernelGGL(k_cold_small, dim3(1), dim3(1024), 0, st, kin, vin, cnt, dbase, kout, vout, words);
    return hipGetLastError();
}
hipError_t launch_post_w(const uint32_t* words, const uint32_t* P, uint32_t nhot, const uint32_t* dec, uint64_t n,
                         uint64_t gbase, uint8_t* ring, uint64_t ring_mask, uint32_t* out, hipStream_t st) {
    const uint32_t nb = (uint32_t)((n + 256 * POSTW_ITEMS - 1) / (256 * POSTW_ITEMS));
    hipLaunchKernelGGL(k_post_w, dim3(nb), dim3(256), 0, st, words, P, nhot, dec, n, gbase, ring, ring_mask, out);
    return hipGetLastError();
}

uint32_t radix_tile() { return RS_TILE; }

hipError_t launch_init_state(Bkt* sec, Bkt* minb, NodeInfo* info, int64_t* borrow, uint32_t nres, hipStream_t st) {
    uint64_t tot = (uint64_t)nres * 60;
    hipLaunchKernelGGL(k_init_state, dim3((uint32_t)((tot + 255) / 256)), dim3(256), 0, st, sec, minb, info, borrow, nres);
    return hipGetLastError();
}
hipError_t launch_set_flags(NodeInfo* info, const uint64_t* upd, uint32_t n, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_set_flags, dim3((n + 255) / 256), dim3(256), 0, st, info, upd, n);
    return hipGetLastError();
}

hipError_t launch_region_copy(const uint64_t* src, uint64_t* dst, const uint64_t* tri, uint32_t n, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_region_copy, dim3(n), dim3(256), 0, st, src, dst, tri);
    return hipGetLastError();
}

// exclusive scan in -> out (may alias); part must hold ceil(n / SC_TILE) + 1 words
// one tile (n <= SC_TILE): the whole exclusive scan in one workgroup (small batches' scans: one launch, not three)
__global__ __launch_bounds__(SC_THREADS) void k_scan_one(const uint32_t* __restrict__ in, uint64_t n,
                                                      uint32_t* __restrict__ out, uint32_t* __restrict__ total) {
    const uint64_t base = (uint64_t)threadIdx.x * SC_ITEMS;
    uint32_t loc[SC_ITEMS];
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < SC_ITEMS; ++k) {
        const uint64_t i = base + k;
        loc[k] = i < n ? in[i] : 0;
        s += loc[k];
    }
    uint32_t tot;
    uint32_t ex = block_excl_scan(s, &tot);  // (its barriers: every item is read before any is written, in == out)
#pragma unroll
    for (int k = 0; k < SC_ITEMS; ++k) {
        const uint64_t i = base + k;
        if (i < n) out[i] = ex;
        ex += loc[k];
    }
    if (threadIdx.x == 0 && total) *total = tot;
}
hipError_t launch_scan(const uint32_t* in, uint32_t* out, uint64_t n, uint32_t* part, uint32_t* total,
                       hipStream_t st) {
    if (n <= SC_TILE) {
        hipLaunchKernelGGL(k_scan_one, dim3(1), dim3(SC_THREADS), 0, st, in, n, out, total);
        return hipGetLastError();
    }
    uint32_t nb = (uint32_t)((n + SC_TILE - 1) / SC_TILE);
    if (nb == 0) nb = 1;
    hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(SC_THREADS), 0, st, in, n, part, (const uint32_t*)nullptr);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SC_THREADS), 0, st, part, nb, total);
    hipLaunchKernelGGL(k_scan_down, dim3(nb), dim3(SC_THREADS), 0, st, in, n, part, out, (const uint32_t*)nullptr);
    return hipGetLastError();
}
// the same over the first min(n, *ndev) elements only (a count known on the device; the rest of out is untouched)
hipError_t launch_scan_n(const uint32_t* in, uint32_t* out, uint64_t n, const uint32_t* ndev, uint32_t* part,
                         uint32_t* total, hipStream_t st) {
    uint32_t nb = (uint32_t)((n + SC_TILE - 1) / SC_TILE);
    if (nb == 0) nb = 1;
    hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(SC_THREADS), 0, st, in, n, part, ndev);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SC_THREADS), 0, st, part, nb, total);
    hipLaunchKernelGGL(k_scan_down, dim3(nb), dim3(SC_THREADS), 0, st, in, n, part, out, ndev);
    return hipGetLastError();
}

hipError_t launch_snapshot(Bkt* minb, NodeInfo* info, uint32_t nres, int64_t now, int32_t max_rt, uint32_t* cnt,
                           uint32_t* off, uint32_t* part, uint32_t* total, sg_metric_node* outp, uint64_t cap,
                           hipStream_t st) {
    uint32_t nb = (nres + 255) / 256;
    hipLaunchKernelGGL(k_snap_count, dim3(nb), dim3(256), 0, st, minb, info, nres, now, max_rt, cnt);
    hipError_t e = launch_scan(cnt, off, nres, part, total, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_snap_emit, dim3(nb), dim3(256), 0, st, minb, info, nres, now, off, outp, cap);
    return hipGetLastError();
}

} // namespace sg
