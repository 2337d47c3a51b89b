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
                                                           uint32_t* __restrict__ pos_of, const uint32_t* __restrict__ ndev) {
    constexpr int NB = 1 << DB;
    if (ndev && *ndev < n) n = *ndev;
    if ((uint64_t)blockIdx.x * RS_TILE >= n) return;  // (a tile past the device count: nothing to move)
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
        const uint64_t dst = (uint64_t)(gdst[(k >> shift) & (NB - 1)] + (int64_t)p);
        keys_out[dst] = k;
        vals_out[dst] = v;
        if (pos_of) pos_of[v & 0x7FFFFFFFu] = (uint32_t)dst | (v & 0x80000000u);
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

__global__ __launch_bounds__(SC_THREADS) void k_scan_reduce(const uint32_t* __restrict__ in, uint64_t n, uint32_t* __restrict__ part) {
    uint64_t base = (uint64_t)blockIdx.x * SC_TILE;
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
                                                       uint32_t* __restrict__ out) {
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
                       kout, vout, (uint32_t*)nullptr, ndev);
    return hipGetLastError();
}
hipError_t launch_radix_scatter(const uint32_t* kin, const uint32_t* vin, uint64_t n, int shift, const uint32_t* goff,
                                uint32_t nblocks, uint32_t* kout, uint32_t* vout, uint32_t* pos_of, hipStream_t st) {
    hipLaunchKernelGGL(k_radix_scatter<8>, dim3(nblocks), dim3(RS_THREADS), 0, st, kin, vin, n, shift, goff, nblocks,
                       kout, vout, pos_of, (const uint32_t*)nullptr);
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
hipError_t launch_scan(const uint32_t* in, uint32_t* out, uint64_t n, uint32_t* part, uint32_t* total,
                       hipStream_t st) {
    uint32_t nb = (uint32_t)((n + SC_TILE - 1) / SC_TILE);
    if (nb == 0) nb = 1;
    hipLaunchKernelGGL(k_scan_reduce, dim3(nb), dim3(SC_THREADS), 0, st, in, n, part);
    hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SC_THREADS), 0, st, part, nb, total);
    hipLaunchKernelGGL(k_scan_down, dim3(nb), dim3(SC_THREADS), 0, st, in, n, part, out);
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
