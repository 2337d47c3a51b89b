// decide.hip -- per-batch decision kernels of the MI355X Sentinel engine.
//
// Pipeline position (engine.cpp sg_submit_async):
//   record build + sort (kernels.hip k_rs_first, k_radix_*) -> k_seg_* (segments + bins) ->
//   k_scatter_rec + k_block_sums (16-byte sorted records, same-batch references mapped to sorted positions)
//   -> k_chain -> decide kernels by bin -> k_post (decisions back to submission order and into
//   the status ring).
//
// A segment is one resource's events of the batch, in event order.  Every resource's slot chain
// is a sequential state machine, so a segment is decided by exactly one owner:
//   * k_lane : one LANE per segment runs the chain event by event (chain.h) -- the Zipf tail,
//              every resource with param rules, and anything outside the cooperative limits;
//   * k_jac  : one wavefront / 256-lane / 1024-lane workgroup per segment (Zipf body and head).
//              Lanes take consecutive events and decide them speculatively: each lane evaluates
//              the chain against the state it would see if every earlier lane had the outcome
//              currently guessed for it (block-wide prefix sums of the counter deltas, max-plus
//              scans for rate limiters, a segmented scan for the RT breaker's passCount).  The
//              first lane whose evaluated outcome differs from its guess is exact, so everything
//              up to it commits; later lanes are re-guessed with their evaluated outcomes
//              (Jacobi iteration).  In the steady states of a hot resource (all pass, or all
//              blocked once its quota is spent) one iteration commits the whole tile.
//              A round never crosses a 500 ms bucket or a breaker reset, so bucket rotation,
//              WarmUp token sync and the ResetTask stay serial points handled by one leader lane.
// No MFMA: nothing here is a dense contraction; the kernels are bound by latency of the
// per-resource dependency chain and by HBM traffic of the event stream.
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <stdint.h>

#include "chain.h"
#include "aux.h"
#include "pmap.h"

using namespace sg;

#define WAVE 64
#define MAXR 16          // rules per resource (engine.cpp enforces)
#define JMAX_FLOW 4      // cooperative kernels: flow stages
#define JMAX_DEG 4       //                      degrade stages
#define JMAX_RL 2        //                      rate-limiter stages

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }
__device__ __forceinline__ uint64_t lanemask_lt() {
    uint32_t l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// =================================================================================
// segments: starts, lengths, bins, bin-ordered dispatch list
// =================================================================================
// Segment detection: a tile of 4096 sorted keys per workgroup, 16 consecutive keys per lane (4 x 16-byte loads);
// k_seg_count writes the tile's segment-start count, a scan over tiles gives the offsets, and
// k_seg_emit recounts and writes each Seg at its offset.  Reads the keys twice instead of
// writing and re-reading an n-wide flag and position array.
#define J8_MAX (1u << 23)  // longest segment of a QPS-DefaultController program on the 512-lane owner
#define SEG_ITEMS 16
#define SEG_TILE (256 * SEG_ITEMS)
// (keys[lo, n) only: lo = the hot / cold group stage's cold region, whose first key starts a segment)
__device__ __forceinline__ uint32_t seg_flags16(const uint32_t* __restrict__ keys, uint64_t n, uint64_t i0,
                                                uint32_t* kout, uint64_t lo = 0) {
    uint32_t f = 0;
    if (i0 >= n || i0 + SEG_ITEMS <= lo) return 0;
    uint32_t prev = i0 <= lo ? 0xFFFFFFFFu : keys[i0 - 1];
    if (i0 + SEG_ITEMS <= n) {
        const uint4* v = reinterpret_cast<const uint4*>(keys + i0);
#pragma unroll
        for (int q = 0; q < SEG_ITEMS / 4; ++q) {
            const uint4 w = v[q];
            kout[4 * q] = w.x; kout[4 * q + 1] = w.y; kout[4 * q + 2] = w.z; kout[4 * q + 3] = w.w;
        }
    } else {
#pragma unroll
        for (int j = 0; j < SEG_ITEMS; ++j) kout[j] = (i0 + j < n) ? keys[i0 + j] : 0u;
    }
#pragma unroll
    for (int j = 0; j < SEG_ITEMS; ++j) {
        const bool valid = i0 + j < n && i0 + j >= lo;
        const bool st = valid && (i0 + j == lo || kout[j] != prev);
        f |= (st ? 1u : 0u) << j;
        prev = valid ? kout[j] : 0xFFFFFFFFu;
    }
    return f;
}
__device__ __forceinline__ uint32_t seg_block_excl_scan(uint32_t v, uint32_t* total) {
    __shared__ uint32_t ws[4];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (l >= o) x += y;
    }
    if (l == 63) ws[w] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) { if (k < w) pre += ws[k]; tot += ws[k]; }
    *total = tot;
    return pre + x - v;
}
// lo (optional, on the device): the first position of the keys (the cold region); sbase (optional): segments written
// from segs[*sbase] on (after the hot ones)
__global__ __launch_bounds__(256) void k_seg_count(const uint32_t* __restrict__ keys, uint64_t n, uint32_t* __restrict__ cnt,
                                                   const uint32_t* __restrict__ lo) {
    const uint64_t b = lo ? *lo : 0u;
    if ((uint64_t)(blockIdx.x + 1) * SEG_TILE <= b) {  // a tile wholly before the region
        if (threadIdx.x == 0) cnt[blockIdx.x] = 0;
        return;
    }
    uint32_t kk[SEG_ITEMS];
    const uint64_t i0 = (uint64_t)blockIdx.x * SEG_TILE + (uint64_t)threadIdx.x * SEG_ITEMS;
    const uint32_t f = seg_flags16(keys, n, i0, kk, b);
    uint32_t tot;
    (void)seg_block_excl_scan((uint32_t)__popc(f), &tot);
    if (threadIdx.x == 0) cnt[blockIdx.x] = tot;
}
__global__ __launch_bounds__(256) void k_seg_emit(const uint32_t* __restrict__ keys, uint64_t n,
                                                  const uint32_t* __restrict__ off, Seg* __restrict__ segs,
                                                  const uint32_t* __restrict__ lo, const uint32_t* __restrict__ sbase) {
    const uint64_t b = lo ? *lo : 0u;
    if ((uint64_t)(blockIdx.x + 1) * SEG_TILE <= b) return;
    uint32_t kk[SEG_ITEMS];
    const uint64_t i0 = (uint64_t)blockIdx.x * SEG_TILE + (uint64_t)threadIdx.x * SEG_ITEMS;
    uint32_t f = seg_flags16(keys, n, i0, kk, b);
    uint32_t tot;
    uint32_t pos = (sbase ? *sbase : 0u) + off[blockIdx.x] + seg_block_excl_scan((uint32_t)__popc(f), &tot);
#pragma unroll
    for (int j = 0; j < SEG_ITEMS; ++j) {
        if ((f >> j) & 1u) {
            Seg sg;
            sg.res = kk[j];
            sg.start = (uint32_t)(i0 + j);
            sg.len = 0;
            sg.bin = 0;
            segs[pos++] = sg;
        }
    }
}
// lengths + bins.  Bins (dev_types.h BIN_*): cooperative kernels for long segments of resources
// inside their limits, one lane per segment for everything else.  Per-block bin counts go to
// blkcnt[bin][block] (a scan turns them into dispatch offsets); the rank inside the block rides
// in Seg.bin's upper bits until k_seg_order places the segment.
// Aux lists (sg_submit_ex batches; aux == null otherwise): the segments whose origin / context nodes the aux.hip
// post-pass updates -- short ones (aux[0] = count, list ashort), long ones (aux[3] = count, list along = seg << 32 |
// first piece; aux[1] = their pieces of AUX_PIECE events, expanded by k_aux_expand), and of those the segments of
// more than one piece, whose pieces' partial results are merged (aux[2] = count, list amulti = seg << 32 | first
// piece).
#define AUX_SHORT 256u
__device__ __forceinline__ uint32_t wave_alloc(uint32_t* ctr, uint32_t k) {  // one atomic per wave
    uint32_t x = k;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if ((int)(threadIdx.x & 63) >= o) x += y;
    }
    const uint32_t tot = __shfl(x, 63, 64);
    uint32_t base = 0;
    if ((threadIdx.x & 63) == 63 && tot) base = atomicAdd(ctr, tot);
    base = __shfl(base, 63, 64);
    return base + x - k;
}
__global__ __launch_bounds__(256) void k_seg_bin(Seg* __restrict__ segs, const uint32_t* __restrict__ mp, uint64_t n,
                                                 const Prog* __restrict__ prog, const uint32_t* __restrict__ prio,
                                                 uint32_t lane_max, uint32_t j1_max,
                                                 uint32_t j4_max, uint32_t force_lane, uint32_t* __restrict__ blkcnt,
                                                 uint32_t nblk, uint32_t pq_ok, uint32_t pq_wide, uint32_t* __restrict__ aux,
                                                 uint32_t* __restrict__ ashort, uint64_t* __restrict__ along,
                                                 uint64_t* __restrict__ amulti, uint32_t* __restrict__ mixc,
                                                 uint32_t* __restrict__ mix, uint32_t mix_cap,
                                                 uint32_t* __restrict__ mixlen, uint32_t mix_wide, uint32_t head_min) {
    __shared__ uint32_t cnt[N_BINS];
    for (uint32_t b = threadIdx.x; b < N_BINS; b += blockDim.x) cnt[b] = 0;
    __syncthreads();
    const uint32_t m = *mp;  // segment count (the grid covers an upper bound: no host round trip)
    const bool pq = pq_ok && !force_lane;
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    bool aux_short = false;
    uint32_t aux_np = 0;
    uint32_t mixk = 0;  // 1: an XF_MIX segment of a cooperative bin (narrow pre / post pass), 2: wide
    Seg sg;
    if (s < m) {
        sg = segs[s];
        const uint32_t end = (s + 1 < m) ? segs[s + 1].start : (uint32_t)n;
        sg.len = end - sg.start;
        const Prog p = prog[sg.res];
        const uint32_t pm = prio[sg.res];
        // decided one lane per segment whatever the length: a live borrow ring (PM_PRIO), events only k_lane takes
        // (PM_LANE), origin / context nodes the rules read (PX_ORIGIN / PX_CHAIN: k_lane<16> keeps them inline)
        const bool lane_only = (pm & (PM_PRIO | PM_LANE)) != 0 || ((pm & PM_AUX) && (p.multi & (PX_ORIGIN | PX_CHAIN)));
        const bool inline_aux = (pm & PM_AUX) && (lane_only || p.multi);  // k_lane<16> updates the nodes itself
        const int nr = p.multi ? 16 : p.n_param + p.n_flow + p.n_degrade;  // PX_*: decided with 16-rule lanes
        // XF_MIX: the param checks run in k_pq's pre pass (args[0] from the key ring: no argument lists)
        const bool mixp = (p.xf & XF_MIX) && pq && mix && !(pm & PM_ARGL);
        // single-rule THREAD-grade / rate-limiter heads (head.hip k_head) leave the lane bins from head_min events on
        const uint32_t cmin = (head_min && (p.xf & (XF_HEADT | XF_HEADR)) && head_min < lane_max) ? head_min : lane_max;
        const bool coop = !force_lane && !(p.pflags & PF_SERIAL) && (p.n_param == 0 || mixp) && sg.len > cmin &&
                          !lane_only && !p.multi;
        if (coop && p.n_param) mixk = sg.len > mix_wide ? 2u : 1u;  // (wide: pvalue.hip's passes, where on)
        if (mixk == 2 && mixlen) atomicAdd(mixlen, sg.len);  // (pvalue.hip's scratch bound)
        uint32_t bin;
        if (pq && (p.pflags & PF_PQ) && !lane_only && !(pm & PM_ARGL) && !((p.xf & XF_PTHREAD) && (pm & PM_XARGS))) {
            bin = sg.len > pq_wide ? BIN_PQ16 : BIN_PQ4;
            // its checks by the value-parallel passes (pvalue.hip), k_pq folding the statistics (long segments)
            if ((p.xf & XF_PVPQ) && mix && mix_wide == 0 && sg.len > lane_max) {
                mixk = 2;
                if (mixlen) atomicAdd(mixlen, sg.len);
            }
        }
        // QPS-DefaultController heads on the 512-lane owner (open stretches), up to J8_MAX events: a longer one (one
        // rank's batch of a strong-scaling run can hold a single resource's 33M events, nearly all in frozen
        // stretches) goes faster through the 1024-lane owner (8-way rehearsal: slowest rank 3.58 vs 2.64 ms)
        else if (coop) bin = (sg.len > j4_max && (p.pflags & PF_J16))
                                 ? (((p.pflags & PF_FROZEN) && sg.len <= J8_MAX) ? BIN_J8 : BIN_J16)
                                 : sg.len > j1_max ? BIN_J4 : BIN_J1;
        else {
            int lb = 31 - __clz(sg.len | 1);
            if (lb > (int)LANE_BINS - 1) lb = LANE_BINS - 1;
            // k_lite: no param rules, <= 2 DefaultController flow stages (QPS or thread), <= 2 breakers
            // (or one QPS DefaultController param rule on args[0] before them, scalar args: k_lite<true>), every
            // flow stage on the ClusterNode (PF_SERIAL: a rule of another strategy, e.g. one whose node is never
            // selected, FlowRuleChecker.selectReferenceNode, is k_lane's)
            const bool lite = (p.n_param == 0 || ((p.xf & XF_PLITE) && !(pm & PM_ARGL))) && !p.multi && !lane_only &&
                              (p.pflags & PF_J16) && !(p.pflags & (PF_WARM | PF_SERIAL));
            bin = (lite ? BIN_LITE : (nr <= 4 && !inline_aux) ? BIN_LANE : BIN_LANE16) + (LANE_BINS - 1 - lb);
        }
        // k_lane<16> keeps a PM_AUX resource's nodes inline; on every other owner the post-pass does
        const bool auxp = aux && (pm & PM_AUX) && !(bin >= BIN_LANE16 && bin < BIN_LANE16 + LANE_BINS);
        if (auxp) {
            if (sg.len <= AUX_SHORT) aux_short = true;
            else aux_np = (sg.len + AUX_PIECE - 1) / AUX_PIECE;
        }
        const uint32_t rank = atomicAdd(&cnt[bin], 1u);
        sg.bin = bin | (auxp ? SEG_AUXP : 0u) | (rank << 8);
        segs[s] = sg;
    }
    if (aux) {  // (wave-uniform: every lane of the wave takes part)
        const uint32_t o = wave_alloc(aux + 0, aux_short ? 1u : 0u);
        if (aux_short) ashort[o] = s;
        const uint32_t q = wave_alloc(aux + 1, aux_np);
        const uint32_t j = wave_alloc(aux + 3, aux_np ? 1u : 0u);
        if (aux_np) along[j] = ((uint64_t)s << 32) | q;
        const uint32_t u = wave_alloc(aux + 2, aux_np > 1 ? 1u : 0u);
        if (aux_np > 1) amulti[u] = ((uint64_t)s << 32) | q;
    }
    if (mix) {  // (wave-uniform)
        const uint32_t a = wave_alloc(mixc + 0, mixk == 1 ? 1u : 0u);
        if (mixk == 1) mix[a] = s;
        const uint32_t b = wave_alloc(mixc + 1, mixk == 2 ? 1u : 0u);
        if (mixk == 2) mix[mix_cap + b] = s;
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < N_BINS; b += blockDim.x) blkcnt[(uint64_t)b * nblk + blockIdx.x] = cnt[b];
}
// bin-major dispatch list: order[off[bin][block] + rank] = segment
__global__ __launch_bounds__(256) void k_seg_order(Seg* __restrict__ segs, const uint32_t* __restrict__ mp,
                                                   const uint32_t* __restrict__ off, uint32_t nblk,
                                                   uint32_t* __restrict__ order) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= *mp) return;
    const uint32_t v = segs[s].bin, bin = v & 0x7F;
    order[off[(uint64_t)bin * nblk + blockIdx.x] + (v >> 8)] = s;
    segs[s].bin = v & 0xFF;  // the bin | SEG_AUXP
}
// per-bin first offsets (+ total) for the host: out[b] = off[b][0], out[N_BINS] = m
__global__ void k_bin_offsets(const uint32_t* __restrict__ off, uint32_t nblk, const uint32_t* __restrict__ mp,
                              uint32_t* __restrict__ out) {
    const uint32_t b = threadIdx.x;
    if (b < N_BINS) out[b] = off[(uint64_t)b * nblk];
    if (b == N_BINS) out[b] = *mp;
}

// =================================================================================
// sorted records
// =================================================================================
// Sorted-order records: reads the submission-order records built by k_rs_first and the inverse
// permutation written by the last radix pass sequentially, maps same-batch references to the ENTRY's
// sorted position (bit 31 of pos_of = the referenced event is an ENTRY; a reference to a non-ENTRY
// resolves like an unknown entry: an EXIT is then the caller asserting the entry passed, a TRACE is not
// counted) and writes each record to its sorted position (random 16-byte writes; gathering through the
// permutation instead -- random 16-byte reads -- over-fetched whole lines, ~6 GB per C4 batch).  Side
// tables for frozen-stretch skipping (k_jac<..., SKIP>) come from one sequential pass over the sorted
// records (k_block_sums): per 1024 positions the ENTRY count sum plus a flag for EXIT/TRACEs that count
// without a same-batch link, and the forward link of every referenced ENTRY.
__global__ __launch_bounds__(256) void k_scatter_rec(const SEv* __restrict__ rec_o, uint64_t n,
                                                     const uint32_t* __restrict__ pos_of, SEv* __restrict__ recs,
                                                     uint32_t* __restrict__ prev, uint32_t* __restrict__ nprev,
                                                     Link* __restrict__ link, uint32_t* __restrict__ bst, uint32_t epoch,
                                                     uint32_t* __restrict__ bflags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    SEv r = rec_o[i];
    const uint32_t p = pos_of[i] & 0x7FFFFFFFu;
    if (r.code == RC_BATCH) {
        const uint32_t po = pos_of[r.x];
        if (po & 0x80000000u) r.x = po & 0x7FFFFFFFu;
        else r.code = r.kind == SG_EV_EXIT ? RC_NONE : RC_NOT;
    } else if (r.code == RC_PREV) {
        prev[atomicAdd(nprev, 1u)] = p;
    }
    if (r.kind == SG_EV_ENTRY) {
        if (r.cnt == 0) atomicOr(bflags, BF_ZERO_CNT);
    } else if (r.code == RC_NONE || r.code == RC_PREV) {
        atomicOr(&bst[p >> 10], BST_STATIC);
    }
    recs[p] = r;  // same-batch forward links are set by k_block_sums, in sorted order (local atomics)
}
// ENTRY count sum of every 1024 sorted positions (one workgroup each, 4 positions per lane), and the
// forward link of every same-batch referenced ENTRY: walked in sorted order, an EXIT/TRACE and its
// ENTRY sit in the same segment a few positions apart, so the link atomics and the key loads stay in
// cache.  The exchange returns the link's previous value: one of this batch's epoch means a second
// EXIT (or TRACE) named the same ENTRY (BF_MULTI_LINK: frozen-stretch skipping is off for the batch).
// A reference must also name an ENTRY of its own resource: the two carry the same sort key (inside a
// STRATEGY_RELATE component the key is the component's).
// skeys: the sorted keys of positions >= *lo (the hot / cold group stage's cold region: k_grp_records checked the
// references of hot events; lo = null: every position, the radix group stage)
__global__ __launch_bounds__(256) void k_block_sums(const SEv* __restrict__ recs, const uint32_t* __restrict__ skeys,
                                                    uint64_t n, uint32_t* __restrict__ bst, Link* __restrict__ link,
                                                    uint32_t epoch, uint32_t* __restrict__ bflags,
                                                    const uint32_t* __restrict__ lo) {
    const uint32_t kmin = lo ? *lo : 0u;
    if ((uint64_t)(blockIdx.x + 1) * 1024 <= kmin) return;  // (the hot region: k_grp_records)
    __shared__ uint32_t wsum[4];
    const uint64_t base = (uint64_t)blockIdx.x * 1024;
    // the four records as whole 16-byte loads (x = dt, y = x, z = cnt | rt << 16, w = kind | flags << 8 | code << 16),
    // then the four exchanges and the four key pairs issued together: one round trip each, not one per item
    uint4 w[4];
    bool in[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // (unconditional loads, clamped into the batch: no wait between them)
        const uint64_t p = base + (uint64_t)k * 256 + threadIdx.x;
        in[k] = p < n && p >= kmin;
        w[k] = reinterpret_cast<const uint4*>(recs)[p < n ? p : n - 1];
    }
    uint32_t v = 0;
    unsigned long long* xd[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t kind = w[k].w & 0xFFu, code = (w[k].w >> 16) & 0xFFu;
        if (in[k] && kind == SG_EV_ENTRY) v += w[k].z & 0xFFFFu;
        xd[k] = nullptr;
        if (in[k] && kind != SG_EV_ENTRY && code == RC_BATCH)
            xd[k] = reinterpret_cast<unsigned long long*>(kind == SG_EV_EXIT ? &link[w[k].y].exit_l : &link[w[k].y].trace_l);
    }
    auto xch = [&](int k) -> uint32_t {
        const uint64_t p = base + (uint64_t)k * 256 + threadIdx.x;
        return xd[k] ? (uint32_t)(atomicExch(xd[k], ((unsigned long long)epoch << 32) | (uint32_t)p) >> 32) : 0u;
    };
    const uint32_t o0 = xch(0), o1 = xch(1), o2 = xch(2), o3 = xch(3);
    // a cold reference to a cold ENTRY: the same sort key (both keys loaded for every item, clamped)
    uint32_t ka[4], kb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t p = base + (uint64_t)k * 256 + threadIdx.x;
        ka[k] = skeys[p < n ? p : n - 1];
        kb[k] = skeys[w[k].y < n ? w[k].y : n - 1];
    }
    bool bad = false;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (xd[k] && w[k].y >= kmin && ka[k] != kb[k]) bad = true;
    const bool multi = o0 == epoch || o1 == epoch || o2 == epoch || o3 == epoch;  // (epochs start at 1)
    if (__ballot(multi) && (threadIdx.x & 63) == 0) atomicOr(bflags, BF_MULTI_LINK);
    if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(bflags, BF_BAD_REF);
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
    if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t sum = wsum[0] + wsum[1] + wsum[2] + wsum[3];
        if (sum) atomicAdd(&bst[blockIdx.x], sum);
    }
}
// references into earlier batches, once those are decided: the ENTRY's status from the ring
// (0xFF = not an ENTRY: an EXIT is then taken as the caller asserting the entry passed)
// (sg_submit_ex: the record's x becomes the event's own origin / context node tag, as for an EXIT naming no ENTRY)
__global__ void k_resolve(const uint32_t* __restrict__ prev, uint32_t np, const uint8_t* __restrict__ ring,
                          SEv* __restrict__ recs, const uint32_t* __restrict__ vals, const sg_event_ext* __restrict__ ext) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np) return;
    const uint32_t p = prev[i];
    SEv r = recs[p];
    const uint8_t st = ring[r.x];
    if (st == ST_NOT_ENTRY) r.code = r.kind == SG_EV_EXIT ? RC_NONE : RC_NOT;
    else r.code = (st == ST_PASS || st == ST_PASS_WAIT) ? RC_PASSED : RC_NOT;
    r.x = 0;
    if (ext) {
        const sg_event_ext x = ext[vals[p] & 0x7FFFFFFFu];
        if (!(x.origin_id >> TAG_ORIGIN_BITS)) r.x = x.origin_id | (x.context_id << TAG_ORIGIN_BITS);
    }
    recs[p] = r;
}

// decisions back to submission order; the status ring keeps every event's status for
// references from later batches (0xFF = not an ENTRY)
// (POST_ITEMS items per lane, all random loads issued before any use: more of them in flight).  Only
// ENTRYs are gathered (bit 31 of pos_of): every other event's word is mk_dec(ST_NOT_ENTRY, 0, 0), which
// the decide kernels need not store.
#define POST_ITEMS 4
__global__ __launch_bounds__(256) void k_post(const uint32_t* __restrict__ pos_of, const uint32_t* __restrict__ dec,
                                              uint64_t n, uint64_t gbase, uint8_t* __restrict__ ring, uint64_t ring_mask,
                                              uint32_t* __restrict__ out) {
    const uint64_t base = (uint64_t)blockIdx.x * (256 * POST_ITEMS) + threadIdx.x;
    uint32_t po[POST_ITEMS], d[POST_ITEMS];
#pragma unroll
    for (int k = 0; k < POST_ITEMS; ++k) {
        const uint64_t i = base + (uint64_t)k * 256;
        po[k] = i < n ? pos_of[i] : 0u;
    }
#pragma unroll
    for (int k = 0; k < POST_ITEMS; ++k)
        d[k] = (po[k] & 0x80000000u) ? dec[po[k] & 0x7FFFFFFFu] : mk_dec(ST_NOT_ENTRY, 0, 0);
#pragma unroll
    for (int k = 0; k < POST_ITEMS; ++k) {
        const uint64_t i = base + (uint64_t)k * 256;
        if (i < n) {
            out[i] = d[k];
            ring[(gbase + i) & ring_mask] = (uint8_t)(d[k] & 0xFF);
        }
    }
}

// Verdicts of the frozen spans recorded by k_jac<..., SKIP> (the map half of a frozen stretch, spread
// over the whole chip): every ENTRY blocks exactly as in k_jac's streaming frozen path.
__global__ __launch_bounds__(256) void k_fill(const Span* __restrict__ spans, const uint32_t* __restrict__ nspan,
                                              uint32_t cap, const SEv* __restrict__ recs, const Prog* __restrict__ prog,
                                              const DRule* __restrict__ rules, uint32_t* __restrict__ dec) {
    const uint32_t ns = *nspan < cap ? *nspan : cap;
    for (uint32_t k = blockIdx.x; k < ns; k += gridDim.x) {
        const Span sp = spans[k];
        if (sp.e <= sp.s) continue;
        const uint32_t res = sp.res & 0x7FFFFFFFu;
        const bool cut = (sp.res >> 31) != 0;
        const Prog pg = prog[res];
        const int nf = pg.n_flow < 4 ? pg.n_flow : 4;
        const uint32_t fo = pg.rule_off + pg.n_param;  // the flow stages (XF_MIX: after the param rules)
        double fc[4];
        uint32_t fd[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            fc[s] = s < nf ? rules[fo + s].count : 0.0;
            fd[s] = s < nf ? mk_dec(ST_BLOCK_FLOW, rules[fo + s].slot, 0) : 0u;
        }
        const uint32_t cdec = (cut && pg.n_degrade) ? mk_dec(ST_BLOCK_DEGRADE, rules[fo + pg.n_flow].slot, 0) : 0u;
        for (uint32_t p = sp.s + threadIdx.x; p < sp.e; p += blockDim.x) {
            const uint4 r = reinterpret_cast<const uint4*>(recs)[p];
            uint32_t d = mk_dec(ST_NOT_ENTRY, 0, 0);
            if ((r.w & 0xFFu) == SG_EV_ENTRY) {
                if ((r.w >> 8) & RF_PBLK) continue;  // the param pre pass's verdict stands
                const double curv = (double)j_iadd(sp.pint, (int)(r.z & 0xFFFFu));
                uint32_t v = 0;
#pragma unroll
                for (int s = 3; s >= 0; --s)
                    if (s < nf && curv > fc[s]) v = fd[s];
                d = v ? v : cdec;
            }
            dec[p] = d;
        }
    }
}

// CtSph.lookProcessChain (core/CtSph.java:206-227): resources touched by this batch with neither a
// chain nor a rejection.  Unbounded cap: grant in place.  Bounded: emit (batch index of the first
// ENTRY, res) candidates for the host, which grants in first-ENTRY order up to the cap.
__global__ void k_chain(const SEv* __restrict__ recs, const uint32_t* __restrict__ vals, const Seg* __restrict__ segs,
                        uint32_t m, NodeInfo* __restrict__ info, uint32_t grant_all, uint32_t* __restrict__ ncand,
                        uint64_t* __restrict__ cand, const sg_event* __restrict__ ev, const Prog* __restrict__ prog,
                        const sg_event_ext* __restrict__ ext, uint32_t max_ctx) {
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= m) return;
    Seg sg = segs[s];
    // an ENTRY in a NullContext never looks its chain up (CtSph.entryWithPriority, CtSph.java:120-127)
    auto looks_up = [&](uint32_t j) {
        return recs[sg.start + j].kind == SG_EV_ENTRY &&
               (!ext || ext[vals[sg.start + j] & 0x7FFFFFFFu].context_id <= max_ctx);
    };
    if (prog[sg.res].multi & PX_MULTI) {  // a STRATEGY_RELATE component: every member's first ENTRY
        for (uint32_t j = 0; j < sg.len; ++j) {
            if (!looks_up(j)) continue;
            const uint32_t vi = vals[sg.start + j] & 0x7FFFFFFFu;
            const uint32_t res = ev[vi].res_id;
            const uint32_t fr = info[res].flags;
            if (fr & (NI_CHAIN | NI_REJECTED)) continue;
            if (grant_all) info[res].flags = fr | NI_CHAIN;
            else cand[atomicAdd(ncand, 1u)] = ((uint64_t)vi << 32) | res;  // the host keeps the first per resource
        }
        return;
    }
    uint32_t f = info[sg.res].flags;
    if (f & (NI_CHAIN | NI_REJECTED)) return;
    for (uint32_t j = 0; j < sg.len; ++j) {
        if (looks_up(j)) {
            if (grant_all) info[sg.res].flags = f | NI_CHAIN;
            else cand[atomicAdd(ncand, 1u)] = ((uint64_t)(vals[sg.start + j] & 0x7FFFFFFFu) << 32) | sg.res;
            return;
        }
    }
}

// =================================================================================
// ParameterMetric's bounded LRU maps (pmap.h).  Every operation below is the CacheMap call the reference makes,
// with ConcurrentLinkedHashMap's access order: get / putIfAbsent of a present key move it to the MRU end, an
// insert into a full map evicts the LRU entry.  A map is private to its resource's owner.
// =================================================================================
__device__ int32_t hot_count(const DevState& S, const DRule& r, uint64_t v, bool* found) {
    for (uint32_t i = 0; i < r.hot_n; ++i) {
        DHot h = S.hot[r.hot_off + i];
        if (h.key == v) { *found = true; return h.count; }
    }
    *found = false;
    return 0;
}
// pm_put (pmap.h) with its memory rounds overlapped, for the lane path: both candidate buckets' keys and stamps
// in one round, the stamp's ring word and the slot's values in the next, ring bits of a hit changed by atomics
// nobody waits for (the lane owns the map: only the order of its own accesses matters).  Same map state and
// result as pm_put; *d = the slot's values before the access (zero for an inserted key).
__device__ int32_t pm_put_lane(PMap& m, const PRef& R, uint64_t v, bool* present, PData* d, uint32_t* bflags) {
    pm_reserve(m, R, 1);
    uint32_t b1, b2;
    pm_buckets(m.nb, v, b1, b2);
    const PBucket B1 = R.B[b1], B2 = R.B[b2];
    int32_t i = -1;
    int64_t st = 0;
#pragma unroll
    for (int j = PM_BKT - 1; j >= 0; --j) if (B2.key[j] == v) { i = (int32_t)(b2 * PM_BKT + j); st = B2.stamp[j]; }
#pragma unroll
    for (int j = PM_BKT - 1; j >= 0; --j) if (B1.key[j] == v) { i = (int32_t)(b1 * PM_BKT + j); st = B1.stamp[j]; }
    const uint64_t RM = (uint64_t)pm_rbits(m) - 1;
    if (i >= 0) {
        const uint64_t p = (uint64_t)st & RM;
        const uint64_t wd = R.bm[p >> 6];
        const PData dd = R.D[i];
        if (st >= m.thr && st < m.clock && ((wd >> (p & 63)) & 1ull)) {
            atomicAnd(reinterpret_cast<unsigned long long*>(&R.bm[p >> 6]), ~(1ull << (p & 63)));
            const int64_t s = m.clock++;
            const uint64_t q = (uint64_t)s & RM;
            atomicOr(reinterpret_cast<unsigned long long*>(&R.bm[q >> 6]), 1ull << (q & 63));
            R.B[i / PM_BKT].stamp[i % PM_BKT] = s;
            *present = true;
            *d = dd;
            return i;
        }
    }
    *present = false;
    PData z;
    z.v0 = 0; z.v1 = 0; z.pad = 0;
    *d = z;
    if (m.live >= m.cap) pm_evict_oldest(m, R);
    m.live++;
    if (i >= 0) {  // the key's own dead slot
        pm_restamp(m, R, i, false);
        R.D[i] = z;
        return i;
    }
    // a free slot (empty, or dead by the ring) of the bucket with fewer live keys: pm_insert_new's choice, the
    // ring words of both buckets' stamps loaded together
    int f1 = -1, f2 = -1, n1 = 0, n2 = 0;
#pragma unroll
    for (int j = 0; j < PM_BKT; ++j) {
        const bool fr1 = B1.key[j] == PK_EMPTY || !pm_live(m, R.bm, B1.stamp[j]);
        const bool fr2 = B2.key[j] == PK_EMPTY || !pm_live(m, R.bm, B2.stamp[j]);
        if (fr1) { if (f1 < 0) f1 = j; } else ++n1;
        if (fr2) { if (f2 < 0) f2 = j; } else ++n2;
    }
    const bool u1 = f1 >= 0 && (f2 < 0 || n1 <= n2);
    if (!u1 && f2 < 0) return pm_insert_new(m, R, v, bflags);  // both full: the displacement walk
    const uint32_t b = u1 ? b1 : b2;
    const int j = u1 ? f1 : f2;
    const int64_t s = m.clock++;
    const uint64_t q = (uint64_t)s & RM;
    atomicOr(reinterpret_cast<unsigned long long*>(&R.bm[q >> 6]), 1ull << (q & 63));
    R.B[b].key[j] = v;
    R.B[b].stamp[j] = s;
    R.D[b * PM_BKT + j] = z;
    return (int32_t)(b * PM_BKT + j);
}
__device__ __forceinline__ uint32_t tmap_of(const DevState& S, uint32_t tm_base, uint32_t idx) {
    return tm_base == NO_ID || idx >= SG_MAX_ARGS ? NO_ID : S.tmid[tm_base + idx];
}
// ParameterMetric.getThreadCount (ParameterMetric.java:233-241): cacheMap.get(value)
__device__ int64_t thread_count_get(const DevState& S, uint32_t tm_base, uint32_t idx, uint64_t v) {
    const uint32_t id = tmap_of(S, tm_base, idx);
    if (id == NO_ID) return 0;
    PMap m = S.pmap[id];
    const PRef R = pm_ref(S, m);
    const int32_t i = pm_get(m, R, v);
    pm_store(S, id, m);
    return i < 0 ? 0 : R.D[i].v0;
}
// addThreadCount / decreaseThreadCount of one value (ParameterMetric.java:117-231):
//   add: putIfAbsent(v, 0) then increment, or put(v, 1) when it was absent;
//   decrease: putIfAbsent(v, 0) -- an absent value stays at 0 -- else decrement, removed at <= 0
__device__ void thread_count_add(const DevState& S, uint32_t tm_base, uint32_t idx, uint64_t v, int64_t d,
                                 uint32_t* bflags) {
    const uint32_t id = tmap_of(S, tm_base, idx);
    if (id == NO_ID) return;
    PMap m = S.pmap[id];
    const PRef R = pm_ref(S, m);
    bool present;
    PData od;
    const int32_t i = pm_put_lane(m, R, v, &present, &od, bflags);
    if (!present) {
        R.D[i].v0 = d > 0 ? 1 : 0;
    } else {
        const int64_t c = od.v0 + (d > 0 ? 1 : -1);
        if (c <= 0 && d < 0) pm_erase(m, R, i);
        else R.D[i].v0 = c;
    }
    pm_store(S, id, m);
}
// ParamFlowChecker.passSingleValueCheck (ParamFlowChecker.java:101-119) of one value
__device__ bool param_check(const DevState& S, uint32_t tm_base, const DRule& r, uint32_t idx, int acquire, uint64_t v,
                            int64_t t, int64_t& wait, uint32_t* bflags) {
    if (r.grade == SG_FLOW_GRADE_QPS) {
        bool hf;
        int32_t hc = hot_count(S, r, v, &hf);
        if (r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER) {  // passThrottleLocalCheck (:198-248)
            int64_t token_count = hf ? (int64_t)hc : r.token_count_l;
            if (token_count == 0) return false;
            int64_t cost = j_round(1.0 * 1000 * acquire * (double)r.duration_sec / (double)token_count);
            PMap m = S.pmap[r.pmap];
            const PRef R = pm_ref(S, m);
            bool present;
            PData od;
            const int32_t i = pm_put_lane(m, R, v, &present, &od, bflags);  // timeRecorderMap.putIfAbsent(value, now)
            bool ok = true;
            if (!present) {
                R.D[i].v0 = t;
            } else {
                const int64_t last = od.v0;
                const int64_t expected = last + cost;
                if (expected <= t || expected - t < r.max_queue) {
                    const int64_t w = expected - t;
                    R.D[i].v0 = w > 0 ? expected : t;
                    if (w > 0) wait += w;
                } else {
                    ok = false;
                }
            }
            pm_store(S, r.pmap, m);
            return ok;
        }
        // passDefaultLocalCheck (:121-196)
        int32_t token_count = hf ? hc : r.token_count;
        if (token_count == 0) return false;
        int32_t max_count = j_iadd(token_count, r.burst);
        if (acquire > max_count) return false;
        PMap m = S.pmap[r.pmap];
        const PRef R = pm_ref(S, m);
        bool present;
        PData od;
        const int32_t i = pm_put_lane(m, R, v, &present, &od, bflags);  // timeCounters.putIfAbsent, then tokenCounters
        bool ok = true;
        if (!present) {
            PData d;
            d.v0 = t;
            d.v1 = j_iadd(max_count, -acquire);
            d.pad = 0;
            R.D[i] = d;
        } else {
            PData d = od;
            const int64_t pass_time = t - d.v0;
            if (pass_time > r.duration_sec * 1000) {
                int32_t to_add = (int32_t)((pass_time * token_count) / (r.duration_sec * 1000));
                int32_t sum = j_iadd(d.v1, to_add);
                int32_t nq = sum > max_count ? j_iadd(max_count, -acquire) : j_iadd(sum, -acquire);
                if (nq < 0) ok = false;
                else { d.v1 = nq; d.v0 = t; R.D[i] = d; }
            } else if (j_iadd(d.v1, -acquire) >= 0) {
                R.D[i].v1 = j_iadd(d.v1, -acquire);
            } else {
                ok = false;
            }
        }
        pm_store(S, r.pmap, m);
        return ok;
    } else if (r.grade == SG_FLOW_GRADE_THREAD) {
        int64_t tc = thread_count_get(S, tm_base, idx, v);
        bool hf;
        int32_t hc = hot_count(S, r, v, &hf);
        if (hf) return ++tc <= hc;
        int64_t threshold = j_d2l(r.count);
        return ++tc <= threshold;
    }
    return true;
}

// The lane path's common XF_MIX shape -- one QPS DefaultController param rule on args[0] beside the thread-count
// map of paramIdx 0 -- keeps both map headers in registers over the segment (the lane owns its resource's maps:
// no other lane reads them) instead of a header load and store per access.
struct PmLane {
    uint32_t mid, tid;  // the rule's map / the thread-count map of paramIdx 0 (NO_ID: not held)
    PMap mp, tm;
};
struct PmLaneRef {      // (k_lite<true>: the headers in LDS)
    uint32_t mid, tid;
    PMap &mp, &tm;
};
// param_check's passDefaultLocalCheck on the held rule map
__device__ __forceinline__ bool param_default_lane(const DevState& S, const DRule& r, PMap& m, int acquire, uint64_t v,
                                                   int64_t t, uint32_t* bflags) {
    bool hf;
    const int32_t hc = hot_count(S, r, v, &hf);
    const int32_t token_count = hf ? hc : r.token_count;
    if (token_count == 0) return false;
    const int32_t max_count = j_iadd(token_count, r.burst);
    if (acquire > max_count) return false;
    const PRef R = pm_ref(S, m);
    bool present;
    PData od;
    const int32_t i = pm_put_lane(m, R, v, &present, &od, bflags);
    if (!present) {
        PData d;
        d.v0 = t;
        d.v1 = j_iadd(max_count, -acquire);
        d.pad = 0;
        R.D[i] = d;
        return true;
    }
    PData d = od;
    const int64_t pass_time = t - d.v0;
    if (pass_time > r.duration_sec * 1000) {
        const int32_t to_add = (int32_t)((pass_time * token_count) / (r.duration_sec * 1000));
        const int32_t sum = j_iadd(d.v1, to_add);
        const int32_t nq = sum > max_count ? j_iadd(max_count, -acquire) : j_iadd(sum, -acquire);
        if (nq < 0) return false;
        d.v1 = nq; d.v0 = t;
        R.D[i] = d;
        return true;
    }
    if (j_iadd(d.v1, -acquire) >= 0) {
        R.D[i].v1 = j_iadd(d.v1, -acquire);
        return true;
    }
    return false;
}
// thread_count_add on the held thread-count map
__device__ __forceinline__ void thread_add_lane(const DevState& S, PMap& m, uint64_t v, int64_t d, uint32_t* bflags) {
    const PRef R = pm_ref(S, m);
    bool present;
    PData od;
    const int32_t i = pm_put_lane(m, R, v, &present, &od, bflags);
    if (!present) {
        R.D[i].v0 = d > 0 ? 1 : 0;
    } else {
        const int64_t c = od.v0 + (d > 0 ? 1 : -1);
        if (c <= 0 && d < 0) pm_erase(m, R, i);
        else R.D[i].v0 = c;
    }
}

// ---- the Context and args of one event (sg_submit_ex, include/sentinel_gpu.h sg_event_ext)
struct EvX {
    uint32_t origin, ctx;  // interned ids (0: no origin / sentinel_default_context)
    uint32_t n;            // args.length
    const sg_arg* a;       // args; null with n == 1: the single key k0 (SG_F_HAS_ARG, or a key-ring key)
    uint64_t k0;
};
__device__ __forceinline__ EvX evx_of(const DevState& S, uint32_t oi, uint32_t flags, uint64_t aux, bool entry) {
    EvX x;
    x.origin = 0; x.ctx = 0; x.n = 0; x.a = nullptr; x.k0 = aux;
    if (S.ext) {
        const sg_event_ext e = S.ext[oi];
        x.origin = e.origin_id;
        x.ctx = e.context_id;
        if (e.n_args) { x.n = e.n_args; x.a = S.args + e.arg_off; return x; }
    }
    if (entry && (flags & SG_F_HAS_ARG)) x.n = 1;
    return x;
}
__device__ __forceinline__ sg_arg evx_arg(const EvX& x, uint32_t i) {
    if (x.a) return x.a[i];
    sg_arg r;
    r.key = x.k0; r.kind = SG_ARG_SCALAR; r.len = 0;
    return r;
}
// ParameterMetric.addThreadCount / decreaseThreadCount (ParameterMetric.java:126-241): every index with a
// thread-count map; a null element of a Collection/array throws inside the try that wraps the whole loop,
// so the remaining elements and indices are skipped.
__device__ void thread_args(const DevState& S, uint32_t tm_base, uint32_t nflags, const EvX& x, int64_t d,
                            uint32_t* bflags) {
    for (uint32_t i = 0; i < x.n && i < SG_MAX_ARGS; ++i) {
        if (!(nflags & ni_tm(i))) continue;
        const sg_arg v = evx_arg(x, i);
        if (v.kind == SG_ARG_LIST) {
            for (uint32_t k = 0; k < v.len; ++k) {
                const sg_arg el = S.args[v.key + k];
                if (el.kind != SG_ARG_SCALAR) return;
                thread_count_add(S, tm_base, i, el.key, d, bflags);
            }
        } else if (v.kind == SG_ARG_SCALAR) {
            thread_count_add(S, tm_base, i, v.key, d, bflags);
        }
    }
}
// the same with the thread-count map of paramIdx 0 held by the lane (L->tid)
__device__ __forceinline__ void thread_args_l(const DevState& S, uint32_t tm_base, uint32_t nflags, const EvX& x,
                                              int64_t d, uint32_t* bflags, PmLane* L) {
    if (!L || L->tid == NO_ID) { thread_args(S, tm_base, nflags, x, d, bflags); return; }
    for (uint32_t i = 0; i < x.n && i < SG_MAX_ARGS; ++i) {
        if (!(nflags & ni_tm(i))) continue;
        const sg_arg v = evx_arg(x, i);
        if (v.kind == SG_ARG_LIST) {
            for (uint32_t k = 0; k < v.len; ++k) {
                const sg_arg el = S.args[v.key + k];
                if (el.kind != SG_ARG_SCALAR) return;
                if (i == 0) thread_add_lane(S, L->tm, el.key, d, bflags);
                else thread_count_add(S, tm_base, i, el.key, d, bflags);
            }
        } else if (v.kind == SG_ARG_SCALAR) {
            if (i == 0) thread_add_lane(S, L->tm, v.key, d, bflags);
            else thread_count_add(S, tm_base, i, v.key, d, bflags);
        }
    }
}

// ---- origin StatisticNodes / context DefaultNodes kept inline by k_lane<16> (aux.h; the other owners' by aux.hip)
// NodeSelectorSlot keeps a DefaultNode per (context, resource) for every entry (NodeSelectorSlot.java:134-176);
// the device keeps those of named contexts always, and that of the default context while a CHAIN rule of the
// resource names it (a CHAIN rule on sentinel_default_context starts from a fresh node)
__device__ __forceinline__ bool chain_ctx_kept(const DRule* flows, int nf, uint32_t ctx) {
    if (ctx != 0) return true;
    for (int k = 0; k < nf; ++k)
        if (flows[k].strategy == SG_STRATEGY_CHAIN && flows[k].chain_ctx == ctx) return true;
    return false;
}
// StatisticSlot bookkeeping on an origin node / DefaultNode: 0 = block, 1 = pass, 2 = PriorityWait (thread only),
// 3 = exit (rt, success, thread)
__device__ void aux_stat(const DevState& S, const DevCfg& cfg, uint32_t res, uint32_t kind, uint32_t id, int what,
                         int64_t t, int cnt, int64_t rt, uint32_t* bflags) {
    AuxNode* a = aux_get(S, res, kind, id, bflags);
    if (!a) return;
    Node NA;
    node_load_aux(NA, a);
    if (what == 2) {
        NA.thread++;
    } else {
        const int sl = sec_current(NA, t, cfg.max_rt);
        if (what == 3) { sec_add(NA, sl, 0, 0, cnt, rt, 0, rt); NA.thread--; }
        else if (what == 1) { NA.thread++; sec_add(NA, sl, cnt, 0, 0, 0, 0, INT64_MAX); aux_add_mpass(a, t, cnt); }
        else sec_add(NA, sl, 0, cnt, 0, 0, 0, INT64_MAX);
    }
    node_store_aux(NA, a);
}

enum { SEL_NONE = 0, SEL_CLUSTER = 1, SEL_ORIGIN = 2, SEL_DEFAULT = 3, SEL_RELATE = 4 };
// FlowRuleChecker.selectNodeByRequesterAndStrategy / selectReferenceNode (FlowRuleChecker.java:67-124)
// "other" also excludes the limitApps of the resource's cluster-only rules, which compile to no check (their
// origin ids ride in the rule's hot list, engine.cpp upload_rules)
__device__ __forceinline__ int flow_select(const DRule& r, const EvX& x, const DRule* flows, int nf, const DHot* hot) {
    bool applies;
    if (r.la_kind == LA_DEFAULT) applies = true;
    else if (r.la_kind == LA_ORIGIN) applies = x.origin != 0 && x.origin == r.la_origin;
    else {  // "other": FlowRuleManager.isOtherOrigin (FlowRuleManager.java:106-125)
        applies = x.origin != 0;
        for (int k = 0; k < nf; ++k)
            if (flows[k].la_origin == x.origin) applies = false;
        for (uint32_t k = 0; k < r.hot_n; ++k)
            if ((uint32_t)hot[r.hot_off + k].key == x.origin) applies = false;
    }
    if (!applies) return SEL_NONE;
    if (r.strategy == SG_STRATEGY_RELATE) return r.ref == NO_REF ? SEL_CLUSTER : SEL_RELATE;
    if (r.strategy == SG_STRATEGY_CHAIN) return x.ctx == r.chain_ctx ? SEL_DEFAULT : SEL_NONE;
    if (r.strategy != SG_STRATEGY_DIRECT) return SEL_NONE;  // selectReferenceNode: no node for other strategies
    return r.la_kind == LA_DEFAULT ? SEL_CLUSTER : SEL_ORIGIN;
}

// =================================================================================
// k_lane: one lane per segment, event by event
// =================================================================================
// FlowRuleChecker.selectReferenceNode for STRATEGY_RELATE (FlowRuleChecker.java:67-88): the controller
// runs on the ClusterNode of ref (ClusterBuilderSlot.getClusterNode: null until an ENTRY of ref was
// processed with a chain -> pass), with its side effects on that node (currentWindow resets)
__device__ int relate_check(const DevState& S, const DevCfg& cfg, const DRule& r, RState& s, int64_t t, int cnt,
                            uint32_t fl, int64_t& wait) {
    const uint32_t b = r.ref;
    if (!(S.info[b].flags & NI_TOUCHED)) return 1;
    Node NB;
    node_load(NB, S, b);
    const Prog pb = S.prog[b];
    const Ctx CB{S.minb + (uint64_t)b * 60, cfg.max_rt, pb.pflags};
    int rc;
    if ((fl & SG_F_PRIORITIZED) && r.behavior == SG_CONTROL_BEHAVIOR_DEFAULT) {
        int64_t w = 0;
        rc = default_can_pass_prio(NB, CB, r, t, cnt, cfg.occupy_timeout, w);
        if (rc == 2) wait += w;
    } else {
        rc = flow_can_pass(NB, CB, r, s, t, cnt, wait) ? 1 : 0;
    }
    min_flush(NB, CB.minb);
    node_store(NB, S, b, pb.pflags);
    return rc;
}
// flow_can_pass (chain.h) on an origin node / DefaultNode: the minute window is the node's pass history (aux.h)
__device__ __forceinline__ bool aux_flow_can_pass(Node& N, AuxNode* a, const DRule& r, RState& s, int64_t t, int acquire,
                                                  int32_t max_rt, int64_t& wait) {
    switch (r.behavior) {
    case SG_CONTROL_BEHAVIOR_WARM_UP: {
        sec_current(N, t, max_rt);
        const int64_t pass_qps = SEC_SUM(N, t, pass);
        warm_sync(r, s, t, aux_prev_pass(a, t));
        const int64_t rest = s.a;
        if (rest >= r.warning_token) return (double)(pass_qps + acquire) <= warm_qps(r, rest);
        return (double)(pass_qps + acquire) <= r.count;
    }
    case SG_CONTROL_BEHAVIOR_RATE_LIMITER:
        if (acquire <= 0) return true;
        if (r.count <= 0) return false;
        return rl_admit(s.c, rl_cost(r, s, acquire), t, r.max_queue, wait);
    case SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER:
        warm_sync(r, s, t, aux_prev_pass(a, t));
        return rl_admit(s.c, rl_cost(r, s, acquire), t, r.max_queue, wait);
    default: {
        int32_t cur;
        if (r.grade == SG_FLOW_GRADE_THREAD) cur = N.thread;
        else { sec_current(N, t, max_rt); cur = j_d2i((double)SEC_SUM(N, t, pass)); }
        return !((double)j_iadd(cur, acquire) > r.count);
    }
    }
}
// default_can_pass_prio (chain.h) on an origin node / DefaultNode
__device__ __forceinline__ int aux_default_prio(Node& N, AuxNode* a, const DRule& r, int64_t t, int acquire,
                                                int32_t occupy_timeout, int32_t max_rt, int64_t& wait) {
    int32_t cur;
    if (r.grade == SG_FLOW_GRADE_THREAD) cur = N.thread;
    else { sec_current(N, t, max_rt); cur = j_d2i((double)SEC_SUM(N, t, pass)); }
    if (!((double)j_iadd(cur, acquire) > r.count)) return 1;
    if (r.grade != SG_FLOW_GRADE_QPS) return 0;
    const Ctx C{nullptr, max_rt, 0};  // tryOccupyNext reads the second window and the borrow ring only
    const int64_t w = try_occupy_next(N, C, t, acquire, r.count, occupy_timeout);
    if (w >= occupy_timeout) return 0;
    const int bs = bor_current(N.bor, t + w);  // addWaitingRequest
    if (bs >= 0) N.bor[2 * bs + 1] += acquire;
    a->flags |= AUXF_BORROW;
    aux_add_mpass(a, t, acquire);              // addOccupiedPass: minute PASS (and OCCUPIED_PASS, never read here)
    wait = w;
    return 2;
}
// the controller of one flow rule on an origin node / DefaultNode (1 pass, 0 block, 2 PriorityWait)
__device__ int aux_check(const DevState& S, const DevCfg& cfg, const DRule& r, RState& s, uint32_t res, uint32_t kind,
                         uint32_t id, int64_t t, int cnt, uint32_t fl, int64_t& wait, uint32_t* bflags) {
    AuxNode* a = aux_get(S, res, kind, id, bflags);
    if (!a) return 1;
    Node NA;
    node_load_aux(NA, a);
    int rc;
    if ((fl & SG_F_PRIORITIZED) && r.behavior == SG_CONTROL_BEHAVIOR_DEFAULT) {
        int64_t w = 0;
        rc = aux_default_prio(NA, a, r, t, cnt, cfg.occupy_timeout, cfg.max_rt, w);
        if (rc == 2) wait += w;
    } else {
        rc = aux_flow_can_pass(NA, a, r, s, t, cnt, cfg.max_rt, wait) ? 1 : 0;
    }
    node_store_aux(NA, a);
    return rc;
}

// One ENTRY through StatisticSlot -> ParamFlowSlot -> [caller's System/Authority] -> FlowSlot -> DegradeSlot
// (param/slots/HotParamSlotChainBuilder.java:38-51, StatisticSlot.entry StatisticSlot.java:54-133).
// rs[] is indexed only with unrolled constants, so for NRMAX <= 4 it stays in registers.  AUX: the
// resource keeps origin nodes / DefaultNodes (k_lane<16> only).
template <int NRMAX, bool MULTI = false>
__device__ __forceinline__ uint32_t lane_entry(Node& N, const Ctx& C, const DevState& S, const DevCfg& cfg,
                                               const Prog& pg, RState (&rs)[NRMAX], uint32_t res, int64_t t, int cnt,
                                               uint32_t fl, const EvX& x, uint32_t* bflags, PmLane* L = nullptr) {
    const DRule* rules = S.rules + pg.rule_off;
    const int np = pg.n_param, nfl = np + pg.n_flow, nr = nfl + pg.n_degrade;
    const bool aux = NRMAX >= 16;  // origin nodes / DefaultNodes (PM_AUX resources and PX_* rules are k_lane<16>'s)
    uint32_t status = ST_PASS, slot = 0;
    int64_t wait = 0;
#pragma unroll
    for (int s = 0; s < NRMAX; ++s) {
        if (s < nr && status == ST_PASS) {
            const DRule r = rules[s];
            if (s < np) {  // ParamFlowSlot.checkFlow (ParamFlowSlot.java:77-101)
                N.flags |= NI_PM;  // initHotParamMetricsFor -> ParameterMetric.initialize
                if (r.behavior == PB_INIT_ONLY && r.param_idx >= 0) {  // maps of a run of never-checked rules
                    N.flags |= (uint32_t)r.burst << NI_TM_SHIFT;
                    continue;
                }
                int idx = r.param_idx;
                if (idx < 0) {  // applyRealParamIdx mutates the rule once (RState.a = resolved index + 1)
                    if (rs[s].a == 0) rs[s].a = 1 + ((-idx <= (int)x.n) ? (int)x.n + idx : -idx);
                    idx = (int)rs[s].a - 1;
                }
                if (idx < SG_MAX_ARGS) N.flags |= ni_tm((uint32_t)idx);
                if (r.behavior == PB_INIT_ONLY || idx >= (int)x.n) continue;
                const sg_arg v = evx_arg(x, (uint32_t)idx);
                bool ok = true;
                int64_t w = 0;
                const bool held = L && L->mid == r.pmap;  // (a QPS DefaultController rule: no wait)
                if (v.kind == SG_ARG_LIST) {  // Collection / array: element by element (ParamFlowChecker.java:75-90)
                    for (uint32_t k = 0; k < v.len && ok; ++k) {
                        const sg_arg el = S.args[v.key + k];
                        if (el.kind != SG_ARG_SCALAR) break;  // a null element throws: passLocalCheck passes
                        ok = held ? param_default_lane(S, r, L->mp, cnt, el.key, t, bflags)
                                  : param_check(S, pg.tm_base, r, (uint32_t)idx, cnt, el.key, t, w, bflags);
                    }
                } else if (v.kind == SG_ARG_SCALAR) {
                    ok = held ? param_default_lane(S, r, L->mp, cnt, v.key, t, bflags)
                              : param_check(S, pg.tm_base, r, (uint32_t)idx, cnt, v.key, t, w, bflags);
                }
                if (!ok) { status = ST_BLOCK_PARAM; slot = r.slot; }
                else wait += w;
            } else if (s < nfl) {  // FlowSlot.checkFlow (FlowSlot.java:146-158)
                if (s == np && (fl & SG_F_BLOCKED_UPSTREAM)) { status = ST_BLOCK_UPSTREAM; slot = 0; continue; }
                const int sel = flow_select(r, x, rules + np, pg.n_flow, S.hot);
                if (sel == SEL_NONE) continue;
                int rc;
                int64_t w = 0;
                if (MULTI && sel == SEL_RELATE) rc = relate_check(S, cfg, r, rs[s], t, cnt, fl, w);
                else if (aux && (sel == SEL_ORIGIN || sel == SEL_DEFAULT))
                    rc = aux_check(S, cfg, r, rs[s], res, sel == SEL_ORIGIN ? AUX_ORIGIN : AUX_CONTEXT,
                                   sel == SEL_ORIGIN ? x.origin : x.ctx, t, cnt, fl, w, bflags);
                else if ((fl & SG_F_PRIORITIZED) && r.behavior == SG_CONTROL_BEHAVIOR_DEFAULT)
                    rc = default_can_pass_prio(N, C, r, t, cnt, cfg.occupy_timeout, w);
                else rc = flow_can_pass(N, C, r, rs[s], t, cnt, w) ? 1 : 0;
                if (rc == 0) { status = ST_BLOCK_FLOW; slot = r.slot; }
                else if (rc == 2) { status = ST_PASS_WAIT; slot = r.slot; wait += w; }  // PriorityWaitException
                else wait += w;
            } else {  // DegradeRuleManager.checkDegrade (DegradeRuleManager.java:72-85)
                if (!degrade_pass(N, C, deg_param(r), rs[s], t)) { status = ST_BLOCK_DEGRADE; slot = r.slot; }
            }
        }
    }
    if (status == ST_PASS && pg.n_flow == 0 && (fl & SG_F_BLOCKED_UPSTREAM)) { status = ST_BLOCK_UPSTREAM; slot = 0; }
    // StatisticSlot.entry (StatisticSlot.java:54-133): DefaultNode -> ClusterNode, origin node
    const int what = status == ST_PASS ? 1 : status == ST_PASS_WAIT ? 2 : 0;
    if (aux) {  // ClusterBuilderSlot's origin node, NodeSelectorSlot's DefaultNode: counted whatever the rules
        if (x.origin) aux_stat(S, cfg, res, AUX_ORIGIN, x.origin, what, t, cnt, 0, bflags);
        if (chain_ctx_kept(rules + np, pg.n_flow, x.ctx)) aux_stat(S, cfg, res, AUX_CONTEXT, x.ctx, what, t, cnt, 0, bflags);
    }
    if (status == ST_PASS_WAIT) {  // StatisticSlot.entry catch PriorityWaitException (StatisticSlot.java:82-96)
        N.thread++;
        if (N.flags & NI_PM) thread_args_l(S, pg.tm_base, N.flags, x, 1, bflags, L);
        return mk_dec(ST_PASS_WAIT, slot, wait);
    }
    const bool passed = status == ST_PASS;
    stat_entry(N, C, t, cnt, passed);
    // ParamFlowStatisticEntryCallback.onPass -> ParameterMetric.addThreadCount(args)
    if (passed && (N.flags & NI_PM)) thread_args_l(S, pg.tm_base, N.flags, x, 1, bflags, L);
    return passed ? mk_dec(ST_PASS, 0, wait) : mk_dec(status, slot, 0);
}

// StatisticSlot.exit of an effective EXIT (StatisticSlot.java:136-173) + ParamFlowStatisticExitCallback.onExit:
// Entry.exit(count, args) releases the thread counts of its args -- the EXIT's own args (sg_submit_ex), else
// args[0] of its ENTRY from the key ring
template <int NRMAX>
__device__ __forceinline__ void lane_exit(Node& N, const Ctx& C, const DevState& S, const DevCfg& cfg, const Prog& pg,
                                          uint32_t res, int64_t t, const SEv& r, const EvX& x, uint64_t ref,
                                          uint32_t* bflags, PmLane* L = nullptr) {
    stat_exit(N, C, t, r.cnt, r.rt);
    if (NRMAX >= 16) {  // the exit runs on the nodes its entry counted on (the same origin and context)
        const DRule* flows = S.rules + pg.rule_off + pg.n_param;
        if (x.origin) aux_stat(S, cfg, res, AUX_ORIGIN, x.origin, 3, t, r.cnt, r.rt, bflags);
        if (chain_ctx_kept(flows, pg.n_flow, x.ctx)) aux_stat(S, cfg, res, AUX_CONTEXT, x.ctx, 3, t, r.cnt, r.rt, bflags);
    }
    if (!(r.flags & SG_F_EXIT_ARGS) || !(N.flags & NI_PM)) return;
    if (x.n) { thread_args_l(S, pg.tm_base, N.flags, x, -1, bflags, L); return; }
    if (!S.key_ring || ref == SG_REF_NONE) return;
    const uint64_t key = S.key_ring[ref & cfg.ring_mask];
    if (key == NO_KEY) return;
    EvX k;
    k.origin = 0; k.ctx = 0; k.n = 1; k.a = nullptr; k.k0 = key;
    thread_args_l(S, pg.tm_base, N.flags, k, -1, bflags, L);
}

// A STRATEGY_RELATE component (one segment, members in event order): each event runs on its own
// resource's node, rules and states, loaded and stored per event -- the flow check of a member may
// read and rotate another member's ClusterNode in between.
template <int NRMAX>
__device__ void lane_multi(const SEv* __restrict__ recs, const sg_event* __restrict__ ev,
                           const uint32_t* __restrict__ vals, const Seg& sg, const DevState& S, const DevCfg& cfg,
                           int64_t t0, uint32_t* __restrict__ dec, uint32_t* __restrict__ bflags) {
    for (uint32_t j = 0; j < sg.len; ++j) {
        const SEv r = recs[sg.start + j];
        const uint32_t oi = vals[sg.start + j] & 0x7FFFFFFFu;
        const sg_event& E = ev[oi];
        const uint32_t res = E.res_id;
        const int64_t t = t0 + r.dt;
        const Prog pg = S.prog[res];
        const int nr = pg.n_param + pg.n_flow + pg.n_degrade;
        Node N;
        node_load(N, S, res);
        const Ctx C{S.minb + (uint64_t)res * 60, cfg.max_rt, pg.pflags};
        RState rs[NRMAX];
#pragma unroll
        for (int s = 0; s < NRMAX; ++s) if (s < nr) rs[s] = S.rstate[pg.rule_off + s];
        const EvX x = evx_of(S, oi, r.flags, E.aux, r.kind == SG_EV_ENTRY);
        const bool has_chain = (N.flags & NI_CHAIN) != 0 && x.ctx <= S.max_ctx;  // NullContext: no chain
        const bool chain = has_chain && cfg.switch_on;
        uint32_t d = mk_dec(ST_NOT_ENTRY, 0, 0);
        if (r.kind == SG_EV_ENTRY) {
            if (!chain) d = mk_dec(ST_NO_CHECK, 0, 0);
            else {
                N.flags |= NI_TOUCHED;  // ClusterBuilderSlot runs before the checks
                d = lane_entry<NRMAX, true>(N, C, S, cfg, pg, rs, res, t, r.cnt, r.flags, x, bflags);
            }
        } else {
            bool eff;
            if (r.code == RC_NONE) eff = r.kind == SG_EV_EXIT ? chain : has_chain;
            else if (r.code == RC_PASSED) eff = true;
            else if (r.code == RC_NOT) eff = false;
            else {
                const uint32_t rel = r.x - sg.start;
                if (rel >= j) { atomicOr(bflags, BF_BAD_REF); eff = false; }
                else eff = st_passed(dec[r.x] & 0xFF);  // written by this lane
            }
            if (eff) {
                if (r.kind == SG_EV_EXIT) {
                    const uint64_t ref = r.code == RC_NONE ? SG_REF_NONE
                                         : r.code == RC_BATCH ? S.gbase + (vals[r.x] & 0x7FFFFFFFu) : (E.aux & SG_REF_NONE);
                    lane_exit<NRMAX>(N, C, S, cfg, pg, res, t, r, x, ref, bflags);
                } else {
                    stat_trace(N, C, t, r.cnt);
                }
            }
        }
        dec[sg.start + j] = d;
        min_flush(N, C.minb);
        node_store(N, S, res, pg.pflags);
#pragma unroll
        for (int s = 0; s < NRMAX; ++s) if (s < nr) S.rstate[pg.rule_off + s] = rs[s];
    }
}

// one segment on one lane (k_lane; the tiny batches' single kernel, k_tiny)
template <int NRMAX>
__device__ __forceinline__ void lane_seg(const SEv* __restrict__ recs, const sg_event* __restrict__ ev,
                                         const uint32_t* __restrict__ vals, const Seg sg, const DevState& S,
                                         const DevCfg& cfg, int64_t t0, uint32_t* __restrict__ dec,
                                         uint32_t* __restrict__ bflags, uint32_t i) {
    const uint32_t res = sg.res;
    const Prog pg = S.prog[res];
    if (NRMAX >= 16 && (pg.multi & PX_MULTI)) {
        lane_multi<NRMAX>(recs, ev, vals, sg, S, cfg, t0, dec, bflags);
        return;
    }
    const int nr = pg.n_param + pg.n_flow + pg.n_degrade;
#ifdef SG_KPROF
    const bool kp = S.dbg && i == 0;  // the longest segment of the launch
    unsigned long long kt0 = kp ? __builtin_amdgcn_s_memtime() : 0, kta = 0, ktb = 0, ktc = 0;
#define LPROF(acc)                                                \
    if (kp) {                                                     \
        unsigned long long _n = __builtin_amdgcn_s_memtime();     \
        acc += _n - kt0;                                          \
        kt0 = _n;                                                 \
    }
#else
#define LPROF(acc)
#endif
    Node N;
    node_load(N, S, res);
    const Ctx C{S.minb + (uint64_t)res * 60, cfg.max_rt, pg.pflags};
    RState rs[NRMAX];
#pragma unroll
    for (int s = 0; s < NRMAX; ++s) if (s < nr) rs[s] = S.rstate[pg.rule_off + s];
    const bool has_chain_r = (N.flags & NI_CHAIN) != 0;
    PmLane L;  // the common XF_MIX shape's map headers, held over the segment (k_lane<4>)
    L.mid = L.tid = NO_ID;
    if (NRMAX <= 4 && pg.n_param) {
        if (pg.n_param == 1) {
            const DRule r0 = S.rules[pg.rule_off];
            if (r0.behavior == SG_CONTROL_BEHAVIOR_DEFAULT && r0.grade == SG_FLOW_GRADE_QPS && r0.param_idx == 0) {
                L.mid = r0.pmap;
                L.mp = S.pmap[L.mid];
            }
        }
        const uint32_t tm0 = tmap_of(S, pg.tm_base, 0);
        if (tm0 != NO_ID && L.mid != NO_ID) {  // (with a THREAD-grade rule n_param > 1: its reads stay in memory)
            L.tid = tm0;
            L.tm = S.pmap[tm0];
        }
    }
    PmLane* LP = NRMAX <= 4 ? &L : nullptr;
    if (sg.len && (t0 + recs[sg.start].dt) < (N.sb[0].ws > N.sb[1].ws ? N.sb[0].ws : N.sb[1].ws))
        atomicOr(bflags, BF_BACKWARD);  // Q3: the clock went back across batches
    uint64_t pm = 0;  // passed bits of the segment's first 64 positions
    SEv rn[2];        // software prefetch, two events ahead
    rn[0] = recs[sg.start];
    if (sg.len > 1) rn[1] = recs[sg.start + 1];
    // the caller's record is read only for an ENTRY's argument key or an EXIT(args) of an earlier batch's ENTRY:
    // its aux (a random load in submission order) is fetched one event ahead
    auto need_ev = [](const SEv& r) {
        return (r.kind == SG_EV_ENTRY && (r.flags & SG_F_HAS_ARG)) ||
               (r.kind == SG_EV_EXIT && r.code == RC_PASSED && (r.flags & SG_F_EXIT_ARGS));
    };
    uint32_t oin = vals[sg.start] & 0x7FFFFFFFu;
    uint64_t auxn = need_ev(rn[0]) ? ev[oin].aux : 0;
    LPROF(kta)
    for (uint32_t j = 0; j < sg.len; ++j) {
        const SEv r = rn[0];
        const uint32_t oi = oin;
        const uint64_t aux = auxn;
        rn[0] = rn[1];
        if (j + 2 < sg.len) rn[1] = recs[sg.start + j + 2];
        if (j + 1 < sg.len) {
            oin = vals[sg.start + j + 1] & 0x7FFFFFFFu;
            auxn = need_ev(rn[0]) ? ev[oin].aux : 0;
        }
        const int64_t t = t0 + r.dt;
        const EvX x = evx_of(S, oi, r.flags, aux, r.kind == SG_EV_ENTRY);
        const bool has_chain = has_chain_r && x.ctx <= S.max_ctx;  // NullContext: no chain, no statistics
        const bool chain = has_chain && cfg.switch_on;
        uint32_t d = mk_dec(ST_NOT_ENTRY, 0, 0);
        if (r.kind == SG_EV_ENTRY) {
            if (!chain) d = mk_dec(ST_NO_CHECK, 0, 0);
            else d = lane_entry<NRMAX>(N, C, S, cfg, pg, rs, res, t, r.cnt, r.flags, x, bflags, LP);
            if (j < 64 && st_passed(d & 0xFF)) pm |= 1ull << j;
            LPROF(ktb)
        } else {
            bool eff;
            if (r.code == RC_NONE) eff = r.kind == SG_EV_EXIT ? chain : has_chain;
            else if (r.code == RC_PASSED) eff = true;
            else if (r.code == RC_NOT) eff = false;
            else {
                uint32_t rel = r.x - sg.start;
                if (rel >= j) { atomicOr(bflags, BF_BAD_REF); eff = false; }  // not an earlier ENTRY of this resource
                else eff = rel < 64 ? ((pm >> rel) & 1) != 0 : st_passed(dec[r.x] & 0xFF);
            }
            if (eff) {
                if (r.kind == SG_EV_EXIT) {
                    const uint64_t ref = r.code == RC_NONE ? SG_REF_NONE
                                         : r.code == RC_BATCH ? S.gbase + (vals[r.x] & 0x7FFFFFFFu) : (aux & SG_REF_NONE);
                    lane_exit<NRMAX>(N, C, S, cfg, pg, res, t, r, x, ref, bflags, LP);
                } else {
                    stat_trace(N, C, t, r.cnt);
                }
            }
            LPROF(ktc)
        }
        if (r.kind == SG_EV_ENTRY) dec[sg.start + j] = d;  // k_post reads ENTRY words only
    }
    min_flush(N, C.minb);
    node_store(N, S, res, pg.pflags);
    if (L.mid != NO_ID) pm_store(S, L.mid, L.mp);
    if (L.tid != NO_ID) pm_store(S, L.tid, L.tm);
#pragma unroll
    for (int s = 0; s < NRMAX; ++s) if (s < nr) S.rstate[pg.rule_off + s] = rs[s];
#ifdef SG_KPROF
    if (kp) {
        S.dbg[32] += kta; S.dbg[33] += ktb; S.dbg[34] += ktc; S.dbg[35] += sg.len; S.dbg[36] += 1;
    }
#endif
#undef LPROF
}
template <int NRMAX>
__global__ __launch_bounds__(256) void k_lane(const SEv* __restrict__ recs, const sg_event* __restrict__ ev,
                                              const uint32_t* __restrict__ vals, const Seg* __restrict__ segs,
                                              const uint32_t* __restrict__ order, uint32_t m, DevState S, DevCfg cfg,
                                              int64_t t0, uint32_t* __restrict__ dec, uint32_t* __restrict__ bflags) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    lane_seg<NRMAX>(recs, ev, vals, segs[order[i]], S, cfg, t0, dec, bflags, i);
}

// =================================================================================
// k_lite: one lane per segment for the common rule shape -- DefaultController flow stages (QPS or
// thread grade, FlowSlot.java:146-158 + DefaultController.java:49-81) and DegradeRule breakers, no
// param rules, no prioritized entries, no STRATEGY_RELATE.  Same chain.h semantics as k_lane, but the
// rules are read once per segment (not per event), the passed bits of the first 256 positions stay in
// registers (EXITs of them never re-read dec[]), and the kernel carries none of the param / warm-up /
// rate-limiter / borrow code, so its code fits the instruction cache and its state fits in VGPRs.
//
// Minute window: a lite segment is a cold resource, a few events per second, so nearly every event
// opens a new second and the read of that second's bucket (to tell "same second, accumulate" from
// "stale slot, reset") would be an HBM round trip on every event's critical path.  No check of a lite
// segment reads the current second's minute bucket (the flow checks read the second window, the
// exception-count breaker a running sum of expired seconds), so the events of a second accumulate
// into register deltas and the bucket is read-modified-written when the segment moves on: its load is
// issued at that second change and consumed at the next one, off the critical path.  (A bucket with a
// later window start -- the clock went back a minute -- would need the old path's "detached" drop;
// that only happens in a batch rejected with BF_BACKWARD.)
// =================================================================================
struct MinDelta {
    int32_t p, b, s, rt, e, minrt;  // per-second deltas of a cold resource (<= 256 events) fit in int32
};
struct LiteMin {
    int64_t T;      // second of the pending deltas (-1: none yet)
    MinDelta pd;    // pending deltas of second T
    bool fly;       // an RMW in flight: bucket fb (loaded at the last second change) + deltas fd of second fT
    int64_t fT;
    MinDelta fd;
    Bkt fb;
};
__device__ __forceinline__ void md_zero(MinDelta& d) { d.p = d.b = d.s = d.rt = d.e = 0; d.minrt = INT32_MAX; }
// LeapArray.currentWindow on the minute bucket of second T, then the second's additions
__device__ __forceinline__ Bkt md_apply(Bkt b, int64_t T, const MinDelta& d, int32_t max_rt) {
    if (b.ws > T) return b;  // detached: the additions are lost (Q3)
    if (b.ws < T) bkt_reset(b, T, max_rt);
    b.pass += d.p; b.block += d.b; b.succ += d.s; b.rt += d.rt; b.exc += d.e;
    if ((int64_t)d.minrt < b.minrt) b.minrt = d.minrt;
    return b;
}
__device__ __forceinline__ void lm_finish(LiteMin& L, Bkt* minb, int32_t max_rt) {
    if (L.fly) {
        minb[(L.fT / 1000) % 60] = md_apply(L.fb, L.fT, L.fd, max_rt);
        L.fly = false;
    }
}
// the event opens second T: the pending second goes in flight, the previous flight lands
__device__ __forceinline__ void lm_roll(LiteMin& L, Node& N, Bkt* minb, int64_t T, int32_t max_rt, uint32_t pflags) {
    lm_finish(L, minb, max_rt);
    if (L.T >= 0) {
        L.fb = minb[(L.T / 1000) % 60];  // consumed at the next second change
        L.fT = L.T;
        L.fd = L.pd;
        L.fly = true;
    }
    L.T = T;
    md_zero(L.pd);
    // StatisticNode.totalException running sum (exc_advance): the seconds it reads are a minute old --
    // never the one in flight -- except on a first full sum, which must see it
    if ((pflags & PF_EXC_COUNT) && N.exc_sum_sec < T) {
        if (N.exc_sum_sec < 0) lm_finish(L, minb, max_rt);
        exc_advance(N, minb, T);
    }
}

// PL (XF_PLITE programs, the launch's other lanes return): ParamFlowSlot's one QPS DefaultController rule on args[0]
// first (ParamFlowSlot.java:77-101, ParamFlowChecker.passDefaultLocalCheck), its map and the thread-count map of
// paramIdx 0 held by the lane (PmLane), ParamFlowStatisticEntryCallback / ExitCallback on them
// (ParameterMetric.java:117-241); args[0]'s key from the key ring (k_rs_first).
#ifndef LITE_PL_WAVES
#define LITE_PL_WAVES 1  // k_lite<true>'s occupancy target (1: 256 VGPRs + 36 AGPRs, no spill; 2: 41 VGPRs spilled,
                         // C6 0.88 vs 0.92 G entries/s, profiles/r06)
#endif
template <bool PL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(PL ? LITE_PL_WAVES : 2))) void k_lite(const SEv* __restrict__ recs, const sg_event* __restrict__ ev,
                                              const uint32_t* __restrict__ vals, const Seg* __restrict__ segs,
                                              const uint32_t* __restrict__ order, uint32_t m, DevState S, DevCfg cfg,
                                              int64_t t0, uint32_t* __restrict__ dec, uint32_t* __restrict__ bflags) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const Seg sg = segs[order[i]];
    const uint32_t res = sg.res;
    const Prog pg = S.prog[res];
    if (((pg.xf & XF_PLITE) != 0) != PL) return;
    const int nf = pg.n_flow, nd = pg.n_degrade;  // <= 2 each (PF_J16)
    const DRule* rules = S.rules + pg.rule_off + (PL ? 1 : 0);  // (flow stages, then breakers)
    // PL: the param rule and the two held map headers live in LDS, one slot a lane (60 KB a workgroup), not in
    // registers (256 VGPRs + 68 AGPRs -> + 36).  Two waves a SIMD still spill (LITE_PL_WAVES).
    __shared__ DRule spr[PL ? 256 : 1];
    __shared__ PMap smp[PL ? 256 : 1], stm[PL ? 256 : 1];
    DRule& pr = spr[PL ? threadIdx.x : 0];
    PmLaneRef PLM{NO_ID, NO_ID, smp[PL ? threadIdx.x : 0], stm[PL ? threadIdx.x : 0]};
    if (PL) {
        pr = S.rules[pg.rule_off];
        PLM.mid = pr.pmap;
        PLM.mp = S.pmap[pr.pmap];
        PLM.tid = tmap_of(S, pg.tm_base, 0);
        if (PLM.tid != NO_ID) PLM.tm = S.pmap[PLM.tid];
    }
    // per-segment rule constants: flow thresholds, degrade grades/thresholds/windows
    double fcnt[2] = {0.0, 0.0};
    bool fthr[2] = {false, false};
    uint32_t fslot[2] = {0, 0};
    DegParam dr[2];       // only the fields the checks read: the whole DRule would cost 28 VGPRs each
    uint32_t dslot[2] = {0, 0};
    RState ds[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        if (k < nf) {
            fcnt[k] = rules[k].count;
            fthr[k] = rules[k].grade == SG_FLOW_GRADE_THREAD;
            fslot[k] = rules[k].slot;
        }
        if (k < nd) {
            dr[k] = deg_param(rules[nf + k]);
            dslot[k] = rules[nf + k].slot;
            ds[k] = S.rstate[pg.rule_off + (PL ? 1 : 0) + nf + k];
        }
    }
#ifdef SG_KPROF
    const bool kp = S.dbg && i == 0;  // the longest segment of the launch
    unsigned long long kt0 = kp ? __builtin_amdgcn_s_memtime() : 0, kta = 0, ktb = 0, ktc = 0, ktd = 0, ktf = 0, ktg = 0, kth = 0;
#define LPROF(acc)                                                \
    if (kp) {                                                     \
        unsigned long long _n = __builtin_amdgcn_s_memtime();     \
        acc += _n - kt0;                                          \
        kt0 = _n;                                                 \
    }
#else
#define LPROF(acc)
#endif
    Node N;
    node_load(N, S, res);
    const Ctx C{S.minb + (uint64_t)res * 60, cfg.max_rt, pg.pflags};
    LiteMin L;
    L.T = -1;
    L.fly = false;
    md_zero(L.pd);
    const bool has_chain = (N.flags & NI_CHAIN) != 0;
    const bool chain = has_chain && cfg.switch_on;
    if (sg.len && (t0 + recs[sg.start].dt) < (N.sb[0].ws > N.sb[1].ws ? N.sb[0].ws : N.sb[1].ws))
        atomicOr(bflags, BF_BACKWARD);  // Q3: the clock went back across batches
    uint64_t pm0 = 0, pm1 = 0, pm2 = 0, pm3 = 0;  // passed bits of positions 0..255
    // records in chunks of 4 with the next chunk in flight: one memory round trip per 4 events (the
    // loads are unconditional with a clamped index, so the compiler's vmcnt waits cannot serialise them)
#ifndef LITE_CH
#define LITE_CH 4
#endif
    constexpr uint32_t CH = LITE_CH;
    const uint4* r4 = reinterpret_cast<const uint4*>(recs + sg.start);
    const uint32_t qmax = sg.len ? sg.len - 1 : 0;
    uint4 cur[CH], nxt[CH];
#pragma unroll
    for (uint32_t k = 0; k < CH; ++k) cur[k] = r4[k < qmax ? k : qmax];
    LPROF(kta)
    for (uint32_t j0 = 0; j0 < sg.len; j0 += CH) {
#pragma unroll
    for (uint32_t k = 0; k < CH; ++k) nxt[k] = r4[j0 + CH + k < qmax ? j0 + CH + k : qmax];
#pragma unroll 1
    for (uint32_t k = 0; k < CH; ++k) {
        const uint4 rw = cur[0];
#pragma unroll
        for (uint32_t m = 0; m + 1 < CH; ++m) cur[m] = cur[m + 1];
        const uint32_t j = j0 + k;
        if (j >= sg.len) break;
        const int32_t rdt = (int32_t)rw.x;
        const uint32_t rx = rw.y;
        const int cntv = (int)(rw.z & 0xFFFFu);
        const int32_t rtv = (int32_t)(rw.z >> 16);
        const uint32_t kind = rw.w & 0xFFu, code = (rw.w >> 16) & 0xFFu;
        const int64_t t = t0 + rdt;
        const int64_t T = t - t % 1000;
        uint32_t d = mk_dec(ST_NOT_ENTRY, 0, 0);
        if (kind == SG_EV_ENTRY) {
            if (!chain) d = mk_dec(ST_NO_CHECK, 0, 0);
            else {
                if (T != L.T) lm_roll(L, N, C.minb, T, C.max_rt, C.pflags);
                uint32_t status = ST_PASS, slot = 0;
                uint64_t key = NO_KEY;
                if (PL) {  // ParamFlowSlot: initHotParamMetricsFor, the rule's index bit, then its check
                    N.flags |= NI_PM | ni_tm(0);
                    if ((rw.w >> 8) & SG_F_HAS_ARG)
                        key = S.key_ring[(S.gbase + (vals[sg.start + j] & 0x7FFFFFFFu)) & cfg.ring_mask];
                    if (key != NO_KEY && !param_default_lane(S, pr, PLM.mp, cntv, key, t, bflags)) {
                        status = ST_BLOCK_PARAM;
                        slot = pr.slot;
                    }
                }
#pragma unroll
                for (int k = 0; k < 2; ++k) {  // FlowSlot: DefaultController on the ClusterNode
                    if (k < nf && status == ST_PASS) {
                        int32_t cur;
                        if (fthr[k]) cur = N.thread;
                        else { sec_current(N, t, C.max_rt); cur = j_d2i((double)SEC_SUM(N, t, pass)); }
                        if ((double)j_iadd(cur, cntv) > fcnt[k]) { status = ST_BLOCK_FLOW; slot = fslot[k]; }
                    }
                }
                LPROF(ktf)
                // StatisticNode.totalException: exc_sum is at T after the roll (PF_EXC_COUNT)
                const int64_t exc_total = N.exc_sum;
#pragma unroll
                for (int k = 0; k < 2; ++k) {  // DegradeSlot
                    if (k < nd && status == ST_PASS && !degrade_pass(N, C, dr[k], ds[k], t, &exc_total)) {
                        status = ST_BLOCK_DEGRADE;
                        slot = dslot[k];
                    }
                }
                LPROF(ktg)
                const bool passed = status == ST_PASS;
                // StatisticSlot.entry: second window + the second's minute deltas
                const int sl = sec_current(N, t, C.max_rt);
                if (passed) {
                    N.thread++;
                    sec_add(N, sl, cntv, 0, 0, 0, 0, INT64_MAX);
                    L.pd.p += cntv;
                } else {
                    sec_add(N, sl, 0, cntv, 0, 0, 0, INT64_MAX);
                    L.pd.b += cntv;
                }
                LPROF(kth)
                // ParamFlowStatisticEntryCallback.onPass -> addThreadCount(args[0])
                if (PL && passed && key != NO_KEY && PLM.tid != NO_ID) thread_add_lane(S, PLM.tm, key, 1, bflags);
                d = passed ? mk_dec(ST_PASS, 0, 0) : mk_dec(status, slot, 0);
                if (passed && j < 256) {
                    const uint64_t b = 1ull << (j & 63);
                    if (j < 64) pm0 |= b; else if (j < 128) pm1 |= b; else if (j < 192) pm2 |= b; else pm3 |= b;
                }
            }
            LPROF(ktb)
        } else {
            bool eff;
            if (code == RC_NONE) eff = kind == SG_EV_EXIT ? chain : has_chain;
            else if (code == RC_PASSED) eff = true;
            else if (code == RC_NOT) eff = false;
            else {
                const uint32_t rel = rx - sg.start;
                if (rel >= j) { atomicOr(bflags, BF_BAD_REF); eff = false; }  // not an earlier ENTRY of this resource
                else if (rel < 256) {
                    const uint64_t w = rel < 64 ? pm0 : rel < 128 ? pm1 : rel < 192 ? pm2 : pm3;
                    eff = ((w >> (rel & 63)) & 1) != 0;
                } else eff = st_passed(dec[rx] & 0xFF);  // written by this lane
            }
            if (eff && kind == SG_EV_EXIT) {  // StatisticSlot.exit
                if (T != L.T) lm_roll(L, N, C.minb, T, C.max_rt, C.pflags);
                const int sl = sec_current(N, t, C.max_rt);
                sec_add(N, sl, 0, 0, cntv, rtv, 0, rtv);
                L.pd.s += cntv;
                L.pd.rt += rtv;
                if (rtv < L.pd.minrt) L.pd.minrt = rtv;
                N.thread--;
                const uint32_t rfl = (rw.w >> 8) & 0xFFu;
                if (PL && (rfl & SG_F_EXIT_ARGS) && (N.flags & NI_PM) && (N.flags & ni_tm(0)) && PLM.tid != NO_ID) {
                    // ParamFlowStatisticExitCallback: its own args[0], else its ENTRY's (lane_exit)
                    uint64_t ref = SG_REF_NONE;
                    if (rfl & RF_OWN_ARGS) ref = S.gbase + (vals[sg.start + j] & 0x7FFFFFFFu);
                    else if (code == RC_BATCH) ref = S.gbase + (vals[rx] & 0x7FFFFFFFu);
                    else if (code == RC_PASSED) ref = ev[vals[sg.start + j] & 0x7FFFFFFFu].aux & SG_REF_NONE;
                    if (ref != SG_REF_NONE) {
                        const uint64_t key = S.key_ring[ref & cfg.ring_mask];
                        if (key != NO_KEY) thread_add_lane(S, PLM.tm, key, -1, bflags);
                    }
                }
            } else if (eff && cntv > 0) {  // ClusterNode.trace
                if (T != L.T) lm_roll(L, N, C.minb, T, C.max_rt, C.pflags);
                const int sl = sec_current(N, t, C.max_rt);
                sec_add(N, sl, 0, 0, 0, 0, cntv, INT64_MAX);
                L.pd.e += cntv;
                if (N.exc_sum_sec == T) N.exc_sum += cntv;
            }
            LPROF(ktc)
        }
        if (kind == SG_EV_ENTRY) dec[sg.start + j] = d;  // k_post reads ENTRY words only
    }
#pragma unroll
    for (uint32_t k = 0; k < CH; ++k) cur[k] = nxt[k];
    }
    // the last two seconds' minute buckets
    lm_finish(L, C.minb, C.max_rt);
    if (L.T >= 0) {
        Bkt* b = C.minb + (L.T / 1000) % 60;
        *b = md_apply(*b, L.T, L.pd, C.max_rt);
    }
    node_store(N, S, res, pg.pflags);
#pragma unroll
    for (int k = 0; k < 2; ++k)
        if (k < nd) S.rstate[pg.rule_off + (PL ? 1 : 0) + nf + k] = ds[k];
    if (PL) {
        pm_store(S, PLM.mid, PLM.mp);
        if (PLM.tid != NO_ID) pm_store(S, PLM.tid, PLM.tm);
    }
    LPROF(ktd)
#ifdef SG_KPROF
    if (kp) {
        S.dbg[32] += kta; S.dbg[33] += ktb; S.dbg[34] += ktc; S.dbg[35] += sg.len; S.dbg[36] += 1; S.dbg[37] += ktd; S.dbg[38] += ktf; S.dbg[39] += ktg; S.dbg[51] += kth;
    }
#endif
#undef LPROF
}

// =================================================================================
// k_jac: cooperative speculative decide of one segment by NW wavefronts
// =================================================================================
// inclusive wave scan with DPP row shifts + row broadcasts (GFX9 family, wave64)
#define DPP_STEP(v, ident, ctrl, rmask, OP) \
    v = OP((uint32_t)__builtin_amdgcn_update_dpp((int)(ident), (int)(v), ctrl, rmask, 0xf, false), v)
#define WAVE_SCAN(v, ident, OP)              \
    do {                                      \
        DPP_STEP(v, ident, 0x111, 0xf, OP);   \
        DPP_STEP(v, ident, 0x112, 0xf, OP);   \
        DPP_STEP(v, ident, 0x114, 0xf, OP);   \
        DPP_STEP(v, ident, 0x118, 0xf, OP);   \
        DPP_STEP(v, ident, 0x142, 0xa, OP);   \
        DPP_STEP(v, ident, 0x143, 0xc, OP);   \
    } while (0)
__device__ __forceinline__ uint32_t op_add(uint32_t a, uint32_t b) { return a + b; }
__device__ __forceinline__ uint32_t op_min(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t op_max(uint32_t a, uint32_t b) { return a > b ? a : b; }
// segmented count: bit31 = "reset here", low bits = count since the last reset; a is the earlier element
__device__ __forceinline__ uint32_t op_seg(uint32_t a, uint32_t b) {
    return (b & 0x80000000u) ? b : ((a & 0x80000000u) | ((a + b) & 0x7fffffffu));
}
__device__ __forceinline__ uint32_t shr1(uint32_t incl, uint32_t ident) {  // exclusive from inclusive
    uint32_t v = (uint32_t)__shfl_up((int)incl, 1, 64);
    return lane_id() == 0 ? ident : v;
}
__device__ __forceinline__ int64_t wscan_i64_add(int64_t x) {
    const uint32_t l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int64_t y = __shfl_up(x, o, 64);
        if (l >= (uint32_t)o) x += y;
    }
    return x;
}
__device__ __forceinline__ int64_t wscan_i64_max(int64_t x) {
    const uint32_t l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int64_t y = __shfl_up(x, o, 64);
        if (l >= (uint32_t)o) x = x > y ? x : y;
    }
    return x;
}
#define NEG_INF64 ((int64_t)0x8000000000000000LL)

#define NO_LANE 0xFFFFFFFFu

// Block-wide exchanges of per-wave values in LDS (a[w], w < NW <= 16): lanes l < NW load a[l] at once and an
// inclusive DPP scan runs within the first 16-lane row; lane NW-1 holds the total, lane wv-1 the waves before wv.
// (A loop over the NW values in every lane issues NW dependent-latency LDS reads per exchange.)
#define ROW_SCAN(v, ident, OP, NWV)                                    \
    do {                                                               \
        if ((NWV) > 1) DPP_STEP(v, ident, 0x111, 0xf, OP);              \
        if ((NWV) > 2) DPP_STEP(v, ident, 0x112, 0xf, OP);              \
        if ((NWV) > 4) DPP_STEP(v, ident, 0x114, 0xf, OP);              \
        if ((NWV) > 8) DPP_STEP(v, ident, 0x118, 0xf, OP);              \
    } while (0)
template <int NW>
__device__ __forceinline__ uint32_t blk_min(const uint32_t* a) {
    static_assert(NW <= 16, "one DPP row");
    uint32_t v = lane_id() < (uint32_t)NW ? a[lane_id()] : NO_LANE;
    ROW_SCAN(v, NO_LANE, op_min, NW);
    return (uint32_t)__builtin_amdgcn_readlane((int)v, NW - 1);
}
// sum over the waves before wv (exclusive) and the total, of a[w * stride]
template <int NW>
__device__ __forceinline__ uint32_t blk_sum_before(const uint32_t* a, uint32_t stride, uint32_t wv, uint32_t* tot) {
    static_assert(NW <= 16, "one DPP row");
    uint32_t v = lane_id() < (uint32_t)NW ? a[lane_id() * stride] : 0u;
    ROW_SCAN(v, 0u, op_add, NW);
    *tot = (uint32_t)__builtin_amdgcn_readlane((int)v, NW - 1);
    return wv == 0 ? 0u : (uint32_t)__builtin_amdgcn_readlane((int)v, (int)wv - 1);
}

// Workgroup barrier that only drains LDS traffic.  __syncthreads() is a release/acquire fence over
// global memory as well, i.e. it waits for every outstanding vector load -- including the next tile
// prefetched into registers -- so each tile would pay a full HBM round trip.  All cross-wave data
// of k_jac lives in LDS; the only cross-wave global data are decisions read back as old references,
// and those are ordered by the full __syncthreads() every FULL_FENCE_TILES tiles plus an L1-bypassing
// (agent-scope) load.
// LDS-broadcast values that steer control flow around barriers are read through readfirstlane:
// provably uniform, they become scalar branches, and the compiler cannot restructure a loop whose
// exit it would otherwise believe divergent into one where lanes of a wave run different numbers
// of barriers.
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ int64_t uni64(int64_t v) {
    const uint32_t lo = uni((uint32_t)(uint64_t)v), hi = uni((uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
#define FULL_FENCE_TILES 8

// u32 quantities scanned block-wide in one Jacobi iteration (counts <= 1024 are packed in halves)
enum { Q_P, Q_B, Q_S, Q_RT, Q_E, Q_TH, Q_MIN, Q_TI /* touch | inr << 16 */, Q_TR /* trip counts, 2 per word */ };

#define NSPAN 64        // skipped spans per segment (LDS list for references into them)
#define OPEN_EPL 4      // open stretches: events per lane per chunk
#define TG_PASSES 2     // closed-form passes per Jacobi iteration of a THREAD-grade program

// the wide owners hold the resource's minute window in LDS (sh.minl) for their lifetime: the round's leader reads and
// writes it every second, from HBM a dependent round trip or two per round; the one-wave owner keeps it in HBM (its
// LDS bounds how many run on a CU)
#define JAC_MINL(NW) ((NW) >= 4)
template <int NW, int MF, int MD>
struct JacSh {
    Bkt minl[JAC_MINL(NW) ? 60 : 1];
    Node node;
    DRule rules[MF + MD];
    RState rs[MF + MD];
    RState syn[MF];  // WarmUp state synced at the round's second
    // round base: the node's window sums at the round's bucket
    int64_t bP, bB, bS, bRT, bE, bEM, bTH;
    int64_t bkt0, next_reset, tnext;
    // committed inside the round (folded into the node by the leader at round end)
    int64_t cP, cB, cS, cRT, cE, cTH;
    uint32_t cminrt, ctouch;
    uint32_t has_sync, warm_reach;
    uint32_t c0, last_out, round_open, pad;
    uint32_t part[NW][Q_TR + (MD + 1) / 2];
    uint32_t pseg[NW][MD];
    int64_t prl[NW][4];
    uint32_t mism[2][NW];
    uint32_t mo[2][NW];        // evaluated outcome of each wave's first mismatching lane
    uint32_t mu[2][NW];        // ... its in-round ENTRY acquire units up to and including it
    int64_t mp[2][NW];         // ... and the round's pass count right after it (when it passed)
    // frozen-stretch skipping
    uint32_t npend;            // live entries of the pending-pass list pend[start, start + npend)
    uint32_t nsp;              // spans of this segment decided by k_fill (their dec[] words are not written yet)
    uint32_t skip_go;
    uint32_t pad2;
    uint2 spn[NSPAN];          // [s, e) relative positions
    unsigned long long fl[NW]; // flagged-block ballots
    uint32_t cg[NW][3];        // closed-form guesses: per-wave totals (entries, effective exits | last entry time, others)
    uint32_t cgm[NW];          // ... per-wave minimum of the thread-grade admission bound
    // open stretches: the stop's evaluated outcome and the RT breakers' segmented passCount state before it; the
    // round machine: the stop's time and the round's pass count at it
    uint32_t os_o;
    uint32_t os_seg[MD];
    int32_t os_t;
    int64_t os_P;
    // the round machine's state (written by the leader, read by every lane after a barrier): the open view before the
    // current chunk (passes, successes, RT sum, exceptions, minute exceptions, blocks), the RT stages' segmented
    // passCount carry and base, the round's event times, the open round's first position, frozen mode, the mode
    int64_t mv[6];
    uint32_t mksg[MD];
    int32_t mpcb[MD];
    int64_t mfzP;
    int32_t mrlo, mrhi;
    uint32_t molo, mfz0, mfcut, mmode;
    double mflim[MF];
};

// leader: fold the round's committed deltas into the node (StatisticSlot bookkeeping of every
// committed event, as one bucket update) and persist WarmUp syncs that some entry reached
template <class SH>
__device__ void round_fold(SH& sh, const Ctx& C, int nf) {
    if (!sh.round_open) return;
    Node& N = sh.node;
    const int64_t tc = sh.bkt0 * 500;
    if (sh.ctouch) {
        int sl = sec_current(N, tc, C.max_rt);
        const int64_t mrt = sh.cminrt == NO_LANE ? INT64_MAX : (int64_t)sh.cminrt;
        sec_add(N, sl, sh.cP, sh.cB, sh.cS, sh.cRT, sh.cE, mrt);
        min_current(N, C.minb, tc, C.max_rt, C.pflags);
        if (!(N.mst & MS_DETACHED)) {
            min_add(N, sh.cP, sh.cB, sh.cS, sh.cRT, sh.cE, mrt);
            if (N.exc_sum_sec == tc - tc % 1000) N.exc_sum += sh.cE;
        }
    }
    N.thread += (int32_t)sh.cTH;
    for (int s = 0; s < nf; ++s)
        if ((sh.has_sync >> s) & 1 & (sh.warm_reach >> s)) { sh.rs[s].a = sh.syn[s].a; sh.rs[s].b = sh.syn[s].b; }
    sh.round_open = 0;
}
// leader: open the round of the 500 ms bucket holding tn.  Side-effect free in Java terms: bucket
// resets happen at fold time, only if a committed event touched the windows.
template <class SH>
__device__ void round_setup(SH& sh, const Ctx& C, int nf, int nd, int64_t tn) {
    Node& N = sh.node;
    const int64_t b0 = tn / 500, T = tn - tn % 1000;
    min_flush(N, C.minb);  // the window (sh.minl) holds the current minute bucket from here on
    int64_t next_reset = INT64_MAX;
    for (int k = 0; k < nd; ++k) {  // ResetTask due (Q12)
        RState& s = sh.rs[nf + k];
        if (s.a && tn >= s.c) { s.a = 0; s.b = 0; }
        if (s.a && s.c < next_reset) next_reset = s.c;
    }
    const Bkt& cur = (b0 & 1) ? N.sb[1] : N.sb[0];
    const Bkt& prv = (b0 & 1) ? N.sb[0] : N.sb[1];
    const bool cv = cur.ws >= b0 * 500;  // else currentWindow resets it before any read
    const bool pv = prv.ws >= 0 && tn - prv.ws <= 1000;
    sh.bP = (cv ? cur.pass : 0) + (pv ? prv.pass : 0);
    sh.bB = (cv ? cur.block : 0) + (pv ? prv.block : 0);
    sh.bS = (cv ? cur.succ : 0) + (pv ? prv.succ : 0);
    sh.bRT = (cv ? cur.rt : 0) + (pv ? prv.rt : 0);
    sh.bE = (cv ? cur.exc : 0) + (pv ? prv.exc : 0);
    sh.bTH = N.thread;
    sh.bEM = 0;
    if (C.pflags & PF_EXC_COUNT) {  // StatisticNode.totalException at T
        if (N.exc_sum_sec < T) exc_advance(N, C.minb, T);
        if (N.exc_sum_sec != T) {
            int64_t s = 0;
            for (int k = 0; k < 60; ++k) {
                Bkt b = C.minb[k];
                if (b.ws >= T - 59000 && b.ws <= T) s += b.exc;
            }
            N.exc_sum = s;
            N.exc_sum_sec = T;
        }
        sh.bEM = N.exc_sum;
    }
    sh.has_sync = 0;
    for (int s = 0; s < nf; ++s) {  // WarmUpController.syncToken at this second (persisted if reached)
        const DRule& r = sh.rules[s];
        if ((r.behavior == SG_CONTROL_BEHAVIOR_WARM_UP || r.behavior == SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER) &&
            T > sh.rs[s].b) {
            const int slot = (int)(((tn - 1000) / 1000) % 60);
            const Bkt b = C.minb[slot];
            int64_t prev = 0;
            if (!(b.ws < 0 || tn - b.ws > 60000 || b.ws + 1000 < tn - 1000)) prev = b.pass;
            RState tmp = sh.rs[s];
            warm_sync(r, tmp, tn, prev);
            sh.syn[s] = tmp;
            sh.has_sync |= 1u << s;
        }
    }
    sh.warm_reach = 0;
    sh.bkt0 = b0;
    sh.next_reset = next_reset;
    sh.cP = sh.cB = sh.cS = sh.cRT = sh.cE = sh.cTH = 0;
    sh.cminrt = NO_LANE;
    sh.ctouch = 0;
    sh.round_open = 1;
}

// leader: the round ends (fold) and the round of tn opens (setup) -- kept out of line: the round machine calls it with a
// chunk of records and its prefetch live in registers, and inlined the set-up's own temporaries spilled the 512-lane
// owner's per-chunk loop (a call per round costs less than scratch traffic per chunk)
template <class SH>
__device__ __attribute__((noinline)) void round_next_leader(SH& sh, const Ctx& C, int nf, int nd, int64_t tn) {
    round_fold(sh, C, nf);
    round_setup(sh, C, nf, nd, tn);
}

__device__ __forceinline__ uint32_t out_to_dec(const DRule* rules, int nr, int nf, uint32_t o, int64_t wait) {
    if (o == (uint32_t)nr) return mk_dec(ST_PASS, 0, wait);
    return mk_dec((int)o < nf ? ST_BLOCK_FLOW : ST_BLOCK_DEGRADE, rules[o].slot, 0);
}

// one event of a k_jac tile, decoded once when its tile is loaded
struct JEv {
    int32_t dt;   // time relative to t0
    uint32_t cz;  // count | rt << 16
    uint32_t kf;  // kind (0xFF: no event) | JK_VALID | JK_WIN | JK_VAL
    uint32_t wi;  // JK_WIN: status-window index of the referenced ENTRY
};
enum : uint32_t { JK_VALID = 0x100u, JK_WIN = 0x200u, JK_VAL = 0x400u, JK_PB = 0x800u /* RF_PBLK ENTRY */ };
// an event's class in one Jacobi iteration: in the round, ENTRY, effective EXIT, effective TRACE, ENTRY a param rule
// blocked (XF_MIX: a block in the statistics, no flow / degrade check)
enum : uint32_t { JC_INR = 1u, JC_ENT = 2u, JC_XE = 4u, JC_TE = 8u, JC_PB = 16u };

// the scanned quantities (Q_*) of one event under its outcome guess g
template <int NQ>
__device__ __forceinline__ void jac_q(uint32_t (&q)[NQ], uint32_t c, uint32_t g, uint32_t cz, uint32_t nr, uint32_t nf) {
    const uint32_t cnt = cz & 0xFFFFu, rtv = cz >> 16;
    const bool ent = (c & JC_ENT) != 0, xe = (c & JC_XE) != 0, te = (c & JC_TE) != 0, pb = (c & JC_PB) != 0;
    const bool gp = ent && g == nr;
    q[Q_P] = gp ? cnt : 0u;
    q[Q_B] = ((ent && !gp) || pb) ? cnt : 0u;
    q[Q_S] = xe ? cnt : 0u;
    q[Q_RT] = xe ? rtv : 0u;
    q[Q_E] = te ? cnt : 0u;
    q[Q_TH] = gp ? 1u : (xe ? 0xFFFFFFFFu : 0u);
    q[Q_MIN] = xe ? rtv : NO_LANE;
    q[Q_TI] = ((ent || xe || te || pb) ? 1u : 0u) | ((c & JC_INR) ? 0x10000u : 0u);
#pragma unroll
    for (int k = Q_TR; k < NQ; ++k) {  // guessed breaker trips, two degrade stages per word
        const uint32_t s0 = nf + 2u * (uint32_t)(k - Q_TR);
        q[k] = (ent && g == s0) ? 1u : (ent && g == s0 + 1u) ? 0x10000u : 0u;
    }
}
template <int NQ>
__device__ __forceinline__ void jac_acc(uint32_t (&a)[NQ], const uint32_t (&q)[NQ]) {
#pragma unroll
    for (int k = 0; k < NQ; ++k) a[k] = k == Q_MIN ? op_min(a[k], q[k]) : a[k] + q[k];
}
template <int NQ>
__device__ __forceinline__ void jac_zero(uint32_t (&a)[NQ]) {
#pragma unroll
    for (int k = 0; k < NQ; ++k) a[k] = k == Q_MIN ? NO_LANE : 0u;
}
// a rate limiter's latestPassedTime moves for this ENTRY under outcome g (it passed stage s)
__device__ __forceinline__ bool rl_upd(const DRule& r, uint32_t c, uint32_t g, int s, int cnt) {
    return (c & JC_ENT) && g > (uint32_t)s &&
           (r.behavior != SG_CONTROL_BEHAVIOR_RATE_LIMITER || (cnt > 0 && r.count > 0));
}

// NW wavefronts own one segment; each lane takes EP consecutive events of a tile (TILE = NW * 64 * EP
// positions), so one chain of scans and barriers -- the latency that bounds an iteration -- decides
// up to TILE events: a lane folds its events' quantities sequentially, the wave and block scans run on
// the lane totals, and each event's view is the lane's exclusive prefix plus its running sum.
// CLS: 0 every segment of the dispatch list; 1 only QPS-DefaultController programs (PF_FROZEN), 2 only the others
// (one bin's list decided by two instantiations, each with the registers its own kind of segment needs)
template <int NW, int EP, int WINLOG, int MF, int MD, bool RL, bool SKIP, int CLS = 0>
#ifndef J4_WAVES
#define J4_WAVES 2  // waves per SIMD the 256-lane owner is compiled for: 2 caps it at 256 registers (the round machine
                    // took it to ~300 and one workgroup a CU: J4 1.75 -> 2.57 ms per C4 batch; capped 1.47 ms)
#endif
__global__ __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(NW == 1 ? (EP == 1 ? 4 : 2) : (EP == 1 ? (NW == 4 ? J4_WAVES : 1) : 2)))) void k_jac(
    const SEv* __restrict__ recs, const Seg* __restrict__ segs, const uint32_t* __restrict__ order, uint32_t m,
    DevState S, DevCfg cfg, int64_t t0, uint32_t* __restrict__ dec, uint32_t* __restrict__ bflags) {
    constexpr uint32_t HW = NW * 64;
    constexpr uint32_t TILE = HW * EP;  // positions per tile; lane l holds [l * EP, l * EP + EP)
    constexpr uint32_t WIN = 1u << WINLOG;
    constexpr int NQ = Q_TR + (MD + 1) / 2;
    static_assert(WIN >= 2 * TILE, "status window must hold two tiles");
    static_assert(TILE < 0x10000u, "counts of a tile are packed in 16 bits");
    __shared__ JacSh<NW, MF, MD> sh;
    __shared__ __attribute__((aligned(16))) uint8_t win[WIN];
    if (blockIdx.x >= m) return;
    const uint32_t tid = threadIdx.x;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint32_t lane = tid & 63;
    const Seg sg = segs[order[blockIdx.x]];
    const uint32_t res = sg.res;
    const Prog pg = S.prog[res];
    if (CLS != 0 && (((pg.pflags & PF_FROZEN) != 0) != (CLS == 1))) return;  // the other instantiation's segment
    if ((NW == 16 || NW == 4 || NW == 1) && (pg.xf & (XF_HEADT | XF_HEADR)) && !(cfg.dbg_flags & HEAD_OFF)) return;  // k_head's
    const int nf = pg.n_flow, nd = pg.n_degrade, nr = nf + nd;
    // the minute window in LDS (sh.minl): loaded here, written back at the segment's end; no other kernel of the
    // decide stage touches this resource's minute buckets while its owner runs
    if (JAC_MINL(NW))
        for (uint32_t i = tid; i < 60u * sizeof(Bkt) / 16u; i += HW)
            reinterpret_cast<uint4*>(sh.minl)[i] = reinterpret_cast<const uint4*>(S.minb + (uint64_t)res * 60)[i];
    const Ctx C{JAC_MINL(NW) ? sh.minl : S.minb + (uint64_t)res * 60, cfg.max_rt, pg.pflags};
    // XF_MIX: the param rules come first in the program and k_pq's pre pass has decided them: an ENTRY one of them
    // blocked carries RF_PBLK (its dec[] word is final) and is a block here, nothing more
    const uint32_t roff = pg.rule_off + pg.n_param;
    const bool mixp = pg.n_param != 0;
    if (tid == 0) {
        node_load(sh.node, S, res);
        sh.round_open = 0;
        sh.c0 = 0;
        sh.last_out = (uint32_t)nr;
        sh.npend = 0;
        sh.nsp = 0;
    }
    if ((int)tid < nr) {
        sh.rules[tid] = S.rules[roff + tid];
        sh.rs[tid] = S.rstate[roff + tid];
    }
    __syncthreads();
    const bool chain = (sh.node.flags & NI_CHAIN) != 0;  // host routes switch_on == 0 to k_lane
    if (!chain) {  // no slot chain: every ENTRY is NO_CHECK, nothing is counted
        for (uint32_t p = tid; p < sg.len; p += HW)
            dec[sg.start + p] = recs[sg.start + p].kind == SG_EV_ENTRY ? mk_dec(ST_NO_CHECK, 0, 0)
                                                                        : mk_dec(ST_NOT_ENTRY, 0, 0);
        return;
    }
    if (tid == 0) {
        const int64_t tf = t0 + recs[sg.start].dt;
        if (tf < (sh.node.sb[0].ws > sh.node.sb[1].ws ? sh.node.sb[0].ws : sh.node.sb[1].ws))
            atomicOr(bflags, BF_BACKWARD);  // Q3: the clock went back across batches
    }
    int rl_s0 = -1, rl_s1 = -1;  // rate-limiter stages (uniform)
    if (RL) {
        for (int s = 0; s < nf; ++s) {
            uint8_t b = sh.rules[s].behavior;
            if (b == SG_CONTROL_BEHAVIOR_RATE_LIMITER || b == SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER) {
                if (rl_s0 < 0) rl_s0 = s; else rl_s1 = s;
            }
        }
    }
    const bool has_rt = (pg.pflags & PF_RT) != 0;
    // frozen / open stretches need every flow stage's verdict to be a function of the round's pass count: QPS
    // DefaultControllers (PF_FROZEN) and QPS WarmUpControllers, whose limit is fixed within a round once its second's
    // token sync is known (WarmUpController.java:83-175: syncToken moves storedTokens once per second)
    uint32_t warmm = 0;  // WarmUp flow stages (uniform)
    bool fz = true;
    for (int s = 0; s < nf; ++s) {
        const DRule& r = sh.rules[s];
        if (r.grade != SG_FLOW_GRADE_QPS) fz = false;
        else if (r.behavior == SG_CONTROL_BEHAVIOR_WARM_UP) warmm |= 1u << s;
        else if (r.behavior != SG_CONTROL_BEHAVIOR_DEFAULT) fz = false;
    }
    const bool frozen_prog = fz;
    // open stretches (all-pass prefix decisions, below): on unless debug flag 64; worth a chunk from one tile left
    // (the 256- and 512-lane owners only: inline in the 1024-lane and one-wave owners, whose 128-register budget the
    // Jacobi iteration already fills, it spilled the iteration's registers and cost more than it saved)
    constexpr bool OPEN = NW == 4 || NW == 8;
    const bool open_on = OPEN && !(cfg.dbg_flags & 64);
    // the round machine (open stretches going on frozen and into the next round in place): the 256-lane owner only --
    // on the 512-lane one (256 registers a lane, two waves a SIMD) its state spilled the chunk loop (A/B: J8 1.40 ->
    // 1.60 ms per C4 batch), so there an open stretch leaves at every stop as before
#ifndef JAC_MACH8
#define JAC_MACH8 0
#endif
    constexpr bool MACH = NW == 4 || (NW == 8 && JAC_MACH8);
    const uint32_t open_min = TILE;
    // single-stage programs with closed-form admission guesses (see the Jacobi iteration)
    // (not with param-blocked ENTRYs in the mix: the closed forms count every ENTRY as an acquire)
    const bool tg_mode = nf == 1 && nd == 0 && sh.rules[0].grade == SG_FLOW_GRADE_THREAD &&
                         sh.rules[0].behavior == SG_CONTROL_BEHAVIOR_DEFAULT && !(cfg.dbg_flags & 16) && !mixp;
    const bool rl_mode = RL && !mixp && nf == 1 && nd == 0 && sh.rules[0].grade == SG_FLOW_GRADE_QPS &&
                         (sh.rules[0].behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER ||
                          sh.rules[0].behavior == SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER) && !(cfg.dbg_flags & 16);

    // diagnostics (SG_DEBUG=1): per-bin iteration counters; phase cycles of the bin's first segment
    // only in builds with -DSG_KPROF (the timers cost registers the 1024-lane kernel does not have)
    const bool prof = S.dbg != nullptr;
    uint32_t n_it = 0, n_round = 0, n_tile = 0, n_mm = 0, n_frz = 0, n_opn = 0;
#ifdef SG_KPROF
    const bool prof0 = prof && tid == 0;  // every block times itself; the longest segment reports
    unsigned long long tmA = prof0 ? __builtin_amdgcn_s_memtime() : 0, tph[14] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t m_nopen = 0, m_nfrz = 0, m_nround = 0;  // the round machine's steps (the slowest segment's, dbg[56..58])
    const unsigned long long tm_start = tmA;
#define PROF_MARK(k)                                          \
    if (prof0) {                                              \
        unsigned long long _n = __builtin_amdgcn_s_memtime(); \
        tph[k] += _n - tmA;                                   \
        tmA = _n;                                             \
    }
#else
#define PROF_MARK(k)
#endif

    // ---- per-lane tile state: EP consecutive events
    uint32_t tbase = 0;
    const uint32_t lp0 = tid * EP;  // tile-relative position of the lane's first event
    SEv nxt[EP];                    // the next tile, in flight
    JEv ev[EP];
    uint32_t gg[EP];  // outcome guesses: index of the blocking stage, nr = pass
    const bool skip_on = SKIP && S.skip_ok && (pg.pflags & PF_FROZEN);
    // positions of skipped spans: blocked ENTRYs whose dec[] words k_fill writes after this kernel
    auto in_span = [&](uint32_t rel) -> bool {
        if (!SKIP) return false;
        const uint32_t ns = sh.nsp;
        for (uint32_t i = 0; i < ns; ++i)
            if (rel >= sh.spn[i].x && rel < sh.spn[i].y) return true;
        return false;
    };
    auto decode = [&](const SEv& r, uint32_t pos) -> JEv {
        JEv x;
        const bool valid = pos < sg.len;
        x.dt = valid ? r.dt : 0;
        x.cz = (uint32_t)r.cnt | ((uint32_t)r.rt << 16);
        x.kf = valid ? ((uint32_t)r.kind | JK_VALID) : 0xFFu;
        if (valid && r.kind == SG_EV_ENTRY && (r.flags & RF_PBLK)) x.kf |= JK_PB;
        x.wi = 0;
        if (valid && r.kind != SG_EV_ENTRY) {
            if (r.code == RC_NONE || r.code == RC_PASSED) x.kf |= JK_VAL;  // the chain exists here
            else if (r.code == RC_BATCH) {
                uint32_t refrel = r.x - sg.start;
                if (refrel >= pos) { atomicOr(bflags, BF_BAD_REF); refrel = 0; }  // not an earlier ENTRY of this resource
                if (refrel + WIN >= tbase + TILE) { x.kf |= JK_WIN; x.wi = refrel & (WIN - 1); }
                else if (!in_span(refrel) &&  // decided >= WIN-TILE positions ago, i.e. before >= 1 full fence
                         st_passed(__hip_atomic_load(&dec[r.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xFF))
                    x.kf |= JK_VAL;
            }
        }
        return x;
    };
    auto load = [&](SEv (&dst)[EP], uint32_t tb) {
#pragma unroll
        for (int e = 0; e < EP; ++e) {
            const uint32_t p = tb + lp0 + (uint32_t)e;
            dst[e].kind = 0xFF;
            if (p < sg.len) dst[e] = recs[sg.start + p];
        }
    };
    // guesses g0 for the tile's events; the window statuses of those at positions >= from
    auto guess_all = [&](uint32_t g0, uint32_t from) {
#pragma unroll
        for (int e = 0; e < EP; ++e) {
            gg[e] = g0;
            if ((ev[e].kf & JK_VALID) && lp0 + (uint32_t)e >= from)
                win[(tbase + lp0 + e) & (WIN - 1)] =
                    ((ev[e].kf & (0xFFu | JK_PB)) == SG_EV_ENTRY && g0 == (uint32_t)nr) ? 1 : 0;
        }
    };
    static_assert(WIN - TILE >= (FULL_FENCE_TILES + 1) * TILE, "old references must be older than one full fence");
    // Decisions committed by the Jacobi iterations wait in registers and are stored when the tile is left:
    // vmcnt counts stores and loads in one in-order counter, so a store issued inside the iterations would
    // make the wait for the next tile's prefetch (whose distance in vector-memory ops the compiler cannot
    // count across the iteration loop) also wait for that store's write acknowledgement.
    uint32_t pdec[EP], pmask = 0;
    auto flush = [&](uint32_t tb) {
#pragma unroll
        for (int e = 0; e < EP; ++e)
            if ((pmask >> e) & 1) dec[sg.start + tb + lp0 + (uint32_t)e] = pdec[e];
        pmask = 0;
    };
    auto advance = [&]() {  // next tile (uniform)
        tbase += TILE;
        // decode first: a (rare) old-reference load must not queue behind the prefetch below,
        // vmcnt retires in order; the finished tile's decisions go out between the two
#pragma unroll
        for (int e = 0; e < EP; ++e) ev[e] = decode(nxt[e], tbase + lp0 + e);
        flush(tbase - TILE);
        load(nxt, tbase + TILE);
        ++n_tile;
        if ((tbase / TILE) % FULL_FENCE_TILES == 0) __syncthreads();  // bound the visibility of dec[] stores
    };
    {
        SEv cur[EP];
        load(cur, 0);
        load(nxt, TILE);
#pragma unroll
        for (int e = 0; e < EP; ++e) ev[e] = decode(cur[e], lp0 + e);
    }
    guess_all((uint32_t)nr, 0);
    if (tid == 0) sh.tnext = t0 + ev[0].dt;
    __syncthreads();
    uint32_t mb = 0;  // mism double-buffer index

    for (;;) {
        uint32_t c0 = uni(sh.c0);
        const uint32_t cnt_t = sg.len - tbase < TILE ? sg.len - tbase : TILE;
        if (c0 >= cnt_t) {  // tile done: advance (uniform)
            if (tbase + TILE >= sg.len) { flush(tbase); break; }
            advance();
            guess_all(sh.last_out, 0);
            lds_barrier();  // everyone has read sh.last_out / sh.c0
            if (tid == 0) { sh.c0 = 0; sh.tnext = t0 + ev[0].dt; }
            lds_barrier();
            c0 = 0;
        }
        ++n_it;
        PROF_MARK(0)
        {  // round check on the event at c0 (uniform)
            const int64_t tn = uni64(sh.tnext);
            const bool need = !uni(sh.round_open) || (tn / 500) != uni64(sh.bkt0) || tn >= uni64(sh.next_reset);
            if (need) {
                PROF_MARK(0)
                lds_barrier();  // every wave has read the round state before the leader rewrites it
                if (tid == 0) {
                    round_fold(sh, C, nf);
                    round_setup(sh, C, nf, nd, tn);
                }
                lds_barrier();
                ++n_round;
                PROF_MARK(6)
            }
        }
        // the round's events: relative times in [dlo, dhi) (its 500 ms bucket, before the next reset)
        const int64_t dlo = uni64(sh.bkt0) * 500 - t0;
        const int64_t nrs = uni64(sh.next_reset) - t0;
        const int64_t dhi = (nrs < dlo + 500) ? nrs : dlo + 500;

        // ================= frozen stretch =================
        // All flow stages are QPS DefaultControllers and either one of them is already saturated
        // for acquire >= 1, or the first breaker is cut: until the round ends no ENTRY can pass, so
        // the pass count and every rule state stay fixed, each verdict is a pure function of the
        // event, and the rest of the round is a map + reduction (one barrier per tile).
        if (frozen_prog) {
            const int64_t Pfix = uni64(sh.bP + sh.cP);
            const int32_t pint = j_d2i((double)Pfix);
            const bool cutk0 = nd > 0 && uni(sh.rs[nf].a != 0);
            // each flow stage's limit in this round: DefaultController count; WarmUp: warningQps above the
            // warning token, else count (the synced state of the round's second)
            double flim[MF];
            auto calc_flim = [&]() {
#pragma unroll
                for (int s = 0; s < MF; ++s) {
                    flim[s] = 0.0;
                    if (s < nf) {
                        const DRule& r = sh.rules[s];
                        flim[s] = r.count;
                        if ((warmm >> s) & 1) {
                            const RState& st = ((sh.has_sync >> s) & 1) ? sh.syn[s] : sh.rs[s];
                            if (st.a >= r.warning_token) flim[s] = warm_qps(r, st.a);
                        }
                    }
                }
            };
            calc_flim();
            // stage s blocks an acquire of c at the round's pass count P
            auto fblock = [&](int s, int64_t P, int c) -> bool {
                return ((warmm >> s) & 1) ? !((double)(P + c) <= flim[s])
                                          : (double)j_iadd(j_d2i((double)P), c) > flim[s];
            };
            bool sat = false;
#pragma unroll
            for (int s = 0; s < MF; ++s)
                if (s < nf) sat |= warmm ? fblock(s, Pfix, 1) : (double)j_iadd(pint, 1) > flim[s];
            sat = uni(sat) != 0;
            if (sat || cutk0) {
                constexpr uint32_t EPL = 4, ST = EPL * HW;  // events per lane, positions per super-tile
                static_assert(WIN - ST >= (FULL_FENCE_TILES + 1) * (ST + HW), "old references must precede a full fence");
                flush(tbase);     // the tile's committed decisions before the stretch
                __syncthreads();  // full fence at every stretch start (see lds_barrier)
                const uint32_t fpos0 = tbase + c0;        // stretch start (segment position)
                double fcount[MF];                        // flow thresholds and verdict words, hoisted
                uint32_t fdec[MF];
#pragma unroll
                for (int s = 0; s < MF; ++s) {
                    fcount[s] = flim[s];
                    fdec[s] = s < nf ? mk_dec(ST_BLOCK_FLOW, sh.rules[s].slot, 0) : 0u;
                }
                uint32_t freach = 0;  // WarmUp stages a committed ENTRY of the stretch reached (token sync persists)
                const uint32_t cdec = nd > 0 ? mk_dec(ST_BLOCK_DEGRADE, sh.rules[nf].slot, 0) : 0u;
                uint32_t aB = 0, aS = 0, aRT = 0, aE = 0, aTI = 0, aMin = NO_LANE, aTH = 0;
                uint32_t fend = 0;
                bool skipped = false;
                // ---- skip: a long stretch is not streamed through this CU.  Its end is found by a
                // block-wide search over event times, its ENTRY counts come from per-block sums (k_block_sums),
                // its effective EXIT/TRACEs are the same-batch EXIT/TRACEs of the passes this owner
                // committed (pending list + forward links) plus the few that count without a link
                // (streamed), and k_fill writes its verdicts after the decide kernels.
                const uint32_t skip_min = S.skip_min * NW / 16 > 0 ? S.skip_min * NW / 16 : 1u;  // scaled to the owner's width
                if (skip_on && sg.len - fpos0 > skip_min && uni(sh.nsp) < NSPAN) {
                    // (1) stretch end E = first position with dt >= dhi (dt is non-decreasing); dt[lo] < dhi.
                    // The first probe round also settles whether the stretch is long enough to skip.
                    uint32_t lo = fpos0, hi = sg.len;
                    bool go = true, first = true;
                    while (hi - lo > 1) {
                        const uint32_t step = (hi - lo + HW - 1) / HW;
                        const uint32_t q = lo + (tid + 1) * step;
                        const bool pr = q < hi && (int64_t)recs[sg.start + q].dt >= dhi;
                        const uint64_t bm = __ballot(pr);
                        if (lane == 0) sh.mism[mb][wv] = bm ? wv * 64 + (uint32_t)(__ffsll((long long)bm) - 1) : NO_LANE;
                        lds_barrier();
                        uint32_t f = NO_LANE;
                        f = blk_min<NW>(sh.mism[mb]);
                        f = uni(f);
                        mb ^= 1;
                        if (f == NO_LANE) {
                            uint32_t kl = (hi - 1 - lo) / step;
                            if (kl > HW) kl = HW;
                            lo += kl * step;
                        } else {
                            hi = lo + (f + 1) * step;
                            lo = lo + f * step;
                        }
                        if (first) {
                            first = false;
                            if (hi <= fpos0 + skip_min) { go = false; break; }  // E <= hi: too short, stream it
                        }
                    }
                    if (go && hi - fpos0 > skip_min) {
                        const uint32_t E = hi;
                        const uint32_t A = sg.start + fpos0, B = sg.start + E;  // absolute positions
                        const uint32_t nch = (B - A + SPAN_CHUNK - 1) / SPAN_CHUNK;
                        // (2) span slots for k_fill; on overflow stream instead (slots already taken are voided)
                        if (tid == 0) {
                            const uint32_t base = atomicAdd(S.nspan, nch);
                            sh.skip_go = base + nch <= S.span_cap ? base : NO_LANE;
                            if (base < S.span_cap && base + nch > S.span_cap)
                                for (uint32_t k = base; k < S.span_cap; ++k) S.spans[k] = Span{0u, 0u, 0u, 0};
                        }
                        lds_barrier();
                        const uint32_t sbase = uni(sh.skip_go);
                        if (sbase != NO_LANE) {
                            skipped = true;
                            fend = E;
                            for (uint32_t c = tid; c < nch; c += HW) {
                                Span sp;
                                sp.s = A + c * SPAN_CHUNK;
                                sp.e = B - sp.s < SPAN_CHUNK ? B : sp.s + SPAN_CHUNK;
                                sp.res = res | (cutk0 ? 0x80000000u : 0u);
                                sp.pint = pint;
                                S.spans[sbase + c] = sp;
                            }
                            // (3) ENTRY counts and link-free EXIT/TRACEs: edge blocks and flagged blocks are
                            // streamed, the other whole blocks contribute their k_block_sums count sums
                            auto stat_ev = [&](uint32_t p) {
                                const uint4 r = reinterpret_cast<const uint4*>(recs)[p];
                                const uint32_t ek = r.w & 0xFFu, ec = r.z & 0xFFFFu, ert = r.z >> 16;
                                const uint32_t code = (r.w >> 16) & 0xFFu;
                                if (ek == SG_EV_ENTRY) { aB += ec; aTI += 1; }
                                else if (code == RC_NONE || code == RC_PASSED) {
                                    if (ek == SG_EV_EXIT) { aS += ec; aRT += ert; aTH -= 1; aMin = op_min(aMin, ert); aTI += 1; }
                                    else if (ec > 0) { aE += ec; aTI += 1; }
                                }
                            };
                            const uint32_t fb = (A + 1023) >> 10, lb = B >> 10;
                            if (fb >= lb) {
                                for (uint32_t p = A + tid; p < B; p += HW) stat_ev(p);
                            } else {
                                for (uint32_t p = A + tid; p < (fb << 10); p += HW) stat_ev(p);
                                for (uint32_t p = (lb << 10) + tid; p < B; p += HW) stat_ev(p);
                                for (uint32_t k0 = fb; k0 < lb; k0 += HW) {
                                    const uint32_t k = k0 + tid;
                                    const uint32_t w = k < lb ? S.bst[k] : 0u;
                                    const bool flg = (w & BST_STATIC) != 0;
                                    if (!flg && (w & BST_CNT)) { aB += w & BST_CNT; aTI += 1; }
                                    const uint64_t bm = __ballot(flg);
                                    if (lane == 0) sh.fl[wv] = bm;
                                    lds_barrier();
                                    for (uint32_t w2 = 0; w2 < (uint32_t)NW; ++w2) {
                                        uint64_t m2 = (uint64_t)uni64((int64_t)sh.fl[w2]);
                                        while (m2) {
                                            const uint32_t b = (uint32_t)(__ffsll((long long)m2) - 1);
                                            m2 &= m2 - 1;
                                            const uint32_t blk = k0 + w2 * 64 + b;
                                            for (uint32_t p = (blk << 10) + tid; p < ((blk + 1) << 10); p += HW) stat_ev(p);
                                        }
                                    }
                                    lds_barrier();  // sh.fl is rewritten by the next chunk
                                }
                            }
                            // (4) pending passes: EXIT/TRACEs inside [A, B) count, those beyond B stay pending
                            const uint32_t np = uni(sh.npend);
                            uint32_t kept = 0;
                            for (uint32_t k0 = 0; k0 < np; k0 += HW) {
                                const uint32_t k = k0 + tid;
                                bool keep = false;
                                uint32_t item = 0;
                                if (k < np) {
                                    item = S.pend[sg.start + k];
                                    const Link L = S.link[sg.start + item];
                                    const uint32_t me = sg.start + item;
                                    if ((uint32_t)(L.exit_l >> 32) == S.epoch) {
                                        const uint32_t x = (uint32_t)L.exit_l;
                                        if (x >= B) keep = true;
                                        else if (x >= A) {
                                            const SEv r = recs[x];
                                            if (r.code == RC_BATCH && r.x == me && r.kind == SG_EV_EXIT) {
                                                aS += r.cnt; aRT += r.rt; aTH -= 1; aMin = op_min(aMin, (uint32_t)r.rt); aTI += 1;
                                            }
                                        }
                                    }
                                    if ((uint32_t)(L.trace_l >> 32) == S.epoch) {
                                        const uint32_t x = (uint32_t)L.trace_l;
                                        if (x >= B) keep = true;
                                        else if (x >= A) {
                                            const SEv r = recs[x];
                                            if (r.code == RC_BATCH && r.x == me && r.kind == SG_EV_TRACE && r.cnt > 0) {
                                                aE += r.cnt; aTI += 1;
                                            }
                                        }
                                    }
                                }
                                const uint64_t km = __ballot(keep);
                                if (lane == 0) sh.mism[mb][wv] = (uint32_t)__popcll(km);
                                lds_barrier();
                                uint32_t tot;
                                const uint32_t before = blk_sum_before<NW>(sh.mism[mb], 1, wv, &tot);
                                mb ^= 1;
                                if (keep) S.pend[sg.start + kept + before + (uint32_t)__popcll(km & lanemask_lt())] = item;
                                kept += uni(tot);
                            }
                            // (5) statuses of the span's ENTRYs as later EXITs see them: blocked
                            {
                                const uint32_t lo2 = (E > WIN && E - WIN > fpos0) ? E - WIN : fpos0;
                                const uint32_t a4 = (lo2 + 3) & ~3u, b4 = E & ~3u;
                                if (a4 <= b4) {
                                    if (tid < a4 - lo2) win[(lo2 + tid) & (WIN - 1)] = 0;
                                    if (tid < E - b4) win[(b4 + tid) & (WIN - 1)] = 0;
                                    uint32_t* w32 = reinterpret_cast<uint32_t*>(win);
                                    for (uint32_t q = a4 / 4 + tid; q < b4 / 4; q += HW) w32[q & (WIN / 4 - 1)] = 0;
                                } else if (tid < E - lo2) {
                                    win[(lo2 + tid) & (WIN - 1)] = 0;
                                }
                            }
                            lds_barrier();  // every wave has read sh.npend / sh.nsp
                            if (tid == 0) {
                                sh.npend = kept;
                                sh.spn[sh.nsp] = make_uint2(fpos0, E);
                                sh.nsp += 1;
                            }
                        }
                    }
                }
                if (!skipped) {
                const uint4* r4 = reinterpret_cast<const uint4*>(recs + sg.start);
                uint4 rr[EPL], rn[EPL];
                uint32_t sb = fpos0, nst = 0;
                // loads are unconditional (clamped index): predicated loads would make the compiler's
                // waitcnt analysis drain the prefetch (vmcnt(0)) before the current tile is touched
                const uint32_t qmax = sg.len - 1;
#pragma unroll
                for (int k = 0; k < (int)EPL; ++k) {
                    const uint32_t q = sb + k * HW + tid;
                    rr[k] = r4[q < qmax ? q : qmax];
                }
                for (;;) {
#pragma unroll
                    for (int k = 0; k < (int)EPL; ++k) {  // prefetch the next super-tile
                        const uint32_t q = sb + ST + k * HW + tid;
                        rn[k] = r4[q < qmax ? q : qmax];
                    }
                    // first position of this lane that cannot be decided frozen
                    uint32_t mystop = NO_LANE;
                    uint32_t fdv[EPL];
#pragma unroll
                    for (int k = 0; k < (int)EPL; ++k) {
                        const uint32_t q = sb + k * HW + tid;
                        const int32_t edt = (int32_t)rr[k].x;
                        const uint32_t ek = rr[k].w & 0xFFu, ec = rr[k].z & 0xFFFFu;
                        const bool in = q < sg.len && edt >= dlo && edt < dhi;
                        const double curv = (double)j_iadd(pint, (int)ec);
                        uint32_t fd = 0;
                        if (!warmm) {
#pragma unroll
                            for (int s = MF - 1; s >= 0; --s)
                                if (s < nf && curv > fcount[s]) fd = fdec[s];
                        } else {
                            const double curw = (double)(Pfix + (int64_t)ec);
#pragma unroll
                            for (int s = MF - 1; s >= 0; --s)
                                if (s < nf && (((warmm >> s) & 1) ? !(curw <= fcount[s]) : curv > fcount[s])) fd = fdec[s];
                        }
                        if (fd == 0 && cutk0) fd = cdec;
                        if ((rr[k].w >> 8) & RF_PBLK) fd = 1u;  // blocked by a param rule: its word is written
                        fdv[k] = fd;
                        const bool stop = q < sg.len && (!in || (ek == SG_EV_ENTRY && fd == 0));
                        if (stop && q < mystop) mystop = q;
                    }
                    uint32_t wmin = mystop;
                    WAVE_SCAN(wmin, NO_LANE, op_min);
                    if (lane == 63) sh.mism[mb][wv] = wmin;
                    lds_barrier();
                    uint32_t f = NO_LANE;
                    f = blk_min<NW>(sh.mism[mb]);
                    f = uni(f);
                    mb ^= 1;
                    ++n_frz;
                    // commit every position before the stop.  The decision stores are unconditional
                    // (masked-off lanes write a per-lane sink word) so vmcnt stays countable.
#pragma unroll
                    for (int k = 0; k < (int)EPL; ++k) {
                        const uint32_t q = sb + k * HW + tid;
                        const bool cm = q < f && q < sg.len;
                        uint32_t d = 0;
                        if (cm) {
                            const uint32_t ek = rr[k].w & 0xFFu, ec = rr[k].z & 0xFFFFu, ert = rr[k].z >> 16;
                            const uint32_t code = (rr[k].w >> 16) & 0xFFu;
                            d = mk_dec(ST_NOT_ENTRY, 0, 0);
                            if (ek == SG_EV_ENTRY) {
                                d = fdv[k];
                                win[q & (WIN - 1)] = 0;
                                aB += ec;
                                aTI += 1;
                                if (warmm && d != 1u) {  // stages up to the blocking one (all flow stages when a breaker blocks)
                                    uint32_t bs = (uint32_t)nf;
#pragma unroll
                                    for (int s = MF - 1; s >= 0; --s)
                                        if (s < nf && d == fdec[s]) bs = (uint32_t)s;
                                    freach |= (2u << bs) - 1u;
                                }
                            } else {
                                bool eff = code == RC_NONE || code == RC_PASSED;
                                if (code == RC_BATCH) {
                                    const uint32_t rel = rr[k].y - sg.start;
                                    if (rel >= q) { atomicOr(bflags, BF_BAD_REF); eff = false; }
                                    else if (rel >= fpos0) eff = false;  // an ENTRY of this stretch: blocked
                                    else if (rel + WIN >= sb + ST) eff = win[rel & (WIN - 1)] != 0;
                                    else eff = !in_span(rel) &&
                                               st_passed(__hip_atomic_load(&dec[rr[k].y], __ATOMIC_RELAXED,
                                                                           __HIP_MEMORY_SCOPE_AGENT) & 0xFF);
                                }
                                win[q & (WIN - 1)] = 0;
                                if (eff && ek == SG_EV_EXIT) {
                                    aS += ec; aRT += ert; aTH -= 1; aMin = op_min(aMin, ert); aTI += 1;
                                } else if (eff && ek == SG_EV_TRACE && ec > 0) {
                                    aE += ec; aTI += 1;
                                }
                            }
                        }
                        *((cm && d != 1u) ? &dec[sg.start + q] : &S.sink[tid]) = d;
                    }
                    if (f != NO_LANE) { fend = f; break; }
                    sb += ST;
                    if (sb >= sg.len) { fend = sg.len; break; }
#pragma unroll
                    for (int k = 0; k < (int)EPL; ++k) rr[k] = rn[k];
                    if (++nst % FULL_FENCE_TILES == 0) __syncthreads();  // bound the visibility of dec[] stores
                }
                }  // !skipped
                PROF_MARK(7)
                if (warmm) {
#pragma unroll
                    for (int s = 0; s < MF; ++s)
                        if (((warmm >> s) & 1) && __ballot((freach >> s) & 1) && lane == 0) atomicOr(&sh.warm_reach, 1u << s);
                }
                // stretch end: reduce the lane accumulators into the round's committed totals
                WAVE_SCAN(aB, 0u, op_add);
                WAVE_SCAN(aS, 0u, op_add);
                WAVE_SCAN(aRT, 0u, op_add);
                WAVE_SCAN(aE, 0u, op_add);
                WAVE_SCAN(aTI, 0u, op_add);
                WAVE_SCAN(aTH, 0u, op_add);
                WAVE_SCAN(aMin, NO_LANE, op_min);
                if (lane == 63) {
                    sh.part[wv][0] = aB; sh.part[wv][1] = aS; sh.part[wv][2] = aRT; sh.part[wv][3] = aE;
                    sh.part[wv][4] = aTI; sh.part[wv][5] = aTH; sh.part[wv][6] = aMin;
                }
                // re-enter the tile machinery at the stop position; guesses = the frozen verdict
                tbase = fend / TILE * TILE;
                c0 = fend - tbase;
                {
                    SEv cur[EP];
                    load(cur, tbase);
                    load(nxt, tbase + TILE);
#pragma unroll
                    for (int e = 0; e < EP; ++e) ev[e] = decode(cur[e], tbase + lp0 + e);
                }
                const uint32_t g = (cutk0 && !sat) ? (uint32_t)nf : 0u;
                guess_all(g, c0);
#pragma unroll
                for (int e = 0; e < EP; ++e)
                    if ((ev[e].kf & JK_VALID) && lp0 + (uint32_t)e == c0) sh.tnext = t0 + ev[e].dt;
                __syncthreads();
                if (tid == 0) {
                    for (uint32_t w = 0; w < (uint32_t)NW; ++w) {
                        sh.cB += sh.part[w][0]; sh.cS += sh.part[w][1]; sh.cRT += sh.part[w][2]; sh.cE += sh.part[w][3];
                        sh.ctouch += sh.part[w][4]; sh.cTH += (int32_t)sh.part[w][5];
                        sh.cminrt = op_min(sh.cminrt, sh.part[w][6]);
                    }
                    sh.last_out = g;
                    sh.c0 = c0;
                }
                lds_barrier();
                PROF_MARK(8)
                continue;
            }

            // ================= open stretch / round machine =================
            // Same program shape, nothing saturated, no breaker cut, and the last committed ENTRY passed:
            // guess that every ENTRY from here on passes.  Under that guess the pass count, the window's
            // success / RT / exception sums and the RT breakers' passCount before an ENTRY are prefix sums
            // of the events before it, so the stretch is decided chunk by chunk at OPEN_EPL events per lane
            // (one chain of scans and barriers per chunk instead of one per tile of Jacobi iterations): every
            // ENTRY is checked against its prefix view in FlowRuleChecker / DegradeRule order, and the first
            // one that does not pass, the first event past the round, or the segment end stops the stretch.
            // Everything before the stop is exact (every earlier ENTRY did pass).
            //
            // The owner's round chain: a hot segment's round is "open until the quota is
            // spent, then frozen until the round ends", and each of those switches used to leave the stretch --
            // a re-entry into the Jacobi tile (its records loaded again), full fences, the next stretch's first
            // chunk loaded again, the leader's round set-up: ~10 dependent memory round trips a round.  Here the
            // stretch keeps going with the chunk already in registers:
            //   * an open stop that is a flow block at a saturated pass count (no acquire of 1 passes any more:
            //     DefaultController.canPass, DefaultController.java:49-81; nothing passes, so the pass count stays)
            //     switches to frozen mode at the stop: every later ENTRY of the round blocks (FlowSlot runs before
            //     DegradeSlot, FlowSlot.java:146-158), a pure map + reduction;
            //   * the first event past the round ends the round in place: the lanes' committed totals are reduced,
            //     the leader folds the round and opens the next one (LDS only: the minute window is in sh.minl),
            //     and the next round goes on frozen (saturated, or the first breaker cut: DegradeRule.java:172-223)
            //     or open (nothing cut) from that event, in the same chunk.
            // Anything else -- a degrade block, a breaker trip, an ENTRY a frozen round could pass, a round that is
            // neither -- leaves the machine into the Jacobi iteration exactly as before, and so does a frozen round
            // that may be longer than the skip threshold, for the frozen-stretch code to skip.  The machine's state
            // lives in LDS (sh.m*: the leader writes it, every lane reads it after a barrier), not in registers.
            // Chunks: open mode reads a chunk lane-blocked (a lane folds OPEN_EPL consecutive events), frozen mode
            // strided (each load instruction one contiguous run of records, as the frozen-stretch loop).
            bool anycut = false;
            if (OPEN) {  // (nothing of this in the owners without open stretches: it sits on every iteration's chain)
#pragma unroll
                for (int k = 0; k < MD; ++k)
                    if (k < nd) anycut |= sh.rs[nf + k].a != 0;
                anycut = uni(anycut ? 1u : 0u) != 0;
            }
            if (OPEN && open_on && !anycut && uni(sh.last_out) == (uint32_t)nr && sg.len - (tbase + c0) >= open_min) {
                constexpr uint32_t OE = OPEN_EPL, OST = OE * HW;
                static_assert(WIN - OST >= (FULL_FENCE_TILES + 1) * (OST + HW), "old references must precede a full fence");
                flush(tbase);
                __syncthreads();  // full fence at every stretch start (see lds_barrier)
                const uint32_t fpos0 = tbase + c0;
                // the owners skip a frozen round from skip_min positions on (the frozen-stretch code does)
                const uint32_t skip_min = S.skip_min * NW / 16 > 0 ? S.skip_min * NW / 16 : 1u;
                // a flow stage's limit in the machine's round (sh.mflim), and whether it blocks an acquire of c at P
                auto mlim = [&](int s) -> double {
                    const uint64_t b = (uint64_t)uni64((int64_t)__builtin_bit_cast(uint64_t, sh.mflim[s]));
                    return __builtin_bit_cast(double, b);
                };
                auto mblock = [&](int s, int64_t P, int c) -> bool {
                    return ((warmm >> s) & 1) ? !((double)(P + c) <= mlim(s)) : (double)j_iadd(j_d2i((double)P), c) > mlim(s);
                };
                auto msat = [&](int64_t P) -> bool {
                    bool r = false;
#pragma unroll
                    for (int s = 0; s < MF; ++s)
                        if (s < nf) r |= mblock(s, P, 1);
                    return r;
                };
                // ---- leader: the machine's round (event times, flow limits), open mode, frozen mode
                auto m_round = [&]() {
                    const int64_t nlo = sh.bkt0 * 500 - t0, nrs = sh.next_reset - t0;
                    const int64_t nhi = (nrs < nlo + 500) ? nrs : nlo + 500;
                    sh.mrlo = (int32_t)nlo;
                    sh.mrhi = nhi > (int64_t)INT32_MAX ? INT32_MAX : (int32_t)nhi;
                    for (int s = 0; s < nf; ++s) {
                        const DRule& r = sh.rules[s];
                        double l = r.count;
                        if ((warmm >> s) & 1) {
                            const RState& st = ((sh.has_sync >> s) & 1) ? sh.syn[s] : sh.rs[s];
                            if (st.a >= r.warning_token) l = warm_qps(r, st.a);
                        }
                        sh.mflim[s] = l;
                    }
                };
                auto m_open = [&](uint32_t from) {
                    sh.mv[0] = sh.bP + sh.cP; sh.mv[1] = sh.bS + sh.cS; sh.mv[2] = sh.bRT + sh.cRT;
                    sh.mv[3] = sh.bE + sh.cE; sh.mv[4] = sh.bEM + sh.cE; sh.mv[5] = sh.bB + sh.cB;
                    for (int k = 0; k < MD; ++k) {
                        sh.mksg[k] = 0;
                        sh.mpcb[k] = k < nd ? (int32_t)sh.rs[nf + k].b : 0;
                    }
                    sh.molo = from;
                    sh.mmode = 0;
                };
                auto m_frozen = [&](uint32_t from, int64_t P) {
                    sh.mfz0 = from;
                    sh.mfzP = P;
                    sh.mfcut = (nd > 0 && sh.rs[nf].a != 0) ? 1u : 0u;
                    sh.mmode = 1;
                };
                auto m_seg = [&]() {  // an open stop's RT passCount state (sh.os_seg) into the breakers
                    for (int k = 0; k < nd; ++k)
                        if (sh.rules[nf + k].grade == SG_DEGRADE_GRADE_RT) {
                            const uint32_t x = sh.os_seg[k];
                            const int32_t cc = (int32_t)(x & 0x7fffffffu);
                            sh.rs[nf + k].b = (x & 0x80000000u) ? cc : sh.rs[nf + k].b + cc;
                        }
                };
                PROF_MARK(0)
                if (tid == 0) {
                    m_round();
                    m_open(fpos0);
                }
                uint32_t aP = 0, aS = 0, aRT = 0, aE = 0, aTI = 0, aTH = 0, aMin = NO_LANE;  // committed (lane)
                uint32_t aB = 0;     // committed blocked units (XF_MIX param blocks; frozen mode: every ENTRY)
                bool oent = false;   // the lane committed a passing ENTRY (WarmUp: every flow stage reached)
                uint32_t freach = 0; // frozen mode: WarmUp stages a committed ENTRY reached
                bool seg_pending = false;  // sh.os_seg holds an open stop's passCount state not in sh.rs yet (uniform)
                bool frz = false;          // the mode (uniform copy of sh.mmode)
                uint32_t g_exit = (uint32_t)nr;
                const uint4* r4 = reinterpret_cast<const uint4*>(recs + sg.start);
                const uint32_t qmax = sg.len - 1;
                uint4 rr[OE], rn[OE];
                uint32_t sb = fpos0, nst = 0, fend = 0;
                uint32_t lay = 0, nlay = 0;  // layout of rr / rn: 0 lane-blocked (open), 1 strided (frozen)
                // a layout's positions are affine in the item k: base + off + k * stride
                auto qoff = [&](uint32_t l) -> uint32_t { return l ? tid : tid * OE; };
                auto qstr = [&](uint32_t l) -> uint32_t { return l ? HW : 1u; };
                auto qpos = [&](uint32_t l, int k) -> uint32_t { return sb + qoff(l) + (uint32_t)k * qstr(l); };
                auto load_chunk = [&](uint4 (&dst)[OE], uint32_t base, uint32_t l) {
                    const uint32_t o = base + qoff(l), st = qstr(l);
#pragma unroll
                    for (int k = 0; k < (int)OE; ++k) {
                        const uint32_t q = o + (uint32_t)k * st;
                        dst[k] = r4[q < qmax ? q : qmax];
                    }
                };
                // the time of the record skip_min (+ a chunk) past the chunk: a frozen round entered in this chunk is
                // long (left to the frozen-stretch code, which skips it) if that record is still in the round
                auto probe_at = [&](uint32_t base) -> int32_t {
                    const uint32_t q = base + OST + skip_min;
                    return q < sg.len ? (int32_t)recs[sg.start + q].dt : INT32_MAX;
                };
                int32_t pr_dt = (MACH && skip_on) ? probe_at(sb) : INT32_MAX, pr_nx = INT32_MAX;
                load_chunk(rr, sb, 0);
                lds_barrier();  // the leader's machine state
                // the lanes' committed totals into the round's (leader), WarmUp reach; accumulators restart
                auto reduce_to_sh = [&]() {
                    if (warmm) {
                        if (__ballot(oent) && lane == 0) atomicOr(&sh.warm_reach, warmm);
#pragma unroll
                        for (int s = 0; s < MF; ++s)
                            if (((warmm >> s) & 1) && __ballot((freach >> s) & 1) && lane == 0) atomicOr(&sh.warm_reach, 1u << s);
                    }
                    WAVE_SCAN(aP, 0u, op_add);
                    WAVE_SCAN(aS, 0u, op_add);
                    WAVE_SCAN(aRT, 0u, op_add);
                    WAVE_SCAN(aE, 0u, op_add);
                    WAVE_SCAN(aTI, 0u, op_add);
                    WAVE_SCAN(aTH, 0u, op_add);
                    WAVE_SCAN(aMin, NO_LANE, op_min);
                    WAVE_SCAN(aB, 0u, op_add);
                    lds_barrier();  // every wave is past its reads of sh.part
                    if (lane == 63) {
                        sh.part[wv][0] = aP; sh.part[wv][1] = aS; sh.part[wv][2] = aRT; sh.part[wv][3] = aE;
                        sh.part[wv][4] = aTI; sh.part[wv][5] = aTH; sh.part[wv][6] = aMin; sh.part[wv][7] = aB;
                    }
                    lds_barrier();
                    if (tid == 0) {
                        for (uint32_t w = 0; w < (uint32_t)NW; ++w) {
                            sh.cP += sh.part[w][0]; sh.cS += sh.part[w][1]; sh.cRT += sh.part[w][2]; sh.cE += sh.part[w][3];
                            sh.ctouch += sh.part[w][4]; sh.cTH += (int32_t)sh.part[w][5];
                            sh.cminrt = op_min(sh.cminrt, sh.part[w][6]);
                            sh.cB += sh.part[w][7];
                        }
                        if (seg_pending) m_seg();
                    }
                    seg_pending = false;
                    aP = aS = aRT = aE = aTI = aTH = aB = 0;
                    aMin = NO_LANE;
                    oent = false;
                    freach = 0;
                };
                // the round of the event at p (time tp) after the current one ended at p: 0 = open from p, 1 = frozen
                // from p, 2 = leave the machine at p
                auto round_next = [&](uint32_t p, int32_t tp) -> uint32_t {
                    reduce_to_sh();
                    if (tid == 0) {
                        round_next_leader(sh, C, nf, nd, t0 + tp);
                        m_round();
                        const int64_t P = sh.bP + sh.cP;
                        bool sat = false, anyc = false;
                        for (int s = 0; s < nf; ++s) {
                            const double l = sh.mflim[s];
                            sat |= ((warmm >> s) & 1) ? !((double)(P + 1) <= l) : (double)j_iadd(j_d2i((double)P), 1) > l;
                        }
                        for (int k = 0; k < nd; ++k) anyc |= sh.rs[nf + k].a != 0;
                        const bool cut0 = nd > 0 && sh.rs[nf].a != 0;
                        if (sat || cut0) {
                            if (pr_dt < sh.mrhi) sh.mmode = 2;  // long: the frozen-stretch code skips it
                            else m_frozen(p, P);
                        } else if (!anyc) m_open(p);
                        else sh.mmode = 2;
                    }
                    lds_barrier();
                    const uint32_t md = uni(sh.mmode);
                    frz = md == 1;
#ifdef SG_KPROF
                    ++m_nround;
#endif
                    PROF_MARK(12)
                    return md;
                };
                for (;;) {
                    nlay = frz ? 1u : 0u;
                    load_chunk(rn, sb + OST, nlay);  // prefetch the next chunk in the current mode's layout
                    if (MACH && skip_on) pr_nx = probe_at(sb + OST);
                    bool leave = false;
                    for (;;) {  // this chunk, in the current mode (again after a mode switch inside it)
                        if (!frz) {
                            // ---------- open mode
                            if (lay) {  // a strided chunk (the round turned open inside it): lane-blocked again
                                load_chunk(rr, sb, 0);
                                lay = 0;
                                if (nlay) { load_chunk(rn, sb + OST, 0); nlay = 0; }
                            }
                            const uint32_t olo = uni(sh.molo);
                            const int32_t rlo = (int32_t)uni((uint32_t)sh.mrlo), rhi = (int32_t)uni((uint32_t)sh.mrhi);
                            // classes under the all-pass guess; 0x80: a stop before evaluation (past the round / segment);
                            // 0: committed already (before olo) or nothing to count
                            uint32_t cl[OE];
                            uint32_t lp = 0, ls = 0, lrt = 0, le = 0, lb = 0;
#pragma unroll
                            for (int k = 0; k < (int)OE; ++k) {
                                const uint32_t q = sb + tid * OE + k;
                                const int32_t edt = (int32_t)rr[k].x;
                                const uint32_t ek = rr[k].w & 0xFFu, ec = rr[k].z & 0xFFFFu;
                                const uint32_t code = (rr[k].w >> 16) & 0xFFu;
                                uint32_t c = 0;
                                if (q < olo) c = 0;
                                else if (q >= sg.len || edt >= rhi || edt < rlo) c = 0x80u;
                                else if (ek == SG_EV_ENTRY) c = ((rr[k].w >> 8) & RF_PBLK) ? JC_PB : JC_ENT;
                                else {
                                    bool eff = code == RC_NONE || code == RC_PASSED;
                                    if (code == RC_BATCH) {
                                        const uint32_t rel = rr[k].y - sg.start;
                                        if (rel >= q) { atomicOr(bflags, BF_BAD_REF); eff = false; }
                                        else if (rel >= olo)  // an ENTRY of this open round: passed, unless a param rule blocked it
                                            eff = !mixp || !((reinterpret_cast<const uint4*>(recs)[rr[k].y].w >> 8) & RF_PBLK);
                                        else if (rel + WIN >= sb + OST) eff = win[rel & (WIN - 1)] != 0;
                                        else eff = !in_span(rel) &&
                                                   st_passed(__hip_atomic_load(&dec[rr[k].y], __ATOMIC_RELAXED,
                                                                               __HIP_MEMORY_SCOPE_AGENT) & 0xFF);
                                    }
                                    if (eff && ek == SG_EV_EXIT) c = JC_XE;
                                    else if (eff && ek == SG_EV_TRACE && ec > 0) c = JC_TE;
                                }
                                cl[k] = c;
                                lp += (c & JC_ENT) ? ec : 0u;
                                ls += (c & JC_XE) ? ec : 0u;
                                lrt += (c & JC_XE) ? (rr[k].z >> 16) : 0u;
                                le += (c & JC_TE) ? ec : 0u;
                                lb += (c & JC_PB) ? ec : 0u;
                            }
                            // block-exclusive prefixes of the lane totals, and the chunk totals
                            uint32_t xp = lp, xs = ls, xrt = lrt, xe = le, xb = lb;
                            WAVE_SCAN(xp, 0u, op_add);
                            WAVE_SCAN(xs, 0u, op_add);
                            WAVE_SCAN(xrt, 0u, op_add);
                            WAVE_SCAN(xe, 0u, op_add);
                            if (mixp) WAVE_SCAN(xb, 0u, op_add);
                            uint32_t tP, tS, tRT, tE, tB = 0;
                            lds_barrier();  // (sh.part may still be read by a reduction of this chunk)
                            if (lane == 63) {
                                sh.part[wv][0] = xp; sh.part[wv][1] = xs; sh.part[wv][2] = xrt; sh.part[wv][3] = xe;
                                sh.part[wv][4] = xb;
                            }
                            lds_barrier();
                            {   // lanes l < NW fetch wave l's totals; a DPP scan gives the waves before wv and the chunk total
                                uint32_t* const xs4[5] = {&xp, &xs, &xrt, &xe, &xb};
                                uint32_t* const ts4[5] = {&tP, &tS, &tRT, &tE, &tB};
#pragma unroll
                                for (int i = 0; i < 5; ++i) {
                                    if (i == 4 && !mixp) break;
                                    uint32_t v = lane < (uint32_t)NW ? sh.part[lane][i] : 0u;
                                    WAVE_SCAN(v, 0u, op_add);
                                    *xs4[i] += wv == 0 ? 0u : (uint32_t)__builtin_amdgcn_readlane((int)v, (int)wv - 1);
                                    *ts4[i] = (uint32_t)__builtin_amdgcn_readlane((int)v, NW - 1);
                                }
                                xp -= lp; xs -= ls; xrt -= lrt; xe -= le; xb -= lb;
                            }
                            // the view before the chunk (after the barriers: the leader's carry of the last chunk)
                            const int64_t P0 = uni64(sh.mv[0]), S0 = uni64(sh.mv[1]), RT0 = uni64(sh.mv[2]);
                            const int64_t E0 = uni64(sh.mv[3]), EM0 = uni64(sh.mv[4]), B0 = uni64(sh.mv[5]);
                            // (the round's flow limits and the RT stages' carry / base, read once a chunk, not per event)
                            double ofl[MF];
                            uint32_t oksg[MD];
                            int32_t opcb[MD];
#pragma unroll
                            for (int s = 0; s < MF; ++s) ofl[s] = s < nf ? mlim(s) : 0.0;
#pragma unroll
                            for (int k = 0; k < MD; ++k) {
                                oksg[k] = uni(sh.mksg[k]);
                                opcb[k] = (int32_t)uni((uint32_t)sh.mpcb[k]);
                            }
                            auto oblock = [&](int s, int64_t P, int c) -> bool {
                                return ((warmm >> s) & 1) ? !((double)(P + c) <= ofl[s])
                                                          : (double)j_iadd(j_d2i((double)P), c) > ofl[s];
                            };
                            // RT breakers: which ENTRYs see an average at the threshold, then the segmented passCount scan
                            uint32_t badb = 0, segl[MD], segt[MD];
#pragma unroll
                            for (int k = 0; k < MD; ++k) segl[k] = segt[k] = 0;
                            if (has_rt) {
                                uint32_t agg[MD];
#pragma unroll
                                for (int k = 0; k < MD; ++k) agg[k] = 0;
                                uint32_t rS = 0, rRT = 0;
#pragma unroll
                                for (int e = 0; e < (int)OE; ++e) {
                                    const int64_t vS = S0 + (int64_t)(xs + rS), vRT = RT0 + (int64_t)(xrt + rRT);
#pragma unroll
                                    for (int k = 0; k < MD; ++k) {
                                        if (k < nd && sh.rules[nf + k].grade == SG_DEGRADE_GRADE_RT) {
                                            const double avg = vS == 0 ? 0.0 : (double)vRT * 1.0 / (double)vS;
                                            const bool bad = !(avg < sh.rules[nf + k].count);
                                            if (bad) badb |= 1u << (e * MD + k);
                                            agg[k] = op_seg(agg[k], (cl[e] & JC_ENT) ? (bad ? 1u : 0x80000000u) : 0u);
                                        }
                                    }
                                    if (cl[e] & JC_XE) { rS += rr[e].z & 0xFFFFu; rRT += rr[e].z >> 16; }
                                }
#pragma unroll
                                for (int k = 0; k < MD; ++k) {
                                    if (k < nd && sh.rules[nf + k].grade == SG_DEGRADE_GRADE_RT) {
                                        uint32_t v = agg[k];
                                        WAVE_SCAN(v, 0u, op_seg);
                                        segl[k] = shr1(v, 0u);
                                        if (lane == 63) sh.pseg[wv][k] = v;
                                    }
                                }
                                lds_barrier();
#pragma unroll
                                for (int k = 0; k < MD; ++k) {
                                    if (k < nd && sh.rules[nf + k].grade == SG_DEGRADE_GRADE_RT) {
                                        uint32_t v = lane < (uint32_t)NW ? sh.pseg[lane][k] : 0u;
                                        WAVE_SCAN(v, 0u, op_seg);
                                        const uint32_t pre = wv == 0 ? 0u : (uint32_t)__builtin_amdgcn_readlane((int)v, (int)wv - 1);
                                        segl[k] = op_seg(pre, segl[k]);
                                        segt[k] = (uint32_t)__builtin_amdgcn_readlane((int)v, NW - 1);
                                    }
                                }
                            }
                            // every ENTRY against its prefix view; the lane's first stop (myo: NO_LANE = past the
                            // round / segment end, else the blocking stage) and the round's pass count before it
                            uint32_t mystop = NO_LANE, myo = NO_LANE, sst[MD];
                            int64_t myP = 0;
                            int32_t myt = 0;
                            uint32_t rp = 0, rs2 = 0, re = 0, rb = 0, rseg[MD];
#pragma unroll
                            for (int k = 0; k < MD; ++k) rseg[k] = sst[k] = 0;
#pragma unroll
                            for (int e = 0; e < (int)OE; ++e) {
                                const uint32_t c = cl[e];
                                const uint32_t ec = rr[e].z & 0xFFFFu;
                                const int64_t vP = P0 + (int64_t)(xp + rp);
                                uint32_t o = (uint32_t)nr;
                                if (c & 0x80u) o = NO_LANE;
                                else if (c & JC_ENT) {
                                    const int64_t vS = S0 + (int64_t)(xs + rs2);
#pragma unroll
                                    for (int s = 0; s < MF; ++s)
                                        if (s < nf && o == (uint32_t)nr && oblock(s, vP, (int)ec)) o = (uint32_t)s;
#pragma unroll
                                    for (int k = 0; k < MD; ++k) {
                                        if (k < nd && o == (uint32_t)nr) {
                                            const DRule& r = sh.rules[nf + k];
                                            bool ok = true;
                                            if (r.grade == SG_DEGRADE_GRADE_RT) {
                                                const uint32_t x = op_seg(oksg[k], op_seg(segl[k], rseg[k]));
                                                const int32_t cc = (int32_t)(x & 0x7fffffffu);
                                                const int32_t pcb = (x & 0x80000000u) ? cc : opcb[k] + cc;
                                                ok = !((badb >> (e * MD + k)) & 1) || (pcb + 1 < 5);
                                            } else if (r.grade == SG_DEGRADE_GRADE_EXCEPTION_RATIO) {
                                                const double exc = (double)(E0 + (int64_t)(xe + re)) / 1.0;
                                                const double succ = (double)vS / 1.0;
                                                const double total = (double)vP / 1.0 + (double)(B0 + (int64_t)(xb + rb)) / 1.0;
                                                if (total < 5) ok = true;
                                                else if (succ - exc <= 0 && exc < 5) ok = true;
                                                else ok = exc / succ < r.count;
                                            } else if (r.grade == SG_DEGRADE_GRADE_EXCEPTION_COUNT) {
                                                ok = (double)(EM0 + (int64_t)(xe + re)) < r.count;
                                            }
                                            if (!ok) o = (uint32_t)(nf + k);
                                        }
                                    }
                                }
                                if (o != (uint32_t)nr && mystop == NO_LANE) {
                                    mystop = sb + tid * OE + (uint32_t)e;
                                    myo = o;
                                    myP = vP;
                                    myt = (int32_t)rr[e].x;
#pragma unroll
                                    for (int k = 0; k < MD; ++k) sst[k] = rseg[k];
                                }
                                rp += (c & JC_ENT) ? ec : 0u;
                                rs2 += (c & JC_XE) ? ec : 0u;
                                re += (c & JC_TE) ? ec : 0u;
                                rb += (c & JC_PB) ? ec : 0u;
                                if (has_rt) {
#pragma unroll
                                    for (int k = 0; k < MD; ++k)
                                        if (k < nd && sh.rules[nf + k].grade == SG_DEGRADE_GRADE_RT)
                                            rseg[k] = op_seg(rseg[k], (c & JC_ENT) ? (((badb >> (e * MD + k)) & 1) ? 1u : 0x80000000u) : 0u);
                                }
                            }
                            uint32_t wmin = mystop;
                            WAVE_SCAN(wmin, NO_LANE, op_min);
                            if (lane == 63) sh.mism[mb][wv] = wmin;
                            lds_barrier();
                            uint32_t f = NO_LANE;
                            f = blk_min<NW>(sh.mism[mb]);
                            f = uni(f);
                            mb ^= 1;
                            ++n_opn;
                            // commit every position of the round before the stop (unconditional stores: masked lanes hit the sink)
                            uint32_t appm = 0;
#pragma unroll
                            for (int k = 0; k < (int)OE; ++k) {
                                const uint32_t q = sb + tid * OE + k;
                                const bool cm = q >= olo && q < f && q < sg.len;
                                const uint32_t c = cl[k];
                                uint32_t d = 0;
                                if (cm) {
                                    const uint32_t ec = rr[k].z & 0xFFFFu, ert = rr[k].z >> 16;
                                    if (c & JC_ENT) {
                                        d = mk_dec(ST_PASS, 0, 0);
                                        win[q & (WIN - 1)] = 1;
                                        aP += ec; aTI += 1; aTH += 1;
                                        oent = true;
                                        appm |= 1u << k;
                                    } else {
                                        d = mk_dec(ST_NOT_ENTRY, 0, 0);
                                        win[q & (WIN - 1)] = 0;
                                        if (c & JC_XE) { aS += ec; aRT += ert; aTH -= 1; aMin = op_min(aMin, ert); aTI += 1; }
                                        else if (c & JC_TE) { aE += ec; aTI += 1; }
                                        else if (c & JC_PB) { aB += ec; aTI += 1; }
                                    }
                                }
                                *((cm && !(c & JC_PB)) ? &dec[sg.start + q] : &S.sink[tid]) = d;
                            }
                            if (skip_on) {  // committed passes join the pending list (their EXIT/TRACE may fall in a skipped span)
                                const uint32_t na = (uint32_t)__popc(appm);
                                uint32_t incl = na;
                                WAVE_SCAN(incl, 0u, op_add);
                                const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
                                if (tot) {
                                    uint32_t base = 0;
                                    if (lane == 0) base = atomicAdd(&sh.npend, tot);
                                    base = (uint32_t)__shfl((int)base, 0, 64) + incl - na;
#pragma unroll
                                    for (int k = 0; k < (int)OE; ++k)
                                        if ((appm >> k) & 1) S.pend[sg.start + base++] = sb + tid * OE + k;
                                }
                            }
#ifdef SG_KPROF
                            ++m_nopen;
#endif
                            PROF_MARK(10)
                            if (f == NO_LANE) {  // the chunk is committed: the leader carries the view into the next one
                                if (tid == 0) {
                                    sh.mv[0] += tP; sh.mv[1] += tS; sh.mv[2] += tRT; sh.mv[3] += tE; sh.mv[4] += tE; sh.mv[5] += tB;
#pragma unroll
                                    for (int k = 0; k < MD; ++k)
                                        if (k < nd) sh.mksg[k] = op_seg(sh.mksg[k], segt[k]);
                                }
                                break;
                            }
                            if (mystop == f) {  // the lane holding the stop
                                sh.os_o = myo;
                                sh.os_P = myP;
                                sh.os_t = myt;
#pragma unroll
                                for (int k = 0; k < MD; ++k) sh.os_seg[k] = op_seg(oksg[k], op_seg(segl[k], sst[k]));
                            }
                            lds_barrier();
                            seg_pending = true;
                            const uint32_t o_f = uni(sh.os_o);
                            if (f >= sg.len) { fend = sg.len; g_exit = (uint32_t)nr; leave = true; break; }
                            if (MACH && o_f == NO_LANE) {  // the round ended: the next one from f, in this chunk
                                if (round_next(f, (int32_t)uni((uint32_t)sh.os_t)) == 2u) {
                                    fend = f; g_exit = (uint32_t)nr; leave = true; break;
                                }
                                continue;
                            }
                            const int64_t Pf = uni64(sh.os_P);
                            if (MACH && o_f < (uint32_t)nf && msat(Pf) && pr_dt >= (int32_t)uni((uint32_t)sh.mrhi)) {
                                // the quota is spent: frozen until the round ends
                                if (tid == 0) {
                                    m_seg();
                                    m_frozen(f, Pf);
                                }
                                seg_pending = false;
                                frz = true;
                                lds_barrier();
                                continue;
                            }
                            fend = f;
                            g_exit = o_f == NO_LANE ? (uint32_t)nr : o_f;
                            leave = true;
                            break;
                        }
                        // ---------- frozen mode: positions [max(sb, fz0), sb + OST) of the round; a stop at the first
                        // event past the round (or an ENTRY that could pass: an acquire of 0)
                        const uint32_t fz0 = uni(sh.mfz0);
                        const int64_t fzP = uni64(sh.mfzP);
                        const bool fcut = uni(sh.mfcut) != 0;
                        const int32_t rlo = (int32_t)uni((uint32_t)sh.mrlo), rhi = (int32_t)uni((uint32_t)sh.mrhi);
                        const int32_t fzi = j_d2i((double)fzP);
                        const double fzd = (double)fzP;
                        double fl[MF];
#pragma unroll
                        for (int s = 0; s < MF; ++s) fl[s] = s < nf ? mlim(s) : 0.0;
                        uint32_t mystop = NO_LANE, myk = 0;
                        int32_t myt = 0;
                        uint32_t fdv[OE], fbs[OE];
#pragma unroll
                        for (int k = 0; k < (int)OE; ++k) {
                            const uint32_t q = qpos(lay, k);
                            const int32_t edt = (int32_t)rr[k].x;
                            const uint32_t ek = rr[k].w & 0xFFu, ec = rr[k].z & 0xFFFFu;
                            const bool act = q >= fz0 && q < sg.len;
                            const bool in = edt >= rlo && edt < rhi;
                            const double curv = (double)j_iadd(fzi, (int)ec);
                            uint32_t bs = (uint32_t)nf;  // the blocking flow stage (nf: none)
#pragma unroll
                            for (int s = MF - 1; s >= 0; --s)
                                if (s < nf && (((warmm >> s) & 1) ? !(fzd + (double)ec <= fl[s]) : curv > fl[s])) bs = (uint32_t)s;
                            uint32_t fd = bs < (uint32_t)nf ? mk_dec(ST_BLOCK_FLOW, sh.rules[bs].slot, 0)
                                                            : (fcut ? mk_dec(ST_BLOCK_DEGRADE, sh.rules[nf].slot, 0) : 0u);
                            if ((rr[k].w >> 8) & RF_PBLK) fd = 1u;  // blocked by a param rule: its word is written
                            fdv[k] = fd;
                            fbs[k] = bs;
                            const bool stop = act && (!in || (ek == SG_EV_ENTRY && fd == 0));
                            if (stop && q < mystop) { mystop = q; myk = in ? 1u : 0u; myt = edt; }
                        }
                        uint32_t wmin = mystop;
                        WAVE_SCAN(wmin, NO_LANE, op_min);
                        if (lane == 63) sh.mism[mb][wv] = wmin;
                        lds_barrier();
                        uint32_t f = NO_LANE;
                        f = blk_min<NW>(sh.mism[mb]);
                        f = uni(f);
                        mb ^= 1;
                        ++n_frz;
#pragma unroll
                        for (int k = 0; k < (int)OE; ++k) {
                            const uint32_t q = qpos(lay, k);
                            const bool cm = q >= fz0 && q < f && q < sg.len;
                            uint32_t d = 0;
                            if (cm) {
                                const uint32_t ek = rr[k].w & 0xFFu, ec = rr[k].z & 0xFFFFu, ert = rr[k].z >> 16;
                                const uint32_t code = (rr[k].w >> 16) & 0xFFu;
                                d = mk_dec(ST_NOT_ENTRY, 0, 0);
                                if (ek == SG_EV_ENTRY) {
                                    d = fdv[k];
                                    win[q & (WIN - 1)] = 0;
                                    aB += ec;
                                    aTI += 1;
                                    // WarmUp: the stages up to the blocking one (every flow stage when a breaker blocks)
                                    if (warmm && d != 1u) freach |= (2u << fbs[k]) - 1u;
                                } else {
                                    bool eff = code == RC_NONE || code == RC_PASSED;
                                    if (code == RC_BATCH) {
                                        const uint32_t rel = rr[k].y - sg.start;
                                        if (rel >= q) { atomicOr(bflags, BF_BAD_REF); eff = false; }
                                        else if (rel >= fz0) eff = false;  // an ENTRY of the frozen part: blocked
                                        else if (rel + WIN >= sb + OST) eff = win[rel & (WIN - 1)] != 0;
                                        else eff = !in_span(rel) &&
                                                   st_passed(__hip_atomic_load(&dec[rr[k].y], __ATOMIC_RELAXED,
                                                                               __HIP_MEMORY_SCOPE_AGENT) & 0xFF);
                                    }
                                    win[q & (WIN - 1)] = 0;
                                    if (eff && ek == SG_EV_EXIT) {
                                        aS += ec; aRT += ert; aTH -= 1; aMin = op_min(aMin, ert); aTI += 1;
                                    } else if (eff && ek == SG_EV_TRACE && ec > 0) {
                                        aE += ec; aTI += 1;
                                    }
                                }
                            }
                            *((cm && d != 1u) ? &dec[sg.start + q] : &S.sink[tid]) = d;
                        }
#ifdef SG_KPROF
                        ++m_nfrz;
#endif
                        PROF_MARK(11)
                        if (f == NO_LANE) break;  // the chunk is committed
                        if (mystop == f) { sh.os_o = myk; sh.os_t = myt; }
                        lds_barrier();
                        if (uni(sh.os_o) == 0u) {  // past the round: the next one from f, in this chunk
                            if (round_next(f, (int32_t)uni((uint32_t)sh.os_t)) == 2u) {
                                fend = f; g_exit = (uint32_t)nr; leave = true; break;
                            }
                            continue;
                        }
                        fend = f;  // an ENTRY that could pass: the Jacobi iteration from it
                        g_exit = (uint32_t)nr;
                        leave = true;
                        break;
                    }
                    if (leave) break;
                    sb += OST;
                    if (sb >= sg.len) {
                        fend = sg.len;
                        g_exit = frz ? ((uni(sh.mfcut) && !msat(uni64(sh.mfzP))) ? (uint32_t)nf : 0u) : (uint32_t)nr;
                        break;
                    }
#pragma unroll
                    for (int k = 0; k < (int)OE; ++k) rr[k] = rn[k];
                    lay = nlay;
                    pr_dt = pr_nx;
                    if (++nst % FULL_FENCE_TILES == 0) __syncthreads();  // bound the visibility of dec[] stores
                }
                // leave the machine: lane accumulators into the round's committed totals, then re-enter the tile
                // machinery at fend with the guess g_exit
                if (warmm) {
                    if (__ballot(oent) && lane == 0) atomicOr(&sh.warm_reach, warmm);
#pragma unroll
                    for (int s = 0; s < MF; ++s)
                        if (((warmm >> s) & 1) && __ballot((freach >> s) & 1) && lane == 0) atomicOr(&sh.warm_reach, 1u << s);
                }
                WAVE_SCAN(aP, 0u, op_add);
                WAVE_SCAN(aS, 0u, op_add);
                WAVE_SCAN(aRT, 0u, op_add);
                WAVE_SCAN(aE, 0u, op_add);
                WAVE_SCAN(aTI, 0u, op_add);
                WAVE_SCAN(aTH, 0u, op_add);
                WAVE_SCAN(aMin, NO_LANE, op_min);
                WAVE_SCAN(aB, 0u, op_add);
                lds_barrier();  // sh.part's chunk exchange is read; sh.os_* is written
                if (lane == 63) {
                    sh.part[wv][0] = aP; sh.part[wv][1] = aS; sh.part[wv][2] = aRT; sh.part[wv][3] = aE;
                    sh.part[wv][4] = aTI; sh.part[wv][5] = aTH; sh.part[wv][6] = aMin; sh.part[wv][7] = aB;
                }
                const uint32_t g = g_exit;
                tbase = fend / TILE * TILE;
                c0 = fend - tbase;
                {
                    SEv cur[EP];
                    load(cur, tbase);
                    load(nxt, tbase + TILE);
#pragma unroll
                    for (int e = 0; e < EP; ++e) ev[e] = decode(cur[e], tbase + lp0 + e);
                }
                guess_all(g, c0);
#pragma unroll
                for (int e = 0; e < EP; ++e)
                    if ((ev[e].kf & JK_VALID) && lp0 + (uint32_t)e == c0) sh.tnext = t0 + ev[e].dt;
                __syncthreads();
                if (tid == 0) {
                    for (uint32_t w = 0; w < (uint32_t)NW; ++w) {
                        sh.cP += sh.part[w][0]; sh.cS += sh.part[w][1]; sh.cRT += sh.part[w][2]; sh.cE += sh.part[w][3];
                        sh.ctouch += sh.part[w][4]; sh.cTH += (int32_t)sh.part[w][5];
                        sh.cminrt = op_min(sh.cminrt, sh.part[w][6]);
                        sh.cB += sh.part[w][7];
                    }
                    if (seg_pending) m_seg();
                    sh.last_out = g;
                    sh.c0 = c0;
                }
                lds_barrier();
                PROF_MARK(13)  // (SG_KPROF: the machine's exit into the tile machinery)
                continue;
            }
        }

        // ================= closed-form guesses of single-stage programs =================
        // A guess only steers how many iterations a tile takes (every verdict is still verified below), but the
        // default re-guess -- every later ENTRY takes the pivot's outcome -- costs two iterations per admission
        // when admissions are sparse and state-driven: a saturated THREAD-grade DefaultController admits one
        // ENTRY per freed thread, a saturated RateLimiter one per `cost` ms (C3's hottest resources).  Both
        // admission sequences have closed forms given the statuses the guesses imply, so the uncommitted ENTRYs
        // of the round are re-guessed with them at the start of every iteration (all in-round ENTRYs acquire 1).
        //   THREAD (DefaultController.java:49-81): thread before ENTRY e = th_c + P(e) - X(e) (P passes, X effective
        //   exits since c0); it passes iff P(e) < Z(e) = max(0, cap - th_c + X(e)) with Z non-decreasing, so
        //   P(e + 1) = min(P(e) + 1, Z(e)), P(n) = E(n) + min(0, min_{j < n} W(j)), W(j) = Z(j) - E(j + 1)
        //   (E: ENTRYs since c0): e passes iff W(e) >= min(0, min_{j < e} W(j)) -- a prefix-min scan.
        //   RateLimiter (RateLimiterController.java:46-91): saturated, the k-th admission after the committed
        //   latestPassedTime L is the first ENTRY with t >= L + k * cost - maxQueue: e passes iff
        //   q(t_e) > q(t of the previous ENTRY), q(t) = max(0, floor((t - L + maxQueue) / cost)).
        // THREAD grade: an EXIT frees a thread only if its ENTRY passed, and in a hot segment half the EXITs name an
        // ENTRY of the same tile (RT ~ Exp(20 ms) against a tile spanning ~16 ms), so the admissions of one pass feed
        // the next: the closed form is re-run on its own guesses (TG_PASSES times) before the Jacobi iteration checks it.
        const int cf_passes = tg_mode ? TG_PASSES : 1;
        for (int cfp = 0; EP == 1 && (tg_mode || rl_mode) && cfp < cf_passes; ++cfp) {
            const uint32_t kf = ev[0].kf, kind = kf & 0xFFu;
            const bool inr = (kf & JK_VALID) && lp0 >= c0 && ev[0].dt >= dlo && ev[0].dt < dhi;
            const bool eff = (kf & JK_WIN) ? (win[ev[0].wi] != 0) : ((kf & JK_VAL) != 0);
            const uint32_t a = (inr && kind == SG_EV_ENTRY) ? 1u : 0u;
            const uint32_t x = (inr && kind == SG_EV_EXIT && eff) ? 1u : 0u;
            const uint32_t bad = (a && (ev[0].cz & 0xFFFFu) != 1u) ? 1u : 0u;
            uint32_t ia = a, ix = tg_mode ? x : (a ? (uint32_t)(ev[0].dt - dlo) + 1u : 0u), ib = bad;
            WAVE_SCAN(ia, 0u, op_add);
            if (tg_mode) WAVE_SCAN(ix, 0u, op_add);
            else WAVE_SCAN(ix, 0u, op_max);
            WAVE_SCAN(ib, 0u, op_add);
            if (lane == 63) { sh.cg[wv][0] = ia; sh.cg[wv][1] = ix; sh.cg[wv][2] = ib; }
            lds_barrier();
            uint32_t pa = 0, px = 0, tb = 0;
            if (NW > 1) {
                uint32_t t0u;
                pa = blk_sum_before<NW>(&sh.cg[0][0], 3, wv, &t0u);
                (void)blk_sum_before<NW>(&sh.cg[0][2], 3, wv, &tb);
                uint32_t v = lane < (uint32_t)NW ? sh.cg[lane][1] : 0u;
                if (tg_mode) ROW_SCAN(v, 0u, op_add, NW);
                else ROW_SCAN(v, 0u, op_max, NW);
                px = wv == 0 ? 0u : (uint32_t)__builtin_amdgcn_readlane((int)v, (int)wv - 1);
            } else {
                tb = sh.cg[0][2];
            }
            const bool use = uni(tb) == 0;
            bool g = false;  // the closed-form outcome of this lane's ENTRY (pass)
            if (use && tg_mode) {
                const int64_t th_c = uni64(sh.bTH + sh.cTH);
                const double cnt_thr = sh.rules[0].count;
                const int64_t cap = cnt_thr <= 0 ? 0 : (cnt_thr >= 2147483647.0 ? 2147483647 : (int64_t)cnt_thr);
                const int64_t Xb = (int64_t)(px + ix - x);        // effective exits strictly before e
                const int64_t Ain = (int64_t)(pa + ia);           // ENTRYs up to and including e
                int64_t Z = cap - th_c + Xb;
                if (Z < 0) Z = 0;
                int64_t W = inr ? Z - Ain : (int64_t)0x3FFFFFFF;
                W = W > 0x3FFFFFFF ? 0x3FFFFFFF : W < -0x3FFFFFFF ? -0x3FFFFFFF : W;
                const uint32_t wb = (uint32_t)(W + 0x40000000LL);  // biased for an unsigned min scan
                uint32_t m = wb;
                WAVE_SCAN(m, 0xFFFFFFFFu, op_min);
                if (lane == 63) sh.cgm[wv] = m;
                const uint32_t mex = shr1(m, 0xFFFFFFFFu);
                lds_barrier();
                uint32_t pm = 0xFFFFFFFFu;
                if (NW > 1) {
                    uint32_t v = lane < (uint32_t)NW ? sh.cgm[lane] : 0xFFFFFFFFu;
                    ROW_SCAN(v, 0xFFFFFFFFu, op_min, NW);
                    pm = wv == 0 ? 0xFFFFFFFFu : (uint32_t)__builtin_amdgcn_readlane((int)v, (int)wv - 1);
                }
                const uint32_t me = op_min(pm, mex);
                const int64_t M = me == 0xFFFFFFFFu ? 0 : ((int64_t)me - 0x40000000LL < 0 ? (int64_t)me - 0x40000000LL : 0);
                g = W >= M;
            } else if (use) {
                const DRule& r = sh.rules[0];
                const RState& st = ((sh.has_sync >> 0) & 1) ? sh.syn[0] : sh.rs[0];
                const int64_t cost = rl_cost(r, st, 1);
                const int64_t L = sh.rs[0].c, mq = r.max_queue;
                auto q = [&](int64_t tt) -> int64_t {
                    const int64_t d = tt - L + mq;
                    return (d < 0 || cost <= 0) ? 0 : d / cost;
                };
                const uint32_t pv = shr1(ix, 0u);                  // previous in-round ENTRY's time (+1), 0: none
                const uint32_t pprev = op_max(px, pv);
                const int64_t qe = q(t0 + ev[0].dt);
                const int64_t qp = pprev ? q(t0 + dlo + (int64_t)pprev - 1) : 0;
                g = cost > 0 && r.count > 0 ? qe > qp : r.count > 0;
            }
            if (use && a) {
                gg[0] = g ? (uint32_t)nr : 0u;
                win[(tbase + lp0) & (WIN - 1)] = g ? 1 : 0;
            }
            lds_barrier();  // the statuses the guesses imply, before the iteration reads them
        }

        // ================= Jacobi iteration =================
        const uint32_t has_sync = sh.has_sync;
        uint32_t cls[EP];  // JC_* of each event under the current guesses
#pragma unroll
        for (int e = 0; e < EP; ++e) {
            const uint32_t kf = ev[e].kf, kind = kf & 0xFFu;
            const bool inr = (kf & JK_VALID) && lp0 + (uint32_t)e >= c0 && ev[e].dt >= dlo && ev[e].dt < dhi;
            const bool eff = (kf & JK_WIN) ? (win[ev[e].wi] != 0) : ((kf & JK_VAL) != 0);
            uint32_t c = 0;
            if (inr) {
                c = JC_INR;
                if (kind == SG_EV_ENTRY) c |= (kf & JK_PB) ? JC_PB : JC_ENT;
                else if (kind == SG_EV_EXIT && eff) c |= JC_XE;
                else if (kind == SG_EV_TRACE && eff && (ev[e].cz & 0xFFFFu) > 0) c |= JC_TE;
            }
            cls[e] = c;
        }

        // ---- phase B: counter deltas under the guesses: lane totals, wave scans
        uint32_t ex[NQ], tq[NQ];
        jac_zero<NQ>(tq);
#pragma unroll
        for (int e = 0; e < EP; ++e) {
            uint32_t q[NQ];
            jac_q<NQ>(q, cls[e], gg[e], ev[e].cz, (uint32_t)nr, (uint32_t)nf);
            jac_acc<NQ>(tq, q);
        }
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            uint32_t v = tq[k];
            if (k == Q_MIN) {
                WAVE_SCAN(v, NO_LANE, op_min);
                ex[k] = shr1(v, NO_LANE);
            } else {
                WAVE_SCAN(v, 0u, op_add);
                ex[k] = v - tq[k];
            }
            if (NW > 1 && lane == 63) sh.part[wv][k] = v;  // one wave: its prefixes are the block's
        }
        // rate limiters: exclusive prefix of the costs (C) and the max-plus term (M) of updating events
        // before the lane (a lane folds its own events: local cost sum, max of t - local inclusive cost)
        int64_t rl_C[2] = {0, 0}, rl_M[2] = {NEG_INF64, NEG_INF64};
        if (RL) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int s = k == 0 ? rl_s0 : rl_s1;
                if (s >= 0) {
                    const DRule& r = sh.rules[s];
                    const RState& st = ((has_sync >> s) & 1) ? sh.syn[s] : sh.rs[s];
                    int64_t cl = 0, ml = NEG_INF64;
#pragma unroll
                    for (int e = 0; e < EP; ++e) {
                        const int cnt = (int)(ev[e].cz & 0xFFFFu);
                        if (rl_upd(r, cls[e], gg[e], s, cnt)) {
                            cl += rl_cost(r, st, cnt);
                            const int64_t v = t0 + ev[e].dt - cl;
                            ml = v > ml ? v : ml;
                        }
                    }
                    const int64_t ci = wscan_i64_add(cl);
                    const int64_t mi = wscan_i64_max(ml == NEG_INF64 ? NEG_INF64 : ml - (ci - cl));
                    if (lane == 63) { sh.prl[wv][2 * k] = ci; sh.prl[wv][2 * k + 1] = mi; }
                    rl_C[k] = ci - cl;
                    const int64_t me = __shfl_up(mi, 1, 64);
                    rl_M[k] = lane == 0 ? NEG_INF64 : me;
                }
            }
        }
        PROF_MARK(1)
        lds_barrier();  // B2
        PROF_MARK(2)
        uint32_t inr_total;
        if (NW == 1) {  // lane 63's inclusive in-round count
            inr_total = (uint32_t)__builtin_amdgcn_readlane((int)((ex[Q_TI] + tq[Q_TI]) >> 16), 63);
        } else {
            // block-wide: lanes l < NW fetch wave l's totals; a DPP scan gives the waves before wv
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                const uint32_t ident = k == Q_MIN ? NO_LANE : 0u;
                uint32_t v = lane < (uint32_t)NW ? sh.part[lane][k] : ident;
                uint32_t incl = v;
                if (k == Q_MIN) WAVE_SCAN(incl, NO_LANE, op_min);
                else WAVE_SCAN(incl, 0u, op_add);
                const uint32_t pre = wv == 0 ? ident : (uint32_t)__builtin_amdgcn_readlane((int)incl, (int)wv - 1);
                ex[k] = k == Q_MIN ? op_min(pre, ex[k]) : ex[k] + pre;
                if (k == Q_TI) inr_total = (uint32_t)__builtin_amdgcn_readlane((int)incl, NW - 1) >> 16;
            }
        }
        if (RL) {
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int s = k == 0 ? rl_s0 : rl_s1;
                if (s >= 0) {
                    int64_t cb = 0, mbx = NEG_INF64;
                    for (uint32_t w = 0; w < wv; ++w) {
                        const int64_t cw = sh.prl[w][2 * k], mw = sh.prl[w][2 * k + 1];
                        if (mw != NEG_INF64 && mw - cb > mbx) mbx = mw - cb;
                        cb += cw;
                    }
                    const int64_t ml = rl_M[k] == NEG_INF64 ? NEG_INF64 : rl_M[k] - cb;
                    rl_M[k] = ml > mbx ? ml : mbx;
                    rl_C[k] += cb;
                }
            }
        }

        // ---- phase C: RT breakers' passCount (segmented scan over the events that check them).  An
        // event's RT average (its view of succ/rt) decides whether it counts or resets: the lane walks its
        // events for those bits, then scans its segmented total.
        uint32_t cutm = 0;  // per degrade stage: the breaker is cut at the round's start
#pragma unroll
        for (int k = 0; k < MD; ++k)
            if (k < nd && sh.rs[nf + k].a) cutm |= 1u << k;
        uint32_t badb = 0;   // bit e * MD + k: stage k's RT average is at its threshold in event e's view
        uint32_t segl[MD];   // RT stages: the segmented count before the lane
#pragma unroll
        for (int k = 0; k < MD; ++k) segl[k] = 0;
        if (has_rt) {
            uint32_t agg[MD];
#pragma unroll
            for (int k = 0; k < MD; ++k) agg[k] = 0;
            uint32_t rS = 0, rRT = 0;
#pragma unroll
            for (int e = 0; e < EP; ++e) {
                const int64_t vS = sh.bS + sh.cS + (int64_t)(ex[Q_S] + rS);
                const int64_t vRT = sh.bRT + sh.cRT + (int64_t)(ex[Q_RT] + rRT);
#pragma unroll
                for (int k = 0; k < MD; ++k) {
                    if (k < nd && sh.rules[nf + k].grade == SG_DEGRADE_GRADE_RT) {
                        const double avg = vS == 0 ? 0.0 : (double)vRT * 1.0 / (double)vS;
                        const bool bad = !(avg < sh.rules[nf + k].count);
                        if (bad) badb |= 1u << (e * MD + k);
                        const bool chk = (cls[e] & JC_ENT) && gg[e] >= (uint32_t)(nf + k);
                        agg[k] = op_seg(agg[k], chk ? (bad ? 1u : 0x80000000u) : 0u);
                    }
                }
                if (cls[e] & JC_XE) { rS += ev[e].cz & 0xFFFFu; rRT += ev[e].cz >> 16; }
            }
#pragma unroll
            for (int k = 0; k < MD; ++k) {
                if (k < nd && sh.rules[nf + k].grade == SG_DEGRADE_GRADE_RT) {
                    uint32_t v = agg[k];
                    WAVE_SCAN(v, 0u, op_seg);
                    segl[k] = shr1(v, 0u);
                    if (lane == 63) sh.pseg[wv][k] = v;
                }
            }
            lds_barrier();  // B3
#pragma unroll
            for (int k = 0; k < MD; ++k) {
                if (k < nd && sh.rules[nf + k].grade == SG_DEGRADE_GRADE_RT) {
                    if (NW > 1) {  // one wave: its prefixes are the block's
                        uint32_t v = lane < (uint32_t)NW ? sh.pseg[lane][k] : 0u;
                        ROW_SCAN(v, 0u, op_seg, NW);
                        const uint32_t pre = wv == 0 ? 0u : (uint32_t)__builtin_amdgcn_readlane((int)v, (int)wv - 1);
                        segl[k] = op_seg(pre, segl[k]);
                    }
                }
            }
        }

        // ---- the lane's running sums over its own events (the view of event e = block prefix + run)
        uint32_t run[NQ], rseg[MD];
        int64_t lc[2], lm[2];
        auto run_reset = [&]() {
            jac_zero<NQ>(run);
#pragma unroll
            for (int k = 0; k < MD; ++k) rseg[k] = 0;
            lc[0] = lc[1] = 0;
            lm[0] = lm[1] = NEG_INF64;
        };
        auto run_step = [&](int e, uint32_t g) {  // fold event e under guess g
            uint32_t q[NQ];
            jac_q<NQ>(q, cls[e], g, ev[e].cz, (uint32_t)nr, (uint32_t)nf);
            jac_acc<NQ>(run, q);
            if (has_rt) {
#pragma unroll
                for (int k = 0; k < MD; ++k) {
                    if (k < nd && sh.rules[nf + k].grade == SG_DEGRADE_GRADE_RT) {
                        const bool chk = (cls[e] & JC_ENT) && g >= (uint32_t)(nf + k);
                        rseg[k] = op_seg(rseg[k], chk ? (((badb >> (e * MD + k)) & 1) ? 1u : 0x80000000u) : 0u);
                    }
                }
            }
            if (RL) {
#pragma unroll
                for (int k = 0; k < 2; ++k) {
                    const int s = k == 0 ? rl_s0 : rl_s1;
                    const int cnt = (int)(ev[e].cz & 0xFFFFu);
                    if (s >= 0 && rl_upd(sh.rules[s], cls[e], g, s, cnt)) {
                        const RState& st = ((has_sync >> s) & 1) ? sh.syn[s] : sh.rs[s];
                        lc[k] += rl_cost(sh.rules[s], st, cnt);
                        const int64_t v = t0 + ev[e].dt - lc[k];
                        lm[k] = v > lm[k] ? v : lm[k];
                    }
                }
            }
        };
        // breaker passCount before event e (RT stage k)
        auto bbefore_of = [&](int k) -> int32_t {
            const uint32_t x = op_seg(segl[k], rseg[k]);
            const int32_t c = (int32_t)(x & 0x7fffffffu);
            return (x & 0x80000000u) ? c : (int32_t)sh.rs[nf + k].b + c;
        };
        // a rate limiter's latestPassedTime before event e
        auto rl_latest = [&](int k, int s) -> int64_t {
            const int64_t L0 = sh.rs[s].c;
            const int64_t mx = lm[k] == NEG_INF64 ? NEG_INF64 : lm[k] - rl_C[k];
            const int64_t me = mx > rl_M[k] ? mx : rl_M[k];
            return rl_C[k] + lc[k] + (me > L0 ? me : L0);
        };

        // ---- evaluation of every event's chain under its view
        uint32_t fe = NO_LANE, fo_m = 0;  // the lane's first mismatching ENTRY and its evaluated outcome
        uint32_t fu_m = 0;                // its ENTRY acquire units through it (from c0)
        int64_t fp_m = 0;                 // the round's pass count after it
        uint32_t wq[EP];                  // queueing waits (rate limiters)
        run_reset();
#pragma unroll
        for (int e = 0; e < EP; ++e) {
            const uint32_t c = cls[e];
            const int cnt = (int)(ev[e].cz & 0xFFFFu);
            const int64_t t = t0 + ev[e].dt;
            const int64_t vP = sh.bP + sh.cP + (int64_t)(ex[Q_P] + run[Q_P]);
            const int64_t vS = sh.bS + sh.cS + (int64_t)(ex[Q_S] + run[Q_S]);
            uint32_t o = (uint32_t)nr;
            int64_t wait = 0;
            if (c & JC_ENT) {
#pragma unroll
                for (int s = 0; s < MF; ++s) {
                    if (s < nf) {
                        const DRule& r = sh.rules[s];
                        bool ok = true;
                        int64_t w = 0;
                        if (r.behavior == SG_CONTROL_BEHAVIOR_WARM_UP) {
                            const RState& st = ((has_sync >> s) & 1) ? sh.syn[s] : sh.rs[s];
                            if (st.a >= r.warning_token) ok = (double)(vP + cnt) <= warm_qps(r, st.a);
                            else ok = (double)(vP + cnt) <= r.count;
                        } else if (RL && (r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER ||
                                          r.behavior == SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER)) {
                            const int k = (s == rl_s0) ? 0 : 1;
                            const RState& st = ((has_sync >> s) & 1) ? sh.syn[s] : sh.rs[s];
                            if (r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER && cnt <= 0) ok = true;
                            else if (r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER && r.count <= 0) ok = false;
                            else {
                                const int64_t expected = rl_latest(k, s) + rl_cost(r, st, cnt);
                                if (expected <= t) ok = true;
                                else { w = expected - t; ok = w <= r.max_queue; }
                            }
                        } else {  // DefaultController
                            const int32_t curv = r.grade == SG_FLOW_GRADE_THREAD
                                                     ? (int32_t)(sh.bTH + sh.cTH + (int64_t)(int32_t)(ex[Q_TH] + run[Q_TH]))
                                                     : j_d2i((double)vP);
                            ok = !((double)j_iadd(curv, cnt) > r.count);
                        }
                        if (o == (uint32_t)nr) {
                            if (!ok) o = (uint32_t)s;
                            else if (w > 0) wait += w;
                        }
                    }
                }
#pragma unroll
                for (int k = 0; k < MD; ++k) {
                    if (k < nd) {
                        const DRule& r = sh.rules[nf + k];
                        const uint32_t trip_ex = ((ex[Q_TR + k / 2] + run[Q_TR + k / 2]) >> (16 * (k & 1))) & 0xFFFFu;
                        bool ok;
                        if (((cutm >> k) & 1) || trip_ex > 0) ok = false;
                        else if (r.grade == SG_DEGRADE_GRADE_RT) ok = !((badb >> (e * MD + k)) & 1) || (bbefore_of(k) + 1 < 5);
                        else if (r.grade == SG_DEGRADE_GRADE_EXCEPTION_RATIO) {
                            const double exc = (double)(sh.bE + sh.cE + (int64_t)(ex[Q_E] + run[Q_E])) / 1.0;
                            const double succ = (double)vS / 1.0;
                            const double total = (double)vP / 1.0 + (double)(sh.bB + sh.cB + (int64_t)(ex[Q_B] + run[Q_B])) / 1.0;
                            if (total < 5) ok = true;
                            else if (succ - exc <= 0 && exc < 5) ok = true;
                            else ok = exc / succ < r.count;
                        } else if (r.grade == SG_DEGRADE_GRADE_EXCEPTION_COUNT)
                            ok = (double)(sh.bEM + sh.cE + (int64_t)(ex[Q_E] + run[Q_E])) < r.count;
                        else ok = true;
                        if (o == (uint32_t)nr && !ok) o = (uint32_t)(nf + k);
                    }
                }
                if (o != gg[e] && fe == NO_LANE) {
                    fe = (uint32_t)e;
                    fo_m = o;
                    fu_m = ex[Q_P] + ex[Q_B] + run[Q_P] + run[Q_B] + (uint32_t)cnt;
                    fp_m = vP + (o == (uint32_t)nr ? cnt : 0);
                }
            }
            wq[e] = (uint32_t)(wait > 0xFFFF ? 0xFFFF : wait);
            run_step(e, gg[e]);
        }
        {   // the wave's first mismatching position and its evaluated outcome
            const uint64_t mm = __ballot(fe != NO_LANE);
            if (mm) {
                const int fl = __ffsll((long long)mm) - 1;
                const uint32_t fel = (uint32_t)__builtin_amdgcn_readlane((int)fe, fl);
                const uint32_t fol = (uint32_t)__builtin_amdgcn_readlane((int)fo_m, fl);
                const uint32_t ful = (uint32_t)__builtin_amdgcn_readlane((int)fu_m, fl);
                const uint32_t fpl = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)fp_m, fl);
                const uint32_t fph = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)fp_m >> 32), fl);
                if (lane == 0) {
                    sh.mism[mb][wv] = (wv * 64 + (uint32_t)fl) * EP + fel;
                    sh.mo[mb][wv] = fol;
                    sh.mu[mb][wv] = ful;
                    sh.mp[mb][wv] = (int64_t)(((uint64_t)fph << 32) | fpl);
                }
            } else if (lane == 0) {
                sh.mism[mb][wv] = NO_LANE;
            }
        }
        PROF_MARK(3)
        lds_barrier();  // B4
        uint32_t f = NO_LANE;
        f = blk_min<NW>(sh.mism[mb]);
        f = uni(f);
        // the pivot's true outcome: the re-guess of every later ENTRY of the round.  Their own evaluated
        // outcomes saw the pivot's wrong guess (e.g. a guessed breaker trip blocks everything after it),
        // while a state change at the pivot (reset breaker, spent quota, trip) mostly holds for the rest.
        const uint32_t of = f != NO_LANE ? uni(sh.mo[mb][f / (64 * EP)]) : 0u;
        // Quota-aware re-guess: when the pivot passed and the first flow stage is a QPS DefaultController,
        // a later ENTRY of the round passes that stage iff the acquire units between the pivot and it still
        // fit the rule's count (FlowRuleChecker order, DefaultController.canPass), so the guess is "pass" for
        // that prefix and "blocked by stage 0" after it instead of "pass" for all -- the iteration that would
        // find the saturation point is saved.  Guesses only steer the iteration count, never a verdict.
        bool qg = false;
        uint32_t q_units = 0;
        int64_t q_pass = 0;
        double q_count = 0.0;
        if (f != NO_LANE && of == (uint32_t)nr && nf > 0 && sh.rules[0].behavior == SG_CONTROL_BEHAVIOR_DEFAULT &&
            sh.rules[0].grade == SG_FLOW_GRADE_QPS) {
            qg = true;
            q_units = uni(sh.mu[mb][f / (64 * EP)]);
            q_pass = uni64(sh.mp[mb][f / (64 * EP)]);
            q_count = sh.rules[0].count;
        }
        mb ^= 1;
        if (f != NO_LANE) ++n_mm;
        const uint32_t e_end = c0 + inr_total;
        const uint32_t cend = f != NO_LANE ? f + 1 : e_end;
        const uint32_t cnt_now = sg.len - tbase < TILE ? sg.len - tbase : TILE;

        // ---- phase D: commit [c0, cend), re-guess the rest (every in-round ENTRY after f: f exists)
        uint32_t appm = 0;  // committed passes (pending list for frozen-stretch skipping)
        uint32_t fmax = 0;  // 1 + the largest outcome of a committed ENTRY (WarmUp sync reach)
        run_reset();
#pragma unroll
        for (int e = 0; e < EP; ++e) {
            const uint32_t c = cls[e];
            const uint32_t pt = lp0 + (uint32_t)e, pos = tbase + pt;
            const uint32_t kind = ev[e].kf & 0xFFu;
            const uint32_t g = gg[e];
            const bool com = (c & JC_INR) && pt < cend;
            const uint32_t fo = (pt == f) ? of : g;
            const int cnt = (int)(ev[e].cz & 0xFFFFu);
            const uint32_t rtv = ev[e].cz >> 16;
            const int64_t t = t0 + ev[e].dt;
#ifdef SG_KPROF
            if (prof && pt == f) {  // what the first mismatching event guessed and evaluated (0 pass, 1 flow, 2 degrade)
                const uint32_t gc = g == (uint32_t)nr ? 0u : g < (uint32_t)nf ? 1u : 2u;
                const uint32_t oc = of == (uint32_t)nr ? 0u : of < (uint32_t)nf ? 1u : 2u;
                atomicAdd(&S.dbg[40 + 3 * gc + oc], 1ull);
                if (f > c0) atomicAdd(&S.dbg[49], 1ull);  // the mismatch is not at the first uncommitted event
                atomicAdd(&S.dbg[50], (unsigned long long)(f - c0));
            }
#endif
            if (com) {
                const bool pbe = (c & JC_PB) != 0;  // its word is the param pre pass's
                pdec[e] = kind == SG_EV_ENTRY ? out_to_dec(sh.rules, nr, nf, fo, wq[e]) : mk_dec(ST_NOT_ENTRY, 0, 0);
                if (!pbe) pmask |= 1u << e;
                win[pos & (WIN - 1)] = ((c & JC_ENT) && fo == (uint32_t)nr) ? 1 : 0;
                gg[e] = fo;
                if (c & JC_ENT) {
                    if (fo == (uint32_t)nr) appm |= 1u << e;
                    if (fo + 1 > fmax) fmax = fo + 1;
                    // the first blocking degrade verdict of a committed ENTRY trips the breaker (DegradeRule.passCheck cut)
#pragma unroll
                    for (int k = 0; k < MD; ++k) {
                        const uint32_t trip_ex = ((ex[Q_TR + k / 2] + run[Q_TR + k / 2]) >> (16 * (k & 1))) & 0xFFFFu;
                        if (k < nd && fo == (uint32_t)(nf + k) && !((cutm >> k) & 1) && trip_ex == 0) {
                            const DRule& r = sh.rules[nf + k];
                            RState& s = sh.rs[nf + k];
                            if (r.grade == SG_DEGRADE_GRADE_RT) s.b = bbefore_of(k) + 1;
                            s.a = 1;
                            s.c = t + (int64_t)r.time_window * 1000;
                        }
                    }
                }
                if (pt == cend - 1) {  // pivot: the last committed event carries the committed totals
                    const bool ce = (c & JC_ENT) != 0, xe = (c & JC_XE) != 0, te = (c & JC_TE) != 0;
                    const bool cp = ce && fo == (uint32_t)nr;
                    sh.cP += (int64_t)(ex[Q_P] + run[Q_P]) + (cp ? cnt : 0);
                    sh.cB += (int64_t)(ex[Q_B] + run[Q_B]) + (((ce && !cp) || pbe) ? cnt : 0);
                    sh.cS += (int64_t)(ex[Q_S] + run[Q_S]) + (xe ? cnt : 0);
                    sh.cRT += (int64_t)(ex[Q_RT] + run[Q_RT]) + (xe ? rtv : 0);
                    sh.cE += (int64_t)(ex[Q_E] + run[Q_E]) + (te ? cnt : 0);
                    sh.cTH += (int64_t)(int32_t)(ex[Q_TH] + run[Q_TH]) + (cp ? 1 : (xe ? -1 : 0));
                    sh.ctouch += ((ex[Q_TI] + run[Q_TI]) & 0xFFFFu) + ((ce || xe || te || pbe) ? 1 : 0);
                    sh.cminrt = op_min(sh.cminrt, op_min(op_min(ex[Q_MIN], run[Q_MIN]), xe ? rtv : NO_LANE));
                    if (RL) {
#pragma unroll
                        for (int k = 0; k < 2; ++k) {
                            const int s = k == 0 ? rl_s0 : rl_s1;
                            if (s >= 0) {
                                const DRule& r = sh.rules[s];
                                const RState& st = ((has_sync >> s) & 1) ? sh.syn[s] : sh.rs[s];
                                const int64_t cost = rl_cost(r, st, cnt);
                                int64_t L = rl_latest(k, s);
                                if (rl_upd(r, c, fo, s, cnt)) L = (t > L + cost) ? t : L + cost;
                                sh.rs[s].c = L;
                            }
                        }
                    }
#pragma unroll
                    for (int k = 0; k < MD; ++k) {
                        const uint32_t trip_ex = ((ex[Q_TR + k / 2] + run[Q_TR + k / 2]) >> (16 * (k & 1))) & 0xFFFFu;
                        if (k < nd && sh.rules[nf + k].grade == SG_DEGRADE_GRADE_RT && !((cutm >> k) & 1) && trip_ex == 0 &&
                            !(ce && fo == (uint32_t)(nf + k))) {
                            int32_t b = bbefore_of(k);
                            if (ce && fo > (uint32_t)(nf + k)) b = ((badb >> (e * MD + k)) & 1) ? b + 1 : 0;
                            sh.rs[nf + k].b = b;
                        }
                    }
                    if (ce) sh.last_out = fo;
                    sh.c0 = cend;
                }
            } else if (c & JC_ENT) {
                uint32_t ng = of;
                if (qg) {
                    const uint32_t before = ex[Q_P] + ex[Q_B] + run[Q_P] + run[Q_B];  // units before this ENTRY
                    const int64_t v = q_pass + (int64_t)(before - q_units);
                    if ((double)j_iadd(j_d2i((double)v), cnt) > q_count) ng = 0u;
                }
                gg[e] = ng;
                win[pos & (WIN - 1)] = (ng == (uint32_t)nr) ? 1 : 0;
            }
            if (pt == cend && cend < cnt_now) sh.tnext = t0 + ev[e].dt;
            run_step(e, g);
        }
        if (skip_on) {  // committed passes join the pending list (their EXIT/TRACE may fall in a skipped span)
            const uint32_t na = (uint32_t)__popc(appm);
            uint32_t incl = na;
            WAVE_SCAN(incl, 0u, op_add);
            const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
            if (tot) {
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&sh.npend, tot);
                base = (uint32_t)__shfl((int)base, 0, 64) + incl - na;
#pragma unroll
                for (int e = 0; e < EP; ++e)
                    if ((appm >> e) & 1) S.pend[sg.start + base++] = tbase + lp0 + e;
            }
        }
        if (has_sync) {
            for (int s = 0; s < nf; ++s) {
                if ((has_sync >> s) & 1) {
                    const uint64_t rb = __ballot(fmax > (uint32_t)s);
                    if (lane == 0 && rb) atomicOr(&sh.warm_reach, 1u << s);
                }
            }
        }
        PROF_MARK(4)
        lds_barrier();  // B1
        PROF_MARK(5)
    }
    if (prof && tid == 0) {
        atomicAdd(&S.dbg[0], (unsigned long long)n_it);
        atomicAdd(&S.dbg[1], (unsigned long long)n_round);
        atomicAdd(&S.dbg[2], (unsigned long long)n_tile);
        atomicAdd(&S.dbg[3], (unsigned long long)n_mm);
        atomicAdd(&S.dbg[4], 1ull);
        atomicAdd(&S.dbg[6], (unsigned long long)n_frz);
        atomicAdd(&S.dbg[7], (unsigned long long)n_opn);
#ifdef SG_KPROF
        const unsigned long long tm_end = __builtin_amdgcn_s_memtime(), tot = tm_end - tm_start;
        if (atomicMax(&S.dbg[18], tot) < tot) {  // slowest segment so far: its phases, length, rounds
            for (int k = 0; k < 10; ++k) S.dbg[8 + k] = tph[k];
            for (int k = 10; k < 14; ++k) S.dbg[52 + k - 10] = tph[k];
            S.dbg[56] = m_nopen;
            S.dbg[57] = m_nfrz;
            S.dbg[58] = m_nround;
            S.dbg[5] = sg.len;
            S.dbg[19] = n_round;
            S.dbg[23] = n_it;
            S.dbg[24] = n_mm;
            S.dbg[25] = pg.pflags | (nf << 8) | (nd << 12) | ((nd ? sh.rules[nf].grade : 0xF) << 16);
            S.dbg[26] = (unsigned long long)sh.rules[0].count;
            S.dbg[27] = n_frz;
            S.dbg[28] = nf ? ((uint64_t)sh.rules[0].behavior | ((uint64_t)sh.rules[0].grade << 8)) : 0xFFFFull;
            S.dbg[29] = n_opn;
        }
        atomicMin(&S.dbg[20], tm_start);  // block start spread (waiting for a CU) and last end
        atomicMax(&S.dbg[21], tm_start);
        atomicMax(&S.dbg[22], tm_end);
#else
        if (blockIdx.x == 0) S.dbg[5] = sg.len;
#endif
    }
#undef PROF_MARK
    // end of segment: fold the last round, write the node and rule states back
    if (tid == 0) {
        round_fold(sh, C, nf);
        min_flush(sh.node, C.minb);
        node_store(sh.node, S, res, pg.pflags);
    }
    __syncthreads();
    if ((int)tid < nr) S.rstate[roff + tid] = sh.rs[tid];
    if (JAC_MINL(NW)) {
        const uint32_t res_u = uni(segs[order[blockIdx.x]].res);  // (recomputed: not held in registers over the kernel)
        for (uint32_t i = tid; i < 60u * sizeof(Bkt) / 16u; i += HW)
            reinterpret_cast<uint4*>(S.minb + (uint64_t)res_u * 60)[i] = reinterpret_cast<const uint4*>(sh.minl)[i];
    }
}

// =================================================================================
// k_tiny: a whole synchronous batch of at most TINY_MAX events in one workgroup (the drop-in's small calls)
// =================================================================================
// The drop-in calls sg_submit_ex synchronously (core/CtSph.java:117-168: every SphU.entry waits for its verdict), so a
// lightly loaded service sends batches of a few events, and the batched pipeline's ~30 launches and its mid-batch host
// round trip set the latency floor.  Here one workgroup runs every stage with a barrier (and an
// agent-scope fence) between them: the group stage's checks, marks and key ring (k_grp_first), a bitonic sort of
// (resource, index) in LDS, the sorted records with same-batch references as sorted positions (k_grp_records) and
// earlier batches' from the status ring (k_resolve), the chain grants (k_chain), the param maps' growth (k_pm_grow),
// the decide stage -- one lane per segment on k_lane<16>'s chain (every rule shape; origin / context nodes inline, as
// k_lane<16> keeps them) -- and the post (decisions in submission order, the status ring: k_post_w).  A batch it
// cannot take alone -- a chain grant under a finite cap (the host orders those), a param pool that must be compacted
// first -- raises BF_TINY_FALLBACK before anything but the marks and the key ring (which the batched path writes the
// same) and growth it would do anyway changed, and the host runs the batched path.
#define TINY_MAX 256u
__global__ __launch_bounds__(TINY_MAX) void k_tiny(const sg_event* __restrict__ ev, uint32_t n, DevState S, DevCfg cfg,
                                                   uint32_t max_res, uint32_t* __restrict__ prio_w,
                                                   const uint32_t* __restrict__ comp, uint64_t n_args, uint32_t grant_all,
                                                   unsigned long long* __restrict__ pool_next, uint64_t pool_nb,
                                                   uint32_t epoch, SEv* __restrict__ recs, uint32_t* __restrict__ vals,
                                                   uint32_t* __restrict__ dec, Seg* __restrict__ segs,
                                                   uint32_t* __restrict__ bflags, uint32_t* __restrict__ out) {
    __shared__ unsigned long long sk[TINY_MAX];  // key << 32 | event index, sorted
    __shared__ uint32_t posof[TINY_MAX];         // event index -> sorted position
    __shared__ uint32_t segat[TINY_MAX + 1];     // segment -> its first position
    __shared__ uint32_t sflags, nseg;
    const uint32_t t = threadIdx.x;
    const uint64_t gbase = S.gbase, ring_mask = cfg.ring_mask;
    if (t == 0) { sflags = 0; nseg = 0; *bflags = 0; }
    __syncthreads();
    const int64_t t0 = ev[0].ts;
    // ---- 1. every event: the batch's checks, the resources' marks, the key ring (k_grp_first)
    uint32_t fl = 0, key = 0xFFFFFFFFu;
    if (t < n) {
        const sg_event e = ev[t];
        if (e.res_id >= max_res) fl |= BF_BAD_RES;
        const int64_t dt = e.ts - t0;
        if (dt < 0 || dt > 0x7FFFFFFFLL) fl |= (dt < 0 ? BF_BACKWARD : BF_TSPAN);
        if (t > 0 && ev[t - 1].ts > e.ts) fl |= BF_BACKWARD;  // ABI: non-decreasing ts
        uint32_t mark = 0;
        uint64_t key0 = (e.flags & SG_F_HAS_ARG) ? e.aux : NO_KEY;
        bool own_args = false;
        if (S.ext) {
            const sg_event_ext x = S.ext[t];
            if (x.n_args > SG_MAX_ARGS || (uint64_t)x.arg_off + x.n_args > n_args) fl |= BF_BAD_ARGS;
            else if (x.n_args) {
                for (uint32_t k = 0; k < x.n_args; ++k) {
                    const sg_arg a = S.args[x.arg_off + k];
                    if (a.kind > SG_ARG_LIST || (a.kind == SG_ARG_LIST && (a.key > n_args || a.len > n_args - a.key)))
                        fl |= BF_BAD_ARGS;
                    else if (a.kind == SG_ARG_LIST) {
                        mark |= PM_ARGL;
                        for (uint32_t q = 0; q < a.len; ++q)
                            if (S.args[a.key + q].kind > SG_ARG_SCALAR) fl |= BF_BAD_ARGS;
                    }
                }
                const sg_arg a0 = S.args[x.arg_off];
                key0 = a0.kind == SG_ARG_SCALAR ? a0.key : NO_KEY;
                own_args = true;
            }
            if (x.context_id > S.max_ctx) mark |= PM_LANE;
            else if (x.origin_id != 0 || x.context_id != 0) {
                mark |= PM_AUX;
                if (x.origin_id >> TAG_ORIGIN_BITS) mark |= PM_LANE;
            }
        }
        if (own_args && e.kind == SG_EV_EXIT && (e.flags & SG_F_EXIT_ARGS)) mark |= PM_XARGS;
        if (e.kind == SG_EV_ENTRY) {
            if (S.key_ring) S.key_ring[(gbase + t) & ring_mask] = key0;
            if (e.flags & SG_F_PRIORITIZED) mark |= PM_PRIO;
            if (e.flags & SG_F_BLOCKED_UPSTREAM) mark |= PM_LANE;
        } else {
            if (e.kind == SG_EV_EXIT && own_args && S.key_ring) S.key_ring[(gbase + t) & ring_mask] = key0;
            const uint64_t ref = e.aux & SG_REF_NONE;
            if (ref != SG_REF_NONE && ref >= gbase && ref - gbase >= t) fl |= BF_BAD_REF;  // must follow its ENTRY
        }
        if (mark && e.res_id < max_res && (prio_w[e.res_id] & mark) != mark) atomicOr(&prio_w[e.res_id], mark);
        key = (comp && e.res_id < max_res) ? comp[e.res_id] : e.res_id;
    }
    sk[t] = t < n ? (((unsigned long long)key << 32) | t) : ~0ull;
    if (fl) atomicOr(&sflags, fl);
    __syncthreads();
    // ---- 2. (resource, index) sorted: every resource's events contiguous, in event order
    for (uint32_t k = 2; k <= TINY_MAX; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            const uint32_t l = t ^ j;
            if (l > t) {
                const unsigned long long a = sk[t], b = sk[l];
                if (((t & k) == 0) == (a > b)) { sk[t] = b; sk[l] = a; }
            }
            __syncthreads();
        }
    const bool first = t < n && (t == 0 || (sk[t] >> 32) != (sk[t - 1] >> 32));
    if (t < n) posof[(uint32_t)sk[t]] = t;
    if (first) segat[atomicAdd(&nseg, 1u)] = t;  // (segment ids in any order: each lane decides its own)
    __syncthreads();
    // ---- 3. the sorted records (k_grp_records, k_resolve)
    if (t < n) {
        const uint32_t i = (uint32_t)sk[t];
        const sg_event e = ev[i];
        SEv r;
        r.dt = (int32_t)(e.ts - t0);
        r.x = 0;
        r.cnt = e.count;
        r.rt = 0;
        r.kind = e.kind;
        r.flags = (uint8_t)(e.flags & 0x3Fu);
        r.code = RC_NONE;
        r.pad = 0;
        uint32_t tag = 0;
        bool own_args = false;
        uint64_t key0 = (e.flags & SG_F_HAS_ARG) ? e.aux : NO_KEY;
        if (S.ext) {
            const sg_event_ext x = S.ext[i];
            if (x.n_args && x.n_args <= SG_MAX_ARGS) {
                const sg_arg a0 = S.args[x.arg_off];
                key0 = a0.kind == SG_ARG_SCALAR ? a0.key : NO_KEY;
                own_args = true;
            }
            if (x.context_id <= S.max_ctx && (x.origin_id != 0 || x.context_id != 0) && !(x.origin_id >> TAG_ORIGIN_BITS))
                tag = x.origin_id | (x.context_id << TAG_ORIGIN_BITS);
        }
        if (own_args) {
            r.flags = (uint8_t)((r.flags & ~SG_F_HAS_ARG) | (key0 != NO_KEY ? SG_F_HAS_ARG : 0));
            if (e.kind == SG_EV_EXIT) r.flags |= RF_OWN_ARGS;
        }
        r.x = tag;
        if (e.kind != SG_EV_ENTRY) {
            if (e.kind == SG_EV_EXIT) {
                const int64_t raw = (int64_t)(e.aux >> 48);
                r.rt = (uint16_t)(raw > cfg.max_rt ? cfg.max_rt : raw);
            }
            const uint64_t ref = e.aux & SG_REF_NONE;
            if (ref != SG_REF_NONE && ref >= gbase && ref - gbase < i) {
                const uint32_t j = (uint32_t)(ref - gbase);
                if (ev[j].kind == SG_EV_ENTRY) {
                    const uint32_t pj = posof[j];
                    if ((sk[pj] >> 32) != (sk[t] >> 32)) atomicOr(&sflags, (uint32_t)BF_BAD_REF);  // another resource's
                    r.code = RC_BATCH;
                    r.x = pj;
                } else {
                    r.code = e.kind == SG_EV_EXIT ? RC_NONE : RC_NOT;  // names a non-ENTRY: as an unknown entry
                }
            } else if (ref != SG_REF_NONE && ref < gbase) {  // an ENTRY of an earlier batch: its status in the ring
                const uint8_t st = S.ring[ref & ring_mask];
                if (st == ST_NOT_ENTRY) r.code = e.kind == SG_EV_EXIT ? RC_NONE : RC_NOT;
                else r.code = (st == ST_PASS || st == ST_PASS_WAIT) ? RC_PASSED : RC_NOT;
            }
        }
        recs[t] = r;
        vals[t] = i | (e.kind == SG_EV_ENTRY ? 0x80000000u : 0u);
    }
    __syncthreads();
    const uint32_t m = nseg;
    // a segment's extent: its start and the next start in position order (starts sorted by a rank among them)
    Seg sg{};
    if (t < m) {
        const uint32_t a = segat[t];
        uint32_t b = n;
        for (uint32_t q = 0; q < m; ++q) { const uint32_t c = segat[q]; if (c > a && c < b) b = c; }
        sg.res = (uint32_t)(sk[a] >> 32);
        sg.start = a;
        sg.len = b - a;
        sg.bin = 0;
        segs[t] = sg;
    }
    if (sflags & (BF_BAD_RES | BF_BACKWARD | BF_TSPAN | BF_BAD_ARGS | BF_BAD_REF)) {  // rejected before any decision
        if (t == 0) *bflags = sflags | BF_TINY_REJECTED;
        return;
    }
    // ---- 4. chain grants (k_chain: CtSph.lookProcessChain) and the param maps' growth (k_pm_grow)
    if (t < m && cfg.switch_on) {
        auto looks_up = [&](uint32_t j) {
            return recs[sg.start + j].kind == SG_EV_ENTRY &&
                   (!S.ext || S.ext[vals[sg.start + j] & 0x7FFFFFFFu].context_id <= S.max_ctx);
        };
        const bool multi = (S.prog[sg.res].multi & PX_MULTI) != 0;
        for (uint32_t j = 0; j < sg.len; ++j) {
            if (!looks_up(j)) continue;
            const uint32_t res = multi ? ev[vals[sg.start + j] & 0x7FFFFFFFu].res_id : sg.res;
            const uint32_t f = S.info[res].flags;
            if (f & (NI_CHAIN | NI_REJECTED)) { if (!multi) break; continue; }
            // grant_all: 1 unbounded cap (grant in place), 0 finite cap not reached (the host grants in first-ENTRY
            // order: fall back), 2 cap reached (no grants; the batched path skips k_chain)
            if (grant_all == 1u) S.info[res].flags = f | NI_CHAIN;
            else if (grant_all == 0u) atomicOr(&sflags, (uint32_t)BF_TINY_FALLBACK);
            if (!multi) break;
        }
    }
    __syncthreads();
    if (t < m && pool_nb && !(sflags & BF_TINY_FALLBACK)) {
        const Prog pg = S.prog[sg.res];
        if (pg.tm_base != NO_ID || pg.n_param != 0) {
            const uint64_t adds = (S.prio && (S.prio[sg.res] & PM_ARGL)) ? 0xFFFFFFFFull : (uint64_t)sg.len;
            for (int k = 0; k < pg.n_param; ++k) {
                const DRule& r = S.rules[pg.rule_off + k];
                if (r.behavior != PB_INIT_ONLY && r.grade == SG_FLOW_GRADE_QPS)
                    pm_grow(S, r.pmap, adds, pool_next, pool_nb, bflags, nullptr, nullptr, 0, epoch);
            }
            if (pg.tm_base != NO_ID)
                for (int i = 0; i < SG_MAX_ARGS; ++i) {
                    const uint32_t id = S.tmid[pg.tm_base + i];
                    if (id != NO_ID) pm_grow(S, id, adds, pool_next, pool_nb, bflags, nullptr, nullptr, 0, epoch);
                }
        }
    }
    __threadfence();
    __syncthreads();
    if (pool_nb && t == 0 && pool_next[PC_RESCUE] == epoch) atomicOr(&sflags, (uint32_t)BF_TINY_FALLBACK);
    __syncthreads();
    if (sflags & BF_TINY_FALLBACK) {
        if (t == 0) atomicOr(bflags, sflags);
        return;
    }
    // ---- 5. decide: one lane per segment (k_lane<16>)
    if (t < m) lane_seg<16>(recs, ev, vals, sg, S, cfg, t0, dec, bflags, t);
    __threadfence();
    __syncthreads();
    // ---- 6. decisions in submission order, the status ring (k_post_w)
    if (t < n) {
        const uint32_t d = ev[t].kind == SG_EV_ENTRY ? dec[posof[t]] : (uint32_t)ST_NOT_ENTRY;
        out[t] = d;
        S.ring[(gbase + t) & ring_mask] = (uint8_t)(d & 0xFF);
    }
    if (t == 0 && sflags) atomicOr(bflags, sflags);
}

// =================================================================================
// host-callable launch wrappers
// =================================================================================
namespace sg {

hipError_t launch_seg(const uint32_t* keys, uint64_t n, uint32_t* flag, uint32_t* pos, Seg* segs, hipStream_t st,
                      hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                      uint32_t* part, uint32_t* nseg) {
    // flag/pos are scratch of >= n words: tile counts in flag, their offsets in pos
    const uint32_t nt = (uint32_t)((n + SEG_TILE - 1) / SEG_TILE);
    hipLaunchKernelGGL(k_seg_count, dim3(nt), dim3(256), 0, st, keys, n, flag, (const uint32_t*)nullptr);
    hipError_t e = scan(flag, pos, nt, part, nseg, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_seg_emit, dim3(nt), dim3(256), 0, st, keys, n, pos, segs, (const uint32_t*)nullptr,
                       (const uint32_t*)nullptr);
    return hipGetLastError();
}
__global__ void k_add2(uint32_t* __restrict__ dst, const uint32_t* __restrict__ a, const uint32_t* __restrict__ b) {
    if (threadIdx.x == 0) *dst = *a + *b;
}
// the cold segments of the hot / cold group stage: keys[*lo, n), written after the *sbase hot ones; nseg = both.
// flag / pos: scratch of >= n / SEG_TILE + 1 words each; ccount: one device word
hipError_t launch_seg_cold(const uint32_t* keys, uint64_t n, const uint32_t* lo, const uint32_t* sbase, uint32_t* flag,
                           uint32_t* pos, Seg* segs, hipStream_t st,
                           hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                           uint32_t* part, uint32_t* ccount, uint32_t* nseg) {
    const uint32_t nt = (uint32_t)((n + SEG_TILE - 1) / SEG_TILE);
    hipLaunchKernelGGL(k_seg_count, dim3(nt), dim3(256), 0, st, keys, n, flag, lo);
    hipError_t e = scan(flag, pos, nt, part, ccount, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_seg_emit, dim3(nt), dim3(256), 0, st, keys, n, pos, segs, lo, sbase);
    hipLaunchKernelGGL(k_add2, dim3(1), dim3(64), 0, st, nseg, sbase, ccount);
    return hipGetLastError();
}
// the sorted-order side tables (bst sums, forward links) of the hot / cold group stage (its records are in place)
hipError_t launch_block_sums(const SEv* recs, uint64_t n, uint32_t* bst, Link* link, uint32_t epoch, uint32_t* bflags,
                             const uint32_t* skeys, const uint32_t* lo, hipStream_t st) {
    hipLaunchKernelGGL(k_block_sums, dim3((uint32_t)((n + 1023) / 1024)), dim3(256), 0, st, recs, skeys, n, bst, link,
                       epoch, bflags, lo);
    return hipGetLastError();
}
// mp: the segment count on the device; mb: an upper bound of it (the grid)
hipError_t launch_seg_bin(Seg* segs, const uint32_t* mp, uint32_t mb, uint64_t n, const Prog* prog, const uint32_t* prio,
                          uint32_t lane_max, uint32_t j1_max, uint32_t j4_max, uint32_t force_lane, uint32_t* blkcnt,
                          uint32_t pq_ok, uint32_t pq_wide, uint32_t* aux, uint32_t* ashort, uint64_t* along,
                          uint64_t* amulti, uint32_t* mixc, uint32_t* mix, uint32_t mix_cap, uint32_t* mixlen,
                          uint32_t mix_wide, uint32_t head_min, hipStream_t st) {
    const uint32_t nblk = (mb + 255) / 256;
    if (!nblk) return hipSuccess;
    hipLaunchKernelGGL(k_seg_bin, dim3(nblk), dim3(256), 0, st, segs, mp, n, prog, prio, lane_max, j1_max, j4_max, force_lane,
                       blkcnt, nblk, pq_ok, pq_wide, aux, ashort, along, amulti, mixc, mix, mix_cap, mixlen, mix_wide,
                       head_min);
    return hipGetLastError();
}
// off = exclusive scan of blkcnt (bin-major); writes the per-bin offsets to bin_off[0..N_BINS]
hipError_t launch_seg_order(Seg* segs, const uint32_t* mp, uint32_t mb, const uint32_t* off, uint32_t* order,
                            uint32_t* bin_off, hipStream_t st) {
    const uint32_t nblk = (mb + 255) / 256;
    if (nblk) hipLaunchKernelGGL(k_seg_order, dim3(nblk), dim3(256), 0, st, segs, mp, off, nblk, order);
    hipLaunchKernelGGL(k_bin_offsets, dim3(1), dim3(64), 0, st, off, nblk ? nblk : 1, mp, bin_off);
    return hipGetLastError();
}
hipError_t launch_gather(const SEv* rec_o, const uint32_t* vals, const uint32_t* skeys, uint64_t n,
                         const uint32_t* pos_of, SEv* recs, uint32_t* prev, uint32_t* nprev, Link* link, uint32_t* bst,
                         uint32_t epoch, uint32_t* bflags, hipStream_t st) {
    uint32_t nb = (uint32_t)((n + 255) / 256);
    hipError_t e = hipMemsetAsync(bst, 0, ((n + 1023) / 1024) * 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_scatter_rec, dim3(nb), dim3(256), 0, st, rec_o, n, pos_of, recs, prev, nprev, link, bst,
                       epoch, bflags);
    hipLaunchKernelGGL(k_block_sums, dim3((uint32_t)((n + 1023) / 1024)), dim3(256), 0, st, recs, skeys, n, bst, link,
                       epoch, bflags, (const uint32_t*)nullptr);
    return hipGetLastError();
}
hipError_t launch_fill(const Span* spans, const uint32_t* nspan, uint32_t cap, const SEv* recs, const Prog* prog,
                       const DRule* rules, uint32_t* dec, hipStream_t st) {
    hipLaunchKernelGGL(k_fill, dim3(2048), dim3(256), 0, st, spans, nspan, cap, recs, prog, rules, dec);
    return hipGetLastError();
}
hipError_t launch_resolve(const uint32_t* prev, uint32_t np, const uint8_t* ring, SEv* recs, const uint32_t* vals,
                          const sg_event_ext* ext, hipStream_t st) {
    if (!np) return hipSuccess;
    hipLaunchKernelGGL(k_resolve, dim3((np + 255) / 256), dim3(256), 0, st, prev, np, ring, recs, vals, ext);
    return hipGetLastError();
}
hipError_t launch_post(const uint32_t* pos_of, const uint32_t* dec, uint64_t n, uint64_t gbase, uint8_t* ring,
                       uint64_t ring_mask, uint32_t* out, hipStream_t st) {
    uint32_t nb = (uint32_t)((n + 256 * POST_ITEMS - 1) / (256 * POST_ITEMS));
    hipLaunchKernelGGL(k_post, dim3(nb), dim3(256), 0, st, pos_of, dec, n, gbase, ring, ring_mask, out);
    return hipGetLastError();
}
hipError_t launch_chain(const SEv* recs, const uint32_t* vals, const Seg* segs, uint32_t m, NodeInfo* info,
                        uint32_t grant_all, uint32_t* ncand, uint64_t* cand, const sg_event* ev, const Prog* prog,
                        const sg_event_ext* ext, uint32_t max_ctx, hipStream_t st) {
    if (!m) return hipSuccess;
    hipLaunchKernelGGL(k_chain, dim3((m + 255) / 256), dim3(256), 0, st, recs, vals, segs, m, info, grant_all, ncand,
                       cand, ev, prog, ext, max_ctx);
    return hipGetLastError();
}
// bin = BIN_J16 / BIN_J8 / BIN_J4 / BIN_J1 / BIN_LANE (range of lane bins, nr <= 4) / BIN_LANE16
hipError_t launch_tiny(const sg_event* ev, uint32_t n, const DevState& S, const DevCfg& cfg, uint32_t max_res,
                       uint32_t* prio_w, const uint32_t* comp, uint64_t n_args, uint32_t grant_all,
                       unsigned long long* pool_next, uint64_t pool_nb, uint32_t epoch, SEv* recs, uint32_t* vals,
                       uint32_t* dec, Seg* segs, uint32_t* bflags, uint32_t* out, hipStream_t st) {
    if (n == 0 || n > TINY_MAX) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_tiny, dim3(1), dim3(TINY_MAX), 0, st, ev, n, S, cfg, max_res, prio_w, comp, n_args, grant_all,
                       pool_next, pool_nb, epoch, recs, vals, dec, segs, bflags, out);
    return hipGetLastError();
}
uint32_t tiny_max() { return TINY_MAX; }
hipError_t launch_head(const SEv* recs, const Seg* segs, const uint32_t* order, uint32_t m, const DevState& S,
                       const DevCfg& cfg, int64_t t0, uint32_t* dec, uint32_t* bflags, hipStream_t st);
hipError_t launch_decide_bin(int bin, const SEv* recs, const sg_event* ev, const uint32_t* vals, const Seg* segs,
                             const uint32_t* order, uint32_t m, const DevState& S, const DevCfg& cfg, int64_t t0,
                             uint32_t* dec, uint32_t* bflags, hipStream_t st) {
    if (!m) return hipSuccess;
    // single-rule THREAD-grade / RateLimiter heads (XF_HEADT / XF_HEADR): the event-driven owner, before the
    // cooperative one (which leaves those segments)
    if ((bin == BIN_J16 || bin == BIN_J4 || bin == BIN_J1) && cfg.heads && !(cfg.dbg_flags & HEAD_OFF)) {
        const hipError_t he = launch_head(recs, segs, order, m, S, cfg, t0, dec, bflags, st);
        if (he != hipSuccess) return he;
    }
    switch (bin) {
    case BIN_J16:  // programs of the J16 shape only (PF_J16): <= 2 flow, <= 2 degrade stages, no rate limiter;
                   // a 128 KiB status window (one workgroup per CU) keeps EXIT references in LDS
        // THREAD-grade / WarmUp heads (no frozen-stretch skipping: without it the iteration fits 128 registers,
        // 1 VGPR spilled against 19), then the QPS-DefaultController heads longer than J8_MAX (skipping)
        hipLaunchKernelGGL((k_jac<16, 1, 17, 2, 2, false, false, 2>), dim3(m), dim3(1024), 0, st, recs, segs, order, m, S, cfg,
                           t0, dec, bflags);
        hipLaunchKernelGGL((k_jac<16, 1, 17, 2, 2, false, true, 1>), dim3(m), dim3(1024), 0, st, recs, segs, order, m, S, cfg,
                           t0, dec, bflags);
        break;
    case BIN_J8:  // the J16 lengths of QPS-DefaultController programs (C2 / C4 heads): 512 lanes with 256 registers a
                  // lane, room for the open stretches (the 1024-lane owner's 128 registers do not hold them);
                  // measured: C4 J16-bin time 1.89 -> 1.53 ms, C2 4.03 -> 4.24 G entries/s.  THREAD-grade / WarmUp
                  // heads keep 1024 lanes (C3: 0.39 vs 0.27 G entries/s)
        hipLaunchKernelGGL((k_jac<8, 1, 17, 2, 2, false, true>), dim3(m), dim3(512), 0, st, recs, segs, order, m, S, cfg, t0,
                           dec, bflags);
        break;
    case BIN_J4:  // 256 lanes, one event each: two events per lane (k_jac<4, 2, ...>) measured 22 % faster alone
                  // but slower in the pipeline (200 VGPRs: less room for the overlapping group stage)
        hipLaunchKernelGGL((k_jac<4, 1, 14, JMAX_FLOW, JMAX_DEG, true, true>), dim3(m), dim3(256), 0, st, recs, segs, order, m, S,
                           cfg, t0, dec, bflags);
        break;
    case BIN_J1:
        hipLaunchKernelGGL((k_jac<1, 1, 12, JMAX_FLOW, JMAX_DEG, true, false>), dim3(m), dim3(64), 0, st, recs, segs, order, m, S,
                           cfg, t0, dec, bflags);
        break;
    case BIN_LITE:
        hipLaunchKernelGGL(k_lite<false>, dim3((m + 255) / 256), dim3(256), 0, st, recs, ev, vals, segs, order, m, S, cfg,
                           t0, dec, bflags);
        if (S.key_ring)  // (param rules exist: XF_PLITE programs may)
            hipLaunchKernelGGL(k_lite<true>, dim3((m + 255) / 256), dim3(256), 0, st, recs, ev, vals, segs, order, m, S,
                               cfg, t0, dec, bflags);
        break;
    case BIN_LANE:
        hipLaunchKernelGGL(k_lane<4>, dim3((m + 255) / 256), dim3(256), 0, st, recs, ev, vals, segs, order, m, S, cfg,
                           t0, dec, bflags);
        break;
    default:
        hipLaunchKernelGGL(k_lane<MAXR>, dim3((m + 255) / 256), dim3(256), 0, st, recs, ev, vals, segs, order, m, S,
                           cfg, t0, dec, bflags);
        break;
    }
    return hipGetLastError();
}

} // namespace sg
