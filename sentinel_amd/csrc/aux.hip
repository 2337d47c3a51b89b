// aux.hip -- the origin / context node post-pass of an sg_submit_ex batch.
//
// ClusterBuilderSlot and NodeSelectorSlot give every entry an origin StatisticNode and a context DefaultNode, and
// StatisticSlot counts the entry (and its exit) on them whatever the rules are (StatisticSlot.java:54-173,
// ClusterBuilderSlot.java:77-106, NodeSelectorSlot.java:136-175).  When no rule of the resource reads those nodes
// (no origin / "other" / STRATEGY_CHAIN flow rule: PX_ORIGIN / PX_CHAIN), nothing the chain decides depends on
// them, so the segment is decided by its usual owner (k_jac, k_lite, k_lane<4>, k_pq) and the nodes are brought
// up to date afterwards from the committed verdicts, here.
//
// A node's update by the events of a batch is a reduction.  Per 500 ms parity p its second-window bucket ends as:
// the latest window W any of its events falls in, holding the sums of the events of W (plus the bucket's own
// counts when W is the bucket's window, or the borrowed pass when W resets it) -- LeapArray.currentWindow resets
// a bucket to a later window in place, so earlier events of the same parity are overwritten.  Per second parity q
// likewise the minute pass history (aux.h), and curThreadNum moves by passes minus exits.  So "later window
// replaces, same window adds" is an associative merge (AuxAcc) and a segment's events can be cut anywhere:
//   * k_aux_cold  : one workgroup per AUX_G segments of <= AUX_SHORT events, their events 256 at a time: an LDS
//                   table of the chunk's nodes, merged in two phases (the latest window of every node-parity, then
//                   the sums of that window), committed one node a thread;
//   * k_aux_piece : one workgroup per AUX_PIECE events of a longer segment, the same table: a one-piece segment
//                   commits its nodes, the pieces of a longer one leave partial AuxAccs;
//   * k_aux_merge : one workgroup per multi-piece segment: the pieces' partials merged the same way, committed.
// An event updates the origin node (origin != 0) and the context node (named context: without a CHAIN rule the
// default context's DefaultNode is not kept, decide.hip chain_ctx_kept) of its tag (SEv.x: the ENTRY's own, an
// EXIT's from its ENTRY when the ENTRY is in the batch): a passed ENTRY pass + thread, a blocked one block, an
// effective EXIT success + rt + minRt - thread (StatisticSlot.exit).  An overflow of the LDS table or the
// partial pool falls back to a sequential walk of the segment (exact, slow).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aux.h"

using namespace sg;

#define AUX_K 4           // aux_walk (the sequential fallback): nodes cached per lane
#define AUX_NONE 0x7FFFFFFF
#define AUX_EMPTY32 0xFFFFFFFFu

enum : uint32_t { AW_NONE = 0, AW_PASS = 1, AW_BLOCK = 2, AW_EXIT = 3 };

// What event p (segment-relative nothing: absolute sorted position) does to its nodes, from the verdicts.
__device__ __forceinline__ uint32_t aux_what(const SEv& r, uint32_t p, const SEv* __restrict__ recs,
                                             const uint32_t* __restrict__ dec, bool chain, uint32_t* tag) {
    if (r.kind == SG_EV_ENTRY) {
        const uint32_t st = dec[p] & 0xFFu;
        *tag = r.x;
        if (st == ST_NO_CHECK || st == ST_NOT_ENTRY) return AW_NONE;
        return st == ST_PASS ? AW_PASS : st == ST_PASS_WAIT ? AW_NONE : AW_BLOCK;  // (PASS_WAIT: k_lane only)
    }
    if (r.kind != SG_EV_EXIT) return AW_NONE;  // Tracer: the ClusterNode only
    bool eff;
    uint32_t tg = r.x;
    if (r.code == RC_NONE) eff = chain;
    else if (r.code == RC_PASSED) eff = true;
    else if (r.code == RC_BATCH) {
        eff = st_passed(dec[r.x] & 0xFFu);
        tg = recs[r.x].x;  // the ENTRY's nodes (its Context)
    } else eff = false;
    *tag = tg;
    return eff ? AW_EXIT : AW_NONE;
}

// ---------------------------------------------------------------- sequential form (lanes, fallback)
// a register accumulator: windows as indices relative to the batch (500 ms / 1 s units)
struct LAcc {
    uint32_t key;
    int32_t thread;
    int32_t W[2], MW[2];
    uint32_t s[2][4];
    uint32_t minrt[2];
    uint32_t mpass[2];
};
__device__ __forceinline__ void lacc_zero(LAcc& a, uint32_t key) {
    a.key = key;
    a.thread = 0;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        a.W[p] = -1; a.MW[p] = -1; a.minrt[p] = 0xFFFFFFFFu; a.mpass[p] = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) a.s[p][k] = 0;
    }
}
// one update, in time order
__device__ __forceinline__ void lacc_add(LAcc& a, uint32_t what, int32_t wi, int32_t si, uint32_t cnt, uint32_t rt) {
    const int p = wi & 1;
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
        if (pp != p) continue;
        if (wi > a.W[pp]) {
            a.W[pp] = wi;
            a.s[pp][0] = a.s[pp][1] = a.s[pp][2] = a.s[pp][3] = 0;
            a.minrt[pp] = 0xFFFFFFFFu;
        }
        if (what == AW_PASS) a.s[pp][0] += cnt;
        else if (what == AW_BLOCK) a.s[pp][1] += cnt;
        else { a.s[pp][2] += cnt; a.s[pp][3] += rt; a.minrt[pp] = rt < a.minrt[pp] ? rt : a.minrt[pp]; }
    }
    if (what == AW_PASS) {
        a.thread += 1;
        const int q = si & 1;
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) {
            if (qq != q) continue;
            if (si > a.MW[qq]) { a.MW[qq] = si; a.mpass[qq] = 0; }
            a.mpass[qq] += cnt;
        }
    } else if (what == AW_EXIT) {
        a.thread -= 1;
    }
}
__device__ __forceinline__ void lacc_commit(const DevState& S, int32_t max_rt, uint32_t res, const LAcc& a,
                                            int64_t b500, int64_t b1000, uint32_t* bflags) {
    AuxAcc A;
    A.key = a.key;
    A.thread = a.thread;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        A.W[p] = a.W[p] < 0 ? -1 : (b500 + a.W[p]) * 500;
        A.MW[p] = a.MW[p] < 0 ? -1 : (b1000 + a.MW[p]) * 1000;
        A.minrt[p] = a.minrt[p];
        A.mpass[p] = a.mpass[p];
#pragma unroll
        for (int k = 0; k < 4; ++k) A.s[p][k] = a.s[p][k];
    }
    aux_commit(S, max_rt, res, A, bflags);
}

// the events [a, b) of one resource's segment, one lane, a cache of AUX_K nodes (an evicted node is committed:
// the merge is associative, so a node may be committed in several parts)
__device__ void aux_walk(const SEv* __restrict__ recs, const uint32_t* __restrict__ dec, const DevState& S,
                         int32_t max_rt, uint32_t res, bool chain, uint32_t a, uint32_t b, int64_t t0, uint32_t* bflags) {
    const int64_t b500 = t0 / 500, b1000 = t0 / 1000;
    LAcc c[AUX_K];
#pragma unroll
    for (int k = 0; k < AUX_K; ++k) lacc_zero(c[k], AUX_EMPTY32);
    uint32_t victim = 0;
    for (uint32_t p = a; p < b; ++p) {
        const SEv r = recs[p];
        uint32_t tag;
        const uint32_t what = aux_what(r, p, recs, dec, chain, &tag);
        if (what == AW_NONE || tag == 0) continue;
        const int64_t t = t0 + r.dt;
        const int32_t wi = (int32_t)(t / 500 - b500), si = (int32_t)(t / 1000 - b1000);
        const uint32_t o = tag_origin(tag), cx = tag_ctx(tag);
        for (int u = 0; u < 2; ++u) {
            const uint32_t id = u == 0 ? o : cx;
            if (id == 0) continue;
            const uint32_t key = ((uint32_t)u << 31) | id;
            int hit = -1;
#pragma unroll
            for (int k = 0; k < AUX_K; ++k) if (c[k].key == key) hit = k;
            if (hit < 0) {  // round-robin eviction
                hit = (int)victim;
                victim = (victim + 1) % AUX_K;
#pragma unroll
                for (int k = 0; k < AUX_K; ++k) {
                    if (k != hit) continue;
                    if (c[k].key != AUX_EMPTY32) lacc_commit(S, max_rt, res, c[k], b500, b1000, bflags);
                    lacc_zero(c[k], key);
                }
            }
#pragma unroll
            for (int k = 0; k < AUX_K; ++k)
                if (k == hit) lacc_add(c[k], what, wi, si, r.cnt, r.rt);
        }
    }
#pragma unroll
    for (int k = 0; k < AUX_K; ++k)
        if (c[k].key != AUX_EMPTY32) lacc_commit(S, max_rt, res, c[k], b500, b1000, bflags);
}

__device__ __forceinline__ bool seg_chain(const DevState& S, const DevCfg& cfg, uint32_t res) {
    return (S.info[res].flags & NI_CHAIN) != 0 && cfg.switch_on;
}

// ---------------------------------------------------------------- the LDS node table
// Slots keyed by a 32-bit node key; windows as indices relative to the batch (500 ms / 1 s units), sums in 32 bits
// (a chunk or piece holds <= AUX_PIECE events of <= 65535 each).  Updates merge in two phases separated by a
// barrier: the latest window of every node-parity first (a read, an atomicMax only when later), then the sums of
// the updates in that window and the thread deltas of all of them.
#define TAB_S 512
struct Tab {
    uint32_t key[TAB_S];
    int32_t W[TAB_S][2], MW[TAB_S][2];
    uint32_t s[TAB_S][2][4];
    uint32_t minrt[TAB_S][2];
    uint32_t mpass[TAB_S][2];
    int32_t thread[TAB_S];
    uint32_t used[TAB_S];
    uint32_t nused, overflow;
};
__device__ __forceinline__ void tab_clear(Tab& T) {  // every slot (the first time)
    for (uint32_t i = threadIdx.x; i < TAB_S; i += blockDim.x) {
        T.key[i] = AUX_EMPTY32;
        T.W[i][0] = T.W[i][1] = T.MW[i][0] = T.MW[i][1] = -1;
        for (int p = 0; p < 2; ++p) {
            for (int k = 0; k < 4; ++k) T.s[i][p][k] = 0;
            T.minrt[i][p] = 0xFFFFFFFFu;
            T.mpass[i][p] = 0;
        }
        T.thread[i] = 0;
    }
    if (threadIdx.x == 0) { T.nused = 0; T.overflow = 0; }
}
__device__ __forceinline__ void tab_reset_used(Tab& T) {  // the used slots only (after a flush)
    const uint32_t nu = T.nused;
    for (uint32_t u = threadIdx.x; u < nu; u += blockDim.x) {
        const uint32_t i = T.used[u];
        T.key[i] = AUX_EMPTY32;
        T.W[i][0] = T.W[i][1] = T.MW[i][0] = T.MW[i][1] = -1;
        for (int p = 0; p < 2; ++p) {
            for (int k = 0; k < 4; ++k) T.s[i][p][k] = 0;
            T.minrt[i][p] = 0xFFFFFFFFu;
            T.mpass[i][p] = 0;
        }
        T.thread[i] = 0;
    }
}
// the slot of key, inserted on first sight (a plain read finds a present key: no atomic); -1 when full
__device__ __forceinline__ int tab_find(Tab& T, uint32_t key) {
    uint32_t h = (uint32_t)(mix64(key) & (TAB_S - 1));
    for (int probe = 0; probe < TAB_S; ++probe) {
        uint32_t k = __hip_atomic_load(&T.key[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (k == AUX_EMPTY32) {
            k = atomicCAS(&T.key[h], AUX_EMPTY32, key);
            if (k == AUX_EMPTY32) { T.used[atomicAdd(&T.nused, 1u)] = h; return (int)h; }
        }
        if (k == key) return (int)h;
        h = (h + 1) & (TAB_S - 1);
    }
    atomicOr(&T.overflow, 1u);
    return -1;
}
__device__ __forceinline__ void tab_p1(Tab& T, int i, uint32_t what, int32_t wi, int32_t si) {
    const int p = wi & 1, q = si & 1;
    if (wi > T.W[i][p]) atomicMax(&T.W[i][p], wi);
    if (what == AW_PASS && si > T.MW[i][q]) atomicMax(&T.MW[i][q], si);
}
__device__ __forceinline__ void tab_p2(Tab& T, int i, uint32_t what, int32_t wi, int32_t si, uint32_t c, uint32_t rt) {
    const int p = wi & 1, q = si & 1;
    const bool in_w = T.W[i][p] == wi;
    if (what == AW_PASS) {
        atomicAdd(&T.thread[i], 1);
        if (in_w) atomicAdd(&T.s[i][p][0], c);
        if (T.MW[i][q] == si) atomicAdd(&T.mpass[i][q], c);
    } else if (what == AW_BLOCK) {
        if (in_w) atomicAdd(&T.s[i][p][1], c);
    } else {
        atomicAdd(&T.thread[i], -1);
        if (in_w) {
            atomicAdd(&T.s[i][p][2], c);
            atomicAdd(&T.s[i][p][3], rt);
            atomicMin(&T.minrt[i][p], rt);
        }
    }
}
// slot i as an AuxAcc (absolute windows; key = kind << 31 | id)
__device__ __forceinline__ void tab_acc(const Tab& T, uint32_t i, uint32_t key, int64_t b500, int64_t b1000, AuxAcc& A) {
    A.key = key;
    A.thread = T.thread[i];
    for (int p = 0; p < 2; ++p) {
        A.W[p] = T.W[i][p] < 0 ? -1 : (b500 + T.W[i][p]) * 500;
        A.MW[p] = T.MW[i][p] < 0 ? -1 : (b1000 + T.MW[i][p]) * 1000;
        A.minrt[p] = T.minrt[i][p];
        A.mpass[p] = T.mpass[i][p];
        for (int k = 0; k < 4; ++k) A.s[p][k] = T.s[i][p][k];
    }
}

// The short segments (<= AUX_SHORT events): a workgroup per AUX_G of them, their events in chunks of 256 (one a
// thread), every chunk's nodes merged in the table and committed (several commits of one node are fine: the merge
// is associative, and one workgroup owns its segments' nodes).  Node key: segment-in-group << 25 | kind << 24 | id.
#define AUX_G 64
__global__ __launch_bounds__(256) void k_aux_cold(const SEv* __restrict__ recs, const Seg* __restrict__ segs,
                                                  const uint32_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                                                  DevState S, DevCfg cfg, int64_t t0, const uint32_t* __restrict__ dec,
                                                  uint32_t* __restrict__ bflags) {
    __shared__ Tab T;
    __shared__ uint32_t gstart[AUX_G], gres[AUX_G], gpre[AUX_G + 1], gchain[AUX_G];
    __shared__ uint32_t claims;
    const uint32_t m = *cnt;
    const int64_t b500 = t0 / 500, b1000 = t0 / 1000;
    tab_clear(T);
    if (threadIdx.x == 0) claims = 0;
    for (uint32_t g0 = blockIdx.x * AUX_G; g0 < m; g0 += gridDim.x * AUX_G) {
        const uint32_t ng = min((uint32_t)AUX_G, m - g0);
        __syncthreads();
        if (threadIdx.x < 64) {  // the group's segments and the exclusive prefix of their lengths (one wave)
            const uint32_t l = threadIdx.x;
            uint32_t len = 0;
            if (l < ng) {
                const Seg sg = segs[list[g0 + l]];
                gstart[l] = sg.start;
                gres[l] = sg.res;
                gchain[l] = seg_chain(S, cfg, sg.res) ? 1u : 0u;
                len = sg.len;
            }
            uint32_t x = len;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(x, o, 64);
                if ((int)l >= o) x += y;
            }
            gpre[l] = x - len;
            if (l == 63) gpre[AUX_G] = x;
        }
        __syncthreads();
        const uint32_t tot = gpre[AUX_G];
        for (uint32_t c0 = 0; c0 < tot; c0 += 256) {
            const uint32_t e = c0 + threadIdx.x;
            uint32_t what = AW_NONE, tag = 0, g = 0, cz = 0;
            int32_t wi = 0, si = 0;
            if (e < tot) {
                uint32_t lo = 0, hi = ng;  // the segment holding event e: gpre[g] <= e < gpre[g + 1]
                while (hi - lo > 1) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if (gpre[mid] <= e) lo = mid; else hi = mid;
                }
                g = lo;
                const uint32_t p = gstart[g] + (e - gpre[g]);
                const SEv r = recs[p];
                what = aux_what(r, p, recs, dec, gchain[g] != 0, &tag);
                const int64_t t = t0 + r.dt;
                wi = (int32_t)(t / 500 - b500);
                si = (int32_t)(t / 1000 - b1000);
                cz = (uint32_t)r.cnt | ((uint32_t)r.rt << 16);
            }
            int sl[2] = {-1, -1};
            if (what != AW_NONE && tag && !(cfg.dbg_flags & 1024)) {
                const uint32_t o = tag_origin(tag), cx = tag_ctx(tag);
                if (o) sl[0] = tab_find(T, (g << 25) | o);
                if (cx) sl[1] = tab_find(T, (g << 25) | (1u << 24) | cx);
            }
#pragma unroll
            for (int u = 0; u < 2; ++u)
                if (sl[u] >= 0) tab_p1(T, sl[u], what, wi, si);
            __syncthreads();
#pragma unroll
            for (int u = 0; u < 2; ++u)
                if (sl[u] >= 0) tab_p2(T, sl[u], what, wi, si, cz & 0xFFFFu, cz >> 16);
            __syncthreads();
            const uint32_t nu = T.nused;  // (<= 512 updates a chunk: the table cannot overflow)
            for (uint32_t u = threadIdx.x; u < nu; u += blockDim.x) {
                const uint32_t i = T.used[u], k = T.key[i];
                AuxAcc A;
                tab_acc(T, i, ((k >> 24) & 1u) << 31 | (k & 0xFFFFFFu), b500, b1000, A);
                if (!(cfg.dbg_flags & 2048)) aux_commit(S, cfg.max_rt, gres[k >> 25], A, bflags, &claims);
            }
            __syncthreads();
            tab_reset_used(T);
            __syncthreads();
            if (threadIdx.x == 0) T.nused = 0;
            __syncthreads();
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) aux_flush_claims(S, claims, bflags);
}

// Long segments: the pieces of every one (apiece[k] = seg << 32 | piece), expanded from the long list
// (along[j] = seg << 32 | first piece) one workgroup a segment
__global__ __launch_bounds__(256) void k_aux_expand(const Seg* __restrict__ segs, const uint64_t* __restrict__ along,
                                                    const uint32_t* __restrict__ cnt, uint64_t* __restrict__ apiece) {
    const uint32_t m = *cnt;
    for (uint32_t j = blockIdx.x; j < m; j += gridDim.x) {
        const uint64_t e = along[j];
        const uint32_t s = (uint32_t)(e >> 32), q = (uint32_t)e;
        const uint32_t np = (segs[s].len + AUX_PIECE - 1) / AUX_PIECE;
        for (uint32_t i = threadIdx.x; i < np; i += blockDim.x) apiece[q + i] = ((uint64_t)s << 32) | i;
    }
}

// One piece of a long segment.  meta[k] = pool offset << 32 | count of its partial AuxAccs (count AUX_NONE: the
// piece overflowed the table or the pool); a one-piece segment commits instead and leaves no meta.
#define PIECE_EPL (AUX_PIECE / 256)
__global__ __launch_bounds__(256) void k_aux_piece(const SEv* __restrict__ recs, const Seg* __restrict__ segs,
                                                   const uint64_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                                                   DevState S, DevCfg cfg, int64_t t0, const uint32_t* __restrict__ dec,
                                                   AuxAcc* __restrict__ pool, uint32_t pool_cap,
                                                   uint32_t* __restrict__ pool_n, uint64_t* __restrict__ meta,
                                                   uint32_t* __restrict__ bflags) {
    __shared__ Tab T;
    __shared__ uint32_t off, claims;
    const uint32_t m = *cnt;
    const int64_t b500 = t0 / 500, b1000 = t0 / 1000;
    tab_clear(T);
    if (threadIdx.x == 0) claims = 0;
    for (uint32_t k = blockIdx.x; k < m; k += gridDim.x) {
        const uint64_t e = list[k];
        const Seg sg = segs[(uint32_t)(e >> 32)];
        const uint32_t piece = (uint32_t)e;
        const uint32_t a = sg.start + piece * AUX_PIECE;
        const uint32_t b = min(a + AUX_PIECE, sg.start + sg.len);
        const bool one = sg.len <= AUX_PIECE;
        const bool chain = seg_chain(S, cfg, sg.res);
        __syncthreads();
        // the piece's updates: (slots, what, windows, count | rt) per event
        int sl[PIECE_EPL][2];
        uint32_t wh[PIECE_EPL], cz[PIECE_EPL];
        int32_t wi[PIECE_EPL], si[PIECE_EPL];
#pragma unroll
        for (int j = 0; j < PIECE_EPL; ++j) {
            const uint32_t p = a + j * 256 + threadIdx.x;
            sl[j][0] = sl[j][1] = -1;
            wh[j] = AW_NONE;
            cz[j] = 0;
            wi[j] = si[j] = 0;
            if (p >= b) continue;
            const SEv r = recs[p];
            uint32_t tag;
            const uint32_t w = aux_what(r, p, recs, dec, chain, &tag);
            if (w == AW_NONE || tag == 0 || (cfg.dbg_flags & 1024)) continue;
            wh[j] = w;
            cz[j] = (uint32_t)r.cnt | ((uint32_t)r.rt << 16);
            const int64_t t = t0 + r.dt;
            wi[j] = (int32_t)(t / 500 - b500);
            si[j] = (int32_t)(t / 1000 - b1000);
            const uint32_t o = tag_origin(tag), cx = tag_ctx(tag);
            if (o) sl[j][0] = tab_find(T, o);
            if (cx) sl[j][1] = tab_find(T, (1u << 31) | cx);
        }
        __syncthreads();
        if (T.overflow) {  // more nodes than slots: the segment is walked by one lane (exact)
            if (one) {
                if (threadIdx.x == 0) aux_walk(recs, dec, S, cfg.max_rt, sg.res, chain, a, b, t0, bflags);
            } else if (threadIdx.x == 0) meta[k] = AUX_NONE;
            __syncthreads();
            tab_clear(T);
            continue;
        }
#pragma unroll
        for (int j = 0; j < PIECE_EPL; ++j)
            for (int u = 0; u < 2; ++u)
                if (sl[j][u] >= 0) tab_p1(T, sl[j][u], wh[j], wi[j], si[j]);
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PIECE_EPL; ++j)
            for (int u = 0; u < 2; ++u)
                if (sl[j][u] >= 0) tab_p2(T, sl[j][u], wh[j], wi[j], si[j], cz[j] & 0xFFFFu, cz[j] >> 16);
        __syncthreads();
        const uint32_t nu = T.nused;
        if (one) {  // the whole segment: commit
            for (uint32_t u = threadIdx.x; u < nu; u += blockDim.x) {
                const uint32_t i = T.used[u];
                AuxAcc A;
                tab_acc(T, i, T.key[i], b500, b1000, A);
                if (!(cfg.dbg_flags & 2048)) aux_commit(S, cfg.max_rt, sg.res, A, bflags, &claims);
            }
        } else {
            if (threadIdx.x == 0) {
                off = atomicAdd(pool_n, nu);
                meta[k] = off + nu <= pool_cap ? (((uint64_t)off << 32) | nu) : (uint64_t)AUX_NONE;
            }
            __syncthreads();
            if (off + nu <= pool_cap)
                for (uint32_t u = threadIdx.x; u < nu; u += blockDim.x) {
                    const uint32_t i = T.used[u];
                    tab_acc(T, i, T.key[i], b500, b1000, pool[off + u]);
                }
        }
        __syncthreads();
        tab_reset_used(T);
        __syncthreads();
        if (threadIdx.x == 0) T.nused = 0;
    }
    __syncthreads();
    if (threadIdx.x == 0) aux_flush_claims(S, claims, bflags);
}

// one multi-piece segment (amulti[k] = seg << 32 | its first piece): the pieces' partials merged in a table with
// 64-bit sums (every thread folds whole pieces), then committed
struct MTab {
    uint32_t key[TAB_S];
    long long W[TAB_S][2], MW[TAB_S][2];
    unsigned long long s[TAB_S][2][4];
    uint32_t minrt[TAB_S][2];
    unsigned long long mpass[TAB_S][2];
    int32_t thread[TAB_S];
    uint32_t used[TAB_S];
    uint32_t nused, overflow;
};
__device__ __forceinline__ int mtab_find(MTab& T, uint32_t key) {
    uint32_t h = (uint32_t)(mix64(key) & (TAB_S - 1));
    for (int probe = 0; probe < TAB_S; ++probe) {
        uint32_t k = __hip_atomic_load(&T.key[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (k == AUX_EMPTY32) {
            k = atomicCAS(&T.key[h], AUX_EMPTY32, key);
            if (k == AUX_EMPTY32) { T.used[atomicAdd(&T.nused, 1u)] = h; return (int)h; }
        }
        if (k == key) return (int)h;
        h = (h + 1) & (TAB_S - 1);
    }
    atomicOr(&T.overflow, 1u);
    return -1;
}
__global__ __launch_bounds__(256) void k_aux_merge(const SEv* __restrict__ recs, const Seg* __restrict__ segs,
                                                   const uint64_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                                                   DevState S, DevCfg cfg, int64_t t0, const uint32_t* __restrict__ dec,
                                                   const AuxAcc* __restrict__ pool, const uint64_t* __restrict__ meta,
                                                   uint32_t* __restrict__ bflags) {
    __shared__ MTab T;
    __shared__ uint32_t bad, claims;
    const uint32_t m = *cnt;
    if (threadIdx.x == 0) claims = 0;
    for (uint32_t k = blockIdx.x; k < m; k += gridDim.x) {
        const uint64_t e = list[k];
        const Seg sg = segs[(uint32_t)(e >> 32)];
        const uint32_t q0 = (uint32_t)e, np = (sg.len + AUX_PIECE - 1) / AUX_PIECE;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < TAB_S; i += blockDim.x) {
            T.key[i] = AUX_EMPTY32;
            T.W[i][0] = T.W[i][1] = T.MW[i][0] = T.MW[i][1] = -1;
            for (int p = 0; p < 2; ++p) {
                for (int c = 0; c < 4; ++c) T.s[i][p][c] = 0;
                T.minrt[i][p] = 0xFFFFFFFFu;
                T.mpass[i][p] = 0;
            }
            T.thread[i] = 0;
        }
        if (threadIdx.x == 0) { bad = 0; T.nused = 0; T.overflow = 0; }
        __syncthreads();
        // phase 1: every thread folds whole pieces (keys, latest windows)
        for (uint32_t q = threadIdx.x; q < np; q += blockDim.x) {
            const uint64_t mt = meta[q0 + q];
            const uint32_t off = (uint32_t)(mt >> 32), n = (uint32_t)mt;
            if (n == AUX_NONE) { bad = 1; continue; }
            for (uint32_t u = 0; u < n; ++u) {
                const AuxAcc& A = pool[off + u];
                const int i = mtab_find(T, A.key);
                if (i < 0) continue;
                for (int p = 0; p < 2; ++p) {
                    if (A.W[p] > T.W[i][p]) atomicMax(&T.W[i][p], (long long)A.W[p]);
                    if (A.MW[p] > T.MW[i][p]) atomicMax(&T.MW[i][p], (long long)A.MW[p]);
                }
            }
        }
        __syncthreads();
        if (bad || T.overflow) {  // a piece without a partial, or more nodes than slots: one lane walks the segment
            if (threadIdx.x == 0)
                aux_walk(recs, dec, S, cfg.max_rt, sg.res, seg_chain(S, cfg, sg.res), sg.start, sg.start + sg.len, t0,
                         bflags);
            continue;
        }
        for (uint32_t q = threadIdx.x; q < np; q += blockDim.x) {
            const uint64_t mt = meta[q0 + q];
            const uint32_t off = (uint32_t)(mt >> 32), n = (uint32_t)mt;
            for (uint32_t u = 0; u < n; ++u) {
                const AuxAcc& A = pool[off + u];
                const int i = mtab_find(T, A.key);
                if (A.thread) atomicAdd(&T.thread[i], A.thread);
                for (int p = 0; p < 2; ++p) {
                    if (A.W[p] >= 0 && A.W[p] == T.W[i][p]) {
                        for (int c = 0; c < 4; ++c)
                            if (A.s[p][c]) atomicAdd(&T.s[i][p][c], (unsigned long long)A.s[p][c]);
                        if (A.minrt[p] != 0xFFFFFFFFu) atomicMin(&T.minrt[i][p], A.minrt[p]);
                    }
                    if (A.MW[p] >= 0 && A.MW[p] == T.MW[i][p] && A.mpass[p])
                        atomicAdd(&T.mpass[i][p], (unsigned long long)A.mpass[p]);
                }
            }
        }
        __syncthreads();
        for (uint32_t u = threadIdx.x; u < T.nused; u += blockDim.x) {
            const uint32_t i = T.used[u];
            AuxAcc A;
            A.key = T.key[i];
            A.thread = T.thread[i];
            for (int p = 0; p < 2; ++p) {
                A.W[p] = T.W[i][p];
                A.MW[p] = T.MW[i][p];
                A.minrt[p] = T.minrt[i][p];
                A.mpass[p] = T.mpass[i][p];
                for (int c = 0; c < 4; ++c) A.s[p][c] = T.s[i][p][c];
            }
            if (!(cfg.dbg_flags & 2048)) aux_commit(S, cfg.max_rt, sg.res, A, bflags, &claims);
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) aux_flush_claims(S, claims, bflags);
}

namespace sg {
// aux[0..3] = short / piece / multi / long counts (device); lists from k_seg_bin
hipError_t launch_aux(const SEv* recs, const Seg* segs, const uint32_t* aux, const uint32_t* ashort,
                      const uint64_t* along, uint64_t* apiece, const uint64_t* amulti, const DevState& S, const DevCfg& cfg,
                      int64_t t0, const uint32_t* dec, AuxAcc* pool, uint32_t pool_cap, uint32_t* pool_n, uint64_t* meta,
                      uint32_t* bflags, hipStream_t st) {
    if (ashort) hipLaunchKernelGGL(k_aux_cold, dim3(2048), dim3(256), 0, st, recs, segs, ashort, aux + 0, S, cfg, t0, dec, bflags);
    hipLaunchKernelGGL(k_aux_expand, dim3(512), dim3(256), 0, st, segs, along, aux + 3, apiece);
    hipLaunchKernelGGL(k_aux_piece, dim3(2048), dim3(256), 0, st, recs, segs, apiece, aux + 1, S, cfg, t0, dec, pool,
                       pool_cap, pool_n, meta, bflags);
    hipLaunchKernelGGL(k_aux_merge, dim3(256), dim3(256), 0, st, recs, segs, amulti, aux + 2, S, cfg, t0, dec, pool, meta,
                       bflags);
    return hipGetLastError();
}
// the short segments' part alone (launch_aux then gets ashort = null)
hipError_t launch_aux_cold(const SEv* recs, const Seg* segs, const uint32_t* aux, const uint32_t* ashort, const DevState& S,
                           const DevCfg& cfg, int64_t t0, const uint32_t* dec, uint32_t* bflags, hipStream_t st) {
    hipLaunchKernelGGL(k_aux_cold, dim3(2048), dim3(256), 0, st, recs, segs, ashort, aux + 0, S, cfg, t0, dec, bflags);
    return hipGetLastError();
}
} // namespace sg
