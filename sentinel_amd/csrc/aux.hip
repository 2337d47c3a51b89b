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
//   * k_aux_short : one lane per segment of <= AUX_SHORT events, walking it with a 4-node register cache;
//   * k_aux_piece : one workgroup per AUX_PIECE events of a longer segment: an LDS table of the piece's nodes,
//                   merged in two phases (the latest window of every node-parity, then the sums of that window);
//                   a one-piece segment commits its nodes, the pieces of a longer one leave partial AuxAccs;
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

#define AUX_K 4           // k_aux_short: nodes cached per lane
#define AUX_S 512         // k_aux_piece / k_aux_merge: LDS node slots (power of two)
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

__global__ __launch_bounds__(256) void k_aux_short(const SEv* __restrict__ recs, const Seg* __restrict__ segs,
                                                   const uint32_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                                                   DevState S, DevCfg cfg, int64_t t0, const uint32_t* __restrict__ dec,
                                                   uint32_t* __restrict__ bflags) {
    const uint32_t m = *cnt;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
        const Seg sg = segs[list[i]];
        aux_walk(recs, dec, S, cfg.max_rt, sg.res, seg_chain(S, cfg, sg.res), sg.start, sg.start + sg.len, t0, bflags);
    }
}

// ---------------------------------------------------------------- the LDS node table (pieces, merges)
struct AuxTab {
    uint32_t key[AUX_S];
    int64_t W[AUX_S][2], MW[AUX_S][2];   // latest windows (absolute ms; -1 none)
    unsigned long long s[AUX_S][2][4];
    uint32_t minrt[AUX_S][2];
    unsigned long long mpass[AUX_S][2];
    int32_t thread[AUX_S];
    uint32_t used[AUX_S];                // slots in use, in insertion order
    uint32_t nused, overflow;
};

__device__ __forceinline__ void tab_init(AuxTab& T) {
    for (uint32_t i = threadIdx.x; i < AUX_S; i += blockDim.x) {
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
// the slot of key (inserted on first sight); -1 when the table is full
__device__ __forceinline__ int tab_slot(AuxTab& T, uint32_t key) {
    uint32_t h = (uint32_t)(mix64(key) & (AUX_S - 1));
    for (int probe = 0; probe < AUX_S; ++probe) {
        const uint32_t old = atomicCAS(&T.key[h], AUX_EMPTY32, key);
        if (old == AUX_EMPTY32) { T.used[atomicAdd(&T.nused, 1u)] = h; return (int)h; }
        if (old == key) return (int)h;
        h = (h + 1) & (AUX_S - 1);
    }
    atomicOr(&T.overflow, 1u);
    return -1;
}
__device__ __forceinline__ void tab_acc(const AuxTab& T, uint32_t i, AuxAcc& A) {
    A.key = T.key[i];
    A.thread = T.thread[i];
    for (int p = 0; p < 2; ++p) {
        A.W[p] = T.W[i][p];
        A.MW[p] = T.MW[i][p];
        A.minrt[p] = T.minrt[i][p];
        A.mpass[p] = T.mpass[i][p];
        for (int k = 0; k < 4; ++k) A.s[p][k] = T.s[i][p][k];
    }
}

// One piece of a long segment: apiece[k] = seg << 32 | piece.  meta[k] = pool offset << 32 | count of its partial
// (count AUX_NONE: the piece overflowed; a one-piece segment commits instead and leaves no meta).
#define PIECE_EPL (AUX_PIECE / 256)
__global__ __launch_bounds__(256) void k_aux_piece(const SEv* __restrict__ recs, const Seg* __restrict__ segs,
                                                   const uint64_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                                                   DevState S, DevCfg cfg, int64_t t0, const uint32_t* __restrict__ dec,
                                                   AuxAcc* __restrict__ pool, uint32_t pool_cap,
                                                   uint32_t* __restrict__ pool_n, uint64_t* __restrict__ meta,
                                                   uint32_t* __restrict__ bflags) {
    __shared__ AuxTab T;
    const uint32_t m = *cnt;
    for (uint32_t k = blockIdx.x; k < m; k += gridDim.x) {
        const uint64_t e = list[k];
        const Seg sg = segs[(uint32_t)(e >> 32)];
        const uint32_t piece = (uint32_t)e;
        const uint32_t a = sg.start + piece * AUX_PIECE;
        const uint32_t b = min(a + AUX_PIECE, sg.start + sg.len);
        const bool one = sg.len <= AUX_PIECE;
        const bool chain = seg_chain(S, cfg, sg.res);
        __syncthreads();  // the previous piece's table is read out
        tab_init(T);
        __syncthreads();
        // the piece's updates: (slot, what, window, second, count, rt) per event, two nodes each
        int sl[PIECE_EPL][2];
        uint32_t wh[PIECE_EPL], cz[PIECE_EPL];
        int64_t tt[PIECE_EPL];
#pragma unroll
        for (int j = 0; j < PIECE_EPL; ++j) {
            const uint32_t p = a + j * 256 + threadIdx.x;
            sl[j][0] = sl[j][1] = -1;
            wh[j] = AW_NONE;
            cz[j] = 0;
            tt[j] = 0;
            if (p >= b) continue;
            const SEv r = recs[p];
            uint32_t tag;
            const uint32_t w = aux_what(r, p, recs, dec, chain, &tag);
            if (w == AW_NONE || tag == 0) continue;
            wh[j] = w;
            cz[j] = (uint32_t)r.cnt | ((uint32_t)r.rt << 16);
            tt[j] = t0 + r.dt;
            const uint32_t o = tag_origin(tag), cx = tag_ctx(tag);
            if (o) sl[j][0] = tab_slot(T, o);
            if (cx) sl[j][1] = tab_slot(T, (1u << 31) | cx);
        }
        __syncthreads();
        if (T.overflow) {  // more nodes than slots: the segment is walked by one lane (exact)
            if (one) {
                if (threadIdx.x == 0) aux_walk(recs, dec, S, cfg.max_rt, sg.res, chain, a, b, t0, bflags);
            } else if (threadIdx.x == 0) meta[k] = AUX_NONE;
            continue;
        }
        // phase 1: the latest window of every node-parity (and pass-second of every node-second-parity)
#pragma unroll
        for (int j = 0; j < PIECE_EPL; ++j) {
            if (wh[j] == AW_NONE) continue;
            const int64_t W = tt[j] - tt[j] % 500, M = tt[j] - tt[j] % 1000;
            const int p = (int)((W / 500) & 1), q = (int)((M / 1000) & 1);
            for (int u = 0; u < 2; ++u) {
                const int i = sl[j][u];
                if (i < 0) continue;
                atomicMax((long long*)&T.W[i][p], (long long)W);
                if (wh[j] == AW_PASS) atomicMax((long long*)&T.MW[i][q], (long long)M);
            }
        }
        __syncthreads();
        // phase 2: the sums of those windows, the thread deltas
#pragma unroll
        for (int j = 0; j < PIECE_EPL; ++j) {
            if (wh[j] == AW_NONE) continue;
            const int64_t W = tt[j] - tt[j] % 500, M = tt[j] - tt[j] % 1000;
            const int p = (int)((W / 500) & 1), q = (int)((M / 1000) & 1);
            const uint32_t c = cz[j] & 0xFFFFu, rt = cz[j] >> 16;
            for (int u = 0; u < 2; ++u) {
                const int i = sl[j][u];
                if (i < 0) continue;
                if (wh[j] == AW_PASS) {
                    atomicAdd(&T.thread[i], 1);
                    if (T.W[i][p] == W) atomicAdd(&T.s[i][p][0], (unsigned long long)c);
                    if (T.MW[i][q] == M) atomicAdd(&T.mpass[i][q], (unsigned long long)c);
                } else if (wh[j] == AW_BLOCK) {
                    if (T.W[i][p] == W) atomicAdd(&T.s[i][p][1], (unsigned long long)c);
                } else {
                    atomicAdd(&T.thread[i], -1);
                    if (T.W[i][p] == W) {
                        atomicAdd(&T.s[i][p][2], (unsigned long long)c);
                        atomicAdd(&T.s[i][p][3], (unsigned long long)rt);
                        atomicMin(&T.minrt[i][p], rt);
                    }
                }
            }
        }
        __syncthreads();
        const uint32_t nu = T.nused;
        if (one) {  // the whole segment: commit
            for (uint32_t u = threadIdx.x; u < nu; u += blockDim.x) {
                AuxAcc A;
                tab_acc(T, T.used[u], A);
                aux_commit(S, cfg.max_rt, sg.res, A, bflags);
            }
            continue;
        }
        __shared__ uint32_t off;
        if (threadIdx.x == 0) {
            off = atomicAdd(pool_n, nu);
            meta[k] = off + nu <= pool_cap ? (((uint64_t)off << 32) | nu) : (uint64_t)AUX_NONE;
        }
        __syncthreads();
        if (off + nu <= pool_cap)
            for (uint32_t u = threadIdx.x; u < nu; u += blockDim.x) tab_acc(T, T.used[u], pool[off + u]);
    }
}

// one multi-piece segment: amulti[k] = seg << 32 | its first piece's index in the piece list
__global__ __launch_bounds__(256) void k_aux_merge(const SEv* __restrict__ recs, const Seg* __restrict__ segs,
                                                   const uint64_t* __restrict__ list, const uint32_t* __restrict__ cnt,
                                                   DevState S, DevCfg cfg, int64_t t0, const uint32_t* __restrict__ dec,
                                                   const AuxAcc* __restrict__ pool, const uint64_t* __restrict__ meta,
                                                   uint32_t* __restrict__ bflags) {
    __shared__ AuxTab T;
    __shared__ uint32_t bad;
    const uint32_t m = *cnt;
    for (uint32_t k = blockIdx.x; k < m; k += gridDim.x) {
        const uint64_t e = list[k];
        const Seg sg = segs[(uint32_t)(e >> 32)];
        const uint32_t q0 = (uint32_t)e, np = (sg.len + AUX_PIECE - 1) / AUX_PIECE;
        __syncthreads();
        tab_init(T);
        if (threadIdx.x == 0) bad = 0;
        __syncthreads();
        for (uint32_t q = threadIdx.x; q < np; q += blockDim.x)
            if ((uint32_t)meta[q0 + q] == AUX_NONE) bad = 1;
        __syncthreads();
        // phase 1 over every partial of every piece: keys, latest windows
        for (uint32_t q = 0; q < np && !bad; ++q) {
            const uint64_t mt = meta[q0 + q];
            const uint32_t off = (uint32_t)(mt >> 32), n = (uint32_t)mt;
            for (uint32_t u = threadIdx.x; u < n; u += blockDim.x) {
                const AuxAcc& A = pool[off + u];
                const int i = tab_slot(T, A.key);
                if (i < 0) continue;
                for (int p = 0; p < 2; ++p) {
                    if (A.W[p] >= 0) atomicMax((long long*)&T.W[i][p], (long long)A.W[p]);
                    if (A.MW[p] >= 0) atomicMax((long long*)&T.MW[i][p], (long long)A.MW[p]);
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
        for (uint32_t q = 0; q < np; ++q) {
            const uint64_t mt = meta[q0 + q];
            const uint32_t off = (uint32_t)(mt >> 32), n = (uint32_t)mt;
            for (uint32_t u = threadIdx.x; u < n; u += blockDim.x) {
                const AuxAcc& A = pool[off + u];
                const int i = tab_slot(T, A.key);
                atomicAdd(&T.thread[i], A.thread);
                for (int p = 0; p < 2; ++p) {
                    if (A.W[p] >= 0 && A.W[p] == T.W[i][p]) {
                        for (int c = 0; c < 4; ++c) atomicAdd(&T.s[i][p][c], (unsigned long long)A.s[p][c]);
                        atomicMin(&T.minrt[i][p], A.minrt[p]);
                    }
                    if (A.MW[p] >= 0 && A.MW[p] == T.MW[i][p]) atomicAdd(&T.mpass[i][p], (unsigned long long)A.mpass[p]);
                }
            }
        }
        __syncthreads();
        for (uint32_t u = threadIdx.x; u < T.nused; u += blockDim.x) {
            AuxAcc A;
            tab_acc(T, T.used[u], A);
            aux_commit(S, cfg.max_rt, sg.res, A, bflags);
        }
    }
}

namespace sg {
// aux[0..2] = short / piece / multi counts (device); lists from k_seg_bin
hipError_t launch_aux(const SEv* recs, const Seg* segs, const uint32_t* aux, const uint32_t* ashort,
                      const uint64_t* apiece, const uint64_t* amulti, const DevState& S, const DevCfg& cfg, int64_t t0,
                      const uint32_t* dec, AuxAcc* pool, uint32_t pool_cap, uint32_t* pool_n, uint64_t* meta,
                      uint32_t* bflags, hipStream_t st) {
    hipLaunchKernelGGL(k_aux_short, dim3(1024), dim3(256), 0, st, recs, segs, ashort, aux + 0, S, cfg, t0, dec, bflags);
    hipLaunchKernelGGL(k_aux_piece, dim3(2048), dim3(256), 0, st, recs, segs, apiece, aux + 1, S, cfg, t0, dec, pool,
                       pool_cap, pool_n, meta, bflags);
    hipLaunchKernelGGL(k_aux_merge, dim3(256), dim3(256), 0, st, recs, segs, amulti, aux + 2, S, cfg, t0, dec, pool, meta,
                       bflags);
    return hipGetLastError();
}
} // namespace sg
