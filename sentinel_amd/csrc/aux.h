// aux.h -- origin StatisticNodes and context DefaultNodes on the device (dev_types.h AuxNode).
//
// ClusterBuilderSlot keeps one StatisticNode per (resource, origin) (ClusterNode.getOrCreateOriginNode,
// core/slots/clusterbuilder/ClusterBuilderSlot.java:77-106) and NodeSelectorSlot one DefaultNode per (context,
// resource) (core/slots/nodeselector/NodeSelectorSlot.java:136-175); StatisticSlot counts every entry on them
// (StatisticSlot.java:54-173).  Here they are one open-addressing table of 256-byte nodes keyed (resource, kind,
// id), claimed by CAS.  Only the owner of a resource's segment (one k_lane<16> lane, or one aux.hip lane /
// workgroup) touches that resource's nodes in a batch; the CAS only keeps different resources from claiming one
// slot.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "chain.h"

namespace sg {

__device__ __forceinline__ void aux_init(AuxNode* a) {
    a->thread = 0;
    a->flags = 0;
    a->mws[0] = -1; a->mws[1] = -1;
    a->mpass[0] = 0; a->mpass[1] = 0;
    Bkt z;
    z.ws = -1; z.pass = 0; z.block = 0; z.exc = 0; z.succ = 0; z.rt = 0; z.occ = 0; z.minrt = 0;
    a->sec[0] = z;
    a->sec[1] = z;
    a->borrow[0] = -1; a->borrow[1] = 0; a->borrow[2] = -1; a->borrow[3] = 0;
}

// the node of (res, kind, id), created on first use (BF_AUX_FULL once more than aux_cap nodes are claimed).  claims:
// where a new node is counted -- a workgroup's LDS counter the kernel adds to aux_count once (aux_flush_claims), or
// null for aux_count itself; *fresh (optional): the node was created here (its state is aux_init's)
__device__ __forceinline__ AuxNode* aux_get(const DevState& S, uint32_t res, uint32_t kind, uint32_t id, uint32_t* bflags,
                                            uint32_t* claims = nullptr, bool* fresh = nullptr) {
    if (fresh) *fresh = false;
    const unsigned long long key = ((unsigned long long)res << 32) | ((unsigned long long)kind << 31) | (id & 0x7FFFFFFFu);
    uint64_t h = mix64(key) & S.aux_mask;
    for (uint64_t probe = 0; probe <= S.aux_mask; ++probe) {
        AuxNode* a = &S.aux_tab[h];
        unsigned long long k = __hip_atomic_load(&a->key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == key) return a;
        if (k == AUX_EMPTY) {
            unsigned long long expect = AUX_EMPTY;
            if (__hip_atomic_compare_exchange_strong(&a->key, &expect, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)) {
                if (claims) atomicAdd(claims, 1u);
                else if (atomicAdd(S.aux_count, 1u) >= S.aux_cap) atomicOr(bflags, BF_AUX_FULL);
                if (fresh) *fresh = true;
                else aux_init(a);
                return a;
            }
            if (expect == key) return a;
        }
        h = (h + 1) & S.aux_mask;
    }
    atomicOr(bflags, BF_AUX_FULL);
    return nullptr;
}

// Minute window of a node: the pass of the second before t (ArrayMetric.previousWindowPass via
// LeapArray.getPreviousWindow, LeapArray.java:216-234): found iff it is its parity's latest pass-second
__device__ __forceinline__ int64_t aux_prev_pass(const AuxNode* a, int64_t t) {
    const int64_t P = t - t % 1000 - 1000;
    const int q = (int)((P / 1000) & 1);
    return a->mws[q] == P ? a->mpass[q] : 0;
}
// addPassRequest / addOccupiedPass on the minute window at t
__device__ __forceinline__ void aux_add_mpass(AuxNode* a, int64_t t, int64_t cnt) {
    const int64_t T = t - t % 1000;
    const int q = (int)((T / 1000) & 1);
    if (a->mws[q] == T) a->mpass[q] += cnt;
    else if (a->mws[q] < T) { a->mws[q] = T; a->mpass[q] = cnt; }
}

__device__ __forceinline__ void node_load_aux(Node& N, AuxNode* a) {
    N.sb[0] = a->sec[0];
    N.sb[1] = a->sec[1];
    N.thread = a->thread;
    N.flags = 0;
    N.exc_sum_sec = -1;
    N.exc_sum = 0;
    N.mslot = -1;
    N.pfslot = -2;
    N.mst = 0;
    N.bor = a->borrow;  // always consulted: a bucket borrows only what a prioritized entry on this node put there
}
__device__ __forceinline__ void node_store_aux(const Node& N, AuxNode* a) {
    a->sec[0] = N.sb[0];
    a->sec[1] = N.sb[1];
    a->thread = N.thread;
}

// One node's merged updates (AuxAcc, times absolute) into the node: per 500 ms parity the later window replaces
// the node's bucket (reset, with the pass its borrow bucket holds: OccupiableBucketLeapArray.resetWindowTo) and the
// same window adds (LeapArray.currentWindow, LeapArray.java:117-208); likewise the minute pass history
__device__ __forceinline__ void aux_commit(const DevState& S, int32_t max_rt, uint32_t res, const AuxAcc& A,
                                           uint32_t* bflags, uint32_t* claims = nullptr) {
    bool fresh;
    AuxNode* a = aux_get(S, res, A.key >> 31, A.key & 0x7FFFFFFFu, bflags, claims, &fresh);
    if (!a) return;
    if (fresh) {  // a new node: its whole state written at once, nothing read back
        a->thread = A.thread;
        a->flags = 0;
#pragma unroll
        for (int q = 0; q < 2; ++q) { a->mws[q] = A.MW[q]; a->mpass[q] = A.MW[q] < 0 ? 0 : (int64_t)A.mpass[q]; }
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            Bkt b;
            const int64_t mrt = A.minrt[p] == 0xFFFFFFFFu ? INT64_MAX : (int64_t)A.minrt[p];
            b.ws = A.W[p];
            b.pass = A.W[p] < 0 ? 0 : (int64_t)A.s[p][0];
            b.block = A.W[p] < 0 ? 0 : (int64_t)A.s[p][1];
            b.exc = 0;
            b.succ = A.W[p] < 0 ? 0 : (int64_t)A.s[p][2];
            b.rt = A.W[p] < 0 ? 0 : (int64_t)A.s[p][3];
            b.occ = 0;
            b.minrt = A.W[p] < 0 ? 0 : (mrt < max_rt ? mrt : max_rt);
            a->sec[p] = b;
        }
        a->borrow[0] = -1; a->borrow[1] = 0; a->borrow[2] = -1; a->borrow[3] = 0;
        return;
    }
    a->thread += A.thread;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        if (A.MW[q] < 0) continue;
        if (A.MW[q] > a->mws[q]) { a->mws[q] = A.MW[q]; a->mpass[q] = (int64_t)A.mpass[q]; }
        else if (A.MW[q] == a->mws[q]) a->mpass[q] += (int64_t)A.mpass[q];
    }
    const uint32_t fl = a->flags;
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        if (A.W[p] < 0) continue;
        Bkt b = a->sec[p];
        const int64_t mrt = A.minrt[p] == 0xFFFFFFFFu ? INT64_MAX : (int64_t)A.minrt[p];
        if (A.W[p] > b.ws) {
            int64_t bp = 0;
            if (fl & AUXF_BORROW) {
                const int64_t bws = a->borrow[2 * p];
                if (bws >= 0 && bws <= A.W[p] && A.W[p] < bws + 500) bp = a->borrow[2 * p + 1];
            }
            b.ws = A.W[p];
            b.pass = bp + (int64_t)A.s[p][0];
            b.block = (int64_t)A.s[p][1];
            b.exc = 0;
            b.succ = (int64_t)A.s[p][2];
            b.rt = (int64_t)A.s[p][3];
            b.occ = 0;
            b.minrt = mrt < max_rt ? mrt : max_rt;
        } else if (A.W[p] == b.ws) {
            b.pass += (int64_t)A.s[p][0];
            b.block += (int64_t)A.s[p][1];
            b.succ += (int64_t)A.s[p][2];
            b.rt += (int64_t)A.s[p][3];
            if (mrt < b.minrt) b.minrt = mrt;
        } else {
            continue;  // an older window than the node's (the clock went back): lost, as a detached bucket
        }
        a->sec[p] = b;
    }
}

// a workgroup's claimed nodes into aux_count (one atomic a workgroup), the capacity check
__device__ __forceinline__ void aux_flush_claims(const DevState& S, uint32_t n, uint32_t* bflags) {
    if (n && atomicAdd(S.aux_count, n) + n > S.aux_cap) atomicOr(bflags, BF_AUX_FULL);
}

} // namespace sg
