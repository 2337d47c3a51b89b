// cluster.hip -- the token server's decision path: batched TokenService.requestToken.
//
// Reference (csrv/ = sentinel-cluster/sentinel-cluster-server-default/.../cluster/):
//   DefaultTokenService.requestToken   csrv/flow/DefaultTokenService.java:37-48
//   ClusterFlowChecker.acquireClusterToken   csrv/flow/ClusterFlowChecker.java:55-112
//   ClusterMetric / ClusterMetricLeapArray    csrv/flow/statistic/metric/ClusterMetric.java:39-98,
//                                             ClusterMetricLeapArray.java:35-91
//   GlobalRequestLimiter / RequestLimiter     csrv/flow/statistic/limit/GlobalRequestLimiter.java:46-54,
//                                             RequestLimiter.java:31-87 (UnaryLeapArray(10, 1000))
//
// A batch of requests (time-ordered) is decided in three device steps:
//   1. k_tok_classify  (parallel)  BAD_REQUEST / NO_RULE_EXISTS, flowId -> flow index (hash table);
//   2. k_tok_limiter   (one wave)  the namespace's GlobalRequestLimiter, in request order.  Inside one
//                                  100 ms bucket the set of valid buckets is fixed, so the passes of a
//                                  bucket are a prefix of its requests: one step per bucket, not per
//                                  request;
//   3. stable radix sort of the limiter-passed requests by flow index (kernels.hip), then
//      k_tok_flow (one lane per flowId) runs acquireClusterToken over the flow's requests in order
//      against the flow's ClusterMetric, kept in HBM between batches.
// Every flowId's window is touched only by its own requests, so step 3 is independent per flowId.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "chain.h"

namespace sg {

#define NO_FLOW 0xFFFFFFFFu

__device__ __forceinline__ uint64_t tab_hash(int64_t k) {
    uint64_t z = (uint64_t)k + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ uint32_t tab_find(const CSlot* __restrict__ tab, uint32_t mask, int64_t key) {
    uint64_t h = tab_hash(key) & mask;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        const CSlot s = tab[h];
        if (s.idx == NO_FLOW) return NO_FLOW;
        if (s.key == key) return s.idx;
        h = (h + 1) & mask;
    }
    return NO_FLOW;
}

// 1. DefaultTokenService.requestToken: notValidRequest -> BAD_REQUEST; no rule -> NO_RULE_EXISTS
__global__ void k_tok_classify(const sg_token_req* __restrict__ req, uint64_t n, const CSlot* __restrict__ tab,
                               uint32_t mask, uint32_t* __restrict__ fidx, sg_token_result* __restrict__ res,
                               uint32_t* __restrict__ flags) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const sg_token_req q = req[i];
    if (i > 0 && q.ts < req[i - 1].ts) atomicOr(flags, 1u);  // requests must be time-ordered
    sg_token_result r;
    r.status = SG_TOKEN_OK; r.remaining = 0; r.wait_in_ms = 0; r.reserved = 0;
    uint32_t f = NO_FLOW;
    if (q.flow_id <= 0 || q.acquire_count <= 0) r.status = SG_TOKEN_BAD_REQUEST;
    else {
        f = tab_find(tab, mask, q.flow_id);
        if (f == NO_FLOW) r.status = SG_TOKEN_NO_RULE_EXISTS;
    }
    fidx[i] = f;
    res[i] = r;
}

// 2. GlobalRequestLimiter.tryPass of the namespace: RequestLimiter.canPass is
//    sum(valid buckets)/1.0 + 1 <= qpsAllowed, then add(1) to the current 100 ms bucket.
//    One wave, 64 requests per step, one sub-step per distinct bucket among them.
__global__ __launch_bounds__(64) void k_tok_limiter(const sg_token_req* __restrict__ req, uint64_t n,
                                                    const uint32_t* __restrict__ fidx, uint32_t nflows,
                                                    NsLimiter* __restrict__ lim, double allowed,
                                                    uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                    sg_token_result* __restrict__ res) {
    const uint32_t lane = threadIdx.x;
    // limiter ring in registers of lanes 0..9: (ws, count); ws < 0 = never created
    int64_t lws = lane < NS_BUCKETS ? lim->ws[lane] : -1;
    int64_t lcnt = lane < NS_BUCKETS ? lim->cnt[lane] : 0;
    const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (uint64_t base = 0; base < n; base += 64) {
        const uint64_t i = base + lane;
        const bool valid = i < n;
        const int64_t t = valid ? req[i].ts : 0;
        const uint32_t f = valid ? fidx[i] : NO_FLOW;
        bool todo = valid && f != NO_FLOW;
        uint32_t key = nflows;
        for (;;) {
            const uint64_t pend = __ballot(todo);
            if (!pend) break;
            const int L = __ffsll((unsigned long long)pend) - 1;
            const int64_t tb = __shfl(t, L, 64);
            const int64_t b = tb / NS_WLEN;
            const uint64_t grp = __ballot(todo && t / NS_WLEN == b);
            const int m = __popcll(grp);
            // LeapArray.currentWindow(tb): create / reset the bucket's slot
            const int64_t wsb = tb - tb % NS_WLEN;
            const int idx = (int)(b % NS_BUCKETS);
            if (lane == (uint32_t)idx && (lws < 0 || wsb > lws)) { lws = wsb; lcnt = 0; }
            // sum over the valid buckets (isWindowDeprecated: t - ws > interval, strict)
            int64_t s = (lane < NS_BUCKETS && lws >= 0 && tb - lws <= NS_INTERVAL) ? lcnt : 0;
#pragma unroll
            for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o, 64);
            s = __shfl(s, 0, 64);
            // passes of this bucket: the first k requests with (double)(s + j) + 1 <= allowed
            int64_t k = 0;
            if ((double)s + 1.0 <= allowed) {
                double room = allowed - 1.0 - (double)s;
                int64_t jm = room >= 64.0 ? 63 : (int64_t)room;
                while (jm + 1 < m && (double)(s + jm + 1) + 1.0 <= allowed) ++jm;
                while (jm >= 0 && !((double)(s + jm) + 1.0 <= allowed)) --jm;
                k = jm + 1 < m ? jm + 1 : m;
            }
            if (lane == (uint32_t)idx) lcnt += k;
            if ((grp >> lane) & 1) {
                const int r = __popcll(grp & lt);
                if (r < k) key = f;
                else res[i].status = SG_TOKEN_TOO_MANY_REQUEST;
                todo = false;
            }
        }
        if (valid) { keys[i] = key; vals[i] = (uint32_t)i; }
    }
    if (lane < NS_BUCKETS) { lim->ws[lane] = lws; lim->cnt[lane] = lcnt; }
}

// ---- ClusterMetric of one flow (thread-private during the batch)
struct CMetric {
    CFlow* f;
    CBkt* b;
    int64_t wlen;
    CBkt scratch;  // LeapArray.currentWindow of a time before the slot's start: a detached bucket
};

// LeapArray.currentWindow + ClusterMetricLeapArray.resetWindowTo/transferOccupyToBucket
__device__ CBkt* cm_current(CMetric& M, int64_t now) {
    const int n = M.f->n;
    const int idx = (int)((now / M.wlen) % n);
    const int64_t ws = now - now % M.wlen;
    CBkt* old = &M.b[idx];
    if (old->ws < 0) {  // newEmptyBucket: no transfer
        old->ws = ws;
        for (int k = 0; k < CF_N; ++k) old->c[k] = 0;
        return old;
    }
    if (ws == old->ws) return old;
    if (ws > old->ws) {
        old->ws = ws;
        for (int k = 0; k < CF_N; ++k) old->c[k] = 0;
        if (M.f->has_occ) {
            old->c[CF_OCC_PASS] += M.f->occ_pass;  // transferOccupiedCount (sum, not reset)
            old->c[CF_PASS] += M.f->occ_pass;      // transferOccupiedThenReset
            old->c[CF_PASS_REQ] += M.f->occ_req;
            M.f->occ_pass = 0;
            M.f->occ_req = 0;
            M.f->has_occ = 0;
        }
        return old;
    }
    M.scratch.ws = ws;
    for (int k = 0; k < CF_N; ++k) M.scratch.c[k] = 0;
    return &M.scratch;
}
__device__ int64_t cm_sum(CMetric& M, int64_t now, int ev) {
    cm_current(M, now);
    int64_t s = 0;
    for (int i = 0; i < M.f->n; ++i) {
        const CBkt& w = M.b[i];
        if (w.ws < 0 || now - w.ws > M.f->interval) continue;
        s += w.c[ev];
    }
    return s;
}
__device__ double cm_avg(CMetric& M, int64_t now, int ev) {
    return (double)cm_sum(M, now, ev) / (M.f->interval / 1000.0);
}
__device__ void cm_add(CMetric& M, int64_t now, int ev, int64_t v) { cm_current(M, now)->c[ev] += v; }

// 3. ClusterFlowChecker.acquireClusterToken over one flow's requests (sorted positions [lo, hi))
__global__ void k_tok_flow(const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ svals, uint64_t n,
                           const sg_token_req* __restrict__ req, CFlow* __restrict__ flows, uint32_t nflows,
                           CBkt* __restrict__ bkts, double exceed, double max_occ_ratio,
                           sg_token_result* __restrict__ res) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nflows) return;
    // lower_bound(skeys, f), lower_bound(skeys, f + 1)
    uint64_t lo = 0, hi = n;
    while (lo < hi) { const uint64_t mid = (lo + hi) / 2; if (skeys[mid] < f) lo = mid + 1; else hi = mid; }
    uint64_t e = lo, h2 = n;
    while (e < h2) { const uint64_t mid = (e + h2) / 2; if (skeys[mid] <= f) e = mid + 1; else h2 = mid; }
    if (lo == e) return;
    CMetric M;
    M.f = &flows[f];
    M.b = bkts + M.f->boff;
    M.wlen = M.f->interval / M.f->n;
    const double thr = M.f->thr_type == SG_CLUSTER_THRESHOLD_GLOBAL ? M.f->count : M.f->count * (double)M.f->connected;
    const double global_threshold = thr * exceed;  // calcGlobalThreshold * exceedCount
    for (uint64_t p = lo; p < e; ++p) {
        const uint32_t i = svals[p];
        const sg_token_req q = req[i];
        const int64_t now = q.ts;
        sg_token_result o;
        o.status = SG_TOKEN_BLOCKED; o.remaining = 0; o.wait_in_ms = 0; o.reserved = 0;
        const double latest_qps = cm_avg(M, now, CF_PASS_REQ);
        const double next_remaining = global_threshold - latest_qps - q.acquire_count;
        if (next_remaining >= 0) {
            cm_add(M, now, CF_PASS, q.acquire_count);
            cm_add(M, now, CF_PASS_REQ, 1);
            if (q.prioritized) cm_add(M, now, CF_OCC_PASS, q.acquire_count);
            o.status = SG_TOKEN_OK;
            o.remaining = j_d2i(next_remaining);  // (int) nextRemaining
            res[i] = o;
            continue;
        }
        if (q.prioritized) {
            const double occupy_avg = cm_avg(M, now, CF_WAITING);
            if (occupy_avg <= max_occ_ratio * global_threshold) {
                // ClusterMetric.tryOccupyNext / canOccupy (ClusterMetric.java:78-98)
                const double lq = cm_avg(M, now, CF_PASS);
                cm_current(M, now);
                int64_t head_pass = 0;  // getFirstCountOfWindow: LeapArray.getValidHead
                {
                    const int hidx = (int)(((now + M.wlen) / M.wlen) % M.f->n);
                    const CBkt& w = M.b[hidx];
                    if (w.ws >= 0 && !(now - w.ws > M.f->interval)) head_pass = w.c[CF_PASS];
                }
                const int64_t occupied = M.f->occ_pass;
                if (lq + (double)((int64_t)q.acquire_count + occupied) - (double)head_pass <= global_threshold) {
                    M.f->occ_pass += q.acquire_count;  // addOccupyPass
                    M.f->occ_req += 1;
                    M.f->has_occ = 1;
                    cm_add(M, now, CF_WAITING, q.acquire_count);
                    const int wait = 1000 / M.f->n;
                    if (wait > 0) {
                        o.status = SG_TOKEN_SHOULD_WAIT;
                        o.wait_in_ms = wait;
                        res[i] = o;
                        continue;
                    }
                }
            }
        }
        cm_add(M, now, CF_BLOCK, q.acquire_count);
        cm_add(M, now, CF_BLOCK_REQ, 1);
        if (q.prioritized) cm_add(M, now, CF_OCC_BLOCK, q.acquire_count);
        res[i] = o;
    }
}

hipError_t launch_tok_classify(const sg_token_req* req, uint64_t n, const CSlot* tab, uint32_t mask, uint32_t* fidx,
                               sg_token_result* res, uint32_t* flags, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_tok_classify, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, req, n, tab, mask, fidx, res,
                       flags);
    return hipGetLastError();
}
hipError_t launch_tok_limiter(const sg_token_req* req, uint64_t n, const uint32_t* fidx, uint32_t nflows,
                              NsLimiter* lim, double allowed, uint32_t* keys, uint32_t* vals, sg_token_result* res,
                              hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_tok_limiter, dim3(1), dim3(64), 0, st, req, n, fidx, nflows, lim, allowed, keys, vals, res);
    return hipGetLastError();
}
hipError_t launch_tok_flow(const uint32_t* skeys, const uint32_t* svals, uint64_t n, const sg_token_req* req,
                           CFlow* flows, uint32_t nflows, CBkt* bkts, double exceed, double max_occ_ratio,
                           sg_token_result* res, hipStream_t st) {
    if (!n || !nflows) return hipSuccess;
    hipLaunchKernelGGL(k_tok_flow, dim3((nflows + 255) / 256), dim3(256), 0, st, skeys, svals, n, req, flows, nflows,
                       bkts, exceed, max_occ_ratio, res);
    return hipGetLastError();
}

// ---- ClusterParamFlowChecker.acquireClusterToken (csrv/flow/ClusterParamFlowChecker.java:42-88)
// One lane per param flow over its requests in time order (sorted positions), like k_tok_flow.  The
// flow's ClusterParameterLeapArray keeps per-bucket value maps; here a value's counts live in a PVal
// slot of an open-addressing table shared by all flows (claimed by CAS on PVal.flow; a lane only ever
// looks up its own flow's values, which it inserted itself, so a lookup never races an insert it needs).
__device__ __forceinline__ int pf_current(PFlow& F, int64_t now) {  // LeapArray.currentWindow (create / reset)
    const int64_t wlen = F.interval / F.n;
    const int idx = (int)((now / wlen) % F.n);
    const int64_t ws = now - now % wlen;
    if (F.fws[idx] < 0 || ws > F.fws[idx]) F.fws[idx] = ws;  // resetWindowTo clears the map: stamps differ
    return idx;
}
__device__ PVal* pv_find(PVal* __restrict__ tab, uint32_t mask, uint32_t f, uint64_t key, bool create,
                         uint32_t* __restrict__ flags) {
    uint64_t h = tab_hash((int64_t)(key ^ ((uint64_t)f * 0xD6E8FEB86659FD93ull))) & mask;
    for (uint32_t probe = 0; probe <= mask; ++probe) {
        PVal* s = &tab[h];
        uint32_t owner = __hip_atomic_load(&s->flow, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (owner == PV_EMPTY) {
            if (!create) return nullptr;
            owner = atomicCAS(&s->flow, PV_EMPTY, f);
            if (owner == PV_EMPTY) {  // claimed: a fresh (flow, value) entry
                s->key = key;
                for (int j = 0; j < CP_MAXN; ++j) { s->ws[j] = -1; s->cnt[j] = 0; }
                return s;
            }
        }
        if (owner == f && s->key == key) return s;
        h = (h + 1) & mask;
    }
    atomicOr(flags, 2u);  // table full
    return nullptr;
}
__global__ void k_ptok_flow(const uint32_t* __restrict__ skeys, const uint32_t* __restrict__ svals, uint64_t n,
                            const sg_param_token_req* __restrict__ req, const uint64_t* __restrict__ values,
                            PFlow* __restrict__ flows, uint32_t nflows, const PHot* __restrict__ hot,
                            PVal* __restrict__ tab, uint32_t mask, sg_token_result* __restrict__ res,
                            uint32_t* __restrict__ flags) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nflows) return;
    uint64_t lo = 0, hi = n;
    while (lo < hi) { const uint64_t mid = (lo + hi) / 2; if (skeys[mid] < f) lo = mid + 1; else hi = mid; }
    uint64_t e = lo, h2 = n;
    while (e < h2) { const uint64_t mid = (e + h2) / 2; if (skeys[mid] <= f) e = mid + 1; else h2 = mid; }
    if (lo == e) return;
    PFlow F = flows[f];
    const double isec = F.interval / 1000.0;  // LeapArray.getIntervalInSecond
    for (uint64_t p = lo; p < e; ++p) {
        const uint32_t i = svals[p];
        const sg_param_token_req q = req[i];
        const int64_t now = q.ts;
        const uint64_t* v = values + q.value_off;
        double remaining = -1.0;
        bool passed = true;
        for (uint32_t k = 0; k < q.n_values; ++k) {
            pf_current(F, now);  // ClusterParamMetric.getSum -> metric.currentWindow()
            int64_t sum = 0;
            const PVal* pv = pv_find(tab, mask, f, v[k], false, flags);
            if (pv) {
                for (int j = 0; j < F.n; ++j) {
                    if (F.fws[j] < 0 || now - F.fws[j] > F.interval) continue;  // isWindowDeprecated (strict >)
                    if (pv->ws[j] == F.fws[j]) sum += pv->cnt[j];
                }
            }
            double raw = F.count;  // getRawThreshold: the exclusive item count, else rule.count
            for (uint32_t hh = 0; hh < F.nhot; ++hh)
                if (hot[F.hoff + hh].key == v[k]) { raw = (double)hot[F.hoff + hh].count; break; }
            const double thr = F.thr_type == SG_CLUSTER_THRESHOLD_GLOBAL ? raw : raw * (double)F.connected;
            const double next = thr - (double)sum / isec - (double)q.acquire_count;
            remaining = next;
            if (next < 0) { passed = false; break; }
        }
        sg_token_result o;
        o.status = SG_TOKEN_BLOCKED; o.remaining = 0; o.wait_in_ms = 0; o.reserved = 0;
        if (passed) {
            for (uint32_t k = 0; k < q.n_values; ++k) {  // addValue to the current bucket of every value
                const int idx = pf_current(F, now);
                PVal* pv = pv_find(tab, mask, f, v[k], true, flags);
                if (!pv) break;
                if (pv->ws[idx] != F.fws[idx]) { pv->ws[idx] = F.fws[idx]; pv->cnt[idx] = 0; }
                pv->cnt[idx] += q.acquire_count;
            }
            if (q.n_values > 1) remaining = -1.0;  // multi-value remaining is unsupported
            o.status = SG_TOKEN_OK;
            o.remaining = j_d2i(remaining);
        }
        res[i] = o;
    }
    flows[f] = F;
}

hipError_t launch_ptok_flow(const uint32_t* skeys, const uint32_t* svals, uint64_t n, const sg_param_token_req* req,
                            const uint64_t* values, PFlow* flows, uint32_t nflows, const PHot* hot, PVal* tab,
                            uint32_t mask, sg_token_result* res, uint32_t* flags, hipStream_t st) {
    if (!n || !nflows) return hipSuccess;
    hipLaunchKernelGGL(k_ptok_flow, dim3((nflows + 255) / 256), dim3(256), 0, st, skeys, svals, n, req, values, flows,
                       nflows, hot, tab, mask, res, flags);
    return hipGetLastError();
}

} // namespace sg
