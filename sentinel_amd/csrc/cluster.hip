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
//   2. the namespace's GlobalRequestLimiter, in request order.  Inside one 100 ms bucket the set of valid
//      buckets is fixed, so the passes of a bucket are a prefix of its candidates: k_lim_walk takes one
//      step per bucket (their candidate counts from a scan), k_lim_apply ranks every request in its
//      bucket (parallel);
//   3. stable radix sort of the limiter-passed requests by flow index (kernels.hip), then k_tok_flow_wg
//      (a workgroup per flowId) runs acquireClusterToken over the flow's requests in time order against
//      the flow's ClusterMetric, kept in HBM between batches.  Inside one window sub-bucket the valid
//      buckets are fixed too, and a request passes iff threshold - (S + P) / intervalSec - acquire >= 0
//      with S the sub-bucket's starting PASS_REQUEST sum and P the passes before it: per request the largest
//      such P (L_j, by bisection on the exact double expression), and the passes follow in a few block-wide
//      phases (one per distinct L_j).  Prioritized requests that fail then try tryOccupyNext in order (one
//      lane: each step is O(1) from prefix sums of the passes).
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

// ---- 2. the limiter, parallel over requests and sequential over 100 ms buckets
// per request: its bucket starts here (first request of its 100 ms bucket), and it is a limiter candidate
__global__ void k_lim_flags(const sg_token_req* __restrict__ req, uint64_t n, const uint32_t* __restrict__ fidx,
                            uint32_t* __restrict__ bflag, uint32_t* __restrict__ cflag) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int64_t b = req[i].ts / NS_WLEN;
    bflag[i] = (i == 0 || req[i - 1].ts / NS_WLEN != b) ? 1u : 0u;
    cflag[i] = fidx[i] != NO_FLOW ? 1u : 0u;
}
// bucket starts: bstart[k] = first request of the k-th bucket (bflag scanned exclusively: its bucket index)
__global__ void k_lim_starts(const uint32_t* __restrict__ bidx, const uint32_t* __restrict__ bflag0, uint64_t n,
                             uint32_t* __restrict__ bstart) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (bflag0[i]) bstart[bidx[i]] = (uint32_t)i;
}
// one lane walks the buckets in order: RequestLimiter.canPass = sum(valid buckets) + 1 <= qpsAllowed, then add(1)
// -- the passes of a bucket are its first kpass[k] candidates (cexcl: candidates before a request)
__global__ void k_lim_walk(const sg_token_req* __restrict__ req, uint64_t n, const uint32_t* __restrict__ bstart,
                           const uint32_t* __restrict__ nbk, const uint32_t* __restrict__ cexcl,
                           const uint32_t* __restrict__ ctot, NsLimiter* __restrict__ lim, double allowed,
                           uint32_t* __restrict__ kpass) {
    if (threadIdx.x != 0) return;
    NsLimiter L = *lim;
    const uint32_t nb = *nbk;
    for (uint32_t k = 0; k < nb; ++k) {
        const uint32_t a = bstart[k];
        const uint32_t m = (k + 1 < nb ? cexcl[bstart[k + 1]] : *ctot) - cexcl[a];
        if (!m) { kpass[k] = 0; continue; }
        const int64_t tb = req[a].ts;  // (every candidate of the bucket: the same bucket, the same valid set)
        const int64_t wsb = tb - tb % NS_WLEN;
        const int idx = (int)((tb / NS_WLEN) % NS_BUCKETS);
        if (L.ws[idx] < 0 || wsb > L.ws[idx]) { L.ws[idx] = wsb; L.cnt[idx] = 0; }
        int64_t s = 0;
        for (int j = 0; j < NS_BUCKETS; ++j)
            if (L.ws[j] >= 0 && tb - L.ws[j] <= NS_INTERVAL) s += L.cnt[j];
        int64_t kp = 0;
        if ((double)s + 1.0 <= allowed) {  // the j-th candidate passes iff (double)(s + j) + 1 <= allowed
            int64_t lo = 0, hi = m;  // largest count kp <= m with (double)(s + kp - 1) + 1 <= allowed
            while (lo < hi) {
                const int64_t mid = (lo + hi + 1) / 2;
                if ((double)(s + mid - 1) + 1.0 <= allowed) lo = mid; else hi = mid - 1;
            }
            kp = lo;
        }
        L.cnt[idx] += kp;
        kpass[k] = (uint32_t)kp;
    }
    *lim = L;
}
// every candidate: passes iff its rank among its bucket's candidates < kpass (else TOO_MANY_REQUEST); the sort key
// (bidx = the exclusive scan of the bucket-start flags: a request's bucket is bidx + bflag - 1)
__global__ void k_lim_apply(const uint64_t n, const uint32_t* __restrict__ fidx, const uint32_t* __restrict__ bflag,
                            const uint32_t* __restrict__ bidx,
                            const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ cexcl,
                            const uint32_t* __restrict__ kpass, uint32_t nflows, uint32_t* __restrict__ keys,
                            uint32_t* __restrict__ vals, sg_token_result* __restrict__ res) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t f = fidx[i];
    uint32_t key = nflows;
    if (f != NO_FLOW) {
        const uint32_t k = bidx[i] + bflag[i] - 1;
        if (cexcl[i] - cexcl[bstart[k]] < kpass[k]) key = f;
        else res[i].status = SG_TOKEN_TOO_MANY_REQUEST;
    }
    keys[i] = key;
    vals[i] = (uint32_t)i;
}

// ---- 3. one flowId's requests, a workgroup of TF_T lanes, chunks of TF_T requests in time order.  A flow's cost is
// one step per chunk plus one per window sub-bucket its requests touch (~20 a flow, up to ~160, over 10k flows), each
// a dozen block-wide scans: a 1024-lane workgroup for a flow with more than `light` requests in the call, a one-wave
// workgroup (the same code, its barriers a single wave's) for the rest, both launches side by side (the engine's
// tok_light, SG_TOK_LIGHT; default 8192).
template <int TF_T>
__device__ __forceinline__ uint32_t tf_scan_excl(uint32_t v, uint32_t* red, uint32_t* total) {
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if ((int)l >= o) x += y;
    }
    __syncthreads();
    if (l == 63) red[w] = x;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
    for (uint32_t k = 0; k < TF_T / 64; ++k) { const uint32_t c = red[k]; if (k < w) pre += c; tot += c; }
    *total = tot;
    return pre + x - v;
}
template <int TF_T>
__device__ __forceinline__ int64_t tf_min(int64_t v, int64_t* red) {
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) { const int64_t y = __shfl_xor(v, o, 64); v = y < v ? y : v; }
    __syncthreads();
    if (l == 0) red[w] = v;
    __syncthreads();
    int64_t m = red[0];
    for (uint32_t k = 1; k < TF_T / 64; ++k) m = red[k] < m ? red[k] : m;
    return m;
}
// six 64-bit sums at once: one wave reduction each, one barrier
template <int TF_T>
__device__ __forceinline__ void tf_sum6(int64_t v[6], int64_t (*red)[6]) {
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 6; ++k)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o, 64);
    __syncthreads();
    if (l == 0)
#pragma unroll
        for (int k = 0; k < 6; ++k) red[w][k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        int64_t m = 0;
        for (uint32_t j = 0; j < TF_T / 64; ++j) m += red[j][k];
        v[k] = m;
    }
}
template <int TF_T>
__device__ __forceinline__ int64_t tf_scan64_excl(int64_t v, int64_t* red) {
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o, 64);
        if ((int)l >= o) x += y;
    }
    __syncthreads();
    if (l == 63) red[w] = x;
    __syncthreads();
    int64_t pre = 0;
    for (uint32_t k = 0; k < w; ++k) pre += red[k];
    return pre + x - v;
}
#define TF_NONE ((int64_t)1 << 62)
#define TF_NB 64  // ClusterMetric windows kept in LDS for the workgroup's life (more samples: in HBM)
enum : uint8_t { TS_BLOCK = 0, TS_PASS = 1, TS_WAIT = 2 };
// bounds[f] = the first sorted position of flow f (lower_bound of the keys), f = 0 .. nflows
__global__ void k_tok_bounds(const uint32_t* __restrict__ skeys, uint64_t n, uint32_t nflows,
                             uint32_t* __restrict__ bounds) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    const int64_t prev = i == 0 ? -1 : (int64_t)skeys[i - 1];
    const int64_t k = i == n ? (int64_t)nflows : (int64_t)skeys[i];
    const int64_t top = k < (int64_t)nflows ? k : (int64_t)nflows;
    for (int64_t f = prev + 1; f <= top; ++f) bounds[f] = (uint32_t)i;
}
// flows with lo_cnt < requests <= hi_cnt
template <int TF_T>
__global__ __launch_bounds__(TF_T) void k_tok_flow_wg(const uint32_t* __restrict__ svals, const uint32_t* __restrict__ bounds,
                                                      uint32_t lo_cnt, uint32_t hi_cnt,
                                                      const sg_token_req* __restrict__ req, CFlow* __restrict__ flows,
                                                      uint32_t nflows, CBkt* __restrict__ bkts, double exceed,
                                                      double max_occ_ratio, sg_token_result* __restrict__ res) {
    __shared__ uint32_t ured[TF_T / 64];
    __shared__ int64_t lred[TF_T / 64];
    __shared__ uint8_t sst[TF_T];     // per position of the chunk: TS_*
    __shared__ int64_t spass[TF_T];   // acquire sum of the run's passes before the position
    __shared__ uint32_t flist[TF_T];  // the run's prioritized requests that failed the normal check, in order
    __shared__ int32_t sacq[TF_T];
    __shared__ int64_t red6[TF_T / 64][6];
    __shared__ CFlow lflow;
    __shared__ CBkt lbkt[TF_NB];
    __shared__ int64_t sh_S, sh_W0, sh_PS0, sh_head, sh_cur0, sh_wadd;
    __shared__ uint32_t sh_seq, sh_headcur;
    const uint32_t f = blockIdx.x, t = threadIdx.x;
    if (f >= nflows) return;
    const uint32_t lo = bounds[f], hi = bounds[f + 1];
    if (hi - lo <= lo_cnt || hi - lo > hi_cnt) return;
    // the flow's metric: its view and windows in LDS while the workgroup runs (lane 0 works on them; written back)
    const CFlow gf = flows[f];
    const bool in_lds = gf.n <= TF_NB;
    if (t == 0) lflow = gf;
    if (in_lds && t < (uint32_t)gf.n) lbkt[t] = bkts[gf.boff + t];
    __syncthreads();
    CMetric M;
    M.f = &lflow;
    M.b = in_lds ? lbkt : bkts + gf.boff;
    M.wlen = M.f->interval / M.f->n;
    const double thr = M.f->thr_type == SG_CLUSTER_THRESHOLD_GLOBAL ? M.f->count : M.f->count * (double)M.f->connected;
    const double gthr = thr * exceed;  // calcGlobalThreshold * exceedCount
    const double isec = M.f->interval / 1000.0;
    const int wait = 1000 / M.f->n;
    for (uint32_t c0 = lo; c0 < hi; c0 += TF_T) {
        const uint32_t cn = min((uint32_t)TF_T, hi - c0);
        uint32_t i = 0;
        int64_t now = 0;
        int32_t acq = 0;
        bool prio = false;
        if (t < cn) {
            i = svals[c0 + t];
            const sg_token_req q = req[i];
            now = q.ts;
            acq = q.acquire_count;
            prio = q.prioritized != 0;
        }
        const int64_t sb = t < cn ? now / M.wlen : -1;
        if (t < cn) sacq[t] = acq;
        // the chunk's sub-bucket runs, one after the other (usually one)
        uint32_t a = 0;
        while (a < cn) {
            __syncthreads();
            if (t == a) {  // the run's window: LeapArray.currentWindow (reset / occupy transfer), then every sum over
                           // the sub-bucket's valid buckets (constant inside it)
                CBkt* cur = cm_current(M, now);
                sh_seq = cur == &M.scratch ? 1u : 0u;  // a time before the slot's window: the sequential path
                sh_S = cm_sum(M, now, CF_PASS_REQ);
                sh_W0 = cm_sum(M, now, CF_WAITING);
                sh_PS0 = cm_sum(M, now, CF_PASS);
                const int hidx = (int)(((now + M.wlen) / M.wlen) % M.f->n);
                const CBkt& hw = M.b[hidx];
                sh_head = (hw.ws >= 0 && !(now - hw.ws > M.f->interval)) ? hw.c[CF_PASS] : 0;
                sh_headcur = &hw == cur ? 1u : 0u;  // (one sample: the head window is the current one)
                sh_cur0 = cur->c[CF_PASS];
                sh_wadd = 0;
                lred[0] = sb;
            }
            __syncthreads();
            const int64_t sba = lred[0];
            uint32_t nrun;
            (void)tf_scan_excl<TF_T>(t < cn && t >= a && sb == sba ? 1u : 0u, ured, &nrun);
            const uint32_t b = a + nrun;  // (positions are time ordered: the run is [a, b))
            const bool in = t >= a && t < b;
            if (sh_seq) {  // the reference's order, request by request
                for (uint32_t c = a; c < b; ++c) {
                    __syncthreads();
                    if (t != c) continue;
                    sg_token_result o;
                    o.status = SG_TOKEN_BLOCKED; o.remaining = 0; o.wait_in_ms = 0; o.reserved = 0;
                    const double nr = gthr - cm_avg(M, now, CF_PASS_REQ) - acq;
                    if (nr >= 0) {
                        cm_add(M, now, CF_PASS, acq);
                        cm_add(M, now, CF_PASS_REQ, 1);
                        if (prio) cm_add(M, now, CF_OCC_PASS, acq);
                        o.status = SG_TOKEN_OK;
                        o.remaining = j_d2i(nr);
                    } else {
                        cm_add(M, now, CF_BLOCK, acq);
                        cm_add(M, now, CF_BLOCK_REQ, 1);
                        if (prio) cm_add(M, now, CF_OCC_BLOCK, acq);
                    }
                    res[i] = o;
                }
                a = b;
                continue;
            }
            const int64_t S = sh_S;
            // L: the largest P >= 0 with gthr - (double)(S + P) / isec - acq >= 0 (-1: none), by bisection on the
            // reference's expression (monotone in P)
            int64_t L = -1;
            if (in && gthr - (double)S / isec - acq >= 0) {
                // near (gthr - acq) * isec - S, then stepped to the exact boundary of the reference's expression
                const double g = (gthr - acq) * isec - (double)S;
                int64_t l2 = g >= 9.0e15 ? ((int64_t)1 << 53) : (g < 0 ? 0 : (int64_t)g);
                while (l2 > 0 && !(gthr - (double)(S + l2) / isec - acq >= 0)) --l2;
                while (l2 < ((int64_t)1 << 53) && gthr - (double)(S + l2 + 1) / isec - acq >= 0) ++l2;
                L = l2;
            }
            // the passes, phase by phase: with P passes so far a request of L < P never passes; the undecided
            // rest pass in order while P <= their smallest L (one phase per distinct L)
            int64_t P = 0, myP = 0;
            bool undec = in, pass = false;
            for (;;) {
                if (undec && L < P) undec = false;
                const int64_t V = tf_min<TF_T>(undec ? L : TF_NONE, lred);
                if (V == TF_NONE) break;
                const int64_t need = V - P + 1;
                uint32_t nu;
                const uint32_t rk = tf_scan_excl<TF_T>(undec ? 1u : 0u, ured, &nu);
                if (undec && (int64_t)rk < need) { pass = true; myP = P + rk; undec = false; }
                if ((int64_t)nu <= need) break;
                P = V + 1;
            }
            // the PASS sum each position sees (the acquire prefix of the run's passes)
            {
                const int64_t ex = tf_scan64_excl<TF_T>(pass ? (int64_t)acq : 0, lred);
                if (in) spass[t] = ex;
            }
            const bool fp = in && !pass && prio;  // tries tryOccupyNext
            uint32_t nfp;
            const uint32_t fr = tf_scan_excl<TF_T>(fp ? 1u : 0u, ured, &nfp);
            if (fp) flist[fr] = t;
            if (in) sst[t] = pass ? TS_PASS : TS_BLOCK;
            __syncthreads();
            if (t == 0 && nfp) {  // tryOccupyNext in request order (ClusterMetric.java:78-98)
                int64_t wadd = 0;
                for (uint32_t k = 0; k < nfp; ++k) {
                    const uint32_t c = flist[k];
                    const double occupy_avg = (double)(sh_W0 + wadd) / isec;
                    if (!(occupy_avg <= max_occ_ratio * gthr)) break;  // (WAITING only grows inside the run)
                    const double lq = (double)(sh_PS0 + spass[c]) / isec;
                    const int64_t head_pass = sh_headcur ? sh_cur0 + spass[c] : sh_head;
                    const int64_t qa = sacq[c];
                    // lq and occupied only grow inside the run and head_pass is fixed (unless the head window is the
                    // current one): once even an acquire of 1 cannot occupy, no later request can
                    if (!sh_headcur && lq + (double)(1 + M.f->occ_pass) - (double)head_pass > gthr) break;
                    if (lq + (double)(qa + M.f->occ_pass) - (double)head_pass <= gthr) {
                        M.f->occ_pass += qa;  // addOccupyPass
                        M.f->occ_req += 1;
                        M.f->has_occ = 1;
                        wadd += qa;
                        if (wait > 0) sst[c] = TS_WAIT;
                    }
                }
                sh_wadd = wadd;
            }
            __syncthreads();
            const uint8_t st = in ? sst[t] : (uint8_t)0xFF;
            if (in) {
                sg_token_result o;
                o.status = st == TS_PASS ? SG_TOKEN_OK : st == TS_WAIT ? SG_TOKEN_SHOULD_WAIT : SG_TOKEN_BLOCKED;
                o.remaining = st == TS_PASS ? j_d2i(gthr - (double)(S + myP) / isec - acq) : 0;
                o.wait_in_ms = st == TS_WAIT ? wait : 0;
                o.reserved = 0;
                res[i] = o;
            }
            // the window's counts of the run
            int64_t cs[6] = {st == TS_PASS ? acq : 0, st == TS_PASS ? 1 : 0, st == TS_PASS && prio ? acq : 0,
                             st == TS_BLOCK ? acq : 0, st == TS_BLOCK ? 1 : 0, st == TS_BLOCK && prio ? acq : 0};
            tf_sum6<TF_T>(cs, red6);
            if (t == 0) {
                CBkt* cur = cm_current(M, sba * M.wlen);
                cur->c[CF_PASS] += cs[0];
                cur->c[CF_PASS_REQ] += cs[1];
                cur->c[CF_OCC_PASS] += cs[2];
                cur->c[CF_WAITING] += sh_wadd;
                cur->c[CF_BLOCK] += cs[3];
                cur->c[CF_BLOCK_REQ] += cs[4];
                cur->c[CF_OCC_BLOCK] += cs[5];
            }
            a = b;
        }
    }
    __syncthreads();
    if (in_lds && t < (uint32_t)gf.n) bkts[gf.boff + t] = lbkt[t];
    if (t == 0) flows[f] = lflow;
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
// bounds: nflows + 1 device words.  The flows of more than `light` requests on hs (after `fork`, recording `join`),
// the rest on st, which then waits for `join`
hipError_t launch_tok_flow(const uint32_t* skeys, const uint32_t* svals, uint64_t n, const sg_token_req* req,
                           CFlow* flows, uint32_t nflows, CBkt* bkts, double exceed, double max_occ_ratio,
                           sg_token_result* res, uint32_t* bounds, uint32_t light, uint32_t wide, hipStream_t st,
                           hipStream_t hs, hipEvent_t fork, hipEvent_t join) {
    if (!n || !nflows) return hipSuccess;
    hipLaunchKernelGGL(k_tok_bounds, dim3((uint32_t)((n + 256) / 256)), dim3(256), 0, st, skeys, n, nflows, bounds);
    hipError_t e = hipEventRecord(fork, st);
    if (e == hipSuccess) e = hipStreamWaitEvent(hs, fork, 0);
    if (e != hipSuccess) return e;
    if (wide == 1024)
        hipLaunchKernelGGL(k_tok_flow_wg<1024>, dim3(nflows), dim3(1024), 0, hs, svals, bounds, light, 0xFFFFFFFFu, req,
                           flows, nflows, bkts, exceed, max_occ_ratio, res);
    else
        hipLaunchKernelGGL(k_tok_flow_wg<512>, dim3(nflows), dim3(512), 0, hs, svals, bounds, light, 0xFFFFFFFFu, req,
                           flows, nflows, bkts, exceed, max_occ_ratio, res);
    if ((e = hipEventRecord(join, hs)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_tok_flow_wg<64>, dim3(nflows), dim3(64), 0, st, svals, bounds, 0u, light, req, flows, nflows,
                       bkts, exceed, max_occ_ratio, res);
    if ((e = hipStreamWaitEvent(st, join, 0)) != hipSuccess) return e;
    return hipGetLastError();
}
// the limiter: bflag / cflag / bidx / cexcl / bstart / kpass are n-word scratch arrays, part the scan partials,
// small = 2 device words (bucket count, candidate count)
hipError_t launch_tok_limiter_par(const sg_token_req* req, uint64_t n, const uint32_t* fidx, uint32_t nflows,
                                  NsLimiter* lim, double allowed, uint32_t* keys, uint32_t* vals, sg_token_result* res,
                                  uint32_t* bflag, uint32_t* cflag, uint32_t* bidx, uint32_t* cexcl, uint32_t* bstart,
                                  uint32_t* kpass, uint32_t* part, uint32_t* small,
                                  hipError_t (*scan)(const uint32_t*, uint32_t*, uint64_t, uint32_t*, uint32_t*, hipStream_t),
                                  hipStream_t st) {
    if (!n) return hipSuccess;
    const uint32_t g = (uint32_t)((n + 255) / 256);
    hipLaunchKernelGGL(k_lim_flags, dim3(g), dim3(256), 0, st, req, n, fidx, bflag, cflag);
    hipError_t e = scan(bflag, bidx, n, part, small, st);
    if (e == hipSuccess) e = scan(cflag, cexcl, n, part, small + 1, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_lim_starts, dim3(g), dim3(256), 0, st, bidx, bflag, n, bstart);
    hipLaunchKernelGGL(k_lim_walk, dim3(1), dim3(64), 0, st, req, n, bstart, small, cexcl, small + 1, lim, allowed, kpass);
    hipLaunchKernelGGL(k_lim_apply, dim3(g), dim3(256), 0, st, n, fidx, bflag, bidx, bstart, cexcl, kpass, nflows, keys,
                       vals, res);
    return hipGetLastError();
}

// ---- ClusterParamFlowChecker.acquireClusterToken (csrv/flow/ClusterParamFlowChecker.java:42-88)
// One lane per param flow over its requests in time order (sorted positions).  The
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
