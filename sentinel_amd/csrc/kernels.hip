// kernels.hip -- gfx950 kernels of the batched Sentinel decision engine.
//
// Per sg_submit batch (n events already in HBM):
//   1. group   : stable LSD radix sort of (res_id, event index) -- keys read straight
//                out of the 24-byte event records on the first pass (k_radix_*)
//   2. segment : one segment per resource touched by the batch (k_seg_*)
//   3. decide  : one 64-lane wavefront per segment, longest segments dispatched first;
//                the wavefront stages 64 events in registers and runs the resource's
//                slot chain over them in event order (k_decide).  State lives in
//                registers / LDS for the whole segment and is written back once.
// The sequential per-resource semantics restated here follow the Java cited at each
// function; the oracle (oracle/sentinel_oracle.c) is the independent CPU restatement
// used to check it.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/sentinel_gpu.h"
#include "dev_types.h"

using namespace sg;

#define WAVE 64

// ---------------------------------------------------------------------------------
// Java arithmetic on the device (identical results to the JVM for these operations)
// ---------------------------------------------------------------------------------
__device__ __forceinline__ int64_t j_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}
__device__ __forceinline__ int32_t j_d2i(double d) {
    if (d != d) return 0;
    if (d >= 2147483647.0) return INT32_MAX;
    if (d <= -2147483648.0) return INT32_MIN;
    return (int32_t)d;
}
__device__ __forceinline__ int32_t j_iadd(int32_t a, int32_t b) { return (int32_t)((uint32_t)a + (uint32_t)b); }
// java.lang.Math.round(double)
__device__ __forceinline__ int64_t j_round(double a) {
    int64_t bits = __double_as_longlong(a);
    int64_t biased = (bits & 0x7ff0000000000000LL) >> 52;
    int64_t shift = (52 - 1 + 1023) - biased;
    if ((shift & -64) == 0) {
        int64_t r = (bits & 0x000fffffffffffffLL) | (0x000fffffffffffffLL + 1);
        if (bits < 0) r = -r;
        return ((r >> shift) + 1) >> 1;
    }
    return j_d2l(a);
}
// java.lang.Math.nextUp(double)
__device__ __forceinline__ double j_next_up(double d) {
    if (d != d || d == __longlong_as_double(0x7ff0000000000000LL)) return d;
    if (d == 0.0) return __longlong_as_double(1LL);
    int64_t b = __double_as_longlong(d);
    b += (d > 0.0) ? 1 : -1;
    return __longlong_as_double(b);
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27; x *= 0x94d049bb133111ebULL;
    x ^= x >> 31; return x;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t rl64(uint64_t v, int i) {
    uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, i);
    uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), i);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
    uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// =================================================================================
// 1. grouping: stable LSD radix sort on res_id
// =================================================================================
#define RS_THREADS 256
#define RS_ITEMS 16
#define RS_TILE (RS_THREADS * RS_ITEMS)
#define RS_BINS 256

// batch flags + key extraction happen on the first histogram pass
__global__ __launch_bounds__(RS_THREADS) void k_radix_hist(const sg_event* __restrict__ ev, const uint32_t* __restrict__ keys,
                                                        uint64_t n, int shift, uint32_t* __restrict__ ghist,
                                                        uint32_t nblocks, uint32_t* __restrict__ bflags, uint32_t max_res) {
    __shared__ uint32_t h[RS_BINS];
    for (int i = threadIdx.x; i < RS_BINS; i += RS_THREADS) h[i] = 0;
    __syncthreads();
    uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
    uint32_t fl = 0;
    for (int it = 0; it < RS_ITEMS; ++it) {
        uint64_t i = base + (uint64_t)it * RS_THREADS + threadIdx.x;
        if (i < n) {
            uint32_t k;
            if (ev) {
                const sg_event& e = ev[i];
                k = e.res_id;
                if (e.kind == SG_EV_ENTRY && (e.flags & SG_F_PRIORITIZED)) fl |= BF_PRIORITIZED;
                if (e.kind == SG_EV_EXIT && (e.flags & SG_F_EXIT_ARGS)) fl |= BF_EXIT_ARGS;
                if (k >= max_res) fl |= BF_BAD_RES;
            } else {
                k = keys[i];
            }
            atomicAdd(&h[(k >> shift) & (RS_BINS - 1)], 1u);
        }
    }
    if (ev && fl) atomicOr(bflags, fl);
    __syncthreads();
    for (int b = threadIdx.x; b < RS_BINS; b += RS_THREADS) ghist[(uint64_t)b * nblocks + blockIdx.x] = h[b];
}

// stable scatter: items of a tile are ranked in (round, wave, lane) order == input order
__global__ __launch_bounds__(RS_THREADS) void k_radix_scatter(const sg_event* __restrict__ ev, const uint32_t* __restrict__ keys_in,
                                                           const uint32_t* __restrict__ vals_in, uint64_t n, int shift,
                                                           const uint32_t* __restrict__ goff, uint32_t nblocks,
                                                           uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out) {
    __shared__ uint32_t wcnt[4][RS_BINS];
    __shared__ uint32_t woff[4][RS_BINS];
    __shared__ uint32_t run[RS_BINS];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    for (int i = threadIdx.x; i < RS_BINS; i += RS_THREADS) {
        run[i] = goff[(uint64_t)i * nblocks + blockIdx.x];
        wcnt[0][i] = wcnt[1][i] = wcnt[2][i] = wcnt[3][i] = 0;
    }
    __syncthreads();
    const uint64_t lt_mask = (l == 0) ? 0ull : (~0ull >> (64 - l));
    uint64_t base = (uint64_t)blockIdx.x * RS_TILE;
    for (int it = 0; it < RS_ITEMS; ++it) {
        uint64_t i = base + (uint64_t)it * RS_THREADS + threadIdx.x;
        bool valid = i < n;
        uint32_t k = 0, v = 0;
        if (valid) {
            if (ev) { k = ev[i].res_id; v = (uint32_t)i; }
            else { k = keys_in[i]; v = vals_in[i]; }
        }
        uint32_t d = (k >> shift) & (RS_BINS - 1);
        // peers: lanes with the same digit (8 ballots)
        uint64_t peers = __ballot(valid);
        #pragma unroll
        for (int b = 0; b < 8; ++b) {
            uint64_t bb = __ballot((d >> b) & 1);
            peers &= ((d >> b) & 1) ? bb : ~bb;
        }
        uint32_t rank = __popcll(peers & lt_mask);
        uint32_t cnt = __popcll(peers);
        bool leader = valid && rank == 0;
        if (leader) wcnt[w][d] = cnt;
        __syncthreads();
        for (int b = threadIdx.x; b < RS_BINS; b += RS_THREADS) {
            uint32_t acc = run[b];
            #pragma unroll
            for (int ww = 0; ww < 4; ++ww) { uint32_t c = wcnt[ww][b]; woff[ww][b] = acc; acc += c; wcnt[ww][b] = 0; }
            run[b] = acc;
        }
        __syncthreads();
        if (valid) {
            uint32_t dst = woff[w][d] + rank;
            keys_out[dst] = k;
            vals_out[dst] = v;
        }
        __syncthreads();
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
// 2. segments
// =================================================================================
__global__ void k_seg_flags(const uint32_t* __restrict__ keys, uint64_t n, uint32_t* __restrict__ flag) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) flag[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

__global__ void k_seg_emit(const uint32_t* __restrict__ keys, uint64_t n, const uint32_t* __restrict__ flag,
                           const uint32_t* __restrict__ pos, Seg* __restrict__ segs, uint32_t* __restrict__ lbucket,
                           const Prog* __restrict__ prog) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n || !flag[i]) return;
    // find the segment end
    uint32_t s = pos[i];
    uint64_t j = i + 1;
    Seg sg;
    sg.res = keys[i];
    sg.start = (uint32_t)i;
    // segment length: scan forward only for the start element (segments average n/m; use binary search on pos)
    uint64_t lo = i + 1, hi = n;
    while (lo < hi) {   // first index > i with flag set == first index whose pos > s
        uint64_t mid = (lo + hi) >> 1;
        uint32_t pm = pos[mid] + flag[mid];
        if (pm > s + 1) hi = mid; else lo = mid + 1;
    }
    (void)j;
    sg.len = (uint32_t)(lo - i);
    sg.pad = prog[sg.res].n_param > 0 ? 1u : 0u;  // class: 1 = serial path
    segs[s] = sg;
    int b = 31 - __clz(sg.len | 1);
    atomicAdd(&lbucket[sg.pad * 32 + b], 1u);
}

// order segments by descending length class so the longest start first
__global__ void k_seg_order(const Seg* __restrict__ segs, uint32_t m, uint32_t* __restrict__ lcursor, uint32_t* __restrict__ order) {
    uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    int b = 31 - __clz(segs[i].len | 1);
    uint32_t p = atomicAdd(&lcursor[segs[i].pad * 32 + b], 1u);
    order[p] = i;
}

// chain cap (CtSph.lookProcessChain, core/CtSph.java:206-227): resources touched by this
// batch with neither a chain nor a rejection, with the batch index of their first ENTRY
__global__ void k_chain_candidates(const sg_event* __restrict__ ev, const uint32_t* __restrict__ vals,
                                   const Seg* __restrict__ segs, uint32_t m, const NodeInfo* __restrict__ info,
                                   uint32_t* __restrict__ ncand, uint64_t* __restrict__ cand) {
    uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= m) return;
    Seg sg = segs[s];
    uint32_t f = info[sg.res].flags;
    if (f & (NI_CHAIN | NI_REJECTED)) return;
    for (uint32_t j = 0; j < sg.len; ++j) {
        uint32_t idx = vals[sg.start + j];
        if (ev[idx].kind == SG_EV_ENTRY) {
            uint32_t p = atomicAdd(ncand, 1u);
            cand[p] = ((uint64_t)idx << 32) | sg.res;
            return;
        }
    }
}

// =================================================================================
// 3. decide
// =================================================================================
#define MAX_RULES_PER_RES 16
#define DEC_WAVES 4

__device__ __forceinline__ uint32_t mk_dec(uint32_t status, uint32_t slot, int64_t wait) {
    if (wait < 0) wait = 0;
    if (wait > 0xFFFF) wait = 0xFFFF;
    return status | ((slot & 0xFFu) << 8) | ((uint32_t)wait << 16);
}

// ---- param table (ParameterMetric maps).  Every key is owned by exactly one
// resource, i.e. by one wavefront at a time; only probing crosses owners. ----
__device__ PSlot* ptab_lookup(PSlot* tab, uint64_t mask, uint64_t khi, uint64_t kval, bool insert, bool* is_new,
                              uint32_t* bflags) {
    uint64_t h = mix64(khi * 0x9e3779b97f4a7c15ULL ^ kval) & mask;
    *is_new = false;
    for (uint32_t probe = 0; probe <= 4096; ++probe) {
        PSlot* s = &tab[h];
        uint64_t k = __hip_atomic_load(&s->khi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == khi && s->kval == kval) return s;
        if (k == 0) {
            if (!insert) return nullptr;
            unsigned long long expect = 0;
            if (__hip_atomic_compare_exchange_strong((unsigned long long*)&s->khi, &expect, (unsigned long long)khi,
                                                     __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                s->kval = kval;
                s->v0 = 0;
                s->v1 = 0;
                *is_new = true;
                return s;
            }
            // lost the race to another owner: this slot now holds a different key, keep probing
        }
        h = (h + 1) & mask;
    }
    atomicOr(bflags, BF_PTAB_FULL);
    return nullptr;
}

struct Wave {
    // constants
    DevState S;
    DevCfg cfg;
    uint32_t res;
    Prog prog;
    uint32_t lane;
    uint32_t* bflags;
    // second window (2 x 500 ms buckets)
    Bkt sb[2];
    // minute window: cached current bucket
    int32_t mslot;
    bool mdirty, mdetached;
    Bkt mb;
    // node info
    int32_t thread;
    uint32_t flags;
    int64_t exc_sum_sec, exc_sum;
    // rule state in LDS
    RState* rs;
};

// ---- LeapArray.currentWindow for the 2-bucket second window (LeapArray.java:117-208);
// returns the slot, or -1 for a detached bucket (clock went back: updates are lost, Q3)
__device__ __forceinline__ void bkt_reset(Bkt& b, int64_t ws, int32_t max_rt) {
    b.ws = ws; b.pass = 0; b.block = 0; b.exc = 0; b.succ = 0; b.rt = 0; b.occ = 0; b.minrt = max_rt;
}
// (explicit branches: a runtime index into W.sb would force the wave state into scratch)
__device__ __forceinline__ int sec_current(Wave& W, int64_t t) {
    int slot = (int)((t / 500) & 1);
    int64_t ws = t - t % 500;
    if (slot == 0) {
        if (W.sb[0].ws == ws) return 0;
        if (W.sb[0].ws < ws) { bkt_reset(W.sb[0], ws, W.cfg.max_rt); return 0; }
        return -1;
    }
    if (W.sb[1].ws == ws) return 1;
    if (W.sb[1].ws < ws) { bkt_reset(W.sb[1], ws, W.cfg.max_rt); return 1; }
    return -1;
}
__device__ __forceinline__ void sec_add(Wave& W, int sl, int64_t dP, int64_t dB, int64_t dS, int64_t dRT, int64_t dE,
                                        int64_t mrt) {
    if (sl == 0) {
        W.sb[0].pass += dP; W.sb[0].block += dB; W.sb[0].succ += dS; W.sb[0].rt += dRT; W.sb[0].exc += dE;
        if (mrt < W.sb[0].minrt) W.sb[0].minrt = mrt;
    } else if (sl == 1) {
        W.sb[1].pass += dP; W.sb[1].block += dB; W.sb[1].succ += dS; W.sb[1].rt += dRT; W.sb[1].exc += dE;
        if (mrt < W.sb[1].minrt) W.sb[1].minrt = mrt;
    }
}
// sum of one counter over values(t) (valid iff t - ws <= 1000)
#define SEC_SUM(W, t, f) (((t) - (W).sb[0].ws <= 1000 && (W).sb[0].ws >= 0 ? (W).sb[0].f : 0) + \
                          ((t) - (W).sb[1].ws <= 1000 && (W).sb[1].ws >= 0 ? (W).sb[1].f : 0))

__device__ __forceinline__ void min_flush(Wave& W) {
    if (W.mslot >= 0 && W.mdirty && !W.mdetached) {
        if (W.lane == 0) W.S.minb[(uint64_t)W.res * 60 + W.mslot] = W.mb;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    W.mdirty = false;
}
// totalException running sum (StatisticNode.totalException = minute EXCEPTION sum over
// the buckets valid at t, i.e. window starts in [T-59000, T]).  Moves the sum to second T;
// the minute ring in HBM must hold every bucket (cache flushed) and slot(T) must not
// have been reset yet, so the seconds that fall out of the window are still readable.
__device__ __forceinline__ void exc_advance(Wave& W, int64_t T) {
    const Bkt* mb = W.S.minb + (uint64_t)W.res * 60;
    if (W.exc_sum_sec < 0 || T - W.exc_sum_sec >= 60000) {
        int64_t s = 0;
        for (int k = 0; k < 60; ++k) {
            Bkt b = mb[k];
            if (b.ws >= T - 59000 && b.ws <= T) s += b.exc;
        }
        W.exc_sum = s;
    } else {
        for (int64_t x = W.exc_sum_sec - 59000; x <= T - 60000; x += 1000) {
            Bkt b = mb[(x / 1000) % 60];
            if (b.ws == x) W.exc_sum -= b.exc;
        }
    }
    W.exc_sum_sec = T;
}
// minute currentWindow(t) (LeapArray.java:117-208): caches the bucket of second T
__device__ __forceinline__ void min_current(Wave& W, int64_t t) {
    int slot = (int)((t / 1000) % 60);
    int64_t ws = t - t % 1000;
    if (W.mslot == slot && W.mb.ws == ws) return;
    min_flush(W);
    if ((W.prog.pflags & PF_EXC_COUNT) && W.exc_sum_sec != ws && W.exc_sum_sec < ws) exc_advance(W, ws);
    Bkt b = W.S.minb[(uint64_t)W.res * 60 + slot];
    W.mslot = slot;
    W.mdetached = false;
    if (b.ws == ws) { W.mb = b; return; }
    bool back = b.ws > ws;
    b.ws = ws; b.pass = 0; b.block = 0; b.exc = 0; b.succ = 0; b.rt = 0; b.occ = 0; b.minrt = W.cfg.max_rt;
    W.mb = b;
    if (back) W.mdetached = true;  // clock went back: a detached bucket, updates are lost (Q3)
    else W.mdirty = true;
}
// ArrayMetric.previousWindowPass on the minute window (LeapArray.getPreviousWindow, LeapArray.java:216-234)
__device__ __forceinline__ int64_t min_prev_pass(Wave& W, int64_t t) {
    min_current(W, t);
    int slot = (int)(((t - 1000) / 1000) % 60);
    Bkt b = W.S.minb[(uint64_t)W.res * 60 + slot];
    if (b.ws < 0) return 0;
    if (t - b.ws > 60000) return 0;
    if (b.ws + 1000 < t - 1000) return 0;
    return b.pass;
}
__device__ __forceinline__ int64_t min_total_exc(Wave& W, int64_t t) {
    min_current(W, t);
    int64_t T = t - t % 1000;
    if (W.exc_sum_sec != T) { // rule added since the last advance: recompute (cached slot from registers)
        int64_t s = 0;
        for (int k = 0; k < 60; ++k) {
            Bkt b = (k == W.mslot) ? W.mb : W.S.minb[(uint64_t)W.res * 60 + k];
            if (b.ws >= T - 59000 && b.ws <= T) s += b.exc;
        }
        W.exc_sum = s;
        W.exc_sum_sec = T;
    }
    return W.exc_sum;
}

// ---- WarmUpController (core/slots/block/flow/controller/WarmUpController.java:119-174)
__device__ __forceinline__ void warm_sync(const DRule& r, RState& s, int64_t now, int64_t pass_qps) {
    int64_t cur = now - now % 1000;
    if (cur <= s.b) return;
    int64_t old = s.a, nv = old;
    if (old < r.warning_token) {
        nv = j_d2l((double)old + (double)(cur - s.b) * r.count / 1000);
    } else if (old > r.warning_token) {
        if (pass_qps < r.count_div_cold) nv = j_d2l((double)old + (double)(cur - s.b) * r.count / 1000);
    }
    if (nv > r.max_token) nv = r.max_token;
    int64_t v = nv - pass_qps;
    s.a = v < 0 ? 0 : v;
    s.b = cur;
}
__device__ __forceinline__ double warm_qps(const DRule& r, int64_t rest) {
    int64_t above = rest - r.warning_token;
    return j_next_up(1.0 / ((double)above * r.slope + 1.0 / r.count));
}
// RateLimiterController / WarmUpRateLimiterController queueing (sleep -> wait_ms, Q10)
__device__ __forceinline__ bool rl_admit(int64_t& latest, int64_t cost, int64_t now, int32_t maxq, int64_t& wait) {
    int64_t expected = cost + latest;
    if (expected <= now) { latest = now; return true; }
    int64_t w = cost + latest - now;
    if (w > maxq) return false;
    latest += cost;
    w = latest - now;
    if (w > maxq) { latest -= cost; return false; }
    if (w > 0) wait += w;
    return true;
}

// TrafficShapingController.canPass on the resource's ClusterNode (FlowRuleChecker.passLocalCheck)
__device__ bool flow_can_pass(Wave& W, const DRule& r, RState& s, int64_t t, int acquire, int64_t& wait) {
    switch (r.behavior) {
    case SG_CONTROL_BEHAVIOR_WARM_UP: {
        sec_current(W, t);
        int64_t pass_qps = SEC_SUM(W, t, pass);          // (long) node.passQps()
        int64_t prev = min_prev_pass(W, t);             // (long) node.previousPassQps()
        warm_sync(r, s, t, prev);
        int64_t rest = s.a;
        if (rest >= r.warning_token) return (double)(pass_qps + acquire) <= warm_qps(r, rest);
        return (double)(pass_qps + acquire) <= r.count;
    }
    case SG_CONTROL_BEHAVIOR_RATE_LIMITER: {
        if (acquire <= 0) return true;
        if (r.count <= 0) return false;
        int64_t cost = j_round(1.0 * acquire / r.count * 1000);
        return rl_admit(s.c, cost, t, r.max_queue, wait);
    }
    case SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER: {
        int64_t prev = min_prev_pass(W, t);
        warm_sync(r, s, t, prev);
        int64_t rest = s.a, cost;
        if (rest >= r.warning_token) cost = j_round(1.0 * acquire / warm_qps(r, rest) * 1000);
        else cost = j_round(1.0 * acquire / r.count * 1000);
        return rl_admit(s.c, cost, t, r.max_queue, wait);
    }
    default: { // DefaultController (DefaultController.java:49-81); prioritized entries are rejected on the host
        int32_t cur;
        if (r.grade == SG_FLOW_GRADE_THREAD) cur = W.thread;
        else { sec_current(W, t); cur = j_d2i((double)SEC_SUM(W, t, pass)); }
        return !((double)j_iadd(cur, acquire) > r.count);
    }
    }
}

// DegradeRule.passCheck (core/slots/block/degrade/DegradeRule.java:172-223); the ResetTask
// fires at cut_until = t_cut + timeWindow*1000 (Q12)
__device__ bool degrade_pass(Wave& W, const DRule& r, RState& s, int64_t t) {
    if (s.a && t >= s.c) { s.a = 0; s.b = 0; }
    if (s.a) return false;
    if (r.grade == SG_DEGRADE_GRADE_RT) {
        sec_current(W, t);
        int64_t succ = SEC_SUM(W, t, succ);
        double avg = succ == 0 ? 0.0 : (double)SEC_SUM(W, t, rt) * 1.0 / (double)succ;
        if (avg < r.count) { s.b = 0; return true; }
        if (++s.b < 5) return true;
    } else if (r.grade == SG_DEGRADE_GRADE_EXCEPTION_RATIO) {
        sec_current(W, t);
        double exc = (double)SEC_SUM(W, t, exc) / 1.0;
        double succ = (double)SEC_SUM(W, t, succ) / 1.0;
        double total = (double)SEC_SUM(W, t, pass) / 1.0 + (double)SEC_SUM(W, t, block) / 1.0;
        if (total < 5) return true;
        double real = succ - exc;
        if (real <= 0 && exc < 5) return true;
        if (exc / succ < r.count) return true;
    } else if (r.grade == SG_DEGRADE_GRADE_EXCEPTION_COUNT) {
        double e = (double)min_total_exc(W, t);
        if (e < r.count) return true;
    }
    s.a = 1;
    s.c = t + (int64_t)r.time_window * 1000;
    return false;
}

// ---- ParamFlowChecker (param/slots/block/flow/param/ParamFlowChecker.java:101-248), lane 0 executes
__device__ int32_t hot_count(const DevState& S, const DRule& r, uint64_t v, bool* found) {
    for (uint32_t i = 0; i < r.hot_n; ++i) {
        DHot h = S.hot[r.hot_off + i];
        if (h.key == v) { *found = true; return h.count; }
    }
    *found = false;
    return 0;
}
__device__ int64_t thread_count_get(Wave& W, uint64_t v) {
    uint64_t khi = (2ULL << 62) | ((uint64_t)(W.prog.tc_epoch & 0x3FFFFFFF) << 32) | W.res;
    bool nw;
    PSlot* s = ptab_lookup(W.S.ptab, W.cfg.ptab_mask, khi, v, false, &nw, W.bflags);
    return s ? s->v0 : 0;
}
__device__ void thread_count_add(Wave& W, uint64_t v, int64_t d) {
    uint64_t khi = (2ULL << 62) | ((uint64_t)(W.prog.tc_epoch & 0x3FFFFFFF) << 32) | W.res;
    bool nw;
    PSlot* s = ptab_lookup(W.S.ptab, W.cfg.ptab_mask, khi, v, true, &nw, W.bflags);
    if (!s) return;
    int64_t c = s->v0 + d;
    if (d < 0 && nw) c = 0; // putIfAbsent(value, new AtomicInteger()) without a decrement
    s->v0 = c < 0 ? 0 : c;
}

__device__ bool param_check_lane0(Wave& W, const DRule& r, int acquire, uint64_t v, int64_t t, int64_t& wait) {
    if (r.grade == SG_FLOW_GRADE_QPS) {
        bool hf;
        int32_t hc = hot_count(W.S, r, v, &hf);
        uint64_t khi = (1ULL << 62) | r.psid;
        if (r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER) {
            int64_t token_count = hf ? (int64_t)hc : r.token_count_l;
            if (token_count == 0) return false;
            int64_t cost = j_round(1.0 * 1000 * acquire * (double)r.duration_sec / (double)token_count);
            bool nw;
            PSlot* s = ptab_lookup(W.S.ptab, W.cfg.ptab_mask, khi, v, true, &nw, W.bflags);
            if (!s) return true;
            if (nw) { s->v0 = t; return true; }
            int64_t expected = s->v0 + cost;
            if (expected <= t || expected - t < r.max_queue) {
                s->v0 = t;
                int64_t w = expected - t;
                if (w > 0) { s->v0 = expected; wait += w; }
                return true;
            }
            return false;
        }
        int32_t token_count = hf ? hc : r.token_count;
        if (token_count == 0) return false;
        int32_t max_count = j_iadd(token_count, r.burst);
        if (acquire > max_count) return false;
        bool nw;
        PSlot* s = ptab_lookup(W.S.ptab, W.cfg.ptab_mask, khi, v, true, &nw, W.bflags);
        if (!s) return true;
        if (nw) { s->v0 = t; s->v1 = j_iadd(max_count, -acquire); return true; }
        int64_t pass_time = t - s->v0;
        if (pass_time > r.duration_sec * 1000) {
            int32_t rest = (int32_t)s->v1;
            int32_t to_add = (int32_t)((pass_time * token_count) / (r.duration_sec * 1000));
            int32_t sum = j_iadd(rest, to_add);
            int32_t nq = sum > max_count ? j_iadd(max_count, -acquire) : j_iadd(sum, -acquire);
            if (nq < 0) return false;
            s->v1 = nq;
            s->v0 = t;
            return true;
        }
        int32_t ov = (int32_t)s->v1;
        if (j_iadd(ov, -acquire) >= 0) { s->v1 = j_iadd(ov, -acquire); return true; }
        return false;
    } else if (r.grade == SG_FLOW_GRADE_THREAD) {
        int64_t tc = thread_count_get(W, v);
        bool hf;
        int32_t hc = hot_count(W.S, r, v, &hf);
        if (hf) return ++tc <= hc;
        int64_t threshold = j_d2l(r.count);
        return ++tc <= threshold;
    }
    return true;
}

// One ENTRY through Statistic -> ParamFlow -> Flow -> Degrade (HotParamSlotChainBuilder.java:38-51,
// StatisticSlot.entry StatisticSlot.java:54-133).  Uniform across the wavefront.
__device__ uint32_t do_entry(Wave& W, int64_t t, int count, uint8_t eflags, uint64_t arg) {
    if (!(W.flags & NI_CHAIN)) return mk_dec(ST_NO_CHECK, 0, 0);
    uint32_t status = ST_PASS, slot = 0;
    int64_t wait = 0;
    const DRule* rules = W.S.rules + W.prog.rule_off;
    int nr = W.prog.n_param + W.prog.n_flow + W.prog.n_degrade;
    // ParamFlowSlot.checkFlow (ParamFlowSlot.java:77-101)
    if (W.prog.n_param) {
        W.flags |= NI_PM;
        if (W.prog.pflags & PF_PARAM_IDX0) W.flags |= NI_TM0;
        if (eflags & SG_F_HAS_ARG) {
            for (int i = 0; i < W.prog.n_param; ++i) {
                DRule r = rules[i];
                int ok = 1;
                int64_t w = 0;
                if (W.lane == 0) ok = param_check_lane0(W, r, count, arg, t, w) ? 1 : 0;
                ok = __builtin_amdgcn_readfirstlane(ok);
                w = (int64_t)rfl64((uint64_t)w);
                if (!ok) { status = ST_BLOCK_PARAM; slot = r.slot; break; }
                wait += w;
            }
        }
    }
    // FlowSlot.checkFlow (FlowSlot.java:146-158)
    if (status == ST_PASS) {
        for (int i = W.prog.n_param; i < W.prog.n_param + W.prog.n_flow; ++i) {
            DRule r = rules[i];
            if (!flow_can_pass(W, r, W.rs[i], t, count, wait)) { status = ST_BLOCK_FLOW; slot = r.slot; break; }
        }
    }
    // DegradeSlot -> DegradeRuleManager.checkDegrade (DegradeRuleManager.java:72-85)
    if (status == ST_PASS) {
        for (int i = W.prog.n_param + W.prog.n_flow; i < nr; ++i) {
            DRule r = rules[i];
            if (!degrade_pass(W, r, W.rs[i], t)) { status = ST_BLOCK_DEGRADE; slot = r.slot; break; }
        }
    }
    int sl = sec_current(W, t);
    min_current(W, t);
    if (status == ST_PASS) {
        W.thread++;
        sec_add(W, sl, count, 0, 0, 0, 0, INT64_MAX);
        if (!W.mdetached) { W.mb.pass += count; W.mdirty = true; }
        // ParamFlowStatisticEntryCallback.onPass -> ParameterMetric.addThreadCount
        if ((W.flags & NI_PM) && (W.flags & NI_TM0) && (eflags & SG_F_HAS_ARG) && W.lane == 0) thread_count_add(W, arg, 1);
        return mk_dec(ST_PASS, 0, wait);
    }
    sec_add(W, sl, 0, count, 0, 0, 0, INT64_MAX);
    if (!W.mdetached) { W.mb.block += count; W.mdirty = true; }
    return mk_dec(status, slot, 0);
}

// StatisticSlot.exit (StatisticSlot.java:136-173) for an entry that passed
__device__ void do_exit(Wave& W, int64_t t, int count, int64_t rt_raw) {
    int64_t rt = rt_raw > W.cfg.max_rt ? W.cfg.max_rt : rt_raw;
    int sl = sec_current(W, t);
    sec_add(W, sl, 0, 0, count, rt, 0, rt);
    min_current(W, t);
    if (!W.mdetached) {
        W.mb.succ += count;
        W.mb.rt += rt;
        if (rt < W.mb.minrt) W.mb.minrt = rt;
        W.mdirty = true;
    }
    W.thread--;
}

// ClusterNode.trace (core/node/ClusterNode.java:99-106)
__device__ void do_trace(Wave& W, int64_t t, int count) {
    if (count <= 0) return;
    int sl = sec_current(W, t);
    sec_add(W, sl, 0, 0, 0, 0, count, INT64_MAX);
    min_current(W, t);
    if (!W.mdetached) {
        W.mb.exc += count;
        W.mdirty = true;
        if (W.exc_sum_sec == t - t % 1000) W.exc_sum += count;
    }
}

__global__ __launch_bounds__(DEC_WAVES * WAVE) void k_decide(const sg_event* __restrict__ ev, const uint32_t* __restrict__ vals,
                                                           const Seg* __restrict__ segs, const uint32_t* __restrict__ order,
                                                           uint32_t m, uint64_t gbase, uint64_t n, DevState S, DevCfg cfg,
                                                           uint32_t* __restrict__ out, uint32_t* __restrict__ bflags) {
    __shared__ RState lds_rs[DEC_WAVES][MAX_RULES_PER_RES];
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t sidx = blockIdx.x * DEC_WAVES + wv;
    if (sidx >= m) return;
    Wave W;
    W.S = S;
    W.cfg = cfg;
    W.lane = lane_id();
    W.bflags = bflags;
    Seg sg = segs[order[sidx]];
    W.res = sg.res;
    W.prog = S.prog[W.res];
    W.rs = lds_rs[wv];
    int nr = W.prog.n_param + W.prog.n_flow + W.prog.n_degrade;
    for (int i = W.lane; i < nr; i += WAVE) W.rs[i] = S.rstate[W.prog.rule_off + i];
    W.sb[0] = S.sec[(uint64_t)W.res * 2 + 0];
    W.sb[1] = S.sec[(uint64_t)W.res * 2 + 1];
    NodeInfo ni = S.info[W.res];
    W.thread = ni.thread;
    W.flags = ni.flags;
    W.exc_sum_sec = ni.exc_sum_sec;
    W.exc_sum = ni.exc_sum;
    W.mslot = -1;
    W.mdirty = false;
    W.mdetached = false;
    __builtin_amdgcn_wave_barrier();

    for (uint32_t base = 0; base < sg.len; base += WAVE) {
        uint32_t cnt = sg.len - base < WAVE ? sg.len - base : WAVE;
        // stage up to 64 events of this resource in registers (one per lane)
        uint32_t idx = 0;
        uint64_t e_ts = 0, e_w1 = 0, e_aux = 0;
        if (W.lane < cnt) {
            idx = vals[sg.start + base + W.lane];
            const uint64_t* p = reinterpret_cast<const uint64_t*>(ev + idx);
            e_ts = p[0];
            e_w1 = p[1];
            e_aux = p[2];
        }
        uint64_t gidx = gbase + idx;
        uint32_t dec_v = mk_dec(ST_NOT_ENTRY, 0, 0);
        uint32_t st_v = ST_NOT_ENTRY;
        for (uint32_t i = 0; i < cnt; ++i) {
            int64_t t = (int64_t)rl64(e_ts, (int)i);
            uint64_t w1 = rl64(e_w1, (int)i);
            uint64_t aux = rl64(e_aux, (int)i);
            uint32_t count = (uint32_t)(w1 >> 32) & 0xFFFFu;
            uint8_t kind = (uint8_t)(w1 >> 48);
            uint8_t fl = (uint8_t)(w1 >> 56);
            if (kind == SG_EV_ENTRY) {
                uint32_t d = cfg.switch_on ? do_entry(W, t, (int)count, fl, aux) : mk_dec(ST_NO_CHECK, 0, 0);
                if (W.lane == i) { dec_v = d; st_v = d & 0xFF; }
            } else {
                // the referenced ENTRY must have passed (EXIT/TRACE of a blocked entry are no-ops)
                uint64_t ref = aux & SG_REF_NONE;
                bool ok;
                if (ref == SG_REF_NONE) {
                    ok = (W.flags & NI_CHAIN) != 0;
                } else {
                    uint64_t hit = __ballot(W.lane < cnt && gidx == ref);
                    uint32_t s;
                    if (hit) s = (uint32_t)__builtin_amdgcn_readlane((int)st_v, (int)(__ffsll((long long)hit) - 1));
                    else s = S.ring[ref & cfg.ring_mask];
                    ok = (s == ST_PASS || s == ST_PASS_WAIT) && (W.flags & NI_CHAIN);
                }
                if (ok) {
                    if (kind == SG_EV_EXIT) do_exit(W, t, (int)count, (int64_t)(aux >> 48));
                    else do_trace(W, t, (int)count);
                }
            }
        }
        if (W.lane < cnt) {
            out[idx] = dec_v;
            if (st_v != ST_NOT_ENTRY) S.ring[gidx & cfg.ring_mask] = (uint8_t)st_v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    // write back
    min_flush(W);
    if (W.lane == 0) {
        S.sec[(uint64_t)W.res * 2 + 0] = W.sb[0];
        S.sec[(uint64_t)W.res * 2 + 1] = W.sb[1];
        NodeInfo o = ni;
        o.thread = W.thread;
        o.flags = W.flags;
        o.exc_sum_sec = (W.prog.pflags & PF_EXC_COUNT) ? W.exc_sum_sec : -1;
        o.exc_sum = W.exc_sum;
        S.info[W.res] = o;
    }
    __builtin_amdgcn_wave_barrier();
    for (int i = W.lane; i < nr; i += WAVE) S.rstate[W.prog.rule_off + i] = W.rs[i];
}


// =================================================================================
// 3b. decide, speculative: Jacobi rounds over the 64 staged events
// ---------------------------------------------------------------------------------
// Every lane evaluates the slot chain for its own event against the state it would
// see if every earlier lane of the round had the outcome currently *guessed* for it
// (prefix scans of the counter deltas, max-plus scans for the rate limiters,
// run-length scans for the RT breaker).  The first lane whose evaluated outcome
// differs from its guess is exact (all earlier guesses were right), so lanes up to
// and including it are committed; the rest are re-guessed with their evaluated
// outcomes and the round repeats.  A round never crosses a 500 ms bucket or a
// breaker reset time, so bucket rotation and ResetTask stay serial points.
// Resources with param rules take the serial path (per-value hash-table state).
// =================================================================================
// inclusive 64-lane prefix sum with DPP row shifts + row broadcasts (GFX9 family)
__device__ __forceinline__ uint32_t wincl_u32(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false); // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false); // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false); // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false); // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false); // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false); // row_bcast:31
    return v;
}
__device__ __forceinline__ uint32_t wex_u32(uint32_t v, uint32_t lane) {
    (void)lane;
    return wincl_u32(v) - v;
}
__device__ __forceinline__ uint32_t wsum_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wincl_u32(v), 63);
}
__device__ __forceinline__ int64_t wex_i64(int64_t v, uint32_t lane) {
    int64_t x = v;
    #pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int64_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x += y;
    }
    return x - v;
}
// exclusive prefix max (identity lo)
__device__ __forceinline__ int64_t wexmax_i64(int64_t v, int64_t lo, uint32_t lane) {
    int64_t x = v;
    #pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int64_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x = x > y ? x : y;
    }
    int64_t e = __shfl_up(x, 1, 64);
    return lane == 0 ? lo : e;
}
__device__ __forceinline__ int32_t wexmax_i32(int32_t v, int32_t lo, uint32_t lane) {
    int32_t x = v;
    #pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int32_t y = __shfl_up(x, o, 64);
        if (lane >= (uint32_t)o) x = x > y ? x : y;
    }
    int32_t e = __shfl_up(x, 1, 64);
    return lane == 0 ? lo : e;
}
__device__ __forceinline__ int64_t wsum_i64(int64_t v) {
    #pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ int64_t wmin_i64(int64_t v) {
    #pragma unroll
    for (int o = 32; o >= 1; o >>= 1) { int64_t y = __shfl_xor(v, o, 64); v = v < y ? v : y; }
    return v;
}
__device__ __forceinline__ int64_t wmax_i64(int64_t v) {
    #pragma unroll
    for (int o = 32; o >= 1; o >>= 1) { int64_t y = __shfl_xor(v, o, 64); v = v > y ? v : y; }
    return v;
}

#define NEG_INF64 ((int64_t)0x8000000000000000LL)

// per-stage uniform info kept in registers for the round (up to MAX_RULES_PER_RES)
struct SpecRound {
    // base counters of the second window visible at the round's times (prev bucket + current bucket)
    int64_t P, B, S, RT, E;
    int64_t TH;       // thread count
    int64_t EM;       // minute exception total (EXC_COUNT)
    int64_t prev_pass_sec; // previous-second pass (WarmUp)
};

// evaluates every lane of the round under the guesses g; returns the lane outcome
// (stage index that blocked, or nr for pass) and the queueing wait for entries.
__device__ __forceinline__ uint32_t spec_eval(Wave& W, const SpecRound& R, const DRule* rules, int nr, uint32_t lane,
                                              bool inr, bool is_entry, bool eff, uint32_t kind, int64_t t, int cnt,
                                              int64_t rtv, uint32_t g, int64_t& wait_out, const RState* synced,
                                              uint32_t has_sync) {
    // ---- counter prefixes under the guesses
    bool gpass = inr && is_entry && g == (uint32_t)nr;
    bool gblock = inr && is_entry && g != (uint32_t)nr;
    bool eexit = inr && kind == SG_EV_EXIT && eff;
    bool etrace = inr && kind == SG_EV_TRACE && eff && cnt > 0;
    int64_t P = R.P + (int64_t)wex_u32(gpass ? (uint32_t)cnt : 0u, lane);
    int64_t B = R.B + (int64_t)wex_u32(gblock ? (uint32_t)cnt : 0u, lane);
    int64_t S = R.S + (int64_t)wex_u32(eexit ? (uint32_t)cnt : 0u, lane);
    int64_t RT = R.RT + (int64_t)wex_u32(eexit ? (uint32_t)rtv : 0u, lane);
    int64_t E = R.E + (int64_t)wex_u32(etrace ? (uint32_t)cnt : 0u, lane);
    int64_t EM = R.EM + (int64_t)wex_u32(etrace ? (uint32_t)cnt : 0u, lane);
    int32_t dth = gpass ? 1 : (eexit ? -1 : 0);
    int64_t TH = R.TH + (int64_t)(int32_t)wex_u32((uint32_t)dth, lane);

    uint32_t out = (uint32_t)nr;
    bool alive = inr && is_entry;
    int64_t wait = 0;
    for (int s = 0; s < nr; ++s) {
        const DRule r = rules[s];
        bool reach_g = inr && is_entry && g >= (uint32_t)s;  // other lanes, by guess
        bool pass_g = inr && is_entry && g > (uint32_t)s;
        bool ok = true;
        if (r.kind == RK_FLOW) {
            switch (r.behavior) {
            case SG_CONTROL_BEHAVIOR_WARM_UP: {
                const RState& st = ((has_sync >> s) & 1) ? synced[s] : W.rs[s];
                int64_t pq = P;
                if (st.a >= r.warning_token) ok = (double)(pq + cnt) <= warm_qps(r, st.a);
                else ok = (double)(pq + cnt) <= r.count;
                break;
            }
            case SG_CONTROL_BEHAVIOR_RATE_LIMITER:
            case SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER: {
                const RState& st = ((has_sync >> s) & 1) ? synced[s] : W.rs[s];
                int64_t cost;
                if (r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER) {
                    cost = (cnt <= 0 || r.count <= 0) ? 0 : j_round(1.0 * cnt / r.count * 1000);
                } else {
                    if (st.a >= r.warning_token) cost = j_round(1.0 * cnt / warm_qps(r, st.a) * 1000);
                    else cost = j_round(1.0 * cnt / r.count * 1000);
                }
                bool upd = pass_g && (r.behavior != SG_CONTROL_BEHAVIOR_RATE_LIMITER || (cnt > 0 && r.count > 0));
                int64_t C = wex_i64(upd ? cost : 0, lane);
                int64_t M = wexmax_i64(upd ? t - (C + cost) : NEG_INF64, NEG_INF64, lane);
                int64_t L0 = W.rs[s].c;
                int64_t L = C + (M > L0 ? M : L0);
                if (r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER && cnt <= 0) { ok = true; break; }
                if (r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER && r.count <= 0) { ok = false; break; }
                int64_t expected = L + cost;
                if (expected <= t) ok = true;
                else {
                    int64_t w = expected - t;
                    ok = w <= r.max_queue;
                    if (ok && alive) wait += w;
                }
                break;
            }
            default: {
                int32_t cur = r.grade == SG_FLOW_GRADE_THREAD ? (int32_t)TH : j_d2i((double)P);
                ok = !((double)j_iadd(cur, cnt) > r.count);
            }
            }
        } else if (r.kind == RK_DEGRADE) {
            // lane-local check value (only meaningful where the lane checks)
            bool bad;
            if (r.grade == SG_DEGRADE_GRADE_RT) {
                double avg = S == 0 ? 0.0 : (double)RT * 1.0 / (double)S;
                bad = !(avg < r.count);
            } else if (r.grade == SG_DEGRADE_GRADE_EXCEPTION_RATIO) {
                double exc = (double)E / 1.0, succ = (double)S / 1.0;
                double total = (double)P / 1.0 + (double)B / 1.0;
                if (total < 5) bad = false;
                else if (succ - exc <= 0 && exc < 5) bad = false;
                else bad = !(exc / succ < r.count);
            } else {
                bad = !((double)EM < r.count);
            }
            // cut before this lane: at round start, or a guessed trip of an earlier lane
            bool trip_g = inr && is_entry && g == (uint32_t)s;
            uint64_t trips = __ballot(trip_g);
            uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
            bool cut = W.rs[s].a != 0 || (trips & lt) != 0;
            if (cut) { ok = false; }
            else if (r.grade == SG_DEGRADE_GRADE_RT) {
                // passCount before this lane: highs since the last low among checking lanes
                bool chk = reach_g;  // lanes before the first guessed trip (later ones are cut)
                bool low_g = chk && !bad;
                bool high_g = chk && bad;
                int32_t last_low = wexmax_i32(low_g ? (int32_t)lane : -1, -1, lane);
                uint32_t highs = wex_u32(high_g ? 1u : 0u, lane);
                int64_t pc;
                if (last_low < 0) pc = W.rs[s].b + highs;
                else {
                    uint32_t h_at = __shfl(highs, last_low, 64);
                    pc = (int64_t)(highs - h_at); // highs strictly after last_low (last_low itself is low)
                }
                ok = !bad || (pc + 1 < 5);
            } else {
                ok = !bad;
            }
        } else {
            ok = true; // param rules never reach this path
        }
        if (alive && !ok) { out = (uint32_t)s; alive = false; }
    }
    wait_out = wait;
    return out;
}

// reductions of the committed lanes into the wavefront state
__device__ __forceinline__ void spec_commit(Wave& W, const SpecRound& R, const DRule* rules, int nr, uint32_t lane,
                                            bool com, bool is_entry, bool eff, uint32_t kind, int64_t t, int cnt,
                                            int64_t rtv, uint32_t g, int64_t tc0, const RState* synced,
                                            uint32_t has_sync, int64_t T) {
    bool cpass = com && is_entry && g == (uint32_t)nr;
    bool cblock = com && is_entry && g != (uint32_t)nr;
    bool cexit = com && kind == SG_EV_EXIT && eff;
    bool ctrace = com && kind == SG_EV_TRACE && eff && cnt > 0;
    int64_t dP = wsum_u32(cpass ? (uint32_t)cnt : 0u);
    int64_t dB = wsum_u32(cblock ? (uint32_t)cnt : 0u);
    int64_t dS = wsum_u32(cexit ? (uint32_t)cnt : 0u);
    int64_t dRT = wsum_u32(cexit ? (uint32_t)rtv : 0u);
    int64_t dE = wsum_u32(ctrace ? (uint32_t)cnt : 0u);
    int64_t dTH = (int64_t)(int32_t)wsum_u32((uint32_t)(cpass ? 1 : (cexit ? -1 : 0)));
    int64_t mrt = wmin_i64(cexit ? rtv : INT64_MAX);
    const bool touch = __ballot(cpass || cblock || cexit || ctrace) != 0;
    int sl = -1;
    if (touch) {
        sl = sec_current(W, tc0);
        min_current(W, tc0);
    }
    sec_add(W, sl, dP, dB, dS, dRT, dE, mrt);
    if (touch && !W.mdetached) {
        W.mb.pass += dP; W.mb.block += dB; W.mb.succ += dS; W.mb.rt += dRT; W.mb.exc += dE;
        if (mrt < W.mb.minrt) W.mb.minrt = mrt;
        if (dP | dB | dS | dRT | dE | (mrt != INT64_MAX)) W.mdirty = true;
        if (W.exc_sum_sec == T) W.exc_sum += dE;
    }
    W.thread += (int32_t)dTH;
    // rule state
    for (int s = 0; s < nr; ++s) {
        const DRule r = rules[s];
        bool reach = com && is_entry && g >= (uint32_t)s;
        bool pass = com && is_entry && g > (uint32_t)s;
        bool any_reach = __ballot(reach) != 0;
        if (r.kind == RK_FLOW) {
            if (r.behavior == SG_CONTROL_BEHAVIOR_WARM_UP || r.behavior == SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER) {
                if (any_reach && ((has_sync >> s) & 1)) { W.rs[s].a = synced[s].a; W.rs[s].b = synced[s].b; }
            }
            if (r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER || r.behavior == SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER) {
                const RState& st = ((has_sync >> s) & 1) ? synced[s] : W.rs[s];
                int64_t cost;
                if (r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER) {
                    cost = (cnt <= 0 || r.count <= 0) ? 0 : j_round(1.0 * cnt / r.count * 1000);
                } else {
                    if (st.a >= r.warning_token) cost = j_round(1.0 * cnt / warm_qps(r, st.a) * 1000);
                    else cost = j_round(1.0 * cnt / r.count * 1000);
                }
                bool upd = pass && (r.behavior != SG_CONTROL_BEHAVIOR_RATE_LIMITER || (cnt > 0 && r.count > 0));
                int64_t C = wex_i64(upd ? cost : 0, lane);
                int64_t v = upd ? t - (C + cost) : NEG_INF64;
                int64_t Ctot = wsum_i64(upd ? cost : 0);
                int64_t Mall = wmax_i64(v);
                int64_t L0 = W.rs[s].c;
                W.rs[s].c = Ctot + (Mall > L0 ? Mall : L0);
            }
        } else if (r.kind == RK_DEGRADE) {
            if (W.rs[s].a) continue; // cut for the whole round: no state change
            bool trip = com && is_entry && g == (uint32_t)s;
            uint64_t trips = __ballot(trip);
            if (r.grade == SG_DEGRADE_GRADE_RT) {
                // recompute the lanes' high/low against committed prefixes
                int64_t S2 = R.S + (int64_t)wex_u32(cexit ? (uint32_t)cnt : 0u, lane);
                int64_t RT2 = R.RT + (int64_t)wex_u32(cexit ? (uint32_t)rtv : 0u, lane);
                double avg = S2 == 0 ? 0.0 : (double)RT2 * 1.0 / (double)S2;
                bool bad = !(avg < r.count);
                int ft = trips ? __ffsll((long long)trips) - 1 : 64;
                bool chk = reach && (int)lane <= ft;
                uint64_t lows = __ballot(chk && !bad);
                uint64_t highs = __ballot(chk && bad);
                if (lows) {
                    int last_low = 63 - __clzll((long long)lows);
                    uint64_t after = last_low == 63 ? 0ull : (~0ull << (last_low + 1));
                    W.rs[s].b = __popcll(highs & after);
                } else {
                    W.rs[s].b += __popcll(highs);
                }
            }
            if (trips) {
                int j = __ffsll((long long)trips) - 1;
                int64_t tj = (int64_t)rl64((uint64_t)t, j);
                W.rs[s].a = 1;
                W.rs[s].c = tj + (int64_t)r.time_window * 1000;
            }
        }
    }
}

__device__ __forceinline__ uint32_t out_to_dec(const DRule* rules, int nr, uint32_t o, int64_t wait) {
    if (o == (uint32_t)nr) return mk_dec(ST_PASS, 0, wait);
    DRule r = rules[o];
    uint32_t st = r.kind == RK_FLOW ? ST_BLOCK_FLOW : r.kind == RK_DEGRADE ? ST_BLOCK_DEGRADE : ST_BLOCK_PARAM;
    return mk_dec(st, r.slot, 0);
}

__global__ __launch_bounds__(DEC_WAVES * WAVE) void k_decide_spec(const sg_event* __restrict__ ev,
                                                                const uint32_t* __restrict__ vals,
                                                                const Seg* __restrict__ segs,
                                                                const uint32_t* __restrict__ order, uint32_t m,
                                                                uint64_t gbase, uint64_t n, DevState S, DevCfg cfg,
                                                                uint32_t* __restrict__ out,
                                                                uint32_t* __restrict__ bflags) {
    __shared__ RState lds_rs[DEC_WAVES][MAX_RULES_PER_RES];
    __shared__ RState lds_sync[DEC_WAVES][MAX_RULES_PER_RES];
    __shared__ DRule lds_rules[DEC_WAVES][MAX_RULES_PER_RES];
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t sidx = blockIdx.x * DEC_WAVES + wv;
    if (sidx >= m) return;
    Wave W;
    W.S = S;
    W.cfg = cfg;
    W.lane = lane_id();
    W.bflags = bflags;
    Seg sg = segs[order[sidx]];
    W.res = sg.res;
    W.prog = S.prog[W.res];
    W.rs = lds_rs[wv];
    const int nr = W.prog.n_param + W.prog.n_flow + W.prog.n_degrade;
    for (int i = W.lane; i < nr; i += WAVE) W.rs[i] = S.rstate[W.prog.rule_off + i];
    W.sb[0] = S.sec[(uint64_t)W.res * 2 + 0];
    W.sb[1] = S.sec[(uint64_t)W.res * 2 + 1];
    NodeInfo ni = S.info[W.res];
    W.thread = ni.thread;
    W.flags = ni.flags;
    W.exc_sum_sec = ni.exc_sum_sec;
    W.exc_sum = ni.exc_sum;
    W.mslot = -1;
    W.mdirty = false;
    W.mdetached = false;
    for (int i = W.lane; i < nr; i += WAVE) lds_rules[wv][i] = S.rules[W.prog.rule_off + i];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const DRule* rules = lds_rules[wv];
    const uint32_t lane = W.lane;
    uint32_t last_out = (uint32_t)nr;
    const bool prof = S.dbg != nullptr && sidx == 0;
    unsigned long long c_tiles = 0, c_rounds = 0, c_iters = 0, t_load = 0, t_ref = 0, t_round = 0, t_eval = 0, t_tail = 0;
    unsigned long long tm0 = prof ? __builtin_amdgcn_s_memtime() : 0, tm1 = 0;

    // software prefetch of the next tile
    uint32_t nidx = 0;
    uint64_t n_ts = 0, n_w1 = 0, n_aux = 0;
    {
        uint32_t c1 = sg.len < WAVE ? sg.len : WAVE;
        if (lane < c1) {
            nidx = vals[sg.start + lane];
            const uint64_t* p = reinterpret_cast<const uint64_t*>(ev + nidx);
            n_ts = p[0]; n_w1 = p[1]; n_aux = p[2];
        }
    }
    for (uint32_t base = 0; base < sg.len; base += WAVE) {
        const uint32_t cnt_t = sg.len - base < WAVE ? sg.len - base : WAVE;
        const uint32_t idx = nidx;
        const int64_t t = (int64_t)n_ts;
        const uint64_t w1 = n_w1, aux = n_aux;
        if (base + WAVE < sg.len) {
            uint32_t c2 = sg.len - base - WAVE < WAVE ? sg.len - base - WAVE : WAVE;
            if (lane < c2) {
                nidx = vals[sg.start + base + WAVE + lane];
                const uint64_t* p = reinterpret_cast<const uint64_t*>(ev + nidx);
                n_ts = p[0]; n_w1 = p[1]; n_aux = p[2];
            }
        }
        if (prof) { tm1 = __builtin_amdgcn_s_memtime(); t_load += tm1 - tm0; tm0 = tm1; ++c_tiles; }
        const bool valid = lane < cnt_t;
        const int cnt = (int)((w1 >> 32) & 0xFFFFu);
        const uint32_t kind = valid ? (uint32_t)((w1 >> 48) & 0xFF) : 0xFFu;
        const uint8_t fl = (uint8_t)(w1 >> 56);
        const bool is_entry = valid && kind == SG_EV_ENTRY;
        const uint64_t gidx = gbase + idx;
        // resolve EXIT/TRACE references: a lane of this tile, or a decided status
        int refl = -1;
        bool known_ok = true;
        int64_t rtv = 0;
        {
            // all lanes take part in the shuffles (ds_bpermute does not read inactive lanes)
            const bool is_ref = valid && kind != SG_EV_ENTRY;
            const uint64_t ref = is_ref ? (aux & SG_REF_NONE) : SG_REF_NONE;
            if (is_ref && kind == SG_EV_EXIT) {
                int64_t raw = (int64_t)(aux >> 48);
                rtv = raw > cfg.max_rt ? cfg.max_rt : raw;
            }
            const uint64_t g0 = rl64(gidx, 0);
            const bool in_tile = ref != SG_REF_NONE && ref >= g0 && ref < gidx;
            int lo = 0, hi = in_tile ? (int)lane : 0;  // gidx strictly increasing across the tile
            #pragma unroll
            for (int k = 0; k < 7; ++k) {
                int mid = (lo + hi) >> 1;
                uint64_t gm = (uint64_t)__shfl((long long)gidx, mid, 64);
                if (lo < hi) { if (gm < ref) lo = mid + 1; else hi = mid; }
            }
            uint64_t gl = (uint64_t)__shfl((long long)gidx, lo, 64);
            if (in_tile) {
                if (gl == ref) refl = lo;
                else known_ok = false; // not an entry of this resource
            } else if (ref != SG_REF_NONE) {
                if (cfg.dbg_flags & 1) known_ok = true;
                else {
                    uint8_t st8 = S.ring[ref & cfg.ring_mask];
                    known_ok = (st8 == ST_PASS || st8 == ST_PASS_WAIT);
                }
            }
        }
        if (prof) { known_ok = __builtin_amdgcn_readfirstlane((int)known_ok) ? known_ok : known_ok; tm1 = __builtin_amdgcn_s_memtime(); t_ref += tm1 - tm0; tm0 = tm1; }
        uint32_t g = is_entry ? last_out : 0u;  // outcome guesses
        uint32_t dec = mk_dec(ST_NOT_ENTRY, 0, 0);
        uint32_t fin = ST_NOT_ENTRY;             // final status per lane (entries)
        int64_t lwait = 0;
        uint32_t c0 = 0;
        const bool chain = (W.flags & NI_CHAIN) != 0 && cfg.switch_on;
        if (!chain) {
            if (is_entry) { dec = mk_dec(ST_NO_CHECK, 0, 0); fin = ST_NO_CHECK; }
            c0 = cnt_t;
        }
        while (c0 < cnt_t) {
            const int64_t tc0 = (int64_t)rl64((uint64_t)t, (int)c0);
            // breaker resets due at tc0 (ResetTask, Q12) and the next reset time
            int64_t next_reset = INT64_MAX;
            for (int s = W.prog.n_param + W.prog.n_flow; s < nr; ++s) {
                if (W.rs[s].a && tc0 >= W.rs[s].c) { W.rs[s].a = 0; W.rs[s].b = 0; }
                if (W.rs[s].a && W.rs[s].c < next_reset) next_reset = W.rs[s].c;
            }
            const int64_t b0 = tc0 / 500;
            const bool inr = valid && lane >= c0 && (t / 500) == b0 && t < next_reset;
            const uint64_t rmask = __ballot(inr);
            const uint32_t e_end = c0 + (uint32_t)__popcll(rmask);
            // base state of the round (buckets are only created/reset by events that write them)
            const bool has_entry = __ballot(inr && is_entry) != 0;
            const int64_t T = tc0 - tc0 % 1000;
            SpecRound R;
            {
                const int cs = (int)(b0 & 1);
                const Bkt cur = cs ? W.sb[1] : W.sb[0];
                const Bkt prv = cs ? W.sb[0] : W.sb[1];
                bool cv = cur.ws == b0 * 500;
                bool pv = prv.ws >= 0 && tc0 - prv.ws <= 1000 && prv.ws <= tc0;
                R.P = (cv ? cur.pass : 0) + (pv ? prv.pass : 0);
                R.B = (cv ? cur.block : 0) + (pv ? prv.block : 0);
                R.S = (cv ? cur.succ : 0) + (pv ? prv.succ : 0);
                R.RT = (cv ? cur.rt : 0) + (pv ? prv.rt : 0);
                R.E = (cv ? cur.exc : 0) + (pv ? prv.exc : 0);
            }
            R.TH = W.thread;
            R.EM = (has_entry && (W.prog.pflags & PF_EXC_COUNT)) ? min_total_exc(W, tc0) : 0;
            RState* synced = lds_sync[wv];
            uint32_t has_sync = 0;
            R.prev_pass_sec = 0;
            bool need_prev = false;
            for (int s = 0; s < nr; ++s) {
                const DRule r = rules[s];
                if (has_entry && r.kind == RK_FLOW && (r.behavior == SG_CONTROL_BEHAVIOR_WARM_UP ||
                                                       r.behavior == SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER)) {
                    if (T > W.rs[s].b) {
                        if (!need_prev) { R.prev_pass_sec = min_prev_pass(W, tc0); need_prev = true; }
                        RState tmp = W.rs[s];
                        warm_sync(r, tmp, tc0, R.prev_pass_sec);
                        synced[s] = tmp;
                        has_sync |= 1u << s;
                    }
                }
            }
            if (prof) { tm1 = __builtin_amdgcn_s_memtime(); t_round += tm1 - tm0; tm0 = tm1; ++c_rounds; }
            // exits/traces: effectiveness under the guesses (referenced lane may be in this round)
            for (;;) {
                if (prof) ++c_iters;
                uint32_t gref = (uint32_t)__shfl((int)g, refl < 0 ? 0 : refl, 64);
                uint32_t fref = (uint32_t)__shfl((int)fin, refl < 0 ? 0 : refl, 64);
                bool eff;
                if (refl < 0) eff = known_ok;
                else if ((uint32_t)refl < c0) eff = (fref == ST_PASS || fref == ST_PASS_WAIT);
                else eff = gref == (uint32_t)nr;
                int64_t wt = 0;
                uint32_t o = spec_eval(W, R, rules, nr, lane, inr, is_entry, eff, kind, t, cnt, rtv, g, wt, synced,
                                       has_sync);
                uint64_t mism = __ballot(inr && is_entry && o != g);
                uint32_t cend = e_end;
                if (mism) cend = (uint32_t)(__ffsll((long long)mism) - 1) + 1;
                // Jacobi update of the guesses
                if (inr && is_entry) g = o;
                const bool com = inr && lane < cend;
                // effectiveness with the final outcomes of the committed lanes
                gref = (uint32_t)__shfl((int)g, refl < 0 ? 0 : refl, 64);
                if (refl >= 0 && (uint32_t)refl >= c0) eff = gref == (uint32_t)nr;
                if (com && is_entry) { dec = out_to_dec(rules, nr, o, wt); fin = dec & 0xFF; lwait = wt; }
                spec_commit(W, R, rules, nr, lane, com, is_entry, eff, kind, t, cnt, rtv, g, tc0, synced, has_sync, T);
                c0 = cend;
                if (prof) { tm1 = __builtin_amdgcn_s_memtime(); t_eval += tm1 - tm0; tm0 = tm1; }
                break;
            }
        }
        // seed the next tile's guesses with the last entry's outcome
        {
            uint64_t em = __ballot(is_entry);
            if (em) {
                int lastl = 63 - __clzll((long long)em);
                uint32_t fo = (uint32_t)__builtin_amdgcn_readlane((int)fin, lastl);
                uint32_t dd = (uint32_t)__builtin_amdgcn_readlane((int)dec, lastl);
                if (fo == ST_PASS) last_out = (uint32_t)nr;
                else if (fo == ST_BLOCK_FLOW || fo == ST_BLOCK_DEGRADE) {
                    // stage index of the blocking rule
                    uint32_t slot = (dd >> 8) & 0xFF;
                    int base_s = fo == ST_BLOCK_FLOW ? W.prog.n_param : W.prog.n_param + W.prog.n_flow;
                    int lim = fo == ST_BLOCK_FLOW ? W.prog.n_flow : W.prog.n_degrade;
                    for (int k = 0; k < lim; ++k) if (rules[base_s + k].slot == slot) { last_out = (uint32_t)(base_s + k); break; }
                }
            }
        }
        (void)lwait;
        if (valid) {
            out[idx] = dec;
            if (is_entry) S.ring[gidx & cfg.ring_mask] = (uint8_t)fin;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (prof) { tm1 = __builtin_amdgcn_s_memtime(); t_tail += tm1 - tm0; tm0 = tm1; }
    }
    if (prof && lane == 0) {
        S.dbg[0] = sg.len; S.dbg[1] = c_tiles; S.dbg[2] = c_rounds; S.dbg[3] = c_iters;
        S.dbg[4] = t_load; S.dbg[5] = t_ref; S.dbg[6] = t_round; S.dbg[7] = t_eval; S.dbg[8] = t_tail;
    }
    min_flush(W);
    if (lane == 0) {
        S.sec[(uint64_t)W.res * 2 + 0] = W.sb[0];
        S.sec[(uint64_t)W.res * 2 + 1] = W.sb[1];
        NodeInfo o = ni;
        o.thread = W.thread;
        o.flags = W.flags;
        o.exc_sum_sec = (W.prog.pflags & PF_EXC_COUNT) ? W.exc_sum_sec : -1;
        o.exc_sum = W.exc_sum;
        S.info[W.res] = o;
    }
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < nr; i += WAVE) S.rstate[W.prog.rule_off + i] = W.rs[i];
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
__global__ void k_init_state(Bkt* __restrict__ sec, Bkt* __restrict__ minb, NodeInfo* __restrict__ info, uint32_t nres) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    Bkt z;
    z.ws = -1; z.pass = 0; z.block = 0; z.exc = 0; z.succ = 0; z.rt = 0; z.occ = 0; z.minrt = 0;
    if (i < (uint64_t)nres * 60) minb[i] = z;
    if (i < (uint64_t)nres * 2) sec[i] = z;
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

// =================================================================================
// host-callable launch wrappers (engine.cpp)
// =================================================================================
namespace sg {

hipError_t launch_radix_hist(const sg_event* ev, const uint32_t* keys, uint64_t n, int shift, uint32_t* ghist,
                             uint32_t nblocks, uint32_t* bflags, uint32_t max_res, hipStream_t st) {
    hipLaunchKernelGGL(k_radix_hist, dim3(nblocks), dim3(RS_THREADS), 0, st, ev, keys, n, shift, ghist, nblocks, bflags,
                       max_res);
    return hipGetLastError();
}
hipError_t launch_radix_scatter(const sg_event* ev, const uint32_t* kin, const uint32_t* vin, uint64_t n, int shift,
                                const uint32_t* goff, uint32_t nblocks, uint32_t* kout, uint32_t* vout, hipStream_t st) {
    hipLaunchKernelGGL(k_radix_scatter, dim3(nblocks), dim3(RS_THREADS), 0, st, ev, kin, vin, n, shift, goff, nblocks,
                       kout, vout);
    return hipGetLastError();
}
uint32_t radix_tile() { return RS_TILE; }

hipError_t launch_init_state(Bkt* sec, Bkt* minb, NodeInfo* info, uint32_t nres, hipStream_t st) {
    uint64_t tot = (uint64_t)nres * 60;
    hipLaunchKernelGGL(k_init_state, dim3((uint32_t)((tot + 255) / 256)), dim3(256), 0, st, sec, minb, info, nres);
    return hipGetLastError();
}
hipError_t launch_set_flags(NodeInfo* info, const uint64_t* upd, uint32_t n, hipStream_t st) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_set_flags, dim3((n + 255) / 256), dim3(256), 0, st, info, upd, n);
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

hipError_t launch_seg(const uint32_t* keys, uint64_t n, uint32_t* flag, uint32_t* pos, uint32_t* part, uint32_t* nseg,
                      Seg* segs, uint32_t* lbucket, const Prog* prog, hipStream_t st) {
    uint32_t nb = (uint32_t)((n + 255) / 256);
    hipLaunchKernelGGL(k_seg_flags, dim3(nb), dim3(256), 0, st, keys, n, flag);
    hipError_t e = launch_scan(flag, pos, n, part, nseg, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_seg_emit, dim3(nb), dim3(256), 0, st, keys, n, flag, pos, segs, lbucket, prog);
    return hipGetLastError();
}
hipError_t launch_seg_order(const Seg* segs, uint32_t m, uint32_t* lcursor, uint32_t* order, hipStream_t st) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(k_seg_order, dim3((m + 255) / 256), dim3(256), 0, st, segs, m, lcursor, order);
    return hipGetLastError();
}
hipError_t launch_chain_candidates(const sg_event* ev, const uint32_t* vals, const Seg* segs, uint32_t m,
                                   const NodeInfo* info, uint32_t* ncand, uint64_t* cand, hipStream_t st) {
    if (m == 0) return hipSuccess;
    hipLaunchKernelGGL(k_chain_candidates, dim3((m + 255) / 256), dim3(256), 0, st, ev, vals, segs, m, info, ncand, cand);
    return hipGetLastError();
}
hipError_t launch_decide(const sg_event* ev, const uint32_t* vals, const Seg* segs, const uint32_t* order, uint32_t m_spec,
                         uint32_t m_serial, uint64_t gbase, uint64_t n, const DevState& S, const DevCfg& cfg,
                         uint32_t* out, uint32_t* bflags, hipStream_t st) {
    const char* mode = getenv("SG_DECIDE_SERIAL");
    bool all_serial = mode && mode[0] == '1';
    uint32_t m = m_spec + m_serial;
    if (all_serial) {
        if (m) hipLaunchKernelGGL(k_decide, dim3((m + DEC_WAVES - 1) / DEC_WAVES), dim3(DEC_WAVES * WAVE), 0, st, ev, vals,
                                  segs, order, m, gbase, n, S, cfg, out, bflags);
        return hipGetLastError();
    }
    if (m_spec)
        hipLaunchKernelGGL(k_decide_spec, dim3((m_spec + DEC_WAVES - 1) / DEC_WAVES), dim3(DEC_WAVES * WAVE), 0, st, ev,
                           vals, segs, order, m_spec, gbase, n, S, cfg, out, bflags);
    if (m_serial)
        hipLaunchKernelGGL(k_decide, dim3((m_serial + DEC_WAVES - 1) / DEC_WAVES), dim3(DEC_WAVES * WAVE), 0, st, ev, vals,
                           segs, order + m_spec, m_serial, gbase, n, S, cfg, out, bflags);
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
