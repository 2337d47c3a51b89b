// chain.h -- lane-local device restatement of one resource's slot chain
// (StatisticSlot -> FlowSlot -> DegradeSlot) over its ClusterNode windows.
//
// Every function here runs on ONE lane and touches only the state passed in:
// the per-lane serial kernel calls them per event, the cooperative (Jacobi)
// kernels call them from a single leader/pivot lane at round boundaries.
// Semantics follow the Java cited at each function (paths as in SURVEY.md §0.1);
// oracle/sentinel_oracle.c is the independent CPU restatement they are checked
// against.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sentinel_gpu.h"
#include "dev_types.h"

namespace sg {

// ---------------------------------------------------------------- Java arithmetic
__device__ __forceinline__ int64_t j_d2l(double d) {  // (long) d
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}
__device__ __forceinline__ int32_t j_d2i(double d) {  // (int) d
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
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ULL;
    x ^= x >> 27; x *= 0x94d049bb133111ebULL;
    x ^= x >> 31; return x;
}
__device__ __forceinline__ uint32_t mk_dec(uint32_t status, uint32_t slot, int64_t wait) {
    if (wait < 0) wait = 0;
    if (wait > 0xFFFF) wait = 0xFFFF;
    return status | ((slot & 0xFFu) << 8) | ((uint32_t)wait << 16);
}
__device__ __forceinline__ bool st_passed(uint32_t st) { return st == ST_PASS || st == ST_PASS_WAIT; }

// ---------------------------------------------------------------- node state
enum : uint32_t { MS_DIRTY = 1u, MS_DETACHED = 2u };

// ClusterNode of one resource: the 2 x 500 ms second window, the cached current
// minute bucket (60 x 1000 ms ring in HBM), curThreadNum and bookkeeping.
struct Node {
    Bkt sb[2];
    Bkt mb;
    int32_t mslot;       // slot of mb, -1 = none cached
    uint32_t mst;        // MS_*
    int32_t thread;
    uint32_t flags;      // NI_*
    int64_t exc_sum_sec; // see NodeInfo
    int64_t exc_sum;
    int64_t* bor;        // borrow ring {ws, pass} x 2 in HBM once a prioritized ENTRY was seen, else null
    // prefetched HBM copy of the minute bucket of the second after mb's (k_lite): -2 = prefetching off,
    // -1 = nothing prefetched.  Only this lane writes the resource's minute buckets, and only mb's slot,
    // so the copy stays exact until mb moves onto its slot.
    int32_t pfslot;
    Bkt pf;
};

__device__ __forceinline__ void node_load(Node& N, const DevState& S, uint32_t res) {
    N.sb[0] = S.sec[(uint64_t)res * 2 + 0];
    N.sb[1] = S.sec[(uint64_t)res * 2 + 1];
    NodeInfo ni = S.info[res];
    N.thread = ni.thread;
    N.flags = ni.flags;
    N.exc_sum_sec = ni.exc_sum_sec;
    N.exc_sum = ni.exc_sum;
    N.mslot = -1;
    N.pfslot = -2;
    N.mst = 0;
    N.bor = S.prio && (S.prio[res] & PM_PRIO) ? S.borrow + (uint64_t)res * 4 : nullptr;
}

__device__ __forceinline__ void bkt_reset(Bkt& b, int64_t ws, int32_t max_rt) {
    b.ws = ws; b.pass = 0; b.block = 0; b.exc = 0; b.succ = 0; b.rt = 0; b.occ = 0; b.minrt = max_rt;
}

// LeapArray.currentWindow for the 2-bucket second window (core/slots/statistic/base/LeapArray.java:117-208):
// returns the slot, or -1 for a detached bucket (clock went back: the update is lost).
// Explicit branches keep sb[] in registers (a runtime index would force it to scratch).
// With a live borrow ring (DevState.prio) a new or reset bucket starts with the pass the borrow bucket of
// t holds (OccupiableBucketLeapArray.newEmptyBucket copies every event, resetWindowTo the pass only,
// OccupiableBucketLeapArray.java:39-64 -- the borrow bucket only ever holds pass, so both are this).
__device__ __forceinline__ void bkt_borrow(Bkt& b, const int64_t* bor, int slot, int64_t t) {
    const int64_t bws = bor[2 * slot];
    if (bws >= 0 && bws <= t && t < bws + 500) b.pass = bor[2 * slot + 1];  // getWindowValue(t)
}
// Both buckets are updated by value selects, never through a pointer chosen by the slot: a selected
// pointer into N.sb makes the compiler keep the node on the stack (scratch), and every scratch access
// then waits for all outstanding memory operations of the lane.
__device__ __forceinline__ void bkt_reset_if(Bkt& b, bool c, int64_t ws, int32_t max_rt) {
    b.ws = c ? ws : b.ws;
    b.pass = c ? 0 : b.pass;
    b.block = c ? 0 : b.block;
    b.exc = c ? 0 : b.exc;
    b.succ = c ? 0 : b.succ;
    b.rt = c ? 0 : b.rt;
    b.occ = c ? 0 : b.occ;
    b.minrt = c ? (int64_t)max_rt : b.minrt;
}
__device__ __forceinline__ int sec_current(Node& N, int64_t t, int32_t max_rt) {
    const int slot = (int)((t / 500) & 1);
    const int64_t ws = t - t % 500;
    const int64_t cws = slot ? N.sb[1].ws : N.sb[0].ws;
    if (cws == ws) return slot;
    if (cws > ws) return -1;
    bkt_reset_if(N.sb[0], slot == 0, ws, max_rt);
    bkt_reset_if(N.sb[1], slot == 1, ws, max_rt);
    if (N.bor) {
        if (slot == 0) bkt_borrow(N.sb[0], N.bor, 0, t);
        else bkt_borrow(N.sb[1], N.bor, 1, t);
    }
    return slot;
}
__device__ __forceinline__ void bkt_add(Bkt& b, int64_t dP, int64_t dB, int64_t dS, int64_t dRT, int64_t dE, int64_t mrt) {
    b.pass += dP; b.block += dB; b.succ += dS; b.rt += dRT; b.exc += dE;
    if (mrt < b.minrt) b.minrt = mrt;
}
__device__ __forceinline__ void bkt_add_if(Bkt& b, bool c, int64_t dP, int64_t dB, int64_t dS, int64_t dRT, int64_t dE,
                                           int64_t mrt) {
    b.pass += c ? dP : 0; b.block += c ? dB : 0; b.succ += c ? dS : 0; b.rt += c ? dRT : 0; b.exc += c ? dE : 0;
    b.minrt = (c && mrt < b.minrt) ? mrt : b.minrt;
}
__device__ __forceinline__ void sec_add(Node& N, int sl, int64_t dP, int64_t dB, int64_t dS, int64_t dRT, int64_t dE,
                                        int64_t mrt) {
    bkt_add_if(N.sb[0], sl == 0, dP, dB, dS, dRT, dE, mrt);
    bkt_add_if(N.sb[1], sl == 1, dP, dB, dS, dRT, dE, mrt);
}
// sum of one counter over LeapArray.values(t): a bucket is valid unless t - ws > 1000 (strict, Q4)
#define SEC_SUM(N, t, f) ((((t) - (N).sb[0].ws <= 1000 && (N).sb[0].ws >= 0) ? (N).sb[0].f : 0) + \
                          (((t) - (N).sb[1].ws <= 1000 && (N).sb[1].ws >= 0) ? (N).sb[1].f : 0))

// write the cached minute bucket back to HBM
__device__ __forceinline__ void min_flush(Node& N, Bkt* minb) {
    if (N.mslot >= 0 && (N.mst & MS_DIRTY) && !(N.mst & MS_DETACHED)) minb[N.mslot] = N.mb;
    N.mst &= ~MS_DIRTY;
}
// StatisticNode.totalException = minute EXCEPTION sum over buckets valid at t (window starts in
// [T-59000, T]), kept as a running sum.  Moves the sum to second T; HBM must hold every bucket
// (cache flushed) and slot(T) must not have been reset yet, so the seconds that fall out of the
// window are still readable.
__device__ __forceinline__ void exc_advance(Node& N, const Bkt* minb, int64_t T) {
    if (N.exc_sum_sec >= 0 && T - N.exc_sum_sec >= 60000) {
        // every bucket was written at or before exc_sum_sec (the sum is advanced on every minute
        // write while the rule exists), so none is valid at T: nothing to read
        N.exc_sum = 0;
    } else if (N.exc_sum_sec < 0) {
        int64_t s = 0;
        for (int k = 0; k < 60; ++k) {
            Bkt b = minb[k];
            if (b.ws >= T - 59000 && b.ws <= T) s += b.exc;
        }
        N.exc_sum = s;
    } else {
        // the seconds that fall out of the window (one bucket a round trip: issuing four at once measured slower in
        // k_lite and k_jac<8>, profiles/r06 A/B)
        const int64_t x1 = T - 60000;
        for (int64_t x = N.exc_sum_sec - 59000; x <= x1; x += 1000) {
            const int sl = (int)((x / 1000) % 60);
            const Bkt b = sl == N.pfslot ? N.pf : minb[sl];
            if (b.ws == x) N.exc_sum -= b.exc;
        }
    }
    N.exc_sum_sec = T;
}
// minute-window currentWindow(t) (LeapArray.java:117-208): caches the bucket of second T in N.mb
__device__ __forceinline__ void min_current(Node& N, Bkt* minb, int64_t t, int32_t max_rt, uint32_t pflags) {
    int slot = (int)((t / 1000) % 60);
    int64_t ws = t - t % 1000;
    if (N.mslot == slot && N.mb.ws == ws) return;
    min_flush(N, minb);
    if ((pflags & PF_EXC_COUNT) && N.exc_sum_sec < ws) exc_advance(N, minb, ws);
    Bkt b = slot == N.pfslot ? N.pf : minb[slot];
    N.mslot = slot;
    N.mst = 0;
    if (N.pfslot >= -1) {  // prefetch the next second's bucket (its load overlaps the events until then)
        N.pfslot = (slot + 1) % 60;
        N.pf = minb[N.pfslot];
    }
    if (b.ws == ws) { N.mb = b; return; }
    bool back = b.ws > ws;
    bkt_reset(b, ws, max_rt);
    N.mb = b;
    N.mst = back ? MS_DETACHED : MS_DIRTY;  // clock went back: a detached bucket (Q3)
}
// ArrayMetric.previousWindowPass on the minute window (LeapArray.getPreviousWindow, LeapArray.java:216-234)
__device__ __forceinline__ int64_t min_prev_pass(Node& N, Bkt* minb, int64_t t, int32_t max_rt, uint32_t pflags) {
    min_current(N, minb, t, max_rt, pflags);
    int slot = (int)(((t - 1000) / 1000) % 60);
    Bkt b = minb[slot];
    if (b.ws < 0) return 0;
    if (t - b.ws > 60000) return 0;
    if (b.ws + 1000 < t - 1000) return 0;
    return b.pass;
}
__device__ __forceinline__ int64_t min_total_exc(Node& N, Bkt* minb, int64_t t, int32_t max_rt, uint32_t pflags) {
    min_current(N, minb, t, max_rt, pflags);
    int64_t T = t - t % 1000;
    if (N.exc_sum_sec != T) {  // rule added since the last advance: recompute (cached slot from registers)
        int64_t s = 0;
        for (int k = 0; k < 60; ++k) {
            Bkt b = (k == N.mslot) ? N.mb : minb[k];
            if (b.ws >= T - 59000 && b.ws <= T) s += b.exc;
        }
        N.exc_sum = s;
        N.exc_sum_sec = T;
    }
    return N.exc_sum;
}
__device__ __forceinline__ void min_add(Node& N, int64_t dP, int64_t dB, int64_t dS, int64_t dRT, int64_t dE, int64_t mrt) {
    if (N.mst & MS_DETACHED) return;
    bkt_add(N.mb, dP, dB, dS, dRT, dE, mrt);
    N.mst |= MS_DIRTY;
}

// ---------------------------------------------------------------- controllers
// WarmUpController.syncToken / coolDownTokens (core/slots/block/flow/controller/WarmUpController.java:141-174)
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
// WarmUpController.canPass warningQps (WarmUpController.java:123-131)
__device__ __forceinline__ double warm_qps(const DRule& r, int64_t rest) {
    int64_t above = rest - r.warning_token;
    return j_next_up(1.0 / ((double)above * r.slope + 1.0 / r.count));
}
// RateLimiterController / WarmUpRateLimiterController queueing (RateLimiterController.java:46-91);
// the sleep becomes wait_ms in the decision (Q10)
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
// cost of one RateLimiter / WarmUpRateLimiter admission at the state s
__device__ __forceinline__ int64_t rl_cost(const DRule& r, const RState& s, int acquire) {
    if (r.behavior == SG_CONTROL_BEHAVIOR_RATE_LIMITER) {
        if (acquire <= 0 || r.count <= 0) return 0;
        return j_round(1.0 * acquire / r.count * 1000);
    }
    if (s.a >= r.warning_token) return j_round(1.0 * acquire / warm_qps(r, s.a) * 1000);
    return j_round(1.0 * acquire / r.count * 1000);
}

struct Ctx {  // per-resource constants
    Bkt* minb;     // the resource's 60 minute buckets
    int32_t max_rt;
    uint32_t pflags;
};

// TrafficShapingController.canPass on the resource's ClusterNode (FlowRuleChecker.passLocalCheck,
// core/slots/block/flow/FlowRuleChecker.java:52-66)
__device__ __forceinline__ bool flow_can_pass(Node& N, const Ctx& C, const DRule& r, RState& s, int64_t t, int acquire,
                                              int64_t& wait) {
    switch (r.behavior) {
    case SG_CONTROL_BEHAVIOR_WARM_UP: {
        sec_current(N, t, C.max_rt);
        int64_t pass_qps = SEC_SUM(N, t, pass);                               // (long) node.passQps()
        int64_t prev = min_prev_pass(N, C.minb, t, C.max_rt, C.pflags);       // (long) node.previousPassQps()
        warm_sync(r, s, t, prev);
        int64_t rest = s.a;
        if (rest >= r.warning_token) return (double)(pass_qps + acquire) <= warm_qps(r, rest);
        return (double)(pass_qps + acquire) <= r.count;
    }
    case SG_CONTROL_BEHAVIOR_RATE_LIMITER: {
        if (acquire <= 0) return true;
        if (r.count <= 0) return false;
        return rl_admit(s.c, rl_cost(r, s, acquire), t, r.max_queue, wait);
    }
    case SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER: {
        int64_t prev = min_prev_pass(N, C.minb, t, C.max_rt, C.pflags);
        warm_sync(r, s, t, prev);
        return rl_admit(s.c, rl_cost(r, s, acquire), t, r.max_queue, wait);
    }
    default: {  // DefaultController (DefaultController.java:49-81)
        int32_t cur;
        if (r.grade == SG_FLOW_GRADE_THREAD) cur = N.thread;
        else { sec_current(N, t, C.max_rt); cur = j_d2i((double)SEC_SUM(N, t, pass)); }
        return !((double)j_iadd(cur, acquire) > r.count);
    }
    }
}

// DegradeRule.passCheck (core/slots/block/degrade/DegradeRule.java:172-223); the ResetTask fires at
// cut_until = t_cut + timeWindow*1000 (Q12).  RState: a = cut, b = passCount, c = cut_until.
// the DegradeRule fields the check reads (k_lite keeps only these in registers)
struct DegParam {
    double count;
    int32_t time_window;
    uint8_t grade;
};
__device__ __forceinline__ DegParam deg_param(const DRule& r) { return DegParam{r.count, r.time_window, r.grade}; }
// exc_total: StatisticNode.totalException at t when the caller keeps it (k_lite), else read through the
// node's cached minute bucket
__device__ __forceinline__ bool degrade_pass(Node& N, const Ctx& C, const DegParam& r, RState& s, int64_t t,
                                             const int64_t* exc_total = nullptr) {
    if (s.a && t >= s.c) { s.a = 0; s.b = 0; }
    if (s.a) return false;
    if (r.grade == SG_DEGRADE_GRADE_RT) {
        sec_current(N, t, C.max_rt);
        int64_t succ = SEC_SUM(N, t, succ);
        double avg = succ == 0 ? 0.0 : (double)SEC_SUM(N, t, rt) * 1.0 / (double)succ;
        if (avg < r.count) { s.b = 0; return true; }
        if (++s.b < 5) return true;
    } else if (r.grade == SG_DEGRADE_GRADE_EXCEPTION_RATIO) {
        sec_current(N, t, C.max_rt);
        double exc = (double)SEC_SUM(N, t, exc) / 1.0;
        double succ = (double)SEC_SUM(N, t, succ) / 1.0;
        double total = (double)SEC_SUM(N, t, pass) / 1.0 + (double)SEC_SUM(N, t, block) / 1.0;
        if (total < 5) return true;
        double real = succ - exc;
        if (real <= 0 && exc < 5) return true;
        if (exc / succ < r.count) return true;
    } else if (r.grade == SG_DEGRADE_GRADE_EXCEPTION_COUNT) {
        double e = (double)(exc_total ? *exc_total : min_total_exc(N, C.minb, t, C.max_rt, C.pflags));
        if (e < r.count) return true;
    }
    s.a = 1;
    s.c = t + (int64_t)r.time_window * 1000;
    return false;
}

// ---------------------------------------------------------------- prioritized entries (k_lane only)
// FutureBucketLeapArray.currentWindow(t) on the borrow ring (LeapArray.java:117-208): slot, or -1
// for a detached bucket (t before the slot's window)
__device__ __forceinline__ int bor_current(int64_t* bor, int64_t t) {
    const int slot = (int)((t / 500) & 1);
    const int64_t ws = t - t % 500;
    const int64_t old = bor[2 * slot];
    if (old < 0 || ws > old) { bor[2 * slot] = ws; bor[2 * slot + 1] = 0; return slot; }
    return ws == old ? slot : -1;
}
// OccupiableBucketLeapArray.currentWaiting: future buckets only (FutureBucketLeapArray.isWindowDeprecated
// is t >= windowStart, FutureBucketLeapArray.java:48-52)
__device__ __forceinline__ int64_t bor_waiting(int64_t* bor, int64_t t) {
    bor_current(bor, t);
    int64_t s = 0;
    if (bor[0] >= 0 && !(t >= bor[0])) s += bor[1];
    if (bor[2] >= 0 && !(t >= bor[2])) s += bor[3];
    return s;
}
// ArrayMetric.getWindowPass(t) of the second window: the bucket whose window holds t (LeapArray.getWindowValue)
__device__ __forceinline__ int64_t sec_window_pass(const Node& N, int64_t t) {
    if (t < 0) return 0;
    const Bkt& b = ((t / 500) & 1) ? N.sb[1] : N.sb[0];
    if (b.ws < 0 || !(b.ws <= t && t < b.ws + 500)) return 0;
    return b.pass;
}
// StatisticNode.tryOccupyNext (core/node/StatisticNode.java:293-325); INTERVAL = 1000, 2 buckets
__device__ __forceinline__ int64_t try_occupy_next(Node& N, const Ctx& C, int64_t now, int acquire, double threshold,
                                                   int32_t occupy_timeout) {
    const double max_count = threshold * 1000 / 1000;
    const int64_t cur_borrow = bor_waiting(N.bor, now);
    if ((double)cur_borrow >= max_count) return occupy_timeout;
    const int64_t wlen = 500;
    int64_t earliest = now - now % wlen + wlen - 1000;
    int64_t idx = 0;
    sec_current(N, now, C.max_rt);
    int64_t cur_pass = SEC_SUM(N, now, pass);
    while (earliest < now) {
        const int64_t wait = idx * wlen + wlen - now % wlen;
        if (wait >= occupy_timeout) break;
        const int64_t wp = sec_window_pass(N, earliest);
        if ((double)(cur_pass + cur_borrow + acquire - wp) <= max_count) return wait;
        earliest += wlen;
        cur_pass -= wp;
        ++idx;
    }
    return occupy_timeout;
}
// DefaultController.canPass with prioritized = true (DefaultController.java:49-81): 1 pass, 0 block,
// 2 PriorityWaitException after addWaitingRequest + addOccupiedPass (wait = waitInMs)
__device__ __forceinline__ int default_can_pass_prio(Node& N, const Ctx& C, const DRule& r, int64_t t, int acquire,
                                                     int32_t occupy_timeout, int64_t& wait) {
    int32_t cur;
    if (r.grade == SG_FLOW_GRADE_THREAD) cur = N.thread;
    else { sec_current(N, t, C.max_rt); cur = j_d2i((double)SEC_SUM(N, t, pass)); }
    if (!((double)j_iadd(cur, acquire) > r.count)) return 1;
    if (r.grade != SG_FLOW_GRADE_QPS || !N.bor) return 0;
    const int64_t w = try_occupy_next(N, C, t, acquire, r.count, occupy_timeout);
    if (w >= occupy_timeout) return 0;
    const int bs = bor_current(N.bor, t + w);  // addWaitingRequest: borrowArray.currentWindow(t + wait).addPass
    if (bs >= 0) N.bor[2 * bs + 1] += acquire;
    min_current(N, C.minb, t, C.max_rt, C.pflags);  // addOccupiedPass: minute window OCCUPIED_PASS + PASS
    if (!(N.mst & MS_DETACHED)) {
        N.mb.occ += acquire;
        N.mb.pass += acquire;
        N.mst |= MS_DIRTY;
    }
    wait = w;
    return 2;
}

// StatisticSlot.entry bookkeeping after the checks (core/slots/statistic/StatisticSlot.java:54-133)
__device__ __forceinline__ void stat_entry(Node& N, const Ctx& C, int64_t t, int count, bool passed) {
    int sl = sec_current(N, t, C.max_rt);
    min_current(N, C.minb, t, C.max_rt, C.pflags);
    if (passed) {
        N.thread++;
        sec_add(N, sl, count, 0, 0, 0, 0, INT64_MAX);
        min_add(N, count, 0, 0, 0, 0, INT64_MAX);
    } else {
        sec_add(N, sl, 0, count, 0, 0, 0, INT64_MAX);
        min_add(N, 0, count, 0, 0, 0, INT64_MAX);
    }
}
// StatisticSlot.exit (StatisticSlot.java:136-173) for an entry that passed; rt already clipped
__device__ __forceinline__ void stat_exit(Node& N, const Ctx& C, int64_t t, int count, int64_t rt) {
    int sl = sec_current(N, t, C.max_rt);
    sec_add(N, sl, 0, 0, count, rt, 0, rt);
    min_current(N, C.minb, t, C.max_rt, C.pflags);
    min_add(N, 0, 0, count, rt, 0, rt);
    N.thread--;
}
// ClusterNode.trace (core/node/ClusterNode.java:99-106)
__device__ __forceinline__ void stat_trace(Node& N, const Ctx& C, int64_t t, int count) {
    if (count <= 0) return;
    int sl = sec_current(N, t, C.max_rt);
    sec_add(N, sl, 0, 0, 0, 0, count, INT64_MAX);
    min_current(N, C.minb, t, C.max_rt, C.pflags);
    if (!(N.mst & MS_DETACHED)) {
        min_add(N, 0, 0, 0, 0, count, INT64_MAX);
        if (N.exc_sum_sec == t - t % 1000) N.exc_sum += count;
    }
}

__device__ __forceinline__ void node_store(const Node& N, const DevState& S, uint32_t res, uint32_t pflags) {
    S.sec[(uint64_t)res * 2 + 0] = N.sb[0];
    S.sec[(uint64_t)res * 2 + 1] = N.sb[1];
    NodeInfo o = S.info[res];
    o.thread = N.thread;
    o.flags = N.flags;
    o.exc_sum_sec = (pflags & PF_EXC_COUNT) ? N.exc_sum_sec : -1;
    o.exc_sum = N.exc_sum;
    S.info[res] = o;
}

} // namespace sg
