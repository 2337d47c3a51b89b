// head.hip -- the event-driven owner of single-rule head segments (C3's THREAD-grade and rate-limiter heads).
//
// A resource whose only rule is one flow rule on its ClusterNode (no degrade, no param rule, DIRECT, limitApp
// default) of these kinds has a decision chain with a single piece of state:
//   XF_HEADT  THREAD-grade DefaultController (core/slots/block/flow/controller/DefaultController.java:49-81): an ENTRY
//             passes iff curThreadNum + acquire <= count; StatisticSlot adds 1 to curThreadNum per pass and takes 1
//             off per effective EXIT (core/slots/statistic/StatisticSlot.java:54-173).  State: the thread count c.
//   XF_HEADR  QPS RateLimiterController (core/slots/block/flow/controller/RateLimiterController.java:46-91): an ENTRY
//             of acquire > 0 passes iff latestPassedTime + cost <= now or latestPassedTime + cost - now <= maxQueue,
//             and then latestPassedTime = max(latestPassedTime + cost, now); WarmUpRateLimiterController likewise, its
//             cost following the stored tokens synced once a second (WarmUpController.java:141-174).  State: L.
// The cooperative owner (decide.hip k_jac) decided such a head by Jacobi iterations over 256- / 1024-lane tiles, whose
// per-iteration chain of block-wide scans and barriers bounded it (C3: 14-17 ms a 2^24-event batch).  Here the owner
// wave walks the segment in chunks of 1,024 positions (16 consecutive a lane), each decided by guess-and-verify rounds
// that need no barrier:
//   THREAD  the passes P_i before position i follow P_{i+1} = min(P_i + [ENTRY], u_i), u_i = max(0, floor(count) -
//           acquire - c + X_i + 1), X_i the effective EXITs before i -- an affine map of the (min, +) semiring, so one
//           wave scan of (a, b) pairs gives every ENTRY's verdict once the EXITs' effectiveness is known.  An EXIT
//           naming an ENTRY of this chunk or the one before is effective iff that ENTRY passed: its guess is that
//           ENTRY's verdict of the round before (a chunk's first round: the last verdict of the chunk before).
//   RATE    with the passes guessed, L before every ENTRY is one wave scan of (max, +) maps x -> max(x + cost, t).
//           Guesses: queueing (L + cost after the round's first arrival) -- the saturated lattice, the n-th pass the
//           first ENTRY at or after L + n * cost - maxQueue, i.e. the THREAD scan over the lattice points up to each
//           arrival; idle -- every ENTRY passes.  A WarmUpRateLimiter round stays inside one second.
// Each round then evaluates every ENTRY exactly at its guessed prefix state; the first event whose evaluation (or, for
// an EXIT, whose ENTRY's verdict) differs from its guess ends the round: everything before it is exact, it takes its
// evaluated outcome, and the next round starts after it.  A round that cannot pass anything (saturated, no effective
// EXIT / no lattice point) is committed as blocked without scans.  Statistics follow once a chunk is decided: per
// 500 ms bucket, folded into the node exactly as k_jac's round_fold folds a round.  EXIT references into earlier
// chunks read a 2^17-position status ring in LDS (older ones the dec[] word).  Seven waves pipeline the chunks
// (head_seg below); one launch takes both kinds (k_head).
#include "chain.h"
#include "dev_types.h"

namespace sg {

#define HD_EP 16u                 // events per lane of a chunk (one 16-bit status word a lane)
#define HD_CH (64u * HD_EP)       // positions per chunk
#define HD_RW 8192u               // status ring words (16 KiB of LDS): 2^17 positions
#define HD_INF 0x3FFFFFFF
#define HD_NONE 0xFFFFFFFFu
#define HD_NEG (-(1ll << 62))

// inclusive wave scans (DPP row shifts + row broadcasts, wave64)
#define HD_DPP(old, v, ctrl, rmask) __builtin_amdgcn_update_dpp((int)(old), (int)(v), ctrl, rmask, 0xf, false)
#define HD_SCAN_STEPS(STEP) \
    STEP(0x111, 0xf) STEP(0x112, 0xf) STEP(0x114, 0xf) STEP(0x118, 0xf) STEP(0x142, 0xa) STEP(0x143, 0xc)

__device__ __forceinline__ uint32_t hd_add_scan(uint32_t v) {
#define S_(c, m) v += (uint32_t)HD_DPP(0, v, c, m);
    HD_SCAN_STEPS(S_)
#undef S_
    return v;
}
__device__ __forceinline__ uint32_t hd_max_scan(uint32_t v) {  // identity 0
#define S_(c, m) { const uint32_t o = (uint32_t)HD_DPP(0, v, c, m); v = o > v ? o : v; }
    HD_SCAN_STEPS(S_)
#undef S_
    return v;
}
__device__ __forceinline__ uint32_t hd_min_red(uint32_t v) {  // wave minimum, uniform
#define S_(c, m) { const uint32_t o = (uint32_t)HD_DPP(0xFFFFFFFFu, v, c, m); v = o < v ? o : v; }
    HD_SCAN_STEPS(S_)
#undef S_
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ uint32_t hd_sum_red(uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)hd_add_scan(v), 63); }
__device__ __forceinline__ uint64_t hd_sum_red64(uint64_t v) {  // in 32 + 16 + 16-bit pieces (no carry lost)
    return ((uint64_t)hd_sum_red((uint32_t)(v >> 32)) << 32) + ((uint64_t)hd_sum_red((uint32_t)v >> 16) << 16) +
           (uint64_t)hd_sum_red((uint32_t)v & 0xFFFFu);
}
// (min, +) maps x -> min(x + a, b), composed in position order: inclusive scan
__device__ __forceinline__ void hd_minplus_scan(int32_t& a, int32_t& b) {
#define S_(c, m) { const int32_t pa = HD_DPP(0, a, c, m), pb = HD_DPP(HD_INF, b, c, m); \
                   const int32_t nb = pb + a; b = nb < b ? nb : b; a = pa + a; }
    HD_SCAN_STEPS(S_)
#undef S_
}
// (max, +) maps x -> max(x + a, b) on int64: inclusive scan
__device__ __forceinline__ void hd_maxplus_scan(int64_t& a, int64_t& b) {
#define D64(old, v, c, m) ((int64_t)(((uint64_t)(uint32_t)HD_DPP((uint32_t)((uint64_t)(old) >> 32), (uint32_t)((uint64_t)(v) >> 32), c, m) << 32) | \
                                    (uint64_t)(uint32_t)HD_DPP((uint32_t)(uint64_t)(old), (uint32_t)(uint64_t)(v), c, m)))
#define S_(c, m) { const int64_t pa = D64(0, a, c, m), pb = D64(HD_NEG, b, c, m); \
                   const int64_t nb = pb + a; b = nb > b ? nb : b; a = pa + a; }
    HD_SCAN_STEPS(S_)
#undef S_
#undef D64
}

__device__ __forceinline__ uint32_t hd_bit(const uint16_t* win, uint32_t p) { return (win[(p >> 4) & (HD_RW - 1)] >> (p & 15)) & 1u; }

// RL: the ENTRY's cost (RateLimiterController.java:53: Math.round(1.0 * acquireCount / count * 1000))
// (WarmUpRateLimiterController.java:50-70: the warming QPS of the second's synced storedTokens, else count)
__device__ __attribute__((noinline)) int64_t hd_cost(double qps, uint32_t cnt, int64_t cost1) {
    if (cnt == 1) return cost1;
    if (cnt == 0 || qps <= 0) return 0;
    return j_round(1.0 * (double)cnt / qps * 1000);
}
// leader, WarmUpRateLimiter: syncToken at the second of the first ENTRY (WarmUpController.java:141-174 with
// previousPassQps: the minute window's pass of the second before, LeapArray.getPreviousWindow), then the QPS its
// cost follows for the rest of the second
__device__ __attribute__((noinline)) double hd_warm_second(const DRule* rp, RState* rs, int64_t now, int64_t prev) {
    const DRule r = *rp;
    RState s = *rs;
    warm_sync(r, s, now, prev);
    *rs = s;
    return s.a >= r.warning_token ? warm_qps(r, s.a) : r.count;
}

// leader: k_jac round_fold of one collected 500 ms bucket (out of line: rare, and its 64-bit node arithmetic would
// otherwise take the round loop's scalar registers)
__device__ __attribute__((noinline)) void hd_fold(Node& node, Ctx C, int64_t cb, uint64_t aP, uint64_t aB, uint64_t aS,
                                                  uint64_t aRT, uint64_t aE, uint32_t aMin) {
    const int64_t tc = cb * 500;
    const int sl = sec_current(node, tc, C.max_rt);
    const int64_t mrt = aMin == HD_NONE ? INT64_MAX : (int64_t)aMin;
    sec_add(node, sl, (int64_t)aP, (int64_t)aB, (int64_t)aS, (int64_t)aRT, (int64_t)aE, mrt);
    min_current(node, C.minb, tc, C.max_rt, C.pflags);
    if (!(node.mst & MS_DETACHED)) {
        min_add(node, (int64_t)aP, (int64_t)aB, (int64_t)aS, (int64_t)aRT, (int64_t)aE, mrt);
        if (node.exc_sum_sec == tc - tc % 1000) node.exc_sum += (int64_t)aE;
    }
}
__device__ __forceinline__ int64_t hd_rl64(int64_t v, uint32_t l) {
    return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)v >> 32), l) << 32) |
                     (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, l));
}
__device__ __forceinline__ int64_t hd_shr64(int64_t v, int64_t ident) {  // the lane below's value (wave_shr:1)
    return (int64_t)(((uint64_t)(uint32_t)HD_DPP((uint32_t)((uint64_t)ident >> 32), (uint32_t)((uint64_t)v >> 32), 0x138, 0xf) << 32) |
                     (uint64_t)(uint32_t)HD_DPP((uint32_t)(uint64_t)ident, (uint32_t)(uint64_t)v, 0x138, 0xf));
}

// one chunk's decoded inputs in LDS, [field][owner lane] (a lane's words in its own bank); three in flight: the
// decoders fill chunk j while the owner decides chunk j - 1 and the statistics wave closes chunk j - 2
#define HD_ND 4u  // decoder waves (four positions of each owner lane apiece)
enum { HM_E = 0, HM_X, HM_T, HM_XS, HM_XD, HM_C1, HM_V, HD_NM };  // ENTRY / EXIT / TRACE kinds, effective (known),
                                                                   // effective iff the ENTRY at ref passed, acquire
                                                                   // != 1, valid
struct HdSlot {
    uint16_t m[HD_ND][HD_NM][64];  // [decoder][mask][owner lane]: bits of the lane's 16 positions
    uint32_t ref[HD_EP][64];
    uint32_t cz[HD_EP][64];
    int32_t dt[HD_EP][64];
    uint32_t wq[HD_EP][64];    // RATE: the passes' waits (the owner writes them, the statistics wave reads them)
};
struct HdShared {
    Node node;
    uint16_t win[HD_RW];       // status ring: a bit a position, a 16-bit word an owner lane's chunk positions
    HdSlot slot[3];
    int32_t hthd;              // RATE: the statistics wave's curThreadNum delta
    RState hrs;                // WarmUpRateLimiter: storedTokens / lastFilledTime as the owner syncs them
    int64_t hmws[60], hmpass[60];
    double hqps;
    unsigned long long tbusy[2];  // diagnostics: a decoder's and the statistics wave's busy cycles
};
__device__ __forceinline__ uint32_t hd_mask(const HdSlot& so, int q, uint32_t lane) {
    uint32_t v = 0;
#pragma unroll
    for (uint32_t h = 0; h < HD_ND; ++h) v |= so.m[h][q][lane];
    return v;
}
__device__ __forceinline__ void hd_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// A workgroup of seven waves per head segment, pipelined over its chunks: waves 1-4 decode chunk j (four positions of
// each owner lane apiece), wave 0 -- the owner -- decides chunk j - 1 (the guess-and-verify rounds), wave 5 writes
// chunk j - 2's verdict words and wave 6 folds its statistics; one LDS barrier a step.  EXIT references into the
// chunk being decided or the one before it are resolved by the owner (their verdicts are not final when decoded).
template <bool RL>
__device__ __forceinline__ void head_seg(HdShared& sh, const SEv* __restrict__ recs, const Seg& sg, const Prog& pg,
                                         const DevState& S, const DevCfg& cfg, int64_t t0, uint32_t* __restrict__ dec,
                                         uint32_t* __restrict__ bflags) {
    Node& node = sh.node;
    uint16_t* win = sh.win;
    HdSlot* slot = sh.slot;
    int32_t& hthd = sh.hthd;
    RState& hrs = sh.hrs;
    int64_t* hmws = sh.hmws;
    int64_t* hmpass = sh.hmpass;
    double& hqps = sh.hqps;
    const uint32_t tid = threadIdx.x;
    const uint32_t wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint32_t lane = tid & 63;
    const uint32_t res = sg.res;
    const double rcount = S.rules[pg.rule_off].count;
    const uint32_t rslot = S.rules[pg.rule_off].slot;
    const int32_t rmaxq = S.rules[pg.rule_off].max_queue;
    if (tid == 0) node_load(node, S, res);
    __syncthreads();
    if (!(node.flags & NI_CHAIN)) {  // no slot chain: every ENTRY is NO_CHECK, nothing is counted
        for (uint32_t p = tid; p < sg.len; p += blockDim.x)
            dec[sg.start + p] = recs[sg.start + p].kind == SG_EV_ENTRY ? mk_dec(ST_NO_CHECK, 0, 0) : mk_dec(ST_NOT_ENTRY, 0, 0);
        return;
    }
    if (tid == 0) {
        const int64_t tf = t0 + recs[sg.start].dt;
        if (tf < (node.sb[0].ws > node.sb[1].ws ? node.sb[0].ws : node.sb[1].ws)) atomicOr(bflags, BF_BACKWARD);
    }
    const Ctx C{S.minb + (uint64_t)res * 60, cfg.max_rt, pg.pflags};
    // WarmUpRateLimiter: the owner syncs the stored tokens at the first ENTRY of every second; previousPassQps is the
    // minute bucket of the second before as the kernel started (its (ws, pass) in LDS) plus this kernel's passes in it
    const bool warm = RL && S.rules[pg.rule_off].behavior == SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER;
    if (warm) {
        if (tid < 60) {
            hmws[tid] = C.minb[tid].ws;
            hmpass[tid] = C.minb[tid].pass;
        }
        if (tid == 0) hrs = S.rstate[pg.rule_off];
    }
    if (tid == 0) hthd = 0;
    __syncthreads();
    const bool prof = S.dbg != nullptr;
    const unsigned long long tm0 = prof ? __builtin_amdgcn_s_memtime() : 0ull;
    const uint32_t nch = (sg.len + HD_CH - 1) / HD_CH;
    const uint32_t lp0 = lane * HD_EP;

    if (wv >= 1 && wv <= HD_ND) {
        // ================= decoders: positions [8h, 8h + 8) of owner lane `lane`, one chunk a step
        const uint32_t h = wv - 1, e0 = h * (HD_EP / HD_ND);
        constexpr uint32_t NE = HD_EP / HD_ND;
        uint4 nxt[NE];
        auto load = [&](uint32_t base) {
#pragma unroll
            for (uint32_t k = 0; k < NE; ++k) {
                const uint32_t p = base + lp0 + e0 + k;
                nxt[k] = make_uint4(0u, 0u, 0u, 0xFFu);
                if (p < sg.len) nxt[k] = reinterpret_cast<const uint4*>(recs + sg.start)[p];
            }
        };
        load(0);
        unsigned long long tbusy = 0;
        for (uint32_t j = 0; j < nch + 2; ++j) {
            if (j < nch) {
                const unsigned long long tb = prof ? __builtin_amdgcn_s_memtime() : 0ull;
                const uint32_t base = j * HD_CH;
                HdSlot& so = slot[j % 3];
                uint32_t mk[HD_NM] = {0, 0, 0, 0, 0, 0, 0};
                uint32_t og = 0, badm = 0;
                uint32_t rref[NE];
#pragma unroll
                for (uint32_t k = 0; k < NE; ++k) {
                    const uint32_t e = e0 + k;
                    const uint4 w = nxt[k];
                    const uint32_t pos = base + lp0 + e;
                    const uint32_t kind = w.w & 0xFFu, code = (w.w >> 16) & 0xFFu;
                    uint32_t rr = w.y - sg.start;
                    const bool isE = kind == SG_EV_ENTRY, isX = kind == SG_EV_EXIT, isT = kind == SG_EV_TRACE;
                    const bool batch = (isX || isT) && code == RC_BATCH;
                    const bool bad = batch && rr >= pos;  // not an earlier ENTRY of this resource
                    rr = bad ? 0u : rr;
                    const bool dyn = batch && rr + HD_CH >= base;                        // this chunk or the one before
                    const bool inr = batch && !dyn && rr + HD_RW * 16u >= base + HD_CH;  // in the LDS ring
                    const uint32_t wb = ((uint32_t)win[(rr >> 4) & (HD_RW - 1)] >> (rr & 15)) & 1u;
                    const bool eff = (isX || isT) && (code == RC_NONE || code == RC_PASSED || (inr && wb));
                    mk[HM_E] |= (uint32_t)isE << e;
                    mk[HM_X] |= (uint32_t)isX << e;
                    mk[HM_T] |= (uint32_t)isT << e;
                    mk[HM_XS] |= (uint32_t)eff << e;
                    mk[HM_XD] |= (uint32_t)dyn << e;
                    mk[HM_C1] |= (uint32_t)(pos < sg.len && (w.z & 0xFFFFu) != 1u) << e;
                    mk[HM_V] |= (uint32_t)(pos < sg.len) << e;
                    og |= (uint32_t)(batch && !dyn && !inr) << e;
                    badm |= (uint32_t)bad << e;
                    rref[k] = rr;
                    so.ref[e][lane] = rr;
                    so.cz[e][lane] = w.z;
                    so.dt[e][lane] = (int32_t)w.x;
                }
                if (badm) atomicOr(bflags, BF_BAD_REF);
                if (og) {  // older than the ring: the dec[] word (stored >= 120 chunks ago)
#pragma unroll
                    for (uint32_t k = 0; k < NE; ++k)
                        if ((og >> (e0 + k)) & 1)
                            if (st_passed(__hip_atomic_load(&dec[sg.start + rref[k]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xFFu))
                                mk[HM_XS] |= 1u << (e0 + k);
                }
#pragma unroll
                for (int q = 0; q < HD_NM; ++q) so.m[h][q][lane] = (uint16_t)mk[q];
                if (j + 1 < nch) load(base + HD_CH);
                if (prof) tbusy += __builtin_amdgcn_s_memtime() - tb;
            }
            hd_lds_barrier();
        }
        if (prof && h == 0 && lane == 0) sh.tbusy[0] = tbusy;
    } else if (wv == 0) {
        // ================= the owner: the guess-and-verify rounds of chunk j - 1
        const double cf = rcount != rcount ? 1e18 : floor(rcount);
        const int32_t Flc = cf > (double)(1 << 29) ? (1 << 29) : cf < -(double)(1 << 29) ? -(1 << 29) : (int32_t)cf;
        int64_t cost1 = (rcount <= 0) ? 0 : j_round(1.0 / rcount * 1000);
        double qps = rcount;  // the QPS the cost of acquire n follows (WarmUpRateLimiter: per second)
        int64_t ksec = INT64_MIN, kcur = 0;  // the second being decided and this kernel's passes in it (uniform)
        const int64_t Q = rmaxq;
        const bool cpos = rcount > 0;
        int32_t c = node.thread;                            // THREAD: curThreadNum (uniform)
        int64_t L = RL ? S.rstate[pg.rule_off].c - t0 : 0;  // RATE: latestPassedTime relative to t0 (uniform)
        bool last_pass = true;                              // the last decided ENTRY passed (round guesses)
        uint32_t n_round = 0;
        unsigned long long ph[4] = {0, 0, 0, 0};  // diagnostics: the owner's round phases
        unsigned long long tround = 0;
        for (uint32_t j = 0; j < nch + 2; ++j) {
            if (j >= 1 && j <= nch) {
                const unsigned long long tr0 = prof ? __builtin_amdgcn_s_memtime() : 0ull;
                const uint32_t q = j - 1, base = q * HD_CH;
                HdSlot& so = slot[q % 3];
                const uint32_t emask = hd_mask(so, HM_E, lane), xk = hd_mask(so, HM_X, lane);
                const uint32_t xs = hd_mask(so, HM_XS, lane), xd = hd_mask(so, HM_XD, lane), c1 = hd_mask(so, HM_C1, lane);
                const uint32_t cnt_t = sg.len - base < HD_CH ? sg.len - base : HD_CH;
                const uint32_t wi = ((base >> 4) + lane) & (HD_RW - 1);
                const bool uni = __ballot(c1 != 0) == 0;  // every event of the chunk counts 1
                // the chunk's times and counts in registers (a round reads them several times; the references stay in
                // LDS, read for the same-chunk EXITs only)
                int32_t dtr[HD_EP];
                uint32_t czr[HD_EP];
                if (RL) {
#pragma unroll
                    for (uint32_t e = 0; e < HD_EP; ++e) {
                        dtr[e] = so.dt[e][lane];
                        czr[e] = so.cz[e][lane];
                    }
                } else if (!uni) {
#pragma unroll
                    for (uint32_t e = 0; e < HD_EP; ++e) {
                        dtr[e] = 0;
                        czr[e] = so.cz[e][lane];
                    }
                } else {
#pragma unroll
                    for (uint32_t e = 0; e < HD_EP; ++e) {
                        dtr[e] = 0;
                        czr[e] = 1u;
                    }
                }
                uint32_t st = last_pass ? emask : 0u;      // committed verdicts below c0, the round's guesses above
                win[wi] = (uint16_t)st;
                if (RL) {
#pragma unroll
                    for (uint32_t e = 0; e < HD_EP; ++e) so.wq[e][lane] = 0;
                }
                uint32_t c0 = 0;
        while (c0 < cnt_t) {
            ++n_round;
            const uint32_t lo = c0 > lp0 ? (c0 - lp0 < HD_EP ? c0 - lp0 : HD_EP) : 0u;
            uint32_t amask = lo >= HD_EP ? 0u : (0xFFFFu << lo) & 0xFFFFu;  // the lane's active positions
            uint32_t act_end = cnt_t;                                         // the round's active range ends here
            unsigned long long pt = prof ? __builtin_amdgcn_s_memtime() : 0ull;
            if (warm) {  // a round stays in the second of its first ENTRY (the cost is fixed there)
                const uint32_t ae = amask & emask;
                const uint64_t eb = __ballot(ae != 0);
                if (eb) {
                    const uint32_t fl = (uint32_t)__ffsll((long long)eb) - 1;
                    const uint32_t fe = (uint32_t)__ffs(__builtin_amdgcn_readlane((int)ae, fl)) - 1;
                    int32_t fdt = 0;
#pragma unroll
                    for (uint32_t e = 0; e < HD_EP; ++e) fdt = e == fe ? dtr[e] : fdt;
                    const int64_t tn = t0 + __builtin_amdgcn_readlane(fdt, fl);
                    const int64_t T = tn - tn % 1000;
                    if (T != ksec) {
                        const int64_t pk = (T - 1000 == ksec) ? kcur : 0;
                        const int sl = (int)(((T - 1000) / 1000) % 60);
                        const int64_t prev = (hmws[sl] == T - 1000 ? hmpass[sl] : 0) + pk;
                        if (lane == 0) hqps = hd_warm_second(S.rules + pg.rule_off, &hrs, tn, prev);
                        __builtin_amdgcn_wave_barrier();  // (one wave: its LDS write lands before its reads)
                        qps = hqps;
                        cost1 = j_round(1.0 / qps * 1000);
                        ksec = T;
                        kcur = 0;
                    }
                    const int64_t se = T + 1000 - t0;  // the second's end, relative
                    const int32_t sei = se > 0x7FFFFFFF ? 0x7FFFFFFF : (int32_t)se;
                    uint32_t after = 0;  // the lane's active positions at or past it
#pragma unroll
                    for (uint32_t e = 0; e < HD_EP; ++e) after |= (uint32_t)(dtr[e] >= sei) << e;
                    after &= amask;
                    const uint64_t ab = __ballot(after != 0);
                    if (ab) {
                        const uint32_t al = (uint32_t)__ffsll((long long)ab) - 1;
                        act_end = al * HD_EP + (uint32_t)__ffs(__builtin_amdgcn_readlane((int)after, al)) - 1;
                    }
                    const uint32_t le = act_end > lp0 ? (act_end - lp0 < HD_EP ? act_end - lp0 : HD_EP) : 0u;
                    amask &= (1u << le) - 1u;
                }
            }
            if (prof) { const unsigned long long _n = __builtin_amdgcn_s_memtime(); ph[0] += _n - pt; pt = _n; }
            const uint32_t am = amask & emask;                                      // ... its active ENTRYs
            uint32_t gm = 0;        // the round's guesses: ENTRYs that pass
            uint32_t mm = 0;        // events whose evaluation differs from the guess
            uint32_t tm = 0;        // evaluated outcomes (ENTRY passes / EXIT effective)
            int64_t mstate = 0;     // the state right after the lane's first mismatch (THREAD c, RATE L)
            int64_t endstate = 0;   // the state after the lane's last position
            if (!RL) {
                // EXITs' effectiveness under the guesses (LDS: committed verdicts / the last round's guesses)
                const uint32_t dx = xd & xk & amask;
                uint32_t dg = 0;
                if (dx) {
#pragma unroll
                    for (uint32_t e = 0; e < HD_EP; ++e) dg |= (hd_bit(win, so.ref[e][lane]) & (dx >> e)) << e;
                }
                const uint32_t xm = (xs | dg) & xk & amask;
                const uint32_t xl = (uint32_t)__popc(xm);
                const uint32_t xin = hd_add_scan(xl);
                const int32_t X0 = (int32_t)(xin - xl);
                // frozen round: saturated (c + 1 > count), unit acquire counts and no effective EXIT among the active
                // positions -- no ENTRY can pass, every guess is exact: all blocked, nothing to scan
                const bool frz = uni && Flc <= c && __builtin_amdgcn_readlane((int)xin, 63) == 0;
                if (frz) {
                    st &= ~amask;
                    win[wi] = (uint16_t)st;
                    endstate = c;
                } else {
                    const int32_t bu = Flc + 1 - c;  // u = max(0, floor(count) - acquire - c + X + 1)
                    int32_t A = 0, B = HD_INF;
                    {
                        int32_t X = X0;
    #pragma unroll
                        for (uint32_t e = 0; e < HD_EP; ++e) {
                            const int32_t a = (int32_t)((am >> e) & 1);
                            int32_t u = bu - (int32_t)(czr[e] & 0xFFFFu) + X;
                            u = u < 0 ? 0 : u > HD_INF ? HD_INF : u;
                            const int32_t nb = B + 1 < u ? B + 1 : u;
                            B = a ? nb : B;
                            A += a;
                            X += (int32_t)((xm >> e) & 1);
                        }
                    }
                    int32_t ia = A, ib = B;
                    hd_minplus_scan(ia, ib);
                    int32_t pa = HD_DPP(0, ia, 0x138, 0xf), pb = HD_DPP(HD_INF, ib, 0x138, 0xf);  // wave_shr:1
                    pa = lane == 0 ? 0 : pa;
                    pb = lane == 0 ? HD_INF : pb;
                    {  // the closed form's guesses (exact for acquire counts of 1 and right EXIT guesses)
                        int32_t P = pa < pb ? pa : pb, X = X0;
    #pragma unroll
                        for (uint32_t e = 0; e < HD_EP; ++e) {
                            const bool a = (am >> e) & 1;
                            int32_t u = bu - (int32_t)(czr[e] & 0xFFFFu) + X;
                            u = u < 0 ? 0 : u > HD_INF ? HD_INF : u;
                            const int32_t Pn = a ? (P + 1 < u ? P + 1 : u) : P;
                            gm |= (uint32_t)(Pn > P) << e;
                            P = Pn;
                            X += (int32_t)((xm >> e) & 1);
                        }
                    }
                    // publish the guesses (same-chunk EXITs read them; a wave's LDS operations complete in order)
                    st = (st & ~amask) | gm;
                    win[wi] = (uint16_t)st;
                    const uint32_t gl = (uint32_t)__popc(gm);
                    const uint32_t gin = hd_add_scan(gl);
                    const int32_t P0 = (int32_t)(gin - gl);
                    if (!uni) {  // mixed acquire counts: the closed form is a guess; evaluate at the counted prefix
                        int32_t Pc = P0, Xc = X0;
    #pragma unroll
                        for (uint32_t e = 0; e < HD_EP; ++e) {
                            const bool a = (am >> e) & 1, g = (gm >> e) & 1;
                            const int32_t ci = c + Pc - Xc;
                            const bool tr = !((double)j_iadd(ci, (int32_t)(czr[e] & 0xFFFFu)) > rcount);
                            mm |= (uint32_t)(a && tr != g) << e;
                            tm |= (uint32_t)(a && tr) << e;
                            Pc += g ? 1 : 0;
                            Xc += (int32_t)((xm >> e) & 1);
                        }
                    } else {
                        tm |= gm;
                    }
                    if (dx) {  // same-chunk EXITs: effective iff their ENTRY's new guess passes
    #pragma unroll
                        for (uint32_t e = 0; e < HD_EP; ++e) {
                            const uint32_t now = hd_bit(win, so.ref[e][lane]), d = (dx >> e) & 1, was = (xm >> e) & 1;
                            mm |= (d & (now ^ was)) << e;
                            tm |= (d & now) << e;
                        }
                    }
                    if (mm) {  // the state right after the lane's first mismatch
                        const uint32_t e1 = (uint32_t)__ffs((int)mm) - 1, below = (1u << e1) - 1u;
                        const int32_t cb1 = c + P0 + __popc(gm & below) - (X0 + __popc(xm & below));
                        const int32_t t1 = (int32_t)((tm >> e1) & 1);
                        mstate = ((emask >> e1) & 1) ? cb1 + t1 : cb1 - t1;
                    }
                    endstate = (int64_t)c + (int32_t)gin - (int32_t)xin;
                }
            } else {
                // RATE: the round's guesses.  Queueing (L + cost after the first active ENTRY's arrival): the saturated
                // lattice -- the n-th pass of the round is the first ENTRY at or after L + n * cost - maxQueue while each
                // pass moves L by exactly cost, i.e. P_{i+1} = min(P_i + 1, k(t_i)) with k(t) the lattice points up to t:
                // the (min, +) scan of the THREAD owner.  Idle (L + cost at or before it): every ENTRY passes.
                uint32_t tf = 0x7FFFFFFFu;
                {
                    const uint64_t eb = __ballot(am != 0);
                    if (eb) {
                        const uint32_t fl = (uint32_t)__ffsll((long long)eb) - 1;
                        const uint32_t fe = (uint32_t)__ffs(__builtin_amdgcn_readlane((int)am, fl)) - 1;
                        int32_t fdt = 0;
#pragma unroll
                        for (uint32_t e = 0; e < HD_EP; ++e) fdt = e == fe ? dtr[e] : fdt;
                        tf = (uint32_t)__builtin_amdgcn_readlane(fdt, fl);
                    }
                }
                const bool lattice = cost1 > 0 && cost1 < (1 << 24) && L + cost1 > (int64_t)(int32_t)tf;
                // lattice points up to t: floor((t - (L - Q)) / cost), in 32-bit arithmetic (lattice: L is within a
                // cost of the round's first arrival, so the offsets of the chunk's times fit; clamped regardless)
                const int64_t lq64 = L - Q;
                const int32_t lq = lq64 > (1 << 30) ? (1 << 30) : lq64 < -(1 << 30) ? -(1 << 30) : (int32_t)lq64;
                const int32_t ci = (int32_t)cost1;
                const float rc = 1.0f / (float)ci;
                auto lat = [&](int32_t t) -> int32_t {  // max(0, floor((t - lq) / cost)), exact
                    int32_t x = t - lq;
                    x = x < 0 ? -1 : x > (1 << 30) ? (1 << 30) : x;
                    int32_t k = (int32_t)((float)x * rc);
                    k = k * ci > x ? k - 1 : k;
                    k = (k + 1) * ci <= x ? k + 1 : k;
                    return k < 0 ? 0 : k;
                };
                // the lattice ENTRYs: acquire > 0 (an acquire-0 ENTRY of a RateLimiter passes without moving L)
                uint32_t lm = 0;
#pragma unroll
                for (uint32_t e = 0; e < HD_EP; ++e)
                    lm |= (uint32_t)(((am >> e) & 1) && (warm || (czr[e] & 0xFFFFu) != 0)) << e;
                // frozen round: queueing, unit acquire counts and no lattice point up to the last active arrival -- every
                // active ENTRY blocks (L + cost - t > maxQueue for all of them) and L stays: nothing to scan
                bool frz = false;
                if (lattice && uni) {
                    const uint64_t lb2 = __ballot(am != 0);
                    const uint32_t ll2 = 63u - (uint32_t)__clzll((long long)lb2);
                    int32_t ldt = 0;
#pragma unroll
                    for (uint32_t e = 0; e < HD_EP; ++e) ldt = ((am >> e) & 1) ? dtr[e] : ldt;
                    frz = lat(__builtin_amdgcn_readlane(ldt, ll2)) == 0;
                }
                uint32_t lg = 0;  // lattice guesses
                if (frz) {
                    endstate = L;
                    st &= ~amask;
                } else {
                if (lattice) {
                    int32_t A2 = 0, B2 = HD_INF;
#pragma unroll
                    for (uint32_t e = 0; e < HD_EP; ++e) {
                        const int32_t u = lat(dtr[e]);
                        const int32_t a2 = (int32_t)((lm >> e) & 1);
                        const int32_t nb = B2 + 1 < u ? B2 + 1 : u;
                        B2 = a2 ? nb : B2;
                        A2 += a2;
                    }
                    int32_t ia2 = A2, ib2 = B2;
                    hd_minplus_scan(ia2, ib2);
                    int32_t pa2 = HD_DPP(0, ia2, 0x138, 0xf), pb2 = HD_DPP(HD_INF, ib2, 0x138, 0xf);
                    pa2 = lane == 0 ? 0 : pa2;
                    pb2 = lane == 0 ? HD_INF : pb2;
                    int32_t P = pa2 < pb2 ? pa2 : pb2;
#pragma unroll
                    for (uint32_t e = 0; e < HD_EP; ++e) {
                        const int32_t u = lat(dtr[e]);
                        const int32_t Pn = ((lm >> e) & 1) ? (P + 1 < u ? P + 1 : u) : P;
                        lg |= (uint32_t)(Pn > P) << e;
                        P = Pn;
                    }
                }
                if (prof) { const unsigned long long _n = __builtin_amdgcn_s_memtime(); ph[1] += _n - pt; pt = _n; }
                int64_t A = 0, B = HD_NEG;
#pragma unroll
                for (uint32_t e = 0; e < HD_EP; ++e) {
                    const bool a = (am >> e) & 1;
                    const uint32_t cnt = czr[e] & 0xFFFFu;
                    const bool g = a && (cnt == 0 || (cpos && (!lattice || ((lg >> e) & 1))));
                    gm |= (uint32_t)g << e;
                    const int64_t cs = uni ? cost1 : hd_cost(qps, cnt, cost1);
                    const bool up = g && (warm || (cnt > 0 && cpos));
                    const int64_t nb = B + cs > (int64_t)dtr[e] ? B + cs : (int64_t)dtr[e];
                    B = up ? nb : B;
                    A += up ? cs : 0;
                }
                int64_t ia = A, ib = B;
                hd_maxplus_scan(ia, ib);
                int64_t pa = hd_shr64(ia, 0), pb = hd_shr64(ib, HD_NEG);
                pa = lane == 0 ? 0 : pa;
                pb = lane == 0 ? HD_NEG : pb;
                int64_t Lc = L + pa > pb ? L + pa : pb;  // L before the lane's first active position
#pragma unroll
                for (uint32_t e = 0; e < HD_EP; ++e) {
                    const bool a = (am >> e) & 1, g = (gm >> e) & 1;
                    const uint32_t cnt = czr[e] & 0xFFFFu;
                    const int64_t t = dtr[e];
                    const int64_t cs = uni ? cost1 : hd_cost(qps, cnt, cost1);
                    const bool up = warm || (cnt > 0 && cpos);  // (WarmUpRateLimiter: acquire 0 is a check of cost 0)
                    const bool tr = (!warm && cnt == 0) || (cpos && ((Lc + cs <= t) || (Lc + cs - t <= Q)));
                    const int64_t Ln = Lc + cs > t ? Lc + cs : t;
                    const int64_t wv = Lc + cs - t;
                    const uint32_t w = (tr && up && wv > 0) ? (wv > 0xFFFF ? 0xFFFFu : (uint32_t)wv) : 0u;
                    if (a) so.wq[e][lane] = w;
                    const bool mis = a && tr != g;
                    mstate = (mis && !mm) ? ((tr && up) ? Ln : Lc) : mstate;
                    mm |= (uint32_t)mis << e;
                    tm |= (uint32_t)(a && tr) << e;
                    Lc = (a && g && up) ? Ln : Lc;
                }
                endstate = Lc;
                st = (st & ~amask) | gm;
                }
            }
            if (prof) { const unsigned long long _n = __builtin_amdgcn_s_memtime(); ph[2] += _n - pt; pt = _n; }
            // the wave's first mismatch (lanes in position order): it takes its evaluated outcome, everything before
            // it stands, positions after it keep the round's guesses for the next round
            const uint64_t bal = __ballot(mm != 0);
            uint32_t cend, ml = 63, me = HD_EP;
            int64_t ns;
            if (bal) {
                ml = (uint32_t)__ffsll((long long)bal) - 1;
                me = (uint32_t)__ffs(__builtin_amdgcn_readlane((int)mm, ml)) - 1;
                const uint32_t mt = ((uint32_t)__builtin_amdgcn_readlane((int)tm, ml) >> me) & 1u;
                cend = ml * HD_EP + me + 1;
                const uint32_t fb = (lane == ml) ? (emask & (1u << me)) : 0u;
                st = (st & ~fb) | (mt ? fb : 0u);
                ns = hd_rl64(mstate, ml);
            } else {
                cend = act_end;
                ns = hd_rl64(endstate, 63);
            }
            win[wi] = (uint16_t)st;
            if (RL) L = ns; else c = (int32_t)ns;
            {  // the last committed ENTRY's verdict seeds the next round's guesses
                const uint32_t cm = lane < ml ? 0xFFFFu : lane == ml ? (me >= HD_EP ? 0xFFFFu : (2u << me) - 1u) : 0u;
                const uint32_t em = am & cm;
                const uint64_t eb = __ballot(em != 0);
                if (eb) {
                    const uint32_t ll = 63u - (uint32_t)__clzll((long long)eb);
                    const uint32_t lem = (uint32_t)__builtin_amdgcn_readlane((int)em, ll);
                    const uint32_t lst = (uint32_t)__builtin_amdgcn_readlane((int)st, ll);
                    last_pass = (lst >> (31u - (uint32_t)__clz(lem))) & 1u;
                }
            }
            if (warm) {  // the round's passes (all in second ksec) for the next second's previousPassQps
                const uint32_t cm = lane < ml ? 0xFFFFu : lane == ml ? (me >= HD_EP ? 0xFFFFu : (2u << me) - 1u) : 0u;
                const uint32_t pm = am & cm & st;
                uint32_t sp = 0;
#pragma unroll
                for (uint32_t e = 0; e < HD_EP; ++e) sp += ((pm >> e) & 1) ? (czr[e] & 0xFFFFu) : 0u;
                kcur += hd_sum_red(sp);
            }
            if (prof) { const unsigned long long _n = __builtin_amdgcn_s_memtime(); ph[3] += _n - pt; pt = _n; }
            c0 = cend;
        }
                if (prof) tround += __builtin_amdgcn_s_memtime() - tr0;
            }
            hd_lds_barrier();
        }
        // the segment's end (after the statistics wave's last fold: the loop's last barrier)
        if (lane == 0) {
            node.thread = RL ? node.thread + hthd : c;
            min_flush(node, C.minb);
            node_store(node, S, res, pg.pflags);
            if (RL) {
                RState o = warm ? hrs : S.rstate[pg.rule_off];
                o.c = L + t0;
                S.rstate[pg.rule_off] = o;
            }
            if (prof) {
                const unsigned long long tot = __builtin_amdgcn_s_memtime() - tm0;
                if (atomicMax(&S.dbg[59], tot) < tot) {
                    S.dbg[60] = sg.len;
                    S.dbg[61] = nch;
                    S.dbg[62] = n_round;
                    S.dbg[30] = tround;
                    S.dbg[44] = sh.tbusy[0];
                    S.dbg[45] = sh.tbusy[1];
                    S.dbg[31] = (unsigned long long)rcount;
                    S.dbg[46] = ph[0]; S.dbg[47] = ph[1]; S.dbg[48] = ph[2]; S.dbg[49] = ph[3];
                }
            }
        }
    } else if (wv == HD_ND + 1) {
        // ================= chunk j - 2's verdict words
        const uint32_t dblock = mk_dec(ST_BLOCK_FLOW, rslot, 0), dnot = mk_dec(ST_NOT_ENTRY, 0, 0);
        for (uint32_t j = 0; j < nch + 2; ++j) {
            if (j >= 2) {
                const uint32_t q = j - 2, base = q * HD_CH;
                const HdSlot& so = slot[q % 3];
                const uint32_t emask = hd_mask(so, HM_E, lane), vmask = hd_mask(so, HM_V, lane);
                const uint32_t st = win[((base >> 4) + lane) & (HD_RW - 1)];
#pragma unroll
                for (uint32_t e = 0; e < HD_EP; ++e) {
                    const uint32_t d = ((emask >> e) & 1) ? (((st >> e) & 1) ? mk_dec(ST_PASS, 0, RL ? (int64_t)so.wq[e][lane] : 0) : dblock) : dnot;
                    if ((vmask >> e) & 1) dec[sg.start + base + lp0 + e] = d;
                }
                if ((q & 31u) == 31u) __threadfence_block();  // (old references read the dec[] words)
            }
            hd_lds_barrier();
        }
    } else if (wv == HD_ND + 2) {
        // ================= chunk j - 2's statistics (per 500 ms bucket, as k_jac's round_fold)
        const int32_t toff = (int32_t)(((t0 % 500) + 500) % 500);
        const int64_t tb0 = (t0 - toff) / 500;  // bucket of relative time -toff
        int64_t cb = -1;                        // the bucket being collected (uniform); per-lane sums
        uint64_t aP = 0, aB = 0, aS = 0, aRT = 0, aE = 0;
        uint32_t aMin = HD_NONE, aT = 0;
        int32_t thd = 0;
        auto fold = [&]() {
            const uint32_t t = hd_sum_red(aT);
            if (t) {
                const uint64_t P = hd_sum_red64(aP), Bk = hd_sum_red64(aB), Su = hd_sum_red64(aS), RT = hd_sum_red64(aRT),
                               Ex = hd_sum_red64(aE);
                const uint32_t mn = hd_min_red(aMin);
                if (lane == 0) hd_fold(node, C, cb, P, Bk, Su, RT, Ex, mn);
            }
            aP = aB = aS = aRT = aE = 0;
            aMin = HD_NONE;
            aT = 0;
        };
        unsigned long long tbusy = 0;
        for (uint32_t j = 0; j < nch + 2; ++j) {
            if (j >= 2) {
                const unsigned long long tb = prof ? __builtin_amdgcn_s_memtime() : 0ull;
                const uint32_t q = j - 2, base = q * HD_CH;
                HdSlot& so = slot[q % 3];
                const uint32_t emask = hd_mask(so, HM_E, lane), xk = hd_mask(so, HM_X, lane), tk = hd_mask(so, HM_T, lane);
                const uint32_t xd = hd_mask(so, HM_XD, lane), c1 = hd_mask(so, HM_C1, lane), vmask = hd_mask(so, HM_V, lane);
                uint32_t xe = hd_mask(so, HM_XS, lane);
                const uint32_t st = win[((base >> 4) + lane) & (HD_RW - 1)];
                if (xd) {
#pragma unroll
                    for (uint32_t e = 0; e < HD_EP; ++e) xe |= (hd_bit(win, so.ref[e][lane]) & (xd >> e)) << e;
                }
                xe &= xk | tk;
                if (RL) thd += (int32_t)hd_sum_red((uint32_t)(__popc(emask & st) - __popc(xe & xk)));
                int32_t dt[HD_EP];
                uint32_t cz[HD_EP];
#pragma unroll
                for (uint32_t e = 0; e < HD_EP; ++e) {
                    dt[e] = so.dt[e][lane];
                    cz[e] = so.cz[e][lane];
                }
                // one bucket for the whole chunk with every count 1 (the usual case): popcounts
                const int32_t dfirst = __builtin_amdgcn_readfirstlane(dt[0]);
                const uint64_t vb = __ballot(vmask != 0);
                const uint32_t ll = 63u - (uint32_t)__clzll((long long)vb);
                int32_t dl = 0;
#pragma unroll
                for (uint32_t e = 0; e < HD_EP; ++e) dl = ((vmask >> e) & 1) ? dt[e] : dl;
                const int32_t dlast = __builtin_amdgcn_readlane(dl, ll);
                auto bkt_of = [&](int32_t d) -> int32_t { const int32_t x = d + toff; return x >= 0 ? x / 500 : -((499 - x) / 500); };
                const int32_t bf = bkt_of(dfirst);
                if (bf == bkt_of(dlast) && __ballot(c1 != 0) == 0) {
                    const int64_t b = tb0 + bf;
                    if (b != cb) {
                        fold();
                        cb = b;
                    }
                    const uint32_t xx = xe & xk, tt = xe & tk, ne = (uint32_t)__popc(emask & vmask), np = (uint32_t)__popc(emask & st);
                    aP += np;
                    aB += ne - np;
                    aS += (uint32_t)__popc(xx);
                    aE += (uint32_t)__popc(tt);
                    aT += ne + (uint32_t)__popc(xx) + (uint32_t)__popc(tt);
                    uint32_t sRT = 0, sMin = HD_NONE;
#pragma unroll
                    for (uint32_t e = 0; e < HD_EP; ++e) {
                        const uint32_t rtv = cz[e] >> 16;
                        const bool x = (xx >> e) & 1;
                        sRT += x ? rtv : 0u;
                        sMin = (x && rtv < sMin) ? rtv : sMin;
                    }
                    aRT += sRT;
                    aMin = sMin < aMin ? sMin : aMin;
                } else {
                    uint32_t left = vmask;  // events not yet in a bucket
                    for (;;) {
                        const uint64_t lb = __ballot(left != 0);
                        if (!lb) break;
                        const uint32_t fl = (uint32_t)__ffsll((long long)lb) - 1;
                        const uint32_t fe = (uint32_t)__ffs((int)left) - 1;
                        int32_t fdt = 0;
#pragma unroll
                        for (uint32_t e = 0; e < HD_EP; ++e) fdt = e == fe ? dt[e] : fdt;
                        const int32_t brel = bkt_of(__builtin_amdgcn_readlane(fdt, fl));
                        const int64_t b = tb0 + brel;
                        if (b != cb) {
                            fold();
                            cb = b;
                        }
                        const int32_t lo_dt = brel * 500 - toff, hi_dt = lo_dt + 500;  // the bucket's relative times
                        uint32_t sP = 0, sB = 0, sS = 0, sRT = 0, sE = 0, sT = 0, sMin = HD_NONE;
#pragma unroll
                        for (uint32_t e = 0; e < HD_EP; ++e) {
                            const bool in = ((left >> e) & 1) && dt[e] >= lo_dt && dt[e] < hi_dt;
                            const uint32_t cnt = cz[e] & 0xFFFFu, rtv = cz[e] >> 16;
                            const bool ent = in && ((emask >> e) & 1), ps = ent && ((st >> e) & 1);
                            const bool x = in && ((xe & xk) >> e) & 1, t = in && ((xe & tk) >> e) & 1 && cnt > 0;
                            sP += ps ? cnt : 0u;
                            sB += (ent && !ps) ? cnt : 0u;
                            sS += x ? cnt : 0u;
                            sRT += x ? rtv : 0u;
                            sMin = (x && rtv < sMin) ? rtv : sMin;
                            sE += t ? cnt : 0u;
                            sT += (ent || x || t) ? 1u : 0u;
                            left &= ~((uint32_t)in << e);
                        }
                        aP += sP;
                        aB += sB;
                        aS += sS;
                        aRT += sRT;
                        aE += sE;
                        aT += sT;
                        aMin = sMin < aMin ? sMin : aMin;
                    }
                }
                if (q + 1 == nch) {
                    fold();
                    if (lane == 0) hthd = thd;
                }
                if (prof) tbusy += __builtin_amdgcn_s_memtime() - tb;
            }
            hd_lds_barrier();
        }
        if (prof && lane == 0) sh.tbusy[1] = tbusy;
    }
}

// one launch for both kinds (a bin's THREAD-grade and rate-limiter heads run side by side)
__global__ __launch_bounds__(64 * (HD_ND + 3)) void k_head(const SEv* __restrict__ recs, const Seg* __restrict__ segs,
                                              const uint32_t* __restrict__ order, uint32_t m, DevState S, DevCfg cfg,
                                              int64_t t0, uint32_t* __restrict__ dec, uint32_t* __restrict__ bflags) {
    __shared__ HdShared sh;
    if (blockIdx.x >= m) return;
    const Seg sg = segs[order[blockIdx.x]];
    const Prog pg = S.prog[sg.res];
    if (pg.xf & XF_HEADT) head_seg<false>(sh, recs, sg, pg, S, cfg, t0, dec, bflags);
    else if (pg.xf & XF_HEADR) head_seg<true>(sh, recs, sg, pg, S, cfg, t0, dec, bflags);
    // (else: the cooperative owner's segment)
}

hipError_t launch_head(const SEv* recs, const Seg* segs, const uint32_t* order, uint32_t m, const DevState& S,
                       const DevCfg& cfg, int64_t t0, uint32_t* dec, uint32_t* bflags, hipStream_t st) {
    if (!m) return hipSuccess;
    hipLaunchKernelGGL(k_head, dim3(m), dim3(64 * (HD_ND + 3)), 0, st, recs, segs, order, m, S, cfg, t0, dec, bflags);
    return hipGetLastError();
}

} // namespace sg
