// dev_types.h -- device-resident state of the MI355X decision engine.
//
// HBM layout (one engine = one GPU = one shard of resources):
//   Bkt     sec[R][2]     rollingCounterInSecond buckets (core/node/StatisticNode.java:102)
//   Bkt     minb[R][60]   rollingCounterInMinute buckets (core/node/StatisticNode.java:111)
//   NodeInfo info[R]      curThreadNum, chain/metric flags, exception running sum
//   Prog    prog[R]       compiled rule program: [param..., flow..., degrade...]
//   DRule   rules[]       compiled rule constants
//   RState  rstate[]      controller / breaker state (one per rule)
//   PSlot   ptab[2^k]     exact open-addressing table: (param rule state id, value) -> token bucket,
//                         (resource, value) -> param thread count (ParameterMetric maps)
//   uint8   ring[2^k]     status of every ENTRY by global event index (EXIT/TRACE references)
// All counters are int64 exactly as the Java LongAdders; RT sums are int64.
#pragma once
#include <stdint.h>

namespace sg {

// one LeapArray bucket: MetricBucket (core/slots/statistic/data/MetricBucket.java:28-139)
struct Bkt {
    int64_t ws;      // window start; -1 = never created (WindowWrap absent)
    int64_t pass;
    int64_t block;
    int64_t exc;
    int64_t succ;
    int64_t rt;
    int64_t occ;
    int64_t minrt;
};
static_assert(sizeof(Bkt) == 64, "Bkt must be 64 B");

enum : uint32_t {
    NI_CHAIN = 1u,       // CtSph chainMap holds this resource (and its ClusterNode exists)
    NI_REJECTED = 2u,    // lookProcessChain returned null once the cap was reached
    NI_PM = 4u,          // ParamFlowSlot.metricsMap has a ParameterMetric for it
    NI_TM0 = 8u,         // ... with a thread-count map for paramIdx 0
};

struct NodeInfo {
    int32_t thread;      // StatisticNode.curThreadNum
    uint32_t flags;      // NI_*
    int64_t exc_sum_sec; // second T for which exc_sum = sum of minute exceptions with ws in [T-59000, T]; -1 unknown
    int64_t exc_sum;
    int64_t last_fetch;  // StatisticNode.lastFetchTime (metrics snapshots)
};
static_assert(sizeof(NodeInfo) == 32, "NodeInfo must be 32 B");

enum : uint8_t { PF_EXC_COUNT = 1, PF_WARM = 2, PF_PARAM_IDX0 = 4 };

struct Prog {
    uint32_t rule_off;
    uint8_t n_param, n_flow, n_degrade, pflags;
    uint32_t tc_epoch;   // epoch of this resource's param thread-count keys
    uint32_t pad;
};
static_assert(sizeof(Prog) == 16, "Prog must be 16 B");

enum : uint8_t { RK_PARAM = 0, RK_FLOW = 1, RK_DEGRADE = 2 };

// compiled rule (host: engine.cpp compile_*)
struct DRule {
    uint8_t kind;
    uint8_t grade;       // flow/param: FLOW_GRADE_*; degrade: DEGRADE_GRADE_*
    uint8_t behavior;    // CONTROL_BEHAVIOR_* (flow, param)
    uint8_t slot;        // index in the resource's full compiled list of this kind (decision rule_slot)
    int32_t max_queue;   // maxQueueingTimeMs
    double count;
    double slope;        // WarmUpController.slope
    int32_t warning_token;
    int32_t max_token;
    int32_t count_div_cold; // (int)count / coldFactor (WarmUpController.coolDownTokens)
    int32_t time_window; // degrade seconds
    int32_t burst;       // param burstCount
    int32_t token_count; // param (int)count
    int64_t duration_sec;// param durationInSec
    int64_t token_count_l; // param (long)count (throttle)
    uint32_t hot_off, hot_n;   // hot items
    uint32_t psid;       // param state id (ParameterMetric maps keyed by rule equality)
    uint32_t pad;
};
static_assert(sizeof(DRule) == 80, "DRule must be 80 B");

struct DHot {
    uint64_t key;
    int32_t count;
    int32_t pad;
};

// controller / breaker state
struct RState {
    int64_t a;   // WarmUp storedTokens      | degrade cut (0/1)
    int64_t b;   // WarmUp lastFilledTime    | degrade passCount
    int64_t c;   // latestPassedTime (RateLimiter, WarmUpRateLimiter) | degrade cut_until
    int64_t d;
};

// param table slot
struct PSlot {
    uint64_t khi;    // 0 = empty; (1<<62)|psid for token buckets; (2<<62)|epoch<<32|res for thread counts
    uint64_t kval;   // parameter value key
    int64_t v0;      // token bucket: last add time / throttle last pass time; thread: count
    int64_t v1;      // token bucket: tokens (int)
};

enum : uint8_t { ST_PASS = 0, ST_PASS_WAIT = 1, ST_BLOCK_FLOW = 2, ST_BLOCK_DEGRADE = 3, ST_BLOCK_PARAM = 4,
                 ST_NO_CHECK = 5, ST_NOT_ENTRY = 0xFF };

struct DevCfg {
    int32_t max_rt;
    int32_t occupy_timeout;
    int32_t max_chain;
    int32_t switch_on;
    uint64_t ptab_mask;
    uint64_t ring_mask;
    uint32_t dbg_flags;  // SG_DEBUG_FLAGS experiment switches (0 in production)
    uint32_t pad;
};

struct Seg {
    uint32_t res;
    uint32_t start;
    uint32_t len;
    uint32_t pad;
};

struct DevState {
    Bkt* sec;
    Bkt* minb;
    NodeInfo* info;
    const Prog* prog;
    const DRule* rules;
    RState* rstate;
    const DHot* hot;
    PSlot* ptab;
    uint8_t* ring;
    unsigned long long* dbg;  // optional per-batch diagnostics (SG_DEBUG=1), else null
};

enum : uint32_t { BF_PRIORITIZED = 1, BF_EXIT_ARGS = 2, BF_PTAB_FULL = 4, BF_BAD_RES = 8 };

} // namespace sg
