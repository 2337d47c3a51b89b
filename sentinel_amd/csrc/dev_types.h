// dev_types.h -- device-resident state of the MI355X decision engine.
//
// HBM layout (one engine = one GPU = one shard of resources):
//   Bkt     sec[R][2]     rollingCounterInSecond buckets (core/node/StatisticNode.java:102)
//   Bkt     minb[R][60]   rollingCounterInMinute buckets (core/node/StatisticNode.java:111)
//   NodeInfo info[R]      curThreadNum, chain/metric flags, exception running sum
//   Prog    prog[R]       compiled rule program: [param..., flow..., degrade...]
//   DRule   rules[]       compiled rule constants
//   RState  rstate[]      controller / breaker state (one per rule)
//   PMap    pmap[]        ParameterMetric's CacheMaps: one bounded LRU map per (param rule state) and per
//                         (resource, paramIdx) thread-count map, each a private region of
//   PBucket pbkt[]        the cuckoo bucket pool (keys + access stamps), PData pdat[] their values, and
//   uint64  pbm[]         the live-stamp rings (recency order, pmap.h)
//   uint8   ring[2^k]     status of every ENTRY by global event index (EXIT/TRACE references)
// All counters are int64 exactly as the Java LongAdders; RT sums are int64.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/sentinel_gpu.h"

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

#define NO_KEY 0xFFFFFFFFFFFFFFFFull  // key-ring value of an ENTRY without an argument

enum : uint32_t {
    NI_CHAIN = 1u,       // CtSph chainMap holds this resource (and its ClusterNode exists)
    NI_REJECTED = 2u,    // lookProcessChain returned null once the cap was reached
    NI_PM = 4u,          // ParamFlowSlot.metricsMap has a ParameterMetric for it
    NI_TOUCHED = 32u,    // ClusterBuilderSlot created its ClusterNode (an ENTRY with a chain was processed);
                         // kept exact for resources in a STRATEGY_RELATE component (ClusterBuilderSlot.getClusterNode)
    NI_TM_SHIFT = 6u     // bit NI_TM_SHIFT + i: ParameterMetric has a thread-count map for paramIdx i (i < SG_MAX_ARGS)
};
__host__ __device__ inline uint32_t ni_tm(uint32_t idx) { return 1u << (NI_TM_SHIFT + idx); }

// sticky per-resource event marks (DevState.prio), set by the group stage: any mark sends the resource's
// segments to the per-lane kernel
enum : uint8_t {
    PM_PRIO = 1,         // a prioritized ENTRY was seen: the second window's borrow ring is live
    PM_LANE = 2,         // an event only k_lane implements was seen: SG_F_BLOCKED_UPSTREAM, a NullContext, an
                         // origin id >= 2^20 (not packable into the record's node tag)
    PM_AUX = 4,          // an event carried an origin or a named context: the resource keeps its origin
                         // StatisticNodes / context DefaultNodes whatever its rules are.  Rules that read them
                         // (PX_ORIGIN / PX_CHAIN) decide on k_lane<16>; otherwise the segment decides on its usual
                         // owner and aux.hip updates the nodes from the committed verdicts afterwards
    PM_ARGL = 8,         // an event's argument was a Collection / array (per-element checks: not k_pq's; its maps
                         // are grown to full size)
    PM_XARGS = 16        // an EXIT released thread counts with args of its own (sg_submit_ex)
};
// SEv.x of an ENTRY (and of an EXIT / TRACE that names no ENTRY of this batch) in an sg_submit_ex batch: the
// origin / context node tag of the event, origin id | context id << 20 (0: no origin, default context)
#define TAG_ORIGIN_BITS 20u
__host__ __device__ inline uint32_t tag_origin(uint32_t tag) { return tag & ((1u << TAG_ORIGIN_BITS) - 1); }
__host__ __device__ inline uint32_t tag_ctx(uint32_t tag) { return tag >> TAG_ORIGIN_BITS; }
// internal SEv.flags bits above the ABI's SG_F_*
#define RF_OWN_ARGS 0x80u  // EXIT of sg_submit_ex with its own args: its args[0] key is in the key ring at its index
#define RF_PBLK 0x40u      // ENTRY of an XF_MIX segment that a param rule blocked (param.hip k_pq pre pass): its dec[]
                           // word is final; the flow / degrade owner counts it as a block and evaluates nothing

struct NodeInfo {
    int32_t thread;      // StatisticNode.curThreadNum
    uint32_t flags;      // NI_*
    int64_t exc_sum_sec; // second T for which exc_sum = sum of minute exceptions with ws in [T-59000, T]; -1 unknown
    int64_t exc_sum;
    int64_t last_fetch;  // StatisticNode.lastFetchTime (metrics snapshots)
};
static_assert(sizeof(NodeInfo) == 32, "NodeInfo must be 32 B");

// Prog.pflags: what the decide kernels need to know about a resource's rule program
enum : uint8_t {
    PF_EXC_COUNT = 1,   // has an EXCEPTION_COUNT breaker (minute exception running sum)
    PF_WARM = 2,        // has a WarmUp / WarmUpRateLimiter controller
    PF_PQ = 4,          // only QPS-grade param rules with a fixed paramIdx and maps of capacity <= PQ_MAX_CAP: the
                        // cooperative param owner (param.hip k_pq) decides it in batches it is enabled for
    PF_SERIAL = 8,      // outside the cooperative (Jacobi) kernels' limits: per-lane serial kernel only
    PF_RL = 16,         // has a RateLimiter / WarmUpRateLimiter controller
    PF_RT = 32,         // has an RT breaker
    PF_FROZEN = 64,     // every flow stage is a QPS DefaultController: saturated / cut stretches are pure
                        // reductions (decide.hip k_jac frozen stretch)
    PF_J16 = 128        // fits the 1024-lane kernel's shape: <= 2 flow, <= 2 degrade stages, no rate limiter
};

struct Prog {
    uint32_t rule_off;
    uint8_t n_param, n_flow, n_degrade, pflags;
    uint32_t tm_base;    // thread-count maps of this resource: DevState.tmid[tm_base + paramIdx] (NO_ID: none)
    uint16_t multi;      // PX_* bits
    uint16_t xf;         // XF_* bits
};
enum : uint16_t {
    XF_PTHREAD = 1,      // a THREAD-grade param rule is checked (k_pq resolves an EXIT's release against its ENTRY's
                         // check of the same tile by key: an EXIT with its own args (PM_XARGS) is k_lane's)
    XF_MIX = 2,          // param rules beside flow / degrade rules, cooperatively decided: k_pq's
                         // pre pass decides the QPS param checks per value first (nothing before ParamFlowSlot
                         // blocks), the Jacobi owner the flow / degrade chain with those verdicts as inputs, and
                         // k_pq's post pass the thread-count map from the final verdicts
    XF_PLITE = 4,        // XF_MIX with exactly one (checked) param rule: its short segments take k_lite<true>
    XF_PVPQ = 8,         // PF_PQ with one QPS rule (DefaultController or throttle) on paramIdx 0: its long segments'
                         // checks by pvalue.hip's passes, k_pq then folding the statistics only (SG_PV_PQ)
    XF_HEADT = 16,       // the only rule is one THREAD-grade DefaultController flow rule on the ClusterNode (DIRECT,
                         // limitApp default): its J16 / J4 segments take the event-driven head owner (head.hip)
    XF_HEADR = 32        // ... one QPS RateLimiter (or WarmUpRateLimiter of count > 0) flow rule likewise
};
enum : uint32_t {
    PX_MULTI = 1,        // representative of a STRATEGY_RELATE component (its members share one segment)
    PX_ORIGIN = 2,       // a flow rule reads an origin StatisticNode (limitApp = an origin / "other", DIRECT):
                         // the resource keeps its origin nodes (ClusterNode.getOrCreateOriginNode)
    PX_CHAIN = 4         // a STRATEGY_CHAIN rule reads the DefaultNode of its context: the resource keeps the
                         // DefaultNodes of the contexts its CHAIN rules name (NodeSelectorSlot)
};
static_assert(sizeof(Prog) == 16, "Prog must be 16 B");

enum : uint8_t { RK_PARAM = 0, RK_FLOW = 1, RK_DEGRADE = 2 };

// compiled rule (host: engine.cpp upload_rules)
enum : uint32_t { LA_DEFAULT = 0, LA_ORIGIN = 1, LA_OTHER = 2 };  // FlowRule.limitApp kinds
#define NO_ID 0xFFFFFFFFu
struct DRule {
    uint8_t kind;
    uint8_t grade;       // flow/param: FLOW_GRADE_*; degrade: DEGRADE_GRADE_*
    uint8_t behavior;    // CONTROL_BEHAVIOR_* (flow, param); param: PB_INIT_ONLY = initialised, never checked
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
    uint32_t pmap;       // param: its ParameterMetric time/token map (DevState.pmap index; maps are keyed by
                         // rule equality, so an equal rule reloaded keeps its map)
    uint32_t ref;        // flow STRATEGY_RELATE: the resource whose ClusterNode is checked (NO_REF: none)
    int32_t param_idx;   // param: ParamFlowRule.paramIdx as loaded (< 0: resolved on first use, RState.a)
    uint32_t la_kind;    // flow: LA_* of limitApp
    uint32_t la_origin;  // flow: origin id of the limitApp string (NO_ID: never interned)
    uint32_t strategy;   // flow: STRATEGY_*
    uint32_t chain_ctx;  // flow STRATEGY_CHAIN: context id of refResource (NO_ID: never interned)
    uint32_t pad[3];
};
#define NO_REF 0xFFFFFFFFu
#define PB_INIT_ONLY 0xFF
static_assert(sizeof(DRule) == 112, "DRule must be 112 B");

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

// ParameterMetric's CacheMap (ConcurrentLinkedHashMapWrapper, param/.../ParameterMetric.java:37-114): at most
// `cap` entries, least-recently-used evicted on insert.  A rule's ruleTimeCounters and ruleTokenCounter maps
// see the same key sequence (every passDefaultLocalCheck touches both, time first), so they always hold the
// same keys in the same LRU order and share one map here (v0 = time, v1 = tokens).  A map is owned by one
// resource and only its owner (a lane of k_lane, or a k_pq workgroup) touches it.
//
// Representation (pmap.h): recency is a per-map access stamp, not a linked list.  Every access gives the key
// the next stamp (clock++); the live keys are exactly the `live` largest stamps of keys not evicted or erased,
// recorded in a ring bitmap of 2^rb_log2 bits (bit stamp mod 2^rb_log2; every live stamp lies in
// [clock - 2^rb_log2, clock)).  The least recently used key is the lowest set bit at or after `thr`; evicting it
// clears the bit and nothing else (its slot is dead from then on and is reused by inserts).  The recency rank of
// a key -- how many live keys are more recent -- is a popcount over the ring, which is what lets k_pq decide a
// whole tile of accesses at once (LRU residency = fewer than `cap` distinct keys accessed since the key's stamp).
// Keys live in a two-choice bucketed cuckoo table: a bucket is one 128-byte line of 8 keys + their 8 stamps.
#define PM_BKT 8
#define PK_EMPTY 0xFFFFFFFFFFFFFFFFull  // never-used key slot (param keys are type-tagged, never all-ones)
struct PBucket {
    uint64_t key[PM_BKT];
    int64_t stamp[PM_BKT];  // stamp of the key's last access (live iff its ring bit is set, see pmap.h)
};
static_assert(sizeof(PBucket) == 128, "PBucket must be one 128-byte line");
struct PData {
    int64_t v0;      // rule map: last add time / throttle last pass time; thread map: count
    int32_t v1;      // rule map: tokens
    uint32_t pad;
};
static_assert(sizeof(PData) == 16, "PData must be 16 B");
// A map's buckets are a region of one pool: CacheMaps grow with their keys (ConcurrentLinkedHashMap allocates per
// entry), so a region starts at PM_MIN_NB buckets and is moved to a larger one (param.hip k_pm_grow) before a batch
// could put more keys in it than half its slots -- up to map_buckets(cap) (<= 50 % load at capacity).  1M resources
// with a rule each would otherwise reserve 2 x 256 KiB of HBM per resource.
#define PM_MIN_NB 2u
// The pool's control words (engine.cpp d_pool_next, 4 x u64): the next free bucket, the buckets taken at the last
// compaction, the on-device compactions so far, and the epoch of the batch whose growth found the pool short (that
// batch compacts on the device and grows again, param.hip launch_pm_grow)
enum { PC_NEXT = 0, PC_FLOOR = 1, PC_RESCUES = 2, PC_RESCUE = 3, PC_WORDS = 4 };
__host__ __device__ inline uint32_t map_buckets(uint32_t cap) { return (2u * cap + PM_BKT - 1) / PM_BKT > 2u ? (2u * cap + PM_BKT - 1) / PM_BKT : 2u; }
struct PMap {
    uint64_t base;   // first bucket in DevState.pbkt (its slots' data at pdat[base * PM_BKT ...])
    uint64_t bm;     // first word of the live-stamp ring in DevState.pbm (and of the rank scratch in pre)
    int64_t clock;   // next stamp
    int64_t thr;     // <= the lowest live stamp (eviction scans start here)
    uint32_t nb;     // buckets (PM_MIN_NB .. map_buckets(cap))
    uint32_t cap;    // min(4000 * durationInSec, 200000) for rule maps, 4000 for thread-count maps
    uint32_t live;   // keys in the map
    uint32_t rb_log2;// ring bits = 2^rb_log2 >= 4 * cap
    uint32_t pad[4];
};
static_assert(sizeof(PMap) == 64, "PMap must be 64 B");
#define PM_BASE_CAP 4000u      // ParameterMetric.BASE_PARAM_MAX_CAPACITY / THREAD_COUNT_MAX_CAPACITY
#define PM_TOTAL_CAP 200000u   // ParameterMetric.TOTAL_MAX_CAPACITY
#define PQ_MAX_CAP 8176u       // largest map k_pq holds (its live-stamp ring of 2^15 bits in LDS: durationInSec <= 2)

enum : uint8_t { ST_PASS = 0, ST_PASS_WAIT = 1, ST_BLOCK_FLOW = 2, ST_BLOCK_DEGRADE = 3, ST_BLOCK_PARAM = 4,
                 ST_NO_CHECK = 5, ST_BLOCK_UPSTREAM = 6, ST_NOT_ENTRY = 0xFF };

#define HEAD_OFF 16384u  // DevCfg.dbg_flags: the cooperative owner decides XF_HEADT / XF_HEADR heads too (A/B)
struct DevCfg {
    int32_t max_rt;
    int32_t occupy_timeout;
    int32_t max_chain;
    int32_t switch_on;
    uint64_t reserved0;
    uint64_t ring_mask;
    uint32_t dbg_flags;  // SG_DEBUG_FLAGS experiment switches (0 in production)
    uint32_t heads;      // some program is XF_HEADT / XF_HEADR: the head owner (head.hip) runs beside the bins
};

// one resource's events inside a batch: sorted positions [start, start+len)
struct Seg {
    uint32_t res;
    uint32_t start;
    uint32_t len;
    uint32_t bin;    // BIN_* (| SEG_AUXP)
};
#define SEG_AUXP 0x80u  // Seg.bin: the segment's origin / context nodes are updated by the aux.hip post-pass
#define SEG_PV 0x40u    // Seg.bin: pvalue.hip decided the segment's param checks (k_pq's pre pass leaves it)
#define SEG_PVT 0x100u  // Seg.bin: pvalue.hip's post pass updated the thread-count map (k_pq's post pass leaves it)

// pvalue.hip: the value-parallel pre pass of long XF_MIX segments
// per listed segment (the wide XF_MIX list): what the pre pass found
struct PvSeg {
    uint32_t ok;        // decided here (else k_pq's pre / post pass)
    uint32_t n;         // accesses
    uint32_t off;       // first access in the dense arrays
    uint32_t mid;       // rule map (the post pass: the thread-count map of paramIdx 0)
    uint32_t rk;        // the checked rule's index in the program
    uint32_t ch0;       // first extraction chunk
    uint32_t nch;       // extraction chunks
    uint32_t fbits;     // post pass: ParameterMetric bits of the rules the segment's ENTRYs visited
    uint32_t freach;    // post pass: segment position + 1 of the first ENTRY visiting rule k0 (EXITs release from it)
    int32_t peak;       // post pass: the thread-count map's largest growth over its start size
    uint32_t tm0;       // post pass: EXITs release from position 0 (the node had the bits already)
    uint32_t sub;       // post pass: the segment releases thread counts (else increments only: LRU residency)
};

struct PvBuf {          // dense per-access arrays (capacity >= the listed segments' events)
    uint64_t* key;
    uint32_t* pos;      // segment-relative position
    int32_t* dt;
    uint32_t* acq;      // acquire | (token count of the value) << 16 is not enough: tc in its own array
    int32_t* tc;
    uint32_t* seg;      // listed segment index
    uint32_t* gid;      // sort keys (group = hash slot) -> after the sort: sorted keys
    uint32_t* idx;      // sort values -> after the sort: accesses in (group, order) order
    uint32_t* gid2;
    uint32_t* idx2;
    int32_t* prev;      // previous access of the value (dense index), PV_NONE
    int32_t* w;         // first access of a value: its recency rank at the start (PV_INF: absent); others -1
    int32_t* sprev;     // prev sorted per block
    int32_t* sw;        // w sorted per block
    int32_t* fslot;     // first access: the value's slot in the map (any liveness), -1
    uint8_t* hit;
    uint8_t* keep;      // last access of a value: the value stays in the map
    int64_t* flast;     // last access of a value: its final (lastAddTime, tokens)
    int32_t* ftok;
    unsigned long long* htab;  // 2 slots per access: the per-segment hash tables of values
    // extraction chunks (PV_CH positions of one segment each): (listed segment, first position), accesses, offsets
    uint2* chunk;
    uint32_t* ccnt;
    uint32_t* cof;
    // the walk's inputs in sorted order: time, acquire | hit << 16, record index
    int32_t* gdt;
    uint32_t* gaw;
    uint32_t* gpos;
    uint4* range;       // blocked stretches the walk jumped over: {first, end, decision word}; count in tot[2]
};



// ---- token server (cluster.hip): ClusterMetric per flowId + the namespace GlobalRequestLimiter
enum { CF_PASS = 0, CF_BLOCK, CF_PASS_REQ, CF_BLOCK_REQ, CF_OCC_PASS, CF_OCC_BLOCK, CF_WAITING, CF_N };  // ClusterFlowEvent
struct CBkt {          // ClusterMetricBucket in a LeapArray slot; ws < 0: slot never created
    int64_t ws;
    int64_t c[CF_N];
};
struct CFlow {         // one flowId: rule view + ClusterMetricLeapArray bookkeeping
    int64_t flow_id;
    double count;                  // FlowRule.count
    int32_t thr_type;              // ClusterFlowConfig.thresholdType
    int32_t n, interval;           // sampleCount, windowIntervalMs of the metric (fixed at creation)
    int32_t connected;             // ConnectionManager.getConnectedCount (AVG_LOCAL)
    uint32_t boff;                 // first bucket in the bucket array
    uint32_t has_occ;              // ClusterMetricLeapArray.hasOccupied
    int64_t occ_pass, occ_req;     // occupyCounter[PASS], occupyCounter[PASS_REQUEST]
};
struct CSlot {         // flowId -> flow index (open addressing, idx 0xFFFFFFFF = empty)
    int64_t key;
    uint32_t idx, pad;
};
// token server view of a cluster-mode ParamFlowRule + its ClusterParamMetric
// (csrv/flow/statistic/metric/ClusterParamMetric.java:36-91, ClusterParameterLeapArray.java:30-58)
#define CP_MAXN 16      // sampleCount bound of the device window (SG_ENOTSUP above)
struct PFlow {
    int64_t flow_id;
    double count;                  // ParamFlowRule.count
    int32_t thr_type;              // ParamFlowClusterConfig.thresholdType
    int32_t n, interval;           // sampleCount, windowIntervalMs (fixed at creation)
    int32_t connected;             // connected count of the namespace (AVG_LOCAL)
    uint32_t hoff, nhot;           // parsed hot items: PHot[hoff, hoff + nhot)
    int64_t fws[CP_MAXN];          // bucket window starts; < 0: never created
};
struct PHot {
    uint64_t key;
    int32_t count, pad;
};
#define PV_EMPTY 0xFFFFFFFFu
struct PVal {                      // (flow, value) counts; live in bucket j while ws[j] == PFlow.fws[j]
    uint64_t key;
    uint32_t flow, pad;            // flow == PV_EMPTY: free slot (claimed by CAS)
    int64_t ws[CP_MAXN];
    int64_t cnt[CP_MAXN];
};
#define NS_BUCKETS 10   // RequestLimiter: UnaryLeapArray(10, 1000)
#define NS_WLEN 100
#define NS_INTERVAL 1000
struct NsLimiter {
    int64_t ws[NS_BUCKETS];   // < 0: never created
    int64_t cnt[NS_BUCKETS];
};

// Forward links of one ENTRY (k_gather): (epoch << 32) | sorted position of the EXIT / TRACE of the same
// batch whose reference names it.  A tag from another batch means "no link".
struct Link {
    uint64_t exit_l;
    uint64_t trace_l;
};
// A frozen span [s, e) of sorted positions (<= SPAN_CHUNK of them) whose verdicts k_fill writes: every
// ENTRY blocks on the first flow stage its count exceeds at pass count pint, else on the first degrade
// stage when that breaker was cut (res bit 31).
struct Span {
    uint32_t s, e, res;
    int32_t pint;
};
#define SPAN_CHUNK 8192u
#define BST_STATIC 0x80000000u  // bst[] flag: the block holds an EXIT/TRACE that is effective without a link
#define BST_CNT 0x7FFFFFFFu

// Origin StatisticNodes (ClusterNode.originCountMap) and context DefaultNodes (NodeSelectorSlot): one
// open-addressing table of nodes keyed (resource, kind, id), 256 B a node, claimed by CAS on the key.
//
// What a node keeps is what the path can read of it.  Its second window is a full 2 x 500 ms LeapArray (flow
// rules on an origin / context read passQps, threadNum; StatisticSlot updates it).  Of its minute window the
// only reader is WarmUpController's previousPassQps (LeapArray.getPreviousWindow: the pass of the second before
// now, LeapArray.java:216-234) and addOccupiedPass / addPassRequest only add to it, so the node keeps, per
// second parity, the latest second in which pass was added and that second's pass: the previous second's pass
// is found iff it is the latest pass-second of its parity, as a 60-slot ring would give it (the other minute
// fields of an origin / context node are never read: MetricTimerListener exports ClusterNodes only).
struct AuxNode {
    unsigned long long key;  // res << 32 | kind << 31 | id; AUX_EMPTY = free
    int32_t thread;          // curThreadNum
    uint32_t flags;          // AUXF_*
    int64_t mws[2];          // minute window, per second parity: the latest second with pass added (-1: none)
    int64_t mpass[2];        //   and its pass
    int64_t pad0[2];
    Bkt sec[2];              // rollingCounterInSecond
    int64_t borrow[4];       // FutureBucketLeapArray {ws, pass} x 2 (prioritized entries on this node)
    int64_t pad1[4];
};
static_assert(sizeof(AuxNode) == 256, "AuxNode size");
#define AUXF_BORROW 1u       // the node's borrow ring was written (a reset reads it)
#define AUX_EMPTY 0xFFFFFFFFFFFFFFFFull
enum : uint32_t { AUX_ORIGIN = 0, AUX_CONTEXT = 1 };
// the aux.hip post-pass: one node's updates of a batch (or of a piece of a segment), merged per 500 ms bucket
// parity as LeapArray.currentWindow merges them (a later window replaces, the same window adds)
struct AuxAcc {
    uint32_t key;            // kind << 31 | id
    int32_t thread;          // curThreadNum delta
    int64_t W[2];            // second window: latest window start per 500 ms parity (-1: none)
    uint64_t s[2][4];        //   pass, block, succ, rt added at W[p]
    uint32_t minrt[2];       //   min rt at W[p] (0xFFFFFFFF: none)
    int64_t MW[2];           // minute window: latest second with pass added, per second parity (-1: none)
    uint64_t mpass[2];
};
static_assert(sizeof(AuxAcc) == 128, "AuxAcc size");
#define AUX_PIECE 4096u      // aux.hip: events of a long segment per piece workgroup

struct DevState {
    Bkt* sec;
    int64_t* borrow;          // [res][2 slots] x {ws, pass}: FutureBucketLeapArray of the second window
    const uint32_t* prio;     // [res] sticky PM_* marks of the group stage (PM_PRIO: the borrow ring is live)
    uint64_t* key_ring;       // arg key of every ENTRY by global event index (ring like the status ring),
                              // NO_KEY if it had none; null until param rules exist
    uint64_t gbase;           // global index of the batch's first event
    Bkt* minb;
    NodeInfo* info;
    const Prog* prog;
    const DRule* rules;
    RState* rstate;
    const DHot* hot;
    PMap* pmap;               // ParameterMetric maps (see PMap)
    PBucket* pbkt;            // their key/stamp buckets
    PData* pdat;              // their values, one per bucket slot
    uint64_t* pbm;            // their live-stamp rings
    uint32_t* ppre;           // per ring word: rank scratch of a lane-side compaction (pmap.h pm_compact)
    const uint32_t* tmid;     // [Prog.tm_base + paramIdx] -> thread-count map (NO_ID: none)
    uint8_t* ring;
    unsigned long long* dbg;  // optional per-batch diagnostics (SG_DEBUG=1), else null
    uint32_t* sink;           // >= 1024 scratch words: target of masked-off unconditional stores
    // frozen-stretch skipping (decide.hip k_jac<..., SKIP>): side tables of the batch built by k_gather
    const Link* link;         // [sorted pos of an ENTRY] -> the EXIT / TRACE of this batch that references it
    const uint32_t* bst;      // [pos >> 10] ENTRY count sum of the 1024-position block | BST_STATIC
    uint32_t* pend;           // [sorted pos] per-segment list of the owner's committed passes (relative positions)
    Span* spans;              // frozen spans whose verdicts k_fill writes after the decide kernels
    uint32_t* nspan;          // span counter (may exceed span_cap: overflow falls back to streaming)
    uint32_t span_cap;
    uint32_t epoch;           // tag of this batch's links
    uint32_t skip_ok;         // 0: no skipping this batch (links not unique / zero-count ENTRYs / SG_DEBUG_FLAGS & 4)
    uint32_t skip_min;        // a stretch is skipped only if it holds more positions than this (SG_SKIP_MIN)
    // sg_submit_ex: per-event context and args (null: none), origin / context nodes
    const sg_event_ext* ext;  // [submission index]
    const sg_arg* args;
    AuxNode* aux_tab;         // origin / context nodes (open addressing, aux_mask + 1 slots)
    uint32_t* aux_count;      // nodes claimed
    uint32_t aux_cap;
    uint32_t max_ctx;         // context ids above this are NullContexts
    uint64_t aux_mask;
};

enum : uint32_t { BF_PRIORITIZED = 1,
                  BF_PQ_INVARIANT = 2,  // k_pq: a tile's presorted key subset is not what it must be (internal error)
                  BF_PTAB_FULL = 4,     // a param map could not place a key (the map then holds a ghost entry)
                  BF_BAD_RES = 8, BF_BAD_REF = 16,
                  BF_BACKWARD = 32, BF_TSPAN = 64,
                  BF_BAD_ARGS = 512,    // an sg_event_ext names args outside the table, or more than SG_MAX_ARGS
                  BF_AUX_FULL = 1024,   // the origin / context node pool is full
                  BF_POOL_FULL = 2048,  // a param map could not grow: the bucket pool (param_table_log2) is used up
                  BF_MULTI_LINK = 128,  // an ENTRY is referenced by two EXITs (or two TRACEs) of the batch
                  BF_ZERO_CNT = 256,    // an ENTRY acquires 0 (it may pass inside a saturated stretch)
                  BF_TINY_FALLBACK = 4096,  // k_tiny: the batch needs the batched path (nothing decided)
                  BF_TINY_REJECTED = 8192 };  // k_tiny: the batch's checks failed before any decision

// One event in resource-sorted order (16 B), built by k_prep from the caller's 24-byte
// sg_event so that every decide kernel streams its segment with coalesced loads.
struct SEv {
    int32_t dt;      // ts - t0 (t0 = ts of the batch's first event)
    uint32_t x;      // EXIT/TRACE with code RC_BATCH: sorted position of the referenced ENTRY
    uint16_t cnt;    // acquire / exit / trace count
    uint16_t rt;     // EXIT: response time clipped to statistic_max_rt (StatisticSlot.exit)
    uint8_t kind;    // SG_EV_*
    uint8_t flags;   // SG_F_*
    uint8_t code;    // EXIT/TRACE: RC_*
    uint8_t pad;
};
static_assert(sizeof(SEv) == 16, "SEv must be 16 B");
// how an EXIT/TRACE's ENTRY reference resolved
enum : uint8_t {
    RC_NONE = 0,    // no reference (or unknown entry): effective iff the resource has a chain
    RC_BATCH = 1,   // ENTRY earlier in this batch, same resource: effective iff it passed
    RC_PASSED = 2,  // ENTRY of an earlier batch that passed
    RC_NOT = 3,     // ENTRY that did not pass (blocked / no chain), or a TRACE of an unknown entry
    RC_PREV = 4     // ENTRY of an earlier batch, status not read yet (x = status-ring index): resolved to
                    // RC_NONE / RC_PASSED / RC_NOT by k_resolve once the earlier batches are decided
};

// decide-kernel bins of a segment (Seg.pad); order[] is laid out bin by bin
enum : uint32_t {
    BIN_J16 = 0,           // one 1024-lane workgroup per segment (Zipf head)
    BIN_J4 = 1,            // one 256-lane workgroup per segment
    BIN_J1 = 2,            // one wavefront per segment
    BIN_PQ16 = 3,          // PF_PQ segments: one 1024-lane k_pq workgroup (long segments)
    BIN_PQ4 = 4,           //                 one 256-lane k_pq workgroup
    BIN_J8 = 5,            // one 512-lane workgroup per segment: the J16 lengths of QPS-DefaultController programs
    BIN_LANE = 6,          // one lane per segment, nr <= 4: bins 6..6+LANE_BINS-1 by descending log2(len)
    LANE_BINS = 19,
    BIN_LANE16 = BIN_LANE + LANE_BINS,  // one lane per segment, nr > 4 (rule state in scratch)
    BIN_LITE = BIN_LANE16 + LANE_BINS,  // one lane per segment, DefaultController flows + breakers only (k_lite)
    N_BINS = BIN_LITE + LANE_BINS       // <= 63: k_bin_offsets runs one 64-lane wave
};

} // namespace sg
