/*
 * sentinel_gpu.h -- C ABI of the MI355X batched decision engine for Sentinel's
 * statistics-and-rule-check hot path.
 *
 * This header is the drop-in boundary.  Everything the Java
 * side needs crosses it as plain pointers, sizes and POD structs; no C++ or
 * torch type appears here.  Each entry point names the reference interface it
 * replaces (paths relative to /root/reference, prefixes as in SURVEY.md §0.1):
 *
 *   core/  = sentinel-core/src/main/java/com/alibaba/csp/sentinel/
 *   param/ = sentinel-extension/sentinel-parameter-flow-control/src/main/java/com/alibaba/csp/sentinel/
 *   csrv/  = sentinel-cluster/sentinel-cluster-server-default/src/main/java/com/alibaba/csp/sentinel/cluster/
 *
 * Threading: one submitting thread per engine.  Every call returns before its
 * buffers may be reused, except sg_submit_async (completion via sg_sync).
 * Errors are returned as negative status codes; sg_last_error() gives the text.
 * No exception ever crosses the ABI (the Java binding turns status codes into
 * BlockException subclasses, core/CtSph.java:157-166).
 */
#ifndef SENTINEL_GPU_H
#define SENTINEL_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SG_ABI_VERSION 1

/* ---- status codes ------------------------------------------------------ */
enum {
    SG_OK = 0,
    SG_EINVAL = -1,     /* bad argument */
    SG_ENOMEM = -2,     /* device or host allocation failed */
    SG_EDEVICE = -3,    /* HIP runtime error / no gfx950 device */
    SG_ESTATE = -4,     /* call out of order (e.g. submit before rules) */
    SG_ENOTSUP = -5,    /* configuration outside what the device path implements */
    SG_ENOTFOUND = -6,  /* unknown resource / flow id */
    SG_ECAPACITY = -7   /* a fixed-capacity table is full */
};

/* ---- rule constants (core/slots/block/RuleConstant.java:26-55) --------- */
enum {
    SG_FLOW_GRADE_THREAD = 0,
    SG_FLOW_GRADE_QPS = 1,
    SG_DEGRADE_GRADE_RT = 0,
    SG_DEGRADE_GRADE_EXCEPTION_RATIO = 1,
    SG_DEGRADE_GRADE_EXCEPTION_COUNT = 2,
    SG_STRATEGY_DIRECT = 0,
    SG_STRATEGY_RELATE = 1,
    SG_STRATEGY_CHAIN = 2,
    SG_CONTROL_BEHAVIOR_DEFAULT = 0,
    SG_CONTROL_BEHAVIOR_WARM_UP = 1,
    SG_CONTROL_BEHAVIOR_RATE_LIMITER = 2,
    SG_CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER = 3,
    /* ClusterRuleConstant (sentinel-core .../cluster/ClusterRuleConstant) */
    SG_CLUSTER_THRESHOLD_AVG_LOCAL = 0,
    SG_CLUSTER_THRESHOLD_GLOBAL = 1
};

/* ---- engine configuration ---------------------------------------------- */
typedef struct sg_config {
    int32_t sample_count;        /* SampleCountProperty.SAMPLE_COUNT = 2 (core/node/SampleCountProperty.java:42) */
    int32_t interval_ms;         /* IntervalProperty.INTERVAL = 1000 (core/node/IntervalProperty.java:41) */
    int32_t statistic_max_rt;    /* Constants.TIME_DROP_VALVE = 4900 (core/Constants.java:62) */
    int32_t cold_factor;         /* ColdFactorProperty.coldFactor = 3 */
    int32_t occupy_timeout_ms;   /* OccupyTimeoutProperty = 500 (core/node/OccupyTimeoutProperty.java:40) */
    int32_t max_slot_chain_size; /* Constants.MAX_SLOT_CHAIN_SIZE = 6000 (core/Constants.java:36); 0 = unbounded */
    int32_t switch_on;           /* Constants.ON (core/Constants.java:67) */
    int32_t device;              /* HIP device ordinal this engine owns */
    uint32_t max_resources;      /* capacity of the resource table (dense ids 0..max-1) */
    uint32_t max_rules;          /* capacity of the compiled rule table (all kinds) */
    uint32_t param_table_log2;   /* cap on the hot-parameter map pool: the bucket slots of every ParameterMetric
                                    CacheMap together (~2x each map's LRU capacity, 32 B a slot) <= 2^log2;
                                    rule loads past it fail SG_ECAPACITY.  Default 28 */
    uint32_t status_ring_log2;   /* entry-status ring for EXIT/TRACE references = 2^log2 events */
    uint32_t max_batch_events;   /* largest n accepted by sg_submit */
    /* token server (csrv/server/config/ServerFlowConfig.java:26-31) */
    int32_t cluster_sample_count;     /* 10 */
    int32_t cluster_interval_ms;      /* 1000 */
    double cluster_exceed_count;      /* 1.0 */
    double cluster_max_occupy_ratio;  /* 1.0 */
    int32_t cluster_max_allowed_qps;  /* GlobalRequestLimiter default 30000 */
    uint32_t aux_node_capacity;       /* origin StatisticNodes + context DefaultNodes kept on the device for the
                                         resources whose flow rules read them (origin / "other" / CHAIN rules);
                                         ~4 KB each, default 65536 */
    int32_t reserved[6];
} sg_config;

/* ---- rules ----------------------------------------------------------------
 * Field meaning and defaults follow the Java beans exactly; strings are
 * NUL-terminated UTF-8 (ASCII hashes like java.lang.String.hashCode). */

/* core/slots/block/flow/FlowRule.java:40-90 + ClusterFlowConfig.java */
typedef struct sg_flow_rule {
    const char* resource;
    const char* limit_app;            /* NULL/""/"default" => "default" */
    const char* ref_resource;         /* RELATE / CHAIN */
    double count;
    int32_t grade;                    /* default QPS */
    int32_t strategy;                 /* default DIRECT */
    int32_t control_behavior;         /* default DEFAULT */
    int32_t warm_up_period_sec;       /* default 10 */
    int32_t max_queueing_time_ms;     /* default 500 */
    int32_t cluster_mode;             /* bool */
    int64_t cluster_flow_id;          /* ClusterFlowConfig.flowId (0 = null) */
    int32_t cluster_threshold_type;   /* default AVG_LOCAL */
    int32_t cluster_fallback_to_local;/* default true */
    int32_t cluster_strategy;         /* default 0 (NORMAL) */
    int32_t cluster_sample_count;     /* default 10 */
    int32_t cluster_window_interval_ms; /* default 1000 */
    int32_t reserved;
} sg_flow_rule;

/* core/slots/block/degrade/DegradeRule.java:60-140 */
typedef struct sg_degrade_rule {
    const char* resource;
    const char* limit_app;
    double count;
    int32_t time_window;              /* seconds */
    int32_t grade;                    /* default RT */
} sg_degrade_rule;

/* param/slots/block/flow/param/ParamFlowItem.java:24-40 */
typedef struct sg_param_item {
    const char* object;               /* value as a string */
    const char* class_type;           /* "int", "java.lang.Long", "java.lang.String", ... */
    int32_t count;                    /* item threshold (Integer; <0 = ignored) */
    int32_t has_count;                /* 0 => Integer null => item ignored */
} sg_param_item;

/* param/slots/block/flow/param/ParamFlowRule.java:40-70 + ParamFlowClusterConfig */
typedef struct sg_param_rule {
    const char* resource;
    const char* limit_app;
    double count;
    int64_t duration_in_sec;          /* default 1 */
    int32_t grade;                    /* default QPS */
    int32_t param_idx;                /* Integer paramIdx (has_param_idx=0 => null => invalid) */
    int32_t has_param_idx;
    int32_t control_behavior;         /* DEFAULT or RATE_LIMITER */
    int32_t max_queueing_time_ms;     /* default 0 */
    int32_t burst_count;              /* default 0 */
    int32_t cluster_mode;
    int32_t n_items;
    const sg_param_item* items;
    int64_t cluster_flow_id;
    int32_t cluster_threshold_type;
    int32_t cluster_fallback_to_local;
    int32_t cluster_sample_count;
    int32_t cluster_window_interval_ms;
} sg_param_rule;

/* ---- events ----------------------------------------------------------------
 * One 24-byte record per SphU.entry / Entry.exit / Tracer.trace, in
 * non-decreasing ts order (ties keep submission order).  ts is the value
 * TimeUtil.currentTimeMillis() had at the event (core/util/TimeUtil.java:49). */
enum {
    SG_EV_ENTRY = 0,  /* SphU.entry(name, type, count, args...)   core/SphU.java:202 */
    SG_EV_EXIT = 1,   /* Entry.exit(count[, args])                core/Entry.java:78-103 */
    SG_EV_TRACE = 2   /* Tracer.trace(t, count)                   core/Tracer.java:47-59 */
};
enum {
    SG_F_PRIORITIZED = 1u << 0, /* SphU.entryWithPriority (ENTRY) */
    SG_F_HAS_ARG = 1u << 1,     /* args = {args[0]}, non-null; aux = its interned 64-bit key (ENTRY; sg_submit_ex
                                   with ext.n_args > 0 takes the args from the table instead) */
    SG_F_EXIT_ARGS = 1u << 2,   /* Entry.exit(count, args): param thread counts are released (EXIT), SURVEY Q14 */
    SG_F_ENTRY_OUT = 1u << 3,   /* EntryType.OUT (ENTRY); informational (SystemSlot is out of scope) */
    SG_F_BLOCKED_UPSTREAM = 1u << 4 /* ENTRY: the caller's SystemSlot / AuthoritySlot threw.  Those slots sit between
                                   ParamFlowSlot and FlowSlot (param/slots/HotParamSlotChainBuilder.java:39-50), so the
                                   param checks still run (and may block first); otherwise the entry is blocked with
                                   SG_BLOCK_UPSTREAM and StatisticSlot counts the block (StatisticSlot.java:97-117) */
};
/* EXIT/TRACE aux: low 48 bits = global index of the ENTRY event this refers
 * to (SG_REF_NONE = the caller asserts the entry passed); EXIT bits 48..63 =
 * raw response time min(exit_ts - entry_ts, 65535) before the TIME_DROP_VALVE clip. */
#define SG_REF_NONE 0xFFFFFFFFFFFFull
#define SG_AUX_EXIT(ref, rt_raw) (((uint64_t)(rt_raw) << 48) | ((uint64_t)(ref) & SG_REF_NONE))

typedef struct sg_event {
    int64_t ts;
    uint32_t res_id;
    uint16_t count;
    uint8_t kind;
    uint8_t flags;
    uint64_t aux;
} sg_event;

/* ---- per-event extension (sg_submit_ex) ---------------------------------------
 * ProcessorSlot.entry(Context, ResourceWrapper, node, count, prioritized, Object... args)
 * (core/slotchain/ProcessorSlot.java:41-50) carries more than an sg_event: the Context -- its
 * name and origin (core/context/Context.java, ContextUtil.enter(name, origin)) -- and every
 * argument.  sg_submit_ex takes one sg_event_ext per event next to the events, and a flat
 * argument table.  An EXIT/TRACE's ext names the origin and context of its ENTRY (the Entry
 * carries its Context); an EXIT's args are those of Entry.exit(count, args). */
enum {
    SG_ARG_NULL = 0,   /* args[i] == null: param rules on index i pass (ParamFlowChecker.java:59-62) */
    SG_ARG_SCALAR = 1, /* key = the interned value (sg_param_key) */
    SG_ARG_LIST = 2    /* a Collection or an array (ParamFlowChecker.java:75-90): its element keys are
                          args_table[key .. key + len), each an SG_ARG_SCALAR / SG_ARG_NULL entry */
};
#define SG_MAX_ARGS 24        /* args per event (and largest paramIdx with a thread-count map + 1) */
#define SG_MAX_CONTEXTS 2000  /* Constants.MAX_CONTEXT_NAME_SIZE (core/Constants.java:35): context ids above it
                                 are ContextUtil's NullContext -- no checks, no statistics (CtSph.java:120-127) */
typedef struct sg_arg {
    uint64_t key;
    uint32_t kind;     /* SG_ARG_* */
    uint32_t len;      /* SG_ARG_LIST: element count */
} sg_arg;

typedef struct sg_event_ext {
    uint32_t origin_id;  /* sg_intern_origin; 0 = "" (no origin) */
    uint32_t context_id; /* sg_intern_context; 0 = sentinel_default_context */
    uint32_t arg_off;    /* args[i] = args_table[arg_off + i], i < n_args */
    uint32_t n_args;     /* <= SG_MAX_ARGS; ENTRY: 0 with SG_F_HAS_ARG = {aux}, 0 without = an empty array */
} sg_event_ext;

/* ---- decisions --------------------------------------------------------------
 * One uint32 per submitted event: status | rule_slot << 8 | wait_ms << 16.
 * rule_slot is the index of the blocking rule inside the resource's compiled
 * rule list of that kind (flow list sorted by FlowRuleComparator, degrade and
 * param lists in java.util.HashSet iteration order). */
enum {
    SG_PASS = 0,          /* entry passed every slot */
    SG_PASS_WAIT = 1,     /* PriorityWaitException: passed after waiting wait_ms (core/slots/block/flow/PriorityWaitException.java) */
    SG_BLOCK_FLOW = 2,    /* FlowException       core/slots/block/flow/FlowSlot.java:154 */
    SG_BLOCK_DEGRADE = 3, /* DegradeException    core/slots/block/degrade/DegradeRuleManager.java:82 */
    SG_BLOCK_PARAM = 4,   /* ParamFlowException  param/slots/block/flow/param/ParamFlowSlot.java:98 */
    SG_NO_CHECK = 5,      /* no slot chain (MAX_SLOT_CHAIN_SIZE), NullContext, or Constants.ON == false */
    SG_BLOCK_UPSTREAM = 6,/* SG_F_BLOCKED_UPSTREAM: SystemBlockException / AuthorityException of the caller's slots */
    SG_NOT_ENTRY = 0xFF   /* EXIT / TRACE record */
};
#define SG_DECISION_STATUS(d) ((d) & 0xFFu)
#define SG_DECISION_RULE(d) (((d) >> 8) & 0xFFu)
#define SG_DECISION_WAIT(d) ((d) >> 16)

/* ---- per-second metric snapshot (core/node/metric/MetricNode.java:30-42) */
typedef struct sg_metric_node {
    int64_t timestamp;
    int64_t pass_qps;
    int64_t block_qps;
    int64_t success_qps;
    int64_t exception_qps;
    int64_t rt;               /* rt / success (integer division) or raw rt when success == 0 */
    int64_t occupied_pass_qps;
    uint32_t res_id;
    uint32_t reserved;
} sg_metric_node;

/* ---- node state read-back (parity tests) ------------------------------- */
typedef struct sg_bucket {
    int64_t window_start;     /* -1 = bucket never created */
    int64_t pass, block, exception, success, rt, occupied_pass;
    int64_t min_rt;
} sg_bucket;

typedef struct sg_node_state {
    sg_bucket second[8];      /* rollingCounterInSecond buckets, slot order (sample_count used) */
    sg_bucket minute[60];     /* rollingCounterInMinute buckets, slot order */
    sg_bucket borrow[8];      /* FutureBucketLeapArray of the second window */
    int32_t cur_thread_num;
    int32_t has_chain;        /* CtSph chainMap membership */
    int64_t reserved[3];
} sg_node_state;

/* ---- token server (csrv/flow/ClusterFlowChecker.java:55-112) ---------- */
typedef struct sg_token_req {
    int64_t ts;
    int64_t flow_id;
    int32_t acquire_count;
    int32_t prioritized;
} sg_token_req;

typedef struct sg_param_token_req { /* ParamFlowRequestData (flowId, count, params) */
    int64_t ts;
    int64_t flow_id;
    int32_t acquire_count;
    uint32_t n_values;
    uint64_t value_off;
} sg_param_token_req;

enum { /* TokenResultStatus (sentinel-core .../cluster/TokenResultStatus.java) */
    SG_TOKEN_BAD_REQUEST = -4,
    SG_TOKEN_TOO_MANY_REQUEST = -2,
    SG_TOKEN_FAIL = -1,
    SG_TOKEN_OK = 0,
    SG_TOKEN_BLOCKED = 1,
    SG_TOKEN_SHOULD_WAIT = 2,
    SG_TOKEN_NO_RULE_EXISTS = 3
};

typedef struct sg_token_result {
    int32_t status;
    int32_t remaining;
    int32_t wait_in_ms;
    int32_t reserved;
} sg_token_result;

typedef struct sg_engine sg_engine;

/* ---- entry points ------------------------------------------------------- */

/* Fill *cfg with the reference defaults listed above. */
void sg_config_default(sg_config* cfg);

/* Create an engine on cfg->device.  Replaces the static state owned by
 * CtSph.chainMap (core/CtSph.java:52), ClusterBuilderSlot.clusterNodeMap
 * (core/slots/clusterbuilder/ClusterBuilderSlot.java:60) and the rule managers. */
int sg_engine_create(const sg_config* cfg, sg_engine** out);
int sg_engine_destroy(sg_engine* e);

/* Resource interning: name -> dense id (idempotent).  Replaces the
 * StringResourceWrapper keyed maps (core/slotchain/ResourceWrapper.java:46-60). */
int sg_register_resources(sg_engine* e, const char* const* names, uint32_t n, uint32_t* out_ids);
int sg_resource_id(sg_engine* e, const char* name, uint32_t* out_id);

/* Rule managers.  Same validation, de-duplication and ordering as
 * FlowRuleManager.loadRules (core/slots/block/flow/FlowRuleManager.java:97-99,
 * FlowRuleUtil.java:89-228), DegradeRuleManager.loadRules
 * (core/slots/block/degrade/DegradeRuleManager.java:112-205) and
 * ParamFlowRuleManager.loadRules (param/.../ParamFlowRuleManager.java:56-166).
 * Loading a list equal to the current one is a no-op (DynamicSentinelProperty
 * .updateValue, core/property/DynamicSentinelProperty.java:49-52); any other
 * list replaces the rules with fresh controller/breaker state.  *n_loaded
 * (optional) receives the number of valid rules kept. */
int sg_load_flow_rules(sg_engine* e, const sg_flow_rule* rules, uint32_t n, uint32_t* n_loaded);
int sg_load_degrade_rules(sg_engine* e, const sg_degrade_rule* rules, uint32_t n, uint32_t* n_loaded);
int sg_load_param_rules(sg_engine* e, const sg_param_rule* rules, uint32_t n, uint32_t* n_loaded);

/* Interns a parameter value exactly as ParamFlowRuleUtil.parseItemValue would
 * type it (param/.../ParamFlowRuleUtil.java:85-121): the key of Integer 1 differs
 * from the key of Long 1 and of String "1".  The Java binding calls this (or an
 * equivalent pure function) for args[0] of every entry. */
int sg_param_key(sg_engine* e, const char* value, const char* class_type, uint64_t* out_key);

/* Decide a batch: the ProcessorSlot chain Statistic -> ParamFlow -> Flow ->
 * Degrade (param/slots/HotParamSlotChainBuilder.java:38-51) for every ENTRY,
 * StatisticSlot.exit (core/slots/statistic/StatisticSlot.java:136-173) for every
 * EXIT and ClusterNode.trace (core/node/ClusterNode.java:99-106) for every TRACE,
 * in event order per resource.  ev and out may be host or device pointers
 * (device pointers avoid the PCIe copy).  sg_submit is synchronous. */
int sg_submit(sg_engine* e, const sg_event* ev, uint64_t n, uint32_t* out);
int sg_submit_async(sg_engine* e, const sg_event* ev, uint64_t n, uint32_t* out);
int sg_sync(sg_engine* e);

/* sg_submit with the Context and the full argument list of every event (see sg_event_ext):
 * origin-specific and `other` flow rules select the origin's StatisticNode, STRATEGY_CHAIN rules the
 * DefaultNode of the entry's context (FlowRuleChecker.selectNodeByRequesterAndStrategy,
 * core/slots/block/flow/FlowRuleChecker.java:90-124); param rules check args[paramIdx] with negative
 * indices resolved on first use and Collection/array values checked element by element
 * (ParamFlowSlot.java:65-101, ParamFlowChecker.java:48-99).  ext may be NULL (= sg_submit); args may be
 * NULL when no ext names any.  All pointers may be host or device memory; sync as sg_submit. */
int sg_submit_ex(sg_engine* e, const sg_event* ev, const sg_event_ext* ext, uint64_t n, const sg_arg* args,
                 uint64_t n_args, uint32_t* out);
int sg_submit_ex_async(sg_engine* e, const sg_event* ev, const sg_event_ext* ext, uint64_t n, const sg_arg* args,
                       uint64_t n_args, uint32_t* out);

/* Context names and origins (ContextUtil.enter(name, origin), core/context/ContextUtil.java:118-166):
 * dense ids, in first-intern order; the name "" interns to origin 0 and "sentinel_default_context"
 * to context 0.  Context ids above SG_MAX_CONTEXTS are NullContexts.  Idempotent. */
int sg_intern_origin(sg_engine* e, const char* origin, uint32_t* out_id);
int sg_intern_context(sg_engine* e, const char* context, uint32_t* out_id);

/* Per-second MetricNode export: StatisticNode.metrics() of every ClusterNode
 * (core/node/StatisticNode.java:124-151, core/node/metric/MetricTimerListener.java:39-71).
 * Writes up to cap nodes, *n receives the number written. */
int sg_snapshot_metrics(sg_engine* e, int64_t now_ms, sg_metric_node* out, uint64_t cap, uint64_t* n);

/* Batched TokenService.requestToken (core/cluster/TokenService.java:26-35,
 * csrv/flow/DefaultTokenService.java:37-48).  Rules come from the flow rules
 * loaded with cluster_mode=1 (the ClusterFlowRuleManager role).  reqs / out may be host or device
 * memory; the call returns when the results are written. */
int sg_cluster_set_connected_count(sg_engine* e, int64_t flow_id, int32_t connected);
int sg_cluster_request_tokens(sg_engine* e, const sg_token_req* reqs, uint64_t n, sg_token_result* out);

/* Batched TokenService.requestParamToken (core/cluster/TokenService.java:37-46,
 * csrv/flow/DefaultTokenService.java:50-61 -> csrv/flow/ClusterParamFlowChecker.java:42-88).
 * Rules come from the param rules loaded with cluster_mode=1 (the ClusterParamFlowRuleManager role,
 * csrv/flow/rule/ClusterParamFlowRuleManager.java:318-369).  Request i names its parameter values
 * as values[value_off, value_off + n_values): interned 64-bit keys (sg_param_key).  Requests are
 * time-ordered and share the namespace's GlobalRequestLimiter with sg_cluster_request_tokens. */
int sg_cluster_request_param_tokens(sg_engine* e, const sg_param_token_req* reqs, uint64_t n, const uint64_t* values,
                                    uint64_t n_values, sg_token_result* out);

/* Node read-back for parity tests: the ClusterNode of res_id. */
int sg_read_node(sg_engine* e, uint32_t res_id, int64_t now_ms, sg_node_state* out);

/* ParameterMetric.getThreadCount(paramIdx, value) of res_id (param/ParameterMetric.java:233-241): the value's
 * thread count in the resource's thread-count map of paramIdx, 0 when the map or the value is absent; *present
 * (optional) tells the two apart.  A read-back: unlike CacheMap.get it does not move the value in the LRU order. */
int sg_param_thread_count(sg_engine* e, uint32_t res_id, int32_t param_idx, uint64_t key, int64_t* count,
                          int32_t* present);

/* Last error message of the calling thread ("" if none). */
const char* sg_last_error(void);

/* Timing of the most recent sg_submit's device stages (HIP events on the engine
 * stream), in ms: [0] group (sort, segments, records, chain grants), [1] decide
 * (every decide kernel, forked over streams and joined), [2] post (decisions back
 * to submission order), [3] their sum; returns the number of values written. */
int sg_last_timings(sg_engine* e, double* ms, int cap);

#ifdef __cplusplus
}
#endif
#endif /* SENTINEL_GPU_H */
