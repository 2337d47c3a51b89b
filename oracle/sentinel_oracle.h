/*
 * sentinel_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * A single-threaded, event-time-clocked CPU restatement of the Sentinel
 * statistics-and-rule-check hot path (vvvvvw/Sentinel 1.6.0-SNAPSHOT), written
 * from the Java sources cited in sentinel_oracle.c.  It is the parity checker
 * for the HIP engine and the "port" CPU baseline in bench.py.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product (sentinel_amd/) never links or calls it.
 *
 * Parity status: pinned against the reference's own deterministic known-answer
 * tests, transcribed in tests/test_oracle_known_answers.py.
 * No JVM exists in this image, so outputs of the real reference could not be
 * generated here (see DESIGN.md "Oracle").
 */
#ifndef SENTINEL_ORACLE_H
#define SENTINEL_ORACLE_H

#include "../include/sentinel_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_engine or_engine;

/* ---- engine ------------------------------------------------------------ */
or_engine* or_create(const sg_config* cfg);
void or_destroy(or_engine* e);
int or_register(or_engine* e, const char* name, uint32_t* out_id);
int or_register_many(or_engine* e, const char* const* names, uint32_t n);
int or_load_flow_rules(or_engine* e, const sg_flow_rule* r, uint32_t n, uint32_t* n_loaded);
int or_load_degrade_rules(or_engine* e, const sg_degrade_rule* r, uint32_t n, uint32_t* n_loaded);
int or_load_param_rules(or_engine* e, const sg_param_rule* r, uint32_t n, uint32_t* n_loaded);
/* Compiled rule order of one resource (kind 0 flow, 1 degrade, 2 param):
 * writes the indices (into the last loaded list) in evaluation order. */
int or_rule_order(or_engine* e, uint32_t res, int kind, int32_t* out, int cap);
uint64_t or_param_key(const char* value, const char* class_type);

/* Replay a batch of sg_event records (same contract as sg_submit / sg_submit_ex). */
int or_submit(or_engine* e, const sg_event* ev, uint64_t n, uint32_t* out);
int or_submit_ex(or_engine* e, const sg_event* ev, const sg_event_ext* ext, uint64_t n, const sg_arg* args,
                 uint64_t n_args, uint32_t* out);
/* sg_intern_origin / sg_intern_context: same ids in the same first-intern order */
int or_intern_origin(or_engine* e, const char* origin, uint32_t* out_id);
int or_intern_context(or_engine* e, const char* context, uint32_t* out_id);

/* Rich entry for integration tests: explicit context name / origin and an
 * args array.  arg_kind[i]: 0 = null, 1 = scalar key arg_key[i], 2 = a
 * Collection/array whose element keys are arg_list[i][0..arg_len[i]).
 * Returns the decision; *handle identifies the entry for or_exit_ex. */
uint32_t or_entry_ex(or_engine* e, int64_t now, uint32_t res, int32_t count, int prioritized,
                     const char* context, const char* origin, int nargs, const int32_t* arg_kind,
                     const uint64_t* arg_key, const uint64_t* const* arg_list, const int32_t* arg_len,
                     uint64_t* handle);
int or_exit_ex(or_engine* e, int64_t now, uint64_t handle, int32_t count, int with_args);
int or_trace_ex(or_engine* e, int64_t now, uint64_t handle, int32_t count);

int or_read_node(or_engine* e, uint32_t res, sg_node_state* out);
int or_read_origin_node(or_engine* e, uint32_t res, const char* origin, sg_node_state* out);
int or_read_default_node(or_engine* e, uint32_t res, const char* context, sg_node_state* out);
/* Derived Node getters of the ClusterNode (core/node/StatisticNode.java:159-248).
 * which: 0 passQps 1 blockQps 2 successQps 3 exceptionQps 4 totalQps 5 avgRt
 * 6 minRt 7 previousPassQps 8 previousBlockQps 9 totalException 10 totalPass
 * 11 totalRequest 12 totalSuccess 13 maxSuccessQps 14 occupiedPassQps 15 curThreadNum 16 waiting */
double or_node_metric(or_engine* e, uint32_t res, int64_t now, int which);
int or_snapshot_metrics(or_engine* e, int64_t now, sg_metric_node* out, uint64_t cap, uint64_t* n);
int or_param_thread_count(or_engine* e, uint32_t res, int32_t param_idx, uint64_t key, int64_t* out);
/* test hook: ParameterMetric.getThreadCount mocked (ParamFlowCheckerTest) */
int or_param_set_thread_count(or_engine* e, uint32_t res, int32_t param_idx, uint64_t key, int64_t v);

/* ---- token server -------------------------------------------------------- */
int or_cluster_set_connected_count(or_engine* e, int64_t flow_id, int32_t connected);
int or_cluster_request_tokens(or_engine* e, const sg_token_req* reqs, uint64_t n, sg_token_result* out);
int or_cluster_request_param_tokens(or_engine* e, const sg_param_token_req* reqs, uint64_t n, const uint64_t* values,
                                    uint64_t n_values, sg_token_result* out);

/* ---- unit-level hooks (mocked Node values, as the reference tests do) ---- */
typedef struct or_ctrl or_ctrl;
/* behavior: CONTROL_BEHAVIOR_*; grade used by DefaultController. */
or_ctrl* or_ctrl_new(int behavior, int grade, double count, int warm_up_period_sec, int max_queueing_ms,
                     int cold_factor);
void or_ctrl_free(or_ctrl* c);
/* canPass(node, acquire) with node.passQps()/previousPassQps()/curThreadNum()
 * mocked; returns 1/0; *wait_ms gets the queueing sleep, if any. */
int or_ctrl_can_pass(or_ctrl* c, int64_t now, double pass_qps, double prev_pass_qps, int32_t cur_thread,
                     int32_t acquire, int64_t* wait_ms);
int64_t or_ctrl_state(or_ctrl* c, int which); /* 0 storedTokens 1 lastFilledTime 2 latestPassedTime 3 warningToken 4 maxToken */
double or_ctrl_slope(or_ctrl* c);

typedef struct or_degrade or_degrade;
or_degrade* or_degrade_new(int grade, double count, int time_window_sec);
void or_degrade_free(or_degrade* d);
/* DegradeRule.passCheck with the ClusterNode's avgRt/exceptionQps/successQps/
 * totalQps/totalException mocked. */
int or_degrade_pass_check(or_degrade* d, int64_t now, double avg_rt, double exception_qps, double success_qps,
                          double total_qps, double total_exception);

/* Generic LeapArray<MetricBucket> (kind 0 BucketLeapArray, 1 OccupiableBucketLeapArray,
 * 2 FutureBucketLeapArray) for the data-structure tests. */
typedef struct or_leap or_leap;
or_leap* or_leap_new(int kind, int sample_count, int interval_ms);
void or_leap_free(or_leap* a);
/* currentWindow(t): returns the slot index, -2 for a detached (clock went back) bucket, -1 for t<0;
 * *ws receives the window start. */
int or_leap_current(or_leap* a, int64_t t, int64_t* ws);
int or_leap_add(or_leap* a, int64_t t, int event, int64_t n); /* currentWindow(t).value().add(event,n) */
int64_t or_leap_get(or_leap* a, int slot, int event);          /* bucket counter of a slot */
int or_leap_values_count(or_leap* a, int64_t t);               /* values(t).size() */
int64_t or_leap_values_sum(or_leap* a, int64_t t, int event);  /* sum over values(t) */
int or_leap_previous(or_leap* a, int64_t t, int64_t* ws);      /* getPreviousWindow(t): slot or -1 */
int or_leap_valid_head(or_leap* a, int64_t t, int64_t* ws);    /* getValidHead(t): slot or -1 */
void or_leap_add_waiting(or_leap* a, int64_t t, int64_t n);    /* OccupiableBucketLeapArray.addWaiting */
int64_t or_leap_current_waiting(or_leap* a, int64_t now);      /* OccupiableBucketLeapArray.currentWaiting */

#ifdef __cplusplus
}
#endif
#endif
