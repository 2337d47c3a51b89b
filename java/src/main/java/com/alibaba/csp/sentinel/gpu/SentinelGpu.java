package com.alibaba.csp.sentinel.gpu;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemoryLayout;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.StructLayout;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;
import java.nio.file.Path;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_BYTE;
import static java.lang.foreign.ValueLayout.JAVA_DOUBLE;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;
import static java.lang.foreign.ValueLayout.JAVA_SHORT;

/**
 * Panama FFM binding of {@code include/sentinel_gpu.h} (the drop-in boundary, SURVEY.md §8(b)): one
 * downcall handle per export and the layout of every struct that crosses it.  No C glue: the engine
 * library is loaded by path ({@code -Dsentinel.gpu.lib=/path/libsentinel_gpu.so}).
 *
 * <p>The struct layouts below are checked against the C compiler's sizes and offsets
 * (tests/abi_sizes.c) by tests/test_java_sources.py, one member per line.
 */
final class SentinelGpu {

    // ---- status codes, constants (sentinel_gpu.h)
    static final int SG_OK = 0;
    static final int EV_ENTRY = 0, EV_EXIT = 1, EV_TRACE = 2;
    static final int F_PRIORITIZED = 1, F_HAS_ARG = 2, F_EXIT_ARGS = 4, F_ENTRY_OUT = 8, F_BLOCKED_UPSTREAM = 16;
    static final int ARG_NULL = 0, ARG_SCALAR = 1, ARG_LIST = 2;
    static final int MAX_ARGS = 24;
    static final long REF_NONE = 0xFFFFFFFFFFFFL;
    static final int PASS = 0, PASS_WAIT = 1, BLOCK_FLOW = 2, BLOCK_DEGRADE = 3, BLOCK_PARAM = 4, NO_CHECK = 5,
        BLOCK_UPSTREAM = 6;

    // ---- struct layouts (one member per line; see the class comment)
    static final StructLayout SG_CONFIG = MemoryLayout.structLayout(
        JAVA_INT.withName("sample_count"),
        JAVA_INT.withName("interval_ms"),
        JAVA_INT.withName("statistic_max_rt"),
        JAVA_INT.withName("cold_factor"),
        JAVA_INT.withName("occupy_timeout_ms"),
        JAVA_INT.withName("max_slot_chain_size"),
        JAVA_INT.withName("switch_on"),
        JAVA_INT.withName("device"),
        JAVA_INT.withName("max_resources"),
        JAVA_INT.withName("max_rules"),
        JAVA_INT.withName("param_table_log2"),
        JAVA_INT.withName("status_ring_log2"),
        JAVA_INT.withName("max_batch_events"),
        JAVA_INT.withName("cluster_sample_count"),
        JAVA_INT.withName("cluster_interval_ms"),
        MemoryLayout.paddingLayout(4),
        JAVA_DOUBLE.withName("cluster_exceed_count"),
        JAVA_DOUBLE.withName("cluster_max_occupy_ratio"),
        JAVA_INT.withName("cluster_max_allowed_qps"),
        JAVA_INT.withName("aux_node_capacity"),
        MemoryLayout.sequenceLayout(6, JAVA_INT).withName("reserved")
    ).withName("sg_config");

    static final StructLayout SG_FLOW_RULE = MemoryLayout.structLayout(
        ADDRESS.withName("resource"),
        ADDRESS.withName("limit_app"),
        ADDRESS.withName("ref_resource"),
        JAVA_DOUBLE.withName("count"),
        JAVA_INT.withName("grade"),
        JAVA_INT.withName("strategy"),
        JAVA_INT.withName("control_behavior"),
        JAVA_INT.withName("warm_up_period_sec"),
        JAVA_INT.withName("max_queueing_time_ms"),
        JAVA_INT.withName("cluster_mode"),
        JAVA_LONG.withName("cluster_flow_id"),
        JAVA_INT.withName("cluster_threshold_type"),
        JAVA_INT.withName("cluster_fallback_to_local"),
        JAVA_INT.withName("cluster_strategy"),
        JAVA_INT.withName("cluster_sample_count"),
        JAVA_INT.withName("cluster_window_interval_ms"),
        JAVA_INT.withName("reserved")
    ).withName("sg_flow_rule");

    static final StructLayout SG_DEGRADE_RULE = MemoryLayout.structLayout(
        ADDRESS.withName("resource"),
        ADDRESS.withName("limit_app"),
        JAVA_DOUBLE.withName("count"),
        JAVA_INT.withName("time_window"),
        JAVA_INT.withName("grade")
    ).withName("sg_degrade_rule");

    static final StructLayout SG_PARAM_ITEM = MemoryLayout.structLayout(
        ADDRESS.withName("object"),
        ADDRESS.withName("class_type"),
        JAVA_INT.withName("count"),
        JAVA_INT.withName("has_count")
    ).withName("sg_param_item");

    static final StructLayout SG_PARAM_RULE = MemoryLayout.structLayout(
        ADDRESS.withName("resource"),
        ADDRESS.withName("limit_app"),
        JAVA_DOUBLE.withName("count"),
        JAVA_LONG.withName("duration_in_sec"),
        JAVA_INT.withName("grade"),
        JAVA_INT.withName("param_idx"),
        JAVA_INT.withName("has_param_idx"),
        JAVA_INT.withName("control_behavior"),
        JAVA_INT.withName("max_queueing_time_ms"),
        JAVA_INT.withName("burst_count"),
        JAVA_INT.withName("cluster_mode"),
        JAVA_INT.withName("n_items"),
        ADDRESS.withName("items"),
        JAVA_LONG.withName("cluster_flow_id"),
        JAVA_INT.withName("cluster_threshold_type"),
        JAVA_INT.withName("cluster_fallback_to_local"),
        JAVA_INT.withName("cluster_sample_count"),
        JAVA_INT.withName("cluster_window_interval_ms")
    ).withName("sg_param_rule");

    static final StructLayout SG_EVENT = MemoryLayout.structLayout(
        JAVA_LONG.withName("ts"),
        JAVA_INT.withName("res_id"),
        JAVA_SHORT.withName("count"),
        JAVA_BYTE.withName("kind"),
        JAVA_BYTE.withName("flags"),
        JAVA_LONG.withName("aux")
    ).withName("sg_event");

    static final StructLayout SG_EVENT_EXT = MemoryLayout.structLayout(
        JAVA_INT.withName("origin_id"),
        JAVA_INT.withName("context_id"),
        JAVA_INT.withName("arg_off"),
        JAVA_INT.withName("n_args")
    ).withName("sg_event_ext");

    static final StructLayout SG_ARG = MemoryLayout.structLayout(
        JAVA_LONG.withName("key"),
        JAVA_INT.withName("kind"),
        JAVA_INT.withName("len")
    ).withName("sg_arg");

    static final StructLayout SG_METRIC_NODE = MemoryLayout.structLayout(
        JAVA_LONG.withName("timestamp"),
        JAVA_LONG.withName("pass_qps"),
        JAVA_LONG.withName("block_qps"),
        JAVA_LONG.withName("success_qps"),
        JAVA_LONG.withName("exception_qps"),
        JAVA_LONG.withName("rt"),
        JAVA_LONG.withName("occupied_pass_qps"),
        JAVA_INT.withName("res_id"),
        JAVA_INT.withName("reserved")
    ).withName("sg_metric_node");

    static final StructLayout SG_TOKEN_REQ = MemoryLayout.structLayout(
        JAVA_LONG.withName("ts"),
        JAVA_LONG.withName("flow_id"),
        JAVA_INT.withName("acquire_count"),
        JAVA_INT.withName("prioritized")
    ).withName("sg_token_req");

    static final StructLayout SG_TOKEN_RESULT = MemoryLayout.structLayout(
        JAVA_INT.withName("status"),
        JAVA_INT.withName("remaining"),
        JAVA_INT.withName("wait_in_ms"),
        JAVA_INT.withName("reserved")
    ).withName("sg_token_result");

    static final StructLayout SG_PARAM_TOKEN_REQ = MemoryLayout.structLayout(
        JAVA_LONG.withName("ts"),
        JAVA_LONG.withName("flow_id"),
        JAVA_INT.withName("acquire_count"),
        JAVA_INT.withName("n_values"),
        JAVA_LONG.withName("value_off")
    ).withName("sg_param_token_req");

    // ---- downcalls (every export of sentinel_gpu.h)
    private static final Linker LINKER = Linker.nativeLinker();
    private static final SymbolLookup LIB = SymbolLookup.libraryLookup(
        Path.of(System.getProperty("sentinel.gpu.lib", "libsentinel_gpu.so")), Arena.global());

    private static MethodHandle fn(String name, FunctionDescriptor fd) {
        return LINKER.downcallHandle(LIB.find(name).orElseThrow(
            () -> new UnsatisfiedLinkError("sentinel_gpu: missing export " + name)), fd);
    }

    private static FunctionDescriptor rc(MemoryLayout... args) {
        return FunctionDescriptor.of(JAVA_INT, args);
    }

    static final MethodHandle CONFIG_DEFAULT = fn("sg_config_default", FunctionDescriptor.ofVoid(ADDRESS));
    static final MethodHandle ENGINE_CREATE = fn("sg_engine_create", rc(ADDRESS, ADDRESS));
    static final MethodHandle ENGINE_DESTROY = fn("sg_engine_destroy", rc(ADDRESS));
    static final MethodHandle REGISTER_RESOURCES = fn("sg_register_resources", rc(ADDRESS, ADDRESS, JAVA_INT, ADDRESS));
    static final MethodHandle RESOURCE_ID = fn("sg_resource_id", rc(ADDRESS, ADDRESS, ADDRESS));
    static final MethodHandle LOAD_FLOW_RULES = fn("sg_load_flow_rules", rc(ADDRESS, ADDRESS, JAVA_INT, ADDRESS));
    static final MethodHandle LOAD_DEGRADE_RULES = fn("sg_load_degrade_rules", rc(ADDRESS, ADDRESS, JAVA_INT, ADDRESS));
    static final MethodHandle LOAD_PARAM_RULES = fn("sg_load_param_rules", rc(ADDRESS, ADDRESS, JAVA_INT, ADDRESS));
    static final MethodHandle PARAM_KEY = fn("sg_param_key", rc(ADDRESS, ADDRESS, ADDRESS, ADDRESS));
    static final MethodHandle SUBMIT = fn("sg_submit", rc(ADDRESS, ADDRESS, JAVA_LONG, ADDRESS));
    static final MethodHandle SUBMIT_ASYNC = fn("sg_submit_async", rc(ADDRESS, ADDRESS, JAVA_LONG, ADDRESS));
    static final MethodHandle SUBMIT_EX = fn("sg_submit_ex",
        rc(ADDRESS, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS));
    static final MethodHandle SUBMIT_EX_ASYNC = fn("sg_submit_ex_async",
        rc(ADDRESS, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS));
    static final MethodHandle SYNC = fn("sg_sync", rc(ADDRESS));
    static final MethodHandle INTERN_ORIGIN = fn("sg_intern_origin", rc(ADDRESS, ADDRESS, ADDRESS));
    static final MethodHandle INTERN_CONTEXT = fn("sg_intern_context", rc(ADDRESS, ADDRESS, ADDRESS));
    static final MethodHandle SNAPSHOT_METRICS = fn("sg_snapshot_metrics",
        rc(ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS));
    static final MethodHandle CLUSTER_SET_CONNECTED_COUNT = fn("sg_cluster_set_connected_count",
        rc(ADDRESS, JAVA_LONG, JAVA_INT));
    static final MethodHandle CLUSTER_REQUEST_TOKENS = fn("sg_cluster_request_tokens",
        rc(ADDRESS, ADDRESS, JAVA_LONG, ADDRESS));
    static final MethodHandle CLUSTER_REQUEST_PARAM_TOKENS = fn("sg_cluster_request_param_tokens",
        rc(ADDRESS, ADDRESS, JAVA_LONG, ADDRESS, JAVA_LONG, ADDRESS));
    static final MethodHandle READ_NODE = fn("sg_read_node", rc(ADDRESS, JAVA_INT, JAVA_LONG, ADDRESS));
    /** ParameterMetric.getThreadCount(paramIdx, value): (engine, res, paramIdx, key, long* count, int* present). */
    static final MethodHandle PARAM_THREAD_COUNT =
        fn("sg_param_thread_count", rc(ADDRESS, JAVA_INT, JAVA_INT, JAVA_LONG, ADDRESS, ADDRESS));
    static final MethodHandle LAST_ERROR = fn("sg_last_error", FunctionDescriptor.of(ADDRESS));
    static final MethodHandle LAST_TIMINGS = fn("sg_last_timings", rc(ADDRESS, ADDRESS, JAVA_INT));

    private SentinelGpu() {}

    /** A negative status becomes an exception carrying sg_last_error(); no exception crosses the ABI. */
    static void check(int rc) {
        if (rc == SG_OK) {
            return;
        }
        String msg;
        try {
            MemorySegment m = ((MemorySegment) LAST_ERROR.invokeExact()).reinterpret(4096);
            msg = m.getString(0);
        } catch (Throwable t) {
            msg = "(sg_last_error unavailable: " + t + ")";
        }
        throw new IllegalStateException("sentinel_gpu error " + rc + ": " + msg);
    }

    /** Decision word fields (SG_DECISION_STATUS / RULE / WAIT). */
    static int status(int d) {
        return d & 0xFF;
    }

    static int ruleSlot(int d) {
        return (d >>> 8) & 0xFF;
    }

    static int waitMs(int d) {
        return d >>> 16;
    }

    /** SG_AUX_EXIT(ref, rt_raw). */
    static long auxExit(long ref, long rtRaw) {
        return (Math.min(Math.max(rtRaw, 0L), 0xFFFFL) << 48) | (ref & REF_NONE);
    }
}
