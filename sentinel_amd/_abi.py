"""ctypes/numpy mirrors of the POD types in include/sentinel_gpu.h.

Layouts only -- no behaviour lives here.  Field order and sizes must match the
header; tests/test_abi.py checks the sizes against the compiled library.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

SG_OK = 0
SG_EINVAL = -1
SG_ENOMEM = -2
SG_EDEVICE = -3
SG_ESTATE = -4
SG_ENOTSUP = -5
SG_ENOTFOUND = -6
SG_ECAPACITY = -7

FLOW_GRADE_THREAD = 0
FLOW_GRADE_QPS = 1
DEGRADE_GRADE_RT = 0
DEGRADE_GRADE_EXCEPTION_RATIO = 1
DEGRADE_GRADE_EXCEPTION_COUNT = 2
STRATEGY_DIRECT = 0
STRATEGY_RELATE = 1
STRATEGY_CHAIN = 2
CONTROL_BEHAVIOR_DEFAULT = 0
CONTROL_BEHAVIOR_WARM_UP = 1
CONTROL_BEHAVIOR_RATE_LIMITER = 2
CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER = 3
CLUSTER_THRESHOLD_AVG_LOCAL = 0
CLUSTER_THRESHOLD_GLOBAL = 1

EV_ENTRY = 0
EV_EXIT = 1
EV_TRACE = 2
F_PRIORITIZED = 1 << 0
F_HAS_ARG = 1 << 1
F_EXIT_ARGS = 1 << 2
F_ENTRY_OUT = 1 << 3
F_BLOCKED_UPSTREAM = 1 << 4
REF_NONE = 0xFFFFFFFFFFFF
ARG_NULL, ARG_SCALAR, ARG_LIST = 0, 1, 2
MAX_ARGS = 24
MAX_CONTEXTS = 2000

PASS = 0
PASS_WAIT = 1
BLOCK_FLOW = 2
BLOCK_DEGRADE = 3
BLOCK_PARAM = 4
NO_CHECK = 5
BLOCK_UPSTREAM = 6
NOT_ENTRY = 0xFF

TOKEN_BAD_REQUEST = -4
TOKEN_TOO_MANY_REQUEST = -2
TOKEN_FAIL = -1
TOKEN_OK = 0
TOKEN_BLOCKED = 1
TOKEN_SHOULD_WAIT = 2
TOKEN_NO_RULE_EXISTS = 3


def aux_exit(ref: int, rt_raw: int) -> int:
    return ((min(int(rt_raw), 0xFFFF)) << 48) | (int(ref) & REF_NONE)


def decision_status(d):
    return np.asarray(d) & 0xFF


def decision_rule(d):
    return (np.asarray(d) >> 8) & 0xFF


def decision_wait(d):
    return np.asarray(d) >> 16


class SgConfig(C.Structure):
    _fields_ = [
        ("sample_count", C.c_int32),
        ("interval_ms", C.c_int32),
        ("statistic_max_rt", C.c_int32),
        ("cold_factor", C.c_int32),
        ("occupy_timeout_ms", C.c_int32),
        ("max_slot_chain_size", C.c_int32),
        ("switch_on", C.c_int32),
        ("device", C.c_int32),
        ("max_resources", C.c_uint32),
        ("max_rules", C.c_uint32),
        ("param_table_log2", C.c_uint32),
        ("status_ring_log2", C.c_uint32),
        ("max_batch_events", C.c_uint32),
        ("cluster_sample_count", C.c_int32),
        ("cluster_interval_ms", C.c_int32),
        ("cluster_exceed_count", C.c_double),
        ("cluster_max_occupy_ratio", C.c_double),
        ("cluster_max_allowed_qps", C.c_int32),
        ("aux_node_capacity", C.c_uint32),
        ("reserved", C.c_int32 * 6),
    ]


class SgFlowRule(C.Structure):
    _fields_ = [
        ("resource", C.c_char_p),
        ("limit_app", C.c_char_p),
        ("ref_resource", C.c_char_p),
        ("count", C.c_double),
        ("grade", C.c_int32),
        ("strategy", C.c_int32),
        ("control_behavior", C.c_int32),
        ("warm_up_period_sec", C.c_int32),
        ("max_queueing_time_ms", C.c_int32),
        ("cluster_mode", C.c_int32),
        ("cluster_flow_id", C.c_int64),
        ("cluster_threshold_type", C.c_int32),
        ("cluster_fallback_to_local", C.c_int32),
        ("cluster_strategy", C.c_int32),
        ("cluster_sample_count", C.c_int32),
        ("cluster_window_interval_ms", C.c_int32),
        ("reserved", C.c_int32),
    ]


class SgDegradeRule(C.Structure):
    _fields_ = [
        ("resource", C.c_char_p),
        ("limit_app", C.c_char_p),
        ("count", C.c_double),
        ("time_window", C.c_int32),
        ("grade", C.c_int32),
    ]


class SgParamItem(C.Structure):
    _fields_ = [
        ("object", C.c_char_p),
        ("class_type", C.c_char_p),
        ("count", C.c_int32),
        ("has_count", C.c_int32),
    ]


class SgParamRule(C.Structure):
    _fields_ = [
        ("resource", C.c_char_p),
        ("limit_app", C.c_char_p),
        ("count", C.c_double),
        ("duration_in_sec", C.c_int64),
        ("grade", C.c_int32),
        ("param_idx", C.c_int32),
        ("has_param_idx", C.c_int32),
        ("control_behavior", C.c_int32),
        ("max_queueing_time_ms", C.c_int32),
        ("burst_count", C.c_int32),
        ("cluster_mode", C.c_int32),
        ("n_items", C.c_int32),
        ("items", C.POINTER(SgParamItem)),
        ("cluster_flow_id", C.c_int64),
        ("cluster_threshold_type", C.c_int32),
        ("cluster_fallback_to_local", C.c_int32),
        ("cluster_sample_count", C.c_int32),
        ("cluster_window_interval_ms", C.c_int32),
    ]


class SgBucket(C.Structure):
    _fields_ = [
        ("window_start", C.c_int64),
        ("pass_", C.c_int64),
        ("block", C.c_int64),
        ("exception", C.c_int64),
        ("success", C.c_int64),
        ("rt", C.c_int64),
        ("occupied_pass", C.c_int64),
        ("min_rt", C.c_int64),
    ]


class SgNodeState(C.Structure):
    _fields_ = [
        ("second", SgBucket * 8),
        ("minute", SgBucket * 60),
        ("borrow", SgBucket * 8),
        ("cur_thread_num", C.c_int32),
        ("has_chain", C.c_int32),
        ("reserved", C.c_int64 * 3),
    ]


class SgMetricNode(C.Structure):
    _fields_ = [
        ("timestamp", C.c_int64),
        ("pass_qps", C.c_int64),
        ("block_qps", C.c_int64),
        ("success_qps", C.c_int64),
        ("exception_qps", C.c_int64),
        ("rt", C.c_int64),
        ("occupied_pass_qps", C.c_int64),
        ("res_id", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class SgTokenReq(C.Structure):
    _fields_ = [
        ("ts", C.c_int64),
        ("flow_id", C.c_int64),
        ("acquire_count", C.c_int32),
        ("prioritized", C.c_int32),
    ]


class SgTokenResult(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("remaining", C.c_int32),
        ("wait_in_ms", C.c_int32),
        ("reserved", C.c_int32),
    ]


EVENT_DTYPE = np.dtype(
    [
        ("ts", "<i8"),
        ("res_id", "<u4"),
        ("count", "<u2"),
        ("kind", "u1"),
        ("flags", "u1"),
        ("aux", "<u8"),
    ],
    align=True,
)
assert EVENT_DTYPE.itemsize == 24

EXT_DTYPE = np.dtype([("origin_id", "<u4"), ("context_id", "<u4"), ("arg_off", "<u4"), ("n_args", "<u4")])
ARG_DTYPE = np.dtype([("key", "<u8"), ("kind", "<u4"), ("len", "<u4")])
assert EXT_DTYPE.itemsize == 16 and ARG_DTYPE.itemsize == 16


def ext_tables(n: int, args_of: dict, origin=None, context=None):
    """sg_event_ext rows + the flat sg_arg table for n events.  args_of[i] = list of per-index values:
    None (null), an int key (scalar) or a list/tuple of int keys / None (a Collection/array).
    origin / context: optional length-n arrays of interned ids."""
    ext = np.zeros(n, dtype=EXT_DTYPE)
    if origin is not None:
        ext["origin_id"] = origin
    if context is not None:
        ext["context_id"] = context
    rows = []
    for i in sorted(args_of):
        vals = args_of[i]
        ext["arg_off"][i] = len(rows)
        ext["n_args"][i] = len(vals)
        rows.extend([None] * len(vals))
        base = ext["arg_off"][i]
        for j, v in enumerate(vals):
            if v is None:
                rows[base + j] = (0, ARG_NULL, 0)
            elif isinstance(v, (list, tuple)):
                rows[base + j] = (len(rows), ARG_LIST, len(v))
                rows.extend((0, ARG_NULL, 0) if x is None else (int(x), ARG_SCALAR, 0) for x in v)
            else:
                rows[base + j] = (int(v), ARG_SCALAR, 0)
    table = np.array(rows, dtype=ARG_DTYPE) if rows else np.zeros(0, dtype=ARG_DTYPE)
    return ext, table


METRIC_NODE_DTYPE = np.dtype(
    [
        ("timestamp", "<i8"),
        ("pass_qps", "<i8"),
        ("block_qps", "<i8"),
        ("success_qps", "<i8"),
        ("exception_qps", "<i8"),
        ("rt", "<i8"),
        ("occupied_pass_qps", "<i8"),
        ("res_id", "<u4"),
        ("reserved", "<u4"),
    ],
    align=True,
)

# bucket fields of SgBucket in order, as a numpy view helper
BUCKET_FIELDS = ("window_start", "pass_", "block", "exception", "success", "rt", "occupied_pass", "min_rt")


def node_state_to_numpy(st: SgNodeState) -> dict:
    """Flatten an SgNodeState into int64 arrays: second/minute/borrow [n, 8] + thread."""
    raw = np.frombuffer(bytes(st), dtype=np.int64)
    sec = raw[0:64].reshape(8, 8).copy()
    minute = raw[64:64 + 480].reshape(60, 8).copy()
    borrow = raw[544:608].reshape(8, 8).copy()
    tail = np.frombuffer(bytes(st)[608 * 8:608 * 8 + 8], dtype=np.int32)
    return {"second": sec, "minute": minute, "borrow": borrow, "thread": int(tail[0]), "has_chain": int(tail[1])}


def flow_rule(resource, count, grade=FLOW_GRADE_QPS, limit_app=None, strategy=STRATEGY_DIRECT, ref_resource=None,
              control_behavior=CONTROL_BEHAVIOR_DEFAULT, warm_up_period_sec=10, max_queueing_time_ms=500,
              cluster_mode=False, cluster_flow_id=0, cluster_threshold_type=CLUSTER_THRESHOLD_AVG_LOCAL,
              cluster_fallback_to_local=True, cluster_sample_count=10, cluster_window_interval_ms=1000):
    """A FlowRule with the Java bean defaults (core/slots/block/flow/FlowRule.java:40-90)."""
    r = SgFlowRule()
    r.resource = resource.encode() if isinstance(resource, str) else resource
    r.limit_app = limit_app.encode() if isinstance(limit_app, str) else limit_app
    r.ref_resource = ref_resource.encode() if isinstance(ref_resource, str) else ref_resource
    r.count = float(count)
    r.grade = grade
    r.strategy = strategy
    r.control_behavior = control_behavior
    r.warm_up_period_sec = warm_up_period_sec
    r.max_queueing_time_ms = max_queueing_time_ms
    r.cluster_mode = int(bool(cluster_mode))
    r.cluster_flow_id = cluster_flow_id
    r.cluster_threshold_type = cluster_threshold_type
    r.cluster_fallback_to_local = int(bool(cluster_fallback_to_local))
    r.cluster_strategy = 0
    r.cluster_sample_count = cluster_sample_count
    r.cluster_window_interval_ms = cluster_window_interval_ms
    return r


def degrade_rule(resource, count, time_window, grade=DEGRADE_GRADE_RT, limit_app=None):
    """A DegradeRule (core/slots/block/degrade/DegradeRule.java:60-140)."""
    r = SgDegradeRule()
    r.resource = resource.encode() if isinstance(resource, str) else resource
    r.limit_app = limit_app.encode() if isinstance(limit_app, str) else limit_app
    r.count = float(count)
    r.time_window = time_window
    r.grade = grade
    return r


def param_rule(resource, param_idx, count, grade=FLOW_GRADE_QPS, duration_in_sec=1, burst_count=0,
               control_behavior=CONTROL_BEHAVIOR_DEFAULT, max_queueing_time_ms=0, items=(), limit_app=None,
               cluster_mode=False, cluster_flow_id=0, cluster_fallback_to_local=False,
               cluster_threshold_type=0, cluster_sample_count=10, cluster_window_interval_ms=1000):
    """A ParamFlowRule (param/slots/block/flow/param/ParamFlowRule.java:40-70).

    items: iterable of (object_str, class_type, count) hot items.
    The returned rule keeps a reference to its item array in ``r._items``.
    """
    r = SgParamRule()
    r.resource = resource.encode() if isinstance(resource, str) else resource
    r.limit_app = limit_app.encode() if isinstance(limit_app, str) else limit_app
    r.count = float(count)
    r.duration_in_sec = duration_in_sec
    r.grade = grade
    r.param_idx = 0 if param_idx is None else param_idx
    r.has_param_idx = 0 if param_idx is None else 1
    r.control_behavior = control_behavior
    r.max_queueing_time_ms = max_queueing_time_ms
    r.burst_count = burst_count
    r.cluster_mode = int(bool(cluster_mode))
    items = list(items)
    arr = (SgParamItem * max(1, len(items)))()
    for i, (obj, ct, cnt) in enumerate(items):
        arr[i].object = None if obj is None else str(obj).encode()
        arr[i].class_type = None if ct is None else ct.encode()
        arr[i].count = 0 if cnt is None else int(cnt)
        arr[i].has_count = 0 if cnt is None else 1
    r.n_items = len(items)
    r.items = C.cast(arr, C.POINTER(SgParamItem))
    r._items = arr  # keep alive
    r.cluster_flow_id = cluster_flow_id
    r.cluster_threshold_type = cluster_threshold_type  # ParamFlowClusterConfig default: AVG_LOCAL (0)
    r.cluster_fallback_to_local = int(bool(cluster_fallback_to_local))
    r.cluster_sample_count = cluster_sample_count
    r.cluster_window_interval_ms = cluster_window_interval_ms
    return r


# numpy views of sg_token_req / sg_token_result for bulk calls
TOKEN_REQ_DTYPE = np.dtype([("ts", "<i8"), ("flow_id", "<i8"), ("acquire_count", "<i4"), ("prioritized", "<i4")])
PARAM_TOKEN_REQ_DTYPE = np.dtype([("ts", "<i8"), ("flow_id", "<i8"), ("acquire_count", "<i4"), ("n_values", "<u4"),
                                  ("value_off", "<u8")])
TOKEN_RES_DTYPE = np.dtype([("status", "<i4"), ("remaining", "<i4"), ("wait_in_ms", "<i4"), ("reserved", "<i4")])


def param_token_arrays(reqs):
    """[(ts, flow_id, acquire, [value keys])] -> (PARAM_TOKEN_REQ_DTYPE array, uint64 values)."""
    arr = np.zeros(len(reqs), dtype=PARAM_TOKEN_REQ_DTYPE)
    vals = []
    for i, (ts, fid, acq, vs) in enumerate(reqs):
        arr[i] = (ts, fid, acq, len(vs), len(vals))
        vals += [int(v) for v in vs]
    return arr, np.array(vals, dtype=np.uint64)
