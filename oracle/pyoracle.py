"""ctypes binding of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module (it is the parity checker, never the product path).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from sentinel_amd import _abi as A

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile liboracle.so with the committed Makefile (gcc only)."""
    if force or not os.path.exists(_LIB_PATH):
        subprocess.run(["make", "-C", _HERE, "-s"], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB_PATH)
        P = C.c_void_p
        L.or_create.restype = P
        L.or_create.argtypes = [C.POINTER(A.SgConfig)]
        L.or_destroy.argtypes = [P]
        L.or_register.argtypes = [P, C.c_char_p, C.POINTER(C.c_uint32)]
        L.or_register_many.argtypes = [P, C.c_void_p, C.c_uint32]
        L.or_load_flow_rules.argtypes = [P, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]
        L.or_load_degrade_rules.argtypes = [P, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]
        L.or_load_param_rules.argtypes = [P, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]
        L.or_rule_order.argtypes = [P, C.c_uint32, C.c_int, C.POINTER(C.c_int32), C.c_int]
        L.or_param_key.restype = C.c_uint64
        L.or_param_key.argtypes = [C.c_char_p, C.c_char_p]
        L.or_submit.argtypes = [P, C.c_void_p, C.c_uint64, C.c_void_p]
        L.or_submit_ex.argtypes = [P, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p]
        L.or_intern_origin.argtypes = [P, C.c_char_p, C.POINTER(C.c_uint32)]
        L.or_intern_context.argtypes = [P, C.c_char_p, C.POINTER(C.c_uint32)]
        L.or_entry_ex.restype = C.c_uint32
        L.or_entry_ex.argtypes = [P, C.c_int64, C.c_uint32, C.c_int32, C.c_int, C.c_char_p, C.c_char_p, C.c_int,
                                  C.POINTER(C.c_int32), C.POINTER(C.c_uint64), C.POINTER(C.POINTER(C.c_uint64)),
                                  C.POINTER(C.c_int32), C.POINTER(C.c_uint64)]
        L.or_exit_ex.argtypes = [P, C.c_int64, C.c_uint64, C.c_int32, C.c_int]
        L.or_trace_ex.argtypes = [P, C.c_int64, C.c_uint64, C.c_int32]
        L.or_read_node.argtypes = [P, C.c_uint32, C.POINTER(A.SgNodeState)]
        L.or_read_origin_node.argtypes = [P, C.c_uint32, C.c_char_p, C.POINTER(A.SgNodeState)]
        L.or_read_default_node.argtypes = [P, C.c_uint32, C.c_char_p, C.POINTER(A.SgNodeState)]
        L.or_node_metric.restype = C.c_double
        L.or_node_metric.argtypes = [P, C.c_uint32, C.c_int64, C.c_int]
        L.or_snapshot_metrics.argtypes = [P, C.c_int64, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
        L.or_param_thread_count.argtypes = [P, C.c_uint32, C.c_int32, C.c_uint64, C.POINTER(C.c_int64)]
        L.or_param_set_thread_count.argtypes = [P, C.c_uint32, C.c_int32, C.c_uint64, C.c_int64]
        L.or_cluster_set_connected_count.argtypes = [P, C.c_int64, C.c_int32]
        L.or_cluster_request_tokens.argtypes = [P, C.c_void_p, C.c_uint64, C.c_void_p]
        L.or_cluster_request_param_tokens.argtypes = [P, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p]
        L.or_ctrl_new.restype = P
        L.or_ctrl_new.argtypes = [C.c_int, C.c_int, C.c_double, C.c_int, C.c_int, C.c_int]
        L.or_ctrl_free.argtypes = [P]
        L.or_ctrl_can_pass.argtypes = [P, C.c_int64, C.c_double, C.c_double, C.c_int32, C.c_int32,
                                       C.POINTER(C.c_int64)]
        L.or_ctrl_state.restype = C.c_int64
        L.or_ctrl_state.argtypes = [P, C.c_int]
        L.or_ctrl_slope.restype = C.c_double
        L.or_ctrl_slope.argtypes = [P]
        L.or_degrade_new.restype = P
        L.or_degrade_new.argtypes = [C.c_int, C.c_double, C.c_int]
        L.or_degrade_free.argtypes = [P]
        L.or_degrade_pass_check.argtypes = [P, C.c_int64, C.c_double, C.c_double, C.c_double, C.c_double,
                                            C.c_double]
        L.or_leap_new.restype = P
        L.or_leap_new.argtypes = [C.c_int, C.c_int, C.c_int]
        L.or_leap_free.argtypes = [P]
        L.or_leap_current.argtypes = [P, C.c_int64, C.POINTER(C.c_int64)]
        L.or_leap_add.argtypes = [P, C.c_int64, C.c_int, C.c_int64]
        L.or_leap_get.restype = C.c_int64
        L.or_leap_get.argtypes = [P, C.c_int, C.c_int]
        L.or_leap_values_count.argtypes = [P, C.c_int64]
        L.or_leap_values_sum.restype = C.c_int64
        L.or_leap_values_sum.argtypes = [P, C.c_int64, C.c_int]
        L.or_leap_previous.argtypes = [P, C.c_int64, C.POINTER(C.c_int64)]
        L.or_leap_valid_head.argtypes = [P, C.c_int64, C.POINTER(C.c_int64)]
        L.or_leap_add_waiting.argtypes = [P, C.c_int64, C.c_int64]
        L.or_leap_current_waiting.restype = C.c_int64
        L.or_leap_current_waiting.argtypes = [P, C.c_int64]
        L.sg_config_default.argtypes = [C.POINTER(A.SgConfig)]
        _lib = L
    return _lib


def default_config(**kw) -> A.SgConfig:
    cfg = A.SgConfig()
    lib().sg_config_default(C.byref(cfg))
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


def param_key(value, class_type="java.lang.String") -> int:
    return int(lib().or_param_key(None if value is None else str(value).encode(),
                                  None if class_type is None else class_type.encode()))


class Oracle:
    """Event-sequential CPU restatement of the Sentinel hot path."""

    def __init__(self, **cfg):
        self._cfg = default_config(**cfg)
        self.h = lib().or_create(C.byref(self._cfg))
        self.n_events = 0

    def close(self):
        if self.h:
            lib().or_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def register(self, name: str) -> int:
        out = C.c_uint32()
        assert lib().or_register(self.h, name.encode(), C.byref(out)) == 0
        return out.value

    def register_ptrs(self, names_ptr, n: int):
        assert lib().or_register_many(self.h, names_ptr, n) == 0

    def _load(self, fn, rules, struct):
        if isinstance(rules, tuple):
            ptr, n = rules
        else:
            arr = (struct * max(1, len(rules)))(*rules)
            ptr, n = C.cast(arr, C.c_void_p), len(rules)
        out = C.c_uint32()
        assert fn(self.h, ptr, n, C.byref(out)) == 0
        return out.value

    def load_flow_rules(self, rules) -> int:
        return self._load(lib().or_load_flow_rules, rules, A.SgFlowRule)

    def load_degrade_rules(self, rules) -> int:
        return self._load(lib().or_load_degrade_rules, rules, A.SgDegradeRule)

    def load_param_rules(self, rules) -> int:
        return self._load(lib().or_load_param_rules, rules, A.SgParamRule)

    def rule_order(self, res: int, kind: int):
        out = (C.c_int32 * 64)()
        k = lib().or_rule_order(self.h, res, kind, out, 64)
        return list(out[:k])

    def submit(self, events: np.ndarray) -> np.ndarray:
        ev = np.ascontiguousarray(events, dtype=A.EVENT_DTYPE)
        out = np.zeros(len(ev), dtype=np.uint32)
        assert lib().or_submit(self.h, ev.ctypes.data, len(ev), out.ctypes.data) == 0
        self.n_events += len(ev)
        return out

    def submit_ex(self, events: np.ndarray, ext: np.ndarray = None, args: np.ndarray = None) -> np.ndarray:
        ev = np.ascontiguousarray(events, dtype=A.EVENT_DTYPE)
        ex = None if ext is None else np.ascontiguousarray(ext, dtype=A.EXT_DTYPE)
        ar = None if args is None or len(args) == 0 else np.ascontiguousarray(args, dtype=A.ARG_DTYPE)
        out = np.zeros(len(ev), dtype=np.uint32)
        rc = lib().or_submit_ex(self.h, ev.ctypes.data, None if ex is None else ex.ctypes.data, len(ev),
                                None if ar is None else ar.ctypes.data, 0 if ar is None else len(ar), out.ctypes.data)
        assert rc == 0, rc
        self.n_events += len(ev)
        return out

    def intern_origin(self, name: str) -> int:
        out = C.c_uint32()
        assert lib().or_intern_origin(self.h, name.encode(), C.byref(out)) == 0
        return out.value

    def intern_context(self, name: str) -> int:
        out = C.c_uint32()
        assert lib().or_intern_context(self.h, name.encode(), C.byref(out)) == 0
        return out.value

    def entry(self, now, res, count=1, prioritized=False, context=None, origin=None, args=None):
        """args: list of None | int key | list[int] keys (Collection/array value)."""
        args = list(args or [])
        n = len(args)
        kinds = (C.c_int32 * max(1, n))()
        keys = (C.c_uint64 * max(1, n))()
        lists = (C.POINTER(C.c_uint64) * max(1, n))()
        lens = (C.c_int32 * max(1, n))()
        keep = []
        for i, a in enumerate(args):
            if a is None:
                kinds[i] = 0
            elif isinstance(a, (list, tuple)):
                kinds[i] = 2
                arr = (C.c_uint64 * max(1, len(a)))(*[0xFFFFFFFFFFFFFFFF if x is None else x for x in a])
                keep.append(arr)
                lists[i] = C.cast(arr, C.POINTER(C.c_uint64))
                lens[i] = len(a)
            else:
                kinds[i] = 1
                keys[i] = int(a)
        h = C.c_uint64()
        d = lib().or_entry_ex(self.h, int(now), res, count, int(bool(prioritized)),
                              None if context is None else context.encode(),
                              None if origin is None else origin.encode(), n, kinds, keys, lists, lens, C.byref(h))
        return int(d), h.value

    def exit(self, now, handle, count=1, with_args=False):
        return lib().or_exit_ex(self.h, int(now), handle, count, int(bool(with_args)))

    def trace(self, now, handle, count=1):
        return lib().or_trace_ex(self.h, int(now), handle, count)

    def read_node(self, res: int) -> dict:
        st = A.SgNodeState()
        assert lib().or_read_node(self.h, res, C.byref(st)) == 0
        return A.node_state_to_numpy(st)

    def read_origin_node(self, res: int, origin: str):
        st = A.SgNodeState()
        rc = lib().or_read_origin_node(self.h, res, origin.encode(), C.byref(st))
        return None if rc != 0 else A.node_state_to_numpy(st)

    def read_default_node(self, res: int, context: str):
        st = A.SgNodeState()
        rc = lib().or_read_default_node(self.h, res, context.encode(), C.byref(st))
        return None if rc != 0 else A.node_state_to_numpy(st)

    def metric(self, res: int, now: int, which: int) -> float:
        return lib().or_node_metric(self.h, res, int(now), which)

    def snapshot(self, now: int, cap: int = 1 << 16) -> np.ndarray:
        out = np.zeros(cap, dtype=A.METRIC_NODE_DTYPE)
        n = C.c_uint64()
        assert lib().or_snapshot_metrics(self.h, int(now), out.ctypes.data, cap, C.byref(n)) == 0
        return out[: min(cap, n.value)]

    def param_thread_count(self, res, idx, key) -> int:
        out = C.c_int64()
        assert lib().or_param_thread_count(self.h, res, idx, key, C.byref(out)) == 0
        return out.value

    def set_param_thread_count(self, res, idx, key, v):
        assert lib().or_param_set_thread_count(self.h, res, idx, key, v) == 0

    def cluster_set_connected(self, flow_id, n):
        return lib().or_cluster_set_connected_count(self.h, flow_id, n)

    def cluster_request(self, reqs):
        """reqs: list of (ts, flow_id, acquire, prioritized) -> list of (status, remaining, wait)."""
        arr = (A.SgTokenReq * max(1, len(reqs)))()
        for i, (ts, fid, acq, pr) in enumerate(reqs):
            arr[i].ts, arr[i].flow_id, arr[i].acquire_count, arr[i].prioritized = ts, fid, acq, int(pr)
        out = (A.SgTokenResult * max(1, len(reqs)))()
        assert lib().or_cluster_request_tokens(self.h, C.cast(arr, C.c_void_p), len(reqs), C.cast(out, C.c_void_p)) == 0
        return [(out[i].status, out[i].remaining, out[i].wait_in_ms) for i in range(len(reqs))]

    def cluster_request_ptr(self, req_ptr, n, out_ptr):
        """Host buffers: n A.TOKEN_REQ_DTYPE rows at req_ptr -> A.TOKEN_RES_DTYPE rows at out_ptr."""
        assert lib().or_cluster_request_tokens(self.h, C.c_void_p(req_ptr), n, C.c_void_p(out_ptr)) == 0

    def cluster_request_array(self, reqs):
        """reqs: A.TOKEN_REQ_DTYPE array -> A.TOKEN_RES_DTYPE array."""
        reqs = np.ascontiguousarray(reqs, dtype=A.TOKEN_REQ_DTYPE)
        out = np.zeros(max(1, len(reqs)), dtype=A.TOKEN_RES_DTYPE)
        if len(reqs):
            self.cluster_request_ptr(reqs.ctypes.data, len(reqs), out.ctypes.data)
        return out[: len(reqs)]

    def cluster_request_param(self, reqs):
        """reqs: list of (ts, flow_id, acquire, [value keys]) -> list of (status, remaining, wait)."""
        arr, vals = A.param_token_arrays(reqs)
        out = np.zeros(max(1, len(reqs)), dtype=A.TOKEN_RES_DTYPE)
        vp = vals.ctypes.data if len(vals) else None
        assert lib().or_cluster_request_param_tokens(self.h, arr.ctypes.data, len(reqs), vp, len(vals),
                                                     out.ctypes.data) == 0
        return [(int(o["status"]), int(o["remaining"]), int(o["wait_in_ms"])) for o in out[:len(reqs)]]


class PartitionedOracle:
    """``threads`` oracles, resources partitioned by splitmix64(res_id) % threads (SURVEY.md §8(d):
    "N threads partitioned by resource"), each deciding its shard of every batch in its own thread
    (ctypes releases the GIL for the call).  Every decision reads and writes only its own resource's
    state, so the merged decisions equal one oracle's -- tests/test_dist.py checks the routing.
    Used as bench.py's multi-core CPU baseline and to replay large traces in the parity tests."""

    def __init__(self, workload, threads: int, **cfg):
        from concurrent.futures import ThreadPoolExecutor
        from sentinel_amd import dist as D
        self.T = threads
        self.D = D
        self.pool = ThreadPoolExecutor(threads)
        self.router = D.EventRouter(threads, ring_log2=20)
        self.orcs = [Oracle(**cfg) for _ in range(threads)]
        owner = D.shard_of(np.arange(workload.n_res), threads)
        subsets = [np.nonzero(owner == r)[0] for r in range(threads)]
        list(self.pool.map(lambda r: workload.install(self.orcs[r], subsets[r]), range(threads)))
        self.n_events = 0

    def submit(self, events: np.ndarray, timed: list = None) -> np.ndarray:
        """Decisions of one batch; with ``timed``, appends the seconds the threads spent deciding
        (routing excluded)."""
        import time
        parts, pos = self.router.route(np.ascontiguousarray(events, dtype=A.EVENT_DTYPE))
        t = time.perf_counter()
        outs = list(self.pool.map(lambda r: self.orcs[r].submit(parts[r]), range(self.T)))
        if timed is not None:
            timed.append(time.perf_counter() - t)
        out = np.zeros(len(events), dtype=np.uint32)
        for p, o in zip(pos, outs):
            out[p] = o
        self.n_events += len(events)
        return out

    def submit_ex(self, events: np.ndarray, ext: np.ndarray, timed: list = None) -> np.ndarray:
        """sg_submit_ex without an args table (contexts and origins only): each shard gets its events' ext rows."""
        import time
        ev = np.ascontiguousarray(events, dtype=A.EVENT_DTYPE)
        parts, pos = self.router.route(ev)
        exs = [np.ascontiguousarray(ext[p]) for p in pos]
        t = time.perf_counter()
        outs = list(self.pool.map(lambda r: self.orcs[r].submit_ex(parts[r], exs[r]), range(self.T)))
        if timed is not None:
            timed.append(time.perf_counter() - t)
        out = np.zeros(len(events), dtype=np.uint32)
        for p, o in zip(pos, outs):
            out[p] = o
        self.n_events += len(events)
        return out

    def orc_of(self, res: int):
        return self.orcs[int(self.D.shard_of(res, self.T))]

    def read_node(self, res: int) -> dict:
        return self.orcs[int(self.D.shard_of(res, self.T))].read_node(res)

    def close(self):
        for o in self.orcs:
            o.close()
        self.pool.shutdown()


class Controller:
    """A TrafficShapingController driven with mocked Node values."""

    def __init__(self, behavior, count, grade=A.FLOW_GRADE_QPS, warm_up_period_sec=10, max_queueing_ms=500,
                 cold_factor=3):
        self.h = lib().or_ctrl_new(behavior, grade, count, warm_up_period_sec, max_queueing_ms, cold_factor)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_ctrl_free(self.h)
            self.h = None

    def can_pass(self, now, pass_qps=0.0, prev_pass_qps=0.0, cur_thread=0, acquire=1):
        w = C.c_int64()
        ok = lib().or_ctrl_can_pass(self.h, int(now), float(pass_qps), float(prev_pass_qps), cur_thread, acquire,
                                    C.byref(w))
        return bool(ok), w.value

    def state(self, which):
        return lib().or_ctrl_state(self.h, which)

    def slope(self):
        return lib().or_ctrl_slope(self.h)


class Degrade:
    def __init__(self, grade, count, time_window):
        self.h = lib().or_degrade_new(grade, count, time_window)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_degrade_free(self.h)
            self.h = None

    def pass_check(self, now, avg_rt=0.0, exception_qps=0.0, success_qps=0.0, total_qps=0.0, total_exception=0.0):
        return bool(lib().or_degrade_pass_check(self.h, int(now), avg_rt, exception_qps, success_qps, total_qps,
                                                total_exception))


LEAP_PLAIN, LEAP_OCCUPIABLE, LEAP_FUTURE = 0, 1, 2
EV_PASS, EV_BLOCK, EV_EXC, EV_SUCC, EV_RT, EV_OCC = range(6)


class Leap:
    def __init__(self, kind, sample_count, interval_ms):
        self.h = lib().or_leap_new(kind, sample_count, interval_ms)

    def __del__(self):
        if getattr(self, "h", None):
            lib().or_leap_free(self.h)
            self.h = None

    def current(self, t):
        ws = C.c_int64()
        slot = lib().or_leap_current(self.h, int(t), C.byref(ws))
        return slot, ws.value

    def add(self, t, ev, n):
        return lib().or_leap_add(self.h, int(t), ev, n)

    def get(self, slot, ev):
        return lib().or_leap_get(self.h, slot, ev)

    def values_count(self, t):
        return lib().or_leap_values_count(self.h, int(t))

    def values_sum(self, t, ev):
        return lib().or_leap_values_sum(self.h, int(t), ev)

    def previous(self, t):
        ws = C.c_int64()
        slot = lib().or_leap_previous(self.h, int(t), C.byref(ws))
        return slot, ws.value

    def valid_head(self, t):
        ws = C.c_int64()
        slot = lib().or_leap_valid_head(self.h, int(t), C.byref(ws))
        return slot, ws.value

    def add_waiting(self, t, n):
        lib().or_leap_add_waiting(self.h, int(t), n)

    def current_waiting(self, now):
        return lib().or_leap_current_waiting(self.h, int(now))
