"""Python binding of libsentinel_gpu.so (include/sentinel_gpu.h).

The engine is the product: every decision is taken by the HIP kernels behind the
C ABI.  There is no CPU fallback -- if the library or a gfx950 device is missing
this module raises instead of computing anything.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _abi as A

_HERE = os.path.dirname(os.path.abspath(__file__))
# SG_LIB_PATH: diagnostics only (e.g. a -DSG_KPROF build for tools/hotprobe.py)
LIB_PATH = os.environ.get("SG_LIB_PATH") or os.path.join(_HERE, "libsentinel_gpu.so")
_lib = None

# every entry point declared in include/sentinel_gpu.h
EXPORTS = (
    "sg_config_default", "sg_engine_create", "sg_engine_destroy", "sg_register_resources", "sg_resource_id",
    "sg_load_flow_rules", "sg_load_degrade_rules", "sg_load_param_rules", "sg_param_key", "sg_submit",
    "sg_submit_async", "sg_sync", "sg_snapshot_metrics", "sg_cluster_set_connected_count",
    "sg_cluster_request_tokens", "sg_cluster_request_param_tokens", "sg_read_node", "sg_last_error", "sg_last_timings",
    "sg_submit_ex", "sg_submit_ex_async", "sg_intern_origin", "sg_intern_context", "sg_param_thread_count",
)


class SentinelError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"sentinel_gpu error {code}: {msg}")
        self.code = code


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise SentinelError(A.SG_EDEVICE, f"{LIB_PATH} is not built (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.sg_config_default.argtypes = [C.POINTER(A.SgConfig)]
        L.sg_engine_create.argtypes = [C.POINTER(A.SgConfig), C.POINTER(C.c_void_p)]
        L.sg_engine_destroy.argtypes = [P]
        L.sg_register_resources.argtypes = [P, C.POINTER(C.c_char_p), C.c_uint32, C.POINTER(C.c_uint32)]
        L.sg_resource_id.argtypes = [P, C.c_char_p, C.POINTER(C.c_uint32)]
        L.sg_load_flow_rules.argtypes = [P, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]
        L.sg_load_degrade_rules.argtypes = [P, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]
        L.sg_load_param_rules.argtypes = [P, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]
        L.sg_param_key.argtypes = [P, C.c_char_p, C.c_char_p, C.POINTER(C.c_uint64)]
        L.sg_submit.argtypes = [P, C.c_void_p, C.c_uint64, C.c_void_p]
        L.sg_submit_async.argtypes = [P, C.c_void_p, C.c_uint64, C.c_void_p]
        L.sg_sync.argtypes = [P]
        L.sg_submit_ex.argtypes = [P, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p]
        L.sg_submit_ex_async.argtypes = [P, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p]
        L.sg_intern_origin.argtypes = [P, C.c_char_p, C.POINTER(C.c_uint32)]
        L.sg_intern_context.argtypes = [P, C.c_char_p, C.POINTER(C.c_uint32)]
        L.sg_snapshot_metrics.argtypes = [P, C.c_int64, C.c_void_p, C.c_uint64, C.POINTER(C.c_uint64)]
        L.sg_cluster_set_connected_count.argtypes = [P, C.c_int64, C.c_int32]
        L.sg_cluster_request_tokens.argtypes = [P, C.c_void_p, C.c_uint64, C.c_void_p]
        L.sg_cluster_request_param_tokens.argtypes = [P, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p]
        L.sg_read_node.argtypes = [P, C.c_uint32, C.c_int64, C.POINTER(A.SgNodeState)]
        L.sg_last_error.restype = C.c_char_p
        L.sg_last_timings.argtypes = [P, C.POINTER(C.c_double), C.c_int]
        _lib = L
    return _lib


def _check(rc: int):
    if rc != 0:
        raise SentinelError(rc, (lib().sg_last_error() or b"").decode(errors="replace"))


def default_config(**kw) -> A.SgConfig:
    cfg = A.SgConfig()
    lib().sg_config_default(C.byref(cfg))
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


def param_key(value, class_type="java.lang.String") -> int:
    out = C.c_uint64()
    _check(lib().sg_param_key(None, None if value is None else str(value).encode(),
                              None if class_type is None else class_type.encode(), C.byref(out)))
    return out.value


class Engine:
    """One MI355X engine (one shard of resources on one GPU)."""

    def __init__(self, **cfg):
        self._cfg = default_config(**cfg)
        h = C.c_void_p()
        _check(lib().sg_engine_create(C.byref(self._cfg), C.byref(h)))
        self.h = h
        self.n_events = 0

    def close(self):
        if getattr(self, "h", None):
            lib().sg_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- resources / rules
    def register(self, name: str) -> int:
        return self.register_many([name])[0]

    def register_many(self, names) -> np.ndarray:
        arr = (C.c_char_p * max(1, len(names)))(*[n.encode() if isinstance(n, str) else n for n in names])
        out = np.zeros(len(names), dtype=np.uint32)
        _check(lib().sg_register_resources(self.h, arr, len(names), out.ctypes.data_as(C.POINTER(C.c_uint32))))
        return out

    def register_ptrs(self, names_ptr, n: int):
        _check(lib().sg_register_resources(self.h, C.cast(names_ptr, C.POINTER(C.c_char_p)), n, None))

    def resource_id(self, name: str) -> int:
        out = C.c_uint32()
        _check(lib().sg_resource_id(self.h, name.encode(), C.byref(out)))
        return out.value

    def _load(self, fn, rules, struct):
        if isinstance(rules, tuple):  # (pointer, n) straight from tracegen
            ptr, n = rules
        else:
            arr = (struct * max(1, len(rules)))(*rules)
            ptr, n = C.cast(arr, C.c_void_p), len(rules)
        out = C.c_uint32()
        _check(fn(self.h, ptr, n, C.byref(out)))
        return out.value

    def load_flow_rules(self, rules) -> int:
        return self._load(lib().sg_load_flow_rules, rules, A.SgFlowRule)

    def load_degrade_rules(self, rules) -> int:
        return self._load(lib().sg_load_degrade_rules, rules, A.SgDegradeRule)

    def load_param_rules(self, rules) -> int:
        return self._load(lib().sg_load_param_rules, rules, A.SgParamRule)

    # ---- decisions
    def submit(self, events: np.ndarray) -> np.ndarray:
        ev = np.ascontiguousarray(events, dtype=A.EVENT_DTYPE)
        out = np.zeros(len(ev), dtype=np.uint32)
        _check(lib().sg_submit(self.h, ev.ctypes.data, len(ev), out.ctypes.data))
        self.n_events += len(ev)
        return out

    def submit_ex(self, events: np.ndarray, ext: np.ndarray = None, args: np.ndarray = None) -> np.ndarray:
        """sg_submit_ex: ext = A.EXT_DTYPE per event (or None), args = A.ARG_DTYPE table (see A.ext_tables)."""
        ev = np.ascontiguousarray(events, dtype=A.EVENT_DTYPE)
        ex = None if ext is None else np.ascontiguousarray(ext, dtype=A.EXT_DTYPE)
        ar = None if args is None or len(args) == 0 else np.ascontiguousarray(args, dtype=A.ARG_DTYPE)
        out = np.zeros(len(ev), dtype=np.uint32)
        _check(lib().sg_submit_ex(self.h, ev.ctypes.data, None if ex is None else ex.ctypes.data, len(ev),
                                  None if ar is None else ar.ctypes.data, 0 if ar is None else len(ar), out.ctypes.data))
        self.n_events += len(ev)
        return out

    def intern_origin(self, name: str) -> int:
        out = C.c_uint32()
        _check(lib().sg_intern_origin(self.h, name.encode(), C.byref(out)))
        return out.value

    def intern_context(self, name: str) -> int:
        out = C.c_uint32()
        _check(lib().sg_intern_context(self.h, name.encode(), C.byref(out)))
        return out.value

    def submit_ptr(self, ev_ptr: int, n: int, out_ptr: int, sync: bool = True):
        """Device (or host) pointers, e.g. torch tensors' data_ptr()."""
        if sync:
            _check(lib().sg_submit(self.h, C.c_void_p(ev_ptr), n, C.c_void_p(out_ptr)))
        else:
            _check(lib().sg_submit_async(self.h, C.c_void_p(ev_ptr), n, C.c_void_p(out_ptr)))
        self.n_events += n

    def submit_ex_ptr(self, ev_ptr: int, ext_ptr: int, n: int, out_ptr: int, sync: bool = True, args_ptr: int = 0,
                      n_args: int = 0):
        """sg_submit_ex(_async) on device (or host) pointers."""
        fn = lib().sg_submit_ex if sync else lib().sg_submit_ex_async
        _check(fn(self.h, C.c_void_p(ev_ptr), C.c_void_p(ext_ptr) if ext_ptr else None, n,
                  C.c_void_p(args_ptr) if args_ptr else None, n_args, C.c_void_p(out_ptr)))
        self.n_events += n

    def sync(self):
        _check(lib().sg_sync(self.h))

    def timings(self):
        """Device time of the last submit in ms: [group, decide, post, total] (sg_last_timings)."""
        ms = (C.c_double * 4)()
        k = lib().sg_last_timings(self.h, ms, 4)
        return list(ms[:k])

    def timing_log(self, cap: int = 4096) -> np.ndarray:
        """Stage times of every batch decided since the last call, [n, 4] ms (group, decide, post,
        total); diagnostics export sgx_timing_log, drains the pipeline first."""
        buf = (C.c_double * (4 * cap))()
        fn = lib().sgx_timing_log
        fn.restype = C.c_int
        fn.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        k = fn(self.h, buf, cap)
        return np.frombuffer(buf, dtype=np.float64, count=4 * k).reshape(k, 4).copy()

    def spans_total(self) -> int:
        """Frozen span slots the cooperative kernels recorded so far (diagnostics export sgx_spans_total)."""
        fn = lib().sgx_spans_total
        fn.restype = C.c_ulonglong
        fn.argtypes = [C.c_void_p]
        return int(fn(self.h))

    def read_aux_node(self, res: int, kind: int, node_id: int):
        """An origin (kind 0, origin id) / context (kind 1, context id) node of res: second window [2, 8], thread,
        minute pass history [2, 2] ({ws, pass} per second parity); None if absent (diagnostics export
        sgx_read_aux_node)."""
        fn = lib().sgx_read_aux_node
        fn.restype = C.c_int
        fn.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_void_p]
        out = np.zeros(21, dtype=np.int64)
        rc = fn(self.h, res, kind, node_id, out.ctypes.data)
        if rc < 0:
            raise SentinelError(A.SG_EDEVICE, "sgx_read_aux_node failed")
        if rc == 0:
            return None
        return {"second": out[:16].reshape(2, 8), "thread": int(out[16]), "mhist": out[17:21].reshape(2, 2)}

    def pv_last(self) -> dict:
        """The last batch's value-parallel pre pass (diagnostics export sgx_pv_last): pre pass segments,
        accesses, blocked stretches its walk jumped; post pass segments eligible, ops, segments committed."""
        fn = lib().sgx_pv_last
        fn.restype = C.c_int
        fn.argtypes = [C.c_void_p, C.c_void_p]
        out = np.zeros(7, dtype=np.uint64)
        if fn(self.h, out.ctypes.data) != 0:
            raise SentinelError(A.SG_EDEVICE, "sgx_pv_last failed")
        return {"segments": int(out[0]), "accesses": int(out[1]), "ranges": int(out[2]),
                "post_segments": int(out[3]), "post_ops": int(out[4]), "post_done": int(out[5]),
                "walk_max": int(out[6])}

    def param_pool(self) -> dict:
        """The param map bucket pool (diagnostics export sgx_param_pool): size, taken, taken at the last compaction,
        compactions between batches, compactions a batch ran on the device when its growth found the pool short."""
        fn = lib().sgx_param_pool
        fn.restype = C.c_int
        fn.argtypes = [C.c_void_p, C.c_void_p]
        out = np.zeros(5, dtype=np.uint64)
        if fn(self.h, out.ctypes.data) != 0:
            raise SentinelError(A.SG_EDEVICE, "sgx_param_pool failed")
        return {"buckets": int(out[0]), "taken": int(out[1]), "floor": int(out[2]), "compactions": int(out[3]),
                "device_compactions": int(out[4])}

    def param_compact(self):
        """Compact the param map pool now, between batches (diagnostics export sgx_param_compact: the same
        on-device compaction a submit runs once growth took half of the free pool)."""
        fn = lib().sgx_param_compact
        fn.restype = C.c_int
        fn.argtypes = [C.c_void_p]
        if fn(self.h) != 0:
            raise SentinelError(A.SG_EDEVICE, "sgx_param_compact failed")

    def param_thread_count(self, res: int, idx: int, key: int, with_presence: bool = False):
        """ParameterMetric.getThreadCount (sg_param_thread_count): the value's count in the thread-count map of
        paramIdx idx, 0 if absent; with_presence: (count, present).  Does not reorder the map's LRU."""
        fn = lib().sg_param_thread_count
        fn.restype = C.c_int
        fn.argtypes = [C.c_void_p, C.c_uint32, C.c_int32, C.c_uint64, C.POINTER(C.c_int64), C.POINTER(C.c_int32)]
        c, p = C.c_int64(), C.c_int32()
        _check(fn(self.h, res, idx, key, C.byref(c), C.byref(p)))
        return (c.value, bool(p.value)) if with_presence else c.value

    def read_node(self, res: int, now: int = 0) -> dict:
        st = A.SgNodeState()
        _check(lib().sg_read_node(self.h, res, now, C.byref(st)))
        return A.node_state_to_numpy(st)

    def snapshot(self, now: int, cap: int = 1 << 16) -> np.ndarray:
        out = np.zeros(cap, dtype=A.METRIC_NODE_DTYPE)
        n = C.c_uint64()
        _check(lib().sg_snapshot_metrics(self.h, int(now), out.ctypes.data, cap, C.byref(n)))
        return out[: min(cap, n.value)]

    def snapshot_to(self, now: int, out_ptr: int, cap: int) -> int:
        """sg_snapshot_metrics into caller memory (a device pointer stays on the device); returns the
        number of MetricNode rows produced (only min(n, cap) are written)."""
        n = C.c_uint64()
        _check(lib().sg_snapshot_metrics(self.h, int(now), C.c_void_p(out_ptr), cap, C.byref(n)))
        return n.value

    # ---- token server (sg_cluster_*; DefaultTokenService.requestToken, csrv/flow/DefaultTokenService.java:37-48)
    def cluster_set_connected(self, flow_id: int, n: int):
        _check(lib().sg_cluster_set_connected_count(self.h, int(flow_id), int(n)))

    def cluster_request_array(self, reqs: np.ndarray) -> np.ndarray:
        """reqs: A.TOKEN_REQ_DTYPE array (time-ordered) -> A.TOKEN_RES_DTYPE array."""
        reqs = np.ascontiguousarray(reqs, dtype=A.TOKEN_REQ_DTYPE)
        out = np.zeros(len(reqs), dtype=A.TOKEN_RES_DTYPE)
        _check(lib().sg_cluster_request_tokens(self.h, reqs.ctypes.data, len(reqs), out.ctypes.data))
        return out

    def cluster_request_ptr(self, req_ptr: int, n: int, out_ptr: int):
        """Device (or host) buffers: n A.TOKEN_REQ_DTYPE rows at req_ptr -> A.TOKEN_RES_DTYPE rows at out_ptr."""
        _check(lib().sg_cluster_request_tokens(self.h, C.c_void_p(req_ptr), n, C.c_void_p(out_ptr)))

    def cluster_request(self, reqs):
        """reqs: list of (ts, flow_id, acquire, prioritized) -> list of (status, remaining, wait)."""
        arr = np.zeros(len(reqs), dtype=A.TOKEN_REQ_DTYPE)
        for i, (ts, fid, acq, pr) in enumerate(reqs):
            arr[i] = (ts, fid, acq, int(pr))
        out = self.cluster_request_array(arr)
        return [(int(o["status"]), int(o["remaining"]), int(o["wait_in_ms"])) for o in out]

    # ---- TokenService.requestParamToken (csrv/flow/DefaultTokenService.java:50-61)
    def cluster_request_param_array(self, reqs: np.ndarray, values: np.ndarray) -> np.ndarray:
        """reqs: A.PARAM_TOKEN_REQ_DTYPE (time-ordered), values: uint64 keys -> A.TOKEN_RES_DTYPE array."""
        reqs = np.ascontiguousarray(reqs, dtype=A.PARAM_TOKEN_REQ_DTYPE)
        values = np.ascontiguousarray(values, dtype=np.uint64)
        out = np.zeros(len(reqs), dtype=A.TOKEN_RES_DTYPE)
        _check(lib().sg_cluster_request_param_tokens(self.h, reqs.ctypes.data, len(reqs), values.ctypes.data,
                                                     len(values), out.ctypes.data))
        return out

    def cluster_request_param(self, reqs):
        """reqs: list of (ts, flow_id, acquire, [value keys]) -> list of (status, remaining, wait)."""
        arr, vals = A.param_token_arrays(reqs)
        out = self.cluster_request_param_array(arr, vals)
        return [(int(o["status"]), int(o["remaining"]), int(o["wait_in_ms"])) for o in out]
