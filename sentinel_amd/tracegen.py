"""Seeded synthetic workloads (C6 = C4 plus a QPS param rule on every resource,
north_star's mixed flow / degrade / param target), generated in C++.

See sentinel_amd/csrc/tracegen.cpp for the trace model.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import _abi as A

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsentinel_trace.so")
_lib = None

SEED_BASE = 20240601  # seed 20240601 + config index

# tg_create variant bits (csrc/tracegen.cpp TG_V_*)
V_WARM_RL = 1   # C3: WarmUpRateLimiter flow rules in the mix
V_HOT = 2       # C5: hot items on every param rule
V_THREAD = 4    # C5: THREAD-grade param rules, exits release their argument (SG_F_EXIT_ARGS)
V_UNIFORM = 8   # C5: half the parameter values uniform (many distinct values: the param maps fill and evict)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            from . import build as _b
            _b.build_trace()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        L.tg_create.restype = P
        L.tg_create.argtypes = [C.c_int, C.c_uint64, C.c_uint32, C.c_uint64, C.c_double, C.c_int64, C.c_uint64,
                                C.c_uint32]
        L.tg_destroy.argtypes = [P]
        L.tg_names.restype = C.c_void_p
        L.tg_names.argtypes = [P, C.POINTER(C.c_uint32)]
        for f in ("tg_flow_rules", "tg_degrade_rules", "tg_param_rules"):
            getattr(L, f).restype = C.c_void_p
            getattr(L, f).argtypes = [P, C.POINTER(C.c_uint32)]
        L.tg_events.restype = C.c_void_p
        L.tg_events.argtypes = [P, C.POINTER(C.c_uint64)]
        L.tg_n_entries.restype = C.c_uint64
        L.tg_n_entries.argtypes = [P]
        L.tg_t_end.restype = C.c_int64
        L.tg_t_end.argtypes = [P]
        _lib = L
    return _lib


class Workload:
    """A generated config: names, rules (as C arrays) and the event trace."""

    def __init__(self, config: int, seed: int | None = None, n_res: int = 0, n_entries: int = 0, rate: float = 0.0,
                 t0: int = 0, n_param_values: int = 0, variant: int = 0):
        self.config = config
        self.seed = SEED_BASE + config if seed is None else seed
        self.variant = variant
        self.h = lib().tg_create(config, self.seed, n_res, n_entries, rate, t0, n_param_values, variant)
        n = C.c_uint32()
        self.names_ptr = lib().tg_names(self.h, C.byref(n))
        self.n_res = n.value
        self.flow = self._rules("tg_flow_rules")
        self.degrade = self._rules("tg_degrade_rules")
        self.param = self._rules("tg_param_rules")
        ne = C.c_uint64()
        ptr = lib().tg_events(self.h, C.byref(ne))
        self.n_events = ne.value
        if ne.value:
            buf = (C.c_char * (ne.value * A.EVENT_DTYPE.itemsize)).from_address(ptr)
            self.events = np.frombuffer(buf, dtype=A.EVENT_DTYPE)
        else:
            self.events = np.zeros(0, dtype=A.EVENT_DTYPE)
        self.n_entries = int(lib().tg_n_entries(self.h))
        self.t_end = int(lib().tg_t_end(self.h))

    def _rules(self, fn):
        n = C.c_uint32()
        ptr = getattr(lib(), fn)(self.h, C.byref(n))
        return (ptr, n.value)

    def names(self):
        arr = C.cast(self.names_ptr, C.POINTER(C.c_char_p))
        return [arr[i].decode() for i in range(self.n_res)]

    _STRUCTS = {"flow": A.SgFlowRule, "degrade": A.SgDegradeRule, "param": A.SgParamRule}

    def install(self, target, res_ids=None):
        """Register names and load the rules into an Engine or an oracle (same calls).  With res_ids,
        every name is still registered (ids stay global) but only the rules of those resources are
        loaded (a resource-partitioned shard)."""
        target.register_ptrs(self.names_ptr, self.n_res)
        for kind, (ptr, n) in (("flow", self.flow), ("degrade", self.degrade), ("param", self.param)):
            if not n:
                continue
            if res_ids is None:
                getattr(target, "load_%s_rules" % kind)((C.c_void_p(ptr), n))
                continue
            sub = self._subset(kind, ptr, n, res_ids)
            getattr(target, "load_%s_rules" % kind)((C.c_void_p(sub.ctypes.data), len(sub)))
            self._keep = getattr(self, "_keep", []) + [sub]

    def _subset(self, kind, ptr, n, res_ids):
        """The rules (raw struct rows, resource-name pointers kept) whose resource is in res_ids."""
        size = C.sizeof(self._STRUCTS[kind])
        raw = np.frombuffer((C.c_char * (n * size)).from_address(ptr), dtype=np.dtype((np.void, size)))
        rptr = np.frombuffer((C.c_char * (n * size)).from_address(ptr), dtype=np.uint64).reshape(n, size // 8)[:, 0]
        names = np.frombuffer((C.c_char * (8 * self.n_res)).from_address(self.names_ptr), dtype=np.uint64)
        order = np.argsort(names)
        k = np.searchsorted(names[order], rptr)
        rid = order[np.minimum(k, self.n_res - 1)]
        if not (names[rid] == rptr).all():
            raise ValueError("a rule names a resource outside the workload's name table")
        keep = np.isin(rid, np.asarray(res_ids))
        return np.ascontiguousarray(raw[keep])

    def intern_names(self, target, n_origins: int = 16, n_contexts: int = 4):
        """Intern the ext workload's origin and context names (ContextUtil.enter(name, origin)) on an Engine or an
        oracle: origins "app-0".., contexts "ctx-0"..; returns their ids (same on every target)."""
        return (np.array([target.intern_origin("app-%d" % k) for k in range(n_origins)], dtype=np.uint32),
                np.array([target.intern_context("ctx-%d" % k) for k in range(n_contexts)], dtype=np.uint32))

    def close(self):
        if getattr(self, "h", None):
            self.events = None
            lib().tg_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def ext_for(events: np.ndarray, origin_ids, context_ids, seed: int) -> np.ndarray:
    """The sg_event_ext of a trace that starts at global index 0 (the drop-in's own input): every
    ENTRY in one of the named contexts, from one of the origins, uniformly; an EXIT / TRACE carries its ENTRY's
    (the Entry keeps its Context).  No args (the C4 rules have none)."""
    n = len(events)
    rng = np.random.default_rng(seed)
    o = rng.integers(0, len(origin_ids), n)
    c = rng.integers(0, len(context_ids), n)
    aux = events["aux"]
    ref = (aux & np.uint64(A.REF_NONE)).astype(np.int64)
    isref = (events["kind"] != A.EV_ENTRY) & (ref != A.REF_NONE) & (ref < n)
    src = np.where(isref, ref, np.arange(n, dtype=np.int64))
    ext = np.zeros(n, dtype=A.EXT_DTYPE)
    ext["origin_id"] = np.asarray(origin_ids, dtype=np.uint32)[o[src]]
    ext["context_id"] = np.asarray(context_ids, dtype=np.uint32)[c[src]]
    return ext
