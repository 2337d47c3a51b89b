"""Diagnostics: per-stage cycle split of the hottest segment in k_decide_spec (SG_DEBUG=1)."""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("SG_DEBUG", "1")
import numpy as np  # noqa: E402

from sentinel_amd import engine as E  # noqa: E402
from sentinel_amd import tracegen as T  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n_entries = int(sys.argv[2]) if len(sys.argv) > 2 else 8_000_000
w = T.Workload(cfg, n_entries=n_entries)
eng = E.Engine(max_resources=1 << 20, max_slot_chain_size=0, param_table_log2=22, status_ring_log2=28,
               max_batch_events=1 << 25)
w.install(eng)
ev = w.events
B = min(len(ev), 1 << 24)
for i in range(2):
    t = time.time()
    d = eng.submit(ev[i * B:(i + 1) * B])
    tm = eng.timings()
    buf = (C.c_ulonglong * 16)()
    E.lib().sgx_debug_counters.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    E.lib().sgx_debug_counters(eng.h, buf, 16)
    v = list(buf)
    names = ["len", "tiles", "rounds", "iters", "load", "ref", "roundsetup", "eval", "tail"]
    print("batch", i, "wall %.1f ms" % ((time.time() - t) * 1e3), "group %.2f decide %.2f ms" % (tm[0], tm[1]))
    print({k: v[j] for j, k in enumerate(names)})
    tot = sum(v[4:9]) or 1
    print({k: "%.1f%%" % (100.0 * v[4 + j] / tot) for j, k in enumerate(names[4:])},
          "cycles/tile %.0f" % (tot / max(1, v[1])), "rounds/tile %.2f" % (v[2] / max(1, v[1])))
