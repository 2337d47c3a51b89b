"""Diagnostics: phase cycles of the wide hot-parameter owner k_pq<16> (SG_KPROF build, SG_PROF_BIN=3) on the
bench's C5 shape.  usage: SG_LIB_PATH=sentinel_amd/libsentinel_gpu_kprof.so python tools/pqprobe.py [n_entries] [variant]
"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("SG_DEBUG", "1")
os.environ.setdefault("SG_PROF_BIN", "3")
import numpy as np  # noqa: E402

from sentinel_amd import engine as E  # noqa: E402
from sentinel_amd import tracegen as T  # noqa: E402

n_entries = int(sys.argv[1]) if len(sys.argv) > 1 else 8_000_000
variant = int(sys.argv[2]) if len(sys.argv) > 2 else 0
w = T.Workload(5, seed=T.SEED_BASE + 5, n_entries=n_entries, variant=variant)
eng = E.Engine(max_resources=max(w.n_res, 1 << 10), max_slot_chain_size=0, param_table_log2=28, status_ring_log2=26,
               max_batch_events=1 << 23)
w.install(eng)
ev = w.events
L = E.lib()
L.sgx_debug_counters.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
L.sgx_debug_reset.argtypes = [C.c_void_p]
names = ["rules-pre+reserve", "sort", "probe", "residency", "walks", "commit+evict", "place", "displace",
         "rule->tmap", "tmap", "decisions", "fold", "load"]
B = 1 << 23
for i in range(min(3, (len(ev) + B - 1) // B)):
    L.sgx_debug_reset(eng.h)
    t = time.time()
    eng.submit(ev[i * B:(i + 1) * B])
    tm = eng.timings()
    buf = (C.c_ulonglong * 64)()
    L.sgx_debug_counters(eng.h, buf, 64)
    v = np.array(list(buf), dtype=np.uint64)
    ph = v[8:21].astype(np.float64)
    order = [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 0]
    print("batch %d: wall %.1f ms decide %.2f ms; k_pq<16> segments %d events %d longest %d" %
          (i, (time.time() - t) * 1e3, tm[1], v[24], v[25], v[26]), flush=True)
    tot = ph.sum() or 1.0
    print("  " + ", ".join("%s %.1f%%" % (names[j], 100 * ph[(order[j])] / tot) for j in range(13)))
    print("  total cycles (all blocks) %.3g" % tot)
