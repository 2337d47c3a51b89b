"""Diagnostics of the event-driven head owner (head.hip k_head, SG_DEBUG=1): the slowest head segment of a bin's
k_head launches -- its length, chunks, guess-and-verify rounds, bucket folds, cycles (total / in rounds) and rule
count -- on a C3 trace.  usage: SG_PROF_BIN=0|1 python tools/headprobe.py [n_entries] [batches]
"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("SG_DEBUG", "1")
import numpy as np  # noqa: E402

from sentinel_amd import engine as E  # noqa: E402
from sentinel_amd import tracegen as T  # noqa: E402

n_entries = int(sys.argv[1]) if len(sys.argv) > 1 else 8_400_000
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 2
w = T.Workload(3, n_entries=n_entries, variant=int(os.environ.get("SG_VARIANT", "1")))
eng = E.Engine(max_resources=1 << 17, max_slot_chain_size=0, status_ring_log2=26, max_batch_events=1 << 24)
w.install(eng)
ev = w.events
B = min(len(ev) // nb, 1 << 24)
L = E.lib()
L.sgx_debug_counters.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
L.sgx_debug_reset.argtypes = [C.c_void_p]
for i in range(nb):
    L.sgx_debug_reset(eng.h)
    t = time.time()
    eng.submit(ev[i * B:(i + 1) * B])
    tm = eng.timings()
    buf = (C.c_ulonglong * 64)()
    L.sgx_debug_counters(eng.h, buf, 64)
    v = np.array(list(buf), dtype=np.uint64)
    print("batch %d: wall %.1f ms decide %.2f ms | slowest head: len %d chunks %d rounds %d folds %d cycles %d "
          "(owner rounds %d, a decoder %d, statistics %d) count %d" % (i, (time.time() - t) * 1e3, tm[1], v[60], v[61], v[62], v[63],
                                                              v[59], v[30], v[44], v[45], v[31]),
          "| owner phases: warm/tf %d, RL guesses %d, scans+evaluation %d, commit %d" % (v[46], v[47], v[48], v[49]),
          flush=True)
