"""Diagnostics: decide-kernel time of a C4 batch with the K hottest resources removed."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from sentinel_amd import engine as E  # noqa: E402
from sentinel_amd import tracegen as T  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
w = T.Workload(4, n_entries=int(sys.argv[2]) if len(sys.argv) > 2 else 16_400_000)
eng = E.Engine(max_resources=1 << 20, max_slot_chain_size=0, param_table_log2=16, status_ring_log2=28,
               max_batch_events=1 << 25)
w.install(eng)
ev = w.events
cnt = np.bincount(ev["res_id"], minlength=w.n_res)
top = np.argsort(-cnt)[:K]
print("top counts", cnt[top][:8].tolist(), "total", len(ev))
keep = ~np.isin(ev["res_id"], top)
ev2 = np.ascontiguousarray(ev[keep])
# references now point at shifted indices: make every EXIT/TRACE unconditional (ref NONE keeps chain semantics)
nz = ev2["kind"] != 0
ev2["aux"][nz] = (ev2["aux"][nz] & ~np.uint64(0xFFFFFFFFFFFF)) | np.uint64(0xFFFFFFFFFFFF)
B = 1 << 25
for i in range(3):
    part = ev2[i * (B // 2):(i + 1) * (B // 2)]
    if len(part) == 0:
        break
    t = time.time()
    eng.submit(part)
    tm = eng.timings()
    print("batch", i, len(part), "wall %.1f ms group %.3f decide %.3f ms" % ((time.time() - t) * 1e3, tm[0], tm[1]))
