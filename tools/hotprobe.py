"""Diagnostics: counters of one cooperative bin (SG_DEBUG=1; SG_PROF_BIN = 0 J16, 1 J4, 2 J1) on a C4 batch
(or another config; SG_VARIANT: tracegen variant bits).

usage: python tools/hotprobe.py [config] [n_entries] [batches] [R/N shard]
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

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n_entries = int(sys.argv[2]) if len(sys.argv) > 2 else 16_400_000
nb = int(sys.argv[3]) if len(sys.argv) > 3 else 2
shard = tuple(int(x) for x in sys.argv[4].split("/")) if len(sys.argv) > 4 else None  # R/N: one rank's shard
t = time.time()
variant = int(os.environ.get("SG_VARIANT", "0"))  # tracegen variant bits (C3: 1 = WarmUpRateLimiter in the mix)
w = T.Workload(cfg, n_entries=n_entries, n_res=1_000_000 if cfg == 4 else 0, variant=variant)
print("generated %d events in %.1f s" % (w.n_events, time.time() - t), flush=True)
eng = E.Engine(max_resources=1 << 20, max_slot_chain_size=0, param_table_log2=22, status_ring_log2=28,
               max_batch_events=1 << 25)
w.install(eng)
ev = w.events
if shard:
    from sentinel_amd import dist as D
    ev, _ = D.shard_stream(ev, shard[1], shard[0])
    print("shard %d/%d: %d events" % (shard[0], shard[1], len(ev)), flush=True)
B = min(len(ev) // nb, 1 << 25)
L = E.lib()
L.sgx_debug_counters.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
L.sgx_debug_reset.argtypes = [C.c_void_p]
prev = np.zeros(64, dtype=np.uint64)
for i in range(nb):
    print("submit batch", i, flush=True)
    t = time.time()
    L.sgx_debug_reset(eng.h)
    eng.submit(ev[i * B:(i + 1) * B])
    tm = eng.timings()
    buf = (C.c_ulonglong * 64)()
    L.sgx_debug_counters(eng.h, buf, 64)
    v = np.array(list(buf), dtype=np.uint64)
    d = v
    print("batch %d: %d events, wall %.1f ms, group %.2f ms, decide %.2f ms" % (i, B, (time.time() - t) * 1e3, tm[0], tm[1]))
    print("  bin %s: segs %d iterations %d rounds %d tiles %d mismatched-iterations %d" % (os.environ.get("SG_PROF_BIN", "0"), d[4], d[0], d[1], d[2], d[3]))
    ph = v[8:18].astype(np.float64)
    tot = ph.sum() or 1
    names = ["top", "phaseB", "B2wait", "evalC", "commitD", "B1wait", "round_setup", "frozen_stretch", "frozen_reduce", "unused"]
    print("  slowest segment (len %d, %d rounds, %d cycles) phase cycles:" % (v[5], v[19], v[18]),
          {k: "%.0f" % ph[j] for j, k in enumerate(names)})
    mph = v[52:56].astype(np.float64)
    print("  slowest segment's round machine: open steps %d, frozen steps %d, round transitions %d; cycles" % (v[56], v[57], v[58]),
          {k: "%.0f" % mph[j] for j, k in enumerate(["open", "frozen", "round_next", "exit"])})
    print("  slowest: iterations %d mismatched %d frozen-tiles %d open-chunks %d prog %#x flow count %d "
          "first flow behaviour|grade<<8 %#x" % (v[23], v[24], v[27], v[29], v[25], v[26], v[28]))
    print("  open-stretch chunks (all segments of the bin): %d" % d[7])
    mm = d[40:49].reshape(3, 3)
    print("  mismatch (guess row: pass/flow/degrade -> evaluated col):", mm.tolist(), "not-first", d[49], "sum(f-c0)", d[50])
    print("  J16 block starts spread %d cycles, first start -> last end %d cycles" % (v[21] - v[20], v[22] - v[20]))
    print("  frozen tiles (all J16 segments):", d[6])
    if d[36]:
        print("  lane kernel longest segment: len %d, cycles start %d entries %d exits %d end %d (per event %.0f)" %
              (d[35], d[32], d[33], d[34], d[37], (d[32] + d[33] + d[34]) / max(1, d[35])))
        print("    entry split: flow %d degrade %d stat_entry %d after %d" % (d[38], d[39], d[51], d[33]))
