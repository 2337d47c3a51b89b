"""Profiling driver: C4 (or C5) batches through sg_submit_ex with contexts / origins (bench.py's C4-ext / C5-ext
sub-lines, without the rest of bench.py), or C6 (mixed rules, sg_submit), for rocprofv3 --kernel-trace --stats."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from sentinel_amd import engine as E, tracegen as T  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "c4ext"
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda", 0)
torch.zeros(1, device=dev)
GB = 1 << 25
if which.startswith("c4"):
    w, ev = bench.make_trace(1_000_000, GB, nb, T.SEED_BASE + 4)
    eng = E.Engine(max_resources=1 << 20, max_slot_chain_size=0, param_table_log2=16, status_ring_log2=28,
                   max_batch_events=GB, aux_node_capacity=1 << 24)
    w.install(eng)
    ext = None
    if which == "c4ext":
        io, ic = w.intern_names(eng)
        ext = T.ext_for(ev, io, ic, seed=T.SEED_BASE + 44)
    t = time.time()
    r = bench.run_batches(eng, ev, GB, dev, ext=ext)
elif which == "c6":
    w = T.Workload(6, seed=T.SEED_BASE + 6, n_entries=int(nb * GB / 2.05) + 1000)
    ev = w.events[:nb * GB]
    eng = E.Engine(max_resources=1 << 20, max_slot_chain_size=0, param_table_log2=29, status_ring_log2=28,
                   max_batch_events=GB, max_rules=1 << 22)
    w.install(eng)
    r = bench.run_batches(eng, ev, GB, dev)
    r["pv"] = eng.pv_last()
    r["pool"] = eng.param_pool()
elif which == "c3":
    # bench.py's C3 sub-line: 100k resources, all five controller kinds (tracegen variant 1)
    w = T.Workload(3, seed=T.SEED_BASE + 3, n_entries=24_000_000, variant=1)
    eng = E.Engine(max_resources=max(w.n_res, 1 << 10), max_slot_chain_size=0, max_batch_events=1 << 24,
                   aux_node_capacity=1 << 20)
    w.install(eng)
    r = bench.run_batches(eng, w.events, 1 << 24, dev)
else:
    w = T.Workload(5, seed=T.SEED_BASE + 5, n_entries=12_000_000)
    eng = E.Engine(max_resources=1 << 14, max_slot_chain_size=0, max_batch_events=1 << 23, param_table_log2=28,
                   status_ring_log2=26, aux_node_capacity=1 << 20)
    w.install(eng)
    ext = args = None
    if which == "c5ext":
        io, ic = w.intern_names(eng)
        ext, args = bench.param_args(w.events)
        oc = T.ext_for(w.events, io, ic, seed=T.SEED_BASE + 45)
        ext["origin_id"], ext["context_id"] = oc["origin_id"], oc["context_id"]
    r = bench.run_batches(eng, w.events, 1 << 23, dev, ext=ext, args=args)
    r["pv"] = eng.pv_last()
print(which, r, flush=True)
