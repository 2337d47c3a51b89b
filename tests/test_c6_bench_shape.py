"""Parity of north_star's mixed-rule workload at the exact shape bench.py's C6 sub-line measures.

bench.py's C6 line (bench.py CONFIGS, config 6): 1M resources, each with a QPS DefaultController flow rule, a
DegradeRule and a QPS ParamFlowRule on args[0] (values Zipf(1.1) over 10M), 2^25-event batches through the
two-stage pipeline, param_table_log2 = 29, max_rules = 1 << 22.  At that size the paths that only a full-size
run reaches all run: the value-parallel pre / post passes over multi-million-event head segments
(pvalue.hip), the k_lite<true> lanes of ~700k cold resources, param maps growing inside the 2^29-slot pool and
the pool's device compaction between batches (engine.cpp compact_pmaps).  This test replays the first two
global batches of that exact trace, then time-shifted copies of them (built on the device as bench.py builds its
fresh batches), with the param map pool compacted on the device before the last two, through the engine and
through the resource-partitioned oracle, and compares every decision, the node windows of the 50 hottest and 300 random
resources and ParameterMetric.getThreadCount of the hot resources' values.

Reference: param/slots/HotParamSlotChainBuilder.java:38-51 (slot order), param/slots/block/flow/param/
ParameterMetric.java:37-39 (map capacities), ParamFlowChecker.java:121-196 (passDefaultLocalCheck).
"""
import os

import numpy as np
import pytest
import torch

import bench
import pyoracle as O
from sentinel_amd import _abi as A
from sentinel_amd import engine as E
from sentinel_amd import tracegen as T

pytestmark = pytest.mark.gpu

GB = 1 << 25


@pytest.mark.timeout(900)
def test_c6_bench_shape():
    cfg, n_entries, gb, kw, var, _ = [c for c in bench.CONFIGS if c[0] == 6][0]
    assert gb == GB and kw["param_table_log2"] == 29
    w = T.Workload(cfg, seed=T.SEED_BASE + cfg, n_entries=n_entries, variant=var)
    assert w.n_res == 1_000_000 and len(w.events) >= 2 * GB
    ev = w.events[:2 * GB]
    n_base = len(ev)
    tspan = int(ev["ts"][-1] - ev["ts"][0]) + 1000
    dev = torch.device("cuda", 0)
    base = torch.from_numpy(np.ascontiguousarray(ev).view(np.uint8).copy()).to(dev)
    base64 = base.view(torch.int64).view(-1, 3)

    def shifted(k, b):
        """Copy k of base batch b: on the device as bench.py builds it, on the host for the oracle."""
        c = torch.empty((GB, 3), dtype=torch.int64, device=dev)
        bench.shifted_batch(base64, b * GB, (b + 1) * GB, k, tspan, n_base, c)
        h = ev[b * GB:(b + 1) * GB].copy()
        h["ts"] += k * tspan
        isref = (h["kind"] != A.EV_ENTRY) & ((h["aux"] & np.uint64(A.REF_NONE)) != np.uint64(A.REF_NONE))
        h["aux"] = np.where(isref, h["aux"] + np.uint64(k * n_base), h["aux"])
        assert np.array_equal(c.cpu().numpy().view(np.uint8).reshape(-1), h.view(np.uint8)), (k, b)
        return c, h

    eng = E.Engine(device=0, max_resources=max(w.n_res, 1 << 10), max_slot_chain_size=0, max_batch_events=GB,
                   aux_node_capacity=1 << 20, **kw)
    w.install(eng)
    threads = min(16, len(os.sched_getaffinity(0)))
    po = O.PartitionedOracle(w, threads, max_slot_chain_size=0)
    # global batches in pairs, each pair back to back through the pipeline as bench.py submits: the two base batches,
    # then time-shifted copies of them (fresh to the engine: windows roll, breakers trip and reset, the maps keep
    # growing).  The maps take ~2.4M of the pool's 67M buckets a batch (bench.py's three batches never compact), so
    # after the second pair the pool is compacted on the device at this size (the submit path's compaction, forced)
    # and a third pair runs on the compacted maps.
    dg, do, allev, pv, pool = [], [], [], None, None
    out = [torch.empty(GB, dtype=torch.int32, device=dev) for _ in range(2)]
    for k in range(3):
        if k == 2:
            eng.param_compact()
        pair = [(base[b * GB * 24:], ev[b * GB:(b + 1) * GB]) for b in range(2)] if k == 0 else \
               [shifted(k, b) for b in range(2)]
        for (d, _), o in zip(pair, out):
            eng.submit_ptr(d.data_ptr(), GB, o.data_ptr(), sync=False)
        eng.sync()
        if k == 0:
            pv = eng.pv_last()
        dg += [o.cpu().numpy().view(np.uint32).copy() for o in out]
        do += [po.submit(h) for _, h in pair]
        allev += [h for _, h in pair]
        pool = eng.param_pool()
    dg, do, allev = np.concatenate(dg), np.concatenate(do), np.concatenate(allev)
    bad = np.nonzero(dg != do)[0]
    assert len(bad) == 0, "decision mismatch at event %d (%s): gpu=%08x oracle=%08x; %d mismatches" % (
        bad[0], allev[bad[0]], dg[bad[0]], do[bad[0]], len(bad))
    print("C6 bench shape: %d global batches, pool %s, pv %s" % (len(allev) // GB, pool, pv))

    cnt = np.bincount(ev["res_id"], minlength=w.n_res)
    rng = np.random.default_rng(7)
    touched = np.nonzero(cnt)[0]
    hot = np.argsort(-cnt)[:50]
    sample = np.unique(np.concatenate([hot, rng.choice(touched, 300, replace=False)]))
    for r in sample:
        g, o = eng.read_node(int(r)), po.read_node(int(r))
        assert g["has_chain"] == o["has_chain"] and g["thread"] == o["thread"], r
        np.testing.assert_array_equal(g["second"][:2], o["second"][:2], err_msg="second window of res %d" % r)
        np.testing.assert_array_equal(g["minute"], o["minute"], err_msg="minute window of res %d" % r)
    # ParameterMetric.getThreadCount of paramIdx 0 for values the hottest resources saw (neither side reorders)
    for r in hot[:8]:
        m = (allev["res_id"] == r) & (allev["kind"] == A.EV_ENTRY) & ((allev["flags"] & A.F_HAS_ARG) != 0)
        keys = np.unique(allev["aux"][m])
        keys = np.concatenate([keys[:400], rng.choice(keys, min(400, len(keys)), replace=False)])
        orc = po.orc_of(int(r))
        g = [eng.param_thread_count(int(r), 0, int(k)) for k in keys]
        o = [orc.param_thread_count(int(r), 0, int(k)) for k in keys]
        badk = [i for i in range(len(keys)) if g[i] != o[i]]
        assert not badk, ("thread count", int(r), hex(int(keys[badk[0]])), g[badk[0]], o[badk[0]], len(badk))

    # the shape really is the bench's: multi-million-event mixed heads through the value-parallel passes, param
    # blocks and flow / degrade blocks, and the map pool compacted on the device inside the run
    assert cnt.max() > 2_000_000
    st = dg[allev["kind"] == A.EV_ENTRY] & 0xFF
    for s in (A.BLOCK_PARAM, A.BLOCK_FLOW, A.BLOCK_DEGRADE, A.PASS):
        assert (st == s).sum() > 0, s
    assert pv["segments"] > 0 and pv["accesses"] > 1_000_000, pv
    assert pool["compactions"] == 1 and pool["taken"] < pool["buckets"], str(pool)
    po.close()
    eng.close()
