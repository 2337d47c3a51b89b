"""Parity at the exact shape bench.py measures.

bench.py decides 1M-resource C4 batches of 2^25 events with the default decide bins, the two-stage
pipeline (sg_submit_async) and device-resident buffers; its Zipf head puts ~4M events of one resource
into one batch, so the cooperative kernels' skip path, their old-reference loads (references older
than the LDS status window) and k_fill all run.  This test replays the first two global batches of
that exact trace, plus the time-shifted copy bench.py builds on the device for the batch after them,
through the engine and through the oracle (resource-partitioned over 16 threads, tests/test_dist.py
checks that partitioning), and compares every decision and the node state of the 50 hottest and of
a random sample of resources.
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


def test_bench_shape_two_batches_and_shifted_copy():
    w, ev = bench.make_trace(1_000_000, GB, 2, T.SEED_BASE + 4)
    n_base = len(ev)
    tspan = int(ev["ts"][-1] - ev["ts"][0]) + 1000
    dev = torch.device("cuda", 0)
    base = torch.from_numpy(np.ascontiguousarray(ev).view(np.uint8).copy()).to(dev)
    base64 = base.view(torch.int64).view(-1, 3)
    # global batch 2 = copy 1 of base batch 0, built on the device exactly as bench.py builds it
    copy = torch.empty((GB, 3), dtype=torch.int64, device=dev)
    bench.shifted_batch(base64, 0, GB, 1, tspan, n_base, copy)
    host_copy = ev[:GB].copy()
    host_copy["ts"] += tspan
    isref = (host_copy["kind"] != A.EV_ENTRY) & ((host_copy["aux"] & np.uint64(A.REF_NONE)) != np.uint64(A.REF_NONE))
    host_copy["aux"] = np.where(isref, host_copy["aux"] + np.uint64(n_base), host_copy["aux"])
    assert np.array_equal(copy.cpu().numpy().view(np.uint8).reshape(-1), host_copy.view(np.uint8))

    eng = E.Engine(max_resources=1 << 20, max_slot_chain_size=0, param_table_log2=16, status_ring_log2=28,
                   max_batch_events=GB)
    w.install(eng)
    outs = [torch.empty(GB, dtype=torch.int32, device=dev) for _ in range(3)]
    ptrs = [base.data_ptr(), base.data_ptr() + GB * 24, copy.data_ptr()]
    for p, o in zip(ptrs, outs):  # back to back through the pipeline, as bench.py submits
        eng.submit_ptr(p, GB, o.data_ptr(), sync=False)
    eng.sync()
    dg = np.concatenate([o.cpu().numpy().view(np.uint32) for o in outs])

    threads = min(16, len(os.sched_getaffinity(0)))
    po = O.PartitionedOracle(w, threads, max_slot_chain_size=0)
    do = np.concatenate([po.submit(ev[:GB]), po.submit(ev[GB:2 * GB]), po.submit(host_copy)])
    allev = np.concatenate([ev[:2 * GB], host_copy])
    bad = np.nonzero(dg != do)[0]
    assert len(bad) == 0, "decision mismatch at event %d (%s): gpu=%08x oracle=%08x; %d mismatches" % (
        bad[0], allev[bad[0]], dg[bad[0]], do[bad[0]], len(bad))
    cnt = np.bincount(ev["res_id"][:2 * GB], minlength=1_000_000)
    rng = np.random.default_rng(7)
    touched = np.nonzero(cnt)[0]
    sample = np.unique(np.concatenate([np.argsort(-cnt)[:50], rng.choice(touched, 300, replace=False)]))
    for r in sample:
        g, o = eng.read_node(int(r)), po.read_node(int(r))
        assert g["has_chain"] == o["has_chain"] and g["thread"] == o["thread"], r
        np.testing.assert_array_equal(g["second"][:2], o["second"][:2], err_msg="second window of res %d" % r)
        np.testing.assert_array_equal(g["minute"], o["minute"], err_msg="minute window of res %d" % r)
    # the shape really is the bench's: a multi-million-event head segment, skipped frozen stretches
    assert cnt.max() > 2_000_000 and eng.spans_total() > 0
    st = dg[allev["kind"] == A.EV_ENTRY] & 0xFF
    assert (st == A.BLOCK_FLOW).sum() > 0 and (st == A.BLOCK_DEGRADE).sum() > 0
    po.close()
