"""The drop-in's own input on the fast path (VERDICT r3 missing #1): sg_submit_ex batches whose every event carries
an origin and a named context, decided by the cooperative / lite / hot-parameter owners, with the origin
StatisticNodes and context DefaultNodes brought up to date by the aux.hip post-pass -- against the oracle.

The reference keeps those nodes for every entry whatever the rules (ClusterBuilderSlot.java:77-106,
NodeSelectorSlot.java:136-175, StatisticSlot.java:54-173).  Checked here: every decision and the ClusterNode of
every resource, and the origin / context nodes of a sample of resources field by field (second window, thread
count, the minute window's previous-second pass; sentinel_amd/csrc/aux.h says why that is all a node keeps of its
minute window), at the three post-pass shapes (one lane per short segment, one workgroup per piece of a long one,
pieces merged), then again after origin / CHAIN rules that read the nodes are loaded (k_lane<16> decides on what
the post-pass left).
"""
import os

import numpy as np
import pytest

import pyoracle as O
from sentinel_amd import _abi as A
from sentinel_amd import engine as E
from sentinel_amd import tracegen as T

pytestmark = pytest.mark.gpu

N_ORIG, N_CTX = 16, 4


def _install(w, eng, orcs, install_orcs=True):
    w.install(eng)
    if install_orcs:
        for o in orcs:
            w.install(o)
    io, ic = w.intern_names(eng, N_ORIG, N_CTX)
    for o in orcs:
        jo, jc = w.intern_names(o, N_ORIG, N_CTX)
        assert np.array_equal(io, jo) and np.array_equal(ic, jc)
    return io, ic


def _check_aux(eng, orc, res, io, ic, t_end):
    """Every origin / context node of res: device vs oracle."""
    n = 0
    for kind, ids, names, read in ((0, io, ["app-%d" % k for k in range(N_ORIG)], orc.read_origin_node),
                                   (1, ic, ["ctx-%d" % k for k in range(N_CTX)], orc.read_default_node)):
        for i, nm in zip(ids, names):
            g, o = eng.read_aux_node(res, kind, int(i)), read(res, nm)
            if o is None:
                assert g is None or (g["thread"] == 0 and (g["second"][:, 0] < 0).all()), (res, kind, nm)
                continue
            assert g is not None, (res, kind, nm)
            n += 1
            assert g["thread"] == o["thread"], (res, nm, g["thread"], o["thread"])
            np.testing.assert_array_equal(g["second"], o["second"][:2], err_msg="second window of %d/%s" % (res, nm))
            # the minute window: per second parity, the latest second with pass must be the device's history
            m = o["minute"]
            for q in range(2):
                ws, ps = g["mhist"][q]
                live = (m[:, 0] >= 0) & (m[:, 0] > t_end - 60_000) & ((m[:, 0] // 1000) % 2 == q) & (m[:, 1] > 0)
                if ws >= 0 and ws > t_end - 59_000:
                    k = np.nonzero(m[:, 0] == ws)[0]
                    assert len(k) == 1 and m[k[0], 1] == ps, (res, nm, q, ws, ps)
                    assert not (live & (m[:, 0] > ws)).any(), (res, nm, q)
                else:
                    assert not (live & (m[:, 0] > t_end - 58_000)).any(), (res, nm, q)
    return n


def _compare(eng, orc, ev, dg, do, n_res, io, ic, sample):
    bad = np.nonzero(dg != do)[0]
    assert len(bad) == 0, "decision mismatch at event %d (%s): gpu=%08x oracle=%08x; %d mismatches" % (
        bad[0], ev[bad[0]], dg[bad[0]], do[bad[0]], len(bad))
    for r in range(n_res):
        g, o = eng.read_node(r), orc.read_node(r)
        assert g["thread"] == o["thread"], r
        np.testing.assert_array_equal(g["second"][:2], o["second"][:2], err_msg="second window of res %d" % r)
        np.testing.assert_array_equal(g["minute"], o["minute"], err_msg="minute window of res %d" % r)
    t_end = int(ev["ts"][-1])
    return sum(_check_aux(eng, orc, int(r), io, ic, t_end) for r in sample)


@pytest.mark.parametrize("cfg", [4, 2, 3])
def test_ext_post_pass_parity(cfg):
    # C4 (flow + degrade: k_jac / k_lite) and C2 (flow only) shapes at 3000 resources: the Zipf head is a
    # segment of ~100k events (pieces + merge), the body single pieces, the tail one lane each; C3 (THREAD-grade /
    # WarmUp / rate-limiter heads: head.hip k_head decides the single-rule heads, the post-pass their nodes)
    n_res = 3000
    var = T.V_WARM_RL if cfg == 3 else 0
    w = T.Workload(cfg, seed=T.SEED_BASE + 40 + cfg, n_res=n_res, n_entries=400_000, variant=var)
    ev = w.events
    eng = E.Engine(max_resources=4096, max_slot_chain_size=0, status_ring_log2=24, aux_node_capacity=1 << 17)
    orc = O.Oracle(max_slot_chain_size=0)
    io, ic = _install(w, eng, [orc])
    ext = T.ext_for(ev, io, ic, seed=5)
    cuts = np.linspace(0, len(ev), 3).astype(np.int64)
    dg = np.concatenate([eng.submit_ex(ev[a:b], ext[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    do = np.concatenate([orc.submit_ex(ev[a:b], ext[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    cnt = np.bincount(ev["res_id"], minlength=n_res)
    assert cnt.max() > 2 * 4096 and ((cnt > 256) & (cnt <= 4096)).sum() > 10  # every post-pass shape ran
    rng = np.random.default_rng(3)
    sample = np.unique(np.concatenate([np.argsort(-cnt)[:12], rng.choice(np.nonzero(cnt)[0], 60, replace=False)]))
    assert _compare(eng, orc, ev, dg, do, n_res, io, ic, sample) > 300
    st = dg[ev["kind"] == A.EV_ENTRY] & 0xFF
    assert (st == A.BLOCK_FLOW).sum() > 0

    # origin / CHAIN rules that read the nodes arrive: k_lane<16> decides on the post-pass's node state
    rules = [A.flow_rule("res-%d" % r, 3, limit_app="app-%d" % (r % N_ORIG)) for r in range(0, n_res, 2)]
    rules += [A.flow_rule("res-%d" % r, 5, strategy=A.STRATEGY_CHAIN, ref_resource="ctx-%d" % (r % N_CTX))
              for r in range(1, n_res, 2)]
    rules += [A.flow_rule("res-%d" % r, 4, limit_app="other", control_behavior=A.CONTROL_BEHAVIOR_WARM_UP,
                          warm_up_period_sec=2) for r in range(0, n_res, 3)]
    for x in (eng, orc):
        x.load_flow_rules(rules)
    w2 = T.Workload(cfg, seed=T.SEED_BASE + 40 + cfg, n_res=n_res, n_entries=60_000, t0=int(ev["ts"][-1]) + 1,
                    variant=var)
    ev2 = w2.events.copy()
    isref = (ev2["kind"] != A.EV_ENTRY) & ((ev2["aux"] & np.uint64(A.REF_NONE)) != np.uint64(A.REF_NONE))
    ext2 = T.ext_for(ev2, io, ic, seed=6)  # (refs still local to ev2 here)
    ev2["aux"] = np.where(isref, ev2["aux"] + np.uint64(len(ev)), ev2["aux"])
    g2, o2 = eng.submit_ex(ev2, ext2), orc.submit_ex(ev2, ext2)
    allev = np.concatenate([ev, ev2])
    n = _compare(eng, orc, allev, np.concatenate([dg, g2]), np.concatenate([do, o2]), n_res, io, ic, sample)
    assert n > 300
    st = g2[ev2["kind"] == A.EV_ENTRY] & 0xFF
    assert (st == A.BLOCK_FLOW).sum() > 100


def test_ext_bench_shape_c4():
    # VERDICT r3 "done" for missing #1: the C4 bench shape (1M resources, 2^25-event batches, the two-stage
    # pipeline) through sg_submit_ex with every event in one of 4 named contexts from one of 16 origins
    import bench
    import torch
    GB = 1 << 25
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)  # torch's HIP runtime first (as bench.py and test_bench_shape do)
    w, ev = bench.make_trace(1_000_000, GB, 2, T.SEED_BASE + 4)
    eng = E.Engine(max_resources=1 << 20, max_slot_chain_size=0, param_table_log2=16, status_ring_log2=28,
                   max_batch_events=GB, aux_node_capacity=1 << 24)
    threads = min(16, len(os.sched_getaffinity(0)))
    po = O.PartitionedOracle(w, threads, max_slot_chain_size=0)
    io, ic = _install(w, eng, po.orcs, install_orcs=False)  # (the partitioned oracle installed its shards)
    ext = T.ext_for(ev, io, ic, seed=9)
    dev_ev = torch.from_numpy(np.ascontiguousarray(ev).view(np.uint8).copy()).to(dev)
    dev_ext = torch.from_numpy(ext.view(np.uint8).copy()).to(dev)
    outs = [torch.empty(GB, dtype=torch.int32, device=dev) for _ in range(2)]
    for b in range(2):  # device buffers, back to back through the pipeline
        eng.submit_ex_ptr(dev_ev.data_ptr() + b * GB * 24, dev_ext.data_ptr() + b * GB * 16, GB, outs[b].data_ptr(),
                          sync=False)
    eng.sync()
    dg = np.concatenate([o.cpu().numpy().view(np.uint32) for o in outs])
    do = np.concatenate([po.submit_ex(ev[:GB], ext[:GB]), po.submit_ex(ev[GB:], ext[GB:])])
    bad = np.nonzero(dg != do)[0]
    assert len(bad) == 0, "decision mismatch at event %d (%s): gpu=%08x oracle=%08x; %d mismatches" % (
        bad[0], ev[bad[0]], dg[bad[0]], do[bad[0]], len(bad))
    cnt = np.bincount(ev["res_id"], minlength=1_000_000)
    rng = np.random.default_rng(7)
    sample = np.unique(np.concatenate([np.argsort(-cnt)[:30], rng.choice(np.nonzero(cnt)[0], 200, replace=False)]))
    t_end = int(ev["ts"][-1])
    n = 0
    for r in sample:
        g, o = eng.read_node(int(r)), po.read_node(int(r))
        assert g["thread"] == o["thread"], r
        np.testing.assert_array_equal(g["second"][:2], o["second"][:2], err_msg="second window of res %d" % r)
        np.testing.assert_array_equal(g["minute"], o["minute"], err_msg="minute window of res %d" % r)
        n += _check_aux(eng, po.orc_of(int(r)), int(r), io, ic, t_end)
    assert n > 1000
    assert cnt.max() > 2_000_000
    po.close()
