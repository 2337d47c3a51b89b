"""The tiny-batch path (decide.hip k_tiny, engine.cpp tiny_impl): a synchronous sg_submit / sg_submit_ex
of at most 256 events runs every stage in one kernel.  Each test replays a trace in batches of 1 ... 256 events through
it (SG_TINY=1, the default) and through the batched path (SG_TINY=0), against the oracle: every decision, every
ClusterNode, and the origin / context nodes the tiny path keeps inline (k_lane<16>'s chain).

* the drop-in's input: contexts, origins, argument tables with Collection / array args, prioritized ENTRYs, upstream
  blocks, param rules (test_gpu_context_args.py's trace);
* the C4 shape with contexts and origins on every event (test_gpu_aux.py's node checks);
* STRATEGY_RELATE components (one segment for a component's members);
* a finite chain cap (CtSph.lookProcessChain, core/CtSph.java:206-227): a batch with a resource the host must grant or
  reject in first-ENTRY order falls back to the batched path; one at the cap is decided in place;
* param maps growing batch by batch in a small pool until its compaction is due (that batch falls back), and a
  malformed tiny batch rejected with nothing changed.
"""
import numpy as np
import pytest

import pyoracle as O
import test_gpu_aux as AX
import test_gpu_context_args as CA
import test_gpu_param_capacity as PC
from sentinel_amd import _abi as A
from sentinel_amd import engine as E
from sentinel_amd import tracegen as T

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 7, 64, 255, 256, 33, 128, 3]


def _cuts(n, sizes=SIZES):
    cuts, i, k = [0], 0, 0
    while i < n:
        i = min(n, i + sizes[k % len(sizes)])
        cuts.append(i)
        k += 1
    return cuts


def _check_decisions(dg, do, ev):
    bad = np.nonzero(dg != do)[0]
    assert len(bad) == 0, "decision mismatch at event %d (%s): gpu=%08x oracle=%08x; %d mismatches" % (
        bad[0], ev[bad[0]], dg[bad[0]], do[bad[0]], len(bad))


@pytest.mark.parametrize("tiny", ["1", "0"])
def test_contexts_args_small_batches(tiny, monkeypatch):
    monkeypatch.setenv("SG_TINY", tiny)
    n_res = 36
    eng, orc, io, ic, _ = CA._pair(n_res, True)
    ev, ext, table = CA._trace(7, n_res, 4_000, io, ic)
    cuts = _cuts(len(ev))
    dg, do = [], []
    for a, b in zip(cuts[:-1], cuts[1:]):
        g, o = CA._replay(eng, orc, ev[a:b], ext[a:b], table, 1)  # (it re-bases the slice's arg offsets)
        dg.append(g)
        do.append(o)
    dg, do = np.concatenate(dg), np.concatenate(do)
    CA._check(eng, orc, ev, dg, do, n_res)
    st = dg[ev["kind"] == A.EV_ENTRY] & 0xFF
    for s in (A.PASS, A.BLOCK_FLOW, A.BLOCK_PARAM, A.BLOCK_UPSTREAM):
        assert (st == s).sum() > 0, s


@pytest.mark.parametrize("tiny", ["1", "0"])
def test_c4_contexts_small_batches(tiny, monkeypatch):
    monkeypatch.setenv("SG_TINY", tiny)
    w = T.Workload(4, n_entries=6_000, n_res=400)
    eng = E.Engine(max_resources=w.n_res, max_slot_chain_size=0, status_ring_log2=22, aux_node_capacity=1 << 16)
    orc = O.Oracle(max_slot_chain_size=0)
    io, ic = AX._install(w, eng, [orc])
    ev = w.events
    ext = T.ext_for(ev, io, ic, seed=T.SEED_BASE + 61)
    cuts = _cuts(len(ev))
    dg = np.concatenate([eng.submit_ex(ev[a:b], ext[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    do = np.concatenate([orc.submit_ex(ev[a:b], ext[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    cnt = np.bincount(ev["res_id"], minlength=w.n_res)
    n = AX._compare(eng, orc, ev, dg, do, w.n_res, io, ic, np.argsort(-cnt)[:30])
    assert n > 0


@pytest.mark.parametrize("tiny", ["1", "0"])
def test_relate_small_batches(tiny, monkeypatch):
    monkeypatch.setenv("SG_TINY", tiny)
    w = T.Workload(2, n_entries=8_000, n_res=300)
    names = ["res-%d" % i for i in range(w.n_res)]
    rules = [A.flow_rule(nm, 3 + (i * 7) % 30) for i, nm in enumerate(names)]
    cnt = np.bincount(w.events["res_id"], minlength=w.n_res)
    hot = [int(x) for x in np.argsort(-cnt)[:12]]
    for k in range(0, 8, 2):
        rules.append(A.flow_rule(names[hot[k]], 4 + k, strategy=A.STRATEGY_RELATE, ref_resource=names[hot[k + 1]]))
    rules.append(A.flow_rule(names[hot[8]], 5, strategy=A.STRATEGY_RELATE, ref_resource=names[hot[9]]))
    rules.append(A.flow_rule(names[hot[9]], 6, strategy=A.STRATEGY_RELATE, ref_resource=names[hot[10]]))
    eng = E.Engine(max_resources=w.n_res + 8, max_slot_chain_size=0, status_ring_log2=22)
    orc = O.Oracle(max_slot_chain_size=0)
    for x in (eng, orc):
        w.install(x)
        x.load_flow_rules(rules)
    ev = w.events
    cuts = _cuts(len(ev))
    dg = np.concatenate([eng.submit(ev[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    do = np.concatenate([orc.submit(ev[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    _check_decisions(dg, do, ev)
    for r in hot[:11]:
        g, o = eng.read_node(r), orc.read_node(r)
        np.testing.assert_array_equal(g["second"][:2], o["second"][:2], err_msg="res %d" % r)
        np.testing.assert_array_equal(g["minute"], o["minute"], err_msg="res %d" % r)


@pytest.mark.parametrize("tiny", ["1", "0"])
def test_chain_cap_small_batches(tiny, monkeypatch):
    # 300 resources, a cap of 120 chains: early batches bring resources the host must grant in first-ENTRY order (the
    # tiny path falls back), later ones only granted, rejected or beyond-the-cap resources (decided in place)
    monkeypatch.setenv("SG_TINY", tiny)
    w = T.Workload(2, n_entries=6_000, n_res=300)
    eng = E.Engine(max_resources=w.n_res, max_slot_chain_size=120, status_ring_log2=22)
    orc = O.Oracle(max_slot_chain_size=120)
    w.install(eng)
    w.install(orc)
    ev = w.events
    cuts = _cuts(len(ev))
    dg = np.concatenate([eng.submit(ev[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    do = np.concatenate([orc.submit(ev[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    _check_decisions(dg, do, ev)
    st = dg[ev["kind"] == A.EV_ENTRY] & 0xFF
    assert (st == A.NO_CHECK).sum() > 0 and (st == A.PASS).sum() > 0


@pytest.mark.parametrize("tiny", ["1", "0"])
def test_param_maps_grow_and_the_pool_compacts_small_batches(tiny, monkeypatch):
    # test_gpu_param_capacity.py's 2^12-slot pool in batches of <= 256 events: the maps grow in the tiny kernel
    # (k_pm_grow's growth in place) until the host's compaction is due, when that batch takes the batched path
    monkeypatch.setenv("SG_TINY", tiny)
    eng = E.Engine(max_resources=64, max_slot_chain_size=0, param_table_log2=12)
    orc = O.Oracle(max_slot_chain_size=0)
    for nm in ("a", "b"):
        assert eng.register(nm) == orc.register(nm)
    rules = [A.param_rule("a", 0, 50), A.param_rule("b", 0, 50)]
    assert eng.load_param_rules(rules) == 2 and orc.load_param_rules(rules) == 2
    v0 = 0
    # a's two maps: 25, 75, 150 buckets after the first three batches (a region doubles at least), 504 of the 512
    # taken: the compaction is due before the fourth, which takes the batched path
    for b, n in enumerate((100, 200, 250, 50, 1)):
        ev = PC._entries(1 if n == 1 else 0, [PC._long(v) for v in range(v0, v0 + n)], t=PC.T0 + 100 * b)
        v0 += n
        np.testing.assert_array_equal(eng.submit(ev), orc.submit(ev), err_msg="batch %d" % b)
    pool = eng.param_pool()
    assert pool["compactions"] + pool["device_compactions"] >= 1 and pool["taken"] <= pool["buckets"], pool
    for v in (0, 99, 100, 350, 599):
        assert eng.param_thread_count(0, 0, PC._long(v)) == orc.param_thread_count(0, 0, PC._long(v)) == 1, v


def test_malformed_tiny_batch_changes_nothing():
    # an EXIT naming a later event: rejected before any decision, the engine as before (the next batch matches the
    # oracle that never saw the bad one)
    w = T.Workload(4, n_entries=2_000, n_res=50)
    eng = E.Engine(max_resources=w.n_res, max_slot_chain_size=0, status_ring_log2=22)
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(eng)
    w.install(orc)
    ev = w.events
    np.testing.assert_array_equal(eng.submit(ev[:100]), orc.submit(ev[:100]))
    bad = ev[100:110].copy()
    bad["kind"][5] = A.EV_EXIT
    bad["aux"][5] = A.aux_exit(100 + 9, 1)  # names a later event
    with pytest.raises(E.SentinelError) as ei:
        eng.submit(bad)
    assert ei.value.code == A.SG_EINVAL and "references" in str(ei.value)
    rest = ev[100:400]
    for a in range(0, len(rest), 37):
        np.testing.assert_array_equal(eng.submit(rest[a:a + 37]), orc.submit(rest[a:a + 37]))
