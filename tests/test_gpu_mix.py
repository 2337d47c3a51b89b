"""Mixed flow / degrade / param resources on the cooperative path (XF_MIX, north_star's target workload).

A resource with QPS ParamFlowRules on args[0] beside its flow and degrade rules is decided in three passes
(sentinel_amd/csrc/param.hip k_pq PQ_PRE / PQ_POST around the decide.hip k_jac owners):
  * ParamFlowSlot's checks first, per value: nothing before it in the chain blocks, so every ENTRY reaches them
    whatever the later slots decide (HotParamSlotChainBuilder.java:38-51, ParamFlowChecker.java:121-248); a blocked
    ENTRY gets its verdict there;
  * the flow / degrade chain on the owner, a param-blocked ENTRY counting as a block (StatisticSlot.java:97-133)
    and checking nothing (frozen / open stretches, skipped spans, the Jacobi iteration);
  * the thread-count map of paramIdx 0 from the final verdicts (ParamFlowStatisticEntryCallback /
    ExitCallback, ParameterMetric.java:126-149).
Everything is compared with the event-sequential oracle: decisions, ClusterNode windows, and -- through a
THREAD-grade rule loaded afterwards, which reads them on the per-lane kernel -- the thread-count maps.
"""
import numpy as np
import pytest

import pyoracle as O
from sentinel_amd import _abi as A
from sentinel_amd import engine as E
from sentinel_amd import tracegen as T

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


def _cmp(eng, orc, ev, what, ext=None):
    if ext is None:
        dg, do = eng.submit(ev), orc.submit(ev)
    else:
        dg, do = eng.submit_ex(ev, ext), orc.submit_ex(ev, ext)
    bad = np.nonzero(dg != do)[0]
    assert not len(bad), (what, "event", int(bad[0]), ev[bad[0]], hex(dg[bad[0]]), hex(do[bad[0]]), len(bad))
    return dg


def _thread_maps(eng, orc, ev, res, per=1500):
    # ParameterMetric.getThreadCount of paramIdx 0 for the values the resources saw (the last read: the oracle's
    # get moves the value in its LRU order)
    for r in res:
        m = (ev["res_id"] == r) & (ev["kind"] == A.EV_ENTRY) & ((ev["flags"] & A.F_HAS_ARG) != 0)
        keys = np.unique(ev["aux"][m])[:per]
        g = [eng.param_thread_count(int(r), 0, int(k)) for k in keys]
        o = [orc.param_thread_count(int(r), 0, int(k)) for k in keys]
        bad = [i for i in range(len(keys)) if g[i] != o[i]]
        assert not bad, ("thread count", int(r), hex(int(keys[bad[0]])), g[bad[0]], o[bad[0]], len(bad))


def _nodes(eng, orc, res):
    for r in res:
        g, o = eng.read_node(int(r)), orc.read_node(int(r))
        assert g["thread"] == o["thread"], r
        np.testing.assert_array_equal(g["second"][:2], o["second"][:2], err_msg="second window of res %d" % r)
        np.testing.assert_array_equal(g["minute"], o["minute"], err_msg="minute window of res %d" % r)


@pytest.mark.parametrize("pv", ["0", "1"])
@pytest.mark.parametrize("nval", [3_000, 300_000])
def test_mix_c6_shapes(nval, pv, monkeypatch):
    # C6 (every resource: a QPS flow rule, a breaker, a QPS param rule on args[0]) at 3000 resources: the Zipf head
    # is a J8 / J16 segment (wide pre / post pass), the body J4 / J1 (narrow), the tail one lane each; few values
    # (maps never evict, hot values get blocked) and many (the maps churn)
    # pv = 1: the long segments' param checks value-parallel (pvalue.hip), the maps rewritten after each segment
    monkeypatch.setenv("SG_PV", pv)
    n_res = 3000
    w = T.Workload(6, seed=T.SEED_BASE + 60, n_res=n_res, n_entries=500_000, n_param_values=nval)
    ev = w.events
    eng = E.Engine(max_resources=4096, max_slot_chain_size=0, param_table_log2=24, status_ring_log2=24)
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(eng)
    w.install(orc)
    cuts = np.linspace(0, len(ev), 4).astype(np.int64)
    dg, sts = [], []
    for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        dg.append(_cmp(eng, orc, ev[a:b], "batch %d" % i))
        sts.append(eng.pv_last())
    dg = np.concatenate(dg)
    if pv == "1":  # the value-parallel passes took the long segments
        tot = {k: sum(st[k] for st in sts) for k in sts[0]}
        assert tot["segments"] >= 9 and tot["accesses"] > 60_000, sts
        assert tot["post_segments"] >= 9 and tot["post_done"] >= 9 and tot["post_ops"] > 1000, sts
    cnt = np.bincount(ev["res_id"], minlength=n_res)
    _thread_maps(eng, orc, ev, np.argsort(-cnt)[:4])
    assert cnt.max() > 3 * 2 * 8192 and ((cnt > 3 * 1100) & (cnt < 3 * 8000)).sum() > 10  # wide and narrow passes
    _nodes(eng, orc, range(n_res))
    st = dg[ev["kind"] == A.EV_ENTRY] & 0xFF
    hot = np.argsort(-cnt)[:10]
    hst = dg[(ev["kind"] == A.EV_ENTRY) & np.isin(ev["res_id"], hot)] & 0xFF
    for s in (A.BLOCK_PARAM, A.BLOCK_FLOW):  # param and flow blocks on the cooperative heads
        assert (hst == s).sum() > 100, s
    assert (st == A.PASS).sum() > 0


def _synthetic(seed, n, gbase, nres, t=T0, span_ms=4000, nval=2000, rt_max=60, exit_args=0.9, trace_p=0.1):
    # n ENTRYs over nres resources (resource 0 gets half of them: a long segment), args[0] Zipf-ish with a uniform
    # tail, acquires mostly 1; about half the ENTRYs get an EXIT (90 % releasing the argument), a tenth a TRACE
    rng = np.random.default_rng(seed)
    ev = np.zeros(3 * n, dtype=A.EVENT_DTYPE)
    ts = t + np.sort(rng.integers(0, span_ms, n))
    k = 0
    pend = []
    for i in range(n):
        while pend and pend[0][0] <= ts[i]:
            tx, kind, ref, rid, rt = pend.pop(0)
            if kind == A.EV_EXIT:
                fl = A.F_EXIT_ARGS if rng.random() < exit_args else 0
                ev[k] = (tx, rid, 1, A.EV_EXIT, fl, A.aux_exit(ref, rt))
            else:
                ev[k] = (tx, rid, int(rng.integers(1, 3)), A.EV_TRACE, 0, ref)
            k += 1
        rid = 0 if rng.random() < 0.5 else int(rng.integers(1, nres))
        v = int(rng.zipf(1.3)) if rng.random() < 0.6 else int(rng.integers(0, nval))
        flags = A.F_HAS_ARG if rng.random() < 0.97 else 0
        cnt = int(rng.choice([1, 1, 1, 1, 2, 3]))  # (no zero acquires: they turn span skipping off)
        ev[k] = (ts[i], rid, cnt, A.EV_ENTRY, flags, E.param_key(str(v), "long"))
        if rng.random() < 0.5:
            rt = int(rng.integers(0, rt_max)) if rng.random() < 0.9 else int(rng.integers(100, 400))
            pend.append((int(ts[i]) + rt, A.EV_EXIT, gbase + k, rid, rt))
            if rng.random() < trace_p:
                pend.append((int(ts[i]) + rt, A.EV_TRACE, gbase + k, rid, 0))
            pend.sort()
        k += 1
    for tx, kind, ref, rid, rt in pend:
        if kind == A.EV_EXIT:
            ev[k] = (tx, rid, 1, A.EV_EXIT, A.F_EXIT_ARGS if rng.random() < exit_args else 0, A.aux_exit(ref, rt))
        else:
            ev[k] = (tx, rid, 1, A.EV_TRACE, 0, ref)
        k += 1
    return ev[:k]


NAMES = ("x0", "x1", "x2", "x3", "x4", "x5")


def _mix_rules(flow_count, thread_rule=False):
    f = [A.flow_rule("x0", flow_count), A.flow_rule("x1", 1e6), A.flow_rule("x2", 400),
         A.flow_rule("x3", 300, control_behavior=A.CONTROL_BEHAVIOR_WARM_UP, warm_up_period_sec=2),
         A.flow_rule("x4", 250), A.flow_rule("x4", 700, grade=A.FLOW_GRADE_THREAD),
         A.flow_rule("x5", 60, control_behavior=A.CONTROL_BEHAVIOR_RATE_LIMITER, max_queueing_time_ms=20)]
    d = [A.degrade_rule("x0", 40, 2, grade=A.DEGRADE_GRADE_RT),
         A.degrade_rule("x1", 0.3, 1, grade=A.DEGRADE_GRADE_EXCEPTION_RATIO),
         A.degrade_rule("x2", 30, 1, grade=A.DEGRADE_GRADE_EXCEPTION_COUNT),
         A.degrade_rule("x2", 45, 1, grade=A.DEGRADE_GRADE_RT),
         A.degrade_rule("x4", 0.5, 1, grade=A.DEGRADE_GRADE_EXCEPTION_RATIO)]
    p = [A.param_rule("x0", 0, 4, burst_count=2, items=[("7", "long", 0), ("8", "long", 60)]),
         A.param_rule("x0", 0, 9),
         A.param_rule("x1", 0, 3),
         A.param_rule("x1", 0, 1, cluster_mode=True, cluster_flow_id=5),  # initialised, never checked
         A.param_rule("x2", 0, 2, burst_count=1),
         A.param_rule("x3", 0, 6),
         A.param_rule("x4", 0, 5, duration_in_sec=1),
         A.param_rule("x4", 1, 1),  # an index the events never carry: its thread-count map exists, no check
         A.param_rule("x5", 0, 8)]
    if thread_rule:  # reads the thread-count maps the post passes kept (per-lane kernel from here on)
        p += [A.param_rule(nm, 0, 2, grade=A.FLOW_GRADE_THREAD) for nm in ("x0", "x1", "x2", "x3")]
    return f, d, p


@pytest.mark.parametrize("pv", ["0", "1"])
@pytest.mark.parametrize("flow_count", [30, 1e5])
def test_mix_stretches_and_thread_maps(flow_count, pv, monkeypatch):
    # one long segment per batch (x0: frozen stretches, skipped spans, the Jacobi iteration with param blocks at a
    # low flow limit; open stretches at a high one), an exception-ratio breaker beside param blocks (x1: the
    # ratio's total counts them), a WarmUp stage, a THREAD-grade flow stage, a rate limiter (x5: the J4 owner);
    # EXIT references across batches; then THREAD-grade param rules read the thread-count maps
    monkeypatch.setenv("SG_PV", pv)
    eng = E.Engine(max_resources=64, max_slot_chain_size=0, param_table_log2=22, status_ring_log2=24)
    orc = O.Oracle(max_slot_chain_size=0)
    for nm in NAMES:
        assert eng.register(nm) == orc.register(nm)

    def load(thread_rule=False):
        f, d, p = _mix_rules(flow_count, thread_rule)
        for x in (eng, orc):
            x.load_flow_rules(f)
            x.load_degrade_rules(d)
            x.load_param_rules(p)

    load()
    t, gbase = T0, 0
    blocked = {}
    for b in range(6):
        if b == 4:
            load(thread_rule=True)
        ev = _synthetic(200 + b, 150_000, gbase, len(NAMES), t=t)
        gbase += len(ev)
        d = _cmp(eng, orc, ev, "batch %d" % b)
        ent = ev["kind"] == A.EV_ENTRY
        for s in (A.BLOCK_PARAM, A.BLOCK_FLOW, A.BLOCK_DEGRADE):
            blocked[s] = blocked.get(s, 0) + int(((d[ent] & 0xFF) == s).sum())
        t = int(ev["ts"].max()) + 1
    _nodes(eng, orc, range(len(NAMES)))
    assert blocked[A.BLOCK_PARAM] > 1000 and blocked[A.BLOCK_FLOW] > 1000


def test_mix_ext_contexts():
    # sg_submit_ex with origins / contexts on mixed resources: the pre / post passes beside the aux post-pass
    n_res = 2000
    w = T.Workload(6, seed=T.SEED_BASE + 61, n_res=n_res, n_entries=300_000, n_param_values=50_000)
    ev = w.events
    eng = E.Engine(max_resources=2048, max_slot_chain_size=0, param_table_log2=24, status_ring_log2=24,
                   aux_node_capacity=1 << 17)
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(eng)
    w.install(orc)
    io, ic = w.intern_names(eng), w.intern_names(orc)
    assert np.array_equal(io[0], ic[0]) and np.array_equal(io[1], ic[1])
    ext = T.ext_for(ev, io[0], io[1], seed=11)
    cuts = np.linspace(0, len(ev), 3).astype(np.int64)
    for i, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        _cmp(eng, orc, ev[a:b], "ext batch %d" % i, ext=ext[a:b])
    _nodes(eng, orc, range(n_res))


@pytest.mark.parametrize("chain_cap", [0, 3])
def test_mix_first_seen_wide_resource(chain_cap):
    # The value-parallel pre pass's extraction runs beside the chain grants of its own batch (and beside the previous
    # batch's post pass) when every chain is granted (chain_cap 0): k_pv_prep then decides the grant's outcome itself.
    # x0 is absent from the first batch and a wide segment with no chain yet in the second; with chain_cap 3 the grants
    # are host-side (CtSph's chain cap: some resources never get one) and the pre pass waits for them.
    eng = E.Engine(max_resources=64, max_slot_chain_size=chain_cap, param_table_log2=22, status_ring_log2=24)
    orc = O.Oracle(max_slot_chain_size=chain_cap)
    for nm in NAMES:
        assert eng.register(nm) == orc.register(nm)
    f, d, p = _mix_rules(1e5)
    for x in (eng, orc):
        x.load_flow_rules(f)
        x.load_degrade_rules(d)
        x.load_param_rules(p)
    t, gbase, pv = T0, 0, []
    for b in range(3):
        ev = _synthetic(300 + b, 40_000, gbase, len(NAMES), t=t)
        if b == 0:
            ev["res_id"][ev["res_id"] == 0] = 1  # (x1 takes x0's events: every reference stays one resource's)
        gbase += len(ev)
        _cmp(eng, orc, ev, "batch %d" % b)
        pv.append(eng.pv_last())
        t = int(ev["ts"].max()) + 1
    _nodes(eng, orc, range(len(NAMES)))
    _thread_maps(eng, orc, ev, [0, 1, 2])
    if chain_cap == 0:  # x0's first batch went through the value-parallel pass
        assert pv[1]["segments"] >= 1 and pv[1]["accesses"] > 10_000, pv
