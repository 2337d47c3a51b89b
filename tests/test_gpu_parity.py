"""Parity of the HIP engine against the CPU oracle (bit-exact decisions and bucket counters).

Every test replays the same seeded trace through the oracle (event-sequential CPU
restatement) and through the C ABI on the GPU, in several batches, then compares
the per-event decisions and the ClusterNode state of the hottest and of a random
sample of resources field by field.
"""
import numpy as np
import pytest

import pyoracle as O
from sentinel_amd import _abi as A
from sentinel_amd import engine as E
from sentinel_amd import tracegen as T

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_123


def _engine(**kw):
    kw.setdefault("max_resources", 1 << 12)
    kw.setdefault("status_ring_log2", 24)
    return E.Engine(**kw)


def _replay(w, eng, orc, batches):
    ev = w.events
    cuts = np.linspace(0, len(ev), batches + 1).astype(np.int64)
    dg, do = [], []
    for a, b in zip(cuts[:-1], cuts[1:]):
        dg.append(eng.submit(ev[a:b]))
        do.append(orc.submit(ev[a:b]))
    return np.concatenate(dg), np.concatenate(do)


def _assert_same_decisions(dg, do, ev):
    bad = np.nonzero(dg != do)[0]
    if len(bad):
        i = bad[0]
        raise AssertionError("decision mismatch at event %d (%s): gpu=%08x oracle=%08x; %d mismatches"
                             % (i, ev[i], dg[i], do[i], len(bad)))


def _compare_nodes(w, eng, orc, res_ids):
    for r in res_ids:
        g, o = eng.read_node(int(r)), orc.read_node(int(r))
        assert g["has_chain"] == o["has_chain"], r
        assert g["thread"] == o["thread"], (r, g["thread"], o["thread"])
        np.testing.assert_array_equal(g["second"][:2], o["second"][:2], err_msg="second window of res %d" % r)
        np.testing.assert_array_equal(g["minute"], o["minute"], err_msg="minute window of res %d" % r)


def _sample(w, k=300, seed=0):
    ev = w.events
    cnt = np.bincount(ev["res_id"], minlength=w.n_res)
    hot = np.argsort(-cnt)[:50]
    rng = np.random.default_rng(seed)
    touched = np.nonzero(cnt)[0]
    rnd = rng.choice(touched, size=min(k, len(touched)), replace=False)
    return np.unique(np.concatenate([hot, rnd]))


# decide-bin modes: the engine reads its bin thresholds at creation (engine.cpp sg_engine_create)
BIN_MODES = {
    "default": {},
    # every eligible segment through the cooperative kernels, all three widths exercised
    "coop": {"SG_LANE_MAX": "0", "SG_J1_MAX": "40", "SG_J4_MAX": "400"},
    # every segment through the one-lane-per-segment kernel
    "lane": {"SG_DEBUG_FLAGS": "2"},
    # cooperative kernels skipping every frozen stretch longer than 16 positions (k_fill writes the verdicts)
    "skip": {"SG_LANE_MAX": "0", "SG_J1_MAX": "40", "SG_J4_MAX": "400", "SG_SKIP_MIN": "16"},
}


@pytest.fixture(params=sorted(BIN_MODES))
def bin_mode(request, monkeypatch):
    for k, v in BIN_MODES[request.param].items():
        monkeypatch.setenv(k, v)
    return request.param


def _run(config, batches=3, chain_cap=0, **kw):
    w = T.Workload(config, **kw)
    eng = _engine(max_resources=max(64, w.n_res), max_slot_chain_size=chain_cap)
    orc = O.Oracle(max_slot_chain_size=chain_cap)
    w.install(eng)
    w.install(orc)
    dg, do = _replay(w, eng, orc, batches)
    _assert_same_decisions(dg, do, w.events)
    _compare_nodes(w, eng, orc, _sample(w))
    return w, eng, orc, dg


def test_c1_flowqpsdemo(bin_mode):
    # FlowQpsDemo (sentinel-demo-basic .../flow/FlowQpsDemo.java:37-66): ~20 pass/s under QPS=20
    w, eng, orc, d = _run(1, batches=4)
    st = d[w.events["kind"] == A.EV_ENTRY] & 0xFF
    assert int((st == A.PASS).sum()) == 2000  # 20 pass/s for 100 s


def test_c2_qps_default(bin_mode):
    _run(2, batches=3, n_entries=400_000)


def test_c3_mixed_controllers(bin_mode):
    _run(3, batches=3, n_entries=400_000, n_res=20_000)


def test_c4_degrade(bin_mode):
    _run(4, batches=3, n_entries=400_000, n_res=50_000)


@pytest.mark.parametrize("config", [2, 4])
def test_cooperative_without_open_stretches(config, monkeypatch):
    # the Jacobi iteration alone (debug flag 64 turns the all-pass open stretches off), every width exercised
    for k, v in BIN_MODES["coop"].items():
        monkeypatch.setenv(k, v)
    monkeypatch.setenv("SG_DEBUG_FLAGS", "64")
    _run(config, batches=3, n_entries=400_000, n_res=50_000 if config == 4 else 0)


def test_c2_full_resource_count():
    # C2 at its configured 10k resources, 4M entries (4 s of trace) in 4 batches, default bins
    _run(2, batches=4, n_entries=4_000_000, n_res=10_000)


def test_c3_full_resource_count():
    # C3 at its configured 100k resources (QPS / thread / WarmUp / RateLimiter / WarmUpRateLimiter mix),
    # 2M entries in 3 batches, default bins
    _run(3, batches=3, n_entries=2_000_000, n_res=100_000, variant=T.V_WARM_RL)


@pytest.mark.parametrize("batches", [8, 2])
def test_c4_minute_window_long_trace(batches, bin_mode):
    # 2000 entries/s for ~150 s: exceptions leave the minute window while exception-count breakers read it
    # (k_lite's running exception sum, chain.h exc_advance), in batches of ~19 s and of ~75 s (a second of
    # the batch expires inside it).
    _run(4, batches=batches, n_entries=300_000, n_res=3_000, rate=2000.0)


def test_c4_wide_keys_three_radix_passes():
    # 200k resources: 18-bit keys take all three 8-bit radix passes of the group stage (as the 1M-resource
    # bench layout does)
    _run(4, batches=2, n_entries=600_000, n_res=200_000)


def test_switch_off_checks_nothing():
    # Constants.ON = false (core/Constants.java:67): CtSph.entryWithPriority hands out an Entry with no
    # chain (CtSph.java:130-133), so nothing is checked or counted; every entry is NO_CHECK on both sides
    w = T.Workload(3, n_entries=200_000, n_res=5_000, variant=T.V_WARM_RL)
    eng = _engine(max_resources=w.n_res, max_slot_chain_size=0, switch_on=0)
    orc = O.Oracle(max_slot_chain_size=0, switch_on=0)
    w.install(eng)
    w.install(orc)
    dg, do = _replay(w, eng, orc, 2)
    _assert_same_decisions(dg, do, w.events)
    ent = w.events["kind"] == A.EV_ENTRY
    assert ((dg[ent] & 0xFF) == A.NO_CHECK).all()
    _compare_nodes(w, eng, orc, _sample(w, k=50))


def test_c5_param(bin_mode):
    _run(5, batches=3, n_entries=400_000, n_param_values=50_000)


def test_c3_warm_up_rate_limiter(bin_mode):
    # WarmUpRateLimiterController (core/slots/block/flow/controller/WarmUpRateLimiterController.java) in the mix
    w, *_ = _run(3, batches=3, n_entries=400_000, n_res=20_000, variant=T.V_WARM_RL)
    assert w.variant == T.V_WARM_RL


def test_c5_hot_items_and_thread_grade(bin_mode):
    # local hot items (ParamFlowChecker.passDefaultLocalCheck / passThrottleLocalCheck exclusion items) and
    # THREAD-grade param rules with exits that release their argument (ParameterMetric.decreaseThreadCount)
    _, _, _, d = _run(5, batches=3, n_entries=400_000, n_param_values=50_000, variant=T.V_HOT | T.V_THREAD)
    assert int(((d & 0xFF) == A.BLOCK_PARAM).sum()) > 0


def test_c5_full_param_maps_evict(bin_mode):
    # 16 resources, ~25k entries each over 200k values: every map fills and evicts its LRU values
    _, _, _, d = _run(5, batches=4, n_entries=400_000, n_res=16, n_param_values=200_000,
                      variant=T.V_UNIFORM | T.V_HOT | T.V_THREAD)
    assert int(((d & 0xFF) == A.BLOCK_PARAM).sum()) > 0


def test_chain_cap_reference_default():
    # Q1: only the first 6000 resources to enter get a slot chain (core/CtSph.java:206-227)
    _run(2, batches=2, chain_cap=6000, n_entries=300_000)


@pytest.mark.parametrize("path", ["default", "hot_cold"])
def test_many_small_batches_and_single_events(bin_mode, path, monkeypatch):
    # default: <= 256 events the one-workgroup k_tiny, larger the radix group stage (below SG_RADIX_BELOW);
    # hot_cold: every batch through the batched pipeline's hot / cold group stage (k_cold_small for one tile)
    if path == "hot_cold":
        monkeypatch.setenv("SG_TINY", "0")
        monkeypatch.setenv("SG_RADIX_BELOW", "0")
    w = T.Workload(4, n_entries=20_000, n_res=2_000)
    eng = _engine(max_resources=w.n_res, max_slot_chain_size=0)
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(eng)
    w.install(orc)
    ev = w.events
    dg, do = [], []
    i = 0
    sizes = [1, 2, 3, 64, 65, 127, 1000, 4097, 4096, 4095]  # (one tile: k_cold_small; more: the radix passes)
    k = 0
    while i < len(ev):
        s = sizes[k % len(sizes)]
        dg.append(eng.submit(ev[i:i + s]))
        do.append(orc.submit(ev[i:i + s]))
        i += s
        k += 1
    dg, do = np.concatenate(dg), np.concatenate(do)
    _assert_same_decisions(dg, do, ev)
    _compare_nodes(w, eng, orc, _sample(w, 200))


# ------------------------------------------------------------------ reference scenarios on the device
def _ev(rows):
    a = np.zeros(len(rows), dtype=A.EVENT_DTYPE)
    for i, (ts, res, kind, count, flags, aux) in enumerate(rows):
        a[i] = (ts, res, count, kind, flags, aux)
    return a


def test_flow_qps_grade_scenario():
    # core-test/slots/block/flow/FlowPartialIntegrationTest.java:51-73 through the C ABI
    eng = _engine()
    rid = eng.register("testQPSGrade")
    eng.load_flow_rules([A.flow_rule("testQPSGrade", 1)])
    d = eng.submit(_ev([(T0, rid, A.EV_ENTRY, 1, 0, 0), (T0, rid, A.EV_EXIT, 1, 0, A.aux_exit(0, 0)),
                        (T0, rid, A.EV_ENTRY, 1, 0, 0)]))
    assert [x & 0xFF for x in d] == [A.PASS, A.NOT_ENTRY, A.BLOCK_FLOW]


def test_thread_grade_scenario():
    # FlowPartialIntegrationTest.java:75-116
    eng = _engine()
    rid = eng.register("testThreadGrade")
    eng.load_flow_rules([A.flow_rule("testThreadGrade", 1, grade=A.FLOW_GRADE_THREAD)])
    d = eng.submit(_ev([(T0, rid, A.EV_ENTRY, 1, 0, 0), (T0 + 1, rid, A.EV_ENTRY, 1, 0, 0),
                        (T0 + 100, rid, A.EV_EXIT, 1, 0, A.aux_exit(0, 100)), (T0 + 101, rid, A.EV_ENTRY, 1, 0, 0)]))
    assert [x & 0xFF for x in d] == [A.PASS, A.BLOCK_FLOW, A.NOT_ENTRY, A.PASS]
    assert eng.read_node(rid)["thread"] == 1


def _submit_ctx(eng, rid, rows):
    """rows: (ts, kind, origin, context, ref) -> decisions through sg_submit_ex (origin / context interned)."""
    ev = np.zeros(len(rows), dtype=A.EVENT_DTYPE)
    ext = np.zeros(len(rows), dtype=A.EXT_DTYPE)
    for i, (ts, kind, origin, ctx, ref) in enumerate(rows):
        aux = 0 if kind == A.EV_ENTRY else A.aux_exit(ref, 0)
        ev[i] = (ts, rid, 1, kind, 0, aux)
        ext[i]["origin_id"] = eng.intern_origin(origin) if origin else 0
        ext[i]["context_id"] = eng.intern_context(ctx) if ctx else 0
    return [int(x) & 0xFF for x in eng.submit_ex(ev, ext)]


def test_origin_flow_rule_scenario():
    # FlowPartialIntegrationTest.java:118-158 (testOriginFlowRule): "other" at 0 blocks app1, app2 has its own rule
    eng = _engine()
    rid = eng.register("testOriginFlowRule")
    eng.load_flow_rules([A.flow_rule("testOriginFlowRule", 0, limit_app="other"),
                         A.flow_rule("testOriginFlowRule", 1, limit_app="app2")])
    d = _submit_ctx(eng, rid, [(T0, A.EV_ENTRY, "app1", "node1", 0), (T0, A.EV_ENTRY, "app2", "node1", 0),
                               (T0, A.EV_EXIT, "app2", "node1", 1)])
    assert d == [A.BLOCK_FLOW, A.PASS, A.NOT_ENTRY]


def test_flow_rule_other_scenario():
    # FlowPartialIntegrationTest.java:160-181 (testFlowRule_other): no origin is not an "other" origin
    eng = _engine()
    rid = eng.register("testOther")
    eng.load_flow_rules([A.flow_rule("testOther", 0, limit_app="other")])
    assert _submit_ctx(eng, rid, [(T0, A.EV_ENTRY, None, None, 0)]) == [A.PASS]


def test_strategy_chain_scenario():
    # FlowPartialIntegrationTest.java:224-255 (testStrategyChain): the rule reads the DefaultNode of context entry1
    eng = _engine()
    rid = eng.register("entry2")
    eng.load_flow_rules([A.flow_rule("entry2", 0, strategy=A.STRATEGY_CHAIN, ref_resource="entry1")])
    d = _submit_ctx(eng, rid, [(T0, A.EV_ENTRY, None, "entry1", 0), (T0, A.EV_ENTRY, None, "entry3", 0)])
    assert d == [A.BLOCK_FLOW, A.PASS]


def test_param_burst_scenario():
    # param-test/slots/block/flow/param/ParamFlowDefaultCheckerTest.java:69-137 through the C ABI
    eng = _engine()
    rid = eng.register("burst")
    eng.load_param_rules([A.param_rule("burst", 0, 5, burst_count=3)])
    k = E.param_key("valueA")
    rows, expect = [], []
    now = T0
    for step, npass in [(0, 8), (1002, 5), (1002, 5), (2000, 8), (1002, 5)]:
        now += step
        for _ in range(npass + 1):
            rows.append((now, rid, A.EV_ENTRY, 1, A.F_HAS_ARG, k))
        expect += [A.PASS] * npass + [A.BLOCK_PARAM]
    d = eng.submit(_ev(rows))
    assert [x & 0xFF for x in d] == expect


def test_backward_clock_across_batches_is_an_error():
    # a resource whose next batch starts before a window it already holds (LeapArray would hand
    # out a detached bucket).  The decide kernels flag it and sg_submit must return SG_EINVAL, not SG_OK.
    eng = _engine()
    rid = eng.register("back")
    eng.load_flow_rules([A.flow_rule("back", 100)])
    assert (eng.submit(_ev([(T0 + 5000, rid, A.EV_ENTRY, 1, 0, 0)]))[0] & 0xFF) == A.PASS
    with pytest.raises(E.SentinelError) as ei:
        eng.submit(_ev([(T0, rid, A.EV_ENTRY, 1, 0, 0)]))
    assert ei.value.code == A.SG_EINVAL and "non-decreasing" in str(ei.value)
    # the engine stays usable for time-ordered batches
    assert (eng.submit(_ev([(T0 + 6000, rid, A.EV_ENTRY, 1, 0, 0)]))[0] & 0xFF) == A.PASS


@pytest.mark.parametrize("kind", [A.EV_EXIT, A.EV_TRACE])
def test_reference_to_other_resource_is_an_error(kind, bin_mode):
    # An EXIT/TRACE naming an earlier ENTRY of another resource (the ABI requires its own resource's ENTRY):
    # BF_BAD_REF raised by the decide kernels surfaces as SG_EINVAL from sg_submit.
    eng = _engine()
    a, b = eng.register("ra"), eng.register("rb")
    eng.load_flow_rules([A.flow_rule("ra", 100), A.flow_rule("rb", 100)])
    rows = [(T0 + i, a if i % 2 else b, A.EV_ENTRY, 1, 0, 0) for i in range(600)]
    aux = A.aux_exit(1, 5) if kind == A.EV_EXIT else 1  # event 1 is an ENTRY of "ra"
    rows.append((T0 + 700, b, kind, 1, 0, aux))
    with pytest.raises(E.SentinelError) as ei:
        eng.submit(_ev(rows))
    assert ei.value.code == A.SG_EINVAL and "references" in str(ei.value)


def test_degrade_rt_scenario():
    # DegradeRule RT breaker (core/slots/block/degrade/DegradeRule.java:181-193): 5 consecutive
    # checks over the threshold cut the resource for timeWindow seconds.
    eng = _engine()
    orc = O.Oracle()
    rows = []
    for eng_or_orc in (eng, orc):
        eng_or_orc.register("rt")
        eng_or_orc.load_degrade_rules([A.degrade_rule("rt", 10, 2)])
    gi = 0
    t = T0
    # one slow call, then a stream of entries
    rows.append((t, 0, A.EV_ENTRY, 1, 0, 0))
    rows.append((t + 50, 0, A.EV_EXIT, 1, 0, A.aux_exit(0, 50)))
    for i in range(12):
        rows.append((t + 60 + i, 0, A.EV_ENTRY, 1, 0, 0))
    rows.append((t + 2100, 0, A.EV_ENTRY, 1, 0, 0))
    rows.append((t + 3000, 0, A.EV_ENTRY, 1, 0, 0))
    ev = _ev(rows)
    dg, do = eng.submit(ev), orc.submit(ev)
    np.testing.assert_array_equal(dg, do)
    st = [x & 0xFF for x in dg]
    assert st[2:6] == [A.PASS] * 4 and st[6] == A.BLOCK_DEGRADE


def test_snapshot_matches_oracle():
    w = T.Workload(2, n_entries=100_000, n_res=500)
    eng = _engine(max_resources=w.n_res, max_slot_chain_size=0)
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(eng)
    w.install(orc)
    eng.submit(w.events)
    orc.submit(w.events)
    for now in (w.t_end + 10, w.t_end + 1500, w.t_end + 70000):
        sg = eng.snapshot(now)
        so = orc.snapshot(now)
        key = lambda a: np.lexsort((a["timestamp"], a["res_id"]))
        np.testing.assert_array_equal(sg[key(sg)], so[key(so)])


# ---------------------------------------------------------------- prioritized entries (A11/A12)
def _run_prioritized(config, frac, batches, **kw):
    """A workload with a fraction of its ENTRYs prioritized: DefaultController.canPass ->
    StatisticNode.tryOccupyNext / addWaitingRequest / addOccupiedPass -> PriorityWaitException
    (core/slots/block/flow/controller/DefaultController.java:49-81, core/node/StatisticNode.java:293-341),
    with the OccupiableBucketLeapArray borrow transfer on window creation and reset (Q6)."""
    w = T.Workload(config, **kw)
    ev = w.events
    rng = np.random.default_rng(11 + config)
    ent = ev["kind"] == A.EV_ENTRY
    pick = ent & (rng.random(len(ev)) < frac)
    ev["flags"] = np.where(pick, ev["flags"] | A.F_PRIORITIZED, ev["flags"])
    eng = _engine(max_resources=max(64, w.n_res), max_slot_chain_size=0)
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(eng)
    w.install(orc)
    dg, do = _replay(w, eng, orc, batches)
    _assert_same_decisions(dg, do, ev)
    res = _sample(w)
    _compare_nodes(w, eng, orc, res)
    for r in res:
        np.testing.assert_array_equal(eng.read_node(int(r))["borrow"][:2], orc.read_node(int(r))["borrow"][:2],
                                      err_msg="borrow ring of res %d" % r)
    return dg, w  # w owns the event buffer


def test_prioritized_flowqps(bin_mode):
    dg, w = _run_prioritized(1, 0.3, 4)
    ent = w.events["kind"] == A.EV_ENTRY
    st = dg[ent] & 0xFF
    assert (st == A.PASS_WAIT).sum() > 0  # the occupy path is exercised
    wait = dg[ent][st == A.PASS_WAIT] >> 16
    assert (wait > 0).all() and (wait < 500).all()


def test_prioritized_zipf(bin_mode):
    _run_prioritized(2, 0.2, 3, n_entries=200_000)


# ---------------------------------------------------------------- exit(count, args) (A25, Q14)
def test_exit_with_args_thread_params(bin_mode):
    """THREAD-grade param rules: onPass increments the value's thread count
    (ParamFlowStatisticEntryCallback.java:33-40) and only exit(count, args) decrements it
    (ParamFlowStatisticExitCallback.java:31-38, core/Entry.java:78-80), so with 70 % of the EXITs
    carrying args the counts -- and the THREAD verdicts -- depend on the exits."""
    w = T.Workload(5, n_entries=150_000, n_res=200, n_param_values=300)
    ev = w.events
    rng = np.random.default_rng(5)
    ex = (ev["kind"] == A.EV_EXIT) & (rng.random(len(ev)) < 0.7)
    ev["flags"] = np.where(ex, ev["flags"] | A.F_EXIT_ARGS, ev["flags"])
    names = ["res-%d" % i for i in range(w.n_res)]
    rules = [A.param_rule(nm, 0, 2 + i % 4, grade=A.FLOW_GRADE_THREAD) if i % 2 == 0 else
             A.param_rule(nm, 0, 20 + i % 30) for i, nm in enumerate(names)]
    eng = _engine(max_resources=max(64, w.n_res), max_slot_chain_size=0)
    orc = O.Oracle(max_slot_chain_size=0)
    for x in (eng, orc):
        w.install(x)
        x.load_param_rules(rules)
    dg, do = _replay(w, eng, orc, 3)
    _assert_same_decisions(dg, do, ev)
    _compare_nodes(w, eng, orc, _sample(w))
    st = dg[ev["kind"] == A.EV_ENTRY] & 0xFF
    assert (st == A.BLOCK_PARAM).sum() > 0 and (st == A.PASS).sum() > 0


# ---------------------------------------------------------------- batch pipeline (sg_submit_async)
@pytest.mark.parametrize("pipeline", ["0", "1"])
@pytest.mark.parametrize("config,kw", [(4, {"n_entries": 300_000, "n_res": 5_000}), (3, {"n_entries": 300_000, "n_res": 20_000}),
                                       (4, {"n_entries": 300_000, "n_res": 40})])
def test_async_pipeline(config, kw, pipeline, monkeypatch):
    """Batches submitted back to back with sg_submit_async: the group stage of batch k+1 runs while
    batch k is decided (SG_PIPELINE=1, the default), and references into earlier batches are resolved
    in the decide stage.  The 40-resource case keeps the cooperative kernels skipping frozen stretches."""
    monkeypatch.setenv("SG_PIPELINE", pipeline)
    monkeypatch.setenv("SG_SKIP_MIN", "64")
    w = T.Workload(config, **kw)
    eng = _engine(max_resources=max(64, w.n_res), max_slot_chain_size=0)
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(eng)
    w.install(orc)
    ev = w.events
    cuts = np.linspace(0, len(ev), 7).astype(np.int64)
    parts = [np.ascontiguousarray(ev[a:b]) for a, b in zip(cuts[:-1], cuts[1:])]
    outs = [np.zeros(len(p), dtype=np.uint32) for p in parts]
    for p, o in zip(parts, outs):
        eng.submit_ptr(p.ctypes.data, len(p), o.ctypes.data, sync=False)
    eng.sync()
    dg = np.concatenate(outs)
    do = np.concatenate([orc.submit(p) for p in parts])
    _assert_same_decisions(dg, do, ev)
    _compare_nodes(w, eng, orc, _sample(w))
    assert len(eng.timing_log()) == len(parts)


# ---------------------------------------------------------------- STRATEGY_RELATE (A13)
def test_relate_components(bin_mode):
    """FlowRuleChecker.selectReferenceNode RELATE (core/slots/block/flow/FlowRuleChecker.java:67-88): the
    rule of A is checked against the ClusterNode of B; A's and B's events are decided in one sequence.
    Pairs, a 3-chain, a self reference (the resource's own node) and a reference to a resource that is
    never entered (no ClusterNode: pass)."""
    w = T.Workload(2, n_entries=200_000, n_res=3_000)
    names = ["res-%d" % i for i in range(w.n_res)]
    rules = [A.flow_rule(nm, 15 + (i * 7) % 300) for i, nm in enumerate(names)]
    cnt = np.bincount(w.events["res_id"], minlength=w.n_res)
    hot = [int(x) for x in np.argsort(-cnt)[:40]]
    for k in range(0, 30, 2):  # pairs among hot resources: a.relate(b)
        a, b = hot[k], hot[k + 1]
        rules.append(A.flow_rule(names[a], 20 + k, strategy=A.STRATEGY_RELATE, ref_resource=names[b]))
    a, b, c = hot[30], hot[31], hot[32]  # chain a -> b -> c
    rules.append(A.flow_rule(names[a], 25, strategy=A.STRATEGY_RELATE, ref_resource=names[b]))
    rules.append(A.flow_rule(names[b], 40, strategy=A.STRATEGY_RELATE, ref_resource=names[c]))
    rules.append(A.flow_rule(names[hot[33]], 30, strategy=A.STRATEGY_RELATE, ref_resource=names[hot[33]]))
    rules.append(A.flow_rule(names[hot[34]], 1, strategy=A.STRATEGY_RELATE, ref_resource="never-entered"))
    eng = _engine(max_resources=max(64, w.n_res + 8), max_slot_chain_size=0)
    orc = O.Oracle(max_slot_chain_size=0)
    for x in (eng, orc):
        w.install(x)
        x.load_flow_rules(rules)
    dg, do = _replay(w, eng, orc, 3)
    _assert_same_decisions(dg, do, w.events)
    _compare_nodes(w, eng, orc, np.unique(np.concatenate([_sample(w), np.asarray(hot[:35])])))


@pytest.mark.parametrize("skip_min", ["16", "1000"])
@pytest.mark.parametrize("config", [2, 4])
def test_frozen_skip_hot_resources(config, skip_min, monkeypatch):
    # a few very hot resources: long saturated / breaker-cut stretches that the cooperative kernels
    # skip (stretch end by search, block count sums, pending passes + forward links, k_fill verdicts),
    # with EXITs referencing entries before, inside and after the skipped spans, across batches
    for k, v in {"SG_LANE_MAX": "0", "SG_J1_MAX": "40", "SG_J4_MAX": "2000", "SG_SKIP_MIN": skip_min}.items():
        monkeypatch.setenv(k, v)
    w, eng, orc, d = _run(config, batches=3, n_entries=300_000, n_res=12)
    assert eng.spans_total() > 0  # the skip path ran


def test_duplicate_exits_disable_skipping(monkeypatch):
    # Two EXITs naming the same ENTRY in one batch: the forward-link check (k_link_verify) must flag
    # the batch so the cooperative kernels decide it without frozen-stretch skipping; decisions and
    # node state still equal the oracle's.  A control batch without duplicates does skip.
    for k, v in {"SG_LANE_MAX": "0", "SG_J1_MAX": "40", "SG_J4_MAX": "2000", "SG_SKIP_MIN": "16"}.items():
        monkeypatch.setenv(k, v)
    w = T.Workload(4, n_entries=200_000, n_res=12)
    ev = w.events
    exits = np.nonzero((ev["kind"] == A.EV_EXIT) & ((ev["aux"] & np.uint64(0xFFFFFFFFFFFF)) != np.uint64(0xFFFFFFFFFFFF)))[0]
    rng = np.random.default_rng(11)
    dup = ev[np.sort(rng.choice(exits, 500, replace=False))].copy()
    dup["ts"] = ev["ts"][-1]
    for events, expect_skip in ((ev, True), (np.concatenate([ev, dup]), False)):
        eng = _engine(max_resources=64, max_slot_chain_size=0)
        orc = O.Oracle(max_slot_chain_size=0)
        w.install(eng)
        w.install(orc)
        dg, do = eng.submit(events), orc.submit(events)
        _assert_same_decisions(dg, do, events)
        _compare_nodes(w, eng, orc, range(w.n_res))
        assert (eng.spans_total() > 0) == expect_skip
