"""The cooperative hot-parameter owner (sentinel_amd/csrc/param.hip k_pq) against the oracle.

k_pq decides the segments of resources whose rules are ParamFlowRules (PF_PQ: QPS-grade rules, at most one
THREAD-grade rule on paramIdx 0 checked last) a tile at a time: LRU residency of the CacheMaps from recency ranks,
one lane per value group through the token bucket / throttle / thread count, the thread-count map's increments
and exit(count, args) releases (with removals: a no-eviction hypothesis checked per tile, else a sequential
replay), statistics per 500 ms bucket.  These tests replay traces in which every such segment goes through it
(batches without sg_submit_ex context) and compare every decision and the ClusterNode windows with the
event-sequential oracle (ParamFlowChecker.java:101-248, ParameterMetric.java:37-241, StatisticSlot.java:54-173).
"""
import numpy as np
import pytest

import pyoracle as O
from sentinel_amd import _abi as A
from sentinel_amd import engine as E
from sentinel_amd import tracegen as T

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


def _check(w, eng, orc, cuts, k_nodes=200):
    ev = w.events
    for a, b in zip(cuts[:-1], cuts[1:]):
        dg, do = eng.submit(ev[a:b]), orc.submit(ev[a:b])
        bad = np.nonzero(dg != do)[0]
        assert not len(bad), ("event", int(a + bad[0]), ev[a + bad[0]], hex(dg[bad[0]]), hex(do[bad[0]]), len(bad))
    cnt = np.bincount(ev["res_id"], minlength=w.n_res)
    hot = np.argsort(-cnt)[:40]
    rnd = np.random.default_rng(1).choice(np.nonzero(cnt)[0], size=min(k_nodes, int((cnt > 0).sum())), replace=False)
    for r in np.unique(np.concatenate([hot, rnd])):
        g, o = eng.read_node(int(r)), orc.read_node(int(r))
        assert g["thread"] == o["thread"], r
        np.testing.assert_array_equal(g["second"][:2], o["second"][:2], err_msg="second window of res %d" % r)
        np.testing.assert_array_equal(g["minute"], o["minute"], err_msg="minute window of res %d" % r)


def test_pq_c5_survey_shape():
    # SURVEY.md §8(d) C5 as tools/config_bench.py runs it: 10k resources, one param rule each (count 5-50, burst
    # 0-5, 1 s, 20 % throttle with maxQueue 100, a fifth THREAD grade), hot items, values Zipf(1.1) over 10M keys
    # plus 50 % uniform, every EXIT releasing its argument; two batches of 2^23 events.  Every hot map fills and
    # evicts.
    w = T.Workload(5, n_res=10_000, n_entries=1 << 23, n_param_values=10_000_000,
                   variant=T.V_HOT | T.V_UNIFORM | T.V_THREAD)
    ev = w.events
    eng = E.Engine(max_resources=w.n_res, max_slot_chain_size=0, param_table_log2=28, status_ring_log2=26,
                   max_batch_events=1 << 23)
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(eng)
    w.install(orc)
    _check(w, eng, orc, [0, 1 << 23, len(ev)])


@pytest.mark.parametrize("pvpq", ["0", "1"])
@pytest.mark.parametrize("wide", ["0", "1073741824"])
@pytest.mark.parametrize("variant", ["hot", "uniform", "thread"])
def test_pq_variants(variant, wide, pvpq, monkeypatch):
    # hot items (per-value token counts, some 0: blocked without a map access), uniform churn (a million
    # distinct values), THREAD-grade rules with exits releasing their argument; every segment on the 1024-lane
    # owner (wide=0) or on the 256-lane one.  pvpq = 1: the long segments of one-rule resources (token bucket or
    # throttle) through the value-parallel passes, k_pvf folding their statistics (XF_PVPQ)
    monkeypatch.setenv("SG_PQ_WIDE", wide)
    monkeypatch.setenv("SG_PV_PQ", pvpq)
    v = {"hot": T.V_HOT, "uniform": T.V_HOT | T.V_UNIFORM, "thread": T.V_HOT | T.V_UNIFORM | T.V_THREAD}[variant]
    w = T.Workload(5, n_res=2_000, n_entries=600_000, n_param_values=2_000_000, variant=v)
    eng = E.Engine(max_resources=w.n_res, max_slot_chain_size=0, param_table_log2=26, status_ring_log2=24)
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(eng)
    w.install(orc)
    _check(w, eng, orc, np.linspace(0, len(w.events), 4).astype(np.int64))
    if pvpq == "1":
        st = eng.pv_last()
        assert st["segments"] > 0 and st["accesses"] > 10_000 and st["post_done"] > 0, st


def _rules(thread_on_m3=False):
    r = [
        # two checked rules on index 0 (token bucket with burst, then a throttle), hot items incl. a zero count
        A.param_rule("m0", 0, 3, burst_count=2, items=[("7", "long", 0), ("8", "long", 50)]),
        A.param_rule("m0", 0, 20, control_behavior=A.CONTROL_BEHAVIOR_RATE_LIMITER, max_queueing_time_ms=40),
        # a rule on index 1 (an argument the events never carry: no check, its thread map exists)
        A.param_rule("m0", 1, 1),
        # cluster mode without fallback: initialised, never checked
        A.param_rule("m1", 0, 1, cluster_mode=True, cluster_flow_id=77),
        A.param_rule("m1", 0, 2),
        A.param_rule("m2", 0, 1, burst_count=1),
        # THREAD grade alone (hot items: a zero and a large threshold)
        A.param_rule("m4", 0, 2, grade=A.FLOW_GRADE_THREAD, items=[("3", "long", 0), ("4", "long", 40)]),
        # QPS only: its thread-count map is kept by the releases and read once a THREAD rule arrives
        A.param_rule("m3", 0, 30, burst_count=3),
    ]
    if thread_on_m3:
        r.append(A.param_rule("m3", 0, 3, grade=A.FLOW_GRADE_THREAD))
    return r


NAMES = ("m0", "m1", "m2", "m3", "m4")


def _synthetic(seed, n, gbase, nres=5, nval=9000, t=T0, rt_max=30, exit_args=0.0):
    # EXIT references name the ENTRY's global event index (batches are numbered consecutively); a fraction
    # exit_args of the EXITs release their ENTRY's argument (Entry.exit(count, args))
    rng = np.random.default_rng(seed)
    ev = np.zeros(2 * n, dtype=A.EVENT_DTYPE)
    ts = t + np.sort(rng.integers(0, 6000, n))
    k = 0
    pend = []

    def put_exit(tx, ref, rid):
        nonlocal k
        fl = A.F_EXIT_ARGS if rng.random() < exit_args else 0
        ev[k] = (tx, rid, 1, A.EV_EXIT, fl, A.aux_exit(ref, 3))
        k += 1

    for i in range(n):
        while pend and pend[0][0] <= ts[i]:
            put_exit(*pend.pop(0))
        rid = int(rng.integers(0, nres))
        v = int(rng.zipf(1.3)) if rng.random() < 0.6 else int(rng.integers(0, nval))
        flags = A.F_HAS_ARG if rng.random() < 0.97 else 0
        cnt = int(rng.choice([1, 1, 1, 2, 0, 6]))
        ev[k] = (ts[i], rid, cnt, A.EV_ENTRY, flags, E.param_key(str(v), "long"))
        if rng.random() < 0.5:
            pend.append((int(ts[i]) + int(rng.integers(0, rt_max)), gbase + k, rid))
            pend.sort()
        k += 1
    for x in pend:
        put_exit(*x)
    return ev[:k]


def _compare(eng, orc, ev, via_ext, what):
    if via_ext:  # sg_submit_ex (an all-zero context/args table): the batch is the per-lane kernel's
        ext = np.zeros(len(ev), dtype=A.EXT_DTYPE)
        dg, do = eng.submit_ex(ev, ext), orc.submit_ex(ev, ext)
    else:
        dg, do = eng.submit(ev), orc.submit(ev)
    bad = np.nonzero(dg != do)[0]
    assert not len(bad), (what, "event", int(bad[0]), ev[bad[0]], hex(dg[bad[0]]), hex(do[bad[0]]), len(bad))
    return dg


@pytest.mark.parametrize("rt_max", [30, 3000])
def test_pq_rule_mix_thread_maps_and_alternating_paths(rt_max):
    # several param rules per resource, hot items, entries without an argument, zero and oversized acquires,
    # > 4000 distinct values per resource (evictions inside and across tiles), exits releasing their argument;
    # with rt_max = 3000 ms about 5000 values per resource are held at once, so the thread-count maps overflow
    # while exits remove keys (the sequential replay).  Batches alternate between k_pq and the per-lane kernel
    # (sg_submit_ex); both work on the same maps.  Then a THREAD rule is added on m3 and reads the thread-count
    # map that m3's releases kept.
    eng = E.Engine(max_resources=64, max_slot_chain_size=0, param_table_log2=20, status_ring_log2=24)
    orc = O.Oracle(max_slot_chain_size=0)
    for nm in NAMES:
        assert eng.register(nm) == orc.register(nm)
    rules = _rules()
    assert eng.load_param_rules(rules) == orc.load_param_rules(rules)
    t, gbase = T0, 0
    for b in range(7):
        if b == 5:
            rules = _rules(thread_on_m3=True)
            assert eng.load_param_rules(rules) == orc.load_param_rules(rules)
        ev = _synthetic(100 + b, 40_000, gbase, t=t, rt_max=rt_max, exit_args=0.9)
        gbase += len(ev)
        d = _compare(eng, orc, ev, b % 3 == 1, "batch %d" % b)
        if b >= 5:  # the THREAD rule on m3 blocks some of its entries
            m3 = (ev["kind"] == A.EV_ENTRY) & (ev["res_id"] == NAMES.index("m3"))
            assert int(((d[m3] & 0xFF) == A.BLOCK_PARAM).sum()) > 0
        t = int(ev["ts"].max()) + 1
    for r in range(len(NAMES)):
        g, o = eng.read_node(r), orc.read_node(r)
        assert g["thread"] == o["thread"]
        np.testing.assert_array_equal(g["second"][:2], o["second"][:2])
        np.testing.assert_array_equal(g["minute"], o["minute"])


def _ext_args(ev, io, ic, seed, list_res_mod=7):
    """The C5 trace as the Java drop-in sends it (sg_submit_ex): contexts / origins on every event, args[0] from the
    table (a few nulls; Collections on the resources res % list_res_mod == 0 now and then: those resources turn to
    the per-lane kernel), and half of the releasing EXITs with args of their own (Entry.exit(count, args): mostly
    the ENTRY's value, sometimes another one)."""
    rng = np.random.default_rng(seed)
    n = len(ev)
    ext = T.ext_for(ev, io, ic, seed)
    ent = ev["kind"] == A.EV_ENTRY
    ext_rows = np.zeros(n, dtype=A.ARG_DTYPE)
    ext_rows["key"] = ev["aux"]
    ext_rows["kind"] = A.ARG_SCALAR
    u = rng.random(n)
    ext_rows["kind"][ent & (u < 0.03)] = A.ARG_NULL
    lst = ent & (u >= 0.03) & (u < 0.05) & (ev["res_id"] % list_res_mod == 0)
    li = np.nonzero(lst)[0]
    extra = np.zeros(2 * len(li), dtype=A.ARG_DTYPE)
    extra["kind"] = A.ARG_SCALAR
    extra["key"][0::2] = ev["aux"][li]
    extra["key"][1::2] = ev["aux"][rng.integers(0, n, len(li))]
    ext_rows["kind"][li] = A.ARG_LIST
    ext_rows["key"][li] = n + 2 * np.arange(len(li), dtype=np.uint64)
    ext_rows["len"][li] = 2
    # EXITs releasing with their own args
    ref = (ev["aux"] & np.uint64(A.REF_NONE)).astype(np.int64)
    own = (ev["kind"] == A.EV_EXIT) & ((ev["flags"] & A.F_EXIT_ARGS) != 0) & (rng.random(n) < 0.5) & (ref < n)
    oi = np.nonzero(own)[0]
    ext_rows["key"][oi] = np.where(rng.random(len(oi)) < 0.9, ev["aux"][ref[oi]], ev["aux"][rng.integers(0, n, len(oi))])
    ext_rows["kind"][oi] = np.where(ent[ref[oi]], A.ARG_SCALAR, A.ARG_NULL)
    ext["arg_off"] = np.arange(n, dtype=np.uint32)
    ext["n_args"] = (ent | own).astype(np.uint32)
    return ext, np.concatenate([ext_rows, extra])


@pytest.mark.parametrize("variant", ["hot", "uniform", "thread"])
def test_pq_ext_args_contexts(variant):
    # VERDICT r3 missing #1: k_pq takes sg_submit_ex batches (args[0] from the table via the key ring; EXITs with
    # their own args), the aux post-pass updates the origin / context nodes of its segments
    v = {"hot": T.V_HOT, "uniform": T.V_HOT | T.V_UNIFORM, "thread": T.V_HOT | T.V_UNIFORM | T.V_THREAD}[variant]
    w = T.Workload(5, n_res=2_000, n_entries=600_000, n_param_values=2_000_000, variant=v)
    ev = w.events
    eng = E.Engine(max_resources=w.n_res, max_slot_chain_size=0, param_table_log2=26, status_ring_log2=24,
                   aux_node_capacity=1 << 16)
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(eng)
    w.install(orc)
    io, ic = w.intern_names(eng)
    assert all(np.array_equal(a, b) for a, b in zip((io, ic), w.intern_names(orc)))
    ext, table = _ext_args(ev, io, ic, seed=17)
    cuts = np.linspace(0, len(ev), 4).astype(np.int64)
    for a, b in zip(cuts[:-1], cuts[1:]):  # one table for the whole trace: arg_off stays global
        dg, do = eng.submit_ex(ev[a:b], ext[a:b], table), orc.submit_ex(ev[a:b], ext[a:b], table)
        bad = np.nonzero(dg != do)[0]
        assert not len(bad), ("event", int(a + bad[0]), ev[a + bad[0]], hex(dg[bad[0]]), hex(do[bad[0]]), len(bad))
    cnt = np.bincount(ev["res_id"], minlength=w.n_res)
    for r in np.unique(np.concatenate([np.argsort(-cnt)[:40], np.random.default_rng(2).choice(w.n_res, 100)])):
        g, o = eng.read_node(int(r)), orc.read_node(int(r))
        assert g["thread"] == o["thread"], r
        np.testing.assert_array_equal(g["second"][:2], o["second"][:2], err_msg="second window of res %d" % r)
        np.testing.assert_array_equal(g["minute"], o["minute"], err_msg="minute window of res %d" % r)
        for k, nm in enumerate(["app-%d" % i for i in range(16)]):
            ga, oa = eng.read_aux_node(int(r), 0, int(io[k])), orc.read_origin_node(int(r), nm)
            if oa is None:
                continue
            assert ga is not None and ga["thread"] == oa["thread"], (r, nm)
            np.testing.assert_array_equal(ga["second"], oa["second"][:2], err_msg="origin node %d/%s" % (r, nm))


@pytest.mark.parametrize("wide", ["0", "1073741824"])
def test_pq_duration_two_maps(wide, monkeypatch):
    # durationInSec = 2: CacheMaps of min(4000 * 2, 200000) = 8000 values (ParameterMetric.java:37-39), a 2^15-bit
    # live-stamp ring in k_pq's LDS; > 8000 distinct values per resource so the maps fill and evict, exits releasing
    # their argument; on the 1024-lane (wide=0) and the 256-lane owner
    monkeypatch.setenv("SG_PQ_WIDE", wide)
    eng = E.Engine(max_resources=64, max_slot_chain_size=0, param_table_log2=22, status_ring_log2=24)
    orc = O.Oracle(max_slot_chain_size=0)
    for nm in NAMES:
        assert eng.register(nm) == orc.register(nm)
    rules = [A.param_rule("m0", 0, 3, duration_in_sec=2, burst_count=2),
             A.param_rule("m1", 0, 2, duration_in_sec=2),
             A.param_rule("m1", 0, 9, duration_in_sec=1),
             A.param_rule("m2", 0, 5, duration_in_sec=2, control_behavior=A.CONTROL_BEHAVIOR_RATE_LIMITER,
                          max_queueing_time_ms=30),
             A.param_rule("m3", 0, 4, duration_in_sec=3)]  # 12000 values: beyond k_pq's rings, the per-lane kernel
    assert eng.load_param_rules(rules) == orc.load_param_rules(rules)
    t, gbase = T0, 0
    for b in range(4):
        ev = _synthetic(300 + b, 60_000, gbase, nres=4, nval=30_000, t=t, exit_args=0.5)
        gbase += len(ev)
        d = _compare(eng, orc, ev, False, "batch %d" % b)
        t = int(ev["ts"].max()) + 1
    assert int(((d & 0xFF) == A.BLOCK_PARAM).sum()) > 0
    for r in range(4):
        g, o = eng.read_node(r), orc.read_node(r)
        assert g["thread"] == o["thread"]
        np.testing.assert_array_equal(g["second"][:2], o["second"][:2])
