"""sg_submit_ex on the device against the oracle: the full ProcessorSlot.entry signature.

ProcessorSlot.entry(Context, ResourceWrapper, node, count, prioritized, Object... args)
(core/slotchain/ProcessorSlot.java:41-50) carries the Context -- name and origin -- and every argument.
These tests replay seeded traces whose events carry origins, context names and argument lists through
sg_submit_ex and through the oracle's or_submit_ex, and require bit-identical decisions and ClusterNode
state:

* FlowRuleChecker.selectNodeByRequesterAndStrategy (core/slots/block/flow/FlowRuleChecker.java:90-124):
  limitApp = an origin and "other" rules on the origin's StatisticNode, STRATEGY_CHAIN rules on the
  DefaultNode of the named context, with DefaultController / WarmUp / RateLimiter controllers and
  prioritized entries on those nodes;
* ParamFlowSlot.checkFlow / applyRealParamIdx (param/.../ParamFlowSlot.java:65-101): paramIdx 1, 2, -1,
  resolved once per rule; Collection/array values checked element by element, null elements
  (ParamFlowChecker.java:48-99); THREAD-grade maps per index, released by Entry.exit(count, args);
* caller-side System/Authority blocks between ParamFlowSlot and FlowSlot (SG_F_BLOCKED_UPSTREAM);
* NullContext past Constants.MAX_CONTEXT_NAME_SIZE (CtSph.java:120-127).
"""
import numpy as np
import pytest

import pyoracle as O
from sentinel_amd import _abi as A
from sentinel_amd import engine as E

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000
ORIGINS = ["appA", "appB", "appC", "appD"]   # appD is named by no rule ("other")
CONTEXTS = ["ctxA", "ctxB", "ctxC"]


def _rules(n_res):
    flow, param, deg = [], [], []
    for i in range(n_res):
        nm = "r%d" % i
        k = i % 6
        if k == 0:  # strategy 3 is a valid rule whose node is never selected: it always passes
            flow += [A.flow_rule(nm, 25), A.flow_rule(nm, 1, strategy=3, ref_resource="ctxA")]
        elif k == 1:
            flow += [A.flow_rule(nm, 4, limit_app="appA"), A.flow_rule(nm, 30)]
        elif k == 2:
            flow += [A.flow_rule(nm, 3, limit_app="other"), A.flow_rule(nm, 2, limit_app="appB",
                                                                        grade=A.FLOW_GRADE_THREAD)]
            if i % 12 == 2:  # a cluster-only rule checks nothing but still names appC: not "other"
                flow.append(A.flow_rule(nm, 1, limit_app="appC", cluster_mode=True, cluster_flow_id=2000 + i,
                                        cluster_fallback_to_local=False))
        elif k == 3:
            flow += [A.flow_rule(nm, 5, strategy=A.STRATEGY_CHAIN, ref_resource="ctxA"),
                     A.flow_rule(nm, 8, limit_app="appA", strategy=A.STRATEGY_CHAIN, ref_resource="ctxB",
                                 control_behavior=A.CONTROL_BEHAVIOR_WARM_UP, warm_up_period_sec=2)]
        elif k == 4:
            flow += [A.flow_rule(nm, 10, limit_app="appC", control_behavior=A.CONTROL_BEHAVIOR_WARM_UP,
                                 warm_up_period_sec=3),
                     A.flow_rule(nm, 20, control_behavior=A.CONTROL_BEHAVIOR_RATE_LIMITER, max_queueing_time_ms=300)]
        else:
            flow += [A.flow_rule(nm, 6, limit_app="other", strategy=A.STRATEGY_CHAIN, ref_resource="sentinel_default_context"),
                     A.flow_rule(nm, 15)]
        j = i % 4
        if j == 0:
            param.append(A.param_rule(nm, 0, 3, burst_count=1))
        elif j == 1:
            param += [A.param_rule(nm, 1, 2, grade=A.FLOW_GRADE_THREAD), A.param_rule(nm, -1, 4)]
        elif j == 2:
            param += [A.param_rule(nm, 2, 5, control_behavior=A.CONTROL_BEHAVIOR_RATE_LIMITER, max_queueing_time_ms=200),
                      A.param_rule(nm, 0, 1, cluster_mode=True, cluster_flow_id=1000 + i,
                                   cluster_fallback_to_local=False)]
        if i % 5 == 0:
            deg.append(A.degrade_rule(nm, 30, 2))
    return flow, param, deg


def _trace(seed, n_res, n_entries, ids_o, ids_c, null_ctx=None):
    """Events + ext/args tables.  ids_o / ids_c: interned ids of ORIGINS / CONTEXTS (same on both sides)."""
    rng = np.random.default_rng(seed)
    vals = [O.param_key("v%d" % v) for v in range(10)]

    def one_arg():
        u = rng.random()
        if u < 0.12:
            return None
        if u < 0.35:
            return [None if rng.random() < 0.1 else vals[int(rng.integers(0, 10))] for _ in range(int(rng.integers(1, 4)))]
        return vals[int(rng.integers(0, 10))]

    raw = []  # (t, order, kind, res, entry_no, flags, rt)
    t = 0.0
    entries = []
    for n in range(n_entries):
        t += rng.exponential(3.0)
        ms = int(t)
        res = int(rng.integers(0, n_res))
        o = int(rng.integers(0, len(ORIGINS) + 1))
        c = int(rng.integers(0, len(CONTEXTS) + 1))
        args = [one_arg() for _ in range(int(rng.integers(0, 4)))]
        fl = 0
        if rng.random() < 0.04:
            fl |= A.F_BLOCKED_UPSTREAM
        if rng.random() < 0.06:
            fl |= A.F_PRIORITIZED
        origin = 0 if o == 0 else ids_o[o - 1]
        ctx = 0 if c == 0 else ids_c[c - 1]
        if null_ctx is not None and rng.random() < 0.05:
            ctx = null_ctx
        entries.append((res, origin, ctx, args))
        raw.append((ms, 0, A.EV_ENTRY, res, n, fl, 0))
        rt = int(rng.exponential(25.0))
        if rng.random() < 0.05:
            raw.append((ms + rt, 1, A.EV_TRACE, res, n, 0, 0))
        xf = A.F_EXIT_ARGS if rng.random() < 0.6 else 0
        raw.append((ms + rt, 2, A.EV_EXIT, res, n, xf, rt))
    raw.sort(key=lambda r: (r[0], r[1]))
    ev = np.zeros(len(raw), dtype=A.EVENT_DTYPE)
    args_of, origin, context = {}, np.zeros(len(raw), np.uint32), np.zeros(len(raw), np.uint32)
    pos_of_entry = {}
    for i, (ms, _, kind, res, n, fl, rt) in enumerate(raw):
        r, o, c, args = entries[n]
        ev[i] = (T0 + ms, res, 1, kind, fl, 0)
        origin[i], context[i] = o, c
        if kind == A.EV_ENTRY:
            pos_of_entry[n] = i
            if args:
                args_of[i] = args
        else:
            ref = pos_of_entry[n]
            ev["aux"][i] = A.aux_exit(ref, rt) if kind == A.EV_EXIT else ref
            if kind == A.EV_EXIT and (fl & A.F_EXIT_ARGS) and args and n % 2 == 0:
                args_of[i] = args  # Entry.exit(count, args) with the entry's args; else the ENTRY's args[0]
    ext, table = A.ext_tables(len(ev), args_of, origin, context)
    return ev, ext, table


def _pair(n_res, intern_first=True, null_ctx=False, **cfg):
    eng = E.Engine(max_resources=max(64, n_res), max_slot_chain_size=0, status_ring_log2=22, **cfg)
    orc = O.Oracle(max_slot_chain_size=0)
    names = ["r%d" % i for i in range(n_res)]
    ids = []

    def intern():
        io = [eng.intern_origin(o) for o in ORIGINS]
        ic = [eng.intern_context(c) for c in CONTEXTS]
        assert io == [orc.intern_origin(o) for o in ORIGINS] and ic == [orc.intern_context(c) for c in CONTEXTS]
        ids[:] = [io, ic]

    if intern_first:
        intern()
    flow, param, deg = _rules(n_res)
    for x in (eng, orc):
        for nm in names:
            x.register(nm)
        x.load_flow_rules(flow)
        x.load_param_rules(param)
        x.load_degrade_rules(deg)
    if not intern_first:  # names interned after the rules that read them: the programs are recompiled
        intern()
    nc = None
    if null_ctx:
        for k in range(A.MAX_CONTEXTS + 1 - len(CONTEXTS)):
            a, b = eng.intern_context("filler%d" % k), orc.intern_context("filler%d" % k)
            assert a == b
        nc = a
        assert nc == A.MAX_CONTEXTS + 1
    return eng, orc, ids[0], ids[1], nc


def _replay(eng, orc, ev, ext, table, batches):
    cuts = np.linspace(0, len(ev), batches + 1).astype(np.int64)
    dg, do = [], []
    for a, b in zip(cuts[:-1], cuts[1:]):
        sub = {}
        # each batch carries its own args table: re-base the ext offsets of the slice
        e2 = ext[a:b].copy()
        rows = []
        for i in range(b - a):
            n = int(e2["n_args"][i])
            if n:
                off = int(e2["arg_off"][i])
                e2["arg_off"][i] = len(rows)
                base = len(rows)
                rows.extend(table[off:off + n].tolist())
                for j in range(n):
                    if table[off + j]["kind"] == A.ARG_LIST:
                        lo, ln = int(table[off + j]["key"]), int(table[off + j]["len"])
                        rows[base + j] = (len(rows), A.ARG_LIST, ln)
                        rows.extend(table[lo:lo + ln].tolist())
        t2 = np.array(rows, dtype=A.ARG_DTYPE) if rows else np.zeros(0, dtype=A.ARG_DTYPE)
        dg.append(eng.submit_ex(ev[a:b], e2, t2))
        do.append(orc.submit_ex(ev[a:b], e2, t2))
    return np.concatenate(dg), np.concatenate(do)


def _check(eng, orc, ev, dg, do, n_res):
    bad = np.nonzero(dg != do)[0]
    assert len(bad) == 0, "decision mismatch at event %d (%s): gpu=%08x oracle=%08x; %d mismatches" % (
        bad[0], ev[bad[0]], dg[bad[0]], do[bad[0]], len(bad))
    for r in range(n_res):
        g, o = eng.read_node(r), orc.read_node(r)
        assert g["thread"] == o["thread"], (r, g["thread"], o["thread"])
        np.testing.assert_array_equal(g["second"][:2], o["second"][:2], err_msg="second window of res %d" % r)
        np.testing.assert_array_equal(g["minute"], o["minute"], err_msg="minute window of res %d" % r)


@pytest.mark.parametrize("intern_first,group", [(True, "default"), (False, "default"), (True, "hot_cold")])
def test_origin_context_args_parity(intern_first, group, monkeypatch):
    if group == "hot_cold":  # (these batches are below SG_RADIX_BELOW: the hot / cold stage's argument checks too)
        monkeypatch.setenv("SG_RADIX_BELOW", "0")
    n_res = 36
    eng, orc, io, ic, _ = _pair(n_res, intern_first)
    ev, ext, table = _trace(7, n_res, 12_000, io, ic)
    dg, do = _replay(eng, orc, ev, ext, table, 3)
    _check(eng, orc, ev, dg, do, n_res)
    st = dg[ev["kind"] == A.EV_ENTRY] & 0xFF
    for s in (A.PASS, A.PASS_WAIT, A.BLOCK_FLOW, A.BLOCK_PARAM, A.BLOCK_UPSTREAM):
        assert (st == s).sum() > 0, s


def test_null_context_parity():
    n_res = 24
    eng, orc, io, ic, nc = _pair(n_res, True, null_ctx=True)
    ev, ext, table = _trace(11, n_res, 6_000, io, ic, null_ctx=nc)
    dg, do = _replay(eng, orc, ev, ext, table, 2)
    _check(eng, orc, ev, dg, do, n_res)
    st = dg[(ev["kind"] == A.EV_ENTRY) & (ext["context_id"] == nc)] & 0xFF
    assert len(st) and (st == A.NO_CHECK).all()


def test_bad_args_table_is_rejected():
    eng = E.Engine(max_resources=64, max_slot_chain_size=0)
    eng.register("r")
    ev = np.zeros(1, dtype=A.EVENT_DTYPE)
    ev["ts"], ev["kind"], ev["count"] = T0, A.EV_ENTRY, 1
    ext = np.zeros(1, dtype=A.EXT_DTYPE)
    ext["n_args"], ext["arg_off"] = 2, 1
    table = np.zeros(2, dtype=A.ARG_DTYPE)
    with pytest.raises(E.SentinelError) as ei:
        eng.submit_ex(ev, ext, table)
    assert ei.value.code == A.SG_EINVAL
    table["kind"][0] = A.ARG_LIST
    table["key"][0], table["len"][0] = 1, 5  # a list running past the table
    ext["arg_off"], ext["n_args"] = 0, 1
    with pytest.raises(E.SentinelError):
        eng.submit_ex(ev, ext, table)
    ext["n_args"] = 0
    assert (eng.submit_ex(ev, ext, table)[0] & 0xFF) == A.PASS  # the engine is still usable


def test_rule_reload_with_entries_in_flight():
    # origin nodes and DefaultNodes are kept for every entry whatever the rules, so origin / CHAIN rules
    # loaded or removed while entries are in flight see the same node history as the reference
    # (ClusterBuilderSlot.java:74-99, NodeSelectorSlot.java:134-176): no thread count leaks or goes negative
    n_res = 36
    eng = E.Engine(max_resources=64, max_slot_chain_size=0, status_ring_log2=22)
    orc = O.Oracle(max_slot_chain_size=0)
    io = [eng.intern_origin(o) for o in ORIGINS]
    ic = [eng.intern_context(c) for c in CONTEXTS]
    assert io == [orc.intern_origin(o) for o in ORIGINS] and ic == [orc.intern_context(c) for c in CONTEXTS]
    for x in (eng, orc):
        for i in range(n_res):
            x.register("r%d" % i)
    flow, param, deg = _rules(n_res)
    plain = [A.flow_rule("r%d" % i, 12) for i in range(n_res)]
    ev, ext, table = _trace(23, n_res, 9_000, io, ic)
    cuts = np.linspace(0, len(ev), 4).astype(np.int64)
    stages = [plain, flow, plain]  # origin / CHAIN rules arrive after batch 1 and leave after batch 2
    dg, do = [], []
    for k, (a, b) in enumerate(zip(cuts[:-1], cuts[1:])):
        for x in (eng, orc):
            x.load_flow_rules(stages[k])
            if k == 1:
                x.load_param_rules(param)
                x.load_degrade_rules(deg)
        g, o = _replay(eng, orc, ev[a:b], ext[a:b], table, 1)
        dg.append(g)
        do.append(o)
    _check(eng, orc, ev, np.concatenate(dg), np.concatenate(do), n_res)
