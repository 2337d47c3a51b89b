"""Oracle pinned against the reference's own deterministic known-answer tests.

Each test transcribes one reference JUnit test (file:line under
/root/reference, prefixes as in SURVEY.md §0.1: core-test/ =
sentinel-core/src/test/java/com/alibaba/csp/sentinel/, param-test/ =
sentinel-extension/sentinel-parameter-flow-control/src/test/java/com/alibaba/csp/sentinel/,
csrv-test/ = sentinel-cluster/sentinel-cluster-server-default/src/test/java/com/alibaba/csp/sentinel/cluster/).
Mocked TimeUtil values become explicit event times; mocked Node getters become
the oracle's unit-level hooks, exactly as the Java tests mock them.
"""
import pytest

import pyoracle as O
from sentinel_amd import _abi as A

T0 = 1_700_000_000_123  # stands in for System.currentTimeMillis() in the Java tests


# ---------------------------------------------------------------- controllers
def test_default_controller_qps():
    # core-test/slots/block/flow/controller/DefaultControllerTest.java:18-29
    c = O.Controller(A.CONTROL_BEHAVIOR_DEFAULT, 10, grade=A.FLOW_GRADE_QPS)
    assert c.can_pass(T0, pass_qps=9)[0]
    assert not c.can_pass(T0, pass_qps=10)[0]


def test_default_controller_thread():
    # DefaultControllerTest.java:31-42
    c = O.Controller(A.CONTROL_BEHAVIOR_DEFAULT, 8, grade=A.FLOW_GRADE_THREAD)
    assert c.can_pass(T0, cur_thread=7)[0]
    assert not c.can_pass(T0, cur_thread=8)[0]


def test_warm_up_controller():
    # core-test/slots/block/flow/controller/WarmUpControllerTest.java:34-62
    c = O.Controller(A.CONTROL_BEHAVIOR_WARM_UP, 10, warm_up_period_sec=10, cold_factor=3)
    assert c.state(3) == 50 and c.state(4) == 100  # warningToken, maxToken
    now = T0
    assert not c.can_pass(now, pass_qps=8, prev_pass_qps=1)[0]
    assert c.can_pass(now, pass_qps=1, prev_pass_qps=1)[0]
    for _ in range(100):
        now += 100
        c.can_pass(now, pass_qps=1, prev_pass_qps=10)
    assert c.can_pass(now, pass_qps=8, prev_pass_qps=10)[0]
    assert not c.can_pass(now, pass_qps=10, prev_pass_qps=10)[0]


def test_rate_limiter_zero_attack():
    # core-test/slots/block/flow/controller/RateLimiterControllerTest.java:89-97
    c = O.Controller(A.CONTROL_BEHAVIOR_RATE_LIMITER, 0.0, max_queueing_ms=500)
    for _ in range(2):
        assert not c.can_pass(T0, acquire=1)[0]
        assert c.can_pass(T0, acquire=0)[0]


def test_warm_up_rate_limiter_pace_can_not_pass():
    # core-test/slots/block/flow/controller/WarmUpRateLimiterControllerTest.java:41-51
    c = O.Controller(A.CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER, 10, warm_up_period_sec=10, max_queueing_ms=10,
                     cold_factor=3)
    assert c.can_pass(T0, pass_qps=100, prev_pass_qps=100)[0]
    assert not c.can_pass(T0, pass_qps=100, prev_pass_qps=100)[0]


def test_rate_limiter_queueing_wait_reported():
    # RateLimiterController.canPass (core/slots/block/flow/controller/RateLimiterController.java:46-91):
    # count 10 -> cost 100 ms; the second request queues 100 ms (sleep reported, clock not advanced, Q10).
    c = O.Controller(A.CONTROL_BEHAVIOR_RATE_LIMITER, 10, max_queueing_ms=500)
    assert c.can_pass(T0) == (True, 0)
    assert c.can_pass(T0) == (True, 100)
    assert c.can_pass(T0) == (True, 200)
    assert c.can_pass(T0)[0] and c.can_pass(T0)[0]  # 300, 400
    assert c.can_pass(T0) == (True, 500)
    assert not c.can_pass(T0)[0]  # 600 > 500


# ---------------------------------------------------------------- degrade
def test_degrade_average_rt():
    # core-test/slots/block/degrade/DegradeTest.java:40-66 (the 2.2 s wall sleep becomes trace time)
    d = O.Degrade(A.DEGRADE_GRADE_RT, 1, 2)
    for _ in range(4):
        assert d.pass_check(T0, avg_rt=2)
    assert not d.pass_check(T0, avg_rt=2)
    assert not d.pass_check(T0, avg_rt=2)
    assert d.pass_check(T0 + 2200, avg_rt=2)


def test_degrade_exception_ratio():
    # DegradeTest.java:68-98
    d = O.Degrade(A.DEGRADE_GRADE_EXCEPTION_RATIO, 0.15, 2)
    assert not d.pass_check(T0, exception_qps=2, total_qps=12, success_qps=8)
    assert d.pass_check(T0 + 2200, exception_qps=2, total_qps=12, success_qps=20)


def test_degrade_exception_count():
    # DegradeTest.java:100-127
    d = O.Degrade(A.DEGRADE_GRADE_EXCEPTION_COUNT, 4, 2)
    assert not d.pass_check(T0, total_exception=4)
    assert d.pass_check(T0 + 2200, total_exception=0)


# ---------------------------------------------------------------- leap arrays
def test_bucket_leap_array_new_window():
    # core-test/slots/statistic/metric/BucketLeapArrayTest.java:45-55
    a = O.Leap(O.LEAP_PLAIN, 2, 2000)
    slot, ws = a.current(T0)
    assert ws == T0 - T0 % 1000 and a.get(slot, O.EV_PASS) == 0


def test_bucket_leap_array_window_after_one_interval():
    # BucketLeapArrayTest.java:69-101
    a = O.Leap(O.LEAP_PLAIN, 2, 2000)
    ws0 = T0 - T0 % 1000
    slot, ws = a.current(ws0)
    assert ws == ws0
    a.add(ws0, O.EV_PASS, 1)
    a.add(ws0, O.EV_BLOCK, 1)
    mid = ws0 + 500
    s2, w2 = a.current(mid)
    assert (s2, w2) == (slot, ws0)
    a.add(mid, O.EV_PASS, 1)
    assert a.get(slot, O.EV_PASS) == 2 and a.get(slot, O.EV_BLOCK) == 1
    s3, w3 = a.current(mid + 500)
    assert w3 - ws0 == 1000
    assert a.get(s3, O.EV_PASS) == 0 and a.get(s3, O.EV_BLOCK) == 0


def test_bucket_leap_array_previous_window():
    # BucketLeapArrayTest.java:151-163
    a = O.Leap(O.LEAP_PLAIN, 2, 2000)
    slot, _ = a.current(T0)
    assert a.previous(T0)[0] == -1
    assert a.previous(T0 + 1000)[0] == slot
    assert a.previous(T0 + 11 * 1000)[0] == -1


def test_bucket_leap_array_list_reset_old():
    # BucketLeapArrayTest.java:165-188 (Thread.sleep -> trace time)
    a = O.Leap(O.LEAP_PLAIN, 10, 1000)
    a.current(T0)
    a.current(T0 + 100)
    assert a.values_count(T0) == 2
    a.add(T0 + 100 + 1000, O.EV_PASS, 1)
    assert a.values_count(T0 + 100 + 1000) == 1


def test_bucket_leap_array_list_new_bucket():
    # BucketLeapArrayTest.java:190-216
    a = O.Leap(O.LEAP_PLAIN, 10, 1000)
    a.current(T0)
    a.current(T0 + 100)
    now = T0 + 1000 + 300
    assert a.values_count(now) == 0
    a.add(now, O.EV_PASS, 1)
    assert a.values_count(now) == 1


def test_occupiable_new_window():
    # core-test/slots/statistic/metric/OccupiableBucketLeapArrayTest.java:29-42
    a = O.Leap(O.LEAP_OCCUPIABLE, 10, 2000)
    slot = a.add(T0, O.EV_PASS, 1)
    assert a.get(slot, O.EV_PASS) == 1
    a.add_waiting(T0 + 200, 1)
    assert a.current_waiting(T0) == 1
    assert a.get(slot, O.EV_PASS) == 1


def test_occupiable_window_in_one_interval():
    # OccupiableBucketLeapArrayTest.java:44-66
    a = O.Leap(O.LEAP_OCCUPIABLE, 10, 2000)
    slot = a.add(T0, O.EV_PASS, 1)
    a.add_waiting(T0 + 200, 2)
    assert a.current_waiting(T0) == 2
    assert a.get(slot, O.EV_PASS) == 1
    a.current(T0 + 200)
    assert a.values_count(T0 + 200) == 2
    assert a.values_sum(T0 + 200, O.EV_PASS) == 3


def test_occupiable_window_after_one_interval():
    # OccupiableBucketLeapArrayTest.java:104-137
    a = O.Leap(O.LEAP_OCCUPIABLE, 10, 2000)
    for i in range(10):
        a.add(T0 + i * 200, O.EV_PASS, 1)
        a.add_waiting(T0 + (i + 1) * 200, 1)
    t = T0 - T0 % 200 + 2000
    assert a.values_count(t) == 10
    assert a.values_sum(t, O.EV_PASS) == 2 * 10 - 1
    assert a.current_waiting(T0) == 10


def test_future_bucket_leap_array():
    # core-test/slots/statistic/metric/FutureBucketLeapArrayTest.java:23-31
    a = O.Leap(O.LEAP_FUTURE, 10, 2000)
    for i in range(0, 2000, 200):
        a.add(T0 + i, O.EV_PASS, 1)
        assert a.values_count(T0 + i) == 0


def test_leap_array_valid_head():
    # core-test/slots/statistic/base/LeapArrayTest.java:32-63 (mocked clock starts at 0)
    a = O.Leap(O.LEAP_PLAIN, 10, 1000)
    now = 0
    e1 = a.add(now, O.EV_PASS, 1)
    now += 100
    e2 = a.add(now, O.EV_PASS, 2)
    for i in range(10 - 2):
        now += 100
        a.add(now, O.EV_PASS, i + 3)
    assert a.valid_head(now)[0] == e1
    now += 100
    assert a.valid_head(now)[0] == e2


def test_array_metric_sums():
    # core-test/slots/statistic/metric/ArrayMetricTest.java:39-71
    a = O.Leap(O.LEAP_PLAIN, 2, 1000)
    a.add(0, O.EV_RT, 21)
    for _ in range(9):
        a.add(0, O.EV_PASS, 1)
    for _ in range(2):
        a.add(0, O.EV_BLOCK, 1)
    for _ in range(9):
        a.add(0, O.EV_SUCC, 1)
    for _ in range(6):
        a.add(0, O.EV_EXC, 1)
    assert [a.values_sum(0, e) for e in (O.EV_PASS, O.EV_BLOCK, O.EV_SUCC, O.EV_EXC, O.EV_RT)] == [9, 2, 9, 6, 21]


# ---------------------------------------------------------------- param flow
def _param_engine(rule):
    o = O.Oracle(max_slot_chain_size=0)
    rid = o.register(rule.resource.decode())
    assert o.load_param_rules([rule]) == 1
    return o, rid


def _pcheck(o, rid, now, key, n):
    out = []
    for _ in range(n):
        d, h = o.entry(now, rid, args=[key])
        out.append(d & 0xFF)
    return out


P, BP = A.PASS, A.BLOCK_PARAM


def test_param_default_single_qps():
    # param-test/slots/block/flow/param/ParamFlowDefaultCheckerTest.java:30-67
    o, rid = _param_engine(A.param_rule("testParamFlowDefaultCheckSingleQps", 0, 5))
    k = O.param_key("valueA")
    now = T0
    assert _pcheck(o, rid, now, k, 6) == [P] * 5 + [BP]
    now += 3000
    assert _pcheck(o, rid, now, k, 6) == [P] * 5 + [BP]


def test_param_default_single_qps_with_burst():
    # ParamFlowDefaultCheckerTest.java:69-137
    o, rid = _param_engine(A.param_rule("testParamFlowDefaultCheckSingleQpsWithBurst", 0, 5, burst_count=3))
    k = O.param_key("valueA")
    now = T0
    assert _pcheck(o, rid, now, k, 9) == [P] * 8 + [BP]
    now += 1002
    assert _pcheck(o, rid, now, k, 6) == [P] * 5 + [BP]
    now += 1002
    assert _pcheck(o, rid, now, k, 6) == [P] * 5 + [BP]
    now += 2000
    assert _pcheck(o, rid, now, k, 9) == [P] * 8 + [BP]
    now += 1002
    assert _pcheck(o, rid, now, k, 6) == [P] * 5 + [BP]


def test_param_default_qps_in_different_duration():
    # ParamFlowDefaultCheckerTest.java:139-188
    o, rid = _param_engine(A.param_rule("testParamFlowDefaultCheckQpsInDifferentDuration", 0, 5, duration_in_sec=60))
    k = O.param_key("helloWorld")
    now = T0
    assert _pcheck(o, rid, now, k, 6) == [P] * 5 + [BP]
    for step in (1000, 10000, 30000):
        now += step
        assert _pcheck(o, rid, now, k, 1) == [BP]
    now += 30000
    assert _pcheck(o, rid, now, k, 6) == [P] * 5 + [BP]


def test_param_pass_check_exceed_args():
    # param-test/slots/block/flow/param/ParamFlowCheckerTest.java:50-63
    o, rid = _param_engine(A.param_rule("testHotParamCheckerPassCheckExceedArgs", 1, 10))
    d, _ = o.entry(T0, rid, args=[O.param_key("abc")])
    assert d & 0xFF == A.PASS


def test_param_throttle_with_exception_items():
    # ParamFlowCheckerTest.java:65-99
    rule = A.param_rule("testSingleValueCheckQpsWithExceptionItems", 0, 5,
                        control_behavior=A.CONTROL_BEHAVIOR_RATE_LIMITER,
                        items=[("valueB", "java.lang.String", 0), ("valueD", "java.lang.String", 7)])
    o, rid = _param_engine(rule)
    assert o.entry(T0, rid, args=[O.param_key("valueA")])[0] & 0xFF == A.PASS
    assert o.entry(T0, rid, args=[O.param_key("valueB")])[0] & 0xFF == A.BLOCK_PARAM


def test_param_thread_count_with_exception_items():
    # ParamFlowCheckerTest.java:101-148 (ParameterMetric.getThreadCount mocked via the oracle hook)
    rule = A.param_rule("testSingleValueCheckThreadCountWithExceptionItems", 0, 5, grade=A.FLOW_GRADE_THREAD,
                        items=[("valueB", "java.lang.String", 3), ("valueD", "java.lang.String", 7)])
    o, rid = _param_engine(rule)
    ka, kb, kc, kd = (O.param_key(v) for v in ("valueA", "valueB", "valueC", "valueD"))

    def check(key, mocked):
        o.set_param_thread_count(rid, 0, key, mocked)
        return o.entry(T0, rid, args=[key])[0] & 0xFF == A.PASS

    assert check(ka, 4)
    assert not check(kb, 4)
    assert check(kc, 4)
    assert check(kd, 6)
    assert not check(ka, 5)
    assert check(kb, 2)
    assert not check(kc, 6)
    assert check(kd, 4)
    assert not check(kd, 7)


def test_param_rule_validity():
    # param-test/slots/block/flow/param/ParamFlowRuleUtilTest.java:17-44
    o = O.Oracle()
    assert o.load_param_rules([A.param_rule("", 1, 1)]) == 0
    assert o.load_param_rules([A.param_rule("abc", 1, -1)]) == 0
    assert o.load_param_rules([A.param_rule("abc", None, 1)]) == 0
    assert o.load_param_rules([A.param_rule("abc", -1, 1)]) == 1
    assert o.load_param_rules([A.param_rule("abc", 1, 10)]) == 1


def test_param_hot_items_parsing():
    # ParamFlowRuleUtilTest.java:46-94: failure cases are dropped, String is the default type,
    # boxed/primitive class names parse to typed values (Float 11.11 != String "11.11").
    items = [(None, "double", 1), ("Sentinel", None, 3), ("6", "java.lang.Integer", -5), ("6", "char", None),
             ("11.11", "", 3), ("1.1", "java.lang.Double", 1), ("6", "java.lang.Integer", 5), ("c", "char", 7)]
    rule = A.param_rule("hot", 0, 100, items=items)
    o, rid = _param_engine(rule)

    def limit(key):
        n = 0
        while o.entry(T0, rid, args=[key])[0] & 0xFF == A.PASS:
            n += 1
            if n > 200:
                break
        return n

    assert limit(O.param_key("Sentinel")) == 3
    assert limit(O.param_key("11.11", "java.lang.String")) == 3
    assert limit(O.param_key("11.11", "java.lang.Float")) == 100  # not a hot item -> global count
    assert limit(O.param_key("1.1", "java.lang.Double")) == 1
    assert limit(O.param_key("6", "java.lang.Integer")) == 5
    assert limit(O.param_key("c", "char")) == 7
    assert limit(O.param_key("6", "java.lang.Long")) == 100  # Long 6 != Integer 6


# ---------------------------------------------------------------- integration through the slot chain
def test_flow_qps_grade():
    # core-test/slots/block/flow/FlowPartialIntegrationTest.java:51-73
    o = O.Oracle()
    rid = o.register("testQPSGrade")
    o.load_flow_rules([A.flow_rule("testQPSGrade", 1)])
    d, h = o.entry(T0, rid)
    assert d & 0xFF == A.PASS
    o.exit(T0, h)
    d, h = o.entry(T0, rid)
    assert d & 0xFF == A.BLOCK_FLOW


def test_flow_thread_grade():
    # FlowPartialIntegrationTest.java:75-116 (the other thread holds its entry while the second enters)
    o = O.Oracle()
    rid = o.register("testThreadGrade")
    o.load_flow_rules([A.flow_rule("testThreadGrade", 1, grade=A.FLOW_GRADE_THREAD)])
    d1, h1 = o.entry(T0, rid)
    assert d1 & 0xFF == A.PASS
    d2, _ = o.entry(T0 + 1, rid)
    assert d2 & 0xFF == A.BLOCK_FLOW
    o.exit(T0 + 100, h1)
    assert o.entry(T0 + 101, rid)[0] & 0xFF == A.PASS


def test_origin_flow_rule():
    # FlowPartialIntegrationTest.java:118-158
    o = O.Oracle()
    rid = o.register("testOriginFlowRule")
    o.load_flow_rules([A.flow_rule("testOriginFlowRule", 0, limit_app="other"),
                       A.flow_rule("testOriginFlowRule", 1, limit_app="app2")])
    assert o.entry(T0, rid, context="node1", origin="app1")[0] & 0xFF == A.BLOCK_FLOW
    d, h = o.entry(T0, rid, context="node1", origin="app2")
    assert d & 0xFF == A.PASS
    o.exit(T0, h)


def test_flow_rule_other():
    # FlowPartialIntegrationTest.java:160-181
    o = O.Oracle()
    rid = o.register("testOther")
    o.load_flow_rules([A.flow_rule("testOther", 0, limit_app="other")])
    assert o.entry(T0, rid)[0] & 0xFF == A.PASS


def test_flow_strategy():
    # FlowPartialIntegrationTest.java:183-222
    o = O.Oracle()
    rid = o.register("testStrategy")
    o.load_flow_rules([A.flow_rule("testStrategy", 0, strategy=A.STRATEGY_DIRECT)])
    assert o.entry(T0, rid, context="testStrategy")[0] & 0xFF == A.BLOCK_FLOW
    # the second rule's resource was overwritten to "entry2": no rule for testStrategy remains
    o.load_flow_rules([A.flow_rule("entry2", 0, strategy=A.STRATEGY_CHAIN)])
    assert o.entry(T0, rid, context="entry1")[0] & 0xFF == A.PASS


def test_flow_strategy_chain():
    # FlowPartialIntegrationTest.java:224-255
    o = O.Oracle()
    rid = o.register("entry2")
    o.load_flow_rules([A.flow_rule("entry2", 0, strategy=A.STRATEGY_CHAIN, ref_resource="entry1")])
    assert o.entry(T0, rid, context="entry1")[0] & 0xFF == A.BLOCK_FLOW
    assert o.entry(T0, rid, context="entry3")[0] & 0xFF == A.PASS


def test_flow_relate_strategy():
    # FlowRuleCheckerTest.java:98-111 + FlowRuleChecker.selectReferenceNode (FlowRuleChecker.java:67-88):
    # a RELATE rule reads the ClusterNode of refResource.
    o = O.Oracle()
    a = o.register("relate_a")
    b = o.register("relate_b")
    o.load_flow_rules([A.flow_rule("relate_a", 1, strategy=A.STRATEGY_RELATE, ref_resource="relate_b")])
    assert o.entry(T0, a)[0] & 0xFF == A.PASS  # ref node absent -> pass
    o.entry(T0, b)
    assert o.entry(T0, a)[0] & 0xFF == A.BLOCK_FLOW  # relate_b already passed 1 in this window


def test_flow_rule_comparator_partition():
    # core-test/slots/block/flow/FlowRuleComparatorTest.java:18-38: specific limitApps sort before "default";
    # ties keep their (HashSet) order.
    o = O.Oracle()
    rid = o.register("abc")
    rules = [A.flow_rule("abc", 10, limit_app="default"), A.flow_rule("abc", 0, limit_app="originA"),
             A.flow_rule("abc", 0, limit_app="originB"), A.flow_rule("abc", 0, limit_app="other"),
             A.flow_rule("abc", 20, limit_app="default")]
    o.load_flow_rules(rules)
    order = o.rule_order(rid, 0)
    assert sorted(order[:3]) == [1, 2, 3] and sorted(order[3:]) == [0, 4]


def test_chain_size_cap():
    # core-test/CtSphTest.java:272-284 + CtSph.lookProcessChain (core/CtSph.java:206-227), Q1
    o = O.Oracle(max_slot_chain_size=6000)
    ids = [o.register("test-resource-%d" % i) for i in range(6001)]
    o.load_flow_rules([A.flow_rule("test-resource-6000", 0)])
    for i in ids[:6000]:
        assert o.entry(T0, i)[0] & 0xFF == A.PASS
    assert o.entry(T0, ids[6000])[0] & 0xFF == A.NO_CHECK  # would block with a chain
    st = o.read_node(ids[6000])
    assert st["has_chain"] == 0 and (st["second"][:, 0] == -1).all()


# ---------------------------------------------------------------- token server
def test_cluster_flow_checker_occupy_sequence():
    # csrv-test/flow/ClusterFlowCheckerTest.java:37-70 (disabled in the reference; its sequence replayed
    # with trace time): threshold 5 GLOBAL, 5 buckets of 200 ms.
    o = O.Oracle()
    o.register("abc")
    o.load_flow_rules([A.flow_rule("abc", 5, cluster_mode=True, cluster_flow_id=98765,
                                   cluster_threshold_type=A.CLUSTER_THRESHOLD_GLOBAL, cluster_sample_count=5)])
    t = T0 - T0 % 1000
    seq = []

    def acq(occupy):
        return o.cluster_request([(t, 98765, 1, occupy)])[0]

    seq += [acq(False), acq(False)]
    t += 200
    seq += [acq(False)]
    t += 200
    seq += [acq(True), acq(False), acq(True)]
    t += 200
    seq += [acq(False), acq(False)]
    t += 200
    seq += [acq(False), acq(True), acq(False)]
    t += 200
    seq += [acq(False)]
    st = [s for s, _, _ in seq]
    OK, BL, W = A.TOKEN_OK, A.TOKEN_BLOCKED, A.TOKEN_SHOULD_WAIT
    assert st == [OK, OK, OK, OK, OK, BL, BL, BL, BL, W, BL, OK]
    assert seq[9][2] == 200


def test_token_service_bad_request_and_no_rule():
    # csrv/flow/DefaultTokenService.java:37-66
    o = O.Oracle()
    assert o.cluster_request([(T0, 0, 1, False)])[0][0] == A.TOKEN_BAD_REQUEST
    assert o.cluster_request([(T0, 5, 0, False)])[0][0] == A.TOKEN_BAD_REQUEST
    assert o.cluster_request([(T0, 5, 1, False)])[0][0] == A.TOKEN_NO_RULE_EXISTS


def _cluster_rule(fid, count, **kw):
    kw.setdefault("cluster_threshold_type", A.CLUSTER_THRESHOLD_GLOBAL)
    return A.flow_rule("abc", count, cluster_mode=True, cluster_flow_id=fid, **kw)


def test_cluster_rule_map_last_rule_wins_and_metric_kept():
    # ClusterFlowRuleManager.applyClusterFlowRule (csrv/flow/rule/ClusterFlowRuleManager.java:323-363):
    # list order, ruleMap.put -> the later rule of a flowId wins; putMetricIfAbsent keeps the metric
    o = O.Oracle()
    o.register("abc")
    o.load_flow_rules([_cluster_rule(7, 2), _cluster_rule(7, 3)])
    t = T0 - T0 % 1000
    st = [s for s, _, _ in o.cluster_request([(t, 7, 1, False)] * 4)]
    assert st == [A.TOKEN_OK] * 3 + [A.TOKEN_BLOCKED]
    # a new list with count 5 and another window shape: the metric (3 passes, 10 x 100 ms) stays
    o.load_flow_rules([_cluster_rule(7, 5, cluster_sample_count=2)])
    st = [s for s, _, _ in o.cluster_request([(t + 10, 7, 1, False)] * 3)]
    assert st == [A.TOKEN_OK, A.TOKEN_OK, A.TOKEN_BLOCKED]
    # remaining = (int)(threshold - passQps - acquire)
    o.load_flow_rules([_cluster_rule(7, 9.5)])
    assert o.cluster_request([(t + 20, 7, 2, False)])[0] == (A.TOKEN_OK, 2, 0)


def test_cluster_dropped_flow_id_and_fresh_metric():
    o = O.Oracle()
    o.register("abc")
    o.load_flow_rules([_cluster_rule(7, 1), _cluster_rule(8, 1)])
    t = T0 - T0 % 1000
    assert [s for s, _, _ in o.cluster_request([(t, 7, 1, False), (t, 7, 1, False)])] == [A.TOKEN_OK, A.TOKEN_BLOCKED]
    o.load_flow_rules([_cluster_rule(8, 1)])  # clearAndResetRulesConditional drops flowId 7
    assert o.cluster_request([(t + 1, 7, 1, False)])[0][0] == A.TOKEN_NO_RULE_EXISTS
    o.load_flow_rules([_cluster_rule(7, 1), _cluster_rule(8, 1)])  # a fresh metric
    assert o.cluster_request([(t + 2, 7, 1, False)])[0][0] == A.TOKEN_OK


def test_global_request_limiter():
    # RequestLimiter.tryPass (csrv/flow/statistic/limit/RequestLimiter.java:72-87): qps + 1 <= allowed over
    # 10 x 100 ms; requests refused here never reach the flow's metric
    o = O.Oracle(cluster_max_allowed_qps=3)
    o.register("abc")
    o.load_flow_rules([_cluster_rule(7, 100)])
    t = T0 - T0 % 1000
    st = [s for s, _, _ in o.cluster_request([(t, 7, 1, False)] * 5)]
    assert st == [A.TOKEN_OK] * 3 + [A.TOKEN_TOO_MANY_REQUEST] * 2
    st = [s for s, _, _ in o.cluster_request([(t + 999, 7, 1, False), (t + 1000, 7, 1, False)])]
    assert st == [A.TOKEN_TOO_MANY_REQUEST, A.TOKEN_OK]
    # BAD_REQUEST / NO_RULE_EXISTS are answered before the limiter and do not consume it
    o2 = O.Oracle(cluster_max_allowed_qps=1)
    o2.register("abc")
    o2.load_flow_rules([_cluster_rule(7, 100)])
    st = [s for s, _, _ in o2.cluster_request([(t, 9, 1, False), (t, 7, 0, False), (t, 7, 1, False)])]
    assert st == [A.TOKEN_NO_RULE_EXISTS, A.TOKEN_BAD_REQUEST, A.TOKEN_OK]


def test_cluster_avg_local_threshold():
    # calcGlobalThreshold: AVG_LOCAL -> count * connectedCount (csrv/flow/ClusterFlowChecker.java:38-48)
    o = O.Oracle()
    o.register("abc")
    o.load_flow_rules([_cluster_rule(7, 2, cluster_threshold_type=A.CLUSTER_THRESHOLD_AVG_LOCAL)])
    t = T0 - T0 % 1000
    assert o.cluster_request([(t, 7, 1, False)])[0][0] == A.TOKEN_BLOCKED  # no client connected
    assert o.cluster_set_connected(7, 3) == 0
    st = [s for s, _, _ in o.cluster_request([(t, 7, 1, False)] * 7)]
    assert st == [A.TOKEN_OK] * 6 + [A.TOKEN_BLOCKED]


# ---------------------------------------------------------------- args: collections, arrays, negative index
def _param_oracle(res, **rule):
    o = O.Oracle()
    rid = o.register(res)
    o.load_param_rules([A.param_rule(res, **rule)])
    return o, rid


def test_param_pass_local_check_for_collection():
    # param-test/slots/block/flow/param/ParamFlowCheckerTest.java:149-166: threshold 1, list [a, B, Cc]:
    # the first check consumes every element's token, the second blocks on the first element
    o, rid = _param_oracle("testPassLocalCheckForCollection", param_idx=0, count=1)
    lst = [O.param_key("a"), O.param_key("B"), O.param_key("Cc")]
    assert o.entry(T0, rid, args=[lst])[0] & 0xFF == A.PASS
    assert o.entry(T0, rid, args=[lst])[0] & 0xFF == A.BLOCK_PARAM


def test_param_pass_local_check_for_array():
    # ParamFlowCheckerTest.java:169-188: RATE_LIMITER, threshold 1, array [a, B, Cc] -> pass, then block
    o, rid = _param_oracle("testPassLocalCheckForArray", param_idx=0, count=1,
                           control_behavior=A.CONTROL_BEHAVIOR_RATE_LIMITER)
    arr = [O.param_key("a"), O.param_key("B"), O.param_key("Cc")]
    assert o.entry(T0, rid, args=[arr])[0] & 0xFF == A.PASS
    assert o.entry(T0, rid, args=[arr])[0] & 0xFF == A.BLOCK_PARAM


def test_param_negative_index():
    # param-test/slots/block/flow/param/ParamFlowSlotTest.java:52-77: paramIdx -1 with 3 args resolves to 2,
    # -100 to 100 (past the args: always passes); the rule object keeps the resolved index
    o, rid = _param_oracle("testNegativeParamIdx", param_idx=-1, count=1)
    k = [O.param_key(v) for v in ("abc", "def", "ghi", "xyz")]
    assert o.entry(T0, rid, args=[k[0], k[1], k[2]])[0] & 0xFF == A.PASS
    assert o.entry(T0, rid, args=[k[3], k[3], k[2]])[0] & 0xFF == A.BLOCK_PARAM  # args[2] = "ghi" again
    assert o.entry(T0, rid, args=[k[2], k[2], k[3]])[0] & 0xFF == A.PASS         # "xyz" is new
    # resolved once: a 2-arg call still checks index 2 (absent -> pass)
    assert o.entry(T0, rid, args=[k[2], k[2]])[0] & 0xFF == A.PASS
    o2, rid2 = _param_oracle("testNegativeParamIdx", param_idx=-100, count=1)
    for _ in range(3):
        assert o2.entry(T0, rid2, args=[k[0], k[1], k[2]])[0] & 0xFF == A.PASS


def test_param_collection_with_null_element():
    # ParamFlowChecker.passLocalCheck (ParamFlowChecker.java:73-99): a null element makes the map lookup throw;
    # the Throwable is caught and the check passes -- elements before it have consumed their tokens
    o, rid = _param_oracle("nullElem", param_idx=0, count=1)
    a, b = O.param_key("a"), O.param_key("b")
    assert o.entry(T0, rid, args=[[a, None, b]])[0] & 0xFF == A.PASS
    assert o.entry(T0, rid, args=[[a, None, b]])[0] & 0xFF == A.BLOCK_PARAM  # a is spent
    assert o.entry(T0, rid, args=[[b]])[0] & 0xFF == A.PASS                  # b was never checked


def test_upstream_block_after_param_before_flow():
    # HotParamSlotChainBuilder (param/slots/HotParamSlotChainBuilder.java:38-51): ParamFlowSlot runs before the
    # System/Authority slots, FlowSlot after them; StatisticSlot counts the block (StatisticSlot.java:97-117)
    o = O.Oracle()
    rid = o.register("up")
    o.load_param_rules([A.param_rule("up", 0, 2)])
    o.load_flow_rules([A.flow_rule("up", 100)])
    k = O.param_key("v")
    ev = A.np.zeros(4, dtype=A.EVENT_DTYPE)
    ev["ts"] = T0
    ev["res_id"] = rid
    ev["count"] = 1
    ev["kind"] = A.EV_ENTRY
    ev["flags"] = [A.F_HAS_ARG | A.F_BLOCKED_UPSTREAM, A.F_HAS_ARG, A.F_HAS_ARG | A.F_BLOCKED_UPSTREAM, A.F_HAS_ARG]
    ev["aux"] = k
    d = o.submit(ev) & 0xFF
    # the upstream-blocked entry still spends a param token; the third is a param block (it comes first)
    assert list(d) == [A.BLOCK_UPSTREAM, A.PASS, A.BLOCK_PARAM, A.BLOCK_PARAM]
    assert o.read_node(rid)["second"][:, 2].sum() == 3 and o.read_node(rid)["second"][:, 1].sum() == 1
