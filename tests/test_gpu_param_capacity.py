"""The device's bounded ParameterMetric maps (dev_types.h PMap) against the oracle's (tests/test_param_capacity.py):
LRU eviction at min(4000 * durationInSec, 200000) / 4000 values, the capacity check at rule load that leaves the
engine unchanged (SG_ECAPACITY), regions that grow with their keys in a pool that is compacted between batches and
whose exhaustion fails the engine, and a C5 trace with more than five million distinct values through a pool sized
by param_table_log2 = 24."""
import numpy as np
import pytest

import pyoracle as O
from sentinel_amd import _abi as A
from sentinel_amd import engine as E
from sentinel_amd import tracegen as T

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000


def _entries(rid, keys, t=T0):
    ev = np.zeros(len(keys), dtype=A.EVENT_DTYPE)
    ev["ts"] = t
    ev["res_id"] = rid
    ev["count"] = 1
    ev["kind"] = A.EV_ENTRY
    ev["flags"] = A.F_HAS_ARG
    ev["aux"] = np.asarray(keys, dtype=np.uint64)
    return ev


def _pair(rule, **cfg):
    eng = E.Engine(max_resources=64, max_slot_chain_size=0, **cfg)
    orc = O.Oracle(max_slot_chain_size=0)
    name = rule.resource.decode()
    rid = eng.register(name)
    assert orc.register(name) == rid
    assert eng.load_param_rules([rule]) == 1 and orc.load_param_rules([rule]) == 1
    return eng, orc, rid


def _long(v):
    return E.param_key(str(v), "java.lang.Long")


@pytest.mark.parametrize("grade", [A.FLOW_GRADE_QPS, A.FLOW_GRADE_THREAD])
@pytest.mark.parametrize("behavior", [A.CONTROL_BEHAVIOR_DEFAULT, A.CONTROL_BEHAVIOR_RATE_LIMITER])
def test_eviction_sequences_match_the_oracle(grade, behavior):
    if grade == A.FLOW_GRADE_THREAD and behavior != A.CONTROL_BEHAVIOR_DEFAULT:
        pytest.skip("the control behaviour only applies to QPS rules")
    eng, orc, rid = _pair(A.param_rule("capk", 0, 1, grade=grade, control_behavior=behavior, max_queueing_time_ms=0))
    k = _long(-1)
    seq = [k, k] + [_long(v) for v in range(3999)] + [k] + [_long(5000)] + [k, _long(0), _long(1)] + \
          [_long(v) for v in range(6000, 12000)] + [k, _long(3000), _long(11999)]
    ev = _entries(rid, seq)
    for a, b in ((0, 2), (2, 4001), (4001, 4010), (4010, len(ev))):   # batches cut inside the sequences
        dg, do = eng.submit(ev[a:b]), orc.submit(ev[a:b])
        bad = np.nonzero(dg != do)[0]
        assert not len(bad), ("event", a + int(bad[0]), hex(dg[bad[0]]), hex(do[bad[0]]))


def test_capacity_follows_the_duration_on_the_device():
    eng, orc, rid = _pair(A.param_rule("capd", 0, 1, duration_in_sec=2))   # 8000 values
    seq = [_long(-1)] + [_long(v) for v in range(7000)] + [_long(-1)] + [_long(v) for v in range(7000, 9000)] + \
          [_long(-1), _long(0), _long(100)]
    ev = _entries(rid, seq)
    np.testing.assert_array_equal(eng.submit(ev), orc.submit(ev))


def test_ecapacity_at_rule_load_leaves_the_engine_unchanged():
    # 2^5 slots hold the first regions of one resource's maps (a rule map + a thread-count map, PM_MIN_NB = 2
    # buckets of 8 each) but not two; a region grows only once live keys + a batch's events exceed 8
    eng = E.Engine(max_resources=64, max_slot_chain_size=0, param_table_log2=5)
    orc = O.Oracle(max_slot_chain_size=0)
    for n in ("a", "b"):
        assert eng.register(n) == orc.register(n)
    first = [A.param_rule("a", 0, 2)]
    assert eng.load_param_rules(first) == 1 and orc.load_param_rules(first) == 1
    ev = _entries(0, [_long(v % 3) for v in range(8)])
    np.testing.assert_array_equal(eng.submit(ev), orc.submit(ev))
    with pytest.raises(E.SentinelError) as ei:
        eng.load_param_rules(first + [A.param_rule("b", 0, 1)])
    assert ei.value.code == A.SG_ECAPACITY and "param_table_log2" in str(ei.value)
    # the rules and the maps of "a" are what they were: the next batch still matches the oracle that never saw
    # the failed load, including the tokens consumed before it
    ev2 = _entries(0, [_long(v % 3) for v in range(4)], t=T0 + 500)  # 3 live keys + 5 events (with b's)
    ev2 = np.concatenate([ev2, _entries(1, [_long(1)], t=T0 + 500)])
    np.testing.assert_array_equal(eng.submit(ev2), orc.submit(ev2))


def test_pool_used_up_fails_the_batch_and_the_engine():
    # the maps' regions grow with their keys (k_pm_grow); 2^8 slots cannot hold a map of 100 keys: the batch
    # fails with SG_ECAPACITY and every later submit is refused (a key may have been lost)
    eng = E.Engine(max_resources=64, max_slot_chain_size=0, param_table_log2=8)
    rid = eng.register("a")
    eng.load_param_rules([A.param_rule("a", 0, 2)])
    np.asarray(eng.submit(_entries(rid, [_long(v) for v in range(6)])))  # fits the first regions
    with pytest.raises(E.SentinelError) as ei:
        eng.submit(_entries(rid, [_long(v) for v in range(100)], t=T0 + 10))
    assert ei.value.code == A.SG_ECAPACITY and "param_table_log2" in str(ei.value)
    with pytest.raises(E.SentinelError):
        eng.submit(_entries(rid, [_long(1)], t=T0 + 20))


def test_batch_that_finds_the_pool_short_compacts_on_the_device():
    # the between-batch compaction runs at half of the free space on counts a batch or two old, so one
    # batch can still find the pool short.  It then compacts on the device and grows again (param.hip
    # launch_pm_grow).  2^12 slots = 512 buckets: batch 1 grows a's two maps to 25 buckets each, batch 2 to 75
    # (54 buckets grown out of, under the host's trigger), batch 3 asks 2 x 175 with 304 free -- short; the live
    # regions compacted (154 buckets) leave room.  Every decision against the oracle, then a's maps still hold
    # their keys (thread counts read back).
    eng = E.Engine(max_resources=64, max_slot_chain_size=0, param_table_log2=12)
    orc = O.Oracle(max_slot_chain_size=0)
    for n in ("a", "b"):
        assert eng.register(n) == orc.register(n)
    rules = [A.param_rule("a", 0, 50), A.param_rule("b", 0, 50)]
    assert eng.load_param_rules(rules) == 2 and orc.load_param_rules(rules) == 2
    v0 = 0
    for b, n in enumerate((100, 200, 400)):
        ev = _entries(0, [_long(v) for v in range(v0, v0 + n)], t=T0 + 100 * b)
        v0 += n
        dg, do = eng.submit(ev), orc.submit(ev)
        np.testing.assert_array_equal(dg, do, err_msg="batch %d" % b)
    pool = eng.param_pool()
    assert pool["device_compactions"] == 1 and pool["compactions"] == 0, pool
    assert pool["taken"] <= pool["buckets"], pool
    for v in (0, 99, 100, 350, 699):
        assert eng.param_thread_count(0, 0, _long(v)) == orc.param_thread_count(0, 0, _long(v)) == 1, v


def test_regions_grow_and_the_pool_compacts():
    # 300 resources, each map growing over 12 batches from 2 buckets towards full size, in a pool a little larger
    # than the final regions: the regions grown out of fill it and are dropped by relayouts between batches
    # (rebuild_pmaps); every decision against the oracle
    n_res = 300
    eng = E.Engine(max_resources=512, max_slot_chain_size=0, param_table_log2=21)
    orc = O.Oracle(max_slot_chain_size=0)
    names = ["g%d" % i for i in range(n_res)]
    for nm in names:
        assert eng.register(nm) == orc.register(nm)
    rules = [A.param_rule(nm, 0, 3, burst_count=1) for nm in names]
    assert eng.load_param_rules(rules) == orc.load_param_rules(rules)
    rng = np.random.default_rng(5)
    for b in range(12):
        rid = rng.integers(0, n_res, 40_000)
        keys = [_long(int(v)) for v in rng.integers(0, 150 * (b + 1), len(rid))]
        ev = np.concatenate([_entries(int(r), [k], t=T0 + 300 * b) for r, k in zip(rid, keys)])
        dg, do = eng.submit(ev), orc.submit(ev)
        bad = np.nonzero(dg != do)[0]
        assert not len(bad), (b, int(bad[0]), hex(dg[bad[0]]), hex(do[bad[0]]))
    pool = eng.param_pool()
    assert pool["compactions"] >= 1 and pool["taken"] <= pool["buckets"], pool


def test_c5_five_million_distinct_values():
    # SURVEY.md §8(d) C5 shape with churn: 14M entries over 1000 resources, half of the values uniform over 10M
    # (5.46M distinct), hot items, THREAD-grade rules; every map fills and evicts.  The pool needs
    # 1000 x 2 x 6016 slots, inside param_table_log2 = 24.
    w = T.Workload(5, n_res=1000, n_entries=14_000_000, n_param_values=10_000_000,
                   variant=T.V_UNIFORM | T.V_HOT | T.V_THREAD)
    ev = w.events
    assert len(np.unique(ev["aux"][ev["kind"] == A.EV_ENTRY])) >= 5_000_000
    eng = E.Engine(max_resources=w.n_res, max_slot_chain_size=0, param_table_log2=24, status_ring_log2=26)
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(eng)
    w.install(orc)
    cuts = np.linspace(0, len(ev), 5).astype(np.int64)
    blocked = 0
    for a, b in zip(cuts[:-1], cuts[1:]):
        dg, do = eng.submit(ev[a:b]), orc.submit(ev[a:b])
        bad = np.nonzero(dg != do)[0]
        assert not len(bad), ("event", int(a + bad[0]), hex(dg[bad[0]]), hex(do[bad[0]]), len(bad))
        blocked += int(((dg & 0xFF) == A.BLOCK_PARAM).sum())
    assert blocked > 100_000


def test_largest_pool_that_fits_loads():
    # the compaction's second pool is allocated with the pool, so the maps take 2 x 2^k x 32 B of HBM at
    # rule load.  8192 rules of durationInSec 50 (200,000 values each) could use more than 2^32 slots, so the pool is
    # the full 2^k: param_table_log2 from 34 down, each load either refused with SG_ECAPACITY (nothing loaded) or
    # taken; the largest k taken decides a batch exactly as the oracle, and every k the device memory holds loads
    # (2^31 slots: 2 x 68.7 GB on one MI355X)
    n_res = 8192
    names = ["big%d" % i for i in range(n_res)]
    rules = [A.param_rule(nm, 0, 5, duration_in_sec=50) for nm in names]
    got = None
    for k in (34, 33, 32, 31, 30):
        eng = E.Engine(max_resources=n_res, max_slot_chain_size=0, param_table_log2=k)
        eng.register_many(names)
        try:
            assert eng.load_param_rules(rules) == n_res
        except E.SentinelError as ex:
            assert ex.code == A.SG_ECAPACITY and "param_table_log2" in str(ex), str(ex)
            eng.close()
            continue
        got = k
        orc = O.Oracle(max_slot_chain_size=0)
        for nm in names[:4]:
            orc.register(nm)
        assert orc.load_param_rules(rules[:4]) == 4
        ev = np.concatenate([_entries(r, [_long(v % 7) for v in range(40)], t=T0 + 10 * r) for r in range(4)])
        ev = ev[np.argsort(ev["ts"], kind="stable")]
        np.testing.assert_array_equal(eng.submit(ev), orc.submit(ev))
        pool = eng.param_pool()
        assert pool["buckets"] * 8 == 1 << k, pool
        orc.close()
        eng.close()
        break
    assert got is not None and got >= 31, got
