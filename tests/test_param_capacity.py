"""ParameterMetric's bounded maps (param/.../ParameterMetric.java:37-114): every rule's time/token CacheMaps
hold at most min(4000 * durationInSec, 200000) values and every thread-count map 4000, evicting the least
recently used value (ConcurrentLinkedHashMap access order: get and putIfAbsent of a present value refresh it).
The reference's own tests never fill a map, and ConcurrentLinkedHashMap is not in /root/reference, so these
cases are derived from that reading ("parity unpinned"); the GPU engine is held to the same oracle
by tests/test_gpu_param_capacity.py."""
import pyoracle as O

from sentinel_amd import _abi as A

T0 = 1_700_000_000_000
P, BP = A.PASS, A.BLOCK_PARAM


def _engine(rule):
    o = O.Oracle(max_slot_chain_size=0)
    rid = o.register(rule.resource.decode())
    assert o.load_param_rules([rule]) == 1
    return o, rid


def _d(o, rid, now, key):
    return o.entry(now, rid, args=[key])[0] & 0xFF


def test_full_rule_map_evicts_the_least_recently_used_value():
    o, rid = _engine(A.param_rule("cap1", 0, 1))          # 1 token per value per second, capacity 4000
    k = O.param_key(-1, "java.lang.Long")
    assert (_d(o, rid, T0, k), _d(o, rid, T0, k)) == (P, BP)
    for v in range(4000):                                  # 4000 newer values push k out
        assert _d(o, rid, T0, O.param_key(v, "java.lang.Long")) == P
    assert _d(o, rid, T0, k) == P                          # a fresh bucket: k was evicted
    assert _d(o, rid, T0, O.param_key(0, "java.lang.Long")) == P   # ... and so, in turn, was value 0
    assert _d(o, rid, T0, O.param_key(3999, "java.lang.Long")) == BP


def test_a_checked_value_is_refreshed():
    o, rid = _engine(A.param_rule("cap2", 0, 1))
    k = O.param_key(-1, "java.lang.Long")
    assert _d(o, rid, T0, k) == P
    for v in range(3999):
        _d(o, rid, T0, O.param_key(v, "java.lang.Long"))
    assert _d(o, rid, T0, k) == BP                         # putIfAbsent of a present value: most recently used
    assert _d(o, rid, T0, O.param_key(5000, "java.lang.Long")) == P   # evicts value 0, the LRU
    assert _d(o, rid, T0, k) == BP
    assert _d(o, rid, T0, O.param_key(0, "java.lang.Long")) == P
    assert _d(o, rid, T0, O.param_key(1, "java.lang.Long")) == P       # evicted by value 0's return


def test_capacity_follows_the_duration():
    o, rid = _engine(A.param_rule("cap3", 0, 1, duration_in_sec=2))   # capacity 8000
    k = O.param_key(-1, "java.lang.Long")
    assert _d(o, rid, T0, k) == P
    for v in range(4500):
        _d(o, rid, T0, O.param_key(v, "java.lang.Long"))
    assert _d(o, rid, T0, k) == BP


def test_thread_count_map_holds_4000_values():
    o, rid = _engine(A.param_rule("cap4", 0, 1, grade=A.FLOW_GRADE_THREAD))
    k = O.param_key(-1, "java.lang.Long")
    assert (_d(o, rid, T0, k), _d(o, rid, T0, k)) == (P, BP)   # one thread holds k (no exit)
    for v in range(4000):
        assert _d(o, rid, T0, O.param_key(v, "java.lang.Long")) == P
    assert _d(o, rid, T0, k) == P                              # k's count was evicted with it
