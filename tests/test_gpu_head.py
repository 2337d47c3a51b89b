"""The event-driven head owner (sentinel_amd/csrc/head.hip k_head) against the oracle.

A resource whose only rule is one THREAD-grade DefaultController or one QPS RateLimiter flow rule (DIRECT,
limitApp default) has its J16 / J4 segments decided by k_head: one wave per segment, chunks of 1,024 positions,
guess-and-verify rounds over a (min, +) scan of the passes (THREAD, DefaultController.java:49-81 with
StatisticSlot.java:54-173's curThreadNum) or a (max, +) scan of latestPassedTime (RateLimiterController.java:46-91).
The trace here is built to reach every branch of those rounds:

* THREAD counts 0.5 / 1 / 3 / 8 / 40 / 1e9, RTs from 1 to 400 ms, rates from 300 to 200k entries/s: saturated and
  open stretches, EXITs naming ENTRYs of the same chunk (the Jacobi fix-ups), of earlier chunks (the LDS status ring),
  of earlier batches (the status ring in HBM), and none at all (RC_NONE: effective, the count can go negative);
* acquire counts of 0 / 1 / 2 / 3 on some resources (the closed form is then only a guess; the verification decides);
* RateLimiter counts 0 (blocks every acquire > 0) / 0.3 / 5 / 50 / 500 / 3,000 (cost 0) with maxQueueingTimeMs
  0 / 20 / 500: the lattice guesses of saturated stretches, the all-pass guesses of open ones, queueing waits;
* WarmUpRateLimiters (WarmUpRateLimiterController.java) warming up over 2-3 s, acquire 0 / 1 / 2 on one: the
  cost changes every second with the stored tokens the leader syncs from the second before's passes;
* one resource with 200k entries/s and 1 % of its RTs at 1.5 s: EXITs naming ENTRYs more than 2^18 positions back
  (past the LDS ring: the dec[] word).

Every decision (with its wait) and every resource's windows and thread count are compared with the oracle, with the
head owner on and off (SG_DEBUG_FLAGS=16384: the cooperative owner decides those heads).
"""
import numpy as np
import pytest

import pyoracle as O
from sentinel_amd import _abi as A
from sentinel_amd import engine as E

T0 = 1_700_000_000_000
BATCH_MS = 2000


def _spec():
    """(rule kwargs, entries per second, mean RT ms, acquire choices) per resource."""
    th = A.FLOW_GRADE_THREAD
    rl = dict(control_behavior=A.CONTROL_BEHAVIOR_RATE_LIMITER)
    s = []
    for cnt in (0.5, 1, 3, 8, 40, 1e9):
        for rate, rtm in ((300, 20), (5000, 5), (40000, 30)):
            s.append((dict(count=cnt, grade=th), rate, rtm, (1,)))
    s.append((dict(count=4, grade=th), 20000, 10, (0, 1, 2, 3)))
    s.append((dict(count=25, grade=th), 8000, 200, (1, 2)))
    for cnt in (0, 0.3, 5, 50, 500, 3000):
        for q in (0, 20, 500):
            s.append((dict(count=cnt, max_queueing_time_ms=q, **rl), 6000, 20, (1,)))
    s.append((dict(count=80, max_queueing_time_ms=300, **rl), 3000, 20, (0, 1, 2)))
    s.append((dict(count=200, max_queueing_time_ms=100, **rl), 300, 10, (1,)))  # sparse: open stretches
    wrl = dict(control_behavior=A.CONTROL_BEHAVIOR_WARM_UP_RATE_LIMITER)
    for cnt, q, rate in ((50, 500, 6000), (500, 20, 6000), (5, 500, 800), (2000, 100, 30000)):
        s.append((dict(count=cnt, max_queueing_time_ms=q, warm_up_period_sec=3, **wrl), rate, 20, (1,)))
    s.append((dict(count=40, max_queueing_time_ms=200, warm_up_period_sec=2, **wrl), 4000, 20, (0, 1, 2)))
    s.append((dict(count=16, grade=th), 200000, None, (1,)))  # the ring-overflow resource (last)
    return s


def _trace(spec, n_batches=3, seed=5):
    rng = np.random.default_rng(seed)
    span = n_batches * BATCH_MS
    ts, res, kind, ref_of, rt, cnt = [], [], [], [], [], []
    for r, (_, rate, rtm, acq) in enumerate(spec):
        k = int(rate * span / 1000)
        if rtm is None:  # the ring-overflow resource: the first batch only
            k = int(rate * BATCH_MS / 1000)
            t = T0 + np.sort(rng.integers(0, BATCH_MS - 1600, k))
            d = np.where(rng.random(k) < 0.01, 1500, rng.integers(0, 40, k))
        else:
            t = T0 + np.sort(rng.integers(0, span, k))
            d = np.minimum(rng.exponential(rtm, k).astype(np.int64), 4900)
        a = rng.choice(np.asarray(acq), k)
        tr = rng.random(k) < 0.05
        noref = rng.random(k) < 0.002
        base = len(ts)
        ts.extend(t.tolist() + (t + d).tolist() + (t[tr] + d[tr]).tolist())
        res.extend([r] * (2 * k + int(tr.sum())))
        kind.extend([A.EV_ENTRY] * k + [A.EV_EXIT] * k + [A.EV_TRACE] * int(tr.sum()))
        ref_of.extend([-1] * k + [(-1 if noref[j] else base + j) for j in range(k)] +
                      [base + j for j in np.nonzero(tr)[0]])
        rt.extend([0] * k + d.tolist() + [0] * int(tr.sum()))
        cnt.extend(a.tolist() + a.tolist() + [1] * int(tr.sum()))
    ts, res, kind, ref_of, rt, cnt = map(np.asarray, (ts, res, kind, ref_of, rt, cnt))
    # time order; in one millisecond ENTRYs first, then TRACEs, then EXITs (an EXIT follows its ENTRY)
    korder = np.where(kind == A.EV_ENTRY, 0, np.where(kind == A.EV_TRACE, 1, 2))
    order = np.lexsort((korder, ts))
    pos = np.empty(len(order), dtype=np.int64)
    pos[order] = np.arange(len(order))
    ev = np.zeros(len(order), dtype=A.EVENT_DTYPE)
    ev["ts"] = ts[order]
    ev["res_id"] = res[order]
    ev["count"] = cnt[order]
    ev["kind"] = kind[order]
    ref = ref_of[order]
    aux = np.full(len(order), A.REF_NONE, dtype=np.uint64)
    has = ref >= 0
    aux[has] = pos[ref[has]].astype(np.uint64)
    ex = ev["kind"] == A.EV_EXIT
    aux[ex] |= rt[order][ex].astype(np.uint64) << np.uint64(48)
    ev["aux"] = aux
    cuts = np.searchsorted(ev["ts"], T0 + BATCH_MS * np.arange(n_batches + 1))
    cuts[-1] = len(ev)
    return ev, cuts


@pytest.mark.gpu
@pytest.mark.parametrize("owner", ["head", "coop"])
def test_head_owner_matches_oracle(owner, monkeypatch):
    for k, v in {"SG_LANE_MAX": "0", "SG_J1_MAX": "40", "SG_J4_MAX": "2000"}.items():
        monkeypatch.setenv(k, v)
    if owner == "coop":
        monkeypatch.setenv("SG_DEBUG_FLAGS", "16384")
    spec = _spec()
    names = ["head-%d" % i for i in range(len(spec))]
    rules = [A.flow_rule(n, **kw) for n, (kw, *_) in zip(names, spec)]
    ev, cuts = _trace(spec)
    eng = E.Engine(max_resources=256, max_slot_chain_size=0, status_ring_log2=24)
    orc = O.Oracle(max_slot_chain_size=0)
    ids = eng.register_many(names)
    assert list(ids) == list(range(len(names)))
    for n in names:
        orc.register(n)
    eng.load_flow_rules(rules)
    orc.load_flow_rules(rules)
    for b, (a, e) in enumerate(zip(cuts[:-1], cuts[1:])):
        dg, do = eng.submit(ev[a:e]), orc.submit(ev[a:e])
        bad = np.nonzero(dg != do)[0]
        assert not len(bad), ("batch", b, int(a + bad[0]), ev[a + bad[0]], hex(dg[bad[0]]), hex(do[bad[0]]), len(bad))
        st = do[ev["kind"][a:e] == A.EV_ENTRY] & 0xFF
        assert (st == A.PASS).any() and (st == A.BLOCK_FLOW).any()
        assert ((do >> 16) > 0).any() or b > 0  # queueing waits are in the words
    for r in range(len(names)):
        g, o = eng.read_node(r), orc.read_node(r)
        assert g["thread"] == o["thread"], (r, g["thread"], o["thread"])
        np.testing.assert_array_equal(g["second"][:2], o["second"][:2], err_msg="second window of res %d" % r)
        np.testing.assert_array_equal(g["minute"], o["minute"], err_msg="minute window of res %d" % r)
    eng.close()
    orc.close()


def test_head_trace_shape():
    """(CPU) the trace reaches what the GPU test is about: long segments, same- and cross-batch references, EXITs
    without one, mixed acquire counts, references more than 2^18 positions back within one resource."""
    spec = _spec()
    ev, cuts = _trace(spec)
    res = ev["res_id"]
    seg = np.bincount(res[cuts[0]:cuts[1]], minlength=len(spec))
    assert (seg > 2000).sum() >= len(spec) - 8
    ex = ev["kind"] == A.EV_EXIT
    ref = (ev["aux"] & np.uint64(A.REF_NONE)).astype(np.int64)
    has = ex & (ref != A.REF_NONE)
    assert (ex & ~has).any()
    idx = np.nonzero(has)[0]
    assert (ref[idx] < cuts[1]).any() and (idx >= cuts[1]).any()
    hot = len(spec) - 1
    hidx = idx[res[idx] == hot]
    rank = np.cumsum(res == hot) - 1  # position within the resource's events
    assert (rank[hidx] - rank[ref[hidx]] > (1 << 18)).any()
    assert set(np.unique(ev["count"][ev["kind"] == A.EV_ENTRY]).tolist()) >= {0, 1, 2, 3}
