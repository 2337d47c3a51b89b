"""Token server on the device (sg_cluster_request_tokens) against the CPU oracle.

DefaultTokenService.requestToken (csrv/flow/DefaultTokenService.java:37-48) ->
GlobalRequestLimiter (csrv/flow/statistic/limit/RequestLimiter.java:72-87) ->
ClusterFlowChecker.acquireClusterToken (csrv/flow/ClusterFlowChecker.java:55-112).
Results must be identical: status, remaining and wait of every request.
"""
import numpy as np
import pytest

import pyoracle as O
from sentinel_amd import _abi as A
from sentinel_amd import engine as E

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_123


def _rule(fid, count, res="abc", **kw):
    kw.setdefault("cluster_threshold_type", A.CLUSTER_THRESHOLD_GLOBAL)
    return A.flow_rule(res, count, cluster_mode=True, cluster_flow_id=fid, **kw)


def _pair(**cfg):
    eng = E.Engine(max_resources=64, **cfg)
    orc = O.Oracle(**cfg)
    for x in (eng, orc):
        x.register("abc")
    return eng, orc


def test_cluster_flow_checker_occupy_sequence():
    # csrv-test/flow/ClusterFlowCheckerTest.java:37-70 (disabled in the reference; replayed on trace time)
    eng, _ = _pair()
    eng.load_flow_rules([_rule(98765, 5, cluster_sample_count=5)])
    t = T0 - T0 % 1000
    seq = []

    def acq(occupy):
        return eng.cluster_request([(t, 98765, 1, occupy)])[0]

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
    OK, BL, W = A.TOKEN_OK, A.TOKEN_BLOCKED, A.TOKEN_SHOULD_WAIT
    assert [s for s, _, _ in seq] == [OK, OK, OK, OK, OK, BL, BL, BL, BL, W, BL, OK]
    assert seq[9][2] == 200


def test_bad_request_no_rule_and_limiter():
    eng, orc = _pair(cluster_max_allowed_qps=3)
    for x in (eng, orc):
        x.load_flow_rules([_rule(7, 100)])
    t = T0 - T0 % 1000
    reqs = [(t, 0, 1, False), (t, 7, 0, False), (t, 9, 1, False)] + [(t, 7, 1, False)] * 5 + \
           [(t + 999, 7, 1, False), (t + 1000, 7, 1, False)]
    got = eng.cluster_request(reqs)
    assert got == orc.cluster_request(reqs)
    assert [s for s, _, _ in got] == [A.TOKEN_BAD_REQUEST, A.TOKEN_BAD_REQUEST, A.TOKEN_NO_RULE_EXISTS] + \
        [A.TOKEN_OK] * 3 + [A.TOKEN_TOO_MANY_REQUEST] * 3 + [A.TOKEN_OK]


def test_rule_reload_keeps_metric_and_drops_flows():
    eng, orc = _pair()
    t = T0 - T0 % 1000
    steps = [
        ([_rule(7, 2), _rule(7, 3), _rule(8, 1)], [(t, 7, 1, False)] * 4 + [(t, 8, 1, False)] * 2),
        ([_rule(7, 5, cluster_sample_count=2)], [(t + 10, 7, 1, False)] * 3 + [(t + 10, 8, 1, False)]),
        ([_rule(7, 9.5), _rule(8, 1)], [(t + 20, 7, 2, False), (t + 20, 8, 1, False)]),
        ([_rule(8, 2, cluster_threshold_type=A.CLUSTER_THRESHOLD_AVG_LOCAL)], [(t + 30, 8, 1, False)] * 2),
    ]
    for rules, reqs in steps:
        for x in (eng, orc):
            x.load_flow_rules(rules)
        assert eng.cluster_request(reqs) == orc.cluster_request(reqs)
    for x in (eng, orc):
        x.cluster_set_connected(8, 3)
    reqs = [(t + 40, 8, 1, False)] * 8
    assert eng.cluster_request(reqs) == orc.cluster_request(reqs)


def _random_requests(rng, n, fids, t0, bad_frac=0.02):
    ts = t0 + np.cumsum(rng.integers(0, 4, n))
    p = 1.0 / np.arange(1, len(fids) + 1) ** 1.1
    p /= p.sum()
    fid = np.asarray(fids)[rng.choice(len(fids), n, p=p)]
    acq = rng.integers(1, 4, n)
    pri = rng.random(n) < 0.3
    bad = rng.random(n)
    fid = np.where(bad < bad_frac / 2, 10 ** 9 + 7, fid)  # no rule
    acq = np.where((bad >= bad_frac / 2) & (bad < bad_frac), 0, acq)  # bad request
    out = np.zeros(n, dtype=A.TOKEN_REQ_DTYPE)
    out["ts"], out["flow_id"], out["acquire_count"], out["prioritized"] = ts, fid, acq, pri
    return out


@pytest.mark.parametrize("allowed,light", [(-1, None), (400, None), (-1, "0"), (400, "1000000")])
def test_random_parity(allowed, light, monkeypatch):
    # light: SG_TOK_LIGHT (cluster.hip: flows of more requests a call on a 1024-lane workgroup, the rest on one wave);
    # "0" every flow on the wide one, "1000000" every flow on one wave
    if light is not None:
        monkeypatch.setenv("SG_TOK_LIGHT", light)
    rng = np.random.default_rng(20240601 + 5)
    eng, orc = _pair(cluster_max_allowed_qps=allowed)
    fids = list(range(101, 141))
    rules = []
    for f in fids:
        sc = int(rng.choice([1, 2, 5, 10, 20]))
        win = int(rng.choice([500, 1000, 2000]))
        thr = A.CLUSTER_THRESHOLD_GLOBAL if f % 3 else A.CLUSTER_THRESHOLD_AVG_LOCAL
        rules.append(_rule(f, float(rng.integers(5, 200)), res="r%d" % f, cluster_sample_count=sc,
                           cluster_window_interval_ms=win, cluster_threshold_type=thr))
    for x in (eng, orc):
        x.load_flow_rules(rules)
        for f in fids:
            if f % 3 == 0:
                x.cluster_set_connected(f, int(f % 5))
    reqs = _random_requests(rng, 60_000, fids, T0)
    for a, b in [(0, 1), (1, 5000), (5000, 30000), (30000, 60000)]:
        got = eng.cluster_request_array(reqs[a:b])
        want = orc.cluster_request([tuple(int(v) for v in r) for r in reqs[a:b]])
        want = np.array(want, dtype=np.int64)
        g = np.stack([got["status"], got["remaining"], got["wait_in_ms"]], axis=1).astype(np.int64)
        bad = np.nonzero((g != want).any(axis=1))[0]
        assert len(bad) == 0, "request %d: gpu %s oracle %s (%d mismatches)" % (a + bad[0], g[bad[0]], want[bad[0]],
                                                                                 len(bad))
    st = np.asarray([s for s in eng.cluster_request_array(reqs[:0])["status"]])
    assert len(st) == 0


def test_unordered_requests_rejected():
    eng, _ = _pair()
    eng.load_flow_rules([_rule(7, 5)])
    with pytest.raises(E.SentinelError):
        eng.cluster_request([(T0 + 5, 7, 1, False), (T0, 7, 1, False)])


def _flows_10k(rng, n_flows=10_000):
    fids = np.arange(1_000_001, 1_000_001 + n_flows)
    rules = []
    for f in fids:
        rules.append(A.flow_rule("r%d" % f, float(int(np.exp(rng.uniform(np.log(1e3), np.log(1e5))))),
                                 cluster_mode=True, cluster_flow_id=int(f),
                                 cluster_threshold_type=A.CLUSTER_THRESHOLD_GLOBAL,
                                 cluster_sample_count=int(rng.choice([1, 2, 5, 10])),
                                 cluster_window_interval_ms=int(rng.choice([500, 1000, 2000]))))
    return fids, rules


def _requests_10k(rng, fids, n, seconds):
    ts = T0 + np.sort(rng.integers(0, seconds * 1000, n))
    p = 1.0 / np.arange(1, len(fids) + 1) ** 1.1
    p /= p.sum()
    out = np.zeros(n, dtype=A.TOKEN_REQ_DTYPE)
    out["ts"], out["flow_id"] = ts, fids[rng.choice(len(fids), n, p=p)]
    out["acquire_count"] = rng.integers(1, 4, n)
    out["prioritized"] = rng.random(n) < 0.2
    return out


def test_ten_thousand_global_flows():
    # SURVEY.md §8(d) C5's cluster half at config size: 10k flowIds with GLOBAL thresholds of
    # 10^3..10^5 per window (1-10 samples of 0.5-2 s), Zipf(1.1) over the flows, 3M requests over 12 s through the
    # token server with device-resident buffers, against the oracle request by request
    rng = np.random.default_rng(20240601 + 15)
    fids, rules = _flows_10k(rng)
    eng = E.Engine(max_resources=16_384, cluster_max_allowed_qps=400_000)  # the namespace limiter above the traffic
    orc = O.Oracle(cluster_max_allowed_qps=400_000)
    for x in (eng, orc):
        for f in fids:
            x.register("r%d" % f)
        x.load_flow_rules(rules)
    reqs = _requests_10k(rng, fids, 3_000_000, 12)
    import torch
    dev = torch.device("cuda", 0)
    dq = torch.from_numpy(reqs.view(np.uint8).copy()).to(dev)
    dr = torch.empty(len(reqs) * A.TOKEN_RES_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    rq, rs = A.TOKEN_REQ_DTYPE.itemsize, A.TOKEN_RES_DTYPE.itemsize
    cuts = [0, 1, 250_000, 1_000_000, 2_000_000, len(reqs)]
    for a, b in zip(cuts[:-1], cuts[1:]):
        eng.cluster_request_ptr(dq.data_ptr() + a * rq, b - a, dr.data_ptr() + a * rs)
    got = dr.cpu().numpy().view(A.TOKEN_RES_DTYPE)
    want = np.concatenate([orc.cluster_request_array(reqs[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    for k in ("status", "remaining", "wait_in_ms"):
        bad = np.nonzero(got[k] != want[k])[0]
        assert len(bad) == 0, "%s of request %d: gpu %s oracle %s (%d mismatches)" % (
            k, bad[0], got[bad[0]], want[bad[0]], len(bad))
    st = np.bincount(got["status"] + 1)
    assert (got["status"] == A.TOKEN_OK).sum() > 0 and (got["status"] == A.TOKEN_BLOCKED).sum() > 1000, st
