"""Edge cases of the hot / cold group stage (kernels.hip k_grp_*).

A batch's resources with >= max(64, n / 8192) events become the next batch's hot ids (k_hot_build, at most
HOT_MAX = 1024, first come); a hot resource's events skip the cold radix passes and land contiguous in one pass.
The hot ids are a batch old, so a resource can be hot-id'd with few or no events, turn cold with many, and EXITs
can name ENTRYs decided on the other path a batch earlier.  This trace forces each case on purpose:

* more than HOT_MAX qualifying resources (2,000 resources with ~140 events a batch: only 1,024 get ids);
* resource 1 flips hot -> short (hot id, 10 ENTRYs) -> long again (cold path, its previous segment was short);
* resource 2 is hot-id'd for a batch in which it has no event at all, then long again on the cold path;
* resource 3 goes cold-long -> hot-id'd-short -> cold-long;
* every ENTRY is followed by its EXIT after an RT of up to 400 ms, so ~1/5 of the EXITs of each resource name an
  ENTRY of the previous batch (decided on the other path), and 5 % are followed by a TRACE.

Every decision and the touched resources' windows are compared with the oracle, with the default decide bins and
with the cooperative owners skipping every frozen stretch (the hot segments' spans, k_fill).
"""
import numpy as np
import pytest

import pyoracle as O
from sentinel_amd import _abi as A
from sentinel_amd import engine as E
from sentinel_amd import tracegen as T

pytestmark = pytest.mark.gpu

T0 = 1_700_000_000_000
N_RES = 4000
MANY = range(100, 2100)  # 2,000 resources past the hot threshold each batch


def _plan():
    """Per batch (1 s of trace time each): {resource: ENTRYs}."""
    many = {r: 70 for r in MANY}
    return [
        {1: 6000, 2: 6000, 3: 10, **many},
        {1: 10, 3: 6000, **many},              # 1: hot id, short; 2: hot id, absent; 3: cold, long
        {1: 6000, 2: 6000, 3: 10, **many},     # 1 and 2 long on the cold path; 3: hot id, short
        {1: 3000, 2: 20, 3: 3000, **many},
    ]


def _trace(plan, seed=11):
    rng = np.random.default_rng(seed)
    ts, res, kind, ref_of, rt = [], [], [], [], []
    for b, spec in enumerate(plan):
        for r, k in spec.items():
            t = T0 + b * 1000 + np.sort(rng.integers(0, 1000, k))
            d = rng.integers(1, 400, k)
            tr = rng.random(k) < 0.05
            base = len(ts)
            n = k + k + int(tr.sum())
            ts.extend(t.tolist() + (t + d).tolist() + (t[tr] + d[tr] - 1).tolist())
            res.extend([r] * n)
            kind.extend([A.EV_ENTRY] * k + [A.EV_EXIT] * k + [A.EV_TRACE] * int(tr.sum()))
            ref_of.extend([-1] * k + list(range(base, base + k)) + [base + j for j in np.nonzero(tr)[0]])
            rt.extend([0] * k + d.tolist() + [0] * int(tr.sum()))
    ts, res, kind, ref_of, rt = map(np.asarray, (ts, res, kind, ref_of, rt))
    # event order: time, then ENTRY before the EXIT / TRACE of the same millisecond (an EXIT follows its ENTRY)
    order = np.lexsort((kind, ts))
    pos = np.empty(len(order), dtype=np.int64)
    pos[order] = np.arange(len(order))
    ev = np.zeros(len(order), dtype=A.EVENT_DTYPE)
    ev["ts"] = ts[order]
    ev["res_id"] = res[order]
    ev["count"] = 1
    ev["kind"] = kind[order]
    ref = ref_of[order]
    aux = np.full(len(order), A.REF_NONE, dtype=np.uint64)
    has = ref >= 0
    aux[has] = pos[ref[has]].astype(np.uint64)
    ex = ev["kind"] == A.EV_EXIT
    aux[ex] |= rt[order][ex].astype(np.uint64) << np.uint64(48)
    ev["aux"] = aux
    cuts = np.searchsorted(ev["ts"], T0 + 1000 * np.arange(len(plan) + 1))
    cuts[-1] = len(ev)
    return ev, cuts


@pytest.mark.parametrize("mode", ["default", "skip"])
def test_hot_cold_flips_cap_and_absent_ids(mode, monkeypatch):
    monkeypatch.setenv("SG_RADIX_BELOW", "0")  # (every batch on the hot / cold stage, whatever its size)
    if mode == "skip":
        monkeypatch.setenv("SG_SKIP_MIN", "16")
    ev, cuts = _trace(_plan())
    assert ((ev["kind"] == A.EV_EXIT) & (ev["aux"] & np.uint64(A.REF_NONE) < cuts[1]) &
            (np.arange(len(ev)) >= cuts[1])).any()  # EXITs across the first batch boundary
    w = T.Workload(4, n_res=N_RES, n_entries=1000)
    eng = E.Engine(max_resources=N_RES, max_slot_chain_size=0, status_ring_log2=24)
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(eng)
    w.install(orc)
    for b, (a, e) in enumerate(zip(cuts[:-1], cuts[1:])):
        dg, do = eng.submit(ev[a:e]), orc.submit(ev[a:e])
        bad = np.nonzero(dg != do)[0]
        assert not len(bad), ("batch", b, int(a + bad[0]), ev[a + bad[0]], hex(dg[bad[0]]), hex(do[bad[0]]), len(bad))
    for r in [1, 2, 3] + list(MANY[:20]) + list(MANY[-20:]):
        g, o = eng.read_node(int(r)), orc.read_node(int(r))
        assert g["thread"] == o["thread"], r
        np.testing.assert_array_equal(g["second"][:2], o["second"][:2], err_msg="second window of res %d" % r)
        np.testing.assert_array_equal(g["minute"], o["minute"], err_msg="minute window of res %d" % r)
    eng.close()
    orc.close()
