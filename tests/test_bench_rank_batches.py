"""bench.py's rank batches (--rank-batches): which events of its shard a rank submits as one batch."""
import numpy as np
import pytest

import bench


def _shard(n_global, nparts, rank, seed=3):
    rng = np.random.default_rng(seed)
    owner = rng.integers(0, nparts, n_global)
    return np.nonzero(owner == rank)[0]


@pytest.mark.parametrize("nparts,spec,k", [(2, "auto", 1), (4, "global", 1), (8, "2", 2), (8, "local", 8)])
def test_rank_batch_k(nparts, spec, k):
    assert bench.rank_batch_k(spec, nparts) == k


@pytest.mark.parametrize("kb", [1, 2, 4])
def test_global_batch_cuts(kb):
    # k global batches per rank batch: every cut sits on a global batch boundary of the shard, the batches tile it
    gb, B, S, nparts = 1000, 8, 16, 8  # (k = N is the rank-local layout)
    pos = _shard(gb * B, nparts, 1)
    LB, per_step, cuts = bench.rank_batch_cuts(pos, len(pos), gb, B, S, nparts, kb)
    assert LB == B // kb and per_step == S // kb and len(cuts) == LB + 1
    assert cuts[0] == 0 and cuts[-1] == len(pos) and (np.diff(cuts) > 0).all()
    for b in range(LB):
        seg = pos[cuts[b]:cuts[b + 1]]
        assert seg.min() >= b * kb * gb and seg.max() < (b + 1) * kb * gb


def test_local_cuts_and_one_gpu():
    gb, B, S = 1000, 8, 48
    pos = _shard(gb * B, 8, 5)
    LB, per_step, cuts = bench.rank_batch_cuts(pos, len(pos), gb, B, S, 8, 8)  # rank-local: one batch of the shard
    assert (LB, per_step) == (1, 6) and list(cuts) == [0, len(pos)]
    LB, per_step, cuts = bench.rank_batch_cuts(None, gb * B, gb, B, S, 1, 1)  # one GPU: the base batches as they are
    assert (LB, per_step) == (B, S) and list(cuts) == [b * gb for b in range(B + 1)]


def test_k_must_divide():
    pos = _shard(8000, 4, 0)
    with pytest.raises(AssertionError):
        bench.rank_batch_cuts(pos, len(pos), 1000, 8, 16, 4, 3)


def test_balanced_table_alpha():
    # a resource's load = its events ** alpha: below 1 the hottest resource's rank takes more of the others
    from sentinel_amd import dist as D
    counts = np.array([10_000] + [100] * 400)
    t1 = D.balanced_table(counts, 4)
    t9 = D.balanced_table(counts, 4, 0.5)
    assert t1[0] == t9[0]
    assert (t9 == t9[0]).sum() > (t1 == t1[0]).sum()
    for t in (t1, t9):
        assert set(np.unique(t)) == {0, 1, 2, 3}


def test_config_alg_bytes_and_roofline(tmp_path, monkeypatch):
    # 24 B per event, 4 B per ENTRY, 608 B per touched resource, 2 x 16 B per distinct
    # (resource, args[0]) of the ENTRYs for the hot-parameter configs
    from sentinel_amd import _abi as A
    ev = np.zeros(6, dtype=A.EVENT_DTYPE)
    ev["res_id"] = [1, 1, 2, 1, 2, 3]
    ev["kind"] = [A.EV_ENTRY, A.EV_EXIT, A.EV_ENTRY, A.EV_ENTRY, A.EV_ENTRY, A.EV_TRACE]
    ev["flags"] = [A.F_HAS_ARG, 0, A.F_HAS_ARG, A.F_HAS_ARG, 0, 0]
    ev["aux"] = [7, 0, 7, 7, 9, 0]
    base = 6 * 24 + 4 * 4 + 3 * 608
    assert bench.alg_bytes(ev, False) == base
    assert bench.alg_bytes(ev, True) == base + 2 * 16 * 2  # (1, 7) and (2, 7)
    r = bench.config_roofline("C9", 2.0, 16e9, 1 << 20)
    assert r["bound"] == "hbm" and abs(r["achieved"] - 8000.0) < 1e-6 and abs(r["frac"] - 1.0) < 1e-9
