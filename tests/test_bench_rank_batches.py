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
