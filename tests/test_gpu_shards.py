"""The multi-GPU partition with HIP engines: every rank's shard of one C4 trace, decided by its
own engine in rank-local batches as bench.py --gpus N submits it, gives exactly the decisions one oracle gives
for those events over the whole trace.  Decisions depend only on the resource's own state
(core/slots/block/degrade/DegradeRule.java:177 reads the resource's own ClusterNode), so any partition of the
resources is exact; this checks the HIP path on the shards (references rewritten to each rank's numbering,
batches spanning N global batches' worth of trace time) for the balanced table and for the hash."""
import numpy as np
import pytest

import pyoracle as O
from sentinel_amd import dist as D
from sentinel_amd import engine as E
from sentinel_amd import tracegen as T

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sharding", ["balanced", "hash"])
def test_hip_shards_equal_whole_trace_oracle(sharding):
    n = 8
    w = T.Workload(4, n_entries=600_000, n_res=50_000)
    ev = w.events
    whole = O.Oracle(max_slot_chain_size=0)
    w.install(whole)
    ref = whole.submit(ev)
    table = D.balanced_table(np.bincount(ev["res_id"], minlength=w.n_res), n) if sharding == "balanced" else None
    seen = 0
    for r in range(n):
        mine, pos = D.shard_stream(ev, n, r, table)
        eng = E.Engine(max_resources=w.n_res, max_slot_chain_size=0, status_ring_log2=22)
        w.install(eng)
        cuts = np.linspace(0, len(mine), 3).astype(np.int64)  # two rank-local batches
        got = np.concatenate([eng.submit(mine[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
        bad = np.nonzero(got != ref[pos])[0]
        assert not len(bad), (r, int(pos[bad[0]]), hex(got[bad[0]]), hex(ref[pos][bad[0]]), len(bad))
        for res in np.unique(mine["res_id"])[:20]:
            g, o = eng.read_node(int(res)), whole.read_node(int(res))
            assert g["thread"] == o["thread"] and np.array_equal(g["minute"], o["minute"]), (r, res)
        seen += len(pos)
        eng.close()
    assert seen == len(ev)
