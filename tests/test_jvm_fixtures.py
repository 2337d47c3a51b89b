"""Fixtures written by the reference itself (java/src/test/.../ReplayHarness.java, imported with
tools/jvm_replay.py): the oracle must decide what the unmodified reference decided and end with
the same ClusterNode buckets.  Decision words are compared on status and rule slot (the harness
cannot observe waits).  This image has no JVM, so no fixture exists yet and the test skips; any
tests/golden/jvm_*.npz dropped in is picked up."""
import glob
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURES = sorted(glob.glob(os.path.join(HERE, "golden", "jvm_*.npz")))


@pytest.mark.skipif(not FIXTURES, reason="no JVM replay fixtures (the image has no JVM; see INTEGRATION.md §3)")
@pytest.mark.parametrize("path", FIXTURES, ids=[os.path.basename(p) for p in FIXTURES])
def test_oracle_matches_the_reference_replay(path):
    import pyoracle as O
    from sentinel_amd import tracegen as T
    z = np.load(path, allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    w = T.Workload(meta["config"], seed=meta["seed"], **meta["kwargs"])
    assert np.array_equal(np.asarray(w.events), z["events"]), "the fixture's trace is not the regenerated one"
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(orc)
    ev = z["events"]
    cuts = np.linspace(0, len(ev), 4).astype(np.int64)
    dec = np.concatenate([orc.submit(ev[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    mask = np.uint32(0xFFFF)
    bad = np.nonzero((dec & mask) != (z["decisions"] & mask))[0]
    assert len(bad) == 0, "first mismatch at event %d: oracle %#x, reference %#x" % (
        bad[0], dec[bad[0]], z["decisions"][bad[0]])
    for i, r in enumerate(z["res"]):
        node = orc.read_node(int(r))
        assert np.array_equal(node["second"][:2], z["second"][i]), int(r)
        assert np.array_equal(node["minute"], z["minute"][i]), int(r)
