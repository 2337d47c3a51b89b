"""Golden vectors (tests/golden/, made by tests/golden/make_golden.py from the oracle).

CPU: the fixtures are intact (SHA-256), the trace generator still produces the same events, and
the oracle still reproduces every decision and bucket.  GPU: the engine reproduces them through
the C ABI.  Rules are rebuilt from the generator arguments in MANIFEST.json.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import pyoracle as O
from sentinel_amd import tracegen as T

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
MANIFEST = json.load(open(os.path.join(HERE, "MANIFEST.json")))
CASES = sorted(MANIFEST)


def _load(name):
    m = MANIFEST[name]
    path = os.path.join(HERE, name + ".npz")
    assert hashlib.sha256(open(path, "rb").read()).hexdigest() == m["sha256"], "fixture %s changed" % name
    return m, np.load(path)  # allow_pickle=False (default): plain arrays only


def _replay(target, m, ev):
    cuts = np.linspace(0, len(ev), m["batches"] + 1).astype(np.int64)
    return np.concatenate([target.submit(ev[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])


def _check_nodes(target, g):
    for i, r in enumerate(g["res"]):
        st = target.read_node(int(r))
        np.testing.assert_array_equal(st["second"][:2], g["second"][i], err_msg="second window res %d" % r)
        np.testing.assert_array_equal(st["minute"], g["minute"][i], err_msg="minute window res %d" % r)


@pytest.mark.parametrize("name", CASES)
def test_golden_oracle(name):
    m, g = _load(name)
    w = T.Workload(m["config"], **m["kwargs"])
    np.testing.assert_array_equal(np.asarray(w.events), g["events"], err_msg="trace generator drifted")
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(orc)
    np.testing.assert_array_equal(_replay(orc, m, g["events"]), g["decisions"])
    _check_nodes(orc, g)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_golden_gpu(name):
    from sentinel_amd import engine as E
    m, g = _load(name)
    w = T.Workload(m["config"], **m["kwargs"])
    eng = E.Engine(max_resources=max(64, w.n_res), max_slot_chain_size=0, status_ring_log2=24)
    w.install(eng)
    np.testing.assert_array_equal(_replay(eng, m, g["events"]), g["decisions"])
    _check_nodes(eng, g)
