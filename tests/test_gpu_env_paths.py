"""Parity of the engine's alternative group-stage paths, selected by environment knobs that the
library reads once per process (so each runs in a child process):

  SG_PIPELINE=0            group and decide stages back to back (no overlap of batch k+1's grouping)
  SG_STREAM_PRIO=1         the decide streams at the higher priority (default: the group stream)
  SG_STREAM_PRIO=0         default stream priorities

Each child replays a seeded C4 trace (DegradeRules + QPS rules, several batches) through the HIP
engine and the oracle and requires bit-identical decisions and node state.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
sys.path[:0] = [%(root)r, %(root)r + '/oracle', %(root)r + '/tests']
import numpy as np
import pyoracle as O
from sentinel_amd import engine as E
from sentinel_amd import tracegen as T
w = T.Workload(4, n_entries=300_000, n_res=30_000)
eng = E.Engine(max_resources=w.n_res, max_slot_chain_size=0, status_ring_log2=24)
orc = O.Oracle(max_slot_chain_size=0)
w.install(eng); w.install(orc)
ev = w.events
cuts = np.linspace(0, len(ev), 4).astype(np.int64)
for a, b in zip(cuts[:-1], cuts[1:]):
    dg, do = eng.submit(ev[a:b]), orc.submit(ev[a:b])
    bad = np.nonzero(dg != do)[0]
    assert not len(bad), ("mismatch", int(a + bad[0]), len(bad))
cnt = np.bincount(ev["res_id"], minlength=w.n_res)
for r in list(np.argsort(-cnt)[:30]) + list(np.nonzero(cnt)[0][::997]):
    g, o = eng.read_node(int(r)), orc.read_node(int(r))
    assert np.array_equal(g["minute"], o["minute"]) and np.array_equal(g["second"][:2], o["second"][:2]), r
print("ok", len(ev))
"""


@pytest.mark.parametrize("env", ["SG_PIPELINE=0", "SG_STREAM_PRIO=1", "SG_STREAM_PRIO=0"])
def test_alternative_path_parity(env):
    k, v = env.split("=")
    child_env = dict(os.environ, **{k: v})
    p = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT}], env=child_env, capture_output=True,
                       text=True, timeout=110)
    assert p.returncode == 0 and p.stdout.startswith("ok"), p.stdout[-2000:] + p.stderr[-2000:]
