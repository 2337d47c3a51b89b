"""Parity of the engine's non-default paths, selected by environment knobs that the library reads once per
engine (each runs in a child process; DESIGN.md §10 lists every switch):

  SG_PIPELINE=0            group and decide stages back to back (no overlap of batch k+1's grouping)
  SG_J1_STREAM=1 / 2       the J1 owners after J16 / J8 on bin_stream[0] instead of after the lane bins / halved over
                           both bin streams
  SG_RADIX_BELOW=0         the hot / cold group stage for batches of every size
  SG_STREAM_PRIO=1 / 0     the decide streams at the higher priority / default stream priorities
  SG_DEBUG_FLAGS=8192      the all-radix group stage (k_rs_first / k_scatter_rec) instead of the hot / cold split
  SG_PQ=0                  hot-parameter resources on the per-lane kernel (no k_pq)
  SG_MIX=0 / SG_MIX_PQ=0   mixed flow / degrade / param resources on one lane (no cooperative passes)
  SG_PV=0, SG_PVT=0        the value-parallel pre pass without its post pass, and the reverse
  SG_DEBUG_FLAGS=4 / 8 / 16 / 128   no frozen-stretch skipping / the decide bins one after another on one stream /
                           no closed-form guesses in the cooperative owners / the 512-lane k_pq for wide segments
  SG_DEBUG_FLAGS=288       k_pq's map phases: sequential key walks (32) and the thread-count map sorted again (256)

Each child replays a seeded trace (C3: THREAD + rate-limiter rules with warm-up rate limiters; C4: DegradeRules + QPS rules; C5: hot-parameter rules; C6: mixed rules;
several batches) through the HIP engine and the oracle and requires bit-identical decisions and node state.
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
cfg = %(cfg)d
w = T.Workload(cfg, n_entries=300_000, n_res={3: 2_000, 4: 30_000, 5: 1_000, 6: 3_000}[cfg],
               **({"n_param_values": 200_000} if cfg in (5, 6) else {"variant": T.V_WARM_RL} if cfg == 3 else {}))
eng = E.Engine(max_resources=w.n_res, max_slot_chain_size=0, status_ring_log2=24,
               **({"param_table_log2": 24} if cfg in (5, 6) else {}))
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


@pytest.mark.parametrize("env,cfg", [("SG_PIPELINE=0", 4), ("SG_STREAM_PRIO=1", 4), ("SG_STREAM_PRIO=0", 4),
                                     ("SG_DEBUG_FLAGS=8192", 4), ("SG_DEBUG_FLAGS=8192", 6), ("SG_PQ=0", 5),
                                     ("SG_MIX=0", 6), ("SG_MIX_PQ=0", 6), ("SG_PVT=0", 6), ("SG_PV=0 SG_PVT=1", 6),
                                     ("SG_DEBUG_FLAGS=4", 3), ("SG_DEBUG_FLAGS=8", 4), ("SG_DEBUG_FLAGS=16", 3),
                                     ("SG_DEBUG_FLAGS=128 SG_PQ_WIDE=512", 5),
                                     ("SG_DEBUG_FLAGS=288", 5), ("SG_J1_STREAM=1", 4), ("SG_J1_STREAM=1", 3),
                                     ("SG_J1_STREAM=2", 4), ("SG_J1_STREAM=2", 3), ("SG_RADIX_BELOW=0", 6),
                                     ("SG_PIPELINE=0", 6), ("SG_STREAM_PRIO=0", 6)])
def test_alternative_path_parity(env, cfg):
    child_env = dict(os.environ)
    for kv in env.split():
        k, v = kv.split("=")
        child_env[k] = v
    p = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT, "cfg": cfg}], env=child_env, capture_output=True,
                       text=True, timeout=110)
    assert p.returncode == 0 and p.stdout.startswith("ok"), p.stdout[-2000:] + p.stderr[-2000:]
