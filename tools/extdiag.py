"""Diagnostics: sg_submit vs sg_submit_ex (contexts / origins) vs the oracle on a small C4/C2 trace."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402
import pyoracle as O  # noqa: E402
from sentinel_amd import engine as E, tracegen as T, _abi as A  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 4
n_ent = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
w = T.Workload(cfg, seed=T.SEED_BASE + 40 + cfg, n_res=3000, n_entries=n_ent)
ev = w.events
orc = O.Oracle(max_slot_chain_size=0)
w.install(orc)
io, ic = w.intern_names(orc)
ext = T.ext_for(ev, io, ic, seed=5)
do = orc.submit_ex(ev, ext)
cnt = np.bincount(ev["res_id"], minlength=3000)


def run(name, use_ext, zero_ext=False, env=None):
    for k, v in (env or {}).items():
        os.environ[k] = v
    eng = E.Engine(max_resources=4096, max_slot_chain_size=0, status_ring_log2=24, aux_node_capacity=1 << 17)
    for k in (env or {}):
        del os.environ[k]
    w.install(eng)
    w.intern_names(eng)
    x = ext.copy()
    if zero_ext:
        x["origin_id"] = 0
        x["context_id"] = 0
    dg = eng.submit_ex(ev, x) if use_ext else eng.submit(ev)
    bad = np.nonzero(dg != do)[0]
    print("%-28s mismatches %d" % (name, len(bad)), flush=True)
    for b in bad[:4]:
        r = int(ev["res_id"][b])
        print("   ev %d %s gpu %08x orc %08x res %d cnt %d" % (b, ev[b], dg[b], do[b], r, cnt[r]), flush=True)
    eng.close()


run("submit", False)
run("submit_ex zero ctx/origin", True, zero_ext=True)
run("submit_ex ctx/origin", True)
run("submit_ex force lane", True, env={"SG_DEBUG_FLAGS": "2"})
run("submit force lane", False, env={"SG_DEBUG_FLAGS": "2"})
