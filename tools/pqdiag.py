"""Diagnostics: replay tests/test_gpu_pq.py's synthetic thread-map trace and print, at the first mismatch, the
history of the mismatching (resource, value) with both sides' decisions.  usage: python tools/pqdiag.py [rt_max]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import pyoracle as O  # noqa: E402
import test_gpu_pq as P  # noqa: E402
from sentinel_amd import _abi as A  # noqa: E402
from sentinel_amd import engine as E  # noqa: E402

rt_max = int(sys.argv[1]) if len(sys.argv) > 1 else 30
eng = E.Engine(max_resources=64, max_slot_chain_size=0, param_table_log2=20, status_ring_log2=24)
orc = O.Oracle(max_slot_chain_size=0)
for nm in P.NAMES:
    eng.register(nm), orc.register(nm)
rules = P._rules()
eng.load_param_rules(rules), orc.load_param_rules(rules)
t, gbase = P.T0, 0
hist_ev, hist_dg, hist_do = [], [], []
for b in range(7):
    if b == 5:
        rules = P._rules(thread_on_m3=True)
        eng.load_param_rules(rules), orc.load_param_rules(rules)
    ev = P._synthetic(100 + b, 40_000, gbase, t=t, rt_max=rt_max, exit_args=0.9)
    if b % 3 == 1:
        ext = np.zeros(len(ev), dtype=A.EXT_DTYPE)
        dg, do = eng.submit_ex(ev, ext), orc.submit_ex(ev, ext)
    else:
        dg, do = eng.submit(ev), orc.submit(ev)
    hist_ev.append(ev), hist_dg.append(dg), hist_do.append(do)
    bad = np.nonzero(dg != do)[0]
    print("batch", b, "events", len(ev), "gbase", gbase, "mismatches", len(bad), flush=True)
    if len(bad):
        allev = np.concatenate(hist_ev)
        alldg = np.concatenate(hist_dg)
        alldo = np.concatenate(hist_do)
        i = gbase + int(bad[0])
        res, key = int(allev["res_id"][i]), int(allev["aux"][i])
        print("first mismatch global", i, "res", res, "key", hex(key), "all bad (batch-local):", bad[:10].tolist())
        ent = np.nonzero((allev["res_id"] == res) & (allev["kind"] == A.EV_ENTRY) & (allev["aux"] == key))[0]
        ex = np.nonzero((allev["res_id"] == res) & (allev["kind"] == A.EV_EXIT))[0]
        refs = allev["aux"][ex] & A.REF_NONE
        rows = []
        for e in ent:
            rows.append((int(e), "ENTRY", int(allev["ts"][e]), int(allev["count"][e]), hex(int(alldg[e])), hex(int(alldo[e]))))
            j = ex[refs == e]
            for x in j:
                rows.append((int(x), "EXIT(ref %d)%s" % (e, " args" if allev["flags"][x] & A.F_EXIT_ARGS else ""),
                             int(allev["ts"][x]), 1, "", ""))
        rows.sort()
        for r in rows:
            if r[0] <= i + 50:
                print("  %8d %-24s ts %d cnt %d gpu %s orc %s" % r)
        break
    gbase += len(ev)
    t = int(ev["ts"].max()) + 1
