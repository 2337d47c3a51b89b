"""Regenerate the golden vectors (run by hand, never by the tests).

For each config C1-C5 a small seeded trace is generated with the repo's
trace generator, replayed through the oracle (oracle/ -- the CPU restatement pinned by the
reference's known-answer tests, tests/test_oracle_known_answers.py) in three batches, and
stored as data: the events, the oracle's decision words, and the ClusterNode state of the
touched resources.  MANIFEST.json records the generator arguments and SHA-256 of every file.

    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

import pyoracle as O  # noqa: E402
from sentinel_amd import tracegen as T  # noqa: E402

# small slices of every config: (config, generator kwargs, batches)
CASES = {
    "c1": (1, dict(n_entries=12), 3),  # FlowQpsDemo, 12 s instead of 100 s (n_entries = seconds for C1)
    "c2": (2, dict(n_entries=6000, n_res=500), 3),
    "c3": (3, dict(n_entries=6000, n_res=500), 3),
    "c4": (4, dict(n_entries=6000, n_res=500), 3),
    "c5": (5, dict(n_entries=6000, n_res=500, n_param_values=2000), 3),
}


def replay(config, kw, batches):
    w = T.Workload(config, **kw)
    orc = O.Oracle(max_slot_chain_size=0)
    w.install(orc)
    ev = np.array(w.events, copy=True)
    cuts = np.linspace(0, len(ev), batches + 1).astype(np.int64)
    dec = np.concatenate([orc.submit(ev[a:b]) for a, b in zip(cuts[:-1], cuts[1:])])
    touched = np.unique(ev["res_id"])
    sec = np.stack([orc.read_node(int(r))["second"][:2] for r in touched])
    minute = np.stack([orc.read_node(int(r))["minute"] for r in touched])
    return w, ev, dec, touched, sec, minute


def sha(path):
    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def main():
    manifest = {}
    for name, (config, kw, batches) in CASES.items():
        w, ev, dec, touched, sec, minute = replay(config, kw, batches)
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, events=ev, decisions=dec, res=touched, second=sec, minute=minute)
        manifest[name] = {"config": config, "kwargs": kw, "seed": w.seed, "batches": batches,
                          "n_events": int(len(ev)), "sha256": sha(path)}
        print(name, len(ev), "events")
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
