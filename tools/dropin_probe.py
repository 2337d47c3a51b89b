"""Drop-in A/B on one box: the latency floor (bench.latency_line) with the tiny-batch path on and off
(SG_TINY), and the 65,536-event operating point (bench.dropin_line) with the hot/cold group stage and the all-radix one
(SG_DEBUG_FLAGS=8192).  One JSON line per variant.  Usage: python tools/dropin_probe.py [n_batches]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    import torch
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    torch.zeros(1, device=dev)
    from sentinel_amd import tracegen as T
    w, ev = bench.make_trace(1_000_000, 1 << 25, 1, T.SEED_BASE + 4)  # (the headline trace's first global batch)
    for tiny in ("1", "0"):
        os.environ["SG_TINY"] = tiny
        r = bench.latency_line(dev, w, ev, sizes=(1, 16, 64, 256, 1024), calls=1000, warm=100)
        print(json.dumps({"variant": "SG_TINY=" + tiny, **r}), flush=True)
    os.environ["SG_TINY"] = "1"
    for fl in ("0", "8192", "0", "8192"):
        os.environ["SG_DEBUG_FLAGS"] = fl
        r = bench.dropin_line(dev, w, ev, n_batches=nb)
        print(json.dumps({"variant": "SG_DEBUG_FLAGS=" + fl, **r}), flush=True)
    os.environ.pop("SG_DEBUG_FLAGS")


if __name__ == "__main__":
    main()
