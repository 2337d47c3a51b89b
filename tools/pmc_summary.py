"""Per-launch HBM traffic of bench.py's kernels from two rocprofv3 --pmc passes.

usage: python tools/pmc_summary.py FETCH_counter_collection.csv WRITE_counter_collection.csv OUT.json

MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced streaming read, so it is doubled here (other access
widths are uncalibrated -- the doubled figure is an upper-bound style estimate for them).
The decide stage's traffic is the sum over its kernels of the mean per-dispatch bytes.
"""
import csv
import json
import sys
from collections import defaultdict

DECIDE = ("k_jac", "k_lane", "k_lite", "k_fill", "k_resolve")


def load(path, counter):
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[name].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in per.items()}


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    names = sorted(set(fetch) | set(write))
    kern = {n: {"fetch_bytes_x2": 2 * fetch.get(n, 0.0), "write_bytes": write.get(n, 0.0)} for n in names}
    for v in kern.values():
        v["traffic_bytes"] = v["fetch_bytes_x2"] + v["write_bytes"]
    decide = sum(v["traffic_bytes"] for n, v in kern.items() if n.startswith(DECIDE))
    pipeline = sum(v["traffic_bytes"] for n, v in kern.items() if n.startswith("k_") and n != "k_init_state")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of `python3 bench.py --steps 3 --warmup 1`",
           "units": "bytes per launch (mean over dispatches); FETCH_SIZE doubled per MI355X_MICROARCH.md",
           "decide_stage_traffic_bytes": decide, "pipeline_traffic_bytes_per_step": pipeline, "kernels": kern}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps({"decide_stage_traffic_bytes": decide, "pipeline_traffic_bytes_per_step": pipeline}))


if __name__ == "__main__":
    main()
