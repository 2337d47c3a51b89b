"""HBM traffic per batch of one bench.py config sub-line (a roofline with traffic on every line).

usage: python tools/pmc_configs.py CFG FETCH.csv WRITE.csv KERNEL_STATS.csv [git_head]
  CFG: C2 | C3 | C5 | C5-ext | C6 -- the rocprofv3 passes are of `python3 bench.py --only-config CFG` (jobs script:
  one `--pmc FETCH_SIZE` pass, one `--pmc WRITE_SIZE` pass, one `--kernel-trace --stats` pass, each its own run).

The bytes are counted as tools/pmc_summary.py counts the headline's (FETCH_SIZE doubled for the streaming kernels,
MI355X_MICROARCH.md; per batch = the run's sum over every dispatch / the batches, one k_grp_first dispatch each,
the untimed first batch included).  The entry for CFG in profiles/pmc_configs.json is replaced and stamped with
bench.src_sha(); bench.py reports it as that line's roofline.traffic only while the sources match.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import bench  # noqa: E402
import pmc_summary as P  # noqa: E402

GB = {"C2": 1 << 25, "C3": 1 << 24, "C5": 1 << 23, "C5-ext": 1 << 23, "C6": 1 << 25, "C4": 1 << 25, "C4-ext": 1 << 25}


def main():
    cfg, fpath, wpath, spath = sys.argv[1:5]
    fetch, fcnt = P.load(fpath, "FETCH_SIZE")
    write, _ = P.load(wpath, "WRITE_SIZE")
    nb = max(1, sum(v for k, v in fcnt.items() if k.startswith(("k_rs_first", "k_grp_first"))))
    kern = {}
    for n in sorted(set(fetch) | set(write)):
        if not n.startswith("k_") or n.startswith(P.SKIP):
            continue
        f1, wb = fetch.get(n, 0.0), write.get(n, 0.0)
        rd = (2 * f1) if n.startswith(P.STREAMING) else f1
        kern[n] = {"read_bytes_per_batch": rd / nb, "write_bytes_per_batch": wb / nb,
                   "traffic_bytes_per_batch": (rd + wb) / nb}
    times = {}
    if os.path.exists(spath):
        import csv
        for r in csv.DictReader(open(spath)):
            times[P.short(r["Name"])] = {"calls": int(r["Calls"]), "ms_per_batch": float(r["TotalDurationNs"]) / 1e6 / nb}
    top = sorted(times.items(), key=lambda kv: -kv[1]["ms_per_batch"])[:12]
    rec = {"src_sha": bench.src_sha(), "git_head": sys.argv[5] if len(sys.argv) > 5 else None,
           "batch_events": GB[cfg], "batches_profiled": nb,
           "traffic_bytes_per_batch": sum(v["traffic_bytes_per_batch"] for v in kern.values()),
           "read_bytes_per_batch": sum(v["read_bytes_per_batch"] for v in kern.values()),
           "write_bytes_per_batch": sum(v["write_bytes_per_batch"] for v in kern.values()),
           "top_kernels_ms_per_batch": {k: v["ms_per_batch"] for k, v in top},
           "kernels": kern,
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE / --kernel-trace --stats passes of "
                     "`python3 bench.py --only-config %s`" % cfg}
    # (on the GPU box: PMC_CONFIGS_JSON under gpurun_out/, copied into profiles/ here afterwards)
    out = os.environ.get("PMC_CONFIGS_JSON") or os.path.join(ROOT, "profiles", "pmc_configs.json")
    allr = {}
    if os.path.exists(out):
        with open(out) as f:
            allr = json.load(f)
    allr[cfg] = rec
    with open(out, "w") as f:
        json.dump(allr, f, indent=1, sort_keys=True)
    print(cfg, "traffic %.3f GB per batch (%d batches)" % (rec["traffic_bytes_per_batch"] / 1e9, nb))


if __name__ == "__main__":
    main()
