"""Per-batch HBM traffic and kernel time of bench.py from rocprofv3 passes (tools/profile.sh).

usage: python tools/pmc_summary.py FETCH.csv WRITE.csv KERNEL_STATS.csv OUT.json [git_head]

MI355X_MICROARCH.md (HBM section): FETCH_SIZE and WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced streaming read, so it is doubled for the kernels whose reads
are coalesced streams (STREAMING below); the reads of the random-access kernels (per-lane segment walks,
gathers) are uncalibrated and taken as counted.  Reads and writes are reported separately, and the
all-doubled figure of earlier rounds is kept as traffic_upper_bytes_per_batch.
Totals are summed over every dispatch of the run and divided by the number of batches (one
k_grp_first or k_rs_first dispatch per batch), so kernels launched several times per batch (radix passes, scans)
count every launch (k_grp_first, the hot / cold group stage's first pass, or k_rs_first, the radix one).  The JSON is stamped with bench.src_sha() of the sources it was measured on;
bench.py reports its traffic only when that stamp matches the sources it runs.
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

DECIDE = ("k_jac", "k_lane", "k_lite", "k_fill", "k_resolve", "k_chain", "k_pq")
# kernels whose loads are wide coalesced streams (events, keys, sorted records, histograms)
STREAMING = ("k_grp_first", "k_grp_records", "k_hot_scan", "k_rs_first", "k_radix_hist", "k_radix_scatter", "k_scan_", "k_seg_count", "k_seg_emit", "k_block_sums",
             "k_scatter_rec", "k_fill", "k_jac")
SKIP = ("k_init_state", "k_snap_", "k_set_flags")


def short(name):
    return name.split("(")[0].replace("void ", "")


def load(path, counter):
    tot, cnt = defaultdict(float), defaultdict(int)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        n = short(r["Kernel_Name"])
        tot[n] += float(r["Counter_Value"]) * 1024.0
        cnt[n] += 1
    return tot, cnt


def main():
    fetch, fcnt = load(sys.argv[1], "FETCH_SIZE")
    write, _ = load(sys.argv[2], "WRITE_SIZE")
    nb = max(1, sum(v for k, v in fcnt.items() if k.startswith(("k_rs_first", "k_grp_first"))))
    names = sorted(set(fetch) | set(write))
    kern = {}
    for n in names:
        if not n.startswith("k_") or n.startswith(SKIP):  # engine kernels only (no torch / rocclr setup copies)
            continue
        f1, wb = fetch.get(n, 0.0), write.get(n, 0.0)
        rd = (2 * f1) if n.startswith(STREAMING) else f1
        kern[n] = {"launches_per_batch": fcnt.get(n, 0) / nb, "fetch_counted_per_batch": f1 / nb,
                   "read_bytes_per_batch": rd / nb, "streaming_reads": n.startswith(STREAMING),
                   "write_bytes_per_batch": wb / nb, "traffic_bytes_per_batch": (rd + wb) / nb,
                   "traffic_upper_bytes_per_batch": (2 * f1 + wb) / nb}
    times = {}
    if len(sys.argv) > 4 and os.path.exists(sys.argv[3]):
        for r in csv.DictReader(open(sys.argv[3])):
            n = short(r["Name"])
            times[n] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                        "ms_per_batch": float(r["TotalDurationNs"]) / 1e6 / nb}
    total = sum(v["traffic_bytes_per_batch"] for v in kern.values())
    reads = sum(v["read_bytes_per_batch"] for v in kern.values())
    writes = sum(v["write_bytes_per_batch"] for v in kern.values())
    upper = sum(v["traffic_upper_bytes_per_batch"] for v in kern.values())
    decide = sum(v["traffic_bytes_per_batch"] for n, v in kern.items() if n.startswith(DECIDE))
    out = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE / --kernel-trace --stats passes of "
                     "`python3 bench.py --steps 2 --warmup 1 --sub-batches 2 --no-cpu-baseline` (tools/profile.sh)",
           "units": "bytes per global batch (sum over the batch's dispatches); FETCH_SIZE doubled for streaming "
                    "kernels per MI355X_MICROARCH.md, as counted for the random-access ones",
           "src_sha": bench.src_sha(), "git_head": sys.argv[5] if len(sys.argv) > 5 else None,
           "batch_events": 1 << 25, "batches_profiled": nb,
           "traffic_bytes_per_batch": total, "read_bytes_per_batch": reads, "write_bytes_per_batch": writes,
           "traffic_upper_bytes_per_batch": upper, "decide_traffic_bytes_per_batch": decide,
           "kernels": kern, "kernel_times": times}
    json.dump(out, open(sys.argv[4], "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("src_sha", "batches_profiled", "traffic_bytes_per_batch", "read_bytes_per_batch",
                                          "write_bytes_per_batch", "traffic_upper_bytes_per_batch",
                                          "decide_traffic_bytes_per_batch")}))


if __name__ == "__main__":
    main()
