"""Per-batch kernel timeline from a rocprofv3 --kernel-trace CSV (tools/timeline.sh): for every decide
stage (k_resolve .. k_post) the start/end of each kernel relative to the batch's k_rs_first, so the
critical path of a batch is visible.  usage: python tools/timeline.py kernel_trace.csv [n_batches]
With --window: every kernel longer than 15 us (with its hardware queue) between the k_rs_first of the
third-last and of the last batch of a pipelined trace, i.e. two overlapped batch periods."""
import csv
import sys


def window(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")[:28],
                 r.get("Queue_Id", "?")) for r in rows)
    firsts = [i for i, k in enumerate(ks) if k[2].startswith("k_rs_first")]
    t0, t1 = ks[firsts[-3]][0], ks[firsts[-1]][0]
    print("two batch periods: %.1f us" % ((t1 - t0) / 1e3))
    for s, e, n, q in ks:
        if t0 <= s < t1 and e - s > 15000:
            print("q%-3s %-28s start %8.1f  end %8.1f  dur %7.1f us" % (q, n, (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))


def main():
    if "--window" in sys.argv:
        return window([a for a in sys.argv[1:] if a != "--window"][0])
    rows = list(csv.DictReader(open(sys.argv[1])))
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows))
    firsts = [i for i, k in enumerate(ks) if k[2].startswith("void k_rs_first") or k[2].startswith("k_rs_first")]
    for bi, i0 in enumerate(firsts[-nb:]):
        t0 = ks[i0][0]
        i1 = firsts[firsts.index(i0) + 1] if firsts.index(i0) + 1 < len(firsts) else len(ks)
        # kernels of this batch: from its rs_first up to (and including) its k_post
        seen_post = False
        print("batch %d" % bi)
        for s, e, n in ks[i0:]:
            if seen_post and n.startswith("k_rs_first"):
                break
            short = n.split("(")[0].replace("void ", "")[:40]
            print("  %-40s start %8.1f us  end %8.1f us  dur %8.1f us" % (short, (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
            if short.startswith("k_post"):
                seen_post = True
                break


if __name__ == "__main__":
    main()
