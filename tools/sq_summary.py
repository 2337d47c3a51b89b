"""Per-kernel SQ counter summary from a rocprofv3 --pmc counter_collection.csv: per kernel the dispatch
count and, per wave, the instruction mix and cycle split (SQ_WAVE_CYCLES etc. count quad-cycles,
MI355X_MICROARCH.md).  usage: python tools/sq_summary.py counter_collection.csv"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    names = sorted({c for v in agg.values() for c in v})
    print("%-34s %6s %10s " % ("kernel", "disp", "waves") + " ".join("%14s" % n.replace("SQ_", "")[:14] for n in names if n != "SQ_WAVES"))
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        w = v.get("SQ_WAVES", 0) or 1
        print("%-34s %6d %10.0f " % (k[:34], len(disp[k]), v.get("SQ_WAVES", 0)) +
              " ".join("%14.1f" % (v[n] / w) for n in names if n != "SQ_WAVES"))


if __name__ == "__main__":
    main()
