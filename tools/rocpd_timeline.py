"""Last batch's kernel timeline from a rocprofv3 rocpd sqlite file: every kernel longer than a threshold (us, default
30) from the batch's k_rs_first on, with its queue, start / end relative to it.
usage: python tools/rocpd_timeline.py results.db [min_us] [batch index from the end, default 1]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cur = db.cursor()
cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = cur.execute("select start, end, %s, queue_id from kernels order by start" % name).fetchall()
min_ns = float(sys.argv[2]) * 1000 if len(sys.argv) > 2 else 30000
back = int(sys.argv[3]) if len(sys.argv) > 3 else 1
firsts = [i for i, r in enumerate(rows) if r[2].replace("void ", "").startswith("k_rs_first")]
i0 = firsts[-back]
i1 = firsts[-back + 1] if back > 1 else len(rows)
t0 = rows[i0][0]
for s, e, n, q in rows[i0:i1]:
    if e - s >= min_ns:
        print("%-44s q%-3s start %9.1f end %9.1f dur %8.1f" % (n.split("(")[0].replace("void ", "")[:44], q,
                                                            (s - t0) / 1e3, (e - t0) / 1e3, (e - s) / 1e3))
