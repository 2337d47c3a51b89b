"""Kernel stats (name, calls, total/avg/min/max ns) from a rocprofv3 rocpd sqlite file (the default output of
rocprofv3 on this image); same columns as rocprofv3's kernel_stats.csv."""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
cur = db.cursor()
cols = [r[1] for r in cur.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else "name"
rows = cur.execute("select %s, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) from kernels "
                   "group by %s order by sum(end-start) desc" % (name, name)).fetchall()
tot = sum(r[2] for r in rows)
out = open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout
out.write('"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"\n')
for n, c, s, a, lo, hi in rows:
    out.write('"%s",%d,%d,%.1f,%.2f,%d,%d\n' % (n.split("(")[0], c, s, a, 100.0 * s / tot, lo, hi))
