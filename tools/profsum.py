"""Summarise a rocprofv3 results database: per-kernel calls, mean/total duration (us)."""
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), avg(duration)/1000.0, sum(duration)/1000.0, max(vgpr_count), "
                 "max(scratch_size), max(lds_size) from kernels group by name order by sum(duration) desc").fetchall()
print("%-44s %6s %12s %12s %5s %7s %6s" % ("kernel", "calls", "mean_us", "total_us", "vgpr", "scratch", "lds"))
for n, k, a, t, v, s, l in rows:
    print("%-44s %6d %12.1f %12.1f %5d %7d %6d" % (n.split("(")[0][:44], k, a, t, v, s, l))
