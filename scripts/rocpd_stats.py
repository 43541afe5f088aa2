"""Kernel statistics (name, calls, average / total duration) from a rocprofv3 SQLite result
(run_results.db, the default output format of rocprofv3 on ROCm 7), as the CSV the
--stats summary used to be: usage python scripts/rocpd_stats.py <results.db> [out.csv]"""
import csv
import sqlite3
import sys

db = sys.argv[1]
c = sqlite3.connect(db)
rows = c.execute("select name, count(*), avg(duration), sum(duration), min(duration), max(duration) from kernels "
                 "group by name order by sum(duration) desc").fetchall()
total = sum(r[3] for r in rows) or 1
out = [("Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs")]
for name, n, avg, tot, mn, mx in rows:
    out.append((name, n, tot, round(avg, 1), round(100.0 * tot / total, 2), mn, mx))
if len(sys.argv) > 2:
    with open(sys.argv[2], "w", newline="") as f:
        csv.writer(f).writerows(out)
for r in out[1:]:
    print(f"{r[0][:78]:80s} {r[1]:6d} {r[3] / 1e3:9.2f} us {r[4]:6.2f}%")
