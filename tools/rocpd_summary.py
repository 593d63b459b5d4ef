"""Summarise a rocprofv3 SQLite output (rocpd) into a kernel-stats CSV like `--stats` writes
(durations in ns, from the per-dispatch kernel table):
    python tools/rocpd_summary.py <results.db> <out.csv>"""
import csv
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                  "from kernels group by name order by sum(duration) desc").fetchall()
total = sum(r[2] for r in rows)
with open(sys.argv[2], "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for r in rows:
        w.writerow([r[0], r[1], r[2], int(r[3]), f"{100.0 * r[2] / total:.2f}", r[4], r[5]])
for r in rows[:12]:
    print(f"{r[0][:70]:70s} {r[1]:5d} {r[3] / 1e3:10.1f} us {100.0 * r[2] / total:6.2f}%")
