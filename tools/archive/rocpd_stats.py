"""Dev tool: kernel statistics (rocprofv3 --stats style CSV) from a rocprofv3 rocpd SQLite
database.  usage: python tools/rocpd_stats.py RESULTS.db OUT.csv"""
import csv
import sqlite3
import sys

db, out = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "name" if "name" in cols else "kernel_name"
# one row per (kernel, grid size): the bench's header read inflates a few blocks with the same
# kernel, which would otherwise pull the average of the full-file launches down
rows = c.execute(f"select {name} || ' [grid ' || grid_x || ']', count(*), sum(end - start), "
                 f"avg(end - start), min(end - start), max(end - start) from kernels "
                 f"group by {name}, grid_x order by sum(end - start) desc").fetchall()
tot = sum(r[2] for r in rows) or 1
with open(out, "w", newline="") as f:
    w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for n, k, s, a, mn, mx in rows:
        w.writerow([n, k, s, round(a, 1), round(100.0 * s / tot, 4), mn, mx])
for n, k, s, a, *_ in rows[:8]:
    print(f"{k:4d} {a / 1e6:10.3f} ms  {100.0 * s / tot:6.2f}%  {n[:90]}")
