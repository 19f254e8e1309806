"""Per-kernel stats (calls, total / average ns) from a rocprofv3 rocpd database (ROCm 7 writes
SQLite by default), in the --stats CSV layout.  usage: python tools/rocpd_stats.py DB [OUT.csv]"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
                     f"from kernels group by {name} order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [(n, k, s, a, 100.0 * s / tot, mn, mx) for n, k, s, a, mn, mx in rows]


if __name__ == "__main__":
    out = stats(sys.argv[1])
    w = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
    for r in out:
        w.writerow(r)
