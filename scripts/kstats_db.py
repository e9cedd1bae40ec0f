#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace results.db (rocpd SQLite) like --stats' kernel_stats.csv:
name, calls, total/avg/min/max ns, percent.  Usage: kstats_db.py results.db [out.csv]"""
import csv
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, count(*), sum(end - start), avg(end - start), min(end - start), max(end - start) "
                     "from kernels group by name order by sum(end - start) desc").fetchall()
    tot = sum(r[2] for r in rows) or 1
    return [(n, k, s, a, lo, hi, 100.0 * s / tot) for n, k, s, a, lo, hi in rows]


if __name__ == "__main__":
    rows = stats(sys.argv[1])
    out = open(sys.argv[2], "w", newline="") if len(sys.argv) > 2 else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    for r in rows:
        w.writerow([r[0], r[1], r[2], f"{r[3]:.1f}", r[4], r[5], f"{r[6]:.2f}"])
