#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace results.db (rocpd SQLite) like --stats' kernel_stats.csv:
name, calls, total/avg/min/max ns, percent.  Usage: kstats_db.py results.db [out.csv] [--skip N]

--skip N drops each kernel's first N dispatches (kprof.py --warmup N: the evaluations before the
measured ones, while the GPU clocks ramp up -- the bench's timed region likewise follows warmup
steps); the raw database keeps every dispatch."""
import csv
import sqlite3
import sys


def stats(db, skip=0):
    c = sqlite3.connect(db)
    per = {}
    for name, dur in c.execute("select name, end - start from kernels order by start"):
        per.setdefault(name, []).append(dur)
    rows = []
    for name, d in per.items():
        d = d[skip:]
        if d:
            rows.append((name, len(d), sum(d), sum(d) / len(d), min(d), max(d)))
    rows.sort(key=lambda r: -r[2])
    tot = sum(r[2] for r in rows) or 1
    return [(n, k, s, a, lo, hi, 100.0 * s / tot) for n, k, s, a, lo, hi in rows]


if __name__ == "__main__":
    args = sys.argv[1:]
    skip = 0
    if "--skip" in args:
        i = args.index("--skip")
        skip = int(args[i + 1])
        del args[i:i + 2]
    rows = stats(args[0], skip)
    out = open(args[1], "w", newline="") if len(args) > 1 else sys.stdout
    w = csv.writer(out)
    w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs", "Percentage"])
    for r in rows:
        w.writerow([r[0], r[1], r[2], f"{r[3]:.1f}", r[4], r[5], f"{r[6]:.2f}"])
