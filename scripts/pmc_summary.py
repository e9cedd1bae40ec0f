#!/usr/bin/env python3
"""Per-launch PMC totals from rocprofv3 output (sqlite .db or counter_collection.csv).

usage: pmc_summary.py <dir> [kernel-substring] -> JSON {counter: mean over dispatches of the
sum over all instances (XCD/SE/...) of that dispatch}, plus the mean kernel duration (ns)."""
import csv
import glob
import json
import sqlite3
import sys
from collections import defaultdict


def collect(d, kernel="k_acro"):
    per = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> sum
    dur = {}
    for db in glob.glob(f"{d}/**/*.db", recursive=True):
        c = sqlite3.connect(db)
        q = "select dispatch_id, kernel_name, counter_name, value, duration from counters_collection"
        for disp, name, ctr, val, du in c.execute(q):
            if kernel in name:
                per[ctr][(db, disp)] += float(val)
                dur[(db, disp)] = du
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if kernel in row["Kernel_Name"]:
                per[row["Counter_Name"]][(f, row["Dispatch_Id"])] += float(row["Counter_Value"])
    out = {k: sum(v.values()) / len(v) for k, v in per.items()}
    out["dispatches"] = max((len(v) for v in per.values()), default=0)
    if dur:
        out["duration_ns"] = sum(dur.values()) / len(dur)
    return out


if __name__ == "__main__":
    print(json.dumps(collect(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "k_acro"), indent=1))
