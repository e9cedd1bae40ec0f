#!/usr/bin/env python3
"""HBM traffic per launch of the fused RK4 kernel from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE in separate passes: TCC slots do not fit both, MI355X_MICROARCH.md
§rocprofv3 PMC slots).  Corrections per the guide's HBM section: FETCH_SIZE reads exactly half
of the bytes of a wide coalesced stream on gfx950 -> x2; both counters are in KiB -> x1024.
WRITE_SIZE is exact for 16-B/lane stores; our trajectory stores are 4-B/lane rows of 256 B per
wave (uncalibrated width -- reported as measured)."""
import csv
import glob
import json
import sys
from collections import defaultdict


def per_launch(d, name, kernel="k_acro"):
    vals = defaultdict(float)
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == name:
                vals[row["Dispatch_Id"]] += float(row["Counter_Value"])
    return sum(vals.values()) / max(len(vals), 1), len(vals)


def main(fetch_dir, write_dir, out):
    f, nf = per_launch(fetch_dir, "FETCH_SIZE")
    w, nw = per_launch(write_dir, "WRITE_SIZE")
    res = {"fetch_bytes_per_launch": f * 1024 * 2, "write_bytes_per_launch": w * 1024,
           "hbm_bytes_per_launch": f * 1024 * 2 + w * 1024, "dispatches": [nf, nw],
           "method": "rocprofv3 --pmc FETCH_SIZE (x2 gfx950 half-count correction, KiB->B) and --pmc WRITE_SIZE "
                     "(KiB->B) in separate passes over scripts/kprof.py (bench C3 workload)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:4])
