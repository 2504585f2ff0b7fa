#!/usr/bin/env python3
"""Dispatches of one kernel from a rocprofv3 kernel trace, grouped by grid
size: count, median duration and median idle gap before each dispatch (from
the previous dispatch's end on the same queue).  Used for the tracker's
per-frame vs micro-batch launches.
usage: tools/kt_grids.py <kernel_trace.csv> [kernel_substring]"""
import collections
import csv
import statistics
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    key = sys.argv[2] if len(sys.argv) > 2 else "k_icp_coop"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    gcol = next(c for c in rows[0] if c.lower().startswith("grid_size"))
    wcol = next(c for c in rows[0] if c.lower().startswith("workgroup_size"))
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    prev_end = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if key in r["Kernel_Name"]:
            wgs = int(r[gcol]) // max(int(r[wcol]), 1)
            dur[wgs].append((e - s) / 1e3)
            if prev_end is not None:
                gap[wgs].append((s - prev_end) / 1e3)
        prev_end = e
    print(f"{'workgroups':>10s} {'n':>6s} {'median_us':>10s} {'gap_before_us':>14s}")
    for w in sorted(dur):
        g = gap.get(w) or [0.0]
        print(f"{w:10d} {len(dur[w]):6d} {statistics.median(dur[w]):10.1f} "
              f"{statistics.median(g):14.1f}")


if __name__ == "__main__":
    main()
