#!/usr/bin/env python3
"""Kernel durations and the idle gaps between consecutive dispatches from a
rocprofv3 kernel trace (one stream): where a latency-bound align spends its
wall time.  usage: tools/kt_gaps.py <kernel_trace.csv> [skip_first_n_dispatches]
"""
import collections
import csv
import sys

from kt_summary import short


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[skip:]
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    for i, r in enumerate(rows):
        k = short(r["Kernel_Name"])
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        dur[k].append((e - s) / 1e3)
        if i:
            gap[k].append((s - int(rows[i - 1]["End_Timestamp"])) / 1e3)
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3
    print(f"{len(rows)} dispatches over {span:.1f} us")
    print(f"{'kernel':24s} {'n':>6s} {'avg_us':>9s} {'gap_before_us':>14s}")
    for k in dur:
        g = gap.get(k, [0.0])
        print(f"{k:24s} {len(dur[k]):6d} {sum(dur[k]) / len(dur[k]):9.2f} "
              f"{sum(g) / max(len(g), 1):14.2f}")


if __name__ == "__main__":
    main()
