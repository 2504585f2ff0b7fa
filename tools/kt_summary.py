#!/usr/bin/env python3
"""Per-kernel durations from a rocprofv3 kernel trace, skipping warm-up calls.

bench.py times its K steps after W warm-up steps; the rocprofv3 stats CSV
averages every dispatch including the warm-ups (first-touch, clock ramp), so
this prints the steady-state average the bench's HIP events should match.

usage: tools/kt_summary.py <kernel_trace.csv> [skip_first_n_per_kernel]
"""
import collections
import csv
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    return re.sub(r"\(.*", "", name).strip()


def main():
    path = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[short(r["Kernel_Name"])].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(f"{'kernel':28s} {'calls':>6s} {'used':>5s} {'avg_us':>10s} {'min_us':>10s} "
          f"{'max_us':>10s}   (first {skip} calls per kernel skipped)")
    for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
        u = v[skip:] if len(v) > skip else v
        print(f"{k:28s} {len(v):6d} {len(u):5d} {sum(u) / len(u):10.1f} {min(u):10.1f} "
              f"{max(u):10.1f}")


if __name__ == "__main__":
    main()
