#!/usr/bin/env python3
"""Overlap of the tracker's frame copies (SDMA copies from the memory-copy
trace, or k_pull_frames dispatches) with k_icp_coop in a rocprofv3 trace
directory: per copy path, the mean copy duration and the fraction of copy
time during which a k_icp_coop ran."""
import csv
import glob
import sys


def rows(pat):
    f = glob.glob(pat, recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


d = sys.argv[1]
ks = rows(f"{d}/**/*kernel_trace.csv")
coop = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks
              if "k_icp_coop" in r["Kernel_Name"])
pull = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in ks if "k_pull_frames" in r["Kernel_Name"]]
cp = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows(f"{d}/**/*memory_copy_trace.csv")
      if "HOST_TO_DEVICE" in r.get("Direction", "") and int(r.get("Size", 0) or 0) >= 600000]


def overlap(a, b):
    return max(0, min(a[1], b[1]) - max(a[0], b[0]))


for name, xs in (("k_pull_frames", pull), ("SDMA H2D", cp)):
    if not xs:
        continue
    tot = sum(e - s for s, e in xs)
    ov = sum(sum(overlap(x, c) for c in coop) for x in xs)
    print(f"{name}: {len(xs)} copies, mean {tot / len(xs) / 1e3:.1f} us, {ov / max(tot, 1):.2f} of copy time "
          f"beside a k_icp_coop; k_icp_coop mean {sum(e - s for s, e in coop) / max(len(coop), 1) / 1e3:.1f} us")
