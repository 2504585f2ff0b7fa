#!/usr/bin/env python3
"""Average rocprofv3 PMC counters per kernel over every pass directory under a
profile root (each pass: <root>/<pass>/*counter_collection.csv)."""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*", "", name)
    return name.strip()


def summarize(root):
    out = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            agg[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in agg.items():
            out[k][c] = sum(v) / len(v)
            out[k]["_dispatches"] = len(v)
    return out


if __name__ == "__main__":
    res = summarize(sys.argv[1])
    keep = sys.argv[2] if len(sys.argv) > 2 else ""
    for k in sorted(res):
        if keep and keep not in k:
            continue
        print(k)
        for c, v in sorted(res[k].items()):
            print(f"    {c:40s} {v:14.6g}")
    if len(sys.argv) > 3:
        json.dump(res, open(sys.argv[3], "w"), indent=1)
