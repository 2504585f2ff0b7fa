#!/usr/bin/env python3
"""Per-launch HBM traffic of k_reduce from rocprofv3 PMC passes -> JSON.

traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 bytes, averaged over the
k_reduce dispatches.  The factor 2 on FETCH_SIZE is MI355X_MICROARCH.md §HBM's
gfx950 correction, re-calibrated here: tools/kbench's k_stream_read of a known
550.5 MB reports FETCH_SIZE = 275.3 MB for both dwordx4 and dword loads
(profiles/r01/pmc_calibration.txt).

usage: tools/pmc_traffic.py <profile_root> <out.json> <pairs> <width> <height> [iters]
(iters: ICP iterations each k_icp launch covers; 1 for per-iteration k_reduce)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import summarize  # noqa: E402


def main():
    root, out, pairs, W, H = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), \
        int(sys.argv[5])
    iters = int(sys.argv[6]) if len(sys.argv) > 6 else 1
    res = summarize(root)
    key = next(k for k in res if k.startswith("k_icp") or k.startswith("k_reduce"))
    r = res[key]
    fetch = r["FETCH_SIZE"] * 1024.0
    write = r.get("WRITE_SIZE", 0.0) * 1024.0
    px = pairs * W * H
    doc = {
        "kernel": key, "pairs": pairs, "width": W, "height": H,
        "fetch_size_bytes": fetch, "write_size_bytes": write,
        "iterations_per_launch": iters,
        "hbm_bytes_per_launch": 2.0 * fetch + write,
        "hbm_bytes_per_iteration": (2.0 * fetch + write) / iters,
        "bytes_per_px": (2.0 * fetch + write) / iters / px,
        "correction": "2 x FETCH_SIZE (gfx950 tallies 128-B requests as 64 B)",
    }
    for k in ("k_prep", "k_solve"):
        m = next((x for x in res if x.startswith(k)), None)
        if m and "FETCH_SIZE" in res[m]:
            doc[k + "_hbm_bytes"] = 2.0 * res[m]["FETCH_SIZE"] * 1024 + \
                res[m].get("WRITE_SIZE", 0.0) * 1024
    json.dump(doc, open(out, "w"), indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
