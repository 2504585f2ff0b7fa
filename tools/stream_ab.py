#!/usr/bin/env python3
"""Streamed-tracker A/B: 300 640x480 frames from host memory through
youth_icp_track_submit/_collect (two in flight) and through track_frame, for
the libyouth_icp.so named by YOUTH_ICP_LIB.  Median of 5 passes.
Usage: YOUTH_ICP_LIB=tools/ab/<name>/libyouth_icp.so python3 tools/stream_ab.py <label>"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-rgbd_amd"))
import youth_icp  # noqa: E402
import youth_synth  # noqa: E402


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else "cur"
    frames, _ = youth_synth.sequence(0, 300, 640, 480)
    ctx = youth_icp.IcpContext(640, 480, 2)
    ctx.track_frame(frames[0])
    ctx.track_frame(frames[1])
    piped, sync = [], []
    for _ in range(5):
        ctx.track_reset()
        t0 = time.perf_counter()
        for f in frames:
            ctx.track_submit(f)
            if ctx.track_pending() == int(os.environ.get("DEPTH", "2")):
                ctx.track_collect()
        while ctx.track_pending():
            ctx.track_collect()
        piped.append(len(frames) / (time.perf_counter() - t0))
        ctx.track_reset()
        t0 = time.perf_counter()
        for f in frames:
            ctx.track_frame(f)
        sync.append(len(frames) / (time.perf_counter() - t0))
    ctx.close()
    print(f"{label:>8s} streamed pipelined: median {np.median(piped):8.0f} frames/s "
          f"(min {min(piped):.0f} max {max(piped):.0f})  one at a time: median {np.median(sync):8.0f}",
          flush=True)


if __name__ == "__main__":
    main()
