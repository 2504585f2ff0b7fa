#!/usr/bin/env python3
"""Tracker micro-batch probe (run alone or under rocprofv3 --kernel-trace):
the same host sequence through (a) the default plan, one launch per frame;
(b) the batch plan (youth_icp_track_set_batch(2)) one launch per frame;
(c) the batch plan in micro-batches of m = 2 .. TRACK_MAX_BATCH frames
through the library's C loop.  Prints frames/s of each."""
import os
import sys
import time

import torch  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "slam-rgbd_amd")]
import numpy as np  # noqa: E402

import youth_icp  # noqa: E402
import youth_synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
frames, _ = youth_synth.sequence(0, n)


def run(ctx, batch_submit):
    ctx.track_reset()
    t0 = time.perf_counter()
    if batch_submit:
        Tb, _ = ctx.track_host_sequence(frames)
    else:
        out = []
        for f in frames:
            ctx.track_submit(f)
            if ctx.track_pending() == 2:
                out.append(ctx.track_collect())
        while ctx.track_pending():
            out.append(ctx.track_collect())
    return n / (time.perf_counter() - t0)


a = youth_icp.IcpContext(640, 480, 4)
run(a, False)
print("default plan, per frame:", round(run(a, False)), a.get_plan(), flush=True)
print("default plan, per frame (C loop):", [round(run(a, True)) for _ in range(3)], flush=True)
for m in range(2, youth_icp.TRACK_MAX_BATCH + 1):
    b = youth_icp.IcpContext(640, 480, 2 * m)
    b.track_set_batch(m)
    run(b, False)
    print(f"batch plan {m}, per frame:", round(run(b, False)), b.get_plan(), flush=True)
    run(b, True)
    print(f"batch plan {m}, micro-batches (C loop):", [round(run(b, True)) for _ in range(3)],
          "chained", b.track_chained(), flush=True)
    b.close()
