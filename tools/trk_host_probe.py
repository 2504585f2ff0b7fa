#!/usr/bin/env python3
"""Where a streamed tracker frame's host time goes: submit (staging memcpy +
stream ops + launch) vs collect (wait), two frames in flight, 300 640x480
frames; plus a plain host memcpy of one depth frame for scale."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-rgbd_amd"))
import youth_icp  # noqa: E402
import youth_synth  # noqa: E402

frames, _ = youth_synth.sequence(0, 300, 640, 480)
ctx = youth_icp.IcpContext(640, 480, 2)
ctx.track_frame(frames[0])
ctx.track_frame(frames[1])
for rep in range(3):
    ctx.track_reset()
    ts = tc = 0.0
    t0 = time.perf_counter()
    for f in frames:
        a = time.perf_counter()
        ctx.track_submit(f)
        b = time.perf_counter()
        ts += b - a
        if ctx.track_pending() == 2:
            ctx.track_collect()
            tc += time.perf_counter() - b
    while ctx.track_pending():
        ctx.track_collect()
    tot = time.perf_counter() - t0
    n = len(frames)
    print(f"pass {rep}: {n / tot:8.0f} frames/s  per frame {tot / n * 1e6:6.1f} us: "
          f"submit {ts / n * 1e6:6.1f} us, collect {tc / n * 1e6:6.1f} us", flush=True)
dst = np.empty_like(frames[0])
a = time.perf_counter()
for f in frames:
    np.copyto(dst, f)
print(f"host memcpy of one frame: {(time.perf_counter() - a) / len(frames) * 1e6:.1f} us", flush=True)
ctx.close()
