#!/usr/bin/env python3
"""A/B of the tracker's staging copy (host_copy.h): a 300-frame host sequence
through youth_icp_track_host_sequence in micro-batches of m frames, with the
copy into page-locked staging done by the submitting thread alone
(YOUTH_ICP_COPY_THREADS=0) or split over it and k helper threads.  The knob is
read at context creation, so one process runs every setting, interleaved.
Prints frames/s (median of the passes) per setting and checks that every
setting's poses are bit-identical.  argv: rounds (default 3)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "slam-rgbd_amd")]
import youth_icp  # noqa: E402
import youth_synth  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
frames, _ = youth_synth.sequence(0, 300)
ref = None
for r in range(rounds):
    for m in (4, 8):
        for k in (0, 1, 3, 7):
            os.environ["YOUTH_ICP_COPY_THREADS"] = str(k)
            ctx = youth_icp.IcpContext(640, 480, 2 * m)
            ctx.track_set_batch(m)
            ctx.track_host_sequence(frames[: 2 * m + 1])  # warm (starts the pool)
            rates = []
            for _ in range(5):
                ctx.track_reset()
                t0 = time.perf_counter()
                T, _ = ctx.track_host_sequence(frames)
                rates.append(len(frames) / (time.perf_counter() - t0))
            ctx.close()
            same = True
            if m == 8:
                if ref is None:
                    ref = T
                same = bool(np.array_equal(T, ref))
            print(f"round {r} batch {m} helpers {k}: {np.median(rates):9.0f} frames/s "
                  f"(passes {[round(x) for x in rates]}) poses equal: {same}", flush=True)
