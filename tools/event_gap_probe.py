#!/usr/bin/env python3
"""Why do consecutive tracker aligns leave ~16 us gaps (profiles/r02/prof_trk)?
One 640x480 pair per call, 400 calls back to back on one torch stream, with
per call: (a) nothing else; (b) an event recorded after the align (default
flags: system-scope fence); (c) the stream waiting on an event recorded on a
second stream before the align; (d) both.  us per call, median of 5 windows."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-rgbd_amd"))
import youth_icp  # noqa: E402
import youth_synth  # noqa: E402


def main():
    src, dst, _ = youth_synth.pairs(0, 1, 640, 480)
    ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
    out = torch.zeros((1, 16), device="cuda")
    s = torch.cuda.Stream()
    x = torch.cuda.Stream()
    ctx = youth_icp.IcpContext(640, 480, 2)
    ev_after = [torch.cuda.Event() for _ in range(4)]
    ev_x = torch.cuda.Event()
    with torch.cuda.stream(x):
        ev_x.record(x)

    def run(mode, calls=400):
        with torch.cuda.stream(s):
            for k in range(calls):
                if mode in ("wait", "both"):
                    s.wait_event(ev_x)
                ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), 1, d_T_out=out.data_ptr(),
                                       stream=s.cuda_stream)
                if mode in ("event", "both"):
                    ev_after[k & 3].record(s)
        s.synchronize()

    for mode in ("plain", "event", "wait", "both"):
        run(mode, 40)
        r = []
        for _ in range(5):
            t0 = time.perf_counter()
            run(mode)
            r.append((time.perf_counter() - t0) / 400 * 1e6)
        print(f"{mode:>6s}: {np.median(r):6.1f} us per align", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
