#!/usr/bin/env python3
"""C2 time per align against the iteration count (k_icp_coop, one 640x480
pair per call, 400 calls x 5 windows per point): the slope is the cost of one
iteration, the intercept the prologue (fused prep, source staging, prep wait),
epilogue and launch.  Usage: python3 tools/c2_iters.py [W H]."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-rgbd_amd"))
import youth_icp  # noqa: E402
import youth_synth  # noqa: E402

W, H = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (640, 480)
src, dst, _ = youth_synth.pairs(0, 1, W, H)
ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
out = torch.zeros((1, 16), device="cuda")
s = torch.cuda.Stream()
pts = []
for iters in (1, 2, 5, 10, 20):
    ctx = youth_icp.IcpContext(W, H, 2, iters=iters)
    calls = 400

    def run(n):
        for _ in range(n):
            ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), 1, d_T_out=out.data_ptr(),
                                   stream=s.cuda_stream)

    run(40)
    torch.cuda.synchronize()
    us = []
    for _ in range(5):
        t0 = time.perf_counter()
        run(calls)
        torch.cuda.synchronize()
        us.append((time.perf_counter() - t0) / calls * 1e6)
    plan = ctx.get_plan() if hasattr(ctx, "get_plan") else ""
    ctx.close()
    pts.append((iters, float(np.median(us))))
    print(f"{W}x{H} iters {iters:2d}: {np.median(us):7.2f} us/align (min {min(us):7.2f}) {plan}",
          flush=True)
x = np.array([p[0] for p in pts], float)
y = np.array([p[1] for p in pts], float)
k, b = np.polyfit(x, y, 1)
print(f"fit: {k:.3f} us per iteration + {b:.2f} us fixed (prologue, epilogue, launch)")
