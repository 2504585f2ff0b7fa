#!/usr/bin/env python3
"""C3 batch (16 pairs 1280x960, 20 iterations, persistent k_icp) for the
chunk target in YOUTH_ICP_TARGET_CHUNKS (read at context creation).
usage: YOUTH_ICP_TARGET_CHUNKS=<n> python3 tools/c3_sweep.py"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-rgbd_amd"))
import youth_icp  # noqa: E402
import youth_synth  # noqa: E402

n, W, H = 16, 1280, 960
src, dst, _ = youth_synth.pairs(0, n, W, H)
ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
out = torch.zeros((n, 16), dtype=torch.float32, device="cuda")
stream = torch.cuda.current_stream().cuda_stream
rates = []
with youth_icp.IcpContext(W, H, n, iters=20) as ctx:
    for rep in range(4):
        for _ in range(3):
            ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n, d_T_out=out.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n, d_T_out=out.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        rates.append(n * 20 / (time.perf_counter() - t0))
    plan = ctx.get_plan()
rates.sort()
print(f"chunks {os.environ.get('YOUTH_ICP_TARGET_CHUNKS', 'default'):>7s}: C3 batch "
      f"{rates[len(rates) // 2]:7.0f} aligns/s (min {rates[0]:.0f} max {rates[-1]:.0f})  {plan.get('kernel')}",
      flush=True)
