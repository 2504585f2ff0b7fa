#!/usr/bin/env python3
"""One point of the C3 batch chunk sweep: 16 pairs @1280x960, 20 iterations,
through the persistent k_icp with YOUTH_ICP_TARGET_CHUNKS (read once per
process) as set in the environment.  Prints the per-call time and k_icp's
HIP-event time.  Run by tools/c3_chunks.sh."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "slam-rgbd_amd")]
import youth_icp  # noqa: E402
import youth_synth  # noqa: E402

n, W, H, iters = 16, 1280, 960, 20
src, dst, _ = youth_synth.pairs(0, n, W, H)
ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
out = torch.zeros((n, 16), dtype=torch.float32, device="cuda")
ctx = youth_icp.IcpContext(W, H, n, iters=iters)
for _ in range(5):
    ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n, d_T_out=out.data_ptr())
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n, d_T_out=out.data_ptr())
torch.cuda.synchronize()
us = (time.perf_counter() - t0) / 20 * 1e6
ctx.set_timing(True, iteration_kernel_only=True)
for _ in range(20):
    ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n, d_T_out=out.data_ptr())
torch.cuda.synchronize()
ms, nl = ctx.get_timing(0)
print(f"chunks {os.environ.get('YOUTH_ICP_TARGET_CHUNKS', 'default')}: {us:8.1f} us per call "
      f"({n / us * 1e6:7.0f} aligns/s), k_icp {ms / max(nl, 1) * 1e3:8.1f} us, "
      f"plan {ctx.get_plan()['kernel']}, sched {ctx.get_sched_stats()}", flush=True)
