#!/usr/bin/env python3
"""C2 align rate (one pair per call, k_icp_coop) on the library's private
stream vs torch-created streams, alone and after a 64-pair align context has
run on the same stream: finds what slows the bench's single-pair leg."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-rgbd_amd"))
import youth_icp  # noqa: E402
import youth_synth  # noqa: E402

bench_stream = torch.cuda.Stream()
src, dst, _ = youth_synth.pairs(0, 64)
ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
out = torch.zeros((64, 16), device="cuda")
ctx1 = youth_icp.IcpContext(640, 480, 2)


def rate(ctx, stream, npairs=1, n=300):
    for _ in range(30):
        ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), npairs, d_T_out=out.data_ptr(),
                               stream=stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), npairs, d_T_out=out.data_ptr(),
                               stream=stream)
    torch.cuda.synchronize()
    return npairs * n / (time.perf_counter() - t0)


print(f"fresh: library {rate(ctx1, 0):7.0f}  bench stream {rate(ctx1, bench_stream.cuda_stream):7.0f}",
      flush=True)
ctx64 = youth_icp.IcpContext(640, 480, 64)
print(f"64-pair ctx on bench stream: {rate(ctx64, bench_stream.cuda_stream, 64, 30):7.0f}", flush=True)
print(f"after: library {rate(ctx1, 0):7.0f}  bench stream {rate(ctx1, bench_stream.cuda_stream):7.0f}",
      flush=True)
ctx64.set_timing(True)
rate(ctx64, bench_stream.cuda_stream, 64, 10)
ctx64.set_timing(False)
print(f"after timing on/off: library {rate(ctx1, 0):7.0f}  bench stream "
      f"{rate(ctx1, bench_stream.cuda_stream):7.0f}", flush=True)
ctx64.close()
print(f"after close: library {rate(ctx1, 0):7.0f}  bench stream "
      f"{rate(ctx1, bench_stream.cuda_stream):7.0f}", flush=True)
ctx2 = youth_icp.IcpContext(640, 480, 2)
print(f"new ctx: library {rate(ctx2, 0):7.0f}  bench stream {rate(ctx2, bench_stream.cuda_stream):7.0f}",
      flush=True)
