#!/usr/bin/env python3
"""C2 align rate (one 640x480 pair per call, k_icp_coop) by launch form and
stream, and after each thing bench.py does before its single-pair leg: finds
what made cooperative launches on the bench's torch stream run at half rate
(VERDICT r01 weak item 4).

Each line: aligns/s on the library's private stream | on a torch-created
stream, for a context whose coop kernel is launched with
hipLaunchCooperativeKernel ("coop") or hipLaunchKernel ("plain",
YOUTH_ICP_COOP_LAUNCH=plain)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-rgbd_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import youth_icp  # noqa: E402
import youth_synth  # noqa: E402

bench_stream = torch.cuda.Stream()
src, dst, _ = youth_synth.pairs(0, 64)
ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
out = torch.zeros((64, 16), device="cuda")
ctx = {}
for k in ("runtime", "plain", "serial"):
    os.environ["YOUTH_ICP_COOP_LAUNCH"] = k
    ctx[k] = youth_icp.IcpContext(640, 480, 2)
os.environ.pop("YOUTH_ICP_COOP_LAUNCH", None)


def rate(c, stream, npairs=1, n=400):
    for _ in range(40):
        c.align_pairs_device(ds.data_ptr(), dd.data_ptr(), npairs, d_T_out=out.data_ptr(),
                             stream=stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        c.align_pairs_device(ds.data_ptr(), dd.data_ptr(), npairs, d_T_out=out.data_ptr(),
                             stream=stream)
    torch.cuda.synchronize()
    return npairs * n / (time.perf_counter() - t0)


def line(tag):
    parts = []
    for k in ("runtime", "plain", "serial"):
        parts.append(f"{k}: lib {rate(ctx[k], 0):7.0f} torch {rate(ctx[k], bench_stream.cuda_stream):7.0f}")
    print(f"{tag:34s} " + " | ".join(parts), flush=True)


def alternating(c, n=400):
    """serial ordering across two streams: every launch waits on the other's"""
    streams = [0, bench_stream.cuda_stream]
    for i in range(n):
        c.align_pairs_device(ds.data_ptr(), dd.data_ptr(), 1, d_T_out=out.data_ptr(),
                             stream=streams[i & 1])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        c.align_pairs_device(ds.data_ptr(), dd.data_ptr(), 1, d_T_out=out.data_ptr(),
                             stream=streams[i & 1])
    torch.cuda.synchronize()
    return n / (time.perf_counter() - t0)


line("fresh")
print(f"alternating lib/torch streams: serial {alternating(ctx['serial']):7.0f} "
      f"runtime {alternating(ctx['runtime']):7.0f}", flush=True)
line("again")
with torch.cuda.stream(bench_stream):
    line("inside torch.cuda.stream(...)")
ctx64 = youth_icp.IcpContext(640, 480, 64)
rate(ctx64, bench_stream.cuda_stream, 64, 30)
line("after a 64-pair ctx on torch stream")
ctx64.set_timing(True, iteration_kernel_only=True)
rate(ctx64, bench_stream.cuda_stream, 64, 10)
ctx64.set_timing(False)
line("after timing on/off")
youth_icp.align_batch(src[:32], dst[:32])
line("after align_batch (xfer stream)")
import oracle  # noqa: E402
oracle.align_batch(src[:16], dst[:16], iters=10, n_threads=16)
line("after 16-thread OpenMP oracle")
time.sleep(1.0)
line("1 s later")
ctx64.close()
