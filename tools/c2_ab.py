#!/usr/bin/env python3
"""C2 rate A/B: one 640x480 pair per call (k_icp_coop) on a torch stream,
400 calls x 5 windows, for the libyouth_icp.so named by YOUTH_ICP_LIB (or the
in-tree build); also 1280x960 / 20 iterations (C3 single pair) and the pose
error vs the C oracle.  Usage: YOUTH_ICP_LIB=tools/ab/<name>/libyouth_icp.so
python3 tools/c2_ab.py <label>   (run several labels in ONE gpurun call)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-rgbd_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import youth_icp  # noqa: E402
import youth_synth  # noqa: E402


def rate(W, H, iters, calls=400, windows=5):
    src, dst, _ = youth_synth.pairs(0, 1, W, H)
    ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
    out = torch.zeros((1, 16), device="cuda")
    s = torch.cuda.Stream()
    ctx = youth_icp.IcpContext(W, H, 2, iters=iters)
    for _ in range(40):
        ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), 1, d_T_out=out.data_ptr(),
                               stream=s.cuda_stream)
    torch.cuda.synchronize()
    rates = []
    for _ in range(windows):
        t0 = time.perf_counter()
        for _ in range(calls):
            ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), 1, d_T_out=out.data_ptr(),
                                   stream=s.cuda_stream)
        torch.cuda.synchronize()
        rates.append(calls / (time.perf_counter() - t0))
    T, _, st = ctx.get_poses(1)
    To, _, sto, _ = oracle.align(src[0], dst[0], iters=iters)
    err = float(np.abs(T[0][:3] - To[:3]).max())
    ctx.close()
    return np.median(rates), max(rates), err, int(st[0])


label = sys.argv[1] if len(sys.argv) > 1 else "cur"
for W, H, it in ((640, 480, 10), (1280, 960, 20)):
    med, best, err, st = rate(W, H, it, calls=400 if W == 640 else 100)
    print(f"{label:>8s} {W}x{H} {it} it: median {med:8.0f} aligns/s  best {best:8.0f}  "
          f"us/align {1e6 / med:7.1f}  pose err {err:.1e}  status {st}", flush=True)
