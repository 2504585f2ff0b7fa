#!/usr/bin/env python3
"""A/B of the viewer point-list kernels (csrc/viewer_cloud.hip) in one process:
pixels per thread (YOUTH_CLOUD_PX 4|8),
64 synthetic 640x480 frames + random RGB per call, HIP events on one stream,
every variant's output compared bitwise with the first's.
usage: python tools/cloud_ab.py [reps] [rounds]"""
import os
import sys

import torch  # noqa: F401  (first: shared HIP runtime)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-rgbd_amd"))
import numpy as np  # noqa: E402

import youth_synth  # noqa: E402
import youth_viewer  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    _, dst, _ = youth_synth.pairs(0, 64)
    n, H, W = dst.shape
    rgb = np.random.default_rng(5).integers(0, 256, size=(n, H, W, 3), dtype=np.uint8)
    d = torch.from_numpy(dst).cuda()
    c = torch.from_numpy(rgb).cuda()
    s = torch.cuda.Stream()   # a real handle: 0 would select the builder's own stream
    ref = None
    for r in range(rounds):
        for px in (8, 4):
            os.environ["YOUTH_CLOUD_PX"] = str(px)
            cb = youth_viewer.CloudBuilder(W, H, max_frames=n)
            v = torch.zeros((n, H * W, 6), dtype=torch.float32, device="cuda")
            k = torch.zeros(n, dtype=torch.int32, device="cuda")

            def call():
                cb.build_device(d.data_ptr(), c.data_ptr(), n, W, H, v.data_ptr(), k.data_ptr(),
                                stream=s.cuda_stream)
            for _ in range(5):
                call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(reps):
                call()
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / reps * 1e3
            cnt = k.cpu().numpy()
            out = v.cpu().numpy()
            same = "ref"
            if ref is None:
                ref = (cnt, out)
            else:
                same = bool(np.array_equal(cnt, ref[0]) and
                            np.array_equal(out.view(np.uint32), ref[1].view(np.uint32)))
            nbytes = n * H * W * 5 + int(cnt.sum()) * 24
            print(f"round {r} px {px}: {us:8.1f} us/call  "
                  f"{nbytes / us / 1e3:7.0f} GB/s  same={same}", flush=True)
            cb.close()


if __name__ == "__main__":
    main()
