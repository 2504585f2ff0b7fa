#!/usr/bin/env python3
"""C3 workload alone (1280x960, 20 iterations), for rocprofv3 passes:
`reps` single-pair calls (k_icp_coop, 64x80 prep tiles fused) and `reps`
16-pair batch calls (k_prep + persistent k_icp) on device-resident inputs,
each pose checked against the C oracle once at the end.

usage: python tools/c3_probe.py [reps]   (under rocprofv3 --pmc ... -- python3 ...)
"""
import os
import sys

import torch  # noqa: F401  (HIP runtime first)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "slam-rgbd_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import youth_icp  # noqa: E402
import youth_synth  # noqa: E402

W, H, IT, N = 1280, 960, 20, 16
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
src, dst, _ = youth_synth.pairs(0, N, W, H)
ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
torch.cuda.synchronize()
ctx = youth_icp.IcpContext(W, H, N, iters=IT)
for k in (1, N):
    for _ in range(reps):
        ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), k)
    ctx.sync()
    T, _, st = ctx.get_poses(k)
    Tc, stc = oracle.align_batch(src[:k], dst[:k], iters=IT, n_threads=min(k, 16))
    err = float(np.abs(T[:, :3] - Tc[:, :3]).max())
    print(f"{k} pair(s) per call: {ctx.get_plan()['kernel']}, pose err {err:.2e}, "
          f"status {int(st.max())}", flush=True)
    assert err <= 1e-5 and not st.any()
ctx.close()
