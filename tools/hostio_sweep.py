#!/usr/bin/env python3
"""Host-buffer batch API (youth_icp_align_batch: H2D + align + pose D2H,
synchronous) over the pipelining chunk size YOUTH_ICP_BATCH_CHUNK (0: one
copy then one align), 64 synthetic 640x480 pairs, pageable and pinned host
buffers; poses compared with the unpipelined call's.
usage: python tools/hostio_sweep.py [reps]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-rgbd_amd"))
import numpy as np  # noqa: E402

import youth_icp  # noqa: E402
import youth_synth  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    src, dst, _ = youth_synth.pairs(0, 64)
    ps, pd = torch.from_numpy(src).pin_memory().numpy(), torch.from_numpy(dst).pin_memory().numpy()
    ref = None
    for chunk in (0, 4, 8, 16, 32, 0):
        os.environ["YOUTH_ICP_BATCH_CHUNK"] = str(chunk)
        line = f"chunk {chunk:2d}:"
        for kind, (s, d) in (("pageable", (src, dst)), ("pinned", (ps, pd))):
            T, _ = youth_icp.align_batch(s, d, iters=10)
            t0 = time.perf_counter()
            for _ in range(reps):
                T, _ = youth_icp.align_batch(s, d, iters=10)
            rate = reps * src.shape[0] / (time.perf_counter() - t0)
            if ref is None:
                ref = T
            err = float(np.abs(T - ref).max())
            line += f"  {kind} {rate:8.0f} aligns/s (max |dT| vs unpipelined {err:.1e})"
        print(line, flush=True)


if __name__ == "__main__":
    main()
