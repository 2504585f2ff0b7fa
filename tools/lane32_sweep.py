#!/usr/bin/env python3
"""CPU sweep (oracle only): poses of spec a9's lane32 reduction (fp32 lane sums
over a given launch partition, fp64 finalize) against the exact reduction, on
the bench's cases and on larger §8d-noise samples.  Test
tooling; takes ~40 s on 8 cores."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "slam-rgbd_amd")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
import youth_synth  # noqa: E402


def sweep(name, src, dst, K, iters, geoms):
    Te, _ = oracle.align_batch(src, dst, K=K, iters=iters)
    for g in geoms:
        with oracle.reduction("lane32", g):
            Tl, _ = oracle.align_batch(src, dst, K=K, iters=iters)
        d = np.abs(Tl - Te)[:, :3, :].max(axis=(1, 2))
        print(f"{name:10s} lanes {g}: max {d.max():.2e} (pair {d.argmax()}), "
              f"> 1e-6: {(d > 1e-6).sum()}, > 1e-5: {(d > 1e-5).sum()} of {len(d)}", flush=True)


K = oracle.viewer_K(640, 480)
s, d, _ = youth_synth.pairs(0, 64)
sweep("C2-64", s, d, K, 10, [(0, 51200, 256, 0), (0, 2048, 256, 0), (1, 0, 512, 3), (2, 0, 512, 3)])
s, d, _ = youth_synth.pairs(0, 2, 1280, 960)
sweep("C3", s, d, oracle.viewer_K(1280, 960), 20, [(2, 0, 512, 10), (0, 51200, 256, 0)])
fr, _ = youth_synth.sequence(0, 201)
sweep("C5-200", fr[1:], fr[:-1], K, 10, [(0, 28672, 256, 0)])
s, d, _ = youth_synth.pairs(0, 16, flags=youth_synth.SURVEY_FLAGS)
sweep("noise16", s, d, K, 10, [(0, 51200, 256, 0), (2, 0, 512, 3)])
s, d, _ = youth_synth.pairs(5000, 128)
sweep("C4-128", s, d, K, 10, [(0, 51200, 256, 0)])
s, d, _ = youth_synth.pairs(1000, 96, flags=youth_synth.SURVEY_FLAGS)
sweep("noise96", s, d, K, 10, [(0, 51200, 256, 0), (1, 0, 512, 3)])
s, d, _ = youth_synth.pairs(100, 21, 160, 120)
sweep("160x120", s, d, oracle.viewer_K(160, 120), 10, [(0, 2048, 256, 0), (1, 0, 512, 3)])
