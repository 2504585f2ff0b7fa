#!/usr/bin/env python3
"""processSlamFrame producer-copy A/B: the backlogged
drop-in rate from one Python producer (bench.py's slam_api leg) and from the
plain-C producer (slam_rate), YOUTH_SLAM_PUSH_COPY=memcpy vs nt (streaming
stores), optionally with YOUTH_SLAM_PUSH_THREADS helpers (mode "nt+2"), interleaved
rounds on one box; each line: mode, rate, push us/frame."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
modes = sys.argv[2:] or ["memcpy", "nt"]
child = r'''
import os, sys, json
sys.path.insert(0, os.path.join(%r, "slam-rgbd_amd")); sys.path.insert(0, %r)
import numpy as np, torch, bench, youth_synth
frames, _ = youth_synth.sequence(0, 300, 640, 480)
r = bench.slam_api_rate(None, frames, None, passes=5)
print(json.dumps({"value": r["value"], "push_us": float(np.median(r["push_us_per_frame"])),
                  "passes": [round(v) for v in r["pass_values"]]}))
''' % (ROOT, ROOT)
for rnd in range(rounds):
    for m in modes:
        # a mode is <copy>[+<helper threads>], e.g. nt+2
        cp, _, th = m.partition("+")
        env = dict(os.environ, YOUTH_SLAM_PUSH_COPY=cp, YOUTH_SLAM_PUSH_THREADS=th or "0")
        r = subprocess.run([sys.executable, "-c", child], env=env, capture_output=True, text=True,
                           timeout=300, cwd=ROOT)
        if r.returncode:
            print(r.stderr[-2000:])
            sys.exit(1)
        py = json.loads(r.stdout.strip().splitlines()[-1])
        c = subprocess.run([os.path.join(ROOT, "slam-rgbd_amd", "slam_rate"), "300", "5", "640", "480"],
                           env=env, capture_output=True, text=True, timeout=300)
        if c.returncode:
            print(c.stderr[-2000:])
            sys.exit(1)
        cj = json.loads(c.stdout.strip().splitlines()[-1])
        cpush = sorted(cj["push_us_per_frame"])[len(cj["push_us_per_frame"]) // 2]
        print(f"round {rnd} {m:>7s}: python {py['value']:8.0f} frames/s push {py['push_us']:5.1f} us "
              f"{py['passes']}   C {cj['value']:8.0f} push {cpush:5.1f} us {cj['pass_values']}",
              flush=True)
