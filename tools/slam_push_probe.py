#!/usr/bin/env python3
"""Where a slow Python-producer pass of processSlamFrame comes from: bench.py's
backlogged slam_api leg with 10 passes in one process, per pass the rate, the
producer's time inside processSlamFrame, the CPU and NUMA node the producer
ran on, and the NUMA nodes holding the source frames (/proc/self/numa_maps).
Usage: python3 tools/slam_push_probe.py [passes]."""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "slam-rgbd_amd"), ROOT]
import numpy as np  # noqa: E402
import psutil  # noqa: E402
import torch  # noqa: E402,F401

import bench  # noqa: E402
import youth_synth  # noqa: E402


def node_of_cpu(c):
    base = f"/sys/devices/system/cpu/cpu{c}"
    for n in os.listdir(base):
        if re.fullmatch(r"node\d+", n):
            return int(n[4:])
    return -1


def numa_of(addr):
    try:
        for line in open("/proc/self/numa_maps"):
            start = int(line.split()[0], 16)
            if start <= addr < start + (1 << 40):
                nodes = dict(re.findall(r"\bN(\d+)=(\d+)", line))
                if nodes:
                    return line.split()[0], nodes
    except OSError as e:
        return str(e), {}
    return None, {}


passes = int(sys.argv[1]) if len(sys.argv) > 1 else 10
print("cpus allowed", len(os.sched_getaffinity(0)), "online", os.cpu_count(),
      "loadavg", os.getloadavg(), flush=True)
frames, _ = youth_synth.sequence(0, 300, 640, 480)
fr = np.ascontiguousarray(frames, np.int16)
p = psutil.Process()
print("frames at", hex(fr.ctypes.data), "numa", numa_of(fr.ctypes.data), "producer cpu",
      p.cpu_num(), "node", node_of_cpu(p.cpu_num()), flush=True)
r = bench.slam_api_rate(None, fr, None, passes=passes)
for i, (v, us) in enumerate(zip(r["pass_values"], r["push_us_per_frame"])):
    print(f"pass {i}: {v:8.0f} frames/s  push {us:6.1f} us/frame", flush=True)
print("after: producer cpu", p.cpu_num(), "node", node_of_cpu(p.cpu_num()), "numa",
      numa_of(fr.ctypes.data), "loadavg", os.getloadavg(), flush=True)
