#!/usr/bin/env python3
"""Benchmark: ICP frame-pair aligns/sec @640x480 on 1..N MI355X.

A "step" = one pass of the hot path over one batch: every rank aligns its
shard of independent 640x480 pairs (back-project both frames, target normals,
10 fixed point-to-plane iterations, final pose on device), then the poses are
all-gathered over RCCL (N > 1).  Inputs are synthetic depth (libyouth_synth),
resident in HBM before the timed region.  Per-GPU work is fixed (weak
scaling); the default shard is BASELINE config C4's per-GPU share (64 pairs),
so N = 8 is exactly C4's 512-pair batch.

Launch: python bench.py [--gpus 1] [--steps K] [--warmup W]
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

# torch first so libyouth_icp binds to torch's HIP runtime
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "slam-rgbd_amd"))

import numpy as np  # noqa: E402

import youth_icp  # noqa: E402
import youth_synth  # noqa: E402

METRIC = "ICP frame-pair aligns/sec @640×480 (1/2/4/8 GPU); SE(3) err vs CPU ref"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
BYTES_PER_PX_ITER = 36       # src XYZ 12 + tgt XYZ 12 + tgt normal 12
KERNEL_BYTES_PER_PX = 18     # k_reduce own bytes: src depth 2 + tgt record {z,n} 16


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pairs-per-gpu", type=int, default=64)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: min(16, cpus)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per reduction launch (from tools/pmc_traffic.py)")
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        a.gpus = world if world > 1 else a.gpus
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    W, H, n = a.width, a.height, a.pairs_per_gpu
    N = W * H
    # rank r aligns global pairs [r*n, (r+1)*n): seeds 0x5EED0000 + global index
    src, dst, _ = youth_synth.pairs(rank * n, n, W, H)
    d_src = torch.from_numpy(src).cuda()
    d_dst = torch.from_numpy(dst).cuda()
    poses = torch.zeros((n, 16), dtype=torch.float32, device="cuda")
    gathered = torch.zeros((world * n, 16), dtype=torch.float32, device="cuda")
    ctx = youth_icp.IcpContext(W, H, 2 * n, iters=a.iters, device=local)
    stream = torch.cuda.current_stream().cuda_stream

    def step():
        ctx.align_pairs_device(d_src.data_ptr(), d_dst.data_ptr(), n,
                               d_T_out=poses.data_ptr(), stream=stream)
        if world > 1:
            dist.all_gather_into_tensor(gathered, poses)

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ctx.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    red_ms, red_n = ctx.get_timing(0)
    solve_ms, solve_n = ctx.get_timing(1)
    prep_ms, prep_n = ctx.get_timing(2)
    ctx.set_timing(False)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # HBM roofline of the dominant kernel (k_reduce): algorithmic bytes per launch
    red_avg_ms = red_ms / max(red_n, 1)
    bytes_per_launch = BYTES_PER_PX_ITER * N * n
    achieved = bytes_per_launch / (red_avg_ms * 1e-3) / 1e9
    traffic = None
    traffic_src = None
    if os.path.exists(a.traffic_json):
        try:
            tj = json.load(open(a.traffic_json))
            if tj.get("pairs") == n and tj.get("width") == W and tj.get("height") == H:
                traffic = tj.get("hbm_bytes_per_launch")
                traffic_src = os.path.relpath(a.traffic_json, ROOT)
        except (OSError, ValueError):
            traffic = None

    T_gpu, _, _ = ctx.get_poses(n)          # fp64 device poses of the last step
    result = {
        "metric": METRIC,
        "value": world * n * a.steps / elapsed,
        "unit": "aligns/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (ray-cast room scene, int16 mm depth, seeds 0x5EED0000+pair)",
        "config": {
            "workload": f"C4 per-GPU shard: {n} independent {W}x{H} pairs/GPU, "
                        f"{a.iters} point-to-plane iters (N=8 -> 512 pairs = C4)",
            "pairs_per_gpu": n, "global_pairs": world * n, "width": W, "height": H,
            "iters": a.iters,
            "parallelism": f"dp{world} (pair shards, RCCL pose all-gather)",
        },
        "roofline": {
            "bound": "hbm", "kernel": "k_reduce",
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": bytes_per_launch,
            "algorithmic_model": "SURVEY §8d: 36 B/px/iter x pixels x pairs",
            "kernel_bytes_per_launch": KERNEL_BYTES_PER_PX * N * n,
            "achieved_kernel_bytes": KERNEL_BYTES_PER_PX * N * n / (red_avg_ms * 1e-3) / 1e9,
            "frac_kernel_bytes": KERNEL_BYTES_PER_PX * N * n / (red_avg_ms * 1e-3) / 1e9
            / HBM_PEAK_GBS,
            "avg_launch_ms": red_avg_ms, "launches": red_n,
        },
        "kernel_ms_per_step": {
            "k_reduce": red_ms / a.steps, "k_solve": solve_ms / a.steps,
            "k_prep": prep_ms / a.steps,
        },
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        result["cpu_baseline"], result["parity"] = cpu_baseline(a, src, dst, T_gpu)
    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(a, src, dst, T_gpu):
    """The C oracle on host cores over a bounded sample of the same pairs
    (OpenMP over pairs); also the SE(3) error of the GPU poses on it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    cpus = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = a.cpu_threads or min(16, cpus or 1)
    S = a.pairs_per_gpu
    oracle.align_batch(src[:1], dst[:1], iters=a.iters, n_threads=1)  # warm
    # repeat passes over the rank-0 pairs until ~1.5 s wall (~10-30 s of CPU work)
    passes, wall, T_cpu, st = 0, 0.0, None, None
    while wall < 1.5 and passes < 50:
        t0 = time.perf_counter()
        T_cpu, st = oracle.align_batch(src, dst, iters=a.iters, n_threads=threads)
        wall += time.perf_counter() - t0
        passes += 1
    err = float(np.abs(T_gpu[:, :3, :] - T_cpu[:, :3, :]).max())
    cpu = {"value": passes * S / wall, "unit": "aligns/s", "cores": threads, "kind": "port",
           "sample": f"{passes} pass(es) over the {S} rank-0 pairs ({a.width}x{a.height}, "
                     f"{a.iters} iters): C oracle -O3 -ffp-contract=off, OpenMP over pairs, "
                     f"{wall:.2f} s wall"}
    parity = {"pose_max_abs_err_vs_cpu": err, "pairs_checked": S, "tolerance": 1e-5,
              "cpu_status_nonzero": int((st != 0).sum())}
    return cpu, parity


if __name__ == "__main__":
    main()
