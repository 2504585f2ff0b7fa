#!/usr/bin/env python3
"""Benchmark: ICP frame-pair aligns/sec @640x480 on 1..N MI355X.

Default workload ("pairs", BASELINE config C4 per-GPU share): a "step" is one
pass of the hot path over one batch — every rank aligns its 64 independent
640x480 pairs (target records, 10 fixed point-to-plane iterations, final
pose on device), then the fp32 poses are all-gathered over RCCL (N > 1).
Inputs are synthetic int16 depth (libyouth_synth), resident in HBM before
the timed region.  Per-GPU work is fixed (weak scaling); N = 8 is exactly
C4's 512-pair batch.

`--workload sequence` (config C5): a streamed synthetic sequence of
--frames frames (default 1000) split over the ranks with a 1-frame halo;
each step aligns every (k, k+1) pair (each frame prepared once), gathers the
relative poses and composes the trajectory on rank 0.  Total work is fixed
(strong scaling).

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

import youth_dist  # noqa: E402
import youth_icp  # noqa: E402
import youth_synth  # noqa: E402
import youth_viewer  # noqa: E402

METRIC = "ICP frame-pair aligns/sec @640×480 (1/2/4/8 GPU); SE(3) err vs CPU ref"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
BYTES_PER_PX_ITER = 36       # src XYZ 12 + tgt XYZ 12 + tgt normal 12
KERNEL_BYTES_PER_PX = 18     # k_reduce own bytes: src depth 2 + tgt record {z,n} 16


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["pairs", "sequence"], default="pairs")
    ap.add_argument("--pairs-per-gpu", type=int, default=64)
    ap.add_argument("--frames", type=int, default=1000, help="sequence workload length")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: min(16, cpus)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-single-pair", action="store_true",
                    help="skip the C2 leg (one pair per align call) / the streamed sequence leg "
                         "(rank 0, N=1)")
    ap.add_argument("--no-viewer", action="store_true",
                    help="skip the viewer point-list leg (SURVEY §8 f4; rank 0, N=1)")
    ap.add_argument("--no-host-io", action="store_true",
                    help="skip the PCIe-inclusive host-buffer API leg (rank 0, N=1)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes per k_reduce launch (tools/pmc_traffic.py)")
    return ap.parse_args()


class Run:
    def __init__(self, a):
        self.a = a
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        # one process per GPU; ranks beyond the visible devices wrap (only for a
        # rehearsal on fewer GPUs with YOUTH_BENCH_BACKEND=gloo: RCCL needs one
        # device per rank)
        self.local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
        torch.cuda.set_device(self.local)
        if self.world > 1:
            backend = os.environ.get("YOUTH_BENCH_BACKEND", "nccl")   # nccl = RCCL over xGMI
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            else:
                dist.init_process_group(backend)

    def barrier_sync(self):
        torch.cuda.synchronize()
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def timed(self, ctx, step):
        a = self.a
        for _ in range(a.warmup):
            step()
        self.barrier_sync()
        # events around the iteration kernel only inside the timed region (the
        # roofline's launch durations); every kernel kind in a short pass after it
        ctx.set_timing(True, iteration_kernel_only=True)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            step()
        self.barrier_sync()
        elapsed = time.perf_counter() - t0
        kt = {"k_reduce": ctx.get_timing(0)}
        ctx.set_timing(True)
        extra = min(a.steps, 5)
        for _ in range(extra):
            step()
        self.barrier_sync()
        for i, k in ((1, "k_solve"), (2, "k_prep")):
            ms, cnt = ctx.get_timing(i)
            kt[k] = (ms * a.steps / extra, cnt)   # scaled to the timed region's step count
        ctx.set_timing(False)
        if self.world > 1:
            dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed, kt

    def roofline(self, kt, pixels_per_iter):
        """k_reduce is timed per launch; the persistent kernel (k_icp) runs
        every iteration of an align in ONE launch, so bytes and the PMC
        traffic are scaled by the iterations each launch covers."""
        red_ms, red_n = kt["k_reduce"]
        avg = red_ms / max(red_n, 1)
        iters_per_launch = max(1, round(self.a.steps * self.a.iters / max(red_n, 1)))
        pixels_per_launch = pixels_per_iter * iters_per_launch
        alg = BYTES_PER_PX_ITER * pixels_per_launch
        own = KERNEL_BYTES_PER_PX * pixels_per_launch
        traffic, src, valu = None, None, None
        if os.path.exists(self.a.traffic_json):
            try:
                tj = json.load(open(self.a.traffic_json))
                if tj.get("width") == self.a.width and tj.get("height") == self.a.height and \
                        tj.get("pairs") * self.a.width * self.a.height == pixels_per_iter:
                    per_iter = tj.get("hbm_bytes_per_iteration", tj.get("hbm_bytes_per_launch"))
                    traffic = per_iter * iters_per_launch
                    src = os.path.relpath(self.a.traffic_json, ROOT)
                    if "valu_cycles_per_instruction" in tj:   # PMC SQ pass, same kernel
                        valu = {k: tj[k] for k in ("valu_cycles_per_instruction",
                                                   "valu_lane_ops_per_px_iteration",
                                                   "effective_clock_ghz") if k in tj}
            except (OSError, ValueError, TypeError):
                traffic = None
        achieved = alg / (avg * 1e-3) / 1e9
        return {
            "bound": "hbm",
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
            "valu_limit": valu,
            "algorithmic_bytes_per_launch": alg,
            "algorithmic_model": "SURVEY §8d: 36 B/px/iter x pixels x pairs",
            "kernel_bytes_per_launch": own,
            "achieved_kernel_bytes": own / (avg * 1e-3) / 1e9,
            "frac_kernel_bytes": own / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "avg_launch_ms": avg, "launches": red_n, "iterations_per_launch": iters_per_launch,
            "kernel": "k_icp (persistent, all iterations)" if iters_per_launch > 1 else "k_reduce",
        }

    def finish(self):
        if self.world > 1:
            dist.destroy_process_group()


def run_pairs(R):
    a, world, rank = R.a, R.world, R.rank
    W, H, n = a.width, a.height, a.pairs_per_gpu
    first, cnt = youth_dist.pair_shard(rank, n)      # seeds 0x5EED0000 + global index
    src, dst, _ = youth_synth.pairs(first, cnt, W, H)
    d_src = torch.from_numpy(src).cuda()
    d_dst = torch.from_numpy(dst).cuda()
    # double-buffered poses: the RCCL gather of step s runs on its own stream
    # while step s+1 aligns; step s+2 waits for it before reusing the buffers
    # (every gather completes inside the timed region: final device sync)
    poses = [torch.zeros((n, 16), dtype=torch.float32, device="cuda") for _ in range(2)]
    gathered = [torch.zeros((world * n, 16), dtype=torch.float32, device="cuda")
                for _ in range(2)]
    pending = [None, None]
    ctx = youth_icp.IcpContext(W, H, max(n, 2), iters=a.iters, device=R.local)
    stream = torch.cuda.current_stream().cuda_stream
    it = [0]

    def step():
        b = it[0] & 1
        it[0] += 1
        if pending[b] is not None:
            pending[b].wait()
        ctx.align_pairs_device(d_src.data_ptr(), d_dst.data_ptr(), n,
                               d_T_out=poses[b].data_ptr(), stream=stream)
        pending[b] = youth_dist.gather_poses_async(poses[b], gathered[b], world)

    elapsed, kt = R.timed(ctx, step)
    T_gpu, _, _ = ctx.get_poses(n)          # fp64 poses of the last step
    lb = (it[0] - 1) & 1                     # the last step's gathered poses: every rank's
    if world > 1 and not np.array_equal(gathered[lb][R.rank * n:(R.rank + 1) * n].cpu().numpy(),
                                        poses[lb].cpu().numpy()):
        raise RuntimeError("pose all-gather: this rank's rows differ from its poses")
    result = base_result(R, world * n * a.steps / elapsed, elapsed)
    result["scaling"] = "weak"
    result["config"] = {
        "workload": f"C4 per-GPU shard: {n} independent {W}x{H} pairs/GPU, "
                    f"{a.iters} point-to-plane iters (N=8 -> 512 pairs = C4)",
        "pairs_per_gpu": n, "global_pairs": world * n, "width": W, "height": H,
        "iters": a.iters, "fastdiv": ctx.fastdiv,
        "parallelism": f"dp{world} (pair shards, RCCL pose all-gather)",
    }
    result["roofline"] = R.roofline(kt, n * W * H)
    result["kernel_ms_per_step"] = {k: v[0] / a.steps for k, v in kt.items()}
    spins, waited = ctx.get_sched_stats()   # last align: persistent-kernel pose waits
    result["sched_last_step"] = {"epoch_polls": spins, "items_waited": waited}
    result["kernel_path"] = ctx.get_plan()
    if rank == 0 and world == 1 and not a.no_host_io:
        result["host_io"] = host_io_rate(a, src, dst)
    T_cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        result["cpu_baseline"], result["parity"], T_cpu = cpu_baseline(a, src, dst, T_gpu)
    if rank == 0 and world == 1 and not a.no_single_pair and n > 1:
        result["single_pair"] = single_pair_rate(R, d_src, d_dst, T_cpu)
    if rank == 0 and world == 1 and not a.no_viewer:
        result["viewer_cloud"] = viewer_cloud_rate(R, d_dst, dst)
    ctx.close()
    return result


def single_pair_rate(R, d_src, d_dst, T_cpu, steps=400, warmup=40):
    """BASELINE configs[1] (C2): ONE 640x480 pair per align call, calls back
    to back on one stream (the latency path: processSlamFrame's tracker),
    inputs resident in HBM.  Reported beside the C4-shard value, never as it;
    the pose is checked against the C oracle's pose of the same pair."""
    a = R.a
    ctx = youth_icp.IcpContext(a.width, a.height, 2, iters=a.iters, device=R.local)
    out = torch.zeros((1, 16), dtype=torch.float32, device="cuda")
    # the library's own (non-blocking) stream: nothing in torch consumes `out`
    # before the final synchronize.  (Cooperative launches on the bench's torch
    # stream ran at half this rate inside this process, 4.5 K vs 9.1 K aligns/s,
    # though not in a standalone probe: tools/stream_probe.py)
    stream = 0
    s0, t0p = d_src[0:1].data_ptr(), d_dst[0:1].data_ptr()
    for _ in range(warmup):
        ctx.align_pairs_device(s0, t0p, 1, d_T_out=out.data_ptr(), stream=stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ctx.align_pairs_device(s0, t0p, 1, d_T_out=out.data_ptr(), stream=stream)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    T1, _, st = ctx.get_poses(1)
    res = {"config": f"C2: one {a.width}x{a.height} pair per call, {a.iters} iters",
           "value": steps / el, "unit": "aligns/s", "us_per_align": el / steps * 1e6,
           "steps": steps, "warmup": warmup, "kernel_path": ctx.get_plan(),
           "status": int(st[0])}
    if T_cpu is not None:
        res["pose_max_abs_err_vs_cpu"] = float(np.abs(T1[0, :3, :] - T_cpu[0, :3, :]).max())
    ctx.close()
    return res


def viewer_cloud_rate(R, d_depth, depth_host, reps=20, warmup=3):
    """the viewer's vertex list (viewerModule.c:336-357) for the
    rank's n frames in one device call (youth_cloud_build_device: count, scan,
    emit), synthetic RGB, inputs resident in HBM; HIP events on the launching
    stream.  Algorithmic bytes: 2 B depth + 3 B colour per pixel read, 24 B
    per vertex written.  Frame 0's list is checked bit-exact against the C
    oracle (oracle_viewer_cloud)."""
    a = R.a
    n, H, W = depth_host.shape
    rgb = np.random.default_rng(0xC0105).integers(0, 256, size=(n, H, W, 3), dtype=np.uint8)
    d_rgb = torch.from_numpy(rgb).cuda()
    verts = torch.empty((n, H * W, 6), dtype=torch.float32, device="cuda")
    counts = torch.zeros(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    cb = youth_viewer.CloudBuilder(W, H, max_frames=n, device=R.local)

    def call():
        cb.build_device(d_depth.data_ptr(), d_rgb.data_ptr(), n, W, H, verts.data_ptr(),
                        counts.data_ptr(), stream=s.cuda_stream)

    for _ in range(warmup):
        call()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        call()
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    cnt = counts.cpu().numpy()
    nbytes = float(n * H * W * 5 + int(cnt.sum()) * 24)
    res = {"frames_per_call": n, "width": W, "height": H, "us_per_call": ms * 1e3,
           "value": n / (ms * 1e-3), "unit": "frames/s",
           "vertices_per_frame": float(cnt.mean()),
           "roofline": {"bound": "hbm", "achieved": nbytes / (ms * 1e-3) / 1e9,
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                        "algorithmic_bytes_per_call": nbytes,
                        "kernels": "k_cloud_count + k_cloud_scan + k_cloud_emit"}}
    if not a.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        want = oracle.viewer_cloud(depth_host[0], rgb[0])
        got = verts[0, : int(cnt[0])].cpu().numpy()
        res["bit_exact_vs_cpu"] = bool(got.shape == want.shape and
                                       np.array_equal(got.view(np.uint32), want.view(np.uint32)))
        t0 = time.perf_counter()
        for f in range(min(n, 8)):
            oracle.viewer_cloud(depth_host[f], rgb[f])
        res["cpu_frames_per_s_1thread"] = min(n, 8) / (time.perf_counter() - t0)
    cb.close()
    return res


def run_sequence(R):
    a, world, rank = R.a, R.world, R.rank
    W, H, F = a.width, a.height, a.frames
    f0, f1 = youth_dist.sequence_shard(F, world, rank)
    nf = f1 - f0
    npairs = max(nf - 1, 0)
    frames, _ = youth_synth.sequence(f0, max(nf, 2), W, H)
    d_frames = torch.from_numpy(frames).cuda()
    rel = torch.zeros((max(npairs, 1), 16), dtype=torch.float32, device="cuda")
    ctx = youth_icp.IcpContext(W, H, max(npairs, 2), iters=a.iters, device=R.local)
    stream = torch.cuda.current_stream().cuda_stream
    max_rows = (F - 1 + world - 1) // world
    counts = [max(0, (lambda f: f[1] - f[0] - 1)(youth_dist.sequence_shard(F, world, r)))
              for r in range(world)]
    traj = {}

    def step():
        if npairs:
            ctx.align_sequence_device(d_frames.data_ptr(), nf, d_T_out=rel.data_ptr(),
                                      stream=stream)
        rows = youth_dist.gather_ragged(rel[:npairs], world, max_rows, counts)
        if rank == 0:
            traj["T"] = rows   # composed after the timed region (host, ordered fp64)

    elapsed, kt = R.timed(ctx, step)
    result = base_result(R, (F - 1) * a.steps / elapsed, elapsed)
    result["scaling"] = "strong"
    result["config"] = {
        "workload": f"C5: {F}-frame synthetic sequence, {W}x{H}, streamed frame-to-frame "
                    f"odometry, {a.iters} iters, {F - 1} pairs split over ranks (1-frame halo)",
        "frames": F, "pairs": F - 1, "width": W, "height": H, "iters": a.iters,
        "parallelism": f"dp{world} (contiguous pair ranges, RCCL pose gather)",
    }
    result["roofline"] = R.roofline(kt, max(npairs, 1) * W * H)
    if rank == 0:
        T = youth_dist.compose_trajectory(traj["T"].cpu().numpy().reshape(-1, 4, 4))
        result["trajectory_frames"] = int(T.shape[0])
        if world == 1 and not a.no_single_pair:
            result["streamed"] = streamed_rate(a, frames, rel[:npairs].cpu().numpy())
    ctx.close()
    return result


def streamed_rate(a, frames, rel_batch, n=300):
    """The same sequence streamed frame by frame from HOST memory through the
    tracker (youth_icp_track_frame: processSlamFrame's path): per frame one
    614 KB H2D, target prep of the new frame + 10 iterations against the
    previous one (one k_icp_coop launch), pose D2H, synchronous.  Reported
    beside the batch value; relative poses checked against the batch run's."""
    n = min(n, frames.shape[0])
    ctx = youth_icp.IcpContext(a.width, a.height, 2, iters=a.iters)
    ctx.track_frame(frames[0])
    ctx.track_frame(frames[1])                         # warm
    ctx.track_reset()
    t0 = time.perf_counter()
    rel = []
    for f in range(n):
        T, st, has = ctx.track_frame(frames[f])
        if has:
            rel.append(T)
    el = time.perf_counter() - t0
    plan = ctx.get_plan()
    ctx.close()
    rel = np.stack(rel)
    err = float(np.abs(rel[:, :3, :] - rel_batch[: n - 1].reshape(-1, 4, 4)[:, :3, :]).max())
    return {"frames": n, "value": n / el, "unit": "frames/s", "us_per_frame": el / n * 1e6,
            "kernel_path": plan, "max_abs_diff_vs_batch_poses": err,
            "note": "host frames, H2D + align + pose D2H per frame, synchronous"}


def base_result(R, value, elapsed):
    a = R.a
    return {
        "metric": METRIC,
        "value": value,
        "unit": "aligns/s",
        "n_gpus": R.world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic (ray-cast room scene, int16 mm depth, seeds 0x5EED0000+pair / "
                "0x5EED1000 sequence)",
    }


def host_io_rate(a, src, dst, reps=5):
    """PCIe-inclusive rate of the one-shot host API (youth_icp_align_batch):
    H2D of both depth stacks + align + D2H of the poses, synchronous, from
    pageable (numpy) and pinned (torch pin_memory) host buffers; the H2D of
    chunk k+1 overlaps the align of chunk k (16-pair chunks).  Reported beside
    the bench value, never as it (inputs there are resident in HBM)."""
    out = {"api": "youth_icp_align_batch", "pairs": int(src.shape[0]),
           "h2d_bytes_per_pair": int(2 * src[0].nbytes)}
    ps = torch.from_numpy(src).pin_memory()
    pd = torch.from_numpy(dst).pin_memory()
    for kind, (s, d) in (("pageable", (src, dst)), ("pinned", (ps.numpy(), pd.numpy()))):
        youth_icp.align_batch(s, d, iters=a.iters)          # warm: batch context, pages
        t0 = time.perf_counter()
        for _ in range(reps):
            youth_icp.align_batch(s, d, iters=a.iters)
        out[kind + "_aligns_per_s"] = reps * src.shape[0] / (time.perf_counter() - t0)
    return out


def cpu_baseline(a, src, dst, T_gpu):
    """The C oracle on the host cores of the GPU box over a bounded sample of
    the same pairs: one warm-up, then the median of >= 5 timed
    passes, (i) OpenMP over pairs on up to 16 threads (the reported value),
    (ii) one thread on a 2-pair sample; also the SE(3) error of the GPU poses."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    cpus = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    threads = a.cpu_threads or min(16, cpus or 1)
    S = src.shape[0]
    oracle.align_batch(src[:threads], dst[:threads], iters=a.iters, n_threads=threads)  # warm
    rates, T_cpu, st = [], None, None
    while len(rates) < 5 or (sum(S / r for r in rates) < 1.5 and len(rates) < 50):
        t0 = time.perf_counter()
        T_cpu, st = oracle.align_batch(src, dst, iters=a.iters, n_threads=threads)
        rates.append(S / (time.perf_counter() - t0))
    single = []
    oracle.align_batch(src[:1], dst[:1], iters=a.iters, n_threads=1)  # warm
    for _ in range(5):
        t0 = time.perf_counter()
        oracle.align_batch(src[:2], dst[:2], iters=a.iters, n_threads=1)
        single.append(2 / (time.perf_counter() - t0))
    err = float(np.abs(T_gpu[:, :3, :] - T_cpu[:, :3, :]).max())
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")),
                         "")
    except OSError:
        pass
    cpu = {"value": float(np.median(rates)), "unit": "aligns/s", "cores": threads, "kind": "port",
           "sample": f"median of {len(rates)} passes over the {S} rank-0 pairs ({a.width}x"
                     f"{a.height}, {a.iters} iters) after 1 warm-up: C oracle -O3 "
                     f"-ffp-contract=off, OpenMP over pairs",
           "single_thread": {"value": float(np.median(single)), "unit": "aligns/s", "cores": 1,
                             "sample": "median of 5 passes over 2 pairs"},
           "host": {"cpu_model": model, "cpus_visible": cpus}}
    parity = {"pose_max_abs_err_vs_cpu": err, "pairs_checked": S, "tolerance": 1e-5,
              "cpu_status_nonzero": int((st != 0).sum())}
    return cpu, parity, T_cpu


def main():
    a = parse()
    R = Run(a)
    # a non-default torch stream: its handle is what every align is issued on,
    # so the pose copies and the RCCL gathers (which wait on torch's current
    # stream) are ordered after the kernels that write the poses (handle 0 would
    # select the library's private stream instead)
    with torch.cuda.stream(torch.cuda.Stream()):
        result = run_pairs(R) if a.workload == "pairs" else run_sequence(R)
    if R.rank == 0:
        print(json.dumps(result), flush=True)
    R.finish()


if __name__ == "__main__":
    main()
