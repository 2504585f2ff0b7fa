#!/usr/bin/env python3
"""Benchmark: ICP frame-pair aligns/sec @640x480 on 1..N MI355X.

Default workload ("pairs", BASELINE config C4): ONE batch of 512 independent
640x480 pairs, split into contiguous shards over the N ranks (SURVEY §8e:
512 / 256 / 128 / 64 pairs per GPU at N = 1 / 2 / 4 / 8; strong scaling).
A "step" is one pass of the hot path over the batch: every rank aligns its
shard (target records, 10 fixed point-to-plane iterations), the fp32 poses
are all-gathered over RCCL (N > 1) and copied into pinned host memory (async
D2H + event, no host sync inside the step), so "final pose available on
host" (§8d) is part of every step.  Inputs are synthetic int16 depth
(libyouth_synth), resident in HBM before the timed region.
`--pairs-per-gpu n` switches to weak scaling (n pairs per GPU).

`--workload sequence` (config C5 over N GPUs): a synthetic sequence of
--frames frames (default 1000) split over the ranks with a 1-frame halo;
each step aligns every (k, k+1) pair (each frame prepared once), gathers the
relative poses and composes the trajectory on rank 0 (strong scaling).

At N = 1, rank 0 also runs, after the timed region and beside the headline
value: the C2 (one pair per call), C3 (1280x960, 20 iterations) and C5
(1000-frame sequence: batch and streamed) legs, each with its pose error
against the C oracle; the PCIe-inclusive host-buffer API; the viewer point
list (§8 f4); and the CPU baseline (the C oracle on the host cores).

Launch: python bench.py [--gpus N] [--steps K] [--warmup W]   (N > 1: bench.py starts
        torch.distributed.run with N ranks as a child process and exits with its code)
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
Rank 0 prints ONE JSON line.
"""
import argparse
import ctypes
import hashlib
import json
import math
import os
import sys
import time



def _launch_ranks(argv=None, environ=None, run=None):
    """`--gpus N` is the rank count (the driver's contract): without a
    launcher (WORLD_SIZE unset) and N > 1, start N ranks through
    torch.distributed.run as a CHILD process with the same arguments, let it
    write to this process's stdout/stderr, and return its exit code.  Under a
    launcher, --gpus must equal WORLD_SIZE (a mismatch would print a line whose
    n_gpus is not the requested N).  Runs before torch is imported and before
    any HIP call, so nothing here has touched the GPU.  Returns None when this
    process is itself the (only) rank."""
    import argparse as _ap
    import socket
    import subprocess
    argv = sys.argv[1:] if argv is None else argv
    environ = os.environ if environ is None else environ
    p = _ap.ArgumentParser(add_help=False)
    p.add_argument("--gpus", type=int, default=1)
    n = p.parse_known_args(argv)[0].gpus
    if n < 1:
        sys.stderr.write(f"bench.py: --gpus {n} < 1\n")
        return 2
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != n:
            sys.stderr.write(f"bench.py: --gpus {n} != WORLD_SIZE {ws} under the launcher\n")
            return 2
        return None
    if n == 1:
        return None
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(n), "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + list(argv)
    env = dict(environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")    # dmabuf IPC only on this pool
    return (run or subprocess.call)(cmd, env=env)


if __name__ == "__main__":
    _rc = _launch_ranks()
    if _rc is not None:
        sys.exit(_rc)

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
ICP_BYTES_PER_PX_ITER = 18   # k_icp per pixel-iteration: src depth 2 + tgt record {z,n} 16
SURVEY_BYTES_PER_PX_ITER = 36  # SURVEY.md §8d model: src XYZ 12 + tgt XYZ 12 + tgt normal 12
PREP_BYTES_PER_PX = 18       # k_prep per target pixel: depth 2 in + record 16 out
KERNEL_SRC = os.path.join(ROOT, "slam-rgbd_amd", "csrc", "icp_kernels.hip")
POSE_TOL = 1e-5              # north star: recovered SE(3) within 1e-5 of the CPU reference


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=["pairs", "sequence"], default="pairs")
    ap.add_argument("--global-pairs", type=int, default=512, help="C4 batch (strong scaling)")
    ap.add_argument("--pairs-per-gpu", type=int, default=0,
                    help="> 0: weak scaling with this many pairs per GPU")
    ap.add_argument("--frames", type=int, default=1000, help="sequence workload length")
    ap.add_argument("--pipeline", type=int, default=0, choices=[0, 1, 2, 3, 4],
                    help="pairs workload: steps in flight per rank; 2 = two contexts on two "
                         "streams, so step s+1's k_prep / k_icp fill step s's k_icp tail "
                         "(independent batches, each completed inside the timed region); "
                         "0 = auto: 2 for shards of <= 192 pairs, each k_icp on half the "
                         "workgroup slots (--share; N = 8's 64 pairs: +4 %%, N = 4's 128: "
                         "+2 %%), else 1 (256 pairs: neutral; profiles/r03/ab_share.txt)")
    ap.add_argument("--share", type=int, default=0, choices=[0, 1, 2, 3, 4],
                    help="pairs workload: k_icp slot share per context "
                         "(youth_icp_set_concurrency); 0 = the steps in flight")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--min-warmup-ms", type=float, default=100.0,
                    help="after the --warmup steps, run more untimed steps until the warm-up has "
                         "lasted this long (the GPU's clock ramps over ~10-20 ms from idle; "
                         "reported as warmup_steps_run); 0 = exactly --warmup steps")
    ap.add_argument("--windows", type=int, default=3,
                    help="extra timed windows of --steps steps after the timed region (spread)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-legs", action="store_true",
                    help="skip the C2 / C3 / C5 legs (rank 0, N=1)")
    ap.add_argument("--no-single-pair", action="store_true", help="skip the C2 leg")
    ap.add_argument("--c3-pairs", type=int, default=16, help="C3 leg batch (1280x960)")
    ap.add_argument("--c5-frames", type=int, default=1000, help="C5 leg sequence length")
    ap.add_argument("--no-viewer", action="store_true",
                    help="skip the viewer point-list leg (SURVEY §8 f4; rank 0, N=1)")
    ap.add_argument("--no-host-io", action="store_true",
                    help="skip the PCIe-inclusive host-buffer API leg (rank 0, N=1)")
    ap.add_argument("--spec", choices=["survey", "fma"],
                    default=os.environ.get("YOUTH_ICP_SPEC", "survey"),
                    help="arithmetic of spec a7/a8 (youth_icp_set_spec): survey = SURVEY.md §8a "
                         "as worded (the default), fma = the opt-in fma-chain form; the oracle "
                         "checks in the same spec")
    ap.add_argument("--reduce", choices=["lane32", "exact"],
                    default=os.environ.get("YOUTH_ICP_REDUCE", "exact"),
                    help="spec a9's reduction (youth_icp_set_reduce): exact = every product exact "
                         "in fp64, launch-independent (the default); lane32 = fp32 lane sums -> "
                         "fp64 finalize (opt-in: depends on the launch's lane partition)")
    ap.add_argument("--no-spec-parity", action="store_true",
                    help="skip the spec-parity leg (rank 0, N=1)")
    ap.add_argument("--dump-poses", default="",
                    help="after the run, every rank writes its shard's fp64 poses (pairs: the last "
                         "step's; sequence: its relative poses) to PATH.rank<r>.npy, and rank 0 "
                         "the C5 world trajectory to PATH.traj.npy (the N-rank rehearsal compares "
                         "them with the N = 1 run's)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic.json"),
                    help="PMC-derived HBM bytes and VALU figures of k_icp (tools/pmc_traffic.py)")
    return ap.parse_args()


def oracle_mod():
    """The C oracle (the checker; legs after the timed region), in the spec
    the library runs (YOUTH_ICP_SPEC, set from --spec in main)."""
    import oracle
    oracle.set_spec(os.environ.get("YOUTH_ICP_SPEC", "survey"))
    return oracle


def kernel_digest():
    with open(KERNEL_SRC, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


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
        # YOUTH_BENCH_DIST=1 brings the process group up at N = 1 too, so the
        # RCCL gather path runs on a one-GPU box (tests/test_gpu_bench.py)
        self.dist_on = self.world > 1 or os.environ.get("YOUTH_BENCH_DIST") == "1"
        if self.dist_on:
            backend = os.environ.get("YOUTH_BENCH_BACKEND", "nccl")   # nccl = RCCL over xGMI
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
            else:
                dist.init_process_group(backend)

    def barrier_sync(self):
        torch.cuda.synchronize()
        if self.dist_on:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(self, x):
        if not self.dist_on:
            return x
        dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def window(self, step, k):
        self.barrier_sync()
        t0 = time.perf_counter()
        for _ in range(k):
            step()
        self.barrier_sync()
        return self.max_over_ranks(time.perf_counter() - t0)

    def timed(self, ctx, step):
        """W warm-up steps, then EXACTLY K timed steps between barrier + sync
        (max over ranks), HIP events around the iteration kernel only; then
        `windows` more K-step windows (spread) and a short pass timing every
        kernel kind (k_prep)."""
        a = self.a
        t0 = time.perf_counter()
        for _ in range(a.warmup):
            step()
        self.warmup_steps_run = a.warmup
        if a.warmup > 0 and a.min_warmup_ms > 0:
            # W steps of a small shard (64 pairs: 5 x 0.9 ms) end before the
            # clock has ramped up: the first timed window then ran 11 % below
            # the steady windows (profiles/r02/warm_probe.txt).  Same count on
            # every rank: a step holds the RCCL gather.
            # one more step timed alone estimates a step (the first warm-up
            # step also carries one-time setup)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            step()
            torch.cuda.synchronize()
            per = time.perf_counter() - t1
            need = a.min_warmup_ms * 1e-3 - (time.perf_counter() - t0)
            extra = min(100000, math.ceil(need / per)) if need > 0 else 0
            extra = int(self.max_over_ranks(float(extra)))
            for _ in range(extra):
                step()
            self.warmup_steps_run += 1 + extra
        ctx.set_timing(True, iteration_kernel_only=True)
        elapsed = self.window(step, a.steps)
        kt = {"k_icp": ctx.get_timing(0)}
        ctx.set_timing(False)
        spread = [self.window(step, a.steps) for _ in range(a.windows)]
        ctx.set_timing(True)
        extra = min(a.steps, 5)
        self.window(step, extra)
        kt["k_prep"] = ctx.get_timing(2)
        kt["prep_pass_steps"] = extra
        ctx.set_timing(False)
        return elapsed, kt, spread

    def finish(self):
        if self.dist_on:
            dist.destroy_process_group()


class CtxGroup:
    """The rank's contexts (one per step in flight) as one for timing:
    events on every context, times and launch counts summed."""

    def __init__(self, ctxs):
        self.ctxs = ctxs

    def set_timing(self, enable, iteration_kernel_only=False):
        for c in self.ctxs:
            c.set_timing(enable, iteration_kernel_only)

    def get_timing(self, kind=0):
        t = [c.get_timing(kind) for c in self.ctxs]
        return sum(x[0] for x in t), sum(x[1] for x in t)


def load_pmc(a, W, H):
    """The committed PMC pass of k_icp (tools/profile.sh + tools/pmc_traffic.py):
    HBM bytes and VALU figures per pixel-iteration, valid only for the kernel
    source it was taken on (sha256 prefix) and the same frame size."""
    try:
        tj = json.load(open(a.traffic_json))
    except (OSError, ValueError):
        return None, "no PMC pass committed"
    if tj.get("kernel_sha16") != kernel_digest():
        return None, f"stale: {os.path.relpath(a.traffic_json, ROOT)} was taken on another build"
    if tj.get("width") != W or tj.get("height") != H:
        return None, "PMC pass taken at another frame size"
    return tj, os.path.relpath(a.traffic_json, ROOT)


# Same-box knockout timings of k_icp: the share of the kernel's time each
# instruction group accounts for when it is removed (timing-only builds, wrong
# sums).  The exact reduction's fp64 update (the default) was 16 % of k_icp
# (profiles/r03/ab_knockout.txt), next to the 32 % the issue account priced
# it at; the opt-in lane32 form's update (28 fp32 FMAs per pixel) is 2.2-2.8 %
# (profiles/r04/ab_r4a.txt: 4724 -> 4622 us, 4699 -> 4569 us).
KNOCKOUTS = {
    "source": "profiles/r03/ab_knockout.txt (exact), profiles/r04/ab_r4a.txt (lane32)",
    "exact_fp64_update": {"measured_time_share": 0.16, "issue_account_share": 0.32,
                          "reduction": "exact (default)"},
    "lane32_fp32_update": {"measured_time_share": 0.025, "reduction": "lane32 (opt-in)"},
    "target_int_to_float": {"measured_time_share": 0.005, "issue_account_share": 0.033},
}


# best 16-B/px non-temporal write stream over 512 x 640 x 480 px measured on
# an MI355X (tools/hbm_write_bw: 0.426 ms for 2.52 GB; 65536 x 512 threads)
WRITE_STREAM_CEILING_GBS = 5903.0
# best 16-B-per-lane streaming read of the same 2.52 GB (0.389 ms; 65536 x 512,
# profiles/r04/hbm_bw_r4w.txt): what a pure read stream reaches on this GPU
READ_STREAM_CEILING_GBS = 6476.0


def roofline_icp(a, kt, n_pairs, W, H, concurrent=1):
    """Roofline of the dominant kernel, k_icp (persistent: all iterations of
    an align in ONE launch).  `achieved` = the kernel's algorithmic bytes
    (18 B per pixel-iteration: 2 B source depth + one 16-B target record,
    DESIGN.md §3) x pixels x iterations per launch / the average launch
    duration from HIP events on the launch stream inside the timed region.
    `traffic` = PMC-measured HBM bytes per launch (same build); `survey_model`
    = the same time against SURVEY §8d's 36 B/px model.  `concurrent` > 1:
    that many launches run side by side, each on 1/concurrent of the
    workgroup slots (youth_icp_set_concurrency), so the chip's rate is
    concurrent x bytes per launch / launch duration."""
    ms, launches = kt["k_icp"]
    avg = ms / max(launches, 1) / concurrent  # chip time per launch
    ipl = max(1, round(a.steps * a.iters / max(launches, 1)))
    px = n_pairs * W * H * ipl
    alg = ICP_BYTES_PER_PX_ITER * px
    achieved = alg / (avg * 1e-3) / 1e9
    tj, src = load_pmc(a, W, H)
    traffic = tj["bytes_per_px"] * px if tj else None
    out = {
        "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
        "kernel": "k_icp (persistent, all iterations of the batch)",
        "algorithmic_bytes_per_launch": alg,
        "algorithmic_model": "18 B per pixel-iteration (src depth 2 + tgt record 16) x pairs x "
                             "W x H x iterations",
        "avg_launch_ms": avg * concurrent, "launches": launches, "iterations_per_launch": ipl,
        "concurrent_launches": concurrent,
        "survey_model": {"bytes_per_px_iter": SURVEY_BYTES_PER_PX_ITER,
                         "achieved": SURVEY_BYTES_PER_PX_ITER * px / (avg * 1e-3) / 1e9,
                         "frac": SURVEY_BYTES_PER_PX_ITER * px / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "note": "SURVEY §8d counts XYZ planes the kernel does not move"},
    }
    if traffic is not None:
        out["traffic_frac"] = traffic / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS
        out["traffic_over_algorithmic"] = traffic / alg
        # k_icp's bytes are reads: against the measured streaming-read ceiling
        out["read_stream_ceiling"] = {
            "value": READ_STREAM_CEILING_GBS, "unit": "GB/s",
            "source": "profiles/r04/hbm_bw_r4w.txt (tools/hbm_write_bw read16)",
            "traffic_frac": traffic / (avg * 1e-3) / 1e9 / READ_STREAM_CEILING_GBS}
    # what bounds k_icp, from same-box knockout timings: the
    # share of the kernel's time each instruction group accounts for when it
    # is removed.  The PMC issue account (below, "valu") is an upper estimate
    # that exceeds 1 when the mixed stream overlaps better than the isolated
    # forms, so it is reported, not used as the limiter.
    out["limiter"] = "VALU issue + exposed memory latency (knockout shares)"
    out["critical_path"] = KNOCKOUTS
    if tj and "valu_busy_frac" in tj:
        out["valu"] = {k: tj[k] for k in ("valu_busy_frac", "valu_lane_ops_per_px_iteration",
                                          "valu_cycles_per_instruction", "effective_clock_ghz",
                                          "valu_busy_definition", "wave_state_frac",
                                          "rocprof_valubusy") if k in tj}
        if "valu_account" in tj:
            acc = tj["valu_account"]
            out["valu"]["busy_frac_range"] = [acc["busy_frac_other_at_2_4_cycles"],
                                              acc["busy_frac"]]
            out["valu"]["issue_cycles_by_class_frac"] = {
                k: v / acc["simd_cycles_available"] for k, v in acc["issue_cycles_by_class"].items()}
    return out




def roofline_prep(a, kt, n_frames, W, H):
    """k_prep (target records, once per align): 2 B depth in + 16 B record out
    per target pixel, HIP events over a short pass after the timed region.
    `traffic` (PMC HBM bytes: the halo re-reads show up here)
    and the VALU issue fraction come from the committed PMC pass of the same
    kernel source, as for k_icp."""
    ms, launches = kt["k_prep"]
    if launches == 0:
        return None
    avg = ms / launches
    px = n_frames * W * H
    alg = PREP_BYTES_PER_PX * px
    ach = alg / (avg * 1e-3) / 1e9
    out = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": ach / HBM_PEAK_GBS, "kernel": "k_prep", "algorithmic_bytes_per_launch": alg,
           "algorithmic_model": "18 B per target pixel (depth 2 in + record 16 out)",
           "avg_launch_ms": avg, "launches": launches}
    tj, src = load_pmc(a, W, H)
    if tj and "k_prep_bytes_per_px" in tj:
        traffic = tj["k_prep_bytes_per_px"] * px
        out.update({"traffic": traffic, "traffic_source": src,
                    "traffic_frac": traffic / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS,
                    "traffic_over_algorithmic": traffic / alg,
                    # 16 of the 18 B/px are writes: against the measured
                    # ceiling of a pure 16-B/px non-temporal write stream
                    "write_stream_ceiling": {
                        "value": WRITE_STREAM_CEILING_GBS, "unit": "GB/s",
                        "source": "profiles/r04/hbm_write_bw_r4u.txt (tools/hbm_write_bw)",
                        "traffic_frac": traffic / (avg * 1e-3) / 1e9 / WRITE_STREAM_CEILING_GBS}})
    if tj and "k_prep_valu_busy_frac" in tj:
        acc = tj["k_prep_valu_account"]
        out["valu_issue_frac"] = tj["k_prep_valu_busy_frac"]
        out["valu_busy_frac_range"] = [acc["busy_frac_other_at_2_4_cycles"], acc["busy_frac"]]
    return out


def parity_sample(n):
    """Shard positions every rank checks against the CPU oracle after the
    timed region: its first two and last two pairs."""
    return sorted({i for i in (0, 1, n - 2, n - 1) if 0 <= i < n})


def shard_parity(a, src, dst, T, idx):
    """max |T - T_cpu| over the pairs `idx` of this rank's shard (src[i] is
    aligned onto dst[i]; T the GPU's fp64 poses), the C oracle in the exact
    reduction, a few threads per rank."""
    if not idx:
        return 0.0
    oracle = oracle_mod()
    idx = np.asarray(idx)
    T_cpu, _ = oracle.align_batch(np.ascontiguousarray(src[idx]), np.ascontiguousarray(dst[idx]),
                                  iters=a.iters, n_threads=min(len(idx), 4))
    return pose_err(np.asarray(T)[idx], T_cpu)


def parity_gate(result):
    """True when every rank's sampled poses are within POSE_TOL of the CPU
    oracle; stored in the line as `parity_all_ranks_ok` (rank 0 then exits
    non-zero if False)."""
    errs = result["ranks"].get("per_rank", {}).get("pose_max_abs_err_vs_cpu", [])
    ok = bool(errs) and max(errs) <= POSE_TOL
    result["parity_all_ranks_ok"] = ok
    return ok


def pose_err(Ta, Tb):
    """max |Ta - Tb| over the 3x4 entries (any leading shape)."""
    Ta = np.asarray(Ta, np.float64).reshape(-1, 4, 4)
    Tb = np.asarray(Tb, np.float64).reshape(-1, 4, 4)
    return float(np.abs(Ta[:, :3, :] - Tb[:, :3, :]).max())


def run_pairs(R):
    a, world, rank = R.a, R.world, R.rank
    W, H = a.width, a.height
    if a.pairs_per_gpu > 0:
        n_glob = world * a.pairs_per_gpu
        first, n = youth_dist.pair_shard(rank, a.pairs_per_gpu)
        scaling = "weak"
    else:
        n_glob = a.global_pairs
        first, n = youth_dist.pair_range(n_glob, world, rank)
        scaling = "strong"
    counts = [youth_dist.pair_range(n_glob, world, r)[1] for r in range(world)]
    src, dst, _ = youth_synth.pairs(first, n, W, H)     # seeds 0x5EED0000 + global index
    d_src = torch.from_numpy(src).cuda()
    d_dst = torch.from_numpy(dst).cuda()
    main = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    # double-buffered: step s aligns into poses[s&1], the RCCL gather of it
    # runs on RCCL's stream and the D2H into pinned host memory on `side`
    # while step s+1 aligns; step s+2 waits for that D2H (event) before
    # reusing the buffers.  Everything completes inside the timed region.
    poses = [torch.zeros((n, 16), dtype=torch.float32, device="cuda") for _ in range(2)]
    gathered = [torch.zeros((n_glob, 16), dtype=torch.float32, device="cuda")
                for _ in range(2)] if R.dist_on else poses
    host = [torch.zeros((n_glob, 16), dtype=torch.float32).pin_memory()
            for _ in range(2)]
    done = [None, None]
    depth = a.pipeline or (2 if n <= 192 else 1)
    # --pipeline 2: step s runs on context / stream s % 2 (each context its
    # own records, poses and queue words), so consecutive steps are
    # independent and the GPU starts step s+1's kernels as step s's
    # persistent k_icp retires its workgroups
    ctxs = [youth_icp.IcpContext(W, H, max(n, 2), iters=a.iters, device=R.local)
            for _ in range(depth)]
    # the steps in flight run side by side, each persistent k_icp on 1/depth
    # of the workgroup slots (DESIGN.md §5 "Small shards")
    share = depth if a.share == 0 else a.share
    for c in ctxs:
        c.set_concurrency(share)
    ctx = ctxs[0]
    streams = [main] + [torch.cuda.Stream() for _ in range(depth - 1)]
    it = [0]

    def step():
        b = it[0] & 1
        q = it[0] % depth
        it[0] += 1
        st = streams[q]
        with torch.cuda.stream(st):
            if done[b] is not None:
                st.wait_event(done[b])
            ctxs[q].align_pairs_device(d_src.data_ptr(), d_dst.data_ptr(), n,
                                       d_T_out=poses[b].data_ptr(), stream=st.cuda_stream)
            work = youth_dist.gather_poses_ragged_async(poses[b], gathered[b], world, counts)
            with torch.cuda.stream(side):
                if work is not None:
                    work.wait()             # side waits for the gather (no host block)
                else:
                    side.wait_stream(st)
                host[b].copy_(gathered[b], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(side)
                done[b] = ev

    elapsed, kt, spread = R.timed(CtxGroup(ctxs), step)
    torch.cuda.synchronize()
    ctx = ctxs[(it[0] - 1) % depth]          # the context of the last step
    T_gpu, _, st_gpu = ctx.get_poses(n)      # fp64 poses of the last step
    lb = (it[0] - 1) & 1
    last_host = host[lb].numpy().reshape(-1, 4, 4)
    mine = last_host[first:first + n]
    if not np.array_equal(mine, poses[lb].cpu().numpy().reshape(-1, 4, 4)):
        raise RuntimeError("host pose copy / all-gather: this rank's rows differ from its poses")
    result = base_result(R, n_glob * a.steps / elapsed, elapsed)
    result["scaling"] = scaling
    result["config"] = {
        "workload": (f"C4: {n_glob} independent {W}x{H} pairs over {world} GPU(s) "
                     f"({n} on rank 0), {a.iters} point-to-plane iters, poses gathered to host"
                     if scaling == "strong" else
                     f"C4 weak: {n} independent {W}x{H} pairs per GPU, {a.iters} iters"),
        "global_pairs": n_glob, "pairs_per_gpu": n, "width": W, "height": H,
        "iters": a.iters, "fastdiv": ctx.fastdiv,
        "parallelism": f"dp{world} (contiguous pair shards, RCCL pose all-gather)",
        "steps_in_flight": depth, "k_icp_slot_share": f"1/{share}",
    }
    result["window_rates"] = [n_glob * a.steps / s for s in spread]
    result["roofline"] = roofline_icp(a, kt, n, W, H, share)
    result["roofline_prep"] = roofline_prep(a, kt, n, W, H)
    result["kernel_ms_per_step"] = {"k_icp": kt["k_icp"][0] / max(kt["k_icp"][1], 1),
                                    "k_prep": kt["k_prep"][0] / max(kt["prep_pass_steps"], 1)}
    spins, waited = ctx.get_sched_stats()   # last align: persistent-kernel pose waits
    result["sched_last_step"] = {"epoch_polls": spins, "items_waited": waited}
    result["kernel_path"] = ctx.get_plan()
    result["status_nonzero"] = int((st_gpu != 0).sum())
    # every rank's own k_icp / k_prep / gather times and the group's size
    # (collective: all ranks), so an N > 1 line shows that N ranks ran and
    # splits compute from the collective
    gms = gather_ms(R, poses[0], gathered[0], world, counts, main, side)
    # every rank checks its shard's first and last two pairs against the CPU
    # oracle (these pairs sit at the shard's own launch geometry)
    idx = parity_sample(n)
    perr = shard_parity(a, src, dst, T_gpu, idx)
    if a.dump_poses:
        np.save(f"{a.dump_poses}.rank{rank}.npy", np.asarray(T_gpu, np.float64).reshape(-1, 4, 4))
    result["ranks"] = youth_dist.rank_report({
        "k_icp_ms": result["kernel_ms_per_step"]["k_icp"],
        "k_prep_ms": result["kernel_ms_per_step"]["k_prep"],
        "gather_ms": gms if gms is not None else 0.0}, world,
        {"pose_max_abs_err_vs_cpu": perr, "pairs_checked": len(idx)})
    result["ranks"]["gather_timed"] = gms is not None
    result["ranks"]["parity_sample"] = "each rank: its shard's first 2 and last 2 pairs vs the C oracle"
    parity_gate(result)
    if rank == 0 and world == 1:
        leg = {}
        if not a.no_cpu_baseline:
            m = min(n, 64)
            result["cpu_baseline"], result["parity"] = cpu_baseline(a, src[:m], dst[:m],
                                                                    T_gpu[:m])
            result["parity"]["survey_noise"] = survey_noise_parity(a, ctx, main)
        if not a.no_host_io:
            result["host_io"] = host_io_rate(a, src[:64], dst[:64])
        if not a.no_legs:
            if not a.no_single_pair:
                leg["c2"] = single_pair_rate(R, d_src, d_dst, src[0], dst[0])
            leg["c3"] = c3_rate(R, n=a.c3_pairs)
            leg["c5"] = c5_rate(R, F=a.c5_frames, stream_frames=min(300, a.c5_frames))
        if not a.no_viewer:
            leg["viewer_cloud"] = viewer_cloud_rate(R, d_dst[:64], dst[:64])
        if not a.no_spec_parity:
            leg["spec_parity"] = spec_parity(a, main)
            leg["spec_parity"]["other_spec_rate"] = other_spec_rate(R, ctxs, step, n_glob)
            leg["spec_parity"]["other_reduce_rate"] = other_reduce_rate(R, ctxs, step, n_glob)
        result.update(leg)
    for c in ctxs:
        c.close()
    return result


def gather_ms(R, local, out, world, counts, main, side, reps=5):
    """Median time of the pose all-gather alone (after the timed region, the
    align idle): HIP events on the launch stream before the collective and
    on the side stream after its wait.  None without a process group."""
    if not R.dist_on:
        return None
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        work = youth_dist.gather_poses_ragged_async(local, out, world, counts)
        with torch.cuda.stream(side):
            if work is not None:
                work.wait()
            else:
                side.wait_stream(main)
            e1.record(side)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return float(np.median(ts))


def other_spec_rate(R, ctxs, step, n_glob):
    """The headline step in the OTHER spec a7/a8 arithmetic on the same
    contexts and inputs (after the timed region): its rate and k_icp time."""
    a = R.a
    other = "fma" if a.spec == "survey" else "survey"
    torch.cuda.synchronize()
    for c in ctxs:
        c.spec = other
    for _ in range(5):
        step()
    g = CtxGroup(ctxs)
    g.set_timing(True, iteration_kernel_only=True)
    el = R.window(step, a.steps)
    ms, n = g.get_timing(0)
    g.set_timing(False)
    for c in ctxs:
        c.spec = a.spec
    return {"spec": other, "value": n_glob * a.steps / el, "unit": "aligns/s",
            "k_icp_ms": ms / max(n, 1)}


def other_reduce_rate(R, ctxs, step, n_glob):
    """The headline step with the OTHER spec a9 reduction (lane32 <-> exact)
    on the same contexts and inputs (after the timed region)."""
    a = R.a
    other = "exact" if a.reduce == "lane32" else "lane32"
    torch.cuda.synchronize()
    for c in ctxs:
        c.reduction = other
    for _ in range(5):
        step()
    g = CtxGroup(ctxs)
    g.set_timing(True, iteration_kernel_only=True)
    el = R.window(step, a.steps)
    ms, n = g.get_timing(0)
    g.set_timing(False)
    for c in ctxs:
        c.reduction = a.reduce
    return {"reduce": other, "value": n_glob * a.steps / el, "unit": "aligns/s",
            "k_icp_ms": ms / max(n, 1)}


def spec_parity(a, main):
    """how far the GPU's poses sit from the
    survey-spec oracle with exact products (SURVEY §8a a7/a8 as worded, the
    strictest sums) in each arithmetic x reduction the kernels implement, on
    C2's 640x480 pairs (64), C3 (2 pairs at 1280x960, 20 iterations), C5 (a
    201-frame sequence: 200 relative poses) and at SURVEY §8d's noise (16
    pairs).  Also each variant against the oracle run in the same variant
    (lane32: the oracle's lane sums over the GPU launch's own lane partition,
    youth_icp_get_lanes): the bit-exactness bar, ~1e-13."""
    oracle = oracle_mod()
    cases = {}
    s64 = youth_synth.pairs(0, 64)
    cases["c2_64_pairs"] = (s64[0], s64[1], 640, 480, 10, None)
    s3 = youth_synth.pairs(0, 2, 1280, 960)
    cases["c3_2_pairs_1280x960_20it"] = (s3[0], s3[1], 1280, 960, 20, None)
    fr, _ = youth_synth.sequence(0, 201)
    cases["c5_200_pairs"] = (fr[1:], fr[:-1], 640, 480, 10, fr)
    sn = youth_synth.pairs(0, 16, flags=youth_synth.SURVEY_FLAGS)
    cases["survey_noise_16_pairs"] = (sn[0], sn[1], 640, 480, 10, None)
    out = {}
    worst, same = {}, {}
    for name, (src, dst, W, H, iters, frames) in cases.items():
        n = src.shape[0]
        K = youth_icp.default_intrinsics(W, H)
        row = {"pairs": n}
        ref = {}

        def oracle_poses(sp, lanes):
            with oracle.spec(sp), oracle.reduction("lane32" if lanes else "exact", lanes):
                return oracle.align_batch(src, dst, K=oracle.viewer_K(W, H), iters=iters,
                                          n_threads=min(n, _cpus()))[0]

        for sp in ("survey", "fma"):
            ref[sp, "exact"] = oracle_poses(sp, None)
        ctx = youth_icp.IcpContext(W, H, max(n, 2), K=K, iters=iters)
        if frames is not None:
            df = torch.from_numpy(frames).cuda()
        else:
            ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
        for sp in ("survey", "fma"):
            for red in ("lane32", "exact"):
                ctx.spec, ctx.reduction = sp, red
                if frames is not None:
                    ctx.align_sequence_device(df.data_ptr(), n + 1, stream=main.cuda_stream)
                else:
                    ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n,
                                           stream=main.cuda_stream)
                T, _, st = ctx.get_poses(n)
                if red == "lane32":
                    lanes = ctx.lanes()
                    row["lanes"] = dict(zip(("kind", "chunk", "threads", "npx"), lanes))
                    ref[sp, red] = oracle_poses(sp, lanes)
                v = sp if red == "exact" else f"{sp}_{red}"
                row[f"gpu_{v}_vs_survey_oracle"] = pose_err(T, ref["survey", "exact"])
                row[f"gpu_{v}_vs_same_variant_oracle"] = pose_err(T, ref[sp, red])
                row[f"gpu_{v}_status_nonzero"] = int((st != 0).sum())
                worst[v] = max(worst.get(v, 0.0), row[f"gpu_{v}_vs_survey_oracle"])
                same[v] = max(same.get(v, 0.0), row[f"gpu_{v}_vs_same_variant_oracle"])
        ctx.close()
        out[name] = row
    out["max_vs_survey_oracle"] = worst
    out["max_vs_same_variant_oracle"] = same
    dv = a.spec if a.reduce == "exact" else f"{a.spec}_{a.reduce}"
    out["default_variant"] = dv
    out["default_within_tol_of_survey_spec"] = bool(worst[dv] <= POSE_TOL)
    return out


def single_pair_rate(R, d_src, d_dst, src0, dst0, steps=400, warmup=40):
    """BASELINE configs[1] (C2): ONE 640x480 pair per align call, calls back
    to back on the caller's (torch) stream: the latency path of
    processSlamFrame's tracker, inputs resident in HBM; pose checked against
    the C oracle's pose of the same pair."""
    oracle = oracle_mod()
    a = R.a
    ctx = youth_icp.IcpContext(a.width, a.height, 2, iters=a.iters, device=R.local)
    out = torch.zeros((1, 16), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
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
    T_cpu, _, _, _ = oracle.align(src0, dst0, iters=a.iters)
    res = {"config": f"C2: one {a.width}x{a.height} pair per call, {a.iters} iters, "
                     "caller's torch stream",
           "value": steps / el, "unit": "aligns/s", "us_per_align": el / steps * 1e6,
           "steps": steps, "warmup": warmup, "kernel_path": ctx.get_plan(),
           "status": int(st[0]), "pose_max_abs_err_vs_cpu": pose_err(T1[0], T_cpu)}
    # k_icp_coop is the whole align (one launch per call, back to back: the
    # kernel trace shows no gaps, profiles/r05/c2_c3_kernel_trace_r5zm.txt)
    nbytes = 18.0 * a.width * a.height * a.iters
    gbs = nbytes / (el / steps) / 1e9
    res["roofline"] = {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": gbs / HBM_PEAK_GBS, "kernel": "k_icp_coop (target prep fused: "
                       "its 18 B/px not counted)", "algorithmic_bytes_per_launch": nbytes,
                       "algorithmic_model": "18 B per pixel-iteration x W x H x iters",
                       "time": "wall clock per call over the timed calls"}
    ctx.close()
    return res


def c3_rate(R, n=16, W=1280, H=960, iters=20):
    """BASELINE configs[2] (C3): 1280x960 pairs with per-pixel normals, 20
    iterations, 1 GPU: one pair per call (the LDS-tiled small-batch kernel)
    and an n-pair batch per call (persistent kernel); every pose checked
    against the C oracle (OpenMP over the 16 pairs)."""
    oracle = oracle_mod()
    src, dst, _ = youth_synth.pairs(0, n, W, H)
    d_src, d_dst = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    out = torch.zeros((n, 16), dtype=torch.float32, device="cuda")
    ctx = youth_icp.IcpContext(W, H, n, iters=iters, device=R.local)
    res = {"config": f"C3: {W}x{H} pairs, {iters} iters, 1 GPU"}
    for tag, k, reps in (("single_pair", 1, 100), ("batch", n, 20)):
        for _ in range(3):
            ctx.align_pairs_device(d_src.data_ptr(), d_dst.data_ptr(), k,
                                   d_T_out=out.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.align_pairs_device(d_src.data_ptr(), d_dst.data_ptr(), k,
                                   d_T_out=out.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        T, _, st = ctx.get_poses(k)
        plan = ctx.get_plan()
        # roofline of the iteration kernel: its own
        # 18 B per pixel-iteration x W x H x iters x pairs per launch over the
        # launch time (HIP events on the launch stream, a separate pass)
        ctx.set_timing(True, iteration_kernel_only=True)
        for _ in range(min(reps, 20)):
            ctx.align_pairs_device(d_src.data_ptr(), d_dst.data_ptr(), k,
                                   d_T_out=out.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        ms, nl = ctx.get_timing(0)
        ctx.set_timing(False)
        avg = ms / max(nl, 1)
        alg = ICP_BYTES_PER_PX_ITER * W * H * iters * k
        ach = alg / (avg * 1e-3) / 1e9
        kname = plan["kernel"]
        res[tag] = {"value": k * reps / el, "unit": "aligns/s", "pairs_per_call": k,
                    "us_per_call": el / reps * 1e6, "kernel_path": plan,
                    "status_nonzero": int((st != 0).sum()),
                    "roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS,
                                 "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
                                 "kernel": ("k_icp_coop (target prep fused: its 18 B/px "
                                            "not counted)") if kname == "k_icp_coop" else
                                           "k_icp (persistent; k_prep separate)",
                                 "algorithmic_bytes_per_launch": alg,
                                 "algorithmic_model": "18 B per pixel-iteration x W x H x "
                                                      "iters x pairs",
                                 "avg_launch_ms": avg, "launches": nl}}
        res[tag]["_T"] = T
    threads = min(n, _cpus())
    t0 = time.perf_counter()
    T_cpu, st_cpu = oracle.align_batch(src, dst, iters=iters, n_threads=threads)
    cpu_s = time.perf_counter() - t0
    for tag in ("single_pair", "batch"):
        T = res[tag].pop("_T")
        res[tag]["pose_max_abs_err_vs_cpu"] = pose_err(T, T_cpu[:T.shape[0]])
    res["cpu"] = {"value": n / cpu_s, "unit": "aligns/s", "cores": threads,
                  "cpu_status_nonzero": int((st_cpu != 0).sum())}
    res["parity_ok"] = bool(max(res[t]["pose_max_abs_err_vs_cpu"]
                                for t in ("single_pair", "batch")) <= POSE_TOL)
    ctx.close()
    return res


def c5_rate(R, F=1000, sample_every=16, stream_frames=300, reps=3):
    """BASELINE configs[4] (C5) on one GPU: the 1000-frame synthetic sequence
    (999 frame pairs, each frame prepared once) as one device-resident batch
    per call, and streamed frame by frame from host memory through the
    tracker (processSlamFrame's path).  Relative poses checked against the C
    oracle on every `sample_every`-th pair; streamed poses against the batch's."""
    oracle = oracle_mod()
    a = R.a
    W, H = a.width, a.height
    frames, _ = youth_synth.sequence(0, F, W, H)
    d_frames = torch.from_numpy(frames).cuda()
    stream = torch.cuda.current_stream().cuda_stream
    rel = torch.zeros((F - 1, 16), dtype=torch.float32, device="cuda")
    ctx = youth_icp.IcpContext(W, H, F - 1, iters=a.iters, device=R.local)
    ctx.align_sequence_device(d_frames.data_ptr(), F, d_T_out=rel.data_ptr(), stream=stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        ctx.align_sequence_device(d_frames.data_ptr(), F, d_T_out=rel.data_ptr(), stream=stream)
    rel_host = rel.cpu().numpy().reshape(-1, 4, 4)     # poses on host inside the timing
    el = time.perf_counter() - t0
    T64, _, st = ctx.get_poses(F - 1)
    ctx.close()
    ks = np.arange(0, F - 1, sample_every)
    threads = min(len(ks), _cpus())
    T_cpu, _ = oracle.align_batch(frames[ks + 1], frames[ks], iters=a.iters, n_threads=threads)
    res = {"config": f"C5: {F}-frame {W}x{H} synthetic sequence, {F - 1} pairs, {a.iters} iters, "
                     "1 GPU",
           "batch": {"value": (F - 1) * reps / el, "unit": "aligns/s",
                     "ms_per_sequence": el / reps * 1e3,
                     "pose_max_abs_err_vs_cpu": pose_err(T64[ks], T_cpu),
                     "pairs_checked": int(len(ks)), "status_nonzero": int((st != 0).sum()),
                     "trajectory_frames": int(youth_dist.compose_trajectory(rel_host).shape[0])}}
    res["streamed"] = streamed_rate(a, frames[:stream_frames], rel_host)
    res["parity_ok"] = bool(res["batch"]["pose_max_abs_err_vs_cpu"] <= POSE_TOL)
    return res


def streamed_rate(a, frames, rel_batch, passes=5):
    """The sequence streamed frame by frame from HOST memory through the
    tracker (processSlamFrame's worker path): per frame one 614 KB copy into
    pinned staging + H2D on a transfer stream, target prep of the new frame +
    10 iterations against the previous one (one k_icp_coop launch), the pose
    written into pinned memory by the kernel.  `value`: the library's own
    loop over a host sequence, two frames in flight as the SLAM worker runs
    them (youth_icp_track_host_sequence: frame k+1's copy and H2D overlap
    frame k's align); `python_pipelined_value`: the same through per-frame
    youth_icp_track_submit / _collect calls from Python; `sync_value`:
    youth_icp_track_frame, one frame at a time.  Median of `passes` passes
    each (host-side timing).  Relative poses checked against the batch run's
    (fp32 output rounding) and the three modes against each other (bitwise)."""
    n = frames.shape[0]
    ctx = youth_icp.IcpContext(a.width, a.height, 2, iters=a.iters)
    ctx.track_frame(frames[0])
    ctx.track_frame(frames[1])                         # warm
    r_sync, r_py, r_c = [], [], []
    for _ in range(passes):
        ctx.track_reset()
        t0 = time.perf_counter()
        sync = []
        for f in range(n):
            T, st, has = ctx.track_frame(frames[f])
            if has:
                sync.append(T)
        r_sync.append(n / (time.perf_counter() - t0))
        ctx.track_reset()
        t0 = time.perf_counter()
        rel = []
        for f in range(n):
            ctx.track_submit(frames[f])
            if ctx.track_pending() == 2:
                T, st, has = ctx.track_collect()
                if has:
                    rel.append(T)
        while ctx.track_pending():
            T, st, has = ctx.track_collect()
            if has:
                rel.append(T)
        r_py.append(n / (time.perf_counter() - t0))
        ctx.track_reset()
        t0 = time.perf_counter()
        Tc, _ = ctx.track_host_sequence(frames)
        r_c.append(n / (time.perf_counter() - t0))
    plan = ctx.get_plan()
    ctx.close()
    # micro-batches of m frames (a backlogged stream, e.g. a .bin replay or a
    # camera burst): youth_icp_track_set_batch(m) -> one cooperative launch
    # per m frames, each pair on the single-pair plan of that mode (the
    # fewest source pixels per lane whose m grids fit the chip), two
    # submissions in flight; per m, the poses must equal track_frame's in the
    # same plan bit for bit
    by_size, equal, launches, diff_vs_default = {}, True, {}, 0.0
    best_m, Tb_best, sync_by_m = None, None, {}
    for m in sorted({2, youth_icp.TRACK_MAX_BATCH // 2, youth_icp.TRACK_MAX_BATCH}):
        ctx2 = youth_icp.IcpContext(a.width, a.height, 2 * m, iters=a.iters)
        ctx2.track_set_batch(m)
        ctx2.track_host_sequence(frames[: 2 * m + 1])  # warm
        r_b = []
        for _ in range(passes):
            ctx2.track_reset()
            t0 = time.perf_counter()
            Tb, _ = ctx2.track_host_sequence(frames)
            r_b.append(n / (time.perf_counter() - t0))
        launches[m] = ctx2.track_chained()
        ctx2.track_reset()
        sync_b = [T for T, _, has in (ctx2.track_frame(f) for f in frames) if has]
        plan_b = ctx2.get_plan()
        ctx2.close()
        sync_by_m[m] = np.stack(sync_b)
        equal &= bool(np.array_equal(Tb, np.stack(sync_b)))
        diff_vs_default = max(diff_vs_default, pose_err(Tb, np.stack(sync)))
        by_size[m] = {"value": float(np.median(r_b)), "pass_values": r_b,
                      "px_per_lane": plan_b.get("px_per_lane"),
                      "workgroups_per_pair": plan_b.get("workgroups_per_pair")}
        if best_m is None or by_size[m]["value"] > by_size[best_m]["value"]:
            best_m, Tb_best = m, Tb
    v1, vp, vs = float(np.median(r_c)), float(np.median(r_py)), float(np.median(r_sync))
    vb = by_size[best_m]["value"]
    slam = slam_api_rate(a, frames, sync_by_m.get(youth_icp.TRACK_MAX_BATCH), passes=passes)
    slam["c_producer"] = slam_rate_c(a, n, passes)
    return {"frames": n, "value": max(v1, vb), "unit": "frames/s", "slam_api": slam,
            "us_per_frame": 1e6 / max(v1, vb),
            "mode": f"micro-batches of {best_m} frames" if vb >= v1 else "one launch per frame",
            "batched_value": vb, "batched_frames_per_launch": best_m,
            "batched_pass_values": by_size[best_m]["pass_values"],
            "batched_by_size": {str(k): v for k, v in by_size.items()},
            "per_frame_value": v1, "per_frame_us": 1e6 / v1,
            "python_pipelined_value": vp, "sync_value": vs, "sync_us_per_frame": 1e6 / vs,
            "passes": passes, "pass_values": r_c, "kernel_path": plan,
            "max_abs_diff_vs_batch_poses": pose_err(Tc, rel_batch[: n - 1]),
            "pipelined_equals_sync": bool(np.array_equal(np.stack(rel), np.stack(sync))
                                          and np.array_equal(Tc, np.stack(sync))),
            "batched_equals_sync": equal,
            "batched_launches": {str(k): v for k, v in launches.items()},
            "batched_max_abs_diff_vs_per_frame_plan": diff_vs_default,
            "batched_best_max_abs_diff_vs_batch_poses": pose_err(Tb_best, rel_batch[: n - 1]),
            "in_flight": 2, "batched_in_flight": "two micro-batches",
            "note": "host frames, copy to pinned + H2D + align + pose to pinned per frame; value: "
                    "the faster of youth_icp_track_host_sequence with one launch per frame (two "
                    "in flight: per_frame_value) and with micro-batches of m frames per launch "
                    "(batched_by_size; batched_value = the best m); every mode's poses equal "
                    "track_frame's in its plan bit for bit (batched_equals_sync); "
                    "python_pipelined_value: track_submit/collect from Python, one launch per "
                    "frame; sync_value: track_frame"}


def slam_api_rate(a, frames, rel_plan, passes=5):
    """The drop-in path itself (SLAM.cpp:126-175 / :32-63 semantics):
    processSlamFrame from one producer thread into the module's ingest queue,
    the module's worker tracking in micro-batches (its default: as many
    queued frames as YOUTH_TRACK_MAX_BATCH per launch, page-locked queue
    buffers submitted in place).  Backlogged: the producer pushes as fast as
    it can but never past the reference's drop threshold (it waits while 10
    frames are queued, so nothing is dropped); timed until the last frame's
    pose is in the trajectory (median of `passes`).  Live: one frame at a
    time, each waited for (the per-frame latency a camera at 30 fps sees).
    World poses checked against the prefix product of track_frame's relative
    poses on a context with the worker's plan (rel_plan: same frames,
    youth_icp_track_set_batch(YOUTH_TRACK_MAX_BATCH)), and the micro-batch
    count (youth_slam_batched_frames)."""
    lib = youth_icp.load_library()
    n = frames.shape[0]
    fr = np.ascontiguousarray(frames, np.int16)
    ptrs = [fr[f].ctypes.data_as(ctypes.POINTER(ctypes.c_int16)) for f in range(n)]
    H, W = fr.shape[1:]
    youth_icp.initSlamModule(None)
    out = {"frames": n, "producer": "one Python thread, ctypes processSlamFrame",
           "worker_batch": os.environ.get("YOUTH_SLAM_TRACK_BATCH",
                                          str(youth_icp.TRACK_MAX_BATCH))}
    try:
        # warm: context, plan, page-locked pool, then one untimed backlogged
        # pass (the first timed pass otherwise ran 5-15 % below the rest:
        # profiles/r06/c2_base_vs_two_level_build_and_push_copy_ab_r6d.txt)
        for f in range(min(n, 24)):
            lib.processSlamFrame(ptrs[f], None, W, H, f)
        youth_icp.slam_wait_idle(20000)
        youth_icp.resetSlam()
        youth_icp.slam_wait_idle(20000)
        for f in range(n):
            while lib.youth_slam_queue_size() >= 10:
                pass
            lib.processSlamFrame(ptrs[f], None, W, H, f)
        youth_icp.slam_wait_idle(20000)
        rates, batched, push_us = [], [], []
        push, qsize, tlen, clock = lib.processSlamFrame, lib.youth_slam_queue_size, \
            lib.youth_slam_trajectory_length, time.perf_counter
        for _ in range(passes):
            youth_icp.resetSlam()
            youth_icp.slam_wait_idle(20000)
            b0 = youth_icp.slam_batched_frames()
            in_push = 0.0
            t0 = clock()
            for f in range(n):
                while qsize() >= 10:
                    pass
                tp = clock()
                push(ptrs[f], None, W, H, f)
                in_push += clock() - tp
            while tlen() < n:
                pass
            rates.append(n / (clock() - t0))
            batched.append(youth_icp.slam_batched_frames() - b0)
            push_us.append(in_push * 1e6 / n)
        ts, T = youth_icp.slam_trajectory()
        out.update({"value": float(np.median(rates)), "unit": "frames/s",
                    "pass_values": rates, "batched_frames_per_pass": batched,
                    # the producer's time inside processSlamFrame (its copy into a
                    # page-locked queue buffer), per frame and pass
                    "push_us_per_frame": push_us,
                    "frames_recorded": int(len(ts)), "timestamps_in_order":
                    bool(np.array_equal(ts, np.arange(n, dtype=np.uint32)))})
        if rel_plan is not None:
            acc = np.eye(4)
            err = 0.0
            for k in range(1, min(len(T), rel_plan.shape[0] + 1)):
                acc = acc @ rel_plan[k - 1]
                err = max(err, pose_err(T[k], acc))
            out["world_pose_max_abs_diff_vs_track_frame_plan"] = err
        youth_icp.resetSlam()
        youth_icp.slam_wait_idle(20000)
        lat = []
        for f in range(min(n, 60)):
            t0 = time.perf_counter()
            lib.processSlamFrame(ptrs[f], None, W, H, f)
            while lib.youth_slam_trajectory_length() < f + 1:
                pass
            lat.append((time.perf_counter() - t0) * 1e6)
        out["live_latency_us_median"] = float(np.median(lat[1:]))
        out["live_latency_us_p90"] = float(np.percentile(lat[1:], 90))
    finally:
        youth_icp.stopSlamModule()
    return out


def slam_rate_c(a, n, passes):
    """The same backlogged / live processSlamFrame runs from a plain-C
    producer thread (examples/slam_rate.c, its own process): the drop-in's
    rate without Python in the producer."""
    import subprocess
    exe = os.path.join(ROOT, "slam-rgbd_amd", "slam_rate")
    if not os.path.exists(exe):
        return {"error": "slam_rate not built"}
    r = subprocess.run([exe, str(n), str(passes), str(a.width), str(a.height)],
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        return {"error": f"rc {r.returncode}", "stderr_tail": r.stderr[-400:]}
    return json.loads(r.stdout.strip().splitlines()[-1])


def survey_noise_parity(a, ctx, main, n=128):
    """Parity on SURVEY §8d's noise level (sigma = 1.5 mm Z^2; the bench's
    default synthetic pairs use 0.25 mm Z^2): n pairs through the
    same context (one launch) vs the C oracle in the exact reduction."""
    oracle = oracle_mod()
    src, dst, _ = youth_synth.pairs(0, n, a.width, a.height, flags=youth_synth.SURVEY_FLAGS)
    ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
    own = ctx.max_frames < n            # a small --global-pairs run: a context of n pairs
    if own:
        ctx = youth_icp.IcpContext(a.width, a.height, n, iters=a.iters)
    ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n, stream=main.cuda_stream)
    T, _, st = ctx.get_poses(n)
    if own:
        ctx.close()
    T_cpu, st_cpu = oracle.align_batch(src, dst, iters=a.iters, n_threads=min(n, _cpus()))
    err = np.abs(np.asarray(T)[:, :3, :] - np.asarray(T_cpu)[:, :3, :]).reshape(n, -1).max(1)
    return {"pairs": n, "noise": "sigma = 1.5 mm * Z^2", "pose_max_abs_err_vs_cpu":
            float(err.max()), "pairs_over_tol": int((err > POSE_TOL).sum()),
            "status_gpu_nonzero": int((st != 0).sum()),
            "status_cpu_nonzero": int((st_cpu != 0).sum())}


def viewer_cloud_rate(R, d_depth, depth_host, reps=20, warmup=3):
    """the viewer's vertex list (viewerModule.c:336-357) for n
    frames in one device call (youth_cloud_build_device: count, scan, emit),
    synthetic RGB, inputs resident in HBM; HIP events on the launching
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
        oracle = oracle_mod()
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

    elapsed, kt, spread = R.timed(ctx, step)
    result = base_result(R, (F - 1) * a.steps / elapsed, elapsed)
    result["scaling"] = "strong"
    result["config"] = {
        "workload": f"C5: {F}-frame synthetic sequence, {W}x{H}, streamed frame-to-frame "
                    f"odometry, {a.iters} iters, {F - 1} pairs split over ranks (1-frame halo)",
        "frames": F, "pairs": F - 1, "width": W, "height": H, "iters": a.iters,
        "parallelism": f"dp{world} (contiguous pair ranges, RCCL pose gather)",
    }
    result["window_rates"] = [(F - 1) * a.steps / s for s in spread]
    result["roofline"] = roofline_icp(a, kt, max(npairs, 1), W, H)
    g_ms = None
    if R.dist_on:
        ts = []
        for _ in range(5):
            R.barrier_sync()
            t0 = time.perf_counter()
            youth_dist.gather_ragged(rel[:npairs], world, max_rows, counts)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        g_ms = float(np.median(ts))
    # every rank checks its first pair and its halo pair (the last, whose
    # source frame is the next shard's first) against the CPU oracle
    idx = sorted({0, npairs - 1}) if npairs else []
    T_rel = ctx.get_poses(npairs)[0] if npairs else None
    perr = shard_parity(a, frames[1:], frames[:-1], T_rel, idx)
    if a.dump_poses:
        np.save(f"{a.dump_poses}.rank{rank}.npy",
                np.asarray(T_rel if npairs else np.zeros((0, 4, 4)), np.float64).reshape(-1, 4, 4))
    result["ranks"] = youth_dist.rank_report({
        "k_icp_ms": kt["k_icp"][0] / max(kt["k_icp"][1], 1),
        "k_prep_ms": kt["k_prep"][0] / max(kt["prep_pass_steps"], 1),
        "gather_ms": g_ms if g_ms is not None else 0.0}, world,
        {"pose_max_abs_err_vs_cpu": perr, "pairs_checked": len(idx)})
    result["ranks"]["gather_timed"] = g_ms is not None
    result["ranks"]["parity_sample"] = "each rank: its first pair and its halo pair vs the C oracle"
    parity_gate(result)
    if rank == 0:
        T = youth_dist.compose_trajectory(traj["T"].cpu().numpy().reshape(-1, 4, 4))
        result["trajectory_frames"] = int(T.shape[0])
        if a.dump_poses:
            np.save(f"{a.dump_poses}.traj.npy", np.asarray(T, np.float64))
    ctx.close()
    return result


def base_result(R, value, elapsed):
    a = R.a
    return {
        "metric": METRIC,
        "value": value,
        "unit": "aligns/s",
        "n_gpus": R.world,
        "steps": a.steps,
        "warmup": a.warmup,
        "warmup_steps_run": getattr(R, "warmup_steps_run", a.warmup),
        "min_warmup_ms": a.min_warmup_ms,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "fp32",
        "spec": {"name": a.spec,
                 "a7_a8": ("SURVEY.md §8a as worded: no FMA, IEEE division fx P'x / P'z"
                           if a.spec == "survey" else
                           "fma chains, one correctly rounded reciprocal (opt-in)"),
                 "a9_reduce": a.reduce,
                 "a9": ("every product exact in fp64, fp64 sums (launch-independent; the default)"
                        if a.reduce == "exact" else
                        "fp32 lane sums (one fma each), fp64 finalize (opt-in; depends on the "
                        "launch's lane partition)")},
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


def _cpus():
    return len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else \
        (os.cpu_count() or 1)


def cpu_baseline(a, src, dst, T_gpu):
    """The C oracle on the host cores of the GPU box over a bounded sample of
    the same pairs: one warm-up, then the median of >= 3 timed
    passes, OpenMP over pairs (i) on the box's CPU share (OMP_NUM_THREADS, 16
    on the GPU pool) and (ii) on min(pairs, visible CPUs) threads; the faster
    is the reported value.  Plus (iii) one thread on a 2-pair sample, and the
    SE(3) error of the GPU poses on every sampled pair."""
    oracle = oracle_mod()

    cpus = _cpus()
    S = src.shape[0]
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, cpus)
    legs = {}
    T_cpu = st = None
    for tag, threads in (("share", min(share, S, cpus)), ("all", min(S, cpus))):
        if tag == "all" and threads == legs["share"]["cores"]:
            legs["all"] = dict(legs["share"])
            continue
        oracle.align_batch(src[:threads], dst[:threads], iters=a.iters, n_threads=threads)
        rates = []
        while len(rates) < 3 or (sum(S / r for r in rates) < 3.0 and len(rates) < 20):
            t0 = time.perf_counter()
            T_cpu, st = oracle.align_batch(src, dst, iters=a.iters, n_threads=threads)
            rates.append(S / (time.perf_counter() - t0))
        legs[tag] = {"value": float(np.median(rates)), "cores": threads, "passes": len(rates)}
    single = []
    oracle.align_batch(src[:1], dst[:1], iters=a.iters, n_threads=1)  # warm
    for _ in range(3):
        t0 = time.perf_counter()
        oracle.align_batch(src[:2], dst[:2], iters=a.iters, n_threads=1)
        single.append(2 / (time.perf_counter() - t0))
    best = max(legs.values(), key=lambda v: v["value"])
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            model = next((ln.split(":", 1)[1].strip() for ln in f if ln.startswith("model name")),
                         "")
    except OSError:
        pass
    cpu = {"value": best["value"], "unit": "aligns/s", "cores": best["cores"], "kind": "port",
           "sample": f"median of >= 3 passes over {S} of the rank-0 pairs ({a.width}x{a.height}, "
                     f"{a.iters} iters) after 1 warm-up: C oracle -O3 -ffp-contract=off, OpenMP "
                     f"over pairs; faster of the CPU-share and all-visible-CPU thread counts",
           "threads_share": legs["share"], "threads_all": legs["all"],
           "single_thread": {"value": float(np.median(single)), "unit": "aligns/s", "cores": 1,
                             "sample": "median of 3 passes over 2 pairs"},
           "host": {"cpu_model": model, "cpus_visible": cpus,
                    "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}}
    parity = {"pose_max_abs_err_vs_cpu": pose_err(T_gpu, T_cpu), "pairs_checked": S,
              "tolerance": POSE_TOL, "cpu_status_nonzero": int((st != 0).sum())}
    return cpu, parity


def legs_summary(result):
    """Every leg's headline in one compact object, emitted as the LAST key of
    the bench line, so the driver's truncated stdout tail still carries them
    (VERDICT r5 item 3).  Values are copied from the full legs above it."""
    def get(*path):
        x = result
        for k in path:
            if not isinstance(x, dict) or k not in x:
                return None
            x = x[k]
        return x

    def r(v, nd=4):
        return None if v is None else float(f"{v:.{nd}g}")

    sa = get("c5", "streamed", "slam_api")
    legs = {
        "c4": {"value": r(get("value")), "frac": r(get("roofline", "frac"), 3)},
        "c2": {"value": r(get("c2", "value")), "us": r(get("c2", "us_per_align"), 3),
               "frac": r(get("c2", "roofline", "frac"), 3)},
        "c3_single": {"value": r(get("c3", "single_pair", "value")),
                      "frac": r(get("c3", "single_pair", "roofline", "frac"), 3)},
        "c3_batch": {"value": r(get("c3", "batch", "value")),
                     "frac": r(get("c3", "batch", "roofline", "frac"), 3)},
        "c5_batch": r(get("c5", "batch", "value")),
        "c5_streamed": r(get("c5", "streamed", "value")),
        "slam_api_py": r(get("c5", "streamed", "slam_api", "value")),
        "slam_api_py_push_us": (None if not sa or "push_us_per_frame" not in sa else
                                r(float(np.median(sa["push_us_per_frame"])), 3)),
        "slam_api_c": r(get("c5", "streamed", "slam_api", "c_producer", "value")),
        "slam_api_c_push_us": (None if not sa or "c_producer" not in sa or
                               "push_us_per_frame" not in sa["c_producer"] else
                               r(float(np.median(sa["c_producer"]["push_us_per_frame"])), 3)),
        "spec_parity_max_vs_survey_oracle": r(get("spec_parity", "max_vs_survey_oracle",
                                                  get("spec_parity", "default_variant") or "survey"), 3),
        "parity_max_vs_cpu": r(get("parity", "pose_max_abs_err_vs_cpu"), 3),
    }
    if get("c2", "roofline", "frac") is None:
        legs["c2"].pop("frac")
    return legs


def main():
    a = parse()
    os.environ["YOUTH_ICP_SPEC"] = a.spec   # every context of this run (youth_icp_create)
    os.environ["YOUTH_ICP_REDUCE"] = a.reduce
    R = Run(a)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))   # the checker (legs after timing)
    # a non-default torch stream: its handle is what every align is issued on,
    # so the pose copies and the RCCL gathers (which wait on torch's current
    # stream) are ordered after the kernels that write the poses
    with torch.cuda.stream(torch.cuda.Stream()):
        result = run_pairs(R) if a.workload == "pairs" else run_sequence(R)
    if R.rank == 0:
        result["legs"] = legs_summary(result)   # last key: survives a truncated tail
        print(json.dumps(result), flush=True)
    R.finish()
    if R.rank == 0 and not result.get("parity_all_ranks_ok", True):
        sys.stderr.write("bench.py: a rank's poses are more than %g from the CPU oracle: %s\n"
                         % (POSE_TOL, result["ranks"].get("per_rank")))
        sys.exit(3)


if __name__ == "__main__":
    main()
