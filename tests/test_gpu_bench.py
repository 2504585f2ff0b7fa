"""bench.py's output contract on the GPU: the one JSON line with the metric,
roofline and cpu_baseline objects (N=1), and the N>1 flow (sharding, pose
gather, max-over-ranks timing) rehearsed with 2 ranks on one GPU over gloo
(RCCL needs one device per rank; the driver's 8-GPU run uses it)."""
import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


def _assert_rank_parity(d, world, per_rank):
    """every rank checked `per_rank` pairs of its own
    shard against the CPU oracle after the timed region, each within 1e-5,
    and the line says so (rank 0 exits non-zero otherwise)."""
    pr = d["ranks"]["per_rank"]
    assert pr["pairs_checked"] == [float(per_rank)] * world
    assert len(pr["pose_max_abs_err_vs_cpu"]) == world
    assert max(pr["pose_max_abs_err_vs_cpu"]) <= 1e-5
    assert d["parity_all_ranks_ok"] is True


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_single_gpu_contract():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1",
                        "--global-pairs", "64", "--windows", "1", "--c3-pairs", "2",
                        "--c5-frames", "41"], cwd=ROOT, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["value"] > 0 and d["scaling"] == "strong"
    assert d["higher_is_better"] is True and d["unit"] == "aligns/s"
    assert d["config"]["workload"].startswith("C4") and d["config"]["global_pairs"] == 64
    assert len(d["window_rates"]) == 1 and d["status_nonzero"] == 0
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "survey_model"):
        assert k in rf, k
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and 0 < rf["frac"] < 1.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    assert rf["iterations_per_launch"] == 10
    rp = d["roofline_prep"]
    assert rp["kernel"] == "k_prep" and 0 < rp["frac"] < 1.0
    if rp.get("traffic_source", "").startswith("profiles/"):    # PMC pass of this source
        assert 1.0 <= rp["traffic_over_algorithmic"] < 1.5
        wc = rp["write_stream_ceiling"]               # 16 of its 18 B/px are writes
        assert wc["unit"] == "GB/s" and 0 < wc["traffic_frac"] < 1.2
        if "valu_issue_frac" in rp:                   # reported, not the limiter evidence
            assert 0 < rp["valu_issue_frac"] < 1.5
    if str(rf.get("traffic_source", "")).startswith("profiles/"):
        assert 1.0 <= rf["traffic_over_algorithmic"] < 1.1
        rc = rf["read_stream_ceiling"]                # k_icp's bytes are reads
        assert rc["unit"] == "GB/s" and 0 < rc["traffic_frac"] < 1.2
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample", "threads_share", "threads_all"):
        assert k in cb, k
    assert cb["kind"] == "port" and cb["value"] > 0
    assert d["parity"]["pose_max_abs_err_vs_cpu"] <= 1e-5
    sn = d["parity"]["survey_noise"]                 # SURVEY §8d noise, >= 128 pairs
    assert sn["pairs"] >= 128 and sn["pose_max_abs_err_vs_cpu"] <= 1e-5
    assert sn["pairs_over_tol"] == 0 and sn["status_gpu_nonzero"] == sn["status_cpu_nonzero"] == 0
    c2 = d["c2"]                            # one pair per call, small-batch kernel
    assert c2["value"] > 0 and c2["status"] == 0 and c2["pose_max_abs_err_vs_cpu"] <= 1e-5
    assert c2["kernel_path"]["kernel"] == "k_icp_coop"
    assert d["c3"]["parity_ok"] and d["c3"]["batch"]["pairs_per_call"] == 2
    for tag in ("single_pair", "batch"):
        rf3 = d["c3"][tag]["roofline"]
        assert rf3["unit"] == "GB/s" and 0 < rf3["frac"] < 1.0 and rf3["launches"] > 0
    assert d["c5"]["parity_ok"] and d["c5"]["batch"]["trajectory_frames"] == 41
    assert d["c5"]["streamed"]["max_abs_diff_vs_batch_poses"] <= 1e-5
    assert d["c5"]["streamed"]["pipelined_equals_sync"]
    assert d["c5"]["streamed"]["batched_equals_sync"]
    bs = d["c5"]["streamed"]["batched_by_size"]      # micro-batches of 2, 4 and 8 frames
    assert set(bs) == {"2", "4", "8"} and all(v["value"] > 0 for v in bs.values())
    assert all(v > 0 for v in d["c5"]["streamed"]["batched_launches"].values())
    assert d["kernel_path"]["kernel"].startswith("k_prep + k_icp")
    assert d["viewer_cloud"]["bit_exact_vs_cpu"]
    # spec a7/a8: the default is SURVEY §8a as worded; a9: exact fp64
    # products (launch-independent).  Every arithmetic x reduction against the
    # oracle in the same variant (lane32 over the launch's own lane partition:
    # ~1e-13); the default against the survey-spec exact oracle (<= 1e-5)
    assert d["spec"]["name"] == "survey" and d["spec"]["a9_reduce"] == "exact"
    sp = d["spec_parity"]
    assert sp["default_variant"] == "survey"
    for case in ("c2_64_pairs", "c3_2_pairs_1280x960_20it", "c5_200_pairs",
                 "survey_noise_16_pairs"):
        for v in ("survey", "fma", "survey_lane32", "fma_lane32"):
            assert sp[case][f"gpu_{v}_vs_same_variant_oracle"] <= 1e-9, (case, v)
        assert sp[case]["gpu_survey_vs_survey_oracle"] <= 1e-5, case
    assert sp["default_within_tol_of_survey_spec"]
    assert sp["other_spec_rate"]["spec"] == "fma" and sp["other_spec_rate"]["value"] > 0
    assert sp["other_reduce_rate"]["reduce"] == "lane32" and sp["other_reduce_rate"]["value"] > 0
    sa = d["c5"]["streamed"]["slam_api"]          # processSlamFrame, worker micro-batches
    assert sa["value"] > 0 and sa["frames_recorded"] == sa["frames"] and sa["timestamps_in_order"]
    assert sa["world_pose_max_abs_diff_vs_track_frame_plan"] <= 1e-12
    assert sum(sa["batched_frames_per_pass"]) > 0
    sc = sa["c_producer"]                         # the same from a plain-C producer
    assert sc["value"] > 0 and sc["frames_recorded"] == sa["frames"] and sc["batched_frames"] > 0
    assert d["ranks"]["rccl_world_size"] == 1 and d["ranks"]["per_rank_ms"]["k_icp_ms"][0] > 0
    _assert_rank_parity(d, 1, 4)


@pytest.mark.parametrize("workload", ["pairs", "sequence"])
def test_bench_two_ranks_rehearsal(workload):
    env = dict(os.environ, YOUTH_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus",
           "2", "--steps", "3", "--warmup", "1", "--windows", "1", "--workload", workload,
           "--global-pairs", "128"]
    if workload == "sequence":
        cmd += ["--frames", "41"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["value"] > 0
    if workload == "pairs":
        assert d["scaling"] == "strong" and d["config"]["global_pairs"] == 128
        assert d["config"]["pairs_per_gpu"] == 64
    else:
        assert d["scaling"] == "strong" and d["config"]["pairs"] == 40
    assert "cpu_baseline" not in d          # rank 0 at N=1 only
    rk = d["ranks"]                         # the N > 1 line's self-report
    assert rk["rccl_world_size"] == 2 and rk["backend"] == "gloo" and rk["gather_timed"]
    for k in ("k_icp_ms", "k_prep_ms", "gather_ms"):
        assert len(rk["per_rank_ms"][k]) == 2, k
    assert min(rk["per_rank_ms"]["k_icp_ms"]) > 0
    _assert_rank_parity(d, 2, 4 if workload == "pairs" else 2)


@pytest.mark.parametrize("workload", ["pairs", "sequence"])
def test_bench_three_ranks_uneven_shards(workload):
    """Three ranks over gloo on one GPU with shards that do not divide evenly
    (100 pairs: 34 + 33 + 33; a 61-frame sequence: 60 pairs, 20 per rank with
    a 1-frame halo): the line's shape, every rank's timings, and bench.py's
    own check that the gathered poses equal each rank's (it raises
    otherwise).  Shards stay above 16 pairs, so no rank launches the
    cooperative kernel (its grids assume one process per GPU)."""
    env = dict(os.environ, YOUTH_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus",
           "3", "--steps", "3", "--warmup", "1", "--windows", "1", "--workload", workload,
           "--global-pairs", "100", "--frames", "61"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 3 and d["value"] > 0 and d["scaling"] == "strong"
    if workload == "pairs":
        assert d["config"]["global_pairs"] == 100
    else:
        assert d["config"]["pairs"] == 60
    rk = d["ranks"]
    assert rk["rccl_world_size"] == 3 and rk["backend"] == "gloo"
    for k in ("k_icp_ms", "k_prep_ms", "gather_ms"):
        assert len(rk["per_rank_ms"][k]) == 3, k
    assert min(rk["per_rank_ms"]["k_icp_ms"]) > 0
    _assert_rank_parity(d, 3, 4 if workload == "pairs" else 2)


@pytest.mark.parametrize("workload", ["pairs", "sequence"])
def test_bench_rccl_gather_one_gpu(workload):
    """The RCCL path itself on hardware: one rank with the process group up
    (YOUTH_BENCH_DIST=1, backend nccl = RCCL): init_process_group(device_id=),
    all_gather_into_tensor(async_op=True) + handle.wait() on the side stream,
    the ragged sequence gather, max-over-ranks timing.  bench.py raises if the
    gathered / host rows differ from the rank's poses."""
    env = dict(os.environ, YOUTH_BENCH_DIST="1")
    env.pop("YOUTH_BENCH_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus",
           "1", "--steps", "3", "--warmup", "1", "--windows", "1", "--workload", workload,
           "--global-pairs", "32", "--frames", "21", "--no-legs", "--no-cpu-baseline",
           "--no-host-io", "--no-viewer"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert d["ranks"]["rccl_world_size"] == 1 and d["ranks"]["backend"] == "nccl"
    assert d["ranks"]["gather_timed"] and d["ranks"]["per_rank_ms"]["gather_ms"][0] > 0


def test_bench_gpus_flag_self_launches_ranks():
    """`python bench.py --gpus 2` with no launcher (the driver's form) starts
    two ranks itself; gloo, so both fit on one GPU."""
    env = dict(os.environ, YOUTH_BENCH_BACKEND="gloo")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--steps", "3", "--warmup",
                        "1", "--windows", "1", "--global-pairs", "64"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["ranks"]["rccl_world_size"] == 2 and d["ranks"]["backend"] == "gloo"
    assert d["config"]["pairs_per_gpu"] == 32
    _assert_rank_parity(d, 2, 4)


@pytest.mark.parametrize("workload", ["pairs", "sequence"])
def test_bench_eight_ranks_rehearsal(workload, tmp_path):
    """The driver's N = 8 run, rehearsed on one GPU:
    `python bench.py --gpus 8` self-launches 8 ranks (gloo, so all of them
    share the one device) on the real shard geometry: pairs with
    --global-pairs 136 (17 per rank: the persistent path), and the C5
    sequence with --frames 1000 (ranges of 125/124 pairs with a 1-frame
    halo).  Every rank reports, every rank's parity sample passes, and the
    poses the 8 ranks computed (fp64, dumped per rank) equal the N = 1 run's
    within 1e-9 (the shards' launch shapes change only fp64 summation
    order); for the sequence, rank 0's gathered and composed 1000-frame
    trajectory too."""
    import time

    import numpy as np
    env = dict(os.environ, YOUTH_BENCH_BACKEND="gloo", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    common = ["--steps", "3", "--warmup", "1", "--windows", "1", "--workload", workload,
              "--global-pairs", "136", "--frames", "1000", "--min-warmup-ms", "0"]
    solo = ["--no-legs", "--no-cpu-baseline", "--no-host-io", "--no-viewer", "--no-spec-parity"]
    p8, p1 = str(tmp_path / "n8"), str(tmp_path / "n1")
    t0 = time.perf_counter()
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "8", "--dump-poses", p8] + common,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    wall8 = time.perf_counter() - t0
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    print(f"\n8-rank {workload} rehearsal: wall {wall8:.1f} s, value {d['value']:.0f} aligns/s")
    assert d["n_gpus"] == 8 and d["value"] > 0 and d["scaling"] == "strong"
    rk = d["ranks"]
    assert rk["rccl_world_size"] == 8 and rk["backend"] == "gloo" and rk["gather_timed"]
    for k in ("k_icp_ms", "k_prep_ms", "gather_ms"):
        assert len(rk["per_rank_ms"][k]) == 8, k
    assert min(rk["per_rank_ms"]["k_icp_ms"]) > 0
    _assert_rank_parity(d, 8, 4 if workload == "pairs" else 2)
    if workload == "pairs":
        assert d["config"]["global_pairs"] == 136 and d["config"]["pairs_per_gpu"] == 17
    else:
        assert d["config"]["pairs"] == 999 and d["trajectory_frames"] == 1000
    env1 = dict(env, OMP_NUM_THREADS="16")
    r1 = subprocess.run([sys.executable, "bench.py", "--dump-poses", p1] + common + solo,
                        cwd=ROOT, env=env1, capture_output=True, text=True, timeout=900)
    assert r1.returncode == 0, r1.stderr[-3000:]
    T8 = np.concatenate([np.load(f"{p8}.rank{k}.npy") for k in range(8)])
    T1 = np.load(f"{p1}.rank0.npy")
    want = 136 if workload == "pairs" else 999
    assert T8.shape == T1.shape == (want, 4, 4)
    err = float(np.abs(T8[:, :3, :] - T1[:, :3, :]).max())
    assert err <= 1e-9, err
    if workload == "sequence":
        # rank 0's trajectory from the gathered fp32 relative poses against the
        # N = 1 run's (each fp32 pose may round differently: a few 1e-8)
        tr8, tr1 = np.load(f"{p8}.traj.npy"), np.load(f"{p1}.traj.npy")
        assert tr8.shape == tr1.shape == (1000, 4, 4)
        assert float(np.abs(tr8[:, :3, :] - tr1[:, :3, :]).max()) <= 1e-5
