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


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_single_gpu_contract():
    r = subprocess.run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1"], cwd=ROOT,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["value"] > 0 and d["scaling"] == "weak"
    assert d["higher_is_better"] is True and d["unit"] == "aligns/s"
    assert d["config"]["workload"].startswith("C4") and d["config"]["pairs_per_gpu"] == 64
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and 0 < rf["frac"] < 1.2
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["kind"] == "port" and cb["value"] > 0
    assert d["parity"]["pose_max_abs_err_vs_cpu"] <= 1e-5
    sp = d["single_pair"]                   # C2 leg: one pair per call, small-batch kernel
    assert sp["value"] > 0 and sp["status"] == 0 and sp["pose_max_abs_err_vs_cpu"] <= 1e-5
    assert sp["kernel_path"]["kernel"] == "k_icp_coop"
    assert d["kernel_path"]["kernel"].startswith("k_prep + k_icp")


@pytest.mark.parametrize("workload", ["pairs", "sequence"])
def test_bench_two_ranks_rehearsal(workload):
    env = dict(os.environ, YOUTH_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus",
           "2", "--steps", "3", "--warmup", "1", "--workload", workload]
    if workload == "sequence":
        cmd += ["--frames", "41"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["value"] > 0
    if workload == "pairs":
        assert d["scaling"] == "weak" and d["config"]["global_pairs"] == 128
    else:
        assert d["scaling"] == "strong" and d["config"]["pairs"] == 40
    assert "cpu_baseline" not in d          # rank 0 at N=1 only
