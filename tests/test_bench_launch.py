"""bench.py's `--gpus N` contract on CPU: without a
launcher, N > 1 starts torch.distributed.run with N ranks as a child process;
under a launcher, --gpus must equal WORLD_SIZE.  No GPU and no rank is
started here: the launcher command is captured, and the argument check runs
before bench.py imports torch."""
import importlib.util
import os
import subprocess
import sys

from conftest import ROOT


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_gpus_n_starts_n_ranks():
    b = _bench()
    seen = {}

    def run(cmd, env):
        seen["cmd"], seen["env"] = cmd, env
        return 7

    rc = b._launch_ranks(["--gpus", "8", "--steps", "5", "--warmup", "2"], {}, run)
    assert rc == 7                                  # the child's exit code is bench.py's
    cmd = seen["cmd"]
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-7:] == [os.path.join(ROOT, "bench.py"), "--gpus", "8", "--steps", "5",
                        "--warmup", "2"]
    assert seen["env"]["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_single_rank_and_launcher_cases():
    b = _bench()
    never = lambda cmd, env: (_ for _ in ()).throw(AssertionError("launched"))  # noqa: E731
    assert b._launch_ranks([], {}, never) is None                  # default N = 1
    assert b._launch_ranks(["--gpus", "1"], {}, never) is None
    assert b._launch_ranks(["--gpus", "4"], {"WORLD_SIZE": "4"}, never) is None
    assert b._launch_ranks(["--gpus=2"], {"WORLD_SIZE": "2"}, never) is None
    assert b._launch_ranks(["--gpus", "8"], {"WORLD_SIZE": "1"}, never) == 2
    assert b._launch_ranks(["--gpus", "0"], {}, never) == 2


def test_mismatch_exits_before_torch():
    env = dict(os.environ, WORLD_SIZE="3")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE 3" in r.stderr


def test_rank_parity_sample_and_gate():
    """each rank's sample (first two and last two pairs of
    its shard) and the gate that makes rank 0 exit non-zero when any rank's
    sampled poses are more than 1e-5 from the CPU oracle."""
    b = _bench()
    assert b.parity_sample(64) == [0, 1, 62, 63]
    assert b.parity_sample(3) == [0, 1, 2] and b.parity_sample(1) == [0]
    assert b.parity_sample(0) == []
    ok = {"ranks": {"per_rank": {"pose_max_abs_err_vs_cpu": [2e-14, 9e-6]}}}
    assert b.parity_gate(ok) and ok["parity_all_ranks_ok"] is True
    bad = {"ranks": {"per_rank": {"pose_max_abs_err_vs_cpu": [2e-14, 1.1e-5]}}}
    assert not b.parity_gate(bad) and bad["parity_all_ranks_ok"] is False
    assert not b.parity_gate({"ranks": {}})                 # nothing checked is not a pass
