"""Race detection for the host-side threading code (VERDICT r1
item 9): tests/tsan/driver.cpp drives the SLAM.h queue + worker
(slam_api.cpp), the AlgorithmModule frame loop and its POSIX-queue transport
(wire.c, algorithm_module.c) from many threads at once, built with
-fsanitize=thread and with -fsanitize=address,undefined.  The device
entry points the worker calls come from tests/tsan/icp_stub.c (a CPU
stand-in linked only into this driver), so it runs without a GPU.  Host code
only: GPU sanitizers are not available on the GPU pool.
"""
import fcntl
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
TSAN = os.path.join(HERE, "tsan")


@pytest.fixture(scope="module")
def drivers():
    # one build at a time (pytest-xdist workers share the object directories)
    with open(os.path.join(TSAN, ".build.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-C", TSAN, "-j2"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail("sanitizer build failed:\n" + r.stdout + r.stderr)
    return TSAN


TSAN_ENV = {"TSAN_OPTIONS": "halt_on_error=1 second_deadlock_stack=1"}
ASAN_ENV = {"ASAN_OPTIONS": "detect_leaks=1 abort_on_error=0",
            "UBSAN_OPTIONS": "halt_on_error=1 print_stacktrace=1"}
BATCH2 = {"YOUTH_SLAM_TRACK_BATCH": "2"}    # the worker's micro-batch modes
BATCH4 = {"YOUTH_SLAM_TRACK_BATCH": "4"}


@pytest.mark.parametrize("kind,env", [
    ("tsan", TSAN_ENV), ("asan", ASAN_ENV),
    ("tsan", {**TSAN_ENV, **BATCH4}), ("asan", {**ASAN_ENV, **BATCH2}),
], ids=["tsan", "asan", "tsan-batch", "asan-batch"])
def test_host_threading_under_sanitizer(drivers, kind, env):
    r = subprocess.run([os.path.join(drivers, "driver_" + kind)], capture_output=True, text=True,
                       timeout=300, env={**os.environ, **env})
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "all scenarios passed" in out
    for marker in ("ThreadSanitizer", "AddressSanitizer", "LeakSanitizer", "runtime error"):
        assert marker not in out, out[-4000:]


@pytest.mark.parametrize("kind,env", [("tsan", TSAN_ENV), ("asan", ASAN_ENV)], ids=["tsan", "asan"])
def test_staging_copy_pool_under_sanitizer(drivers, kind, env):
    """host_copy.h, the tracker's parallel staging copy (track_submit_batch /
    track_host_sequence): random jobs on 0-4 helpers checked byte for byte,
    pools driven from several threads, pools torn down idle and right after
    a job."""
    r = subprocess.run([os.path.join(drivers, "copy_pool_" + kind)], capture_output=True,
                       text=True, timeout=300, env={**os.environ, **env})
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "copy pool: all scenarios passed" in out
    for marker in ("ThreadSanitizer", "AddressSanitizer", "LeakSanitizer", "runtime error"):
        assert marker not in out, out[-4000:]
