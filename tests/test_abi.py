"""CPU tests of the C-ABI boundary: the library loads, exports every function
include/*.h declares, and the host-only logic (queue policy, YAML intrinsics,
no-device behaviour, synthetic source) behaves as the reference's API says.
No compute calls here."""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

import youth_icp
import youth_synth
from conftest import GOLDEN, PKG, ROOT

HEADERS = {
    "youth_icp.h": os.path.join(PKG, "libyouth_icp.so"),
    "youth_wire.h": os.path.join(PKG, "libyouth_icp.so"),
    "youth_viewer.h": os.path.join(PKG, "libyouth_icp.so"),
    "youth_synth.h": os.path.join(PKG, "libyouth_synth.so"),
    "youth_dist.h": os.path.join(PKG, "libyouth_dist.so"),
}


def _exported(lib_path):
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], capture_output=True,
                         text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


@pytest.mark.parametrize("header", sorted(HEADERS))
def test_every_declared_symbol_is_exported(header):
    names = youth_icp.declared_functions(os.path.join(ROOT, "include", header))
    assert len(names) >= (35 if header == "youth_icp.h" else 4)
    exported = _exported(HEADERS[header])
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    lib = ctypes.CDLL(HEADERS[header])
    for n in names:
        getattr(lib, n)


def test_reference_api_names_present():
    """SLAM.h:11-38 + algorithmModule.h:6, exactly these names."""
    ref = ["initSlamModule", "stopSlamModule", "processSlamFrame", "saveSlamMap",
           "isSlamModuleRunning", "getSlamMapPoints", "resetSlam", "algorithmModule"]
    assert set(ref) <= _exported(HEADERS["youth_icp.h"])


def test_header_compiles_as_c99_and_cpp():
    src = ('#include "youth_icp.h"\n#include "youth_synth.h"\n#include "youth_wire.h"\n'
           'int main(void){return 0;}\n')
    inc = os.path.join(ROOT, "include")
    for cc, std in (("gcc", "-std=c99"), ("g++", "-std=c++11")):
        r = subprocess.run([cc, std, "-Wall", "-Werror", "-fsyntax-only", "-I", inc, "-x",
                            "c" if cc == "gcc" else "c++", "-"], input=src, text=True,
                           capture_output=True)
        assert r.returncode == 0, r.stderr


def test_default_intrinsics_follow_viewer_convention():
    K = youth_icp.default_intrinsics(640, 480)
    assert K.as_tuple() == (np.float32(570.3), np.float32(570.3), 320.0, 240.0, 1000.0)
    K = youth_icp.default_intrinsics(1281, 961)
    assert (K.cx, K.cy) == (640.0, 480.0)           # integer W/2 (viewerModule.c:344)
    P = youth_icp.default_params()
    assert P.iters == 10 and abs(P.dist_thresh - 0.1) < 1e-7


def test_no_device_fails_loudly(has_gpu):
    if has_gpu:
        pytest.skip("only meaningful without a GPU")
    assert youth_icp.device_count() == 0
    with pytest.raises(youth_icp.IcpError) as e:
        youth_icp.IcpContext(64, 48, 2)
    assert e.value.code == youth_icp.YOUTH_ENODEV
    src = np.ones((1, 48, 64), np.int16)
    with pytest.raises(youth_icp.IcpError):
        youth_icp.align_batch(src, src)
    with pytest.raises(youth_icp.IcpError) as e:
        youth_icp.align_batch_multi(src, src)
    assert e.value.code == youth_icp.YOUTH_ENODEV
    # SLAM.h API: the module refuses to start, so frames are rejected (return 0)
    youth_icp.initSlamModule(None)
    assert youth_icp.isSlamModuleRunning() == 0
    assert youth_icp.processSlamFrame(src[0], None, 64, 48, 0) == 0
    assert youth_icp.saveSlamMap("/tmp/youth_nomap") == 0
    assert youth_icp.getSlamMapPoints() == 0
    lib = youth_icp.load_library()
    assert lib.algorithmModule(None) is None     # returns instead of hanging
    # viewer point list (youth_viewer.h): no builder without a device
    import youth_viewer
    with pytest.raises(youth_icp.IcpError) as e:
        youth_viewer.CloudBuilder(64, 48)
    assert e.value.code == youth_icp.YOUTH_ENODEV


def test_shard_range_matches_bench_split():
    """youth_icp_shard_range (the multi-GPU host API's split) == the bench
    ranks' youth_dist.pair_range, and the shards tile [0, n) contiguously."""
    import youth_dist
    for n in (1, 2, 7, 64, 511, 512, 999):
        for k in (1, 2, 3, 4, 8):
            nxt = 0
            for r in range(k):
                f, c = youth_icp.shard_range(n, k, r)
                assert (f, c) == youth_dist.pair_range(n, k, r)
                assert f == nxt and c >= 0
                nxt = f + c
            assert nxt == n
    with pytest.raises(youth_icp.IcpError):
        youth_icp.shard_range(8, 0, 0)
    with pytest.raises(youth_icp.IcpError):
        youth_icp.shard_range(8, 2, 2)


def test_rccl_gather_row_mapping_and_no_device(has_gpu):
    """youth_dist.h (libyouth_dist.so, the multi-process RCCL pose gather):
    the row -> (rank, row-in-shard) mapping its compaction kernel applies
    inverts youth_icp_shard_range for every split; without a device the
    communicator is refused loudly."""
    import youth_dist
    for n in (1, 5, 8, 63, 64, 512, 999):
        for k in (1, 2, 3, 4, 7, 8):
            for r in range(n):
                q, i = youth_dist.row_source(n, k, r)
                f, c = youth_icp.shard_range(n, k, q)
                assert f + i == r and 0 <= i < c
    if not has_gpu:
        with pytest.raises(youth_icp.IcpError) as e:
            youth_dist.RcclPoseGather(1, 0, 0, bytes(youth_dist.DIST_ID_BYTES))
        assert e.value.code == youth_icp.YOUTH_ENODEV


def test_queue_overflow_policy_matches_reference():
    """SLAM.cpp:159-169: push, then if size > 10 drop oldest until size == 5."""
    q = youth_icp.FrameQueue(10, 5)
    frames = [np.full((4, 6), i, np.int16) for i in range(12)]
    dropped = [q.push(f, timestamp=100 + i) for i, f in enumerate(frames)]
    assert dropped[:10] == [0] * 10 and dropped[10] == 6 and dropped[11] == 0
    assert len(q) == 6
    out = [q.pop() for _ in range(6)]
    assert [ts for _, ts in out] == [106, 107, 108, 109, 110, 111]
    assert all((d == ts - 100).all() and d.shape == (4, 6) for d, ts in out)
    assert q.pop() is None and len(q) == 0
    q.push(frames[0])
    q.clear()
    assert len(q) == 0
    q.close()


def test_queue_copies_frames():
    q = youth_icp.FrameQueue()
    f = np.arange(12, dtype=np.int16).reshape(3, 4)
    q.push(f, 1)
    f[:] = -1                                   # caller reuses its buffer immediately
    d, ts = q.pop()
    assert (d == np.arange(12).reshape(3, 4)).all() and ts == 1


def test_ingest_trace_records_pushes_and_drops():
    """youth_slam_trace_*: the producer side of the ingest path traces every
    push (queue depth before, whether the buffer was pooled or new) and the
    >10 -> 5 drops, lock-free, on any queue; reading returns the count
    recorded; capacity 0 stops it."""
    youth_icp.slam_trace_enable(64)
    try:
        q = youth_icp.FrameQueue(10, 5)
        f = np.zeros((4, 6), np.int16)
        for i in range(11):
            q.push(f, i)
        q.pop()
        q.push(f, 11)                          # a buffer from the pool
        t, k, a = youth_icp.slam_trace_read()
        q.close()
    finally:
        youth_icp.slam_trace_enable(0)
    names = [youth_icp.SLAM_EVENTS[int(v)] for v in k]
    assert names.count("push_begin") == 12 and names.count("push_end") == 12
    assert names.count("drop") == 1 and a[names.index("drop")] == 6
    depth = [int(x) for x, n in zip(a, names) if n == "push_begin"]
    assert depth[:11] == list(range(11)) and depth[11] == 4
    kinds = [int(x) for x, n in zip(a, names) if n == "push_end"]
    assert kinds[0] == 2 and kinds[-1] == 0      # new pageable, then pooled
    assert (np.diff(t) >= 0).all()
    assert youth_icp.slam_trace_read()[0].size == 0


def test_parse_camera_yaml():
    K, W, H = youth_icp.parse_camera_yaml(os.path.join(GOLDEN, "astra_camera.yaml"))
    assert (K.fx, K.fy, K.cx, K.cy, K.depth_scale) == (np.float32(570.3), np.float32(570.3),
                                                       320.0, 240.0, 1000.0)
    assert (W, H) == (640, 480)
    assert youth_icp.parse_camera_yaml("/nonexistent.yaml") is None


def test_synth_deterministic_and_valid():
    a = youth_synth.pairs(0, 2, 160, 120)
    b = youth_synth.pairs(0, 2, 160, 120)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    src, dst, T = a
    valid = src[src > 0]
    assert 400 <= valid.min() and valid.max() <= 8000
    assert 0.95 < (src > 0).mean() < 0.995          # ~2 % holes
    R = T[:, :3, :3]
    assert np.allclose(R @ R.transpose(0, 2, 1), np.eye(3), atol=1e-12)
    ang = np.degrees(np.arccos(np.clip((np.trace(R, axis1=1, axis2=2) - 1) / 2, -1, 1)))
    assert (ang <= 1.5 + 1e-9).all() and (np.abs(T[:, :3, 3]) <= 0.015).all()
    g = np.load(os.path.join(GOLDEN, "pair_160x120.npz"), allow_pickle=False)
    K = youth_icp.Intrinsics(*[float(v) for v in g["K"]])
    s2, d2, _ = youth_synth.pairs(1, 1, 160, 120, K=K)
    assert np.array_equal(s2[0], g["src"]) and np.array_equal(d2[0], g["dst"])


def test_synth_sequence_shards_consistent():
    full, T = youth_synth.sequence(0, 6, 64, 48)
    part, T2 = youth_synth.sequence(3, 3, 64, 48)
    assert np.array_equal(full[3:], part) and np.array_equal(T[3:], T2)


def test_host_wrappers_reject_mismatched_shapes():
    """Shape checks run before any library call (no GPU needed): a frame stack
    whose src and dst differ, or that is not [n, H, W], is a ValueError, not an
    out-of-bounds read in the library."""
    a = np.zeros((2, 8, 8), np.int16)
    with pytest.raises(ValueError):
        youth_icp.align_batch(a, np.zeros((2, 8, 9), np.int16))
    with pytest.raises(ValueError):
        youth_icp.align_batch_multi(a, np.zeros((3, 8, 8), np.int16))
    with pytest.raises(ValueError):
        youth_icp.align_batch(np.zeros(64, np.int16), np.zeros(64, np.int16))


_NULL_SWEEP = r"""
import ctypes, re, sys
text = open(sys.argv[1]).read()
text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
text = re.sub(r"typedef[^;]*;", "", text)
lib = ctypes.CDLL(sys.argv[2])
for ret, name, args in re.findall(r"\n\s*([A-Za-z_][\w ]*?\**)\s*\b(youth_\w+)\(([^;{]*)\)\s*;", text):
    ret = ret.strip()
    args = " ".join(args.split())
    if not (args.startswith(("youth_icp_ctx*", "const youth_icp_ctx*", "youth_frame_queue*"))
            or name.startswith("youth_slam_")):
        continue
    n = 0 if args in ("", "void") else args.count(",") + 1
    f = getattr(lib, name)
    f.restype = (None if ret == "void" else ctypes.c_longlong if ret.startswith("long long")
                 else ctypes.c_void_p if ret.endswith("*") else ctypes.c_int)
    f.argtypes = [ctypes.c_void_p] * n
    print(name, ret, f(*([None] * n)), flush=True)
"""


def test_null_arguments_are_refused_not_dereferenced(tmp_path):
    """Every entry point that takes a context or a queue, and every
    youth_slam_* query, called with NULL / zero for all of its arguments (no
    module running): it returns an error or an empty answer, and nothing
    dereferences the NULL.  Calls run in a child process, so a crash fails the
    test instead of the test runner."""
    script = tmp_path / "sweep.py"
    script.write_text(_NULL_SWEEP)
    r = subprocess.run([sys.executable, str(script), os.path.join(ROOT, "include", "youth_icp.h"),
                        HEADERS["youth_icp.h"]], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = {}
    for line in r.stdout.splitlines():
        name, *_, val = line.split()
        res[name] = val
    assert len(res) >= 45, sorted(res)
    einval = str(youth_icp.YOUTH_EINVAL)
    must_fail = [n for n in res if n.startswith(("youth_icp_align", "youth_icp_track_submit",
                                                  "youth_icp_track_collect", "youth_icp_track_frame",
                                                  "youth_icp_track_realign", "youth_icp_get_",
                                                  "youth_icp_set_", "youth_icp_sync",
                                                  "youth_icp_track_host", "youth_queue_p"))
                 and n != "youth_icp_track_realigned"]
    assert len(must_fail) >= 20
    assert all(res[n] == einval for n in must_fail), {n: res[n] for n in must_fail}
    # counters and sizes of nothing are 0; void calls return
    for n in ("youth_icp_track_pending", "youth_icp_track_chained", "youth_icp_track_realigned",
              "youth_queue_size", "youth_slam_trajectory_length", "youth_slam_get_trajectory",
              "youth_slam_realigned", "youth_slam_queue_size"):
        assert res[n] == "0", (n, res[n])
    assert res["youth_icp_destroy"] == "None" and res["youth_slam_wait_stopped"] == "None"
    # the reference API with NULL buffers (SLAM.h: 0 = failure)
    lib = ctypes.CDLL(HEADERS["youth_icp.h"])
    lib.processSlamFrame.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_uint32]
    assert lib.processSlamFrame(None, None, 640, 480, 0) == 0
    lib.saveSlamMap.argtypes = [ctypes.c_char_p]
    assert lib.saveSlamMap(None) == 0
