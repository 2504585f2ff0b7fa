"""The pipeline side of the drop-in on the GPU.

f2: a synthetic sequence recorded in the logger's .bin format and replayed
    through the SLAM.h API gives the same trajectory as the C oracle's
    composed frame-to-frame poses.
f1: the AlgorithmModule frame loop pulls the logger's chunked messages from
    a 4th POSIX queue, tracks, and publishes one YOUTH_MSG_TYPE_POSE message
    per frame (trajectory index, frame id, timestamp, T_wc).
"""
import ctypes
import os
import threading

import numpy as np
import pytest

import oracle
import youth_icp
import youth_synth
import youth_wire
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-5
CFG = os.path.join(GOLDEN, "astra_camera.yaml")


def _expected(frames):
    """World poses: prefix product of the oracle's relative poses."""
    out, acc = [np.eye(4)], np.eye(4)
    for k in range(1, len(frames)):
        T64, _, _, _ = oracle.align(frames[k], frames[k - 1])
        acc = acc @ T64
        out.append(acc.copy())
    return out


def _err(A, B):
    return float(np.abs(np.asarray(A)[:3, :4] - np.asarray(B)[:3, :4]).max())


def test_recording_playback_through_slam_api(tmp_path):
    frames, _ = youth_synth.sequence(0, 6)
    rng = np.random.default_rng(0)
    colour = [rng.integers(0, 256, (480, 640, 3)).astype(np.uint8) for _ in range(6)]
    path = str(tmp_path / "seq.bin")
    assert youth_wire.write_recording(
        path, [(k, 1000 + 33 * k, frames[k], colour[k]) for k in range(6)]) == 6
    youth_icp.initSlamModule(CFG, "ORBvoc.txt")
    try:
        assert youth_wire.play(path) == 6
        assert youth_icp.slam_wait_idle(20000) == 1
        ts, T = youth_icp.slam_trajectory()
    finally:
        youth_icp.stopSlamModule()
    assert list(ts) == [1000 + 33 * k for k in range(6)]
    for k, E in enumerate(_expected(frames)):
        assert _err(T[k], E) <= POSE_TOL, k


def test_algorithm_loop_in_process():
    """The frame loop (reassembly -> processSlamFrame -> pose messages) over
    an in-process transport: runs on boxes where POSIX queues are refused."""
    frames, _ = youth_synth.sequence(0, 5)
    msgs = []
    for k in range(5):
        msgs += youth_wire.frame_messages(300 + k, 4000 + 33 * k, frames[k])
    poses = []
    it = iter(msgs)

    def next_message(_timeout_ms):
        m = next(it, None)
        if m is not None:
            return m
        if len(poses) == 5:
            return False                      # everything published: end the loop
        youth_icp.slam_wait_idle(100)
        return None

    youth_icp.initSlamModule(CFG, "ORBvoc.txt")
    try:
        n = youth_wire.run_loop(next_message, lambda h, p: poses.append(
            (h.msgType, h.frameId, h.timestamp, p.index, np.array(p.T_wc[:]).reshape(4, 4))))
    finally:
        youth_icp.stopSlamModule()
    assert n == 5 and len(poses) == 5
    exp = _expected(frames)
    for k, (typ, fid, ts, idx, T) in enumerate(poses):
        assert (typ, fid, ts, idx) == (youth_wire.MSG_TYPE_POSE, 300 + k, 4000 + 33 * k, k)
        assert _err(T, exp[k]) <= POSE_TOL, k


def test_algorithm_loop_over_queues():
    # the reference's queue attributes (10 x 8192 B, sensorModule.c:73-77,
    # loggingModule.c:138-141) need ~82 KB of RLIMIT_MSGQUEUE per queue:
    # raise the soft limit to the hard one first
    youth_wire.mq_raise_limit()
    if not youth_wire.mq_available():
        pytest.skip("POSIX message queues refused here: " + youth_wire.mq_diagnose())
    fq = f"/youth_t_frames_{os.getpid()}"
    pq = f"/youth_t_poses_{os.getpid()}"
    L = youth_wire.lib()
    frames, _ = youth_synth.sequence(0, 5)
    youth_icp.initSlamModule(CFG, "ORBvoc.txt")
    stop = ctypes.c_int(0)
    res = []
    t = threading.Thread(target=lambda: res.append(
        L.youth_algorithm_loop(fq.encode(), pq.encode(), ctypes.byref(stop))))
    try:
        t.start()
        for k in range(5):
            # one frame = METADATA + 79 depth chunks (no colour); blocking sends
            assert youth_wire.mq_send_frame(fq, 700 + k, 2000 + 33 * k, frames[k]) == 80
            got = youth_wire.mq_recv_pose(pq, 30000)   # one pose per frame, in order
            assert got is not None, k
            h, p = got
            assert h.msgType == youth_wire.MSG_TYPE_POSE and p.index == k
            assert (h.frameId, h.timestamp) == (700 + k, 2000 + 33 * k)
            T = np.array(p.T_wc[:]).reshape(4, 4)
            assert _err(T, _expected(frames[:k + 1])[k]) <= POSE_TOL, k
    finally:
        stop.value = 1
        t.join(timeout=30)
        youth_icp.stopSlamModule()
        youth_wire.mq_unlink(fq)
        youth_wire.mq_unlink(pq)
    assert not t.is_alive() and res == [5]
