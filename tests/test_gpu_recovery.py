"""A tracker align that times out is never used: it is realigned.

k_icp_coop is launched as a plain kernel sized to an idle device, so on a
shared GPU its grid may not be co-resident; its waits then end at the spin
bound with YOUTH_STATUS_TIMEOUT and a partly iterated pose (youth_icp.h).  The
test hook YOUTH_ICP_TEST_COOP_STALL=<chunk>[:<launches>] makes the context's
first <launches> cooperative launches lose one partial row, so they time out
the same way; YOUTH_ICP_TEST_REALIGN_STALL=1 does it to every realign's
cooperative launch.  Required:
  * youth_icp_track_realign gives the timed-out frame exactly the pose an
    undisturbed run gives (the cooperative single-pair plan again), and the
    frames around it are untouched;
  * when the realign's own cooperative launch times out too, the persistent
    kernel (no co-residency assumption) gives it within fp64 summation order;
  * through the SLAM.h drop-in (processSlamFrame backlog -> micro-batches ->
    worker), the recorded trajectory and the saveSlamMap files equal an
    undisturbed run's bit for bit, with the retry counted and traced.
Reference: SLAM.cpp:32-63 (worker), :177-198 (saveSlamMap).
"""
import os
import tempfile

import numpy as np
import pytest

import oracle
import youth_icp
import youth_synth
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-5
CFG = os.path.join(GOLDEN, "astra_camera.yaml")


def _pose_err(A, B):
    return float(np.abs(np.asarray(A)[:3, :4] - np.asarray(B)[:3, :4]).max())


def _reference_sequence(frames, batch=8):
    with youth_icp.IcpContext(640, 480, 2 * batch) as ctx:
        ctx.track_set_batch(batch)
        T, st = ctx.track_host_sequence(frames)
        assert ctx.track_realigned() == {"coop": 0, "persistent": 0, "failed": 0}
    assert not (st & youth_icp.STATUS_TIMEOUT).any()
    return T, st


def test_track_micro_batch_timeout_realigned_bit_identical(monkeypatch):
    """(a) track_submit_batch: the micro-batch launch stalls; its timed-out
    frames are realigned by hand to the undisturbed poses bit for bit, the
    other frames of the batch and the frame tracked after it are unchanged;
    then track_host_sequence does the same by itself."""
    F = 9
    frames, _ = youth_synth.sequence(0, F)
    want_T, want_st = _reference_sequence(frames)
    monkeypatch.setenv("YOUTH_ICP_TEST_COOP_STALL", "7")
    with youth_icp.IcpContext(640, 480, 16) as ctx:
        ctx.track_set_batch(8)
        ctx.track_submit_batch(frames[:8])          # frame 0 prepped, frames 1-7 one chain
        assert ctx.track_chained() == 1
        got = [ctx.track_collect() for _ in range(8)]
        assert not got[0][2]                        # frame 0: no reference
        timed_out = [k for k in range(1, 8) if got[k][1] & youth_icp.STATUS_TIMEOUT]
        assert 1 in timed_out, [g[1] for g in got]  # pair 0 of the chain lost its row
        for k in range(1, 8):
            if k in timed_out:
                if k == 1:                          # stopped after iteration 0
                    assert _pose_err(got[k][0], want_T[k - 1]) > 0
                T, st = ctx.track_realign(frames[k - 1], frames[k])
                assert np.array_equal(T, want_T[k - 1]) and st == want_st[k - 1], k
            else:
                assert np.array_equal(got[k][0], want_T[k - 1]) and got[k][1] == want_st[k - 1]
        assert ctx.track_realigned() == {"coop": len(timed_out), "persistent": 0, "failed": 0}
        # the tracker's reference (frame 7) was not disturbed by the realigns
        ctx.track_submit(frames[8])
        T8, st8, has = ctx.track_collect()
        assert has and np.array_equal(T8, want_T[7]) and st8 == want_st[7]
    with youth_icp.IcpContext(640, 480, 16) as ctx:
        ctx.track_set_batch(8)
        T, st = ctx.track_host_sequence(frames)
        re = ctx.track_realigned()
    assert re["coop"] >= 1 and re["persistent"] == 0 and re["failed"] == 0, re
    assert np.array_equal(T, want_T) and np.array_equal(st, want_st)


def test_track_realign_falls_back_to_persistent_kernel(monkeypatch):
    """The realign's own cooperative launch stalls too (REALIGN_STALL): the
    persistent k_prep + k_icp aligns the frame; its pose equals the
    undisturbed one up to fp64 summation order and is within 1e-5 of the
    oracle."""
    F = 9
    frames, _ = youth_synth.sequence(2, F)
    want_T, want_st = _reference_sequence(frames)
    monkeypatch.setenv("YOUTH_ICP_TEST_COOP_STALL", "7")
    monkeypatch.setenv("YOUTH_ICP_TEST_REALIGN_STALL", "1")
    with youth_icp.IcpContext(640, 480, 16) as ctx:
        ctx.track_set_batch(8)
        T, st = ctx.track_host_sequence(frames)
        re = ctx.track_realigned()
    assert re["persistent"] >= 1 and re["coop"] == 0 and re["failed"] == 0, re
    assert not (st & youth_icp.STATUS_TIMEOUT).any() and np.array_equal(st, want_st)
    err = max(_pose_err(T[k], want_T[k]) for k in range(F - 1))
    assert err <= 1e-12, err
    for k in range(F - 1):
        To = oracle.align(frames[k + 1], frames[k])[0]
        assert _pose_err(T[k], To) <= POSE_TOL, k


def _slam_run(frames, trace=False):
    """All frames pushed at once (a backlog under the drop threshold of 10),
    tracked by the worker; returns the trajectory, statuses, the counters and
    the saveSlamMap text."""
    youth_icp.initSlamModule(CFG, "ORBvoc.txt")
    try:
        if trace:
            youth_icp.slam_trace_enable(1 << 14)
        for k in range(frames.shape[0]):
            assert youth_icp.processSlamFrame(frames[k], None, 640, 480, 1000 + 33 * k) == 1
        assert youth_icp.slam_wait_idle(30000) == 1
        ts, T = youth_icp.slam_trajectory()
        st, few, deg = youth_icp.slam_status()
        re = youth_icp.slam_realigned()
        batched = youth_icp.slam_batched_frames()
        events = youth_icp.slam_trace_read()[1:] if trace else None
        with tempfile.TemporaryDirectory() as td:
            base = os.path.join(td, "map")
            assert youth_icp.saveSlamMap(base) == 1
            text = open(base + "_trajectory.txt").read()
    finally:
        if trace:
            youth_icp.slam_trace_enable(0)
        youth_icp.stopSlamModule()
    return dict(ts=ts, T=T, st=st, re=re, batched=batched, text=text, events=events)


def test_slam_backlog_timeout_never_composed(monkeypatch):
    """(b) processSlamFrame backlog through the drop-in: with the stall hook
    the worker's first cooperative launch times out; the worker realigns the
    frame from its held reference buffer, and the trajectory, statuses and the
    saveSlamMap file equal the undisturbed run's bit for bit."""
    F = 9
    frames, _ = youth_synth.sequence(0, F)
    base = _slam_run(frames)
    assert base["re"] == {"coop": 0, "persistent": 0, "lost": 0}
    monkeypatch.setenv("YOUTH_ICP_TEST_COOP_STALL", "7")
    got = _slam_run(frames, trace=True)
    assert got["re"]["coop"] >= 1 and got["re"]["persistent"] == 0 and got["re"]["lost"] == 0
    assert got["batched"] >= 2                       # micro-batches ran
    assert list(got["ts"]) == list(base["ts"]) == [1000 + 33 * k for k in range(F)]
    assert np.array_equal(got["T"], base["T"])
    assert np.array_equal(got["st"], base["st"]) and not (got["st"] & youth_icp.STATUS_TIMEOUT).any()
    assert got["text"] == base["text"]
    kind, arg = got["events"]
    realigns = [int(a) for k, a in zip(kind, arg) if youth_icp.SLAM_EVENTS[int(k)] == "realign"]
    assert realigns and all(a == 0 for a in realigns), realigns
    # and the undisturbed trajectory is the oracle's
    acc = np.eye(4)
    for k in range(1, F):
        acc = acc @ oracle.align(frames[k], frames[k - 1])[0]
        assert _pose_err(base["T"][k], acc) <= POSE_TOL


def test_slam_backlog_timeout_persistent_fallback(monkeypatch):
    """The worker's realign times out on the cooperative plan too
    (REALIGN_STALL):
    the persistent kernel's pose is composed; the trajectory is within fp64
    summation order of the undisturbed one."""
    F = 9
    frames, _ = youth_synth.sequence(4, F)
    base = _slam_run(frames)
    monkeypatch.setenv("YOUTH_ICP_TEST_COOP_STALL", "7")
    monkeypatch.setenv("YOUTH_ICP_TEST_REALIGN_STALL", "1")
    got = _slam_run(frames)
    assert got["re"]["persistent"] >= 1 and got["re"]["coop"] == 0 and got["re"]["lost"] == 0, got["re"]
    assert list(got["ts"]) == list(base["ts"])
    err = max(_pose_err(a, b) for a, b in zip(got["T"], base["T"]))
    assert err <= 1e-12, err
    assert np.array_equal(got["st"], base["st"])


def test_entry_wait_gives_up_fast_and_tracker_recovers(monkeypatch):
    """A grid whose entry barrier never completes (hook: chunk 7's
    iteration-0 row is lost, with the product's own spin bound, not the
    hook's shorter one) is what a grid that is not co-resident looks like:
    its waits give up after kCoopSpinMax polls (~35-65 ms; ~4 s before round
    6), the frame comes back TIMEOUT, and the realign gives the undisturbed
    pose."""
    import time
    frames, _ = youth_synth.sequence(1, 3)
    with youth_icp.IcpContext(640, 480, 2) as ctx:
        want = [ctx.track_frame(f)[:2] for f in frames][1:]
    monkeypatch.setenv("YOUTH_ICP_TEST_COOP_STALL", "7")
    monkeypatch.setenv("YOUTH_ICP_TEST_COOP_STALL_ITER", "0")
    with youth_icp.IcpContext(640, 480, 2) as ctx:
        assert not ctx.track_frame(frames[0])[2]
        t0 = time.perf_counter()
        T1, st1, has = ctx.track_frame(frames[1])
        dt = time.perf_counter() - t0
        assert has and st1 & youth_icp.STATUS_TIMEOUT, st1
        assert dt < 1.5, dt                        # the bound, not round 5's ~4 s
        T, st = ctx.track_realign(frames[0], frames[1])
        assert np.array_equal(T, want[0][0]) and st == want[0][1]
        T2, st2, _ = ctx.track_frame(frames[2])    # the tracker carries on
        assert np.array_equal(T2, want[1][0]) and st2 == want[1][1]
        print(f"\nspin-bound timeout after {dt * 1e3:.1f} ms")


def test_host_batch_api_realigns_a_timed_out_chunk(monkeypatch, capfd):
    """The host batch API (youth_icp_align_batch / _multi) never hands out a
    TIMEOUT pose: a chunk whose cooperative launch timed out is aligned again
    on the persistent kernel from the frames still on the device.  The cached
    batch context is recreated under the stall hook (intrinsics switched away
    and back); the poses equal an undisturbed call's within fp32 rounding,
    every status is 0, every pose is within 1e-5 of the oracle, and the retry
    is reported on stderr."""
    src, dst, _ = youth_synth.pairs(71, 4)
    Kb = youth_icp.Intrinsics(571.25, 571.25, 320.0, 240.0, 1000.0)
    Ka = youth_icp.Intrinsics(571.5, 571.5, 320.0, 240.0, 1000.0)
    want = youth_icp.align_batch(src, dst, K=Kb, iters=10)[0]
    youth_icp.align_batch(src[:1], dst[:1], K=Ka, iters=10)     # the cached context moves to Ka
    monkeypatch.setenv("YOUTH_ICP_TEST_COOP_STALL", "7")
    capfd.readouterr()
    got, st = youth_icp.align_batch_multi(src, dst, K=Kb, iters=10, devices=[0])   # recreated: hook on
    err = capfd.readouterr().err
    monkeypatch.delenv("YOUTH_ICP_TEST_COOP_STALL")
    assert "realigned on the persistent kernel" in err, err[-2000:]
    assert not np.asarray(st).any(), st
    assert float(np.abs(np.asarray(got) - np.asarray(want)).max()) <= 1e-6
    Ko = [Kb.fx, Kb.fy, Kb.cx, Kb.cy, Kb.depth_scale]
    for i in range(src.shape[0]):
        To = oracle.align(src[i], dst[i], K=Ko)[0]
        assert _pose_err(np.asarray(got[i], np.float64), To) <= POSE_TOL


def test_slam_few_matches_frames_are_composed_with_their_status():
    """YOUTH_STATUS_FEW_MATCHES (youth_icp.h): a frame with no valid depth
    skips every update, so its relative pose is the identity ("no motion"),
    which is composed; the status bits are kept with the pose and counted.
    The frame after it (aligned against the empty frame) likewise."""
    frames, _ = youth_synth.sequence(0, 4)
    seq = np.stack([frames[0], np.zeros_like(frames[0]), frames[2], frames[3]])
    youth_icp.initSlamModule(CFG, "ORBvoc.txt")
    try:
        for k in range(seq.shape[0]):
            assert youth_icp.processSlamFrame(seq[k], None, 640, 480, 10 + k) == 1
            assert youth_icp.slam_wait_idle(20000) == 1
        ts, T = youth_icp.slam_trajectory()
        st, few, deg = youth_icp.slam_status()
        re = youth_icp.slam_realigned()
    finally:
        youth_icp.stopSlamModule()
    assert list(ts) == [10, 11, 12, 13]
    assert list(st) == [0, youth_icp.STATUS_FEW_MATCHES, youth_icp.STATUS_FEW_MATCHES, 0], st
    assert few == 2 and deg == 0 and re == {"coop": 0, "persistent": 0, "lost": 0}
    assert np.array_equal(T[1], np.eye(4)) and np.array_equal(T[2], np.eye(4))
    T3 = oracle.align(seq[3], seq[2])[0]
    assert _pose_err(T[3], T3) <= POSE_TOL
