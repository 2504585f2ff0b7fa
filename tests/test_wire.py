"""Wire formats and the recording format, CPU only.

The C implementation (slam-rgbd_amd/csrc/wire.c) is checked against an
independent restatement of the reference's byte layouts with Python's struct
module: FrameHeader '<IIHHH2xIII' (frameDefinitions.h:11-20), MessageHeader
'<9i256s' (:45-56), the end marker (loggingModule.c:224-226), the chunking
of sendDataInChunks (:447-485) and the logger's reassembly rule (:299-354).
tests/golden/rec_24x16_3f.bin was written by that restatement
(tests/golden/make_golden.py), not by the C code.

The second half pins the same paths to the REFERENCE itself:
tests/golden/ref_logger_rec.bin and ref_logger_play.msgs were written by the
reference's loggingModule.c, compiled unchanged (oracle/Makefile `ref`,
tests/golden/make_ref_fixtures.py).
"""
import os
import struct

import numpy as np
import pytest

import youth_wire as yw
from conftest import GOLDEN

FH = struct.Struct("<IIHHH2xIII")   # FrameHeader, 28 B
MH = struct.Struct("<9i256s")        # MessageHeader, 292 B (timestamp packed as int here)


def _frames(n=3, W=24, H=16, seed=7, color=True):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        d = rng.integers(-5, 9000, (H, W)).astype(np.int16)
        c = rng.integers(0, 256, (H, W, 3)).astype(np.uint8) if color else None
        out.append((100 + k, 1000 + 33 * k, d, c))
    return out


def _pack(frames):
    """Independent restatement of saveFrameToFile + the end marker."""
    b = bytearray()
    for fid, ts, d, c in frames:
        H, W = d.shape
        b += FH.pack(fid, ts, 1, W, H, W * H * 2, W * H * 3, 0)
        b += d.astype("<i2").tobytes()
        b += (c if c is not None else np.zeros((H, W, 3), np.uint8)).tobytes()
    b += FH.pack(0, 0, 0xFF, 0, 0, 0, 0, 0)
    return bytes(b)


def test_layouts_mirror_frame_definitions():
    assert yw.ctypes.sizeof(yw.FrameHeader) == FH.size == 28
    assert yw.ctypes.sizeof(yw.MsgHeader) == MH.size == 292
    assert yw.MSG_PAYLOAD == 7900
    assert yw.FrameHeader.depthDataSize.offset == 16      # 2 padding bytes after height
    assert yw.MsgHeader.ctrlCommand.offset == 32 and yw.MsgHeader.filename.offset == 36


def test_writer_bytes_equal_independent_packer(tmp_path):
    frames = _frames() + _frames(1, 97, 53, seed=3, color=False)
    p = str(tmp_path / "a.bin")
    assert yw.write_recording(p, frames) == len(frames)
    assert open(p, "rb").read() == _pack(frames)


def test_reader_round_trip_and_golden(tmp_path):
    frames = _frames()
    got, end = yw.read_recording(os.path.join(GOLDEN, "rec_24x16_3f.bin"))
    assert end == 0 and len(got) == 3
    for (h, d, c), (fid, ts, d0, c0) in zip(got, frames):
        assert (h.frameId, h.timestamp, h.frameType, h.width, h.height) == (fid, ts, 1, 24, 16)
        assert np.array_equal(d, d0) and np.array_equal(c, c0)
    # the C writer reproduces the golden file byte for byte
    p = str(tmp_path / "b.bin")
    yw.write_recording(p, frames)
    assert open(p, "rb").read() == open(os.path.join(GOLDEN, "rec_24x16_3f.bin"), "rb").read()


def test_reader_edge_cases(tmp_path):
    # no end marker: clean end at EOF
    p = str(tmp_path / "nomark.bin")
    open(p, "wb").write(_pack(_frames(2))[:-FH.size])
    got, end = yw.read_recording(p)
    assert len(got) == 2 and end == 0
    # truncated plane: error after the intact frames
    p = str(tmp_path / "trunc.bin")
    open(p, "wb").write(_pack(_frames(2))[:-FH.size - 10])
    got, end = yw.read_recording(p)
    assert len(got) == 1 and end == -1
    # truncated header
    p = str(tmp_path / "hdr.bin")
    open(p, "wb").write(_pack(_frames(1))[:-FH.size] + b"\x01\x02\x03")
    got, end = yw.read_recording(p)
    assert len(got) == 1 and end == -1
    # the logger's 1 MiB playback cap: 640x480 fits (colour 921,600 B), 1280x960 does not
    d = np.zeros((480, 640), np.int16)
    p = str(tmp_path / "vga.bin")
    yw.write_recording(p, [(1, 1, d, None)])
    assert yw.read_recording(p)[1] == 0 and len(yw.read_recording(p)[0]) == 1
    d = np.zeros((960, 1280), np.int16)
    p = str(tmp_path / "sxga.bin")
    yw.write_recording(p, [(1, 1, d, None)])
    got, end = yw.read_recording(p)
    assert got == [] and end == -1
    got, end = yw.read_recording(p, max_plane_bytes=8 << 20)
    assert len(got) == 1 and end == 0
    # empty recording: just the marker
    p = str(tmp_path / "empty.bin")
    assert yw.write_recording(p, []) == 0
    assert open(p, "rb").read() == FH.pack(0, 0, 0xFF, 0, 0, 0, 0, 0)
    assert yw.read_recording(p) == ([], 0)


@pytest.mark.parametrize("W,H,color", [(640, 480, True), (97, 53, False), (24, 16, True)])
def test_chunking_matches_send_data_in_chunks(W, H, color):
    rng = np.random.default_rng(W)
    d = rng.integers(0, 9000, (H, W)).astype(np.int16)
    c = rng.integers(0, 256, (H, W, 3)).astype(np.uint8) if color else None
    msgs = yw.frame_messages(42, 777, d, c)
    nd = -(-2 * W * H // 7900)
    nc = -(-3 * W * H // 7900) if color else 0
    assert len(msgs) == 1 + nd + nc
    hdrs = [MH.unpack(m[:292]) for m in msgs]
    assert hdrs[0][:7] == (1, W, H, 0, 0, 0, 42) and len(msgs[0]) == 292
    planes = {2: bytearray(), 3: bytearray()}
    for m, h in zip(msgs[1:], hdrs[1:]):
        typ, w, hh, idx, tot, size, fid, ts = h[:8]
        assert len(m) == 292 + size <= 8192 and (w, hh, fid, ts) == (W, H, 42, 777)
        assert size == (7900 if idx < tot - 1 else len(m) - 292)
        assert len(planes[typ]) == idx * 7900   # in order, contiguous
        planes[typ] += m[292:]
    assert bytes(planes[2]) == d.tobytes()
    if color:
        assert bytes(planes[3]) == c.tobytes()


def test_assembler_follows_logger_rule():
    rng = np.random.default_rng(1)
    d0 = rng.integers(0, 9000, (48, 64)).astype(np.int16)
    c0 = rng.integers(0, 256, (48, 64, 3)).astype(np.uint8)
    d1 = rng.integers(0, 9000, (48, 64)).astype(np.int16)
    msgs = yw.frame_messages(5, 50, d0, c0) + yw.frame_messages(6, 83, d1, None)
    # need_color = 1 (the logger's rule): frame 5 completes at its last colour
    # chunk; frame 6 (no colour) never completes
    a = yw.Assembler(need_color=True)
    out = [(i, r) for i, m in enumerate(msgs) if (r := a.push(m)) not in (None,)]
    assert len(out) == 1 and out[0][0] == len(yw.frame_messages(5, 50, d0, c0)) - 1
    h, d, c = out[0][1]
    assert (h.frameId, h.timestamp, h.width, h.height) == (5, 50, 64, 48)
    assert np.array_equal(d, d0) and np.array_equal(c, c0)
    # need_color = 0 (ICP): each frame completes at its last depth chunk, once
    a = yw.Assembler(need_color=False)
    done = [r for m in msgs if (r := a.push(m)) is not None]
    assert [r[0].frameId for r in done] == [5, 6]
    assert np.array_equal(done[1][1], d1) and done[1][2] is None
    # malformed: short message, payload shorter than dataSize
    assert a.push(b"\x00" * 10) == -1
    bad = bytearray(msgs[1])
    assert a.push(bytes(bad[:300])) == -1
    # chunks before any METADATA are ignored; control messages are not frame data
    b = yw.Assembler()
    assert b.push(msgs[1]) is None
    ctrl = MH.pack(4, 0, 0, 0, 0, 0, 0, 0, 1, b"x.bin")
    assert b.push(ctrl) is None


def test_mq_transport_round_trip():
    """Frames through a POSIX queue (youth_wire_mq_send_frame) reassemble
    bit-exactly; pose messages come back through youth_wire_mq_recv_pose."""
    if not yw.mq_available():
        pytest.skip("POSIX message queues refused here (RLIMIT_MSGQUEUE)")
    import ctypes
    import threading
    q = f"/youth_t_wire_{os.getpid()}"
    libc = yw._libc_mq()
    libc.mq_open.restype = ctypes.c_int
    libc.mq_open.argtypes = [ctypes.c_char_p, ctypes.c_int]
    libc.mq_receive.restype = ctypes.c_ssize_t
    rng = np.random.default_rng(3)
    d = rng.integers(0, 9000, (96, 128)).astype(np.int16)
    c = rng.integers(0, 256, (96, 128, 3)).astype(np.uint8)
    sent = []
    try:
        t = threading.Thread(target=lambda: sent.append(yw.mq_send_frame(q, 9, 99, d, c)))
        t.start()                                  # blocks when the 10-deep queue is full
        fd = -1
        for _ in range(100):
            fd = libc.mq_open(q.encode(), os.O_RDONLY)
            if fd >= 0:
                break
            t.join(0.01)
        assert fd >= 0
        a, buf, frame = yw.Assembler(need_color=True), ctypes.create_string_buffer(8192), None
        while frame is None:
            n = libc.mq_receive(fd, buf, 8192, None)
            assert n > 0
            frame = a.push(buf.raw[:n])
        t.join(10)
        libc.mq_close(fd)
        h, dd, cc = frame
        assert sent == [1 + 4 + 5] and (h.frameId, h.timestamp) == (9, 99)
        assert np.array_equal(dd, d) and np.array_equal(cc, c)
        # a pose message, sent raw, is decoded by the consumer helper
        p = yw.PoseMsg(7, 0, (ctypes.c_double * 16)(*np.arange(16.0)))
        hdr = yw.MsgHeader(yw.MSG_TYPE_POSE, 0, 0, 0, 0, ctypes.sizeof(p), 9, 99, 0, b"")
        raw = bytes(hdr) + bytes(p)
        fd = libc.mq_open(q.encode(), os.O_WRONLY)
        assert libc.mq_send(fd, raw, len(raw), 0) == 0
        libc.mq_close(fd)
        got = yw.mq_recv_pose(q, 1000)
        assert got is not None and got[1].index == 7 and got[0].frameId == 9
        assert list(got[1].T_wc) == list(np.arange(16.0))
        assert yw.mq_recv_pose(q, 50) is None        # timeout
    finally:
        yw.mq_unlink(q)


# ---- pinned to the REFERENCE's own logger ----------------------------------
# tests/golden/ref_logger_rec.bin / ref_logger_play.msgs were produced by
# /root/reference/Youth.Source/LoggingModule/loggingModule.c compiled
# unchanged (oracle/Makefile `ref`, oracle/ref_logger_harness.c,
# tests/golden/make_ref_fixtures.py): the logger's saveFrameToFile recording
# of 5 frames (80x60 x3, 24x16, 97x53) and its playback stream
# (sendMetadata + sendDataInChunks), header bytes 32..291 zeroed (the
# reference leaves them uninitialised).

REF_REC = os.path.join(GOLDEN, "ref_logger_rec.bin")
REF_MSGS = os.path.join(GOLDEN, "ref_logger_play.msgs")


def _ref_frames():
    """Frames parsed from the reference recording with struct (independent
    of the C reader)."""
    b = open(REF_REC, "rb").read()
    off, out = 0, []
    while True:
        fid, ts, typ, W, H, dn, cn, _ = FH.unpack_from(b, off)
        off += FH.size
        if typ == 0xFF:
            assert off == len(b)
            return out
        assert typ == 1 and dn == 2 * W * H and cn == 3 * W * H
        d = np.frombuffer(b, "<i2", W * H, off).reshape(H, W)
        c = np.frombuffer(b, np.uint8, cn, off + dn).reshape(H, W, 3)
        off += dn + cn
        out.append((fid, ts, d, c))


def _ref_msgs():
    b = open(REF_MSGS, "rb").read()
    (n,), off, out = struct.unpack_from("<I", b), 4, []
    for _ in range(n):
        (ln,) = struct.unpack_from("<I", b, off)
        out.append(b[off + 4: off + 4 + ln])
        off += 4 + ln
    assert off == len(b)
    return out


def test_reference_recording_fixture_shape():
    fr = _ref_frames()
    assert [(f[2].shape[1], f[2].shape[0]) for f in fr] == [(80, 60)] * 3 + [(24, 16), (97, 53)]
    assert [f[0] for f in fr] == [100, 101, 102, 103, 104]
    assert [f[1] for f in fr] == [1000, 1033, 1066, 1099, 1132]
    assert min(int(f[2].min()) for f in fr) < 0          # negative depths travel as-is


def test_writer_reproduces_reference_recording(tmp_path):
    """youth_rec_write_frame + youth_rec_close == the reference logger's
    saveFrameToFile + end marker (loggingModule.c:101-130, 224-226), byte for byte."""
    p = str(tmp_path / "ours.bin")
    fr = _ref_frames()
    assert yw.write_recording(p, fr) == len(fr)
    assert open(p, "rb").read() == open(REF_REC, "rb").read()


def test_reader_reads_reference_recording():
    got, end = yw.read_recording(REF_REC)
    assert end == 0
    fr = _ref_frames()
    assert len(got) == len(fr)
    for (h, d, c), (fid, ts, d0, c0) in zip(got, fr):
        assert (h.frameId, h.timestamp, h.frameType) == (fid, ts, 1)
        assert (h.width, h.height, h.depthDataSize, h.colorDataSize) == (
            d0.shape[1], d0.shape[0], d0.nbytes, c0.nbytes)
        assert np.array_equal(d, d0) and np.array_equal(c, c0)


def test_send_frame_reproduces_reference_playback_stream():
    """youth_wire_send_frame's messages == the reference playback thread's
    sendMetadata + sendDataInChunks (loggingModule.c:447-502, 584-590), byte
    for byte (our headers are zero where the reference's are uninitialised)."""
    ours = [m for fid, ts, d, c in _ref_frames() for m in yw.frame_messages(fid, ts, d, c)]
    ref = _ref_msgs()
    assert len(ours) == len(ref) == 23
    for k, (a, b) in enumerate(zip(ours, ref)):
        assert a == b, f"message {k} differs"


def test_assembler_on_reference_playback_stream():
    """The reference's playback stream through youth_asm (the logger's rule,
    colour required, and the ICP rule) yields every recorded frame once."""
    fr = _ref_frames()
    for need_color in (True, False):
        a = yw.Assembler(need_color=need_color)
        done = [r for m in _ref_msgs() if (r := a.push(m)) is not None]
        assert len(done) == len(fr)
        for (h, d, c), (fid, ts, d0, c0) in zip(done, fr):
            assert (h.frameId, h.timestamp) == (fid, ts)
            assert np.array_equal(d, d0)
            # ICP rule: complete at the last depth chunk, before the colour
            assert np.array_equal(c, c0) if need_color else c is None
        a.close()


@pytest.mark.skipif(not os.path.isdir("/root/reference/Youth.Source/LoggingModule"),
                    reason="the reference source is only in the build container")
def test_reference_logger_regenerates_fixtures(tmp_path):
    """Where the reference is present: rebuild and rerun its logger; its
    outputs must equal the committed fixtures."""
    if not yw.mq_available():
        pytest.skip("POSIX message queues refused here (RLIMIT_MSGQUEUE)")
    import subprocess
    import sys
    sys.path.insert(0, GOLDEN)
    import make_ref_fixtures as mrf
    subprocess.run(["make", "-C", os.path.join(os.path.dirname(GOLDEN), "..", "oracle"), "ref"],
                   check=True, stdout=subprocess.DEVNULL)
    exe = os.path.join(os.path.dirname(GOLDEN), "..", "oracle", "_ref", "ref_logger")
    raw = tmp_path / "frames.raw"
    with open(raw, "wb") as f:
        fr = mrf.frames()
        f.write(struct.pack("<I", len(fr)))
        for fid, ts, d, c in fr:
            f.write(struct.pack("<4I", fid, ts, d.shape[1], d.shape[0]))
            f.write(d.astype("<i2").tobytes() + c.tobytes())
    rec, msgs = tmp_path / "rec.bin", tmp_path / "play.msgs"
    subprocess.run([exe, str(raw), str(rec), str(msgs)], check=True, timeout=120,
                   stdout=subprocess.DEVNULL)
    assert rec.read_bytes() == open(REF_REC, "rb").read()
    assert msgs.read_bytes() == open(REF_MSGS, "rb").read()
