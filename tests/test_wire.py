"""Wire formats and the recording format, CPU only.

The C implementation (slam-rgbd_amd/csrc/wire.c) is checked against an
independent restatement of the reference's byte layouts with Python's struct
module: FrameHeader '<IIHHH2xIII' (frameDefinitions.h:11-20), MessageHeader
'<9i256s' (:45-56), the end marker (loggingModule.c:224-226), the chunking
of sendDataInChunks (:447-485) and the logger's reassembly rule (:299-354).
tests/golden/rec_24x16_3f.bin was written by that restatement
(tests/golden/make_golden.py), not by the C code.
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
