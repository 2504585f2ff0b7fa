"""ctypes mirror of include/youth_wire.h: recordings, wire
chunking and reassembly, the AlgorithmModule frame loop and its queues.

The structs mirror Youth.Source/frameDefinitions.h (FrameHeader :11-20,
MessageHeader :45-56); tests/test_wire.py checks sizes and offsets.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_char, c_double, c_int, c_int16, c_int32, c_size_t
from ctypes import c_uint8, c_uint16, c_uint32, c_void_p

import numpy as np

import youth_icp

FRAME_TYPE_DEPTH_COLOR = 1
FRAME_TYPE_END_OF_FILE = 0xFF
MSG_TYPE_METADATA, MSG_TYPE_DEPTH_DATA, MSG_TYPE_COLOR_DATA, MSG_TYPE_CONTROL = 1, 2, 3, 4
MSG_TYPE_POSE = 5
MAX_MSG_SIZE = 8192
MQ_LOGGER_TO_ALGORITHM = "/logger_algorithm_queue"
MQ_ALGORITHM_POSE = "/algorithm_pose_queue"


class FrameHeader(Structure):
    _fields_ = [("frameId", c_uint32), ("timestamp", c_uint32), ("frameType", c_uint16),
                ("width", c_uint16), ("height", c_uint16), ("depthDataSize", c_uint32),
                ("colorDataSize", c_uint32), ("reserved", c_uint32)]


class MsgHeader(Structure):
    _fields_ = [("msgType", c_int), ("width", c_int), ("height", c_int), ("chunkIndex", c_int),
                ("totalChunks", c_int), ("dataSize", c_int), ("frameId", c_int),
                ("timestamp", c_uint32), ("ctrlCommand", c_int), ("filename", c_char * 256)]


class PoseMsg(Structure):
    _fields_ = [("index", c_int32), ("reserved", c_int32), ("T_wc", c_double * 16)]


MSG_PAYLOAD = MAX_MSG_SIZE - ctypes.sizeof(MsgHeader)
SINK = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_size_t)
SOURCE = ctypes.CFUNCTYPE(c_int, c_void_p, c_void_p, c_size_t, c_int)

_bound = False


def lib():
    global _bound
    L = youth_icp.load_library()
    if _bound:
        return L
    P16, PU8 = POINTER(c_int16), POINTER(c_uint8)
    sig = {
        "youth_rec_create": (c_void_p, [ctypes.c_char_p]),
        "youth_rec_write_frame": (c_int, [c_void_p, c_uint32, c_uint32, c_int, c_int, P16, PU8]),
        "youth_rec_close": (c_int, [c_void_p]),
        "youth_rec_open": (c_void_p, [ctypes.c_char_p, c_uint32]),
        "youth_rec_next": (c_int, [c_void_p, POINTER(FrameHeader), POINTER(P16),
                                   POINTER(PU8)]),
        "youth_rec_close_reader": (None, [c_void_p]),
        "youth_wire_send_frame": (c_int, [SINK, c_void_p, c_uint32, c_uint32, c_int, c_int,
                                          P16, PU8]),
        "youth_asm_create": (c_void_p, [c_int]),
        "youth_asm_destroy": (None, [c_void_p]),
        "youth_asm_push": (c_int, [c_void_p, c_void_p, c_size_t, POINTER(FrameHeader),
                                   POINTER(P16), POINTER(PU8)]),
        "youth_algorithm_loop": (c_int, [ctypes.c_char_p, ctypes.c_char_p, POINTER(c_int)]),
        "youth_algorithm_run": (c_int, [SOURCE, c_void_p, SINK, c_void_p, POINTER(c_int)]),
        "youth_wire_mq_send_frame": (c_int, [ctypes.c_char_p, c_uint32, c_uint32, c_int, c_int,
                                             P16, PU8]),
        "youth_wire_mq_recv_pose": (c_int, [ctypes.c_char_p, c_int, POINTER(MsgHeader),
                                            POINTER(PoseMsg)]),
        "youth_rec_play": (c_int, [ctypes.c_char_p, c_int]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _bound = True
    return L


def _p16(a):
    return None if a is None else a.ctypes.data_as(POINTER(c_int16))


def _pu8(a):
    return None if a is None else a.ctypes.data_as(POINTER(c_uint8))


def write_recording(path: str, frames) -> int:
    """frames: iterable of (frame_id, timestamp_ms, depth[H,W] int16, color[H,W,3] u8 | None).
    Returns youth_rec_close's count (-1 on error)."""
    L = lib()
    w = L.youth_rec_create(path.encode())
    if not w:
        raise OSError(f"youth_rec_create({path}) failed")
    for fid, ts, d, c in frames:
        d = np.ascontiguousarray(d, np.int16)
        c = None if c is None else np.ascontiguousarray(c, np.uint8)
        if L.youth_rec_write_frame(w, fid, ts, d.shape[1], d.shape[0], _p16(d), _pu8(c)) != 1:
            L.youth_rec_close(w)
            raise OSError("youth_rec_write_frame failed")
    return L.youth_rec_close(w)


def read_recording(path: str, max_plane_bytes: int = 0):
    """All frames of a recording: (list of (FrameHeader, depth, color|None), end code) where
    end code is 0 (marker / end of file) or -1 (error)."""
    L = lib()
    r = L.youth_rec_open(path.encode(), max_plane_bytes)
    if not r:
        raise OSError(f"youth_rec_open({path}) failed")
    out = []
    try:
        while True:
            h = FrameHeader()
            d, c = POINTER(c_int16)(), POINTER(c_uint8)()
            rc = L.youth_rec_next(r, ctypes.byref(h), ctypes.byref(d), ctypes.byref(c))
            if rc != 1:
                return out, rc
            n = h.width * h.height
            depth = np.ctypeslib.as_array(d, (n,)).reshape(h.height, h.width).copy()
            color = (np.ctypeslib.as_array(c, (3 * n,)).reshape(h.height, h.width, 3).copy()
                     if c else None)
            out.append((h, depth, color))
    finally:
        L.youth_rec_close_reader(r)


def frame_messages(frame_id, ts, depth, color=None):
    """The wire messages of one frame (youth_wire_send_frame), as bytes objects."""
    L = lib()
    d = np.ascontiguousarray(depth, np.int16)
    c = None if color is None else np.ascontiguousarray(color, np.uint8)
    msgs = []

    def sink(_user, msg, length):
        msgs.append(ctypes.string_at(msg, length))
        return 0

    cb = SINK(sink)
    n = L.youth_wire_send_frame(cb, None, frame_id, ts, d.shape[1], d.shape[0], _p16(d), _pu8(c))
    assert n == len(msgs), (n, len(msgs))
    return msgs


class Assembler:
    def __init__(self, need_color: bool = False):
        self.L = lib()
        self.h = self.L.youth_asm_create(1 if need_color else 0)

    def push(self, msg: bytes):
        """-1 / None (no frame yet) / (FrameHeader, depth, color|None)."""
        h = FrameHeader()
        d, c = POINTER(c_int16)(), POINTER(c_uint8)()
        buf = ctypes.create_string_buffer(msg, len(msg))
        rc = self.L.youth_asm_push(self.h, buf, len(msg), ctypes.byref(h), ctypes.byref(d),
                                   ctypes.byref(c))
        if rc < 0:
            return -1
        if rc == 0:
            return None
        n = h.width * h.height
        depth = np.ctypeslib.as_array(d, (n,)).reshape(h.height, h.width).copy()
        color = (np.ctypeslib.as_array(c, (3 * n,)).reshape(h.height, h.width, 3).copy()
                 if c else None)
        return h, depth, color

    def close(self):
        if self.h:
            self.L.youth_asm_destroy(self.h)
            self.h = None

    __del__ = close


def mq_send_frame(queue: str, frame_id, ts, depth, color=None) -> int:
    d = np.ascontiguousarray(depth, np.int16)
    c = None if color is None else np.ascontiguousarray(color, np.uint8)
    return lib().youth_wire_mq_send_frame(queue.encode(), frame_id, ts, d.shape[1], d.shape[0],
                                          _p16(d), _pu8(c))


def mq_recv_pose(queue: str, timeout_ms: int = 1000):
    """(MsgHeader, PoseMsg) or None on timeout; raises on a queue error."""
    h, p = MsgHeader(), PoseMsg()
    rc = lib().youth_wire_mq_recv_pose(queue.encode(), timeout_ms, ctypes.byref(h),
                                       ctypes.byref(p))
    if rc < 0:
        raise OSError(f"youth_wire_mq_recv_pose({queue}) failed")
    return (h, p) if rc == 1 else None


def run_loop(next_message, on_pose, stop=None) -> int:
    """youth_algorithm_run with Python callbacks: next_message(timeout_ms) ->
    bytes | None (nothing yet) | False (end); on_pose(MsgHeader, PoseMsg)."""
    def src(_u, buf, cap, timeout_ms):
        m = next_message(timeout_ms)
        if m is False:
            return -1
        if not m:
            return 0
        ctypes.memmove(buf, m, min(len(m), cap))
        return len(m)

    def pub(_u, msg, length):
        raw = ctypes.string_at(msg, length)
        h = MsgHeader.from_buffer_copy(raw[:ctypes.sizeof(MsgHeader)])
        p = PoseMsg.from_buffer_copy(raw[ctypes.sizeof(MsgHeader):])
        on_pose(h, p)
        return 0

    cs, cp = SOURCE(src), SINK(pub)
    flag = stop if stop is not None else c_int(0)
    return lib().youth_algorithm_run(cs, None, cp, None, ctypes.byref(flag))


def _libc_mq():
    libc = ctypes.CDLL(None, use_errno=True)
    if not hasattr(libc, "mq_open"):
        libc = ctypes.CDLL("librt.so.1", use_errno=True)
    return libc


def mq_raise_limit() -> None:
    """Raise the soft RLIMIT_MSGQUEUE to the hard limit (a queue with the
    reference's attributes, 10 x 8192 B, needs ~82 KB of it)."""
    import resource
    soft, hard = resource.getrlimit(resource.RLIMIT_MSGQUEUE)
    if hard == resource.RLIM_INFINITY or soft < hard:
        try:
            resource.setrlimit(resource.RLIMIT_MSGQUEUE, (hard, hard))
        except (ValueError, OSError):
            pass


def mq_diagnose() -> str:
    """Why a queue with the reference's attributes cannot be opened: errno of
    the probe, RLIMIT_MSGQUEUE and the /proc/sys/fs/mqueue limits."""
    import resource
    parts = [f"rlimit_msgqueue={resource.getrlimit(resource.RLIMIT_MSGQUEUE)}"]
    for k in ("msg_max", "msgsize_max", "queues_max"):
        try:
            parts.append(f"{k}={open('/proc/sys/fs/mqueue/' + k).read().strip()}")
        except OSError as e:
            parts.append(f"{k}=?({e.errno})")
    parts.append(f"probe_errno={_probe()[1]}")
    return ", ".join(parts)


def mq_available() -> bool:
    """POSIX queues usable here (RLIMIT_MSGQUEUE may be 0 for the user)."""
    return _probe()[0]


def _probe():
    class Attr(Structure):
        _fields_ = [("flags", ctypes.c_long), ("maxmsg", ctypes.c_long),
                    ("msgsize", ctypes.c_long), ("curmsgs", ctypes.c_long),
                    ("pad", ctypes.c_long * 4)]
    libc = _libc_mq()
    libc.mq_open.restype = c_int
    libc.mq_open.argtypes = [ctypes.c_char_p, c_int, c_int, POINTER(Attr)]
    name = f"/youth_probe_{os.getpid()}".encode()
    a = Attr(0, 10, MAX_MSG_SIZE, 0)
    fd = libc.mq_open(name, os.O_CREAT | os.O_RDWR, 0o600, ctypes.byref(a))
    if fd < 0:
        return False, ctypes.get_errno()
    libc.mq_close(fd)
    libc.mq_unlink(name)
    return True, 0


def mq_unlink(name: str) -> None:
    _libc_mq().mq_unlink(name.encode())


def play(path: str, realtime: bool = False) -> int:
    return lib().youth_rec_play(path.encode(), 1 if realtime else 0)
