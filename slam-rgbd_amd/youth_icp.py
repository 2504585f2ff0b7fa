"""Python host mirror of the C-ABI in include/youth_icp.h (ctypes, no torch).

Two layers, mirroring the reference's interface for this path:

* The reference's own AlgorithmModule API — same names, argument meaning and
  1/0 return convention as Youth.Source/AlgorithmModule/SLAM.h:11-38
  (``initSlamModule``, ``stopSlamModule``, ``processSlamFrame``,
  ``saveSlamMap``, ``isSlamModuleRunning``, ``getSlamMapPoints``,
  ``resetSlam``) so a parity test reads like a caller of SLAM.h.
* The additive batch / device API (``IcpContext``, ``align_batch``).

The library is built in-tree (``make -C slam-rgbd_amd``) and loaded from
next to this file.  There is no CPU fallback: if ``libyouth_icp.so`` is
missing, importing the wrappers raises, and every compute call on a machine
without a HIP device returns ``YOUTH_ENODEV`` -> ``IcpError``.
"""
from __future__ import annotations

import ctypes
import os
import re
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int16, c_int32
from ctypes import c_size_t, c_uint8, c_uint32, c_void_p

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("YOUTH_ICP_LIB") or os.path.join(HERE, "libyouth_icp.so")  # override: A/B builds (tools/ab.sh)
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "youth_icp.h")

YOUTH_OK = 0
YOUTH_EINVAL = -1
YOUTH_ENOMEM = -2
YOUTH_EHIP = -3
YOUTH_ENODEV = -4
YOUTH_NEQ = 29
SPEC_FMA = 0       # YOUTH_SPEC_FMA: opt-in, spec a7/a8 on fma chains
SPEC_SURVEY = 1    # YOUTH_SPEC_SURVEY (default): SURVEY.md §8a a7/a8 as worded (no FMA, IEEE division)
REDUCE_EXACT = 0   # YOUTH_REDUCE_EXACT (default): every product exact in fp64, launch-independent
REDUCE_LANE32 = 1  # YOUTH_REDUCE_LANE32 (opt-in): fp32 lane sums -> fp64, launch-shape dependent
LANES_STRIDED, LANES_COOP, LANES_COOP_TILE = 0, 1, 2   # youth_lanes.kind
STATUS_DEGENERATE = 1
STATUS_FEW_MATCHES = 2
STATUS_TIMEOUT = 4  # a kernel hit its spin bound (youth_icp.h YOUTH_STATUS_TIMEOUT)


class IcpError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"youth_icp error {code}: {msg}")
        self.code = code


class Intrinsics(ctypes.Structure):
    _fields_ = [("fx", c_float), ("fy", c_float), ("cx", c_float), ("cy", c_float),
                ("depth_scale", c_float)]

    def as_tuple(self):
        return (self.fx, self.fy, self.cx, self.cy, self.depth_scale)


class Lanes(ctypes.Structure):
    """youth_lanes: how one align partitioned an iteration's pixels into lanes."""
    _fields_ = [("kind", c_int), ("chunk", c_int), ("threads", c_int), ("npx", c_int)]

    def as_tuple(self):
        return (self.kind, self.chunk, self.threads, self.npx)


class Params(ctypes.Structure):
    _fields_ = [("iters", c_int), ("dist_thresh", c_float)]


_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libyouth_icp.so (raises OSError when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"{path} not built: run `make -C {HERE}` (HIP extension missing)")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    P16, PU8, PF, PD, PI32 = POINTER(c_int16), POINTER(c_uint8), POINTER(c_float), \
        POINTER(c_double), POINTER(c_int32)
    sig = {
        "initSlamModule": (None, [c_char_p, c_char_p]),
        "stopSlamModule": (None, []),
        "processSlamFrame": (c_int, [P16, PU8, c_int, c_int, c_uint32]),
        "saveSlamMap": (c_int, [c_char_p]),
        "isSlamModuleRunning": (c_int, []),
        "getSlamMapPoints": (c_int, []),
        "resetSlam": (None, []),
        "algorithmModule": (c_void_p, [c_void_p]),
        "youth_default_intrinsics": (Intrinsics, [c_int, c_int]),
        "youth_default_params": (Params, []),
        "youth_icp_last_error": (c_char_p, []),
        "youth_icp_device_count": (c_int, []),
        "youth_icp_fastdiv_enabled": (c_int, [c_void_p]),
        "youth_icp_set_spec": (c_int, [c_void_p, c_int]),
        "youth_icp_set_concurrency": (c_int, [c_void_p, c_int]),
        "youth_icp_get_spec": (c_int, [c_void_p]),
        "youth_icp_set_reduce": (c_int, [c_void_p, c_int]),
        "youth_icp_get_reduce": (c_int, [c_void_p]),
        "youth_icp_get_lanes": (c_int, [c_void_p, POINTER(Lanes)]),
        "youth_icp_selftest_projquot": (c_int, [c_int, ctypes.c_longlong, ctypes.c_ulonglong,
                                                POINTER(ctypes.c_longlong),
                                                POINTER(ctypes.c_longlong),
                                                POINTER(ctypes.c_longlong)]),
        "youth_icp_align_batch": (c_int, [P16, P16, c_int, c_int, c_int, POINTER(Intrinsics),
                                          c_int, PF, PI32]),
        "youth_icp_align_batch_multi": (c_int, [P16, P16, c_int, c_int, c_int,
                                                POINTER(Intrinsics), c_int, PI32, c_int, PF,
                                                PI32]),
        "youth_icp_shard_range": (c_int, [c_int, c_int, c_int, POINTER(c_int), POINTER(c_int)]),
        "youth_icp_create": (c_void_p, [c_int, c_int, c_int, c_int, POINTER(Intrinsics),
                                        POINTER(Params)]),
        "youth_icp_destroy": (None, [c_void_p]),
        "youth_icp_align_pairs_device": (c_int, [c_void_p, c_void_p, c_void_p, c_int, PD,
                                                 c_void_p, c_void_p]),
        "youth_icp_align_sequence_device": (c_int, [c_void_p, c_void_p, c_int, c_void_p,
                                                    c_void_p]),
        "youth_icp_sync": (c_int, [c_void_p, c_void_p]),
        "youth_icp_get_poses": (c_int, [c_void_p, c_int, PD, PF, PI32]),
        "youth_icp_get_stats": (c_int, [c_void_p, c_int, c_int, PD, PD]),
        "youth_icp_set_timing": (c_int, [c_void_p, c_int]),
        "youth_icp_get_timing": (c_int, [c_void_p, c_int, PD, POINTER(c_int)]),
        "youth_icp_get_sched_stats": (c_int, [c_void_p, POINTER(c_uint32), POINTER(c_uint32)]),
        "youth_icp_get_plan": (c_int, [c_void_p, POINTER(c_int), POINTER(c_int)]),
        "youth_icp_selftest_projdiv": (c_int, [c_int, ctypes.c_longlong, ctypes.c_ulonglong,
                                               POINTER(ctypes.c_longlong),
                                               POINTER(ctypes.c_longlong)]),
        "youth_icp_selftest_normalize": (c_int, [c_int, ctypes.c_longlong, ctypes.c_ulonglong,
                                                 POINTER(ctypes.c_longlong),
                                                 POINTER(ctypes.c_longlong),
                                                 POINTER(ctypes.c_longlong)]),
        "youth_icp_prepare_host": (c_int, [c_void_p, P16, c_int, c_int, PF, PF, PF, PF, PF,
                                           PF]),
        "youth_icp_reduce_host": (c_int, [c_void_p, P16, P16, PF, PI32, PD]),
        "youth_icp_solve_host": (c_int, [c_void_p, PD, PD]),
        "youth_icp_track_frame": (c_int, [c_void_p, P16, PD, PD, POINTER(c_int)]),
        "youth_icp_track_reset": (None, [c_void_p]),
        "youth_icp_track_submit": (c_int, [c_void_p, P16, PD]),
        "youth_icp_track_collect": (c_int, [c_void_p, PD, POINTER(c_int)]),
        "youth_icp_track_pending": (c_int, [c_void_p]),
        "youth_icp_track_submit_batch": (c_int, [c_void_p, P16, c_int]),
        "youth_icp_track_set_batch": (c_int, [c_void_p, c_int]),
        "youth_icp_track_chained": (ctypes.c_longlong, [c_void_p]),
        "youth_icp_track_chained_frames": (ctypes.c_longlong, [c_void_p]),
        "youth_icp_track_submit_pinned": (c_int, [c_void_p, POINTER(P16), c_int]),
        "youth_icp_host_alloc": (P16, [c_size_t]),
        "youth_icp_host_free": (None, [P16]),
        "youth_icp_track_host_sequence": (c_int, [c_void_p, P16, c_int, PD, POINTER(c_int32)]),
        "youth_parse_camera_yaml": (c_int, [c_char_p, POINTER(Intrinsics), POINTER(c_int),
                                            POINTER(c_int)]),
        "youth_queue_create": (c_void_p, [c_int, c_int]),
        "youth_queue_destroy": (None, [c_void_p]),
        "youth_queue_push": (c_int, [c_void_p, P16, c_int, c_int, c_uint32]),
        "youth_queue_pop": (c_int, [c_void_p, P16, c_size_t, POINTER(c_int), POINTER(c_int),
                                    POINTER(c_uint32)]),
        "youth_queue_size": (c_int, [c_void_p]),
        "youth_queue_clear": (None, [c_void_p]),
        "youth_slam_trajectory_length": (c_int, []),
        "youth_slam_get_trajectory": (c_int, [c_int, POINTER(c_uint32), PD]),
        "youth_slam_wait_idle": (c_int, [c_int]),
        "youth_slam_batched_frames": (ctypes.c_longlong, []),
        "youth_slam_queue_size": (c_int, []),
        "youth_slam_wait_stopped": (None, []),
        "youth_slam_trace_enable": (c_int, [c_int]),
        "youth_slam_trace_read": (c_int, [c_int, PD, POINTER(c_int), POINTER(c_int)]),
        "youth_icp_track_realign": (c_int, [c_void_p, P16, P16, PD, PD]),
        "youth_icp_track_realigned": (ctypes.c_longlong, [c_void_p, POINTER(ctypes.c_longlong),
                                                          POINTER(ctypes.c_longlong)]),
        "youth_slam_realigned": (ctypes.c_longlong, [POINTER(ctypes.c_longlong),
                                                     POINTER(ctypes.c_longlong)]),
        "youth_slam_get_status": (c_int, [c_int, PI32, POINTER(ctypes.c_longlong),
                                          POINTER(ctypes.c_longlong)]),
    }
    ab_build = bool(os.environ.get("YOUTH_ICP_LIB"))  # tools/ab_*.sh: older builds
    for name, (res, args) in sig.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            if ab_build:
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def declared_functions(header: str = HEADER_PATH) -> list[str]:
    """Function names declared in an include/*.h header (for the ABI test);
    function-pointer typedefs and keywords are not functions."""
    text = open(header).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"typedef[^;]*;", "", text)
    names = re.findall(r"\b([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", text)
    keywords = {"sizeof", "int", "void", "char", "unsigned", "double", "float", "long", "short",
                "const", "return", "if", "while", "for", "struct"}
    return sorted({n for n in names if n not in keywords})


def _p(arr, ctype):
    return None if arr is None else arr.ctypes.data_as(POINTER(ctype))


def _err(code: int) -> IcpError:
    lib = load_library()
    return IcpError(code, (lib.youth_icp_last_error() or b"").decode())


TRACK_MAX_IN_FLIGHT = 16  # YOUTH_TRACK_MAX_IN_FLIGHT (include/youth_icp.h)
TRACK_MAX_BATCH = 8       # YOUTH_TRACK_MAX_BATCH
MAX_CONCURRENCY = 4       # YOUTH_ICP_MAX_CONCURRENCY


def _check(code: int) -> int:
    if code < 0:
        raise _err(code)
    return code


def default_intrinsics(width: int, height: int) -> Intrinsics:
    return load_library().youth_default_intrinsics(width, height)


def default_params() -> Params:
    return load_library().youth_default_params()


def device_count() -> int:
    return load_library().youth_icp_device_count()


# ----------------------------------------------------------- SLAM.h mirror --
def initSlamModule(config_file: str | None, vocabulary_file: str | None = None) -> None:
    load_library().initSlamModule(config_file.encode() if config_file else None,
                                  vocabulary_file.encode() if vocabulary_file else None)


def stopSlamModule() -> None:
    load_library().stopSlamModule()


def processSlamFrame(depth_data: np.ndarray, color_data: np.ndarray | None, width: int,
                     height: int, timestamp: int) -> int:
    depth = np.ascontiguousarray(depth_data, dtype=np.int16)
    if depth.size < width * height:
        return 0
    color = None if color_data is None else np.ascontiguousarray(color_data, dtype=np.uint8)
    return load_library().processSlamFrame(_p(depth, c_int16), _p(color, c_uint8), width,
                                           height, timestamp)


def saveSlamMap(map_file: str) -> int:
    return load_library().saveSlamMap(map_file.encode())


def isSlamModuleRunning() -> int:
    return load_library().isSlamModuleRunning()


def getSlamMapPoints() -> int:
    return load_library().getSlamMapPoints()


def resetSlam() -> None:
    load_library().resetSlam()


def slam_wait_idle(timeout_ms: int = 10000) -> int:
    return load_library().youth_slam_wait_idle(timeout_ms)


def slam_batched_frames() -> int:
    """Frames the SLAM worker aligned in chained micro-batch launches."""
    return int(load_library().youth_slam_batched_frames())


def slam_queue_size() -> int:
    """Frames waiting in the SLAM module's ingest queue."""
    return load_library().youth_slam_queue_size()


SLAM_EVENTS = {1: "push_begin", 2: "push_end", 3: "take", 4: "submit_begin", 5: "submit_end",
               6: "collect_begin", 7: "collect_end", 8: "idle_begin", 9: "idle_end",
               10: "pool", 11: "drop", 12: "submit_step",
               13: "realign"}   # YOUTH_SLAM_EV_* (youth_icp.h)


def slam_trace_enable(capacity: int) -> None:
    """youth_slam_trace_enable: record the ingest path's events (0 = off)."""
    _check(load_library().youth_slam_trace_enable(int(capacity)))


def slam_trace_read(n: int = 1 << 20) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(t seconds CLOCK_MONOTONIC, kind, arg) of the recorded events."""
    t = np.zeros(n, np.float64)
    k = np.zeros(n, np.int32)
    a = np.zeros(n, np.int32)
    m = min(n, load_library().youth_slam_trace_read(n, _p(t, c_double), _p(k, c_int),
                                                     _p(a, c_int)))
    return t[:m], k[:m], a[:m]


def slam_realigned() -> dict:
    """youth_slam_realigned: timed-out aligns the worker realigned on the
    cooperative plan / the persistent kernel, and those it lost."""
    p, lost = ctypes.c_longlong(0), ctypes.c_longlong(0)
    coop = load_library().youth_slam_realigned(ctypes.byref(p), ctypes.byref(lost))
    return {"coop": int(coop), "persistent": int(p.value), "lost": int(lost.value)}


def slam_status() -> tuple[np.ndarray, int, int]:
    """youth_slam_get_status: (status bits per trajectory entry, frames with
    FEW_MATCHES, frames with DEGENERATE)."""
    lib = load_library()
    n = lib.youth_slam_trajectory_length()
    st = np.zeros(max(n, 1), np.int32)
    few, deg = ctypes.c_longlong(0), ctypes.c_longlong(0)
    m = lib.youth_slam_get_status(n, _p(st, c_int32), ctypes.byref(few), ctypes.byref(deg))
    return st[:m], int(few.value), int(deg.value)


def slam_trajectory() -> tuple[np.ndarray, np.ndarray]:
    lib = load_library()
    n = lib.youth_slam_trajectory_length()
    ts = np.zeros(n, np.uint32)
    T = np.zeros((n, 4, 4), np.float64)
    m = lib.youth_slam_get_trajectory(n, _p(ts, c_uint32), _p(T, c_double))
    return ts[:m], T[:m]


def parse_camera_yaml(path: str, width: int = 640, height: int = 480):
    """(Intrinsics, W, H) from an ORB-SLAM3-style YAML; None if unreadable."""
    lib = load_library()
    K = lib.youth_default_intrinsics(width, height)
    W, H = c_int(0), c_int(0)
    ok = lib.youth_parse_camera_yaml(path.encode(), ctypes.byref(K), ctypes.byref(W),
                                     ctypes.byref(H))
    return (K, W.value, H.value) if ok else None


# ---------------------------------------------------------- ingest queue --
class FrameQueue:
    """The bounded ingest queue (SLAM.cpp:159-169 policy)."""

    def __init__(self, high_water: int = 10, low_water: int = 5):
        self._lib = load_library()
        self._q = self._lib.youth_queue_create(high_water, low_water)
        if not self._q:
            raise IcpError(YOUTH_EINVAL, "bad queue watermarks")

    def push(self, depth: np.ndarray, timestamp: int = 0) -> int:
        d = np.ascontiguousarray(depth, dtype=np.int16)
        return _check(self._lib.youth_queue_push(self._q, _p(d, c_int16), d.shape[1],
                                                 d.shape[0], timestamp))

    def pop(self, cap: int = 4096 * 4096):
        buf = np.empty(cap, np.int16)
        w, h, ts = c_int(0), c_int(0), c_uint32(0)
        rc = _check(self._lib.youth_queue_pop(self._q, _p(buf, c_int16), cap, ctypes.byref(w),
                                              ctypes.byref(h), ctypes.byref(ts)))
        if rc == 0:
            return None
        return buf[: w.value * h.value].reshape(h.value, w.value).copy(), ts.value

    def __len__(self):
        return self._lib.youth_queue_size(self._q)

    def clear(self):
        self._lib.youth_queue_clear(self._q)

    def close(self):
        if self._q:
            self._lib.youth_queue_destroy(self._q)
            self._q = None

    __del__ = close


class PinnedFrame:
    """One page-locked host frame (youth_icp_host_alloc) as a numpy view."""

    def __init__(self, height: int, width: int):
        self._lib = load_library()
        self.ptr = self._lib.youth_icp_host_alloc(width * height)
        if not self.ptr:
            raise IcpError(YOUTH_ENOMEM, "youth_icp_host_alloc failed")
        self.array = np.ctypeslib.as_array(self.ptr, shape=(height, width))

    def close(self):
        if getattr(self, "ptr", None):
            self.array = None
            self._lib.youth_icp_host_free(self.ptr)
            self.ptr = None

    __del__ = close


# -------------------------------------------------------- additive API --
class IcpContext:
    """Device workspace for W x H frames (youth_icp_create)."""

    def __init__(self, width: int, height: int, max_frames: int, K: Intrinsics | None = None,
                 iters: int = 10, dist_thresh: float = 0.10, device: int = 0, spec=None,
                 reduction=None):
        self._lib = load_library()
        self.W, self.H, self.max_frames = width, height, max_frames
        self.K = K if K is not None else default_intrinsics(width, height)
        self.params = Params(iters, dist_thresh)
        self._ctx = self._lib.youth_icp_create(device, width, height, max_frames,
                                               ctypes.byref(self.K), ctypes.byref(self.params))
        if not self._ctx:
            msg = (self._lib.youth_icp_last_error() or b"").decode()
            raise IcpError(YOUTH_ENODEV if "no HIP device" in msg else YOUTH_EHIP, msg)
        if spec is not None:
            self.spec = spec
        if reduction is not None:
            self.reduction = reduction

    @property
    def handle(self) -> int:
        return self._ctx

    @property
    def fastdiv(self) -> bool:
        """True when the verified 3-op back-projection division is in use."""
        return bool(self._lib.youth_icp_fastdiv_enabled(self._ctx))

    @property
    def spec(self) -> int:
        """Spec a7/a8 arithmetic of the next aligns (SPEC_FMA / SPEC_SURVEY)."""
        return _check(self._lib.youth_icp_get_spec(self._ctx))

    @spec.setter
    def spec(self, value) -> None:
        code = {"fma": SPEC_FMA, "survey": SPEC_SURVEY}.get(value, value)
        _check(self._lib.youth_icp_set_spec(self._ctx, int(code)))

    @property
    def reduction(self) -> int:
        """Spec a9 reduction of the next aligns (REDUCE_LANE32 / REDUCE_EXACT)."""
        return _check(self._lib.youth_icp_get_reduce(self._ctx))

    @reduction.setter
    def reduction(self, value) -> None:
        code = {"exact": REDUCE_EXACT, "lane32": REDUCE_LANE32}.get(value, value)
        _check(self._lib.youth_icp_set_reduce(self._ctx, int(code)))

    def lanes(self) -> tuple:
        """(kind, chunk, threads, npx) of the last align's lane partition
        (youth_icp_get_lanes), the geometry oracle.set_reduce("lane32", ...)
        restates."""
        g = Lanes()
        _check(self._lib.youth_icp_get_lanes(self._ctx, ctypes.byref(g)))
        return g.as_tuple()

    def set_concurrency(self, contexts: int) -> int:
        """Declare `contexts` contexts aligning concurrently on this device
        (youth_icp_set_concurrency): the persistent kernel takes 1/contexts of
        the workgroup slots and chunks.  Returns the previous value."""
        return _check(self._lib.youth_icp_set_concurrency(self._ctx, int(contexts)))

    def close(self):
        if getattr(self, "_ctx", None):
            self._lib.youth_icp_destroy(self._ctx)
            self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        self.close()

    # device-pointer API (pointers as ints, e.g. torch tensor.data_ptr())
    def align_pairs_device(self, d_src: int, d_dst: int, n_pairs: int, T_init=None,
                           d_T_out: int = 0, stream: int = 0) -> None:
        Ti = None if T_init is None else np.ascontiguousarray(T_init, np.float64)
        _check(self._lib.youth_icp_align_pairs_device(self._ctx, d_src, d_dst, n_pairs,
                                                      _p(Ti, c_double), d_T_out or None,
                                                      stream or None))

    def align_sequence_device(self, d_frames: int, n_frames: int, d_T_out: int = 0,
                              stream: int = 0) -> None:
        _check(self._lib.youth_icp_align_sequence_device(self._ctx, d_frames, n_frames,
                                                         d_T_out or None, stream or None))

    def sync(self, stream: int = 0) -> None:
        _check(self._lib.youth_icp_sync(self._ctx, stream or None))

    def get_poses(self, n: int):
        T64 = np.zeros((n, 4, 4), np.float64)
        T32 = np.zeros((n, 4, 4), np.float32)
        st = np.zeros(n, np.int32)
        _check(self._lib.youth_icp_get_poses(self._ctx, n, _p(T64, c_double), _p(T32, c_float),
                                             _p(st, c_int32)))
        T64[:, 3, :] = (0.0, 0.0, 0.0, 1.0)
        return T64, T32, st

    def get_stats(self, n: int, iters: int):
        cnt = np.zeros((n, iters), np.float64)
        r2 = np.zeros((n, iters), np.float64)
        _check(self._lib.youth_icp_get_stats(self._ctx, n, iters, _p(cnt, c_double),
                                             _p(r2, c_double)))
        return cnt, r2

    def set_timing(self, enable, iteration_kernel_only: bool = False) -> None:
        """HIP-event timing of the launches (every kernel kind, or only the
        iteration kernel: fewer markers inside a timed region)."""
        mode = (2 if iteration_kernel_only else 1) if enable else 0
        _check(self._lib.youth_icp_set_timing(self._ctx, mode))

    def get_timing(self, kind: int = 0):
        ms, n = c_double(0.0), c_int(0)
        _check(self._lib.youth_icp_get_timing(self._ctx, kind, ctypes.byref(ms),
                                              ctypes.byref(n)))
        return ms.value, n.value

    def get_sched_stats(self):
        """(epoch polls, items that waited) of the last persistent align."""
        spins, waited = c_uint32(0), c_uint32(0)
        _check(self._lib.youth_icp_get_sched_stats(self._ctx, ctypes.byref(spins),
                                                   ctypes.byref(waited)))
        return spins.value, waited.value

    def get_plan(self) -> dict:
        """Kernel path of the last align: the small-batch cooperative kernel
        (workgroups per pair, source pixels per lane) or the persistent one."""
        g, px = c_int(0), c_int(0)
        r = self._lib.youth_icp_get_plan(self._ctx, ctypes.byref(g), ctypes.byref(px))
        _check(min(r, 0))
        if r == 1:
            return {"kernel": "k_icp_coop", "workgroups_per_pair": g.value, "threads": 512,
                    "px_per_lane": px.value}
        if r == 2:
            return {"kernel": "k_prep + k_init + k_reduce x iters (per-iteration)"}
        return {"kernel": "k_prep + k_icp (persistent)"}

    # host-array stage entry points (parity tests)
    def prepare(self, depth: np.ndarray, want_normals: bool = True, want_xyz: bool = True):
        """Stage a2/a6 on host frames: X, Y, Z planes and the record normals
        (NX, NY, NZ).  want_xyz=False asks for the normals only, which runs the
        align path's record kernel exactly as an align does (no X/Y/Z planes
        stored; X/Y/Z come back as zeros)."""
        d = np.ascontiguousarray(depth, np.int16).reshape(-1, self.H, self.W)
        n = d.shape[0]
        outs = [np.zeros((n, self.H, self.W), np.float32) for _ in range(6)]
        ptrs = [_p(o, c_float) if (k >= 3 or want_xyz) else None for k, o in enumerate(outs)]
        _check(self._lib.youth_icp_prepare_host(self._ctx, _p(d, c_int16), n,
                                                1 if want_normals else 0, *ptrs))
        return outs

    def reduce(self, src: np.ndarray, dst: np.ndarray, T12: np.ndarray, want_assoc=True):
        s, _ = self._frame_args(src, None)
        d, _ = self._frame_args(dst, None)
        T = np.ascontiguousarray(np.asarray(T12, np.float32).reshape(-1)[:12])
        if T.size != 12:
            raise ValueError("T12 must hold 12 values (3x4)")
        assoc = np.zeros(self.W * self.H, np.int32) if want_assoc else None
        neq = np.zeros(YOUTH_NEQ, np.float64)
        _check(self._lib.youth_icp_reduce_host(self._ctx, _p(s, c_int16), _p(d, c_int16),
                                               _p(T, c_float), _p(assoc, c_int32),
                                               _p(neq, c_double)))
        return assoc, neq

    def solve(self, neq: np.ndarray, T64: np.ndarray):
        nq = np.ascontiguousarray(neq, np.float64)
        T = np.ascontiguousarray(np.array(T64, np.float64).reshape(4, 4))
        st = _check(self._lib.youth_icp_solve_host(self._ctx, _p(nq, c_double),
                                                   _p(T, c_double)))
        return T, st

    def _frame_args(self, depth, T_init):
        d = np.ascontiguousarray(depth, np.int16)
        if d.size != self.W * self.H:
            raise ValueError(f"depth frame of {d.size} pixels; the context is {self.W}x{self.H}")
        Ti = None if T_init is None else np.ascontiguousarray(T_init, np.float64)
        if Ti is not None and Ti.size != 16:
            raise ValueError("T_init must be a 4x4 matrix")
        return d, Ti

    def track_frame(self, depth: np.ndarray, T_init=None):
        d, Ti = self._frame_args(depth, T_init)
        T = np.zeros((4, 4), np.float64)
        has = c_int(0)
        st = _check(self._lib.youth_icp_track_frame(self._ctx, _p(d, c_int16), _p(Ti, c_double),
                                                    _p(T, c_double), ctypes.byref(has)))
        return T, st, bool(has.value)

    def track_reset(self) -> None:
        self._lib.youth_icp_track_reset(self._ctx)

    def track_submit(self, depth: np.ndarray, T_init=None) -> None:
        """Pipelined tracking: enqueue one host frame (copied before the call
        returns) and return without waiting; at most TRACK_MAX_IN_FLIGHT in
        flight."""
        d, Ti = self._frame_args(depth, T_init)
        _check(self._lib.youth_icp_track_submit(self._ctx, _p(d, c_int16), _p(Ti, c_double)))

    def track_collect(self):
        """(T_rel, status, has_ref) of the OLDEST submitted frame (waits for it)."""
        T = np.zeros((4, 4), np.float64)
        has = c_int(0)
        st = _check(self._lib.youth_icp_track_collect(self._ctx, _p(T, c_double),
                                                      ctypes.byref(has)))
        return T, st, bool(has.value)

    def track_submit_batch(self, frames: np.ndarray) -> None:
        """Micro-batch of consecutive frames [m, H, W] (m <= TRACK_MAX_BATCH):
        one cooperative launch when it fits, each frame then collected by its
        own track_collect with track_frame's result bit for bit."""
        f = np.ascontiguousarray(frames, np.int16).reshape(-1, self.H, self.W)
        _check(self._lib.youth_icp_track_submit_batch(self._ctx, _p(f, c_int16), f.shape[0]))

    def track_set_batch(self, frames: int) -> int:
        """Frames per submission of track_host_sequence; returns the previous."""
        return _check(self._lib.youth_icp_track_set_batch(self._ctx, frames))

    def track_chained(self) -> int:
        """Micro-batch launches run so far on this context."""
        return int(self._lib.youth_icp_track_chained(self._ctx))

    def track_chained_frames(self) -> int:
        """Frames those micro-batch launches aligned."""
        return int(self._lib.youth_icp_track_chained_frames(self._ctx))

    def track_submit_pinned(self, frames) -> None:
        """Submit PinnedFrames rows (or a list of them) without a staging copy
        (youth_icp_track_submit_pinned); keep them unchanged until collected."""
        ptrs = (POINTER(c_int16) * len(frames))(*[f.ptr for f in frames])
        _check(self._lib.youth_icp_track_submit_pinned(self._ctx, ptrs, len(frames)))

    def track_pending(self) -> int:
        return int(self._lib.youth_icp_track_pending(self._ctx))

    def track_realign(self, ref_depth: np.ndarray, depth: np.ndarray, T_init=None):
        """(T_rel, status) of depth aligned to ref_depth again after a timed-out
        tracker align (youth_icp_track_realign): the cooperative plan first
        (bit-identical to an undisturbed align), the persistent kernel if that
        times out too.  Waits for the frames in flight; leaves them collectable."""
        r, _ = self._frame_args(ref_depth, None)
        d, Ti = self._frame_args(depth, T_init)
        T = np.zeros((4, 4), np.float64)
        st = _check(self._lib.youth_icp_track_realign(self._ctx, _p(r, c_int16), _p(d, c_int16),
                                                      _p(Ti, c_double), _p(T, c_double)))
        return T, st

    def track_realigned(self) -> dict:
        """Realigns that completed on the cooperative plan / the persistent
        kernel, and those that still timed out."""
        p, f = ctypes.c_longlong(0), ctypes.c_longlong(0)
        coop = self._lib.youth_icp_track_realigned(self._ctx, ctypes.byref(p), ctypes.byref(f))
        return {"coop": int(coop), "persistent": int(p.value), "failed": int(f.value)}

    def track_host_sequence(self, frames: np.ndarray):
        """youth_icp_track_host_sequence: (T_rel [m, 4, 4], status [m]) of the
        frames that had a reference (m = n or n - 1)."""
        f = np.ascontiguousarray(frames, np.int16).reshape(-1, self.H, self.W)
        n = f.shape[0]
        T = np.zeros((max(n, 1), 4, 4), np.float64)
        st = np.zeros(max(n, 1), np.int32)
        m = _check(self._lib.youth_icp_track_host_sequence(self._ctx, _p(f, c_int16), n,
                                                           _p(T, c_double), _p(st, c_int32)))
        return T[:m], st[:m]


def selftest_projdiv(n: int, seed: int = 1, device: int = 0) -> tuple[int, int]:
    """youth_icp_selftest_projdiv: (bit mismatches, projection mismatches) of the
    kernels' shared-reciprocal projection division vs IEEE a/b on n cases."""
    lib = load_library()
    b, p = ctypes.c_longlong(0), ctypes.c_longlong(0)
    _check(lib.youth_icp_selftest_projdiv(device, n, seed, ctypes.byref(b), ctypes.byref(p)))
    return b.value, p.value


def selftest_projquot(n: int, seed: int = 1, device: int = 0) -> tuple[int, int, int]:
    """youth_icp_selftest_projquot: (quotient mismatches, projection mismatches,
    one-instruction floor mismatches over all 2^32 floats) of
    YOUTH_SPEC_SURVEY's projection vs IEEE num / den and floorf."""
    lib = load_library()
    q, p, f = ctypes.c_longlong(0), ctypes.c_longlong(0), ctypes.c_longlong(0)
    _check(lib.youth_icp_selftest_projquot(device, n, seed, ctypes.byref(q), ctypes.byref(p),
                                           ctypes.byref(f)))
    return q.value, p.value, f.value


def selftest_normalize(n: int, seed: int = 1, device: int = 0) -> tuple[int, int, int]:
    """youth_icp_selftest_normalize: (sqrt mismatches over [2^-96, 2^118],
    quotient mismatches, fast-path cases) of k_prep's fast normalisation vs IEEE."""
    lib = load_library()
    s, q, f = ctypes.c_longlong(0), ctypes.c_longlong(0), ctypes.c_longlong(0)
    _check(lib.youth_icp_selftest_normalize(device, n, seed, ctypes.byref(s), ctypes.byref(q),
                                            ctypes.byref(f)))
    return s.value, q.value, f.value


def align_batch(src: np.ndarray, dst: np.ndarray, K: Intrinsics | None = None, iters: int = 10,
                want_assoc: bool = False):
    """youth_icp_align_batch: src/dst [n, H, W] int16 -> (T [n,4,4] fp32, assoc|None)."""
    s = np.ascontiguousarray(src, np.int16)
    d = np.ascontiguousarray(dst, np.int16)
    if s.ndim == 2:
        s, d = s[None], d[None]
    if s.ndim != 3 or s.shape != d.shape:
        raise ValueError(f"src {s.shape} and dst {d.shape} must both be [n, H, W]")
    n, H, W = s.shape
    T = np.zeros((n, 4, 4), np.float32)
    assoc = np.zeros((n, H * W), np.int32) if want_assoc else None
    lib = load_library()
    Kp = ctypes.byref(K) if K is not None else None
    _check(lib.youth_icp_align_batch(_p(s, c_int16), _p(d, c_int16), n, W, H, Kp, iters,
                                     _p(T, c_float), _p(assoc, c_int32)))
    return T, assoc


def align_batch_multi(src: np.ndarray, dst: np.ndarray, K: Intrinsics | None = None,
                      iters: int = 10, devices=None):
    """youth_icp_align_batch_multi: contiguous pair shards over `devices`
    (None: every visible device), one host thread each -> (T [n,4,4] fp32,
    status [n] int32)."""
    s = np.ascontiguousarray(src, np.int16)
    d = np.ascontiguousarray(dst, np.int16)
    if s.ndim == 2:
        s, d = s[None], d[None]
    if s.ndim != 3 or s.shape != d.shape:
        raise ValueError(f"src {s.shape} and dst {d.shape} must both be [n, H, W]")
    n, H, W = s.shape
    T = np.zeros((n, 4, 4), np.float32)
    st = np.zeros(n, np.int32)
    dv = None if devices is None else np.ascontiguousarray(devices, np.int32)
    lib = load_library()
    Kp = ctypes.byref(K) if K is not None else None
    _check(lib.youth_icp_align_batch_multi(_p(s, c_int16), _p(d, c_int16), n, W, H, Kp, iters,
                                           _p(dv, c_int32), 0 if dv is None else len(dv),
                                           _p(T, c_float), _p(st, c_int32)))
    return T, st


def shard_range(n_pairs: int, n_parts: int, part: int):
    """youth_icp_shard_range -> (first, count)."""
    f, c = c_int(0), c_int(0)
    _check(load_library().youth_icp_shard_range(n_pairs, n_parts, part, ctypes.byref(f),
                                                ctypes.byref(c)))
    return f.value, c.value
