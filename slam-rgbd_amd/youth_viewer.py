"""Python host mirror of include/youth_viewer.h (ctypes, no torch): the viewer's
point list.

The reference's 3-D view, Youth.Source/ViewerModule/viewerModule.c:336-357
(display_3d_color), emits one glColor3f + glVertex3f per pixel with depth > 0.
``CloudBuilder`` builds that vertex list on the GPU as a packed float array
[n_valid, 6] = {-x, -y, -z, r, g, b} in the loop's raster order — a vertex
buffer a renderer uploads in one call (stride 24 B).

Lives in libyouth_icp.so; no CPU fallback (a missing library raises, a
machine without a HIP device raises ``IcpError(YOUTH_ENODEV)``).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_int, c_int16, c_uint8, c_void_p

import numpy as np

import youth_icp
from youth_icp import YOUTH_EHIP, YOUTH_ENODEV, IcpError, Intrinsics

HEADER_PATH = os.path.join(os.path.dirname(youth_icp.HERE), "include", "youth_viewer.h")
FLOATS_PER_VERTEX = 6

_bound = False


def load_library() -> ctypes.CDLL:
    global _bound
    lib = youth_icp.load_library()
    if not _bound:
        PI = POINTER(Intrinsics)
        lib.youth_cloud_create.restype = c_void_p
        lib.youth_cloud_create.argtypes = [c_int, c_int, c_int, c_int]
        lib.youth_cloud_destroy.restype = None
        lib.youth_cloud_destroy.argtypes = [c_void_p]
        lib.youth_cloud_last_error.restype = c_char_p
        lib.youth_cloud_last_error.argtypes = []
        lib.youth_cloud_build_device.restype = c_int
        lib.youth_cloud_build_device.argtypes = [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                                 PI, c_void_p, c_void_p, c_void_p]
        lib.youth_cloud_build_device_posed.restype = c_int
        lib.youth_cloud_build_device_posed.argtypes = [c_void_p, c_void_p, c_void_p, c_int, c_int,
                                                       c_int, PI, c_void_p, c_void_p, c_void_p,
                                                       c_void_p]
        lib.youth_cloud_build_host.restype = c_int
        lib.youth_cloud_build_host.argtypes = [c_void_p, POINTER(c_int16), POINTER(c_uint8), c_int,
                                               c_int, PI, POINTER(ctypes.c_float), c_int]
        lib.youth_cloud_sync.restype = c_int
        lib.youth_cloud_sync.argtypes = [c_void_p, c_void_p]
        _bound = True
    return lib


def _check(lib, code: int) -> int:
    if code < 0:
        raise IcpError(code, (lib.youth_cloud_last_error() or b"").decode())
    return code


class CloudBuilder:
    """Device workspace for W x H frames, up to max_frames per device call
    (youth_cloud_create)."""

    def __init__(self, width: int, height: int, max_frames: int = 1, device: int = 0):
        self._lib = load_library()
        self.W, self.H, self.max_frames = width, height, max_frames
        self._ctx = self._lib.youth_cloud_create(device, width, height, max_frames)
        if not self._ctx:
            msg = (self._lib.youth_cloud_last_error() or b"").decode()
            raise IcpError(YOUTH_ENODEV if "no HIP device" in msg else YOUTH_EHIP, msg)

    def close(self):
        if getattr(self, "_ctx", None):
            self._lib.youth_cloud_destroy(self._ctx)
            self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        self.close()

    def build(self, depth: np.ndarray, rgb: np.ndarray | None = None,
              K: Intrinsics | None = None) -> np.ndarray:
        """One host frame -> [n_valid, 6] float32 vertices (synchronous)."""
        d = np.ascontiguousarray(depth, np.int16)
        H, W = d.shape
        c = None if rgb is None else np.ascontiguousarray(rgb, np.uint8).reshape(H, W, 3)
        out = np.empty((H * W, FLOATS_PER_VERTEX), np.float32)
        n = _check(self._lib, self._lib.youth_cloud_build_host(
            self._ctx, d.ctypes.data_as(POINTER(c_int16)),
            None if c is None else c.ctypes.data_as(POINTER(c_uint8)), W, H,
            None if K is None else ctypes.byref(K),
            out.ctypes.data_as(POINTER(ctypes.c_float)), H * W))
        return out[:n].copy()

    def build_device(self, d_depth: int, d_rgb: int, n_frames: int, W: int, H: int,
                     d_vertices: int, d_counts: int, K: Intrinsics | None = None,
                     stream: int = 0) -> None:
        """Device pointers (ints, e.g. torch data_ptr()); asynchronous on `stream`
        (0: the builder's own stream)."""
        _check(self._lib, self._lib.youth_cloud_build_device(
            self._ctx, d_depth, d_rgb or None, n_frames, W, H,
            None if K is None else ctypes.byref(K), d_vertices, d_counts, stream or None))

    def build_device_posed(self, d_depth: int, d_rgb: int, n_frames: int, W: int, H: int,
                           d_T_world: int, d_vertices: int, d_counts: int,
                           K: Intrinsics | None = None, stream: int = 0) -> None:
        """build_device in the world frame: d_T_world = device [n_frames][12]
        fp32 row-major 3x4 camera -> world poses (0: camera frame)."""
        _check(self._lib, self._lib.youth_cloud_build_device_posed(
            self._ctx, d_depth, d_rgb or None, n_frames, W, H,
            None if K is None else ctypes.byref(K), d_T_world or None, d_vertices, d_counts,
            stream or None))

    def sync(self, stream: int = 0) -> None:
        _check(self._lib, self._lib.youth_cloud_sync(self._ctx, stream or None))
