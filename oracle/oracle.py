"""ctypes wrapper of the CPU ORACLE (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, and there only as the checker / timed CPU
baseline.  The shipped library never loads it.  See icp_oracle.h for what is
pinned (back-projection: SURVEY.md §4 KAT table) and what is parity-unpinned
(the ICP maths: the reference has none).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_double, c_float, c_int, c_int16, c_int32

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
NEQ = 29


class OracleIntrinsics(ctypes.Structure):
    _fields_ = [("fx", c_float), ("fy", c_float), ("cx", c_float), ("cy", c_float),
                ("depth_scale", c_float)]


_lib = None


def build() -> None:
    subprocess.run(["make", "-C", HERE], check=True, stdout=subprocess.DEVNULL)


def load_library() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    PF, PD, P16, PI32 = POINTER(c_float), POINTER(c_double), POINTER(c_int16), POINTER(c_int32)
    PK = POINTER(OracleIntrinsics)
    lib.oracle_backproject.argtypes = [P16, c_int, c_int, PK, PF, PF, PF]
    lib.oracle_normals.argtypes = [PF, PF, PF, c_int, c_int, PF, PF, PF]
    lib.oracle_associate.argtypes = [PF] * 9 + [c_int, c_int, PK, PF, c_float, PI32]
    lib.oracle_reduce.argtypes = [PF] * 9 + [c_int, c_int, PK, PF, c_float, PD]
    lib.oracle_solve.argtypes = [PD, PD]
    lib.oracle_solve.restype = c_int
    lib.oracle_solve_ldlt.argtypes = [PD, PD]
    lib.oracle_solve_ldlt.restype = c_int
    lib.oracle_set_solve.argtypes = [c_int]
    lib.oracle_set_solve.restype = c_int
    lib.oracle_se3_exp.argtypes = [PD, PD]
    lib.oracle_align.argtypes = [P16, P16, c_int, c_int, PK, c_int, c_float, PD, PD, PF, PD]
    lib.oracle_align.restype = c_int
    lib.oracle_align_batch.argtypes = [P16, P16, c_int, c_int, c_int, PK, c_int, c_float, PD,
                                       PI32, PD, c_int]
    lib.oracle_set_spec.argtypes = [c_int]
    lib.oracle_set_spec.restype = c_int
    lib.oracle_get_spec.restype = c_int
    lib.oracle_set_reduce.argtypes = [c_int, ctypes.c_void_p]
    lib.oracle_set_reduce.restype = c_int
    lib.oracle_get_reduce.restype = c_int
    lib.oracle_max_threads.restype = c_int
    lib.oracle_viewer_cloud.argtypes = [P16, POINTER(ctypes.c_uint8), c_int, c_int, PK, PF]
    lib.oracle_viewer_cloud.restype = c_int
    lib.oracle_viewer_cloud_posed.argtypes = [P16, POINTER(ctypes.c_uint8), c_int, c_int, PK, PF, PF]
    lib.oracle_viewer_cloud_posed.restype = c_int
    for n in ("oracle_backproject", "oracle_normals", "oracle_associate", "oracle_reduce",
              "oracle_se3_exp", "oracle_align_batch"):
        getattr(lib, n).restype = None
    _lib = lib
    return lib


SPEC_FMA = 0      # ORACLE_SPEC_FMA: DESIGN.md §2's opt-in fma form
SPEC_SURVEY = 1   # ORACLE_SPEC_SURVEY (default): SURVEY.md §8a a7/a8 + §7 literally
SPECS = {"fma": SPEC_FMA, "survey": SPEC_SURVEY}


def set_spec(spec) -> int:
    """Select spec a7/a8's arithmetic ("fma" | "survey" or 0 | 1); returns the
    previous one."""
    code = SPECS.get(spec, spec)
    old = load_library().oracle_set_spec(int(code))
    if old < 0:
        raise ValueError(f"unknown spec {spec!r}")
    return old


def get_spec() -> int:
    return load_library().oracle_get_spec()


class spec:
    """Context manager: ``with oracle.spec("survey"): ...``."""

    def __init__(self, name):
        self.name = name

    def __enter__(self):
        self.old = set_spec(self.name)
        return self

    def __exit__(self, *exc):
        set_spec(self.old)


REDUCE_EXACT = 0   # ORACLE_REDUCE_EXACT: exact fp64 products, pixel order
REDUCE_LANE32 = 1  # ORACLE_REDUCE_LANE32: fp32 lanes -> fp64 finalize
REDUCES = {"exact": REDUCE_EXACT, "lane32": REDUCE_LANE32}
LANES_STRIDED, LANES_COOP, LANES_COOP_TILE = 0, 1, 2


class OracleLanes(ctypes.Structure):
    _fields_ = [("kind", c_int), ("chunk", c_int), ("threads", c_int), ("npx", c_int)]


def set_reduce(mode, lanes=None) -> int:
    """Select spec a9's reduction ("exact" | "lane32" or 0 | 1).  LANE32 needs
    the lane partition of the kernel launch it restates: a (kind, chunk,
    threads, npx) tuple, e.g. youth_icp.Context.lanes().  Returns the
    previous mode."""
    global _lanes
    code = REDUCES.get(mode, mode)
    g = None if lanes is None else OracleLanes(*[int(v) for v in lanes])
    lib = load_library()
    old = lib.oracle_set_reduce(int(code), None if g is None else ctypes.byref(g))
    if old < 0:
        raise ValueError(f"bad reduce mode {mode!r} / lanes {lanes!r}")
    if int(code) == REDUCE_LANE32:
        _lanes = tuple(int(v) for v in lanes)
    return old


_lanes = None   # the geometry of the last LANE32 selection


def get_reduce() -> int:
    return load_library().oracle_get_reduce()


class reduction:
    """Context manager: ``with oracle.reduction("lane32", lanes): ...``;
    restores the previous mode (and geometry) on exit."""

    def __init__(self, mode, lanes=None):
        self.mode, self.lanes = mode, lanes

    def __enter__(self):
        self.prev_lanes = _lanes
        self.old = set_reduce(self.mode, self.lanes)
        return self

    def __exit__(self, *exc):
        set_reduce(self.old, self.prev_lanes if self.old == REDUCE_LANE32 else None)


def K_of(K) -> OracleIntrinsics:
    if isinstance(K, OracleIntrinsics):
        return K
    if hasattr(K, "fx"):
        return OracleIntrinsics(K.fx, K.fy, K.cx, K.cy, K.depth_scale)
    return OracleIntrinsics(*K)


def viewer_K(W: int, H: int) -> OracleIntrinsics:
    return OracleIntrinsics(570.3, 570.3, float(W // 2), float(H // 2), 1000.0)


def _p(a, t):
    return None if a is None else a.ctypes.data_as(POINTER(t))


def backproject(depth: np.ndarray, K=None):
    d = np.ascontiguousarray(depth, np.int16)
    H, W = d.shape
    K = K_of(K) if K is not None else viewer_K(W, H)
    X, Y, Z = (np.zeros((H, W), np.float32) for _ in range(3))
    load_library().oracle_backproject(_p(d, c_int16), W, H, ctypes.byref(K), _p(X, c_float),
                                      _p(Y, c_float), _p(Z, c_float))
    return X, Y, Z


def viewer_cloud(depth: np.ndarray, rgb: np.ndarray | None = None, K=None,
                 T_world=None) -> np.ndarray:
    """display_3d_color's vertex list (viewerModule.c:336-357): [n_valid, 6]
    float32 rows {-x, -y, -z, r, g, b} in raster order; with T_world (3x4 or
    4x4 camera -> world) the points are moved to the world frame first
    (youth_cloud_build_device_posed)."""
    d = np.ascontiguousarray(depth, np.int16)
    H, W = d.shape
    K = K_of(K) if K is not None else viewer_K(W, H)
    c = None if rgb is None else np.ascontiguousarray(rgb, np.uint8).reshape(H, W, 3)
    T = None if T_world is None else np.ascontiguousarray(
        np.asarray(T_world, np.float32).reshape(-1)[:12])
    out = np.zeros((H * W, 6), np.float32)
    n = load_library().oracle_viewer_cloud_posed(_p(d, c_int16), _p(c, ctypes.c_uint8), W, H,
                                                 ctypes.byref(K), _p(T, c_float),
                                                 _p(out, c_float))
    return out[:n].copy()


def normals(X, Y, Z):
    H, W = X.shape
    NX, NY, NZ = (np.zeros((H, W), np.float32) for _ in range(3))
    a = [np.ascontiguousarray(v, np.float32) for v in (X, Y, Z)]
    load_library().oracle_normals(*[_p(v, c_float) for v in a], W, H, _p(NX, c_float),
                                  _p(NY, c_float), _p(NZ, c_float))
    return NX, NY, NZ


def _frames(src, dst, K):
    H, W = src.shape
    K = K_of(K) if K is not None else viewer_K(W, H)
    sX, sY, sZ = backproject(src, K)
    tX, tY, tZ = backproject(dst, K)
    nX, nY, nZ = normals(tX, tY, tZ)
    return K, W, H, [sX, sY, sZ, tX, tY, tZ, nX, nY, nZ]


def associate(src, dst, T12, K=None, dist_thresh: float = 0.10):
    K, W, H, planes = _frames(src, dst, K)
    T = np.ascontiguousarray(np.asarray(T12, np.float32).reshape(-1)[:12])
    idx = np.zeros(W * H, np.int32)
    load_library().oracle_associate(*[_p(v, c_float) for v in planes], W, H, ctypes.byref(K),
                                    _p(T, c_float), dist_thresh, _p(idx, c_int32))
    return idx


def reduce(src, dst, T12, K=None, dist_thresh: float = 0.10):
    K, W, H, planes = _frames(src, dst, K)
    T = np.ascontiguousarray(np.asarray(T12, np.float32).reshape(-1)[:12])
    out = np.zeros(NEQ, np.float64)
    load_library().oracle_reduce(*[_p(v, c_float) for v in planes], W, H, ctypes.byref(K),
                                 _p(T, c_float), dist_thresh, _p(out, c_double))
    return out


def solve(neq):
    """Spec a10: block elimination with 3x3 adjugates (oracle_solve)."""
    n = np.ascontiguousarray(neq, np.float64)
    xi = np.zeros(6, np.float64)
    st = load_library().oracle_solve(_p(n, c_double), _p(xi, c_double))
    return xi, st


class solve_mode:
    """Context manager selecting the solve oracle_align runs: ``with
    oracle.solve_mode("ldlt"): ...`` (the round 1-4 spec a10, for the
    fixtures' T64_ldlt poses); "block" is the default and what the kernels
    run."""

    def __init__(self, name):
        self.code = {"block": 0, "ldlt": 1}[name]

    def __enter__(self):
        self.old = load_library().oracle_set_solve(self.code)
        return self

    def __exit__(self, *exc):
        load_library().oracle_set_solve(self.old)


def solve_ldlt(neq):
    """The round 1-4 spec a10 (LDL^T), for the fixtures' T64_ldlt poses."""
    n = np.ascontiguousarray(neq, np.float64)
    xi = np.zeros(6, np.float64)
    st = load_library().oracle_solve_ldlt(_p(n, c_double), _p(xi, c_double))
    return xi, st


def se3_exp(xi):
    x = np.ascontiguousarray(xi, np.float64)
    E = np.zeros((4, 4), np.float64)
    load_library().oracle_se3_exp(_p(x, c_double), _p(E, c_double))
    return E


def align(src, dst, K=None, iters: int = 10, dist_thresh: float = 0.10, T_init=None):
    """-> (T64 [4,4], T32 [3,4] fp32, status, stats [iters, 2] (count, sum r^2))."""
    s = np.ascontiguousarray(src, np.int16)
    d = np.ascontiguousarray(dst, np.int16)
    H, W = s.shape
    K = K_of(K) if K is not None else viewer_K(W, H)
    T64 = np.zeros((4, 4), np.float64)
    T32 = np.zeros((3, 4), np.float32)
    stats = np.zeros((max(iters, 1), 2), np.float64)
    Ti = None if T_init is None else np.ascontiguousarray(T_init, np.float64)
    st = load_library().oracle_align(_p(s, c_int16), _p(d, c_int16), W, H, ctypes.byref(K),
                                     iters, dist_thresh, _p(Ti, c_double), _p(T64, c_double),
                                     _p(T32, c_float), _p(stats, c_double))
    return T64, T32, st, stats[:iters]


def align_batch(src, dst, K=None, iters: int = 10, dist_thresh: float = 0.10,
                n_threads: int = 0, want_stats: bool = False):
    """-> (T64 [n,4,4], status [n]) or, with want_stats, (T64, status, stats
    [n, iters, 2] = per-iteration (count, sum r^2))."""
    s = np.ascontiguousarray(src, np.int16)
    d = np.ascontiguousarray(dst, np.int16)
    n, H, W = s.shape
    K = K_of(K) if K is not None else viewer_K(W, H)
    T = np.zeros((n, 4, 4), np.float64)
    st = np.zeros(n, np.int32)
    stats = np.zeros((n, max(iters, 1), 2), np.float64) if want_stats else None
    load_library().oracle_align_batch(_p(s, c_int16), _p(d, c_int16), n, W, H, ctypes.byref(K),
                                      iters, dist_thresh, _p(T, c_double), _p(st, c_int32),
                                      _p(stats, c_double), n_threads)
    if want_stats:
        return T, st, stats[:, :iters]
    return T, st


def max_threads() -> int:
    return load_library().oracle_max_threads()
