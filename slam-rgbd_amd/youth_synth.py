"""ctypes wrapper of the synthetic depth source (include/youth_synth.h).

Stands in for the reference's Astra SensorModule (sensorModule.c:69-264):
produces int16 [H][W] millimetre depth frames, 0 = invalid.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_int, c_int16, c_uint64

import numpy as np

from youth_icp import HERE, Intrinsics

LIB_PATH = os.path.join(HERE, "libyouth_synth.so")
PAIR_SEED = 0x5EED0000
SEQ_SEED = 0x5EED1000
NOISE = 1
HOLES = 2
NOISE_SURVEY = 4   # SURVEY §8d sigma = 1.5 mm * Z^2 (instead of NOISE's 0.25)
SURVEY_FLAGS = NOISE_SURVEY | HOLES
DEFAULT_FLAGS = NOISE | HOLES

_lib = None


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise OSError(f"{path} not built: run `make -C {HERE}`")
    lib = ctypes.CDLL(path)
    P16, PD, PK = POINTER(c_int16), POINTER(c_double), POINTER(Intrinsics)
    lib.youth_synth_render.argtypes = [PD, c_int, c_int, PK, c_uint64, c_int, P16]
    lib.youth_synth_render.restype = None
    lib.youth_synth_pair.argtypes = [c_uint64, c_int, c_int, PK, c_int, P16, P16, PD]
    lib.youth_synth_pair.restype = None
    lib.youth_synth_pairs.argtypes = [c_uint64, c_int, c_int, c_int, c_int, PK, c_int, P16, P16,
                                      PD]
    lib.youth_synth_pairs.restype = None
    lib.youth_synth_sequence.argtypes = [c_uint64, c_int, c_int, c_int, c_int, PK, c_int, P16,
                                         PD]
    lib.youth_synth_sequence.restype = None
    _lib = lib
    return lib


def viewer_intrinsics(width: int, height: int) -> Intrinsics:
    """viewerModule.c:343-345 convention without loading the HIP library."""
    return Intrinsics(570.3, 570.3, float(width // 2), float(height // 2), 1000.0)


def _p(a, t):
    return a.ctypes.data_as(POINTER(t))


def pairs(first_index: int, n: int, width: int = 640, height: int = 480, K=None,
          flags: int = DEFAULT_FLAGS, base_seed: int = PAIR_SEED):
    """n pairs with seeds base_seed + first_index + p -> (src, dst, T_gt)."""
    K = K if K is not None else viewer_intrinsics(width, height)
    src = np.zeros((n, height, width), np.int16)
    dst = np.zeros((n, height, width), np.int16)
    T = np.zeros((n, 4, 4), np.float64)
    load_library().youth_synth_pairs(base_seed, first_index, n, width, height,
                                     ctypes.byref(K), flags, _p(src, c_int16),
                                     _p(dst, c_int16), _p(T, c_double))
    return src, dst, T


def sequence(first_frame: int, n: int, width: int = 640, height: int = 480, K=None,
             flags: int = DEFAULT_FLAGS, seed: int = SEQ_SEED):
    """Frames [first_frame, first_frame+n) of the synthetic sequence -> (frames, T_wc)."""
    K = K if K is not None else viewer_intrinsics(width, height)
    frames = np.zeros((n, height, width), np.int16)
    T = np.zeros((n, 4, 4), np.float64)
    load_library().youth_synth_sequence(seed, first_frame, n, width, height, ctypes.byref(K),
                                        flags, _p(frames, c_int16), _p(T, c_double))
    return frames, T


def render(T_wc: np.ndarray, width: int, height: int, K=None, noise_seed: int = 0,
           flags: int = 0):
    K = K if K is not None else viewer_intrinsics(width, height)
    T = np.ascontiguousarray(T_wc, np.float64)
    out = np.zeros((height, width), np.int16)
    load_library().youth_synth_render(_p(T, c_double), width, height, ctypes.byref(K),
                                      noise_seed, flags, _p(out, c_int16))
    return out
