"""GPU tests of the C-ABI's argument checks with a live context (youth_icp.h):
every documented bad argument is refused with YOUTH_EINVAL before anything is
launched, the error text names the call, and the context aligns bit for bit
as before afterwards.  The NULL-context sweep is CPU-side (test_abi.py)."""
import ctypes

import numpy as np
import pytest
import torch

import youth_icp
import youth_synth

pytestmark = pytest.mark.gpu

E = youth_icp.YOUTH_EINVAL


def test_create_refuses_bad_sizes_and_devices():
    lib = youth_icp.load_library()
    for W, H, mf in ((2, 480, 2), (640, 2, 2), (16385, 8, 2), (8, 16385, 2),
                     (16384, 4097, 2), (640, 480, 1), (640, 480, 0), (-640, 480, 2)):
        assert not lib.youth_icp_create(0, W, H, mf, None, None), (W, H, mf)
        assert b"bad size" in lib.youth_icp_last_error()
    assert not lib.youth_icp_create(lib.youth_icp_device_count(), 64, 48, 2, None, None)
    assert b"no HIP device" in lib.youth_icp_last_error()
    assert not lib.youth_icp_create(-1, 64, 48, 2, None, None)


def test_bad_arguments_refused_context_unchanged():
    W, H, n = 160, 120, 4
    src, dst, _ = youth_synth.pairs(0, n, W, H)
    ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
    seq = torch.from_numpy(np.concatenate([src, dst[-1:]])).cuda()
    ctx = youth_icp.IcpContext(W, H, n)
    lib, h = ctx._lib, ctx.handle
    ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n)
    T0, _, st0 = ctx.get_poses(n)
    assert (st0 == 0).all()

    P16 = ctypes.POINTER(ctypes.c_int16)
    host = np.zeros(W * H, np.int16)
    hp = host.ctypes.data_as(P16)
    T = np.zeros(16, np.float64)
    Tp = T.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    has = ctypes.c_int()
    ms, cnt = ctypes.c_double(), ctypes.c_int()
    calls = {
        "align_pairs null src": lambda: lib.youth_icp_align_pairs_device(
            h, None, dd.data_ptr(), 1, None, None, None),
        "align_pairs null dst": lambda: lib.youth_icp_align_pairs_device(
            h, ds.data_ptr(), None, 1, None, None, None),
        "align_pairs 0 pairs": lambda: lib.youth_icp_align_pairs_device(
            h, ds.data_ptr(), dd.data_ptr(), 0, None, None, None),
        "align_pairs -1 pairs": lambda: lib.youth_icp_align_pairs_device(
            h, ds.data_ptr(), dd.data_ptr(), -1, None, None, None),
        "align_pairs > max_frames": lambda: lib.youth_icp_align_pairs_device(
            h, ds.data_ptr(), dd.data_ptr(), n + 1, None, None, None),
        "align_sequence 1 frame": lambda: lib.youth_icp_align_sequence_device(
            h, seq.data_ptr(), 1, None, None),
        "align_sequence > max_frames": lambda: lib.youth_icp_align_sequence_device(
            h, seq.data_ptr(), n + 2, None, None),
        "get_poses > max_frames": lambda: lib.youth_icp_get_poses(h, n + 1, None, None, None),
        "get_poses -1": lambda: lib.youth_icp_get_poses(h, -1, None, None, None),
        "get_stats other iters": lambda: lib.youth_icp_get_stats(h, n, 11, None, None),
        "get_timing kind 3": lambda: lib.youth_icp_get_timing(h, 3, ctypes.byref(ms),
                                                              ctypes.byref(cnt)),
        "set_spec 7": lambda: lib.youth_icp_set_spec(h, 7),
        "set_reduce 9": lambda: lib.youth_icp_set_reduce(h, 9),
        "set_concurrency 0": lambda: lib.youth_icp_set_concurrency(h, 0),
        "set_concurrency > max": lambda: lib.youth_icp_set_concurrency(h, 99),
        "track_set_batch 0": lambda: lib.youth_icp_track_set_batch(h, 0),
        "track_set_batch > max": lambda: lib.youth_icp_track_set_batch(h, 99),
        "track_collect nothing in flight": lambda: lib.youth_icp_track_collect(
            h, Tp, ctypes.byref(has)),
        "track_collect null T": lambda: lib.youth_icp_track_collect(h, None, ctypes.byref(has)),
        "track_submit null frame": lambda: lib.youth_icp_track_submit(h, None, None),
        "track_submit_batch 0 frames": lambda: lib.youth_icp_track_submit_batch(h, hp, 0),
        "track_submit_batch > max": lambda: lib.youth_icp_track_submit_batch(h, hp, 99),
        "track_submit_pinned null list": lambda: lib.youth_icp_track_submit_pinned(h, None, 1),
        "track_submit_pinned null frame": lambda: lib.youth_icp_track_submit_pinned(
            h, (P16 * 1)(), 1),
        "track_frame null T_rel": lambda: lib.youth_icp_track_frame(h, hp, None, None, None),
        "track_realign null ref": lambda: lib.youth_icp_track_realign(h, None, hp, None, Tp),
        "track_host_sequence -1 frames": lambda: lib.youth_icp_track_host_sequence(
            h, hp, -1, Tp, None),
    }
    for name, call in calls.items():
        rc = call()
        assert rc == E, (name, rc)
        assert lib.youth_icp_last_error(), name
    # still the same context: same plan, same spec / reduction, bit-identical poses
    assert ctx.spec == youth_icp.SPEC_SURVEY
    assert lib.youth_icp_track_pending(h) == 0
    ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n)
    T1, _, st1 = ctx.get_poses(n)
    assert (st1 == 0).all() and np.array_equal(T0, T1)
    ctx.close()
