"""GPU parity of the viewer point list (include/youth_viewer.h):
the HIP builder against the C oracle's restatement of
viewerModule.c:336-357 (itself pinned to the reference loop and the §4 KAT in
tests/test_oracle.py).  Bar: bit-exact vertices (fp32 bit patterns, -0.0
included) and identical counts — the list is integer/byte work plus IEEE
quotients, so nothing is tolerance-based."""
import numpy as np
import pytest
import torch

import oracle
import youth_icp
import youth_synth
import youth_viewer

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _frame(W, H, seed, holes=0.1, negative=True):
    rng = np.random.default_rng(seed)
    lo = -500 if negative else 0
    depth = rng.integers(lo, 32768, size=(H, W)).astype(np.int16)
    depth[rng.random((H, W)) < holes] = 0
    rgb = rng.integers(0, 256, size=(H, W, 3)).astype(np.uint8)
    return depth, rgb


def test_cloud_640x480_synthetic_scene_bit_exact():
    src, _, _ = youth_synth.pairs(0, 1)
    depth = src[0]
    rgb = np.random.default_rng(7).integers(0, 256, size=depth.shape + (3,)).astype(np.uint8)
    with youth_viewer.CloudBuilder(640, 480) as cb:
        got = cb.build(depth, rgb)
    want = oracle.viewer_cloud(depth, rgb)
    assert got.shape == want.shape and want.shape[0] == int((depth > 0).sum())
    assert np.array_equal(_bits(got), _bits(want))


@pytest.mark.parametrize("W,H", [(97, 53), (640, 480), (5, 7), (1, 1), (1, 300), (2049, 3)])
def test_cloud_ragged_and_narrow_frames(W, H):
    """Odd sizes run the scalar-load path; W < 8 wraps rows inside one thread's
    8 pixels; 2049-wide rows straddle tiles."""
    depth, rgb = _frame(W, H, W * 7 + H)
    with youth_viewer.CloudBuilder(W, H) as cb:
        got = cb.build(depth, rgb)
        got_nc = cb.build(depth, None)
    want = oracle.viewer_cloud(depth, rgb)
    assert np.array_equal(_bits(got), _bits(want))
    assert np.array_equal(_bits(got_nc), _bits(oracle.viewer_cloud(depth, None)))


def test_cloud_empty_full_and_negative_frames():
    W, H = 64, 48
    with youth_viewer.CloudBuilder(W, H) as cb:
        assert cb.build(np.zeros((H, W), np.int16)).shape == (0, 6)
        assert cb.build(np.full((H, W), -1, np.int16)).shape == (0, 6)   # d > 0 only
        full = np.full((H, W), 32767, np.int16)
        got = cb.build(full)
        assert got.shape == (W * H, 6)
        assert np.array_equal(_bits(got), _bits(oracle.viewer_cloud(full)))
        # a smaller frame through the same builder
        d, c = _frame(33, 17, 5)
        assert np.array_equal(_bits(cb.build(d, c)), _bits(oracle.viewer_cloud(d, c)))


def test_cloud_explicit_intrinsics():
    W, H = 160, 120
    depth, rgb = _frame(W, H, 11, negative=False)
    K = youth_icp.Intrinsics(525.0, 523.5, 81.25, 59.5, 5000.0)
    with youth_viewer.CloudBuilder(W, H) as cb:
        got = cb.build(depth, rgb, K)
    want = oracle.viewer_cloud(depth, rgb, K.as_tuple())
    assert np.array_equal(_bits(got), _bits(want))


@pytest.mark.parametrize("px", [8, 4])
@pytest.mark.parametrize("offset", [0, 1])
def test_cloud_device_batch(offset, px, monkeypatch):
    """Device API over a stacked batch on a torch stream; offset 1 misaligns the
    depth/colour pointers (scalar-load path) and the output run alignment; both
    tile widths (pixels per thread, read at builder creation)."""
    monkeypatch.setenv("YOUTH_CLOUD_PX", str(px))
    W, H, n = 320, 240, 5
    frames = [_frame(W, H, 100 + f) for f in range(n)]
    d_all = torch.zeros(n * H * W + offset, dtype=torch.int16, device="cuda")
    c_all = torch.zeros(n * H * W * 3 + offset, dtype=torch.uint8, device="cuda")
    d_all[offset:] = torch.from_numpy(np.stack([f[0] for f in frames]).reshape(-1)).cuda()
    c_all[offset:] = torch.from_numpy(np.stack([f[1] for f in frames]).reshape(-1)).cuda()
    verts = torch.zeros((n, H * W, 6), dtype=torch.float32, device="cuda")
    counts = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    with youth_viewer.CloudBuilder(W, H, max_frames=n) as cb:
        cb.build_device(d_all.data_ptr() + offset * 2, c_all.data_ptr() + offset, n, W, H,
                        verts.data_ptr(), counts.data_ptr(), stream=stream)
        torch.cuda.synchronize()
    counts = counts.cpu().numpy()
    verts = verts.cpu().numpy()
    for f, (d, c) in enumerate(frames):
        want = oracle.viewer_cloud(d, c)
        assert counts[f] == want.shape[0]
        assert np.array_equal(_bits(verts[f, : counts[f]]), _bits(want))


def _pose(rng, big=False):
    """A random camera -> world pose, row-major 3x4 fp32."""
    w = rng.normal(size=3) * (1.0 if big else 0.05)
    th = np.linalg.norm(w)
    Kx = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]]) / max(th, 1e-12)
    R = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
    t = rng.normal(size=3) * (5.0 if big else 0.1)
    return np.hstack([R, t[:, None]]).astype(np.float32)


@pytest.mark.parametrize("offset", [0, 1])
def test_cloud_world_frame_batch(offset):
    """youth_cloud_build_device_posed: every frame's points moved by its own
    camera -> world pose (the tracker's trajectory), then the display flip;
    bit-exact against the oracle with the same fma chains, small and large
    poses, aligned and misaligned inputs; a null pose array is the camera
    frame list."""
    W, H, n = 320, 240, 4
    rng = np.random.default_rng(5)
    frames = [_frame(W, H, 200 + f) for f in range(n)]
    T = np.stack([_pose(rng, big=f % 2 == 1) for f in range(n)])
    d_all = torch.zeros(n * H * W + offset, dtype=torch.int16, device="cuda")
    c_all = torch.zeros(n * H * W * 3 + offset, dtype=torch.uint8, device="cuda")
    d_all[offset:] = torch.from_numpy(np.stack([f[0] for f in frames]).reshape(-1)).cuda()
    c_all[offset:] = torch.from_numpy(np.stack([f[1] for f in frames]).reshape(-1)).cuda()
    d_T = torch.from_numpy(T.reshape(n, 12)).cuda()
    verts = torch.zeros((n, H * W, 6), dtype=torch.float32, device="cuda")
    counts = torch.full((n,), -1, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    with youth_viewer.CloudBuilder(W, H, max_frames=n) as cb:
        cb.build_device_posed(d_all.data_ptr() + offset * 2, c_all.data_ptr() + offset, n, W, H,
                              d_T.data_ptr(), verts.data_ptr(), counts.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        got = verts.cpu().numpy(), counts.cpu().numpy()
        cb.build_device_posed(d_all.data_ptr() + offset * 2, c_all.data_ptr() + offset, n, W, H,
                              0, verts.data_ptr(), counts.data_ptr(), stream=stream)
        torch.cuda.synchronize()
        cam = verts.cpu().numpy()
    for f, (d, c) in enumerate(frames):
        want = oracle.viewer_cloud(d, c, T_world=T[f])
        assert got[1][f] == want.shape[0]
        assert np.array_equal(_bits(got[0][f, : got[1][f]]), _bits(want))
        assert np.array_equal(_bits(cam[f, : got[1][f]]), _bits(oracle.viewer_cloud(d, c)))


def test_cloud_rejects_bad_arguments():
    with youth_viewer.CloudBuilder(64, 48, max_frames=2) as cb:
        with pytest.raises(youth_icp.IcpError):
            cb.build(np.zeros((49, 64), np.int16))      # taller than the builder
        with pytest.raises(youth_icp.IcpError):
            cb.build_device(0, 0, 1, 64, 48, 0, 0)       # null device pointers
    with pytest.raises(youth_icp.IcpError):
        youth_viewer.CloudBuilder(20000, 2)
