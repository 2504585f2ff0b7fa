"""Randomised parity of the HIP path against the C oracle (SURVEY §8 c):
random poses and scenes beyond the fixed cases of test_gpu_parity.py.

- Association (spec a7) bit-exact and the normal equations (a8-a9) within
  rel 1e-11, for 96 random (pair, pose) draws: rotations up to 30 degrees
  about a random axis, translations up to 20 cm, both noise models.
- Full aligns from random non-identity initial poses through both kernel
  paths (the persistent k_icp for a 64-pair batch, k_icp_coop one pair at a
  time): every fp64 pose within 1e-5 of the oracle's from the same T_init,
  same status.
The draws are seeded (reproducible); the oracle runs on the host (a few
seconds)."""
import numpy as np
import pytest
import torch

import oracle
import youth_icp
import youth_synth
from conftest import oracle_like

pytestmark = pytest.mark.gpu
POSE_TOL = 1e-5


def _pose(rng, max_deg, max_t):
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    th = np.deg2rad(rng.uniform(0, max_deg))
    Kx = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    T = np.eye(4)
    T[:3, :3] = np.eye(3) + np.sin(th) * Kx + (1 - np.cos(th)) * Kx @ Kx
    T[:3, 3] = rng.uniform(-max_t, max_t, size=3)
    return T


def _pose_err(a, b):
    return float(np.abs(np.asarray(a)[:3] - np.asarray(b)[:3]).max())


def test_association_and_sums_random_poses():
    rng = np.random.default_rng(0x5EED)
    K = oracle.viewer_K(640, 480)
    with youth_icp.IcpContext(640, 480, 2) as ctx:
        for draw in range(96):
            flags = youth_synth.SURVEY_FLAGS if draw % 3 == 0 else 0
            src, dst, _ = youth_synth.pairs(1000 + draw, 1, 640, 480, flags=flags)
            T32 = _pose(rng, 30.0 if draw % 2 else 5.0, 0.20)[:3].astype(np.float32)
            g_idx, g_neq = ctx.reduce(src[0], dst[0], T32)
            o_idx = oracle.associate(src[0], dst[0], T32, K)
            with oracle_like(ctx):
                o_neq = oracle.reduce(src[0], dst[0], T32, K)
            assert np.array_equal(g_idx, o_idx), draw
            np.testing.assert_allclose(g_neq, o_neq, rtol=1e-11, atol=1e-9, err_msg=str(draw))


def test_align_from_random_initial_poses_both_paths():
    rng = np.random.default_rng(0xF022)
    n = 64
    src, dst, _ = youth_synth.pairs(2000, n, 640, 480)
    T_init = np.stack([_pose(rng, 2.0, 0.02) for _ in range(n)])
    want = [oracle.align(src[p], dst[p], iters=10, T_init=T_init[p]) for p in range(n)]
    ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
    N = 640 * 480
    with youth_icp.IcpContext(640, 480, n) as ctx:
        ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n, T_init=T_init)
        T64, _, st = ctx.get_poses(n)
        assert ctx.get_plan()["kernel"] != "k_icp_coop"
        for p in range(n):
            assert st[p] == want[p][2] and _pose_err(T64[p], want[p][0]) <= POSE_TOL, p
        for p in range(0, n, 8):           # one pair per call: the cooperative kernel
            ctx.align_pairs_device(ds.data_ptr() + p * N * 2, dd.data_ptr() + p * N * 2, 1,
                                   T_init=T_init[p])
            T1, _, s1 = ctx.get_poses(1)
            assert ctx.get_plan()["kernel"] == "k_icp_coop"
            assert s1[0] == want[p][2] and _pose_err(T1[0], want[p][0]) <= POSE_TOL, p


def _rand_intrinsics(rng, W, H):
    """Intrinsics away from the viewer's defaults: focal lengths 300-900 px
    with fractional parts, a principal point anywhere in the middle 80 % of
    the frame (off-centre ones exercise the aligned loop's exactness guard),
    depth scale 1000 / 5000 / 1000.5 (the fast-division verification decides
    per context)."""
    return dict(fx=float(np.float32(rng.uniform(300, 900))), fy=float(np.float32(rng.uniform(300, 900))),
                cx=float(np.float32(rng.uniform(0.1, 0.9) * W)),
                cy=float(np.float32(rng.uniform(0.1, 0.9) * H)),
                ds=float(rng.choice([1000.0, 5000.0, 1000.5])))


@pytest.mark.parametrize("W,H", [(640, 480), (162, 122)])
def test_random_intrinsics_every_path(W, H, monkeypatch):
    """Random intrinsics (6 draws per size; 162 x 122 has W % 4 == 2, the
    unaligned loops): the stage kernel's association bit-exact and its sums
    within rel 1e-11 of the oracle in the same reduction; full aligns through
    the persistent kernel (4 pairs) and k_icp_coop (1 pair) with per-iteration
    counts equal to the oracle's and poses within 1e-9 of it."""
    rng = np.random.default_rng(0x1F0C + W)
    src, dst, _ = youth_synth.pairs(95, 4, W, H)
    ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
    torch.cuda.synchronize()
    iters = 6
    for draw in range(6):
        k = _rand_intrinsics(rng, W, H)
        K = youth_icp.default_intrinsics(W, H)
        Ko = oracle.viewer_K(W, H)
        for obj in (K, Ko):
            obj.fx, obj.fy, obj.cx, obj.cy, obj.depth_scale = k["fx"], k["fy"], k["cx"], k["cy"], k["ds"]
        T32 = _pose(rng, 2.0, 0.02)[:3].astype(np.float32)
        with youth_icp.IcpContext(W, H, 4, K=K) as ctx:
            g_idx, g_neq = ctx.reduce(src[0], dst[0], T32)
            with oracle_like(ctx):
                o_neq = oracle.reduce(src[0], dst[0], T32, Ko)
        assert np.array_equal(g_idx, oracle.associate(src[0], dst[0], T32, Ko)), (draw, k)
        assert g_neq[28] == o_neq[28], (draw, k)
        np.testing.assert_allclose(g_neq, o_neq, rtol=1e-11, atol=1e-9, err_msg=str((draw, k)))
        for n, env in ((4, "1"), (1, None)):
            if env:
                monkeypatch.setenv("YOUTH_ICP_NO_COOP", env)
            else:
                monkeypatch.delenv("YOUTH_ICP_NO_COOP", raising=False)
            with youth_icp.IcpContext(W, H, max(n, 2), K=K, iters=iters) as ctx:
                ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n)
                ctx.sync()
                T64, _, st = ctx.get_poses(n)
                cnt, _ = ctx.get_stats(n, iters)
                plan = ctx.get_plan()
                with oracle_like(ctx):
                    To, sto, stats = oracle.align_batch(src[:n], dst[:n], K=Ko, iters=iters,
                                                        n_threads=n, want_stats=True)
            assert np.array_equal(st, sto), (draw, k, plan["kernel"])
            assert np.array_equal(cnt, stats[..., 0]), (draw, k, plan["kernel"],
                                                        np.argwhere(cnt != stats[..., 0])[:4])
            err = float(np.abs(np.asarray(T64)[..., :3, :4] - np.asarray(To)[..., :3, :4]).max())
            assert err <= 1e-9, (draw, k, plan["kernel"], err)


@pytest.mark.parametrize("W,H", [(4, 3), (5, 4), (8, 8), (31, 7), (65, 3), (3, 65), (130, 66)])
def test_tiny_and_ragged_frames_every_path(W, H, monkeypatch):
    """Frames down to 4 x 3 and single-tile-row / single-column shapes (the
    prep tiles, the halo's edge words and the lane partitions all clipped):
    the stage kernel's association bit-exact and sums within rel 1e-11 of the
    oracle; full aligns through the persistent kernel (2 pairs) and
    k_icp_coop (1 pair) with equal per-iteration counts and statuses, poses
    within 1e-9 + 4e-16 cond(A): the GPU and the oracle add the same exact
    products in different fp64 orders (~1e-16 relative), and the one-row /
    one-column frames' normal equations have cond(A) up to ~3e8, which the
    solve (any exact solve: round 1-4's LDL^T was as sensitive) amplifies.
    cond(A) is taken at the oracle's final pose."""
    rng = np.random.default_rng(0x7111 + W * 131 + H)
    src, dst, _ = youth_synth.pairs(96, 2, W, H)
    ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
    torch.cuda.synchronize()
    Ko = oracle.viewer_K(W, H)
    iters = 5
    T32 = _pose(rng, 1.0, 0.01)[:3].astype(np.float32)
    with youth_icp.IcpContext(W, H, 2) as ctx:
        g_idx, g_neq = ctx.reduce(src[0], dst[0], T32)
        with oracle_like(ctx):
            o_neq = oracle.reduce(src[0], dst[0], T32, Ko)
    assert np.array_equal(g_idx, oracle.associate(src[0], dst[0], T32, Ko))
    assert g_neq[28] == o_neq[28]
    np.testing.assert_allclose(g_neq, o_neq, rtol=1e-11, atol=1e-9)
    for n, env in ((2, "1"), (1, None)):
        if env:
            monkeypatch.setenv("YOUTH_ICP_NO_COOP", env)
        else:
            monkeypatch.delenv("YOUTH_ICP_NO_COOP", raising=False)
        with youth_icp.IcpContext(W, H, 2, iters=iters) as ctx:
            ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n)
            ctx.sync()
            T64, _, st = ctx.get_poses(n)
            cnt, _ = ctx.get_stats(n, iters)
            plan = ctx.get_plan()
            with oracle_like(ctx):
                To, sto, stats = oracle.align_batch(src[:n], dst[:n], K=Ko, iters=iters,
                                                    n_threads=n, want_stats=True)
        assert np.array_equal(st, sto), (plan["kernel"], st, sto)
        assert np.array_equal(cnt, stats[..., 0]), (plan["kernel"], cnt, stats[..., 0])
        for p in np.flatnonzero(st == 0):
            err = float(np.abs(np.asarray(T64)[p][:3, :4] - np.asarray(To)[p][:3, :4]).max())
            neq = oracle.reduce(src[p], dst[p], np.asarray(To)[p][:3].astype(np.float32), Ko)
            A = np.zeros((6, 6))
            A[np.triu_indices(6)] = neq[:21]
            A = A + np.triu(A, 1).T
            bound = 1e-9 + 4e-16 * np.linalg.cond(A)
            assert err <= bound, (plan["kernel"], p, err, bound)
