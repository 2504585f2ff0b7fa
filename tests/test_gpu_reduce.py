"""GPU parity of spec a9's two reductions (youth_icp_set_reduce), each against
the oracle run in the same reduction:

  * YOUTH_REDUCE_EXACT (the default since round 5): every product of two
    fp32 values exact in fp64, accumulated in fp64.  It does not depend on
    the launch: the same pair in a 512-pair batch, a 64-pair shard or a
    single-pair cooperative launch gives the same pose up to fp64 summation
    order, within 1e-5 of the CPU oracle at SURVEY §8d noise
    (test_default_reduction_is_launch_independent_at_survey_noise);
  * YOUTH_REDUCE_LANE32 (opt-in): "fp32 lanes -> fp64 finalize".  Every lane
    sums its matched pixels' 28 products in fp32 (one fma each) over its
    whole share of an iteration; the lane sums are converted once and added
    in fp64.  The oracle restates it given the launch's lane partition
    (youth_icp_get_lanes -> oracle_set_reduce): each lane's fp32 sums are
    then the GPU's bit for bit, so the 28 sums differ only by the fp64 order
    of the lane additions (rel 1e-11 here, observed ~1e-15), correspondence
    counts are equal at every iteration and poses agree to ~1e-13.  Against
    the exact reduction its poses move by the fp32 rounding of the lane sums
    (<= 1e-6 on the cases below; up to ~5e-5 at §8d noise).
"""
import os

import numpy as np
import pytest
import torch

import oracle
import youth_icp
import youth_synth
from conftest import lanes_of, oracle_like

pytestmark = pytest.mark.gpu
POSE_TOL = 1e-5
SAME_VARIANT_TOL = 1e-9     # poses vs the oracle in the same reduction (observed ~1e-13)


def _err(a, b):
    return float(np.abs(np.asarray(a)[..., :3, :4] - np.asarray(b)[..., :3, :4]).max())


def test_reduce_selection_api(monkeypatch):
    with youth_icp.IcpContext(64, 48, 2) as ctx:
        assert ctx.reduction == youth_icp.REDUCE_EXACT           # the default
        with pytest.raises(youth_icp.IcpError):
            ctx.lanes()                                          # no align has run
        with pytest.raises(youth_icp.IcpError):
            ctx.reduction = 5
        assert ctx.reduction == youth_icp.REDUCE_EXACT
        ctx.reduction = "lane32"
        assert ctx.reduction == youth_icp.REDUCE_LANE32
    monkeypatch.setenv("YOUTH_ICP_REDUCE", "exact")
    with youth_icp.IcpContext(64, 48, 2) as ctx:
        assert ctx.reduction == youth_icp.REDUCE_EXACT
    monkeypatch.setenv("YOUTH_ICP_REDUCE", "lane32")
    with youth_icp.IcpContext(64, 48, 2) as ctx:
        assert ctx.reduction == youth_icp.REDUCE_LANE32


@pytest.mark.parametrize("W,H", [(640, 480), (97, 53), (160, 120)])
def test_lane32_sums_match_oracle(W, H):
    """k_reduce (the stage kernel; W % 4 != 0 takes the unaligned depth path)
    at the identity and 8 random poses: indices bit-exact, the 28 sums within
    rel 1e-11 of the oracle's lane32 restatement over the reported partition,
    the count exact; and the two reductions within the fp32 rounding of each
    other (rel 1e-4 of the largest sum)."""
    rng = np.random.default_rng(0x1A9E)
    src, dst, _ = youth_synth.pairs(70, 1, W, H)
    K = oracle.viewer_K(W, H)
    with youth_icp.IcpContext(W, H, 2) as ctx:
        for draw in range(9):
            if draw == 0:
                T32 = np.eye(4, dtype=np.float32)[:3]
            else:
                axis = rng.normal(size=3)
                axis /= np.linalg.norm(axis)
                Tr = oracle.se3_exp(np.r_[axis * np.deg2rad(rng.uniform(0, 4)),
                                          rng.uniform(-0.03, 0.03, 3)])
                T32 = Tr[:3].astype(np.float32)
            ctx.reduction = "lane32"
            g_idx, g_neq = ctx.reduce(src[0], dst[0], T32)
            kind, chunk, threads, npx = ctx.lanes()
            assert kind == youth_icp.LANES_STRIDED and threads == 256 and chunk % 1024 == 0
            with oracle_like(ctx):
                o_neq = oracle.reduce(src[0], dst[0], T32, K)
            assert np.array_equal(g_idx, oracle.associate(src[0], dst[0], T32, K)), draw
            assert g_neq[28] == o_neq[28], draw
            np.testing.assert_allclose(g_neq, o_neq, rtol=1e-11, atol=1e-9, err_msg=str(draw))
            ctx.reduction = "exact"
            _, e_neq = ctx.reduce(src[0], dst[0], T32)
            e_o = oracle.reduce(src[0], dst[0], T32, K)
            np.testing.assert_allclose(e_neq, e_o, rtol=1e-11, atol=1e-9, err_msg=str(draw))
            scale = np.abs(e_neq[:28]).max()
            assert np.abs(g_neq[:28] - e_neq[:28]).max() <= 1e-4 * scale, draw


PATHS = {
    # name: (env, W, H, iters, n, expected kernel)
    "coop_tile": ({}, 640, 480, 10, 1, "k_icp_coop"),
    "coop_contiguous": ({"YOUTH_ICP_COOP_TILE_SRC": "0"}, 640, 480, 10, 1, "k_icp_coop"),
    "coop_tall_1280x960": ({}, 1280, 960, 20, 1, "k_icp_coop"),
    "coop_8_pairs": ({}, 640, 480, 10, 8, "k_icp_coop"),
    "persistent_64": ({}, 640, 480, 10, 64, "k_prep + k_icp"),
    "persistent_97x53": ({"YOUTH_ICP_NO_COOP": "1"}, 97, 53, 10, 5, "k_prep + k_icp"),
    "per_iteration": ({"YOUTH_ICP_NO_COOP": "1", "YOUTH_ICP_NO_PERSISTENT": "1"}, 640, 480,
                      10, 3, "k_prep + k_init + k_reduce"),
}


@pytest.mark.parametrize("path", sorted(PATHS))
def test_every_kernel_path_in_both_reductions(path, monkeypatch):
    """Each kernel path of an align (its lane partition: strided chunks,
    contiguous or tile-shaped coop chunks, the 64x80-tile coop kernel) in
    both reductions: counts per iteration equal to the oracle's in the same
    reduction, poses within 1e-9 of it, and within 1e-5 of the exact
    oracle (the other reduction)."""
    env, W, H, iters, n, kern = PATHS[path]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    src, dst, _ = youth_synth.pairs(90, n, W, H)
    K = youth_icp.default_intrinsics(W, H)
    ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
    torch.cuda.synchronize()
    exact_T = None
    for red in ("exact", "lane32"):
        with youth_icp.IcpContext(W, H, max(n, 2), K=K, iters=iters, reduction=red) as ctx:
            ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n)
            ctx.sync()
            T64, _, st = ctx.get_poses(n)
            cnt, r2 = ctx.get_stats(n, iters)
            plan = ctx.get_plan()
            lanes = lanes_of(ctx)
        assert plan["kernel"].startswith(kern), plan
        with oracle_like(lanes):
            To, sto, stats = oracle.align_batch(src, dst, K=oracle.viewer_K(W, H), iters=iters,
                                                n_threads=min(n, 16), want_stats=True)
        assert np.array_equal(st, sto) and not st.any(), red
        assert np.array_equal(cnt, stats[..., 0]), (red, np.argwhere(cnt != stats[..., 0])[:4])
        np.testing.assert_allclose(r2, stats[..., 1], rtol=1e-6)
        assert _err(T64, To) <= SAME_VARIANT_TOL, (red, _err(T64, To))
        if red == "exact":
            exact_T = To
        else:
            assert _err(T64, exact_T) <= POSE_TOL, _err(T64, exact_T)


def test_tracker_lane32_matches_oracle():
    """The tracker (k_icp_coop with the fused next-reference prep) in the
    lane32 reduction: every relative pose within 1e-9 of the oracle's lane32
    restatement over the tracker's own partition, status equal."""
    frames, _ = youth_synth.sequence(13, 6)
    with youth_icp.IcpContext(640, 480, 2, reduction="lane32") as ctx:
        got = [ctx.track_frame(f) for f in frames]
        lanes = lanes_of(ctx)
    assert lanes is not None and lanes[0] in (youth_icp.LANES_COOP, youth_icp.LANES_COOP_TILE)
    with oracle_like(lanes):
        for k in range(1, len(frames)):
            T64, _, sto, _ = oracle.align(frames[k], frames[k - 1])
            assert got[k][2] and got[k][1] == sto
            assert _err(got[k][0], T64) <= SAME_VARIANT_TOL, (k, _err(got[k][0], T64))


def test_oracle_reduction_restored():
    """oracle_like leaves the oracle in the mode it found (tests share the
    process-wide oracle)."""
    assert oracle.get_reduce() == oracle.REDUCE_EXACT
    with oracle.reduction("lane32", (youth_icp.LANES_STRIDED, 2048, 256, 0)):
        assert oracle.get_reduce() == oracle.REDUCE_LANE32
    assert oracle.get_reduce() == oracle.REDUCE_EXACT


def test_off_centre_principal_point(monkeypatch):
    """k_icp's aligned pixel loop forms a lane's centred columns as
    ((float)u0 - cx) + q, which equals the spec's (float)u - cx only while the
    difference keeps cx's ulp.  For a principal point far to one side (cx =
    20.9316 at W = 640: 9 columns round differently) the context takes the
    unaligned loop instead: per-iteration counts equal to the oracle's and
    poses within 1e-9 of it, on the persistent kernel and the stage kernel."""
    W, H, n, iters = 640, 480, 4, 10
    cols = np.arange(W)
    cx = np.float32(20.9316)
    assert ((np.float32(cols) - cx) != ((np.float32(cols & ~3) - cx) + np.float32(cols & 3))).any()
    monkeypatch.setenv("YOUTH_ICP_NO_COOP", "1")
    src, dst, _ = youth_synth.pairs(91, n, W, H)
    K = youth_icp.default_intrinsics(W, H)
    K.cx = float(cx)
    Ko = oracle.viewer_K(W, H)
    Ko.cx = float(cx)
    ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
    torch.cuda.synchronize()
    with youth_icp.IcpContext(W, H, n, K=K, iters=iters) as ctx:
        ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n)
        ctx.sync()
        T64, _, st = ctx.get_poses(n)
        cnt, _ = ctx.get_stats(n, iters)
        lanes = lanes_of(ctx)
        T32 = np.asarray(T64[0], np.float32)[:3]
        g_idx, g_neq = ctx.reduce(src[0], dst[0], T32)
        rl = lanes_of(ctx)
    with oracle_like(lanes):
        To, sto, stats = oracle.align_batch(src, dst, K=Ko, iters=iters, n_threads=n,
                                            want_stats=True)
    assert np.array_equal(st, sto) and not st.any()
    assert np.array_equal(cnt, stats[..., 0]), np.argwhere(cnt != stats[..., 0])[:4]
    assert _err(T64, To) <= SAME_VARIANT_TOL, _err(T64, To)
    assert np.array_equal(g_idx, oracle.associate(src[0], dst[0], T32, Ko))
    with oracle_like(rl):
        o_neq = oracle.reduce(src[0], dst[0], T32, Ko)
    assert g_neq[28] == o_neq[28]
    np.testing.assert_allclose(g_neq, o_neq, rtol=1e-11, atol=1e-9)


def test_default_reduction_is_launch_independent_at_survey_noise():
    """the default reduction at SURVEY §8d noise (sigma =
    1.5 mm Z^2) through three launch shapes -- all 512 pairs in ONE launch
    (the C4 headline geometry: persistent k_icp, 3072 chunks), pairs 0..127
    as two 64-pair shards on two streams with set_concurrency(2) (the N = 8
    shard), and pairs 0..127 one pair per call (k_icp_coop) -- every pose
    within 1e-5 of the CPU oracle in EXACT mode (launch-independent, no GPU
    parameter), and the shapes within 1e-9 of each other (fp64 order)."""
    W, H, iters = 640, 480, 10
    src, dst, _ = youth_synth.pairs(0, 512, W, H, flags=youth_synth.SURVEY_FLAGS)
    assert oracle.get_reduce() == oracle.REDUCE_EXACT
    T_cpu, st_cpu = oracle.align_batch(src, dst, iters=iters, n_threads=16)
    assert not st_cpu.any()
    ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
    torch.cuda.synchronize()
    with youth_icp.IcpContext(W, H, 512, iters=iters) as ctx:
        assert ctx.reduction == youth_icp.REDUCE_EXACT
        ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), 512)
        ctx.sync()
        T_batch, _, st = ctx.get_poses(512)
        assert ctx.get_plan()["kernel"].startswith("k_prep + k_icp")
    assert not st.any()
    assert _err(T_batch, T_cpu) <= POSE_TOL, _err(T_batch, T_cpu)
    # 64-pair shards, two contexts side by side on half the slots each
    streams = [torch.cuda.Stream() for _ in range(2)]
    ctxs = [youth_icp.IcpContext(W, H, 64, iters=iters) for _ in range(2)]
    try:
        for c in ctxs:
            c.set_concurrency(2)
        for k, (c, s) in enumerate(zip(ctxs, streams)):
            c.align_pairs_device(ds[64 * k:].data_ptr(), dd[64 * k:].data_ptr(), 64,
                                 stream=s.cuda_stream)
        torch.cuda.synchronize()
        T_shard = np.concatenate([c.get_poses(64)[0] for c in ctxs])
        st = np.concatenate([c.get_poses(64)[2] for c in ctxs])
    finally:
        for c in ctxs:
            c.close()
    assert not st.any()
    assert _err(T_shard, T_cpu[:128]) <= POSE_TOL, _err(T_shard, T_cpu[:128])
    # one pair per call: the cooperative single-pair kernel
    T_one = []
    with youth_icp.IcpContext(W, H, 2, iters=iters) as ctx:
        for p in range(128):
            ctx.align_pairs_device(ds[p:].data_ptr(), dd[p:].data_ptr(), 1)
            ctx.sync()
            T_one.append(ctx.get_poses(1)[0][0])
            assert ctx.get_plan()["kernel"] == "k_icp_coop"
    T_one = np.stack(T_one)
    assert _err(T_one, T_cpu[:128]) <= POSE_TOL, _err(T_one, T_cpu[:128])
    # the launch shape moves a pose by fp64 summation order only
    assert _err(T_shard, T_batch[:128]) <= SAME_VARIANT_TOL, _err(T_shard, T_batch[:128])
    assert _err(T_one, T_batch[:128]) <= SAME_VARIANT_TOL, _err(T_one, T_batch[:128])
