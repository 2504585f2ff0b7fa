"""GPU parity of both arithmetics of spec a7/a8, each against the oracle run
in the same spec:
  * YOUTH_SPEC_SURVEY (the default): SURVEY.md §8a a7/a8 as worded (no FMA:
    products and sums rounded separately in a fixed order; the projection
    quotient fx P'x / P'z an IEEE division).  Its oracle (ORACLE_SPEC_SURVEY)
    reproduces the round-1 fixtures bit for bit (tests/test_oracle.py) and
    equals an independent numpy restatement (tests/test_oracle_numpy.py);
  * YOUTH_SPEC_FMA (opt-in): fma chains, one correctly rounded reciprocal
    (fixtures tests/golden/fma/).

Every kernel of the iteration runs in this spec: the stage kernel k_reduce
(association indices, normal equations), the persistent k_icp (batches), the
cooperative k_icp_coop (single pairs at 640x480 and 1280x960, the tracker)
and the sequence path.  Bar as in test_gpu_parity.py: indices bit-exact given
the same fp32 pose, sums within rel 1e-11, poses within 1e-5 (observed
~1e-13), correspondence counts per iteration equal.
"""
import os

import numpy as np
import pytest
import torch

import oracle
import youth_icp
import youth_synth
from conftest import GOLDEN, lanes_of, oracle_like

pytestmark = pytest.mark.gpu
POSE_TOL = 1e-5
GOLDEN_DIR = {"survey": GOLDEN, "fma": os.path.join(GOLDEN, "fma")}
SPECS = ["survey", "fma"]


def _err(a, b):
    return float(np.abs(np.asarray(a)[..., :3, :4] - np.asarray(b)[..., :3, :4]).max())


def test_projquot_selftest():
    """The survey projection's quotient (correctly rounded reciprocal + one
    correction) equals IEEE num / den bitwise on 2^27 cases (half next to a
    rounding midpoint) and projects to the same pixel on 2^27 more; its
    one-instruction floor equals floorf (and its in-range test) on all 2^32
    floats but NaN and denormals."""
    q, p, f = youth_icp.selftest_projquot(1 << 27, seed=3)
    assert (q, p, f) == (0, 0, 0)


def test_spec_selection_api(monkeypatch):
    monkeypatch.delenv("YOUTH_ICP_SPEC", raising=False)
    with youth_icp.IcpContext(64, 48, 2) as ctx:
        assert ctx.spec == youth_icp.SPEC_SURVEY      # the default
        ctx.spec = "survey"
        assert ctx.spec == youth_icp.SPEC_SURVEY
        ctx.spec = "fma"
        assert ctx.spec == youth_icp.SPEC_FMA
        with pytest.raises(youth_icp.IcpError):
            ctx.spec = 5
        assert ctx.spec == youth_icp.SPEC_FMA


@pytest.mark.parametrize("spec", SPECS)
@pytest.mark.parametrize("name", ["pair_80x60", "pair_160x120", "pair_97x53"])
def test_golden_fixtures_per_spec(name, spec):
    """The spec's fixtures (survey: the round-1 files, written before the fma
    spec existed): indices at identity and at the final pose bit-exact,
    identity normal equations, and the final pose and per-iteration counts
    through the cooperative and the persistent kernel."""
    g = np.load(os.path.join(GOLDEN_DIR[spec], name + ".npz"), allow_pickle=False)
    K = youth_icp.Intrinsics(*[float(v) for v in g["K"]])
    H, W = g["src"].shape
    it, d = int(g["iters"]), float(g["dist_thresh"])
    with youth_icp.IcpContext(W, H, 4, K=K, iters=it, dist_thresh=d, spec=spec,
                              reduction="exact") as ctx:    # the fixtures' reduction
        assoc, neq = ctx.reduce(g["src"], g["dst"], np.eye(4, dtype=np.float32)[:3])
        assert np.array_equal(assoc, g["idx_identity"])
        np.testing.assert_allclose(neq, g["neq_identity"], rtol=1e-12, atol=1e-12)
        assoc, _ = ctx.reduce(g["src"], g["dst"], g["T32"])
        assert np.array_equal(assoc, g["idx_final"])
        ds = torch.from_numpy(np.stack([g["src"]] * 4)).cuda()
        dd = torch.from_numpy(np.stack([g["dst"]] * 4)).cuda()
        torch.cuda.synchronize()
        ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), 1)
        T1, _, s1 = ctx.get_poses(1)
        cnt, _ = ctx.get_stats(1, it)
        assert ctx.get_plan()["kernel"] == "k_icp_coop"
        assert s1[0] == int(g["status"]) and _err(T1[0], g["T64"]) <= POSE_TOL
        assert np.array_equal(cnt[0], g["stats"][:, 0])
    os.environ["YOUTH_ICP_NO_COOP"] = "1"
    try:
        with youth_icp.IcpContext(W, H, 4, K=K, iters=it, dist_thresh=d, spec=spec,
                              reduction="exact") as ctx:    # the fixtures' reduction
            ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), 4)
            T4, _, s4 = ctx.get_poses(4)
            cnt, _ = ctx.get_stats(4, it)
            assert ctx.get_plan()["kernel"].startswith("k_prep + k_icp")
    finally:
        del os.environ["YOUTH_ICP_NO_COOP"]
    for p in range(4):
        assert s4[p] == int(g["status"]) and _err(T4[p], g["T64"]) <= POSE_TOL
        assert np.array_equal(cnt[p], g["stats"][:, 0])


@pytest.mark.parametrize("spec", SPECS)
def test_assoc_bit_exact_every_iteration_640x480(spec):
    """Index bit-exactness given the SAME fp32 pose: the oracle's T_k (same
    spec) fed to both sides at every iteration, plus random poses up to
    30 deg / 20 cm under both noise models."""
    oracle.set_spec(spec)
    src, dst, _ = youth_synth.pairs(0, 1)
    src, dst = src[0], dst[0]
    K = oracle.viewer_K(640, 480)
    rng = np.random.default_rng(0x5BEE)
    with youth_icp.IcpContext(640, 480, 2, spec=spec) as ctx:
        T = np.eye(4)
        for it in range(10):
            T32 = T[:3].astype(np.float32)
            g_idx, g_neq = ctx.reduce(src, dst, T32)
            assert np.array_equal(g_idx, oracle.associate(src, dst, T32, K)), it
            with oracle_like(ctx):
                o_neq = oracle.reduce(src, dst, T32, K)
            np.testing.assert_allclose(g_neq, o_neq, rtol=1e-11, atol=1e-9)
            xi, st = oracle.solve(o_neq)
            assert st == 0
            T = oracle.se3_exp(xi) @ T
        for draw in range(24):
            flags = youth_synth.SURVEY_FLAGS if draw % 3 == 0 else 0
            s, t, _ = youth_synth.pairs(3000 + draw, 1, 640, 480, flags=flags)
            axis = rng.normal(size=3)
            axis /= np.linalg.norm(axis)
            th = np.deg2rad(rng.uniform(0, 30.0 if draw % 2 else 5.0))
            Tr = oracle.se3_exp(np.r_[axis * th, rng.uniform(-0.2, 0.2, 3)])
            T32 = Tr[:3].astype(np.float32)
            g_idx, g_neq = ctx.reduce(s[0], t[0], T32)
            assert np.array_equal(g_idx, oracle.associate(s[0], t[0], T32, K)), draw
            with oracle_like(ctx):
                o_neq = oracle.reduce(s[0], t[0], T32, K)
            np.testing.assert_allclose(g_neq, o_neq, rtol=1e-11, atol=1e-9, err_msg=str(draw))


@pytest.mark.parametrize("spec", SPECS)
def test_assoc_extreme_poses(spec):
    """The projection's rare paths, given the same fp32 pose on both sides:
    rotations up to 180 deg and translations along z of up to +-5 m put
    source points behind the camera (P'_z <= 0), at P'_z next to 0 (the
    quotient's range guard, the IEEE fallback) and far off the frame
    (saturated coordinates, the row clamp into the record pad).  Indices
    bit-exact, sums within rel 1e-11, match counts equal (k_reduce, which
    shares the pixel code with k_icp and k_icp_coop)."""
    oracle.set_spec(spec)
    K = oracle.viewer_K(640, 480)
    rng = np.random.default_rng(0xE47E)
    src, dst, _ = youth_synth.pairs(77, 1)
    Ts = []
    with youth_icp.IcpContext(640, 480, 2, spec=spec) as ctx:
        for draw in range(16):
            axis = rng.normal(size=3)
            axis /= np.linalg.norm(axis)
            th = np.deg2rad(rng.uniform(60.0, 180.0))
            t = np.r_[rng.uniform(-1.0, 1.0, 2), rng.uniform(-5.0, 5.0)]
            if draw % 4 == 0:
                t[2] = -float(np.median(src[src > 0])) / 1000.0   # the scene at the camera plane
            Tr = oracle.se3_exp(np.r_[axis * th, t])
            T32 = Tr[:3].astype(np.float32)
            g_idx, g_neq = ctx.reduce(src[0], dst[0], T32)
            o_idx = oracle.associate(src[0], dst[0], T32, K)
            assert np.array_equal(g_idx, o_idx), draw
            with oracle_like(ctx):
                o_neq = oracle.reduce(src[0], dst[0], T32, K)
            assert g_neq[28] == o_neq[28], draw
            np.testing.assert_allclose(g_neq, o_neq, rtol=1e-11, atol=1e-9, err_msg=str(draw))
            Ts.append(Tr)
    # the first iteration's match count from the same initial poses through
    # the cooperative kernel (one pair per call) and the persistent one (4
    # pairs, YOUTH_ICP_NO_COOP): the same pixel code with the other match
    # gate (masked normal / skipped update) and per-wave counts
    want = [int(oracle.align(src[0], dst[0], iters=1, T_init=T)[3][0, 0]) for T in Ts]
    ds = torch.from_numpy(np.stack([src[0]] * 4)).cuda()
    dd = torch.from_numpy(np.stack([dst[0]] * 4)).cuda()
    torch.cuda.synchronize()
    with youth_icp.IcpContext(640, 480, 4, iters=1, spec=spec) as ctx:
        for draw, T in enumerate(Ts):
            ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), 1, T_init=T[None])
            assert ctx.get_plan()["kernel"] == "k_icp_coop"
            cnt, _ = ctx.get_stats(1, 1)
            assert int(cnt[0, 0]) == want[draw], draw
    os.environ["YOUTH_ICP_NO_COOP"] = "1"
    try:
        with youth_icp.IcpContext(640, 480, 4, iters=1, spec=spec) as ctx:
            for d0 in range(0, len(Ts), 4):
                ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), 4,
                                       T_init=np.stack(Ts[d0:d0 + 4]))
                assert ctx.get_plan()["kernel"].startswith("k_prep + k_icp")
                cnt, _ = ctx.get_stats(4, 1)
                assert [int(v) for v in cnt[:, 0]] == want[d0:d0 + 4], d0
    finally:
        del os.environ["YOUTH_ICP_NO_COOP"]


@pytest.mark.parametrize("spec", SPECS)
def test_projections_below_the_frame(spec):
    """the survey arithmetic's projection has no explicit v' < H
    test; a row past the frame is clamped to H and rejected because its
    record index lands in the zeroed pad [N, P) or past the buffer.  Pinned
    here against the oracle's explicit test: camera moves along +y and tilts
    that push the lower rows of the scene to v' = H, H + 1, ... (counted
    below with the survey formula in numpy float32): indices bit-exact, sums
    within rel 1e-11, first-iteration match counts equal through k_icp_coop
    and the persistent k_icp."""
    oracle.set_spec(spec)
    W, H = 640, 480
    K = oracle.viewer_K(W, H)
    src, dst, _ = youth_synth.pairs(78, 1)
    X, Y, Z = oracle.backproject(src[0], K)
    f32 = np.float32
    Ts, at_H, below = [], 0, 0
    for ty in np.linspace(0.002, 0.30, 12):
        for tilt in (0.0, 2.0):
            Tr = oracle.se3_exp(np.r_[np.deg2rad(tilt), 0.0, 0.0, 0.0, ty, 0.0])
            T = Tr[:3].astype(np.float32)
            qy = ((T[1, 0] * X + T[1, 1] * Y) + T[1, 2] * Z) + T[1, 3]
            qz = ((T[2, 0] * X + T[2, 1] * Y) + T[2, 2] * Z) + T[2, 3]
            with np.errstate(divide="ignore", invalid="ignore"):
                fv = np.floor(((f32(K.fy) * qy) / qz + f32(K.cy)) + f32(0.5))
            live = (Z > 0) & (qz > 0)
            at_H += int((live & (fv == H)).sum())
            below += int((live & (fv >= H)).sum())
            Ts.append(Tr)
    assert at_H > 100 and below > 10000, (at_H, below)
    with youth_icp.IcpContext(W, H, 2, spec=spec) as ctx:
        for draw, Tr in enumerate(Ts):
            T32 = Tr[:3].astype(np.float32)
            g_idx, g_neq = ctx.reduce(src[0], dst[0], T32)
            assert np.array_equal(g_idx, oracle.associate(src[0], dst[0], T32, K)), draw
            with oracle_like(ctx):
                o_neq = oracle.reduce(src[0], dst[0], T32, K)
            assert g_neq[28] == o_neq[28], draw
            np.testing.assert_allclose(g_neq, o_neq, rtol=1e-11, atol=1e-9, err_msg=str(draw))
    want = [int(oracle.align(src[0], dst[0], iters=1, T_init=T)[3][0, 0]) for T in Ts]
    ds = torch.from_numpy(np.stack([src[0]] * 4)).cuda()
    dd = torch.from_numpy(np.stack([dst[0]] * 4)).cuda()
    torch.cuda.synchronize()
    with youth_icp.IcpContext(W, H, 4, iters=1, spec=spec) as ctx:
        for draw in range(0, len(Ts), 3):
            ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), 1, T_init=Ts[draw][None])
            assert int(ctx.get_stats(1, 1)[0][0, 0]) == want[draw], draw
    os.environ["YOUTH_ICP_NO_COOP"] = "1"
    try:
        with youth_icp.IcpContext(W, H, 4, iters=1, spec=spec) as ctx:
            for d0 in range(0, len(Ts), 4):
                ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), 4,
                                       T_init=np.stack(Ts[d0:d0 + 4]))
                cnt, _ = ctx.get_stats(4, 1)
                assert [int(v) for v in cnt[:, 0]] == want[d0:d0 + 4], d0
    finally:
        del os.environ["YOUTH_ICP_NO_COOP"]


@pytest.mark.parametrize("spec", SPECS)
@pytest.mark.parametrize("W,H,iters,n", [(640, 480, 10, 1), (640, 480, 10, 8),
                                         (640, 480, 10, 64), (1280, 960, 20, 1),
                                         (1280, 960, 20, 2)])
def test_align_all_kernel_paths_per_spec(W, H, iters, n, spec):
    """C2 (one pair: k_icp_coop), 8 pairs (k_icp_coop), 64 pairs (persistent
    k_icp: N = 8's shard of C4), C3 (1280x960, 20 iterations: the 64x80-tile
    coop kernel, and a 2-pair call), at the bench's noise and one pair at
    SURVEY §8d's: every pose within 1e-5 of the survey oracle, counts per
    iteration equal."""
    oracle.set_spec(spec)
    src, dst, _ = youth_synth.pairs(0, n, W, H)
    if n >= 8:
        s2, d2, _ = youth_synth.pairs(0, 1, W, H, flags=youth_synth.SURVEY_FLAGS)
        src[n - 1], dst[n - 1] = s2[0], d2[0]
    K = youth_icp.default_intrinsics(W, H)
    ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
    torch.cuda.synchronize()
    with youth_icp.IcpContext(W, H, max(n, 2), K=K, iters=iters, spec=spec) as ctx:
        ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n)
        T64, _, st = ctx.get_poses(n)
        cnt, _ = ctx.get_stats(n, iters)
        plan = ctx.get_plan()
        lanes = lanes_of(ctx)
    if n == 1:
        assert plan["kernel"] == "k_icp_coop"
    if n == 64:
        assert plan["kernel"].startswith("k_prep + k_icp")
    with oracle_like(lanes):
        T_cpu, st_cpu, stats = oracle.align_batch(src, dst, K=oracle.viewer_K(W, H),
                                                  iters=iters, n_threads=min(n, 16),
                                                  want_stats=True)
    assert np.array_equal(st, st_cpu) and not st.any()
    assert _err(T64, T_cpu) <= POSE_TOL
    assert np.array_equal(cnt, stats[..., 0])


@pytest.mark.parametrize("spec", SPECS)
def test_sequence_and_tracker_per_spec(spec):
    """C5 in each spec: a 65-frame 640x480 sequence through
    align_sequence_device (persistent path) and frame by frame through the
    tracker (k_icp_coop with the fused next-reference prep): every relative
    pose within 1e-5 of the oracle in the same spec."""
    oracle.set_spec(spec)
    F = 65
    frames, _ = youth_synth.sequence(0, F)
    d = torch.from_numpy(frames).cuda()
    torch.cuda.synchronize()
    T_cpu, _ = oracle.align_batch(frames[1:], frames[:-1], iters=10, n_threads=16)
    with youth_icp.IcpContext(640, 480, F - 1, spec=spec) as ctx:
        ctx.align_sequence_device(d.data_ptr(), F)
        T64, _, st = ctx.get_poses(F - 1)
        assert not st.any() and _err(T64, T_cpu) <= POSE_TOL
    with youth_icp.IcpContext(640, 480, 2, spec=spec) as ctx:
        Tseq, stseq = ctx.track_host_sequence(frames[:17])
    assert not stseq.any() and _err(Tseq, T_cpu[:16]) <= POSE_TOL


@pytest.fixture(autouse=True)
def _restore_oracle_spec():
    yield
    oracle.set_spec("survey")


def test_env_selects_spec(monkeypatch):
    monkeypatch.setenv("YOUTH_ICP_SPEC", "survey")
    with youth_icp.IcpContext(64, 48, 2) as ctx:
        assert ctx.spec == youth_icp.SPEC_SURVEY
    monkeypatch.setenv("YOUTH_ICP_SPEC", "fma")
    with youth_icp.IcpContext(64, 48, 2) as ctx:
        assert ctx.spec == youth_icp.SPEC_FMA
