"""A second, independent restatement of spec a6-a9 in numpy, checked BIT FOR
BIT against the C oracle (oracle/icp_oracle.c) on the committed golden pairs
and on 640x480 synthetic pairs.  CPU only.

The reference has no ICP (a6-a10 are parity-unpinned at the
reference boundary), so the C oracle restates this build's own spec
(DESIGN.md §2).  This file guards that restatement against implementation
slips with a second implementation written from the spec text, not from the
C code's structure: whole-frame numpy array expressions instead of a pixel
loop, numpy float32 arithmetic (IEEE single, one rounding per operation, no
contraction) and an exact emulation of fmaf (fma32 below).  The 29 normal-
equation sums are compared exactly too: the products are exact in float64
and np.cumsum adds in pixel order, the oracle's summation order.
The SE(3) exp and the 6x6 solve (a10) are cross-checked against scipy /
numpy in test_oracle.py.

Spec a7/a8 exists in two arithmetics (oracle_set_spec): the default fma
chains, and SURVEY.md §8a a7/a8 as worded (no FMA, IEEE division), which is
plain numpy float32 evaluated left to right (``spec="survey"`` below).
"""
import numpy as np
import pytest

import oracle
import youth_synth
from conftest import GOLDEN

f32, f64 = np.float32, np.float64


def fma32(a, b, c):
    """Correctly rounded float32 fma(a, b, c), elementwise.  a*b is exact in
    float64; s = a*b + c rounds once in float64 and e (TwoSum) is its exact
    error.  round32(s + e) == round32(s) unless s sits exactly on a float32
    midpoint, where the sign of e breaks the tie."""
    a, b, c = (np.asarray(x, f32) for x in (a, b, c))
    p = a.astype(f64) * b.astype(f64)
    c64 = c.astype(f64)
    s = p + c64
    bb = s - p
    e = (p - (s - bb)) + (c64 - bb)
    r = s.astype(f32)
    r64 = r.astype(f64)
    up = np.nextafter(r, f32(np.inf))
    dn = np.nextafter(r, f32(-np.inf))
    tie_up = (s == (r64 + up.astype(f64)) / 2) & (e > 0)   # rounded down at a tie, true value above
    tie_dn = (s == (r64 + dn.astype(f64)) / 2) & (e < 0)   # rounded up at a tie, true value below
    return np.where(tie_up, up, np.where(tie_dn, dn, r)).astype(f32)


def test_fma32_exact_on_constructed_ties():
    # a*b = 1 + 2^-24 exactly (a float32 midpoint); c = +-2^-60 decides the rounding
    a = f32(1 + 2.0 ** -12)
    b = f32(1 + 2.0 ** -12)          # a*b = 1 + 2^-11 + 2^-24
    for c, want in ((f32(2.0 ** -60), f32(1 + 2.0 ** -11 + 2.0 ** -23)),
                    (f32(-(2.0 ** -60)), f32(1 + 2.0 ** -11)),
                    (f32(0.0), f32(1 + 2.0 ** -11))):     # exact tie: to even
        assert fma32(a, b, c) == want


def backproject_np(depth, K):
    """Spec a2: z = d / depth_scale; x = ((u - cx) * z) / fx; y likewise."""
    H, W = depth.shape
    d = depth.astype(f32)
    valid = depth > 0
    z = np.where(valid, d / f32(K.depth_scale), f32(0)).astype(f32)
    u = np.arange(W, dtype=f32)[None, :]
    v = np.arange(H, dtype=f32)[:, None]
    x = np.where(valid, ((u - f32(K.cx)) * z) / f32(K.fx), f32(0)).astype(f32)
    y = np.where(valid, ((v - f32(K.cy)) * z) / f32(K.fy), f32(0)).astype(f32)
    return x, y, z


def normals_np(X, Y, Z):
    """Spec a6: n = normalize((P(u+1)-P(u-1)) x (P(v+1)-P(v-1))), zero on the
    1-px border, where the centre or a 4-neighbour is invalid, or where the
    cross product vanishes; oriented so n . P <= 0."""
    H, W = Z.shape
    N = [np.zeros((H, W), f32) for _ in range(3)]
    c = (slice(1, H - 1), slice(1, W - 1))
    l, r = (slice(1, H - 1), slice(0, W - 2)), (slice(1, H - 1), slice(2, W))
    up, dn = (slice(0, H - 2), slice(1, W - 1)), (slice(2, H), slice(1, W - 1))
    ok = (Z[c] > 0) & (Z[l] > 0) & (Z[r] > 0) & (Z[up] > 0) & (Z[dn] > 0)
    ax, ay, az = X[r] - X[l], Y[r] - Y[l], Z[r] - Z[l]
    bx, by, bz = X[dn] - X[up], Y[dn] - Y[up], Z[dn] - Z[up]
    cx = ay * bz - az * by
    cy = az * bx - ax * bz
    cz = ax * by - ay * bx
    len2 = (cx * cx + cy * cy) + cz * cz
    ok &= len2 > 0
    with np.errstate(invalid="ignore", divide="ignore"):
        ln = np.sqrt(len2)
        nx, ny, nz = cx / ln, cy / ln, cz / ln
    flip = ((nx * X[c] + ny * Y[c]) + nz * Z[c]) > 0
    for k, n in enumerate((nx, ny, nz)):
        N[k][c] = np.where(ok, np.where(flip, -n, n), f32(0))
    return N


def associate_np(S, Tg, Nt, T12, K, thr, spec="fma"):
    """Spec a7 for every source pixel: target index or -1, and P'."""
    sx, sy, sz = (a.ravel() for a in S)
    tX, tY, tZ = (a.ravel() for a in Tg)
    nX, nY, nZ = (a.ravel() for a in Nt)
    H, W = S[2].shape
    T = np.asarray(T12, f32).ravel()
    if spec == "survey":
        # P' = R P + t, fixed order, no FMA;
        # u' = floor(fx P'x / P'z + cx + 0.5), left to right, IEEE division
        qx = ((T[0] * sx + T[1] * sy) + T[2] * sz) + T[3]
        qy = ((T[4] * sx + T[5] * sy) + T[6] * sz) + T[7]
        qz = ((T[8] * sx + T[9] * sy) + T[10] * sz) + T[11]
    else:
        qx = fma32(T[2], sz, fma32(T[1], sy, fma32(T[0], sx, T[3])))
        qy = fma32(T[6], sz, fma32(T[5], sy, fma32(T[4], sx, T[7])))
        qz = fma32(T[10], sz, fma32(T[9], sy, fma32(T[8], sx, T[11])))
    ok = (sz > 0) & (qz > 0)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        if spec == "survey":
            fu = np.floor(((f32(K.fx) * qx) / qz + f32(K.cx)) + f32(0.5))
            fv = np.floor(((f32(K.fy) * qy) / qz + f32(K.cy)) + f32(0.5))
        else:
            rz = f32(1) / qz
            fu = np.floor(fma32(f32(K.fx) * qx, rz, f32(K.cx) + f32(0.5)))
            fv = np.floor(fma32(f32(K.fy) * qy, rz, f32(K.cy) + f32(0.5)))
    ok &= (fu >= 0) & (fu < W) & (fv >= 0) & (fv < H)
    j = np.where(ok, np.where(ok, fv, 0).astype(np.int64) * W + np.where(ok, fu, 0).astype(np.int64), 0)
    ok &= tZ[j] > 0
    ok &= ~((nX[j] == 0) & (nY[j] == 0) & (nZ[j] == 0))
    dx, dy, dz = qx - tX[j], qy - tY[j], qz - tZ[j]
    d2 = (dx * dx + dy * dy) + dz * dz if spec == "survey" else fma32(dz, dz, fma32(dy, dy, dx * dx))
    thr2 = f32(thr) * f32(thr)
    ok &= d2 < thr2
    return np.where(ok, j, -1).astype(np.int32), (qx, qy, qz)


def reduce_np(S, Tg, Nt, T12, K, thr, spec="fma"):
    """Spec a8-a9: r = n . (P' - P_t), J = [P' x n, n]; the 21 + 6 + 1 + 1
    sums of exact float64 products in pixel order."""
    idx, (qx, qy, qz) = associate_np(S, Tg, Nt, T12, K, thr, spec)
    m = idx >= 0
    j = idx[m]
    tX, tY, tZ = (a.ravel()[j] for a in Tg)
    nx, ny, nz = (a.ravel()[j] for a in Nt)
    q0, q1, q2 = qx[m], qy[m], qz[m]
    dx, dy, dz = q0 - tX, q1 - tY, q2 - tZ
    if spec == "survey":
        r = (nx * dx + ny * dy) + nz * dz
        J = [q1 * nz - q2 * ny, q2 * nx - q0 * nz, q0 * ny - q1 * nx, nx, ny, nz]
    else:
        r = fma32(nz, dz, fma32(ny, dy, nx * dx))
        J = [fma32(q1, nz, -(q2 * ny)), fma32(q2, nx, -(q0 * nz)), fma32(q0, ny, -(q1 * nx)),
             nx, ny, nz]
    J64 = [a.astype(f64) for a in J]
    r64 = r.astype(f64)
    terms = [J64[a] * J64[b] for a in range(6) for b in range(a, 6)]
    terms += [J64[a] * r64 for a in range(6)] + [r64 * r64, np.ones_like(r64)]
    return np.array([np.cumsum(t)[-1] if t.size else 0.0 for t in terms], f64), idx


def _cases():
    g = np.load(GOLDEN + "/pair_160x120.npz")
    yield "pair_160x120", g["src"], g["dst"], oracle.K_of(g["K"]), float(g["dist_thresh"])
    src, dst, _ = youth_synth.pairs(7, 2, 640, 480)
    for p in range(2):
        yield f"synth640_{p}", src[p], dst[p], oracle.viewer_K(640, 480), 0.10
    src, dst, _ = youth_synth.pairs(9, 1, 640, 480, flags=youth_synth.SURVEY_FLAGS)
    yield "synth640_survey_noise", src[0], dst[0], oracle.viewer_K(640, 480), 0.10


@pytest.mark.parametrize("spec", ["fma", "survey"])
@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: c[0])
def test_numpy_restatement_equals_oracle_bitwise(case, spec):
    _, src, dst, K, thr = case
    S = backproject_np(src, K)
    Tg = backproject_np(dst, K)
    oS = oracle.backproject(src, K)
    oT = oracle.backproject(dst, K)
    for a, b in zip(S + Tg, oS + oT):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    Nt = normals_np(*Tg)
    oN = oracle.normals(*oT)
    for a, b in zip(Nt, oN):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert sum(int((n != 0).sum()) for n in Nt) > 0
    # identity, a small motion and a larger one (about 3 degrees, 4 cm)
    th = np.deg2rad(3.0)
    R = np.array([[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]])
    for T in (np.eye(4)[:3], np.hstack([np.eye(3), [[0.004], [-0.002], [0.003]]]),
              np.hstack([R, [[0.04], [0.01], [-0.02]]])):
        T12 = T.astype(f32)
        neq, idx = reduce_np(S, Tg, Nt, T12, K, thr, spec)
        with oracle.spec(spec):
            o_idx = oracle.associate(src, dst, T12, K, thr).ravel()
            o_neq = oracle.reduce(src, dst, T12, K, thr)
        assert np.array_equal(idx, o_idx)
        assert np.array_equal(neq.view(np.uint64), o_neq.view(np.uint64))
        assert neq[28] > 0


def test_world_frame_viewer_list_equals_numpy():
    """oracle_viewer_cloud_posed (youth_cloud_build_device_posed's checker)
    against the same three fma chains in numpy (fma32), bit for bit."""
    src, _, _ = youth_synth.pairs(4, 1, 160, 120)
    d = src[0]
    K = oracle.viewer_K(160, 120)
    th = 0.7
    T = np.array([[np.cos(th), -np.sin(th), 0, 1.5], [np.sin(th), np.cos(th), 0, -2.0],
                  [0, 0, 1, 0.25]], np.float32)
    x, y, z = backproject_np(d, K)
    m = (d > 0).ravel()
    x, y, z = x.ravel()[m], y.ravel()[m], z.ravel()[m]
    want = np.stack([-fma32(T[0, 2], z, fma32(T[0, 1], y, fma32(T[0, 0], x, T[0, 3]))),
                     -fma32(T[1, 2], z, fma32(T[1, 1], y, fma32(T[1, 0], x, T[1, 3]))),
                     -fma32(T[2, 2], z, fma32(T[2, 1], y, fma32(T[2, 0], x, T[2, 3])))], 1)
    got = oracle.viewer_cloud(d, None, K, T_world=T)
    assert np.array_equal(got[:, :3].view(np.uint32), want.view(np.uint32))
    assert not got[:, 3:].any()


# --------------------------------------------------- spec a9, lane32 mode --
def lane_np(kind, chunk, threads, npx, W, H):
    """Lane of every pixel (raster index) under a launch's partition, from
    include/youth_icp.h's description of youth_lanes."""
    i = np.arange(W * H, dtype=np.int64)
    T = threads
    if kind == oracle.LANES_STRIDED:
        c, o = i // chunk, i % chunk
        return c * T + (o % (4 * T)) // 4
    if kind == oracle.LANES_COOP:
        C = npx * T
        return (i // C) * T + (i % C) % T
    th = npx * T // 64
    u, v = i % W, i // W
    tx, ty = u // 64, v // th
    k = (v - ty * th) * 64 + (u - tx * 64)
    return (ty * ((W + 63) // 64) + tx) * T + k % T


def reduce_lane32_np(S, Tg, Nt, T12, K, thr, lanes, spec):
    """SURVEY §8a a9 as worded: per lane, fp32 sums (fma32, from +0, pixel
    order) of the matched pixels' 28 products; then the lanes' sums in fp64,
    in lane order; the count exact."""
    idx, (qx, qy, qz) = associate_np(S, Tg, Nt, T12, K, thr, spec)
    H, W = S[2].shape
    m = idx >= 0
    j = idx[m]
    tX, tY, tZ = (a.ravel()[j] for a in Tg)
    nx, ny, nz = (a.ravel()[j] for a in Nt)
    q0, q1, q2 = qx[m], qy[m], qz[m]
    dx, dy, dz = q0 - tX, q1 - tY, q2 - tZ
    if spec == "survey":
        r = (nx * dx + ny * dy) + nz * dz
        J = [q1 * nz - q2 * ny, q2 * nx - q0 * nz, q0 * ny - q1 * nx, nx, ny, nz]
    else:
        r = fma32(nz, dz, fma32(ny, dy, nx * dx))
        J = [fma32(q1, nz, -(q2 * ny)), fma32(q2, nx, -(q0 * nz)), fma32(q0, ny, -(q1 * nx)),
             nx, ny, nz]
    pairs = [(J[a], J[b]) for a in range(6) for b in range(a, 6)]
    pairs += [(J[a], r) for a in range(6)] + [(r, r)]
    lane = lane_np(*lanes, W, H)[m]
    n_lanes = int(lane_np(*lanes, W, H).max()) + 1
    order = np.argsort(lane, kind="stable")          # within a lane: pixel order
    ls = lane[order]
    first = np.r_[0, np.flatnonzero(np.diff(ls)) + 1]
    rank = np.arange(ls.size) - np.repeat(first, np.diff(np.r_[first, ls.size]))
    acc = np.zeros((n_lanes, 28), f32)
    for step in range(int(rank.max()) + 1 if rank.size else 0):
        sel = order[rank == step]
        L = lane[sel]
        for k, (a, b) in enumerate(pairs):
            acc[L, k] = fma32(a[sel], b[sel], acc[L, k])
    out = np.zeros(29, f64)
    for k in range(28):
        out[k] = np.cumsum(np.r_[0.0, acc[:, k].astype(f64)])[-1]
    out[28] = float(m.sum())
    return out


@pytest.mark.parametrize("spec", ["fma", "survey"])
@pytest.mark.parametrize("lanes", [(0, 2048, 256, 0), (0, 51200, 256, 0), (1, 0, 512, 3),
                                   (2, 0, 512, 3), (2, 0, 512, 10)],
                         ids=["strided2048", "strided51200", "coop3", "tile64x24", "tile64x80"])
def test_lane32_restatement_equals_oracle_bitwise(lanes, spec):
    """oracle_set_reduce(LANE32, partition) against the numpy restatement
    above, bit for bit, at 640x480 (the partitions k_icp, k_icp_coop and the
    tall-tile kernel use) and at a larger motion; and LANE32 against EXACT
    within the fp32 rounding of the lane sums."""
    src, dst, _ = youth_synth.pairs(7, 1, 640, 480)
    K = oracle.viewer_K(640, 480)
    S, Tg = backproject_np(src[0], K), backproject_np(dst[0], K)
    Nt = normals_np(*Tg)
    th = np.deg2rad(2.0)
    R = np.array([[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]])
    for T in (np.eye(4)[:3], np.hstack([R, [[0.02], [0.01], [-0.01]]])):
        T12 = T.astype(f32)
        want = reduce_lane32_np(S, Tg, Nt, T12, K, 0.10, lanes, spec)
        with oracle.spec(spec), oracle.reduction("lane32", lanes):
            got = oracle.reduce(src[0], dst[0], T12, K)
        with oracle.spec(spec):
            exact = oracle.reduce(src[0], dst[0], T12, K)
        assert np.array_equal(got.view(np.uint64), want.view(np.uint64))
        assert got[28] == exact[28] > 0
        assert np.abs(got[:28] - exact[:28]).max() <= 1e-4 * np.abs(exact[:28]).max()
    assert oracle.get_reduce() == oracle.REDUCE_EXACT


def test_lane32_rejects_bad_partitions():
    for mode, lanes in (("lane32", None), ("lane32", (0, 0, 256, 0)), ("lane32", (0, 2048, 100, 0)),
                        ("lane32", (1, 0, 512, 0)), ("lane32", (7, 2048, 256, 1)), (3, None)):
        with pytest.raises(ValueError):
            oracle.set_reduce(mode, lanes)
    assert oracle.get_reduce() == oracle.REDUCE_EXACT
