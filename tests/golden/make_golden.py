"""Generate the committed golden fixtures (tests/golden/*.npz).

Run from the repo root:  python tests/golden/make_golden.py

Provenance, case by case:
  * kat_backproject — the back-projection known-answer table of SURVEY.md §4,
    computed by the survey from the reference formula viewerModule.c:343-345
    with gcc -O2 -ffp-contract=off (x86-64 SSE fp32).  These are the only
    vectors pinned to the REFERENCE; they are written out here verbatim.
  * pair_* / seq_* — inputs from the synthetic depth source
    (libyouth_synth.so), expected outputs from the C oracle
    (oracle/liboracle.so) in its default spec, spec a7/a8 as SURVEY.md §8a
    words it (ORACLE_SPEC_SURVEY: no FMA, IEEE division).  The committed
    files are the round-1 fixtures, written by the round-1 oracle before the
    fma spec existed (identical to git 1041b06^:tests/golden/); running this
    script regenerates them with today's oracle and leaves their arrays
    equal (tests/test_oracle.py checks that without writing).
  * Round 5 changed spec a10's solve (LDL^T -> block elimination with 3x3
    adjugates).  T64 / T32 / status / stats / idx_final
    (pairs) and T_rel (sequences) are the block solve's; the round-1 LDL^T
    results stay in the files verbatim as T64_ldlt / T32_ldlt and T_rel_ldlt
    (the oracle reproduces them in oracle.solve_mode("ldlt")).  Everything
    before the solve (xyz, normals, association, neq) is unchanged.
  * fma/pair_* / fma/seq_* — the same cases in the opt-in fma spec
    (ORACLE_SPEC_FMA, `--fma`).  The reference has no ICP, so
    these pin this build's own spec against regressions: "parity unpinned"
    with respect to the reference beyond back-projection.

Fixtures are data only (numpy .npz, loaded with allow_pickle=False).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "slam-rgbd_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
import youth_synth  # noqa: E402

# (W, H, u, v, d_mm, X_bits, Y_bits, Z_bits)
KAT = [
    (640, 480, 0, 0, 1000, 0xBF0FA4C9, 0xBED7772E, 0x3F800000),
    (640, 480, 639, 479, 4000, 0x400F31DF, 0x3FD6915A, 0x40800000),
    (640, 480, 320, 240, 1234, 0x00000000, 0x00000000, 0x3F9DF3B6),
    (640, 480, 17, 401, 32767, 0xC18B45CE, 0x41140186, 0x42031168),
    (1280, 960, 1279, 0, 2500, 0x40334629, 0xC006AA7D, 0x40200000),
]


def scaled_K(W, H):
    """Focal length scaled with the width so small frames keep a 58 deg FOV."""
    return oracle.OracleIntrinsics(570.3 * W / 640.0, 570.3 * W / 640.0, float(W // 2),
                                   float(H // 2), 1000.0)


def make_pair_case(name, W, H, index, iters=10, dist=0.10, out=HERE):
    K = scaled_K(W, H)
    src, dst, Tgt = youth_synth.pairs(index, 1, W, H, K=_yk(K))
    src, dst = src[0], dst[0]
    sX, sY, sZ = oracle.backproject(src, K)
    tX, tY, tZ = oracle.backproject(dst, K)
    nX, nY, nZ = oracle.normals(tX, tY, tZ)
    I12 = np.eye(4, dtype=np.float32)[:3]
    idx0 = oracle.associate(src, dst, I12, K, dist)
    neq0 = oracle.reduce(src, dst, I12, K, dist)
    T64, T32, st, stats = oracle.align(src, dst, K, iters, dist)
    with oracle.solve_mode("ldlt"):
        T64l, T32l, _, _ = oracle.align(src, dst, K, iters, dist)
    idxF = oracle.associate(src, dst, T32, K, dist)
    np.savez_compressed(
        os.path.join(out, name + ".npz"), src=src, dst=dst,
        K=np.array([K.fx, K.fy, K.cx, K.cy, K.depth_scale], np.float32),
        iters=np.int32(iters), dist_thresh=np.float32(dist), T_gt=Tgt[0],
        src_xyz=np.stack([sX, sY, sZ]), dst_xyz=np.stack([tX, tY, tZ]),
        dst_nrm=np.stack([nX, nY, nZ]), idx_identity=idx0, neq_identity=neq0,
        T64=T64, T32=T32, status=np.int32(st), stats=stats, idx_final=idxF,
        T64_ldlt=T64l, T32_ldlt=T32l)
    print(f"{name}: status={st} matches0={int((idx0 >= 0).sum())} "
          f"final count={stats[-1, 0]:.0f}")


def _yk(K):
    from youth_icp import Intrinsics
    return Intrinsics(K.fx, K.fy, K.cx, K.cy, K.depth_scale)


def make_seq_case(name, W, H, n_frames, iters=10, dist=0.10, out=HERE):
    K = scaled_K(W, H)
    frames, Twc = youth_synth.sequence(0, n_frames, W, H, K=_yk(K))
    rel, rel_l = [], []
    for k in range(n_frames - 1):
        T64, T32, st, _ = oracle.align(frames[k + 1], frames[k], K, iters, dist)
        rel.append(T64)
        with oracle.solve_mode("ldlt"):
            rel_l.append(oracle.align(frames[k + 1], frames[k], K, iters, dist)[0])
    np.savez_compressed(os.path.join(out, name + ".npz"), frames=frames,
                        K=np.array([K.fx, K.fy, K.cx, K.cy, K.depth_scale], np.float32),
                        iters=np.int32(iters), dist_thresh=np.float32(dist), T_wc=Twc,
                        T_rel=np.stack(rel), T_rel_ldlt=np.stack(rel_l))
    print(f"{name}: {n_frames} frames")


def make_recording(name, n=3, W=24, H=16, seed=7):
    """A .bin recording written with Python's struct module from the
    reference's layouts (FrameHeader '<IIHHH2xIII', frameDefinitions.h:11-20;
    frame = header + int16 depth + uint8 RGB, loggingModule.c:101-130; end
    marker = zero header with frameType 0xFF, :224-226) — independent of the
    C writer it is used to check (tests/test_wire.py)."""
    import struct
    fh = struct.Struct("<IIHHH2xIII")
    rng = np.random.default_rng(seed)
    b = bytearray()
    for k in range(n):
        d = rng.integers(-5, 9000, (H, W)).astype(np.int16)
        c = rng.integers(0, 256, (H, W, 3)).astype(np.uint8)
        b += fh.pack(100 + k, 1000 + 33 * k, 1, W, H, W * H * 2, W * H * 3, 0)
        b += d.astype("<i2").tobytes() + c.tobytes()
    b += fh.pack(0, 0, 0xFF, 0, 0, 0, 0, 0)
    with open(os.path.join(HERE, name), "wb") as f:
        f.write(bytes(b))
    print(f"{name}: {n} frames, {len(b)} bytes")


PAIR_CASES = [("pair_80x60", 80, 60, 0), ("pair_160x120", 160, 120, 1),
              ("pair_97x53", 97, 53, 2)]
SEQ_CASES = [("seq_128x96", 128, 96, 6)]


def main():
    if "--fma" in sys.argv:
        out = os.path.join(HERE, "fma")
        os.makedirs(out, exist_ok=True)
        with oracle.spec("fma"):
            for args in PAIR_CASES:
                make_pair_case(*args, out=out)
            for args in SEQ_CASES:
                make_seq_case(*args, out=out)
        return
    make_recording("rec_24x16_3f.bin")
    np.savez_compressed(os.path.join(HERE, "kat_backproject.npz"),
                        table=np.array(KAT, dtype=np.int64))
    with oracle.spec("survey"):
        for args in PAIR_CASES:
            make_pair_case(*args)
        for args in SEQ_CASES:
            make_seq_case(*args)


if __name__ == "__main__":
    main()
