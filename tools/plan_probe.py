"""Which kernel path align_pairs_device takes per (max_frames, iters, pairs)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-rgbd_amd"))
import torch  # noqa: E402
import youth_icp  # noqa: E402
import youth_synth  # noqa: E402

src, dst, _ = youth_synth.pairs(52, 16)
ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
for mf, it, n in ((2, 10, 1), (16, 10, 1), (2, 1, 1), (16, 1, 1), (2, 2, 1), (16, 3, 3), (16, 10, 16)):
    with youth_icp.IcpContext(640, 480, mf, iters=it) as ctx:
        ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n)
        T, _, st = ctx.get_poses(n)
        print(mf, it, n, ctx.get_plan(), st, flush=True)
