"""k_icp designated-summer probe: persistent path only (YOUTH_ICP_NO_COOP=1),
1 / 8 / 64 pairs, status and wall time per call."""
import os
import sys
import time
os.environ["YOUTH_ICP_NO_COOP"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-rgbd_amd"))
import torch  # noqa: E402
import youth_icp  # noqa: E402
import youth_synth  # noqa: E402

src, dst, _ = youth_synth.pairs(7, 64)
ds, dd = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
cases = ((1, 1), (1, 2), (1, 10), (8, 10), (64, 10))
if len(sys.argv) > 2:
    cases = ((int(sys.argv[1]), int(sys.argv[2])),)
for n, iters in cases:
    with youth_icp.IcpContext(640, 480, 64, iters=iters) as ctx:
        t0 = time.time()
        ctx.align_pairs_device(ds.data_ptr(), dd.data_ptr(), n)
        T, _, st = ctx.get_poses(n)
        print(n, iters, ctx.get_plan()["kernel"], "status", st[:4], "s", round(time.time() - t0, 3),
              ctx.get_sched_stats() if hasattr(ctx, "get_sched_stats") else "", flush=True)
