#!/bin/bash
# Round-4 GPU call m: drop-in backlogged rate with the tracker's collect
# polling its event (default) vs the blocking hipEventSynchronize
# (YOUTH_ICP_TRACK_WAIT=sync), interleaved; the trace build (tools/ab/slamtrace,
# blocking wait) for reference.
set -o pipefail
O=gpurun_out/slam_wait_r4m.txt
: > $O
for r in 1 2 3; do
  for m in sync poll; do
    echo "wait=$m" >> $O
    YOUTH_ICP_TRACK_WAIT=$m timeout -k 10 120 slam-rgbd_amd/slam_rate 300 9 2>/dev/null >> $O || exit 1
  done
done
echo all done
