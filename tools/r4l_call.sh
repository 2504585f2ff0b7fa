#!/bin/bash
# Round-4 GPU call l: kernel + memory-copy timeline of the drop-in's
# backlogged passes (slam_rate), to see whether slow passes are H2D or kernel.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/slamprof_r4l -o run \
    -- slam-rgbd_amd/slam_rate 300 9 > gpurun_out/slamprof_r4l.json 2>/dev/null || exit 1
echo all done
