#!/bin/bash
# Round-4 GPU call k: the drop-in's backlogged passes with the worker's
# per-submission trace (tools/ab/slamtrace: batch size, frames in flight,
# queue depth, time waiting on collects / idle), to find the slow passes.
set -o pipefail
LD_LIBRARY_PATH=tools/ab/slamtrace timeout -k 10 120 slam-rgbd_amd/slam_rate 300 9 \
    > gpurun_out/slamtrace_r4k.json 2> gpurun_out/slamtrace_r4k.txt || exit 1
echo all done
