#!/bin/bash
# The drop-in path's backlogged passes (examples/slam_rate, plain-C producer)
# under a rocprofv3 kernel trace with the module's event trace on, then
# tools/slam_trace.py per pass.  Output: gpurun_out/slamtrace/.
set -eo pipefail
export TMPDIR=/tmp
O=gpurun_out/slamtrace
mkdir -p $O
YOUTH_SLAM_TRACE=$O/events.txt timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace \
    --output-format csv -d $O/kt -o kt -- slam-rgbd_amd/slam_rate 300 9 > $O/slam_rate.json 2> $O/slam_rate.err
KT=$(find $O/kt -name '*kernel_trace.csv' -print -quit)
python3 tools/slam_trace.py $O/events.txt $KT > $O/summary.txt
cat $O/summary.txt
# the same without the profiler (its overhead can shift the timing)
YOUTH_SLAM_TRACE=$O/events_noprof.txt timeout -k 10 120 slam-rgbd_amd/slam_rate 300 9 > $O/slam_rate_noprof.json
python3 tools/slam_trace.py $O/events_noprof.txt > $O/summary_noprof.txt
cat $O/summary_noprof.txt
